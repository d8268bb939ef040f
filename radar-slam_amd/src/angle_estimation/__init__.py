"""Reference-compatible subpackage (see src/__init__.py)."""
