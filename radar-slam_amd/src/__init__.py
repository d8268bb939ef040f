"""Reference-compatible package ``src`` (zaidcontractor/radar-slam module paths), MI355X-native.

Same dotted paths, class names, constructor kwargs, public attributes, method signatures and return
dict keys as the reference's ``src`` namespace package; the compute runs as HIP kernels of
``librsl.so`` through ``rsl``.  Importing fails loudly when the library has not been built.
"""
import os as _os
import sys as _sys

_PKG = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _PKG not in _sys.path:
    _sys.path.insert(0, _PKG)

from rsl import _lib as _rsl_lib  # noqa: E402

if not _os.path.exists(_rsl_lib.LIB_PATH):
    raise ImportError(f"librsl.so is not built ({_rsl_lib.LIB_PATH}); run __graft_entry__.build()")
