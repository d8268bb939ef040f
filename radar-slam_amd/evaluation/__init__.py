"""Drop-in for the reference's ``evaluation`` package (device-backed pose-error evaluation)."""
