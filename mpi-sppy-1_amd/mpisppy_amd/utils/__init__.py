"""Utilities (W / x̄ CSV I/O, config helpers)."""
