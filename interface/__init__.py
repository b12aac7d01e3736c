"""Reference-compatible ``interface`` package (GTP wrapper and match harness)."""
