"""Compatibility module for ``interface/Play.py`` (reference)."""
from rocalphago_amd.gtp.match import PlayMatch as play_match  # noqa: F401
