"""Compatibility module for ``interface/TestPlay.py`` (reference)."""
from rocalphago_amd.gtp.match import AXIS, RESULT, PlayMatch as play_match  # noqa: F401
from rocalphago_amd.engine.gamestate import BLACK, EMPTY, WHITE  # noqa: F401
