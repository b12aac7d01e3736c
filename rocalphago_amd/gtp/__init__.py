"""GTP serving and the match harness (C46)."""
from .engine import (PASS, RESIGN, ExtendedGtpEngine, GtpEngine, GtpError, GTPGameConnector,  # noqa: F401
                     format_vertex, parse_color, parse_move, parse_vertex, run_gtp)
from .match import PlayMatch, play_match  # noqa: F401
