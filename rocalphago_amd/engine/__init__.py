"""Go rules engine (native C++ core + reference-compatible python facade)."""
from .gamestate import BLACK, EMPTY, PASS_MOVE, WHITE, GameState, IllegalMove  # noqa: F401
