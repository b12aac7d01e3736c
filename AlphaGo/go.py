"""AlphaGo.go — rules engine (native C++ core). See rocalphago_amd/engine/gamestate.py."""
from rocalphago_amd.engine.gamestate import (BLACK, EMPTY, PASS_MOVE, WHITE, GameState,  # noqa: F401
                                             IllegalMove)
