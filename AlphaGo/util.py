"""AlphaGo.util — SGF / index helpers. See rocalphago_amd/utils/go_util.py."""
from rocalphago_amd.utils.go_util import (LETTERS, _parse_sgf_move, _sgf_init_gamestate,  # noqa: F401
                                          flatten_idx, plot_network_output,
                                          save_gamestate_to_sgf, sgf_iter_states,
                                          sgf_to_gamestate, unflatten_idx)
