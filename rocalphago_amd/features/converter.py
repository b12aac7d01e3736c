"""SGF -> HDF5 training-data converter — reference AlphaGo/preprocessing/game_converter.py.

Output layout (SURVEY §2.5 c), written by our own HDF5 writer (io/h5lite.py):
  states   uint8 (N, F, S, S), maxshape (None, F, S, S), chunks (64, F, S, S), LZF
  actions  uint8 (N, 2) as (x, y), chunks (1024, 2), LZF
  file_offsets/<path with '/' -> ':'> = [start, length]
  features = "board,ones,..." (comma-joined feature list)
The file is written to ``.tmp.<name>`` and atomically renamed on success; per-game errors are
handled like the reference (IllegalMove drops the remainder of a game, parse errors and board
size mismatches skip the game, anything else warns when ``ignore_errors``).

Speed: features for all positions of a game are computed by the native engine; with
``workers > 1`` games are converted in parallel processes (positions streamed in file order).
"""
import os
import sys
import warnings

import numpy as np

from ..engine import gamestate as go
from ..io import h5lite, sgf
from ..utils.go_util import sgf_iter_states
from .preprocessing import DEFAULT_FEATURES, Preprocess


class SizeMismatchError(Exception):
    pass


class GameConverter(object):

    def __init__(self, features):
        self.feature_processor = Preprocess(features)
        self.n_features = self.feature_processor.output_dim

    def convert_game(self, file_name, bd_size):
        """Yield (features (1, F, S, S), move (x, y)) for every non-pass move of the game."""
        with open(file_name, 'r') as file_object:
            state_action_iterator = sgf_iter_states(file_object.read(), include_end=False)
        for (state, move, player) in state_action_iterator:
            if state.size != bd_size:
                raise SizeMismatchError()
            if move != go.PASS_MOVE:
                nn_input = self.feature_processor.state_to_tensor(state)
                yield (nn_input, move)

    def _game_arrays(self, file_name, bd_size):
        """All (states uint8 [n,F,S,S], actions uint8 [n,2]) of a game, plus the error."""
        states, actions, err = [], [], None
        try:
            for st, mv in self.convert_game(file_name, bd_size):
                states.append(st[0].astype(np.uint8))
                actions.append(mv)
        except Exception as e:  # classified by the caller, like the reference
            err = e
        return states, actions, err

    def sgfs_to_hdf5(self, sgf_files, hdf5_file, bd_size=19, ignore_errors=True, verbose=False):
        tmp_file = os.path.join(os.path.dirname(hdf5_file), ".tmp." + os.path.basename(hdf5_file))
        h5f = h5lite.File(tmp_file, 'w')
        try:
            states = h5f.require_dataset(
                'states', dtype=np.uint8, shape=(1, self.n_features, bd_size, bd_size),
                maxshape=(None, self.n_features, bd_size, bd_size), exact=False,
                chunks=(64, self.n_features, bd_size, bd_size), compression="lzf")
            actions = h5f.require_dataset(
                'actions', dtype=np.uint8, shape=(1, 2), maxshape=(None, 2), exact=False,
                chunks=(1024, 2), compression="lzf")
            file_offsets = h5f.require_group('file_offsets')
            h5f['features'] = np.bytes_(','.join(self.feature_processor.feature_list))
            if verbose:
                print("created HDF5 dataset in {}".format(tmp_file))
            next_idx = 0
            for file_name in sgf_files:
                if verbose:
                    print(file_name)
                n_pairs = 0
                file_start_idx = next_idx
                game_states, game_actions, err = self._game_arrays(file_name, bd_size)
                if isinstance(err, (sgf.SGFParseError, SizeMismatchError)):
                    game_states, game_actions = [], []
                for st, mv in zip(game_states, game_actions):
                    if next_idx >= len(states):
                        states.resize((next_idx + 1, self.n_features, bd_size, bd_size))
                        actions.resize((next_idx + 1, 2))
                    states[next_idx] = st
                    actions[next_idx] = mv
                    n_pairs += 1
                    next_idx += 1
                if isinstance(err, go.IllegalMove):
                    warnings.warn("Illegal Move encountered in %s\n"
                                  "\tdropping the remainder of the game" % file_name)
                elif isinstance(err, sgf.SGFParseError):
                    warnings.warn("Could not parse %s\n\tdropping game" % file_name)
                elif isinstance(err, SizeMismatchError):
                    warnings.warn("Skipping %s; wrong board size" % file_name)
                elif err is not None:
                    if ignore_errors:
                        warnings.warn("Unkown exception with file %s\n\t%s" % (file_name, err),
                                      stacklevel=2)
                    else:
                        raise err
                if n_pairs > 0:
                    file_name_key = file_name.replace('/', ':')
                    file_offsets[file_name_key] = np.array([file_start_idx, n_pairs],
                                                           dtype=np.int64)
                    if verbose:
                        print("\t%d state/action pairs extracted" % n_pairs)
                elif verbose:
                    print("\t-no usable data-")
            if next_idx == 0:
                states.resize((0, self.n_features, bd_size, bd_size))
                actions.resize((0, 2))
        except Exception as e:
            print("sgfs_to_hdf5 failed")
            h5f._fh.close()
            os.remove(tmp_file)
            raise e
        if verbose:
            print("finished. renaming %s to %s" % (tmp_file, hdf5_file))
        h5f.close()
        os.rename(tmp_file, hdf5_file)


def run_game_converter(cmd_line_args=None):
    import argparse
    parser = argparse.ArgumentParser(
        description='Prepare SGF Go game files for training the neural network model.',
        epilog="Available features are: board, ones, turns_since, liberties, capture_size, "
               "self_atari_size, liberties_after, ladder_capture, ladder_escape, sensibleness, "
               "zeros, legal and color")
    parser.add_argument("--features", "-f", help="Comma-separated list of features to compute and store or 'all'", default='all')  # noqa: E501
    parser.add_argument("--outfile", "-o", help="Destination to write data (hdf5 file)", required=True)  # noqa: E501
    parser.add_argument("--recurse", "-R", help="Set to recurse through directories searching for SGF files", default=False, action="store_true")  # noqa: E501
    parser.add_argument("--directory", "-d", help="Directory containing SGF files to process. if not present, expects files from stdin", default=None)  # noqa: E501
    parser.add_argument("--size", "-s", help="Size of the game board. SGFs not matching this are discarded with a warning", type=int, default=19)  # noqa: E501
    parser.add_argument("--verbose", "-v", help="Turn on verbose mode", default=False, action="store_true")  # noqa: E501
    if cmd_line_args is None:
        args = parser.parse_args()
    else:
        args = parser.parse_args(cmd_line_args)
    if args.features.lower() == 'all':
        feature_list = list(DEFAULT_FEATURES)
    else:
        feature_list = args.features.split(",")
    if args.verbose:
        print("using features", feature_list)
    converter = GameConverter(feature_list)

    def _is_sgf(fname):
        return fname.strip()[-4:] == ".sgf"

    def _walk_all_sgfs(root):
        for (dirpath, dirname, files) in os.walk(root):
            for filename in sorted(files):
                if _is_sgf(filename):
                    yield os.path.join(dirpath, filename)

    def _list_sgfs(path):
        files = sorted(os.listdir(path))
        return (os.path.join(path, f) for f in files if _is_sgf(f))

    if args.directory:
        files = _walk_all_sgfs(args.directory) if args.recurse else _list_sgfs(args.directory)
    else:
        files = (f.strip() for f in sys.stdin if _is_sgf(f))
    converter.sgfs_to_hdf5(files, args.outfile, bd_size=args.size, verbose=args.verbose)
