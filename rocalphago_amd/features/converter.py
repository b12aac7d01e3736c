"""SGF -> HDF5 training-data converter (reference AlphaGo/preprocessing/game_converter.py API).

Bulk path: game files are read in batches, the native converter (csrc/engine/converter.cpp)
replays and featurises every game of a batch in parallel on the shared thread pool, and the
rows are appended to the datasets in file order as whole 64-row LZF chunks (io/h5lite.py
``WDataset.append``). A game the native parser does not reproduce exactly (parse error, a board
size other than ``bd_size``, non-ASCII syntax, unusual coordinates) is converted by the Python
replay below instead, which raises and is reported exactly as by the reference.

Output layout (SURVEY §2.5 c, a file-format contract):
  states   uint8 (N, F, S, S), maxshape (None, F, S, S), chunks (64, F, S, S), LZF
  actions  uint8 (N, 2) as (x, y), chunks (1024, 2), LZF
  file_offsets/<path with '/' -> ':'> = [start, length]
  features = "board,ones,..." (comma-joined feature list)
The file is written as ``.tmp.<name>`` and renamed when complete. Per-game outcomes follow the
reference: an illegal move keeps the game's positions up to it, unparsable games and games of
another board size are skipped, anything else is a warning (``ignore_errors``) or raised.
"""
import os
import sys
import time
import warnings

import numpy as np

from .._native import engine as _engine
from ..engine import gamestate as go
from ..io import h5lite, sgf
from ..utils.go_util import sgf_iter_states
from .preprocessing import DEFAULT_FEATURES, Preprocess

_rg = _engine()
_NATIVE_OK, _NATIVE_ILLEGAL = 0, 1
_CHUNK = 64  # rows per states chunk (the layout contract)


class SizeMismatchError(Exception):
    pass


def _addr(a):
    return a.__array_interface__["data"][0]


def _join(arrs):
    """Concatenate row blocks; a view when they are adjacent slices of one C-contiguous base."""
    if len(arrs) == 1:
        return arrs[0]
    a0 = arrs[0]
    base = a0.base
    pos = _addr(a0)
    adjacent = base is not None and a0.flags.c_contiguous
    for a in arrs:
        if not adjacent:
            break
        adjacent = a.base is base and a.flags.c_contiguous and _addr(a) == pos and \
            a.shape[1:] == a0.shape[1:] and a.dtype == a0.dtype
        pos += a.nbytes
    if adjacent:
        rows = sum(a.shape[0] for a in arrs)
        return np.lib.stride_tricks.as_strided(a0, shape=(rows,) + a0.shape[1:],
                                               strides=a0.strides, writeable=False)
    return np.concatenate(arrs)


class _Sink(object):
    """The output file: datasets + per-file offsets, rows appended in order."""

    def __init__(self, path, features, n_planes, size):
        self.path = path
        self.f = h5lite.File(path, "w")
        shp = (n_planes, size, size)
        self.states = self.f.require_dataset(
            "states", dtype=np.uint8, shape=(0,) + shp, maxshape=(None,) + shp, exact=False,
            chunks=(_CHUNK,) + shp, compression="lzf")
        self.actions = self.f.require_dataset(
            "actions", dtype=np.uint8, shape=(0, 2), maxshape=(None, 2), exact=False,
            chunks=(1024, 2), compression="lzf")
        self.offsets = self.f.require_group("file_offsets")
        self.f["features"] = np.bytes_(",".join(features))
        self.rows = 0
        self._queue = []

    def add(self, file_name, states, actions, rows_only=False):
        """Queue one game's rows (written by flush(), in order). rows_only: the states come
        with the batch's fused chunks (flush_fused); only the actions are queued."""
        n = len(actions)
        if n == 0:
            return 0
        st = None if rows_only else np.asarray(states, dtype=np.uint8)
        self._queue.append((st, np.asarray(actions, dtype=np.uint8).reshape(n, 2)))
        self.offsets[file_name.replace("/", ":")] = np.array([self.rows, n], dtype=np.int64)
        self.rows += n
        return n

    def flush_fused(self, lead, chunks, tail):
        """Append a batch converted on the fused path: its actions, then its states as the
        lead rows + precompressed whole chunks + tail rows."""
        if self._queue:
            self.actions.append(_join([q[1] for q in self._queue]))
            self._queue = []
        self.states.append_chunks(lead, chunks, tail)

    def flush(self):
        """Append the queued games as one block: whole 64-row chunks compress in parallel. Rows
        of consecutive games that already sit back to back in one native block are appended as
        a view of it (no concatenation)."""
        if not self._queue:
            return
        st = _join([q[0] for q in self._queue])
        ac = _join([q[1] for q in self._queue])
        self._queue = []
        self.states.append(st)
        self.actions.append(ac)

    def close(self):
        self.flush()
        self.f.close()

    def abort(self):
        self.f._fh.close()
        os.remove(self.path)


class GameConverter(object):

    def __init__(self, features):
        self.feature_processor = Preprocess(features)
        self.n_features = self.feature_processor.output_dim
        self.games_per_s = None

    # ---- reference API: one game as a python generator --------------------------------------
    def convert_game(self, file_name, bd_size):
        """Yield (features (1, F, S, S), move (x, y)) for every non-pass move of the game."""
        with open(file_name, "r") as fh:
            replay = sgf_iter_states(fh.read(), include_end=False)
        for state, move, _player in replay:
            if state.size != bd_size:
                raise SizeMismatchError()
            if move is not go.PASS_MOVE:
                yield self.feature_processor.state_to_tensor(state), move

    def _python_game(self, file_name, bd_size):
        """(states [n, F, S, S] uint8, actions [(x, y)], the exception that ended the game)."""
        planes, moves = [], []
        try:
            for tensor, move in self.convert_game(file_name, bd_size):
                planes.append(tensor[0].astype(np.uint8))
                moves.append(move)
        except Exception as e:  # classified by the caller
            return planes, moves, e
        return planes, moves, None

    # ---- bulk conversion ----------------------------------------------------------------------
    def _batch(self, names, bd_size, nthreads, lead=None):
        """Per game of a batch: (states array or list, actions, error or None). ``nthreads``
        0 converts every game with the Python replay (the reference's path; benchmarks).

        ``lead`` (the rows the writer's pending chunk still needs): the fused path -- the
        native converter LZF-compresses every whole 64-row chunk of the batch while it is
        cache-hot and returns only the lead and tail rows as planes. Returns (games, fused)
        with fused = (lead rows, [(bytes, compressed)], tail rows) or None when a game of the
        batch took the Python replay (its rows then go through the unfused path)."""
        if nthreads == 0:
            return [self._python_game(name, bd_size) for name in names], None
        texts, native_idx = [], []
        for i, name in enumerate(names):
            try:
                with open(name, "rb") as fh:
                    raw = fh.read()
                raw.decode("utf-8")  # undecodable files take the python path (and its error)
            except (OSError, UnicodeDecodeError):
                continue
            texts.append(raw)
            native_idx.append(i)
        fuse = lead is not None and len(native_idx) == len(names)
        done = [None] * len(names)
        fused = None
        if texts:
            zw, zb, _ = go._zobrist(bd_size)
            args = (texts, list(self.feature_processor.feature_ids), bd_size,
                    np.ascontiguousarray(zw.ravel()), np.ascontiguousarray(zb.ravel()),
                    nthreads)
            if fuse:
                status, rows, block, acts, chunks, L = _rg.convert_games(
                    *args, chunk_rows=_CHUNK, lead=int(lead))
                if any(c not in (_NATIVE_OK, _NATIVE_ILLEGAL) and n
                       for c, n in zip(status.tolist(), rows.tolist())):
                    # rows of a game the writer will not keep sit inside the chunks: unfused
                    return self._batch(names, bd_size, nthreads, None)
                fused = (block[:L], chunks, block[L:])
                block = None
            else:
                status, rows, block, acts = _rg.convert_games(*args)
            at = 0
            for i, code, n in zip(native_idx, status.tolist(), rows.tolist()):
                st = block[at:at + n] if block is not None else n
                ac = acts[at:at + n]
                at += n
                if code == _NATIVE_OK:
                    done[i] = (st, ac, None)
                elif code == _NATIVE_ILLEGAL:
                    done[i] = (st, ac, go.IllegalMove("illegal move in SGF replay"))
        for i, name in enumerate(names):
            if done[i] is None:
                done[i] = self._python_game(name, bd_size)
                if fused is not None and len(done[i][1]):
                    # a game the native parser rejected but the replay converts: its rows
                    # belong between the batch's native rows -- redo the batch unfused
                    return self._batch(names, bd_size, nthreads, None)
        return done, fused

    def sgfs_to_hdf5(self, sgf_files, hdf5_file, bd_size=19, ignore_errors=True, verbose=False,
                     batch=32, nthreads=8, fused=True):
        tmp = os.path.join(os.path.dirname(hdf5_file), ".tmp." + os.path.basename(hdf5_file))
        sink = _Sink(tmp, self.feature_processor.feature_list, self.n_features, bd_size)
        if verbose:
            print("created HDF5 dataset in {}".format(tmp))
        sink.states.nthreads = max(1, nthreads)
        fuse = bool(fused)
        t0, ngames = time.time(), 0
        files = iter(sgf_files)
        # the next batch converts on a helper thread (the native converter releases the GIL)
        # while this one is written; batches are small so that even a few hundred games overlap
        from concurrent.futures import ThreadPoolExecutor
        ex = ThreadPoolExecutor(1)

        def submit(lead):
            names = [n for _, n in zip(range(batch), files)]
            if not names:
                return None
            return names, ex.submit(self._batch, names, bd_size, nthreads,
                                    lead if fuse else None)
        try:
            nxt = submit(sink.states.lead_rows())
            while nxt is not None:
                names, fut = nxt
                results, fused = fut.result()
                # rows of this batch that reach the file (unparsable / wrong-size games drop)
                kept = 0
                for states, moves, err in results:
                    if not isinstance(err, (sgf.SGFParseError, SizeMismatchError)):
                        kept += len(moves)
                nxt = submit((sink.states.lead_rows() - kept) % _CHUNK)
                for name, (states, moves, err) in zip(names, results):
                    ngames += 1
                    if verbose:
                        print(name)
                    if isinstance(err, (sgf.SGFParseError, SizeMismatchError)):
                        states, moves = [], []
                    n = sink.add(name, states, moves, rows_only=fused is not None)
                    self._report(name, err, ignore_errors)
                    if verbose:
                        print("\t%d state/action pairs extracted" % n if n else
                              "\t-no usable data-")
                if fused is not None:
                    sink.flush_fused(*fused)
                else:
                    sink.flush()
        except Exception:
            print("sgfs_to_hdf5 failed")
            ex.shutdown(wait=True)
            sink.abort()
            raise
        ex.shutdown(wait=True)
        self.games_per_s = ngames / max(time.time() - t0, 1e-9)
        if verbose:
            print("finished (%.1f games/s). renaming %s to %s" % (self.games_per_s, tmp,
                                                                 hdf5_file))
        sink.close()
        os.rename(tmp, hdf5_file)

    @staticmethod
    def _report(name, err, ignore_errors):
        if err is None:
            return
        if isinstance(err, go.IllegalMove):
            warnings.warn("Illegal Move encountered in %s\n\tdropping the remainder of the game"
                          % name)
        elif isinstance(err, sgf.SGFParseError):
            warnings.warn("Could not parse %s\n\tdropping game" % name)
        elif isinstance(err, SizeMismatchError):
            warnings.warn("Skipping %s; wrong board size" % name)
        elif ignore_errors:
            warnings.warn("Unknown exception with file %s\n\t%s" % (name, err), stacklevel=2)
        else:
            raise err


def _sgf_files(directory, recurse):
    if not recurse:
        return (os.path.join(directory, f) for f in sorted(os.listdir(directory))
                if f.strip().endswith(".sgf"))
    return (os.path.join(d, f) for d, _, fs in os.walk(directory) for f in sorted(fs)
            if f.strip().endswith(".sgf"))


def run_game_converter(cmd_line_args=None):
    """CLI of the reference converter (game_converter.py:154-229), plus --threads."""
    import argparse
    ap = argparse.ArgumentParser(
        description="Prepare SGF Go game files for training the neural network model.",
        epilog="Available features are: board, ones, turns_since, liberties, capture_size, "
               "self_atari_size, liberties_after, ladder_capture, ladder_escape, sensibleness, "
               "zeros, legal and color")
    ap.add_argument("--features", "-f", default="all",
                    help="Comma-separated list of features to compute and store or 'all'")
    ap.add_argument("--outfile", "-o", required=True, help="Destination to write data (hdf5 file)")
    ap.add_argument("--recurse", "-R", default=False, action="store_true",
                    help="Set to recurse through directories searching for SGF files")
    ap.add_argument("--directory", "-d", default=None,
                    help="Directory containing SGF files to process. if not present, expects "
                         "files from stdin")
    ap.add_argument("--size", "-s", type=int, default=19,
                    help="Size of the game board. SGFs not matching this are discarded with a "
                         "warning")
    ap.add_argument("--verbose", "-v", default=False, action="store_true",
                    help="Turn on verbose mode")
    ap.add_argument("--threads", type=int, default=8,
                    help="native converter threads (games of a batch in parallel)")
    args = ap.parse_args(cmd_line_args)
    features = list(DEFAULT_FEATURES) if args.features.lower() == "all" else \
        args.features.split(",")
    if args.verbose:
        print("using features", features)
    if args.directory:
        files = _sgf_files(args.directory, args.recurse)
    else:
        files = (line.strip() for line in sys.stdin if line.strip().endswith(".sgf"))
    GameConverter(features).sgfs_to_hdf5(files, args.outfile, bd_size=args.size,
                                         verbose=args.verbose, nthreads=args.threads)
