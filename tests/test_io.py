"""h5lite HDF5 reader/writer, LZF codec, SGF parsing/writing, and parity with reference fixtures."""
import os

import numpy as np
import pytest

from rocalphago_amd import _native
from rocalphago_amd.engine import BLACK, WHITE, GameState
from rocalphago_amd.features.preprocessing import Preprocess
from rocalphago_amd.io import h5lite, sgf
from rocalphago_amd.utils import go_util


def test_lzf_roundtrip():
    rg = _native.engine()
    rng = np.random.RandomState(0)
    for data in [b"", b"a", b"abcabcabcabcabcabc" * 100, rng.bytes(5000),
                 (rng.rand(20000) > 0.9).astype(np.uint8).tobytes()]:
        c = rg.lzf_compress(data)
        if c is None:
            continue
        assert rg.lzf_decompress(c, len(data)) == data
    sparse = np.zeros(100000, np.uint8).tobytes()
    assert len(rg.lzf_compress(sparse)) < 2000


def test_h5_write_read_roundtrip(tmp_path):
    p = str(tmp_path / "x.h5")
    rng = np.random.RandomState(1)
    big = (rng.rand(300, 5, 7, 7) > 0.7).astype(np.uint8)
    with h5lite.File(p, "w") as f:
        f.attrs["layer_names"] = [b"conv_a", b"conv_bb"]
        g = f.create_group("conv_a")
        g.attrs["weight_names"] = [b"conv_a_W", b"conv_a_b"]
        g["conv_a_W"] = np.arange(24, dtype=np.float32).reshape(2, 3, 2, 2)
        g["conv_a_b"] = np.array([1.5, -2.0], dtype=np.float32)
        ds = f.require_dataset("states", dtype=np.uint8, shape=(1, 5, 7, 7),
                               maxshape=(None, 5, 7, 7), chunks=(64, 5, 7, 7), compression="lzf")
        for i in range(300):
            if i >= len(ds):
                ds.resize((i + 1, 5, 7, 7))
            ds[i] = big[i]
        fo = f.require_group("file_offsets")
        for k in range(40):  # more entries than one symbol-table leaf holds
            fo["game_%03d.sgf" % k] = [k * 3, 3]
        f["features"] = np.bytes_("board,ones")
        f["i64"] = np.arange(5, dtype=np.int64)
    r = h5lite.File(p)
    assert sorted(r.keys()) == ["conv_a", "features", "file_offsets", "i64", "states"]
    assert list(r.attrs["layer_names"]) == [b"conv_a", b"conv_bb"]
    assert np.array_equal(r["conv_a/conv_a_W"][()], np.arange(24).reshape(2, 3, 2, 2))
    assert r["conv_a"].attrs["weight_names"][1] == b"conv_a_b"
    s = r["states"]
    assert s.shape == (300, 5, 7, 7) and s.chunks == (64, 5, 7, 7)
    assert np.array_equal(s[()], big)
    assert np.array_equal(s[130], big[130]) and np.array_equal(s[10:200], big[10:200])
    assert len(r["file_offsets"].keys()) == 40
    assert list(r["file_offsets"]["game_017.sgf"][()]) == [51, 3]
    assert r["features"][()] == b"board,ones"
    assert "features" in r and "nope" not in r
    assert r["i64"][()].dtype == np.int64


def test_reads_reference_keras_weights(ref_data):
    f = h5lite.File(os.path.join(ref_data, "hdf5", "random_minimodel_weights.hdf5"))
    names = [n.decode() for n in f.attrs["layer_names"]]
    assert names[:2] == ["convolution2d_1", "convolution2d_2"] and names[-1] == "activation_1"
    assert f["convolution2d_1/convolution2d_1_W"].shape == (16, 12, 5, 5)
    assert f["bias_1/param_0"].shape == (361,)


def test_reference_dataset_parity(ref_data):
    """Our engine + features regenerate the reference converter's output exactly."""
    d = h5lite.File(os.path.join(ref_data, "hdf5", "alphago-vs-lee-sedol-features.hdf5"))
    states, actions = d["states"][()], d["actions"][()]
    assert states.shape == (1033, 12, 19, 19)
    pp = Preprocess(["board", "ones", "turns_since"])
    root = os.path.dirname(os.path.dirname(ref_data))
    fo = d["file_offsets"]
    seen = 0
    for key in fo.keys():
        start, n = fo[key][()]
        path = os.path.join(root, key.replace(":", "/").replace("//", "/"))
        with open(path) as fh:
            txt = fh.read()
        i = start
        for (st, mv, pl) in go_util.sgf_iter_states(txt, include_end=False):
            if mv is None:
                continue
            assert tuple(actions[i]) == mv
            assert np.array_equal(pp.state_to_tensor(st)[0].astype(np.uint8), states[i])
            i += 1
        seen += i - start
    assert seen == 1033


def test_sgf_parser_variations_and_escapes():
    txt = "(;SZ[9]C[a \\] b];B[aa](;W[bb];B[cc])(;W[dd]))"
    game = sgf.parse(txt)[0]
    assert game.root.properties["C"] == ["a ] b"]
    moves = [n.properties for n in game.rest]
    assert moves == [{"B": ["aa"]}, {"W": ["bb"]}, {"B": ["cc"]}]
    with pytest.raises(sgf.SGFParseError):
        sgf.parse("(;B[aa]")


def test_sgf_roundtrip_with_handicap(tmp_path):
    gs = GameState(19)
    gs.place_handicaps([(3, 3), (15, 15)])
    for m in [(10, 10), (4, 4), None, (5, 5)]:
        gs.do_move(m)
    go_util.save_gamestate_to_sgf(gs, str(tmp_path), "g.sgf")
    txt = open(str(tmp_path / "g.sgf")).read()
    assert "HA[2]" in txt and "[tt]" in txt
    back = go_util.sgf_to_gamestate(txt)
    assert np.array_equal(back.board, gs.board)


def test_setup_stones_sgf(ref_data):
    with open(os.path.join(ref_data, "sgf_with_handicap", "ab_aw.sgf")) as fh:
        gs = go_util.sgf_to_gamestate(fh.read())
    assert (gs.board == BLACK).sum() > 0 and (gs.board == WHITE).sum() > 0


def test_flatten_helpers():
    assert go_util.flatten_idx((2, 3), 19) == 41
    assert go_util.unflatten_idx(41, 19) == (2, 3)


def test_plot_network_output_writes_png(tmp_path):
    """Heat map of a policy distribution (optional matplotlib; reference util.py:131-231)."""
    pytest.importorskip("matplotlib")
    import numpy as np
    from rocalphago_amd.engine.gamestate import GameState
    from rocalphago_amd.utils import go_util
    gs = GameState(size=9)
    for mv in [(2, 2), (6, 6), (2, 6)]:
        gs.do_move(mv)
    p = np.random.RandomState(0).dirichlet(np.ones(81))
    go_util.plot_network_output(p, gs.board, gs.history, str(tmp_path), "h.png")
    go_util.plot_network_output(p, gs.board, gs.history, str(tmp_path), "h2.png",
                                western_column_notation=False)
    assert (tmp_path / "h.png").stat().st_size > 1000
    assert (tmp_path / "h2.png").stat().st_size > 1000
