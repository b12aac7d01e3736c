"""CPU checks of the HIP engine's launch-geometry invariants (no GPU needed)."""
import itertools

import pytest

from rocalphago_amd.models.engine import ConvSpec, pack_grid_width

_PT = 16  # pack.h pack_trunk_block: 16 (n) x 16 (c) all-tap tiles


def _pack_tiles(spec, width):
    """Tiles the blocks x < width of a pack_trunk launch (pack.h pack_trunk_block) visit for one
    layer (each block grid-strides over the layer's tiles: the kernel's own loop, restated)."""
    ntiles = -(-spec.coutp // _PT) * -(-spec.cinp // _PT)
    seen = []
    for x in range(width):
        seen.extend(range(x, ntiles, width))
    return seen, ntiles


def _tile_elements(taps):
    """(n offset, c offset, tap) of the elements thread tid handles in chunk i0 (the kernel's
    idx = tid + 256 i, i = i0 + k < taps, k < 16; row = 16 taps contiguous masters per n)."""
    row = _PT * taps
    out = []
    for tid in range(256):
        for i0 in range(0, taps, 16):
            for k in range(16):
                i = i0 + k
                if i >= taps:
                    break
                idx = tid + 256 * i
                r, e = divmod(idx, row)
                cl, tap = divmod(e, taps)
                out.append((r, cl, tap))
    return out


def test_pack_trunk_grid_covers_every_tile_once():
    """The grid width is a multiple of 8 and at least the widest layer's tile count, and every
    16x16 tile of every layer in a launch is packed exactly once."""
    shapes = [ConvSpec(5, 48, 192, True), ConvSpec(3, 192, 192, True), ConvSpec(1, 192, 1, False),
              ConvSpec(3, 128, 128, True), ConvSpec(3, 40, 64, True), ConvSpec(5, 64, 128, True),
              ConvSpec(3, 256, 256, True), ConvSpec(7, 48, 48, True)]
    for k in range(1, 4):
        for specs in itertools.combinations(shapes, k):
            width = pack_grid_width(specs)
            assert width % 8 == 0
            for s in specs:
                seen, ntiles = _pack_tiles(s, width)
                assert sorted(seen) == list(range(ntiles))
                assert width >= ntiles  # one tile per block at the widest layer


@pytest.mark.parametrize("ks", [1, 3, 5, 7])
def test_pack_trunk_tile_elements_each_once(ks):
    """Inside a tile the 256 threads cover the 16 x 16 x taps masters exactly once, each thread's
    loads in chunks of 16 (kernels up to 7x7: 49 taps)."""
    taps = ks * ks
    el = _tile_elements(taps)
    assert len(el) == len(set(el)) == _PT * _PT * taps
    assert set(el) == {(r, c, t) for r in range(_PT) for c in range(_PT) for t in range(taps)}


def test_trunk_rejects_kernels_above_7x7():
    """pack_trunk_kernel stages at most 49 taps per tile: larger kernels are refused up front."""
    import torch
    from rocalphago_amd.models.engine import HipTrunk
    with pytest.raises(ValueError, match="7x7"):
        HipTrunk([ConvSpec(9, 48, 64, True)], 19, torch.device("cpu"))


def test_wino_pack_grid_covers_every_tile():
    """pack.h wino_pack_block: one block per 32 (n) x 16 (c) tile; rag_wino_pack
    launches 8 blocks per 64 x 64 tile of the widest layer, which covers every layer's tiles."""
    for coutp, cinp in [(192, 192), (128, 128), (192, 64), (384, 192), (64, 32), (256, 96)]:
        max_tiles = -(-coutp // 64) * -(-cinp // 64)
        assert -(-coutp // 32) * -(-cinp // 16) <= 8 * max_tiles
