"""CPU checks of the HIP engine's launch-geometry invariants (no GPU needed)."""
import itertools

from rocalphago_amd.models.engine import ConvSpec, pack_grid_width


def _pack_blocks(spec, width):
    """(tile, tap) pairs the blocks x < width of conv.hip pack_trunk_kernel cover for one layer
    (the kernel's own index arithmetic, restated)."""
    taps = spec.ks * spec.ks
    ntn, ntc = -(-spec.coutp // 64), -(-spec.cinp // 64)
    seen = []
    for x in range(width):
        xcd, j = x & 7, x >> 3
        g, tap = (j // taps) * 8 + xcd, j % taps
        if g < ntn * ntc:
            seen.append((g, tap))
    return seen, ntn * ntc, taps


def test_pack_trunk_grid_covers_every_tile_tap_once():
    """The XCD-grouped pack order: the grid width is a multiple of 8 (block x runs on XCD x % 8
    for every layer row of the 2-D grid), every (64x64 tile, tap) of every layer is packed
    exactly once, and all taps of one tile run on one XCD."""
    shapes = [ConvSpec(5, 48, 192, True), ConvSpec(3, 192, 192, True), ConvSpec(1, 192, 1, False),
              ConvSpec(3, 128, 128, True), ConvSpec(3, 40, 64, True), ConvSpec(5, 64, 128, True),
              ConvSpec(3, 256, 256, True)]
    for k in range(1, 4):
        for specs in itertools.combinations(shapes, k):
            width = pack_grid_width(specs)
            assert width % 8 == 0
            for s in specs:
                seen, ntiles, taps = _pack_blocks(s, width)
                assert sorted(seen) == [(g, t) for g in range(ntiles) for t in range(taps)]
                xcd_of = {}
                for x in range(width):
                    j = x >> 3
                    g = (j // taps) * 8 + (x & 7)
                    if g < ntiles:
                        xcd_of.setdefault(g, set()).add(x & 7)
                assert all(len(v) == 1 for v in xcd_of.values())
