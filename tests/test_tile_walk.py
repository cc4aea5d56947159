"""The one-wave-per-SIMD GEMM's XCD-banded tile order (csrc/include/gemm_impl.h band_tile, round 6), replicated
in Python: a bijection on the tiles whenever band_ok() admits the shape, every XCD (hardware blocks with
blockIdx % 8 == x) computes exactly the tile-rows of its own band, and the static walk gives every block
the same number of items.  (The cfg-11 GPU tests — tests/test_gemm_w1_gpu.py SHAPES (65536, 768, 768),
(65536, 512, 128) and the fp8 (65536, 3072, 1024) case — run the device code on banded shapes against fp32.)"""

import pytest

GROUP_M = 8


def xcd_remap(bid, n):
    xcd, loc = bid & 7, bid >> 3
    q, r = n >> 3, n & 7
    return (xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q) + loc


def group_tile_g(i, tm_, tn_, gm):
    per = gm * tn_
    gid = i // per
    first = gid * gm
    gsz = min(tm_ - first, gm)
    inn = i % per
    return first + inn % gsz, inn // gsz


def band_ok(grid, tm_, tn_):
    return grid % 8 == 0 and tm_ % 8 == 0 and (tm_ * tn_) % grid == 0


def band_tile(u, grid, tm_, tn_, gm):
    per = grid >> 3
    s, r = divmod(u, grid)
    x = r // per
    bx = tm_ >> 3
    a, b = group_tile_g(r - x * per + s * per, bx, tn_, gm)
    return a + x * bx, b


@pytest.mark.parametrize("grid,tm_,tn_", [(256, 256, 3), (256, 256, 9), (256, 256, 12), (256, 256, 197),
                                          (256, 128, 4), (256, 128, 12), (256, 128, 16), (248, 248, 8),
                                          (128, 64, 6), (256, 32, 8)])
def test_band_walk_is_a_per_xcd_bijection(grid, tm_, tn_):
    assert band_ok(grid, tm_, tn_)
    tiles = tm_ * tn_
    seen = {}
    for hw in range(grid):  # hardware block id: XCD hw % 8
        bid = xcd_remap(hw, grid)
        s = 0
        while bid + s * grid < tiles:
            t = band_tile(bid + s * grid, grid, tm_, tn_, GROUP_M)
            assert t not in seen
            seen[t] = hw % 8
            s += 1
        assert s == tiles // grid  # every block the same number of items
    assert len(seen) == tiles
    bx = tm_ // 8
    for (m, n), x in seen.items():
        assert m // bx == x, "a tile-row computed outside its XCD's band"


def test_band_not_taken_for_uneven_shapes():
    assert not band_ok(256, 394, 3)   # ViT-B/16 tokens (b512 x 197): tile-rows % 8 != 0
    assert not band_ok(256, 128, 197)  # GPT-2-medium LM head: 25216 tiles % 256 != 0
    assert not band_ok(252, 256, 3)    # a grid with reserved CUs that is not a multiple of 8
