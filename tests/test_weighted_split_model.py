"""CPU model of the XCD-weighted split (csrc/kernels/reduce_kernels.hpp weighted_tiles /
weighted_tail / XcdAnchor, csrc/kernels/reduce.hip plan_reduce / make_args).

The kernel's own bijection test runs on the GPU (tests/test_kernels_gpu.py::test_xcd_weighted_split
and ::test_xcd_weighted_split_follows_the_xccs). This mirrors the same integer formulas in Python so
that every (ntiles, grid, skew, favoured parity) corner can be swept in milliseconds: whichever
parity the anchor picks, every tile is streamed exactly once.
"""
import pytest


def plan_skew(ntiles, grid, permille):
    """plan_reduce: permille of the rounds -> extra rounds d, kept only with >= 1 common round."""
    rounds = ntiles // grid
    q = rounds * permille + (500 if permille >= 0 else -500)
    d = abs(q) // 1000 * (1 if q >= 0 else -1)  # C++ division truncates toward zero
    return d if grid % 2 == 0 and abs(d) * (grid // 2) + grid <= ntiles else 0


def args(ntiles, grid, xskew):
    """make_args: common rounds ra and extra rounds dd."""
    if xskew == 0:
        return ntiles // grid, 0
    d = abs(xskew)
    return (ntiles - d * (grid // 2)) // grid, d


def tiles_of(b, ntiles, grid, xskew, fpar):
    """The tiles workgroup b streams (run 0, then runs 1 and 2), fpar = favoured blockIdx parity."""
    ra, dd = args(ntiles, grid, xskew)
    out = [b + k * grid for k in range(ra)]
    base1 = ra * grid
    if xskew == 0:
        if b < ntiles - base1:
            out.append(base1 + b)
        return out
    half = grid // 2
    fav = (b & 1) == fpar
    if fav:
        out += [base1 + (b >> 1) + k * half for k in range(dd)]
    base2 = base1 + dd * half
    rank2 = (b >> 1) if fav else half + (b >> 1)
    if rank2 < ntiles - base2:
        out.append(base2 + rank2)
    return out


@pytest.mark.parametrize("grid", [2, 8, 256, 512])
@pytest.mark.parametrize("ntiles", [2, 255, 256, 257, 6347, 30517, 244140])
@pytest.mark.parametrize("permille", [-300, -20, 0, 16, 20, 40, 400, 5000])
def test_every_tile_once_for_either_parity(grid, ntiles, permille):
    xskew = plan_skew(ntiles, grid, permille)
    for fpar in (0, 1):
        seen = [0] * ntiles
        for b in range(grid):
            for t in tiles_of(b, ntiles, grid, xskew, fpar):
                assert 0 <= t < ntiles, (b, t)
                seen[t] += 1
        assert all(c == 1 for c in seen), (grid, ntiles, xskew, fpar)
        if xskew:
            ra, _ = args(ntiles, grid, xskew)
            assert ra >= 1  # the kernel resolves the anchor at the end of the common rounds


def test_favoured_parity_gets_the_extra_rounds():
    ntiles, grid = 244140, 256  # 1e9 float64 in 32 KB tiles
    xskew = plan_skew(ntiles, grid, 20)
    assert xskew == 19
    for fpar in (0, 1):
        n = [len(tiles_of(b, ntiles, grid, xskew, fpar)) for b in range(grid)]
        fav = [n[b] for b in range(grid) if b % 2 == fpar]
        other = [n[b] for b in range(grid) if b % 2 != fpar]
        assert min(fav) > max(other)
