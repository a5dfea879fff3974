"""CPU tests of the multi-GPU partition logic (msm_amd.dist): point shards, signed-digit window
ranges and the points x windows split every rank and every device-list thread takes its share
from.  The GPU side (partials of window ranges joining to the MSM) is in
tests/test_gpu_windows.py; here: every (point, window) pair is computed exactly once."""
import pytest

import msm_amd as M
from msm_amd.dist import SPLIT_HALF_WINDOWS, SPLIT_WINDOW_BITS, parse_split, shard_range, split_part, window_ranges


@pytest.mark.parametrize("c", range(4, 21))
@pytest.mark.parametrize("q", range(1, 9))
@pytest.mark.parametrize("halves", [False, True])
def test_window_ranges_cover_and_balance(c, q, halves):
    wm = M.window_count(c)
    u = 2 if halves else 1
    rs = window_ranges(wm, q, halves)
    assert len(rs) == q
    assert all(len(r) == (3 if halves else 2) and (not halves or r[2] == 2) for r in rs)
    # contiguous, starting at 0, ending at u wm (the overflow window in the top range)
    assert rs[0][0] == 0 and rs[-1][1] == u * wm
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    assert all(r[0] < r[1] for r in rs)
    # the main windows balanced: range sizes (overflow window aside) differ by at most one unit
    sizes = [r[1] - r[0] for r in rs]
    sizes[-1] -= u
    assert max(sizes) - min(sizes) <= 1
    if halves and q == 2:
        assert sizes[0] == sizes[1]  # any main-window count splits evenly in half windows


def test_parse_split():
    assert parse_split("points", 8) == (8, 1)
    assert parse_split("auto", 4) == (4, 1)
    assert parse_split("", 2) == (2, 1)
    assert parse_split("4x2", 8) == (4, 2)
    assert parse_split("1X8", 8) == (1, 8)
    for bad in ("3x2", "0x8", "4x4", "8x0"):
        with pytest.raises(ValueError):
            parse_split(bad, 8)


@pytest.mark.parametrize("world,split", [(1, "points"), (2, "points"), (2, "1x2"), (4, "2x2"), (4, "1x4"),
                                         (8, "points"), (8, "4x2"), (8, "2x4"), (8, "1x8"), (3, "3x1")])
@pytest.mark.parametrize("n", [1 << 20, (1 << 18) + 7, 5])
def test_split_part_covers_every_point_and_window_once(world, split, n):
    P, Q = parse_split(split, world)
    c = SPLIT_WINDOW_BITS if Q > 1 else None
    wm = M.window_count(c) if c else None
    seen = {}
    for rank in range(world):
        lo, hi, win, cw = split_part(n, rank, world, split)
        assert (lo, hi) == shard_range(n, rank // Q, P)
        if Q == 1:
            assert win is None and cw is None
            win = (0, 1)  # all windows, one token
        else:
            units = 2 if len(win) > 2 else 1
            assert cw == SPLIT_WINDOW_BITS and 0 <= win[0] < win[1] <= units * wm
        key = (lo, hi)
        seen.setdefault(key, []).append(tuple(win))
    # P disjoint point shards covering [0, n), each split into the same complete window partition
    shards = sorted(seen)
    assert len(shards) == P and shards[0][0] == 0 and shards[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))
    for wins in seen.values():
        wins.sort()
        assert len(wins) == Q
        if Q > 1:
            assert wins == window_ranges(wm, Q, SPLIT_HALF_WINDOWS)
