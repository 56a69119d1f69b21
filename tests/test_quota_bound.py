"""The level-list capacity of the device retain path (orbx_geometry.cpp:
level_cap = nDesired + 2 nCells + 64) rests on a bound on what the
reference's quota redistribution (src/ORBextractor.cc:622-670) can retain
per level: sum_c min(nTotal_c, nToRetain_c) <= nDesired + 2 nCells - 1.
This replays the reference loop (float ceil included) on random and
adversarial cell totals and checks the bound."""
import math

import numpy as np
import pytest


def retained(n_desired, totals, valid):
    n_cells = len(totals)
    nfc = math.ceil(np.float32(n_desired) / np.float32(n_cells))
    ret = [0] * n_cells
    nomore = [False] * n_cells
    to_dist, n_nomore = 0, 0
    for c in range(n_cells):
        if not valid[c]:
            continue                      # `continue` before nTotal is set (:567-596)
        if totals[c] > nfc:
            ret[c] = nfc
        else:
            ret[c] = totals[c]
            to_dist += nfc - totals[c]
            nomore[c] = True
            n_nomore += 1
    tot = [t if v else 0 for t, v in zip(totals, valid)]
    while to_dist > 0 and n_nomore < n_cells:
        n_new = nfc + math.ceil(np.float32(to_dist) / np.float32(n_cells - n_nomore))
        to_dist = 0
        for c in range(n_cells):
            if not nomore[c]:
                if tot[c] > n_new:
                    ret[c] = n_new
                else:
                    ret[c] = tot[c]
                    to_dist += n_new - tot[c]
                    nomore[c] = True
                    n_nomore += 1
    return sum(min(t, r) for t, r in zip(tot, ret))


@pytest.mark.parametrize("seed", range(40))
def test_quota_bound_random(seed):
    r = np.random.default_rng(seed)
    n_cells = int(r.integers(1, 257))
    n_desired = int(r.integers(1, 4097))
    shape = seed % 4
    if shape == 0:
        totals = r.integers(0, 3 * n_desired // n_cells + 3, n_cells)
    elif shape == 1:   # a few rich cells, many poor ones
        totals = np.where(r.random(n_cells) < 0.1, r.integers(0, 5000, n_cells), r.integers(0, 3, n_cells))
    elif shape == 2:   # graded totals: many redistribution rounds
        totals = np.sort(r.integers(0, 2 * n_desired // n_cells + 2, n_cells))
    else:
        totals = r.geometric(1.0 / (1 + n_desired / n_cells), n_cells)
    valid = r.random(n_cells) > (0.05 if seed % 5 == 0 else 0.0)
    got = retained(n_desired, [int(t) for t in totals], list(valid))
    assert got <= n_desired + 2 * n_cells - 1, (got, n_desired, n_cells)


def test_quota_bound_staircase():
    """Totals 1, 2, 3, ... force one cell out per round (the worst case for
    the loose nCells^2 bound the capacity used to be sized with)."""
    for n_cells in (8, 30, 60, 128, 256):
        for n_desired in (n_cells, 3 * n_cells + 1, 1000, 4096):
            totals = list(range(1, n_cells + 1))
            got = retained(n_desired, totals, [True] * n_cells)
            assert got <= n_desired + 2 * n_cells - 1
