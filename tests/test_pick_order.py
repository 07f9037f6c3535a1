"""The batch picks of the 19x19 shared expansions (mzgo_search.hpp: pick_all)
decode all of a batch's choices at once instead of one after another.

Simulation sim0 + i takes the r_i-th (ascending) of the still-unexpanded
eligible children -- select_leaf's random.choice over them
(self_play.py:283-287) -- so pick i depends on every earlier pick.  pick_all
lifts the ranks backwards (q_j += q_j >= r_i for j > i, i = count-2 .. 0) and
maps ranks to actions through a rank table.  This checks that restatement of
the device algorithm against the sequential definition, on random masks and
on the edge cases (one pick, every element picked, more than 64 picks, a
single element).
"""
import numpy as np
import pytest


def sequential_picks(actions, ranks):
    remaining = sorted(actions)
    out = []
    for r in ranks:
        out.append(remaining.pop(r))
    return out


def lifted_picks(actions, ranks):
    table = sorted(actions)
    q = list(ranks)
    for i in range(len(ranks) - 2, -1, -1):     # the device's reverse steps
        s = ranks[i]
        for j in range(i + 1, len(ranks)):
            q[j] += 1 if q[j] >= s else 0
    return [table[p] for p in q]


@pytest.mark.parametrize("A", [26, 82, 362])
def test_lift_matches_sequential(A):
    rng = np.random.default_rng(A)
    for _ in range(200):
        n = int(rng.integers(1, A + 1))
        actions = sorted(rng.choice(A, size=n, replace=False).tolist())
        count = int(rng.integers(1, n + 1))
        ranks = [int(rng.integers(0, n - i)) for i in range(count)]
        assert lifted_picks(actions, ranks) == sequential_picks(actions, ranks)


def test_lift_edge_cases():
    acts = list(range(0, 362, 3))
    n = len(acts)
    # every element, always the last one / always the first one
    assert lifted_picks(acts, [n - 1 - i for i in range(n)]) == acts[::-1]
    assert lifted_picks(acts, [0] * n) == acts
    # one pick, one element
    assert lifted_picks([7], [0]) == [7]
    assert lifted_picks(acts, [5]) == [acts[5]]
