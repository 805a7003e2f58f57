"""The work-root selection (bre_gather.hip k_roots), restated on the host.

Round 4 chose the S work roots by a serial greedy expansion: starting from the root, replace the
frontier's largest interior node (leaf tiles below it; ties: the lowest frontier position) by its
children while the frontier stays within S entries.  Round 5 computes the result in parallel: every
expanded node is larger than its children, so the expansions come in decreasing order of size and
the expanded set is the S - 1 largest interior nodes (ties by node index), the roots being their
children outside the set.  These tests check that claim on random binary trees: both forms partition
the leaves into the same number of roots, expand interior nodes of the same sizes, and expand the same
nodes (so give the same roots) whenever the size at the cut is not tied.  (CPU only: the GPU kernel's roots are checked end to end by
tests/test_split_gpu.py, which gathers with S = 1 / 64 / 256 / 1024 and compares the counts.)"""
import random
import sys

import pytest


def random_tree(n_leaves, rng):
    """A random full binary tree over n_leaves leaf tiles: nodes as (left, right) with children either
    node indices (>= 0) or leaves (~k); returns (children, nleaf) with node 0 the root."""
    children, nleaf = [], []

    def build(lo, hi):
        idx = len(children)
        children.append(None)
        nleaf.append(hi - lo)
        mid = rng.randint(lo + 1, hi - 1)
        kids = []
        for a, b in ((lo, mid), (mid, hi)):
            kids.append(~a if b - a == 1 else build(a, b))
        children[idx] = tuple(kids)
        return idx

    build(0, n_leaves)
    return children, nleaf


def greedy_roots(children, nleaf, S):
    """Round 4's serial expansion (k_roots before round 5); returns (roots, expanded nodes)."""
    size = lambda c: nleaf[c] if c >= 0 else 1  # noqa: E731
    cur, expanded = [0], []
    while True:
        best = None
        for p, c in enumerate(cur):
            if c >= 0 and (best is None or size(c) > size(cur[best])):
                best = p
        if best is None or len(cur) + 1 > S:
            return cur, expanded
        expanded.append(cur[best])
        c0, c1 = children[cur[best]]
        cur[best] = c0
        cur.append(c1)


def parallel_roots(children, nleaf, S):
    """Round 5's form: E = the S - 1 largest interior nodes by (leaf tiles, -index); roots = E's
    children outside E (the root itself when S = 1); returns (roots, E)."""
    interior = sorted(range(len(children)), key=lambda x: (-nleaf[x], x))
    E = set(interior[:S - 1])
    if not E:
        return [0], E
    return [c for e in E for c in children[e] if not (c >= 0 and c in E)], E


def leaves_below(children, c):
    if c < 0:
        return {~c}
    out = set()
    for k in children[c]:
        out |= leaves_below(children, k)
    return out


@pytest.mark.parametrize("seed", range(12))
def test_parallel_selection_matches_the_greedy(seed):
    sys.setrecursionlimit(20000)
    rng = random.Random(seed)
    n = rng.choice([2, 3, 17, 200, 1500])
    children, nleaf = random_tree(n, rng)
    for S in (1, 2, 4, 16, 64, 256):
        (g, ge), (p, pe) = greedy_roots(children, nleaf, S), parallel_roots(children, nleaf, S)
        # both partition the leaves into the same number (<= S) of roots
        assert len(g) == len(p) == min(S, n)
        for roots in (g, p):
            cover = [leaves_below(children, r) for r in roots]
            assert sum(len(c) for c in cover) == n and set().union(*cover) == set(range(n))
        # the greedy expands the S - 1 largest interior nodes: the same sizes as E ...
        assert sorted(nleaf[x] for x in ge) == sorted(nleaf[x] for x in pe), S
        # ... and the same nodes whenever the size at the cut is not tied
        sizes = sorted(nleaf, reverse=True)
        if S - 1 < len(sizes) and (S - 1 == 0 or sizes[S - 2] != sizes[S - 1]):
            assert set(ge) == set(pe) and set(g) == set(p), S
