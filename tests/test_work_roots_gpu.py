"""The work roots the GPU computes (k_roots, bre_gather.hip; read through bre_device_check kind 5)
against the host restatements of tests/test_work_roots.py: random trees, deep and
unbalanced ones (a caterpillar of 20,000 interior nodes puts far more heavy nodes than the kernel's
4096 cache slots in reach: its overflow path), S from 1 to kMaxSplit.  The roots must be exactly the
parallel form's (the S - 1 largest interior nodes by (leaf tiles, -index), their children outside the
set, ordered by leaf tiles descending and child index), partition the leaves, and equal the greedy
expansion's whenever the size at the cut is not tied."""
import random
import sys

import pytest

from test_work_roots import greedy_roots, parallel_roots, random_tree

pytestmark = pytest.mark.gpu


def caterpillar(n_inner):
    """Node i has leaf ~i and interior child i + 1 (the last one two leaves): depth n_inner."""
    children, nleaf = [], []
    for i in range(n_inner):
        last = i == n_inner - 1
        children.append((~i, ~(i + 1) if last else i + 1))
        nleaf.append(n_inner + 1 - i)
    return children, nleaf


def leaves_under(children, c):
    """leaves_below without recursion (the caterpillar is 20,000 levels deep)."""
    out, stack = set(), [c]
    while stack:
        x = stack.pop()
        if x < 0:
            out.add(~x)
        else:
            stack.extend(children[x])
    return out


def check(g, children, nleaf, S):
    size = lambda c: nleaf[c] if c >= 0 else 1  # noqa: E731
    got = g.work_roots(children, nleaf, S)
    p, _ = parallel_roots(children, nleaf, S)
    assert sorted(got) == sorted(p), S
    # largest first, ties by ascending (signed) child index: k_roots step 4's key (leaf tiles, then
    # 0xffffffff - (index ^ 0x80000000)), larger keys first
    assert got == sorted(got, key=lambda c: (-size(c), c))
    n = nleaf[0]
    cover = [leaves_under(children, r) for r in got]
    assert sum(len(c) for c in cover) == n and set().union(*cover) == set(range(n))
    gr, _ = greedy_roots(children, nleaf, S)
    sizes = sorted(nleaf, reverse=True)
    if S - 1 < len(sizes) and (S - 1 == 0 or sizes[S - 2] != sizes[S - 1]):
        assert set(gr) == set(got), S


@pytest.mark.parametrize("seed", range(6))
def test_gpu_roots_random_trees(bre, seed):
    sys.setrecursionlimit(50000)
    rng = random.Random(100 + seed)
    n = rng.choice([2, 3, 17, 300, 3000])
    children, nleaf = random_tree(n, rng)
    with bre.BeamGather(0) as g:
        for S in (1, 2, 16, 256, 1024):
            check(g, children, nleaf, S)


def test_gpu_roots_deep_unbalanced_tree(bre):
    sys.setrecursionlimit(100000)
    children, nleaf = caterpillar(20_000)
    with bre.BeamGather(0) as g:
        for S in (1, 64, 256, 1024):
            check(g, children, nleaf, S)
