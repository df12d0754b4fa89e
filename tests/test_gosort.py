"""Properties of the oracle's Go sort.Slice (pdqsort_func) restatement."""
import ctypes as C

import numpy as np
import pytest

from oracle import pyoracle


def go_sort(keys):
    n = len(keys)
    k = (C.c_int64 * max(1, n))(*keys)
    p = (C.c_uint32 * max(1, n))()
    pyoracle.lib().oracle_go_sort_ints(k, p, n)
    return list(k)[:n], list(p)[:n]


@pytest.mark.parametrize("seed", range(40))
def test_sorted_permutation(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 400))
    keys = [int(x) for x in rng.integers(0, max(1, n // 4 + 1), size=n)]
    out, perm = go_sort(keys)
    assert out == sorted(keys)
    assert sorted(perm) == list(range(n))
    assert [keys[i] for i in perm] == out


@pytest.mark.parametrize("n", range(0, 13))
def test_small_is_insertion_sort_stable(n):
    rng = np.random.default_rng(n)
    keys = [int(x) for x in rng.integers(0, 3, size=n)]
    _, perm = go_sort(keys)
    assert perm == sorted(range(n), key=lambda i: (keys[i], i))


def test_large_ties_are_not_stable():
    """pdqsort is unstable beyond 12 elements: the order of ties is a property of
    the algorithm that the product must reproduce exactly"""
    keys = [1, 0] * 40
    _, perm = go_sort(keys)
    zeros = [i for i in perm if keys[i] == 0]
    assert zeros != sorted(zeros)
