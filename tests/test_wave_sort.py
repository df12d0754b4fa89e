"""The single-wave sort.Slice restatement (WaveSort in ffd_wave.hpp: the
Solve's per-pod `sort.Slice(newNodeClaims, len(Pods) asc)`) against the
oracle's restatement of Go's pdqsort (oracle/gosort.h), permutation for
permutation, on the inputs the Solve hands it: a sorted array with one key
raised by one (anywhere, and on choosePivot's samples), arrays of two or three
key values, the e2e shape (a long run of low counts, then the raised claim and
the active runs), and random keys.  Ties decide which NodeClaim a pod lands
on, so the permutation -- not just the sorted keys -- must match."""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

from oracle import pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))
HEAP_INPUTS = json.load(open(os.path.join(HERE, "golden", "heapsort_inputs.json")))


def go_perm(keys):
    n = len(keys)
    k = (C.c_int64 * max(1, n))(*keys)
    p = (C.c_uint32 * max(1, n))()
    pyoracle.lib().oracle_go_sort_ints(k, p, n)
    return list(p)[:n]


def wave_perm(keys):
    from gpusched import lib
    L = lib.load()
    n = len(keys)
    f = L.gs_debug_go_sort
    f.argtypes = [C.POINTER(C.c_uint16), C.c_uint32, C.POINTER(C.c_uint32)]
    f.restype = C.c_int
    k = (C.c_uint16 * max(1, n))(*keys)
    p = (C.c_uint32 * max(1, n))()
    assert f(k, n, p) == 0
    return list(p)[:n]


def wave_perm_known(keys, x):
    from gpusched import lib
    L = lib.load()
    n = len(keys)
    f = L.gs_debug_go_sort_known
    f.argtypes = [C.POINTER(C.c_uint16), C.c_uint32, C.c_int32, C.POINTER(C.c_uint32)]
    f.restype = C.c_int
    k = (C.c_uint16 * max(1, n))(*keys)
    p = (C.c_uint32 * max(1, n))()
    assert f(k, n, x, p) == 0
    return list(p)[:n]


def check(keys, x=None):
    """x: the one position out of order (the Solve's one-change sorts: in a
    GS_KNOWN_PARTITION=1 build the first partition then searches the
    boundary, WaveSort::partition_known; the default build ignores x)"""
    keys = [int(v) for v in keys]
    want = go_perm(keys)
    assert wave_perm(keys) == want, keys if len(keys) < 80 else len(keys)
    if x is not None:
        assert wave_perm_known(keys, x) == want, (x, keys if len(keys) < 80 else len(keys))


def raised(runs, pos):
    """the sorted array given as (key, length) runs, with the key at `pos` raised by one"""
    a = [k for k, n in runs for _ in range(n)]
    a[pos] += 1
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("n", [13, 20, 49, 50, 51, 64, 100, 200, 333])
def test_one_raised_key_every_position(n):
    rng = np.random.default_rng(n)
    for pos in range(n):
        runs = [(3, int(rng.integers(1, n))), (4, n)]
        a = raised(runs, pos)[:n]
        check(a, pos)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [100, 250, 1000, 1999, 4096])
def test_raised_on_pivot_samples(n):
    q = n // 4
    for s in (q, 2 * q, 3 * q):
        for d in (-2, -1, 0, 1):
            for lo in (0, n // 8, n // 2, n - 3):
                runs = [(16, lo), (17, n - lo)]
                x = max(0, min(n - 1, s + d))
                check(raised(runs, x), x)


@pytest.mark.parametrize("low,mid,m", [(500, 1, 19), (500, 1, 2), (500, 1, 100), (250, 1, 40), (10, 1, 5),
                                       (700, 1, 150)])
@pytest.mark.gpu
def test_e2e_shape(low, mid, m):
    """a run of idle claims at a low count, then the raised claim and the
    active runs (tests/golden e2e Solve: 12,494 of 30k sorts look like this)"""
    n = 1000
    a = [16] * low + [18] * mid + [17] * m + [18] * (n - low - mid - m)
    check(a[:n], low if mid == 1 else None)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(60))
def test_random_few_values(seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(0, 3000))
    vals = int(rng.integers(1, 5))
    check(rng.integers(0, vals, size=n))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_random_sorted_runs_with_swaps(seed):
    rng = np.random.default_rng(200 + seed)
    n = int(rng.integers(13, 4096))
    a = np.sort(rng.integers(0, int(rng.integers(1, 40)), size=n))
    for _ in range(int(rng.integers(0, 4))):
        i, j = rng.integers(0, n, size=2)
        a[i], a[j] = a[j], a[i]
    check(a)


@pytest.mark.gpu
@pytest.mark.parametrize("n", range(0, 65))
def test_register_frames_every_size(n):
    """arrays of <= 64 NodeClaims sort in registers (RegSort, ffd_wave.hpp):
    every length, keys from two values to distinct, sorted-with-swaps and
    reversed inputs (choosePivot's decreasing hint), permutation for permutation"""
    rng = np.random.default_rng(400 + n)
    for vals in (2, 3, 8, 1000):
        check(rng.integers(0, vals, size=n))
    a = np.sort(rng.integers(0, 6, size=n))
    for _ in range(2):
        if n:
            i, j = rng.integers(0, n, size=2)
            a[i], a[j] = a[j], a[i]
    check(a)
    check(np.sort(rng.integers(0, 50, size=n))[::-1])
    check(list(range(n)))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_random_keys(seed):
    rng = np.random.default_rng(300 + seed)
    n = int(rng.integers(0, 4096))
    check(rng.integers(0, 65535, size=n))


def test_heapsort_inputs_reach_heapsort_on_the_oracle():
    """CPU: the committed inputs do reach Go's heapSort fallback (the Python
    restatement in make_heapsort_inputs.py counts it), and the oracle's
    permutation of them equals that restatement's"""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_heapsort_inputs as M
    assert set(HEAP_INPUTS) == {"30", "45", "64", "100"}
    for keys in HEAP_INPUTS.values():
        class K:  # sort (key, index) pairs by key only, as sort.Slice's Less
            __slots__ = ("k", "i")

            def __init__(self, k, i):
                self.k, self.i = k, i

            def __lt__(self, o):
                return self.k < o.k
        d = [K(k, i) for i, k in enumerate(keys)]
        heap, _ = M.go_pdqsort(d)
        assert heap >= 1
        assert [x.i for x in d] == go_perm(keys)


@pytest.mark.gpu
@pytest.mark.parametrize("n", ["30", "45", "64", "100"])
def test_heapsort_inputs(n):
    """the heapSort fallback: in registers' frame (<= 64: RegSort stores the
    frame and runs lane 0's heapSort) and on the wave path (100)"""
    check(HEAP_INPUTS[n])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_one_change_random_runs(seed):
    """the Solve's one-change inputs over many runs of pod counts: one count
    raised by one (MOD_INC) anywhere, or a NodeClaim appended with any count
    (MOD_APPEND), through the boundary-search first partition"""
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(65, 2500))
    a = np.sort(rng.integers(0, int(rng.integers(2, 60)), size=n))
    for _ in range(6):
        x = int(rng.integers(0, n))
        b = a.copy()
        b[x] += 1
        check(b, x)
    for _ in range(3):
        b = a.copy()
        b[n - 1] = int(rng.integers(0, int(a.max()) + 2))
        check(b, n - 1)


@pytest.mark.parametrize("seed", range(12))
def test_oracle_gosort_matches_python_restatement(seed):
    """CPU: the oracle's pdqsort_func restatement (oracle/gosort.h, the
    checker of every wave-sort test above) against the independent Python
    restatement in tests/golden/make_heapsort_inputs.py, permutation for
    permutation, on random keys with many ties and on one-change orders"""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_heapsort_inputs as M
    rng = np.random.default_rng(900 + seed)

    class K:
        __slots__ = ("k", "i")

        def __init__(self, k, i):
            self.k, self.i = k, i

        def __lt__(self, o):
            return self.k < o.k
    for _ in range(10):
        n = int(rng.integers(0, 400))
        keys = [int(v) for v in rng.integers(0, int(rng.integers(1, 50)), size=n)]
        if rng.random() < 0.5 and n:
            keys = sorted(keys)
            keys[int(rng.integers(0, n))] += 1
        d = [K(k, i) for i, k in enumerate(keys)]
        M.go_pdqsort(d)
        assert [x.i for x in d] == go_perm(keys)
