"""Autoplacement ranking: FilterInstanceTypes + rankInstanceTypes
(pkg/providers/common/instancetype/instancetype.go:259-379).

CPU tests pin the oracle: the reference's score KATs
(instancetype_test.go:104-159), the filter semantics (:319-344), and the tie
order against the oracle's Go sort.Slice restatement (test_gosort.py).  GPU
tests compare gs_rank_instance_types with the oracle bit for bit (indices and
float64 scores), ties included.
"""
import ctypes as C

import numpy as np
import pytest

from gpusched import abi
from oracle import pyoracle

GI = 1 << 30


def test_score_kats():
    # instancetype_test.go:104-159 (got != want: exact float64 equality)
    st, order, score = pyoracle.rank_instance_types([4000, 2000, 16000], [16 * GI, 8 * GI, 64 * GI],
                                                    [0.5, 0.0, 2.0], [0, 0, 0])
    assert st == abi.GS_OK
    assert order == [0, 2, 1]
    assert score == [0.0763888888888889, 0.0769927536231884, 11.0]


def test_filters():
    cpu = [2000, 4000, 8000, 16000, 4000]
    mem = [8 * GI, 16 * GI, 32 * GI, 64 * GI, 16 * GI - 1]
    price = [0.1, 0.2, 0.4, 0.8, 0.2]
    arch = [0, 0, 1, 0, 0]
    run = lambda **kw: pyoracle.rank_instance_types(cpu, mem, price, arch, **kw)[1]  # noqa: E731
    assert sorted(run()) == [0, 1, 2, 3, 4]
    assert sorted(run(want_arch=1)) == [2]
    assert sorted(run(min_cpu=4)) == [1, 2, 3, 4]
    # memoryGB = bytes / 2^30 (float64) < MinimumMemory drops the type
    assert sorted(run(min_memory_gb=16)) == [1, 2, 3]
    assert sorted(run(max_price=0.4)) == [0, 1, 2, 4]
    assert sorted(run(max_price=-1.0)) == [0, 1, 2, 3, 4]  # maxPrice > 0 gate (:339)
    assert run(want_arch=1, min_cpu=16) == []


def test_refusals():
    assert pyoracle.rank_instance_types([-1], [GI], [0.1], [0])[0] == abi.GS_E_INVALID
    assert pyoracle.rank_instance_types([1000], [GI], [float('nan')], [0])[0] == abi.GS_E_INVALID
    n = abi.GS_RANK_MAX + 1
    assert pyoracle.rank_instance_types([1000] * n, [GI] * n, [0.1] * n, [0] * n)[0] == abi.GS_E_CAPACITY
    assert pyoracle.rank_instance_types([], [], [], []) == (abi.GS_OK, [], [])


def catalog(seed, n, distinct=8):
    """few distinct shapes and prices -> many exact score ties"""
    rng = np.random.default_rng(seed)
    vcpu = rng.choice([2, 4, 8, 16, 32, 48, 64][:max(1, distinct // 2 + 1)], size=n)
    ratio = rng.choice([2, 4, 8], size=n)
    cpu = (vcpu * 1000).astype(np.int64)
    mem = (vcpu * ratio * GI).astype(np.int64)
    price = np.round(vcpu * ratio * rng.choice([0.01, 0.0125, 0.02], size=n), 4)
    price[rng.random(n) < 0.1] = 0.0  # failed price lookups
    arch = rng.integers(0, 2, size=n).astype(np.uint32)
    return cpu, mem, price, arch


@pytest.mark.parametrize("seed", range(12))
def test_tie_order_is_go_sort_slice(seed):
    """sort.Slice depends only on Less outcomes, so ranking the scores by
    their dense integer rank through oracle_go_sort_ints gives the same
    permutation"""
    n = [0, 1, 12, 13, 49, 50, 51, 200, 1188, 2000, 4096, 777][seed]
    cpu, mem, price, arch = catalog(seed, n)
    st, order, score = pyoracle.rank_instance_types(cpu, mem, price, arch)
    assert st == abi.GS_OK and len(order) == n
    scores = [pyoracle.lib().oracle_instance_score(int(c), int(m), float(p)) for c, m, p in zip(cpu, mem, price)]
    dense = {s: i for i, s in enumerate(sorted(set(scores)))}
    keys = (C.c_int64 * max(1, n))(*[dense[s] for s in scores])
    perm = (C.c_uint32 * max(1, n))()
    pyoracle.lib().oracle_go_sort_ints(keys, perm, n)
    assert order == list(perm)[:n]
    assert score == sorted(scores)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_gpu_rank_parity(seed):
    from gpusched import lib
    n = [0, 1, 12, 13, 49, 50, 51, 200, 1188, 2000, 4096, 777, 256, 257, 1024, 3000][seed]
    cpu, mem, price, arch = catalog(seed, n)
    rng = np.random.default_rng(1000 + seed)
    filters = [dict(), dict(want_arch=int(rng.integers(0, 2))), dict(min_cpu=8), dict(min_memory_gb=64),
               dict(max_price=float(np.median(price)) if n else 1.0),
               dict(want_arch=0, min_cpu=4, min_memory_gb=16, max_price=2.0)]
    for kw in filters:
        st, want_order, want_score = pyoracle.rank_instance_types(cpu, mem, price, arch, **kw)
        assert st == abi.GS_OK
        got_order, got_score = lib.rank_instance_types(cpu, mem, price, arch, **kw)
        assert got_order == want_order, kw
        assert np.array_equal(np.array(got_score).view(np.uint64), np.array(want_score).view(np.uint64)), kw


@pytest.mark.gpu
def test_gpu_rank_kats_and_refusals():
    from gpusched import lib
    order, score = lib.rank_instance_types([4000, 2000, 16000], [16 * GI, 8 * GI, 64 * GI], [0.5, 0.0, 2.0], [0] * 3)
    assert order == [0, 2, 1]
    assert score == [0.0763888888888889, 0.0769927536231884, 11.0]
    with pytest.raises(lib.GpuSchedError):
        lib.rank_instance_types([-1], [GI], [0.1], [0])
    with pytest.raises(lib.GpuSchedError):
        lib.rank_instance_types([1000], [GI], [float('nan')], [0])
    n = abi.GS_RANK_MAX + 1
    with pytest.raises(lib.GpuSchedError):
        lib.rank_instance_types([1000] * n, [GI] * n, [0.1] * n, [0] * n)


def _kats():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")) as f:
        return json.load(f)


RANK_ORDER_CASES = _kats()["rank_orders"]["cases"]


def _check_rank_order(case, order):
    names = [t[0] for t in case["types"]]
    got = [names[i] for i in order]
    if "want" in case:
        assert got == case["want"], case["name"]
    if "want_first" in case:
        assert got[0] == case["want_first"], case["name"]
    if "want_set" in case:
        assert sorted(got) == sorted(case["want_set"]), case["name"]


def _rank_cols(case):
    t = case["types"]
    return [x[1] for x in t], [x[2] for x in t], [x[3] for x in t], [0] * len(t)


@pytest.mark.parametrize("case", RANK_ORDER_CASES, ids=[c["name"] for c in RANK_ORDER_CASES])
def test_rank_order_kats(case):
    """rankInstanceTypes orders (instancetype_mock_test.go:221-361) through the oracle"""
    st, order, _ = pyoracle.rank_instance_types(*_rank_cols(case))
    assert st == abi.GS_OK
    _check_rank_order(case, order)


def test_score_zero_resources_kat():
    k = _kats()["score_zero_resources"]  # instancetype_mock_test.go:372-383
    assert pyoracle.lib().oracle_instance_score(k["cpu_milli"], k["memory_bytes"], k["price"]) == k["want"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", RANK_ORDER_CASES, ids=[c["name"] for c in RANK_ORDER_CASES])
def test_gpu_rank_order_kats(case):
    from gpusched import lib
    order, score = lib.rank_instance_types(*_rank_cols(case))
    _check_rank_order(case, order)
    assert order == pyoracle.rank_instance_types(*_rank_cols(case))[1]


@pytest.mark.gpu
def test_gpu_rank_zero_resources_kat():
    from gpusched import lib
    _, score = lib.rank_instance_types([0], [0], [0.0], [0])
    assert score == [_kats()["score_zero_resources"]["want"]]


@pytest.mark.gpu
def test_gpu_rank_runs_on_current_device():
    """gs_rank_instance_types keeps one buffer per device and launches on the
    calling thread's current device (rank.hip per-device buffers);
    a gs_create on the last visible device makes it current."""
    import torch
    from gpusched import lib
    n = torch.cuda.device_count()
    cpu, mem, price, arch = catalog(3, 300)
    want = pyoracle.rank_instance_types(cpu, mem, price, arch)[1]
    for dev in sorted({0, n - 1}):
        s = lib.Solver(device=dev)
        assert lib.rank_instance_types(cpu, mem, price, arch)[0] == want
        s.close()
    assert lib.rank_instance_types(cpu, mem, price, arch)[0] == want
