"""Library-owned multi-GPU (gs_config.n_shards, csrc/multi.cpp): one context
drives several shard contexts from one calling thread — the single-process
flow a Go controller uses.  Shards may share a device, so a
one-GPU box exercises the whole path (child contexts, per-shard host threads,
merge, host policy replay).

Every sharded result must equal the single-device result bit for bit:
consolidation commands / chosen / multi options (SINGLE, MULTI, EVAL, and the
reruns), the static feasibility matrix (rows, cheapest, offering counts,
OrderByPrice keys, sub-ranges of words), and the Solve (parent device).
"""
import numpy as np
import pytest

from gpusched import abi, synth
from gpusched.consolidation import ConsolidationInput

pytestmark = pytest.mark.gpu

SHARDS = [[0, 0], [0, 0, 0]]


@pytest.fixture(scope="module")
def single():
    from gpusched import lib
    s = lib.Solver()
    yield s
    s.close()


@pytest.fixture(scope="module", params=SHARDS, ids=["2shards", "3shards"])
def sharded(request):
    from gpusched import lib
    s = lib.Solver(shard_devices=request.param)
    yield s
    s.close()


def _cons(kind, seed):
    if kind == "rand":
        return synth.random_consolidation(seed)
    return synth.make_c4(n_nodes=60, n_pending=4, seed=seed, util=(0.9, 0.99), full_frac=0.5, big_frac=1.0, pack=True)


@pytest.mark.parametrize("kind,seed", [("rand", s) for s in range(6)] + [("c4", 0), ("c4", 1)])
@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_sharded_consolidation_equals_single(single, sharded, kind, seed, mode):
    p = _cons(kind, seed)
    cands = list(range(len(p.nodes)))
    want = single.consolidate(ConsolidationInput(p, cands, mode=mode))[:3]
    got = sharded.consolidate(ConsolidationInput(p, cands, mode=mode))[:3]
    assert got == want
    assert sharded.consolidate_rerun()[:3] == want


def test_sharded_eval_sets(single, sharded):
    p = synth.random_consolidation(7, n_nodes=12, n_pending=2)
    sets = [(0, 1), (1, 3), (0, 0), (4, 8), (2, 10)]
    want = single.consolidate(ConsolidationInput(p, list(range(12)), mode=abi.CONSOLIDATE_EVAL, sets=sets))[:3]
    got = sharded.consolidate(ConsolidationInput(p, list(range(12)), mode=abi.CONSOLIDATE_EVAL, sets=sets))[:3]
    assert got == want


def test_sharded_refuses_caller_sharding(sharded):
    from gpusched import lib
    p = synth.random_consolidation(1)
    with pytest.raises(lib.GpuSchedError):
        sharded.consolidate(ConsolidationInput(p, list(range(len(p.nodes))), shard=(0, 2)))


def _feas_equal(a, b):
    for k in ("rows", "cheapest", "n_feasible_offerings", "cheapest_key"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("make", [lambda: synth.make_c2(n_pods=3000), lambda: synth.make_c3(n_pods=2000),
                                  lambda: synth.random_problem(4), lambda: synth.make_c5(n_pods=5000)],
                         ids=["c2", "c3", "random", "c5"])
def test_sharded_feasibility_equals_single(single, sharded, make):
    p = make()
    single.prepare(p)
    want, _ = single.feasibility()
    sharded.prepare(p)
    got, _ = sharded.feasibility()
    _feas_equal(got, want)
    W = want["rows"].shape[2]
    lo, hi = W // 3, max(W // 3 + 1, W - 1)
    want_part, _ = single.feasibility_shard(lo, hi)
    got_part, _ = sharded.feasibility_shard(lo, hi)
    _feas_equal(got_part, want_part)


def test_sharded_solve_runs_on_parent(single, sharded):
    p = synth.random_problem(11)
    assert sharded.solve(p)[0] == single.solve(p)[0]


def _device_result(solver, lo, hi):
    import torch
    from gpusched.feasibility import device_views
    res = solver.feasibility_shard_device(lo, hi)
    rows, nfo, key = (x.clone() for x in device_views(res, torch.device("cuda", 0)))
    S = res.row_stride
    rows = rows.view(-1, S)[:, lo:min(hi, res.words)].cpu()
    return rows, nfo.cpu(), key.cpu(), res


@pytest.mark.parametrize("make", [lambda: synth.make_c3(n_pods=2000), lambda: synth.random_problem(2),
                                  lambda: synth.make_c5(n_pods=5000)], ids=["c3", "random", "c5"])
def test_sharded_device_results_equal_single(single, sharded, make):
    """gs_feasibility_shard_device on a sharded context: the shards' slices
    gathered and their counts / keys reduced ON the parent's device (the
    merge kernel) equal one device's matrix, whole and over a word sub-range"""
    p = make()
    single.prepare(p)
    sharded.prepare(p)
    W = single.feasibility_shard_device(0, 0).words
    for lo, hi in ((0, W), (W // 3, max(W // 3 + 1, W - 1))):
        want = _device_result(single, lo, hi)
        got = _device_result(sharded, lo, hi)
        for a, b in zip(got[:3], want[:3]):
            assert torch_equal(a, b)
        assert got[3].t_merge_ms > 0


def torch_equal(a, b):
    import torch
    return bool(torch.equal(a, b))


def test_rccl_shards():
    """GS_CFG_RCCL: the shards' counts / keys are all-reduced by RCCL before
    the gather.  RCCL refuses a communicator whose ranks repeat a device --
    gs_create then returns GS_E_RCCL; where it accepts them the all-reduced
    matrix must equal one device's"""
    from gpusched import lib
    try:
        s = lib.Solver(shard_devices=[0, 0], flags=abi.GS_CFG_RCCL)
    except lib.GpuSchedError as e:
        assert e.status == abi.GS_E_RCCL
        pytest.skip("RCCL refused the repeated device (GS_E_RCCL): the all-reduce path did not run")
    one = lib.Solver()
    try:
        p = synth.make_c3(n_pods=2000)
        one.prepare(p)
        s.prepare(p)
        W = one.feasibility_shard_device(0, 0).words
        want = _device_result(one, 0, W)
        got = _device_result(s, 0, W)
        for a, b in zip(got[:3], want[:3]):
            assert torch_equal(a, b)
    finally:
        s.close()
        one.close()


def _hip_device_count():
    import ctypes
    n = ctypes.c_int(0)
    ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(n))
    return n.value


@pytest.mark.parametrize("flags", [0, abi.GS_CFG_RCCL], ids=["peer", "rccl"])
@pytest.mark.parametrize("make", [lambda: synth.make_c3(n_pods=2000), lambda: synth.make_c5(n_pods=5000)],
                         ids=["c3", "c5"])
def test_distinct_devices_equal_single(single, make, flags):
    """shards on DISTINCT devices [0, 1], so the merge kernel reads
    the other shard's slice over xGMI peer access (and, with GS_CFG_RCCL, the
    RCCL all-reduce runs between two real ranks); the merged device matrix and
    the consolidation commands equal one device's.  Skipped on a one-GPU box."""
    if _hip_device_count() < 2:
        pytest.skip("one visible device: the peer-read / RCCL path needs two")
    from gpusched import lib
    s = lib.Solver(shard_devices=[0, 1], flags=flags)
    try:
        p = make()
        single.prepare(p)
        s.prepare(p)
        W = single.feasibility_shard_device(0, 0).words
        for lo, hi in ((0, W), (W // 3, max(W // 3 + 1, W - 1))):
            want = _device_result(single, lo, hi)
            got = _device_result(s, lo, hi)
            for a, b in zip(got[:3], want[:3]):
                assert torch_equal(a, b)
        c = synth.make_c4(n_nodes=60, n_pending=4, seed=3, util=(0.9, 0.99), full_frac=0.5, big_frac=1.0, pack=True)
        cands = list(range(len(c.nodes)))
        assert s.consolidate(ConsolidationInput(c, cands))[:3] == single.consolidate(ConsolidationInput(c, cands))[:3]
    finally:
        s.close()
