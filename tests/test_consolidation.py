"""Consolidation: the HIP simulations through the
C-ABI against the oracle's naive SimulateScheduling + computeConsolidation.

CPU tests pin the host-only policy replay (gs_consolidation_choose) against
the oracle's own SINGLE / MULTI choices; GPU tests require every per-
simulation command (decision, reason, NodeClaim count, failed pods,
replacement NodePool and options with prices) and the chosen command to be
identical.  Consolidation semantics are <U> (karpenter v1.13.0, not in the
container): parity unpinned against the reference itself.
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.consolidation import ConsolidationInput, n_multi_sims, pack_commands, unpack_commands
from oracle import pyoracle


def _cases():
    out = []
    for s in range(12):
        out.append(("rand", s))
    out.append(("c4", 0))
    return out


def _problem(kind, seed):
    if kind == "rand":
        return synth.random_consolidation(seed)
    return synth.make_c4(n_nodes=40, n_pending=3, seed=seed, util=(0.85, 0.99), full_frac=0.6, big_frac=0.6)


@pytest.mark.parametrize("kind,seed", _cases())
@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_host_policy_replay_matches_oracle(kind, seed, mode):
    p = _problem(kind, seed)
    cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=mode)
    st, cmds, chosen, multi = pyoracle.consolidate(cin)
    assert st == abi.GS_OK
    if mode == abi.CONSOLIDATE_MULTI:
        assert len(cmds) == n_multi_sims(len(p.nodes))
    got, got_multi = lib.choose(cin, cmds)
    assert (got, got_multi) == (chosen, multi)


def test_pack_roundtrip():
    p = _problem("c4", 0)
    cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=abi.CONSOLIDATE_SINGLE)
    _, cmds, _, _ = pyoracle.consolidate(cin)
    assert unpack_commands(pack_commands(cmds)) == cmds


def test_oracle_decisions_cover_every_outcome():
    seen = set()
    for s in range(12):
        p = _problem("rand", s)
        _, cmds, _, _ = pyoracle.consolidate(ConsolidationInput(p, list(range(len(p.nodes)))))
        seen |= {(c["decision"], c["reason"]) for c in cmds}
    p = _problem("c4", 0)
    _, cmds, _, _ = pyoracle.consolidate(ConsolidationInput(p, list(range(len(p.nodes)))))
    seen |= {(c["decision"], c["reason"]) for c in cmds}
    assert (abi.DECISION_DELETE, 0) in seen and (abi.DECISION_REPLACE, 0) in seen
    assert (abi.DECISION_NOOP, abi.NOOP_UNSCHEDULABLE) in seen


# ------------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def solver():
    from gpusched.lib import Solver
    s = Solver(0)
    yield s
    s.close()


def check(solver, p, mode, cands=None, sets=None, shard=(0, 0)):
    cands = list(range(len(p.nodes))) if cands is None else cands
    cin = ConsolidationInput(p, cands, mode=mode, sets=sets)
    st, want, want_chosen, want_multi = pyoracle.consolidate(cin)
    assert st == abi.GS_OK
    gin = ConsolidationInput(p, cands, mode=mode, sets=sets, shard=shard)
    got, chosen, multi, _ = solver.consolidate(gin)
    for i, (g, w) in enumerate(zip(got, want)):
        if shard[1] and i % shard[1] != shard[0]:
            assert g["decision"] == abi.DECISION_SKIPPED
            continue
        assert g == w, (i, g, w)
    assert len(got) == len(want)
    if not shard[1]:
        assert (chosen, multi) == (want_chosen, want_multi)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("kind,seed", _cases())
@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_gpu_consolidation_matches_oracle(solver, kind, seed, mode):
    check(solver, _problem(kind, seed), mode)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20, 40))
def test_gpu_consolidation_random_single(solver, seed):
    check(solver, synth.random_consolidation(seed, n_nodes=24, n_pending=int(seed % 3)), abi.CONSOLIDATE_SINGLE)


@pytest.mark.gpu
def test_gpu_consolidation_eval_sets(solver):
    p = synth.random_consolidation(7, n_nodes=12, n_pending=2)
    sets = [(0, 1), (1, 3), (0, 0), (4, 8), (2, 10)]
    check(solver, p, abi.CONSOLIDATE_EVAL, cands=list(range(12)), sets=sets)


@pytest.mark.gpu
def test_gpu_consolidation_sharded_union_equals_whole(solver):
    p = _problem("c4", 1)
    parts = [check(solver, p, abi.CONSOLIDATE_SINGLE, shard=(r, 3)) for r in range(3)]
    whole = check(solver, p, abi.CONSOLIDATE_SINGLE)
    merged = [parts[i % 3][i] for i in range(len(whole))]
    assert merged == whole
    cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=abi.CONSOLIDATE_SINGLE)
    want_chosen = pyoracle.consolidate(cin)[2]
    assert lib.choose(cin, merged)[0] == want_chosen


@pytest.mark.gpu
def test_gpu_consolidation_rerun_identical(solver):
    p = _problem("c4", 2)
    cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=abi.CONSOLIDATE_SINGLE)
    a = solver.consolidate(cin)[:3]
    b = solver.consolidate_rerun()[:3]
    assert a == b


@pytest.mark.gpu
def test_gpu_consolidation_c4_scale_invariants(solver):
    # full C4 scale: no oracle (minutes on CPU); size-independent checks
    p = synth.make_c4(n_nodes=5000, n_pending=0)
    cin = ConsolidationInput(p, list(range(5000)), mode=abi.CONSOLIDATE_SINGLE)
    cmds, chosen, _, res = solver.consolidate(cin)
    assert len(cmds) == 5000
    assert all(c["decision"] in (0, 1, 2) for c in cmds)
    first = next((i for i, c in enumerate(cmds) if c["decision"] != abi.DECISION_NOOP), -1)
    assert chosen == first
    for c in cmds:
        if c["decision"] == abi.DECISION_REPLACE:
            assert c["n_new_claims"] == 1 and c["options"]
            assert all(x < c["candidate_price"] for x in c["option_prices"])
            assert c["option_prices"] == sorted(c["option_prices"])
        if c["decision"] == abi.DECISION_DELETE:
            assert c["n_new_claims"] == 0 and c["n_failed_pods"] == 0
    # a sampled subset against the oracle
    sub = list(range(0, 5000, 250))
    st, want, _, _ = pyoracle.consolidate(ConsolidationInput(p, sub, mode=abi.CONSOLIDATE_SINGLE))
    assert st == abi.GS_OK
    assert [cmds[i] for i in sub] == want


@pytest.mark.gpu
def test_gpu_consolidation_narrow_equals_wide(solver):
    """5,000 simulations run in the 128-thread shape; each of 5 shards holds
    1,000 (< 4 per CU) and runs the 256-thread shape (ffd.hip FB_SIM_NARROW,
    consolidate.cpp plan_sims).  Mixed Delete / Replace / NoOp (bench c4_mixed)."""
    p = synth.make_c4(n_nodes=5000, n_pending=0, util=(0.9, 0.99), full_frac=0.5, big_frac=1.0, pack=True)
    cands = list(range(5000))
    cin = ConsolidationInput(p, cands, mode=abi.CONSOLIDATE_SINGLE)
    whole, chosen, _, _ = solver.consolidate(cin)
    assert {c["decision"] for c in whole} == {abi.DECISION_DELETE, abi.DECISION_REPLACE, abi.DECISION_NOOP}
    for r in range(5):
        part = solver.consolidate(ConsolidationInput(p, cands, mode=abi.CONSOLIDATE_SINGLE, shard=(r, 5)))[0]
        for i in range(r, 5000, 5):
            assert part[i] == whole[i], i
    sub = list(range(3, 5000, 500))
    st, want, _, _ = pyoracle.consolidate(ConsolidationInput(p, sub, mode=abi.CONSOLIDATE_SINGLE))
    assert st == abi.GS_OK
    assert [whole[i] for i in sub] == want


@pytest.mark.gpu
def test_gpu_consolidation_rerun_after_input_overwritten(solver):
    """gs_consolidate copies what the reruns need (no borrowed
    cluster / candidate pointers survive the call): scribbling over every
    caller array afterwards leaves the rerun's commands unchanged"""
    import numpy as np
    p = _problem("c4", 3)
    cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=abi.CONSOLIDATE_SINGLE)
    a = solver.consolidate(cin)[:3]
    rng = np.random.default_rng(0)
    for arr in (p.quantities, p.reqs, p.labels, p.offerings, p.instance_types, p.nodes, p.pods, p.bound_pods,
                p.value_ids, p.bound_node, cin.candidates):
        if len(arr):
            raw = arr.view(np.uint8)
            raw[:] = rng.integers(0, 256, size=raw.shape, dtype=np.uint8)
    b = solver.consolidate_rerun()[:3]
    assert a == b
