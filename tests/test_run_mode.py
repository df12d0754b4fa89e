"""Run mode of the single-wave Solve (round 5).

Runs of identical simple pods are placed from a register window of the
sorted NodeClaims: the pending one-claim rotation, the scan from the
infeasible-prefix bound, the fast accept, the exact CanAdd of the window's
candidates, a window rebase when a run of equal keys leaves the window and a
touched choosePivot sample sorted in place.  Run mode needs >= 50 in-flight
NodeClaims, so the random suites (small problems) never reach it; these
problems do: CM- and C2-distributed batches of 2,500-8,000 pods (queue order
interleaves pods with node selectors and GPU requests among each spec's
simple pods) and CM pods onto 150 state nodes, compared bit for bit with the
oracle (the first-fit CanAdd counters too), with the kernel's own counters
showing each run-mode path was taken.
"""
import ctypes as C

import pytest

from gpusched import abi, synth
from oracle import pyoracle

CASES = [("cm", 2500 + 700 * k, 0x5EED0100 + k) for k in range(8)] + \
        [("c2", 3000 + 900 * k, 0x5EED0200 + k) for k in range(6)] + \
        [("c4", 4000 + 1000 * k, 0x5EED0300 + k) for k in range(4)]


def _problem(kind, n, seed):
    if kind == "cm":
        return synth.make_cm(n_pods=n, seed=seed)
    if kind == "c4":
        # CM-distributed pods onto 150 state nodes first (runs start once
        # the nodes are full for a spec: the node hint covers every node)
        return synth.make_c4(n_nodes=150, n_pending=n, seed=seed)
    return synth.make_c2(n_pods=n, seed=seed)


@pytest.fixture(scope="module")
def wave():
    from gpusched.lib import Solver
    s = Solver(0, 0)
    yield s
    s.close()


def _run_counters(s):
    out = (C.c_uint64 * 16)()
    s.L.gs_debug_ctrl.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
    s.L.gs_debug_ctrl(s.ctx, out, 16)
    # dbg[8..13]: pods placed in runs, entries, exits (pivot, window, spec,
    # scan); dbg[14]: exact batches in runs (ffd_wave.hpp)
    return {"pods": out[8], "entries": out[9], "pivot": out[10], "window": out[11], "spec": out[12],
            "scan": out[13], "exact": out[14]}


_SEEN = []


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(CASES)), ids=[f"{c[0]}-{c[1]}" for c in CASES])
def test_gpu_run_mode_parity(wave, k):
    from test_gpu_parity import _diff
    kind, n, seed = CASES[k]
    p = _problem(kind, n, seed)
    st, want, raw = pyoracle.solve(p)
    assert st == abi.GS_OK
    wave.prepare(p)
    wave.run()
    got, res = wave.fetch()
    d = _diff(got, want)
    assert d is None, d
    # the first-fit NodeClaim.CanAdd / ExistingNode.CanAdd call counts
    assert (int(res.claim_prefix), int(res.node_prefix)) == (int(raw.claim_prefix), int(raw.node_prefix))
    ctr = _run_counters(wave)
    _SEEN.append(ctr)
    if len(want["claims"]) >= 60:
        assert ctr["pods"] > 0, ctr  # the run mode engaged


@pytest.mark.gpu
def test_gpu_run_mode_paths_taken():
    """across the cases above: runs, their exact batches and window rebases"""
    if len(_SEEN) < len(CASES):
        pytest.skip("needs the parity cases of this module first")
    tot = {key: sum(c[key] for c in _SEEN) for key in _SEEN[0]}
    assert tot["pods"] > 1000 and tot["exact"] > 0 and tot["window"] > 0, tot
    assert sum(c["pods"] for c in _SEEN[-4:]) > 0  # with existing nodes too


@pytest.mark.gpu
@pytest.mark.parametrize("nodes,pods", [(1000, 20000), (2500, 30000)])
def test_gpu_run_mode_state_nodes_midsize(wave, nodes, pods):
    """CM-distributed pods onto 1,000 / 2,500 C4-style state nodes: the nodes
    fill first, then the runs take over behind the node hint (the bench's
    CM_C4 shape at a size the oracle finishes in seconds)"""
    from test_gpu_parity import _diff
    p = synth.make_c4(n_nodes=nodes, n_pending=pods, seed=0x5EED0400 + nodes)
    st, want, raw = pyoracle.solve(p)
    assert st == abi.GS_OK
    wave.prepare(p)
    wave.run()
    got, res = wave.fetch()
    d = _diff(got, want)
    assert d is None, d
    assert (int(res.claim_prefix), int(res.node_prefix)) == (int(raw.claim_prefix), int(raw.node_prefix))
    assert _run_counters(wave)["pods"] > 0

