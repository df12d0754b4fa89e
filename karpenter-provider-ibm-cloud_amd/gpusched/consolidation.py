"""Host-side mirror of karpenter's disruption consolidation entry points over
the C-ABI (gs_consolidate / gs_consolidation_choose in include/gpusched.h).

<U> sigs.k8s.io/karpenter@v1.13.0 pkg/controllers/disruption:
  SingleNodeConsolidation.ComputeCommand  -> mode SINGLE (first non-NoOp)
  MultiNodeConsolidation.firstNConsolidationOption -> mode MULTI (binary search)
  computeConsolidation(candidates...)     -> mode EVAL, one command per set
The reference provider reaches these through karpenter-core's disruption
controller (reference cmd/controller/main.go:76-86); each simulation is an
independent SimulateScheduling Solve, sharded across GPUs by `shard`.
"""
import ctypes as C

import numpy as np

from . import abi


class ConsolidationInput:
    """Owns the arrays behind one gs_consolidation struct."""

    def __init__(self, problem, candidates, mode=abi.CONSOLIDATE_SINGLE, sets=None, max_candidates=0,
                 shard=(0, 0)):
        self.problem = problem
        self.candidates = np.asarray(candidates, dtype=np.uint32)
        sets = sets or []
        self.sets = np.zeros(len(sets), dtype=[("begin", "<u4"), ("count", "<u4")])
        for i, (b, c) in enumerate(sets):
            self.sets[i] = (b, c)
        self.struct = abi.GsConsolidation()
        st = self.struct
        st.cluster = C.pointer(problem.struct)
        bp, bn = problem.bound_pods, problem.bound_node
        st.bound_pods = bp.ctypes.data if len(bp) else None
        st.n_bound_pods = len(bp)
        st.bound_pod_node = bn.ctypes.data if len(bn) else None
        st.candidates = self.candidates.ctypes.data if len(self.candidates) else None
        st.n_candidates = len(self.candidates)
        st.sets = self.sets.ctypes.data if len(self.sets) else None
        st.n_sets = len(self.sets)
        st.mode = int(mode)
        st.max_candidates = int(max_candidates)
        st.shard_index, st.shard_count = int(shard[0]), int(shard[1])


def n_multi_sims(n_candidates, max_candidates=100):
    """number of prefix simulations MULTI evaluates (firstNConsolidationOption's mids)"""
    mx = min(n_candidates, max_candidates or 100)
    if n_candidates < 2:
        return 0
    if n_candidates <= mx:
        mx = n_candidates - 1
    return mx


def pack_commands(cmds):
    """fixed-size records (for an all-gather across ranks): [n, 9 + 2*60] float64"""
    rec = np.zeros((len(cmds), 9 + 120), dtype=np.float64)
    for i, c in enumerate(cmds):
        rec[i, :8] = [c["decision"], c["reason"], c["n_new_claims"], c["n_failed_pods"], c["n_candidates"],
                      -1 if c["nodepool"] is None else c["nodepool"], c["spot_only"], c["candidate_price"]]
        n = len(c["options"])
        rec[i, 8] = n
        rec[i, 9:9 + n] = c["options"]
        rec[i, 69:69 + n] = c["option_prices"]
    return rec


def unpack_commands(rec):
    out = []
    for r in rec:
        n = int(r[8])
        out.append({"decision": int(r[0]), "reason": int(r[1]), "n_new_claims": int(r[2]),
                    "n_failed_pods": int(r[3]), "n_candidates": int(r[4]),
                    "nodepool": None if r[5] < 0 else int(r[5]), "spot_only": int(r[6]),
                    "candidate_price": float(r[7]), "options": [int(x) for x in r[9:9 + n]],
                    "option_prices": [float(x) for x in r[69:69 + n]]})
    return out
