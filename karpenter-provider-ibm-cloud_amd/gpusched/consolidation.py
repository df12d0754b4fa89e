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


DT_COMMAND = np.dtype([("decision", "<u4"), ("reason", "<u4"), ("n_new_claims", "<u4"), ("n_failed_pods", "<u4"),
                       ("n_candidates", "<u4"), ("nodepool", "<u4"), ("spot_only", "<u4"),
                       ("options", [("begin", "<u4"), ("count", "<u4")]), ("candidate_price", "<f8")], align=True)
assert DT_COMMAND.itemsize == C.sizeof(abi.GsCommand)
REC_BYTES = DT_COMMAND.itemsize + 60 * 4 + 60 * 8  # one simulation's command + options + prices


def result_arrays(res):
    """zero-Python-loop copy of a gs_consolidation_result: (commands [DT_COMMAND], options u32, prices f64)"""
    n = res.n_commands
    if n == 0:
        return np.zeros(0, DT_COMMAND), np.zeros(0, np.uint32), np.zeros(0, np.float64)
    raw = np.ctypeslib.as_array(C.cast(res.commands, C.POINTER(C.c_uint8)), shape=(n * DT_COMMAND.itemsize,))
    cmds = raw.view(DT_COMMAND).copy()
    no = int((cmds["options"]["begin"] + cmds["options"]["count"]).max())
    opts = np.ctypeslib.as_array(res.options, shape=(no,)).copy() if no else np.zeros(0, np.uint32)
    prices = np.ctypeslib.as_array(res.option_prices, shape=(no,)).copy() if no else np.zeros(0, np.float64)
    return cmds, opts, prices


def _pack(cmds, opts, prices, sel):
    c = cmds[sel]
    rec = np.zeros((len(sel), REC_BYTES), np.uint8)
    o = np.zeros((len(sel), 60), np.uint32)
    p = np.zeros((len(sel), 60), np.float64)
    cnt = c["options"]["count"].astype(np.int64)
    if cnt.sum():
        rows = np.repeat(np.arange(len(sel)), cnt)
        cols = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        src = np.repeat(c["options"]["begin"].astype(np.int64), cnt) + cols
        o[rows, cols] = opts[src]
        p[rows, cols] = prices[src]
    rec[:, :DT_COMMAND.itemsize] = c.view(np.uint8).reshape(len(sel), -1)
    rec[:, DT_COMMAND.itemsize:DT_COMMAND.itemsize + 240] = o.view(np.uint8)
    rec[:, DT_COMMAND.itemsize + 240:] = p.view(np.uint8)
    return rec


def _unpack(rec):
    n = len(rec)
    cmds = np.ascontiguousarray(rec[:, :DT_COMMAND.itemsize]).view(DT_COMMAND).reshape(n).copy()
    o = np.ascontiguousarray(rec[:, DT_COMMAND.itemsize:DT_COMMAND.itemsize + 240]).view(np.uint32).reshape(n, 60)
    p = np.ascontiguousarray(rec[:, DT_COMMAND.itemsize + 240:]).view(np.float64).reshape(n, 60)
    cmds["options"]["begin"] = np.arange(n, dtype=np.uint32) * 60
    return cmds, o.reshape(-1).copy(), p.reshape(-1).copy()


def gather_arrays(cmds, opts, prices, rank, world, dist, device=None):
    """all-gather of sharded commands (simulation s is evaluated on rank
    s % world): every rank sends only its own simulations as fixed-size
    records (RCCL over xGMI when `device` is a GPU, gloo on CPU)"""
    n = len(cmds)
    if world <= 1:
        return cmds, opts, prices
    import torch
    n_local = (n + world - 1) // world
    mine = np.arange(rank, n, world)
    rec = np.zeros((n_local, REC_BYTES), np.uint8)
    rec[:len(mine)] = _pack(cmds, opts, prices, mine)
    t = torch.from_numpy(rec)
    if device is not None:
        t = t.to(device)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    allrec = torch.stack(bufs).cpu().numpy()  # [world, n_local, REC]
    s = np.arange(n)
    return _unpack(allrec[s % world, s // world])


def choose_arrays(cin, cmds, opts, prices):
    """gs_consolidation_choose over numpy command arrays -> (chosen, multi_options)"""
    from . import lib
    L = lib.load()
    cmds = np.ascontiguousarray(cmds)
    opts = np.ascontiguousarray(opts, dtype=np.uint32)
    prices = np.ascontiguousarray(prices, dtype=np.float64)
    chosen = C.c_int32(-1)
    mo = (C.c_uint32 * 60)()
    nmo = C.c_uint32(0)
    st = L.gs_consolidation_choose(C.byref(cin.struct), cmds.ctypes.data_as(C.POINTER(abi.GsCommand)), len(cmds),
                                   opts.ctypes.data_as(C.POINTER(C.c_uint32)),
                                   prices.ctypes.data_as(C.POINTER(C.c_double)), C.byref(chosen), mo, C.byref(nmo))
    if st != abi.GS_OK:
        raise lib.GpuSchedError(st, "gs_consolidation_choose failed")
    return int(chosen.value), [int(mo[i]) for i in range(nmo.value)]


def arrays_to_list(cmds, opts, prices):
    out = []
    for c in cmds:
        b, n = int(c["options"]["begin"]), int(c["options"]["count"])
        out.append({"decision": int(c["decision"]), "reason": int(c["reason"]), "n_new_claims": int(c["n_new_claims"]),
                    "n_failed_pods": int(c["n_failed_pods"]), "n_candidates": int(c["n_candidates"]),
                    "nodepool": int(c["nodepool"]) if c["decision"] == abi.DECISION_REPLACE else None,
                    "spot_only": int(c["spot_only"]), "options": [int(x) for x in opts[b:b + n]],
                    "option_prices": [float(x) for x in prices[b:b + n]],
                    "candidate_price": float(c["candidate_price"])})
    return out


def gather_commands(cmds, rank, world, dist, device=None):
    """list-of-dict form of gather_arrays (tests)"""
    if world <= 1:
        return cmds
    rec = pack_commands(cmds)
    n = len(cmds)
    arr = np.zeros(n, DT_COMMAND)
    opts, prices = [], []
    for i, c in enumerate(cmds):
        arr[i] = (c["decision"], c["reason"], c["n_new_claims"], c["n_failed_pods"], c["n_candidates"],
                  c["nodepool"] or 0, c["spot_only"], (len(opts), len(c["options"])), c["candidate_price"])
        opts += c["options"]
        prices += c["option_prices"]
    del rec
    g = gather_arrays(arr, np.asarray(opts, np.uint32), np.asarray(prices, np.float64), rank, world, dist, device)
    return arrays_to_list(*g)
def sharded_consolidation(evaluate, problem, candidates, mode, rank=0, world=1, dist=None, device=None,
                          max_candidates=0):
    """One consolidation pass sharded over `world` ranks: every rank evaluates
    its simulations (evaluate(ConsolidationInput) -> commands, others Skipped),
    the commands are all-gathered and every rank replays the policy with the
    host-only gs_consolidation_choose.  -> (commands, chosen, multi_options)"""
    from . import lib
    shard = (rank, world) if world > 1 else (0, 0)
    cin = ConsolidationInput(problem, candidates, mode=mode, shard=shard, max_candidates=max_candidates)
    cmds = gather_commands(evaluate(cin), rank, world, dist, device)
    full = ConsolidationInput(problem, candidates, mode=mode, max_candidates=max_candidates)
    chosen, multi = lib.choose(full, cmds)
    return cmds, chosen, multi
