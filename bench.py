#!/usr/bin/env python3
"""bench.py — BASELINE.json metric on MI355X:
pod x offering feasibility checks/sec + Solve latency (ms), 100k pods.

Headline (`value`, `ms_per_step`): a step = one provisioning Solve of the CM
workload (BASELINE configs[1]) through the C-ABI with the problem resident in
HBM (gs_run: K1/K2 feasibility -> K4 first-fit-decreasing -> K3
OrderByPrice/Truncate(60)); checks per step = pods x offerings reachable from
the NodePool.  `solve_latency_ms` is §8(d)'s latency: the wall
clock of complete gs_solve calls (encode + H2D + kernels + D2H + decode into
the result memory), timed separately over the same workload; the device-only
step is `device_ms_per_step`.  The Solve is sequential in pod order, so
--gpus N runs N independent replicas (one cluster's Solve per rank, no
data-path collective): weak scaling; value = sum of checks over ranks / max
step time.

Every BASELINE config has a leg with its own roofline and CPU baseline:
  configs.C1/C2/C3  provisioning Solve legs (same step definition as CM)
  consolidation     C4: SingleNodeConsolidation over 5,000 state nodes
                    (sharded round-robin over ranks, commands all-gathered
                    over RCCL, policy replayed: strong scaling), plus a packed
                    C4 variant with mixed Delete/Replace/NoOp decisions and a
                    MultiNodeConsolidation leg (binary-search prefixes)
  stress            C5: the static pod x offering matrix, 200k pods x 24,000
                    offerings, instance-type words sharded over ranks
  create_filter     the launch-time re-filter of every CM NodeClaim
  ranking           autoplacement ranking over a C5-sized catalog
The CPU baselines run the oracle (oracle/, a C++ restatement of the
reference algorithm) on the GPU box's host: Solve legs on the full config
(1 thread: the Solve is sequential), consolidation on a bounded candidate
sample with 1 and `pool` worker processes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "karpenter-provider-ibm-cloud_amd"))
sys.path.insert(0, ROOT)

from gpusched import abi, synth  # noqa: E402
from gpusched.consolidation import (ConsolidationInput, arrays_to_list, choose_arrays, gather_arrays,  # noqa: E402
                                    n_multi_sims, result_arrays)
from gpusched.lib import Solver  # noqa: E402

METRIC = "pod×offering feasibility checks/sec + Solve latency (ms) at 100k pods, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: aggregate L2 bandwidth (8 XCDs)
CM_WORKLOAD = ("CM: 100k pods x C2 synthetic IBM VPC catalog (198 profiles x 3 zones x {on-demand, spot} = "
               "1,188 offerings), 1 NodePool, 1% GPU pods, 10% nodeSelectors")


# ------------------------------------------------------------------ roofline
def ffd_bytes(res, n_types):
    """SURVEY §8(d) K4 algorithmic bytes per launch: per pod Σ_in-flight
    ⌈N_IT/8⌉ (the option bitset of every NodeClaim a sequential first fit
    visits: res.claim_prefix, pinned equal to the oracle's NodeClaim.CanAdd
    calls by tests/test_gpu_fullsize.py) + 32 B of request sums per pop +
    40 B per existing node visited (res.node_prefix)"""
    return int(res.claim_prefix) * ((n_types + 7) // 8) + 32 * int(res.pops) + 40 * int(res.node_prefix)


def ffd_unique_bytes(res, n_types, n_res, n_claims, n_nodes):
    """unique HBM bytes of one K4 launch: every popped pod's variant record and
    requests (128 + 8 R B) and its add-log entry (16 B), every NodeClaim's
    record and option words written (192 + 8 OW B), every existing node read
    once (184 B).  The claim visits of ffd_bytes() are served from LDS and L2,
    so they are priced against the L2 in a second roofline object."""
    words = (n_types + 63) // 64
    ow = max(4, (words + 3) // 4 * 4)
    return int(res.pops) * (128 + 8 * n_res + 16) + n_claims * (192 + 8 * ow) + n_nodes * 184


def feas_bytes(V, T, O, words):
    """per-launch algorithmic bytes of feas_kernel over `words` instance-type
    words: variant records (128 B), the offering list (48 B), rows + cheapest
    key + offering count written per (variant, template)"""
    return V * 128 + O * 48 + V * T * (words * 8 + 12)


def node_check_bytes(R, K=4):
    """algorithmic bytes of one ExistingNode.CanAdd: available + requests (R x i64),
    taints (8), ok flag (4), K label value ids (4 each), zone/capacity-type ids (8)"""
    return 16 * R + 8 + 4 + 4 * K + 8


def load_traffic(path):
    """{leg: {kernel: HBM bytes per launch}} from the committed PMC profile (empty when absent)"""
    if not path or not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def traffic_of(traffic, leg, *kernels):
    """PMC HBM bytes per launch of a leg's kernel(s), summed (None when not profiled)"""
    tot, seen = 0, False
    for k in kernels:
        x = traffic.get(leg, {}).get(k)
        if x is not None:
            tot += x["bytes"] if isinstance(x, dict) else x
            seen = True
    return tot if seen else None


# where `traffic` comes from: a committed PMC pass (tools/profile_round.sh ->
# tools/pmc_traffic.py), not a counter read inside this run
TRAFFIC_SOURCE = {"path": None}


def roofline(kernel, algo_bytes, avg_ms, traffic=None, peak=HBM_PEAK_GBS, bound="hbm"):
    ach = algo_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    out = {"kernel": kernel, "bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": "GB/s",
           "frac": ach / peak, "algorithmic_bytes": int(algo_bytes), "avg_ms": round(avg_ms, 4), "traffic": traffic}
    if traffic is not None and TRAFFIC_SOURCE["path"]:
        out["traffic_source"] = "committed PMC profile " + TRAFFIC_SOURCE["path"] + " (not measured in this run)"
    if traffic and avg_ms > 0:
        # the rate the PMC bytes imply: a frac above it by more than 1.2x is not HBM evidence
        out["pmc_rate_gbs"] = round(traffic / (avg_ms * 1e-3) / 1e9, 3)
    return out


def digest(res_dict):
    import hashlib
    return hashlib.sha256(json.dumps(res_dict, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


# ------------------------------------------------------------ output lines
HEADLINE_MAX_BYTES = 6144  # the driver keeps the last 8 KB of stdout: the headline must fit wholly
HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "solve_latency_ms",
                 "ffd_us_per_pop")


def _r(x, nd=4):
    """round floats for the compact line (None and ints pass through)"""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}") if abs(x) >= 1e5 or (x != 0 and abs(x) < 1e-3) else round(x, nd)
    return x


def _compact_roofline(rf):
    if not rf:
        return None
    keep = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_source", "basis",
            "algorithmic_bytes", "avg_ms")
    return {k: _r(rf.get(k)) for k in keep if k in rf}


def _compact_cpu(cb):
    if not cb:
        return cb
    out = {k: _r(cb[k]) for k in ("value", "unit", "cores", "kind", "solve_ms", "ms_per_call", "value_1_core",
                                  "gpu_result_bit_exact") if k in cb}
    out["sample"] = (cb.get("sample") or "")[:160]
    return out


def _leg_summary(leg):
    """a few numbers per leg for the headline; the whole leg is in the detail file"""
    s = {}
    for k in ("ms_per_step", "ms_per_sweep", "solve_latency_ms", "ffd_us_per_pop", "ms_per_call_pcie_inclusive",
              "kernel_ms"):
        if k in leg and leg[k] is not None:
            v = leg[k]
            s[k] = {a: _r(b) for a, b in v.items() if a != "trunc"} if isinstance(v, dict) else _r(v)
    rf = leg.get("roofline")
    if rf:
        s["frac"] = _r(rf.get("frac"), 3)
    cb = leg.get("cpu_baseline")
    if cb:
        s["cpu"] = _r(cb.get("solve_ms") or cb.get("ms_per_call") or cb.get("value"))
        if "gpu_result_bit_exact" in cb:
            s["cpu_exact"] = cb["gpu_result_bit_exact"]
    for k in ("oracle_digest_equal", "shards_equal_whole"):
        if leg.get(k) is not None:
            s[k] = leg[k]
    if leg.get("oracle_full_solve_offline"):
        s["cpu_full_offline_s"] = leg["oracle_full_solve_offline"]["seconds"]
    return s


def headline(line):
    """the driver's line: the contract keys, the K4 roofline on SURVEY §8(d)'s
    claim-visit bytes (the unique-byte and L2 views beside it), the CPU
    baseline, latency, and one small summary per leg; <= HEADLINE_MAX_BYTES"""
    h = {k: line.get(k) for k in HEADLINE_KEYS}
    for k in ("value", "ms_per_step", "solve_latency_ms", "ffd_us_per_pop"):
        h[k] = _r(h[k], 6)
    h["roofline"] = _compact_roofline(line.get("roofline"))
    views = {}
    for name, key in (("unique_hbm_bytes", "roofline_unique_bytes"), ("l2_claim_visits", "roofline_l2_claim_visits"),
                      ("feasibility_kernel", "roofline_feasibility_kernel")):
        rf = line.get(key)
        if rf:
            views[name] = {k: _r(rf.get(k)) for k in ("kernel", "bound", "achieved", "peak", "frac", "traffic",
                                                      "algorithmic_bytes") if k in rf}
    if views:
        h["roofline_views"] = views
    h["cpu_baseline"] = _compact_cpu(line.get("cpu_baseline"))
    if line.get("strong_scaling"):
        h["strong_scaling"] = line["strong_scaling"]
    for k in ("solve_latency_phases_ms", "queue_pops", "new_nodeclaims", "pod_errors", "go_sort_emulation",
              "device_kernel_ms"):
        if line.get(k) is not None:
            h[k] = line[k]
    legs = {}
    for grp in ("configs", "consolidation_legs"):
        for name, leg in (line.get(grp) or {}).items():
            legs[name] = _leg_summary(leg)
    for name in ("stress", "create_filter", "ranking"):
        if line.get(name):
            legs[name] = _leg_summary(line[name])
    if legs:
        h["legs"] = legs
    if line.get("detail_file"):
        h["detail_file"] = line["detail_file"]
    # shed detail (never the contract keys) until the line fits
    for drop in ("legs", "roofline_views", "solve_latency_phases_ms", "go_sort_emulation", "device_kernel_ms",
                 "strong_scaling"):
        if len(json.dumps(h)) <= HEADLINE_MAX_BYTES:
            break
        h.pop(drop, None)
    return h


def strong_scaling_section(per_rank, world, backend, max_over_ranks):
    """N > 1: the legs that shard a fixed job over the ranks,
    for the headline -- the C5 static matrix split by instance-type words
    (each rank's kernel, then the RCCL all-gather of the word slices + SUM /
    MIN) and the C4 consolidation sweep split by candidate (each rank's
    simulation kernel, then the all-gather of the commands + the host policy
    replay).  per_rank: this rank's {leg: {timing: ms}}; every timing is the
    max over ranks (the job waits for the slowest), taken with
    max_over_ranks; the other fields come from rank 0's record."""
    out = {"ranks": world, "backend": backend, "scaling": "strong"}
    for leg in sorted(per_rank):
        rec = dict(per_rank[leg])
        for k in sorted(rec):
            if k.endswith("_ms"):
                rec[k] = _r(max_over_ranks(float(rec[k])))
        out[leg] = rec
    return out


def emit(line, detail_path, rank):
    """rank 0: the whole record to `detail_path`, one `# leg <name> {...}`
    line per leg on stdout, then the compact headline as the LAST stdout line"""
    if rank != 0:
        return None
    if detail_path:
        d = os.path.dirname(detail_path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(detail_path, "w") as f:
            json.dump(line, f, indent=1)
        line["detail_file"] = os.path.relpath(detail_path, ROOT)
    for grp in ("configs", "consolidation_legs"):
        for name, leg in (line.get(grp) or {}).items():
            print(f"# leg {name} " + json.dumps(leg))
    for name in ("stress", "create_filter", "ranking"):
        if line.get(name):
            print(f"# leg {name} " + json.dumps(line[name]))
    h = headline(line)
    print(json.dumps(h), flush=True)
    return h


# ------------------------------------------------------------- Solve legs
def solve_leg(problem, solver, steps, warmup, latency_steps, barrier=None, max_over_ranks=None, traffic=None,
              leg=None):
    """device-resident steps (gs_run) and complete gs_solve calls on one problem"""
    t0 = time.perf_counter()
    solver.prepare(problem)
    prep_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(warmup):
        solver.run()
    kt = []
    if barrier:
        barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        solver.run()  # synchronous: returns after the stream's last event
        kt.append(solver.last_run_ms())
    if barrier:
        barrier()
    elapsed = time.perf_counter() - t0
    if max_over_ranks:
        elapsed = max_over_ranks(elapsed)
    t1 = time.perf_counter()
    out, res = solver.fetch()
    fetch_py_ms = (time.perf_counter() - t1) * 1e3
    # §8(d) latency: whole gs_solve calls, C-ABI wall clock (no Python-side copy)
    lat, phases = [], []
    for _ in range(latency_steps):
        t2 = time.perf_counter()
        r = solver.solve_raw(problem)
        lat.append((time.perf_counter() - t2) * 1e3)
        phases.append((r.t_encode_ms, r.t_upload_ms, r.t_feas_ms, r.t_ffd_ms, r.t_truncate_ms, r.t_fetch_ms,
                       r.t_run_wall_ms, r.t_wall_ms))
    kms = {k: sum(x[i] for x in kt) / len(kt) for i, k in enumerate(("feas", "ffd", "trunc"))}
    n_types = len(problem.instance_types)
    ab = {"feas": feas_bytes(res.n_variants, res.n_templates, len(problem.offerings), res.words),
          "ffd": ffd_bytes(res, n_types)}
    names = {"feas": "feas_kernel", "ffd": "ffdw_kernel" if solver.flags == 0 and len(problem.nodes) <= 6144
             else "ffd_kernel"}
    ph = np.mean(np.array(phases), axis=0) if phases else np.zeros(8)
    return {
        "ms_per_step": elapsed * 1e3 / steps,
        "checks": problem.checks(),
        "device_kernel_ms": {k: round(v, 4) for k, v in kms.items()},
        "solve_latency_ms": round(float(np.mean(lat)), 3) if lat else None,
        "solve_latency_ms_each": [round(x, 2) for x in lat],
        "solve_latency_phases_ms": {"encode": round(ph[0], 2), "upload": round(ph[1], 2), "feas": round(ph[2], 3),
                                    "ffd": round(ph[3], 2), "truncate": round(ph[4], 3),
                                    "fetch_decode": round(ph[5], 2),
                                    # the host wall clock of gs_run (kernels + launches + synchronisation),
                                    # the C-ABI call's own wall clock and what the phases leave of it
                                    "run_wall": round(ph[6], 2), "gs_solve_wall": round(ph[7], 2),
                                    "unaccounted": round(ph[7] - ph[0] - ph[1] - ph[5] - ph[6], 2)},
        "prepare_ms_first_call": round(prep_ms, 2),
        "python_result_copy_ms": round(fetch_py_ms, 2),
        "new_nodeclaims": len(out["claims"]),
        "pod_errors": len(out["errors"]),
        "queue_pops": int(res.pops),
        "first_fit_claim_visits": int(res.claim_prefix),
        "first_fit_node_visits": int(res.node_prefix),
        "ffd_candidates_scanned": int(res.cand_evals),
        "ffd_candidates_exact_checked": int(res.cand_full),
        "go_sort_emulation": {"fast": int(res.sorts_fast), "generic": int(res.sorts_generic)},
        # SURVEY §8(d)'s K4 figure (claim visits + request sums + node visits)
        # priced against HBM; beside it the unique HBM bytes (PMC-comparable)
        # and the claim visits priced against the L2 they are served from;
        # and the latency per pod §8(d) asks for
        "roofline": dict(roofline(names["ffd"], ab["ffd"], kms["ffd"], traffic_of(traffic or {}, leg, "ffd")),
                         basis="SURVEY 8(d) claim-visit bytes, served from LDS/L2; HBM-unique bytes: "
                               "roofline_views.unique_hbm_bytes"),
        "roofline_unique_bytes": roofline(names["ffd"], ffd_unique_bytes(
            res, n_types, min(8, len(np.unique(problem.quantities["resource"]))), len(out["claims"]),
            len(problem.nodes)), kms["ffd"], traffic_of(traffic or {}, leg, "ffd")),
        "roofline_l2_claim_visits": roofline(names["ffd"], ab["ffd"], kms["ffd"], None, L2_PEAK_GBS, "l2"),
        "ffd_us_per_pop": round(kms["ffd"] * 1e3 / max(int(res.pops), 1), 4),
        "roofline_feasibility_kernel": roofline("feas_cursor_kernel + feas_kernel", ab["feas"], kms["feas"],
                                                traffic_of(traffic or {}, leg, "feas", "feas_cursor")),
        "_result": out,
    }


def cpu_baseline_solve(problem, got):
    """the oracle's Solve (1 thread) on the SAME full problem; its own input
    build is reported apart from the Solve, like the product's encode"""
    from oracle import pyoracle
    t0 = time.perf_counter()
    st, want, raw = pyoracle.solve(problem)
    wall = (time.perf_counter() - t0) * 1e3
    build_ms = float(raw.t_encode_ms)
    solve_ms = wall - build_ms
    return {"value": problem.checks() / (solve_ms * 1e-3), "unit": "checks/s", "cores": 1, "kind": "port",
            "sample": f"full problem ({len(problem.pods)} pods); oracle Solve {solve_ms:.0f} ms + its input build "
                      f"{build_ms:.0f} ms = {wall:.0f} ms wall (the Solve is sequential: 1 thread)",
            "solve_ms": round(solve_ms, 1), "wall_ms": round(wall, 1),
            "gpu_result_bit_exact": bool(st == abi.GS_OK and got == want)}


def config_leg(name, problem, args, traffic):
    solver = Solver(0)
    try:
        r = solve_leg(problem, solver, max(1, min(args.steps, 5)), 1, args.latency_steps, traffic=traffic, leg=name)
    finally:
        solver.close()
    got = r.pop("_result")
    r["value"] = r["checks"] / (r["ms_per_step"] * 1e-3)
    r["unit"] = "checks/s"
    r["result_sha256"] = digest(got)
    if args.no_cpu_baseline:
        r["cpu_baseline"] = None
    elif name in ("c5_solve", "cm_c4"):
        # the full oracle Solve takes minutes: a bounded, evenly spaced pod
        # sample (its own Solve, same cluster) is timed instead; exactness at
        # full size is the committed oracle digest (C5) or the sample itself
        n_s = args.cpu_sample_c5_solve_pods if name == "c5_solve" else args.cpu_sample_cm_c4_pods
        idx = np.linspace(0, len(problem.pods) - 1, n_s).astype(np.int64)
        sub = problem.with_pods(idx)
        solver = Solver(0)
        try:
            sgot, _ = solver.solve(sub)
        finally:
            solver.close()
        cb = cpu_baseline_solve(sub, sgot)
        cb["sample"] = f"{name}, {len(idx)} evenly spaced pods as their own Solve: " + cb["sample"]
        r["cpu_baseline"] = cb
    else:
        r["cpu_baseline"] = cpu_baseline_solve(problem, got)
    return r


# ------------------------------------------------------- consolidation legs
_POOL = None  # worker processes, forked before this process touches the GPU
_WORKER_PROBLEMS = {}


C4_GENERATORS = {"c4": "make_c4", "e2e": "e2e_consolidation_cluster"}


def c4_problem(spec):
    """spec = (n_nodes, generator kwargs[, generator]): workers rebuild the
    cluster themselves (deterministic generator) instead of inheriting
    GPU-process state"""
    key = json.dumps(spec, sort_keys=True)
    if key not in _WORKER_PROBLEMS:
        _WORKER_PROBLEMS.clear()
        gen = getattr(synth, C4_GENERATORS[spec[2] if len(spec) > 2 else "c4"])
        _WORKER_PROBLEMS[key] = gen(n_nodes=spec[0], **spec[1])
    return _WORKER_PROBLEMS[key]


def _oracle_chunk(job):
    spec, cands, mode, sets = job
    from oracle import pyoracle
    cin = ConsolidationInput(c4_problem(spec), cands, mode=mode, sets=sets)
    st, cmds, _, _ = pyoracle.consolidate(cin)
    return st, cmds


def _warm(spec):
    c4_problem(spec)
    return True


def oracle_consolidation_timed(spec, jobs, workers):
    """oracle consolidation jobs on 1 process (here) or on the pool's
    `workers` processes (the oracle keeps global state: processes, not
    threads); the clusters are built before the clock starts"""
    if workers <= 1 or _POOL is None:
        c4_problem(spec)
        t0 = time.perf_counter()
        outs = [_oracle_chunk(j) for j in jobs]
    else:
        _POOL.map(_warm, [spec] * workers * 2, chunksize=1)
        t0 = time.perf_counter()
        outs = _POOL.map(_oracle_chunk, jobs, chunksize=1)
    return time.perf_counter() - t0, outs


def cpu_baseline_single(spec, n, cmds, n_sample, workers):
    """oracle SingleNodeConsolidation simulations on an evenly spaced sample
    of the candidates, 1 process and `workers` processes; the GPU commands are
    compared on the sample"""
    sub = list(range(0, n, max(1, n // n_sample)))[:n_sample]
    one = sub[:max(1, len(sub) // max(workers, 1))]
    t1, o1 = oracle_consolidation_timed(spec, [(spec, one, abi.CONSOLIDATE_SINGLE, None)], 1)
    chunks = [sub[i::workers] for i in range(workers)]
    tw, ow = oracle_consolidation_timed(spec, [(spec, c, abi.CONSOLIDATE_SINGLE, None) for c in chunks if c],
                                        workers)
    want = {}
    for c, (st, out) in zip([c for c in chunks if c], ow):
        for i, cmd in zip(c, out or []):
            want[i] = cmd
    same = all(cmds[i] == want.get(i) for i in sub)
    return {"value": len(sub) / tw, "unit": "simulations/s", "cores": workers, "kind": "port",
            "value_1_core": len(one) / t1,
            "sample": f"{len(sub)} evenly spaced single-node candidates on {workers} processes ({tw:.1f} s); "
                      f"{len(one)} of them on 1 process ({t1:.1f} s); GPU commands on the sample identical: {same}"}


def consolidation_leg(problem, mode, args, rank, world, local, dist, device, barrier, max_over_ranks, traffic, leg,
                      max_candidates=0):
    n = len(problem.nodes)
    cands = list(range(n))
    shard = (rank, world) if world > 1 else (0, 0)
    cin = ConsolidationInput(problem, cands, mode=mode, shard=shard, max_candidates=max_candidates)
    full = ConsolidationInput(problem, cands, mode=mode, max_candidates=max_candidates)
    solver = Solver(local)
    t0 = time.perf_counter()
    solver.consolidate(cin)  # encode + upload + first run
    prep_ms = (time.perf_counter() - t0) * 1e3

    gch = []

    def sweep():
        r = solver.consolidate_rerun(raw=True)
        if world == 1:
            return None, int(r.chosen), r
        t1 = time.perf_counter()
        merged = gather_arrays(*result_arrays(r), rank, world, dist, device)
        chosen, _ = choose_arrays(full, *merged)
        gch.append((time.perf_counter() - t1) * 1e3)
        return merged, chosen, r

    for _ in range(args.warmup):
        sweep()
    gch.clear()
    kt = []
    steps = args.steps
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        merged, chosen, r = sweep()
        kt.append((r.t_feas_ms, r.t_sim_ms, r.t_truncate_ms, r.t_fetch_ms))
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    if merged is None:
        merged = result_arrays(r)
    merged = arrays_to_list(*merged)
    ms = elapsed * 1e3 / steps
    feas_ms, sim_ms, trunc_ms, decide_ms = (sum(k[i] for k in kt) / len(kt) for i in range(4))
    R = len(set(int(x) for x in problem.quantities["resource"]))
    nb = node_check_bytes(R)
    n_sims = len(merged)
    n_local = (n_sims + world - 1) // world
    # HBM-unique algorithmic bytes of one launch: the shared node table once,
    # every simulated pod's variant record + requests + add-log entry, the
    # control block per simulation.  The node checks each simulation repeats
    # (node_prefix visits) are served by L2 / MALL: priced against L2 apart.
    uniq_bytes = n * nb + int(r.pods_simulated) * (128 + 8 * R + 16) + n_local * 256
    visit_bytes = r.node_prefix * nb + r.pops * (104 + 8 * R) + n_local * 256
    counts = {}
    for c in merged:
        k = abi.DECISION_NAMES[c["decision"]]
        counts[k] = counts.get(k, 0) + 1
    out = {
        "mode": {abi.CONSOLIDATE_SINGLE: "SingleNodeConsolidation",
                 abi.CONSOLIDATE_MULTI: "MultiNodeConsolidation"}[mode],
        "simulations": n_sims,
        "value": n_sims / (ms * 1e-3),
        "unit": "simulations/s",
        "ms_per_sweep": ms,
        "scaling": "strong",
        "node_checks_per_s": r.checks * world / (ms * 1e-3),
        "kernel_ms": {"feas": round(feas_ms, 4), "sim": round(sim_ms, 4), "trunc": round(trunc_ms, 4)},
        "host_decide_fetch_ms": round(decide_ms, 3),
        # N > 1: all-gather of the command tables over the ranks + the host policy replay (this rank)
        "gather_choose_ms": round(sum(gch) / len(gch), 3) if gch else 0.0,
        "prepare_ms_encode_plus_pcie_upload": round(prep_ms, 1),
        "pods_simulated": int(r.pods_simulated),
        "node_prefix": int(r.node_prefix),
        "chosen": chosen,
        "decisions": counts,
        "roofline": roofline("ffd_kernel<SIM>", uniq_bytes, sim_ms, traffic_of(traffic, leg, "sim")),
        "roofline_l2_node_visits": roofline("ffd_kernel<SIM>", visit_bytes, sim_ms, None, L2_PEAK_GBS, "l2"),
        "cpu_baseline": None,
        "_commands": merged,
    }
    solver.close()
    return out


def cpu_baseline_multi(spec, n, cmds, n_prefixes, workers):
    """oracle MultiNodeConsolidation prefix simulations (the binary search's
    candidates[0:mid+1]) on a sample of prefix lengths, as EVAL sets, on
    `workers` processes; GPU commands compared on the sample"""
    n_sims = len(cmds)
    mids = sorted(set(int(x) for x in np.linspace(0, n_sims - 1, n_prefixes)))
    cands = list(range(n))
    jobs = [(spec, cands, abi.CONSOLIDATE_EVAL, [(0, m + 2)]) for m in mids]
    tw, outs = oracle_consolidation_timed(spec, jobs, workers)
    same = all(st == abi.GS_OK and out and out[0] == cmds[m] for m, (st, out) in zip(mids, outs))
    return {"value": len(mids) / tw, "unit": "simulations/s", "cores": workers, "kind": "port",
            "sample": f"{len(mids)} prefix simulations (lengths {[m + 2 for m in mids]}) on {workers} processes "
                      f"({tw:.1f} s); GPU commands on the sample identical: {same}"}


# ---------------------------------------------------------------- C5 stress
def cpu_baseline_stress(problem, n_pods):
    """oracle static matrix (1 thread) on an evenly spaced pod sample of C5;
    checks the GPU matrix on that sample"""
    from oracle import pyoracle
    idx = np.linspace(0, len(problem.pods) - 1, n_pods).astype(np.int64)
    sub = problem.with_pods(idx)
    t0 = time.perf_counter()
    st, want = pyoracle.feasibility(sub)
    dt = time.perf_counter() - t0
    s = Solver(0)
    try:
        s.prepare(sub)
        got, _ = s.feasibility()
    finally:
        s.close()
    same = all(np.array_equal(got[k], want[k]) for k in ("rows", "cheapest", "n_feasible_offerings"))
    return {"value": sub.checks() / dt, "unit": "checks/s", "cores": 1, "kind": "port",
            "sample": f"C5, {n_pods} evenly spaced pods; oracle static matrix {dt * 1e3:.0f} ms; GPU matrix on the "
                      f"sample bit-exact: {bool(same)}"}


def bench_stress(args, rank, world, local, dist, device, barrier, max_over_ranks, traffic):
    """C5 (BASELINE configs[4]): the static pod x offering matrix, instance-type
    words sharded over the ranks and combined in place by RCCL: strong scaling"""
    from gpusched.feasibility import device_combine, word_range
    problem = synth.make_c5(n_pods=args.c5_pods)
    solver = Solver(local)
    t0 = time.perf_counter()
    solver.prepare(problem)
    prep_ms = (time.perf_counter() - t0) * 1e3
    W = (len(problem.instance_types) + 63) // 64
    wb, we = word_range(W, rank, world)

    comb = []

    def step():
        r = solver.feasibility_shard_device(wb, we)  # returns after the kernel
        if world > 1:
            t1 = time.perf_counter()
            device_combine(r, dist, device)
            import torch
            torch.cuda.synchronize(device)
            comb.append((time.perf_counter() - t1) * 1e3)
        return r

    for _ in range(args.warmup):
        step()
    comb.clear()
    kms = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = step()
        kms.append(r.t_kernel_ms)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms = elapsed * 1e3 / args.steps
    k_ms = sum(kms) / len(kms)
    combine_ms = sum(comb) / len(comb) if comb else 0.0
    equal = None
    if world > 1:
        import torch
        from gpusched.feasibility import device_views
        got = [x.clone() for x in device_views(r, device)]
        whole = solver.feasibility_shard_device(0, W)
        ref = device_views(whole, device)
        S = r.row_stride
        equal = bool(torch.equal(got[0].view(-1, S)[:, :W], ref[0].view(-1, S)[:, :W]) and
                     torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2]))
        equal = bool(max_over_ranks(0.0 if equal else 1.0) == 0.0)
    ab = feas_bytes(r.n_variants, r.n_templates, len(problem.offerings), we - wb)
    out = {
        "workload": f"C5: {len(problem.pods)} pods x {len(problem.instance_types)} instance types x 6 zones x "
                    f"2 capacity types ({len(problem.offerings)} offerings), static feasibility matrix + cheapest "
                    f"offering per pod and NodePool",
        "value": r.checks / (ms * 1e-3),
        "unit": "checks/s",
        "ms_per_step": ms,
        "scaling": "strong",
        "parallelism": f"it-columns{world}" if world > 1 else "single",
        "words_per_rank": we - wb,
        "variants": r.n_variants,
        "kernel_ms": round(k_ms, 4),
        "combine_ms": round(combine_ms, 4),  # N > 1: RCCL all-gather of the word slices + SUM / MIN (this rank)
        "prepare_ms_encode_plus_pcie_upload": round(prep_ms, 1),
        "shards_equal_whole": equal,
        "roofline": roofline("feas_cursor_kernel + feas_kernel", ab, k_ms, traffic_of(traffic, "c5", "feas", "feas_cursor")),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1:
        out["library_shards"] = library_shards(problem, solver, W, args.steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_stress(problem, args.cpu_sample_c5_pods)
    solver.close()
    return out


def _hip_device_count():
    """devices the HIP runtime the library links sees (torch bundles its own
    runtime; initialising it after the library's can fail in one process)"""
    import ctypes
    n = ctypes.c_int(0)
    try:
        ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(n))
    except OSError:
        return 1
    return n.value


def library_shards(problem, single, W, steps):
    """the library's own multi-GPU (gs_config.n_shards = 2, csrc/multi.cpp):
    each shard computes half the words on its device, the merge kernel on the
    parent's device gathers the slices over xGMI peer reads and reduces the
    counts / keys.  Two devices when the node shows them, else both shards on
    device 0; merge_ms is the merge kernel alone"""
    devs = [0, 1] if _hip_device_count() > 1 else [0, 0]
    s = Solver(devs[0], shard_devices=devs)
    try:
        s.prepare(problem)
        s.feasibility_shard_device(0, W)
        merge, kern, wall = [], [], []
        for _ in range(max(steps, 3)):
            t0 = time.perf_counter()
            r = s.feasibility_shard_device(0, W)
            wall.append((time.perf_counter() - t0) * 1e3)
            merge.append(r.t_merge_ms)
            kern.append(r.t_kernel_ms)
        # the merged device matrix through the host API (same buffers, copied out)
        got, _ = s.feasibility()
        want, _ = single.feasibility()
        equal = all(np.array_equal(got[k], want[k]) for k in ("rows", "cheapest", "n_feasible_offerings", "cheapest_key"))
    finally:
        s.close()
    return {"shard_devices": devs, "merge_ms": round(sum(merge) / len(merge), 4),
            "shard_kernel_ms_max": round(sum(kern) / len(kern), 4), "call_ms": round(sum(wall) / len(wall), 3),
            "equal_single_device": equal}


# ------------------------------------------------------------ small legs
def bench_ranking(args):
    """Autoplacement ranking (FilterInstanceTypes + rankInstanceTypes,
    instancetype.go:259-379) over a C5-sized catalog of 2,000 instance types
    with all filters off.  One call = host buffers in, ranked indices out
    (PCIe-inclusive); rank 0 at N=1 only."""
    from gpusched import lib
    rng = np.random.default_rng(5)
    n = 2000
    vcpu = rng.choice([2, 4, 8, 16, 32, 48, 64, 96], size=n)
    ratio = rng.choice([2, 4, 8], size=n)
    cpu = (vcpu * 1000).astype(np.int64)
    mem = (vcpu * ratio * (1 << 30)).astype(np.int64)
    price = np.round(vcpu * ratio * rng.choice([0.01, 0.0125, 0.02], size=n), 4)
    arch = np.zeros(n, dtype=np.uint32)
    for _ in range(max(args.warmup, 1)):
        lib.rank_instance_types(cpu, mem, price, arch)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        order, score = lib.rank_instance_types(cpu, mem, price, arch)
    ms = (time.perf_counter() - t0) * 1000 / args.steps
    out = {"workload": f"RankInstanceTypes over {n} instance types (C5 catalog size), exact score ties",
           "types": n, "ms_per_call_pcie_inclusive": round(ms, 4), "cpu_baseline": None}
    if not args.no_cpu_baseline:
        from oracle import pyoracle
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            st, want, _ = pyoracle.rank_instance_types(cpu, mem, price, arch)
        cms = (time.perf_counter() - t0) * 1000 / reps
        out["cpu_baseline"] = {"ms_per_call": round(cms, 4), "cores": 1, "kind": "port",
                               "sample": f"same {n} types, {reps} calls; GPU order identical: {want == order}"}
    return out


def claim_queries(problem, result):
    """ToNodeClaim: each emitted NodeClaim's requirements + instance-type
    In[options] and its requests, as gs_claim_query rows"""
    names = [problem.strings[i] for i in problem.instance_types["name"]]

    def add(b):
        for c in result["claims"]:
            reqs = []
            for line in c["requirements"].split("\n") if c["requirements"] else []:
                key, op, vals, gt, lt, _ = line.split("|")
                if key == "node.kubernetes.io/instance-type":
                    continue
                if not (op == "Exists" and (gt != "-" or lt != "-")):
                    reqs.append((key, op, vals.split(",") if vals else []))
                if gt != "-":
                    reqs.append((key, "Gt", [gt]))
                if lt != "-":
                    reqs.append((key, "Lt", [lt]))
            reqs.append(("node.kubernetes.io/instance-type", "In", [names[i] for i in c["its"]]))
            b.add_claim_query(reqs, c["requests"])
    return problem.extended(add)


def bench_create_filter(problem, result, args):
    """CloudProvider.Create's re-filter + instanceTypes[0] + ResolveCapacityType
    for every NodeClaim the CM Solve emitted, one gs_create_filter call
    (host buffers in, results out: PCIe-inclusive)"""
    p2 = claim_queries(problem, result)
    solver = Solver(0)
    try:
        for _ in range(max(args.warmup, 1)):
            solver.create_filter(p2, raw=True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            solver.create_filter(p2, raw=True)
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        kernel_ms = solver_filter_ms(solver)
        got = solver.create_filter(p2)
    finally:
        solver.close()
    nq, n = p2.n_claim_queries, len(p2.instance_types)
    out = {"workload": f"{nq} CM NodeClaims x {n} instance types (List order), requirement algebra + offerings "
                       f"+ Fits", "pairs": nq * n, "ms_per_call_pcie_inclusive": round(ms, 3),
           "kernel_ms": kernel_ms, "pairs_per_s": nq * n / (ms * 1e-3), "cpu_baseline": None}
    if not args.no_cpu_baseline:
        from oracle import pyoracle
        t0 = time.perf_counter()
        st, want = pyoracle.create_filter(p2)
        cms = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"ms_per_call": round(cms, 2), "pairs_per_s": nq * n / (cms * 1e-3), "cores": 1,
                               "kind": "port", "sample": f"same {nq} claims; GPU results identical: {got == want}"}
    return out


def solver_filter_ms(solver):
    return None  # the kernel time is inside the call; rocprofv3 stats carry it


# --------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=100_000)
    ap.add_argument("--latency-steps", type=int, default=3)
    ap.add_argument("--c4-nodes", type=int, default=5000)
    ap.add_argument("--cpu-sample-sims", type=int, default=160)
    ap.add_argument("--cpu-sample-prefixes", type=int, default=16)
    ap.add_argument("--pool", type=int, default=min(16, os.cpu_count() or 1),
                    help="worker processes for the consolidation CPU baselines (the box's CPU share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-consolidation", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the C1/C2/C3 Solve legs")
    ap.add_argument("--c5-pods", type=int, default=200_000)
    ap.add_argument("--cpu-sample-c5-pods", type=int, default=2000)
    ap.add_argument("--cpu-sample-c5-solve-pods", type=int, default=20000)
    ap.add_argument("--cpu-sample-cm-c4-pods", type=int, default=10000)
    ap.add_argument("--no-stress", action="store_true")
    ap.add_argument("--only", default=None, help="run one leg only: cm | c1 | c2 | c3 | e2e | e2e200 | c5_solve | cm_c4 | "
                                                 "c4 | c4_mixed | c4_multi | c4_e2e | c4_e2e_multi | c5 | filter | "
                                                 "ranking (profiling passes)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r6", "traffic.json"),
                    help="PMC-derived HBM bytes per launch per leg (tools/pmc_traffic.py, committed under profiles/)")
    ap.add_argument("--detail-json", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="the whole record (every leg); stdout's last line is the compact headline")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    device = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    traffic = load_traffic(args.traffic_json)
    if traffic:
        TRAFFIC_SOURCE["path"] = os.path.relpath(os.path.abspath(args.traffic_json), ROOT)
    only = args.only
    solo = rank == 0 and world == 1
    global _POOL
    if solo and not args.no_cpu_baseline and not args.no_consolidation and args.pool > 1 and \
            only in (None, "c4", "c4_mixed", "c4_multi", "c4_e2e", "c4_e2e_multi"):
        import multiprocessing as mp
        _POOL = mp.get_context("fork").Pool(args.pool)  # before any GPU call in this process
    line = {"metric": METRIC, "value": None, "unit": "checks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic"}

    if only in (None, "cm", "filter"):
        problem = synth.make_cm(n_pods=args.pods, seed=0x5EED0006 + rank)
        solver = Solver(local)
        r = solve_leg(problem, solver, args.steps, args.warmup, args.latency_steps if only != "filter" else 0,
                      barrier, max_over_ranks, traffic, "cm")
        solver.close()
        result = r.pop("_result")
        ms = r.pop("ms_per_step")
        line.update({
            "value": r["checks"] * world / (ms * 1e-3),
            "ms_per_step": ms,
            "device_ms_per_step": ms,
            "config": {"workload": CM_WORKLOAD, "pods": len(problem.pods),
                       "instance_types": len(problem.instance_types), "offerings": len(problem.offerings),
                       "nodepools": len(problem.nodepools), "checks_per_step": r["checks"],
                       "parallelism": f"replicas{world}" if world > 1 else "single"},
        })
        line.update({k: v for k, v in r.items() if k != "checks"})
        line["result_sha256"] = digest(result)
        line["cpu_baseline"] = None
        if solo and not args.no_cpu_baseline and only is None:
            line["cpu_baseline"] = cpu_baseline_solve(problem, result)
        if solo and only in (None, "filter"):
            line["create_filter"] = bench_create_filter(problem, result, args)
        del problem, result

    if solo and not args.no_configs and only in (None, "c1", "c2", "c3", "e2e", "e2e200", "c5_solve", "cm_c4"):
        configs = {}
        gens = {"c1": (synth.make_c1, "C1: 500 pods x 8 fake profiles x 3 zones (24 offerings), 1 NodePool"),
                "c2": (synth.make_c2, "C2: 10k pods x C2 catalog (1,188 offerings), 1 NodePool"),
                "c3": (synth.make_c3, "C3: 50k pods x C2 catalog, 4 weighted NodePools, taints/tolerations, "
                                      "required + preferred node affinity, 20% zone topology spread"),
                # the reference e2e suite's deployment shape at scale (test/e2e/config.go:455-490)
                "e2e": (lambda: synth.e2e_deployments(n_deployments=60, replicas=500),
                        "e2e: 30k pods in 60 deployments x 500 replicas, each with a preferred (weight 100) "
                        "kubernetes.io/hostname podAntiAffinity on its own app label, 16-type catalog x 3 zones x "
                        "{on-demand, spot}"),
                "e2e200": (lambda: synth.e2e_deployments(n_deployments=200, replicas=150),
                           "e2e200: 30k pods in 200 deployments x 150 replicas (200 topology groups), the e2e "
                           "deployment shape above"),
                # BASELINE configs[4] as a Solve: 200k pods x 2,000 types x 6 zones x 2 capacity types
                "c5_solve": (synth.make_c5, "C5 Solve: 200k pods x 2,000 synthetic instance types x 6 zones x "
                                            "{on-demand, spot} (24,000 offerings), 1 NodePool"),
                # CM's pods provisioned into C4's cluster: 5,000 state nodes first (single-wave kernel's LDS
                # node codes, existing-node fast accept and infeasible-prefix hint)
                "cm_c4": (lambda: synth.make_c4(n_nodes=5000, n_pending=100_000),
                          "CM pods onto C4: 100k CM-distribution pending pods into a cluster of 5,000 state nodes "
                          "(C2 catalog, 2 NodePools, 60-90% cpu used), then new NodeClaims")}
        for name, (gen, desc) in gens.items():
            if only not in (None, name):
                continue
            leg = config_leg(name, gen(), args, traffic)
            leg["workload"] = desc
            configs[name.upper()] = leg
            if name == "c5_solve":
                # the oracle's C5 200k result digest (tests/golden/fullsize.json, 6.5 min on one core)
                with open(os.path.join(ROOT, "tests", "golden", "fullsize.json")) as f:
                    gold = json.load(f)["c5_200k"]
                leg["oracle_digest_equal"] = leg.pop("result_sha256") == gold["sha256"]
                # the full 200k oracle Solve is too long for the bench: its
                # offline time (build container, 1 core) is reported as such
                leg["oracle_full_solve_offline"] = {
                    "seconds": gold["oracle_s"], "cores": 1, "kind": "port",
                    "where": "build container (not the GPU box), tests/golden/make_fullsize_golden.py; the same "
                             "container times CM's oracle Solve ~3x slower than the GPU box's host"}
        line["configs"] = configs

    if not args.no_consolidation and only in (None, "c4", "c4_mixed", "c4_multi", "c4_e2e", "c4_e2e_multi"):
        legs = {}
        specs = {
            "c4": (dict(), abi.CONSOLIDATE_SINGLE, 0,
                   "C4: {n} state nodes (C2 catalog, 2 NodePools, 60-90% cpu used, {b} bound pods), "
                   "SingleNodeConsolidation over all {n} candidates"),
            "c4_mixed": (dict(util=(0.9, 0.99), full_frac=0.5, big_frac=1.0, pack=True), abi.CONSOLIDATE_SINGLE, 0,
                         "C4 packed: {n} state nodes filled until no pod of their shape fits (90-99% cpu, "
                         "{b} bound 1-6 vCPU pods): mixed Delete / Replace / NoOp, SingleNodeConsolidation"),
            "c4_multi": (dict(), abi.CONSOLIDATE_MULTI, 100,
                         "C4: {n} state nodes, MultiNodeConsolidation: every binary-search prefix "
                         "candidates[0:mid+1] of the first 100 candidates as one simulation"),
            # the reference's consolidation e2e workload (test/e2e/scheduling_test.go:38-122) at C4 scale:
            # every pod carries a preferred hostname anti-affinity (general simulation variant)
            "c4_e2e": (dict(), abi.CONSOLIDATE_SINGLE, 0,
                       "C4 e2e shape: {n} state nodes of the C2 catalog running {b} pods of 4-replica deployments, "
                       "1 vCPU / 1 GiB each with a preferred (weight 100) kubernetes.io/hostname podAntiAffinity on "
                       "its own app (reference test/e2e/scheduling_test.go:38-122), SingleNodeConsolidation over "
                       "all {n} candidates (topology variant of the simulation kernel)"),
            "c4_e2e_multi": (dict(), abi.CONSOLIDATE_MULTI, 100,
                             "C4 e2e shape: {n} state nodes as c4_e2e, MultiNodeConsolidation prefixes of the first "
                             "100 candidates (topology variant)"),
        }
        for name, (kw, mode, maxc, desc) in specs.items():
            if only not in (None, name):
                continue
            spec = (args.c4_nodes, kw, "e2e" if name.startswith("c4_e2e") else "c4")
            problem = c4_problem(spec)
            leg = consolidation_leg(problem, mode, args, rank, world, local, dist, device, barrier, max_over_ranks,
                                    traffic, name, max_candidates=maxc)
            cmds = leg.pop("_commands")
            leg["workload"] = desc.format(n=len(problem.nodes), b=len(problem.bound_pods))
            if solo and not args.no_cpu_baseline:
                n = len(problem.nodes)
                if mode == abi.CONSOLIDATE_SINGLE:
                    leg["cpu_baseline"] = cpu_baseline_single(spec, n, cmds, args.cpu_sample_sims, args.pool)
                else:
                    leg["cpu_baseline"] = cpu_baseline_multi(spec, n, cmds, args.cpu_sample_prefixes, args.pool)
            legs[name] = leg
        line["consolidation"] = legs.get("c4")
        line["consolidation_legs"] = legs

    if not args.no_stress and only in (None, "c5"):
        line["stress"] = bench_stress(args, rank, world, local, dist, device, barrier, max_over_ranks, traffic)
    if solo and only in (None, "ranking"):
        line["ranking"] = bench_ranking(args)
    if world > 1:
        per_rank = {}
        st = line.get("stress")
        if st:
            per_rank["c5_static_matrix_it_columns"] = {
                "ms_per_step": st["ms_per_step"], "kernel_ms": st["kernel_ms"], "combine_ms": st["combine_ms"],
                "words_per_rank": st["words_per_rank"], "checks_per_s": _r(st["value"]),
                "shards_equal_whole": st["shards_equal_whole"]}
        for name, leg in (line.get("consolidation_legs") or {}).items():
            per_rank[f"{name}_candidates"] = {
                "ms_per_sweep": leg["ms_per_sweep"], "sim_kernel_ms": leg["kernel_ms"]["sim"],
                "gather_choose_ms": leg["gather_choose_ms"], "simulations": leg["simulations"],
                "simulations_per_s": _r(leg["value"])}
        backend = dist.get_backend() if dist is not None else None
        line["strong_scaling"] = strong_scaling_section(per_rank, dist.get_world_size(), backend, max_over_ranks)
    if _POOL is not None:
        _POOL.close()
        _POOL.join()
    emit(line, args.detail_json, rank)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
