#!/usr/bin/env python3
"""bench.py — BASELINE.json metric on MI355X:
pod x offering feasibility checks/sec + Solve latency (ms), 100k pods.

Headline (`value`): a step = one device-resident provisioning Solve of the CM
workload through the C-ABI (gs_run: K1/K2 feasibility -> K4 first-fit-
decreasing -> K3 OrderByPrice/Truncate(60)); encode + host->HBM upload happen
once before the timed region and are reported separately.  checks per step =
pods x offerings reachable from the NodePool.  The Solve is
sequential in pod order, so --gpus N runs N independent replicas (one
independent cluster's Solve per rank, no data-path collective): weak scaling;
value = sum of checks over ranks / max step time.

`consolidation`: the C4 workload (BASELINE configs[3]): a SingleNodeConsolidation
sweep over all 5,000 state nodes, each an independent SimulateScheduling Solve
(one workgroup per simulation).  Simulations are sharded round-robin over the
N ranks, their commands all-gathered (RCCL over xGMI), and the policy replayed
on every rank: strong scaling.

`stress`: the C5 workload (BASELINE configs[4]): the static pod x offering
matrix of 200k pods x 2,000 instance types x 6 zones x 2 capacity types with
instance-type columns sharded over the ranks and combined by RCCL all-reduces
(SUM rows / SUM offering counts / MIN OrderByPrice key): strong scaling.
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
                                    result_arrays)
from gpusched.lib import Solver  # noqa: E402

METRIC = "pod×offering feasibility checks/sec + Solve latency (ms) at 100k pods, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(res, problem, n_claims):
    """per-launch ALGORITHMIC bytes from the run's counters"""
    V, T, W = res.n_variants, res.n_templates, res.words
    R = res.n_resources
    O = len(problem.offerings)
    N = len(problem.instance_types)
    feas = V * 128 + O * 48 + V * T * (W * 8 + 12)
    per_cand = 24 + W * 8 * (2 + R) + R * 8      # header, opts, row, R threshold sets, totals
    per_pop = R * 8 + 96                          # pod requests + variant record
    adds = len(problem.pods) - res.n_errors
    per_add = W * 8 + R * 8 + 24 + 16             # claim update + add-log record
    ffd = res.pops * per_pop + res.cand_evals * per_cand + adds * per_add
    trunc = n_claims * (W * 8 + 24 + 60 * 4) + N * 16
    return {"feas": feas, "ffd": ffd, "trunc": trunc}


def load_traffic(path):
    """{kernel: HBM bytes per launch} from the committed PMC profile (null when absent)"""
    if not path or not os.path.exists(path):
        return {}
    return {k: v["bytes"] for k, v in json.load(open(path)).items()}


def node_check_bytes(R, K=4):
    """algorithmic bytes of one ExistingNode.CanAdd: available + requests (R x i64),
    taints (8), ok flag (4), K label value ids (4 each), zone/capacity-type ids (8)"""
    return 16 * R + 8 + 4 + 4 * K + 8


def cpu_baseline(n_pods):
    """oracle (C++ port of the reference algorithm, 1 thread) on a bounded
    sample of the same workload; also checks the GPU result on that sample"""
    from oracle import pyoracle
    problem = synth.make_cm(n_pods=n_pods)
    t0 = time.perf_counter()
    st, want, _ = pyoracle.solve(problem)
    dt = time.perf_counter() - t0
    s = Solver(0)
    try:
        got, _ = s.solve(problem)
    finally:
        s.close()
    return {
        "value": problem.checks() / dt,
        "unit": "checks/s",
        "cores": 1,
        "kind": "port",
        "sample": f"CM distribution, first {n_pods} pods (same C2 catalog, 1 NodePool); oracle Solve "
                  f"{dt * 1e3:.0f} ms; GPU result on the sample bit-exact: {got == want}",
        "solve_ms": dt * 1e3,
    }


def cpu_baseline_consolidation(problem, cmds, n_sample):
    """oracle SingleNodeConsolidation simulations (1 thread) on a bounded sample
    of the candidates; checks the GPU commands on that sample"""
    from oracle import pyoracle
    n = len(problem.nodes)
    sub = list(range(0, n, max(1, n // n_sample)))[:n_sample]
    t0 = time.perf_counter()
    st, want, _, _ = pyoracle.consolidate(ConsolidationInput(problem, sub, mode=abi.CONSOLIDATE_SINGLE))
    dt = time.perf_counter() - t0
    return {
        "value": len(sub) / dt,
        "unit": "simulations/s",
        "cores": 1,
        "kind": "port",
        "sample": f"C4 cluster, {len(sub)} evenly spaced single-node candidates; oracle {dt * 1e3:.0f} ms; "
                  f"GPU commands on the sample identical: {st == 0 and [cmds[i] for i in sub] == want}",
    }


def bench_consolidation(args, rank, world, local, dist, device, barrier, max_over_ranks):
    problem = synth.make_c4(n_nodes=args.c4_nodes)
    n = len(problem.nodes)
    cands = list(range(n))
    shard = (rank, world) if world > 1 else (0, 0)
    cin = ConsolidationInput(problem, cands, mode=abi.CONSOLIDATE_SINGLE, shard=shard)
    full = ConsolidationInput(problem, cands, mode=abi.CONSOLIDATE_SINGLE)
    solver = Solver(local)
    t0 = time.perf_counter()
    cmds, _, _, res = solver.consolidate(cin)  # encode + upload + first run
    prep_ms = (time.perf_counter() - t0) * 1e3

    def sweep():
        # device simulations + host decisions, then (N > 1) the all-gather of
        # every rank's commands and the policy replay
        r = solver.consolidate_rerun(raw=True)
        if world == 1:
            return None, int(r.chosen), r
        merged = gather_arrays(*result_arrays(r), rank, world, dist, device)
        chosen, _ = choose_arrays(full, *merged)
        return merged, chosen, r

    for _ in range(args.warmup):
        sweep()
    kt = []
    barrier()
    t0 = time.perf_counter()
    steps_ms = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        merged, chosen, r = sweep()
        steps_ms.append((time.perf_counter() - ts) * 1e3)
        kt.append((r.t_feas_ms, r.t_sim_ms, r.t_truncate_ms, r.t_fetch_ms))
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    if merged is None:
        merged = result_arrays(r)
    merged = arrays_to_list(*merged)
    ms = elapsed * 1e3 / args.steps
    feas_ms = sum(k[0] for k in kt) / len(kt)
    sim_ms = sum(k[1] for k in kt) / len(kt)
    trunc_ms = sum(k[2] for k in kt) / len(kt)
    decide_ms = sum(k[3] for k in kt) / len(kt)
    R = len(set(int(x) for x in problem.quantities["resource"]))  # encoded resource dimensions
    nb = node_check_bytes(R)
    # per-launch algorithmic bytes of the simulation kernel on THIS rank: the
    # node records a sequential first-fit visits + per pop (variant record
    # 104 B + requests 8R) + per simulation (candidate ids, control block)
    n_local = (n + world - 1) // world
    sim_bytes = r.node_prefix * nb + r.pops * (104 + 8 * R) + n_local * 256
    ach = sim_bytes / (sim_ms * 1e-3) / 1e9 if sim_ms > 0 else 0.0
    counts = {}
    for c in merged:
        k = abi.DECISION_NAMES[c["decision"]]
        counts[k] = counts.get(k, 0) + 1
    out = {
        "workload": f"C4: {n} state nodes (C2 catalog, 2 NodePools, 60-90% cpu used, {len(problem.bound_pods)} "
                    f"bound pods), SingleNodeConsolidation over all {n} candidates",
        "simulations": n,
        "value": n / (ms * 1e-3),
        "unit": "simulations/s",
        "ms_per_sweep": ms,
        "scaling": "strong",
        "node_checks_per_s": r.checks * world / (ms * 1e-3),
        "kernel_ms": {"feas": round(feas_ms, 4), "sim": round(sim_ms, 4), "trunc": round(trunc_ms, 4)},
        "host_decide_fetch_ms": round(decide_ms, 3),
        "sweep_ms_each": [round(x, 3) for x in steps_ms],
        "prepare_ms_encode_plus_pcie_upload": round(prep_ms, 1),
        "pods_simulated": int(r.pods_simulated),
        "node_evals": int(r.node_evals),
        "node_prefix": int(r.node_prefix),
        "chosen": chosen,
        "decisions": counts,
        "roofline": {"kernel": "ffd_kernel<SIM>", "bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes": int(sim_bytes),
                     "avg_ms": round(sim_ms, 4), "traffic": load_traffic(args.traffic_json).get("sim")},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_consolidation(problem, merged, args.cpu_sample_sims)
    solver.close()
    return out


def feas_bytes(V, T, O, words):
    """per-launch algorithmic bytes of feas_kernel over `words` instance-type
    words: variant records, the offering list, rows + counts + keys written"""
    return V * 128 + O * 48 + V * T * (words * 8 + 12)


def cpu_baseline_stress(n_pods):
    """oracle static matrix (1 thread) on the first n_pods of the C5 workload;
    checks the GPU matrix on that sample"""
    from oracle import pyoracle
    problem = synth.make_c5(n_pods=n_pods)
    t0 = time.perf_counter()
    st, want = pyoracle.feasibility(problem)
    dt = time.perf_counter() - t0
    s = Solver(0)
    try:
        s.prepare(problem)
        got, _ = s.feasibility()
    finally:
        s.close()
    same = all(np.array_equal(got[k], want[k]) for k in ("rows", "cheapest", "n_feasible_offerings"))
    return {"value": problem.checks() / dt, "unit": "checks/s", "cores": 1, "kind": "port",
            "sample": f"C5, first {n_pods} pods; oracle static matrix {dt * 1e3:.0f} ms; GPU matrix on the "
                      f"sample bit-exact: {bool(same)}"}


def bench_stress(args, rank, world, local, dist, device, barrier, max_over_ranks):
    """C5 (BASELINE configs[4]): the static pod x offering matrix of 200k pods x
    2,000 types x 6 zones x 2 capacity types, instance-type words sharded over
    the ranks and combined in place by three RCCL all-reduces: strong scaling"""
    from gpusched.feasibility import device_combine, word_range
    problem = synth.make_c5(n_pods=args.c5_pods)
    solver = Solver(local)
    t0 = time.perf_counter()
    solver.prepare(problem)
    prep_ms = (time.perf_counter() - t0) * 1e3
    W = (len(problem.instance_types) + 63) // 64
    wb, we = word_range(W, rank, world)

    def step():
        r = solver.feasibility_shard_device(wb, we)  # returns after the kernel
        if world > 1:
            device_combine(r, dist, device)
            import torch
            torch.cuda.synchronize(device)
        return r

    for _ in range(args.warmup):
        step()
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
    ach = ab / (k_ms * 1e-3) / 1e9
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
        "prepare_ms_encode_plus_pcie_upload": round(prep_ms, 1),
        "shards_equal_whole": equal,
        "roofline": {"kernel": "feas_kernel", "bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes": int(ab),
                     "avg_ms": round(k_ms, 4), "traffic": load_traffic(args.traffic_json).get("feas_c5")},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_stress(args.cpu_sample_c5_pods)
    solver.close()
    return out


def bench_ranking(args):
    """Autoplacement ranking (FilterInstanceTypes + rankInstanceTypes,
    instancetype.go:259-379) over a C5-sized catalog of 2,000 instance types
    with all filters off (RankInstanceTypes).  One call = host buffers in,
    ranked indices out, so the time is PCIe- and allocation-inclusive; rank 0
    at N=1 only (replicas: the call does not shard)."""
    import numpy as np
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=100_000)
    ap.add_argument("--cpu-sample-pods", type=int, default=40_000)
    ap.add_argument("--c4-nodes", type=int, default=5000)
    ap.add_argument("--cpu-sample-sims", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-consolidation", action="store_true")
    ap.add_argument("--c5-pods", type=int, default=200_000)
    ap.add_argument("--cpu-sample-c5-pods", type=int, default=1000)
    ap.add_argument("--no-stress", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r1", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output, committed under profiles/)")
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
            # RCCL over xGMI: barriers, the max-over-ranks time and the
            # consolidation all-gather
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

    problem = synth.make_cm(n_pods=args.pods, seed=0x5EED0006 + rank)
    solver = Solver(local)
    t0 = time.perf_counter()
    solver.prepare(problem)
    prep_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(args.warmup):
        solver.run()

    kt = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solver.run()  # synchronous: returns after the stream's last event
        kt.append(solver.last_run_ms())
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    t1 = time.perf_counter()
    out, res = solver.fetch()
    fetch_ms = (time.perf_counter() - t1) * 1e3
    checks = problem.checks()
    ms_per_step = elapsed * 1e3 / args.steps
    value = checks * world / elapsed * args.steps

    feas_ms = sum(k[0] for k in kt) / len(kt)
    ffd_ms = sum(k[1] for k in kt) / len(kt)
    trunc_ms = sum(k[2] for k in kt) / len(kt)
    ab = algorithmic_bytes(res, problem, len(out["claims"]))
    kms = {"feas": feas_ms, "ffd": ffd_ms, "trunc": trunc_ms}
    dom = max(kms, key=kms.get)
    traffic = load_traffic(args.traffic_json)

    def roof(k):
        ach = ab[k] / (kms[k] * 1e-3) / 1e9
        return {"kernel": {"feas": "feas_kernel", "ffd": "ffd_kernel", "trunc": "trunc_kernel"}[k],
                "bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes": ab[k], "avg_ms": round(kms[k], 4)}

    roofline = roof(dom)
    roofline["traffic"] = traffic.get(dom)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "checks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {
            "workload": "CM: 100k pods x C2 synthetic IBM VPC catalog (198 profiles x 3 zones x "
                        "{on-demand, spot} = 1,188 offerings), 1 NodePool, 1% GPU pods, 10% nodeSelectors",
            "pods": len(problem.pods),
            "instance_types": len(problem.instance_types),
            "offerings": len(problem.offerings),
            "nodepools": len(problem.nodepools),
            "checks_per_step": checks,
            "parallelism": f"replicas{world}" if world > 1 else "single",
        },
        "solve_latency_ms": ms_per_step,
        "kernel_ms": {k: round(v, 4) for k, v in kms.items()},
        "prepare_ms_encode_plus_pcie_upload": round(prep_ms, 2),
        "fetch_decode_ms": round(fetch_ms, 2),
        "new_nodeclaims": len(out["claims"]),
        "pod_errors": len(out["errors"]),
        "queue_pops": int(res.pops),
        "ffd_candidates_scored": int(res.cand_evals),
        "ffd_candidates_full_check": int(res.cand_full),
        "ffd_phase_ms": {"sort": round(res.t_ffd_sort_ms, 2), "scan": round(res.t_ffd_scan_ms, 2),
                         "template": round(res.t_ffd_template_ms, 2)},
        "go_sort_emulation": {"fast": int(res.sorts_fast), "generic": int(res.sorts_generic)},
        "roofline": roofline,
        "roofline_feasibility_kernel": dict(roof("feas"), traffic=traffic.get("feas")),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample_pods)
    solver.close()
    if not args.no_consolidation:
        line["consolidation"] = bench_consolidation(args, rank, world, local, dist, device, barrier, max_over_ranks)
    if not args.no_stress:
        line["stress"] = bench_stress(args, rank, world, local, dist, device, barrier, max_over_ranks)
    if rank == 0 and world == 1:
        line["ranking"] = bench_ranking(args)
    if rank == 0:
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
