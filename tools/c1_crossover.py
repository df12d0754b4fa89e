"""C1's GPU/CPU crossover.

BASELINE configs[0] (C1: 500 pods x 8 fake profiles x 3 zones) is the
reference-sized Solve.  At that size the wave Solve is latency-bound (one
dependent pop after another on one wave) and the 1-core oracle restatement
is as fast or faster.  This measures both on the C1 catalog at growing pod
counts and reports the pod count where the GPU wins:

  gpu_ms   = gs_run wall per step (device-resident input, like bench.py's
             ms_per_step), median of --steps runs after 2 warmups
  cpu_ms   = the oracle's Solve (1 thread), its input build subtracted, the
             best of --cpu-reps runs (like bench.py's cpu_baseline)

Both results are compared (bit-exact) at every size.  Run on the GPU box:
  python tools/c1_crossover.py --out gpurun_out/c1_crossover.json
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-provider-ibm-cloud_amd"))
sys.path.insert(0, ROOT)

from gpusched import abi, synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="125,250,500,1000,2000,4000,8000,16000")
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from oracle import pyoracle  # the checker and the CPU baseline, never the product path

    rows = []
    solver = Solver(0)
    try:
        for n in [int(x) for x in args.sizes.split(",")]:
            p = synth.make_c1(n_pods=n)
            solver.prepare(p)
            for _ in range(2):
                solver.run()
            wall = []
            for _ in range(args.steps):
                t0 = time.perf_counter()
                solver.run()
                wall.append((time.perf_counter() - t0) * 1e3)
            got, res = solver.fetch()
            cpu = []
            want = None
            for _ in range(args.cpu_reps):
                t0 = time.perf_counter()
                st, want, raw = pyoracle.solve(p)
                cpu.append((time.perf_counter() - t0) * 1e3 - float(raw.t_encode_ms))
            row = {"pods": n, "gpu_ms": round(statistics.median(wall), 4), "gpu_min_ms": round(min(wall), 4),
                   "cpu_ms": round(min(cpu), 4), "claims": len(got["claims"]), "pops": int(res.pops),
                   "generic_sorts": int(res.sorts_generic), "fast_sorts": int(res.sorts_fast),
                   "bit_exact": bool(st == abi.GS_OK and got == want)}
            row["gpu_over_cpu"] = round(row["gpu_ms"] / row["cpu_ms"], 3) if row["cpu_ms"] > 0 else None
            rows.append(row)
            print(json.dumps(row), flush=True)
    finally:
        solver.close()
    cross = next((r["pods"] for r in rows if r["gpu_ms"] < r["cpu_ms"]), None)
    out = {"what": "C1 catalog (8 fake profiles x 3 zones, 1 NodePool) at growing pod counts: wave Solve gs_run "
                   "wall per step vs the 1-core oracle Solve (input build excluded)",
           "rows": rows, "crossover_pods": cross}
    print(json.dumps({"crossover_pods": cross}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
