"""Diagnostic: C5 (200k pods x 2,000 ITs x 6 zones x 2 capacity types) feasibility
kernel timing and, optionally, the full Solve."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "karpenter-provider-ibm-cloud_amd"))
from gpusched import synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
t0 = time.time()
p = synth.make_c5(n_pods=n)
print("gen_s", round(time.time() - t0, 1), "pods", len(p.pods), "its", len(p.instance_types), "offerings",
      len(p.offerings), flush=True)
s = Solver(0)
t0 = time.time()
s.prepare(p)
print("prepare_ms", round((time.time() - t0) * 1e3, 1), flush=True)
ts = []
for _ in range(5):
    f, r = s.feasibility()
    ts.append(r.t_kernel_ms)
print("feas_kernel_ms", [round(x, 3) for x in ts], "checks", r.checks, flush=True)
s.run()
print("solve_feas_kernel_ms (rows only)", round(s.last_run_ms()[0], 4), flush=True) if "--solve" not in sys.argv else None
if "--solve" in sys.argv:
    t0 = time.time()
    s.run()
    out, res = s.fetch()
    print("solve_ms", round((time.time() - t0) * 1e3, 1), "kernel_ms", s.last_run_ms(), "claims", len(out["claims"]),
          "errors", len(out["errors"]), "pops", res.pops, flush=True)
