"""Diagnostic: consolidation sweep wall-time breakdown on the C4 workload."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "karpenter-provider-ibm-cloud_amd"))
from gpusched import abi, synth  # noqa: E402
from gpusched.consolidation import ConsolidationInput  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

import gc
if "--after-cm" in sys.argv:
    cm = synth.make_cm()
    s0 = Solver(0)
    s0.prepare(cm)
    s0.run()
    out_cm = s0.fetch()
    s0.close()
p = synth.make_c4(n_nodes=5000)
s = Solver(0)
cin = ConsolidationInput(p, list(range(len(p.nodes))), mode=abi.CONSOLIDATE_SINGLE)
s.consolidate(cin)
for _ in range(3):
    s.consolidate_rerun(raw=True)
ts = []
if "--nogc" in sys.argv:
    gc.disable()
for _ in range(10):
    t0 = time.perf_counter()
    r = s.consolidate_rerun(raw=True)
    ts.append((time.perf_counter() - t0) * 1e3)
print({"all_ms": [round(x, 3) for x in ts], "wall_ms": sorted(ts)[len(ts) // 2], "feas": r.t_feas_ms, "sim": r.t_sim_ms, "trunc": r.t_truncate_ms,
       "fetch_decide": r.t_fetch_ms, "node_evals": r.node_evals, "node_prefix": r.node_prefix, "pops": r.pops})
