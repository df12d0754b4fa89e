"""c4_multi probe: the MULTI prefixes' simulation stats (pods re-solved, node
CanAdd evaluations, first-fit prefix, pops) and per-prefix sim time"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'karpenter-provider-ibm-cloud_amd'))
from gpusched import abi, synth  # noqa: E402
from gpusched.consolidation import ConsolidationInput  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

gen = synth.e2e_consolidation_cluster if "--e2e" in sys.argv else synth.make_c4
p = gen(n_nodes=5000)
cands = list(range(5000))
s = Solver(0)
for mode, name in ((abi.CONSOLIDATE_MULTI, "multi"), (abi.CONSOLIDATE_SINGLE, "single")):
    cin = ConsolidationInput(p, cands, mode=mode)
    s.consolidate(cin)
    for _ in range(3):
        t0 = time.perf_counter()
        res = s.consolidate_rerun(raw=True)
        wall = (time.perf_counter() - t0) * 1e3
    print(name, {"sims": res.n_commands, "pods_simulated": res.pods_simulated, "node_evals": res.node_evals,
                 "node_prefix": res.node_prefix, "pops": res.pops, "t_sim_ms": round(res.t_sim_ms, 3),
                 "t_feas_ms": round(res.t_feas_ms, 3), "wall_ms": round(wall, 2)}, flush=True)
# the largest MULTI prefix alone (EVAL of one set)
for m in (10, 50, 100):
    cin = ConsolidationInput(p, cands[:m], mode=abi.CONSOLIDATE_EVAL, sets=[(0, m)])
    s.consolidate(cin)
    res = s.consolidate_rerun(raw=True)
    print("prefix", m, {"pods": res.pods_simulated, "node_evals": res.node_evals, "node_prefix": res.node_prefix,
                        "pops": res.pops, "t_sim_ms": round(res.t_sim_ms, 3)}, flush=True)
s.close()
