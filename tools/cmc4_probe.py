"""Probe: provisioning Solve of CM-distribution pods into C4's 5,000 state
nodes on the single-wave and block kernels (device time per run)."""
import sys
import time

sys.path.insert(0, "karpenter-provider-ibm-cloud_amd")
from gpusched import abi, synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

for n_pending in [int(x) for x in sys.argv[1:]] or [20000]:
    p = synth.make_c4(n_nodes=5000, n_pending=n_pending)
    for name, flags in (("wave", 0), ("block", abi.GS_CFG_BLOCK_SOLVE)):
        s = Solver(0, flags)
        try:
            s.prepare(p)
            t0 = time.perf_counter()
            s.run()
            wall = (time.perf_counter() - t0) * 1e3
            _, res = s.fetch()
            print(f"pods {n_pending} {name}: run {wall:.1f} ms kernels {s.last_run_ms()} pops {res.pops} "
                  f"node_prefix {res.node_prefix} claim_prefix {res.claim_prefix}", flush=True)
        finally:
            s.close()
