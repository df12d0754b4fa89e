"""Quick GPU-vs-oracle parity probe of one library build (GPUSCHED_LIB):
prints the first difference per problem.  Diagnostic, not a test."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'karpenter-provider-ibm-cloud_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
from gpusched import synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402
from oracle import pyoracle  # noqa: E402
from test_gpu_parity import _diff  # noqa: E402

flags = 1 if "--block" in sys.argv else 0
s = Solver(0, flags)
probs = [("c1", synth.make_c1())] + [(f"rand{k}", synth.random_problem(k)) for k in range(20)] + \
        [(f"many{k}", synth.random_problem(1000 + k, n_pods=400, with_nodes=False)) for k in range(5)]
bad = 0
for name, p in probs:
    st, want, _ = pyoracle.solve(p)
    got, _ = s.solve(p)
    d = _diff(got, want)
    if d:
        bad += 1
        print(name, d[:300])
print(os.environ.get("GPUSCHED_LIB", "libgpusched.so"), "mismatches", bad, "of", len(probs))
