"""Diagnostic: pod-loop segment cycles of one pod category (GS_CAT_SEG build,
GPUSCHED_LIB=libgpusched_seg<k>.so) on the CM workload (--c3: C3)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'karpenter-provider-ibm-cloud_amd'))
from gpusched import synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

p = synth.make_c3() if "--c3" in sys.argv else synth.make_cm()
s = Solver(0, 0)
s.prepare(p)
s.run()
out = (C.c_uint64 * 16)()
s.L.gs_debug_ctrl.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
s.L.gs_debug_ctrl(s.ctx, out, 16)
d, res = s.fetch()
n = max(int(out[12]), 1)
names = ["pop_record", "nodes", "sort", "scan_add", "new_claim", "scanA_lds", "scanB_exact", "tail"]
print(json.dumps({"lib": os.environ.get("GPUSCHED_LIB"), "ffd_ms": res.t_ffd_ms, "pods_in_category": int(out[12]),
                  "cycles_per_pod": {k: round(out[i] / n, 1) for i, k in enumerate(names)},
                  "total": round(sum(out[i] for i in range(8)) / n, 1)}))
