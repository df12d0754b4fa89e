"""Diagnostic: FFD kernel phase breakdown (barrier-to-barrier timers)."""
import sys, json, ctypes as C
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'karpenter-provider-ibm-cloud_amd'))
from gpusched import synth
from gpusched.lib import Solver
p = synth.make_cm(n_pods=int(sys.argv[1]) if len(sys.argv)>1 else 100000)
s = Solver(0); s.prepare(p); s.run()
out = (C.c_uint64*16)()
s.L.gs_debug_ctrl.argtypes=[C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
s.L.gs_debug_ctrl(s.ctx, out, 16)
d, res = s.fetch()
print(json.dumps({"ffd_ms": res.t_ffd_ms, "sort": res.t_ffd_sort_ms, "scan": res.t_ffd_scan_ms, "tmpl": res.t_ffd_template_ms,
  "scan_tid0_work_ms": out[0]*1e-5, "scan_wait_ms": out[1]*1e-5, "chunks": out[2], "sort_decide_ms": out[3]*1e-5, "pop_ms": out[4]*1e-5, "shader_clock_mhz": out[7] / (res.t_ffd_ms * 1e3),
  "pops": res.pops, "claims": len(d['claims']), "cand_evals": res.cand_evals, "cand_full": res.cand_full,
  # GS_FFD_DIAG build only: per-wave cycles to record test / cursor probe / option words, tid0 chunk cycles
  "wave_rec_cyc": out[8] / max(out[11], 1), "wave_probe_cyc": out[9] / max(out[12], 1), "wave_words_cyc": out[10] / max(out[12], 1),
  "waves_rec": out[11], "waves_full": out[12], "chunk_cyc_tid0": out[13] / max(out[2], 1)}))
