"""Diagnostic: FFD kernel phase breakdown on the CM workload (--c1 / --c2 / --c3 / --c5 / --e2e: those workloads).

default build: barrier-to-barrier wall-clock timers (Ctrl.dbg);
`make tl` build + --tl: shader cycles per pod-loop segment (GS_FFD_TL)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'karpenter-provider-ibm-cloud_amd'))
from gpusched import synth  # noqa: E402
from gpusched.lib import Solver  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
if "--c1" in sys.argv:
    p = synth.make_c1()
elif "--c3" in sys.argv:
    p = synth.make_c3()
elif "--e2e" in sys.argv:
    p = synth.e2e_deployments(n_deployments=60, replicas=500)
elif "--c5" in sys.argv:
    p = synth.make_c5(n_pods=int(args[0]) if args else 200000)
elif "--c2" in sys.argv:
    p = synth.make_c2()
else:
    p = synth.make_cm(n_pods=int(args[0]) if args else 100000)
s = Solver(0, 1 if "--block" in sys.argv else 0)
s.prepare(p)
s.run()
out = (C.c_uint64 * 16)()
s.L.gs_debug_ctrl.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
s.L.gs_debug_ctrl(s.ctx, out, 16)
d, res = s.fetch()
base = {"ffd_ms": res.t_ffd_ms, "pops": res.pops, "claims": len(d['claims']), "cand_evals": res.cand_evals,
        "cand_full": res.cand_full, "sorts_fast": res.sorts_fast, "sorts_generic": res.sorts_generic}
if "--tl" in sys.argv and "--block" not in sys.argv:
    names = ["pop_record", "nodes", "sort", "scan_add", "new_claim", "scanA_lds", "scanB_exact", "tail"]
    base["cycles_per_pop"] = {n: round(out[i] / max(res.pops, 1), 1) for i, n in enumerate(names) if n != "-"}
    base["cycles_per_pop_total"] = round(sum(out[i] for i in range(8)) / max(res.pops, 1), 1)
    base["generic_sort_cycles_per_pop"] = round(out[8] / max(res.pops, 1), 1)
    base["cycles_per_generic_sort"] = round(out[8] / max(res.sorts_generic, 1), 1)
    base["fast_accepts"] = out[15]
    if "--sorttl" in sys.argv:  # GS_SORT_TL build: the generic sort's parts (shader cycles per generic sort)
        base["generic_sort_parts_per_sort"] = {n: round(out[9 + i] / max(res.sorts_generic, 1), 1) for i, n in enumerate(
            ["seq_breakpatterns", "uniform", "pivot", "partial_insertion", "partition_equal", "partition", "frames"])}
    if "--sorttl2" in sys.argv:  # GS_SORT_TL2 build: the wave partition's parts (shader cycles per generic sort)
        base["partition_parts_per_sort"] = {n: round(out[i] / max(res.sorts_generic, 1), 1) for i, n in enumerate(
            ["swap_in", "count_split", "lists", "swaps_out"])}
    base["exact_cands_nonsimple"] = out[9]
    base["exact_batches"] = out[10]
    base["exact_wins"] = out[11]
    base["nonsimple_pops"] = out[12]
    base["rotations"] = out[13]
    base["mean_rotation_len"] = round(out[14] / max(out[13], 1), 1)
elif "--tl" in sys.argv:
    names = ["to_top", "publish", "pop", "stage_nodes", "sort_decide", "rotate", "chunk_lds", "reduce2", "exact",
             "winner_end", "new_claim"]
    base["cycles_per_pop"] = {n: round(out[i] / max(res.pops, 1), 1) for i, n in enumerate(names)}
    base["cycles_per_pop_total"] = round(sum(out[i] for i in range(11)) / max(res.pops, 1), 1)
    base["last_wave_lateness_vs_wave0"] = round(out[11] / max(res.pops, 1), 1)
    base["last_wave_hist_w0_w1_w2_w3plus"] = [out[12], out[13], out[14], out[15]]
else:
    # single-wave kernel: run-mode counters (pods placed in runs, entries, exits by cause)
    base["runs"] = {n: int(out[8 + i]) for i, n in enumerate(["pods", "entries", "x_pivot", "x_window", "x_spec",
                                                            "x_scan"])}
    # dbg[14]: s_memtime ticks in run mode (GS_RUN_TL builds), else run-mode exact batches
    base["runs"]["exact_batches_or_run_ticks"] = int(out[14])
    base["runs"]["batches"] = int(out[6])
    base["runs"]["batch_pods"] = int(out[5])
    base["runs"]["batch_ticks_all_or_sort_decide"] = int(out[3])
    base["runs"]["batch_ticks_placed_or_pop"] = int(out[4])
    if "--cat" in sys.argv:  # GS_CAT_TL build: shader cycles per pod category
        names = ["run_mode", "simple_claim", "-", "other_claim", "new_claim", "failed", "existing_node", "unknown"]
        base["categories"] = {n: {"pods": int(out[8 + i]), "mcycles": round(out[i] / 1e6, 2),
                                  "cycles_per_pod": round(out[i] / max(out[8 + i], 1), 1)}
                              for i, n in enumerate(names) if n != "-"}
        del base["runs"]
    base.update({"sort": res.t_ffd_sort_ms, "scan": res.t_ffd_scan_ms, "tmpl": res.t_ffd_template_ms,
                 "scan_tid0_work_ms": out[0] * 1e-5, "scan_wait_ms": out[1] * 1e-5, "chunks": out[2],
                 "sort_decide_ms": out[3] * 1e-5, "pop_ms": out[4] * 1e-5, "end_to_pop_ms": out[5] * 1e-5,
                 "fast_accepts": out[15], "shader_clock_mhz": out[7] / (res.t_ffd_ms * 1e3)})
print(json.dumps(base))
