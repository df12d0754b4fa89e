"""Full-size consolidation goldens for BASELINE configs[3] (C4, 5,000 state
nodes): the sha256 of the oracle's commands for every SingleNodeConsolidation
candidate of the c4 / c4_mixed / c4_e2e sweeps (5,000 simulations each) and
for all 100 MultiNodeConsolidation prefix simulations candidates[0:j+2] of
the c4 and c4_e2e clusters -- the same clusters and command lists as bench.py's
consolidation legs.  Run here (CPU, a process pool):

    python tests/golden/make_c4_golden.py [names] [--procs N]

Writes tests/golden/c4_consolidation.json; tests/test_c4_fullsize.py compares
the simulation kernel's command digests (narrow and wide shapes) with it.
The inputs are the deterministic generators of gpusched.synth."""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-provider-ibm-cloud_amd"))
from gpusched import abi, synth  # noqa: E402
from gpusched.consolidation import ConsolidationInput  # noqa: E402

N_NODES = 5000
N_PREFIXES = 100
# name -> (generator, kwargs, mode); the bench legs' clusters (bench.py specs)
SWEEPS = {
    "c4_single": ("make_c4", {}, "single"),
    "c4_mixed_single": ("make_c4", {"util": (0.9, 0.99), "full_frac": 0.5, "big_frac": 1.0, "pack": True}, "single"),
    "c4_e2e_single": ("e2e_consolidation_cluster", {}, "single"),
    "c4_multi": ("make_c4", {}, "multi"),
    "c4_e2e_multi": ("e2e_consolidation_cluster", {}, "multi"),
}

_CACHE = {}


def cluster(name):
    gen, kw, _ = SWEEPS[name]
    key = (gen, json.dumps(kw, sort_keys=True))
    if key not in _CACHE:
        _CACHE.clear()
        _CACHE[key] = getattr(synth, gen)(n_nodes=N_NODES, **kw)
    return _CACHE[key]


def _job(args):
    name, cands, mode, sets = args
    from oracle import pyoracle
    st, cmds, _, _ = pyoracle.consolidate(ConsolidationInput(cluster(name), cands, mode=mode, sets=sets))
    assert st == abi.GS_OK, st
    return cmds


def digest(cmds):
    return hashlib.sha256(json.dumps(cmds, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


def oracle_commands(name, pool, procs):
    """the command list the product's sweep returns: SINGLE, one command per
    candidate in candidate order; MULTI, multi[j] = candidates[0:j+2]"""
    _, _, kind = SWEEPS[name]
    if kind == "single":
        chunk = 50
        jobs = [(name, list(range(i, min(i + chunk, N_NODES))), abi.CONSOLIDATE_SINGLE, None)
                for i in range(0, N_NODES, chunk)]
    else:
        jobs = [(name, list(range(N_PREFIXES + 1)), abi.CONSOLIDATE_EVAL, [(0, j + 2)])
                for j in range(N_PREFIXES)]
    out = []
    for cmds in pool.imap(_job, jobs, chunksize=1):
        out.extend(cmds)
    return out


def summary(cmds):
    dec = {}
    for c in cmds:
        dec[str(c["decision"])] = dec.get(str(c["decision"]), 0) + 1
    return dec


def main(argv):
    procs = 8
    if "--procs" in argv:
        procs = int(argv[argv.index("--procs") + 1])
        del argv[argv.index("--procs"):argv.index("--procs") + 2]
    names = argv or list(SWEEPS)
    path = os.path.join(HERE, "c4_consolidation.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    ctx = mp.get_context("fork")
    for name in names:
        t0 = time.time()
        with ctx.Pool(procs) as pool:
            cmds = oracle_commands(name, pool, procs)
        out[name] = {"n_commands": len(cmds), "decisions": summary(cmds), "sha256": digest(cmds),
                     "oracle_s": round(time.time() - t0, 1), "procs": procs}
        print(name, out[name], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
