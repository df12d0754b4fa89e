"""Full-size Solve goldens: sha256 of the oracle's result on the BASELINE
configs whose oracle run is too long for a GPU test (C5 200k: minutes of
CPU).  Run here (CPU): python tests/golden/make_fullsize_golden.py [names]
Writes tests/golden/fullsize.json; tests/test_gpu_fullsize.py compares the
product's result digest with it.  The inputs are the deterministic synthetic
generators of gpusched.synth (numpy default_rng with fixed seeds)."""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-provider-ibm-cloud_amd"))
from gpusched import synth  # noqa: E402
from oracle import pyoracle  # noqa: E402

CONFIGS = {
    "c5_200k": lambda: synth.make_c5(),
    "cm_100k": lambda: synth.make_cm(),
    "c3_50k": lambda: synth.make_c3(),
}


def digest(res):
    return hashlib.sha256(json.dumps(res, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


def main(names):
    path = os.path.join(HERE, "fullsize.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        p = CONFIGS[name]()
        t0 = time.time()
        st, res, _ = pyoracle.solve(p)
        assert st == 0, st
        out[name] = {"claims": len(res["claims"]), "errors": len(res["errors"]),
                     "pods_on_claims": sum(len(c["pods"]) for c in res["claims"]),
                     "sha256": digest(res), "oracle_s": round(time.time() - t0, 1)}
        print(name, out[name], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS))
