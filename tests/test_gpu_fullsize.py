"""Full-size parity at BASELINE.json's configs ("configs_untested").

Solve results are compared with the oracle bit for bit — the complete
result: every NodeClaim's pods, NodePool, truncated instance-type options,
requirements and requests, the existing-node placements and the unschedulable
pods — on both Solve kernels (single-wave ffd_wave.hip and the block kernel):
  CM 100k  (configs[1], the headline)  live oracle (~16 s CPU)
  C3 50k   (topology + affinity mix)   live oracle (~9 s CPU)
  C5 50k   (2000 types, 6 zones)       live oracle (~27 s CPU)
  C5 200k  (configs[4] at full size)   oracle digest committed in
           tests/golden/fullsize.json (the oracle takes ~6.5 min; generated
           by tests/golden/make_fullsize_golden.py)
The C5 200k static feasibility matrix is checked through size-independent
properties (each row inside its NodePool's instance types, the cheapest type
inside its row and the minimum of the row's OrderByPrice keys, shards
unioning to the whole) and exactly against the oracle on a 2000-pod sample.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from gpusched import abi, synth
from oracle import pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))


def gold():
    with open(os.path.join(HERE, "golden", "fullsize.json")) as f:
        return json.load(f)

pytestmark = pytest.mark.gpu


def digest(res):
    return hashlib.sha256(json.dumps(res, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


@pytest.fixture(scope="module", params=["wave", "block"])
def solver(request):
    from gpusched import lib
    s = lib.Solver(flags=abi.GS_CFG_BLOCK_SOLVE if request.param == "block" else 0)
    yield s
    s.close()


_cache = {}


def _case(name):
    if name not in _cache:
        p = {"cm_100k": synth.make_cm, "c3_50k": synth.make_c3,
             "c5_50k": lambda: synth.make_c5(n_pods=50_000)}[name]()
        st, want, raw = pyoracle.solve(p)
        assert st == abi.GS_OK
        want["_calls"] = (int(raw.claim_prefix), int(raw.node_prefix))
        _cache.clear()  # one full-size problem resident at a time
        _cache[name] = (p, want)
    return _cache[name]


def _compare(got, want):
    assert len(got["claims"]) == len(want["claims"])
    for i, (g, w) in enumerate(zip(got["claims"], want["claims"])):
        assert g == w, f"claim {i}"
    assert got["nodes"] == want["nodes"]
    assert got["errors"] == want["errors"]


@pytest.mark.parametrize("name", ["cm_100k", "c3_50k", "c5_50k"])
def test_fullsize_solve_matches_live_oracle(solver, name):
    p, want = _case(name)
    got, raw = solver.solve(p)
    _compare(got, want)
    # the kernels' first-fit counters equal the reference's CanAdd calls
    # (the roofline's algorithmic bytes are priced on them)
    assert (int(raw.claim_prefix), int(raw.node_prefix)) == want["_calls"]
    if name in gold():
        assert digest(got) == gold()[name]["sha256"]


def test_c5_200k_solve_matches_oracle_digest(solver):
    g = gold()["c5_200k"]
    p = synth.make_c5()
    got, _ = solver.solve(p)
    assert len(got["claims"]) == g["claims"] and len(got["errors"]) == g["errors"]
    assert sum(len(c["pods"]) for c in got["claims"]) == g["pods_on_claims"]
    assert digest(got) == g["sha256"]


@pytest.fixture(scope="module")
def c5_full():
    return synth.make_c5()


def test_c5_200k_static_matrix_properties(c5_full):
    from gpusched import lib
    p = c5_full
    s = lib.Solver()
    s.prepare(p)
    whole, _ = s.feasibility()
    rows, cheapest, keys = whole["rows"], whole["cheapest"], whole["cheapest_key"]
    P, T, W = rows.shape
    assert P == 200_000 and T == len(p.nodepools)
    # each row lies inside its NodePool's GetInstanceTypes list
    for t, np_ in enumerate(p.nodepools):
        b, c = np_["instance_types"]
        allowed = np.zeros(W, np.uint64)
        for i in p.it_refs[b:b + c]:
            allowed[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
        assert not np.any(rows[:, t, :] & ~allowed)
    # cheapest: in its row, -1 exactly on empty rows
    nonempty = rows.any(axis=2)
    assert np.array_equal(cheapest >= 0, nonempty)
    pi, ti = np.nonzero(cheapest >= 0)
    ci = cheapest[pi, ti].astype(np.int64)
    assert np.all((rows[pi, ti, ci >> 6] >> (ci & 63).astype(np.uint64)) & np.uint64(1))
    assert np.all(keys[~nonempty] == np.iinfo(np.int64).max)
    # shards over instance-type words union to the whole (3 uneven shards)
    acc = np.zeros_like(rows)
    best = np.full(keys.shape, np.iinfo(np.int64).max, dtype=np.int64)
    for lo, hi in [(0, 5), (5, 17), (17, W)]:
        part, _ = s.feasibility_shard(lo, hi)
        assert not np.any(part["rows"][:, :, :lo]) and not np.any(part["rows"][:, :, hi:])
        acc |= part["rows"]
        best = np.minimum(best, part["cheapest_key"].astype(np.int64))
    assert np.array_equal(acc, rows)
    assert np.array_equal(best, keys.astype(np.int64))
    s.close()


def test_c5_200k_static_matrix_sample_matches_oracle(c5_full):
    from gpusched import lib
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(200_000, size=2000, replace=False))
    idx = np.concatenate([[0, 1, 199_999], idx])
    sub = c5_full.with_pods(idx)
    st, want = pyoracle.feasibility(sub)
    assert st == abi.GS_OK
    s = lib.Solver()
    s.prepare(sub)
    got, _ = s.feasibility()
    s.close()
    assert np.array_equal(got["rows"], want["rows"])
    assert np.array_equal(got["cheapest"], want["cheapest"])
    assert np.array_equal(got["n_feasible_offerings"], want["n_feasible_offerings"])
    # and the sample's rows are the full matrix's rows for the same pods
    s = lib.Solver()
    s.prepare(c5_full)
    full, _ = s.feasibility()
    s.close()
    assert np.array_equal(full["rows"][idx], got["rows"])
