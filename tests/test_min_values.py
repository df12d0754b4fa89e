"""NodePool minValues, Strict policy (<U>
karpenter InstanceTypes.SatisfiesMinValues in filterInstanceTypesByRequirements
and Results.TruncateInstanceTypes; CRD field charts/crds/
karpenter.sh_nodepools.yaml:281).

CPU known-answer tests pin the oracle's restatement on hand-derived cases:
a NodeClaim keeps a pod only while its options still cover the minimum
number of distinct values per key; a NodePool whose options miss it is
skipped; a NodeClaim whose top 60 by price miss it is dropped after the
Solve and its pods become pod errors.  GPU tests require the HIP Solve (both
kernels) and the static matrix to equal the oracle bit for bit.  minValues
is upstream behaviour recalled, not vendored: parity unpinned.
"""
import numpy as np
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

FAM = synth.FAMILY_KEY
ITK = synth.IT_KEY
Z = "topology.kubernetes.io/zone"


def _base(np_reqs, pods=((500, None),), profiles=None):
    b = ProblemBuilder()
    profs = profiles or synth.FAKE_PROFILES
    synth.build_catalog(b, profs, synth.FAKE_ZONES, spot=False, prices=synth.price_table(profs))
    b.add_nodepool("default", requirements=np_reqs)
    for i, (cpu, sel) in enumerate(pods):
        b.add_pod(f"p{i}", 0, {"cpu": cpu, "memory": 1 << 30, "pods": 1000}, node_selector=sel or {})
    return b


def _solve(b):
    st, res, _ = pyoracle.solve(b.build())
    assert st == abi.GS_OK
    return res


def _fam_line(res, i=0):
    return [ln for ln in res["claims"][i]["requirements"].split("\n") if ln.startswith(FAM + "|")]


def test_satisfied_min_values_are_kept_in_the_requirements():
    res = _solve(_base([(FAM, "In", ["bx2", "cx2", "mx2"], 2)], pods=[(500, None)] * 3))
    assert [c["pods"] for c in res["claims"]] == [[0, 1, 2]] and not res["errors"]
    assert _fam_line(res) == [FAM + "|In|bx2,cx2,mx2|-|-|2"]


def test_pod_selector_below_the_minimum_cannot_join():
    # the pod pins one family: the NodeClaim's options would hold one family
    res = _solve(_base([(FAM, "In", ["bx2", "cx2", "mx2"], 2)], pods=[(500, {FAM: "bx2"})]))
    assert res["errors"] == [0] and not res["claims"]


def test_requests_that_narrow_below_the_minimum():
    # 3.5 vCPU fits the types with >= 4 vCPU (allocatable vcpu*1000 - 200 m);
    # 3.7 vCPU still does
    its = synth.FAKE_PROFILES
    n4 = sum(1 for p in its if p[1] >= 4)
    res = _solve(_base([(ITK, "Exists", [], n4)], pods=[(3500, None), (200, None)]))
    assert not res["errors"] and [c["pods"] for c in res["claims"]] == [[0, 1]]
    res = _solve(_base([(ITK, "Exists", [], n4 + 1)], pods=[(3500, None)]))
    assert res["errors"] == [0]


def test_second_pod_would_break_the_minimum_opens_a_new_nodeclaim():
    # p0 (1.5 vCPU) keeps every type with allocatable >= 1.5 vCPU; with p1
    # (1.5 vCPU) only the >= 4-vCPU types remain, one short of the minimum
    its = synth.FAKE_PROFILES
    n4 = sum(1 for p in its if p[1] >= 4)
    res = _solve(_base([(ITK, "Exists", [], n4 + 1)], pods=[(1500, None), (1500, None)]))
    assert [c["pods"] for c in res["claims"]] == [[0], [1]] and not res["errors"]


def test_nodepool_below_the_minimum_is_skipped():
    n = len(synth.FAKE_PROFILES)
    res = _solve(_base([(ITK, "Exists", [], n + 1)], pods=[(500, None)]))
    assert res["errors"] == [0] and not res["claims"]
    # instance types carry no zone value: any zone minimum is unsatisfiable
    res = _solve(_base([(Z, "In", synth.FAKE_ZONES, 1)], pods=[(500, None)]))
    assert res["errors"] == [0]


def test_truncation_drops_the_nodeclaim():
    st, res, _ = pyoracle.solve(synth.min_values_truncation())
    assert st == abi.GS_OK
    assert not res["claims"] and res["errors"] == [0, 1, 2]
    # with 58 cheap types the top 60 include both mx2 types
    st, res, _ = pyoracle.solve(synth.min_values_truncation(n_cheap=58))
    assert st == abi.GS_OK and not res["errors"] and len(res["claims"]) == 1


def test_static_matrix_rows_under_the_minimum_are_empty():
    b = _base([(FAM, "In", ["bx2", "cx2", "mx2"], 2)], pods=[(500, {FAM: "bx2"}), (500, None)])
    st, f = pyoracle.feasibility(b.build())
    assert st == abi.GS_OK
    assert not f["rows"][0].any() and f["cheapest"][0][0] == -1
    assert f["rows"][1].any()


def test_refusals_and_pass_through():
    b = _base([])
    b.add_pod("x", 0, {"cpu": 1}, required_terms=[[(FAM, "In", ["bx2"], 1)]])
    assert pyoracle.solve(b.build())[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(_base([(FAM, "In", ["bx2", "cx2"], 2)]).build())[0] == abi.GS_OK


@pytest.mark.parametrize("seed", range(40))
def test_oracle_and_encoder_accept_random_min_values(seed):
    p = synth.random_min_values(seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK, msg


def test_random_min_values_bind():
    # the generator exercises the constraint: some pods fail or split claims
    # only because of minValues
    errs = 0
    for s in range(40):
        st, res, _ = pyoracle.solve(synth.random_min_values(s))
        errs += len(res["errors"])
    assert errs > 0


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module", params=["wave", "block", "hbm"])
def solver(request):
    from gpusched.lib import Solver
    s = Solver(0, {"wave": 0, "block": abi.GS_CFG_BLOCK_SOLVE, "hbm": abi.GS_CFG_CLAIMS_HBM}[request.param])
    yield s
    s.close()


def _check(solver, p):
    from test_gpu_parity import _diff
    st, want, _ = pyoracle.solve(p)
    assert st == abi.GS_OK
    got, _ = solver.solve(p)
    d = _diff(got, want)
    assert d is None, d


def _check_feas(solver, p):
    st, want = pyoracle.feasibility(p)
    assert st == abi.GS_OK
    solver.prepare(p)
    got, _ = solver.feasibility()
    assert np.array_equal(got["rows"], want["rows"])
    assert np.array_equal(got["cheapest"], want["cheapest"])
    assert np.array_equal(got["n_feasible_offerings"], want["n_feasible_offerings"])


@pytest.mark.gpu
def test_gpu_min_values_kats(solver):
    n4 = sum(1 for p in synth.FAKE_PROFILES if p[1] >= 4)
    _check(solver, _base([(FAM, "In", ["bx2", "cx2", "mx2"], 2)], pods=[(500, None)] * 3).build())
    _check(solver, _base([(FAM, "In", ["bx2", "cx2", "mx2"], 2)], pods=[(500, {FAM: "bx2"})]).build())
    _check(solver, _base([(ITK, "Exists", [], n4 + 1)], pods=[(1500, None), (1500, None)]).build())
    _check(solver, synth.min_values_truncation())
    _check(solver, synth.min_values_truncation(n_cheap=58))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100))
def test_gpu_min_values_random(solver, seed):
    _check(solver, synth.random_min_values(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(5))
def test_gpu_min_values_random_many_pods(solver, seed):
    _check(solver, synth.random_min_values(500 + seed, n_pods=400))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_gpu_min_values_static_matrix(solver, seed):
    _check_feas(solver, synth.random_min_values(seed))
