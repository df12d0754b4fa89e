"""Launch-time re-filter: CloudProvider.Create's instance-type filter
(reference pkg/cloudprovider/cloudprovider.go:322-346), GetInstanceTypes'
NodePool filter (:574-577), instanceTypes[0] (vpc/instance/provider.go:215-221)
and ResolveCapacityType (common/capacitytype/capacitytype.go:27-42).

CPU tests pin the oracle against the reference's own cases
(capacitytype_test.go:30-169, cloudprovider_test.go:686-798) and check its
internal invariants; GPU tests compare gs_create_filter with the oracle bit
for bit (three bitsets, selected index, capacity type) on the same KATs, on
randomised catalogs exercising the full requirement algebra
(In/NotIn/Exists/DoesNotExist/Gt/Lt, custom and well-known keys, label-key
normalisation) and on the NodeClaims a Solve emits.
"""
import json
import os

import numpy as np
import pytest

from gpusched import abi
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "reference_kats.json")) as f:
    KATS = json.load(f)

GI = 1 << 30
ZONE, CT, ITK = "topology.kubernetes.io/zone", "karpenter.sh/capacity-type", "node.kubernetes.io/instance-type"


def _kat_problem(case):
    """capacitytype_test.go: instance types carrying only offerings"""
    b = ProblemBuilder()
    for k, offs in enumerate(case["types"]):
        b.add_instance_type(f"it-{k}", [], {}, {}, [(z, ct, p, av) for ct, z, p, av in offs])
    b.add_claim_query(case["requirements"] or [])
    return b.build()


CT_CASES = KATS["resolve_capacity_type"]["cases"]


@pytest.mark.parametrize("case", CT_CASES, ids=[c["name"] for c in CT_CASES])
def test_resolve_capacity_type_kats(case):
    p = _kat_problem(case)
    st, got = pyoracle.resolve_capacity_type(p, 0, list(range(len(case["types"]))))
    assert st == abi.GS_OK
    assert got == (abi.GS_CAPACITY_SPOT if case["want"] == "spot" else abi.GS_CAPACITY_ON_DEMAND)


def _test_instance_type(b, name="test-instance-type"):
    """getTestInstanceType (cloudprovider_test.go:254-284)"""
    return b.add_instance_type(name, [(ITK, "In", [name]), (CT, "In", ["on-demand"]), (ZONE, "In", ["us-south-1"])],
                               {"cpu": 4000, "memory": 16 * GI * 1000, "pods": 110000},
                               {"cpu": 100, "memory": GI * 1000}, [("us-south-1", "on-demand", 1.0, True)])


def _git_problem(case):
    b = ProblemBuilder()
    if case["n_types"] >= 1:
        _test_instance_type(b)
    if case["n_types"] >= 2:  # second type: no requirements, no offerings
        b.add_instance_type("test-instance-type-2", [], {"cpu": 8000, "memory": 32 * GI * 1000}, {}, [])
    b.add_claim_query([])  # NodePool without requirements
    return b.build()


GIT_CASES = KATS["get_instance_types_counts"]["cases"]


@pytest.mark.parametrize("case", GIT_CASES, ids=[c["name"] for c in GIT_CASES])
def test_get_instance_types_count_kats(case):
    st, out = pyoracle.create_filter(_git_problem(case))
    assert st == abi.GS_OK
    assert len(out[0]["requirements"]) == case["want"]


# ------------------------------------------------------------ random catalogs
CUSTOM = "example.com/team"


def random_catalog(seed, n_types=150, n_claims=40):
    """IBM-shaped catalog plus the corners of the requirement algebra"""
    rng = np.random.default_rng(seed)
    zones = ["us-south-1", "us-south-2", "us-south-3"]
    fams = ["bx2", "cx2", "mx2", "gx2", "ux2"]
    b = ProblemBuilder()
    names = []
    for i in range(n_types):
        fam = fams[rng.integers(len(fams))]
        cpu = int(rng.choice([2, 4, 8, 16, 32, 48]))
        mem = cpu * int(rng.choice([2, 4, 8]))
        name = f"{fam}-{cpu}x{mem}-{i}"
        names.append(name)
        reqs = [(ITK, "In", [name]), ("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "s390x"]))]),
                ("karpenter-ibm.sh/instance-family", "In", [fam]),
                ("karpenter-ibm.sh/instance-cpu", "In", [str(cpu)])]
        u = rng.random()
        if u < 0.08:
            reqs.append((CUSTOM, "In", [str(rng.choice(["a", "b"]))]))  # custom key: must be defined by the claim
        elif u < 0.14:
            reqs.append((CUSTOM, "NotIn", ["a"]))  # custom NotIn: exempt
        elif u < 0.18:
            reqs.append((CUSTOM, "DoesNotExist", []))
        elif u < 0.22:
            reqs.append(("beta.kubernetes.io/os", "In", ["linux"]))  # normalised to kubernetes.io/os
        elif u < 0.25:
            reqs.append((ZONE, "In", [zones[rng.integers(3)]]))  # zone pinned on the type itself
        offs = []
        for z in zones:
            for ct in ("on-demand", "spot"):
                if rng.random() < 0.75:
                    offs.append((z, ct, float(rng.integers(1, 400)) / 100, bool(rng.random() < 0.85)))
        overhead = {"cpu": 100 + 50 * int(rng.integers(0, 3)), "memory": GI * 1000}
        if rng.random() < 0.03:
            overhead["cpu"] = cpu * 1000 + 500  # Allocatable() < 0: never fits
        b.add_instance_type(name, reqs, {"cpu": cpu * 1000, "memory": mem * GI * 1000, "pods": 110000},
                            overhead, offs)
    for q in range(n_claims):
        reqs = []
        u = rng.random()
        if u < 0.5:
            k = min(int(rng.integers(1, 60)), n_types)
            reqs.append((ITK, "In", list(rng.choice(names, size=k, replace=False))))
        if rng.random() < 0.5:
            reqs.append((CT, "In", list(rng.choice(["spot", "on-demand"], size=int(rng.integers(1, 3)), replace=False))))
        if rng.random() < 0.4:
            reqs.append((ZONE, str(rng.choice(["In", "NotIn"])), list(rng.choice(zones, size=int(rng.integers(1, 3)),
                                                                                   replace=False))))
        if rng.random() < 0.25:
            reqs.append(("karpenter-ibm.sh/instance-cpu", str(rng.choice(["Gt", "Lt", "Gte", "Lte"])), [str(rng.choice([4, 8, 16]))]))
        if rng.random() < 0.15:
            reqs.append(("karpenter-ibm.sh/instance-cpu", "Gt", ["2"]))
            reqs.append(("karpenter-ibm.sh/instance-cpu", "Lt", ["3"]))  # bounds cross: DoesNotExist
        if rng.random() < 0.2:
            reqs.append((CUSTOM, str(rng.choice(["In", "Exists", "NotIn", "DoesNotExist"])), ["a"]))
        if rng.random() < 0.2:
            reqs.append(("failure-domain.beta.kubernetes.io/zone", "Exists", []))
        if rng.random() < 0.1:
            reqs.append(("karpenter-ibm.sh/instance-family", "In", ["bx2", "cx2"]))
            reqs.append(("karpenter-ibm.sh/instance-family", "NotIn", ["cx2"]))  # repeated key: Add intersects
        if rng.random() < 0.1:
            reqs.append(("kubernetes.io/os", "NotIn", ["windows"]))
        req = {"cpu": int(rng.integers(0, 40)) * 500, "memory": int(rng.integers(0, 64)) * GI * 1000}
        if rng.random() < 0.1:
            req["nvidia.com/gpu"] = 1000  # no type has it: nothing fits
        if rng.random() < 0.1:
            req = {}
        b.add_claim_query([(k, op, [str(v) for v in vals]) for k, op, vals in reqs], req)
    return b.build()


@pytest.mark.parametrize("seed", range(6))
def test_oracle_invariants(seed):
    p = random_catalog(seed, n_types=80, n_claims=20)
    st, out = pyoracle.create_filter(p)
    assert st == abi.GS_OK
    for q in out:
        assert set(q["compatible"]) <= set(q["requirements"])
        assert q["selected"] == (q["compatible"][0] if q["compatible"] else -1)
        if not q["compatible"]:
            assert q["capacity_type"] == abi.GS_CAPACITY_ON_DEMAND
    # the corners are exercised: some claims keep nothing, some keep types
    assert any(q["compatible"] for q in out) and any(not q["compatible"] for q in out)


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def solver():
    from gpusched import lib
    s = lib.Solver()
    yield s
    s.close()


def _same(got, want):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CT_CASES, ids=[c["name"] for c in CT_CASES])
def test_gpu_resolve_capacity_type_kats(solver, case):
    """through Create's filter: ResolveCapacityType over the compatible list
    gives the reference's answer for every case (an unavailable offering
    drops the type, and an empty list resolves to on-demand)"""
    p = _kat_problem(case)
    got = solver.create_filter(p)
    assert got[0]["capacity_type"] == (abi.GS_CAPACITY_SPOT if case["want"] == "spot" else abi.GS_CAPACITY_ON_DEMAND)
    _same(got, pyoracle.create_filter(p)[1])


@pytest.mark.gpu
@pytest.mark.parametrize("case", GIT_CASES, ids=[c["name"] for c in GIT_CASES])
def test_gpu_get_instance_types_count_kats(solver, case):
    p = _git_problem(case)
    got = solver.create_filter(p)
    assert len(got[0]["requirements"]) == case["want"]
    _same(got, pyoracle.create_filter(p)[1])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_gpu_create_filter_parity(solver, seed):
    n_types = [150, 1, 63, 64, 65, 300, 1188, 150, 257, 511, 150, 150, 2000, 700, 129, 150][seed]
    n_claims = [40, 5, 30, 30, 30, 60, 100, 1, 40, 40, 200, 0, 20, 80, 30, 40][seed]
    p = random_catalog(100 + seed, n_types, n_claims)
    want = pyoracle.create_filter(p)[1]
    got = solver.create_filter(p)
    _same(got, want)


@pytest.mark.gpu
def test_gpu_create_filter_refusals(solver):
    from gpusched import lib
    b = ProblemBuilder()
    _test_instance_type(b)
    b.add_claim_query([("karpenter-ibm.sh/instance-cpu", "Gt", ["x"])])
    with pytest.raises(lib.GpuSchedError) as e:
        solver.create_filter(b.build())
    assert e.value.status == abi.GS_E_INVALID
    # minValues: Compatible ignores it (cloudprovider.go:321-325)
    b = ProblemBuilder()
    _test_instance_type(b)
    b.add_claim_query([(ITK, "In", ["test-instance-type"], 2)])
    b2 = ProblemBuilder()
    _test_instance_type(b2)
    b2.add_claim_query([(ITK, "In", ["test-instance-type"])])
    got, want = solver.create_filter(b.build()), solver.create_filter(b2.build())
    assert repr(got) == repr(want)


def claim_queries_from_solve(p, res, builder):
    """NodeClaimTemplate.ToNodeClaim: the claim's requirements (canonical
    text) plus instance-type In[its truncated options], and its requests"""
    names = [p.strings[i] for i in p.instance_types["name"]]
    ops = {"In": "In", "NotIn": "NotIn", "Exists": "Exists", "DoesNotExist": "DoesNotExist"}
    for c in res["claims"]:
        reqs = []
        for line in c["requirements"].split("\n") if c["requirements"] else []:
            key, op, vals, gt, lt, _mv = line.split("|")
            vals = vals.split(",") if vals else []
            if key == ITK:
                continue
            if op == "Exists" and (gt != "-" or lt != "-"):
                pass  # bounds only
            else:
                reqs.append((key, ops[op], vals))
            if gt != "-":
                reqs.append((key, "Gt", [gt]))
            if lt != "-":
                reqs.append((key, "Lt", [lt]))
        reqs.append((ITK, "In", [names[i] for i in c["its"]]))
        builder.add_claim_query(reqs, c["requests"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_create_filter_after_solve(solver, seed):
    """the NodeClaims a Solve emits, re-filtered at launch: bit-exact with the
    oracle, every kept type is one of the claim's options, and every claim
    keeps at least one (the Solve only opens claims some option can launch)"""
    from gpusched import synth
    p = synth.random_problem(seed, n_pods=300, with_nodes=False, with_limits=False)
    res, _ = solver.solve(p)
    if not res["claims"]:
        pytest.skip("no claims")
    p2 = p.extended(lambda b: claim_queries_from_solve(p, res, b))
    got = solver.create_filter(p2)
    _same(got, pyoracle.create_filter(p2)[1])
    for c, g in zip(res["claims"], got):
        assert set(g["compatible"]) <= set(c["its"])
        assert g["n_compatible"] >= 1 and g["selected"] in c["its"]


@pytest.mark.parametrize("seed", range(4))
def test_oracle_create_filter_after_oracle_solve(seed):
    """the same chain through the oracle alone (CPU)"""
    from gpusched import synth
    p = synth.random_problem(seed, n_pods=300, with_nodes=False, with_limits=False)
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and res["claims"]
    p2 = p.extended(lambda b: claim_queries_from_solve(p, res, b))
    st, out = pyoracle.create_filter(p2)
    assert st == abi.GS_OK
    for c, g in zip(res["claims"], out):
        assert set(g["compatible"]) <= set(c["its"])
        assert g["n_compatible"] >= 1 and g["selected"] in c["its"]


@pytest.mark.gpu
def test_gpu_create_filter_rejects_bad_inputs_before_allocating(solver):
    """nq > 65535 and null arrays with non-zero counts return
    GS_E_INVALID (no dereference, no device allocation)"""
    import ctypes as C
    p = random_catalog(7, 20, 3)
    res = abi.GsClaimFilterResult()
    st = solver.L.gs_create_filter(solver.ctx, C.byref(p.struct), p.claim_queries, 70000, C.byref(res))
    assert st == abi.GS_E_INVALID
    for field in ("instance_types", "offerings", "quantities", "reqs", "value_ids"):
        bad = abi.GsProblem()
        C.memmove(C.byref(bad), C.byref(p.struct), C.sizeof(bad))
        setattr(bad, field, None)
        st = solver.L.gs_create_filter(solver.ctx, C.byref(bad), p.claim_queries, p.n_claim_queries, C.byref(res))
        assert st == abi.GS_E_INVALID, field
    # the context still works afterwards
    assert solver.create_filter(p) == solver.create_filter(p)
