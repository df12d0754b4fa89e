"""Zone-key pod anti-affinity (VERDICT r2 Missing 2).

<U> karpenter Topology, TopologyTypePodAntiAffinity on
topology.kubernetes.io/zone: nextDomainAntiAffinity allows every known zone
whose count is 0 and that both the pod and the NodeClaim allow, so a
NodeClaim's zone requirement narrows to a SET of zones (not one domain as
for spread); Record counts every zone of the NodeClaim's non-complement zone
requirement.  The inverse group of a required term keeps the term's targets
out of the carriers' zones.  The reference's own e2e suite runs this shape
(reference test/e2e/multizone_test.go:83-174, preferred weight 100).

CPU tests pin the oracle restatement on hand-derived cases; GPU tests require
both HIP Solve kernels to equal the oracle bit for bit.
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
WEB = {"labels": {"app": "web"}}
ZONES = synth.FAKE_ZONES


def zones_of(claim):
    """the zone values of a NodeClaim's requirement text (None: no zone requirement)"""
    for line in claim["requirements"].split("\n"):
        f = line.split("|")
        if f[0] == Z:
            return (f[1], sorted(v for v in f[2].split(",") if v))
    return None


def _base(n_pods=4, anti=(), zones=ZONES, cpu=500):
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, ZONES, spot=False, prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("default", requirements=[(Z, "In", list(zones))])
    for i in range(n_pods):
        b.add_pod(f"p{i}", 0, {"cpu": cpu, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  anti_affinity=list(anti))
    return b


def _solve(b):
    st, res, _ = pyoracle.solve(b.build())
    assert st == abi.GS_OK
    return res


def _zone_anti(required, weight=100, selector=WEB):
    return {"key": Z, "required": required, "weight": weight, "selector": selector}


def test_required_zone_anti_affinity_first_claim_blocks_every_zone():
    # the first NodeClaim may still land in any zone, so Record counts it in
    # all three ("where the pods could be"): no zone is empty for the others
    res = _solve(_base(anti=[_zone_anti(True)]))
    assert [c["pods"] for c in res["claims"]] == [[0]] and res["errors"] == [1, 2, 3]
    assert zones_of(res["claims"][0]) == ("In", sorted(ZONES))


def test_preferred_zone_anti_affinity_relaxes():
    res = _solve(_base(anti=[_zone_anti(False)]))
    assert [c["pods"] for c in res["claims"]] == [[0, 1, 2, 3]] and not res["errors"]


def test_zone_anti_affinity_avoids_bound_pods_zone():
    # a web pod runs in zone 1: the first pending web pod gets zones {2, 3}
    b = _base(n_pods=2, anti=[_zone_anti(True)])
    b.add_node("n0", {Z: ZONES[0], H: "n0"}, {"cpu": 100, "memory": 1 << 30, "pods": 110_000})
    b.add_bound_pod(0, "b0", 0, {"cpu": 100}, labels={"app": "web"})
    res = _solve(b)
    assert [c["pods"] for c in res["claims"]] == [[0]] and res["errors"] == [1]
    assert zones_of(res["claims"][0]) == ("In", sorted(ZONES[1:]))


def test_inverse_zone_anti_affinity_of_a_bound_carrier():
    # a db pod in zone 1 requires no web pod in its zone: plain web pods skip
    # the roomy node n0 and open a NodeClaim restricted to zones {2, 3}
    b = _base(n_pods=3)
    b.add_node("n0", {Z: ZONES[0], H: "n0"}, {"cpu": 8000, "memory": 32 << 30, "pods": 110_000})
    b.add_bound_pod(0, "b0", 0, {"cpu": 100}, labels={"app": "db"}, anti_affinity=[_zone_anti(True)])
    res = _solve(b)
    assert res["nodes"][0] == [] and not res["errors"]
    assert [c["pods"] for c in res["claims"]] == [[0, 1, 2]]
    assert zones_of(res["claims"][0]) == ("In", sorted(ZONES[1:]))


def test_zone_anti_affinity_and_spread_intersect():
    # zone spread (maxSkew 1) and zone anti-affinity on the same pods
    spread = {"key": Z, "max_skew": 1, "selector": WEB, "when": "DoNotSchedule", "node_affinity_policy": "Ignore"}
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, ZONES, spot=False, prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("default", requirements=[(Z, "In", ZONES)])
    for i in range(4):
        b.add_pod(f"p{i}", 0, {"cpu": 500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  anti_affinity=[_zone_anti(False)], spreads=[spread])
    res = _solve(b)
    assert not res["errors"]
    for c in res["claims"]:
        assert zones_of(c)[0] == "In" and len(zones_of(c)[1]) == 1


def test_zone_pod_affinity_still_refused():
    b = _base(n_pods=0)
    b.add_pod("x", 0, {"cpu": 1}, affinity=[{"key": Z, "required": True, "selector": WEB}])
    assert pyoracle.solve(b.build())[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


def random_zone_anti(seed, n_pods=None):
    """random problems mixing zone anti-affinity (required / preferred,
    self-selecting or not, namespaces), its inverse groups from pending and
    bound carriers, zone spread and hostname anti-affinity, over NodePools
    with zone subsets, existing nodes in some zones and NodePool limits"""
    import numpy as np
    rng = np.random.default_rng(0xA7170000 + seed)
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3", "z4"][: int(rng.integers(2, 5))]
    profs = [("bx2-2x8", 2, 8, None), ("bx2-4x16", 4, 16, None), ("cx2-8x16", 8, 16, None)]
    synth.build_catalog(b, profs, zones, spot=bool(rng.random() < 0.5), prices=synth.price_table(profs), rng=rng,
                        unavailable_frac=0.1)
    for j in range(int(rng.integers(1, 3))):
        sub = sorted(set(rng.choice(zones, size=int(rng.integers(1, len(zones) + 1))).tolist()))
        limits = {"cpu": int(rng.choice([8, 16, 64])) * 1000} if rng.random() < 0.3 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=[(Z, "In", sub)], limits=limits)
    apps = ["web", "db", "cache"]
    pal = []
    for _ in range(int(rng.integers(1, 4))):
        pal.append({"key": Z if rng.random() < 0.7 else H, "required": bool(rng.random() < 0.4),
                    "weight": int(rng.choice([1, 10, 100])), "selector": {"labels": {"app": str(rng.choice(apps))}}})
    spread = {"key": Z, "max_skew": int(rng.choice([1, 2])), "selector": {"labels": {"app": str(rng.choice(apps))}},
              "when": "ScheduleAnyway" if rng.random() < 0.5 else "DoNotSchedule", "node_affinity_policy": "Ignore"}
    for k in range(int(rng.integers(0, 4))):
        b.add_node(f"n{k}", {Z: str(rng.choice(zones)), H: f"n{k}"},
                   {"cpu": int(rng.choice([1000, 4000])), "memory": 16 << 30, "pods": 110_000})
        for q in range(int(rng.integers(0, 3))):
            anti = [dict(pal[0], required=True)] if rng.random() < 0.3 else []
            b.add_bound_pod(k, f"b{k}-{q}", 0, {"cpu": 100}, labels={"app": str(rng.choice(apps))}, anti_affinity=anti)
    n = int(n_pods if n_pods is not None else rng.integers(1, 30))
    for i in range(n):
        k = int(rng.integers(0, 3))
        anti = [pal[x] for x in sorted(set(rng.choice(len(pal), size=k).tolist()))] if k else []
        b.add_pod(f"p{i:03d}", int(rng.integers(0, 3)), {"cpu": int(rng.choice([250, 500, 1000])),
                                                          "memory": 1 << 30, "pods": 1000},
                  labels={"app": str(rng.choice(apps))}, anti_affinity=anti,
                  spreads=[spread] if rng.random() < 0.2 else [])
    return b.build()


@pytest.mark.parametrize("seed", range(30))
def test_oracle_and_encoder_accept_random_zone_anti(seed):
    p = random_zone_anti(seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK, msg


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


_KATS = [
    lambda: _base(anti=[_zone_anti(True)]),
    lambda: _base(n_pods=3, anti=[_zone_anti(True)]),
    lambda: _base(anti=[_zone_anti(False)]),
    lambda: _base(n_pods=6, anti=[_zone_anti(False), {"key": H, "required": True, "selector": WEB}]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(_KATS)))
def test_gpu_zone_anti_kats(solver, k):
    _check(solver, _KATS[k]().build())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(60))
def test_gpu_zone_anti_random(solver, seed):
    _check(solver, random_zone_anti(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_zone_anti_random_many_pods(solver, seed):
    _check(solver, random_zone_anti(100 + seed, n_pods=300))
