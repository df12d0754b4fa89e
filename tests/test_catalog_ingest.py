"""Catalog ingest (gs_build_catalog): IBMInstanceTypeProvider.List
over VPC profile wire data (reference pkg/providers/common/instancetype/
instancetype.go:221-246,433-537,659-858), with the UnavailableOfferings
overlay (pkg/cache/unavailable_offerings.go:36-77).

CPU tests pin the oracle's restatement (oracle_convert_profile) on the new
overlay semantics (expiry, per-zone prices); the reference KATs already pin
the rest of it (tests/test_oracle_kats.py).  GPU tests require the product's
converted catalog — names, requirements, capacity, Overhead.Total(), and every
offering's zone, capacity type, float64 price bits and availability — to equal
the oracle's on the reference KAT inputs and on randomised profile lists, and
the refused profiles to be exactly the ones the oracle refuses.
"""
import json
import os
import struct

import numpy as np
import pytest

from oracle import pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "reference_kats.json")) as f:
    KATS = json.load(f)

NOW = 1_760_000_000_000_000_000


def _ac(x):
    return None if x is None else (x[0], x[1])


def oracle_list(profiles, zones, price_rows=(), unavailable=(), now_ns=NOW, spot_discount_percent=0, kubelet=None):
    """per profile: the oracle's converted type (parsed) or None when refused"""
    out = []
    for p in profiles:
        st, text = pyoracle.convert_profile(
            p.get("name"), vcpu=p.get("vcpu"), memory_gib=p.get("memory_gib"), arch=p.get("arch"),
            gpu=p.get("gpu"), availability_class=p.get("availability_class"), zones=zones,
            spot_discount_percent=spot_discount_percent, unavailable=[k for k, _ in unavailable],
            unavailable_expiry=[x for _, x in unavailable], now_ns=now_ns, price_rows=list(price_rows),
            kubelet=kubelet, vcpu_kind=p.get("vcpu_kind"), memory_kind=p.get("memory_kind"),
            gpu_kind=p.get("gpu_kind"))
        out.append(pyoracle.parse_text(text) if st == 0 else None)
    return out


def normalize_oracle(it):
    reqs = sorted(tuple(r.split("|")) for r in it["requirements"].split(";"))
    ovh = it["overhead"]
    total = {"cpu": ovh["kube.cpu"] + ovh["system.cpu"],
             "memory": ovh["kube.memory"] + ovh["system.memory"] + ovh["eviction.memory"]}
    return {"name": it["name"], "requirements": reqs, "capacity": it["capacity"], "overhead": total,
            "offerings": [(z, ct, struct.pack("<d", p), a) for z, ct, p, a in it["offerings"]]}


def normalize_product(it):
    return {"name": it["name"], "requirements": sorted((k, op, v[0]) for k, op, v in it["requirements"]),
            "capacity": it["capacity"], "overhead": it["overhead"],
            "offerings": [(z, ct, struct.pack("<d", p), a) for z, ct, p, a in it["offerings"]]}


# ----------------------------------------------------------- CPU: the oracle
def test_oracle_overlay_expiry():
    """IsUnavailable: present and !now.After(expiry) (unavailable_offerings.go:51-77)"""
    base = dict(vcpu=2, memory_gib=8, zones=["z1"], availability_class=("enum", ["standard", "spot"]))
    for expiry, want in [(NOW + 1, False), (NOW, False), (NOW - 1, True)]:
        st, text = pyoracle.convert_profile("bx2-2x8", unavailable=["bx2-2x8:z1:spot"], unavailable_expiry=[expiry],
                                            now_ns=NOW, **base)
        offs = pyoracle.parse_text(text)["offerings"]
        assert [o[3] for o in offs] == [True, want]
    # a repeated key keeps the last Add
    st, text = pyoracle.convert_profile("bx2-2x8", unavailable=["bx2-2x8:z1:on-demand"] * 2,
                                        unavailable_expiry=[NOW + 5, NOW - 5], now_ns=NOW, **base)
    assert pyoracle.parse_text(text)["offerings"][0][3] is True


def test_oracle_zone_prices():
    st, text = pyoracle.convert_profile("bx2-2x8", vcpu=2, memory_gib=8, zones=["z1", "z2"],
                                        price_rows=[("bx2-2x8", None, 0.5), ("bx2-2x8", "z2", 0.7)])
    offs = pyoracle.parse_text(text)["offerings"]
    assert [o[2] for o in offs] == [0.5, 0.7]


# --------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def solver():
    from gpusched import lib
    s = lib.Solver()
    yield s
    s.close()


def check(solver, profiles, zones, **kw):
    kw.setdefault("now_ns", NOW)
    want = oracle_list(profiles, zones, **kw)
    if all(w is None for w in want):
        from gpusched import lib
        with pytest.raises(lib.GpuSchedError):
            solver.build_catalog(profiles, zones, **kw)
        return []
    got, skipped, _ = solver.build_catalog(profiles, zones, **kw)
    assert [i for i, _ in skipped] == [i for i, w in enumerate(want) if w is None]
    kept = [w for w in want if w is not None]
    assert len(got) == len(kept)
    for g, w in zip(got, kept):
        assert normalize_product(g) == normalize_oracle(w), g["name"]
    return got


@pytest.mark.gpu
def test_gpu_fake_catalog(solver):
    k = KATS["fake_profiles"]
    profs = [dict(name=n, vcpu=v, memory_gib=m, gpu=g) for n, v, m, g in k["profiles"]]
    got = check(solver, profs, k["zones"])
    assert len(got) == 8 and all(o[2] == 0.0 for it in got for o in it["offerings"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", KATS["overhead"]["cases"])
def test_gpu_overhead_kats(solver, case):
    check(solver, [dict(name="bx2-2x8", vcpu=2, memory_gib=8)], ["z1"], kubelet=case["kubelet"])


@pytest.mark.gpu
@pytest.mark.parametrize("ac,want", KATS["supported_capacity_types"]["cases"])
def test_gpu_capacity_types_kats(solver, ac, want):
    got = check(solver, [dict(name="bx2-2x8", vcpu=2, memory_gib=8, availability_class=_ac(ac))], ["z1"])
    assert [o[1] for o in got[0]["offerings"]] == want


@pytest.mark.gpu
def test_gpu_spot_price_and_overlay_kats(solver):
    for key in ("spot_price", "offerings_per_zone_captype"):
        k = KATS[key]
        p = dict(k["profile"])
        p["availability_class"] = _ac(p["availability_class"])
        got = check(solver, [p], k["zones"], price_rows=[(n, None, v) for n, v in k["prices"].items()],
                    unavailable=[(u, NOW + 3600 * 10**9) for u in k.get("unavailable", [])],
                    spot_discount_percent=k.get("spot_discount_percent", 0))
        if key == "spot_price":
            assert [(o[1], o[2]) for o in got[0]["offerings"]] == [("on-demand", 0.19), ("spot", 0.076)]
        else:
            assert [(o[0], o[1]) for o in got[0]["offerings"] if not o[3]] == [("us-south-2", "spot")]


@pytest.mark.gpu
@pytest.mark.parametrize("case", KATS["conversion_errors"]["cases"][:3])
def test_gpu_conversion_errors(solver, case):
    prof, _, want = case
    good = dict(name="bx2-2x8", vcpu=2, memory_gib=8)
    got, skipped, _ = solver.build_catalog([prof, good], ["z1"])
    assert [i for i, _ in skipped] == [0] and want in skipped[0][1]
    assert [it["name"] for it in got] == ["bx2-2x8"]


@pytest.mark.gpu
def test_gpu_no_zones_refused(solver):
    from gpusched import lib
    with pytest.raises(lib.GpuSchedError):
        solver.build_catalog([dict(name="bx2-2x8", vcpu=2, memory_gib=8)], [])


def random_profiles(seed, n):
    rng = np.random.default_rng(seed)
    fams = ["bx2", "cx2", "mx2", "gx3", "ux2d", "", "vx2d"]
    out = []
    for i in range(n):
        fam = fams[rng.integers(len(fams))]
        v = int(rng.choice([1, 2, 3, 4, 8, 16, 48]))
        m = v * int(rng.choice([2, 4, 8, 14]))
        name = f"{fam}-{v}x{m}" if rng.random() < 0.9 else f"{fam}{i}"
        if rng.random() < 0.05:
            name = f"{name}-"
        p = dict(name=f"{name}-{i}" if rng.random() < 0.5 else name, vcpu=v, memory_gib=m)
        u = rng.random()
        if u < 0.03:
            p["name"] = None
        elif u < 0.05:
            p["name"] = ""
        elif u < 0.08:
            p["vcpu"] = None
        elif u < 0.10:
            p["vcpu_kind"] = 2
        elif u < 0.12:
            p["memory_gib"] = None
        elif u < 0.14:
            p["memory_kind"] = 2
        if rng.random() < 0.3:
            p["arch"] = str(rng.choice(["amd64", "s390x", "arm64"]))
        g = rng.random()
        if g < 0.1:
            p["gpu"] = int(rng.integers(1, 5))
        elif g < 0.13:
            p["gpu"], p["gpu_kind"] = 3, 2  # another GpuCount variant: 0
        a = rng.random()
        if a < 0.3:
            p["availability_class"] = ("enum", list(rng.choice(["standard", "spot", "reserved"],
                                                               size=int(rng.integers(0, 3)))))
        elif a < 0.45:
            p["availability_class"] = ("fixed", None if rng.random() < 0.2 else str(rng.choice(["spot", "standard"])))
        out.append(p)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_gpu_random_catalogs(solver, seed):
    rng = np.random.default_rng(1000 + seed)
    profs = random_profiles(seed, [5, 40, 200, 1188, 2000, 64, 65, 1, 300, 500][seed])
    zones = [f"us-south-{i}" for i in range(1, int(rng.integers(1, 7)) + 1)]
    names = [p["name"] for p in profs if p.get("name")]
    price_rows = []
    for nm in names:
        if rng.random() < 0.8:
            price_rows.append((nm, None, float(rng.integers(1, 5000)) / 1000))
        if rng.random() < 0.2:
            price_rows.append((nm, zones[rng.integers(len(zones))], float(rng.integers(1, 5000)) / 997))
    unavailable = []
    for _ in range(len(names) // 3):
        nm = names[rng.integers(len(names))]
        key = f"{nm}:{zones[rng.integers(len(zones))]}:{rng.choice(['spot', 'on-demand'])}"
        unavailable.append((key, NOW + int(rng.integers(-10, 10)) * 10**9))
    unavailable.append(("garbage-key", NOW + 1))
    kub = None
    if seed % 3 == 1:
        kub = {"kubeReserved": {"cpu": "250m", "memory": "1.5Gi"}, "systemReserved": {"cpu": "bad"},
               "evictionHard": {"memory.available": "200Mi"}}
    check(solver, profs, zones, price_rows=price_rows, unavailable=unavailable,
          spot_discount_percent=[0, 40, 75, 33][seed % 4], kubelet=kub)


@pytest.mark.gpu
def test_gpu_catalog_feeds_solve(solver):
    """the ingested C2 catalog equals the harness catalog the Solve benches
    use (gpusched.catalog), and a problem built from it solves exactly as the
    oracle does"""
    from gpusched import catalog as cat, synth
    from gpusched.problem import ProblemBuilder
    profs = synth.c2_profiles(200)
    prices = synth.price_table(profs)
    zones = synth.FAKE_ZONES
    ac = ("enum", ["standard", "spot"])
    wire = [dict(name=n, vcpu=v, memory_gib=m, arch="amd64", gpu=g, availability_class=ac) for n, v, m, g in profs]
    unav = [(f"{profs[k][0]}:{zones[k % 3]}:spot", NOW + 10**9) for k in range(0, 200, 7)]
    got, skipped, _ = solver.build_catalog(wire, zones, price_rows=[(n, None, v) for n, v in prices.items()],
                                           unavailable=unav, now_ns=NOW)
    assert not skipped
    mine = cat.list_instance_types([cat.Profile(n, v, m, "amd64", g, ac) for n, v, m, g in profs], zones,
                                   lambda n, z: prices.get(n), unavailable={k for k, _ in unav})
    for g, m in zip(got, mine):
        assert g["name"] == m.name and g["capacity"] == m.capacity and g["overhead"] == m.overhead
        assert sorted((k, op, v[0]) for k, op, v in g["requirements"]) == sorted((k, op, v[0]) for k, op, v in m.requirements)
        assert [(z, ct, struct.pack("<d", pr), a) for z, ct, pr, a in g["offerings"]] == \
               [(z, ct, struct.pack("<d", pr), a) for z, ct, pr, a in m.offerings]
    b = ProblemBuilder()
    for it in got:
        b.add_instance_type(it["name"], it["requirements"], it["capacity"], it["overhead"], it["offerings"])
    b.add_nodepool("default", requirements=[("kubernetes.io/arch", "In", ["amd64"])])
    rng = np.random.default_rng(3)
    for i in range(2000):
        b.add_pod(f"pod-{i:05d}", 1_700_000_000 + int(rng.integers(0, 8)),
                  {"cpu": int(rng.choice([100, 250, 500, 1000, 2000])),
                   "memory": int(rng.choice([128, 512, 2048])) * (1 << 20) * 1000, "pods": 1000})
    p = b.build()
    want = pyoracle.solve(p)[1]
    res, _ = solver.solve(p)
    assert res == want
