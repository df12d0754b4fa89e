"""Pin the oracle (and the host-side catalog mirror) to the reference's own
known-answer tests (tests/golden/reference_kats.json, transcribed from the
reference Go test tables, each with its file:line)."""
import json
import os
import struct

import pytest

from gpusched import catalog as cat
from oracle import pyoracle

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def _ac(x):
    return None if x is None else (x[0], x[1])


@pytest.mark.parametrize("name,want", KATS["instance_family"]["cases"])
def test_instance_family(name, want):
    assert pyoracle.lib().oracle_instance_family(name.encode()).decode() == want
    assert cat.instance_family(name) == want


@pytest.mark.parametrize("name,want", KATS["instance_size"]["cases"])
def test_instance_size(name, want):
    assert pyoracle.lib().oracle_instance_size(name.encode()).decode() == want
    assert cat.instance_size(name) == want


@pytest.mark.parametrize("ac,want", KATS["supported_capacity_types"]["cases"])
def test_supported_capacity_types(ac, want):
    assert cat.supported_capacity_types(_ac(ac)) == want
    # the oracle's conversion must expose the same capacity types, in order
    st, text = pyoracle.convert_profile("bx2-2x8", vcpu=2, memory_gib=8, availability_class=_ac(ac),
                                        zones=["z1"])
    assert st == 0
    assert [o[1] for o in pyoracle.parse_text(text)["offerings"]] == want


@pytest.mark.parametrize("cpu,mem,price,want", KATS["instance_score"]["cases"])
def test_instance_score(cpu, mem, price, want):
    cpu_m = cat.parse_quantity_milli(cpu)
    mem_b = cat.parse_quantity_milli(mem) // 1000
    assert cat.instance_type_score(cpu_m, mem_b, price) == want
    assert pyoracle.lib().oracle_instance_score(cpu_m, mem_b, price) == want


@pytest.mark.parametrize("case", KATS["overhead"]["cases"])
def test_overhead(case):
    want = {k: cat.parse_quantity_milli(v) for k, v in case["want"].items()}
    kub = case["kubelet"]
    st, text = pyoracle.convert_profile("bx2-2x8", vcpu=2, memory_gib=8, zones=["z1"], kubelet=kub)
    assert st == 0
    assert pyoracle.parse_text(text)["overhead"] == want
    k = None if kub is None else cat.Kubelet(kub.get("kubeReserved", {}), kub.get("systemReserved", {}),
                                             kub.get("evictionHard", {}))
    ovh = cat.calculate_overhead(k)
    flat = {f"{part}.{r}": v for part, d in ovh.items() for r, v in d.items()}
    assert flat == want


def test_offerings_per_zone_captype():
    k = KATS["offerings_per_zone_captype"]
    p = k["profile"]
    st, text = pyoracle.convert_profile(p["name"], vcpu=p["vcpu"], memory_gib=p["memory_gib"], arch=p["arch"],
                                        gpu=p["gpu"], availability_class=_ac(p["availability_class"]),
                                        zones=k["zones"], prices=k["prices"], unavailable=k["unavailable"])
    assert st == 0
    offs = pyoracle.parse_text(text)["offerings"]
    assert len(offs) == k["want_offerings"]
    for z, ct, _, avail in offs:
        assert avail == ([z, ct] not in k["want_unavailable"])
    it = cat.convert_profile(cat.Profile(p["name"], p["vcpu"], p["memory_gib"], p["arch"], p["gpu"],
                                         _ac(p["availability_class"])), k["zones"],
                             lambda n, z: k["prices"].get(n), unavailable=k["unavailable"])
    assert it.offerings == offs


def test_spot_price_exact():
    k = KATS["spot_price"]
    p = k["profile"]
    st, text = pyoracle.convert_profile(p["name"], vcpu=p["vcpu"], memory_gib=p["memory_gib"], arch=p["arch"],
                                        gpu=p["gpu"], availability_class=_ac(p["availability_class"]),
                                        zones=k["zones"], prices=k["prices"],
                                        spot_discount_percent=k["spot_discount_percent"])
    assert st == 0
    offs = pyoracle.parse_text(text)["offerings"]
    assert len(offs) == 2
    for _, ct, price, _ in offs:
        # bit-exact float64, as assert.Equal in the Go test
        assert struct.pack("<d", price) == struct.pack("<d", k["want"][ct])
    it = cat.convert_profile(cat.Profile(p["name"], p["vcpu"], p["memory_gib"], p["arch"], p["gpu"],
                                         _ac(p["availability_class"])), k["zones"],
                             lambda n, z: k["prices"].get(n), spot_discount_percent=k["spot_discount_percent"])
    assert [(o[1], o[2]) for o in it.offerings] == [("on-demand", 0.190), ("spot", 0.076)]


@pytest.mark.parametrize("case", KATS["conversion_errors"]["cases"])
def test_conversion_errors(case):
    prof, has_client, want = case
    st, text = pyoracle.convert_profile(prof.get("name"), vcpu=prof.get("vcpu"), memory_gib=prof.get("memory_gib"),
                                        arch=prof.get("arch"), gpu=prof.get("gpu"), zones=["z1"],
                                        has_client=has_client)
    assert st != 0
    assert want in text


def test_fake_catalog_capacity_and_pods():
    """pods heuristic 30/60/110 and the always-present nvidia.com/gpu (instancetype.go:705-718,784)"""
    k = KATS["fake_profiles"]
    for name, v, m, g in k["profiles"]:
        st, text = pyoracle.convert_profile(name, vcpu=v, memory_gib=m, gpu=g, zones=k["zones"])
        assert st == 0
        it = pyoracle.parse_text(text)
        pods = 30 if v <= 2 else 60 if v <= 4 else 110
        assert it["capacity"] == {"cpu": v * 1000, "memory": m * (1 << 30) * 1000, "pods": pods * 1000,
                                  "nvidia.com/gpu": (g or 0) * 1000}
        assert len(it["offerings"]) == 3
        mine = cat.convert_profile(cat.Profile(name, v, m, None, g), k["zones"], lambda n, z: None)
        assert mine.capacity == it["capacity"]
        assert all(o[2] == 0.0 for o in mine.offerings)  # missing price -> 0.0 (instancetype.go:753)


@pytest.mark.parametrize("q", ["100m", "1Gi", "500Mi", "2", "1.5", "0.1m", "1e3", "2Ki", "-1", "3k", "1.25Gi"])
def test_quantity_parse_agrees(q):
    import ctypes as C
    v = C.c_int64()
    assert pyoracle.lib().oracle_parse_quantity_milli(q.encode(), C.byref(v)) == 0
    assert v.value == cat.parse_quantity_milli(q)


@pytest.mark.parametrize("q", ["not-a-quantity", "also-bad", "", "1Qi", "--1"])
def test_quantity_parse_rejects(q):
    import ctypes as C
    v = C.c_int64()
    assert pyoracle.lib().oracle_parse_quantity_milli(q.encode(), C.byref(v)) != 0
    with pytest.raises(ValueError):
        cat.parse_quantity_milli(q)


def test_no_zones_reason_names_region():
    """"no zones found for region %s" carries client.GetRegion() (instancetype.go:738-740)"""
    st, text = pyoracle.convert_profile("bx2-2x8", vcpu=2, memory_gib=8, zones=[], region="us-south")
    assert st != 0 and text == "no zones found for region us-south"
    with pytest.raises(ValueError, match="^no zones found for region us-south$"):
        cat.convert_profile(cat.Profile("bx2-2x8", 2, 8), [], lambda n, z: None, region="us-south")
