"""IBM VPC catalog -> cloudprovider.InstanceType list (host-side mirror).

Mirrors IBMInstanceTypeProvider.convertVPCProfileToInstanceType and helpers
(reference pkg/providers/common/instancetype/instancetype.go:659-877) and
capacitytype.GetSupportedCapacityTypes (capacitytype.go:48-85).  This is the
provider seam that feeds Solve; its outputs go into ProblemBuilder
add_instance_type() exactly as GetInstanceTypes would return them.
"""
from dataclasses import dataclass, field
from fractions import Fraction
import re

GI = 1 << 30
MI = 1 << 20

_QTY = re.compile(r"^([+-]?)(\d+(?:\.\d*)?|\.\d+)(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E|[eE][+-]?\d+)?$")
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}


def parse_quantity_milli(s: str) -> int:
    """resource.ParseQuantity(s).MilliValue() (rounds up); ValueError if invalid."""
    m = _QTY.match(s or "")
    if not m:
        raise ValueError(f"invalid quantity {s!r}")
    sign, num, suf = m.group(1), m.group(2), m.group(3) or ""
    x = Fraction(num)
    if suf in _BIN:
        x *= 1 << _BIN[suf]
    elif suf in _DEC:
        x *= Fraction(10) ** _DEC[suf]
    else:
        x *= Fraction(10) ** int(suf[1:])
    x *= 1000
    q = -(-x.numerator // x.denominator)  # ceil
    return -q if sign == "-" else q


def instance_family(name: str) -> str:
    """getInstanceFamily (instancetype.go:861-867)"""
    first = name.split("-", 1)[0]
    return first if first else "balanced"


def instance_size(name: str) -> str:
    """getInstanceSize (instancetype.go:870-877)"""
    for i, c in enumerate(name):
        if c == "-" and i + 1 < len(name):
            return name[i + 1:]
    return "small"


def capacity_type_from_availability_class(cls: str) -> str:
    """GetCapacityTypeFromAvailabilityClass (capacitytype.go:75-85)"""
    return "spot" if cls == "spot" else "on-demand"


def supported_capacity_types(availability_class) -> list:
    """GetSupportedCapacityTypes (capacitytype.go:48-73).
    availability_class: None | ("enum", [values]) | ("fixed", value-or-None)"""
    out = []
    if availability_class is None:
        return ["on-demand"]
    kind, val = availability_class
    if kind == "enum":
        out = [capacity_type_from_availability_class(v) for v in val]
    elif kind == "fixed" and val is not None:
        out = [capacity_type_from_availability_class(val)]
    return out or ["on-demand"]


def instance_type_score(cpu_milli: int, memory_bytes: int, price: float) -> float:
    """calculateInstanceTypeScore (instancetype.go:90-110)"""
    cpu = float(-(-cpu_milli // 1000))
    mem_gb = float(-(-memory_bytes // 1_000_000_000))
    if price <= 0:
        return cpu + mem_gb
    return (price / cpu + price / mem_gb) / 2


@dataclass
class Kubelet:
    kube_reserved: dict = field(default_factory=dict)
    system_reserved: dict = field(default_factory=dict)
    eviction_hard: dict = field(default_factory=dict)


def calculate_overhead(kubelet) -> dict:
    """calculateOverhead (instancetype.go:792-858) -> milli quantities"""
    kc, km = parse_quantity_milli("100m"), parse_quantity_milli("1Gi")
    sc, sm = parse_quantity_milli("100m"), parse_quantity_milli("1Gi")
    ev = parse_quantity_milli("500Mi")

    def over(d, k, cur):
        if k in d:
            try:
                return parse_quantity_milli(d[k])
            except ValueError:
                return cur
        return cur

    if kubelet is not None:
        kc = over(kubelet.kube_reserved, "cpu", kc)
        km = over(kubelet.kube_reserved, "memory", km)
        sc = over(kubelet.system_reserved, "cpu", sc)
        sm = over(kubelet.system_reserved, "memory", sm)
        ev = over(kubelet.eviction_hard, "memory.available", ev)
    return {"kube": {"cpu": kc, "memory": km}, "system": {"cpu": sc, "memory": sm}, "eviction": {"memory": ev}}


def overhead_total(ovh: dict) -> dict:
    """InstanceTypeOverhead.Total() = Merge(kube, system, eviction)"""
    tot = {}
    for part in ("kube", "system", "eviction"):
        for k, v in ovh[part].items():
            tot[k] = tot.get(k, 0) + v
    return tot


@dataclass
class Profile:
    """vpcv1.InstanceProfile fields used by the conversion"""
    name: str
    vcpu: int
    memory_gib: int
    arch: str = None
    gpu: int = None
    availability_class: object = None


@dataclass
class InstanceType:
    name: str
    requirements: list
    capacity: dict
    overhead: dict
    offerings: list  # (zone, ct, price, available)


def convert_profile(p: Profile, zones, price_of, spot_discount_percent=60, unavailable=(), kubelet=None,
                    region=""):
    """convertVPCProfileToInstanceType.  price_of(name, zone) -> float or None
    (None = GetPrice error -> 0.0, reference instancetype.go:753)."""
    if not p.name:
        raise ValueError("instance profile has empty name")
    if not zones:
        raise ValueError(f"no zones found for region {region}")  # instancetype.go:738-740
    arch = p.arch or "amd64"
    gpu = p.gpu or 0
    pods = 110
    if p.vcpu <= 2:
        pods = 30
    elif p.vcpu <= 4:
        pods = 60
    capacity = {"cpu": p.vcpu * 1000, "memory": p.memory_gib * GI * 1000, "pods": pods * 1000,
                "nvidia.com/gpu": gpu * 1000}
    reqs = [("node.kubernetes.io/instance-type", "In", [p.name]),
            ("kubernetes.io/arch", "In", [arch]),
            ("karpenter-ibm.sh/instance-family", "In", [instance_family(p.name)]),
            ("karpenter-ibm.sh/instance-size", "In", [instance_size(p.name)])]
    pct = spot_discount_percent or 60
    unav = set(unavailable)
    offerings = []
    for z in zones:
        for ct in supported_capacity_types(p.availability_class):
            price = price_of(p.name, z)
            price = 0.0 if price is None else float(price)
            if ct == "spot":
                price = price * float(pct) / 100.0
            offerings.append((z, ct, price, f"{p.name}:{z}:{ct}" not in unav))
    return InstanceType(p.name, reqs, capacity, overhead_total(calculate_overhead(kubelet)), offerings)


def list_instance_types(profiles, zones, price_of, **kw):
    """IBMInstanceTypeProvider.List: convert in VPC order, skip failures"""
    out = []
    for p in profiles:
        try:
            out.append(convert_profile(p, zones, price_of, **kw))
        except ValueError:
            continue
    if not out:
        raise ValueError("no instance types found from VPC API")
    return out
