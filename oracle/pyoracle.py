"""ctypes loader for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product path (gpusched) never does.
"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "karpenter-provider-ibm-cloud_amd"))
from gpusched import abi  # noqa: E402


class OracleProfile(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("vcpu_kind", C.c_int32), ("vcpu", C.c_int64),
        ("memory_kind", C.c_int32), ("memory_gib", C.c_int64), ("arch", C.c_char_p),
        ("gpu_kind", C.c_int32), ("gpu", C.c_int64), ("avail_kind", C.c_int32),
        ("avail_values", C.POINTER(C.c_char_p)), ("n_avail_values", C.c_uint32),
    ]


class OracleEnv(C.Structure):
    _fields_ = [
        ("has_client", C.c_int32), ("zones", C.POINTER(C.c_char_p)), ("n_zones", C.c_uint32),
        ("spot_discount_percent", C.c_int32),
        ("price_names", C.POINTER(C.c_char_p)), ("prices", C.POINTER(C.c_double)), ("n_prices", C.c_uint32),
        ("unavailable", C.POINTER(C.c_char_p)), ("n_unavailable", C.c_uint32),
        ("has_nodeclass", C.c_int32), ("has_kubelet", C.c_int32),
        ("kube_reserved_cpu", C.c_char_p), ("kube_reserved_memory", C.c_char_p),
        ("system_reserved_cpu", C.c_char_p), ("system_reserved_memory", C.c_char_p),
        ("eviction_memory_available", C.c_char_p),
        ("price_zones", C.POINTER(C.c_char_p)),
        ("unavailable_expiry", C.POINTER(C.c_int64)),
        ("now_ns", C.c_int64),
        ("region", C.c_char_p),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_solve.argtypes = [C.POINTER(abi.GsProblem), C.POINTER(abi.GsResult)]
        L.oracle_solve.restype = C.c_int
        L.oracle_feasibility.argtypes = [C.POINTER(abi.GsProblem), C.POINTER(abi.GsFeasResult)]
        L.oracle_feasibility.restype = C.c_int
        L.oracle_convert_profile.argtypes = [C.POINTER(OracleProfile), C.POINTER(OracleEnv),
                                             C.POINTER(C.c_char_p)]
        L.oracle_convert_profile.restype = C.c_int
        L.oracle_parse_quantity_milli.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.oracle_parse_quantity_milli.restype = C.c_int
        for f in ("oracle_instance_family", "oracle_instance_size", "oracle_capacity_type"):
            getattr(L, f).argtypes = [C.c_char_p]
            getattr(L, f).restype = C.c_char_p
        L.oracle_instance_score.argtypes = [C.c_int64, C.c_int64, C.c_double]
        L.oracle_instance_score.restype = C.c_double
        L.oracle_rank_instance_types.argtypes = abi.RANK_ARGTYPES
        L.oracle_rank_instance_types.restype = C.c_int
        L.oracle_consolidate.argtypes = [C.POINTER(abi.GsConsolidation), C.POINTER(abi.GsConsolidationResult),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_consolidate.restype = C.c_int
        L.oracle_create_filter.argtypes = [C.POINTER(abi.GsProblem), C.POINTER(abi.GsClaimQuery), C.c_uint32,
                                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_uint32)]
        L.oracle_create_filter.restype = C.c_int
        L.oracle_resolve_capacity_type.argtypes = [C.POINTER(abi.GsProblem), C.POINTER(abi.GsClaimQuery),
                                                   C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]
        L.oracle_resolve_capacity_type.restype = C.c_int
        L.oracle_go_sort_ints.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_uint32), C.c_uint32]
        _lib = L
    return _lib


def solve(problem):
    res = abi.GsResult()
    st = lib().oracle_solve(C.byref(problem.struct), C.byref(res))
    if st != abi.GS_OK:
        return st, None, res
    return st, abi.result_to_dict(res, problem), res


def last_groups_created():
    """Spread groups the last solve() created mid-Solve (Topology.Update
    after a relaxation that changed an owner's node filter)."""
    L = lib()
    L.oracle_last_groups_created.restype = C.c_uint64
    return int(L.oracle_last_groups_created())


def feasibility(problem):
    res = abi.GsFeasResult()
    st = lib().oracle_feasibility(C.byref(problem.struct), C.byref(res))
    if st != abi.GS_OK:
        return st, None
    return st, abi.feas_to_dict(res)


def consolidate(cin):
    """cin: gpusched.consolidation.ConsolidationInput -> (status, commands, chosen, multi_options)"""
    res = abi.GsConsolidationResult()
    chosen = C.c_int32(-1)
    mo = (C.c_uint32 * 60)()
    nmo = C.c_uint32(0)
    st = lib().oracle_consolidate(C.byref(cin.struct), C.byref(res), C.byref(chosen), mo, C.byref(nmo))
    if st != abi.GS_OK:
        return st, None, None, None
    return st, abi.commands_to_list(res), int(chosen.value), [int(mo[i]) for i in range(nmo.value)]


def _cstrs(xs):
    arr = (C.c_char_p * max(1, len(xs)))(*[x.encode() for x in xs])
    return arr, len(xs)


def convert_profile(name, vcpu=None, memory_gib=None, arch=None, gpu=None, availability_class=None,
                    zones=(), prices=None, spot_discount_percent=0, unavailable=(), has_client=True,
                    kubelet=None, vcpu_kind=None, memory_kind=None, price_rows=None, unavailable_expiry=None,
                    now_ns=0, gpu_kind=None, region=None):
    """returns (status, text).  price_rows: [(name, zone or None, price)]
    instead of the name-keyed `prices`; unavailable_expiry: per key expiry (ns)"""
    keep = []
    p = OracleProfile()
    p.name = name.encode() if name is not None else None
    p.vcpu_kind = vcpu_kind if vcpu_kind is not None else (0 if vcpu is None else 1)
    p.vcpu = vcpu or 0
    p.memory_kind = memory_kind if memory_kind is not None else (0 if memory_gib is None else 1)
    p.memory_gib = memory_gib or 0
    p.arch = arch.encode() if arch else None
    p.gpu_kind = gpu_kind if gpu_kind is not None else (0 if gpu is None else 1)
    p.gpu = gpu or 0
    if availability_class is None:
        p.avail_kind = 0
    else:
        kind, val = availability_class
        vals = list(val) if kind == "enum" else ([] if val is None else [val])
        arr, n = _cstrs(vals)
        keep.append(arr)
        p.avail_kind = 1 if kind == "enum" else 2
        p.avail_values, p.n_avail_values = arr, n
    e = OracleEnv()
    e.has_client = 1 if has_client else 0
    e.region = region.encode() if region is not None else None
    za, zn = _cstrs(list(zones))
    keep.append(za)
    e.zones, e.n_zones = za, zn
    e.spot_discount_percent = spot_discount_percent
    if price_rows is None:
        price_rows = [(k, None, v) for k, v in (prices or {}).items()]
    pn, n = _cstrs([r[0] for r in price_rows])
    pz = (C.c_char_p * max(1, n))(*[None if r[1] is None else r[1].encode() for r in price_rows])
    pv = (C.c_double * max(1, n))(*[r[2] for r in price_rows])
    keep += [pn, pv, pz]
    e.price_names, e.prices, e.n_prices = pn, pv, n
    e.price_zones = pz
    ua, un = _cstrs(list(unavailable))
    keep.append(ua)
    e.unavailable, e.n_unavailable = ua, un
    if unavailable_expiry is not None:
        ux = (C.c_int64 * max(1, un))(*unavailable_expiry)
        keep.append(ux)
        e.unavailable_expiry = ux
    e.now_ns = now_ns
    if kubelet is not None:
        e.has_nodeclass = 1
        e.has_kubelet = 1
        kr, sr, eh = kubelet.get("kubeReserved", {}), kubelet.get("systemReserved", {}), kubelet.get("evictionHard", {})
        enc = lambda d, k: d[k].encode() if k in d else None  # noqa: E731
        e.kube_reserved_cpu = enc(kr, "cpu")
        e.kube_reserved_memory = enc(kr, "memory")
        e.system_reserved_cpu = enc(sr, "cpu")
        e.system_reserved_memory = enc(sr, "memory")
        e.eviction_memory_available = enc(eh, "memory.available")
    out = C.c_char_p()
    st = lib().oracle_convert_profile(C.byref(p), C.byref(e), C.byref(out))
    return st, out.value.decode()


def parse_text(text):
    """parse oracle_convert_profile's canonical rendering"""
    it = {"offerings": []}
    for line in text.strip().split("\n"):
        k, v = line.split("=", 1)
        if k == "offering":
            z, ct, hexp, _, av = v.split("|")
            import struct
            price = struct.unpack("<d", bytes.fromhex(hexp)[::-1])[0]
            it["offerings"].append((z, ct, price, av == "1"))
        elif k in ("capacity", "overhead"):
            it[k] = {a: int(b) for a, b in (x.split(":") for x in v.split(","))}
        else:
            it[k] = v
    return it


def rank_instance_types(cpu_milli, memory_bytes, price, arch, want_arch=abi.GS_ARCH_ANY, min_cpu=0,
                        min_memory_gb=0, max_price=0.0):
    """oracle_rank_instance_types -> (status, List indices ranked, scores)"""
    return abi.call_rank(lib().oracle_rank_instance_types, cpu_milli, memory_bytes, price, arch, want_arch,
                         min_cpu, min_memory_gb, max_price)


def create_filter(problem):
    """oracle_create_filter over problem.claim_queries -> (status, list like
    gpusched.lib.Solver.create_filter)"""
    nq, n = problem.n_claim_queries, len(problem.instance_types)
    W = (n + 63) // 64
    comp = (C.c_uint64 * max(1, nq * W))()
    reqs = (C.c_uint64 * max(1, nq * W))()
    sel = (C.c_int32 * max(1, nq))()
    ct = (C.c_uint32 * max(1, nq))()
    st = lib().oracle_create_filter(C.byref(problem.struct), problem.claim_queries, nq, comp, reqs, sel, ct)
    if st != abi.GS_OK:
        return st, None
    out = []
    for q in range(nq):
        c = abi._bits(comp, q, W, n)
        out.append(dict(compatible=c, requirements=abi._bits(reqs, q, W, n), n_compatible=len(c),
                        selected=int(sel[q]), capacity_type=int(ct[q])))
    return st, out


def resolve_capacity_type(problem, query_index, its):
    """ResolveCapacityType(claim, [catalog[i] for i in its]) -> (status, GS_CAPACITY_*)"""
    arr = (C.c_uint32 * max(1, len(its)))(*its)
    out = C.c_uint32(0)
    st = lib().oracle_resolve_capacity_type(C.byref(problem.struct), C.byref(problem.claim_queries[query_index]),
                                            arr, len(its), C.byref(out))
    return st, int(out.value)
