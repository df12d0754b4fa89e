"""ctypes / numpy mirror of include/gpusched.h (the C-ABI boundary).

Struct layouts here must match the header byte for byte; tests/test_abi.py
checks sizes against the compiled library's own sizeof table (gs_abi_sizes).
"""
import ctypes as C

import numpy as np

GS_OK, GS_E_INVALID, GS_E_UNSUPPORTED, GS_E_CAPACITY, GS_E_HIP, GS_E_RCCL, GS_E_NO_DEVICE = range(7)
STATUS_NAMES = {
    0: "GS_OK", 1: "GS_E_INVALID", 2: "GS_E_UNSUPPORTED", 3: "GS_E_CAPACITY",
    4: "GS_E_HIP", 5: "GS_E_RCCL", 6: "GS_E_NO_DEVICE",
}

OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_GTE, OP_LTE = range(8)
OPS = {"In": OP_IN, "NotIn": OP_NOTIN, "Exists": OP_EXISTS, "DoesNotExist": OP_DNE,
       "Gt": OP_GT, "Lt": OP_LT, "Gte": OP_GTE, "Lte": OP_LTE}
TOL_EQUAL, TOL_EXISTS = 0, 1

POD_TOPOLOGY_SPREAD = 1 << 0
POD_AFFINITY = 1 << 1
POD_ANTI_AFFINITY = 1 << 2
POD_HOST_PORTS = 1 << 3
POD_VOLUMES = 1 << 4

# numpy dtypes (align=True reproduces the C layout on x86-64)
RANGE = [("begin", "<u4"), ("count", "<u4")]
DT_REQ = np.dtype([("key", "<u4"), ("op", "<u4"), ("values", RANGE), ("min_values", "<i4")], align=True)
DT_QTY = np.dtype([("resource", "<u4"), ("milli", "<i8")], align=True)
DT_LABEL = np.dtype([("key", "<u4"), ("value", "<u4")], align=True)
DT_TAINT = np.dtype([("key", "<u4"), ("value", "<u4"), ("effect", "<u4")], align=True)
DT_TOL = np.dtype([("key", "<u4"), ("op", "<u4"), ("value", "<u4"), ("effect", "<u4")], align=True)
DT_TERM = np.dtype([("requirements", RANGE), ("weight", "<i4")], align=True)
DT_OFFERING = np.dtype([("requirements", RANGE), ("price", "<f8"), ("available", "<u4")], align=True)
DT_IT = np.dtype([("name", "<u4"), ("requirements", RANGE), ("capacity", RANGE), ("overhead", RANGE),
                  ("offerings", RANGE)], align=True)
DT_NODEPOOL = np.dtype([("name", "<u4"), ("weight", "<i4"), ("requirements", RANGE), ("labels", RANGE),
                        ("taints", RANGE), ("limits", RANGE), ("has_limits", "<u4"),
                        ("daemon_requests", RANGE), ("instance_types", RANGE)], align=True)
DT_POD = np.dtype([("uid", "<u4"), ("creation_ns", "<i8"), ("requests", RANGE), ("node_selector", RANGE),
                   ("required_terms", RANGE), ("preferred_terms", RANGE), ("tolerations", RANGE),
                   ("flags", "<u4"), ("ns", "<u4"), ("labels", RANGE), ("spreads", RANGE),
                   ("anti_affinity", RANGE), ("host_ports", RANGE), ("affinity", RANGE), ("volumes", RANGE)],
                  align=True)
DT_VOLUME = np.dtype([("driver", "<u4"), ("id", "<u4")], align=True)
DT_VOLUME_LIMIT = np.dtype([("driver", "<u4"), ("limit", "<i4")], align=True)
DT_AFFINITY = np.dtype([("topology_key", "<u4"), ("required", "<u4"), ("weight", "<i4"), ("has_selector", "<u4"),
                    ("match_labels", RANGE), ("match_expressions", RANGE), ("namespaces", RANGE),
                    ("has_ns_selector", "<u4"), ("ns_match_labels", RANGE), ("ns_match_expressions", RANGE)],
                   align=True)
DT_NAMESPACE = np.dtype([("name", "<u4"), ("labels", RANGE)], align=True)
DT_HOSTPORT = np.dtype([("protocol", "<u4"), ("ip", "<u4"), ("port", "<i4")], align=True)
SPREAD_DO_NOT_SCHEDULE, SPREAD_SCHEDULE_ANYWAY = 0, 1
POLICY_HONOR, POLICY_IGNORE = 0, 1
DT_SPREAD = np.dtype([("topology_key", "<u4"), ("max_skew", "<i4"), ("when_unsatisfiable", "<u4"),
                      ("min_domains", "<i4"), ("has_selector", "<u4"), ("match_labels", RANGE),
                      ("match_expressions", RANGE), ("node_affinity_policy", "<u4"),
                      ("node_taints_policy", "<u4"), ("match_label_keys", RANGE)], align=True)
DT_NODE = np.dtype([("name", "<u4"), ("initialized", "<u4"), ("labels", RANGE), ("taints", RANGE),
                    ("available", RANGE), ("requests", RANGE), ("volume_limits", RANGE), ("managed", "<u4"),
                    ("claim_taints", RANGE), ("startup_taints", RANGE)], align=True)
# <U> scheduling.KnownEphemeralTaints (key, effect): StateNode.Taints() drops them
EPHEMERAL_TAINTS = (("node.kubernetes.io/not-ready", "NoSchedule"), ("node.kubernetes.io/unreachable", "NoSchedule"),
                    ("node.cloudprovider.kubernetes.io/uninitialized", "NoSchedule"),
                    ("karpenter.sh/unregistered", "NoExecute"))

_P = C.c_void_p
_U32 = C.c_uint32


class GsProblem(C.Structure):
    _fields_ = [
        ("strings", C.POINTER(C.c_char_p)), ("n_strings", _U32),
        ("value_ids", _P), ("n_value_ids", _U32),
        ("reqs", _P), ("n_reqs", _U32),
        ("quantities", _P), ("n_quantities", _U32),
        ("labels", _P), ("n_labels", _U32),
        ("taints", _P), ("n_taints", _U32),
        ("tolerations", _P), ("n_tolerations", _U32),
        ("terms", _P), ("n_terms", _U32),
        ("it_refs", _P), ("n_it_refs", _U32),
        ("offerings", _P), ("n_offerings", _U32),
        ("instance_types", _P), ("n_instance_types", _U32),
        ("nodepools", _P), ("n_nodepools", _U32),
        ("pods", _P), ("n_pods", _U32),
        ("nodes", _P), ("n_nodes", _U32),
        ("spreads", _P), ("n_spreads", _U32),
        ("bound_pods", _P), ("n_bound_pods", _U32),
        ("bound_pod_node", _P),
        ("affinity_terms", _P), ("n_affinity_terms", _U32),
        ("host_ports", _P), ("n_host_ports", _U32),
        ("volumes", _P), ("n_volumes", _U32),
        ("volume_limits", _P), ("n_volume_limits", _U32),
        ("namespaces", _P), ("n_namespaces", _U32),
    ]


class GsResult(C.Structure):
    _fields_ = [
        ("n_claims", _U32),
        ("claim_nodepool", C.POINTER(C.c_uint32)),
        ("claim_pod_offsets", C.POINTER(C.c_uint32)),
        ("claim_pods", C.POINTER(C.c_uint32)),
        ("claim_it_offsets", C.POINTER(C.c_uint32)),
        ("claim_its", C.POINTER(C.c_uint32)),
        ("claim_requirements", C.POINTER(C.c_char_p)),
        ("n_resources", _U32),
        ("resource_names", C.POINTER(C.c_uint32)),
        ("claim_requests", C.POINTER(C.c_int64)),
        ("n_nodes", _U32),
        ("node_pod_offsets", C.POINTER(C.c_uint32)),
        ("node_pods", C.POINTER(C.c_uint32)),
        ("n_errors", _U32),
        ("error_pods", C.POINTER(C.c_uint32)),
        ("checks", C.c_uint64),
        ("pops", C.c_uint64),
        ("cand_evals", C.c_uint64),
        ("cand_full", C.c_uint64),
        ("sorts_fast", C.c_uint64), ("sorts_generic", C.c_uint64),
        ("words", _U32), ("n_templates", _U32), ("n_variants", _U32),
        ("t_encode_ms", C.c_double), ("t_upload_ms", C.c_double), ("t_feas_ms", C.c_double),
        ("t_ffd_ms", C.c_double), ("t_truncate_ms", C.c_double), ("t_fetch_ms", C.c_double),
        ("t_total_ms", C.c_double),
        ("t_ffd_sort_ms", C.c_double), ("t_ffd_scan_ms", C.c_double), ("t_ffd_template_ms", C.c_double),
        ("claim_prefix", C.c_uint64), ("node_prefix", C.c_uint64),
        ("t_run_wall_ms", C.c_double), ("t_wall_ms", C.c_double),
    ]


class GsFeasDevice(C.Structure):
    """gs_feas_device: one shard of the static matrix left in HBM (variant granularity)"""
    _fields_ = [
        ("n_variants", _U32), ("n_templates", _U32), ("words", _U32), ("row_stride", _U32),
        ("word_begin", _U32), ("word_end", _U32),
        ("rows", C.c_void_p), ("n_feasible_offerings", C.c_void_p), ("cheapest_key", C.c_void_p),
        ("variant_of_pod", C.POINTER(C.c_uint32)), ("template_nodepool", C.POINTER(C.c_uint32)),
        ("it_name_rank", C.POINTER(C.c_uint32)),
        ("n_pods", _U32), ("n_its", _U32),
        ("checks", C.c_uint64),
        ("t_kernel_ms", C.c_double), ("t_merge_ms", C.c_double),
    ]


class GsFeasResult(C.Structure):
    _fields_ = [
        ("n_pods", _U32), ("n_nodepools", _U32), ("n_its", _U32), ("words", _U32),
        ("rows", C.POINTER(C.c_uint64)),
        ("cheapest_it", C.POINTER(C.c_int32)),
        ("n_feasible_offerings", C.POINTER(C.c_uint32)),
        ("checks", C.c_uint64),
        ("t_kernel_ms", C.c_double),
        ("cheapest_key", C.POINTER(C.c_uint64)),
        ("it_name_rank", C.POINTER(C.c_uint32)),
        ("word_begin", _U32), ("word_end", _U32),
    ]


GS_CFG_BLOCK_SOLVE = 1  # gs_config.flags: run the Solve on the block kernel
GS_CFG_CLAIMS_HBM = 2   # gs_config.flags: single-wave Solve with its claim scan state in HBM
GS_CFG_RCCL = 4         # gs_config.flags: sharded context with an RCCL communicator over the shard devices


class GsConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_claims", _U32), ("flags", _U32), ("n_shards", _U32),
                ("shard_devices", C.POINTER(C.c_int32))]


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def result_to_dict(res: GsResult, problem) -> dict:
    """Canonical, comparable form of a gs_result (copied out of library memory)."""
    nc = res.n_claims
    cpo = _arr(res.claim_pod_offsets, nc + 1, np.uint32)
    cpods = _arr(res.claim_pods, int(cpo[-1]) if nc else 0, np.uint32)
    cio = _arr(res.claim_it_offsets, nc + 1, np.uint32)
    cits = _arr(res.claim_its, int(cio[-1]) if nc else 0, np.uint32)
    npool = _arr(res.claim_nodepool, nc, np.uint32)
    nr = res.n_resources
    rnames = [problem.strings[i] for i in _arr(res.resource_names, nr, np.uint32)]
    creq = _arr(res.claim_requests, nc * nr, np.int64).reshape(nc, nr) if nr else np.zeros((nc, 0), np.int64)
    claims = []
    for c in range(nc):
        claims.append({
            "nodepool": int(npool[c]),
            "pods": [int(x) for x in cpods[cpo[c]:cpo[c + 1]]],
            "its": [int(x) for x in cits[cio[c]:cio[c + 1]]],
            "requirements": res.claim_requirements[c].decode(),
            "requests": {rnames[k]: int(creq[c, k]) for k in range(nr) if creq[c, k] != 0},
        })
    nn = res.n_nodes
    npo = _arr(res.node_pod_offsets, nn + 1, np.uint32)
    npods = _arr(res.node_pods, int(npo[-1]) if nn else 0, np.uint32)
    nodes = [[int(x) for x in npods[npo[i]:npo[i + 1]]] for i in range(nn)]
    errors = [int(x) for x in _arr(res.error_pods, res.n_errors, np.uint32)]
    return {"claims": claims, "nodes": nodes, "errors": errors}


def feas_to_dict(res: GsFeasResult) -> dict:
    P, T, W = res.n_pods, res.n_nodepools, res.words
    rows = _arr(res.rows, P * T * W, np.uint64).reshape(P, T, W) if P * T * W else np.zeros((P, T, W), np.uint64)
    cheapest = _arr(res.cheapest_it, P * T, np.int32).reshape(P, T)
    nfo = _arr(res.n_feasible_offerings, P * T, np.uint32).reshape(P, T)
    out = {"rows": rows, "cheapest": cheapest, "n_feasible_offerings": nfo, "checks": int(res.checks)}
    if res.cheapest_key:  # product results (the oracle reports no keys)
        out["cheapest_key"] = _arr(res.cheapest_key, P * T, np.uint64).reshape(P, T)
        out["it_name_rank"] = _arr(res.it_name_rank, res.n_its, np.uint32)
        out["word_range"] = (int(res.word_begin), int(res.word_end))
    return out


# ------------------------------------------------------------ consolidation
CONSOLIDATE_EVAL, CONSOLIDATE_SINGLE, CONSOLIDATE_MULTI = 0, 1, 2
DECISION_NOOP, DECISION_DELETE, DECISION_REPLACE, DECISION_SKIPPED = 0, 1, 2, 3
DECISION_NAMES = {0: "NoOp", 1: "Delete", 2: "Replace", 3: "Skipped"}
(NOOP_NONE, NOOP_UNSCHEDULABLE, NOOP_MULTIPLE_CLAIMS, NOOP_PRICE_UNKNOWN, NOOP_SPOT_TO_SPOT,
 NOOP_NOT_CHEAPER, NOOP_SAME_TYPE, NOOP_MIN_VALUES) = range(8)


class GsRange(C.Structure):
    _fields_ = [("begin", _U32), ("count", _U32)]


class GsConsolidation(C.Structure):
    _fields_ = [
        ("cluster", C.POINTER(GsProblem)),
        ("candidates", _P), ("n_candidates", _U32),
        ("sets", _P), ("n_sets", _U32),
        ("mode", _U32), ("max_candidates", _U32),
        ("shard_index", _U32), ("shard_count", _U32),
    ]


class GsCommand(C.Structure):
    _fields_ = [
        ("decision", _U32), ("reason", _U32), ("n_new_claims", _U32), ("n_failed_pods", _U32),
        ("n_candidates", _U32), ("nodepool", _U32), ("spot_only", _U32), ("options", GsRange),
        ("candidate_price", C.c_double),
    ]


class GsConsolidationResult(C.Structure):
    _fields_ = [
        ("n_commands", _U32),
        ("commands", C.POINTER(GsCommand)),
        ("options", C.POINTER(C.c_uint32)),
        ("option_prices", C.POINTER(C.c_double)),
        ("chosen", C.c_int32),
        ("n_multi_options", _U32),
        ("multi_options", C.POINTER(C.c_uint32)),
        ("pods_simulated", _U32),
        ("checks", C.c_uint64),
        ("node_evals", C.c_uint64),
        ("node_prefix", C.c_uint64),
        ("pops", C.c_uint64),
        ("t_encode_ms", C.c_double), ("t_upload_ms", C.c_double), ("t_feas_ms", C.c_double),
        ("t_sim_ms", C.c_double), ("t_truncate_ms", C.c_double), ("t_fetch_ms", C.c_double),
    ]


class GsClaimQuery(C.Structure):
    _fields_ = [("requirements", GsRange), ("requests", GsRange)]


GS_CAPACITY_ON_DEMAND, GS_CAPACITY_SPOT = 0, 1


class GsClaimFilterResult(C.Structure):
    _fields_ = [
        ("n_queries", _U32), ("words", _U32),
        ("compatible", C.POINTER(C.c_uint64)),
        ("requirements", C.POINTER(C.c_uint64)),
        ("n_compatible", C.POINTER(C.c_uint32)),
        ("selected", C.POINTER(C.c_int32)),
        ("capacity_type", C.POINTER(C.c_uint32)),
    ]


def _bits(ptr, q, words, n):
    return [64 * w + i for w in range(words) for i in range(64)
            if (ptr[q * words + w] >> i) & 1 and 64 * w + i < n]


def claim_filter_to_list(res: GsClaimFilterResult, n_types: int) -> list:
    """per query: {compatible: [catalog indices], requirements: [...],
    selected, capacity_type} (List order)"""
    out = []
    for q in range(res.n_queries):
        out.append(dict(compatible=_bits(res.compatible, q, res.words, n_types),
                        requirements=_bits(res.requirements, q, res.words, n_types),
                        n_compatible=int(res.n_compatible[q]), selected=int(res.selected[q]),
                        capacity_type=int(res.capacity_type[q])))
    return out


GS_VPC_NIL, GS_VPC_VALUE, GS_VPC_OTHER = 0, 1, 2
GS_AVAIL_NIL, GS_AVAIL_ENUM, GS_AVAIL_FIXED = 0, 1, 2


class GsVpcProfile(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("vcpu_kind", C.c_int32), ("vcpu", C.c_int64),
        ("memory_kind", C.c_int32), ("memory_gib", C.c_int64), ("arch", C.c_char_p),
        ("gpu_kind", C.c_int32), ("gpu", C.c_int64), ("avail_kind", C.c_int32),
        ("avail_values", C.POINTER(C.c_char_p)), ("n_avail_values", _U32),
    ]


class GsPrice(C.Structure):
    _fields_ = [("name", C.c_char_p), ("zone", C.c_char_p), ("price", C.c_double)]


class GsUnavailable(C.Structure):
    _fields_ = [("key", C.c_char_p), ("expiry_unix_ns", C.c_int64)]


class GsCatalogEnv(C.Structure):
    _fields_ = [
        ("zones", C.POINTER(C.c_char_p)), ("n_zones", _U32),
        ("spot_discount_percent", C.c_int32),
        ("prices", C.POINTER(GsPrice)), ("n_prices", _U32),
        ("unavailable", C.POINTER(GsUnavailable)), ("n_unavailable", _U32),
        ("now_unix_ns", C.c_int64),
        ("has_kubelet", C.c_int32),
        ("kube_reserved_cpu", C.c_char_p), ("kube_reserved_memory", C.c_char_p),
        ("system_reserved_cpu", C.c_char_p), ("system_reserved_memory", C.c_char_p),
        ("eviction_memory_available", C.c_char_p),
        ("region", C.c_char_p),
    ]


class GsCatalog(C.Structure):
    _fields_ = [
        ("strings", C.POINTER(C.c_char_p)), ("n_strings", _U32),
        ("value_ids", C.POINTER(C.c_uint32)), ("n_value_ids", _U32),
        ("reqs", _P), ("n_reqs", _U32),
        ("quantities", _P), ("n_quantities", _U32),
        ("offerings", _P), ("n_offerings", _U32),
        ("instance_types", _P), ("n_instance_types", _U32),
        ("n_skipped", _U32), ("skipped", C.POINTER(C.c_uint32)),
        ("skip_reasons", C.POINTER(C.c_char_p)),
    ]


def _np_view(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n * np.dtype(dtype).itemsize,))
    return raw.view(dtype).copy()


def catalog_to_list(cat: GsCatalog) -> list:
    """gs_catalog -> [{name, requirements [(key, op, [values])], capacity {res: milli},
    overhead {res: milli}, offerings [(zone, ct, price, available)]}] in List order"""
    strs = [cat.strings[i].decode() for i in range(cat.n_strings)]
    vals = [int(cat.value_ids[i]) for i in range(cat.n_value_ids)]
    reqs = _np_view(cat.reqs, cat.n_reqs, DT_REQ)
    qty = _np_view(cat.quantities, cat.n_quantities, DT_QTY)
    offs = _np_view(cat.offerings, cat.n_offerings, DT_OFFERING)
    its = _np_view(cat.instance_types, cat.n_instance_types, DT_IT)
    ops = {v: k for k, v in OPS.items()}

    def rl(b, n):
        out = []
        for r in reqs[b:b + n]:
            vb, vn = r["values"]
            out.append((strs[r["key"]], ops[int(r["op"])], [strs[v] for v in vals[vb:vb + vn]]))
        return out

    def ql(b, n):
        d = {}
        for q in qty[b:b + n]:
            d[strs[q["resource"]]] = d.get(strs[q["resource"]], 0) + int(q["milli"])
        return d

    out = []
    for it in its:
        ob, on = it["offerings"]
        ol = []
        for o in offs[ob:ob + on]:
            rb, rn = o["requirements"]
            d = {k: v[0] for k, _, v in rl(rb, rn)}
            ol.append((d["topology.kubernetes.io/zone"], d["karpenter.sh/capacity-type"], float(o["price"]),
                       bool(o["available"])))
        out.append({"name": strs[it["name"]], "requirements": rl(*it["requirements"]),
                    "capacity": ql(*it["capacity"]), "overhead": ql(*it["overhead"]), "offerings": ol})
    return out


def commands_to_list(res: GsConsolidationResult) -> list:
    """Canonical, comparable form of the commands (copied out of library memory)."""
    out = []
    for i in range(res.n_commands):
        c = res.commands[i]
        opts = [int(res.options[c.options.begin + k]) for k in range(c.options.count)]
        prices = [float(res.option_prices[c.options.begin + k]) for k in range(c.options.count)]
        out.append({"decision": int(c.decision), "reason": int(c.reason), "n_new_claims": int(c.n_new_claims),
                    "n_failed_pods": int(c.n_failed_pods), "n_candidates": int(c.n_candidates),
                    "nodepool": int(c.nodepool) if c.decision == DECISION_REPLACE else None,
                    "spot_only": int(c.spot_only), "options": opts, "option_prices": prices,
                    "candidate_price": float(c.candidate_price)})
    return out


# gs_rank_instance_types / oracle_rank_instance_types (include/gpusched.h)
GS_ARCH_ANY = 0xFFFFFFFF
GS_RANK_MAX = 4096
RANK_ARGTYPES = [C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                 C.POINTER(C.c_uint32), C.c_uint32, C.c_int64, C.c_int64, C.c_double,
                 C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_double)]


def call_rank(fn, cpu_milli, memory_bytes, price, arch, want_arch=GS_ARCH_ANY, min_cpu=0, min_memory_gb=0,
              max_price=0.0):
    """marshal one ranking call -> (status, List indices in ranked order, scores)"""
    n = len(cpu_milli)
    m = max(n, 1)
    cpu = np.ascontiguousarray(cpu_milli, dtype=np.int64)
    mem = np.ascontiguousarray(memory_bytes, dtype=np.int64)
    pr = np.ascontiguousarray(price, dtype=np.float64)
    ar = np.ascontiguousarray(arch, dtype=np.uint32)
    order = np.zeros(m, dtype=np.uint32)
    score = np.zeros(m, dtype=np.float64)
    kept = C.c_uint32(0)
    p = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    st = fn(n, p(cpu, C.c_int64), p(mem, C.c_int64), p(pr, C.c_double), p(ar, C.c_uint32), want_arch,
            int(min_cpu), int(min_memory_gb), float(max_price), p(order, C.c_uint32), C.byref(kept),
            p(score, C.c_double))
    k = kept.value
    return st, order[:k].tolist(), score[:k].tolist()
