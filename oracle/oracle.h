/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference algorithm used as the parity checker for
 * the MI355X product library.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so.  The product never
 * links, loads or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *  - catalog conversion (oracle_convert_profile) is PINNED by the reference's
 *    own known-answer tests (instancetype_test.go, capacitytype_test.go);
 *  - Solve / OrderByPrice / Fits semantics live in sigs.k8s.io/karpenter
 *    v1.13.0, which is absent from the container (no Go toolchain, module not
 *    vendored): that part is "parity unpinned" — restated from upstream
 *    behaviour, flagged <U> in comments.
 */
#ifndef GPUSCHED_ORACLE_H
#define GPUSCHED_ORACLE_H

#include "../include/gpusched.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Scheduler.Solve(...).TruncateInstanceTypes(60) restated with string sets.
 * Result memory is owned by the oracle until the next call. */
gs_status oracle_solve(const gs_problem* problem, gs_result* out);

/* static per (pod, nodepool) feasibility: a fresh NodeClaim for the pod */
gs_status oracle_feasibility(const gs_problem* problem, gs_feas_result* out);

/* vpcv1.InstanceProfile subset used by convertVPCProfileToInstanceType */
typedef struct oracle_profile {
  const char* name;        /* NULL = nil */
  int32_t vcpu_kind;       /* 0 nil, 1 InstanceProfileVcpu{Value}, 2 other type */
  int64_t vcpu;
  int32_t memory_kind;     /* 0 nil, 1 InstanceProfileMemory{Value}, 2 other type */
  int64_t memory_gib;
  const char* arch;        /* NULL = VcpuArchitecture nil */
  int32_t gpu_kind;        /* 0 nil, 1 InstanceProfileGpu{Value}, 2 other type */
  int64_t gpu;
  int32_t avail_kind;      /* 0 nil, 1 Enum{Values}, 2 Fixed{Value} */
  const char* const* avail_values; uint32_t n_avail_values; /* Fixed: 0 (nil) or 1 */
} oracle_profile;

typedef struct oracle_catalog_env {
  int32_t has_client;                  /* p.client != nil */
  const char* const* zones; uint32_t n_zones; /* getZonesForRegion result */
  int32_t spot_discount_percent;       /* options.FromContext(ctx).SpotDiscountPercent */
  const char* const* price_names; const double* prices; uint32_t n_prices; /* GetPrice table */
  const char* const* unavailable; uint32_t n_unavailable; /* "name:zone:ct" keys */
  int32_t has_nodeclass, has_kubelet;
  const char* kube_reserved_cpu;       /* NULL = key absent */
  const char* kube_reserved_memory;
  const char* system_reserved_cpu;
  const char* system_reserved_memory;
  const char* eviction_memory_available;
  const char* const* price_zones;      /* NULL, or per price entry its zone (NULL entry: every zone) */
  const int64_t* unavailable_expiry;   /* NULL: entries never expire; else unavailable while now <= expiry */
  int64_t now_ns;
  const char* region;                  /* p.client.GetRegion() (NULL = "") */
} oracle_catalog_env;

/* convertVPCProfileToInstanceType.  On success returns GS_OK and a
 * canonical text rendering (see oracle/catalog.cpp) valid until next call;
 * on a conversion error returns GS_E_INVALID and the error text. */
gs_status oracle_convert_profile(const oracle_profile* profile, const oracle_catalog_env* env,
                                 const char** text_out);

/* resource.ParseQuantity(s).MilliValue(); returns 0 on success */
int oracle_parse_quantity_milli(const char* s, int64_t* milli_out);

/* getInstanceFamily / getInstanceSize (instancetype.go:861-877) */
const char* oracle_instance_family(const char* name);
const char* oracle_instance_size(const char* name);
/* GetCapacityTypeFromAvailabilityClass (capacitytype.go:75-85) */
const char* oracle_capacity_type(const char* availability_class);
/* calculateInstanceTypeScore (instancetype.go:90-110) for cpu/memory quantities */
double oracle_instance_score(int64_t cpu_milli, int64_t memory_bytes, double price);
/* FilterInstanceTypes (instancetype.go:259-356) + rankInstanceTypes (:358-379):
 * the CPU restatement of gs_rank_instance_types (same arguments and result;
 * GS_E_INVALID / GS_E_CAPACITY on the same inputs, no device needed). */
gs_status oracle_rank_instance_types(uint32_t n, const int64_t* cpu_milli, const int64_t* memory_bytes,
                                     const double* price, const uint32_t* arch, uint32_t want_arch, int64_t min_cpu,
                                     int64_t min_memory_gb, double max_price, uint32_t* out_order, uint32_t* out_n,
                                     double* out_score);

/* <U> disruption consolidation (SimulateScheduling + computeConsolidation and
 * the single/multi-node policies), one naive Solve per simulation.  For MULTI
 * the surviving options of the chosen command (after filterOutSameInstanceType)
 * go to multi_opts (capacity 60). */
gs_status oracle_consolidate(const gs_consolidation* in, gs_consolidation_result* out, int32_t* chosen,
                             uint32_t* multi_opts, uint32_t* n_multi_opts);

/* CloudProvider.Create's filter + instanceTypes[0] + ResolveCapacityType and
 * GetInstanceTypes' requirement filter, per claim: the CPU restatement of
 * gs_create_filter.  Bitsets [n][ceil(n_instance_types/64)], caller-owned. */
gs_status oracle_create_filter(const gs_problem* catalog, const gs_claim_query* queries, uint32_t n,
                               uint64_t* compatible, uint64_t* requirements, int32_t* selected,
                               uint32_t* capacity_type);
/* capacitytype.ResolveCapacityType(nodeClaim, instanceTypes) over an explicit
 * list of catalog indices (capacitytype.go:27-42) */
gs_status oracle_resolve_capacity_type(const gs_problem* catalog, const gs_claim_query* query, const uint32_t* its,
                                       uint32_t n, uint32_t* out);

/* Go sort.Slice (pdqsort_func) applied to an int array with Less = a[i] < a[j];
 * perm receives the resulting permutation of original indices. */
void oracle_go_sort_ints(int64_t* keys, uint32_t* perm, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
