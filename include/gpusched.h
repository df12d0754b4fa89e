/*
 * gpusched.h — C-ABI of the MI355X (gfx950) provisioning-solve library.
 *
 * This is the drop-in boundary a Go `pkg/gpusched` (cgo) binds. It replaces,
 * for one call, the in-process work that karpenter-core performs between
 *   CloudProvider.GetInstanceTypes   (reference pkg/cloudprovider/cloudprovider.go:553-583)
 * and the NodeClaims the provisioner creates, i.e. sigs.k8s.io/karpenter@v1.13.0
 *   scheduling.NewScheduler(...).Solve(pods).TruncateInstanceTypes(60)
 * (reached from reference cmd/controller/main.go:76-86; source not vendored,
 * see SURVEY.md §8(b)/(c)).  The IBM catalog that feeds it is produced by
 *   IBMInstanceTypeProvider.List / convertVPCProfileToInstanceType
 *   (reference pkg/providers/common/instancetype/instancetype.go:221-246,659-790).
 *
 * Conventions
 *  - Every string is referenced by an index into gs_problem.strings
 *    (NUL-terminated UTF-8, compared bytewise like Go strings). The empty
 *    string must be present when a field is "unset" (e.g. toleration key "").
 *  - Quantities are int64 milli-units (resource.Quantity.MilliValue()).
 *  - All arrays are caller-owned and only read during the call.
 *  - Result memory (gs_result / gs_feas_result) is owned by the context and
 *    stays valid until the next call on that context or gs_destroy.
 *  - No exceptions cross the ABI; every entry point returns gs_status and
 *    gs_last_error() holds a human-readable message for the last failure.
 *  - One context is single-threaded and not reentrant.
 */
#ifndef GPUSCHED_H
#define GPUSCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum gs_status {
  GS_OK = 0,
  GS_E_INVALID = 1,     /* malformed input (bad index, bad operator, ...) */
  GS_E_UNSUPPORTED = 2, /* input uses a scheduling feature this build does not implement */
  GS_E_CAPACITY = 3,    /* a device capacity limit was exceeded */
  GS_E_HIP = 4,         /* HIP runtime error */
  GS_E_RCCL = 5,        /* RCCL error */
  GS_E_NO_DEVICE = 6    /* no gfx950 device visible */
} gs_status;

/* k8s NodeSelectorOperator (+ Gt/Lt and the v1.13 CRD's Gte/Lte,
 * charts/crds/karpenter.sh_nodepools.yaml:292-300).  Gte x / Lte x are
 * integer bounds, evaluated as Gt x-1 / Lt x+1 (<U>: parity unpinned);
 * their value must parse as an integer (GS_E_INVALID otherwise). */
enum {
  GS_OP_IN = 0,
  GS_OP_NOTIN = 1,
  GS_OP_EXISTS = 2,
  GS_OP_DOES_NOT_EXIST = 3,
  GS_OP_GT = 4,
  GS_OP_LT = 5,
  GS_OP_GTE = 6,
  GS_OP_LTE = 7
};

/* corev1.TolerationOperator ("" is Equal) */
enum { GS_TOL_EQUAL = 0, GS_TOL_EXISTS = 1 };

/* gs_pod.flags: scheduling features present on the pod that this build
 * refuses (GS_E_UNSUPPORTED) rather than silently ignoring.  Pod (anti-)
 * affinity terms, host ports and volumes are passed in their gs_pod ranges;
 * the flags remain for forms those cannot express (for example an affinity
 * term's matchLabelKeys / mismatchLabelKeys). */
enum {
  GS_POD_TOPOLOGY_SPREAD = 1u << 0,
  GS_POD_AFFINITY = 1u << 1,   /* forms gs_pod.affinity cannot express */
  GS_POD_ANTI_AFFINITY = 1u << 2,
  GS_POD_HOST_PORTS = 1u << 3,
  GS_POD_VOLUMES = 1u << 4      /* forms gs_pod.volumes cannot express */
};

typedef struct gs_range {
  uint32_t begin;
  uint32_t count;
} gs_range;

/* one NodeSelectorRequirementWithMinValues */
typedef struct gs_requirement {
  uint32_t key;          /* string id */
  uint32_t op;           /* GS_OP_* */
  gs_range values;       /* into gs_problem.value_ids (string ids) */
  int32_t min_values;    /* -1 when unset.  NodePool requirements: <U> Strict
                            minValues (SatisfiesMinValues in CanAdd, at
                            NewScheduler and after Truncate(60)); claim queries:
                            ignored; pod terms: GS_E_UNSUPPORTED; consolidation
                            and static-matrix column shards: GS_E_UNSUPPORTED */
} gs_requirement;

typedef struct gs_quantity {
  uint32_t resource; /* string id, e.g. "cpu", "memory", "pods", "nvidia.com/gpu" */
  int64_t milli;
} gs_quantity;

typedef struct gs_label {
  uint32_t key;   /* string id */
  uint32_t value; /* string id */
} gs_label;

typedef struct gs_taint {
  uint32_t key, value, effect; /* string ids */
} gs_taint;

typedef struct gs_toleration {
  uint32_t key;    /* string id ("" = any key) */
  uint32_t op;     /* GS_TOL_* */
  uint32_t value;  /* string id */
  uint32_t effect; /* string id ("" = any effect) */
} gs_toleration;

/* a NodeSelectorTerm (required: weight ignored) or a
 * PreferredSchedulingTerm (weight = its weight) */
typedef struct gs_term {
  gs_range requirements; /* into gs_problem.reqs */
  int32_t weight;
} gs_term;

/* cloudprovider.Offering (reference instancetype.go:764-771) */
typedef struct gs_offering {
  gs_range requirements; /* zone In[z], capacity-type In[ct] */
  double price;
  uint32_t available;
} gs_offering;

/* cloudprovider.InstanceType (reference instancetype.go:778-789) */
typedef struct gs_instance_type {
  uint32_t name;         /* string id */
  gs_range requirements; /* into reqs */
  gs_range capacity;     /* into quantities */
  gs_range overhead;     /* into quantities: Overhead.Total() = kube+system+eviction */
  gs_range offerings;    /* into offerings, in reference order (zones x capacity types) */
} gs_instance_type;

/* karpv1.NodePool as seen by NewNodeClaimTemplate */
typedef struct gs_nodepool {
  uint32_t name;            /* string id */
  int32_t weight;
  gs_range requirements;    /* spec.template.spec.requirements */
  gs_range labels;          /* spec.template.metadata.labels */
  gs_range taints;          /* spec.template.spec.taints */
  gs_range limits;          /* spec.limits minus current usage (remaining) */
  uint32_t has_limits;
  gs_range daemon_requests; /* RequestsForPods(compatible daemonset pods) */
  gs_range instance_types;  /* into it_refs: GetInstanceTypes(nodePool) in order */
} gs_nodepool;

/* corev1.TopologySpreadConstraint (<U> karpenter Topology: spread groups on
 * topology.kubernetes.io/zone or kubernetes.io/hostname; other keys and a
 * Honor nodeTaintsPolicy are refused).  matchLabelKeys: for every listed key
 * the pod carries, the selector also requires key In [the pod's value]. */
enum { GS_SPREAD_DO_NOT_SCHEDULE = 0, GS_SPREAD_SCHEDULE_ANYWAY = 1 };
enum { GS_POLICY_HONOR = 0, GS_POLICY_IGNORE = 1 };
typedef struct gs_spread {
  uint32_t topology_key;         /* string id */
  int32_t max_skew;              /* >= 1 */
  uint32_t when_unsatisfiable;   /* GS_SPREAD_* */
  int32_t min_domains;           /* <= 0: unset */
  uint32_t has_selector;         /* 0: nil labelSelector (selects no pod) */
  gs_range match_labels;         /* into labels */
  gs_range match_expressions;    /* into reqs: In / NotIn / Exists / DoesNotExist over pod labels */
  uint32_t node_affinity_policy; /* GS_POLICY_HONOR (default) or GS_POLICY_IGNORE */
  uint32_t node_taints_policy;   /* GS_POLICY_IGNORE (default); HONOR is accepted where every taint of the problem is tolerated by the owner (it then equals IGNORE), else GS_E_UNSUPPORTED */
  gs_range match_label_keys;     /* into value_ids: label keys (string ids) */
} gs_spread;

/* corev1.PodAffinityTerm of spec.affinity.podAffinity or .podAntiAffinity: a
 * required term, or a preferred one with its weight (<U> karpenter Topology:
 * required and not-yet-relaxed preferred terms both constrain the pod).
 *  - anti-affinity (TopologyTypePodAntiAffinity): only domains where no
 *    selected pod runs; a required term also constrains, through the inverse
 *    group, every pod its selector selects;
 *  - affinity (TopologyTypePodAffinity): only domains where a selected pod
 *    runs, or, while none runs anywhere, the pod's own domain when the pod
 *    is selected itself (nextDomainAffinity's bootstrap).
 * topologyKey must be kubernetes.io/hostname (other keys GS_E_UNSUPPORTED:
 * upstream picks a zone bootstrap domain in map order). */
typedef struct gs_affinity_term {
  uint32_t topology_key;       /* string id */
  uint32_t required;           /* 1: requiredDuringScheduling..., 0: preferred */
  int32_t weight;              /* preferred terms: the term's weight */
  uint32_t has_selector;       /* 0: nil labelSelector (selects no pod) */
  gs_range match_labels;       /* into labels */
  gs_range match_expressions;  /* into reqs: In / NotIn / Exists / DoesNotExist */
  gs_range namespaces;         /* into value_ids (string ids) */
  uint32_t has_ns_selector;    /* namespaceSelector set ({} selects every namespace) */
  gs_range ns_match_labels;    /* into labels: over gs_problem.namespaces' labels */
  gs_range ns_match_expressions; /* into reqs */
  /* <U> buildNamespaceList: no namespaces and no selector = the pod's
   * namespace; else the listed ones plus those the selector matches */
} gs_affinity_term;

/* a namespace and its labels (namespaceSelector of pod (anti-)affinity terms) */
typedef struct gs_namespace {
  uint32_t name;    /* string id */
  gs_range labels;  /* into labels */
} gs_namespace;

/* a containers[].ports[] entry with hostPort != 0 (<U> scheduling
 * HostPortUsage: two entries conflict when protocol and port are equal and
 * either hostIP is unspecified or both are equal) */
typedef struct gs_host_port {
  uint32_t protocol;  /* string id; "" = TCP */
  uint32_t ip;        /* string id; "", "0.0.0.0" and "::" = unspecified */
  int32_t port;       /* 1..65535 */
} gs_host_port;

/* a pod volume that counts toward a node's CSI attach limit (<U>
 * scheduling.Volumes from GetVolumes: the CSI driver and the volume's
 * identity, e.g. the bound PV name; two pods naming the same volume share it) */
typedef struct gs_volume {
  uint32_t driver;  /* string id */
  uint32_t id;      /* string id */
} gs_volume;

/* CSINode allocatable attach count of one driver on an existing node */
typedef struct gs_volume_limit {
  uint32_t driver;  /* string id */
  int32_t limit;
} gs_volume_limit;

/* a pod; requests = resources.RequestsForPods(pod) (incl. pods=1) */
typedef struct gs_pod {
  uint32_t uid;             /* string id */
  int64_t creation_ns;      /* metadata.creationTimestamp (ns) */
  gs_range requests;        /* into quantities */
  gs_range node_selector;   /* into labels */
  gs_range required_terms;  /* into terms: requiredDuringScheduling nodeSelectorTerms (OR) */
  gs_range preferred_terms; /* into terms: preferredDuringScheduling, with weights */
  gs_range tolerations;     /* into tolerations */
  uint32_t flags;           /* GS_POD_* */
  uint32_t ns;              /* metadata.namespace (string id) */
  gs_range labels;          /* metadata.labels, into labels (topology selectors) */
  gs_range spreads;         /* spec.topologySpreadConstraints, into spreads */
  gs_range anti_affinity;   /* spec.affinity.podAntiAffinity terms, into affinity_terms */
  gs_range host_ports;      /* host ports of all containers, into host_ports */
  gs_range affinity;        /* spec.affinity.podAffinity terms, into affinity_terms */
  gs_range volumes;         /* CSI volumes, into volumes (<U> ExistingNode.CanAdd VolumeUsage) */
} gs_pod;

/* an existing (state) node: ExistingNode inputs.
 *
 * Taints.  ExistingNode.CanAdd tolerates against <U> StateNode.Taints()
 * (karpenter pkg/controllers/state/statenode.go), which the library computes
 * from the raw fields below, so the caller marshals them as the cluster state
 * holds them and applies no filter of its own:
 *   source   = (managed && !initialized) ? claim_taints : taints
 *   rejected = KnownEphemeralTaints, plus startup_taints when managed && !initialized
 *   Taints() = the source taints that match no rejected taint
 * where a taint matches another when key and effect are equal (corev1
 * Taint.MatchTaint: the value is not compared) and KnownEphemeralTaints are
 *   node.kubernetes.io/not-ready:NoSchedule, node.kubernetes.io/unreachable:NoSchedule,
 *   node.cloudprovider.kubernetes.io/uninitialized:NoSchedule, karpenter.sh/unregistered:NoExecute.
 * So an in-flight node that karpenter launched (its NodeClaim's
 * spec.startupTaints, e.g. NodePool startupTaints, reference test/e2e/
 * e2e_taints_test.go:105-115, CRD karpenter.sh_nodepools.yaml:334) takes the
 * pods its NodeClaim's taints admit while it initializes. */
typedef struct gs_node {
  uint32_t name;        /* string id (also its hostname) */
  uint32_t initialized; /* StateNode.Initialized() */
  gs_range labels;      /* node labels */
  gs_range taints;      /* Node.Spec.Taints (a registered node's current taints) */
  gs_range available;   /* StateNode.Available() */
  gs_range requests;    /* remaining daemonset requests already owed */
  gs_range volume_limits; /* into volume_limits; a driver without an entry has no limit */
  uint32_t managed;     /* StateNode.Managed(): a NodeClaim owns the node (karpenter launched it) */
  gs_range claim_taints;   /* into taints: NodeClaim.Spec.Taints (managed nodes) */
  gs_range startup_taints; /* into taints: NodeClaim.Spec.StartupTaints (managed nodes) */
} gs_node;

typedef struct gs_problem {
  const char* const* strings; uint32_t n_strings;
  const uint32_t* value_ids; uint32_t n_value_ids;
  const gs_requirement* reqs; uint32_t n_reqs;
  const gs_quantity* quantities; uint32_t n_quantities;
  const gs_label* labels; uint32_t n_labels;
  const gs_taint* taints; uint32_t n_taints;
  const gs_toleration* tolerations; uint32_t n_tolerations;
  const gs_term* terms; uint32_t n_terms;
  const uint32_t* it_refs; uint32_t n_it_refs;
  const gs_offering* offerings; uint32_t n_offerings;
  const gs_instance_type* instance_types; uint32_t n_instance_types;
  const gs_nodepool* nodepools; uint32_t n_nodepools;
  const gs_pod* pods; uint32_t n_pods;       /* pending pods (the Solve's pods) */
  const gs_node* nodes; uint32_t n_nodes;
  const gs_spread* spreads; uint32_t n_spreads;
  /* pods bound to state nodes: counted by topology spread selectors; the
   * reschedulable ones are what consolidation simulations move */
  const gs_pod* bound_pods; uint32_t n_bound_pods;
  const uint32_t* bound_pod_node;             /* [n_bound_pods] index into nodes */
  const gs_affinity_term* affinity_terms; uint32_t n_affinity_terms;
  const gs_host_port* host_ports; uint32_t n_host_ports;
  const gs_volume* volumes; uint32_t n_volumes;
  const gs_volume_limit* volume_limits; uint32_t n_volume_limits;
  const gs_namespace* namespaces; uint32_t n_namespaces;
} gs_problem;

/* Results.TruncateInstanceTypes(60) of Scheduler.Solve */
typedef struct gs_result {
  uint32_t n_claims;                 /* new NodeClaims, creation order */
  const uint32_t* claim_nodepool;    /* [n_claims] index into gs_problem.nodepools */
  const uint32_t* claim_pod_offsets; /* [n_claims+1] */
  const uint32_t* claim_pods;        /* pod indices, add order */
  const uint32_t* claim_it_offsets;  /* [n_claims+1] */
  const uint32_t* claim_its;         /* catalog indices, OrderByPrice, <= 60 each */
  const char* const* claim_requirements; /* [n_claims] canonical text */
  uint32_t n_resources;              /* resource vocabulary for claim_requests */
  const uint32_t* resource_names;    /* [n_resources] string ids, ascending by name */
  const int64_t* claim_requests;     /* [n_claims*n_resources] milli */
  uint32_t n_nodes;
  const uint32_t* node_pod_offsets;  /* [n_nodes+1] existing-node assignments */
  const uint32_t* node_pods;
  uint32_t n_errors;
  const uint32_t* error_pods;        /* pods left unschedulable, ascending index */
  /* instrumentation (product only; the oracle reports total only) */
  uint64_t checks;                   /* pod x offering checks of the static matrix */
  uint64_t pops;                     /* queue pops performed */
  uint64_t cand_evals;               /* in-flight NodeClaim candidates scored */
  uint64_t cand_full;                /* ... of which passed the slack prefilter */
  uint64_t sorts_fast, sorts_generic;/* Go sort.Slice emulations by path */
  uint32_t words, n_templates, n_variants; /* encoded sizes: IT words, templates, pod variants */
  double t_encode_ms, t_upload_ms, t_feas_ms, t_ffd_ms, t_truncate_ms, t_fetch_ms, t_total_ms;
  double t_ffd_sort_ms, t_ffd_scan_ms, t_ffd_template_ms; /* in-kernel phase split of t_ffd_ms; -1 = not
                                        measured (the phase timers sit on the pod loop's critical path and
                                        are built only into the GS_FFD_PHASES diagnostic library) */
  uint64_t claim_prefix;             /* in-flight NodeClaims a sequential first-fit visits (first feasible
                                        position + 1, or all): the reference's NodeClaim.CanAdd calls */
  uint64_t node_prefix;              /* ... and existing nodes (ExistingNode.CanAdd calls) */
  double t_run_wall_ms;              /* host wall clock of the last gs_run (launches, kernels, synchronisation) */
  double t_wall_ms;                  /* gs_solve: wall clock of the whole call (prepare + run + fetch); 0 from gs_fetch */
} gs_result;

/* Static pod x offering feasibility (K1/K2): for every (pod, nodepool) the
 * instance types a NodeClaim opened for that pod alone could keep
 * (filterInstanceTypesByRequirements of NodeClaim.CanAdd on a fresh
 * NodeClaim) and the cheapest of them (first of OrderByPrice). */
typedef struct gs_feas_result {
  uint32_t n_pods, n_nodepools, n_its;
  uint32_t words;                  /* u64 words per row = ceil(n_its/64) */
  const uint64_t* rows;            /* [n_pods][n_nodepools][words], bit i = catalog IT i */
  const int32_t* cheapest_it;      /* [n_pods][n_nodepools], -1 if row empty */
  const uint32_t* n_feasible_offerings; /* [n_pods][n_nodepools] */
  uint64_t checks;
  double t_kernel_ms;
  /* OrderByPrice key of the cheapest type: (price_rank << 32) | name_rank,
   * INT64_MAX when the row is empty.  Keys order exactly like Go's
   * (price, name) comparison, signed or unsigned, so a MIN over shards is
   * the global cheapest. */
  const uint64_t* cheapest_key;   /* [n_pods][n_nodepools] */
  const uint32_t* it_name_rank;   /* [n_its] bytewise rank of each type's name */
  uint32_t word_begin, word_end;  /* instance-type words this result covers */
} gs_feas_result;

typedef struct gs_ctx gs_ctx;

/* gs_config.flags */
enum {
  /* run the provisioning Solve on the multi-wave block kernel even when the
   * single-wave kernel applies (both are bit-identical; tests compare them) */
  GS_CFG_BLOCK_SOLVE = 1u << 0,
  /* keep the single-wave Solve's claim scan state in HBM from the first run
     (it moves there by itself when a Solve outgrows the LDS NodeClaims; this
     flag exercises that mode on any problem) */
  GS_CFG_CLAIMS_HBM = 1u << 1,
  /* n_shards > 1 on distinct devices: gs_create also builds an RCCL
     communicator over the shard devices (ncclCommInitAll); the static
     matrix's offering counts (SUM) and cheapest keys (MIN) are then all-reduced
     over it before the row gather.  GS_E_RCCL when RCCL refuses (e.g. a device
     repeats) */
  GS_CFG_RCCL = 1u << 2
};

/* One Go process, several devices: with n_shards > 1 the context owns one
 * child context per shard (HIP device shard_devices[k], a device may repeat)
 * and, from ONE calling thread, runs
 *  - gs_consolidate / gs_consolidate_rerun: simulation s on shard s % n, in
 *    parallel (one host thread per shard), then merges the command tables and
 *    replays SingleNode/MultiNode selection (gs_consolidation_choose) on the
 *    host: the result is identical to the single-device call;
 *  - gs_feasibility / gs_feasibility_shard / gs_feasibility_shard_device:
 *    the requested instance-type words split evenly over the shards, each
 *    shard computes its word slice on its device; a merge kernel on `device`
 *    gathers the slices (peer reads over xGMI; local on a repeated device),
 *    adds the offering counts and keeps the minimum OrderByPrice key (with
 *    GS_CFG_RCCL: counts and keys all-reduced over RCCL first).  The merged
 *    matrix is left in `device`'s memory (gs_feas_device.t_merge_ms);
 *  - the provisioning Solve (gs_prepare/gs_run/gs_fetch) on `device` only: it
 *    is sequential in pod order and does not shard.
 * gs_prepare encodes the problem once and uploads it to every shard (in
 * parallel). */
typedef struct gs_config {
  int32_t device;        /* HIP device ordinal (the Solve's device) */
  uint32_t max_claims;   /* 0 = default */
  uint32_t flags;        /* GS_CFG_* */
  uint32_t n_shards;     /* 0 or 1: single device */
  const int32_t* shard_devices; /* [n_shards] device per shard; NULL: `device` for every shard */
} gs_config;

/* ------------------------------------------------------------------------
 * Consolidation (<U> pkg/controllers/disruption: SimulateScheduling +
 * computeConsolidation, SingleNodeConsolidation, MultiNodeConsolidation;
 * SURVEY.md §3.2).  Each simulation removes a candidate set of state nodes
 * and re-Solves their reschedulable pods together with the pending pods
 * against the remaining nodes.  Every simulation is an independent Solve:
 * the device runs one workgroup per simulation.
 * ------------------------------------------------------------------------ */
enum {
  GS_CONSOLIDATE_EVAL = 0,   /* evaluate the candidate sets in `sets` */
  GS_CONSOLIDATE_SINGLE = 1, /* SingleNodeConsolidation: one set per candidate, in order */
  GS_CONSOLIDATE_MULTI = 2   /* MultiNodeConsolidation: prefixes candidates[0:mid+1] of the binary search */
};

enum { GS_DECISION_NOOP = 0, GS_DECISION_DELETE = 1, GS_DECISION_REPLACE = 2, GS_DECISION_SKIPPED = 3 };

/* why a simulation is a NoOp (computeConsolidation's early returns, in order) */
enum {
  GS_NOOP_NONE = 0,
  GS_NOOP_UNSCHEDULABLE = 1,   /* !AllNonPendingPodsScheduled (incl. uninitialized-node placements) */
  GS_NOOP_MULTIPLE_CLAIMS = 2, /* more than one new NodeClaim */
  GS_NOOP_PRICE_UNKNOWN = 3,   /* getCandidatePrices: no offering of a candidate's type matches its labels */
  GS_NOOP_SPOT_TO_SPOT = 4,    /* all candidates spot, replacement may be spot, SpotToSpotConsolidation off */
  GS_NOOP_NOT_CHEAPER = 5,     /* RemoveInstanceTypeOptionsByPriceAndMinValues left no option */
  GS_NOOP_SAME_TYPE = 6,       /* multi-node: filterOutSameInstanceType left no option */
  GS_NOOP_MIN_VALUES = 7       /* RemoveInstanceTypeOptionsByPriceAndMinValues: the cheaper options miss a minValues requirement */
};

typedef struct gs_consolidation {
  const gs_problem* cluster;        /* catalog, NodePools, ACTIVE state nodes, PENDING pods and the
                                       reschedulable bound pods (cluster->bound_pods) */
  const uint32_t* candidates;       /* candidate node indices, disruption order (sortCandidates) */
  uint32_t n_candidates;
  const gs_range* sets;             /* GS_CONSOLIDATE_EVAL: candidate sets, ranges into candidates[] */
  uint32_t n_sets;
  uint32_t mode;                    /* GS_CONSOLIDATE_* */
  uint32_t max_candidates;          /* MULTI: batch cap (upstream 100); 0 = 100 */
  uint32_t shard_index, shard_count;/* evaluate only sims s with s % shard_count == shard_index (0,0 = all) */
} gs_consolidation;

/* one computeConsolidation outcome */
typedef struct gs_command {
  uint32_t decision;       /* GS_DECISION_* */
  uint32_t reason;         /* GS_NOOP_* */
  uint32_t n_new_claims;   /* NodeClaims the simulation opened */
  uint32_t n_failed_pods;  /* non-pending pods left without a place */
  uint32_t n_candidates;   /* size of the simulated candidate set */
  uint32_t nodepool;       /* REPLACE: the replacement's NodePool index */
  uint32_t spot_only;      /* REPLACE: capacity-type requirement narrowed to spot (OD -> [OD, spot]) */
  gs_range options;        /* REPLACE: catalog IT indices in OrderByPrice order, into result.options */
  double candidate_price;  /* getCandidatePrices */
} gs_command;

typedef struct gs_consolidation_result {
  uint32_t n_commands;     /* one per simulation */
  const gs_command* commands;
  const uint32_t* options;        /* replacement options of all commands */
  const double* option_prices;    /* [same] cheapest available compatible offering price */
  int32_t chosen;          /* SINGLE/MULTI (unsharded): the command the policy returns, -1 = none */
  uint32_t n_multi_options;/* MULTI: the chosen Replace's options after filterOutSameInstanceType */
  const uint32_t* multi_options;
  uint32_t pods_simulated; /* sum over simulations of the pods re-solved */
  uint64_t checks;         /* sum over simulations of pod x (existing node + offering) checks */
  uint64_t node_evals;     /* ExistingNode.CanAdd evaluations the device performed (first-fit scans) */
  uint64_t node_prefix;    /* node positions a sequential first-fit visits */
  uint64_t pops;           /* queue pops over all simulations */
  double t_encode_ms, t_upload_ms, t_feas_ms, t_sim_ms, t_truncate_ms, t_fetch_ms;
} gs_consolidation_result;

/* evaluate consolidation simulations on the device (encode + upload + run + decide) */
gs_status gs_consolidate(gs_ctx* ctx, const gs_consolidation* in, gs_consolidation_result* out);
/* re-run the device part on the same input (bench: inputs stay resident) */
gs_status gs_consolidate_rerun(gs_ctx* ctx, gs_consolidation_result* out);
/* host-only policy replay over a complete command table (e.g. after an
 * all-gather of sharded evaluations): SINGLE = first non-NoOp in order,
 * MULTI = firstNConsolidationOption's binary search with filterOutSameInstanceType.
 * `options`/`option_prices` back the commands' option ranges.  Writes the chosen index (-1 none)
 * and, for MULTI, the surviving options of the chosen command into
 * multi_options (capacity 60) / *n_multi_options. */
gs_status gs_consolidation_choose(const gs_consolidation* in, const gs_command* commands, uint32_t n_commands,
                                  const uint32_t* options, const double* option_prices, int32_t* chosen,
                                  uint32_t* multi_options, uint32_t* n_multi_options);

gs_status gs_create(const gs_config* cfg, gs_ctx** out);
void gs_destroy(gs_ctx* ctx);

/* encode + upload (host -> HBM); inputs become device-resident */
gs_status gs_prepare(gs_ctx* ctx, const gs_problem* problem);
/* run the device solve on the prepared problem (no host<->device traffic
 * except a completion flag); can be called repeatedly */
gs_status gs_run(gs_ctx* ctx);
/* device time (HIP events on the context's stream) of the last gs_run:
 * out[0] feasibility (K1/K2), out[1] FFD (K4), out[2] truncate (K3), ms */
gs_status gs_last_run_ms(const gs_ctx* ctx, double out[3]);
/* fetch + decode the last run's result */
gs_status gs_fetch(gs_ctx* ctx, gs_result* out);
/* prepare + run + fetch */
gs_status gs_solve(gs_ctx* ctx, const gs_problem* problem, gs_result* out);

/* static feasibility matrix only (K1/K2) on a prepared problem */
gs_status gs_feasibility(gs_ctx* ctx, gs_feas_result* out);
/* one instance-type column shard of it: only words
 * [word_begin, word_end) are evaluated; rows carry only those words,
 * n_feasible_offerings counts only those types and cheapest_key is the
 * shard's minimum.  Shards combine exactly: rows OR (disjoint words, so an
 * integer SUM all-reduce works), offering counts SUM, cheapest_key MIN. */
gs_status gs_feasibility_shard(gs_ctx* ctx, uint32_t word_begin, uint32_t word_end, gs_feas_result* out);

/* The same shard left in HBM for an in-place collective (one process per
 * GPU): the matrix at pod-variant granularity (pods with equal scheduling
 * inputs share a variant), device pointers owned by the context and valid
 * until the next call.  Combine over ranks with
 *   ncclAllReduce(rows, rows, n_variants*n_templates*row_stride, ncclUint64, ncclSum)
 *   ncclAllReduce(n_feasible_offerings, ..., n_variants*n_templates, ncclUint32, ncclSum)
 *   ncclAllReduce(cheapest_key, ..., n_variants*n_templates, ncclInt64, ncclMin)
 * then pod p, NodePool template t reads [variant_of_pod[p]][t].  The call
 * returns after the kernel has finished (the buffers are ready for any
 * stream). */
typedef struct gs_feas_device {
  uint32_t n_variants, n_templates, words, row_stride; /* row_stride >= words (u64 units) */
  uint32_t word_begin, word_end;
  uint64_t* rows;                  /* device [n_variants][n_templates][row_stride] */
  uint32_t* n_feasible_offerings;  /* device [n_variants][n_templates] */
  int64_t* cheapest_key;           /* device [n_variants][n_templates] */
  const uint32_t* variant_of_pod;  /* host [n_pods] */
  const uint32_t* template_nodepool; /* host [n_templates] */
  const uint32_t* it_name_rank;    /* host [n_its] */
  uint32_t n_pods, n_its;
  uint64_t checks;                 /* pod x offering checks of the WHOLE matrix */
  double t_kernel_ms;              /* sharded context: the slowest shard's kernels */
  double t_merge_ms;               /* sharded context: the device merge (RCCL reduce + gather kernel) */
} gs_feas_device;

gs_status gs_feasibility_shard_device(gs_ctx* ctx, uint32_t word_begin, uint32_t word_end, gs_feas_device* out);

/* Autoplacement ranking.  Replaces
 * IBMInstanceTypeProvider.FilterInstanceTypes (pkg/providers/common/instancetype/
 * instancetype.go:259-356) + rankInstanceTypes (:358-379); with every filter
 * off it is RankInstanceTypes (:381-420).  Input: n instance types in List
 * order (host buffers): capacity cpu (milli) and memory (bytes), both >= 0,
 * the GetPrice result (0 when the lookup failed), an architecture id.
 * Type i is kept when
 *   (want_arch == GS_ARCH_ANY || arch[i] == want_arch)           :321
 *   && (min_cpu <= 0 || ceil(cpu_milli/1000) >= min_cpu)           :326
 *   && (min_memory_gb <= 0 || bytes / 2^30 >= min_memory_gb)       :331-335 (float64)
 *   && (max_price <= 0 || price <= max_price)                      :339
 * (max_price is the parsed MaximumHourlyPrice; the caller parses the string,
 * as :311-317 does).  The kept types are ordered by calculateInstanceTypeScore
 * (:90-110, float64, lower first) with Go's sort.Slice (pdqsort_func), so
 * ties come out exactly as the reference's.  Writes out_order[0..*out_n)
 * (List indices, ranked) and out_score (same order).  One workgroup on the
 * current device; n <= GS_RANK_MAX (GS_E_CAPACITY above), negative
 * quantities and NaN prices GS_E_INVALID.  Runs on the calling thread's
 * current HIP device (hipSetDevice, or the device of the last gs_* call on
 * this thread); device buffers are kept per device. */
#define GS_ARCH_ANY 0xFFFFFFFFu
#define GS_RANK_MAX 4096u
gs_status gs_rank_instance_types(uint32_t n, const int64_t* cpu_milli, const int64_t* memory_bytes,
                                 const double* price, const uint32_t* arch, uint32_t want_arch, int64_t min_cpu,
                                 int64_t min_memory_gb, double max_price, uint32_t* out_order, uint32_t* out_n,
                                 double* out_score);

/* ------------------------------------------------ launch-time re-filter
 * One NodeClaim as CloudProvider.Create sees it (reference
 * pkg/cloudprovider/cloudprovider.go:284-346): spec.requirements and
 * spec.resources.requests, as ranges into the catalog gs_problem's reqs /
 * quantities arrays (append the claims' requirements to the same pools). */
typedef struct gs_claim_query {
  gs_range requirements; /* NodeClaim spec.requirements (NewNodeSelectorRequirementsWithMinValues) */
  gs_range requests;     /* spec.resources.requests */
} gs_claim_query;

enum { GS_CAPACITY_ON_DEMAND = 0, GS_CAPACITY_SPOT = 1 };

/* Results of gs_create_filter, owned by the ctx (valid until the next
 * gs_create_filter or gs_destroy).  Bitsets are [n_queries][words], bit i of
 * word w = catalog instance type 64*w + i (List order). */
typedef struct gs_claim_filter_result {
  uint32_t n_queries;
  uint32_t words;               /* ceil(n_instance_types / 64) */
  const uint64_t* compatible;   /* Create's filter: reqs.Compatible(it.Requirements, AllowUndefinedWellKnownLabels)
                                   && len(it.Offerings.Compatible(reqs).Available()) > 0
                                   && resources.Fits(requests, it.Allocatable())   cloudprovider.go:322-329 */
  const uint64_t* requirements; /* GetInstanceTypes' filter: reqs.Compatible(it.Requirements, ...) only
                                   (cloudprovider.go:574-577), the claim's requirements standing for the
                                   NodePool template's */
  const uint32_t* n_compatible; /* popcount of `compatible` (0: Create returns InsufficientCapacityError, :345) */
  const int32_t* selected;      /* instanceTypes[0] of the compatible list (vpc/instance/provider.go:215-221),
                                   -1 when empty */
  const uint32_t* capacity_type; /* GS_CAPACITY_*: capacitytype.ResolveCapacityType(nodeClaim, compatible)
                                   (pkg/providers/common/capacitytype/capacitytype.go:27-42) */
} gs_claim_filter_result;

/* Batched CloudProvider.Create re-filter + instance selection + capacity type
 * for n_queries NodeClaims against the catalog's instance types (only the
 * catalog fields of `catalog` are read: strings, value_ids, reqs, quantities,
 * offerings, instance_types).  Requirements use the full scheduling.Requirement
 * algebra (In/NotIn/Exists/DoesNotExist/Gt/Lt/Gte/Lte, any key, label-key
 * normalisation); minValues is ignored, as Compatible ignores it.  One device
 * pass over all (claim, instance type) pairs on the ctx's device. */
gs_status gs_create_filter(gs_ctx* ctx, const gs_problem* catalog, const gs_claim_query* queries,
                           uint32_t n_queries, gs_claim_filter_result* out);

/* ------------------------------------------------------ catalog ingest
 * IBMInstanceTypeProvider.List over the VPC wire data (reference
 * pkg/providers/common/instancetype/instancetype.go:221-246,433-537,659-858;
 * profiles as ListInstanceProfiles returns them, pkg/cloudprovider/ibm/vpc.go:489-495). */

/* the vpcv1.InstanceProfile fields convertVPCProfileToInstanceType reads */
enum { GS_VPC_NIL = 0, GS_VPC_VALUE = 1, GS_VPC_OTHER = 2 };          /* *_kind: nil / the Value variant / another variant */
enum { GS_AVAIL_NIL = 0, GS_AVAIL_ENUM = 1, GS_AVAIL_FIXED = 2 };     /* AvailabilityClass variants */
typedef struct gs_vpc_profile {
  const char* name;                 /* NULL: nil */
  int32_t vcpu_kind; int64_t vcpu;  /* VcpuCount (InstanceProfileVcpu{Value}) */
  int32_t memory_kind; int64_t memory_gib; /* Memory (InstanceProfileMemory{Value}, GiB) */
  const char* arch;                 /* VcpuArchitecture.Value, NULL: nil ("amd64") */
  int32_t gpu_kind; int64_t gpu;    /* GpuCount (InstanceProfileGpu{Value}; other variants count 0) */
  int32_t avail_kind;               /* GS_AVAIL_* */
  const char* const* avail_values; uint32_t n_avail_values; /* Enum values / Fixed value (0 or 1 entries) */
} gs_vpc_profile;

/* PricingProvider.GetPrice(name, zone): the last entry matching name and
 * (zone == NULL or zone); no entry -> 0.0 (instancetype.go:753 drops the error) */
typedef struct gs_price {
  const char* name;
  const char* zone;
  double price;
} gs_price;

/* UnavailableOfferings entries ("<profile>:<zone>:<capacity type>", reference
 * pkg/cache/unavailable_offerings.go:36-77): unavailable while now <= expiry */
typedef struct gs_unavailable {
  const char* key;
  int64_t expiry_unix_ns;
} gs_unavailable;

typedef struct gs_catalog_env {
  const char* const* zones; uint32_t n_zones; /* getZonesForRegion, in order (0: every profile fails) */
  int32_t spot_discount_percent;              /* options.SpotDiscountPercent (0 -> 60) */
  const gs_price* prices; uint32_t n_prices;
  const gs_unavailable* unavailable; uint32_t n_unavailable;
  int64_t now_unix_ns;
  int32_t has_kubelet;                        /* nodeClass != nil && nodeClass.Spec.Kubelet != nil */
  const char* kube_reserved_cpu;              /* NULL: key absent; unparsable: the default (calculateOverhead) */
  const char* kube_reserved_memory;
  const char* system_reserved_cpu;
  const char* system_reserved_memory;
  const char* eviction_memory_available;      /* evictionHard["memory.available"] */
  const char* region;                         /* client.GetRegion(), only for the "no zones found for region %s"
                                                 reason (instancetype.go:738-740); NULL reads as "" */
} gs_catalog_env;

/* The converted catalog in gs_problem form (its own string table): splice
 * strings / value_ids / reqs / quantities / offerings / instance_types into a
 * gs_problem, offsetting the ids, or use them as they are.  Owned by the ctx,
 * valid until the next gs_build_catalog or gs_destroy. */
typedef struct gs_catalog {
  const char* const* strings; uint32_t n_strings;
  const uint32_t* value_ids; uint32_t n_value_ids;
  const gs_requirement* reqs; uint32_t n_reqs;
  const gs_quantity* quantities; uint32_t n_quantities;
  const gs_offering* offerings; uint32_t n_offerings;
  const gs_instance_type* instance_types; uint32_t n_instance_types;
  uint32_t n_skipped;                 /* profiles the conversion refused (List logs and skips them) */
  const uint32_t* skipped;            /* their indices */
  const char* const* skip_reasons;    /* the conversion error text, per skipped profile */
} gs_catalog;

/* List: convert every profile in VPC order, skipping the ones the conversion
 * refuses; GS_E_INVALID when none converts ("no instance types found").
 * Capacity {cpu, memory, pods, nvidia.com/gpu}, requirements {instance-type,
 * arch, instance-family, instance-size}, Overhead.Total() from
 * calculateOverhead, offerings zones x GetSupportedCapacityTypes with the
 * spot discount and the UnavailableOfferings overlay (the price / overlay
 * expansion of all profiles x zones x capacity types runs on the device). */
gs_status gs_build_catalog(gs_ctx* ctx, const gs_vpc_profile* profiles, uint32_t n_profiles,
                           const gs_catalog_env* env, gs_catalog* out);

/* host-only: run the encoder (no device needed) and report whether this
 * build can solve the problem exactly; GS_E_UNSUPPORTED names the feature.
 * A Go caller uses it to choose between this library and upstream Solve. */
gs_status gs_validate(const gs_problem* problem, char* err, size_t err_len);

/* sizeof of every ABI struct, in this order: gs_range, gs_requirement,
 * gs_quantity, gs_label, gs_taint, gs_toleration, gs_term, gs_offering,
 * gs_instance_type, gs_nodepool, gs_pod, gs_node, gs_problem, gs_result,
 * gs_feas_result, gs_config, gs_consolidation, gs_command,
 * gs_consolidation_result, gs_claim_query, gs_claim_filter_result,
 * gs_vpc_profile, gs_price, gs_unavailable, gs_catalog_env, gs_catalog.
 * Bindings check their layouts against it.
 * Returns the number of entries (26); writes min(n, 26). */
uint32_t gs_abi_sizes(uint32_t* out, uint32_t n);

size_t gs_last_error(const gs_ctx* ctx, char* buf, size_t len);
const char* gs_version(void);
/* the first 16 hex digits of the sha256 of the library's sources
 * (karpenter-provider-ibm-cloud_amd/csrc/Makefile SRC_SHA): a binding or a
 * test compares it with the tree it ships with, so a stale prebuilt library
 * is caught before it runs */
const char* gs_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* GPUSCHED_H */
