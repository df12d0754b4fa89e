// layout.hpp — HBM layout shared by the host encoder and the gfx950 kernels.
//
// Everything the device touches is plain-old-data in structure-of-arrays form:
//  * label vocabularies: every requirement key gets a value vocabulary; a
//    requirement on a key becomes a "has" bitset over that vocabulary
//    (Requirement.Has(v) for every vocabulary value) plus, for complement
//    sets, the explicit excluded values and integer bounds;
//  * instance types (ITs) are columns: one bit per IT in u64 words (W words);
//  * offerings are folded per IT into a (zone x capacity-type) "pair" grid
//    bitmask (Z*C <= 64 bits) of AVAILABLE offerings;
//  * resources are int64 milli-units, R <= RMAX per vector.
#pragma once
#include <stdint.h>
#include <stddef.h>

// host-only builds of the encoder (g++ with sanitizers, tools/encode_harness.cpp)
// see the shared records without the HIP function attributes
#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace gsd {

constexpr int RMAX = 8;        // resource dimensions per vector
constexpr int KMAX_IT = 8;     // requirement keys carried by instance types
// simulations with at most OVH_MAX overlay entries keep their node -> entry
// map in an LDS hash (2 slots per entry, power of two) instead of a per-block
// NN-entry array in HBM
constexpr uint32_t OVH_MAX = 128;
inline uint32_t ovh_slots_for(uint32_t ov_cap) {
  if (ov_cap > OVH_MAX) return 0;
  uint32_t s = 16;
  while (s < 2 * ov_cap) s <<= 1;
  return s;
}
constexpr int FMAX = 16;       // "free" key slots (keys on neither ITs nor offerings)
constexpr int TMAX = 64;       // NodeClaim templates (NodePools)
constexpr uint32_t THR_LDS_MAX = 2048;   // fit thresholds staged in the FFD kernel's LDS
constexpr uint32_t SLOT_LDS_MAX = 1024;  // (zone, capacity-type) pair type-set words in LDS
constexpr int SMAX = 16;       // offerings per instance type
constexpr int TGMAX = 4096;    // topology groups (spread, pod (anti-)affinity, inverse, host ports)
constexpr int OWNMAX = 64;     // topology groups one pod variant owns
constexpr int ZVMAX = 64;      // zone vocabulary (topology domains) when zone groups are used
// topology group kinds (TGroupRec.kind, and the top byte of a selection-list entry)
// selection-list kind bits (entry >> 24); TK_LAZY: a spread group created by
// a relaxation (Topology.Update), lazy index in entry bits 12..23, slot in
// bits 0..11; Record skips it until some pod has relaxed into it
enum : uint32_t { TK_HOST = 1u, TK_AFF = 2u, TK_ANTI = 4u, TK_LAZY = 8u };
constexpr uint32_t LZ_HOST = 1u << 31;  // lazy_slot: a hostname group (its slot is a column of hc)
// a NodeClaim's count cell of a lazy hostname group created after the claim:
// the claim is no domain of it (Topology.Register ran before the group
// existed), so every owner check fails there; Record makes it a domain with
// count 1 (TopologyGroup.Record), hence count = (cell & HC_COUNT) + 1
constexpr int32_t HC_UNKNOWN = 0x40000000, HC_COUNT = 0x3FFFFFFF;
// own-list entry: group id | TL_SELF (the owner is counted by the group itself)
constexpr uint32_t TL_SELF = 0x80000000u;
constexpr uint32_t TL_GID = 0xFFFFu;
enum : uint32_t { ZF_COMP = 1u };  // zone requirement is a complement (Exists / NotIn / absent)
constexpr uint32_t NONE = 0xFFFFFFFFu;
// capacity-type requirement bits (consolidation's spot-to-spot rule)
enum : uint32_t { CT_SPOT = 1u, CT_OD = 2u };
// VarRec.ctb flag: the variant has no requirements and no topology spread, so
// NodeClaim.Add changes nothing but the requests (claims never carry it:
// their ctb is the template's AND the pods')
// VarRec.ctb flags: VF_SIMPLE no requirements and no owned topology group;
// VF_ZSPREAD owns a zone spread group; VF_HOSTFA no requirements and 1..4
// owned groups, all hostname groups admitted by count + self <= skew
enum : uint32_t { VF_SIMPLE = 1u << 31, VF_ZSPREAD = 1u << 30, VF_HOSTFA = 1u << 29 };

// requirement on one free key, vocabulary <= 64 values (last one is the
// "unmentioned value" omega used for hostname placeholders)
enum : uint32_t { FK_PRESENT = 1u, FK_COMP = 2u, FK_GT = 4u, FK_LT = 8u };
#ifndef GS_FKW
#define GS_FKW 4
#endif
constexpr int FKW = GS_FKW;     // words of a free key's value bitsets (<= 256 vocabulary values, omega included)
constexpr int FKV = 64 * FKW;
struct FK {
  uint64_t has[FKW];   // Has(v) for each vocabulary value
  uint64_t excl[FKW];  // complement: explicit excluded values (after bound filtering)
  int64_t gt, lt;      // bounds (complement sets only)
  uint32_t flags;
  uint32_t pad;
};

struct FKEntry {
  uint32_t slot, pad;
  FK st;
};

// one pod "variant": the pod's requirement set after k relaxations
// (<U> Preferences.Relax is deterministic, so every variant is known up front)
struct VarRec {
  uint32_t pod;
  uint32_t fk_begin, fk_count;
  uint32_t ctb;                  // CT_SPOT | CT_OD: capacity-type requirement Has(spot) / Has(on-demand)
  uint32_t itmask_off[KMAX_IT];  // word offset into itmask arena, NONE = unconstrained
  uint32_t zfull_off, cfull_off; // full-vocabulary zone / capacity-type masks (existing nodes)
  uint64_t zm, cm;               // Has over catalog zones / capacity types
  uint64_t tol;                  // tolerated taint-vocabulary mask
  uint64_t tolt;                 // templates whose taints this variant tolerates
  // topology (<U> Topology): the groups the variant owns and the groups that
  // select (count) the pod, as lists in DevProblem::tg_list (own entries:
  // group id | TL_SELF; selection entries: slot | kind << 24), and the zone
  // Has over the zone vocabulary of the strict (podDomains) and full
  // (nodeDomains) requirements
  uint32_t own_off, own_n, sel_off, sel_n;
  uint64_t zs, zn;
  uint32_t zflags;               // ZF_COMP of the full zone requirement
  uint32_t vix;                  // this record's own variant index
};
static_assert(sizeof(VarRec) == 128, "VarRec layout");

struct TmplRec {
  uint32_t np_index;
  uint32_t has_limits;
  uint32_t limit_rmask;  // resources present in the remaining-limits map
  uint32_t ctb;          // CT_SPOT | CT_OD of the template requirements
  uint64_t zm, cm;       // template Has over catalog zones / capacity types
  uint64_t taints;       // taint-vocabulary mask
  int64_t daemon[RMAX];
  int64_t limits[RMAX];  // initial remaining limits
  uint64_t zfull;        // zone Has over the zone vocabulary
  uint32_t zflags;       // ZF_COMP
  uint32_t mv_mask;      // IT keys with a minValues requirement (Strict policy)
  uint16_t mv[KMAX_IT];  // minValues per IT key
};

// one topology group (<U> TopologyGroup, empty node filter)
struct TGroupRec {
  int32_t skew;          // maxSkew (hostname anti-affinity / host ports: self, so the rule is count == 0)
  int32_t mind;          // minDomains (0 = unset; -(k + 1): lazy group k's, set when a relaxation creates it)
  uint32_t slot;         // TK_HOST: row in hn / column in hc; zone groups: row in the zone count table
  uint32_t kind;         // TK_HOST (hostname key, else zone), TK_AFF (pod affinity), TK_ANTI (anti-affinity / inverse)
  uint64_t known0;       // zone groups: domains known before the Solve (universe + counted)
};
static_assert(sizeof(TGroupRec) == 24, "TGroupRec layout");

// LDS bytes of the single-wave Solve's existing-node state: slack and room
// codes (u64 each) and a flag byte per node, 8-B aligned after the topology state
__host__ __device__ inline uint32_t wave_node_lds_bytes(uint32_t nn) { return nn ? 8u + nn * 17u : 0u; }

// LDS bytes of the Solve kernels' topology state: known domains [TGZ] u64,
// per-owned-group minimum counts [OWNMAX] i64, zone counts [TGZ][ZS] i32,
// hostname totals [TGH] i32, then the lazy groups' created bitset and their
// minDomains [nl] i32 (none of it without groups)
__host__ __device__ inline uint32_t topo_lazy_off(uint32_t tgz, uint32_t zs, uint32_t tgh) {
  return (tgz * 8u + (uint32_t)OWNMAX * 8u + tgz * zs * 4u + tgh * 4u + 7u) & ~7u;
}
__host__ __device__ inline uint32_t topo_lds_bytes(uint32_t tgz, uint32_t zs, uint32_t tgh, uint32_t nl) {
  if (!tgz && !tgh) return 0;
  return topo_lazy_off(tgz, zs, tgh) + ((nl + 63u) / 64u) * 8u + ((nl * 4u + 7u) & ~7u);
}

// per-claim record (device-owned, AoS: one candidate = one 192-B record read
// in a single round trip)
struct alignas(64) ClaimRec {
  // hot 64-B header: everything the candidate scan reads for R <= 4, one
  // line and four 16-B loads per lane
  int64_t tot_lo[4];     // requests: daemon overhead + pods (Merge), resources 0..3
  uint16_t thr_lo[4];    // threshold cursors: lower_bound(thr_val_r, tot_r)
  uint64_t zm, cm;       // Has over catalog zones / capacity types
  uint32_t tmpl, count;
  // resources 4..7
  int64_t tot_hi[RMAX - 4];
  uint16_t thr_hi[RMAX - 4];
  uint32_t ctb;          // CT_SPOT | CT_OD of the claim requirements (template AND pods)
  uint32_t zflags;       // ZF_COMP of the claim's zone requirement
  uint64_t zfull;        // zone Has over the zone vocabulary (topology spread)
  uint32_t pad[2];
  int64_t maxa[RMAX];    // max allocatable over the claim's initial options (slack bound)
  __host__ __device__ int64_t& tot(uint32_t r) { return r < 4 ? tot_lo[r] : tot_hi[r - 4]; }
  __host__ __device__ int64_t tot(uint32_t r) const { return r < 4 ? tot_lo[r] : tot_hi[r - 4]; }
  __host__ __device__ uint16_t& thr(uint32_t r) { return r < 4 ? thr_lo[r] : thr_hi[r - 4]; }
  __host__ __device__ uint16_t thr(uint32_t r) const { return r < 4 ? thr_lo[r] : thr_hi[r - 4]; }
};
static_assert(sizeof(ClaimRec) == 192, "ClaimRec layout");
static_assert(offsetof(ClaimRec, tot_hi) == 64, "ClaimRec hot header");

// existing (state) node: <U> ExistingNode
struct NodeRec {
  int64_t avail[RMAX];   // StateNode.Available()
  int64_t req[RMAX];     // remaining daemonset requests + pods added in this Solve
  uint64_t taints;       // taint-vocabulary mask
  uint32_t ok;           // 0 if any available quantity is negative (never fits)
  uint32_t zvid, cvid;   // zone / capacity-type label value ids (NONE = unlabeled)
  uint32_t vid[KMAX_IT]; // instance-type-key label value ids (NONE = unlabeled)
  uint16_t init;         // StateNode.Initialized()
  uint16_t dvid;         // the topology domain key's label value id (zone, capacity type or NodePool; DVID_NONE)
};
constexpr uint16_t DVID_NONE = 0xFFFFu;

// <U> VolumeUsage of an existing node over the CSI drivers that pending pods
// use (<= VDMAX): which of the pending pods' volumes (<= 64) it already
// mounts, its distinct volume count and its limit per driver
constexpr int VDMAX = 4;
struct NodeVol {
  uint64_t present;
  int32_t cnt[VDMAX];
  int32_t lim[VDMAX];  // INT32_MAX: no limit
};

// add-log entry: pod popped & placed, in order
struct LogRec {
  uint32_t pod, var, target, pad;  // target: claim id, or (node id | 0x80000000)
};

// FFD kernel control block (device <-> host)
// Ctrl.status values
enum : uint32_t { ST_OK = 0, ST_CLAIMS = 1, ST_INTERNAL = 2, ST_POD_COUNT = 3 };

struct Ctrl {
  uint32_t status;       // ST_*: 0 ok, 1 claim capacity exceeded, 2 internal error, 3 u16 pod count overflow
  uint32_t n_claims;
  uint32_t n_log;
  uint32_t qhead, qlen;
  uint32_t epoch;
  uint64_t pops;
  uint64_t generic_sorts, fast_sorts;
  uint64_t cand_evals;   // in-flight NodeClaim candidates scored
  uint64_t cand_full;    // candidates that passed the slack prefilter
  uint64_t node_evals;   // existing-node ExistingNode.CanAdd evaluations (whole scan chunks)
  uint64_t node_prefix;  // node positions a sequential first-fit visits (found index + 1, or all)
  uint64_t claim_prefix; // in-flight NodeClaims a sequential first-fit visits (the reference's CanAdd calls)
  uint32_t failed;       // simulations: non-pending pods unplaced or placed on uninitialized nodes
  uint32_t pad;
  uint64_t t_sort, t_scan, t_tmpl, t_total;  // wall_clock64 ticks (100 MHz) per phase
  uint64_t dbg[16];                            // diagnostic phase counters
};

// a consolidation simulation's outcome: one 16-B store per simulation (the
// counters of Ctrl are summed per workgroup into DevProblem::sim_blk)
struct SimCtrl {
  uint32_t status, n_claims, n_log, failed;
};

struct DevProblem {
  // sizes
  uint32_t N, W, R, Z, C, T, F, V, P, K, NT;  // K = IT keys, NT = taint vocab
  uint32_t NN;                                // existing nodes
  uint32_t RQ;                                // resources in the LDS slack prefilter (<= 4)
  uint32_t OW;                                // row / option / threshold stride: max(4, W rounded up to 4)
  uint32_t n_thr;                             // thr_off[R] (host copy: sizes the dynamic LDS)
  uint32_t max_claims;
  uint32_t max_claims_wave;   // the single-wave kernel's LDS NodeClaims (<= max_claims: node codes share its LDS)
  uint32_t claim_cap;         // NodeClaim slots of the claim arrays (c_rec, c_opts, c_fk, hc, c_its, ...)
  uint64_t wk_slots;  // free slots whose key is well-known
  // catalog
  const uint32_t* it_vid;      // [K][N]
  const uint16_t* it_dvid;     // [K][N] dense id of the type's value among the catalog's (minValues)
  uint32_t it_key_unique;      // IT keys whose value differs for every type (minValues counts types)
  uint32_t any_mv;             // a template carries minValues: the Solve runs the general (TOPO) variant
  const int64_t* it_alloc;     // [R][N]
  const int64_t* it_cap;       // [R][N]
  const uint64_t* it_pair;     // [N] available (zone,ct) pairs
  const uint32_t* it_prank;    // [N][64] price rank per pair, NONE if none
  const uint32_t* it_namerank; // [N]
  const uint32_t* rank_to_it;  // [N]
  const uint64_t* slot_set;    // [64][W] ITs with an available offering on pair g
  // OrderByPrice per distinct offering grid G (gs_feasibility only, built
  // on first use): grid_list sorted; the instance types with an available
  // offering in G as keys (min price rank over G << 32 | name rank), ascending,
  // at grid_keys[grid_off[g] .. grid_off[g+1])
  // grid_its: the same instance types' indices; grid_planes[g][b][W]: bit b
  // of |available offerings of i in G| for every instance type i (the
  // offering count of a row is sum_b popcount(row AND plane b) << b)
  const uint64_t* grid_list;
  const uint32_t* grid_off;
  const uint64_t* grid_keys;
  const uint32_t* grid_its;
  const uint64_t* grid_planes;
  // grid_blocks[g][k][W] (may be null): the instance types at list positions
  // [64k, 64k + 64) of grid g's OrderByPrice list, as a bitset; the cheapest
  // type in a row is in the first block the row intersects
  const uint64_t* grid_blocks;
  uint32_t n_grids, n_planes, grid_nb;
  const int64_t* thr_val;      // thresholds: sorted distinct alloc per resource
  const uint32_t* thr_off;     // [R+1] offsets into thr_val
  const uint64_t* thr_set;     // [(n_r+1) per r][OW], offsets thr_off[r]+r
  const int64_t* fk_ival;      // [F][FKV] integer value of vocabulary entries
  const uint64_t* fk_isint;    // [F][FKW] entries that are integers
  // templates
  const TmplRec* tmpl;         // [T]
  const uint64_t* t_opts;      // [T][W]
  const uint64_t* t_limopts;   // [T][W] t_opts within the NodePool limits (static matrix)
  const FK* t_fk;              // [T][F]
  // pods
  const int64_t* pod_req;      // [P][R]
  const uint32_t* var_begin;   // [P]
  const uint32_t* var_count;   // [P]
  const VarRec* vars;          // [V]
  const uint64_t* itmask;      // arena
  const uint32_t* var_itclass; // [V] IT-key requirement class of each variant (NONE: no IT keys)
  const uint32_t* var_pod;     // [V] each variant's pod (the K1 cursor pass reads 4 B, not the 128-B VarRec)
  const uint64_t* itclass_mask;// [classes][W] instance types each class's IT-key requirements allow
  const FKEntry* fk_entries;
  const uint32_t* queue0;      // [P] initial queue order
  const VarRec* qvars;         // [P] first variant of queue0[k], in queue order (first-pass prefetch)
  const int64_t* qreqs;        // [P][R] requests of queue0[k]
  const uint32_t* qcodes;      // [P][4] their slack-test codes: floor lo/hi dword, ceil lo/hi dword (16 bits per resource 0..3)
  const uint32_t* qrun;        // [P] first-pass records k.. (<= 16) equal to record k but for pod and variant index
  const NodeRec* nodes0;       // [NN] in <U> order: initialized first, then name
  const FK* n_fk0;             // [NN][F] free-key requirement state per node
  NodeRec* nodes;              // working copies (reset at every run)
  const NodeVol* n_vol0;       // [NN] volume usage before the Solve (any_vol)
  NodeVol* n_vol;              // [NN] working copies
  const uint64_t* pod_vol;     // [P][VDMAX] the pod's shared-volume bits per driver (volumes other pods mount too)
  const uint32_t* pod_vfresh;  // [P][VDMAX] the pod's volumes no other pod mounts, per driver (never present on a node)
  uint32_t any_vol;            // pending pods mount CSI volumes: the general (TOPO) variant checks limits
  FK* n_fk;
  // feasibility outputs
  uint64_t* rows;              // [V][T][OW]
  uint32_t* cheapest;          // [V][T] IT index or NONE
  uint64_t* cheapest_key;      // [V][T] (price_rank << 32 | name_rank), INT64_MAX = none
  uint32_t* nfo;               // [V][T]
  uint32_t* fk_ok;             // [V][T] free-key Compatible vs the fresh template
  uint32_t* pair_cur;          // [V][T][R] Fits threshold cursors (feas_cursor_kernel)
  // FFD state
  uint32_t* queue;             // [P]
  uint32_t* last_len;          // [P]
  uint32_t* last_epoch;        // [P]
  uint32_t* cur_var;           // [P]
  ClaimRec* c_rec;             // [max_claims]
  uint64_t* c_opts;            // [max_claims][OW]
  FK* c_fk;                    // [max_claims][F]
  int64_t* t_rem;              // [T][R] remaining limits (dynamic)
  LogRec* log;                 // [P]
  uint32_t* c_sorted;          // [max_claims] final sort order (debug)
  // the single-wave kernel's claim scan state in HBM (a Solve that outgrows
  // the LDS NodeClaims; <= 65,535 claims): the LDS arrays' global twins
  uint64_t* ch_slk;            // [claim_cap] slack codes
  uint64_t* ch_rm;             // [claim_cap] room codes
  uint32_t* ch_so;             // [claim_cap] sorted order (count | id << 16)
  uint16_t* ch_scr;            // [claim_cap] sort scratch
  uint8_t* ch_tmpl;            // [claim_cap] template
  Ctrl* ctrl;
  // topology groups
  uint32_t TG, TGH, NZV;       // groups, hostname groups, zone vocabulary size
  uint32_t TGZ, ZS;            // zone groups, zone-count stride (max(NZV, 1))
  uint32_t dom_ct;             // the "zone" groups' domain key is the capacity type (zone_cat -> catalog capacity types)
  uint32_t dom_np;             // ... is the NodePool (a template's fixed domain: no catalog narrowing)
  uint32_t n_lazy;             // spread groups created by relaxations (<= TGMAX)
  uint64_t zknown0;            // zone domains known before the Solve (universe + counted), every zone group
  const TGroupRec* tgroups;    // [TG]
  const uint32_t* tg_list;     // own / selection list arena (VarRec own_off / sel_off)
  const uint32_t* lazy_slot;   // [n_lazy] slot | LZ_HOST
  const uint32_t* var_lz_off;  // [2V]: variant v owns the lazy groups lz_idx[var_lz_off[2v] .. var_lz_off[2v + 1])
  const uint32_t* lz_idx;
  const int32_t* lz_mind;      // the variant's minDomains for each (a group takes its creator's)
  const int32_t* zcnt0;        // [TGZ][ZS] zone counts before the Solve
  const int32_t* htot0;        // [TGH] hostname groups: counted pods over all domains before the Solve
  const uint32_t* zone_order;  // [NZV] zone vocabulary ids in name order (omega excluded)
  const uint32_t* zone_cat;    // [64] zone vocabulary id -> catalog zone index (NONE)
  const int32_t* hn0;          // [TGH][NN] hostname counts per existing node before the Solve
  // simulations: each node's nonzero counts before the Solve, node-major
  // sparse (CSR): entries (group << 32 | count), group < TGZ a zone group,
  // else hostname group (group - TGZ).  Excluding a candidate's pods reads
  // its few entries, not a TGZ + TGH row
  const uint32_t* nsp_off;     // [NN + 1]
  const uint64_t* nsp;         // [nsp_off[NN]]
  int32_t* hn;                 // [TGH][NN] working copy
  int32_t* hc;                 // [max_claims][TGH] per NodeClaim (one row per claim)
  // truncation outputs
  uint32_t* c_its;             // [max_claims][60] (simulations: [n_sims][60])
  uint32_t* c_nits;            // [max_claims]     (simulations: [n_sims])
  // simulations with minValues: OrderByPrice + Truncate(60) of every NodeClaim
  // arena slot and whether its top 60 miss a minimum (TruncateInstanceTypes drop)
  uint32_t* slot_its;          // [sim claim slots][60]
  uint32_t* slot_nits;         // [sim claim slots]
  uint32_t* slot_drop;         // [sim claim slots]
  // consolidation simulations (n_sims > 0: one workgroup per simulation).
  // Per simulation s the pod range [sim_pod_off[s], sim_pod_off[s+1]) indexes
  // sim_pods and is also the simulation's arena in queue/last_len/last_epoch/
  // cur_var/log and in the claim arrays (a simulation opens at most one
  // NodeClaim per pod).  Existing nodes are the shared read-only nodes0/n_fk0
  // plus a per-block overlay of the nodes the simulation touched.
  uint32_t n_sims;
  uint32_t sim_nt;             // threads per simulation workgroup (128 or 256)
  uint32_t ov_cap;             // overlay entries per block (candidates + pods of a simulation)
  uint32_t nb_words;           // ceil(NN / 32): LDS touched-node bitmap
  uint32_t n_pending;          // pod ids < n_pending are pending (their errors do not count)
  const uint32_t* sim_pod_off; // [n_sims + 1]
  const uint32_t* sim_pods;    // pod ids, queue order within each simulation
  const uint32_t* sim_cand_off;// [n_sims + 1]
  const uint32_t* sim_cands;   // node positions removed by each simulation
  int64_t* ov_req;             // [grid][ov_cap][RMAX]
  FK* ov_fk;                   // [grid][ov_cap][F]
  SimCtrl* sim_ctrl;           // [n_sims]
  Ctrl* sim_blk;               // [grid] per-workgroup sums of the simulations' counters
  ClaimRec* sim_hdr;           // [n_sims] header of the single NodeClaim (trunc_kernel copies it)
  uint32_t* sim_next;          // work counter (reset before each launch)
  // simulations with topology groups / volumes: per simulation the zone
  // domains known without the candidates; the counted bound pods per zone
  // group and node (the candidates' pods are rescheduled, not counted); per
  // block the hostname counts and volume usage of the overlay nodes
  const uint64_t* sim_known;   // [n_sims]
  // [grid][ov_cap][TGH] (stamp << 32 | count): a hostname count a
  // simulation wrote on one of its overlay nodes, stamp = ov_epoch << 20 |
  // simulation + 1; a cell with another stamp is unwritten (the node's hn0
  // count holds), so an entry's cells are never cleared
  uint64_t* ov_hn;
  NodeVol* ov_vol;             // [grid][ov_cap]
  uint32_t ov_epoch;            // 1..4095: the launch's stamp prefix (ov_hn zeroed when it wraps)
  uint32_t* ov_map;            // [grid][NN] a touched node's overlay entry (valid where the LDS bitmap bit is set)
  uint32_t ovh_slots;          // > 0: simulations this small keep node -> entry in an LDS hash of that many slots instead
  uint32_t sim_lds;            // simulations keep queue / staleness / variant / add log in LDS (32 B per pod)
};

// the parent-side merge of a sharded static matrix (kernels.hip
// merge_shards_kernel): the shards' device buffers and word slices
constexpr int SHARDS_MAX = 16;
struct ShardSrc {
  const uint64_t* rows;  // [VT][OW] (words [lo, hi) valid)
  const uint32_t* nfo;   // [VT]
  const uint64_t* key;   // [VT]
  uint32_t lo, hi;
};
struct ShardMerge {
  ShardSrc src[SHARDS_MAX];
  uint32_t K, K_red;     // shards; shards whose counts / keys still need reducing (1 after RCCL)
  uint32_t VT, OW, wb, we;
  uint64_t* rows;
  uint32_t* nfo;
  uint64_t* key;
  uint32_t* cheapest;
  const uint32_t* rank_to_it;
};

}  // namespace gsd
