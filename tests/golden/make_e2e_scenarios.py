"""Writes tests/golden/e2e_scenarios.json: the reference e2e suite's Solve-level
expectations, transcribed as data (VERDICT r2 Missing 3).  Each scenario names
the reference test (file:line) it restates, the NodePool and workloads that
test creates, how the workload arrives, and the property the test asserts.

The e2e tests run against a live IBM cloud (test/e2e/, build tag e2e); what a
single provisioning Solve (and the consolidation simulation) must do for
their assertions to hold is restated here.  `arrival` "together" is one Solve
of every replica; "one_by_one" is one Solve per replica, each after the
previous NodeClaims were launched as nodes (zone: the first the claim allows
with an available offering of its first instance type).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ZONES = ["us-south-1", "us-south-2", "us-south-3"]
# GetMultipleInstanceTypes(n) (reference test/e2e/instance_discovery.go:39-66):
# the first n of the 2-4 vCPU / 4-16 GB profiles sorted by vCPU, then memory,
# then bx2 first, then name (filterSmallProfiles, instance_profiles.go:26-67),
# over the fake catalog (pkg/fake/zz_generated_ibm_test_data.go:27-243)
FAKE = [("bx2-2x8", 2, 8), ("bx2-4x16", 4, 16), ("bx2-8x32", 8, 32), ("cx2-2x4", 2, 4), ("cx2-4x8", 4, 8),
        ("mx2-2x16", 2, 16), ("mx2-4x32", 4, 32), ("gx2-8x64x1v100", 8, 64)]
SMALL = [n for n, v, m in sorted(((n, v, m) for n, v, m in FAKE if 2 <= v <= 4 and 4 <= m <= 16),
                                 key=lambda x: (x[1], x[2], not x[0].startswith("bx2-"), x[0]))]
SMALL3 = SMALL[:3]
SMALL4 = SMALL[:4]
IT = "node.kubernetes.io/instance-type"
Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"

# createTestNodePool (reference test/e2e/resources.go:232-269)
TEST_NODEPOOL = {"requirements": [[IT, "In", SMALL3]]}
# createMultiZoneNodePool (reference test/e2e/multizone_test.go:474-521)
MULTIZONE_NODEPOOL = {"requirements": [[IT, "In", ["bx2-4x16", "bx2-2x8"]], [Z, "In", ZONES]]}
# createTestNodePoolWithMultipleInstanceTypes (reference test/e2e/resources.go:311-368)
MULTI_TYPE_NODEPOOL = {"requirements": [[IT, "In", SMALL4], ["kubernetes.io/arch", "In", ["amd64"]],
                                        ["karpenter.sh/capacity-type", "In", ["on-demand"]]],
                       "labels": {"provisioner": "karpenter-vpc", "cluster-type": "self-managed", "test": "e2e",
                                  "test-name": "nodepool-instance-selection"}}
# TestE2ETaintsBasicScheduling's NodePool (reference test/e2e/e2e_taints_test.go:495-531): one instance type
# (GetMultipleInstanceTypes(t, 1)), a NoSchedule taint, template label test=<testName>.  The workload's own
# comment sizes it for an 8 GB 2-vCPU profile (bx2a-2x8, :1106-1110): 1000m / 4Gi does not fit the first small
# fake profile (cx2-2x4: 4 GB - 2.5 GiB calculateOverhead), so the fake catalog's 8 GB 2-vCPU profile stands in.
TAINTED_NODEPOOL = {"requirements": [[IT, "In", ["bx2-2x8"]]], "labels": {"test": "basic-taints"},
                    "taints": [["dedicated", "gpu-workload", "NoSchedule"]]}
# TestE2EStartupTaints' NodePool (reference test/e2e/e2e_taints_test.go:80-119): one instance type (the same
# bx2-2x8 stand-in as above for the 1000m / 4Gi workload), template label test=<testName>, two startup taints
STARTUP_NODEPOOL = {"requirements": [[IT, "In", ["bx2-2x8"]]], "labels": {"test": "startup-taints"},
                    "startup_taints": [["node.kubernetes.io/not-ready", "", "NoSchedule"],
                                       ["example.com/initializing", "true", "NoSchedule"]]}
# TestE2ETaintValues' NodePool (reference test/e2e/e2e_taints_test.go:650-691): a NoSchedule and a
# PreferNoSchedule taint with values
TAINT_VALUES_NODEPOOL = {"requirements": [[IT, "In", ["bx2-2x8"]]], "labels": {"test": "taint-values"},
                         "taints": [["workload-type", "batch-processing", "NoSchedule"],
                                    ["priority", "high", "PreferNoSchedule"]]}

SCENARIOS = [
    {
        "id": "pod_anti_affinity_hostname",
        "ref": "test/e2e/scheduling_test.go:246-344 (TestE2EPodAntiAffinity)",
        "nodepool": TEST_NODEPOOL,
        "workloads": [{"app": "anti-affinity-app", "replicas": 3, "cpu_m": 500, "memory_mi": 512,
                       "anti_affinity": [{"key": H, "required": True}]}],
        "arrival": "together",
        "expect": {"kind": "distinct_nodeclaims", "app": "anti-affinity-app", "n": 3},
    },
    {
        "id": "node_affinity_instance_type",
        "ref": "test/e2e/scheduling_test.go:359-475 (TestE2ENodeAffinity)",
        "nodepool": TEST_NODEPOOL,
        # createTestWorkload (resources.go:461-545): 3 replicas, 1 CPU / 1 GiB,
        # launched first; the second deployment requires the first node's type
        "workloads": [{"app": "initial-workload", "replicas": 3, "cpu_m": 1000, "memory_mi": 1024},
                      {"app": "node-affinity-app", "replicas": 2, "cpu_m": 500, "memory_mi": 512,
                       "node_affinity_first_node_type": True}],
        "arrival": "by_workload",
        "expect": {"kind": "instance_type_is_first_node_type", "app": "node-affinity-app"},
    },
    {
        "id": "topology_spread_zone",
        "ref": "test/e2e/multizone_test.go:188-289 (TestE2ETopologySpreadConstraints)",
        "nodepool": MULTIZONE_NODEPOOL,
        "workloads": [{"app": "topology-spread-app", "replicas": 6, "cpu_m": 500, "memory_mi": 512,
                       "spread": {"key": Z, "max_skew": 1, "when": "DoNotSchedule"}}],
        "arrival": "together",
        "expect": {"kind": "zone_skew", "app": "topology-spread-app", "max_skew": 1, "min_zones": 2},
    },
    {
        "id": "zone_anti_affinity_preferred",
        "ref": "test/e2e/multizone_test.go:83-174 (TestE2EZoneAntiAffinity)",
        "nodepool": MULTIZONE_NODEPOOL,
        "workloads": [{"app": "zone-anti-affinity-app", "replicas": 3, "cpu_m": 1000, "memory_mi": 1024,
                       "anti_affinity": [{"key": Z, "required": False, "weight": 100}]}],
        "arrival": "one_by_one",
        "expect": {"kind": "min_zones", "app": "zone-anti-affinity-app", "min_zones": 2},
    },
    {
        "id": "consolidation_with_pdb",
        "ref": "test/e2e/scheduling_test.go:38-176 (TestE2EConsolidationWithPDB)",
        "nodepool": TEST_NODEPOOL,
        "workloads": [{"app": "consolidation-pdb-app", "replicas": 4, "cpu_m": 1000, "memory_mi": 1024,
                       "anti_affinity": [{"key": H, "required": False, "weight": 100}]}],
        "arrival": "together",
        # more than one node after the Solve (:120-122); scaled to 2 replicas
        # (:152-156) the emptied nodes consolidate
        "expect": {"kind": "multi_node_then_consolidate", "app": "consolidation-pdb-app", "min_nodes": 2,
                   "scale_to": 2},
    },
    {
        "id": "tainted_nodepool_tolerant_split",
        "ref": "test/e2e/e2e_taints_test.go:458-611 (TestE2ETaintsBasicScheduling), workload :1074-1119",
        "nodepool": TAINTED_NODEPOOL,
        # createResourceIntensiveWorkload: 1 replica, 1000m / 4Gi; the tolerant one tolerates
        # dedicated=gpu-workload:NoSchedule (Equal) and selects the template label; the intolerant one
        # (created after the first is ready, :598-608) has neither and must stay pending
        "workloads": [{"app": "tolerant-deployment", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "tolerations": [["dedicated", "Equal", "gpu-workload", "NoSchedule"]],
                       "node_selector": {"test": "basic-taints"}},
                      {"app": "intolerant-deployment", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "node_selector": {}}],
        "arrival": "by_workload",
        "expect": {"kind": "taint_split", "app": "tolerant-deployment", "pending_app": "intolerant-deployment",
                   "taint": ["dedicated", "gpu-workload", "NoSchedule"]},
    },
    {
        "id": "instance_types_within_allowed",
        "ref": "test/e2e/basic_workflow_test.go:76-115 (TestE2ENodePoolInstanceTypeSelection), NodePool "
               "resources.go:311-368, workload resources.go:548-623, assertion verification.go:102-132 and "
               "verifyNodePoolRequirementsOnNodes :135-",
        "nodepool": MULTI_TYPE_NODEPOOL,
        # 2 replicas, 1500m / 2Gi, required hostname anti-affinity on their own app
        "workloads": [{"app": "nodepool-instance-selection-workload", "replicas": 2, "cpu_m": 1500,
                       "memory_mi": 2048, "anti_affinity": [{"key": H, "required": True}]}],
        "arrival": "together",
        "expect": {"kind": "types_within_allowed", "app": "nodepool-instance-selection-workload",
                   "allowed": SMALL4, "n": 2},
    },
    {
        "id": "zone_spread_survives_scale_up",
        "ref": "test/e2e/multizone_test.go:384-431 (TestE2EZoneFailover), deployment :578-649",
        "nodepool": MULTIZONE_NODEPOOL,
        # 4 replicas of 500m / 512Mi with a preferred (weight 50) zone anti-affinity on their own app;
        # once placed, the Deployment scales to 8 (:410-416) and the pods must still span > 1 zone (:425)
        "workloads": [{"app": "zone-failover-app", "replicas": 4, "cpu_m": 500, "memory_mi": 512,
                       "anti_affinity": [{"key": Z, "required": False, "weight": 50}]}],
        "arrival": "scale",
        "scale_to": 8,
        "expect": {"kind": "min_zones", "app": "zone-failover-app", "min_zones": 2, "placed": 8},
    },
    {
        "id": "startup_taints_inflight_node",
        "ref": "test/e2e/e2e_taints_test.go:43-258 (TestE2EStartupTaints), workload :1074-1119",
        "nodepool": STARTUP_NODEPOOL,
        # the reference deployment: 1 replica, 1000m / 4Gi, tolerating both startup taints (:129-141) and
        # selecting the template label; it must get a NodeClaim of this pool (:149-184) and schedule (:242-254).
        # Derived step (marked "derived"): while that node initializes (managed, not initialized, its Node
        # carrying the startup taints and not-ready), a second pod WITHOUT those tolerations packs onto it:
        # <U> StateNode.Taints() ignores startup and ephemeral taints until initialization; once the node is
        # initialized and a startup taint is still there, the same pod opens a NodeClaim instead.
        "workloads": [{"app": "startup-taints-deployment", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "tolerations": [["node.kubernetes.io/not-ready", "Equal", "", "NoSchedule"],
                                       ["example.com/initializing", "Equal", "true", "NoSchedule"]],
                       "node_selector": {"test": "startup-taints"}},
                      {"app": "startup-followup", "replicas": 1, "cpu_m": 500, "memory_mi": 1024,
                       "node_selector": {"test": "startup-taints"}, "derived": True}],
        "arrival": "startup",
        "expect": {"kind": "startup_taints", "app": "startup-taints-deployment", "followup_app": "startup-followup"},
    },
    {
        "id": "taint_values_equal_tolerations",
        "ref": "test/e2e/e2e_taints_test.go:614-776 (TestE2ETaintValues), workload :1074-1119",
        "nodepool": TAINT_VALUES_NODEPOOL,
        # the reference deployment tolerates both taints with Operator Equal and their exact values
        # (:700-715) and must become ready on this pool's node (:723-735).  Derived workloads: one tolerating
        # only the NoSchedule taint schedules after <U> Preferences.Relax tolerates PreferNoSchedule (the
        # pool carries such a taint); one whose Equal toleration names another value stays pending.
        "workloads": [{"app": "taint-values-deployment", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "tolerations": [["workload-type", "Equal", "batch-processing", "NoSchedule"],
                                       ["priority", "Equal", "high", "PreferNoSchedule"]],
                       "node_selector": {"test": "taint-values"}},
                      {"app": "prefer-relaxed", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "tolerations": [["workload-type", "Equal", "batch-processing", "NoSchedule"]],
                       "node_selector": {"test": "taint-values"}, "derived": True},
                      {"app": "value-mismatch", "replicas": 1, "cpu_m": 1000, "memory_mi": 4096,
                       "tolerations": [["workload-type", "Equal", "streaming", "NoSchedule"],
                                       ["priority", "Equal", "high", "PreferNoSchedule"]],
                       "node_selector": {"test": "taint-values"}, "derived": True}],
        "arrival": "together",
        "expect": {"kind": "taint_values", "app": "taint-values-deployment", "relaxed_app": "prefer-relaxed",
                   "pending_app": "value-mismatch"},
    },
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "e2e_scenarios.json"), "w") as f:
        json.dump({"zones": ZONES, "scenarios": SCENARIOS}, f, indent=1)
        f.write("\n")
