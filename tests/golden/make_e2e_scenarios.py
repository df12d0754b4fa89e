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
# GetMultipleInstanceTypes(3): the first three 2-4 vCPU / 4-16 GB profiles
# (reference test/e2e/instance_discovery.go:39-66) of the fake catalog order
# (pkg/fake/zz_generated_ibm_test_data.go:27-243)
SMALL3 = ["bx2-2x8", "bx2-4x16", "cx2-2x4"]
IT = "node.kubernetes.io/instance-type"
Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"

# createTestNodePool (reference test/e2e/resources.go:232-269)
TEST_NODEPOOL = {"requirements": [[IT, "In", SMALL3]]}
# createMultiZoneNodePool (reference test/e2e/multizone_test.go:474-521)
MULTIZONE_NODEPOOL = {"requirements": [[IT, "In", ["bx2-4x16", "bx2-2x8"]], [Z, "In", ZONES]]}

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
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "e2e_scenarios.json"), "w") as f:
        json.dump({"zones": ZONES, "scenarios": SCENARIOS}, f, indent=1)
        f.write("\n")
