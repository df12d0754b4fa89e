"""Writes tests/golden/reference_kats.json: the known-answer vectors that the
reference's own Go tests hold for the catalog path that feeds Solve.

Values are transcribed (data only) from these reference test tables; each
entry carries its file:line.  Re-run: python tests/golden/make_reference_kats.py
"""
import json
import os

KATS = {
    "instance_family": {  # pkg/providers/common/instancetype/instancetype_test.go:754-801
        "source": "instancetype_test.go:754-801",
        "cases": [["bx2-2x8", "bx2"], ["cx2-4x8", "cx2"], ["mx2-8x64", "mx2"], ["ab", "ab"], ["", "balanced"],
                  ["bx3d-2x8", "bx3d"]],
    },
    "instance_size": {  # instancetype_test.go:803-842
        "source": "instancetype_test.go:803-842",
        "cases": [["bx2-2x8", "2x8"], ["cx2-16x32", "16x32"], ["bx2", "small"], ["", "small"], ["bx2-", "small"]],
    },
    "supported_capacity_types": {  # pkg/providers/common/capacitytype/capacitytype_test.go:171-248
        "source": "capacitytype_test.go:171-248",
        "cases": [
            [None, ["on-demand"]],
            [["enum", ["standard"]], ["on-demand"]],
            [["enum", ["spot"]], ["spot"]],
            [["enum", ["standard", "spot"]], ["on-demand", "spot"]],
            [["fixed", "standard"], ["on-demand"]],
            [["fixed", "spot"], ["spot"]],
            [["fixed", None], ["on-demand"]],
            [["enum", []], ["on-demand"]],
        ],
    },
    "instance_score": {  # instancetype_test.go:103-159
        "source": "instancetype_test.go:103-159",
        "cases": [  # cpu quantity, memory quantity, price, want
            ["4", "16Gi", 0.5, 0.0763888888888889],
            ["2", "8Gi", 0.0, 11.0],
            ["16", "64Gi", 2.0, 0.0769927536231884],
        ],
    },
    "overhead": {  # instancetype_test.go:237-350 (and provider_test.go:250-352)
        "source": "instancetype_test.go:237-350",
        "cases": [
            {"kubelet": None, "want": {"kube.cpu": "100m", "kube.memory": "1Gi", "system.cpu": "100m",
                                       "system.memory": "1Gi", "eviction.memory": "500Mi"}},
            {"kubelet": {"kubeReserved": {"cpu": "1", "memory": "2Gi"},
                         "systemReserved": {"cpu": "500m", "memory": "1Gi"},
                         "evictionHard": {"memory.available": "500Mi"}},
             "want": {"kube.cpu": "1", "kube.memory": "2Gi", "system.cpu": "500m", "system.memory": "1Gi",
                      "eviction.memory": "500Mi"}},
            {"kubelet": {"kubeReserved": {"cpu": "2"}},
             "want": {"kube.cpu": "2", "kube.memory": "1Gi", "system.cpu": "100m", "system.memory": "1Gi",
                      "eviction.memory": "500Mi"}},
            {"kubelet": {"kubeReserved": {"cpu": "not-a-quantity", "memory": "also-bad"},
                         "systemReserved": {"cpu": "still-bad", "memory": "nope"},
                         "evictionHard": {"memory.available": "broken"}},
             "want": {"kube.cpu": "100m", "kube.memory": "1Gi", "system.cpu": "100m", "system.memory": "1Gi",
                      "eviction.memory": "500Mi"}},
        ],
    },
    "offerings_per_zone_captype": {  # instancetype_test.go:1082-1148
        "source": "instancetype_test.go:1082-1148",
        "profile": {"name": "bx2-4x16", "vcpu": 4, "memory_gib": 16, "arch": "amd64", "gpu": 0,
                    "availability_class": ["enum", ["standard", "spot"]]},
        "zones": ["us-south-1", "us-south-2"],
        "prices": {"bx2.2x8": 0.095, "bx2.4x16": 0.190, "bx2-4x16": 0.190},  # MockPricingProvider :86-95
        "unavailable": ["bx2-4x16:us-south-2:spot"],
        "want_offerings": 4,
        "want_unavailable": [["us-south-2", "spot"]],
    },
    "spot_price": {  # instancetype_test.go:1150-1202
        "source": "instancetype_test.go:1150-1202",
        "profile": {"name": "bx2-4x16", "vcpu": 4, "memory_gib": 16, "arch": "amd64", "gpu": 0,
                    "availability_class": ["enum", ["standard", "spot"]]},
        "zones": ["us-south-1"],
        "prices": {"bx2.2x8": 0.095, "bx2.4x16": 0.190, "bx2-4x16": 0.190},
        "spot_discount_percent": 40,
        "want": {"on-demand": 0.190, "spot": 0.076},
    },
    "conversion_errors": {  # instancetype_test.go:968-1026, 1029-1080, 845-866
        "source": "instancetype_test.go:968-1080,845-866",
        "cases": [
            [{"name": None}, False, "instance profile name is nil"],
            [{"name": "test-profile", "vcpu": None}, False, "has no CPU count"],
            [{"name": "test-profile", "vcpu": 2, "memory_gib": None}, False, "has no memory"],
            [{"name": "gx2-8x64x1v100", "vcpu": 8, "memory_gib": 64, "arch": "amd64", "gpu": 1}, False,
             "IBM client not initialized"],
            [{"name": "test-profile", "vcpu": 2, "memory_gib": 16}, False, "IBM client not initialized"],
        ],
    },
    "fake_profiles": {  # pkg/fake/zz_generated_ibm_test_data.go:27-243 (C1 catalog)
        "source": "pkg/fake/zz_generated_ibm_test_data.go:27-243,286-314",
        "profiles": [["bx2-2x8", 2, 8, None], ["bx2-4x16", 4, 16, None], ["bx2-8x32", 8, 32, None],
                     ["cx2-2x4", 2, 4, None], ["cx2-4x8", 4, 8, None], ["mx2-2x16", 2, 16, None],
                     ["mx2-4x32", 4, 32, None], ["gx2-8x64x1v100", 8, 64, 1]],
        "zones": ["us-south-1", "us-south-2", "us-south-3"],
    },
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1, sort_keys=True)
    print("wrote", out)
