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
    "rank_orders": {  # pkg/providers/common/instancetype/instancetype_mock_test.go:221-361
        # makeInstanceType(name, cpu milli, memory bytes, arch) + the price the
        # ranking sees (RankInstanceTypes with a nil pricing provider or nil
        # client prices every type at 0.0, :300-353)
        "source": "instancetype_mock_test.go:221-361",
        "cases": [
            {"name": "ByPrice", "types": [["expensive", 4000, 16 * 2**30, 1.00], ["cheap", 4000, 16 * 2**30, 0.10],
                                          ["mid", 4000, 16 * 2**30, 0.50]],
             "want": ["cheap", "mid", "expensive"]},
            {"name": "NoPricing_FallsBackToResourceSize",
             "types": [["large", 8000, 32 * 2**30, 0.0], ["small", 2000, 8 * 2**30, 0.0]], "want": ["small", "large"]},
            {"name": "MixedPricingAndNoPricing",
             "types": [["no-price", 4000, 8 * 2**30, 0.0], ["has-price", 4000, 8 * 2**30, 0.10]],
             "want_first": "has-price"},
            {"name": "NilPricingProvider",
             "types": [["bx2-8x32", 8000, 32 * 2**30, 0.0], ["bx2-2x8", 2000, 8 * 2**30, 0.0]],
             "want": ["bx2-2x8", "bx2-8x32"]},
            {"name": "EmptyInput", "types": [], "want": []},
            {"name": "SingleInstance", "types": [["bx2-4x16", 4000, 16 * 2**30, 0.0]], "want": ["bx2-4x16"]},
            {"name": "ClientNilWithPricingProvider",
             "types": [["bx2-4x16", 4000, 16 * 2**30, 0.0], ["bx2-2x8", 2000, 8 * 2**30, 0.0]],
             "want": ["bx2-2x8", "bx2-4x16"]},
            {"name": "EqualScores_PreservesAll",
             "types": [["bx2-2x8", 2000, 8 * 2**30, 0.0], ["cx2-2x8", 2000, 8 * 2**30, 0.0]],
             "want_set": ["bx2-2x8", "cx2-2x8"]},
        ],
    },
    "score_zero_resources": {  # instancetype_mock_test.go:372-383
        "source": "instancetype_mock_test.go:372-383",
        "cpu_milli": 0, "memory_bytes": 0, "price": 0.0, "want": 0.0,
    },
    "resolve_capacity_type": {  # pkg/providers/common/capacitytype/capacitytype_test.go:30-169
        # nodeClaim requirements (None = nil Requirements), instance types as
        # lists of offerings [capacity type, zone, price, available]
        "source": "capacitytype_test.go:30-169",
        "cases": [
            {"name": "nil requirements defaults to on-demand", "requirements": None, "types": [], "want": "on-demand"},
            {"name": "empty requirements defaults to on-demand", "requirements": [], "types": [],
             "want": "on-demand"},
            {"name": "on-demand only requirement returns on-demand",
             "requirements": [["karpenter.sh/capacity-type", "In", ["on-demand"]]], "types": [], "want": "on-demand"},
            {"name": "spot allowed but no available spot offering returns on-demand",
             "requirements": [["karpenter.sh/capacity-type", "In", ["spot", "on-demand"]]],
             "types": [[["on-demand", "us-south-1", 0.1, True]]], "want": "on-demand"},
            {"name": "spot allowed with available spot offering returns spot",
             "requirements": [["karpenter.sh/capacity-type", "In", ["spot", "on-demand"]]],
             "types": [[["spot", "us-south-1", 0.06, True]]], "want": "spot"},
            {"name": "spot allowed but spot offering unavailable returns on-demand",
             "requirements": [["karpenter.sh/capacity-type", "In", ["spot"]]],
             "types": [[["spot", "us-south-1", 0.06, False]]], "want": "on-demand"},
        ],
    },
    "get_instance_types_counts": {  # pkg/cloudprovider/cloudprovider_test.go:686-798 (+ getTestInstanceType)
        # a NodePool without requirements keeps every listed type, whatever its
        # offerings (GetInstanceTypes filters on Compatible only, cloudprovider.go:574-577)
        "source": "cloudprovider_test.go:686-798",
        "cases": [
            {"name": "successful get instance types", "n_types": 2, "second_has_offerings": False, "want": 2},
            {"name": "empty instance types", "n_types": 0, "want": 0},
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
