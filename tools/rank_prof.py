"""Profile target: 20 gs_rank_instance_types calls over the bench.py ranking
catalog (2,000 types with exact ties).  Run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "karpenter-provider-ibm-cloud_amd"))
from gpusched import lib  # noqa: E402

rng = np.random.default_rng(5)
n = 2000
vcpu = rng.choice([2, 4, 8, 16, 32, 48, 64, 96], size=n)
ratio = rng.choice([2, 4, 8], size=n)
cpu = (vcpu * 1000).astype(np.int64)
mem = (vcpu * ratio * (1 << 30)).astype(np.int64)
price = np.round(vcpu * ratio * rng.choice([0.01, 0.0125, 0.02], size=n), 4)
arch = np.zeros(n, dtype=np.uint32)
for _ in range(20):
    order, score = lib.rank_instance_types(cpu, mem, price, arch)
print("ranked", len(order))
