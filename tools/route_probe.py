"""Probe: packet_route_kernel time on the C5 window (10 M packets over the C4 table)."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

top = sa.Topology.synthetic(seed=20261015)
pk = top.synth_packets(20261015, 100_000, 10_000_000, 10**9, 10**7)
top.build()
jump = int(top.getMinimumLatency()) * 1_000_000
cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
a = [cu(pk["src_col"]), cu(pk["dst_col"]), cu(pk["payload"].view(np.int32)),
     cu(pk["state_in"].view(np.int32)), cu(pk["now"].view(np.int64))]
n = len(pk["src_col"])
t = torch.empty(n, dtype=torch.int64, device="cuda")
s = torch.empty(n, dtype=torch.int32, device="cuda")
d = torch.empty(n, dtype=torch.uint8, device="cuda")
ms = []
for i in range(30):
    top.route_batch_device(*a, jump, 1, t, s, d)
    if i >= 5:
        ms.append(top.stats()["route_kernel_ms"])
print("route kernel ms: median %.4f min %.4f" % (np.median(ms), np.min(ms)), flush=True)
