"""Time SA2's grouped MLP (the lean x3 kernel, lidar_sa_group_mlp_x3_f32) alone over one 128-frame
launch at the bench's shape (1 024 centres x 64 rows per frame, 4 096 per-point layer-1 rows of 128 per
frame, widths 128-128-256), on whatever library LIDAR_AMD_LIB names: the diagnostic LIDAR_SA_ABL builds
(sa_mlp_x3.hip) drop the weight streaming (1), the per-pass barriers (2) or the row gather (4), so
the difference to the product build prices each part.  Random operands (the clock depends on the data).

    for a in 0 1 2 4 7; do LIDAR_AMD_LIB=tools/ablib/liblidar_abl$a.so python tools/micro/sa2_ablate.py; done
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402

B, N, M, NS, C1, C2, C3 = 128, 4096, 1024, 64, 128, 128, 256
FLOP = 2.0 * B * M * NS * (C1 * C2 + C2 * C3)  # fp32-equivalent, layers 2-3
PEAK = 2.5e15 / 3  # x3: three bf16 products per fp32 product

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
layers = [(rng.standard_normal((131, C1)).astype(np.float32) * 0.1, rng.standard_normal(C1).astype(np.float32) * 0.1),
          (rng.standard_normal((C1, C2)).astype(np.float32) * 0.1, rng.standard_normal(C2).astype(np.float32) * 0.1),
          (rng.standard_normal((C2, C3)).astype(np.float32) * 0.1, rng.standard_normal(C3).astype(np.float32) * 0.1)]
packed = torch.from_numpy(pn.pack_branch_x3(layers, False)).to(dev)
p = torch.randn(B * N, C1, device=dev)
q = torch.randn(B * M, C1, device=dev) * 0.5
idx = torch.randint(0, N, (B, M, NS), device=dev, dtype=torch.int32)
out = torch.empty(B * M, C3, device=dev)

for _ in range(3):
    pn.group_mlp_x3(p, q, idx, N, packed, (C1, C2, C3), out)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
reps = 20
ev[0].record()
for _ in range(reps):
    pn.group_mlp_x3(p, q, idx, N, packed, (C1, C2, C3), out)
ev[1].record()
torch.cuda.synchronize()
ms = ev[0].elapsed_time(ev[1]) / reps
print("%s abl=%s %.3f ms per 128-frame launch, %.3f of the x3 peak" % (
    os.path.basename(os.environ.get("LIDAR_AMD_LIB", "product")), os.environ.get("ABL", "?"), ms,
    FLOP / (ms * 1e-3) / PEAK), flush=True)
