"""Phase cycles of the voxel bucket kernel (diagnostic build -DVX_DIAG_PHASES: s_memtime and
s_memrealtime stamps of workgroup thread 0, written into the scratch tail of the counts output,
16 words per bucket).  usage:
LIDAR_AMD_LIB=tools/ablib/liblidar_vx_PHASES.so python tools/micro/voxel_phases.py [B] [voxel]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
voxel = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
N = 65536
x = torch.from_numpy(unit_frames(B, N, 0)).to("cuda:0")
for _ in range(3):
    c, vid, cnt, nv = pn.voxel_downsample_batch(x, voxel)
torch.cuda.synchronize()
nb = (N + 2047) // 2048
cnt = cnt.cpu().numpy().astype(np.int64)
d = np.stack([cnt[:, N - 16 * (b + 1):N - 16 * b] for b in range(nb)], 1)  # (B, nb, 16)
ph = d[:, :, :7].astype(np.float64)
names = ["range", "load+rank", "scan", "runs+place", "look-back", "ids", "sums"]
print(f"B={B} voxel={voxel} buckets/frame={nb}: mean cycles per phase " +
      ", ".join(f"{k} {v:.0f}" for k, v in zip(names, ph.mean(axis=(0, 1)))))
for k, nm in enumerate(names):
    print(f"{nm:10s} by bucket:", np.round(ph[:, :, k].mean(0)).astype(int).tolist())
print("spins by bucket:", np.round(d[:, :, 7].mean(0), 1).tolist())
rt = d[:, :, 8:16].astype(np.float64)  # realtime (100 MHz = 10 ns) stamps 0..7
t0 = rt[:, :, 0].min()
us = (rt - t0) * 0.01
for f in (0, 8, 1, 31 if B > 31 else B - 1):
    print(f"frame {f}: start us", np.round(us[f, :, 0], 1).tolist())
    print(f"frame {f}: look-back start us", np.round(us[f, :, 4], 1).tolist())
    print(f"frame {f}: look-back end us", np.round(us[f, :, 5], 1).tolist())
print("kernel span us", round(us[:, :, 7].max(), 1))
rd = np.mod(np.diff(rt, axis=2), 2.0 ** 31) * 0.01  # (B, nb, 7) realtime per phase, us (stamps kept mod 2^31)
print("realtime us per phase: " + ", ".join(f"{k} {v:.2f}" for k, v in zip(names, rd.mean(axis=(0, 1)))) +
      f"; workgroup life {rd.sum(2).mean():.1f} us")
