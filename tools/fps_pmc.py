"""One FPS launch (B frames x 65 536 points -> 4 096) for a PMC pass: python tools/fps_pmc.py B THREADS."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
N, M = 65536, 4096
dev = torch.device("cuda:0")
x = torch.from_numpy(unit_frames(B, N, 0)).to(dev)
idx = torch.empty((B, M), dtype=torch.int32, device=dev)
for _ in range(2):
    nat.call("lidar_fps_ex_f32", nat.handle(0), nat.ptr(x), B, N, M, nat.ptr(idx), None, None, None, T,
             nat.stream_ptr())
torch.cuda.synchronize()
print("ok", idx[0, :4].tolist())
