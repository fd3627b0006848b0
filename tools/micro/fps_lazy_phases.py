"""(lazy kernel, 512 threads) Where an FPS step's time goes: the DIAG build of fps_bucket_kernel<1024, 1> (lidar_diag_fps_lazy_phases)
stamps the shader clock around each phase of every step, per wave.  Prints, per step averaged over
frames and waves: [0] bucket tests + active-bucket updates (loads, distances, DPP reductions),
[1] wave argmax + LDS publish, [2] barrier wait, [3] 16-way merge, plus active-bucket batches per
wave-step, and the same for the first / last 256 steps.

usage (the diagnostic library, `make -C lidar_ai_recommendation_software_amd/csrc diag`):
LIDAR_AMD_LIB=lidar_ai_recommendation_software_amd/liblidar_amd_diag.so python tools/micro/fps_phases.py [B] [N] [M]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
M = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
dev = torch.device("cuda:0")
lib = nat.load_library()
f = lib.lidar_diag_fps_lazy_phases
f.argtypes = [nat.P, nat.P, nat.I64, nat.I64, nat.I64, nat.P, nat.P, nat.P]
x = torch.from_numpy(unit_frames(B, N, seed=5)).to(dev)
idx = torch.empty((B, M), dtype=torch.int32, device=dev)
diag = torch.zeros((B, 8, 8), dtype=torch.int64, device=dev)
h = nat.handle(0)
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nat.check(f(h, nat.ptr(x), B, N, M, nat.ptr(idx), nat.ptr(diag), nat.stream_ptr()), "diag")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
d = diag.cpu().numpy().astype(np.float64)
steps = d[..., 7].mean()
per = d[..., :7].sum(axis=(0, 1)) / (B * 8 * steps)
tot = per[:5].sum()
print(f"lazy B={B} N={N} M={M}: wall {wall * 1e3:.2f} ms ({wall * 1e6 / M:.2f} us/step); per wave-step cycles: "
      f"tests+L+defer {per[0]:.0f}, refresh {per[1]:.0f}, recount+publish {per[2]:.0f}, barrier {per[3]:.0f}, "
      f"merge {per[4]:.0f} (sum {tot:.0f} = {tot / 2.4e3:.2f} us at 2.4 GHz); batches per wave-step {per[5]:.2f}, "
      f"recounts per wave-step {per[6]:.2f}")
