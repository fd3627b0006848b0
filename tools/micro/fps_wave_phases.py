"""Where a one-wave FPS step's time goes: the DIAG build of fps_wave_kernel<16> (lidar_diag_fps_wave)
stamps the shader clock around each phase of every step.  Prints per step, averaged over frames:
cycles of [0] slot tests + active-bucket list, [1] batches (loads, distances, reductions),
[2] slot re-keys, [3] frame argmax; and active slots, active buckets, batches, re-keyed slots.

usage: python tools/micro/fps_wave_phases.py [B,...] [N] [M]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

BS = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 128]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
M = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
dev = torch.device("cuda:0")
lib = nat.load_library()
f = lib.lidar_diag_fps_wave
f.argtypes = [nat.P, nat.P, nat.I64, nat.I64, nat.I64, nat.P, nat.P, nat.P]
h = nat.handle(0)
for B in BS:
    x = torch.from_numpy(unit_frames(B, N, seed=5)).to(dev)
    idx = torch.empty((B, M), dtype=torch.int32, device=dev)
    diag = torch.zeros((B, 9), dtype=torch.int64, device=dev)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nat.check(f(h, nat.ptr(x), B, N, M, nat.ptr(idx), nat.ptr(diag), nat.stream_ptr()), "diag")
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    d = diag.cpu().numpy().astype(np.float64)
    steps = d[:, 8].mean()
    per = d[:, :8].sum(axis=0) / (B * steps)
    tot = per[:4].sum()
    print(f"B={B} N={N} M={M}: wall {wall * 1e3:.2f} ms ({wall * 1e6 / M:.2f} us/step); cycles per step: "
          f"slots+list {per[0]:.0f}, batches {per[1]:.0f}, re-key {per[2]:.0f}, argmax {per[3]:.0f} "
          f"(sum {tot:.0f} = {tot / 2.4e3:.2f} us at 2.4 GHz); per step: active slots {per[4]:.2f}, "
          f"active buckets {per[5]:.2f}, batches {per[6]:.2f}, re-keyed slots {per[7]:.2f}", flush=True)
