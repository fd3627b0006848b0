"""The SA1 FPS step phases INSIDE the bench's pipeline, beside the same kernel alone.

The diagnostic library's lidar_diag_fps_record makes every SA1 FPS launch of 512 threads (no prefix_ok)
take the DIAG instantiation of fps_bucket_kernel<512, BPL> and append its per-(frame, wave) phase totals:
[0] bucket tests + active-bucket updates, [1] wave argmax + LDS publish, [2] barrier wait, [3] merge,
[4] active-bucket batches, [5] steps.  The pipeline is bench.py's (SSG, 32 x 65 536-point batches,
StreamingSSG depth 3, G batches per group, bq "bin", l2_side); only the launches of the timed window are
recorded.  Then the same kernel alone at the window's launch size.  Prints cycles per wave-step per phase
(s_memtime) and a JSON record.

usage: LIDAR_AMD_LIB=lidar_ai_recommendation_software_amd/liblidar_amd_diag.so \\
       python tools/micro/fps_pipe_phases.py [steps] [G] [out.json]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
out = sys.argv[3] if len(sys.argv) > 3 else None
B, N, depth = 32, 65536, 3
M = N // 16
dev = torch.device("cuda:0")
lib = nat.load_library()
assert hasattr(lib, "lidar_diag_fps_record"), "needs the diagnostic library (LIDAR_AMD_LIB=...diag.so)"
lib.lidar_diag_fps_record.argtypes = [nat.P, nat.I64]
lib.lidar_diag_fps_recorded.restype = nat.I64
lib.lidar_diag_fps_recorded.argtypes = []

bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
xs = [torch.from_numpy(unit_frames(B, N, seed=100 + i)).to(dev) for i in range(8)]
ready = torch.cuda.Event()
ready.record()
pipe = pn.StreamingSSG(bb, B, N, depth=depth, fps_group=G, fps_threads=512, ramp=False, bq="bin", l2_side=True)
feed = pipe.feed()
nwarm = (depth + 1) * G
for i in range(nwarm):
    feed.push(xs[i % 8], ready)
cap = (steps // G + 2) * G * B * 8 * 6
rec = torch.zeros(cap, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
nat.check(lib.lidar_diag_fps_record(nat.ptr(rec), cap), "record")
t0 = time.perf_counter()
for i in range(nwarm, nwarm + steps):
    feed.push(xs[i % 8], ready)
torch.cuda.synchronize()
wall = time.perf_counter() - t0
used = lib.lidar_diag_fps_recorded()
nat.check(lib.lidar_diag_fps_record(None, 0), "stop")
feed.flush()
d_pipe = rec[:used].view(-1, 8, 6).cpu().numpy().astype(np.float64)


def summary(d):
    st = d[..., 5].sum()
    per = d[..., :5].sum(axis=(0, 1)) / st
    return {"update": per[0], "argmax_publish": per[1], "barrier": per[2], "merge": per[3],
            "sum": per[:4].sum(), "batches_per_wave_step": per[4], "frames": int(d.shape[0])}


# the same kernel alone, at the window's launch size (G * B frames), recorded the same way
GB = G * B
xa = torch.cat(xs[:G])
rec2 = torch.zeros(GB * 8 * 6, dtype=torch.int64, device=dev)
pn.farthest_point_sample(xa, M, threads=512)  # warm-up (workspace)
torch.cuda.synchronize()
nat.check(lib.lidar_diag_fps_record(nat.ptr(rec2), rec2.numel()), "record")
t1 = time.perf_counter()
pn.farthest_point_sample(xa, M, threads=512)
torch.cuda.synchronize()
alone_ms = (time.perf_counter() - t1) * 1e3
nat.check(lib.lidar_diag_fps_record(None, 0), "stop")
d_alone = rec2.view(-1, 8, 6).cpu().numpy().astype(np.float64)
res = {"config": {"frames_per_launch": GB, "points_per_frame": N, "samples": M, "steps": steps, "depth": depth,
                  "fps_threads": 512},
       "unit": "shader cycles (s_memtime) per wave and step",
       "pipeline": summary(d_pipe), "alone": summary(d_alone),
       "pipeline_M_points_per_s_diag_build": B * N * steps / wall / 1e6, "alone_launch_ms": alone_ms}
for k in ("pipeline", "alone"):
    s = res[k]
    print(f"{k:8s}: update {s['update']:6.0f}  argmax+publish {s['argmax_publish']:5.0f}  barrier {s['barrier']:6.0f}  "
          f"merge {s['merge']:5.0f}  sum {s['sum']:6.0f} cycles/wave-step; batches {s['batches_per_wave_step']:.2f}; "
          f"{s['frames']} frames", flush=True)
print(json.dumps(res))
if out:
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
