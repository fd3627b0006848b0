"""Where the host-frame SSG feed's time goes: the bench's pipeline (32 x 65 536-point batches, depth 3, G 4) fed
by push_host, the wall time per batch against (a) the host time inside push_host per call and (b) the same
pinned fill done alone (4 threads), and the device-resident feed's time per batch beside it.
usage: python tools/host_feed_probe.py [steps] [threads]"""
import concurrent.futures
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B, N, depth, G = 32, 65536, 3, 4
dev = torch.device("cuda:0")
bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
hx = [unit_frames(B, N, seed=300 + i) for i in range(8)]
xs = [torch.from_numpy(h).to(dev) for h in hx]
ready = torch.cuda.Event()
ready.record()


def run(host):
    pipe = pn.StreamingSSG(bb, B, N, depth=depth, fps_group=G, fps_threads=512, ramp=False, bq="bin", l2_side=True)
    feed = pipe.feed()
    push = (lambda i: feed.push_host(hx[i % 8], threads=threads)) if host else (lambda i: feed.push(xs[i % 8], ready))
    for i in range((depth + 2) * G):
        push(i)
    torch.cuda.synchronize()
    inside = 0.0
    t0 = time.perf_counter()
    for i in range(steps):
        a = time.perf_counter()
        push(i)
        inside += time.perf_counter() - a
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    feed.flush()
    return wall / steps * 1e3, inside / steps * 1e3


for host in (False, True, False, True):
    w, ins = run(host)
    print(f"{'host' if host else 'device':6s}: {w:.3f} ms per batch wall, {ins:.3f} ms inside push per call "
          f"({B * N / w / 1e3:.0f} M points/s)", flush=True)
pin = torch.empty((B, N, 3), dtype=torch.float32, pin_memory=True).numpy()
pool = concurrent.futures.ThreadPoolExecutor(max_workers=threads)
step = -(-B // threads)
for rep in range(3):
    t0 = time.perf_counter()
    fs = [pool.submit(lambda lo: [np.copyto(pin[j], hx[rep][j]) for j in range(lo, min(B, lo + step))], lo)
          for lo in range(0, B, step)]
    for f in fs:
        f.result()
    print(f"fill alone ({threads} threads): {(time.perf_counter() - t0) * 1e3:.3f} ms per batch", flush=True)
