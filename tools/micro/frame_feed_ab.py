"""frame_feed.HostFrameFeed (host NumPy frames -> the reference's density dicts, PCIe included) per batch size and
number of lanes,
on `frames` uniform 65 536-point frames, against the drop-in API one frame per call; results checked equal.
usage: python tools/micro/frame_feed_ab.py [frames]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import data_processing as dp  # noqa: E402
from lidar_ai_recommendation_software_amd.crowd_density_model import CrowdDensityModel  # noqa: E402
from lidar_ai_recommendation_software_amd.frame_feed import HostFrameFeed  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import uniform_frame  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 192
n = 65536
xs = [uniform_frame(n, 7000 + i) for i in range(frames)]
model = CrowdDensityModel()
want = [model.analyze(dp.preprocess_lidar_data(x)) for x in xs[:8]]
for rep in range(2):
    for batch, lanes in ((8, 1), (32, 1), (16, 3), (32, 3), (64, 3), (32, 2)):
        feed = HostFrameFeed(batch=batch, lanes=lanes)
        feed.run(xs[:batch * lanes])  # warm-up: every lane's pinned buffers, handle and workspaces sized
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = feed.run(xs)
        dt = time.perf_counter() - t0
        assert all(a["total_people"] == b["total_people"] and np.array_equal(a["density_map"], b["density_map"])
                   for a, b in zip(want, got[:8]))
        print(f"batch {batch:3d} lanes {lanes}: {frames * n / dt / 1e6:7.1f} M points/s ({dt / frames * 1e3:.3f} ms "
              "per frame)", flush=True)
