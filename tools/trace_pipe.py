"""Run a StreamingSSG pipeline for the timeline (use under rocprofv3 --kernel-trace)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

cfg_name, dtype, B, N, steps, depth = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
group = int(sys.argv[7]) if len(sys.argv) > 7 else 1
mlp16 = {"0": False, "1": True}.get(sys.argv[8], sys.argv[8]) if len(sys.argv) > 8 else False
dev = torch.device("cuda:0")
x3 = {"0": False, "1": True}.get(sys.argv[9], sys.argv[9]) if len(sys.argv) > 9 else False
bb = pn.PointNet2Backbone(pn.CONFIGS[cfg_name], device=dev, seed=0, dtype=dtype, mlp16=mlp16, x3=x3)
x = torch.from_numpy(unit_frames(B, N, 0)).to(dev)
bqm = len(sys.argv) > 10 and sys.argv[10] == "1"
fpst = int(sys.argv[11]) if len(sys.argv) > 11 else 0
pipe = pn.StreamingSSG(bb, B, N, depth=depth, fps_group=group, bq_on_main=bqm, fps_threads=fpst)
pipe.run([x] * 3)
torch.cuda.synchronize()
t0 = time.perf_counter()
pipe.run([x] * steps)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"{cfg_name} {dtype} B={B} N={N} depth={depth} group={group} mlp16={mlp16} x3={x3} bq_main={int(bqm)}: {dt / steps * 1e3:.2f} ms/step, {B * N * steps / dt / 1e6:.1f} M pts/s", flush=True)
