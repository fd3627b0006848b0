"""Run one Tier R golden case N times in one process and report byte-equality per run."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
from golden_cases import FRAMES, META, digest  # noqa: E402
from lidar_ai_recommendation_software_amd import data_processing as dp  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
pts = FRAMES[name]()
want = META["cases"][name]
for r in range(reps):
    pd = dp.preprocess_lidar_data(pts)
    ok = {k: digest(pd[k])["sha256"] == want[k]["sha256"] for k in ("points", "colors", "normals", "clusters")}
    lab = pd["clusters"]
    print(name, r, ok, "n_clusters", int(lab.max()) + 1, "noise", int((lab < 0).sum()), flush=True)
