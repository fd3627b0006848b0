"""Per-run scalars + label digest of one Tier R case (nondeterminism hunt)."""
import hashlib
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from golden_cases import FRAMES  # noqa: E402
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2])
pts = FRAMES[name]()
n = len(pts)
dev = torch.device("cuda:0")
x = torch.from_numpy(np.ascontiguousarray(pts, dtype=np.float64)).to(dev)
for r in range(reps):
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    colors = torch.empty((n, 3), dtype=torch.float64, device=dev)
    normals = torch.empty((n, 3), dtype=torch.float64, device=dev)
    comp = torch.empty((n, 3), dtype=torch.float64, device=dev)
    labels = torch.empty(n, dtype=torch.int64, device=dev)
    scal = torch.empty(64, dtype=torch.float64, device=dev)
    nat.call("lidar_preprocess_f64", nat.handle(0), nat.ptr(x), n, nat.ptr(mask), nat.ptr(colors), nat.ptr(normals),
             nat.ptr(comp), nat.ptr(labels), nat.ptr(scal), nat.stream_ptr())
    torch.cuda.synchronize()
    S = scal.cpu().numpy()
    lab = labels.cpu().numpy()
    print(r, "eps", S[4].hex(), "smean", [v.hex() for v in S[22:25]], "sscale", [v.hex() for v in S[25:28]],
          "ncl", int(S[39]), "labels", hashlib.sha256(lab.tobytes()).hexdigest()[:12],
          "noise", int((lab < 0).sum()), flush=True)
