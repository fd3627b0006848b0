"""Tier N feature precision, measured: for the x3 (split-bf16) and native fp32-MFMA kernels,
the max pure relative error |got - want| / |want| over elements with |want| >= f * RMS(want)
for several floors f, against the fp32 oracle.  Prints one JSON record (GPU)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import tier_n  # noqa: E402
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

FLOORS = (1e-4, 1e-3, 1e-2, 1e-1)


def stats(got, want):
    got = np.asarray(got, np.float64).ravel()
    want = np.asarray(want, np.float64).ravel()
    rms = float(np.sqrt(np.mean(want ** 2))) + 1e-30
    err = np.abs(got - want)
    out = {"rms": rms, "max_abs_over_rms": float(err.max() / rms)}
    for f in FLOORS:
        big = np.abs(want) >= f * rms
        out[f"rel@{f:g}"] = float((err[big] / np.abs(want[big])).max()) if big.any() else 0.0
    return out


def main():
    dev = torch.device("cuda:0")
    rec = {}
    for cfg_name, n in (("ssg", 16384), ("ssg", 65536), ("msg", 16384)):
        for x3 in (True, False):
            cfg = pn.CONFIGS[cfg_name]
            bb = pn.PointNet2Backbone(cfg, device=dev, seed=0, x3=x3)
            x = unit_frames(1, n, 21)
            g, levels = bb.forward(torch.from_numpy(x).to(dev), keep_levels=True)
            torch.cuda.synchronize()
            want, wl = tier_n.sa_stack(x[0], {"levels": pn.resolve(cfg, n)}, bb.weights)
            key = f"{cfg_name}_{n}_{'x3' if x3 else 'fp32'}"
            rec[key] = {f"level{li + 1}": stats(lv[1].cpu().numpy()[0], w[1]) for li, (lv, w) in
                        enumerate(zip(levels, wl))}
            rec[key]["global"] = stats(g.cpu().numpy()[0], want)
            # the oracle in float64 (what the fp32 oracle itself carries)
            print(key, json.dumps(rec[key]["global"]), flush=True)
    # a single x3 GEMM against the float64 product
    rng = np.random.default_rng(1)
    for rows, k, cout in ((1024, 256, 512), (1024, 144, 128)):
        xa = rng.standard_normal((rows, k)).astype(np.float32)
        w = (rng.standard_normal((k, cout)) / np.sqrt(k)).astype(np.float32)
        b = np.zeros(cout, np.float32)
        T = lambda a: torch.from_numpy(a).to(dev)
        got = pn.dense_x3s(T(xa), pn.pack_dense_x3(T(w)), T(b), cout, relu=False).cpu().numpy()
        want64 = xa.astype(np.float64) @ w.astype(np.float64)
        want32 = xa @ w
        rec[f"dense_x3_{rows}x{k}x{cout}_vs_f64"] = stats(got, want64)
        rec[f"numpy_fp32_{rows}x{k}x{cout}_vs_f64"] = stats(want32, want64)
        gotn = pn.dense(T(xa), T(w), T(b), relu=False).cpu().numpy()
        rec[f"dense_fp32mfma_{rows}x{k}x{cout}_vs_f64"] = stats(gotn, want64)
    out = os.path.join(REPO, "gpurun_out", "precision_probe.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
