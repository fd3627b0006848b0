"""Micro-benchmarks of single kernels (GPU box): python tools/micro.py [fps|mlp|bq]."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    what = sys.argv[1:] or ["fps", "mlp", "bq"]
    dev = torch.device("cuda:0")
    for B, N in ((32, 65536), (1, 65536), (256, 65536)):
        x = torch.from_numpy(unit_frames(B, N, 0)).to(dev)
        if "fps" in what:
            M = N // 16
            ms = timeit(lambda: pn.farthest_point_sample(x, M, return_xyz=True))
            print(f"fps B={B} N={N} M={M}: {ms:.3f} ms  ({ms * 1e3 / M:.2f} us/step)", flush=True)
            if B == 32:
                c = pn.farthest_point_sample(x, M, return_xyz=True)[1]
                ms2 = timeit(lambda: pn.farthest_point_sample(c, N // 64, return_xyz=True))
                print(f"fps2 (no shortcut) B={B} N={M} M={N // 64}: {ms2:.3f} ms", flush=True)
        if "bq" in what and B == 32:
            c = x[:, : N // 16].contiguous()
            ms = timeit(lambda: pn.ball_query(0.2, 32, x, c))
            print(f"ball_query B={B} N={N} M={N // 16} r0.2 ns32 (random centres): {ms:.3f} ms", flush=True)
            c = pn.farthest_point_sample(x, N // 16, return_xyz=True)[1]
            ms = timeit(lambda: pn.ball_query(0.2, 32, x, c))
            print(f"ball_query B={B} N={N} M={N // 16} r0.2 ns32 (FPS centres): {ms:.3f} ms", flush=True)


if __name__ == "__main__" and not ({"phases", "mlp", "tier_r", "dense", "tier_r_batch"} & set(sys.argv)):
    main()


def fps_phases():
    import ctypes
    from lidar_ai_recommendation_software_amd import _native as nat
    lib = nat.load_library()
    lib.lidar_diag_fps_phases.argtypes = [nat.P, nat.P, nat.I64, nat.I64, nat.I64, nat.P, nat.P, nat.P]
    dev = torch.device("cuda:0")
    for B in (1, 32):
        N, M = 65536, 4096
        x = torch.from_numpy(unit_frames(B, N, 0)).to(dev)
        idx = torch.empty((B, M), dtype=torch.int32, device=dev)
        diag = torch.zeros((B, 16, 6), dtype=torch.int64, device=dev)
        for _ in range(2):
            nat.check(lib.lidar_diag_fps_phases(nat.handle(0), nat.ptr(x), B, N, M, nat.ptr(idx), nat.ptr(diag),
                                                nat.stream_ptr()), "diag")
        torch.cuda.synchronize()
        d = diag.cpu().numpy().astype(np.float64)
        steps = d[..., 5].mean()
        per = d[..., :4].mean(axis=(0, 1)) / steps
        print(f"B={B}: cycles/step  test+update={per[0]:.0f} wave-argmax={per[1]:.0f} "
              f"submit+barrier={per[2]:.0f} broadcast={per[3]:.0f}  (slowest wave's test+update: "
              f"{d[..., 0].max(axis=1).mean() / steps:.0f}; update batches/step/wave {d[..., 4].mean() / steps:.2f})",
              flush=True)


if __name__ == "__main__" and "phases" in sys.argv:
    fps_phases()


def mlp_micro():
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    w = pn.init_weights(pn.SSG, 0)
    B = 32
    for name, (N, M, ns, cf, layers, widths) in {
            "sa1": (65536, 4096, 32, 0, w[0][0], [64, 64, 128]),
            "sa2": (4096, 1024, 64, 128, w[1][0], [128, 128, 256])}.items():
        x = torch.from_numpy(unit_frames(B, N, 1)).to(dev)
        f = torch.from_numpy(rng.standard_normal((B, N, cf)).astype(np.float32)).to(dev) if cf else None
        c = x[:, :M].contiguous()
        gi = torch.from_numpy(rng.integers(0, N, (B, M, ns)).astype(np.int32)).to(dev)
        packed = torch.from_numpy(pn.pack_branch(layers, cf)).to(dev)
        out = torch.empty((B, M, widths[-1]), dtype=torch.float32, device=dev)
        ms = timeit(lambda: pn.group_mlp(x, f, c, gi, packed, widths, out=out), reps=10)
        dims = [3 + cf] + widths
        flops = 2 * B * M * ns * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
        print(f"{name} group_mlp: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s ({flops / ms / 1e9 / 157.3 * 100:.1f}% of fp32 peak)",
              flush=True)
        pk16 = torch.from_numpy(pn.pack_branch16(layers, cf == 0)).to(dev)
        pkx3 = torch.from_numpy(pn.pack_branch_x3(layers, cf == 0)).to(dev)
        if cf == 0:
            ms = timeit(lambda: pn.group_mlp16(x, c, gi, N, pk16, widths, out, xyz_level=True), reps=10)
            print(f"{name} group_mlp16: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s", flush=True)
            ms = timeit(lambda: pn.group_mlp_x3(x, c, gi, N, pkx3, widths, out, xyz_level=True), reps=10)
            print(f"{name} group_mlp_x3: {ms:.3f} ms  {flops / ms / 1e9:.1f} fp32-equivalent TFLOP/s", flush=True)
        if cf:
            P = torch.from_numpy(rng.standard_normal((B * N, widths[0])).astype(np.float32)).to(dev)
            Q = torch.from_numpy(rng.standard_normal((B * M, widths[0])).astype(np.float32)).to(dev)
            ms = timeit(lambda: pn.group_mlp_pre(P, Q, gi, N, packed, cf, widths, out), reps=10)
            flops = 2 * B * M * ns * sum(a * b for a, b in zip(widths[:-1], widths[1:]))
            print(f"{name} group_mlp_pre (layers 2-3): {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s "
                  f"({flops / ms / 1e9 / 157.3 * 100:.1f}% of fp32 peak)", flush=True)
            ms = timeit(lambda: pn.group_mlp16(P, Q, gi, N, pk16, widths, out), reps=10)
            print(f"{name} group_mlp16 (layers 2-3): {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s", flush=True)
            ms = timeit(lambda: pn.group_mlp_x3(P, Q, gi, N, pkx3, widths, out), reps=10)
            print(f"{name} group_mlp_x3 (layers 2-3): {ms:.3f} ms  {flops / ms / 1e9:.1f} fp32-equivalent TFLOP/s",
                  flush=True)


if __name__ == "__main__" and "mlp" in sys.argv:
    mlp_micro()


def tier_r_micro():
    """Per-stage device time of the reference density path (Tier R) per frame."""
    from lidar_ai_recommendation_software_amd import _native as nat
    from lidar_ai_recommendation_software_amd import data_processing as dp
    from lidar_ai_recommendation_software_amd.crowd_density_model import CrowdDensityModel
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame, crowd_frame
    dev = torch.device("cuda:0")
    for kind, n in (("uniform", 65536), ("crowd", 65536), ("uniform", 131072)):
        pts = uniform_frame(n, 0) if kind == "uniform" else crowd_frame(n, 0)
        x = torch.from_numpy(np.ascontiguousarray(pts, dtype=np.float64)).to(dev)
        mask = torch.empty(n, dtype=torch.uint8, device=dev)
        colors = torch.empty((n, 3), dtype=torch.float64, device=dev)
        normals = torch.empty((n, 3), dtype=torch.float64, device=dev)
        comp = torch.empty((n, 3), dtype=torch.float64, device=dev)
        labels = torch.empty(n, dtype=torch.int64, device=dev)
        scal = torch.empty(64, dtype=torch.float64, device=dev)
        h = nat.handle(0)

        def pre():
            nat.call("lidar_preprocess_f64", h, nat.ptr(x), n, nat.ptr(mask), nat.ptr(colors), nat.ptr(normals),
                     nat.ptr(comp), nat.ptr(labels), nat.ptr(scal), nat.stream_ptr())
        ms_pre = timeit(pre, reps=5)
        model = CrowdDensityModel(1.0)
        t0 = time.perf_counter()
        for _ in range(3):
            pd = dp.preprocess_lidar_data(pts)
            res = model.analyze(pd)
        ms_all = (time.perf_counter() - t0) / 3 * 1e3
        print(f"tier_r {kind} N={n}: preprocess+dbscan device {ms_pre:.3f} ms; drop-in preprocess+analyze "
              f"(host in/out) {ms_all:.2f} ms; people {res['total_people']}", flush=True)


if __name__ == "__main__" and "tier_r" in sys.argv and "tier_r_batch" not in sys.argv:
    tier_r_micro()


def dense_micro():
    """group_all's three dense layers: liblidar_amd dense kernel vs hipBLASLt (torch)."""
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    rows = 64 * 1024
    for k, n in ((144, 128), (272, 256), (256, 512), (512, 1024)):
        x = torch.from_numpy(rng.standard_normal((rows, k)).astype(np.float32)).to(dev)
        w = torch.from_numpy((rng.standard_normal((k, n)) / np.sqrt(k)).astype(np.float32)).to(dev)
        b = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
        ms_own = timeit(lambda: pn.dense(x, w, b), reps=10)
        wp = pn.pack_dense_x3(w)
        ms_x3 = timeit(lambda: pn.dense(x, w, b, x3=True, wpack=wp), reps=10)
        print(f"dense x3 {k}x{n}: {ms_x3:.3f} ms ({2 * rows * k * n / ms_x3 / 1e9:.0f} fp32-equivalent TF)", flush=True)
        sp = pn.split_x3(x)
        for name, a in (("planes", sp), ("fp32", x)):
            for mode, kw in (("rows", {}), ("split", {"split_out": True}), ("pool", {"pool_rows": 1024})):
                ms_s = timeit(lambda: pn.dense_x3s(a, wp, b, n, **kw), reps=10)
                print(f"  x3s {name:6s} -> {mode:5s} {k}x{n}: {ms_s:.3f} ms ({2 * rows * k * n / ms_s / 1e9:.0f} TF)",
                      flush=True)
        ms_sp = timeit(lambda: pn.split_x3(x), reps=10)
        print(f"  split_x3 {rows}x{k}: {ms_sp:.3f} ms ({rows * k * 8 / ms_sp / 1e6:.0f} GB/s)", flush=True)
        ms_blas = timeit(lambda: torch._addmm_activation(b, x, w), reps=10)
        ms_mm = timeit(lambda: torch.relu_(torch.addmm(b, x, w)), reps=10)
        fl = 2 * rows * k * n
        err = (pn.dense(x, w, b) - torch._addmm_activation(b, x, w)).abs().max().item()
        print(f"dense {k}x{n}: own {ms_own:.3f} ms ({fl / ms_own / 1e9:.0f} TF)  hipblaslt+relu {ms_blas:.3f} ms "
              f"({fl / ms_blas / 1e9:.0f} TF)  addmm+relu {ms_mm:.3f} ms  maxdiff {err:.2e}", flush=True)


if __name__ == "__main__" and "dense" in sys.argv:
    dense_micro()


def tier_r_batch_micro():
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    dev = torch.device("cuda:0")
    for F in (8, 32, 64):
        xs = [torch.from_numpy(uniform_frame(65536, 1000 + i)).to(dev) for i in range(F)]
        ds = DensityStream(dev, workers=4)
        ds.run_batch(xs)
        ds.run(xs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ds.run_batch(xs)
        tb = (time.perf_counter() - t0) / 3
        t0 = time.perf_counter()
        for _ in range(3):
            ds.run(xs)
        tw = (time.perf_counter() - t0) / 3
        print(f"tier_r F={F} x 65536: batch {tb * 1e3:.1f} ms ({F * 65536 / tb / 1e6:.1f} M pts/s)  "
              f"4 workers {tw * 1e3:.1f} ms ({F * 65536 / tw / 1e6:.1f} M pts/s)", flush=True)


if __name__ == "__main__" and "tier_r_batch" in sys.argv:
    tier_r_batch_micro()
