#!/usr/bin/env python3
"""bench.py — M points/s through the PointNet++ SetAbstraction stack on 65 536-point frames.

BASELINE.json metric: "M points/sec through SetAbstraction, 65k-pt frames; 1->8 GPU
scaling".  Workload (configs[2] / configs[3]): the 3-level SSG encoder
(SA1 N/16 r=0.2 ns=32 [64,64,128]; SA2 N/64 r=0.4 ns=64 [128,128,256]; group_all
[256,512,1024]) in fp32 on 65 536-point frames; per GPU a batch of 32 frames — the
per-GPU share of configs[3] (256 frames over 8 GPUs) — so N GPUs process 32*N frames
per step (weak scaling, per-frame data parallel, no collective on the data path).

A step = FPS + ball query + fused group/MLP/max-pool for SA1 and SA2, then group_all
(three MFMA dense layers with a fused max-pool) over the batch, inputs resident in HBM.
Steps run through pointnet2.StreamingSSG — the steady state of a continuous LiDAR feed:
later batches' SA1 FPS (latency-bound, one 512-thread workgroup per frame) and the SA1
ball-query binning run on side streams (--depth 3 groups in flight) while earlier batches'
ball queries and MFMA levels run on the main stream; groups of three batches share one
FPS launch and one main-stream pass (--fps-group 3; every operator is per frame, outputs
are bit-identical to one-batch forward()).  K steps = K batches of 32 frames fully
processed inside the timed region (pipeline fill included).
Synthetic data: uniform [-1, 1]^3 float32 frames (seeded per rank), random-init weights.

Run:  python bench.py [--gpus N --steps K --warmup W]  (N>1 via torch.distributed.run)
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# per-frame algorithmic work of each kernel of the SSG stack at N points
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 matrix (= vector) peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 dense matrix peak
# the x3 kernels carry each fp32 product as 3 bf16 MFMA products: their fp32-equivalent peak
X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0


def mlp_flops(rows, widths_in):
    return 2 * rows * sum(a * b for a, b in zip(widths_in[:-1], widths_in[1:]))


def ssg_kernel_work(n):
    m1, m2 = n // 16, n // 64
    return {
        "sa1_group_mlp": ("mfma", mlp_flops(m1 * 32, [3, 64, 64, 128])),
        # SA2 layer 1 runs per point (N/16 rows of [f, x] W1 + b1, N/64 centre rows of
        # c W1_xyz); the fused kernel computes layers 2-3 of every grouped row
        "sa2_layer1_points": ("mfma", 2 * m1 * 131 * 128 + 2 * m2 * 3 * 128),
        "sa2_group_mlp": ("mfma", mlp_flops(m2 * 64, [128, 128, 256])),
        "sa3_dense1": ("mfma", mlp_flops(m2, [259, 256])),
        "sa3_dense2": ("mfma", mlp_flops(m2, [256, 512])),
        "sa3_dense3_pool": ("mfma", mlp_flops(m2, [512, 1024])),
        # compulsory bytes: read xyz, write idx + new_xyz
        "sa1_fps": ("hbm", 12 * n + 16 * m1),
        "sa2_fps": ("hbm", 12 * m1 + 16 * m2),
        "sa1_ball_query": ("hbm", 12 * (n + m1) + 4 * m1 * 32),
        # the grid ball query's binning (side stream): read xyz, write (x, y, z, index) + slot table
        "sa1_bq_bin": ("hbm", 12 * n + 16 * n + 4 * 16385),
        "sa2_ball_query": ("hbm", 12 * (m1 + m2) + 4 * m2 * 64),
    }


def pmc_traffic(B, N):
    """Memory-side bytes per launch from the committed PMC passes (tools/pmc_traffic.py),
    when they were taken on this same workload; None otherwise."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_traffic.json")))
    if not files:
        return {}
    with open(files[-1]) as f:
        d = json.load(f)
    c = d.get("config", {})
    if c.get("points_per_frame") != N or c.get("frames_per_gpu") != B:
        return {}
    return {k: v["traffic_bytes"] for k, v in d.get("kernels", {}).items()}


def cpu_baseline(n, budget_s=20.0):
    """The oracle SA stack (C FPS / ball query + numpy MLP, BLAS pinned to 1 thread) on
    one frame of the same workload, on this host.  kind = "port" (the reference has no
    SetAbstraction code to time)."""
    from threadpoolctl import threadpool_limits
    from oracle import tier_n
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    cfg = pn.SSG
    w = pn.init_weights(cfg, 0)
    frames, t0 = 0, time.perf_counter()
    with threadpool_limits(limits=1):
        while True:
            x = unit_frames(1, n, 1000 + frames)[0]
            tier_n.sa_stack(x, {"levels": pn.resolve(cfg, n)}, w)
            frames += 1
            if time.perf_counter() - t0 > budget_s or frames >= 64:
                break
    dt = time.perf_counter() - t0
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    return {"value": frames * n / dt / 1e6, "unit": "M points/s", "cores": 1, "kind": "port",
            "sample": f"{frames} x {n}-point SSG frame(s) through oracle/tier_n.sa_stack "
                      f"(C FPS + C ball query + numpy fp32 MLP, 1 thread) in {dt:.1f} s on {cpu}; "
                      f"host has {os.cpu_count()} logical CPUs"}


def tier_r_cpu_baseline(n, budget_s=12.0):
    """oracle/tier_r (the byte-identical CPU restatement of the reference density path:
    numpy + the C DBSCAN of the same neighbourhood rule) on uniform +-15 m frames."""
    from oracle import tier_r
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    frames, t0 = 0, time.perf_counter()
    while True:
        pd = tier_r.preprocess_lidar_data(uniform_frame(n, 2000 + frames))
        tier_r.analyze(pd)
        frames += 1
        if time.perf_counter() - t0 > budget_s or frames >= 32:
            break
    dt = time.perf_counter() - t0
    return {"value": frames * n / dt / 1e6, "unit": "M points/s", "cores": 1, "kind": "port",
            "sample": f"{frames} x {n}-point uniform frame(s) through oracle/tier_r preprocess + analyze "
                      f"(byte-identical restatement of the reference's numpy/sklearn path, 1 thread) in {dt:.1f} s"}


def tier_r_leg(dev, rank, world, frames=32, n=65536, workers=4, steps=3, cpu=True, cpu_budget=12.0):
    """The reference's own path (Tier R: preprocess -> DBSCAN -> people -> density grid) on
    device-resident uniform +-15 m frames: batches of `frames` frames through
    density_stream.DensityStream.run_batch (one launch per phase over the CSR batch)."""
    import torch
    from lidar_ai_recommendation_software_amd import sharding
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    xs = [torch.from_numpy(uniform_frame(n, sharding.frame_seed(rank, base=1000 + i))).to(dev) for i in range(frames)]
    ds = DensityStream(dev, workers=workers)
    ds.run_batch(xs)  # warm-up: workspaces sized
    el = sharding.timed(lambda: [ds.run_batch(xs) for _ in range(steps)], dev, world)
    rec = {"metric": "M points/s through the reference density path (preprocess + DBSCAN + people + "
                     "density grid), device-resident frames",
           "value": sharding.aggregate_rate(frames * n * steps, world, el) / 1e6, "unit": "M points/s",
           "ms_per_frame": el / (frames * steps) * 1e3, "frames_per_gpu": frames, "points_per_frame": n,
           "executor": "DensityStream.run_batch (CSR batch, one launch per phase)", "dtype": "f64",
           "parity": "byte-identical to the reference (tests/golden)",
           "cpu_baseline": None}
    if cpu and rank == 0 and world == 1:
        rec["cpu_baseline"] = tier_r_cpu_baseline(n, cpu_budget)
        rec["speedup_vs_cpu"] = rec["value"] / rec["cpu_baseline"]["value"]
    return rec


def voxel_leg(dev, rank, world, B=32, n=65536, voxel=0.05, steps=20, cpu=True):
    """voxel downsampling of the SA batch (B x n uniform frames, device-resident)
    on the chip-wide path (lidar_voxel_downsample_batch_f32).  Roofline: algorithmic bytes per
    launch (12 B per point in + 4 B voxel id out + 16 B per voxel out) over 8 TB/s."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    from lidar_ai_recommendation_software_amd import sharding
    x = torch.from_numpy(unit_frames(B, n, seed=sharding.frame_seed(rank, base=77))).to(dev)
    out = pn.voxel_downsample_batch(x, voxel)
    torch.cuda.synchronize(dev)
    el = sharding.timed(lambda: [pn.voxel_downsample_batch(x, voxel) for _ in range(steps)], dev, world)
    nv = int(out[3].sum().item())
    per_launch = el / steps
    algo = B * n * 16 + nv * 16
    rec = {"metric": "M points/s through voxel_downsample (batched, device-resident frames)",
           "value": sharding.aggregate_rate(B * n * steps, world, el) / 1e6, "unit": "M points/s",
           "ms_per_launch": per_launch * 1e3, "frames": B, "points_per_frame": n, "voxel": voxel,
           "voxels_per_frame": nv / B, "parity": "bit-exact vs oracle/tier_n.voxel_downsample "
           "(tests/test_gpu_tier_r.py::test_voxel_downsample_batch_vs_oracle)",
           "roofline": {"kernel": "voxel_downsample_batch (11 launches)", "bound": "hbm",
                        "achieved": algo / per_launch / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": algo / per_launch / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "work_per_launch": algo, "avg_launch_ms": per_launch * 1e3,
                        "peak_basis": "HBM peak; algorithmic bytes (the radix sort moves ~5x more)"},
           "cpu_baseline": None}
    if cpu and rank == 0 and world == 1:
        from oracle import tier_n
        xs = x[:2].cpu().numpy()
        t0 = time.perf_counter()
        for f in xs:
            tier_n.voxel_downsample(f, voxel)
        dt = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": len(xs) * n / dt / 1e6, "unit": "M points/s", "cores": 1, "kind": "port",
                               "sample": f"{len(xs)} x {n}-point frame(s) through oracle/tier_n.voxel_downsample "
                                         f"(C keys + numpy unique + the sequential sums) in {dt:.1f} s"}
    return rec


def variant_leg(rank, world, frames=8, n=65536, cpu=True, cpu_budget=6.0):
    """the Streamlit apps' own pipeline (app_simplified.py:76-137 ->
    :234-316, DBSCAN eps 0.3 on unscaled points + KDTree r = 2 cell counts) through the
    drop-in API, host NumPy frame in -> host dicts out (PCIe included), crowd frames."""
    import torch
    from lidar_ai_recommendation_software_amd import variant_pipeline as vp
    from lidar_ai_recommendation_software_amd.synthetic import crowd_frame
    xs = [crowd_frame(n, 500 + 97 * rank + i) for i in range(frames)]
    vp.analyze_crowd_density(vp.preprocess_point_cloud(xs[0]))  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x in xs:
        vp.analyze_crowd_density(vp.preprocess_point_cloud(x))
    dt = time.perf_counter() - t0
    rec = {"metric": "M points/s through app_simplified.py's preprocess_point_cloud + analyze_crowd_density "
                     "(drop-in API, host frames in / dicts out, one frame per call)",
           "value": frames * n / dt / 1e6, "unit": "M points/s", "ms_per_frame": dt / frames * 1e3,
           "points_per_frame": n, "frames": frames, "data": "synthetic crowd frames (people clumps, metres)",
           "parity": "byte-identical to scikit-learn's DBSCAN / KDTree results (tests/golden/variant.json)",
           "cpu_baseline": None}
    if cpu and rank == 0 and world == 1:
        from oracle import tier_r
        k, t0 = 0, time.perf_counter()
        while True:
            tier_r.variant_analyze_crowd_density(tier_r.variant_preprocess_point_cloud(xs[k % frames]))
            k += 1
            if time.perf_counter() - t0 > cpu_budget or k >= frames:
                break
        dtc = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": k * n / dtc / 1e6, "unit": "M points/s", "cores": 1, "kind": "port",
                               "sample": f"{k} x {n}-point crowd frame(s) through oracle/tier_r's variant "
                                         f"restatement (numpy + the C DBSCAN, 1 thread) in {dtc:.1f} s"}
        rec["speedup_vs_cpu"] = rec["value"] / rec["cpu_baseline"]["value"]
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=240,
                    help="timed steps; the pipeline fill (one SA1-FPS latency, ~12 ms) is inside the window")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--points", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU work per baseline sample")
    ap.add_argument("--depth", type=int, default=3, help="side streams (SA1-FPS groups in flight ahead of the MLPs)")
    ap.add_argument("--side-priority", type=int, default=0, help="HIP priority of the FPS streams (<0 = high)")
    ap.add_argument("--fps-group", type=int, default=3, help="batches per SA1-FPS launch (StreamingSSG fps_group)")
    ap.add_argument("--side-cus", type=int, default=0, help="CUs reserved for the SA1 FPS streams (0 = shared)")
    ap.add_argument("--fps-threads", type=int, default=512, choices=[256, 512, 1024],
                    help="SA1 FPS workgroup size in the pipeline (512: half the CU footprint beside the MLPs)")
    ap.add_argument("--cu-layout", default="xcd", choices=["xcd", "low"])
    ap.add_argument("--mlp16", default="pre", choices=["0", "1", "pre", "xyz"],
                    help="SA branches on the 16-row MFMA kernels: 1 all, pre / xyz only those levels")
    ap.add_argument("--x3", default="1", choices=["0", "1", "pre", "xyz"],
                    help="SA layers 2-3 on the split-bf16 (x3) kernels: fp32 arithmetic within the 1e-4 "
                         "contract; 0 = native fp32 MFMA kernels")
    ap.add_argument("--shared-bin", type=int, default=0,
                    help="1: one ball-query binning per group for all branches (MSG: 452 vs 468-494 M pts/s, off)")
    ap.add_argument("--ramp", type=int, default=1, help="1: first groups of 1, 2, .. batches (shorter fill)")
    ap.add_argument("--reserve", type=int, default=1, help="1: size the side handles' workspaces at setup")
    ap.add_argument("--x3s", type=int, default=1, help="1: dense layers on the split-plane x3 GEMM")
    ap.add_argument("--bq-main", type=int, default=0, help="1: SA1 ball queries on the main stream (0: on the FPS side streams)")
    ap.add_argument("--l1-side", type=int, default=0,
                    help="1: SA2's FPS and ball queries (they need only SA1's centres) on the side streams")
    ap.add_argument("--no-fp32-mfma-leg", action="store_true",
                    help="skip the extra measurement of the native fp32-MFMA kernels (when --x3 is on)")
    ap.add_argument("--msg-batch", type=int, default=32,
                    help="frames per GPU per step of the configs[4] MSG leg (32: the per-GPU share of 256 frames)")
    ap.add_argument("--msg-steps", type=int, default=30)
    ap.add_argument("--msg-x3", type=int, default=0, help="1: also time the MSG leg in fp32 on the x3 kernels")
    ap.add_argument("--no-extras", action="store_true", help="skip the configs[1]/[4] side measurements")
    ap.add_argument("--no-density", action="store_true", help="skip the Tier R density-path leg")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames

    from lidar_ai_recommendation_software_amd import sharding
    rank, world, local = sharding.world_info()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    B, N = args.batch, args.points

    x3_opt = {"0": False, "1": True}.get(args.x3, args.x3)

    def measure(cfg, dtype, B, N, steps, warmup, depth, events_in_window=True, x3=None):
        """events_in_window: HIP events around every launch inside the timed window (the
        headline: the roofline durations come from the same window).  False: the window
        runs clean and the per-kernel durations come from a second, instrumented window
        of the same length (with ~25 launches per step, as MSG has, the events cost ~1/3)."""
        bb = pn.PointNet2Backbone(cfg, device=dev, seed=0, dtype=dtype,
                                  mlp16={"0": False, "1": True}.get(args.mlp16, args.mlp16),
                                  x3=x3_opt if x3 is None else x3, x3s=bool(args.x3s))
        x = torch.from_numpy(unit_frames(B, N, seed=sharding.frame_seed(rank))).to(dev)
        # the streaming executor overlaps batch k+1's SA1 FPS + ball queries (latency-bound,
        # one workgroup per frame) with batch k's MFMA levels; results are identical to forward()
        pipe = pn.StreamingSSG(bb, B, N, depth=depth, side_priority=args.side_priority,
                               side_cus=args.side_cus, cu_layout=args.cu_layout, fps_group=args.fps_group,
                               bq_on_main=bool(args.bq_main), fps_threads=args.fps_threads,
                               level1_on_side=bool(args.l1_side), shared_bin=bool(args.shared_bin),
                               reserve=bool(args.reserve), ramp=bool(args.ramp))
        ref, _ = bb.forward(x)
        outs = pipe.run([x] * max(2, warmup))
        torch.cuda.synchronize(dev)
        assert all(torch.equal(ref, o) for o in outs), "streaming executor diverged from forward()"
        timers = pn._Timers()
        if events_in_window:
            bb.timers = timers  # HIP events around every launch, on the stream it is launched on
            elapsed = sharding.timed(lambda: pipe.run([x] * steps), dev, world)  # max over ranks
        else:
            elapsed = sharding.timed(lambda: pipe.run([x] * steps), dev, world)
            bb.timers = timers
            pipe.run([x] * steps)
            torch.cuda.synchronize(dev)
        bb.timers = None
        return elapsed, timers.mean_ms()

    elapsed, kern = measure(pn.SSG, "f32", B, N, args.steps, args.warmup, args.depth)
    fp32_mfma = None
    if x3_opt and not args.no_fp32_mfma_leg:
        # the same workload on the native fp32-MFMA kernels (clean window), for comparison
        el_f, k_f = measure(pn.SSG, "f32", B, N, args.steps, args.warmup, args.depth, events_in_window=False,
                            x3=False)
        fp32_mfma = {"value": sharding.aggregate_rate(B * N * args.steps, world, el_f) / 1e6, "unit": "M points/s",
                     "ms_per_step": el_f / args.steps * 1e3,
                     "sa2_group_mlp_ms": k_f.get("sa2_group_mlp"), "sa1_group_mlp_ms": k_f.get("sa1_group_mlp")}
    extras = {}
    if not args.no_extras:
        # the other BASELINE.json configs, measured the same way (not the headline metric)
        legs = [("configs[1]_sa1_16k_f32", pn.SA1_ONLY, "f32", 32, 16384, 40),
                ("configs[4]_msg_131k_bf16", pn.MSG, "bf16", args.msg_batch, 131072, args.msg_steps)]
        if args.msg_x3:  # the same MSG stack in fp32 arithmetic on the x3 kernels (bf16 MFMA products)
            legs.append(("configs[4]_msg_131k_f32x3", pn.MSG, "f32", args.msg_batch, 131072, args.msg_steps))
        for key, cfg, dtype, b2, n2, st in legs:
            el2, k2 = measure(cfg, dtype, b2, n2, st, 2, 3, events_in_window=False)
            extras[key] = {"M_points_per_s": sharding.aggregate_rate(b2 * n2 * st, world, el2) / 1e6, "ms_per_step": el2 / st * 1e3,
                           "frames_per_gpu": b2, "points_per_frame": n2, "dtype": dtype,
                           "kernel_ms": k2}

    density = None if args.no_density else tier_r_leg(dev, rank, world, cpu=not args.no_cpu_baseline, cpu_budget=args.cpu_budget)
    variant = None if args.no_density else variant_leg(rank, world, cpu=not args.no_cpu_baseline)
    voxel = None if args.no_density else voxel_leg(dev, rank, world, cpu=not args.no_cpu_baseline)
    work = ssg_kernel_work(N)
    traffic = pmc_traffic(B, N)
    # Two chains per group of batches: the side streams' SA1 FPS + ball queries (`depth`
    # groups in flight; FPS is one workgroup per frame, latency-bound: read as us/step) and
    # the main stream's full-chip kernels.  The roofline is reported for the kernel that
    # dominates the main chain's device time; the chain lengths say which chain bounds a step.
    # issued on the side streams, overlapped with the rest
    side = ("sa1_fps", "sa1_bq_bin") if args.bq_main else ("sa1_fps", "sa1_ball_query")
    if args.l1_side:
        side += ("sa2_fps", "sa2_ball_query")
    main = {k: v for k, v in kern.items() if k not in side}
    side_ms = sum(kern.get(k, 0) for k in side) / args.depth
    dom = max(main, key=lambda k: main[k])
    chains = {"side_ms_per_group": side_ms, "main_ms_per_group": sum(main.values()),
              "bound_by": "side (SA1 FPS latency)" if side_ms > sum(main.values()) else "main (MFMA levels)",
              "sa1_fps_us_per_step": kern.get("sa1_fps", 0) * 1e3 / max(1, N // 16)}

    def roof(name):
        bound, per_frame = work[name]
        per_launch = per_frame * B * args.fps_group  # one launch covers a group of batches
        avg_s = kern[name] / 1e3
        if bound == "mfma":
            # with x3 on, the grouped SA kernels AND the dense GEMMs (SA2's per-point layer 1,
            # group_all's three layers: dense_x3p) issue 3 bf16 MFMA products per fp32 product
            x3k = x3_opt and name in ("sa1_group_mlp", "sa2_group_mlp", "sa2_layer1_points",
                                      "sa3_dense1", "sa3_dense2", "sa3_dense3_pool")
            a, p, u = per_launch / avg_s / 1e12, X3_PEAK_TFLOPS if x3k else FP32_MFMA_PEAK_TFLOPS, "TFLOP/s"
        else:
            a, p, u = per_launch / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
        return {"kernel": name, "bound": bound, "achieved": a, "peak": p, "unit": u, "frac": a / p,
                "traffic": traffic.get(name), "traffic_unit": "bytes per launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
                "work_per_launch": per_launch, "avg_launch_ms": kern[name],
                "peak_basis": ("bf16 MFMA dense peak / 3 (x3: 3 bf16 products per fp32 product)"
                               if bound == "mfma" and p == X3_PEAK_TFLOPS else
                               "fp32 MFMA peak" if bound == "mfma" else "HBM peak")}

    value = sharding.aggregate_rate(B * N * args.steps, world, elapsed) / 1e6
    if rank == 0:
        rec = {
            "metric": "M points/sec through SetAbstraction, 65k-pt frames; 1->8 GPU scaling",
            "value": value, "unit": "M points/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" + (" (MLP products as split-bf16 x3 MFMA products, fp32 accumulation)" if x3_opt else ""),
            "precision": ("fp32 inputs/weights/outputs; SA layers 2-3, SA2's per-point layer 1 and group_all: each "
                          "fp32 operand split exactly into bf16 hi+lo, products ah*bh + ah*bl + al*bh accumulated in "
                          "fp32 (<= ~2^-15 per product); SA1 layer 1 (K = 3) on fp32 MFMA; features within the 1e-4 "
                          "rel contract of the fp32 oracle (tests/test_gpu_tier_n.py::test_group_mlp_x3, "
                          "test_dense_x3s, test_backbone_vs_oracle)") if x3_opt else
                         "fp32 MFMA (v_mfma_f32_*_f32)",
            "data": "synthetic: uniform [-1,1]^3 float32 frames (seeded per rank), random-init SSG weights",
            "config": {"workload": "PointNet++ SSG encoder (SA1 N/16 r0.2 ns32 [64,64,128]; "
                                   "SA2 N/64 r0.4 ns64 [128,128,256]; group_all [256,512,1024]) fp32",
                       "points_per_frame": N, "frames_per_gpu": B, "global_batch_frames": B * world,
                       "parallelism": f"per-frame data parallel x{world} (no collectives)"},
            "roofline": roof(dom),
            # the north_star's MFMA figure: the grouped MLP (SA2 layers 2-3), whatever dominates
            "roofline_grouped_mlp": roof("sa2_group_mlp") if "sa2_group_mlp" in kern else None,
            "roofline_all": {k: roof(k) for k in kern if k in work},
            "kernel_ms": kern,
            "pipeline": {"executor": "pointnet2.StreamingSSG", "side_streams": args.depth,
                         "batches_per_group": args.fps_group, "ball_query_stream": "main" if args.bq_main else "side",
                         **chains},
            "fp32_mfma_kernels": fp32_mfma,
            "other_configs": extras,
            "density_path": density,
            "variant_path": variant,
            "voxel_downsample": voxel,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(N, args.cpu_budget)
            rec["speedup_vs_cpu"] = value / rec["cpu_baseline"]["value"]
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
