"""bench.py's driver-facing output, on CPU: the last stdout line must stay small enough for the
driver's stdout tail (LINE_MAX bytes) and still carry the contract keys, the headline roofline,
the CPU baseline and the distributed record; `--gpus N` outside torch.distributed.run must start
N ranks itself."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (module level imports numpy only)

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "speedup_vs_cpu", "distributed")


def _full_record():
    """The round-3 full record (the 23 KB line the driver could not parse)."""
    with open(os.path.join(REPO, "profiles", "r03", "recheck_bench_final.json")) as f:
        return json.loads(f.readline())


def _with_ranks(rec, world):
    rec = json.loads(json.dumps(rec))
    rec["n_gpus"] = world
    rec["distributed"] = {"backend": "nccl", "world_size": world, "device_count": world,
                          "ranks": [{"rank": r, "device": r, "frames": 640, "ms": 32.948751933872 + r / 7}
                                    for r in range(world)]}
    stats = {"max_rel": 3.1415926e-05, "n_rel": 131000, "n": 131072, "max_tol_ratio": 0.123456789}
    rec["arithmetic_short"] = ("h3: fp32 as fp16 hi+lo on fp16 MFMA (3 products), fp32 accumulate; "
                               "<=1e-4 rel on every element >=1e-2 RMS")
    msg = rec.setdefault("other_configs", {}).setdefault("configs[4]_msg_131k_bf16", {"M_points_per_s": 479.3})
    msg["roofline"] = {"kernel": "sa1_b2_group_mlp", "bound": "mfma", "achieved": 543.0, "peak": 2500.0,
                       "unit": "TFLOP/s", "frac": 0.2172, "traffic": None, "stack_mfma_frac": 0.19,
                       "work_per_launch": 3.75e12, "avg_launch_ms": 6.9, "launches": 6, "frames": 576}
    msg["chains_ms_per_group"] = {"main": 19.87654, "side": 10.34567, "step_ms_per_group": 22.123456}
    rec["ssg_host_feed"] = {"value": 1049.123456, "unit": "M points/s", "ms_per_step": 2.0012345,
                            "long_window": {"batches": 80, "value": 1172.3456}}
    rec["precision"] = {"contract": "max |got-want|/|want| over |want| >= 1e-2 RMS, and max err/(1e-4|want| + "
                                    "1e-4 RMS)", "frames": [0, 31, 64, 127], "fps_exact": True,
                        "per_frame": {str(f): {"level1": 3.1e-05, "level2": 2.9e-05, "global": 3.1e-05}
                                      for f in (0, 31, 64, 127)},
                        "level1": stats, "level2": stats, "global": stats}
    return rec


@pytest.mark.parametrize("world", [1, 2, 8, 16])
def test_compact_line_fits_and_keeps_the_contract(world):
    rec = _with_ranks(_full_record(), world)
    line = bench.compact_line(rec, "gpurun_out/bench_detail.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX, len(text)
    d = json.loads(text)
    for k in CONTRACT:
        assert k in d, k
    assert d["value"] == pytest.approx(rec["value"], rel=1e-3) and d["n_gpus"] == world
    r = d["roofline"]
    for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=2e-3)
    assert d["ssg_host_feed"]["value"] == pytest.approx(1049.123456, rel=1e-3)  # SURVEY §8(d), always kept
    assert d["ssg_host_feed"]["value_80_batches"] == pytest.approx(1172.3, rel=1e-3)
    assert r["achieved"] == pytest.approx(r["work_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=2e-3)
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1 and d["cpu_baseline"]["kind"] == "port"
    assert d["distributed"]["world_size"] == world == len(d["distributed"]["ranks"])
    assert d["precision"]["global"]["max_rel"] == pytest.approx(3.142e-05)
    assert d["precision"]["frames"] == [0, 31, 64, 127] and "per_frame" not in d["precision"]
    # the line says what "f32" means, where ball_query stands against north_star's HBM target, and
    # prices the configs[4] MSG leg's dominant kernel on the bf16 peak
    assert d["arithmetic"].startswith("h3: fp32 as fp16 hi+lo")
    bq = d["ball_query_hbm"]
    assert bq["target"] == 0.5 and bq["met"] is False and 0 < bq["frac_compulsory"] < 0.5
    # north_star's MFMA figure is on the line whichever kernel dominates the window (the fused SA1 kernel and
    # the SA2 grouped MLP tie within box noise; SA1's time includes its ball queries, said in a note)
    if rec.get("roofline_grouped_mlp"):
        g = d["roofline_grouped_mlp"]
        assert g["kernel"] == "sa2_group_mlp" and 0 < g["frac"] < 1
    rec2 = json.loads(json.dumps(rec))
    rec2["roofline"]["kernel"] = "sa1_group_mlp"
    assert "ball queries" in bench.compact_line(rec2)["roofline"]["note"]
    if world <= 8:  # the optional parts survive at the driver's world sizes
        assert "legs_M_points_per_s" in d and "kernels" in d and d["detail"] == "gpurun_out/bench_detail.json"
        r = d["roofline_configs[4]"]
        assert r["kernel"] == "sa1_b2_group_mlp" and r["peak"] == 2500.0 and r["frac"] == pytest.approx(0.2172)


def test_compact_line_drops_optional_parts_last_first():
    rec = _with_ranks(_full_record(), 8)
    rec["distributed"]["ranks"] *= 40  # an absurd rank list: the optional parts go, the contract stays
    line = bench.compact_line(rec)
    for k in CONTRACT:
        assert k in line


def test_committed_r04_lines_are_driver_readable():
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r0[4-9]", "*bench*.log")))
    if not files:
        pytest.skip("no committed round-4 bench log")
    for f in files:
        lines = [l for l in open(f).read().splitlines() if l.strip()]
        last = lines[-1]
        assert len(last.encode()) <= bench.LINE_MAX, f"{f}: last line {len(last)} bytes"
        d = json.loads(last)
        for k in CONTRACT:
            assert k in d, f"{f}: {k}"


def test_launch_ranks_starts_n_ranks(tmp_path):
    """--gpus N without WORLD_SIZE: a child torch.distributed.run with N ranks, output relayed,
    exit code returned (a stand-in script: this container has no GPU)."""
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\n"
                      "print('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'], sys.argv[1:], flush=True)\n"
                      "sys.exit(3 if os.environ['RANK'] == '1' and '--fail' in sys.argv else 0)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, sys.argv[1:], script=%r))" % (REPO, str(script)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code, "--x", "1"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = sorted(l for l in r.stdout.splitlines() if l.startswith("rank"))
    assert got == ["rank 0 of 2 ['--x', '1']", "rank 1 of 2 ['--x', '1']"]
    r = subprocess.run([sys.executable, "-c", code, "--fail"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=60, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
