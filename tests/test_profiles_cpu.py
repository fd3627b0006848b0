"""The committed profiles reproduce the bench: every kernel the rocprofv3 summaries of the bench
name has a label in tools/pmc_traffic.py (so its PMC traffic and VALU figures can be attributed),
and the committed PMC reductions were taken on pipeline launches of the bench's own shape."""
import csv
import glob
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pmc_traffic  # noqa: E402


def _latest(pattern):
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", pattern)))
    return files[-1] if files else None


@pytest.mark.parametrize("pattern", ["*rocprof_kernel_stats_bench.csv"])
def test_every_bench_kernel_has_a_label(pattern):
    f = _latest(pattern)
    if f is None:
        pytest.skip("no committed rocprof summary")
    names = [r["Name"] for r in csv.DictReader(open(f))]
    assert names
    missing = [n for n in names if pmc_traffic.label(n) is None]
    assert not missing, f"{os.path.relpath(f, REPO)}: kernels without a label: {missing}"


def test_headline_kernel_labels():
    # the north_star's grouped MLP (the lean SA2 kernel, PFX on) and the SA1 fused kernel
    assert pmc_traffic.label("void (anonymous namespace)::sa_x3_lean_kernel<128, 128, 256, 64, true>(float const*)") \
        == "sa2_group_mlp"
    assert pmc_traffic.label("void (anonymous namespace)::sa_x3_kernel<64, 64, 128, 32, 0, 2, false, true>(float)") \
        == "sa1_group_mlp"
    assert pmc_traffic.label("void (anonymous namespace)::fps_bucket_kernel<512, 2, false>(float const*)") == "sa1_fps"


def test_pmc_reductions_are_per_pipeline_launch():
    f = _latest("pmc_traffic.json")
    if f is None:
        pytest.skip("no committed PMC reduction")
    d = json.load(open(f))
    F = d["config"]["frames_per_launch"]
    assert F == 128, "PMC taken at the driver's shape (--steps 20: G = 4 batches of 32 frames)"
    for k in ("sa1_fps", "sa2_group_mlp", "sa1_group_mlp"):
        v = d["kernels"][k]
        assert v["traffic_bytes"] > 0 and abs(v["traffic_per_frame"] * F - v["traffic_bytes"]) < 1e-3 * v["traffic_bytes"]
    v = json.load(open(_latest("pmc_valu.json")))
    assert v["config"]["frames_per_launch"] == F and v["kernels"]["sa2_group_mlp"]["valu_issue_frac"] is not None


def _bench_lines():
    out = []
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r03", "*bench*.json"))):
        line = open(f).readline().strip()
        if line.startswith("{"):
            out.append((os.path.relpath(f, REPO), json.loads(line)))
    return out


def test_committed_bench_lines_keep_the_contract():
    # every committed bench line carries the driver's keys, a self-consistent roofline for the
    # dominant kernel, the 1-rank CPU baseline and the distributed record of the ranks it saw
    lines = _bench_lines()
    if not lines:
        pytest.skip("no committed bench line")
    for name, d in lines:
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "dtype", "data", "config", "roofline", "cpu_baseline"):
            assert k in d, f"{name}: missing {k}"
        r = d["roofline"]
        assert r["kernel"] == "sa2_group_mlp" and r["bound"] == "mfma"
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
        assert abs(r["achieved"] - r["work_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12) < 1e-6 * r["achieved"]
        assert 0 < r["frac"] < 1
        if "distributed" in d:
            dist = d["distributed"]
            assert dist["world_size"] == d["n_gpus"] == len(dist["ranks"])
            if d["cpu_baseline"] is not None:
                assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
