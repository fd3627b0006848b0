"""World-size-2 gloo coverage of the N>1 path (no GPU).

The multi-GPU design is per-frame data parallelism: ranks take
disjoint frame shards and share nothing on the data path; bench.py's only collectives
are the timing barrier and the MAX-over-ranks all-reduce (`sharding.timed`).  These
tests run exactly that bookkeeping over gloo with two CPU processes, and check that
sharded per-frame processing gives the single-process results frame for frame.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lidar_ai_recommendation_software_amd import sharding


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, _ = sharding.world_info()
    assert (r, w) == (rank, world)
    # timing: rank 1 is slower; every rank must report the slowest rank's time
    delay = 0.05 + 0.25 * rank
    elapsed = sharding.timed(lambda: time.sleep(delay), None, world)
    # data path: this rank's frames, processed independently (oracle Tier R, CPU)
    from oracle import tier_r
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    lo, hi = sharding.shard(n_frames, rank, world)
    res = {}
    for f in range(lo, hi):
        pts = uniform_frame(1024, seed=sharding.frame_seed(0, base=f))
        pd = tier_r.preprocess_lidar_data(pts)
        res[f] = (pd["clusters"], tier_r.extract_people_positions(pd))
    shards = [None] * world
    dist.all_gather_object(shards, (lo, hi))  # test-only check of coverage
    np.save(os.path.join(out_dir, f"rank{rank}.npy"),
            np.array([elapsed, *[x for s in shards for x in s]], dtype=np.float64))
    np.savez(os.path.join(out_dir, f"res{rank}.npz"),
             **{f"c{f}": v[0] for f, v in res.items()}, **{f"p{f}": v[1] for f, v in res.items()})
    dist.destroy_process_group()


def test_shard_partition_is_disjoint_and_complete():
    for n in (0, 1, 7, 32, 256, 1001):
        for world in (1, 2, 3, 8):
            ranges = [sharding.shard(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [hi - lo for lo, hi in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        sharding.shard(10, 2, 2)


def test_aggregate_rate_is_whole_job():
    assert sharding.aggregate_rate(32 * 65536, 8, 2.0) == 32 * 65536 * 8 / 2.0


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_world2_timing_and_sharded_frames(tmp_path, world):
    n_frames = 5  # world 4: ragged shards (2/1/1/1)
    port = _free_port()
    mp.spawn(_worker, args=(world, port, n_frames, str(tmp_path)), nprocs=world, join=True)
    recs = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    # every rank reports the MAX elapsed (>= the slowest rank's 0.05 + 0.25 (world - 1) s sleep)
    assert all(rec[0] == recs[0][0] for rec in recs) and recs[0][0] >= 0.05 + 0.25 * (world - 1)
    # gathered shard table: disjoint, complete
    table = recs[0][1:].reshape(world, 2).astype(int)
    assert table[0, 0] == 0 and table[-1, 1] == n_frames
    assert all(table[r, 1] == table[r + 1, 0] for r in range(world - 1))
    # per-frame results from the sharded run equal the single-process run
    from oracle import tier_r
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    got = {}
    for r in range(world):
        with np.load(tmp_path / f"res{r}.npz") as z:
            got.update({k: z[k] for k in z.files})
    assert len(got) == 2 * n_frames
    for f in range(n_frames):
        pd = tier_r.preprocess_lidar_data(uniform_frame(1024, seed=sharding.frame_seed(0, base=f)))
        np.testing.assert_array_equal(got[f"c{f}"], pd["clusters"])
        np.testing.assert_array_equal(got[f"p{f}"], tier_r.extract_people_positions(pd))


def _venue_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import tier_r
    from lidar_ai_recommendation_software_amd.global_density import VenueGrid
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    xr, yr = (-15.0, 15.0), (-15.0, 15.0)
    vg = VenueGrid(xr, yr, 1.0, device="cpu")
    # this rank's people (the GPU path bins them with lidar_venue_counts_f64; here the oracle's
    # histogram of the same edges stands in, the collective is what is under test)
    people = uniform_frame(200 + 50 * rank, seed=40 + rank)[:, :2]
    h = tier_r.calculate_grid_density(people, xr, yr, 1.0)[2]
    vg.counts += torch.from_numpy(h.astype(np.int32))
    vg.all_reduce()
    np.save(os.path.join(out_dir, f"venue{rank}.npy"), vg.density())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_world2_venue_grid_all_reduce(tmp_path, world):
    """SURVEY §8e's optional global density: per-rank venue counts summed by one all_reduce
    (RCCL on the GPU box; gloo here) equal the grid density of all ranks' people together.
    World 4 rehearses more ranks than one GPU box holds (the driver's 8-GPU node runs RCCL)."""
    from oracle import tier_r
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    mp.spawn(_venue_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    allp = np.concatenate([uniform_frame(200 + 50 * r, seed=40 + r)[:, :2] for r in range(world)])
    want = tier_r.calculate_grid_density(allp, (-15.0, 15.0), (-15.0, 15.0), 1.0)[2]
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"venue{r}.npy"), want)


def _report_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    el, local = sharding.timed_detail(lambda: time.sleep(0.05 + 0.2 * rank), None, world)
    rep = sharding.group_report(None, world, 32 * (rank + 1), local)
    np.save(os.path.join(out_dir, f"rep{rank}.npy"),
            np.array([el, local] + [v for r in rep["ranks"] for v in (r["rank"], r["frames"], r["ms"])]
                     + [rep["world_size"], float(rep["backend"] == "gloo")], dtype=np.float64))
    dist.destroy_process_group()


def test_gloo_world2_group_report(tmp_path):
    """bench.py's `distributed` record: every rank's frames and own window time, gathered over the
    group, the backend and world size the group reports; the max equals the slowest rank's time."""
    world = 2
    mp.spawn(_report_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    recs = [np.load(tmp_path / f"rep{r}.npy") for r in range(world)]
    for rec in recs:
        el, local = rec[0], rec[1]
        rows = rec[2:2 + 3 * world].reshape(world, 3)
        assert list(rows[:, 0]) == [0, 1] and list(rows[:, 1]) == [32, 64]
        assert el == recs[0][0] and abs(el * 1e3 - rows[:, 2].max()) < 1e-6 and local <= el
        assert rec[-2] == world and rec[-1] == 1.0
    assert recs[1][1] >= 0.25


def test_check_backend_rules():
    sharding.check_backend(1, None, 1, local=1)          # one rank: nothing to check
    sharding.check_backend(8, "nccl", 8, local=8)        # one rank per GPU over RCCL
    sharding.check_backend(2, "gloo", 1, local=2)        # two ranks sharing one GPU: gloo by design
    with pytest.raises(RuntimeError):
        sharding.check_backend(8, "gloo", 8, local=8)    # a GPU per rank but not RCCL
    with pytest.raises(RuntimeError):
        sharding.check_backend(16, "gloo", 8, local=8)   # two 8-GPU nodes, 8 ranks each: RCCL
    sharding.check_backend(16, "gloo", 8, local=16)      # 16 ranks on one 8-GPU node share GPUs


def test_local_world_from_env(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert sharding.local_world() == 8
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert sharding.local_world() == 16
