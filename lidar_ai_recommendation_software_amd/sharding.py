"""Per-frame data parallelism: one process per GPU, frames sharded across ranks.

Frames are independent through the whole path (preprocess -> DBSCAN -> people ->
density grid, and the SetAbstraction stack), so N GPUs shard the frame stream with no
collective on the data path.  The only collectives are the timing
barrier and the MAX-over-ranks of the elapsed time, which `timed` performs on whatever
process group is initialised: RCCL ("nccl") on the GPU box, gloo in the CPU tests.
"""
import os
import time

import torch
import torch.distributed as dist


def world_info():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_frames, rank, world):
    """Contiguous, balanced frame range [lo, hi) of `rank`; the ranges of all ranks are
    disjoint and cover 0..n_frames-1 (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    q, r = divmod(int(n_frames), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def frame_seed(rank, step=0, base=0):
    """Seed of the synthetic frame batch a rank processes (distinct per rank)."""
    return base + 1_000_003 * step + rank


def timed(run, device=None, world=1):
    """Barrier + device sync, run(), device sync + barrier; returns the elapsed wall
    time MAXED over ranks (the whole job finishes when the slowest rank does)."""
    return timed_detail(run, device, world)[0]


def _host_collectives(device):
    """True when the process group reduces host tensors (gloo: the CPU tests, or ranks sharing
    one GPU), False for RCCL, which reduces device tensors."""
    return not (device is not None and device.type == "cuda" and dist.get_backend() == "nccl")


def timed_detail(run, device=None, world=1):
    """`timed`, returning (max-over-ranks elapsed, this rank's own elapsed)."""
    cuda = device is not None and device.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(device)

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run()
    sync()
    if world > 1:
        dist.barrier()
    local = elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if _host_collectives(device) else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, local


def group_report(device, world, frames, elapsed_local):
    """What the process group saw, for the bench line: the backend, the world size, the GPUs this
    node exposes, and every rank's (device index, frames processed, own elapsed ms), gathered with
    one all_gather over the group (the reporting path, not the data path).  With world 1 no
    collective runs."""
    ndev = torch.cuda.device_count()
    dev_idx = device.index if device is not None and device.type == "cuda" else -1
    mine = [float(dist.get_rank() if world > 1 else 0), float(dev_idx), float(frames), elapsed_local * 1e3]
    if world > 1:
        t = torch.tensor(mine, dtype=torch.float64, device="cpu" if _host_collectives(device) else device)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rows = [p.cpu().tolist() for p in parts]
        backend, ws = dist.get_backend(), dist.get_world_size()
    else:
        rows, backend, ws = [mine], None, 1
    return {"backend": backend, "world_size": ws, "device_count": ndev,
            "ranks": [{"rank": int(r[0]), "device": int(r[1]), "frames": int(r[2]), "ms": r[3]} for r in rows]}


def local_world():
    """Ranks on this node (torch.distributed.run's LOCAL_WORLD_SIZE; WORLD_SIZE when unset)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))


def check_backend(world, backend, device_count, local=None):
    """One process per GPU must talk RCCL: a multi-rank run whose node has at least as many visible
    GPUs as ranks on it, but ended up on another backend, is a misconfiguration (init_distributed
    picks gloo only when ranks on a node share a GPU).  The comparison is per node, so a 16-rank
    job over two 8-GPU nodes is held to RCCL as well."""
    local = local_world() if local is None else local
    if world > 1 and local <= device_count and backend != "nccl":
        raise RuntimeError(f"{local} ranks per node over {device_count} GPUs must use RCCL ('nccl'), got {backend!r}")


def init_distributed(world, local):
    """One process per GPU (torch.distributed.run).  Returns the local device index.  Ranks that
    share a GPU (more ranks on this node than visible devices: a rehearsal of the N-GPU path on a 1-GPU box)
    use gloo for the timing collectives; otherwise RCCL ("nccl") over xGMI.  Counting devices
    does not initialise the GPU, so this runs before any GPU call."""
    ndev = max(1, torch.cuda.device_count())
    dev = local % ndev
    if world > 1:
        if local_world() > ndev:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    return dev


def aggregate_rate(units_per_rank, world, elapsed):
    """Whole-job throughput: units processed by ALL ranks / the max-over-ranks time."""
    return units_per_rank * world / elapsed
