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
    elapsed = time.perf_counter() - t0
    if world > 1:
        # RCCL reduces device tensors; gloo (the CPU tests, or ranks sharing one GPU) host ones
        on_dev = cuda and dist.get_backend() == "nccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def init_distributed(world, local):
    """One process per GPU (torch.distributed.run).  Returns the local device index.  Ranks that
    share a GPU (more ranks than visible devices: a rehearsal of the N-GPU path on a 1-GPU box)
    use gloo for the timing collectives; otherwise RCCL ("nccl") over xGMI.  Counting devices
    does not initialise the GPU, so this runs before any GPU call."""
    ndev = max(1, torch.cuda.device_count())
    dev = local % ndev
    if world > 1:
        if world > ndev:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    return dev


def aggregate_rate(units_per_rank, world, elapsed):
    """Whole-job throughput: units processed by ALL ranks / the max-over-ranks time."""
    return units_per_rank * world / elapsed
