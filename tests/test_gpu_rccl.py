"""The RCCL branch of the optional global density (`global_density.VenueGrid.all_reduce`)
executed on the GPU: a one-rank "nccl" process group (RCCL needs a device per rank, and the box has
one) runs the product's `all_reduce(int32, SUM)` on the device counts, which must leave them equal to
`calculate_grid_density` of the same people, bit for bit.  The rank runs in a child process so the
test runner's own process never holds a process group; the multi-rank reduction itself is covered
by the gloo world-2/4 tests (tests/test_distributed_cpu.py) and runs over RCCL in the driver's
8-GPU run, whose bench line records the backend and the ranks it saw."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import tier_r

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from lidar_ai_recommendation_software_amd.global_density import VenueGrid
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
people = np.load(sys.argv[2])
vg = VenueGrid((-15.0, 15.0), (-15.0, 15.0), 1.0).add(people)
before = vg.counts.clone()
vg.all_reduce()
torch.cuda.synchronize()
assert VenueGrid.backend() == "nccl" and dist.get_world_size() == 1
assert torch.equal(before, vg.counts)
np.save(sys.argv[3], vg.density())
dist.destroy_process_group()
print("rccl ok", flush=True)
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_venue_grid_rccl_all_reduce_one_rank(tmp_path):
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    people = np.concatenate([uniform_frame(300 + 40 * r, seed=70 + r)[:, :2] for r in range(3)])
    np.save(tmp_path / "people.npy", people)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "-c", CHILD, REPO, str(tmp_path / "people.npy"),
                          str(tmp_path / "density.npy")], env=env, cwd=REPO, capture_output=True, text=True,
                         timeout=180)
    assert out.returncode == 0 and "rccl ok" in out.stdout, out.stdout[-2000:] + out.stderr[-4000:]
    want = tier_r.calculate_grid_density(people, (-15.0, 15.0), (-15.0, 15.0), 1.0)[2]
    assert np.array_equal(np.load(tmp_path / "density.npy"), want)
