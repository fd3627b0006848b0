"""Known-byte copy for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on this box.

Runs a 1 GiB -> 1 GiB device copy (torch's elementwise copy kernel: 16-B vector loads
and stores) 4 times; each launch moves exactly 2^30 bytes in and 2^30 bytes out, well
past the 256 MiB Infinity Cache.  tools/pmc_traffic.py divides the counters of that
kernel by 2^30 to get the scale factors applied to the SA-stack kernels."""
import torch

x = torch.rand(1 << 28, device="cuda")  # 1 GiB of float32
y = torch.empty_like(x)
for _ in range(4):
    y.copy_(x)
torch.cuda.synchronize()
print("calib ok", float(y[123]))
