"""bench.py's density-path leg alone (no CPU baseline), printed as one JSON line: phase times per
launch, 32-frame / lanes / 256-frame rates.  usage: python tools/tier_r_leg.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

rec = bench.tier_r_leg(torch.device("cuda:0"), 0, 1, cpu=False)
print(json.dumps({"value": rec["value"], "phase_ms_per_launch": rec["phase_ms_per_launch"],
                  "pipelined": rec.get("pipelined_batches", {}).get("value"),
                  "wide": rec.get("wide_batch", {}).get("value")}))
