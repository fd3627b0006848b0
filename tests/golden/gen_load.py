"""Capture golden results of ``load_lidar_data`` by running the REFERENCE itself (this container).

Writes every ``load_cases`` file into a temporary directory, loads it with the reference's
``utils/data_processing.load_lidar_data`` (:8-125, imported read-only from /root/reference) and
records per case either the points (sha256 of the bytes, shape, dtype) or the exception's type and
message.  Output: ``load.json``.  Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_load.py
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference")

import load_cases  # noqa: E402
from utils.data_processing import load_lidar_data  # noqa: E402


def main():
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name in load_cases.NAMES:
            fname, data = load_cases.build(name)
            path = os.path.join(d, name + "_" + fname)
            with open(path, "wb") as f:
                f.write(data)
            try:
                a = np.ascontiguousarray(load_lidar_data(path))
                out[name] = {"ok": True, "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
                             "shape": list(a.shape), "dtype": str(a.dtype)}
            except Exception as e:  # noqa: BLE001 — the exception IS the expected result
                out[name] = {"ok": False, "type": type(e).__name__,
                             "message": str(e).replace(path, "<path>")}
            print(name, out[name].get("shape", out[name].get("message")))
    with open(os.path.join(HERE, "load.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{len(out)} cases -> load.json")


if __name__ == "__main__":
    main()
