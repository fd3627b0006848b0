"""Capture golden results of the desktop loader by running the REFERENCE itself (this container).

Writes every ``loader_cases`` file into a temporary directory, loads it with
``windows_implementation/core/data_loader.py``'s ``DataLoader().load_file`` (imported read-only
from /root/reference), and records per case either the points (sha256 of the bytes, shape, dtype)
plus the metadata (``file_path`` dropped), or the exception's type and message. Output:
``loader.json``. Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_loader.py
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
sys.path.insert(0, "/root/reference/windows_implementation/core")

import loader_cases  # noqa: E402
from data_loader import DataLoader  # noqa: E402


def record(ds):
    a = np.ascontiguousarray(ds.points)
    meta = {k: v for k, v in ds.metadata.items() if k != "file_path"}
    return {"ok": True, "sha256": hashlib.sha256(a.tobytes()).hexdigest(), "shape": list(a.shape),
            "dtype": str(a.dtype), "metadata": json.loads(json.dumps(meta, default=str))}


def main():
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name in loader_cases.NAMES:
            fname, data = loader_cases.build(name)
            path = os.path.join(d, name + "_" + fname)
            with open(path, "wb") as f:
                f.write(data)
            try:
                out[name] = record(DataLoader().load_file(path))
            except Exception as e:  # noqa: BLE001 — the exception IS the expected result
                out[name] = {"ok": False, "type": type(e).__name__, "message": str(e)}
    with open(os.path.join(HERE, "loader.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{len(out)} cases -> loader.json")


if __name__ == "__main__":
    main()
