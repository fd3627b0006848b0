"""Capture golden vectors for the flow model by running the REFERENCE itself (this container).

``models/crowd_flow_model.py`` imports (numpy, scikit-learn, scipy) from ``/root/reference``
read-only.  Two kinds of cases:

* frames: the reference's ``preprocess_lidar_data`` -> ``CrowdFlowModel().analyze`` on
  seeded synthetic frames (``analyze`` end to end, people positions included);
* extents: ``_generate_simulated_flow`` + ``_identify_bottlenecks`` on processed-data dicts
  holding only ``dimensions`` (the only key they read), over varied scene extents — small,
  large, offset, fractional — so the flow field and the KD-tree neighbourhoods see many
  grids.

Writes ``flow.json`` (sha256 of the arrays, float.hex scalars, directions, bottlenecks, the
RNG state digest after the call).  Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_flow.py
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, "/root/reference")

from utils.data_processing import preprocess_lidar_data  # noqa: E402
from models.crowd_flow_model import CrowdFlowModel  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import crowd_frame, blob_frame, lattice_frame  # noqa: E402


def sha(a):
    a = np.ascontiguousarray(a)
    return {"sha256": hashlib.sha256(a.tobytes()).hexdigest(), "shape": list(a.shape), "dtype": str(a.dtype)}


def fhex(v):
    return float(v).hex()


def rng_digest():
    st = np.random.get_state()
    return hashlib.sha256(st[1].tobytes() + str(st[2]).encode()).hexdigest()


def flow_entry(fv):
    return {"positions": sha(fv["positions"]), "vectors": sha(fv["vectors"]), "magnitudes": sha(fv["magnitudes"])}


def bn_entry(bs):
    return [[fhex(b["x"]), fhex(b["y"]), int(b["severity"]), type(b["severity"]).__name__] for b in bs]


FRAMES = {
    "crowd_10000_s42": lambda: crowd_frame(10000, 42),
    "crowd_16384_s7": lambda: crowd_frame(16384, 7),
    "crowd_65536_s3": lambda: crowd_frame(65536, 3),
    "blobs_8980_s1": lambda: blob_frame(200, 40, 500, 1, 15, 0.3),
    "lattice_8163_s4": lambda: lattice_frame(4, 120, 60, 4, 15, 0.4),
}


def extents():
    rng = np.random.default_rng(2024)
    out = {"square_30": (-15.0, 15.0, -15.0, 15.0), "narrow": (0.0, 1.5, -3.0, 20.0),
           "tiny": (2.0, 2.4, 5.0, 5.3), "wide_60x40": (-30.2, 29.9, -20.1, 19.7),
           "offset": (100.25, 131.75, -250.5, -219.0), "integer_edges": (-12.0, 12.0, -8.0, 8.0)}
    for i in range(14):
        x0, y0 = rng.uniform(-40, 40, 2)
        w, h = rng.uniform(0.5, 45, 2)
        out[f"random_{i}"] = (x0, x0 + w, y0, y0 + h)
    return out


def main():
    import scipy
    import sklearn
    meta = {"generator": "tests/golden/gen_flow.py", "numpy": np.__version__, "sklearn": sklearn.__version__,
            "scipy": scipy.__version__, "frames": {}, "extents": {}}
    for name, make in FRAMES.items():
        pd = preprocess_lidar_data(make())
        res = CrowdFlowModel().analyze(pd)
        meta["frames"][name] = {"flow": flow_entry(res["flow_vectors"]), "avg_speed": fhex(res["avg_speed"]),
                                "avg_speed_type": type(res["avg_speed"]).__name__,
                                "dominant_direction": res["dominant_direction"],
                                "bottlenecks": bn_entry(res["bottlenecks"]), "rng_after": rng_digest()}
        print(name, res["dominant_direction"], len(res["bottlenecks"]), flush=True)
    for name, (x0, x1, y0, y1) in extents().items():
        pd = {"dimensions": {"x_range": (np.float64(x0), np.float64(x1)), "y_range": (np.float64(y0), np.float64(y1))}}
        model = CrowdFlowModel()
        fv = model._generate_simulated_flow(np.zeros((1, 2)), pd)
        bs = model._identify_bottlenecks(fv, pd)
        meta["extents"][name] = {"range": [fhex(v) for v in (x0, x1, y0, y1)], "flow": flow_entry(fv),
                                 "bottlenecks": bn_entry(bs), "rng_after": rng_digest()}
        print(name, len(fv["positions"]), "nodes", len(bs), "bottlenecks", flush=True)
    with open(os.path.join(HERE, "flow.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
