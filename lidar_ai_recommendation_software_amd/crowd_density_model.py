"""Drop-in for the reference's ``models/crowd_density_model.py`` on MI355X.

``CrowdDensityModel(grid_size=1.0).analyze(processed_data)`` returns the reference's
result dict (``models/crowd_density_model.py:23-98``) bit for bit: people positions,
density grid, statistics and hotspots come from the gfx950 kernels behind
``data_processing.extract_people_positions`` / ``lidar_density_grid_f64`` (the numpy
pairwise mean of the occupied cells and the stable top-5 ordering are restated on the
device).  The optional ``backbone`` ("ssg" / "msg") adds a PointNet++ global feature of
the frame, computed with ``backbone_weights`` when given (trained weights: the
nested [level][branch][layer] = (W, b) lists of ``pointnet2.init_weights``'s layout, or an ``.npz``
written by ``pointnet2.save_weights``) and with the deterministic random init otherwise; the result
says which (``backbone_weights``: "supplied" / "random-init").  The default ``None`` keeps the
reference behaviour exactly.
"""
import numpy as np

from . import data_processing as dp


class CrowdDensityModel:
    """Model for analyzing crowd density from LiDAR point cloud data."""

    def __init__(self, grid_size=1.0, backbone=None, backbone_weights=None):
        """grid_size as the reference (models/crowd_density_model.py:14-22); backbone None / "ssg" / "msg";
        backbone_weights: the backbone's weights (validated against its configuration here, so a
        mismatched set fails at construction), or None for the seed-0 random init."""
        self.grid_size = grid_size
        self.backbone = backbone
        self._net = None
        self._weights = None
        if backbone_weights is not None:
            from . import pointnet2 as pn
            if backbone is None:
                raise ValueError("backbone_weights given without a backbone")
            cfg = pn.CONFIGS[backbone]
            if isinstance(backbone_weights, (str, bytes)) or hasattr(backbone_weights, "__fspath__"):
                self._weights = pn.load_weights(backbone_weights, cfg)
            else:
                self._weights = pn.check_weights(cfg, backbone_weights)

    def analyze(self, processed_data):
        people = dp.extract_people_positions(processed_data)
        if len(people) == 0:
            return {
                "total_people": 0,
                "avg_density": 0.0,
                "max_density": 0.0,
                "density_map": np.zeros((1, 1)),
                "grid_coordinates": (np.array([0]), np.array([0])),
                "density_values": np.array([0]),
                "hotspots": [],
            }
        dims = processed_data["dimensions"]
        gx, gy, dens, flat_x, flat_y, stats, hot = dp._grid(people, dims["x_range"], dims["y_range"],
                                                            self.grid_size)
        flat = dens.flatten()
        hotspots = [{"x": flat_x[i], "y": flat_y[i], "density": flat[i]} for i in hot]
        res = {
            "total_people": len(people),
            "avg_density": np.float64(stats[1]),
            "max_density": np.float64(stats[0]),
            "density_map": dens,
            "grid_coordinates": (flat_x, flat_y),
            "density_values": flat,
            "hotspots": hotspots,
        }
        if self.backbone is not None:
            res["backbone_feature"] = self.encode(processed_data["points"])
            res["backbone_weights"] = "supplied" if self._weights is not None else "random-init"
        return res

    @staticmethod
    def normalise(points):
        """The backbone's input: the frame centred on its bounding box and scaled so that the
        box's longest side spans [-1, 1] (fp32; the SA radii 0.2 / 0.4 are in these units)."""
        p = np.asarray(points, dtype=np.float64)
        lo, hi = p.min(axis=0), p.max(axis=0)
        return ((p - (lo + hi) / 2) / max(float((hi - lo).max()) / 2, 1e-9)).astype(np.float32)

    def encode(self, points):
        """PointNet++ (SSG/MSG) global feature of one frame over ALL its points (1 <= N <= 4 194 304:
        the FPS kernel's limit, lidar_fps_ex_f32; frames above 262 144 points run it on buckets of
        64 x PPL points; a larger frame raises LidarError naming the limit).  SA levels take
        max(1, N/16) and max(1, N/64) centres.  Not part of the reference."""
        import torch
        from . import pointnet2 as pn
        if self._net is None:
            self._net = pn.PointNet2Backbone(pn.CONFIGS[self.backbone], weights=self._weights, device="cuda")
        unit = self.normalise(points)
        g, _ = self._net.forward(torch.from_numpy(np.ascontiguousarray(unit))[None].cuda())
        return g[0].cpu().numpy()

    def calculate_risk_level(self, density):
        """models/crowd_density_model.py:100-117."""
        if density < 1.0:
            return "Low"
        elif density < 2.5:
            return "Moderate"
        elif density < 4.0:
            return "High"
        else:
            return "Critical"
