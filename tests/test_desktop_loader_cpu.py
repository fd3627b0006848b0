"""desktop_loader.DataLoader against the REFERENCE's desktop loader
(windows_implementation/core/data_loader.py), pinned by tests/golden/loader.json, which
tests/golden/gen_loader.py captured by running the reference on the files that
tests/golden/loader_cases.py builds. The cases are ASCII PCD / PLY (C parser and Python
fallbacks), binary PCD / PLY rejection, LAS (record cap, short final record, bad signature,
truncated header), LAZ, XYZ delimiters and CSV column rules. Host code only: no GPU."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from lidar_ai_recommendation_software_amd import desktop_loader as dl

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import loader_cases  # noqa: E402

with open(os.path.join(HERE, "golden", "loader.json")) as _f:
    GOLD = json.load(_f)


def test_every_case_has_a_fixture():
    assert sorted(GOLD) == loader_cases.NAMES


@pytest.mark.parametrize("name", loader_cases.NAMES)
def test_desktop_loader_matches_reference(tmp_path, name):
    fname, data = loader_cases.build(name)
    path = str(tmp_path / (name + "_" + fname))
    with open(path, "wb") as f:
        f.write(data)
    want = GOLD[name]
    if not want["ok"]:
        with pytest.raises(Exception) as ei:
            dl.DataLoader().load_file(path)
        assert type(ei.value).__name__ == want["type"]
        assert str(ei.value) == want["message"]
        return
    ds = dl.DataLoader().load_file(path)
    a = np.ascontiguousarray(ds.points)
    assert list(a.shape) == want["shape"] and str(a.dtype) == want["dtype"]
    assert hashlib.sha256(a.tobytes()).hexdigest() == want["sha256"]
    assert ds.metadata.pop("file_path") == path
    assert json.loads(json.dumps(ds.metadata, default=str)) == want["metadata"]


def test_missing_file_raises_file_not_found(tmp_path):
    with pytest.raises(FileNotFoundError, match="File not found"):
        dl.DataLoader().load_file(str(tmp_path / "absent.pcd"))


def test_large_ascii_sections_take_the_c_parser(tmp_path, monkeypatch):
    """The 65 536-row PCD must come from lidar_parse_ascii_xyz, not the Python loop."""
    fname, data = loader_cases.build("pcd_ascii_65536")
    path = str(tmp_path / fname)
    with open(path, "wb") as f:
        f.write(data)

    def boom(_lines):
        raise AssertionError("python fallback used")

    monkeypatch.setattr(dl, "_rows_skipping", boom)
    ds = dl.DataLoader().load_file(path)
    assert ds.points.shape == (65536, 3)
