"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol
``include/lidar_amd.h`` declares (no GPU needed — nothing is launched), the host-side
weight packer is deterministic, and the product package never imports the oracle."""
import os
import re
import subprocess

import pytest

from lidar_ai_recommendation_software_amd import _native as nat

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "lidar_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lidar_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = nat.load_library()
    missing = [s for s in declared_symbols() if getattr(lib, s, None) is None]
    assert not missing, f"declared in include/lidar_amd.h but not exported: {missing}"
    assert len(declared_symbols()) >= 15


def test_abi_version_matches_integration_doc():
    # a host call (no GPU needed); INTEGRATION.md lists what changed in this version
    v = nat.load_library().lidar_version()
    assert v == 5
    assert f"### ABI version {v} (`lidar_version() == {v}`" in open(os.path.join(REPO, "INTEGRATION.md")).read()


def test_binding_covers_header():
    assert sorted(nat.SIGNATURES) == declared_symbols()


def test_exported_symbols_are_c_abi():
    out = subprocess.check_output(["nm", "-D", "--defined-only", nat.LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for s in declared_symbols():
        assert s in exported, s  # unmangled extern "C"


def test_library_is_gfx950_only():
    # the target string embedded in the fat binary's code objects
    data = open(nat.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "lidar_ai_recommendation_software_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f


def test_errors_without_gpu_are_loud():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(nat.NativeUnavailable):
        nat.handle(0)


def test_pack_is_deterministic_and_sized():
    import numpy as np
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    w = pn.init_weights(pn.SSG, 0)
    a = pn.pack_branch_x3(w[1][0], False)
    b = pn.pack_branch_x3(w[1][0], False)
    assert np.array_equal(a, b)
    assert a.size == nat.load_library().lidar_mlp_packed_size_x3(0, 128, 128, 256)
    assert pn.pack_branch16(w[0][0], True).size * 4 >= nat.load_library().lidar_mlp_packed_size16(1, 64, 64, 128)


def test_invalid_arguments_return_einval():
    lib = nat.load_library()
    rc = lib.lidar_mlp_pack_x3_f32(1, 64, 64, 128, None, None, None, None, None, None, None)
    assert rc == -1 and b"null" in lib.lidar_last_error()
    rc = lib.lidar_profile(None, 1)
    assert rc == -1 and b"null handle" in lib.lidar_last_error()
    assert lib.lidar_gather_rows(None, None, 0, 0, None, 0, None, None) == -1
    import ctypes
    nx, ny = nat.I64(), nat.I64()
    assert lib.lidar_grid_dims(0.0, 1.0, 0.0, 1.0, -1.0, ctypes.byref(nx), ctypes.byref(ny)) == -1
