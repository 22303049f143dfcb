"""The C-ABI library loads and exports every symbol include/cvlite.h declares (CPU; no compute)."""
import os
import re

from conftest import ROOT


def test_library_exports_header_symbols():
    from cvlite import _lib
    hdr = open(os.path.join(ROOT, "include", "cvlite.h")).read()
    names = set(re.findall(r"\b(cvl_[a-z0-9_]+)\s*\(", hdr))
    assert names, "no declarations parsed"
    lib = _lib.load()
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert set(_lib.SIGNATURES) == names, sorted(set(_lib.SIGNATURES) ^ names)
    assert lib.cvl_version() >= 100


def test_no_cpu_fallback_in_product_path():
    """Without a GPU every cvlite op raises (there is no CPU fallback on the product path)."""
    import numpy as np
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the loud-failure path is for CPU-only hosts")
    from cvlite import _lib
    from cvlite.retinanet import RetinaNet
    from cvlite import fcos
    net = RetinaNet(80, {})
    with pytest.raises(_lib.CvlError):
        net.cpu_nms(np.zeros((3, 6), np.float32), 0.5)
    with pytest.raises(_lib.CvlError):
        net.prediction_to_corners(np.zeros((4, 4, 4), np.float32), net.anchor_boxes[0][0], 8)
    with pytest.raises(_lib.CvlError):
        fcos.prediction_to_corners(np.zeros((4, 4, 4), np.float32), 8)
