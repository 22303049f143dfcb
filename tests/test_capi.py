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


def _header_decls():
    """(name -> (return C type, [argument C types])) for every cvl_* function in the header."""
    hdr = open(os.path.join(ROOT, "include", "cvlite.h")).read()
    hdr = re.sub(r"/\*.*?\*/", " ", hdr, flags=re.S)
    hdr = re.sub(r"//[^\n]*", " ", hdr)
    out = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_ \*]*?)\b(cvl_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", hdr):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        ret = ret.split("\n")[-1].strip()
        argl = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        types = []
        for a in argl:
            a = " ".join(a.split())
            if "*" in a:
                types.append("ptr")
            else:
                types.append(" ".join(a.split(" ")[:-1]).replace("const ", ""))
        out[name] = ("ptr" if "*" in ret else ret.replace("const ", "").strip(), types)
    return out


def test_ctypes_signatures_match_header_types():
    """Every argument and return type in _lib.SIGNATURES agrees with the C declaration (an
    int / int64 / size_t / float / double / pointer drift fails here, not on the GPU)."""
    import ctypes
    from cvlite import _lib
    cmap = {"int": ctypes.c_int, "int32_t": ctypes.c_int, "int64_t": ctypes.c_int64, "long": ctypes.c_long,
            "size_t": ctypes.c_size_t, "float": ctypes.c_float, "double": ctypes.c_double,
            "cvl_stream_t": ctypes.c_void_p, "ptr": ctypes.c_void_p}
    decls = _header_decls()
    assert set(decls) == set(_lib.SIGNATURES), sorted(set(decls) ^ set(_lib.SIGNATURES))
    for name, (ret, args) in decls.items():
        res, argt = _lib.SIGNATURES[name]
        exp_args = [cmap[a] for a in args]
        assert len(argt) == len(exp_args), (name, len(argt), len(exp_args))
        for i, (got, exp) in enumerate(zip(argt, exp_args)):
            assert ctypes.sizeof(got) == ctypes.sizeof(exp) and (got is exp or (
                issubclass(got, ctypes._SimpleCData) and got._type_ == exp._type_)), (name, i, got, exp)
        if ret == "ptr":
            assert res in (ctypes.c_void_p, ctypes.c_char_p), (name, res)
        else:
            assert res is cmap[ret] or res._type_ == cmap[ret]._type_, (name, res, ret)


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


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of the header's structs (cvl_conv_desc incl. the parity-mode `prec`
    field, cvl_conv_seg, cvl_pack_item, cvl_bias_item) have the C layout: sizes and the offsets
    of every field, as gcc lays out include/cvlite.h."""
    import ctypes
    import shutil
    import subprocess
    from cvlite import ops_nn as nn
    if shutil.which("gcc") is None:
        import pytest
        pytest.skip("no gcc")
    checks = [("cvl_conv_desc", nn.ConvDesc), ("cvl_conv_seg", nn.ConvSeg), ("cvl_pack_item", nn.PackItem),
              ("cvl_bias_item", nn.BiasItem)]
    lines = []
    for cname, cls in checks:
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\nint main(void){%s return 0;}\n'
                   % (os.path.join(ROOT, "include", "cvlite.h"), "\n".join(lines)))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I/opt/rocm/include", str(src), "-o", str(exe)])
    got = dict(ln.rsplit(" ", 1) for ln in subprocess.check_output([str(exe)], text=True).splitlines())
    for cname, cls in checks:
        assert int(got["%s size" % cname]) == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert int(got["%s.%s" % (cname, f[0])]) == getattr(cls, f[0]).offset, (cname, f[0])


def test_bias_grad_plan_workspace_sizes():
    """The bias-gradient partial-row plan (host code, nn_ops.hip bias_multi_plan): chunks of
    >= 4 rounds of 8 rows per thread, <= 256 partial rows per item, never across an image; the
    workspace is one fp32 row of round_up(ncol, 8) per partial row.  Invalid items size to 0."""
    from cvlite import _lib
    from cvlite import ops_nn as nn
    lib = _lib.load()
    ws = lambda ncol, HW, B: int(lib.cvl_bias_grad_workspace_size(ncol, HW, B))
    # FPN level 0 at 512 / bs 16: 8 rows per pass, 64-row rounds -> 256-row chunks, 16 per image
    assert ws(256, 4096, 16) == 4 * 256 * 256
    # FCOS cls head (20 -> 24 columns, 4 threads per row, 64 rows per pass): 2048-row chunks
    assert ws(20, 4096, 16) == 4 * (16 * 2) * 24
    # the 256-partial-row cap: chunks grow beyond the minimum for large levels
    assert ws(256, 16384, 16) == 4 * (16 * 16) * 256
    # single-row images: one chunk per image
    assert ws(516, 1, 3) == 4 * 3 * 520
    assert ws(0, 10, 1) == 0 and ws(8, 0, 1) == 0
    arr = (nn.BiasItem * 2)()
    for i in range(2):
        arr[i] = nn.BiasItem(16, 16, 0, 4096, 256, 0, 256, 4096, 16, 0.0)
    assert int(lib.cvl_bias_grad_multi_workspace_size(arr, 2)) == 2 * 4 * 256 * 256
    arr[1] = nn.BiasItem(16, 16, 0, 4096, 256, 8, 256, 4096, 16, 0.0)      # coff + 256 > ld
    assert int(lib.cvl_bias_grad_multi_workspace_size(arr, 2)) == 0
