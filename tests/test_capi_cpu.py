"""CPU: the C-ABI library builds, loads after torch, and exports every entry point include/nconv.h
declares with the declared ABI version; descriptor validation rejects malformed calls before any
launch (no GPU needed: validation happens on the host)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nconv.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(nconv_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points(nconv_amd):
    assert set(header_functions()) == set(nconv_amd._lib.EXPORTED)


def test_library_exports_all_symbols(nconv_amd):
    lib = nconv_amd._lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), f"libnconv.so does not export {name}"
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_abi_version_matches_header(nconv_amd):
    v = int(re.search(r"#define NCONV_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert nconv_amd._lib.lib().nconv_abi_version() == v == nconv_amd._lib.ABI_VERSION


def _layer(nconv_amd, **kw):
    L = nconv_amd._lib.NconvLayer()
    L.B, L.Cin, L.H, L.W, L.Cout, L.Ho, L.Wo = 1, 8, 16, 16, 8, 16, 16
    L.KH = L.KW = 5
    L.SH = L.SW = L.DH = L.DW = L.groups = 1
    L.PH = L.PW = 2
    L.eps = 1e-7
    L.load_mode = nconv_amd._lib.PLAIN
    fake = 0x1000  # never dereferenced: validation fails or passes on the host first
    L.a.x, L.a.c, L.a.C, L.a.H, L.a.W = fake, fake, 8, 16, 16
    L.weight = L.bias = L.wsum = fake
    for k, v in kw.items():
        setattr(L, k, v)
    return L


@pytest.mark.parametrize("bad,msg", [
    (dict(Ho=15), "Ho/Wo inconsistent"),
    (dict(groups=3), "groups"),
    (dict(load_mode=9), "unknown load mode"),
    (dict(Cin=4), "PLAIN"),
    (dict(weight=None), "null weight"),
])
def test_fwd_rejects_bad_descriptors(nconv_amd, bad, msg):
    lib = nconv_amd._lib.lib()
    L = _layer(nconv_amd, **bad)
    rc = lib.nconv_fwd(ctypes.byref(L), ctypes.c_void_p(0x2000), ctypes.c_void_p(0x3000), None)
    assert rc == -22
    assert msg in lib.nconv_last_error().decode()


def test_bwd_workspace_query_is_host_only(nconv_amd):
    lib = nconv_amd._lib.lib()
    L = _layer(nconv_amd)
    assert lib.nconv_bwd_workspace_bytes(ctypes.byref(L)) > 0
    bad = _layer(nconv_amd, Ho=3)
    assert lib.nconv_bwd_workspace_bytes(ctypes.byref(bad)) == 0


def test_product_path_refuses_cpu_tensors(nconv_amd):
    """No CPU fallback: the NConv modules compute only on the ROCm device and say so."""
    import torch
    net = nconv_amd.SETP1_NCONV()
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        net(torch.zeros(1, 1, 16, 16))
    layer = nconv_amd.NConv2d(8, 8, (5, 5))
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        layer(torch.zeros(1, 8, 8, 8), torch.zeros(1, 8, 8, 8))
