"""CPU: a non-Python host compiled against include/nconv.h agrees with the ctypes binding.

tests/host/capi_host.c is built with gcc against the public header and linked to libnconv.so. It
reports sizeof/offsetof of every ABI struct field, which must equal the ctypes structures of
realtime-depth-estimation-nconv_amd/_lib.py (so header, binding and INTEGRATION.md cannot drift
apart silently), and makes host-validated calls that must return -EINVAL with a message."""
import ctypes
import json
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def host_report(nconv_amd, tmp_path_factory):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    lib = nconv_amd._lib.LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("libnconv.so not built")
    exe = str(tmp_path_factory.mktemp("host") / "capi_host")
    libdir = os.path.dirname(lib)
    subprocess.run([gcc, "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "host", "capi_host.c"), "-o", exe, lib,
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    r = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120)
    return json.loads(r.stdout)


def _ctypes_layout(struct):
    out = {struct.__name__: [0, ctypes.sizeof(struct)]}
    for name, _ in struct._fields_:
        f = getattr(struct, name)
        out[f"{struct.__name__}.{name}"] = [f.offset, f.size]
    return out


@pytest.mark.parametrize("c_name,py_name", [("nconv_src", "NconvSrc"), ("nconv_layer", "NconvLayer"),
                                            ("nconv_dense_conv", "NconvDenseConv"),
                                            ("nconv_dense_wgrad", "NconvDenseWgrad"),
                                            ("nconv_bwd_io", "NconvBwdIo"),
                                            ("nconv_bn_train", "NconvBnTrain")])
def test_struct_layout_matches_ctypes(nconv_amd, host_report, c_name, py_name):
    py = _ctypes_layout(getattr(nconv_amd._lib, py_name))
    c = {k.replace(c_name, py_name, 1): v for k, v in host_report.items() if k == c_name or k.startswith(c_name + ".")}
    assert c == py


def test_host_validation_and_abi(host_report):
    assert host_report["abi"][0] == host_report["abi"][1]
    for key, msg in (("rc_bad_ho", "Ho/Wo inconsistent"), ("rc_bad_math", "unknown math"),
                     ("rc_bad_mode", "unknown load mode")):
        rc, err = host_report[key]
        assert rc == -22 and msg in err, (key, rc, err)
    assert host_report["bwd_ws_ok"][0] > 0
    # zero-initialised math: NCONV_MATH_FP32, VALU forward / input gradient, fp32-MFMA weight gradient
    assert host_report["plan_zero"] == [0, 1, 1, 1, 2]


def test_integration_doc_binding_matches_ctypes(nconv_amd):
    """The ctypes NconvLayer / NconvSrc field lists shown in INTEGRATION.md §4 equal the binding's."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for cls in ("NconvSrc", "NconvLayer"):
        m = re.search(r"class %s\(ctypes\.Structure\):\s*_fields_ = \[(.*?)\]\n" % cls, doc, re.S)
        assert m, f"INTEGRATION.md has no {cls} binding"
        names = re.findall(r'\("(\w+)"', m.group(1))
        assert names == [n for n, _ in getattr(nconv_amd._lib, cls)._fields_], cls
