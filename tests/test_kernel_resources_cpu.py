"""Kernel resource metadata of the built gfx950 code objects (CPU; no GPU needed).

Every csrc/*.hip object in the package's _build/ carries its device code object in .hip_fatbin;
the AMDGPU metadata notes give each kernel's scratch size and spill counts. A hot kernel that
suddenly needs scratch is a regression the GPU suite's numerics cannot see (this round's training
head went from 262 to 696 us when the compiler stopped inlining a lambda: 240 B/lane of scratch and
waterfall loops around its stores), so scratch is allowed only in the listed opt-in kernels.
"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "realtime-depth-estimation-nconv_amd", "_build")
LLVM = "/opt/rocm/lib/llvm/bin"
# opt-in bf16 matrix-core forward of the pooled down layers (NCONV_MATH_BF16X9 / BF16X3)
SCRATCH_ALLOWED = ("fwd_mfmaILi8ELi5ELi2E",)


def _kernels(obj, tmp):
    fat, co = os.path.join(tmp, "f.bin"), os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                       capture_output=True, text=True)
    if r.returncode != 0:  # an object without device code (host-only source)
        return {}
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    out, name = {}, None
    for line in notes.splitlines():
        m = re.search(r"\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
            out.setdefault(name, {})
        m = re.search(r"\.(private_segment_fixed_size|sgpr_spill_count|vgpr_spill_count):\s+(\d+)", line)
        if m and name:
            out[name][m.group(1)] = int(m.group(2))
    return out


@pytest.mark.skipif(not glob.glob(os.path.join(BUILD, "*.o")) or not shutil.which(f"{LLVM}/llvm-readelf"),
                    reason="needs the built objects (build.py) and the ROCm llvm tools")
def test_no_scratch_outside_opt_in_kernels(tmp_path):
    seen, bad = 0, []
    for obj in sorted(glob.glob(os.path.join(BUILD, "*.hip.o"))):
        for name, md in _kernels(obj, str(tmp_path)).items():
            if not name.startswith("_Z"):
                continue
            seen += 1
            if md.get("private_segment_fixed_size", 0) > 0 and not any(a in name for a in SCRATCH_ALLOWED):
                bad.append((os.path.basename(obj), name, md))
    assert seen > 50, seen
    assert not bad, bad


@pytest.mark.skipif(not glob.glob(os.path.join(BUILD, "*.o")) or not shutil.which(f"{LLVM}/llvm-readelf"),
                    reason="needs the built objects (build.py) and the ROCm llvm tools")
def test_exact_head_has_no_scratch_and_few_spills(tmp_path):
    md = _kernels(os.path.join(BUILD, "nconv_fwd_head.hip.o"), str(tmp_path))
    heads = {k: v for k, v in md.items() if "fwd_head_exact" in k}
    assert len(heads) == 2, list(md)
    for k, v in heads.items():
        assert v.get("private_segment_fixed_size", 0) == 0, (k, v)
        assert v.get("vgpr_spill_count", 0) == 0, (k, v)
        assert v.get("sgpr_spill_count", 0) <= 24, (k, v)


def _kernel_blocks(obj, tmp):
    """{kernel name: {field: int}} from the code object's metadata, split per kernel entry (fields
    that sort before .name, such as .group_segment_fixed_size, stay with their own kernel)."""
    fat, co = os.path.join(tmp, "f.bin"), os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.agpr_count", notes):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if m:
            out[m.group(1)] = {k: int(v) for k, v in re.findall(r"\.(\w+):\s+(\d+)\s*$", blk, re.M)}
    return out


@pytest.mark.skipif(not glob.glob(os.path.join(BUILD, "*.o")) or not shutil.which(f"{LLVM}/llvm-readelf"),
                    reason="needs the built objects (build.py) and the ROCm llvm tools")
def test_training_input_gradients_occupancy(tmp_path):
    """nconv2's input gradient (dgrad_tiled, pooled stager + fused nconv1 weight gradient) at five
    waves per SIMD and the tail's (dgrad_phase) at six: the one-plane-ahead stagers' register budgets
    and the head epilogue's halved LDS (profiles/r5_ab_dgrad_occupancy.log,
    r5_ab_dgrad_phase_one_ahead.log). A change that pushes them back to four waves shows here."""
    md = _kernel_blocks(os.path.join(BUILD, "nconv_bwd.hip.o"), str(tmp_path))
    head = [v for k, v in md.items() if "dgrad_tiledILi8ELi8ELi5ELi0ELb1ELb1E" in k]
    phase = [v for k, v in md.items() if "dgrad_phaseILi4ELb1E" in k]
    assert len(head) == 1 and len(phase) == 1, sorted(md)
    assert head[0]["vgpr_count"] <= 96 and head[0]["group_segment_fixed_size"] <= 160 * 1024 // 5, head[0]
    assert phase[0]["vgpr_count"] <= 80 and phase[0]["group_segment_fixed_size"] <= 160 * 1024 // 6, phase[0]
    for v in head + phase:
        assert v.get("private_segment_fixed_size", 0) == 0, v
