"""Build libnconv.so in-tree for gfx950 (hipcc, no torch involvement).

    python realtime-depth-estimation-nconv_amd/build.py [--force]

Each csrc/*.hip is compiled to an object next to the library (parallel, incremental on mtime,
headers included), then linked into realtime-depth-estimation-nconv_amd/libnconv.so. The .so is
git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libnconv.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("NCONV_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-Wall",
          "-Wno-unused-function"]


def _newest_dep():
    deps = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(p) for p in deps), default=0.0)


def _compile(src, force, dep_mtime):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), dep_mtime):
        return obj, None
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    dep = _newest_dep()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        results = list(ex.map(lambda s: _compile(s, force, dep), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("libnconv build failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"libnconv link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[nconv] built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
