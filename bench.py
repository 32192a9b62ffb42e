#!/usr/bin/env python3
"""Benchmark of the NConv depth-completion hot path on MI355X.

Headline (BASELINE.json metric, config 2): frames/sec of the unguided NConv U-Net (DNET /
SETP1_NCONV, models/step1.py:15-94) forward on B=8 synthetic KITTI-shaped 352x1216 sparse depth
per GPU, inputs resident in HBM, computed in EXACT fp32 (every product an fp32 product, as the
reference's F.conv2d; include/nconv.h NCONV_MATH_FP32). Also on the same JSON line:
  fwd_bf16x3         the same forward with split-bf16 matrix-core products (NCONV_MATH_BF16X3,
                     <= ~1.1e-5 relative per product: narrower than fp32, reported separately)
  config5            B=16 1024x2048 forward (BASELINE configs[4]), both arithmetics, own roofline
  train_fwd_bwd_adamw  config 4b: EnforcePos drift + calculate_loss on the whole batch
                     (train_step1.py:63) + backward + AdamW, hipGraph-replayed, with its roofline
  guided_fwd / guided_train_fwd_bwd_adamw  configs 3 / 4 with their fraction of the fp32 MFMA peak
                     in reference flops, under the default dense math (bf16x9: exact products on
                     the bf16 matrix cores) and, in other_dense_math, the fp32-MFMA and bf16x6 ones
  layer_us / roofline  per-kernel device time of the headline forward and the roofline of its
                     dominant kernel (HIP events on the launch stream; profiles/ has the rocprofv3
                     summary of the same command)
  cpu_baseline       the oracle (the reference's op sequence) on this host's cores: the config-2
                     workload (B=8, generalized crop) and config 1 (3-layer forward, B=1)

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 8] [--height 352] [--width 1216]
    torchrun --nproc-per-node N bench.py --gpus N ...      # one process per GPU, RCCL

`--gpus N` without a launcher (no WORLD_SIZE in the environment) starts the N rank processes
itself (launch_ranks: one child per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1
set, before this process touches the GPU) and exits with their status; N greater than the visible
devices is an error. Under torchrun, --gpus must equal WORLD_SIZE.

Multi-GPU: frames are independent units, so each rank runs its own B frames (weak scaling) with
no collective in the forward; the training step all-reduces gradients over RCCL (one bucket).
"""
import argparse
import faulthandler
import json
import os
import socket
import subprocess
import sys
import time

faulthandler.enable()  # a host fault (SIGSEGV / SIGABRT) leaves every thread's Python stack on stderr

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, chip-level parameters (spec)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 matrix peak (no sparsity)
FP32_PEAK_TFLOPS = 157.3        # FP32 vector = FP32 matrix peak (same table)
PASS_BYTES_PER_FRAME = 238.44e6  # fused per-layer forward, 352x1216
PASS_FLOPS_PER_FRAME = 6.620e9
BWD_BYTES_PER_FRAME = 373.9e6    # SURVEY.md 8(d) backward estimate, 352x1216
BWD_FLOPS_PER_FRAME = 12.79e9
GUIDED_DENSE_FLOPS_PER_FRAME = 133.6e9  # RGB encoder 7.94 + fusion decoder 125.69 GFLOP
MATH_DTYPE = {"fp32": "fp32", "bf16x9": "fp32", "bf16x3": "fp32 io and accumulation, bf16x3 products"}
MATH_ARITH = {
    "fp32": "exact fp32: every product an fp32 fmaf product on the vector ALU, fp32 accumulation (NCONV_MATH_FP32)",
    "bf16x9": "exact products: both operands split into three bf16 parts (an exact decomposition), all nine "
              "partial products (each exact in fp32) accumulated in fp32 on the matrix cores; nconv7 and "
              "non-DNET shapes on the vector ALU (NCONV_MATH_BF16X9)",
    "bf16x3": "8-channel layers' products as two-part split-bf16 matrix-core terms (<= ~1.1e-5 relative per "
              "product, inside the 1e-4 forward tolerance; narrower than fp32) (NCONV_MATH_BF16X3)"}
LAYERS = ("nconv1", "nconv2", "nconv_down1", "nconv_down2", "nconv_down3", "nconv4", "nconv5", "nconv6", "nconv7")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (= rank processes, one per GPU); default: WORLD_SIZE under a launcher, else 1")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--height", type=int, default=352)
    p.add_argument("--width", type=int, default=1216)
    p.add_argument("--train-steps", type=int, default=None, help="timed fwd+bwd steps (default: --steps)")
    p.add_argument("--no-train", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--math", default="fp32", choices=("fp32", "bf16x9", "bf16x3"),
                   help="forward arithmetic of the headline (include/nconv.h enum nconv_math)")
    p.add_argument("--alt-math", default="bf16x9,bf16x3", type=lambda v: [x for x in v.split(",") if x],
                   help="other arithmetics measured beside the headline (comma list; '' for none)")
    p.add_argument("--no-config5", action="store_true", help="skip the B=16 1024x2048 forward (config 5)")
    p.add_argument("--no-guided", action="store_true", help="skip the config-3 guided forward measurement")
    p.add_argument("--no-guided-train", action="store_true", help="skip the config-4 guided training step")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU time of each CPU-baseline sample")
    p.add_argument("--graph", type=int, default=1, help="capture the forward in a hipGraph (1) or run eager (0)")
    p.add_argument("--fused-head", type=int, default=1, help="nconv1 inside nconv2's kernel (nconv_fwd_head)")
    p.add_argument("--inference-streams", type=int, default=None,
                   help="DNET.inference_streams: batch slices on that many streams (default: the module's)")
    p.add_argument("--inference-shares", default=None, type=_shares,
                   help="DNET.inference_shares: relative frames per inference stream, e.g. 5,3 (one positive "
                        "number per stream of --inference-streams, default 2)")
    p.add_argument("--guided-alt-math", default="fp32,bf16x6", type=lambda v: [x for x in v.split(",") if x],
                   help="also time configs 3 / 4 (graphed) with these dense maths (separately labelled)")
    p.add_argument("--guided-train-graph", type=int, default=1,
                   help="replay the config-4 guided training step from a hipGraph (1) or eager (0)")
    p.add_argument("--head-density", type=float, default=0.40,
                   help="also time the forward's kernels at this depth density (0: skip); the headline is 5 %%")
    p.add_argument("--train-graph", type=int, default=1,
                   help="replay the training step from a hipGraph (1, every world size: the RCCL all-reduce is "
                        "captured in the graph) or eager (0); on one GPU the eager step is reported beside it")
    a = p.parse_args(argv)
    if a.inference_shares is not None and len(a.inference_shares) != (a.inference_streams or 2):
        p.error(f"--inference-shares has {len(a.inference_shares)} entries for {a.inference_streams or 2} "
                "inference streams")
    return a


def _shares(v):
    """--inference-shares: comma list of positive finite numbers."""
    try:
        sh = [float(x) for x in v.split(",")]
    except ValueError:
        raise argparse.ArgumentTypeError(f"not a comma list of numbers: {v!r}")
    if not sh or not all(x > 0 and x != float("inf") for x in sh):
        raise argparse.ArgumentTypeError(f"shares must be positive and finite: {v!r}")
    return sh


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv, device_count=None, script=None, poll_s=0.2):
    """Start n rank processes of `script` (default: this file) with `argv`, one per GPU, as
    torch.distributed.run would (RANK = LOCAL_RANK = r, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1, a free
    MASTER_PORT), wait for them and return the exit status (the first failing rank's; the others are
    then terminated, so no rank waits forever in a collective). This parent may load the HIP
    runtime to count devices (torch.cuda.device_count() falls back to hipGetDeviceCount on builds
    without amdsmi) but never launches a kernel and is never re-exec'd: the ranks are fresh child
    processes started with Popen."""
    ndev = torch.cuda.device_count() if device_count is None else device_count
    if n > ndev:
        raise SystemExit(f"bench.py: --gpus {n} but only {ndev} GPU(s) are visible")
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    status = 0
    while True:
        codes = [p.poll() for p in procs]  # (every child polled each round)
        if all(c is not None for c in codes):
            break
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            status = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            break
        time.sleep(poll_s)
    for p in procs:
        rc = p.wait()
        if rc and not status:
            status = rc
    return status if status >= 0 else 128 - status


def log(*msg):
    """Progress on stderr (a long silent run looks hung to the GPU harness)."""
    print("[bench]", *msg, file=sys.stderr, flush=True)


def sparse_depth(g, B, H, W, device, density=0.05):
    d = torch.rand(B, 1, H, W, generator=g) * 79 + 1
    d = d * (torch.rand(B, 1, H, W, generator=g) < density)
    return d.to(device)


WARMUP_MIN_S = 0.2  # untimed warm-up per leg: at least --warmup calls and at least this long


def warm_up(fn, min_calls, min_seconds=WARMUP_MIN_S):
    """Run fn() at least min_calls times and until min_seconds of device time have passed (synchronised
    every call after the first few, so the clock is real). A box whose clocks ramp up under load
    reaches its steady state before the timed region. Returns (calls, seconds)."""
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        if n >= min_calls:
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            if el >= min_seconds:
                return n, el


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_state(dev):
    """The clock / power state the box exposes for this GPU through sysfs (amdgpu: pp_dpm_sclk /
    pp_dpm_mclk current level -- the line marked '*' --, hwmon power cap / average power / edge
    temperature), or None where it is not readable (a container may hide /sys/class/drm)."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    except Exception:  # noqa: BLE001 -- an informational field only
        bus = None
    base = None
    if bus is not None:
        for cand in (f"/sys/bus/pci/devices/{bus}.0",):
            if os.path.isdir(cand):
                base = cand
    if base is None:
        return None
    st = {"pci": bus}
    for key in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk"):
        txt = _read(os.path.join(base, key))
        if txt:
            cur = [ln.split(":", 1)[1].strip(" *") for ln in txt.splitlines() if ln.rstrip().endswith("*")]
            st[key] = cur[0] if cur else txt.splitlines()[-1]
    st["power_dpm_force_performance_level"] = _read(os.path.join(base, "power_dpm_force_performance_level"))
    try:
        hw = os.path.join(base, "hwmon")
        hw = os.path.join(hw, sorted(os.listdir(hw))[0])
        for key, name, scale in (("power1_cap", "power_cap_w", 1e-6), ("power1_average", "power_avg_w", 1e-6),
                                 ("power1_input", "power_w", 1e-6), ("temp1_input", "temp_edge_c", 1e-3),
                                 ("freq1_input", "sclk_hz", 1.0)):
            v = _read(os.path.join(hw, key))
            if v is not None:
                st[name] = round(float(v) * scale, 1)
    except (OSError, IndexError, ValueError):
        pass
    return st


# ---- algorithmic cost per kernel -------------------------------------------------
def kernel_costs(B, H, W):
    """(bytes, flops) per launch of each kernel of the inference forward. Bytes: the kernel's
    sources read once at their native resolution and its outputs written once (including the
    2x2 max-pooled copies the pooled launches write for the next down layer); fp32, 4 B.
    Flops: 2 convolutions x 2 flop/FMA x Cin k^2 Cout per output pixel, + 4 Cout (div, bias, conf).
    Per unit (one output pixel of the layer): nconv1 68 B / 832 flop; nconv2 (pooled) 144 B /
    6432; head (nconv1+2, pooled) 84 B / 7264; down1/down2 (pooled) 144 B / 6432; down3 128 B /
    6432; nconv4/5 64 B + 64 B per skip / low-res source pixel / 4640; tail 64 B per nconv2 pixel
    + 64 B per nconv5 pixel + 4 B output / 4640 (nconv6) + 36 (nconv7)."""
    f4 = 4
    H2, W2, H4, W4, H8, W8, H16, W16 = H // 2, W // 2, H // 4, W // 4, H // 8, W // 8, H // 16, W // 16
    px = lambda h, w: B * h * w
    F5, F3 = 2 * 2 * 8 * 25 * 8 + 32, 2 * 2 * 16 * 9 * 8 + 32
    c = {
        "nconv1": (px(H, W) * (1 + 16) * f4, px(H, W) * (2 * 2 * 1 * 25 * 8 + 32)),
        "nconv2": (px(H, W) * (16 + 16 + 4) * f4, px(H, W) * F5),
        "nconv1+nconv2_head": (px(H, W) * (1 + 16 + 4) * f4, px(H, W) * (F5 + 2 * 2 * 25 * 8 + 32)),
        "nconv_down1": (px(H2, W2) * (16 + 16 + 4) * f4, px(H2, W2) * F5),
        "nconv_down2": (px(H4, W4) * (16 + 16 + 4) * f4, px(H4, W4) * F5),
        "nconv_down3": (px(H8, W8) * (16 + 16) * f4, px(H8, W8) * F5),
        "nconv4": ((px(H4, W4) * 32 + px(H8, W8) * 16) * f4, px(H4, W4) * F3),
        "nconv5": ((px(H2, W2) * 32 + px(H4, W4) * 16) * f4, px(H2, W2) * F3),
        "nconv6+7_tail": ((px(H, W) * (16 + 1) + px(H2, W2) * 16) * f4,
                          px(H - 2, W - 2) * F3 + px(H + 2, W + 2) * (2 * 2 * 8 + 4)),
    }
    del H16, W16
    return c


def inference_calls(m, net, S):
    """The inference forward's launches, one callable each (same kernels and order as
    DNET._infer), for per-kernel timing."""
    lib = m._lib
    d = net.d_net
    layers = [getattr(d, n) for n in LAYERS]
    wsum = d._prologue(layers, S)
    l1, l2, d1, d2, d3, l4, l5, l6, l7 = layers
    s1, s2, sd1, sd2, sd3, s4, s5, s6, s7 = wsum
    fwd, fpool, fhead = m.nconv.layer_forward_raw, m.nconv.layer_forward_pooled, m.nconv.layer_forward_head
    H, W = S.shape[2], S.shape[3]
    oh, ow = m.crop_hw(H, W, d.crop)
    head = d._use_head(l1, l2)
    wph = d._phase_weights(S.device)
    w4, w5, w6 = (None, None, None) if wph is None else tuple(wph)
    w21 = None
    if head and m.nconv.FORWARD_MATH == lib.MATH_FP32:
        w21 = m.nconv.head_weights(l1.spec(lib.THRESH, 0.01), l2.spec(), S, l1.weight, l1.bias, s1, l2.weight,
                                   l2.bias, s2)
    with torch.no_grad():
        if head:
            x1b, c1b, p1, q1 = fhead(l1.spec(lib.THRESH, 0.01), l2.spec(), S, l1.weight, l1.bias, s1, l2.weight,
                                     l2.bias, s2, w21)
        else:
            x1, c1 = fwd(l1.spec(lib.THRESH, 0.01), S, None, None, None, l1.weight, l1.bias, s1)
            x1b, c1b, p1, q1 = fpool(l2.spec(), x1, c1, None, None, l2.weight, l2.bias, s2)
        x2, c2, p2, q2 = fpool(d1.spec(), p1, q1, None, None, d1.weight, d1.bias, sd1)
        x3, c3, p3, q3 = fpool(d2.spec(), p2, q2, None, None, d2.weight, d2.bias, sd2)
        x4, c4 = fwd(d3.spec(), p3, q3, None, None, d3.weight, d3.bias, sd3)
        x34, c34 = fwd(l4.spec(lib.UPCAT_SKIP_FIRST), x3, c3, x4, c4, l4.weight, l4.bias, s4, wphase=w4)
        x23, c23 = fwd(l5.spec(lib.UPCAT_SKIP_FIRST), x2, c2, x34, c34, l5.weight, l5.bias, s5, wphase=w5)
    tail_out = torch.empty((S.shape[0], 1, oh, ow), device=S.device, dtype=torch.float32)
    first = {"nconv1+nconv2_head": lambda: fhead(l1.spec(lib.THRESH, 0.01), l2.spec(), S, l1.weight, l1.bias, s1,
                                                 l2.weight, l2.bias, s2, w21)} if head else {
        "nconv1": lambda: fwd(l1.spec(lib.THRESH, 0.01), S, None, None, None, l1.weight, l1.bias, s1),
        "nconv2": lambda: fpool(l2.spec(), x1, c1, None, None, l2.weight, l2.bias, s2)}
    return {
        **first,
        "nconv_down1": lambda: fpool(d1.spec(), p1, q1, None, None, d1.weight, d1.bias, sd1),
        "nconv_down2": lambda: fpool(d2.spec(), p2, q2, None, None, d2.weight, d2.bias, sd2),
        "nconv_down3": lambda: fwd(d3.spec(), p3, q3, None, None, d3.weight, d3.bias, sd3),
        "nconv4": lambda: fwd(l4.spec(lib.UPCAT_SKIP_FIRST), x3, c3, x4, c4, l4.weight, l4.bias, s4, wphase=w4),
        "nconv5": lambda: fwd(l5.spec(lib.UPCAT_SKIP_FIRST), x2, c2, x34, c34, l5.weight, l5.bias, s5, wphase=w5),
        "nconv6+7_tail": lambda: d._fused_tail(l6, l7, s6, s7, x1b, c1b, x23, c23, tail_out, w6),
    }


def time_layers(m, net, S, reps=20):
    """Average device time (us) per launch of each kernel of the inference forward: one HIP-event
    pair per launch, recorded on the stream the kernel is launched on. The launches run in the
    forward's own order, pass after pass (not one kernel repeated back to back), so each kernel
    meets the clock and cache state it has inside the real forward."""
    calls = inference_calls(m, net, S)
    stream = torch.cuda.current_stream()
    ev = {name: [] for name in calls}
    with torch.no_grad():
        for fn in calls.values():
            fn()
        for _ in range(reps):
            for name, fn in calls.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                ev[name].append((e0, e1))
    torch.cuda.synchronize()
    return {name: sum(e0.elapsed_time(e1) for e0, e1 in pairs) / len(pairs) * 1e3 for name, pairs in ev.items()}


def time_concurrent_halves(m, net, S, name, reps=20):
    """Device span (us) of kernel `name`'s two B/2 launches run concurrently on two streams -- the
    launch shape the replayed headline graph runs (DNET's two-stream inference split), as opposed to
    time_layers' isolated B launch on one stream: HIP events on the current stream around the fork
    (side stream waits for it), the two launches, and the join."""
    B = S.shape[0]
    if B < 2:
        return None
    h = B // 2
    ca, cb = inference_calls(m, net, S[:h])[name], inference_calls(m, net, S[h:])[name]
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    spans = []
    with torch.no_grad():
        for it in range(reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            side.wait_stream(cur)
            ca()
            with torch.cuda.stream(side):
                cb()
            cur.wait_stream(side)
            e1.record(cur)
            if it >= 2:
                spans.append((e0, e1))
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in spans) / len(spans) * 1e3


def pmc_traffic(kernel, math, B, H, W):
    """HBM bytes per launch of `kernel` from the committed PMC summary (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction), or None if this kernel was not
    measured at this configuration."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if tuple(d.get("config", ())) != (B, H, W):
            return None
        e = d.get("kernels", {}).get(math, {}).get(kernel)
        return e["hbm_bytes_per_launch"] if e else None
    except (ValueError, KeyError, TypeError, AttributeError):
        return None


def sq_exec(kernel, math, B, H, W):
    """The kernel's executed VALU work per launch from the committed SQ counters
    (profiles/sq_exec.json, tools/gpu_runs/r4_sq.sh + tools/sq_report.py), or None."""
    path = os.path.join(ROOT, "profiles", "sq_exec.json")
    try:
        d = json.load(open(path))
        if tuple(d.get("config", ())) != (B, H, W):
            return None
        return d["kernels"][math].get(kernel)
    except (OSError, ValueError, KeyError, TypeError, AttributeError):
        return None


def roofline(layer_us, costs, math, B, H, W, issued_mfma=None):
    """The roofline object of the dominant (longest) kernel of the forward. Its bound is the roof
    its arithmetic intensity (algorithmic flop per algorithmic byte) meets first:
    above the fp32 ridge (157.3 TF/s / 8 TB/s = 19.7 flop/B) the compute roof -- "fp32-valu" for the
    exact-fp32 kernels (packed FP32 FMAs on the vector ALU; its peak equals the dense fp32 matrix
    peak of MI355X_MICROARCH.md and the two do not add, tools/microbench/fp32_rates.hip), "mfma" for
    the bf16x3 / bf16x9 maths -- with achieved = the reference's algorithmic fp32 flops per launch /
    the launch time; below it HBM. Both fractions are reported, and, where the committed SQ
    counters (profiles/sq_exec.json) hold the kernel, the executed rate: the fp32 flops its FMA-class
    VALU instructions actually performed per launch over the same time."""
    dom = max(layer_us, key=lambda n: layer_us[n])
    byt, fl = costs[dom]
    us = layer_us[dom]
    gbs = byt / (us * 1e-6) / 1e9
    tfs = fl / (us * 1e-6) / 1e12
    compute = fl / byt > FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    # the compute roof of the exact-fp32 kernels is the packed-FP32 vector ALU ("fp32-valu"); the
    # bf16x3 / bf16x9 maths run their products on the matrix cores ("mfma")
    r = {"bound": ("fp32-valu" if math == "fp32" else "mfma") if compute else "hbm",
         "achieved": round(tfs, 2) if compute else round(gbs, 1),
         "peak": FP32_PEAK_TFLOPS if compute else HBM_PEAK_GBS,
         "unit": "TFLOP/s" if compute else "GB/s",
         "frac": round(tfs / FP32_PEAK_TFLOPS, 4) if compute else round(gbs / HBM_PEAK_GBS, 4),
         "traffic": pmc_traffic(dom, math, B, H, W),
         "kernel": dom, "kernel_us": round(us, 2), "algorithmic_bytes_per_launch": byt, "flops_per_launch": fl,
         "arithmetic_intensity_flop_per_byte": round(fl / byt, 2),
         "compute_roof": "fp32: packed FMA on the vector ALU (exact products); peak = the dense fp32 MFMA peak, "
                         "which equals the vector peak" if math == "fp32" else f"{math} products on the bf16 matrix cores",
         "hbm_achieved_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
         "fp32_tflops": round(tfs, 2), "fp32_frac": round(tfs / FP32_PEAK_TFLOPS, 4)}
    ex = sq_exec(dom, math, B, H, W)
    if ex:  # what the hardware executed: FMA-class VALU instructions x 64 lanes x 4 flop (packed)
        etf = ex["executed_flops_per_launch"] / (us * 1e-6) / 1e12
        r["executed"] = {"fp32_flops_per_launch": ex["executed_flops_per_launch"], "tflops": round(etf, 2),
                         "frac": round(etf / FP32_PEAK_TFLOPS, 4),
                         "valu_busy_frac": round(ex["valu_cycles_per_simd"] / (us * 1e-6 * 2.4e9), 4),
                         "source": "profiles/sq_exec.json (SQ_INSTS_VALU_FMA_F32, SQ_INSTS_VALU per launch)"}
        if ex.get("mfma_insts_per_launch"):  # the head's exact confidence mass on the bf16 matrix cores
            # v_mfma_f32_16x16x32_bf16: 16384 flop = 16 cycles of one SIMD at the dense bf16 rate
            r["executed"]["bf16_mfma_busy_frac"] = round(
                ex["mfma_insts_per_launch"] * 16 / 1024 / (us * 1e-6 * 2.4e9), 4)
    if issued_mfma:
        r["mfma_issued_bf16_tflops"] = round(issued_mfma(dom) / (us * 1e-6) / 1e12, 2)
        r["mfma_bf16_dense_peak_tflops"] = MFMA_BF16_PEAK_TFLOPS
    return r


# Layers on the matrix-core kernel (fwd_mfma): output rows per tile, k-steps and resolution
MFMA_LAYERS = {"nconv1+nconv2_head": (8, 8, 1), "nconv2": (8, 8, 1), "nconv_down1": (8, 8, 2),
               "nconv_down2": (8, 8, 4), "nconv_down3": (8, 8, 8), "nconv4": (8, 6, 4), "nconv5": (8, 6, 2),
               "nconv6+7_tail": (16, 6, 1)}
# v_mfma_f32_16x16x32_bf16 per {N, D} k-step and per head nconv1 k-step (N terms + D terms)
MFMA_TERMS = {"bf16x3": (6, 5), "bf16x9": (18, 12)}


def mfma_issued_flops(layer, B, H, W, math):
    """bf16 MFMA flops one fwd_mfma launch issues (the split terms per k-step and row pair /
    column half, plus the fused head's nconv1 MFMAs: 3 x 3 blocks x 2 row pairs x 2 k-steps)."""
    if layer not in MFMA_LAYERS or math not in MFMA_TERMS:
        return 0
    th, nt, div = MFMA_LAYERS[layer]
    if math == "bf16x9" and layer == "nconv6+7_tail":
        th = 8
    per_k, head_k = MFMA_TERMS[math]
    h, w = H // div, W // div
    tiles = -(-h // th) * -(-w // 32) * B
    extra = 3 * 3 * 2 * 2 * head_k if layer == "nconv1+nconv2_head" else 0
    return tiles * ((th // 2) * 2 * nt * per_k + extra) * 16384


# ---- CPU baseline ----------------------------------------------------------------------------------
def host_cores():
    """(threads the CPU baseline uses, the machine's physical cores, how the first was found).
    The thread count is what this process can actually run at once: its CPU affinity, capped by
    the cgroup CPU quota when one is set (a GPU box's job may see every CPU of the machine but be
    given a 16-CPU share; oversubscribing torch's thread pool on it is ~30x slower)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    how = "affinity"
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
            if path.endswith("cpu.max"):
                quota, period = txt[0], float(txt[1])
            else:
                quota, period = txt[0], float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if quota != "max" and float(quota) > 0:
                q = max(1, int(float(quota) / period))
                if q < usable:
                    usable, how = q, f"cgroup quota ({path})"
            break
        except (OSError, ValueError, IndexError):
            continue
    phys = None
    try:
        seen = set()
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (s.strip() for s in line.split(":", 1))
                cur[k] = v
            elif cur:
                seen.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            seen.add((cur.get("physical id"), cur.get("core id")))
        phys = len(seen) or None
    except OSError:
        pass
    return usable, phys, how


def cpu_baseline(B, H, W, seconds):
    """The oracle (oracle/nconv_ref.py: the reference's DNET forward restated with the same torch
    CPU ops; bitwise equal to the reference on the same torch build) timed on this host on every
    core this process may use: the config-2 workload (B frames, generalized crop, the GPU's crop),
    and config 1 (nconv1 -> nconv2 -> nconv7, B=1, step1.py:38-39,49)."""
    from oracle import nconv_ref as R
    import nconv_pkg
    m = nconv_pkg.load()
    usable, phys, how = host_cores()
    threads = usable
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = m.SETP1_NCONV()
    params = R.dnet_params_from_state_dict({k: R.softplus_pos(v) if k.endswith(".weight") and "bnorm" not in k
                                            else v for k, v in net.state_dict().items()})
    g = torch.Generator().manual_seed(0)
    S = sparse_depth(g, B, H, W, "cpu")

    def timed(fn, max_n):
        fn()  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= max_n:
                return n, el

    with torch.no_grad():
        n, el = timed(lambda: R.dnet_forward(S, params, "generalized"), 200)
        S1 = S[:1]
        nc = {k: params[k] for k in ("nconv1", "nconv2", "nconv7")}

        def three_layer():
            c0 = (S1 > 0.01).float()
            x, c = R.nconv2d(S1, c0, *nc["nconv1"], (1, 1), (2, 2))
            x, c = R.nconv2d(x, c, *nc["nconv2"], (1, 1), (2, 2))
            return R.nconv2d(x, c, *nc["nconv7"], (1, 1), (2, 2))
        n1, el1 = timed(three_layer, 2000)
    return {"value": round(n * B / el, 3), "unit": "frames/sec", "cores": threads, "kind": "port",
            "physical_cores_on_host": phys, "threads_from": how,
            "sample": f"{n} B={B} {H}x{W} DNET forwards (config-2 workload, generalized crop; "
                      f"oracle/nconv_ref.dnet_forward, fp32, torch CPU, {threads} threads = every CPU this "
                      f"process may run on at once) in {el:.1f} s",
            "config1_3layer_frames_per_sec": round(n1 / el1, 2),
            "config1_sample": f"{n1} single-frame {H}x{W} nconv1->nconv2->nconv7 forwards in {el1:.1f} s"}


# ---- guided configs ---------------------------------------------------------------------------------
# the arithmetic of the guided model's 3x3 stride-1 convolutions (dense.MATH; other kinds: fp32 MFMA)
DENSE_ARITH = {
    "bf16x9": "exact products on the bf16 matrix cores (three-part split operands, all nine partial "
              "products, fp32 accumulation); the 1x1 convolutions fp32 MFMA",
    "fp32": "v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation) for every convolution",
    "bf16x6": "the six largest split-bf16 partial products (each product within ~2^-23 relative), "
              "fp32 accumulation; the 1x1 convolutions fp32 MFMA",
}


def guided_forward(m, dev, B, H, W, steps, warmup, rank):
    """Config 3: SETP2 (RGB-guided, models/step2.py:80-126) forward on B/2 + B/2 frames per GPU,
    eval, hipGraph-captured; step 1 and every dense convolution on libnconv kernels. Returns the
    timed seconds of this rank."""
    torch.manual_seed(1)
    net = m.SETP2_BP_EXPORT(step1_crop="generalized").to(dev).eval()
    g = torch.Generator().manual_seed(3000 + rank)
    h = B // 2
    rgb0 = (torch.rand(h, 3, H, W, generator=g) * 255).to(dev)
    rgb1 = (torch.rand(h, 3, H, W, generator=g) * 255).to(dev)
    d0 = sparse_depth(g, h, H, W, dev)
    d1 = sparse_depth(g, h, H, W, dev)
    with torch.no_grad():
        for _ in range(max(warmup, 1)):
            net(rgb0, d0, rgb1, d1)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                net(rgb0, d0, rgb1, d1)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            net(rgb0, d0, rgb1, d1)
        warm_up(graph.replay, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            graph.replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    return el


def make_guided_train_step(m, dev, B, H, W, rank, graph=True):
    """Config 4 per GPU: one SETP2_BP_TRAIN iteration as train_step2.py:60-66 (train mode, frozen
    step 1 still EnforcePos-drifted, batch-statistics BatchNorm), forward on B/2 + B/2 frames,
    calculate_loss_multi_resolution (MSE, train_step2.py:21), backward, RCCL all-reduce with
    several ranks, AdamW lr 1e-4 / wd 1e-7. graph=True replays the iteration from a hipGraph
    (train.GraphedTrainStep; fused capturable AdamW, the same update rule)."""
    torch.manual_seed(1)
    model = m.SETP2_BP_TRAIN(None, step1_crop="generalized").to(dev)
    net = m.dp.DataParallelRCCL(model)
    opt = m.train.get_optimizer(net, "adam", 1e-4, 1e-7, capturable=graph, fused=graph)
    g = torch.Generator().manual_seed(4000 + rank)
    h = B // 2
    rgb0 = (torch.rand(h, 3, H, W, generator=g) * 255).to(dev)
    rgb1 = (torch.rand(h, 3, H, W, generator=g) * 255).to(dev)
    d0 = sparse_depth(g, h, H, W, dev)
    d1 = sparse_depth(g, h, H, W, dev)
    gt = sparse_depth(g, h, 480, 640, dev)
    net.train()

    def loss_fn(model_, rgb0_, d0_, rgb1_, d1_, gt_):
        est, _ = model_(rgb0_, d0_, rgb1_, d1_)
        return m.train.calculate_loss_multi_resolution(est, gt_, False)

    if graph:
        gstep = m.train.GraphedTrainStep(net, opt, loss_fn, (rgb0, d0, rgb1, d1, gt))
        return lambda: gstep()

    def step():
        opt.zero_grad()
        loss = loss_fn(net, rgb0, d0, rgb1, d1, gt)
        loss.backward()
        net.allreduce_grads()
        opt.step()
    return step


def make_train_step(m, dev, B, H, W, rank, graph=True):
    """One step-1 training iteration as train_step1.py:59-65: train-mode forward (EnforcePos drift),
    calculate_loss(estimated_depth, gt) on the whole batch with the gradient loss (train_step1.py:63),
    backward, (RCCL gradient all-reduce when several ranks run), AdamW lr 1e-2 / wd 1e-7
    (train_step1.py:16-17, utils.py:55). graph=True replays the iteration from a hipGraph."""
    torch.manual_seed(0)
    net = m.dp.DataParallelRCCL(m.SETP1_NCONV(crop="generalized").to(dev))
    opt = m.train.get_optimizer(net, "adam", 1e-2, 1e-7, capturable=graph, fused=graph)
    g = torch.Generator().manual_seed(2000 + rank)
    S = sparse_depth(g, B, H, W, dev)
    gt = sparse_depth(g, B, H, W, dev)
    net.train()

    def loss_fn(model, S, gt):
        return m.train.calculate_loss(model(S), gt, True)

    if graph:
        gstep = m.train.GraphedTrainStep(net, opt, loss_fn, (S, gt))
        return lambda: gstep()

    def step():
        opt.zero_grad()
        loss = loss_fn(net, S, gt)
        loss.backward()
        net.allreduce_grads()
        opt.step()
    return step


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:  # no launcher: start the ranks here
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import nconv_pkg
    m = nconv_pkg.load()
    lib = m._lib
    B, H, W = a.batch, a.height, a.width
    torch.manual_seed(0)
    net = m.SETP1_NCONV(crop="generalized").to(dev)
    net.train()
    with torch.no_grad():
        net(torch.zeros(1, 1, 32, 32, device=dev))  # one EnforcePos: positive (trained-like) weights
    net.eval()
    net.d_net.fused_head = bool(a.fused_head)
    if a.inference_streams is not None:
        net.d_net.inference_streams = a.inference_streams
    if a.inference_shares is not None:
        net.d_net.inference_shares = tuple(a.inference_shares)
    g = torch.Generator().manual_seed(1000 + rank)
    S = sparse_depth(g, B, H, W, dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(el):
        if world > 1:
            t = torch.tensor([el], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.item()
        return el

    warm = {}
    math_key = lambda mth, Sx: f"{mth}:{'x'.join(map(str, Sx.shape))}"

    def time_forward(Sx, steps, math):
        """Warm-up passes (hipGraph capture when --graph; then replays for at least --warmup calls
        and WARMUP_MIN_S seconds), then `steps` timed passes between barrier + synchronize; returns
        the max over ranks of the timed seconds."""
        m.nconv.FORWARD_MATH = math
        graph = None
        with torch.no_grad():
            for _ in range(max(a.warmup, 1)):
                net(Sx)
            if a.graph:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(2):
                        net(Sx)
                torch.cuda.current_stream().wait_stream(s)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    net(Sx)
            one = graph.replay if graph is not None else (lambda: net(Sx))
            warm[math_key(math, Sx)] = warm_up(one, a.warmup)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            for _ in range(steps):
                one()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        del graph
        return max_over_ranks(el)

    MATHS = {"fp32": lib.MATH_FP32, "bf16x9": lib.MATH_BF16X9, "bf16x3": lib.MATH_BF16X3}
    HEAD = MATHS[a.math]
    pass_frac = lambda t, k: round(PASS_BYTES_PER_FRAME * B * k / t / 1e9 / HBM_PEAK_GBS, 4) \
        if (H, W) == (352, 1216) else None

    # ---- headline: config 2 forward ----
    log(f"config 2 forward, {a.math}")
    state0 = gpu_state(dev)
    t_fwd = time_forward(S, a.steps, HEAD)
    state1 = gpu_state(dev)
    fps = world * B * a.steps / t_fwd
    # per-kernel times of each forward right after its timed run (rank 0), so the roofline's kernel
    # time is taken in the same conditions as the headline, not after the heavier legs below
    lt_of = {}
    head_density = None
    if rank == 0:
        log("per-kernel times")
        m.nconv.FORWARD_MATH = HEAD
        lt_of[a.math] = time_layers(m, net, S)
        dom = max(lt_of[a.math], key=lambda n: lt_of[a.math][n])
        lt_of["replayed_shape"] = time_concurrent_halves(m, net, S, dom)
        if a.head_density > 0 and a.math == "fp32":
            # the exact head skips nconv1's zero taps, so its time depends on the input density: the
            # same forward's kernels at f10's 40 % (golden fixture density) beside the 5 % headline
            log(f"per-kernel times at density {a.head_density}")
            S40 = sparse_depth(torch.Generator().manual_seed(1100 + rank), B, H, W, dev, a.head_density)
            lt_of["density"] = time_layers(m, net, S40)
            del S40

    # ---- the same forward in the other arithmetics ----
    alt = {}
    for name in a.alt_math:
        if name == a.math:
            continue
        log(f"config 2 forward, {name}")
        t = time_forward(S, a.steps, MATHS[name])
        if rank == 0:
            m.nconv.FORWARD_MATH = MATHS[name]
            lt_of[name] = time_layers(m, net, S)
        alt[name] = {"frames_per_sec": round(world * B * a.steps / t, 2), "ms_per_step": round(t / a.steps * 1e3, 4),
                     "dtype": MATH_DTYPE[name], "arith": MATH_ARITH[name], "whole_pass_hbm_frac": pass_frac(t, a.steps)}

    # ---- config 5: B=16 1024x2048 ----
    c5 = None
    S5 = None
    if not a.no_config5:
        B5, H5, W5 = 16, 1024, 2048
        log("config 5 forward (B=16 1024x2048)")
        S5 = sparse_depth(torch.Generator().manual_seed(5000 + rank), B5, H5, W5, dev)
        k5 = max(3, a.steps // 4)
        t5 = time_forward(S5, k5, HEAD)
        if rank == 0:
            m.nconv.FORWARD_MATH = HEAD
            lt_of["config5"] = time_layers(m, net, S5, reps=5)
        c5 = {"workload": f"config5: DNET forward, B=16 1024x2048 per GPU, generalized crop, {a.math}",
              "frames_per_sec": round(world * B5 * k5 / t5, 2), "ms_per_step": round(t5 / k5 * 1e3, 3),
              "steps": k5, "per_gpu_batch": B5}
        for name in a.alt_math:
            if name != a.math:
                t5b = time_forward(S5, k5, MATHS[name])
                c5[f"{name}_frames_per_sec"] = round(world * B5 * k5 / t5b, 2)
    m.nconv.FORWARD_MATH = lib.MATH_FP32

    # ---- config 4b: fwd + bwd + AdamW ----
    train = None
    if not a.no_train:
        log("config 4b training step")
        tg = a.train_graph != 0
        ks = a.train_steps or a.steps

        def time_train(graphed):
            step = make_train_step(m, dev, B, H, W, rank, graph=graphed)
            wn, ws = warm_up(step, max(a.warmup, 1))
            torch.cuda.synchronize()
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(ks):
                step()
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.perf_counter() - t0)
            del step
            return el, wn, ws
        tt, wn, ws = time_train(tg)
        ms = tt / ks * 1e3
        eager = None
        if tg and world == 1:  # the same step eager, so a 1 -> N curve can be read in either mode
            log("config 4b training step, eager")
            te, _, _ = time_train(False)
            eager = {"frames_per_sec": round(world * B * ks / te, 2), "ms_per_step": round(te / ks * 1e3, 4)}
        fl = (PASS_FLOPS_PER_FRAME + BWD_FLOPS_PER_FRAME) * B * (H * W) / (352 * 1216)
        by = (PASS_BYTES_PER_FRAME + BWD_BYTES_PER_FRAME) * B * (H * W) / (352 * 1216)
        train = {"frames_per_sec": round(world * B * ks / tt, 2), "ms_per_step": round(ms, 4), "steps": ks,
                 "mode": "hipgraph" if tg else "eager", "hipgraph": tg, "eager": eager,
                 "warmup_calls": wn, "warmup_s": round(ws, 3),
                 "loss": "calculate_loss(est, gt) on the whole batch (train_step1.py:63)",
                 "forward_math": "exact fp32 (training forward), exact fp32 backward",
                 "roofline": {"bound": "fp32", "flops_per_step": fl, "bytes_per_step": by,
                              "achieved_tflops": round(fl / (ms * 1e-3) / 1e12, 2), "peak_tflops": FP32_PEAK_TFLOPS,
                              "frac": round(fl / (ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4),
                              "hbm_frac": round(by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "basis": "SURVEY.md 8(d): forward 6.62 GFLOP / 238.4 MB + backward 12.79 GFLOP / "
                                       "373.9 MB per 352x1216 frame"}}
        torch.cuda.empty_cache()

    # ---- config 3: guided forward ----
    guided = None
    if not a.no_guided:
        log("config 3 guided forward")
        gsteps = max(5, a.steps // 5)
        el = max_over_ranks(guided_forward(m, dev, B, H, W, gsteps, min(a.warmup, 3), rank))
        fl = (GUIDED_DENSE_FLOPS_PER_FRAME + PASS_FLOPS_PER_FRAME) * B * (H * W) / (352 * 1216)
        guided = {"frames_per_sec": round(world * B * gsteps / el, 2), "ms_per_step": round(el / gsteps * 1e3, 3),
                  "steps": gsteps, "frames_per_step": B * world,
                  "workload": "config3: SETP2_BP_EXPORT forward, B/2+B/2 frames per GPU, hipGraph",
                  "dense_math": m.dense.MATH, "arith": DENSE_ARITH[m.dense.MATH],
                  "fp32_tflops": round(fl / (el / gsteps) / 1e12, 2),
                  "fp32_mfma_frac": round(fl / (el / gsteps) / 1e12 / FP32_PEAK_TFLOPS, 4)}
        torch.cuda.empty_cache()
        if world == 1:  # the other dense maths, separately labelled
            base = m.dense.MATH
            guided["other_dense_math"] = {}
            for mm in a.guided_alt_math:
                if mm == base:
                    continue
                m.dense.MATH = mm
                try:
                    el2 = guided_forward(m, dev, B, H, W, gsteps, min(a.warmup, 3), rank)
                finally:
                    m.dense.MATH = base
                guided["other_dense_math"][mm] = {"ms_per_step": round(el2 / gsteps * 1e3, 3),
                                                  "frames_per_sec": round(B * gsteps / el2, 2),
                                                  "arith": DENSE_ARITH[mm]}
                torch.cuda.empty_cache()

    # ---- config 4: guided training step ----
    guided_train = None
    if not a.no_guided_train:
        log("config 4 guided training step")
        gts = max(3, a.steps // 10)
        # forward + input gradient + weight gradient of every dense conv; frozen step 1 forward only
        fl = (3 * GUIDED_DENSE_FLOPS_PER_FRAME + PASS_FLOPS_PER_FRAME) * B * (H * W) / (352 * 1216)

        def time_guided_train(graphed):
            st = make_guided_train_step(m, dev, B, H, W, rank, graph=graphed)
            warm_up(st, max(min(a.warmup, 2), 1))
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            for _ in range(gts):
                st()
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.perf_counter() - t0)
            del st
            torch.cuda.empty_cache()
            return el
        gmode = a.guided_train_graph != 0
        tt = time_guided_train(gmode)
        guided_train = {"frames_per_sec": round(world * B * gts / tt, 2), "ms_per_step": round(tt / gts * 1e3, 3),
                        "steps": gts, "frames_per_step": B * world,
                        "workload": "config4: SETP2_BP_TRAIN fwd+bwd+AdamW, B/2+B/2 frames per GPU, "
                                    + ("hipGraph" if gmode else "eager"),
                        "mode": "hipgraph" if gmode else "eager",
                        "dense_math": m.dense.MATH, "arith": DENSE_ARITH[m.dense.MATH],
                        "fp32_tflops": round(fl / (tt / gts) / 1e12, 2),
                        "fp32_mfma_frac": round(fl / (tt / gts) / 1e12 / FP32_PEAK_TFLOPS, 4)}
        if gmode and world == 1:  # the eager step beside it
            log("config 4 guided training step, eager")
            te = time_guided_train(False)
            guided_train["eager"] = {"frames_per_sec": round(world * B * gts / te, 2),
                                     "ms_per_step": round(te / gts * 1e3, 3)}
        if gmode and world == 1:  # the other dense maths (graphed), separately labelled
            base = m.dense.MATH
            guided_train["other_dense_math"] = {}
            for mm in a.guided_alt_math:
                if mm == base:
                    continue
                log(f"config 4 guided training step, dense math {mm}")
                m.dense.MATH = mm
                try:
                    t2 = time_guided_train(True)
                finally:
                    m.dense.MATH = base
                guided_train["other_dense_math"][mm] = {"ms_per_step": round(t2 / gts * 1e3, 3),
                                                        "frames_per_sec": round(B * gts / t2, 2),
                                                        "arith": DENSE_ARITH[mm]}

    # ---- per-kernel times, rooflines, CPU baseline (rank 0) ----
    if rank == 0:
        costs = kernel_costs(B, H, W)
        lt = lt_of[a.math]
        issued = (lambda k: mfma_issued_flops(k, B, H, W, a.math)) if a.math in MFMA_TERMS else None
        roof = roofline(lt, costs, a.math, B, H, W, issued_mfma=issued)
        roof["whole_pass_hbm_frac"] = pass_frac(t_fwd, a.steps)
        roof["launch"] = f"kernel_us: one isolated B={B} launch on one stream (HIP events, outside the graph)"
        if lt_of.get("replayed_shape"):
            span = lt_of["replayed_shape"]
            fl_dom = costs[roof["kernel"]][1]
            roof["replayed_shape"] = {
                "launches": f"two concurrent B={B // 2} launches on two streams (the headline graph's split)",
                "span_us": round(span, 2), "reference_flop_frac": round(fl_dom / (span * 1e-6) / 1e12 / FP32_PEAK_TFLOPS, 4)}
        if "density" in lt_of:
            dom = roof["kernel"]
            head_density = {}
            for dens, lt_d in ((0.05, lt), (a.head_density, lt_of["density"])):
                r_d = roofline({dom: lt_d[dom]}, costs, a.math, B, H, W)
                ex = sq_exec(dom if dens == 0.05 else f"{dom}@{dens:.2f}", a.math, B, H, W)
                ent = {"kernel_us": r_d["kernel_us"], "reference_flop_frac": r_d["fp32_frac"],
                       "executed_frac": None, "layer_us": {k: round(v, 2) for k, v in lt_d.items()}}
                if ex:
                    ent["executed_frac"] = round(ex["executed_flops_per_launch"] / (lt_d[dom] * 1e-6) / 1e12
                                                 / FP32_PEAK_TFLOPS, 4)
                    ent["executed_fp32_flops_per_launch"] = ex["executed_flops_per_launch"]
                head_density[f"{dens:.2f}"] = ent
            head_density["note"] = ("reference_flop_frac counts nconv1 + nconv2 densely (the reference's flops); "
                                    "executed_frac = the fp32 flops the kernel's FMA instructions performed "
                                    "(SQ counters at that density, profiles/sq_exec.json) over the same time")
        for name, rec in alt.items():
            lt_a = lt_of[name]
            rec["layer_us"] = {k: round(v, 2) for k, v in lt_a.items()}
            rec["roofline"] = roofline(lt_a, costs, name, B, H, W,
                                       issued_mfma=(lambda k, n=name: mfma_issued_flops(k, B, H, W, n))
                                       if name in MFMA_TERMS else None)
        if c5 is not None:
            lt5 = lt_of["config5"]
            c5["layer_us"] = {k: round(v, 2) for k, v in lt5.items()}
            c5["roofline"] = roofline(lt5, kernel_costs(16, 1024, 2048), a.math, 16, 1024, 2048)
            c5["whole_pass_hbm_frac"] = round(1169.4e6 * 16 / (c5["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        m.nconv.FORWARD_MATH = lib.MATH_FP32
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            log("CPU baseline")
            cpu = cpu_baseline(B, H, W, a.cpu_seconds)
        result = {
            "metric": "frames/sec (352x1216 sparse depth, DNET NConv U-Net forward, B=8 per GPU)",
            "value": round(fps, 2), "unit": "frames/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(t_fwd / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": MATH_DTYPE[a.math],
            "data": "synthetic (seeded 5%-dense U(1,80) depth, seeded init + one EnforcePos)",
            "config": {"workload": f"config2: SETP1_NCONV/DNET forward, fused HIP NConv kernels, {a.math}",
                       "global_batch": B * world, "per_gpu_batch": B, "height": H, "width": W,
                       "crop": "generalized [1:H+1,1:W+1]", "parallelism": f"frame-sharded x{world}",
                       "hipgraph": bool(a.graph), "fused_head": bool(a.fused_head)},
            "arith": MATH_ARITH[a.math],
            "layer_us": {k: round(v, 2) for k, v in lt.items()},
            "roofline": roof,
            "head_density": head_density,
            "warmup_replays": {k: {"calls": n, "seconds": round(t, 3)} for k, (n, t) in warm.items()},
            "gpu_state": {"before": state0, "after_forward": state1},
            "fwd_other_arith": alt,
            "config5": c5,
            "train_fwd_bwd_adamw": train,
            "guided_fwd": guided,
            "guided_train_fwd_bwd_adamw": guided_train,
            "cpu_baseline": cpu,
        }
        if cpu:
            result["speedup_vs_cpu"] = round(fps / cpu["value"], 1)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
