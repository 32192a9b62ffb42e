"""ctypes binding of libnconv.so (the C ABI in include/nconv.h).

Loaded lazily on first use, after `import torch`, so the dynamic loader resolves the library's
libamdhip64.so.7 to the HIP runtime torch already mapped (one HIP runtime per process).
There is deliberately no fallback: a missing or unloadable library raises.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# NCONV_LIB: an alternative build of the same library (kernel-tuning experiments)
LIB_PATH = os.environ.get("NCONV_LIB") or os.path.join(_HERE, "libnconv.so")
ABI_VERSION = 22
BWD_ACCUMULATE = 1
BWD_DEFER_REDUCE = 2
BWD_SEPARATE = 4  # accepted and ignored since ABI 21 (include/nconv.h)

# enum nconv_load_mode
PLAIN, THRESH, POOL2, UPCAT_SKIP_FIRST, UPCAT_UP_FIRST = 0, 1, 2, 3, 4
# enum nconv_math
MATH_FP32, MATH_BF16X3, MATH_BF16X9 = 0, 1, 2
# enum nconv_kernel (nconv_plan)
KERNEL_GENERIC, KERNEL_TILED_FP32, KERNEL_MFMA_FP32, KERNEL_MFMA_BF16X3, KERNEL_MFMA_BF16X9 = 0, 1, 2, 3, 4
KERNEL_TILED_FP32_PHASE = 5
KERNEL_NAMES = ("generic", "tiled_fp32", "mfma_fp32", "mfma_bf16x3", "mfma_bf16x9", "tiled_fp32_phase")
# enum nconv_dense_kind
DENSE_3X3, DENSE_1X1, DENSE_TRANSPOSED_4X4, DENSE_CONV4X4_S2 = 0, 1, 2, 3
# enum nconv_dense_math
DENSE_MATHS = {"fp32": 0, "bf16x9": 2, "bf16x6": 3}

EXPORTED = (
    "nconv_abi_version",
    "nconv_last_error",
    "nconv_weight_prep",
    "nconv_fwd",
    "nconv_fwd_pooled",
    "nconv_fwd_tail",
    "nconv_fwd_head",
    "nconv_head_weights",
    "nconv_plan",
    "nconv_phase_weights_floats",
    "nconv_phase_weights",
    "nconv_weight_prologue",
    "nconv_train_prologue",
    "nconv_bwd_workspace_bytes",
    "nconv_bwd",
    "nconv_bwd_ex",
    "nconv_bwd_head_workspace_bytes",
    "nconv_bwd_tail_workspace_bytes",
    "nconv_wgrad_reduce",
    "nconv_wgrad_reduce_ex",
    "nconv_sum_workspace_bytes",
    "nconv_dense_packed_floats",
    "nconv_dense_pack",
    "nconv_dense_conv_fwd",
    "nconv_conv3x3_c1",
    "nconv_bilinear_ac",
    "nconv_dense_wgrad_workspace_bytes",
    "nconv_dense_conv_wgrad",
    "nconv_bn_workspace_bytes",
    "nconv_bn_train_fwd",
    "nconv_bn_train_bwd",
    "nconv_relu_bias_bwd_workspace_bytes",
    "nconv_relu_bias_bwd",
    "nconv_depth_loss_workspace_bytes",
    "nconv_depth_loss_fwd",
    "nconv_depth_loss_bwd",
)


class NconvSrc(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("c", ctypes.c_void_p), ("C", ctypes.c_int),
                ("H", ctypes.c_int), ("W", ctypes.c_int)]


class NconvLayer(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("Cin", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("Cout", ctypes.c_int), ("Ho", ctypes.c_int), ("Wo", ctypes.c_int),
                ("KH", ctypes.c_int), ("KW", ctypes.c_int), ("SH", ctypes.c_int), ("SW", ctypes.c_int),
                ("PH", ctypes.c_int), ("PW", ctypes.c_int), ("DH", ctypes.c_int), ("DW", ctypes.c_int),
                ("groups", ctypes.c_int), ("eps", ctypes.c_float), ("load_mode", ctypes.c_int),
                ("thresh", ctypes.c_float), ("a", NconvSrc), ("b", NconvSrc),
                ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("wsum", ctypes.c_void_p),
                ("math", ctypes.c_int), ("bwd_math", ctypes.c_int), ("waux", ctypes.c_void_p)]


class NconvBwdIo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("y", "cout", "gy", "gcout", "gxa", "gca", "gxb", "gcb", "gw",
                                               "gbias", "gy_pool", "gcout_pool", "pool_argmax")] + [
        ("head", ctypes.POINTER(NconvLayer)), ("head_workspace", ctypes.c_void_p),
        ("head_workspace_bytes", ctypes.c_size_t), ("head_gw", ctypes.c_void_p), ("head_gbias", ctypes.c_void_p),
        ("head_nparts", ctypes.c_int), ("tail", ctypes.POINTER(NconvLayer)), ("tail_y", ctypes.c_void_p),
        ("tail_cout", ctypes.c_void_p), ("tail_gy", ctypes.c_void_p), ("tail_workspace", ctypes.c_void_p),
        ("tail_workspace_bytes", ctypes.c_size_t), ("tail_gw", ctypes.c_void_p), ("tail_nparts", ctypes.c_int),
        ("box_weights", ctypes.c_void_p), ("tail_crop0", ctypes.c_int), ("tail_h", ctypes.c_int),
        ("tail_w", ctypes.c_int)]


class NconvDenseConv(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("x0", ctypes.c_void_p), ("C0", ctypes.c_int),
                ("x1", ctypes.c_void_p), ("C1", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("Cout", ctypes.c_int), ("Ho", ctypes.c_int), ("Wo", ctypes.c_int),
                ("kind", ctypes.c_int), ("stride", ctypes.c_int), ("wpack", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("relu", ctypes.c_int), ("wshort", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("out_C", ctypes.c_int), ("out_c0", ctypes.c_int),
                ("math", ctypes.c_int)]


class NconvDenseWgrad(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("kind", ctypes.c_int), ("stride", ctypes.c_int),
                ("x0", ctypes.c_void_p), ("C0", ctypes.c_int), ("x1", ctypes.c_void_p), ("C1", ctypes.c_int),
                ("H", ctypes.c_int), ("W", ctypes.c_int), ("gy", ctypes.c_void_p), ("Cout", ctypes.c_int),
                ("Ho", ctypes.c_int), ("Wo", ctypes.c_int), ("gw", ctypes.c_void_p), ("math", ctypes.c_int)]


class NconvBnTrain(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("x", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p),
                ("running_mean", ctypes.c_void_p), ("running_var", ctypes.c_void_p),
                ("momentum", ctypes.c_float), ("eps", ctypes.c_float), ("relu", ctypes.c_int),
                ("y", ctypes.c_void_p), ("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p)]


_lib = None
_lock = threading.Lock()


def _declare(lib):
    P = ctypes.c_void_p
    lib.nconv_abi_version.restype = ctypes.c_int
    lib.nconv_abi_version.argtypes = []
    lib.nconv_last_error.restype = ctypes.c_char_p
    lib.nconv_last_error.argtypes = []
    lib.nconv_weight_prep.restype = ctypes.c_int
    lib.nconv_weight_prep.argtypes = [ctypes.c_int, P, P, P, P, P, P]
    lib.nconv_fwd.restype = ctypes.c_int
    lib.nconv_fwd.argtypes = [ctypes.POINTER(NconvLayer), P, P, P]
    lib.nconv_fwd_pooled.restype = ctypes.c_int
    lib.nconv_fwd_pooled.argtypes = [ctypes.POINTER(NconvLayer), P, P, P, P, P, P]
    lib.nconv_fwd_head.restype = ctypes.c_int
    lib.nconv_fwd_head.argtypes = [ctypes.POINTER(NconvLayer), ctypes.POINTER(NconvLayer), P, P, P, P, P, P, P, P]
    lib.nconv_head_weights.restype = ctypes.c_int
    lib.nconv_head_weights.argtypes = [ctypes.POINTER(NconvLayer), ctypes.POINTER(NconvLayer), P, P]
    lib.nconv_fwd_tail.restype = ctypes.c_int
    lib.nconv_fwd_tail.argtypes = [ctypes.POINTER(NconvLayer), P, P, P, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_float, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
    lib.nconv_plan.restype = ctypes.c_int
    lib.nconv_plan.argtypes = [ctypes.POINTER(NconvLayer), P, P, P]
    lib.nconv_phase_weights_floats.restype = ctypes.c_size_t
    lib.nconv_phase_weights_floats.argtypes = [ctypes.POINTER(NconvLayer)]
    lib.nconv_phase_weights.restype = ctypes.c_int
    lib.nconv_phase_weights.argtypes = [ctypes.c_int, P, P, P, P, P]
    lib.nconv_weight_prologue.restype = ctypes.c_int
    lib.nconv_weight_prologue.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, ctypes.c_int, P, P, P, P, P]
    lib.nconv_bwd_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_bwd_workspace_bytes.argtypes = [ctypes.POINTER(NconvLayer)]
    lib.nconv_bwd.restype = ctypes.c_int
    lib.nconv_bwd.argtypes = [ctypes.POINTER(NconvLayer), P, P, P, P, P, P, P, P, P, P, P,
                              ctypes.c_size_t, ctypes.c_uint, P]
    lib.nconv_bwd_ex.restype = ctypes.c_int
    lib.nconv_bwd_ex.argtypes = [ctypes.POINTER(NconvLayer), ctypes.POINTER(NconvBwdIo), P, ctypes.c_size_t,
                                 ctypes.c_uint, P]
    lib.nconv_bwd_head_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_bwd_head_workspace_bytes.argtypes = [ctypes.POINTER(NconvLayer)]
    lib.nconv_bwd_tail_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_bwd_tail_workspace_bytes.argtypes = [ctypes.POINTER(NconvLayer)]
    lib.nconv_wgrad_reduce.restype = ctypes.c_int
    lib.nconv_wgrad_reduce.argtypes = [ctypes.c_int, ctypes.POINTER(NconvLayer), P, P, P, P, P]
    lib.nconv_wgrad_reduce_ex.restype = ctypes.c_int
    lib.nconv_wgrad_reduce_ex.argtypes = [ctypes.c_int, ctypes.POINTER(NconvLayer), P, P, P, P, ctypes.c_int, P, P,
                                          P, P, ctypes.c_size_t, P]
    lib.nconv_sum_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_sum_workspace_bytes.argtypes = [ctypes.c_int]
    lib.nconv_train_prologue.restype = ctypes.c_int
    lib.nconv_train_prologue.argtypes = [ctypes.c_int, P, P, P, P, P, ctypes.c_int, ctypes.c_int, P, P,
                                         ctypes.c_int, P, P, P, P, P]
    I = ctypes.c_int
    lib.nconv_dense_packed_floats.restype = ctypes.c_size_t
    lib.nconv_dense_packed_floats.argtypes = [I, I, I]
    lib.nconv_dense_pack.restype = I
    lib.nconv_dense_pack.argtypes = [I, I, I, P, P, P, P]
    lib.nconv_dense_conv_fwd.restype = I
    lib.nconv_dense_conv_fwd.argtypes = [ctypes.POINTER(NconvDenseConv), P]
    lib.nconv_conv3x3_c1.restype = I
    lib.nconv_conv3x3_c1.argtypes = [P, I, I, I, I, P, P, P, P]
    lib.nconv_bilinear_ac.restype = I
    lib.nconv_bilinear_ac.argtypes = [P, I, I, I, I, P, I, I, P]
    lib.nconv_dense_wgrad_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_dense_wgrad_workspace_bytes.argtypes = [ctypes.POINTER(NconvDenseWgrad)]
    lib.nconv_dense_conv_wgrad.restype = I
    lib.nconv_dense_conv_wgrad.argtypes = [ctypes.POINTER(NconvDenseWgrad), P, ctypes.c_size_t, P]
    lib.nconv_bn_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_bn_workspace_bytes.argtypes = [ctypes.POINTER(NconvBnTrain)]
    lib.nconv_bn_train_fwd.restype = I
    lib.nconv_bn_train_fwd.argtypes = [ctypes.POINTER(NconvBnTrain), P, ctypes.c_size_t, P]
    lib.nconv_bn_train_bwd.restype = I
    lib.nconv_bn_train_bwd.argtypes = [ctypes.POINTER(NconvBnTrain), P, P, P, P, P, ctypes.c_size_t, P]
    lib.nconv_relu_bias_bwd_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_relu_bias_bwd_workspace_bytes.argtypes = [I, I, I, I]
    lib.nconv_relu_bias_bwd.restype = I
    lib.nconv_relu_bias_bwd.argtypes = [I, I, I, I, P, P, P, P, P, ctypes.c_size_t, P]
    L = ctypes.c_longlong
    lib.nconv_depth_loss_workspace_bytes.restype = ctypes.c_size_t
    lib.nconv_depth_loss_workspace_bytes.argtypes = [I, I, I]
    lib.nconv_depth_loss_fwd.restype = I
    lib.nconv_depth_loss_fwd.argtypes = [P, L, L, P, L, L, I, I, I, I, P, P, ctypes.c_size_t, P]
    lib.nconv_depth_loss_bwd.restype = I
    lib.nconv_depth_loss_bwd.argtypes = [P, L, L, P, L, L, I, I, I, I, P, P, ctypes.c_size_t, P, P]


def lib():
    """The loaded library. Raises RuntimeError if it is missing or incompatible."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libnconv.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no fallback path exists)")
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(handle)
            v = handle.nconv_abi_version()
            if v != ABI_VERSION:
                raise RuntimeError(f"libnconv ABI {v} != expected {ABI_VERSION}")
            _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().nconv_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def src(x, c):
    """NconvSrc for a (B, C, H, W) pair (c may be None)."""
    s = NconvSrc()
    if x is not None:
        s.x = x.data_ptr()
        s.c = c.data_ptr() if c is not None else None
        s.C, s.H, s.W = x.shape[1], x.shape[2], x.shape[3]
    return s
