"""nconv_amd — MI355X-native normalized-convolution (NConv) depth completion.

Drop-in for the hot path of lllllcf/Realtime-Depth-Estimation-Nconv (models/step1.py, models/step2.py):
the same nn.Module classes, signatures and state_dict keys, computed by hand-written gfx950 HIP
kernels behind the C ABI of include/nconv.h (libnconv.so, built in-tree).

The directory name is not a Python identifier; import it through the repo-root helper
`nconv_pkg.load()`, which registers it as the module `nconv_amd`.
"""
from . import _lib, data, dense, dp, export, guided, train
from .nconv import EnforcePos, LayerSpec, NConv2d, NConvLayerFn, nconv_layer, weight_prep
from .dnet import DNET, SETP1_NCONV, crop_hw
from .guided import SETP2_BP_EXPORT, SETP2_BP_TRAIN, RGBEncoder

__all__ = ["EnforcePos", "LayerSpec", "NConv2d", "NConvLayerFn", "nconv_layer", "weight_prep", "DNET",
           "SETP1_NCONV", "crop_hw", "SETP2_BP_EXPORT", "SETP2_BP_TRAIN", "RGBEncoder"]
