"""Drop-in for the reference's models/step2.py: same names, backed by nconv_amd.

    from models.step2 import SETP2_BP_TRAIN, SETP2_BP_EXPORT
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import nconv_pkg  # noqa: E402

_m = nconv_pkg.load()
_g = _m.guided
SETP2_BP_TRAIN = _g.SETP2_BP_TRAIN
SETP2_BP_EXPORT = _g.SETP2_BP_EXPORT
RGBEncoder = _g.RGBEncoder
Conv1x1, Conv3x3, UpCat, Basic2d, Basic2dTrans = _g.Conv1x1, _g.Conv3x3, _g.UpCat, _g.Basic2d, _g.Basic2dTrans
NewFusionBlock, FusionResolutionBlock, FusionResolution0, ConvBlock = (
    _g.NewFusionBlock, _g.FusionResolutionBlock, _g.FusionResolution0, _g.ConvBlock)
