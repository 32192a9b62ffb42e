"""Drop-in for the reference's models/step1.py: same names, backed by nconv_amd (libnconv on MI355X).

    from models.step1 import SETP1_NCONV, DNET, NConv2d, EnforcePos
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import nconv_pkg  # noqa: E402

_m = nconv_pkg.load()
SETP1_NCONV = _m.SETP1_NCONV
DNET = _m.DNET
NConv2d = _m.NConv2d
EnforcePos = _m.EnforcePos
