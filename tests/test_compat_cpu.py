"""CPU: the compat `models` package resolves the reference's import lines to nconv_amd classes."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_import_lines_resolve():
    code = ("from models.step1 import SETP1_NCONV, NConv2d, EnforcePos, DNET\n"
            "from models.step2 import SETP2_BP_TRAIN, SETP2_BP_EXPORT\n"
            "import torch; torch.manual_seed(0); n = SETP1_NCONV()\n"
            "print(type(n).__module__, round(float(n.d_net.nconv1.weight.sum()), 4))\n")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "compat"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    mod, s = out.stdout.split()
    assert mod.startswith("nconv_amd") and s == "111.0923"
