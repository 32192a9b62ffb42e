"""Layer-by-layer gradient comparison GPU vs fp64 oracle for DNET (developer diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
import nconv_pkg
from oracle import nconv_ref as R
m = nconv_pkg.load(); L = m._lib
dev = torch.device("cuda")
torch.manual_seed(0)
net = m.SETP1_NCONV().to(dev)
net.train()
with torch.no_grad(): net(torch.zeros(1,1,32,32,device=dev))
H, W = int(sys.argv[1]) if len(sys.argv) > 1 else 64, int(sys.argv[2]) if len(sys.argv) > 2 else 96
g = torch.Generator().manual_seed(11)
S = (torch.rand(2,1,H,W,generator=g)*79+1)*(torch.rand(2,1,H,W,generator=g)<0.05)
sd = {k: v.detach().double().cpu() for k, v in net.state_dict().items()}
P = R.dnet_params_from_state_dict(sd)

def run(dt, device, ours):
    d = net.d_net
    names = R.DNET_LAYERS
    acts = {}
    params = {n: (P[n][0].detach().to(device, dt).clone().requires_grad_(True), P[n][1].detach().to(device, dt).clone().requires_grad_(True)) for n in names}
    Sd = S.to(device, dt)
    def lay(name, mode, xa, ca, xb=None, cb=None):
        w, b = params[name]
        if ours:
            mod = getattr(d, name)
            spec = mod.spec(mode, 0.01)
            ws = torch.empty(w.shape[0], device=device); m.weight_prep([w.detach()], [False], [ws])
            y, c = m.nconv_layer(spec, xa, ca, xb, cb, w, b, ws)
        else:
            import importlib; sys.path.insert(0, 'tests'); from nconv_cases import oracle_layer
            st, pad = R.DNET_GEOMETRY[name]
            y, c = oracle_layer(mode, xa, ca, xb, cb, w, b, st, pad)
        y.retain_grad(); c.retain_grad(); acts[name] = (y, c)
        return y, c
    x1, c1 = lay("nconv1", L.THRESH, Sd, None)
    x1, c1 = lay("nconv2", L.PLAIN, x1, c1)
    x2, c2 = lay("nconv_down1", L.POOL2, x1, c1)
    x3, c3 = lay("nconv_down2", L.POOL2, x2, c2)
    x4, c4 = lay("nconv_down3", L.POOL2, x3, c3)
    x34, c34 = lay("nconv4", L.UPCAT_SKIP_FIRST, x3, c3, x4, c4)
    x23, c23 = lay("nconv5", L.UPCAT_SKIP_FIRST, x2, c2, x34, c34)
    xo, co = lay("nconv6", L.UPCAT_UP_FIRST, x1, c1, x23, c23)
    xo, co = lay("nconv7", L.PLAIN, xo, co)
    out = xo[:, :, 1:481, 1:641]
    g2 = torch.Generator().manual_seed(5)
    gt = torch.rand(out.shape, generator=g2, dtype=torch.float64)*80
    gt = (gt*(torch.rand(out.shape, generator=g2, dtype=torch.float64)<0.3)).to(device, dt)
    R.calculate_loss(out[0], gt[0], True).backward()
    return acts, params

A64, P64 = run(torch.float64, "cpu", False)
A32, P32 = run(torch.float32, "cpu", False)
AG, PG = run(torch.float32, dev, True)
rel = lambda a, b: float("nan") if (a is None or b is None) else ((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-300)).item()
print(f"{'layer':12s} {'gy cpu32':>9s} {'gy gpu':>9s} {'gc cpu32':>9s} {'gc gpu':>9s} | {'gW cpu32':>9s} {'gW gpu':>9s} {'gb cpu32':>9s} {'gb gpu':>9s} | y gpu")
for n in reversed(R.DNET_LAYERS):
    (y64, c64), (y32, c32), (yg, cg) = A64[n], A32[n], AG[n]
    print(f"{n:12s} {rel(y32.grad, y64.grad):9.2e} {rel(yg.grad, y64.grad):9.2e} {rel(c32.grad, c64.grad):9.2e} {rel(cg.grad, c64.grad):9.2e} | "
          f"{rel(P32[n][0].grad, P64[n][0].grad):9.2e} {rel(PG[n][0].grad, P64[n][0].grad):9.2e} {rel(P32[n][1].grad, P64[n][1].grad):9.2e} {rel(PG[n][1].grad, P64[n][1].grad):9.2e} | {rel(yg.detach(), y64.detach()):9.2e}")

# ---- isolate per-layer kernel error: exact (fp64) upstream grads and inputs fed to one layer ----
print("\nisolated layer backward, exact fp64 inputs/upstream grads cast to fp32:")
print(f"{'layer':12s} {'gW gpu':>9s} {'gW cpu32':>9s} {'gb gpu':>9s} {'gb cpu32':>9s}")
names = R.DNET_LAYERS
# rebuild the fp64 layer inputs by re-running the fp64 oracle forward with hooks
acts_in = {}
def lay64(name, mode, xa, ca, xb=None, cb=None):
    acts_in[name] = (mode, xa, ca, xb, cb)
    w, b = P[name]
    sys.path.insert(0, 'tests'); from nconv_cases import oracle_layer
    st, pad = R.DNET_GEOMETRY[name]
    return oracle_layer(mode, xa, ca, xb, cb, w, b, st, pad)
Sd = S.double()
x1, c1 = lay64("nconv1", L.THRESH, Sd, None)
x1, c1 = lay64("nconv2", L.PLAIN, x1, c1)
x2, c2 = lay64("nconv_down1", L.POOL2, x1, c1)
x3, c3 = lay64("nconv_down2", L.POOL2, x2, c2)
x4, c4 = lay64("nconv_down3", L.POOL2, x3, c3)
x34, c34 = lay64("nconv4", L.UPCAT_SKIP_FIRST, x3, c3, x4, c4)
x23, c23 = lay64("nconv5", L.UPCAT_SKIP_FIRST, x2, c2, x34, c34)
xo, co = lay64("nconv6", L.UPCAT_UP_FIRST, x1, c1, x23, c23)
lay64("nconv7", L.PLAIN, xo, co)
from nconv_cases import oracle_layer
for n in names:
    mode, xa, ca, xb, cb = acts_in[n]
    gy64 = A64[n][0].grad
    gc64 = A64[n][1].grad if A64[n][1].grad is not None else torch.zeros_like(gy64)
    st, pad = R.DNET_GEOMETRY[n]
    def leaf(t, dt, device):
        return None if t is None else t.detach().to(device, dt).clone().requires_grad_(True)
    res = {}
    for tag, dt, device in (("64", torch.float64, "cpu"), ("32", torch.float32, "cpu"), ("gpu", torch.float32, dev)):
        w = leaf(P[n][0], dt, device); b = leaf(P[n][1], dt, device)
        ins = [leaf(t, dt, device) for t in (xa, ca, xb, cb)]
        if tag == "gpu":
            ws = torch.empty(w.shape[0], device=device); m.weight_prep([w.detach()], [False], [ws])
            y, c = m.nconv_layer(getattr(net.d_net, n).spec(mode, 0.01), *ins, w, b, ws)
        else:
            y, c = oracle_layer(mode, *ins, w, b, st, pad)
        (y * gy64.to(device, dt) + c * gc64.to(device, dt)).sum().backward()
        res[tag] = (w.grad, b.grad)
    print(f"{n:12s} {rel(res['gpu'][0], res['64'][0]):9.2e} {rel(res['32'][0], res['64'][0]):9.2e} "
          f"{rel(res['gpu'][1], res['64'][1]):9.2e} {rel(res['32'][1], res['64'][1]):9.2e}")
