"""Do GPU fp32 forward activations pick different max-pool winners than the fp64 oracle?"""
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch, torch.nn.functional as F
import nconv_pkg; m = nconv_pkg.load(); L = m._lib
from oracle import nconv_ref as R
from test_gpu_dnet import make_net, oracle_params, sparse_depth
from nconv_cases import oracle_layer
gpu = torch.device('cuda')
for H, W in [(64, 96), (45, 67)]:
    net = make_net(m, "literal", gpu); net.train()
    with torch.no_grad(): net(torch.zeros(1,1,8,8,device=gpu))  # second softplus like the test
    net.eval()
    g = torch.Generator().manual_seed(11)
    S = sparse_depth(g, 2, H, W)
    P = oracle_params(net)
    d = net.d_net
    def run(ours):
        acts = {}
        dt = torch.float32 if ours else torch.float64
        dev = gpu if ours else 'cpu'
        def lay(n, mode, xa, ca, xb=None, cb=None):
            w, b = (t.to(dev, dt) for t in P[n])
            if ours:
                ws = torch.empty(w.shape[0], device=dev); m.weight_prep([w], [False], [ws])
                y, c = m.nconv.layer_forward_raw(getattr(d, n).spec(mode, 0.01), xa, ca, xb, cb, w, b, ws)
            else:
                y, c = oracle_layer(mode, xa, ca, xb, cb, w, b, *R.DNET_GEOMETRY[n])
            acts[n] = (y, c); return y, c
        Sd = S.to(dev, dt)
        x1, c1 = lay("nconv1", L.THRESH, Sd, None); x1, c1 = lay("nconv2", L.PLAIN, x1, c1)
        x2, c2 = lay("nconv_down1", L.POOL2, x1, c1); x3, c3 = lay("nconv_down2", L.POOL2, x2, c2)
        lay("nconv_down3", L.POOL2, x3, c3)
        return acts
    with torch.no_grad():
        A, B = run(True), run(False)
    for n in ("nconv2", "nconv_down1", "nconv_down2"):
        for i, lab in ((0, 'x'), (1, 'c')):
            _, ig = F.max_pool2d(A[n][i].double().cpu(), 2, 2, return_indices=True)
            _, ir = F.max_pool2d(B[n][i], 2, 2, return_indices=True)
            mism = (ig != ir).sum().item()
            print(H, W, n, lab, 'argmax mismatches', mism, 'of', ig.numel())
    n = "nconv2"
    xg = A[n][0].double().cpu(); xr = B[n][0]
    _, ig = F.max_pool2d(xg, 2, 2, return_indices=True)
    _, ir = F.max_pool2d(xr, 2, 2, return_indices=True)
    bad = (ig != ir).nonzero()[:4]
    for b_, c_, i_, j_ in bad.tolist():
        wg = xg[b_, c_, 2*i_:2*i_+2, 2*j_:2*j_+2].flatten().tolist()
        wr = xr[b_, c_, 2*i_:2*i_+2, 2*j_:2*j_+2].flatten().tolist()
        cg = A[n][1][b_, c_, 2*i_:2*i_+2, 2*j_:2*j_+2].flatten().tolist()
        print('gpu', ['%.9g' % v for v in wg], 'f64', ['%.9g' % v for v in wr], 'c', ['%.3g' % v for v in cg])
