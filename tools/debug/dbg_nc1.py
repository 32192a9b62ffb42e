import sys, os; sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch
import nconv_pkg; m = nconv_pkg.load()
from oracle import nconv_ref as R
from test_gpu_dnet import make_net, oracle_params, sparse_depth
gpu = torch.device('cuda')
for H, W in [(45, 67), (45, 64), (48, 67), (64, 67), (45, 96)]:
    net = make_net(m, "literal", gpu); net.train()
    g = torch.Generator().manual_seed(11)
    S = sparse_depth(g, 2, H, W)
    params0 = oracle_params(net)
    params = {n: (R.softplus_pos(w).detach().requires_grad_(True), b.detach().requires_grad_(True)) for n, (w, b) in params0.items()}
    ref = R.dnet_forward(S.double(), params, "literal")
    g2 = torch.Generator().manual_seed(5)
    gt = torch.rand(ref.shape, generator=g2, dtype=torch.float64) * 80
    gt = gt * (torch.rand(ref.shape, generator=g2, dtype=torch.float64) < 0.3)
    R.calculate_loss(ref[0], gt[0], True).backward()
    out = net(S.to(gpu))
    R.calculate_loss(out[0], gt[0].to(gpu, torch.float32), True).backward()
    gw = net.d_net.nconv1.weight.grad.double().cpu(); rw = params['nconv1'][0].grad
    d = (gw - rw).abs()
    print(H, W, 'nconv1 gW rel', (d.max()/rw.abs().max()).item(), 'worst idx', divmod(int(d.argmax()), 25), 'nconv2', ((net.d_net.nconv2.weight.grad.double().cpu()-params['nconv2'][0].grad).abs().max()/params['nconv2'][0].grad.abs().max()).item())
    print('   per-o max err', d.amax(dim=(1,2,3)).tolist())
