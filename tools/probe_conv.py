import torch, torch.nn.functional as F
g = torch.Generator().manual_seed(0)
x = torch.rand(2, 8, 64, 96, generator=g) * 10
w = torch.rand(8, 8, 5, 5, generator=g) + 0.05
ref = F.conv2d(x.double(), w.double(), None, 1, 2)
for tf32 in (True, False):
    torch.backends.cudnn.allow_tf32 = tf32
    torch.backends.cuda.matmul.allow_tf32 = tf32
    y = F.conv2d(x.cuda(), w.cuda(), None, 1, 2).double().cpu()
    print("allow_tf32", tf32, "max rel err", ((y - ref).abs() / ref.abs()).max().item())
print(torch.backends.cudnn.allow_tf32, torch.backends.cudnn.enabled)
