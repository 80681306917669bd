"""Debug: which part of bench.C3Lsq.check fails on the GPU."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
W = bench.C3Lsq(dev, 2, 0)
for i in range(3):
    assert W.launch(i) == 0
torch.cuda.synchronize()
s = W.slots[0]
k = 1 << 21
x, g = s["x"].reshape(-1)[:k].cpu(), s["g"].reshape(-1)[:k].cpu()
s32 = torch.tensor(W.scale0, dtype=torch.float64).float()
r = torch.round(x / s32)
y = torch.clamp(r, -128, 127) * s32
m = (r >= -128) & (r <= 127)
gx = torch.where(m, (g * s32) / s32, torch.zeros_like(g))
print("y eq", torch.equal(y.view(torch.int32), s["y"].reshape(-1)[:k].cpu().view(torch.int32)))
print("gx eq", torch.equal(gx.view(torch.int32), s["gx"].reshape(-1)[:k].cpu().view(torch.int32)))
xd, gd, sd = s["x"].double(), s["g"].double(), float(s32)
rd = torch.round(xd / sd)
md = (rd >= -128) & (rd <= 127)
term = gd * (torch.clamp(rd, -128, 127) - torch.where(md, xd / sd, torch.zeros_like(xd)))
want = float(term.sum()) * W.gscale
print("grads", s["grads"].tolist(), "want", want)
from oracle import fakequant_np as O
xn, gn = s["x"].reshape(-1)[:k].cpu().numpy(), s["g"].reshape(-1)[:k].cpu().numpy()
yo, gxo, gso, _ = O.lsq_forward_backward(xn, gn, W.scale0, 0, -128, 127, W.gscale)
print("oracle y eq", (yo.view('u4') == s["y"].reshape(-1)[:k].cpu().numpy().view('u4')).all())
