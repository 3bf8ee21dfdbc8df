"""Which bf16 rounding points does the implicit-GEMM subsampling backward have?  Compares the
HIP bf16 gradients with float64 restatements that round at different subsets of points."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "espnet-1_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.nn.functional as F

def bf(x):
    return x.to(torch.bfloat16).to(torch.float64)

def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())

def run(B=4, T=1000, C=512):
    from espnet_amd.arena import ParamArena
    from espnet_amd.layers import subsampling as S
    torch.manual_seed(0)
    sub = S.Conv2dSubsampling(80, C, 0.0)
    dev = torch.device("cuda", 0)
    arena = ParamArena(sub, dev, [], shadow_dtype=torch.bfloat16)
    sub.bind(arena, "", torch.bfloat16)
    sub._anchor = torch.zeros(1, device=dev, requires_grad=True)
    sub.train()
    g = torch.Generator().manual_seed(5)
    feats = torch.randn(B, T, 80, generator=g)
    T2 = ((T - 1) // 2 - 1) // 2
    gy = torch.randn(B, T2, C, generator=g)
    y = sub(feats.to(dev), 0)
    y.backward(gy.to(dev))
    torch.cuda.synchronize()
    gh = {k: p.grad.detach().double().cpu() for k, p in sub.named_parameters()}
    P = {k: p.detach().double().cpu() for k, p in sub.named_parameters()}
    x = feats.double().unsqueeze(1)
    W1, b1, W2, b2, Wl = P["conv.0.weight"], P["conv.0.bias"], P["conv.2.weight"], P["conv.2.bias"], P["out.0.weight"]
    xs = math.sqrt(C)
    torch.set_num_threads(16)
    for name, rx1, rw2, rx2, rdv, rdh in [("all", 1, 1, 1, 1, 1), ("no dh2 round", 1, 1, 1, 1, 0),
                                           ("no dv round", 1, 1, 1, 0, 1), ("no x2 round", 1, 1, 0, 1, 1),
                                           ("no x1 round", 0, 1, 1, 1, 1), ("no w2 round", 1, 0, 1, 1, 1)]:
        with torch.no_grad():
            x1 = torch.relu(F.conv2d(x, W1, b1, stride=2)); x1 = bf(x1) if rx1 else x1
            W2r = bf(W2) if rw2 else W2
            x2 = torch.relu(F.conv2d(x1, W2r, b2, stride=2)); x2 = bf(x2) if rx2 else x2
            Bn, _, T2_, F2 = x2.shape
            Wlr = bf(Wl)
            gs = gy.double() * xs
            dv = bf(gs) if rdv else gs
            dxr = (dv @ Wlr).reshape(Bn, T2_, C, F2).transpose(1, 2)
            dh2 = dxr * (x2 > 0); dh2 = bf(dh2) if rdh else dh2
            gb2 = dh2.sum((0, 2, 3))
            gw2 = torch.nn.grad.conv2d_weight(x1, W2.shape, dh2, stride=2)
        print(f"{name:14s} conv.2.bias {rel(gh['conv.2.bias'], gb2):.2e} conv.2.weight {rel(gh['conv.2.weight'], gw2):.2e}",
              flush=True)

run()
