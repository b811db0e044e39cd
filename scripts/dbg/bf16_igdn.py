import sys
sys.path.insert(0, ".")
import torch, torch.nn.functional as F
from oracle import codec
from imagecompression_adversarial_amd import hip_ops as K
DEV = torch.device("cuda:0")
def rnd(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo
C, H, W = 128, 16, 24
x = rnd((2, C, H, W), 11)
beta = rnd((C,), 12, 0.5, 1.5)
gamma = (0.1 * torch.eye(C) + 0.02 * rnd((C, C), 13, 0, 1)).reshape(C, C, 1, 1)
w = rnd((C, C, 5, 5), 14) * (1.0 / (C * 25) ** 0.5)
b = rnd((C,), 15) * 0.1
for prec in (0, 1):
    gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
    p = K.PackedConv(w.to(DEV), b.to(DEV), "deconv", 2, prec)
    y4, _, ss = K.conv_up(K.to_nc4(x.to(DEV)), C, p.fwd, p.bias, C, K.EPI_IGDN, gdn, True, prec=p.fwd_prec)
    xx = x.bfloat16().float() if prec else x
    ww = w.bfloat16().float() if prec else w
    pre = F.conv_transpose2d(xx, ww, b, stride=2, padding=2, output_padding=1)
    be, ge = codec.gdn_effective(beta, gamma)
    norm = F.conv2d(pre ** 2, ge.reshape(C, C, 1, 1), be)
    s_ref = torch.sqrt(norm)
    s = K.from_nc4(ss, C).cpu()
    d = (s - s_ref).abs()
    print("prec", prec, "max diff", float(d.max()), "argmax", [int(v) for v in torch.nonzero(d == d.max())[0]], "count>1e-3", int((d > 1e-3).sum()), "of", d.numel())
    bad = torch.nonzero(d > 1e-3)
    print(" bad rows sample", bad[:10].tolist())
    print(" y err", float((K.from_nc4(y4, C).cpu() - pre * s_ref).abs().max()))
    for dim, name in enumerate("nchw"):
        u = torch.unique(bad[:, dim])
        print("  ", name, u.tolist() if len(u) < 40 else (int(u.min()), int(u.max()), len(u)))
