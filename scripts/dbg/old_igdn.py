# same check through the HEAD library (fp32 only: prec 0)
import os, sys
os.environ["ICA_HIP_LIB"] = os.path.abspath("scripts/dbg/libold.so")
sys.path.insert(0, ".")
import torch, torch.nn.functional as F
from oracle import codec
from imagecompression_adversarial_amd import _lib
for k in ("ica_pack_conv_weight_bf16", "ica_pack_gdn_bf16"):
    _lib._SIGS.pop(k)
class _CA(_lib.C.Structure):
    _fields_ = _lib.ConvArgs._fields_[:-1]
_lib.ConvArgs = _CA
from imagecompression_adversarial_amd import hip_ops as K
K.ConvArgs = _CA
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
gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
p = K.PackedConv(w.to(DEV), b.to(DEV), "deconv", 2)
y4, _, ss = K.conv_up(K.to_nc4(x.to(DEV)), C, p.fwd, p.bias, C, K.EPI_IGDN, gdn, True)
pre = F.conv_transpose2d(x, w, b, stride=2, padding=2, output_padding=1)
be, ge = codec.gdn_effective(beta, gamma)
s_ref = torch.sqrt(F.conv2d(pre ** 2, ge.reshape(C, C, 1, 1), be))
d = (K.from_nc4(ss, C).cpu() - s_ref).abs()
print("OLD lib: max diff", float(d.max()), "count>1e-3", int((d > 1e-3).sum()))

bad = torch.nonzero(d > 1e-3)
for dim, name in enumerate("nchw"):
    u = torch.unique(bad[:, dim])
    print("  ", name, u.tolist() if len(u) < 40 else (int(u.min()), int(u.max()), len(u)))
