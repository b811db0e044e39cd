"""Where the step-0 attack gradient of the cheng2020 HIP paths departs from float64 (seed 34, 2 x 64x64):
output_s (eval forward), x_ = g_s(g_a(im_s)), the loss gradient d = out_s - clamp(x_) and the input gradient,
each as max abs error / max abs value against the float64 oracle.  GPU box:
    python scripts/cheng_grad_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import codec as oc           # noqa: E402  (checker only)
from imagecompression_adversarial_amd import hip_ops as K                      # noqa: E402
from imagecompression_adversarial_amd.attack import AttackLoop                 # noqa: E402
from imagecompression_adversarial_amd.engine_cheng import ChengKernels        # noqa: E402

DEV = torch.device("cuda:0")
P = oc.perturb_params(oc.init_params("cheng2020", 6, seed=0), seed=1)
P64 = {k: v.double() for k, v in P.items()}
g = torch.Generator().manual_seed(34)
x = torch.rand((2, 3, 64, 64), generator=g)
x64 = x.double().requires_grad_(True)
with torch.no_grad():
    out_s64 = oc.forward(P64, x.double(), "cheng2020")["x_hat"].clamp(0, 1)
xh64 = oc.transforms(P64, x64, "cheng2020")
d64 = (out_s64 - xh64.clamp(0, 1)).detach()
(1.0 - ((out_s64 - oc.bound01(xh64)) ** 2).flatten(1).mean(1)).sum().backward()
gx64 = x64.grad


def err(a, ref):
    return float((a.double().cpu() - ref).abs().max() / ref.abs().max())


print(f"float64: max|d| {float(d64.abs().max()):.3e}, median |d| {float(d64.abs().median()):.3e}, "
      f"max|grad| {float(gx64.abs().max()):.3e}")
for pr in ("fp32", "x6"):
    kern = ChengKernels({k: v.to(DEV) for k, v in P.items()}, precision=pr)
    loop = AttackLoop(kern, x.to(DEV), steps=1, noise_thr=1e-5)
    im4 = K.to_nc4(x.to(DEV))
    y4, sa = kern.g_a(im4, save=True)
    xh4, ss = kern.g_s(y4, save=True)
    xh = K.from_nc4(xh4, 3)
    d = loop.output_s - xh.clamp(0, 1)
    loop.noise.zero_()
    loop.step(0)
    gx = K.from_nc4(loop.network_grad(), 3)   # im_in4 of step 0 (noise 0): im_s
    scale = float(gx64.abs().max() / gx.abs().max())
    print(f"{pr}: output_s {err(loop.output_s, out_s64):.2e}  x_ {err(xh, xh64.detach()):.2e}  "
          f"d {err(d, d64):.2e}  input grad {err(gx * scale, gx64):.2e} (scale {scale:.4e})", flush=True)

# the same input gradient under a random output gradient at three scales (the attack's is ~1e-7 per element)
xr = x.double().requires_grad_(True)
xhr = oc.transforms(P64, xr, "cheng2020")
gg = torch.Generator().manual_seed(31)
gout = torch.rand(xhr.shape, generator=gg, dtype=torch.float64) * 2 - 1
xhr.backward(gout)
for pr in ("fp32", "x6"):
    kern = ChengKernels({k: v.to(DEV) for k, v in P.items()}, precision=pr)
    line = []
    for sc in (1.0, 1e-4, 1e-7, 1e-10):
        y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
        xh4, ss = kern.g_s(y4, save=True)
        gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4((gout * sc).float().to(DEV)), ss), sa)
        line.append(f"scale {sc:.0e}: {err(K.from_nc4(gx4, 3) / sc, xr.grad):.2e}")
    print(pr, " ".join(line), flush=True)
