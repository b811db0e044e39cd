"""Per-kernel timing of the k5 s2 conv launches on the bench shapes (hyper q3, 512x768, B=32), fp32-MFMA vs the
fp32-accurate bf16x6 kernels.  Interleaved rounds in one process; median ms and TFLOP/s.
    python scripts/kbench_x6.py [B] [--only substring] [--dump out.pt]
--dump saves every case's output (one more call) so that two libraries (ICA_HIP_LIB) can be compared bit for bit:
    python scripts/kbench_x6.py --cmp a.pt b.pt"""
import statistics
import sys

import torch

if "--cmp" in sys.argv:
    a, b = (torch.load(f, weights_only=True) for f in sys.argv[sys.argv.index("--cmp") + 1:][:2])
    bad = 0
    for k in a:
        if k in b:
            same = torch.equal(a[k], b[k])
            bad += not same
            print(f"{k:22s} {'identical' if same else 'DIFFERENT max|d|=%.3g' % float((a[k] - b[k]).abs().max())}")
    sys.exit(1 if bad else 0)
sys.path.insert(0, ".")
from imagecompression_adversarial_amd import hip_ops as K  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)   # the activation / saved-tensor inputs come from the default generator: same bits per process
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 32
only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else ""
N = 128
g = torch.Generator(device=dev).manual_seed(0)


def r(*shape):
    return torch.rand(shape, generator=g, device=dev) * 2 - 1


gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
W1, W2, b = r(N, N, 5, 5) * 0.02, r(N, N, 5, 5) * 0.02, r(N) * 0.1
P = {pr: (K.PackedConv(W1, b, "conv", 2, pr), K.PackedConv(W2, b, "deconv", 2, pr)) for pr in (K.PREC_FP32, K.PREC_X6)}
x_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(-1, 1)
x_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(-1, 1)
sx_hi, ss_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(0, 1), K.empty_nc4(B, N, 256, 384, dev).uniform_(0.5, 1)
sx_lo, ss_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(0, 1), K.empty_nc4(B, N, 128, 192, dev).uniform_(0.5, 1)
flop = 2 * N * N * 25 * 128 * 192 * B
cases = {}
for pr, nm in ((K.PREC_FP32, "fp32"), (K.PREC_X6, "x6")):
    wc, wd = P[pr]
    cases.update({
        f"{nm} down.bias": lambda wc=wc, pr=pr: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS, prec=wc.fwd_prec),
        f"{nm} down.gdn(save)": lambda wc=wc: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_GDN, gd, save=True,
                                                        prec=wc.fwd_prec),
        f"{nm} down.igdn_bwd": lambda wd=wd: K.conv_down(x_hi, N, wd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd,
                                                       saved=(sx_lo, ss_lo), prec=wd.bwd_prec),
        f"{nm} up.bias": lambda wd=wd: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_BIAS, prec=wd.fwd_prec),
        f"{nm} up.igdn(save)": lambda wd=wd: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_IGDN, gd, save=True,
                                                     prec=wd.fwd_prec),
        f"{nm} up.gdn_bwd": lambda wc=wc: K.conv_up(x_lo, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(sx_hi, ss_hi),
                                                  prec=wc.bwd_prec),
    })
W3 = r(N, 3, 5, 5) * 0.1
R = {pr: (K.PackedConv(W3, b, "conv", 2, pr), K.PackedConv(W3, None, "deconv", 2, pr)) for pr in (K.PREC_FP32, K.PREC_X6)}
x_rgb = K.empty_nc4(B, 3, 512, 768, dev).uniform_(0, 1)
flop_rgb = 2 * N * 3 * 25 * 256 * 384 * B
for pr, nm in ((K.PREC_FP32, "fp32"), (K.PREC_X6, "x6")):
    rc, rd = R[pr]
    cases.update({
        f"{nm} rgb.gdn(save)": lambda rc=rc: K.conv_down(x_rgb, 3, rc.fwd, rc.bias, N, 5, 2, K.EPI_GDN, gd, save=True,
                                                       prec=rc.fwd_prec),
        f"{nm} rgb.igdn_bwd": lambda rd=rd: K.conv_down(x_rgb, 3, rd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd,
                                                      saved=(sx_hi, ss_hi), prec=rd.bwd_prec),
    })
U3 = {pr: K.PackedConv(W3, b[:3].contiguous(), "deconv", 2, pr) for pr in (K.PREC_FP32, K.PREC_X6)}
for pr, nm in ((K.PREC_FP32, "fp32"), (K.PREC_X6, "x6")):
    cases[f"{nm} up3.bias"] = lambda u=U3[pr]: K.conv_up(x_hi, N, u.fwd, u.bias, 3, K.EPI_BIAS, prec=u.fwd_prec)
cases = {k: f for k, f in cases.items() if only in k}
times = {k: [] for k in cases}
for rnd in range(6):
    for k, f in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = f()
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            times[k].append(e0.elapsed_time(e1))
        del out
for k, v in times.items():
    ms = statistics.median(v)
    fl = flop_rgb if ("rgb" in k or "up3" in k) else flop
    print(f"{k:22s} {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TFLOP/s (conv only)", flush=True)
if "--dump" in sys.argv:
    res = {}
    for k, f in cases.items():
        o = f()
        o = [t for t in o if isinstance(t, torch.Tensor)] if isinstance(o, tuple) else [o]
        res[k] = torch.cat([t.float().reshape(-1).cpu() for t in o])
    torch.save(res, sys.argv[sys.argv.index("--dump") + 1])
