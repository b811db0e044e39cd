"""Per-kernel timing of the bf16 conv kernels at BASELINE config-5 shapes (hyper q3, 8 x 2048x2048):
level-1 (1024^2) <-> level-2 (512^2) layers and the RGB ends.  Median of 7 launches (HIP events, launch
stream), printed with algorithmic TFLOP/s and the HBM bytes of the activation tensors they move.
    python scripts/kbench_bf16.py [lib path] [--only name-substring]"""
import os
import sys

ONLY = None
args = sys.argv[1:]
if "--only" in args:
    i = args.index("--only")
    ONLY = args[i + 1]
    del args[i:i + 2]
if args:
    os.environ["ICA_HIP_LIB"] = os.path.abspath(args[0])
sys.path.insert(0, ".")
import torch  # noqa: E402

from imagecompression_adversarial_amd import hip_ops as K  # noqa: E402

dev = torch.device("cuda:0")
B, N = 8, 128
g = torch.Generator(device=dev).manual_seed(0)
BF = torch.bfloat16


def r(*shape):
    return torch.rand(shape, generator=g, device=dev) * 2 - 1


gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
wc = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "conv", 2, K.PREC_BF16)
wd = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "deconv", 2, K.PREC_BF16)
w0 = K.PackedConv(r(N, 3, 5, 5) * 0.1, r(N) * 0.1, "conv", 2, K.PREC_BF16)        # g_a.0
w6 = K.PackedConv(r(N, 3, 5, 5) * 0.05, r(3) * 0.1, "deconv", 2, K.PREC_BF16)     # g_s.6
L1, L2 = (1024, 1024), (512, 512)
x1 = K.empty_nc4(B, N, *L1, dev, BF).uniform_(-1, 1)
x2 = K.empty_nc4(B, N, *L2, dev, BF).uniform_(-1, 1)
s1 = K.empty_nc4(B, N, *L1, dev, BF).uniform_(0.5, 1)
s2 = K.empty_nc4(B, N, *L2, dev, BF).uniform_(0.5, 1)
img = K.empty_nc4(B, 3, 2048, 2048, dev).uniform_(0, 1)
img[:, :, :, :, 3] = 0
FL = 2.0 * N * N * 25 * 512 * 512 * B            # level-1 <-> level-2 conv
FL0 = 2.0 * N * 3 * 25 * 1024 * 1024 * B         # RGB <-> level-1
cases = {
    "down_gdn   (g_a.2.fwd)": (lambda: K.conv_down(x1, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_GDN, gd, True, prec=1), FL),
    "down_bias  (no GDN)": (lambda: K.conv_down(x1, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS, prec=1), FL),
    "down_igdnb (g_s.4.dgrad)": (lambda: K.conv_down(x1, N, wd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd,
                                                      saved=(x2, s2), prec=1), FL),
    "up_igdn    (g_s.4.fwd)": (lambda: K.conv_up(x2, N, wd.fwd, wd.bias, N, K.EPI_IGDN, gd, True, prec=1), FL),
    "up_bias    (no GDN)": (lambda: K.conv_up(x2, N, wd.fwd, wd.bias, N, K.EPI_BIAS, prec=1), FL),
    "up_gdnb    (g_a.2.dgrad)": (lambda: K.conv_up(x2, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(x1, s1),
                                                    prec=1), FL),
    "rgb_gdn    (g_a.0.fwd)": (lambda: K.conv_down(img, 3, w0.fwd, w0.bias, N, 5, 2, K.EPI_GDN, gd, True, prec=1), FL0),
    "rgb_igdnb  (g_s.6.dgrad)": (lambda: K.conv_down(img, 3, w6.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd,
                                                      saved=(x1, s1), prec=1), FL0),
    "up3        (g_s.6.fwd)": (lambda: K.conv_up(x1, N, w6.fwd, w6.bias, 3, prec=1), FL0),
}
for name, (fn, fl) in cases.items():
    if ONLY and ONLY not in name:
        continue
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts)[3]
    print(f"{name:26s} {t:7.3f} ms  {fl / t / 1e9:7.1f} TFLOP/s", flush=True)
