"""Per-kernel ablation timing on the bench shapes (hyper q3, 512x768, B=32): main loop vs epilogues.
Interleaved rounds in one process (cdna_hip_programming.md rule 24); prints median ms and TFLOP/s."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from imagecompression_adversarial_amd import hip_ops as K  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
N = 128
g = torch.Generator(device=dev).manual_seed(0)


def r(*shape):
    return torch.rand(shape, generator=g, device=dev) * 2 - 1


gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
wc = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "conv", 2)
wd = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "deconv", 2)
x_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(-1, 1)   # level-1 activations
x_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(-1, 1)   # level-2 activations
sx_hi, ss_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(0, 1), K.empty_nc4(B, N, 256, 384, dev).uniform_(0.5, 1)
sx_lo, ss_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(0, 1), K.empty_nc4(B, N, 128, 192, dev).uniform_(0.5, 1)

flop_down = 2 * N * N * 25 * 128 * 192 * B
flop_up = 2 * N * N * 25 * 128 * 192 * B
cases = {
    "down.bias": lambda: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS),
    "down.gdn(save)": lambda: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_GDN, gd, save=True),
    "down.igdn_bwd": lambda: K.conv_down(x_hi, N, wd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd, saved=(sx_lo, ss_lo)),
    "up.bias": lambda: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_BIAS),
    "up.igdn(save)": lambda: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_IGDN, gd, save=True),
    "up.gdn_bwd": lambda: K.conv_up(x_lo, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(sx_hi, ss_hi)),
}
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
    fl = flop_down if k.startswith("down") else flop_up
    print(f"{k:18s} {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TFLOP/s (conv only)")
