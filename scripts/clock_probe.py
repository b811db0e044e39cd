"""In-kernel clock of the x6 k5 conv kernels at the config-2 shapes (MI355X_MICROARCH.md, DVFS give-back item 6).

Needs a diagnostic library built with -DICA_CLOCK_STAMP (the product library has no stamps):
    bash scripts/build_variant.sh clk imagecompression_adversarial_amd/csrc/ica_conv_x6.hip \
         imagecompression_adversarial_amd/csrc/ica_conv_x6.hip -DICA_CLOCK_STAMP
    ICA_HIP_LIB=scripts/variants/libclk.so python scripts/clock_probe.py [--only substr] [--secs 2.5]
Per case: >= --secs seconds of back-to-back launches on random data, then one stamped launch; per block (wave 0)
clock = d(s_memtime) / d(s_memrealtime) * 100 MHz, the block's wall time in cycles, and the kernel's MFMA-cycle
demand per SIMD against its stamped duration (the MFMA issue fraction the clock leaves)."""
import ctypes
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from imagecompression_adversarial_amd import hip_ops as K   # noqa: E402
from imagecompression_adversarial_amd._lib import lib       # noqa: E402

dev = torch.device("cuda:0")
only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else ""
secs = float(sys.argv[sys.argv.index("--secs") + 1]) if "--secs" in sys.argv else 2.5
B, N = 32, 128
g = torch.Generator(device=dev).manual_seed(0)


def r(*shape):
    return torch.rand(shape, generator=g, device=dev) * 2 - 1


gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
W1, W2, b = r(N, N, 5, 5) * 0.02, r(N, N, 5, 5) * 0.02, r(N) * 0.1
wc, wd = K.PackedConv(W1, b, "conv", 2, K.PREC_X6), K.PackedConv(W2, b, "deconv", 2, K.PREC_X6)
x_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(-1, 1)
x_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(-1, 1)
sx_hi, ss_hi = K.empty_nc4(B, N, 256, 384, dev).uniform_(0, 1), K.empty_nc4(B, N, 256, 384, dev).uniform_(0.5, 1)
sx_lo, ss_lo = K.empty_nc4(B, N, 128, 192, dev).uniform_(0, 1), K.empty_nc4(B, N, 128, 192, dev).uniform_(0.5, 1)
flop = 2 * N * N * 25 * 128 * 192 * B           # conv MACs x 2 per launch
gflop = 2 * N * N * 256 * 384 * B               # the fused gamma' GEMM of a GDN epilogue
# x6 MFMA cycles per launch summed over SIMDs: 6 bf16 32x32x16 MFMAs (32 cycles each) per 32x32x16 fp32-equivalent
mfma_cycles = lambda fl: fl / (2 * 32 * 32 * 16) * 6 * 32   # noqa: E731
cases = {
    "down.bias (conv_down_x6w)": (lambda: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS, prec=wc.fwd_prec),
                                  flop),
    "down.igdn_bwd (conv_down_x6w)": (lambda: K.conv_down(x_hi, N, wd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd,
                                                          saved=(sx_lo, ss_lo), prec=wd.bwd_prec), flop + gflop // 4),
    "up.bias (conv_up_x6w)": (lambda: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_BIAS, prec=wd.fwd_prec), flop),
    "up.gdn_bwd": (lambda: K.conv_up(x_lo, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(sx_hi, ss_hi),
                                     prec=wc.bwd_prec), flop + gflop),
}
if "--bf16" in sys.argv:   # config-5 shapes (8 x 2048^2: level 1 = 1024^2), bf16 kernels of ica_conv.hip (a
    # -DICA_CLOCK_STAMP build of ica_conv.hip; phases: class A main / epilogue, class B main / epilogue)
    BFT = torch.bfloat16
    wcb = K.PackedConv(W1, b, "conv", 2, K.PREC_BF16)
    x2b = K.empty_nc4(8, N, 512, 512, dev, BFT).uniform_(-1, 1)
    y1b, s1b = K.empty_nc4(8, N, 1024, 1024, dev, BFT).uniform_(-1, 1), K.empty_nc4(8, N, 1024, 1024, dev, BFT).uniform_(0.5, 1)
    fl5 = 2 * N * N * 25 * 512 * 512 * 8
    cases = {"bf16 up.gdn_bwd 4w (config 5)": (lambda: K.conv_up(x2b, N, wcb.bwd, None, N, K.EPI_GDN_BWD, gd,
                                                                  saved=(y1b, s1b), prec=1),
                                               fl5 + 2 * N * N * 1024 * 1024 * 8)}
    mfma_cycles = lambda fl: fl / (2 * 32 * 32 * 16) * 32   # noqa: E731  (one bf16 MFMA per 32x32x16)
cases = {k: v for k, v in cases.items() if only in k}
L = lib()
L.ica_diag_stamp_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint]
L.ica_diag_stamp_buffer.restype = ctypes.c_int
slots = 1 << 16
buf = torch.zeros(slots * 16, dtype=torch.int64, device=dev)
n_simd = torch.cuda.get_device_properties(dev).multi_processor_count * 4
for name, (f, fl) in cases.items():
    assert L.ica_diag_stamp_buffer(None, 0) == 0
    t0, n = time.perf_counter(), 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            f()
        n += 20
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    buf.zero_()
    assert L.ica_diag_stamp_buffer(ctypes.c_void_p(buf.data_ptr()), slots) == 0
    f()
    torch.cuda.synchronize()
    assert L.ica_diag_stamp_buffer(None, 0) == 0
    st16 = buf.view(-1, 16).cpu()
    st16 = st16[st16[:, 7] > 0]
    st = st16[:, :8]
    st = st[st[:, 7] > 0]
    dt, dr = (st[:, 6] - st[:, 0]).double(), (st[:, 7] - st[:, 1]).double()
    clk = (dt / dr * 100.0).tolist()            # MHz
    span_r = float(st[:, 7].max() - st[:, 1].min())   # first entry .. last exit, 100 MHz ticks
    clk_med = statistics.median(clk)
    cyc = span_r / 100e6 * clk_med * 1e6          # kernel span in shader cycles at the median clock
    busy = mfma_cycles(fl) / n_simd / cyc
    q = statistics.quantiles(clk, n=10)
    print(f"{name:34s} {ms:6.3f} ms/launch ({n} launches, {fl / ms / 1e9:6.1f} TFLOP/s)  clock median "
          f"{clk_med:6.0f} MHz (p10 {q[0]:.0f}, p90 {q[-1]:.0f}) over {len(clk)} blocks; stamped span "
          f"{span_r / 100:.0f} us; MFMA issue fraction {busy:.3f}; median block {statistics.median(dt.tolist()):.0f} "
          "cycles", flush=True)
    ph = st[:, 2:6]
    if bool((ph > 0).all()):
        marks = torch.cat([st[:, :1], ph, st[:, 6:7]], 1).double()
        d = (marks[:, 1:] - marks[:, :-1]).median(0).values.tolist()
        # conv_up_x6 (4 waves): class A main / epilogue, class B main / epilogue; conv_up_x6w GDN backward: main
        # loop, block barrier, epilogue of pixel tile 0, of pixel tile 1
        lab = (("fill+main A", "epilogue A", "main B", "epilogue B", "tail") if "4w" in name else
               ("fill+main", "barrier", "epilogue t0", "epilogue t1", "tail"))
        mean = (marks[:, 1:] - marks[:, :-1]).mean(0).tolist()
        print("    wave-0 phases (median / mean cycles): " + ", ".join(
            f"{k} {v:.0f} / {m:.0f}" for k, v, m in zip(lab, d, mean)), flush=True)
    print(f"    block cycles mean {float(dt.mean()):.0f}, p90 {float(dt.quantile(0.9)):.0f}", flush=True)
    wv = st16[:, 8:16]
    if bool((wv > 0).any()):
        rel = (wv - st16[:, :1]).double()
        rel[wv == 0] = float("nan")
        med = [float(rel[:, w][~rel[:, w].isnan()].median()) if bool((~rel[:, w].isnan()).any()) else float("nan")
               for w in range(8)]
        print("    per-wave stamp (median cycles after block entry): " + ", ".join(f"w{w} {m:.0f}" for w, m in
                                                                               enumerate(med)), flush=True)
