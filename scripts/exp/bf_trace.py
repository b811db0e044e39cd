"""Phase timing inside the bf16 conv kernels (s_memtime stamps per block and wave, ICA_BF_TRACE build) at the
config-5 shapes (hyper q3, 8 x 2048^2: level-1 1024^2 <-> level-2 512^2).

    python scripts/exp/bf_trace.py build [-Dflag]  # here (CPU): scripts/exp/libica_bftrace.so
    python scripts/exp/bf_trace.py run [case...]   # GPU box: median cycles per phase
conv_up stamps: 0 start, 1 after the LDS fill, 2 / 4 after class A / B main loop, 3 / 5 after their epilogues.
conv_down stamps: 0 start, 2 after the main loop (chunk fills included), 3 after the epilogue.
"""
import ctypes
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "imagecompression_adversarial_amd", "csrc")
LIB = os.path.join(HERE, os.environ.get("BF_TRACE_LIB", "libica_bftrace.so"))


def build(extra=()):
    obj = LIB[:-3] + ".o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-Wno-pass-failed", "-DICA_BF_TRACE", *extra, "-c", os.path.join(CSRC, "ica_conv.hip"),
                           "-o", obj])
    objs = [o for o in glob.glob(os.path.join(CSRC, "*.o")) if not o.endswith("ica_conv.o")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, obj] + objs)
    print("built", LIB)


def run(names):
    os.environ["ICA_HIP_LIB"] = LIB
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd._lib import lib
    dev = torch.device("cuda:0")
    B, N = 8, 128
    BF = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape):
        return torch.rand(shape, generator=g, device=dev) * 2 - 1
    gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
    wc = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "conv", 2, K.PREC_BF16)
    wd = K.PackedConv(r(N, N, 5, 5) * 0.02, r(N) * 0.1, "deconv", 2, K.PREC_BF16)
    L1, L2 = (1024, 1024), (512, 512)
    x1 = K.empty_nc4(B, N, *L1, dev, BF).uniform_(-1, 1)
    x2 = K.empty_nc4(B, N, *L2, dev, BF).uniform_(-1, 1)
    s1 = K.empty_nc4(B, N, *L1, dev, BF).uniform_(0.5, 1)
    s2 = K.empty_nc4(B, N, *L2, dev, BF).uniform_(0.5, 1)
    cases = {
        "down.bias": lambda: K.conv_down(x1, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS, prec=1),
        "down.gdn": lambda: K.conv_down(x1, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_GDN, gd, True, prec=1),
        "down.igdn_bwd": lambda: K.conv_down(x1, N, wd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd, saved=(x2, s2),
                                             prec=1),
        "up.bias": lambda: K.conv_up(x2, N, wd.fwd, wd.bias, N, K.EPI_BIAS, prec=1),
        "up.igdn": lambda: K.conv_up(x2, N, wd.fwd, wd.bias, N, K.EPI_IGDN, gd, True, prec=1),
        "up.gdn_bwd": lambda: K.conv_up(x2, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(x1, s1), prec=1),
    }
    L = lib()
    L.ica_bf_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.ica_bf_trace_clear.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(32768 * 4 * 8, dtype=np.uint64)  # first 32768 blocks
    for nm in names or list(cases):
        f = cases[nm]
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        buf[:] = 0
        assert L.ica_bf_trace_clear(buf.ctypes.data, buf.nbytes) == 0   # stamps of earlier cases must not survive
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        assert L.ica_bf_trace_read(buf.ctypes.data, buf.nbytes) == 0
        t = buf.reshape(32768, 4, 8).astype(np.int64)
        nb = int((t[:, 0, 0] != 0).sum())
        t = t[:nb]
        up = nm.startswith("up")
        ph = ([("fill", 0, 1), ("mainA", 1, 2), ("epiA", 2, 3), ("mainB", 3, 4), ("epiB", 4, 5)] if up
              else [("main", 0, 2), ("epi", 2, 3)])
        last = 5 if up else 3
        blk = t[:, :, last].max(1) - t[:, :, 0].min(1)
        # block residency: blocks started per CU-slot; total cycles x CUs / blocks = cycles between block starts
        span = t[:, :, last].max() - t[:, :, 0].min()
        line = [f"{nm:14s} {ms:6.3f} ms  blocks {nb}  block cycles med {np.median(blk):9.0f}  "
                f"span {span:.0f} cyc -> {span * 256 / max(nb, 1):.0f} CU-cycles per block"]
        for w in ((0, 1), (2, 3)) if up else ((0, 1, 2, 3),):
            parts = []
            for pn, a, bb in ph:
                d = t[:, list(w), bb] - t[:, list(w), a]
                parts.append(f"{pn} {np.median(d):8.0f}")
            line.append(f"  waves{w}: " + " ".join(parts))
        line.append(f"  block cycles p10 {np.percentile(blk, 10):.0f} p90 {np.percentile(blk, 90):.0f}")
        print("\n".join(line), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(sys.argv[2:])
