"""Phase timing inside the x6 conv kernels (s_memtime stamps per block and wave, ICA_X6_TRACE build).

    python scripts/exp/x6_trace.py build [-Dflag]  # here (CPU): scripts/exp/libica_trace.so
    python scripts/exp/x6_trace.py run [case...]  # GPU box: median cycles per phase
conv_up stamps: 0 start, 1 after the LDS fill, 2 / 4 after class A / B main loop, 3 / 5 after their epilogues.
conv_down stamps: 0 start, 2 after the main loop, 3 after the epilogue.
"""
import ctypes
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "imagecompression_adversarial_amd", "csrc")
LIB = os.path.join(HERE, os.environ.get("X6_TRACE_LIB", "libica_trace.so"))


def build(extra=()):
    obj = LIB[:-3] + ".o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-DICA_X6_TRACE", *extra, "-c", os.path.join(CSRC, "ica_conv_x6.hip"), "-o", obj])
    objs = [o for o in glob.glob(os.path.join(CSRC, "*.o")) if not o.endswith("ica_conv_x6.o")]
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
    W3 = r(N, 3, 5, 5) * 0.1
    rc, rd = K.PackedConv(W3, b, "conv", 2, K.PREC_X6), K.PackedConv(W3, None, "deconv", 2, K.PREC_X6)
    x_rgb = K.empty_nc4(B, 3, 512, 768, dev).uniform_(0, 1)
    cases = {
        "rgb.gdn": lambda: K.conv_down(x_rgb, 3, rc.fwd, rc.bias, N, 5, 2, K.EPI_GDN, gd, save=True, prec=rc.fwd_prec),
        "rgb.igdn_bwd": lambda: K.conv_down(x_rgb, 3, rd.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, gd, saved=(sx_hi, ss_hi),
                                            prec=rd.bwd_prec),
        "down.bias": lambda: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_BIAS, prec=wc.fwd_prec),
        "down.gdn": lambda: K.conv_down(x_hi, N, wc.fwd, wc.bias, N, 5, 2, K.EPI_GDN, gd, save=True, prec=wc.fwd_prec),
        "up.bias": lambda: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_BIAS, prec=wd.fwd_prec),
        "up.igdn": lambda: K.conv_up(x_lo, N, wd.fwd, wd.bias, N, K.EPI_IGDN, gd, save=True, prec=wd.fwd_prec),
        "up.gdn_bwd": lambda: K.conv_up(x_lo, N, wc.bwd, None, N, K.EPI_GDN_BWD, gd, saved=(sx_hi, ss_hi),
                                        prec=wc.bwd_prec),
    }
    L = lib()
    L.ica_x6_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.ica_x6_trace_clear.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(32768 * 4 * 8, dtype=np.uint64)  # first 32768 blocks
    for nm in names or list(cases):
        f = cases[nm]
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        buf[:] = 0
        assert L.ica_x6_trace_clear(buf.ctypes.data, buf.nbytes) == 0   # stamps of earlier cases must not survive
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        assert L.ica_x6_trace_read(buf.ctypes.data, buf.nbytes) == 0
        t = buf.reshape(32768, 4, 8).astype(np.int64)
        nb = int((t[:, 0, 0] != 0).sum())
        t = t[:nb]
        up = nm.startswith("up")
        ph = ([("fill", 0, 1), ("mainA", 1, 2), ("epiA", 2, 3), ("mainB", 3, 4), ("epiB", 4, 5)] if up
              else [("fill", 0, 1), ("main", 1, 2), ("epi", 2, 3)] if nm.startswith("rgb")
              else [("main", 0, 2), ("epi", 2, 3)])
        last = 5 if up else 3
        blk = t[:, :, last].max(1) - t[:, :, 0].min(1)
        line = [f"{nm:11s} {ms:6.3f} ms  blocks {nb}  block cycles med {np.median(blk):9.0f}"]
        for w in ((0, 1), (2, 3)) if up else ((0, 1, 2, 3),):
            parts = []
            for pn, a, bb in ph:
                d = t[:, list(w), bb] - t[:, list(w), a]
                parts.append(f"{pn} {np.median(d):8.0f}")
            line.append(f"  waves{w}: " + " ".join(parts))
        # start-to-start spacing of consecutive blocks on the same CU is not observable; report the spread of
        # block durations instead
        line.append(f"  block cycles p10 {np.percentile(blk, 10):.0f} p90 {np.percentile(blk, 90):.0f}")
        print("\n".join(line), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])   # extra hipcc flags, e.g. -DICA_X6_DENSE
    else:
        run(sys.argv[2:])
