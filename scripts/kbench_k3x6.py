"""Per-kernel timing of the cheng2020 k3 s1 x6 conv launches (the X6O conv_down) on the config-3 shard shapes:
q6 (N = 192), the 256x384 level of a 512x768 image, B images.  Interleaved rounds in one process; median ms and
TFLOP/s of the conv (the GDN gamma' GEMMs not counted).  Same --only / --dump / --cmp as scripts/kbench_x6.py:
    python scripts/kbench_k3x6.py [B] [--only substring] [--dump out.pt]
    python scripts/kbench_x6.py --cmp a.pt b.pt"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from imagecompression_adversarial_amd import hip_ops as K  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 32
only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else ""
N, H, W = 192, 256, 384
g = torch.Generator(device=dev).manual_seed(0)


def r(*shape):
    return torch.rand(shape, generator=g, device=dev) * 2 - 1


from imagecompression_adversarial_amd.engine_cheng import Conv3  # noqa: E402

gd = K.PackedGDN(torch.ones(N, device=dev) * 1.01, (0.1 * torch.eye(N, device=dev) + 0.001).sqrt())
cv = Conv3(r(N, N, 3, 3) * 0.02, r(N) * 0.1, 1, x6=True)
assert cv.fwd6 is not None and cv.bwd6 is not None
cv2 = Conv3(r(N, N, 3, 3) * 0.02, r(N) * 0.1, 2, x6=True)
assert cv2.fwd6 is not None


def nc4(lo, hi):
    return K.empty_nc4(B, N, H, W, dev).uniform_(lo, hi)


x, m, res = nc4(-1, 1), nc4(-1, 1), nc4(-1, 1)
sx, ss, a1 = nc4(0, 1), nc4(0.5, 1), nc4(-1, 1)
yg, s_, gs = nc4(0, 0), nc4(0, 0), nc4(0, 0)
flop = 2 * N * N * 9 * H * W * B
# the engine's launches (engine_cheng.py: ResidualBlock / WithStride / Upsample fwd and dgrad)
cases = {
    "k3 lrelu": lambda: cv.forward(x, K.EPI_LRELU),
    "k3 lrelu+res": lambda: cv.forward(x, K.EPI_LRELU, res=res, save_x=yg),
    "k3 gdn+res": lambda: cv.forward(x, K.EPI_GDN, gdn=gd, res=res, save_x=yg, save_s=s_),
    "k3 igdn+res": lambda: cv.forward(x, K.EPI_IGDN, gdn=gd, res=res, save_x=yg, save_s=s_),
    "k3 masked lrelu_bwd": lambda: cv.dgrad(x, K.EPI_LRELU_BWD, fill_mode=K.FILL_LRELU_MASK, mask=m, saved=(a1, None)),
    "k3 gdn_bwd": lambda: cv.dgrad(x, K.EPI_GDN_BWD, gdn=gd, res=res, save_x=gs, saved=(sx, ss)),
    "k3 igdn_bwd": lambda: cv.dgrad(x, K.EPI_IGDN_BWD, gdn=gd, res=res, save_x=gs, saved=(sx, ss)),
    # g_a.2 conv1: k3 stride 2 (256x384 -> 128x192), leaky ReLU (a quarter of the other cases' FLOPs)
    "k3s2 lrelu": lambda: cv2.forward(x, K.EPI_LRELU),
}
cases = {k: f for k, f in cases.items() if only in k}
times = {k: [] for k in cases}
for rnd in range(5):
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
    fl = flop / 4 if "s2" in k else flop
    print(f"{k:22s} {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TFLOP/s (conv only)", flush=True)
if "--dump" in sys.argv:
    dump = {}
    for k, f in cases.items():
        o = f()
        o = [t for t in o if isinstance(t, torch.Tensor)] if isinstance(o, tuple) else [o]
        # a fingerprint of the output bits (the full tensors are GBs): int32 sum and position-weighted sum
        fp = []
        for t in o:
            v = t.contiguous().view(torch.int32).reshape(-1).long()
            fp += [v.sum(), (v * torch.arange(v.numel(), device=v.device) % 1000003).sum()]
            del v
        dump[k] = torch.stack(fp).cpu()
    torch.save(dump, sys.argv[sys.argv.index("--dump") + 1])
