"""Which x6 launch of the cheng2020 backward carries the input-gradient error (seed 34, 2 x 64x64, random output
gradient): every x6 pack disabled, then the x6 input gradient (bwd6) or forward (fwd6) of one layer at a time
enabled; each line is the input gradient's max abs error / max against float64.  GPU box:
    python scripts/cheng_x6_layer_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import codec as oc           # noqa: E402  (checker only)
from imagecompression_adversarial_amd import hip_ops as K                      # noqa: E402
from imagecompression_adversarial_amd.engine_cheng import ChengKernels, Conv3, Subpel   # noqa: E402

DEV = torch.device("cuda:0")
P = oc.perturb_params(oc.init_params("cheng2020", 6, seed=0), seed=1)
P64 = {k: v.double() for k, v in P.items()}
g = torch.Generator().manual_seed(34)
x = torch.rand((2, 3, 64, 64), generator=g)
xr = x.double().requires_grad_(True)
xhr = oc.transforms(P64, xr, "cheng2020")
gout = torch.rand(xhr.shape, generator=torch.Generator().manual_seed(31), dtype=torch.float64) * 2 - 1
xhr.backward(gout)
kern = ChengKernels({k: v.to(DEV) for k, v in P.items()}, precision="x6")


def layers(obj, path, seen):
    if id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, (Conv3, Subpel)):
        yield path, obj
        return
    if isinstance(obj, (list, tuple)):
        for i, o in enumerate(obj):
            yield from layers(o, f"{path}[{i}]", seen)
    elif hasattr(obj, "__dict__") and type(obj).__module__.startswith("imagecompression"):
        for k, o in vars(obj).items():
            yield from layers(o, f"{path}.{k}", seen)


L = list(layers(kern, "kern", set()))
packs = {p: (l.fwd6, l.bwd6) for p, l in L}
for p, l in L:
    l.fwd6 = l.bwd6 = None


def run():
    y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
    xh4, ss = kern.g_s(y4, save=True)
    gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4(gout.float().to(DEV)), ss), sa)
    gx = K.from_nc4(gx4, 3).double().cpu()
    return float((gx - xr.grad).abs().max() / xr.grad.abs().max())


print(f"all fp32: {run():.2e}", flush=True)


def enable(pred):
    for p, l in L:
        f6, b6 = packs[p]
        l.fwd6 = f6 if pred(p, "fwd6") else None
        l.bwd6 = b6 if pred(p, "bwd6") else None


groups = {
    "all": lambda p, n: True,
    "g_a only": lambda p, n: ".ga." in p,
    "g_s only": lambda p, n: ".gs." in p,
    "fwd6 only": lambda p, n: n == "fwd6",
    "bwd6 only": lambda p, n: n == "bwd6",
    "g_s fwd6": lambda p, n: ".gs." in p and n == "fwd6",
    "g_s bwd6": lambda p, n: ".gs." in p and n == "bwd6",
    "g_a fwd6": lambda p, n: ".ga." in p and n == "fwd6",
    "g_a bwd6": lambda p, n: ".ga." in p and n == "bwd6",
}
for name, pred in groups.items():
    enable(pred)
    print(f"{name}: {run():.2e}", flush=True)
# cumulative: layers switched on one by one in order
enable(lambda p, n: False)
for p, l in L:
    f6, b6 = packs[p]
    l.fwd6, l.bwd6 = f6, b6
    print(f"+ {p}: {run():.2e}", flush=True)
