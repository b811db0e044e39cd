"""Accuracy diagnostics against float64 (GPU box; the oracle is only the checker here).

    python scripts/accuracy_diag.py cheng      # cheng2020 q6 g_a+g_s input gradient at 512x768: x6 / fp32 HIP /
                                               # fp32 oracle, each vs the float64 oracle
    python scripts/accuracy_diag.py t100b      # hyper q1 (traj100 t100b weights): the attack's network gradient at
                                               # the reference trajectory's step-9 / 24 / 49 states, same comparison,
                                               # and the Adam direction m/sqrt(v) sensitivity it implies

Prints, per path: max |err| / max|ref|, the 99.99 % quantile of that ratio, how many elements exceed 1e-4 of the
max, and where the largest error sits (so a localized difference -- a leaky-ReLU kink or a rounding tie -- is told
apart from a uniform one)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import codec  # noqa: E402  (checker only)
from imagecompression_adversarial_amd import hip_ops as K  # noqa: E402

DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def report(name, got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    d = (got - ref).abs() / ref.abs().max()
    flat = d.flatten()
    i = int(flat.argmax())
    idx = np.unravel_index(i, tuple(d.shape))
    print(f"  {name:10s} max {float(flat.max()):.3e}  p99.99 {float(torch.quantile(flat[::7].float(), 0.9999)):.3e}  "
          f"n>1e-4 {int((flat > 1e-4).sum())}/{flat.numel()}  argmax {idx}  ref there {float(ref[idx]):.3e}", flush=True)


def cheng():
    from imagecompression_adversarial_amd.engine_cheng import ChengKernels
    torch.set_num_threads(16)
    H, W = 512, 768
    P = codec.perturb_params(codec.init_params("cheng2020", 6, seed=0), seed=1)
    x = rnd((1, 3, H, W), 48)
    gout = None
    res = {}
    for prec in ("x6", "fp32"):
        kern = ChengKernels({k: v.to(DEV) for k, v in P.items()}, precision=prec)
        y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
        xh4, ss = kern.g_s(y4, save=True)
        if gout is None:
            gout = rnd(K.from_nc4(xh4, 3).shape, 49, -1, 1)
        gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4(gout.to(DEV)), ss), sa)
        res[prec] = (K.from_nc4(y4, 192).cpu(), K.from_nc4(xh4, 3).cpu(), K.from_nc4(gx4, 3).cpu())
        del kern
    for dt in (torch.float32, torch.float64):
        Pd = {k: v.to(dt) for k, v in P.items()}
        xr = x.to(dt).clone().requires_grad_(True)
        yr = codec.cheng_g_a(Pd, xr)
        xhr = codec.cheng_g_s(Pd, yr)
        xhr.backward(gout.to(dt))
        res["oracle32" if dt == torch.float32 else "f64"] = (yr.detach(), xhr.detach(), xr.grad)
    for k, name in enumerate(("y", "x_hat", "input grad")):
        print(name)
        for path in ("x6", "fp32", "oracle32"):
            report(path, res[path][k], res["f64"][k])
        report("x6-vs-o32", res["x6"][k], res["oracle32"][k])


def t100b():
    from imagecompression_adversarial_amd.attack import AttackLoop
    from imagecompression_adversarial_amd.engine import CodecKernels
    torch.set_num_threads(16)
    t100 = np.load(os.path.join(REPO, "tests", "golden", "traj100.npz"))
    snap = np.load(os.path.join(REPO, "tests", "golden", "traj100_snap.npz"))
    P = codec.perturb_params(codec.init_params("hyper", 1, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * float(t100["t100b_scale"])
    xs = rnd((1, 3, 256, 256), 101)
    os_ = torch.from_numpy(t100["t100b_output_s"])
    eps = 16 / 255.0
    for k, step in enumerate(int(v) for v in snap["snap_steps"]):
        noise = torch.from_numpy(snap["t100b_snap"][k])
        im_in = torch.clamp(xs + torch.clamp(noise, -eps, eps), 0, 1)
        grads = {}
        for prec in ("x6", "fp32"):
            kern = CodecKernels({kk: v.to(DEV) for kk, v in P.items()}, "hyper", precision=prec)
            loop = AttackLoop(kern, xs.to(DEV), steps=1)
            loop.output_s.copy_(os_.to(DEV))
            loop.noise.copy_(noise.to(DEV))
            call_prologue(loop)
            g4 = loop.network_grad()
            grads[prec] = K.from_nc4(g4, 3).cpu()
        for dt in (torch.float32, torch.float64):
            Pd = {kk: v.to(dt) for kk, v in P.items()}
            xi = im_in.to(dt).clone().requires_grad_(True)
            o = codec.bound01(codec.g_s(Pd, codec.g_a(Pd, xi)), 0.0, 1.0)
            loss = 1.0 - torch.mean((os_.to(dt) - o) * (os_.to(dt) - o))
            loss.backward()
            grads["oracle32" if dt == torch.float32 else "f64"] = xi.grad
        print(f"t100b network gradient at the reference state after step {step}")
        for path in ("x6", "fp32", "oracle32"):
            report(path, grads[path], grads["f64"])
        g64 = grads["f64"].abs()
        print(f"  |g| quantiles (of max): p1 {float(torch.quantile((g64 / g64.max()).flatten(), 0.01)):.2e} "
              f"p10 {float(torch.quantile((g64 / g64.max()).flatten(), 0.1)):.2e}", flush=True)


def call_prologue(loop):
    from imagecompression_adversarial_amd._lib import call, ptr, stream
    call("ica_attack_prologue", ptr(loop.noise), ptr(loop.im_s), ptr(loop.im_in4), ptr(loop.part), loop.B, loop.H,
         loop.W, loop.eps, stream())


if __name__ == "__main__":
    {"cheng": cheng, "t100b": t100b}[sys.argv[1]]()
