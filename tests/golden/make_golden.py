"""Generate the committed golden vectors from the REFERENCE's own modules.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Imports (read-only, nothing copied): /root/reference/utils/ops.py
(Low_bound, Up_bound, GDN), /root/reference/anchors/utils.py (conv, deconv),
/root/reference/utils/torch_msssim.py (MS_SSIM; its hard-coded ``.cuda()``
calls are neutralised by a golden-generation-only shim
``torch.Tensor.cuda = identity``).

Large tensors (weights, inputs) are NOT stored: they are regenerated from
seeds by ``oracle.codec.init_params`` / ``torch.Generator`` (deterministic on
CPU); the fixtures hold the reference modules' outputs and gradients.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = "/root/reference"

from oracle import codec  # noqa: E402


def _ref_modules():
    sys.path.insert(0, REF)
    torch.Tensor.cuda = lambda self, *a, **k: self  # shim: reference hard-codes .cuda()
    from utils import ops as rops  # noqa
    from utils import torch_msssim as rtm  # noqa
    from anchors import utils as rau  # noqa
    return rops, rtm, rau


def rand(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def ref_gdn(rops, beta, gamma, inverse):
    C = beta.shape[0]
    m = rops.GDN(C, inverse=inverse)
    with torch.no_grad():
        m.beta.copy_(beta)
        m.gama.copy_(gamma.reshape(C, C, 1, 1))
    return m


def ref_stack(rops, rau, P, N, M):
    """g_a / g_s built from the reference's own layers (anchors/utils.py conv/deconv + utils/ops.GDN)."""
    ga = nn.Sequential(rau.conv(3, N), ref_gdn(rops, P["g_a.1.beta"], P["g_a.1.gamma"], False),
                       rau.conv(N, N), ref_gdn(rops, P["g_a.3.beta"], P["g_a.3.gamma"], False),
                       rau.conv(N, N), ref_gdn(rops, P["g_a.5.beta"], P["g_a.5.gamma"], False),
                       rau.conv(N, M))
    gs = nn.Sequential(rau.deconv(M, N), ref_gdn(rops, P["g_s.1.beta"], P["g_s.1.gamma"], True),
                       rau.deconv(N, N), ref_gdn(rops, P["g_s.3.beta"], P["g_s.3.gamma"], True),
                       rau.deconv(N, N), ref_gdn(rops, P["g_s.5.beta"], P["g_s.5.gamma"], True),
                       rau.deconv(N, 3))
    with torch.no_grad():
        for pre, seq in (("g_a", ga), ("g_s", gs)):
            for i in (0, 2, 4, 6):
                seq[i].weight.copy_(P[f"{pre}.{i}.weight"])
                seq[i].bias.copy_(P[f"{pre}.{i}.bias"])
    for p in list(ga.parameters()) + list(gs.parameters()):
        p.requires_grad_(False)
    return ga, gs


def main():
    torch.set_num_threads(8)
    rops, rtm, rau = _ref_modules()
    out = {}

    # 1. bounds (utils/ops.py:28-56), incl. equality and g == 0 cases
    x = torch.tensor([-0.2, 0.0, 0.05, 0.5, 1.0, 1.2, -1e-9, 1.0 + 1e-7])
    for tag, gval in (("gpos", 1.0), ("gneg", -1.0), ("gzero", 0.0)):
        xx = x.clone().requires_grad_(True)
        y = rops.Up_bound.apply(rops.Low_bound.apply(xx, 0.0), 1.0)
        y.backward(torch.full_like(y, gval))
        out[f"bounds_x"] = x.numpy()
        out[f"bounds_y"] = y.detach().numpy()
        out[f"bounds_dx_{tag}"] = xx.grad.numpy()
    xr = rand((4, 3, 17, 23), 11, -0.2, 0.2)
    gr = rand((4, 3, 17, 23), 12, -1, 1)
    xx = xr.clone().requires_grad_(True)
    y = rops.Up_bound.apply(rops.Low_bound.apply(xx, -16 / 255.0), 16 / 255.0)
    y.backward(gr)
    out["bounds_eps_y"] = y.detach().numpy()
    out["bounds_eps_dx"] = xx.grad.numpy()

    # 2. GDN / IGDN fwd + bwd (utils/ops.py:58-97) on perturbed params
    for C, shape, seed in ((16, (2, 16, 9, 11), 21), (128, (2, 128, 6, 10), 22)):
        P = codec.perturb_params(dict(zip(("a.beta", "a.gamma"), codec.gdn_init(C))), seed=seed)
        for inv in (False, True):
            m = ref_gdn(rops, P["a.beta"], P["a.gamma"], inv)
            xg = (rand(shape, seed + 1) * 2 - 1).requires_grad_(True)
            y = m(xg)
            g = rand(shape, seed + 2) * 2 - 1
            y.backward(g)
            tag = f"gdn{C}_{'inv' if inv else 'fwd'}"
            out[f"{tag}_y"] = y.detach().numpy()
            out[f"{tag}_dx"] = xg.grad.numpy()
            out[f"{tag}_dbeta"] = m.beta.grad.numpy()
            out[f"{tag}_dgamma"] = m.gama.grad.reshape(C, C).numpy()

    # 3. conv / deconv geometry (anchors/utils.py:112-130), fwd + input grad
    geoms = [("conv_3_16_k5", rau.conv(3, 16), (2, 3, 32, 48)),
             ("conv_16_24_k5", rau.conv(16, 24), (2, 16, 16, 24)),
             ("conv_24_16_k3s1", rau.conv(24, 16, kernel_size=3, stride=1), (2, 24, 8, 12)),
             ("deconv_24_16_k5", rau.deconv(24, 16), (2, 24, 8, 12)),
             ("deconv_16_3_k5", rau.deconv(16, 3), (2, 16, 16, 24))]
    for i, (tag, m, shape) in enumerate(geoms):
        torch.manual_seed(100 + i)
        m.reset_parameters()
        xg = (rand(shape, 200 + i) * 2 - 1).requires_grad_(True)
        y = m(xg)
        g = rand(tuple(y.shape), 300 + i) * 2 - 1
        y.backward(g)
        out[f"{tag}_w"] = m.weight.detach().numpy()
        out[f"{tag}_b"] = m.bias.detach().numpy()
        out[f"{tag}_y"] = y.detach().numpy()
        out[f"{tag}_dx"] = xg.grad.numpy()

    # 4. composed hyper g_a + g_s (q3 widths N=128, M=192), weights from
    #    oracle.codec.init_params(seed=0) + perturb_params(seed=1); 64x64 input.
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    ga, gs = ref_stack(rops, rau, P, 128, 192)
    xs = rand((1, 3, 64, 64), 7)
    with torch.no_grad():
        os_ = torch.clamp(gs(torch.round(ga(xs))), 0, 1)  # stand-in for the eval target
    xin = rand((1, 3, 64, 64), 8, -0.03, 0.03)
    xi = rops.Up_bound.apply(rops.Low_bound.apply(xs + xin, 0.0), 1.0).detach().requires_grad_(True)
    y = ga(xi)
    xh = gs(y)
    o = rops.Up_bound.apply(rops.Low_bound.apply(xh, 0.0), 1.0)
    loss = 1.0 - torch.mean((os_ - o) * (os_ - o))  # attack_rd.py:364
    loss.backward()
    out["stack_y"] = y.detach().numpy()
    out["stack_xhat"] = xh.detach().numpy()
    out["stack_output_s"] = os_.numpy()
    out["stack_loss"] = np.array(loss.item())
    out["stack_dx"] = xi.grad.numpy()

    # 5. short attack trajectories on the reference stack (attack_rd.py:496-559
    #    restated with the reference's own Low_bound/Up_bound and torch Adam).
    #    thr 1e-4 (default -noise) stays in the network branch; thr 1e-5 flips.
    for tag, thr in (("traj", 1e-4), ("traj2", 1e-5)):
        steps, eps_n = 12, 16 / 255.0
        noise = torch.zeros_like(xs).requires_grad_(True)
        opt = torch.optim.Adam([noise], lr=0.01)
        sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
        loss_is, branch = [], []
        for i in range(steps):
            nc = rops.Up_bound.apply(rops.Low_bound.apply(noise, -eps_n), eps_n)
            im_in = rops.Up_bound.apply(rops.Low_bound.apply(xs + nc, 0.0), 1.0)
            loss_i = torch.mean((xs - im_in) ** 2)
            if loss_i > thr:
                loss = loss_i
                branch.append(1)
            else:
                o = rops.Up_bound.apply(rops.Low_bound.apply(gs(ga(im_in)), 0.0), 1.0)
                loss = 1.0 - torch.mean((os_ - o) * (os_ - o))
                branch.append(0)
            loss_is.append(loss_i.item())
            opt.zero_grad()
            loss.backward()
            opt.step()
            if i % (steps // 3) == 0:
                sch.step()
        out[f"{tag}_thr"] = np.array(thr)
        out[f"{tag}_loss_i"] = np.array(loss_is)
        out[f"{tag}_branch"] = np.array(branch)
        out[f"{tag}_noise"] = noise.detach().numpy()
        out[f"{tag}_im_in"] = im_in.detach().numpy()

    # 6. utils/torch_msssim.MS_SSIM value + grad (adv_train loss), 192x192 pair
    a = rand((1, 3, 192, 192), 31)
    b = torch.clamp(a + (rand((1, 3, 192, 192), 32) - 0.5) * 0.2, 0, 1).requires_grad_(True)
    v = rtm.MS_SSIM(max_val=1.0)(a, b)
    v.backward()
    out["tmssim_val"] = np.array(v.item())
    out["tmssim_grad"] = b.grad.numpy()

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"), {k: v.shape for k, v in out.items()})


# Long-horizon trajectories (config 1: hyper q1 widths N=128, M=192, one 256x256 image, 100 steps, default
# -noise 1e-4 / -lr_attack 0.01 / -e 16).  The weights are oracle.codec.init_params("hyper", 1, seed=0) +
# perturb_params(seed=1) with g_a.6.weight scaled by LSCALE: CompressAI's random init gives |y| << 0.5, so
# round(y) == 0, the eval reconstruction never changes and the attack never leaves the network branch; the
# scale brings |y| to the O(1) range of a trained codec, where the run hovers at the -noise budget and
# crosses the lr milestones at 34 / 67 with both branches in play (attack_rd.py:502-503,553-554).
TRAJ100 = {"t100a": 10.0, "t100b": 40.0}


def traj100_params(tag):
    P = codec.perturb_params(codec.init_params("hyper", 1, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * TRAJ100[tag]
    return P


def traj100_image():
    return rand((1, 3, 256, 256), 101)


def main_traj100():
    """attack_rd.attack_ (attack_rd.py:496-559) for 100 steps on the reference's own layers, Adam and
    MultiStepLR, then the eval metrics of self_ensemble.eval (self_ensemble.py:190-246) on the same layers:
    out = clamp(g_s(round(g_a(x))), 0, 1) (the hyperprior's eval reconstruction, means=None -> round(y))."""
    torch.set_num_threads(8)
    rops, rtm, rau = _ref_modules()
    out = {}
    xs = traj100_image()
    steps, eps_n, thr = 100, 16 / 255.0, 1e-4
    B = lambda v, lo, hi: rops.Up_bound.apply(rops.Low_bound.apply(v, lo), hi)  # noqa: E731
    for tag in TRAJ100:
        P = traj100_params(tag)
        ga, gs = ref_stack(rops, rau, P, 128, 192)
        with torch.no_grad():
            os_ = torch.clamp(gs(torch.round(ga(xs))), 0, 1)   # attack_rd.py:406-411 (eval reconstruction)
        noise = torch.zeros_like(xs).requires_grad_(True)
        opt = torch.optim.Adam([noise], lr=0.01)
        sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
        loss_is, branch, lrs = [], [], []
        for i in range(steps):
            nc = B(noise, -eps_n, eps_n)
            im_in = B(xs + nc, 0.0, 1.0)
            loss_i = torch.mean((xs - im_in) ** 2)
            if loss_i > thr:                                   # attack_rd.py:334
                loss = loss_i
                branch.append(1)
            else:
                o = B(gs(ga(im_in)), 0.0, 1.0)
                loss = 1.0 - torch.mean((os_ - o) * (os_ - o))  # attack_rd.py:364
                branch.append(0)
            loss_is.append(loss_i.item())
            lrs.append(opt.param_groups[0]["lr"])
            opt.zero_grad()
            loss.backward()
            opt.step()
            if i % (steps // 3) == 0:
                sch.step()
        with torch.no_grad():
            im_ = torch.clamp(im_in, 0, 1)
            o_adv = torch.clamp(gs(torch.round(ga(im_))), 0, 1)
            mse_in = torch.mean((im_ - xs) ** 2).item()
            mse_out = torch.mean((o_adv - os_) ** 2).item()
        out[f"{tag}_scale"] = np.array(TRAJ100[tag])
        out[f"{tag}_loss_i"] = np.array(loss_is, dtype=np.float32)
        out[f"{tag}_branch"] = np.array(branch, dtype=np.int8)
        out[f"{tag}_lr"] = np.array(lrs)
        out[f"{tag}_noise"] = noise.detach().numpy()
        out[f"{tag}_output_s"] = os_.numpy()
        out[f"{tag}_mse_in"] = np.array(mse_in)
        out[f"{tag}_mse_out"] = np.array(mse_out)
        out[f"{tag}_vi"] = np.array(10.0 * np.log10(mse_out / mse_in) if mse_out > 0 else np.nan)
        print(tag, "".join("c" if b else "E" for b in branch), mse_in, mse_out, flush=True)
    np.savez_compressed(os.path.join(HERE, "traj100.npz"), **out)
    print("wrote", os.path.join(HERE, "traj100.npz"))


# noise snapshots of the same trajectories (after these step indexes) and per-step noise fingerprints, so that a
# run whose branch sequence leaves the reference's at step d can still be checked element-wise up to d
SNAP_STEPS = (9, 24, 49)


def fingerprint_pattern(shape):
    return rand(shape, 977) * 2.0 - 1.0


def main_traj100_snap():
    """traj100.npz's runs again (same layers, weights, image and loop), recording noise after SNAP_STEPS and, per
    step, (sum |noise|, sum noise^2, <noise, pattern>) with pattern a fixed seeded U(-1, 1) tensor."""
    torch.set_num_threads(8)
    rops, rtm, rau = _ref_modules()
    out = {}
    xs = traj100_image()
    pat = fingerprint_pattern(xs.shape).double()
    steps, eps_n, thr = 100, 16 / 255.0, 1e-4
    B = lambda v, lo, hi: rops.Up_bound.apply(rops.Low_bound.apply(v, lo), hi)  # noqa: E731
    ref = np.load(os.path.join(HERE, "traj100.npz"))
    for tag in TRAJ100:
        P = traj100_params(tag)
        ga, gs = ref_stack(rops, rau, P, 128, 192)
        with torch.no_grad():
            os_ = torch.clamp(gs(torch.round(ga(xs))), 0, 1)
        noise = torch.zeros_like(xs).requires_grad_(True)
        opt = torch.optim.Adam([noise], lr=0.01)
        sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
        fp, snaps, branch = [], [], []
        for i in range(steps):
            nc = B(noise, -eps_n, eps_n)
            im_in = B(xs + nc, 0.0, 1.0)
            loss_i = torch.mean((xs - im_in) ** 2)
            if loss_i > thr:
                loss = loss_i
                branch.append(1)
            else:
                o = B(gs(ga(im_in)), 0.0, 1.0)
                loss = 1.0 - torch.mean((os_ - o) * (os_ - o))
                branch.append(0)
            opt.zero_grad()
            loss.backward()
            opt.step()
            if i % (steps // 3) == 0:
                sch.step()
            n = noise.detach().double()
            fp.append([float(n.abs().sum()), float((n * n).sum()), float((n * pat).sum())])
            if i in SNAP_STEPS:
                snaps.append(noise.detach().numpy().copy())
        assert branch == [int(v) for v in ref[f"{tag}_branch"]], tag   # the same run as traj100.npz
        assert np.array_equal(noise.detach().numpy(), ref[f"{tag}_noise"]), tag
        out[f"{tag}_fp"] = np.array(fp, dtype=np.float64)
        out[f"{tag}_snap"] = np.stack(snaps)
        print(tag, "snapshots", SNAP_STEPS, flush=True)
    out["snap_steps"] = np.array(SNAP_STEPS)
    np.savez_compressed(os.path.join(HERE, "traj100_snap.npz"), **out)
    print("wrote", os.path.join(HERE, "traj100_snap.npz"))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "traj100":
        main_traj100()
    elif len(sys.argv) > 1 and sys.argv[1] == "traj100_snap":
        main_traj100_snap()
    else:
        main()
