"""CPU fp32 restatement of the reference's eval-time defences (self_ensemble.py:34-252).

TEST INFRASTRUCTURE (see oracle/__init__.py).  rotates / bitdepth_reduction / random_resize are the
reference's own torch calls (self_ensemble.py:34-83: torch.flip, torch.rot90, torch.round,
F.interpolate(mode="bicubic", antialias=True)) restated; self_ensemble.py itself is not importable here
(lpips, pytorch_msssim, compressai absent), so no fixture pins them beyond these torch semantics.

  * ``self_ensemble``  self_ensemble.py:85-131, per image (the reference runs B = 1)
  * ``eval_defend``    self_ensemble.eval with args.defend (self_ensemble.py:173-252)
  * ``adv_expensive``  the --adv expensive branch (self_ensemble.py:259-262): x_ of defend(net, im_in) in
                       training mode, differentiable, for oracle.attack.attack(expensive=...)
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import codec
from .attack import _per_image_mean
from .msssim import ms_ssim_per_image


def rotates(x, reverse=-1):
    """self_ensemble.py:34-57."""
    if reverse == -1:
        x0 = torch.flip(x, [2])
        x1 = torch.flip(x, [3])
        x2 = torch.flip(x0, [3])
        x3 = torch.rot90(x, 1, [2, 3])
        x4 = torch.flip(x3, [2])
        x5 = torch.flip(x3, [3])
        x6 = torch.flip(x4, [3])
        return x, x0, x1, x2, x3, x4, x5, x6
    cases = {
        0: lambda: x,
        1: lambda: torch.flip(x, [2]),
        2: lambda: torch.flip(x, [3]),
        3: lambda: torch.flip(torch.flip(x, [3]), [2]),
        4: lambda: torch.rot90(x, -1, [2, 3]),
        5: lambda: torch.rot90(torch.flip(x, [2]), -1, [2, 3]),
        6: lambda: torch.rot90(torch.flip(x, [3]), -1, [2, 3]),
        7: lambda: torch.rot90(torch.flip(torch.flip(x, [3]), [2]), -1, [2, 3]),
    }
    return cases[reverse]()


def bitdepth_reduction(x, bits=6):
    """self_ensemble.py:59-70 (inference=True)."""
    scale = 2 ** bits - 1
    return torch.round(x * scale) / scale


def random_resize(x, scale=0.5):
    """self_ensemble.py:72-83 (random=False)."""
    x_down = F.interpolate(x, scale_factor=scale, mode="bicubic", align_corners=False, antialias=True)
    return F.interpolate(x_down, scale_factor=1 / scale, mode="bicubic", align_corners=False, antialias=True)


def self_ensemble(P, x, model="hyper"):
    """Per image: the variant with the smallest mean((x_v - x_hat_v)^2) (strict <, first wins)."""
    out = []
    for b in range(x.shape[0]):
        xs = rotates(x[b:b + 1])
        best = (float("inf"), 0)
        for i, xv in enumerate(xs):
            xh = codec.forward(P, xv, model)["x_hat"]
            m = float(torch.mean((xv - xh) ** 2))
            if m < best[0]:
                best = (m, i)
        out.append((best[0], xs[best[1]], best[1]))
    return out


def eval_defend(P, im_adv, im_s, output_s, method="ensemble", model="hyper", clamp=True, adv=False, msssim=True,
                pre=None):
    """self_ensemble.eval with args.defend: per-image dicts {bpp, mse_in, mse_out, vi, vi_msim[, mse_pre, vi_pre]
    [, best_idx]} and the defended (clamped) reconstructions.  ``pre`` (tests) replaces the preprocessed image
    of 'resize' / 'bitdepth', so that the codec part is compared on identical inputs."""
    with torch.no_grad():
        B, _, H, W = im_adv.shape
        im_ = torch.clamp(im_adv, 0.0, 1.0) if clamp else im_adv
        mse_in = _per_image_mean((im_ - im_s) ** 2)
        extra = [{} for _ in range(B)]
        if method == "ensemble":
            se = self_ensemble(P, im_, model)
            xs = [s[1] for s in se]
            for b in range(B):
                extra[b]["best_idx"] = se[b][2]
        else:
            xp = bitdepth_reduction(im_) if method == "bitdepth" else random_resize(im_, 243 / 256)
            if pre is not None:
                assert float((pre - xp).abs().max()) < 2e-6   # the preprocessing itself agrees
                xp = pre
            mse_pre = _per_image_mean((im_s - xp) ** 2)
            xs = [xp[b:b + 1] for b in range(B)]
        outs, bpps = [], []
        for b in range(B):
            res = codec.forward(P, xs[b], model)
            outs.append(torch.clamp(res["x_hat"], 0.0, 1.0) if clamp else res["x_hat"])
            bpps.append(codec.bpp(res["likelihoods"], H * W))
        output_ = torch.cat(outs, 0)
        mse_out = _per_image_mean((output_ - output_s) ** 2)
        msim_in = ms_ssim_per_image(im_, im_s) if msssim else None
        msim_out = ms_ssim_per_image(output_, output_s) if msssim else None
        results = []
        for b in range(B):
            mi, mo = float(mse_in[b]), float(mse_out[b])
            r = {"bpp": float(bpps[b]), "mse_in": mi, "mse_out": mo, "vi": None, "vi_msim": None, **extra[b]}
            if method != "ensemble":
                r["mse_pre"] = float(mse_pre[b])
                r["vi_pre"] = 10.0 * math.log10(r["mse_pre"] / mi)
            if mi > 1e-20 and mo > 1e-20:
                r["vi"] = 10.0 * math.log10(mo / mi)
                if not adv and msssim and float(msim_in[b]) < 0.9999 and float(msim_out[b]) < 1.0:
                    r["vi_msim"] = 10.0 * math.log10((1 - float(msim_out[b])) / (1 - float(msim_in[b])))
            results.append(r)
    return results, output_


def adv_expensive(P, method="ensemble", noise_fn=None, model="hyper", chosen=None):
    """f(im_in, step) -> x_ of defend(net, im_in, method) with net.training (self_ensemble.py:85-131, :156-171):
      ensemble : per image, g_s(g_a(.)) of the variants as two cat-of-4 batches, the first least
                 mean((x_v - x_hat_v)^2) wins, x_ = clamp(rotates(x_hat_best, reverse=best), 0, 1)
      bitdepth : x_ = g_s(g_a((x * 63 + u) / 63) + u_y)     (net(x_)["x_hat"] in training mode)
      resize   : x_ = g_s(g_a(random_resize(x, 243/256)) + u_y)
    noise_fn(step, name, shape) supplies the U(-0.5, 0.5) draws ("x", "y"); chosen (list) records best
    indices per call."""
    def f(x, step):
        if method == "ensemble":
            outs, picks = [], []
            for b in range(x.shape[0]):
                xs = rotates(x[b:b + 1])
                best = (float("inf"), 0, None)
                for grp, base in ((xs[:4], 0), (xs[4:], 4)):
                    xh = codec.transforms(P, torch.cat(grp, 0), model)
                    for j in range(4):
                        m = torch.mean((grp[j] - xh[j:j + 1]) ** 2)
                        if m < best[0]:
                            best = (m, base + j, xh[j:j + 1])
                picks.append(best[1])
                outs.append(torch.clamp(rotates(best[2], reverse=best[1]), 0.0, 1.0))
            if chosen is not None:
                chosen.append(picks)
            return torch.cat(outs, 0)
        if method == "bitdepth":
            scale = 2 ** 6 - 1
            xp = (x * scale + noise_fn(step, "x", tuple(x.shape))) / scale
        elif method == "resize":
            xp = random_resize(x, 243 / 256)
        else:
            raise ValueError(method)
        y = codec.g_a(P, xp)
        return codec.g_s(P, y + noise_fn(step, "y", tuple(y.shape)))
    return f
