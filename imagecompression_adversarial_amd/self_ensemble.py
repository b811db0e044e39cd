"""Eval-time defences of the reference's self_ensemble.py on the HIP kernels.

    python -m imagecompression_adversarial_amd.self_ensemble -m hyper -q 3 -metric mse -s 'kodim*.png' \\
        --defend --defend_m ensemble|resize|bitdepth

rotates             self_ensemble.py:34-57   8 dihedral variants / their inverses (ica_flip_rot)
bitdepth_reduction  self_ensemble.py:59-70   round(x * (2^bits - 1)) / (2^bits - 1)   (ica_bitdepth)
random_resize       self_ensemble.py:72-83   bicubic antialiased down (243/256) and up (ica_resample_axis with
                                             torch's float32 _compute_weights_aa restated in aa_table)
self_ensemble       self_ensemble.py:85-131  best of the 8 variants by mse(variant, its reconstruction)
defend              self_ensemble.py:156-171
evaluate_defend     self_ensemble.py:173-252 (eval with args.defend)
attack_/main        self_ensemble.py:275-444 (the L2 attack loop == attack.attack_batch, then eval with defend)

Reference semantics kept as they are (SURVEY Appendix B style):
  * ensemble: eval re-runs net(best_x) and compares its reconstruction, in the transformed frame of the
    best variant, with output_s (self_ensemble.py:210-217); a rotated best variant of a non-square image
    has another shape there, which raises like the reference's mse would.
  * resize / bitdepth: eval encodes the preprocessed adversarial image; mse_pre = mean((im_s - x_pre)^2),
    vi_pre = 10 log10(mse_pre / mse_in).  The reference's other products of defend() (the noisy bit-depth
    forward, output_pre) never reach a reported number and are not computed.
  * random_resize(random=False) only (eval uses scale 243/256); output sizes follow F.interpolate
    (floor(size * scale)), so the resized image keeps the input size only for sizes divisible by 256.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from . import coder
from . import hip_ops as K
from . import msssim as MS
from ._lib import call, ptr, stream
from .attack import attack_batch, eval_forward

RESIZE_SCALE = 243.0 / 256.0  # self_ensemble.py:160 random_resize(x, scale=243/256, random=False)


# --------------------------------------------------------------------------- #
# Transforms
# --------------------------------------------------------------------------- #
def _dev(x):
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("defences run on HIP fp32 tensors (no CPU fallback)")
    return x.contiguous()


def _flip_rot(x, op):
    x = _dev(x)
    B, C, H, W = x.shape
    y = torch.empty((B, C, W, H) if op >= 2 else (B, C, H, W), dtype=x.dtype, device=x.device)
    call("ica_flip_rot", ptr(x), ptr(y), B * C, H, W, op, stream())
    return y


FLIP_H, FLIP_W, ROT_P, ROT_M = 0, 1, 2, 3   # flip dim 2, flip dim 3, rot90(k=1), rot90(k=-1)


def rotates(x, reverse=-1):
    """self_ensemble.rotates: reverse=-1 gives the 8 variants (x, x0..x6); reverse=k inverts variant k."""
    if reverse == -1:
        x0 = _flip_rot(x, FLIP_H)
        x1 = _flip_rot(x, FLIP_W)
        x2 = _flip_rot(x0, FLIP_W)
        x3 = _flip_rot(x, ROT_P)
        x4 = _flip_rot(x3, FLIP_H)
        x5 = _flip_rot(x3, FLIP_W)
        x6 = _flip_rot(x4, FLIP_W)
        return x, x0, x1, x2, x3, x4, x5, x6
    cases = {
        0: lambda: x,
        1: lambda: _flip_rot(x, FLIP_H),
        2: lambda: _flip_rot(x, FLIP_W),
        3: lambda: _flip_rot(_flip_rot(x, FLIP_W), FLIP_H),
        4: lambda: _flip_rot(x, ROT_M),
        5: lambda: _flip_rot(_flip_rot(x, FLIP_H), ROT_M),
        6: lambda: _flip_rot(_flip_rot(x, FLIP_W), ROT_M),
        7: lambda: _flip_rot(_flip_rot(_flip_rot(x, FLIP_W), FLIP_H), ROT_M),
    }
    return cases[reverse]()


def bitdepth_reduction(x, bits=6, inference=True):
    """self_ensemble.bitdepth_reduction (inference=True: the rounding the eval reports)."""
    assert bits > 0
    if not inference:
        raise NotImplementedError("the noisy (inference=False) bit-depth path never reaches a reported metric")
    x = _dev(x)
    y = torch.empty_like(x)
    call("ica_bitdepth", ptr(x), ptr(y), x.numel(), float(2 ** bits - 1), stream())
    return y


def aa_table(in_size: int, out_size: int, scale_factor: float):
    """Weights of torch's antialiased bicubic interpolation along one axis (ATen UpSampleKernel.cpp
    _compute_weights_aa with interp_size 4 and aa_filter a = -0.5), restated in float32 as torch computes
    them: scale = 1/scale_factor, support = 2*scale (downsampling) or 2, center = scale*(i+0.5),
    xmin = max(int(center - support + 0.5), 0), xsize = min(int(center + support + 0.5), in) - xmin,
    w_j = filter((j + xmin - center + 0.5) * invscale) normalised to sum 1.
    Returns (xmin int32[out], xsize int32[out], w float32[out, K])."""
    f32 = np.float32
    scale = f32(1.0 / scale_factor)
    support = f32(2.0) * scale if scale >= 1.0 else f32(2.0)
    invscale = f32(1.0) / scale if scale >= 1.0 else f32(1.0)
    a = f32(-0.5)

    def filt(x):
        x = abs(x)
        if x < 1.0:
            return ((a + f32(2)) * x - (a + f32(3))) * x * x + f32(1)
        if x < 2.0:
            return (((x - f32(5)) * x + f32(8)) * x - f32(4)) * a
        return f32(0)

    xmins, xsizes, ws = [], [], []
    for i in range(out_size):
        center = scale * f32(i + 0.5)
        xmin = max(int(center - support + f32(0.5)), 0)
        xsize = min(int(center + support + f32(0.5)), in_size) - xmin
        w = [filt((f32(j + xmin) - center + f32(0.5)) * invscale) for j in range(xsize)]
        tot = f32(0)
        for v in w:
            tot = f32(tot + v)
        ws.append([f32(v / tot) if tot != 0 else f32(0) for v in w])
        xmins.append(xmin)
        xsizes.append(xsize)
    K_ = max(xsizes)
    wt = np.zeros((out_size, K_), np.float32)
    for i, w in enumerate(ws):
        wt[i, :len(w)] = w
    return np.asarray(xmins, np.int32), np.asarray(xsizes, np.int32), wt


def _resample(x, axis, out_len, tab):
    xmin, xsize, wt = (torch.from_numpy(t).to(x.device) for t in tab)
    B, C, H, W = x.shape
    shape = (B, C, out_len, W) if axis == 0 else (B, C, H, out_len)
    y = torch.empty(shape, dtype=x.dtype, device=x.device)
    call("ica_resample_axis", ptr(x), ptr(y), B * C, H, W, axis, out_len, ptr(xmin), ptr(xsize), ptr(wt),
         wt.shape[1], stream())
    return y


def interpolate_aa_bicubic(x, scale_factor: float):
    """F.interpolate(x, scale_factor=s, mode="bicubic", align_corners=False, antialias=True): output size
    floor(size * s) per axis; columns then rows."""
    x = _dev(x)
    B, C, H, W = x.shape
    Ho, Wo = math.floor(H * scale_factor), math.floor(W * scale_factor)
    t = _resample(x, 1, Wo, aa_table(W, Wo, scale_factor))
    return _resample(t, 0, Ho, aa_table(H, Ho, scale_factor))


def random_resize(x, scale=0.5, random=False):
    """self_ensemble.random_resize: bicubic antialiased down by `scale` and back up by 1/scale."""
    if random:
        raise NotImplementedError("random_resize(random=True) is not used by the reference's eval")
    return interpolate_aa_bicubic(interpolate_aa_bicubic(x, scale), 1.0 / scale), scale


# --------------------------------------------------------------------------- #
# Defended evaluation
# --------------------------------------------------------------------------- #
def _forward(kern, x):
    """net(x) in eval mode: (x_hat NCHW unclamped, bpp[B]) — one HIP forward."""
    B, _, H, W = x.shape
    res = kern.forward(K.to_nc4(x))
    return K.from_nc4(res["x_hat4"], 3), K.bits_to_bpp(res["sumlog"], H * W)


def self_ensemble(kern, x):
    """self_ensemble.self_ensemble for a batch (each image on its own, as the reference's B = 1 call):
    returns (best_mse[B], best_x (list of [1,3,h,w]), best_idx list)."""
    B = x.shape[0]
    xs = rotates(x)
    mses = []
    for group in (xs[:4], xs[4:]):
        xcat = torch.cat(group, dim=0)   # variant-major, like the reference's cat(xs[:4])
        xh, _ = _forward(kern, xcat)
        mses.append(K.sqdiff_mean(xcat, xh).view(4, B))   # mean((x - x_hat)^2), x_hat unclamped
    m = torch.cat(mses, 0).cpu()                           # [8, B]
    best_idx, best_mse, best_x = [], [], []
    for b in range(B):
        i_best, v_best = 0, float("inf")
        for i in range(8):
            if float(m[i, b]) < v_best:                    # strict: the first minimum wins
                i_best, v_best = i, float(m[i, b])
        best_idx.append(i_best)
        best_mse.append(v_best)
        best_x.append(xs[i_best][b:b + 1])
    return best_mse, best_x, best_idx


def defend(kern, x, method="ensemble"):
    """self_ensemble.defend: the preprocessed input the eval encodes (and, for 'ensemble', the variants)."""
    assert method in ("ensemble", "resize", "bitdepth"), f"{method} not in 'ensemble', 'resize'"
    if method == "ensemble":
        return self_ensemble(kern, x)
    if method == "bitdepth":
        return bitdepth_reduction(x, inference=True)
    return random_resize(x, scale=RESIZE_SCALE, random=False)[0]


def evaluate_defend(kern, im_adv, im_s, output_s, method="ensemble", clamp=True, adv=False, msssim=True):
    """self_ensemble.eval with args.defend (self_ensemble.py:173-252), per image.  Returns a list of dicts
    {bpp, mse_in, mse_out, vi, vi_msim[, mse_pre, vi_pre][, best_idx]} and the defended outputs."""
    B = im_adv.shape[0]
    im_ = K.clamp01(im_adv) if clamp else im_adv
    mse_in = K.sqdiff_mean(im_, im_s)
    extra = [{} for _ in range(B)]
    if method == "ensemble":
        _, best_x, best_idx = self_ensemble(kern, im_)
        xs = best_x
        for b in range(B):
            extra[b]["best_idx"] = best_idx[b]
    else:
        xp = defend(kern, im_, method)
        if xp.shape != im_s.shape:
            raise RuntimeError(f"defend '{method}' changed the image size {tuple(im_s.shape)} -> {tuple(xp.shape)}"
                               " (the reference's mse_pre fails the same way)")
        mse_pre = K.sqdiff_mean(im_s, xp)
        xs = [xp[b:b + 1] for b in range(B)]
    outs, bpps = [], []
    for b in range(B):
        x = xs[b]
        if x.shape[2:] != output_s.shape[2:]:
            raise RuntimeError("defended reconstruction and output_s differ in shape (rotated best variant of a "
                               "non-square image; the reference's mse_out fails the same way)")
        out, bpp = eval_forward(kern, x, clamp)
        outs.append(out)
        bpps.append(bpp)
    output_ = torch.cat(outs, 0)
    bpp = torch.cat(bpps, 0)
    mse_out = K.sqdiff_mean(output_, output_s)
    msim_in = msim_out = None
    if msssim:
        msim_in = MS.ms_ssim_per_image(im_, im_s).tolist()
        msim_out = MS.ms_ssim_per_image(output_, output_s).tolist()
    results = []
    for b in range(B):
        mi, mo = float(mse_in[b]), float(mse_out[b])
        r = {"bpp": float(bpp[b]), "mse_in": mi, "mse_out": mo, "vi": None, "vi_msim": None, **extra[b]}
        if method in ("resize", "bitdepth"):
            r["mse_pre"] = float(mse_pre[b])
            r["vi_pre"] = 10.0 * math.log10(r["mse_pre"] / mi) if mi > 0 and r["mse_pre"] > 0 else None
        if mi > 1e-20 and mo > 1e-20:
            r["vi"] = 10.0 * math.log10(mo / mi)
            if not adv and msim_in is not None and msim_in[b] < 0.9999 and msim_out[b] < 1.0:
                # (msim_out >= 1 makes the reference's log10 raise; reported as None here)
                r["vi_msim"] = 10.0 * math.log10((1 - msim_out[b]) / (1 - msim_in[b]))
        results.append(r)
    return results, output_


# --------------------------------------------------------------------------- #
# CLI (self_ensemble.py:317-444): attack, then the defended eval
# --------------------------------------------------------------------------- #
def batch_attack(args):
    from .attack_rd import _sources
    if args.adv:
        raise NotImplementedError("attacking through the self-ensemble (--adv) is not supported")
    print("==================== ATTACK SETTINGS ====================")
    print("[ IMAGE ]:", args.source, "->", args.target)
    print("Attack Loss Metric:", args.att_metric)
    print("Noise Threshold (L2):", args.noise, f"(epsilon={args.epsilon})")
    print(f"{args.steps} Steps")
    print("=========================================================")
    if args.defend:
        print("==================== DEFENSE SETTINGS ====================")
        print("Defense Method:", args.method)
        print("=========================================================")
    net = coder.load_model(args, training=False).to(args.device)
    for p in net.parameters():
        p.requires_grad_(False)
    kern = net.kernels(getattr(args, "precision", "fp32"))
    pre = args.method in ("resize", "bitdepth")
    bpp_ori_, bpp_, vi_, vi_pre_, n = 0.0, 0.0, 0.0, 0.0, 0
    for name, t, _, _ in _sources(args.source):
        start = time.time()
        im_s = (t if t is not None else coder.read_image(name)[0]).to(args.device)
        res = attack_batch(kern, im_s, steps=args.steps, epsilon=args.epsilon, noise_thr=args.noise,
                           lr=args.lr_attack, clamp=args.clamp, eval_msssim=False)
        if args.defend:
            r = evaluate_defend(kern, res.im_adv, im_s, res.output_s, args.method, args.clamp,
                                msssim=min(im_s.shape[2:]) > 160)[0][0]
            bpp, vi = r["bpp"], r["vi"]
            if pre:
                vi_pre_ += r["vi_pre"] if r["vi_pre"] is not None else 0.0
        else:
            bpp, vi = float(res.bpp[0]), res.vi[0]
        bpp_ori = float(res.bpp_ori[0])
        print(name, bpp_ori, bpp, vi, "Time:", time.time() - start)
        bpp_ori_ += bpp_ori
        bpp_ += bpp
        vi_ += vi if vi is not None else 0.0
        n += 1
    n = max(n, 1)
    bpp_ori, bpp, vi = bpp_ori_ / n, bpp_ / n, vi_ / n
    if args.defend and pre:
        print("AVG:", args.quality, bpp_ori, bpp, (bpp - bpp_ori) / bpp_ori, vi, vi_pre_ / n)
    else:
        print("AVG:", args.quality, bpp_ori, bpp, (bpp - bpp_ori) / bpp_ori, vi)
    return {"bpp_ori": bpp_ori, "bpp": bpp, "vi": vi}


def main(argv=None):
    args = coder.config().parse_args(argv)
    return batch_attack(args)


if __name__ == "__main__":
    main()
