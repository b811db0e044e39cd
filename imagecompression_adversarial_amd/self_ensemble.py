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
DefendedAttackLoop  self_ensemble.py:253-326 with --adv: the attack through defend() (ensemble / bitdepth / resize)

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
from .attack import AttackLoop, attack_batch, eval_forward, evaluate

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
# Attacking through the defence (--adv; self_ensemble.py:253-326)
# --------------------------------------------------------------------------- #
BITDEPTH_SCALE = float(2 ** 6 - 1)   # bitdepth_reduction(bits=6)


def variant(x, i):
    """rotates(x)[i] alone (the forward transform of dihedral variant i)."""
    if i == 0:
        return x
    if i in (1, 2, 3):
        t = _flip_rot(x, FLIP_H) if i != 2 else _flip_rot(x, FLIP_W)
        return _flip_rot(t, FLIP_W) if i == 3 else t
    r = _flip_rot(x, ROT_P)
    if i == 4:
        return r
    t = _flip_rot(r, FLIP_H) if i != 6 else _flip_rot(r, FLIP_W)
    return _flip_rot(t, FLIP_W) if i == 7 else t


def aa_table_t(tab, in_size: int):
    """Transpose of one resample pass (its input gradient) as a gather table over the pass's outputs: for input
    index i the outputs whose support holds i form one contiguous range (xmin, xsize nondecreasing)."""
    xmin, xsize, wt = tab
    rows = [[] for _ in range(in_size)]
    for o in range(len(xmin)):
        for k in range(int(xsize[o])):
            rows[int(xmin[o]) + k].append((o, wt[o, k]))
    Kt = max(1, max(len(r) for r in rows))
    xm = np.zeros(in_size, np.int32)
    xs = np.zeros(in_size, np.int32)
    w = np.zeros((in_size, Kt), np.float32)
    for i, r in enumerate(rows):
        if r:
            os_ = [o for o, _ in r]
            if os_ != list(range(os_[0], os_[0] + len(os_))):
                raise AssertionError("resample support is not contiguous")
            xm[i], xs[i] = os_[0], len(os_)
            w[i, :len(r)] = [v for _, v in r]
    return xm, xs, w


class _ResizePair:
    """random_resize(x, 243/256) as four separable passes plus their transposes (input gradient)."""

    def __init__(self, H, W, scale=RESIZE_SCALE):
        Ho, Wo = math.floor(H * scale), math.floor(W * scale)
        H2, W2 = math.floor(Ho / scale), math.floor(Wo / scale)
        if (H2, W2) != (H, W):
            raise RuntimeError(f"resize {H}x{W} -> {Ho}x{Wo} -> {H2}x{W2} changes the image size (the reference's "
                               "loss against output_s fails the same way)")
        self.fw = [(1, Wo, aa_table(W, Wo, scale)), (0, Ho, aa_table(H, Ho, scale)),
                   (1, W, aa_table(Wo, W, 1.0 / scale)), (0, H, aa_table(Ho, H, 1.0 / scale))]
        ins = [W, H, Wo, Ho]
        self.bw = [(ax, n_in, aa_table_t(tab, n_in)) for (ax, _, tab), n_in in zip(self.fw, ins)][::-1]

    def forward(self, x):
        for ax, n, tab in self.fw:
            x = _resample(x, ax, n, tab)
        return x

    def backward(self, g):
        for ax, n, tab in self.bw:
            g = _resample(g, ax, n, tab)
        return g


def _select(saved, rows):
    """index_select every tensor of a saved-activation structure along the batch dimension."""
    if saved is None:
        return None
    if isinstance(saved, torch.Tensor):
        return saved.index_select(0, rows)
    out = type(saved)(_select(s, rows) for s in saved)
    if hasattr(saved, "__dict__"):   # engine.Saved: keep the layout record (split / exact) of the selection
        out.__dict__.update(saved.__dict__)
    return out


class DefendedAttackLoop(AttackLoop):
    """self_ensemble.attack_ with args.adv: the expensive branch encodes defend(net, im_in, method) in training
    mode (self_ensemble.py:259-262) and the loss gradient flows back through the defence:
      ensemble : all 8 dihedral variants through g_s(g_a(.)) (two cat-of-4 batches, :85-131); the variant with
                 the least mse(variant, reconstruction) (first minimum) carries the gradient:
                 output_ = clamp(rotate_back(x_hat_best)) -> torch.clamp mask -> variant transform -> g_s/g_a
                 input gradient -> inverse transform.
      bitdepth : x_ = (x * 63 + u) / 63, x_hat = g_s(g_a(x_) + u_y) (net(x_) in training mode: y_hat = y + noise
                 for every model), the usual bounded L2 output loss.
      resize   : x_ = up(down(x)) (antialiased bicubic 243/256), x_hat = g_s(g_a(x_) + u_y); gradient through the
                 transposed resample passes.
    noise_fn(step, name, shape) may supply the uniform draws ("x": bit-depth noise, "y": latent noise); default:
    torch's device generator, U(-0.5, 0.5) as the reference draws them."""

    def __init__(self, kern, im_s, method="ensemble", noise_fn=None, **kw):
        if method not in ("ensemble", "resize", "bitdepth"):
            raise ValueError(f"{method} not in 'ensemble', 'resize', 'bitdepth'")
        if kw.get("att_metric", "L2") != "L2" or kw.get("target") is not None or kw.get("coupled"):
            raise NotImplementedError("self_ensemble's attack is the per-image L2 attack")
        super().__init__(kern, im_s, **kw)
        # the defences draw their noise for the whole batch each step (the reference's draw shapes), so the
        # network runs on the full batch here: no branch compaction
        self.compact = False
        self.method, self.noise_fn = method, noise_fn
        self.resize = _ResizePair(self.H, self.W) if method == "resize" else None
        self.best_hist = []   # per step: the best variant index of each image (ensemble)

    def _uniform(self, name, shape, i):
        if self.noise_fn is not None:
            return self.noise_fn(i, name, shape).to(self.im_s.device, torch.float32).contiguous()
        return torch.empty(shape, device=self.im_s.device).uniform_(-0.5, 0.5)

    def step(self, i, record_im_in=False, census=False):
        self._i = i
        return super().step(i, record_im_in, census)

    def network_grad(self, idx=None, E=None):
        assert idx is None, "DefendedAttackLoop runs the network on the full batch"
        if self.method == "ensemble":
            return self._grad_ensemble()
        return self._grad_noisy()

    def _grad_noisy(self):
        kern, B, H, W = self.kern, self.B, self.H, self.W
        x = K.from_nc4(self.im_in4, 3)
        if self.method == "bitdepth":
            u = self._uniform("x", x.shape, self._i)
            xp = torch.empty_like(x)
            call("ica_bitdepth_noise", ptr(x), ptr(u), ptr(xp), x.numel(), BITDEPTH_SCALE, stream())
        else:
            xp = self.resize.forward(x)
        y4, sa = kern.g_a(K.to_nc4(xp), save=True)
        uy = self._uniform("y", (B, kern.M, y4.shape[2], y4.shape[3]), self._i)
        yh4 = torch.empty_like(y4)
        call("ica_add", ptr(y4), ptr(K.to_nc4(uy)), ptr(yh4), y4.numel(), stream())
        del y4
        xh4, ss = kern.g_s(yh4, save=True)
        call("ica_attack_loss", ptr(xh4), ptr(self.output_s), ptr(self.grad4), ptr(self.part), B, H, W,
             self.gscale, int(self.clamp), 0, stream())
        g = K.from_nc4(kern.g_a_backward(kern.g_s_backward(self.grad4, ss), sa), 3)
        if self.method == "bitdepth":
            gx = torch.empty_like(g)
            call("ica_bitdepth_noise_bwd", ptr(g), ptr(gx), g.numel(), BITDEPTH_SCALE, stream())
        else:
            gx = self.resize.backward(g)
        return K.to_nc4(gx)

    def _grad_ensemble(self):
        kern, B = self.kern, self.B
        x = K.from_nc4(self.im_in4, 3)
        xs = rotates(x)
        groups, mses = [], []
        for grp in (xs[:4], xs[4:]):
            xcat = torch.cat(grp, dim=0)                     # variant-major, as cat(xs[:4]) per image
            y4, sa = kern.g_a(K.to_nc4(xcat), save=True)
            xh4, ss = kern.g_s(y4, save=True)
            del y4
            xh = K.from_nc4(xh4, 3)
            mses.append(K.sqdiff_mean(xcat, xh).view(4, B))
            groups.append((xh, sa, ss))
        best = torch.argmin(torch.cat(mses, 0), dim=0).tolist()   # first minimum, like the strict '<' scan
        self.best_hist.append(best)
        gx = torch.empty_like(x)
        for gi, (xh, sa, ss) in enumerate(groups):
            imgs = [b for b in range(B) if best[b] // 4 == gi]
            if not imgs:
                continue
            rows = torch.tensor([(best[b] % 4) * B + b for b in imgs], device=x.device)
            gv = []
            for b in imgs:
                o = rotates(xh[(best[b] % 4) * B + b:(best[b] % 4) * B + b + 1], reverse=best[b]).contiguous()
                g = torch.empty_like(o)
                call("ica_ensemble_grad", ptr(o), ptr(self.output_s[b:b + 1]), ptr(g), o.numel(), self.gscale,
                     stream())
                gv.append(variant(g, best[b]))
            g4 = K.to_nc4(torch.cat(gv, 0))
            gxv = K.from_nc4(kern.g_a_backward(kern.g_s_backward(g4, _select(ss, rows)), _select(sa, rows)), 3)
            for j, b in enumerate(imgs):
                gx[b:b + 1] = rotates(gxv[j:j + 1].contiguous(), reverse=best[b])
        return K.to_nc4(gx)


def adv_attack_batch(kern, im_s, method="ensemble", steps=1001, epsilon=16.0, noise_thr=1e-4, lr=0.01, clamp=True,
                     noise_fn=None, defend_eval=False, eval_msssim=True, record=False):
    """self_ensemble.attack_ with --adv (per image), then its eval (with --defend when defend_eval).
    Returns (AttackResult-like dict of the eval, the loop)."""
    loop = DefendedAttackLoop(kern, im_s, method, noise_fn, steps=steps, epsilon=epsilon, noise_thr=noise_thr,
                              lr=lr, clamp=clamp)
    branches = loop.run(record=record)
    if defend_eval:
        res, out = evaluate_defend(kern, loop.im_in, loop.im_s, loop.output_s, method, clamp, adv=True,
                                   msssim=eval_msssim)
    else:
        im_, out, bpp, mse_in, mse_out, msim_in, msim_out, vi, vi_msim = evaluate(
            kern, loop.im_in, loop.im_s, loop.output_s, clamp, adv=True, msssim=eval_msssim)
        res = [{"bpp": float(bpp[b]), "mse_in": float(mse_in[b]), "mse_out": float(mse_out[b]), "vi": vi[b],
                "vi_msim": vi_msim[b]} for b in range(loop.B)]
    return res, out, loop, branches


# --------------------------------------------------------------------------- #
# CLI (self_ensemble.py:317-444): attack, then the defended eval
# --------------------------------------------------------------------------- #
def batch_attack(args):
    from .attack_rd import _sources
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
    kern = net.kernels(net.attack_precision(getattr(args, "precision", None)))
    pre = args.method in ("resize", "bitdepth")
    bpp_ori_, bpp_, vi_, vi_pre_, n = 0.0, 0.0, 0.0, 0.0, 0
    for name, t, _, _ in _sources(args.source):
        start = time.time()
        im_s = (t if t is not None else coder.read_image(name)[0]).to(args.device)
        if args.adv:   # attack through defend(net, im_in, args.method) (self_ensemble.py:259-262)
            rs, _, loop, _ = adv_attack_batch(kern, im_s, args.method, steps=args.steps, epsilon=args.epsilon,
                                              noise_thr=args.noise, lr=args.lr_attack, clamp=args.clamp,
                                              defend_eval=args.defend, eval_msssim=min(im_s.shape[2:]) > 160)
            r = rs[0]
            bpp, vi = r["bpp"], r["vi"]
            if args.defend and pre:
                vi_pre_ += r["vi_pre"] if r["vi_pre"] is not None else 0.0
            bpp_ori = float(loop.bpp_ori[0])
            print(name, bpp_ori, bpp, vi, "Time:", time.time() - start)
            bpp_ori_ += bpp_ori
            bpp_ += bpp
            vi_ += vi if vi is not None else 0.0
            n += 1
            continue
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
