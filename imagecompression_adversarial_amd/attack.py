"""The attack step loops on the HIP kernels (no autograd, no host round-trips
inside a step except the optional per-step branch census).

``attack_batch`` == attack_rd.attack_ (attack_rd.py:381-575) with attack_our
(:332-379) and self_ensemble.eval (self_ensemble.py:173-252), batched with
PER-IMAGE semantics: image b of the batch follows exactly the trajectory a
B == 1 reference run would (own loss_i, own branch, own Adam state).  The
branch `loss_i > -noise` is decided ON DEVICE per image inside the Adam kernel.

``coupled=True`` gives the batch-coupled semantics the adversarial fine-tune
uses (train.py:342 -> attack_rd.py:333-334, adv_train.py:146-155): loss_i is
the mean over the WHOLE batch and one branch is taken for all images.  With a
process group the batch is the union of every rank's shard: the per-image
loss_i are summed across ranks by one 4-byte-per-rank all-reduce per step
(RCCL on the GPU box), and all gradients are normalised by the global image
count, so N ranks reproduce one B_global run.

``target=`` / ``roi=`` give the targeted / ROI attack (DESIGN.md "Targeted / ROI
attack"): box-weighted masked means for the input budget and a minimised output loss that pulls the
target region toward the codec's reconstruction of the target image and keeps the background at
output_s.  Same step loop, schedule, branch rule and per-image semantics as above.

``ifgsm_batch`` == attack_ifgsm.attack_ifgsm (attack_ifgsm.py:364-438) without
random start (the reference default path), per image.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from . import dist as D
from . import hip_ops as K
from . import msssim as MS
from ._lib import call, ptr, stream
from .engine import CodecKernels


# HIP-graph replay of the whole-batch network step (g_a, g_s, loss, g_s^T, g_a^T: ~25 launches) while every image
# stays on the expensive branch: captured once per AttackLoop (its weights and buffers are fixed), replayed by one
# launch per step.  The replay runs the captured kernels on the same buffers, so the bits equal the eager step's
# (tests/test_gpu_graph.py).  ICA_ATTACK_GRAPH=0 turns it off.
ATTACK_GRAPH = os.environ.get("ICA_ATTACK_GRAPH", "1") != "0"
GRAPH_STATS = {"captures": 0, "replays": 0}   # process-wide counters (bench.py --config 4 reports them)


def _lr_table(steps, lr):
    # replicate torch's float arithmetic: lr is multiplied by gamma at each milestone
    out, cur, sch = [], lr, 0
    period = max(steps // 3, 1)
    for i in range(steps):
        out.append(cur)
        if i % period == 0:
            sch += 1
            if sch in (1, 2, 3):
                cur = cur * 0.33
    return out


@dataclass
class AttackResult:
    im_adv: torch.Tensor          # clamp(im_in_final, 0, 1)          [B,3,H,W]
    output_adv: torch.Tensor      # clamp(x_hat(im_adv), 0, 1)
    output_s: torch.Tensor        # clamp(x_hat(im_s), 0, 1)
    bpp_ori: torch.Tensor         # [B]
    bpp: torch.Tensor             # [B]
    mse_in: torch.Tensor          # [B]
    mse_out: torch.Tensor         # [B]
    msim_in: torch.Tensor | None  # [B]
    msim_out: torch.Tensor | None
    vi: list = field(default_factory=list)
    vi_msim: list = field(default_factory=list)
    noise: torch.Tensor | None = None
    branches: list = field(default_factory=list)
    output_t: torch.Tensor | None = None   # targeted mode: clamp(x_hat(target))
    tar_mse: torch.Tensor | None = None    # targeted mode: per-image mean_roi((out - output_t)^2)


def eval_forward(kern: CodecKernels, x: torch.Tensor, clamp=True):
    """net.eval(); net(x) -> (output_ = clamp?(x_hat) NCHW, bpp[B])."""
    B, _, H, W = x.shape
    res = kern.forward(K.to_nc4(x))
    out = torch.empty_like(x)
    call("ica_nc4_bound_to_nchw", ptr(res["x_hat4"]), ptr(out), B, H, W, int(clamp), stream())
    return out, K.bits_to_bpp(res["sumlog"], H * W)


def padded_eval_forward(kern: CodecKernels, x: torch.Tensor, pad: int, mode="reflect"):
    """attack_rd.py:389-419 with -p: net(F.pad(x, (p, p, p, p), mode)) -> crop(clamp(x_hat)), bits / (H * W).
    The padded pre-eval clamps whatever --clamp says (attack_rd.py:417 clamps unconditionally)."""
    import torch.nn.functional as F
    B, _, H, W = x.shape
    xp = F.pad(x, (pad, pad, pad, pad), mode=mode).contiguous()
    Hp, Wp = xp.shape[2:]
    if Hp % 64 or Wp % 64:
        raise ValueError(f"-p {pad}: the padded size {Hp}x{Wp} must be a multiple of 64 (the codec's latent grid; "
                         "the reference's crop fails otherwise)")
    out_p, bpp_p = eval_forward(kern, xp, True)
    out = out_p[:, :, pad:pad + H, pad:pad + W].contiguous()
    return out, bpp_p * (Hp * Wp / (H * W))


def evaluate(kern, im_in, im_s, output_s, clamp=True, adv=False, msssim=True):
    """self_ensemble.eval (self_ensemble.py:173-252), per image."""
    im_ = K.clamp01(im_in) if clamp else im_in
    out, bpp = eval_forward(kern, im_, clamp)
    mse_in = K.sqdiff_mean(im_, im_s)
    mse_out = K.sqdiff_mean(out, output_s)
    msim_in = msim_out = None
    if msssim:
        msim_in = MS.ms_ssim_per_image(im_, im_s)
        msim_out = MS.ms_ssim_per_image(out, output_s)
    vi, vi_msim = [], []
    mi_l, mo_l = mse_in.tolist(), mse_out.tolist()
    si_l = msim_in.tolist() if msssim else [None] * len(mi_l)
    so_l = msim_out.tolist() if msssim else [None] * len(mi_l)
    for mi, mo, si, so in zip(mi_l, mo_l, si_l, so_l):
        v = vm = None
        if mi > 1e-20 and mo > 1e-20:
            v = 10.0 * math.log10(mo / mi)
            if not adv and si is not None and si < 0.9999:
                vm = 10.0 * math.log10((1 - so) / (1 - si))
        vi.append(v)
        vi_msim.append(vm)
    return im_, out, bpp, mse_in, mse_out, msim_in, msim_out, vi, vi_msim


class AttackLoop:
    """Holds the device state of one batched attack_rd.attack_ run."""

    def __init__(self, kern: CodecKernels, im_s: torch.Tensor, steps=1001, epsilon=16.0, noise_thr=1e-4,
                 lr=0.01, att_metric="L2", clamp=True, init_noise=None, coupled=False, group=None,
                 target=None, roi=None, la_tar=1.0, la_bkg_in=1.0, la_bkg_out=1.0, pad=None, padding_mode="reflect"):
        if att_metric not in ("L2", "ms-ssim"):
            raise ValueError(f"att_metric {att_metric!r} not supported (reference: L2, ms-ssim)")
        if target is not None and (att_metric != "L2" or coupled):
            raise NotImplementedError("the targeted / ROI attack is defined for att_metric L2, per-image")
        self.kern = kern
        self.im_s = im_s.contiguous()
        B, C, H, W = im_s.shape
        assert C == 3
        self.B, self.H, self.W = B, H, W
        self.steps, self.eps, self.thr = steps, float(epsilon) / 255.0, float(noise_thr)
        self.metric, self.clamp = att_metric, clamp
        self.invN = float(1.0 / (3 * H * W))  # torch: grad / numel in fp32
        self.coupled, self.group = coupled, group
        self.B_global = D.global_count(B, im_s.device, group) if coupled else B
        # gradient scale of the mean-type losses: per image (1/numel) or over the whole batch
        self.gscale = float(1.0 / (self.B_global * 3 * H * W)) if coupled else self.invN
        self.dval = 1.0 / self.B_global if coupled else 1.0
        dev = im_s.device
        # the debug model (ae_onelayer) attacks an unclamped input from a random start (attack_rd.py:493-494, 514-515)
        self.clamp_in = bool(getattr(kern, "clamp_input", True))
        if init_noise is not None:
            self.noise = init_noise.clone().contiguous()
        elif not self.clamp_in:
            r = float(noise_thr) ** 0.5
            self.noise = torch.empty(tuple(im_s.shape)).uniform_(-r, r).to(dev)
        else:
            self.noise = torch.zeros_like(self.im_s)
        if target is not None and not self.clamp_in:
            raise NotImplementedError("the targeted / ROI attack is defined for the clamped-input models")
        self.m = torch.zeros_like(self.im_s)
        self.v = torch.zeros_like(self.im_s)
        self.im_in4 = K.empty_nc4(B, 3, H, W, dev)
        self.part = torch.empty(B * K.blocks_per_image(), device=dev)
        self.loss_i = torch.empty(B, device=dev)
        self.grad4 = K.empty_nc4(B, 3, H, W, dev)
        self.branch = torch.zeros(B, dtype=torch.int32, device=dev)
        self.im_in = torch.empty_like(self.im_s)
        self.lrs = _lr_table(steps, lr)
        self.t = 0
        # branch compaction (attack_rd.py:334: the network runs only for images with loss_i <= -noise):
        # per step one device->host read of the expensive-image list, then g_a/g_s on that sub-batch only.
        # census[b] counts image b's cheap-branch steps (device-side, no sync).
        self.compact = True
        self.sel = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        self.gpos = torch.zeros(B, dtype=torch.int32, device=dev)
        self.sel_host = torch.zeros(B + 1, dtype=torch.int32).pin_memory() if dev.type == "cuda" else None
        # speculation: after a step whose images were all on the expensive branch, the next step runs the network on
        # the whole batch without waiting for its own selection (read one step later, when the GPU still has that
        # step's network work queued).  The Adam kernel takes each image's branch from the device, and an image's
        # gradient does not depend on the batch it runs in, so the results are the same bits either way; a cheap
        # image costs one step of unused network work.
        self._sel_ev = torch.cuda.Event() if dev.type == "cuda" else None
        self._sel_pending = False
        self.census = torch.zeros(B, dtype=torch.int32, device=dev)
        self.steps_done = 0
        # host-side cost of the branch read: steps whose network launch waited for the device's selection, and the
        # wall time spent blocked in those waits (bench.py --mixed reports them)
        self.sync_steps = 0
        self.sync_wait_s = 0.0
        # the whole-batch network step as a HIP graph (L2 losses, the ROI attack's included; the ms-ssim loss path and
        # subclasses with their own network step -- the defended attack's, which reads its variant choice on the host
        # -- run eager)
        self.graph_ok = (ATTACK_GRAPH and dev.type == "cuda" and att_metric == "L2"
                         and type(self).network_grad is AttackLoop.network_grad)
        self._graph, self._graph_out = None, None
        self.graph_replays = 0
        # pre-eval: output_s, bpp_ori (attack_rd.py:401-419)
        if pad:
            # -p P (attack_rd.py:389-413): the pre-eval codes the image padded by P (-padmode, reflect by default),
            # output_s is the crop back to the image, bpp_ori counts the padded bits per UNPADDED pixel (:419);
            # the step loop and the post-eval run unpadded, as in the reference
            self.output_s, self.bpp_ori = padded_eval_forward(kern, self.im_s, int(pad), padding_mode)
        else:
            self.output_s, self.bpp_ori = eval_forward(kern, self.im_s, clamp)
        self.output_s4 = None
        self.roi = None
        if target is not None:
            t = target.to(self.im_s.device).contiguous()
            if t.shape[0] == 1 and B > 1:
                t = t.expand(B, -1, -1, -1).contiguous()
            if t.shape != self.im_s.shape:
                raise ValueError(f"target {tuple(t.shape)} must match the source batch {tuple(self.im_s.shape)}")
            self.output_t, _ = eval_forward(kern, t, True)   # attack_cv.py:136-137: the target's reconstruction
            self.roi = roi_weights(H, W, roi, la_tar, la_bkg_in, la_bkg_out)

    def _adam_scalars(self, i):
        t = i + 1
        bc1 = 1 - 0.9 ** t
        bc2 = 1 - 0.999 ** t
        step_size = self.lrs[i] / bc1
        return float(bc2 ** 0.5), float(-step_size)

    def _select(self):
        """Expensive images of this step: (E, idx) with idx the sorted host list (None when E == B)."""
        B = self.B
        if not self.compact:
            return B, None
        call("ica_branch_select", ptr(self.loss_i), self.thr, B, ptr(self.sel), ptr(self.gpos), stream())
        prev_all = False
        if self._sel_pending:   # the previous step's selection (its copy was queued one step ago)
            self._sel_ev.synchronize()
            prev_all = int(self.sel_host[0]) == B
            self._sel_pending = False
        self.sel_host.copy_(self.sel, non_blocking=True)
        self._sel_ev.record()
        # (ms-ssim needs the host to know whether any image is cheap: its cheap-branch gradient is a separate launch)
        if prev_all and (self.metric == "L2" or self.roi is not None):   # speculate: the whole batch, no wait
            self._sel_pending = True
            return B, None
        t0 = time.perf_counter()
        self._sel_ev.synchronize()
        self.sync_wait_s += time.perf_counter() - t0
        self.sync_steps += 1
        E = int(self.sel_host[0])
        if E == B:
            self._sel_pending = True   # (already complete) lets the next step speculate
            return B, None
        return E, self.sel[1:1 + E]

    def _gather(self, x, idx, E):
        if idx is None:
            return x
        per = x[0].numel()
        out = torch.empty((E,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        call("ica_gather_images", ptr(x), ptr(out), ptr(idx), E, per, stream())
        return out

    def network_grad(self, idx=None, E=None):
        """x_hat = g_s(g_a(im_in)); d loss_o / d im_in (nChw4c, C=3) for the images idx (all when None): the
        expensive-branch work of attack_our (attack_rd.py:340-379), on a compacted sub-batch."""
        kern = self.kern
        H, W = self.H, self.W
        Bn = self.B if idx is None else E
        im4 = self._gather(self.im_in4, idx, Bn)
        out_s = self._gather(self.output_s, idx, Bn)
        grad4, part = self.grad4[:Bn], self.part[:Bn * K.blocks_per_image()]
        y4, sa = kern.g_a(im4, save=True)
        del im4
        xh4, ss = kern.g_s(y4, save=True)
        del y4
        if self.roi is not None:
            x0, x1, y0, y1, _, _, wot, wob = self.roi
            out_t = self._gather(self.output_t, idx, Bn)
            call("ica_roi_loss", ptr(xh4), ptr(out_s), ptr(out_t), ptr(grad4), ptr(part),
                 Bn, H, W, x0, x1, y0, y1, wot, wob, int(self.clamp), stream())
        elif self.metric == "L2":
            call("ica_attack_loss", ptr(xh4), ptr(out_s), ptr(grad4), ptr(part), Bn, H, W,
                 self.gscale, int(self.clamp), 0, stream())
        else:
            # loss_o = ms_ssim(out, output_s) per image (attack_rd.py:362)
            out = torch.empty_like(out_s)
            call("ica_nc4_bound_to_nchw", ptr(xh4), ptr(out), Bn, H, W, int(self.clamp), stream())
            ones = torch.full((Bn,), self.dval, device=out.device)
            _, gout, _ = MS.ms_ssim_value_and_grad(out, out_s, ones)
            call("ica_bound_bwd_nc4", ptr(xh4), ptr(gout), ptr(grad4), Bn, H, W, int(self.clamp), stream())
        gy4 = kern.g_s_backward(grad4, ss)
        del ss, xh4
        return kern.g_a_backward(gy4, sa)

    def _network_graph(self):
        """network_grad() on the whole batch through a HIP graph: captured on first use (the capture does not run
        the kernels, so it is replayed right away), one replay per step after that.  The per-launch timing hooks of
        hip_ops (bench.py) see only the eager launches."""
        if self._graph is None:
            hooks = (K.EVENT_HOOK, K.LAUNCH_HOOK)
            K.EVENT_HOOK = K.LAUNCH_HOOK = None
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, capture_error_mode="relaxed"):
                    out = self.network_grad(None, self.B)
            finally:
                K.EVENT_HOOK, K.LAUNCH_HOOK = hooks
            self._graph, self._graph_out = g, out
            GRAPH_STATS["captures"] += 1
        self._graph.replay()
        self.graph_replays += 1
        GRAPH_STATS["replays"] += 1
        return self._graph_out

    def step(self, i, record_im_in=False, census=False):
        B, H, W = self.B, self.H, self.W
        if self.roi is not None:
            return self._step_roi(i, record_im_in, census)
        call("ica_attack_prologue_ex", ptr(self.noise), ptr(self.im_s), ptr(self.im_in4), ptr(self.part), B, H, W,
             self.eps, int(self.clamp_in), stream())
        K.reduce_rows(self.part, B, self.invN, out=self.loss_i)
        if self.coupled:
            D.couple_loss_i(self.loss_i, self.B_global, self.group)
        E, idx = self._select()
        if E == B and idx is None and self.graph_ok:
            gx4 = self._network_graph()
        else:
            gx4 = self.network_grad(idx, E) if E > 0 else None
        cheap_grad = None
        if self.metric == "ms-ssim" and E < B:
            # cheap branch loss = 1 - ms_ssim(im_s, im_in): d/d im_in = -dMS/dY
            im_in = torch.empty_like(self.im_s)
            call("ica_nc4_bound_to_nchw", ptr(self.im_in4), ptr(im_in), B, H, W, 0, stream())
            _, _, gY = MS.ms_ssim_value_and_grad(self.im_s, im_in, torch.full((B,), -self.dval, device=im_in.device))
            cheap_grad = gY
        bc2s, neg_step = self._adam_scalars(i)
        call("ica_attack_adam_ex", ptr(self.noise), ptr(self.im_s), ptr(gx4), ptr(self.loss_i), ptr(cheap_grad),
             ptr(self.m), ptr(self.v), ptr(self.im_in if record_im_in else None), B, H, W, self.eps, self.thr,
             self.gscale, bc2s, neg_step, ptr(self.branch), ptr(self.gpos if idx is not None else None),
             ptr(self.census), int(self.clamp_in), stream())
        self.steps_done += 1
        if census:
            return self.branch.tolist()
        return None

    def _step_roi(self, i, record_im_in, census):
        B, H, W = self.B, self.H, self.W
        x0, x1, y0, y1, wit, wib, _, _ = self.roi
        call("ica_roi_prologue", ptr(self.noise), ptr(self.im_s), ptr(self.im_in4), ptr(self.part), B, H, W,
             self.eps, x0, x1, y0, y1, wit, wib, stream())
        K.reduce_rows(self.part, B, 1.0, out=self.loss_i)
        E, idx = self._select()
        if E == B and idx is None and self.graph_ok:
            gx4 = self._network_graph()
        else:
            gx4 = self.network_grad(idx, E) if E > 0 else None
        bc2s, neg_step = self._adam_scalars(i)
        call("ica_roi_adam", ptr(self.noise), ptr(self.im_s), ptr(gx4), ptr(self.loss_i), ptr(self.m), ptr(self.v),
             ptr(self.im_in if record_im_in else None), B, H, W, self.eps, self.thr, bc2s, neg_step,
             ptr(self.branch), x0, x1, y0, y1, wit, wib, ptr(self.gpos if idx is not None else None),
             ptr(self.census), stream())
        self.steps_done += 1
        if census:
            return self.branch.tolist()
        return None

    def expensive_image_steps(self):
        """Image-steps that ran the network so far (B * steps - the device census of cheap steps)."""
        return self.B * self.steps_done - int(self.census.sum())

    def run(self, record=False):
        branches = []
        for i in range(self.steps):
            br = self.step(i, record_im_in=(i == self.steps - 1), census=record)
            if record:
                branches.append(br)
        return branches


def roi_weights(H, W, roi, la_tar=1.0, la_bkg_in=1.0, la_bkg_out=1.0):
    """(x0, x1, y0, y1, w_in_tar, w_in_bkg, w_out_tar, w_out_bkg) of the masked means; roi = (x0, x1, y0, y1)
    in pixels (x = width, attack_cv.py:159-161), None = the whole image is the target region."""
    x0, x1, y0, y1 = (0, W, 0, H) if roi is None else (int(v) for v in roi)
    x0, x1 = max(0, min(x0, W)), max(0, min(x1, W))
    y0, y1 = max(0, min(y0, H)), max(0, min(y1, H))
    area = max(x1 - x0, 0) * max(y1 - y0, 0)
    if area == 0:
        raise ValueError(f"empty ROI {roi} for a {W}x{H} image")
    cnt_t, cnt_b = 3.0 * area, 3.0 * (H * W - area)
    wb = (lambda la: float(la / cnt_b) if cnt_b > 0 else 0.0)
    return (x0, x1, y0, y1, float(1.0 / cnt_t), wb(la_bkg_in), float(la_tar / cnt_t), wb(la_bkg_out))


def roi_mse(a, b, roi4):
    """Per-image mean over the target box of (a - b)^2 (NCHW)."""
    x0, x1, y0, y1 = roi4
    d = (a - b)[:, :, y0:y1, x0:x1]
    return (d * d).flatten(1).mean(1)


def attack_batch(kern: CodecKernels, im_s, steps=1001, epsilon=16.0, noise_thr=1e-4, lr=0.01, att_metric="L2",
                 clamp=True, init_noise=None, eval_msssim=True, record=False, coupled=False,
                 group=None, target=None, roi=None, la_tar=1.0, la_bkg_in=1.0, la_bkg_out=1.0, pad=None,
                 padding_mode="reflect") -> AttackResult:
    loop = AttackLoop(kern, im_s, steps, epsilon, noise_thr, lr, att_metric, clamp, init_noise, coupled, group,
                      target, roi, la_tar, la_bkg_in, la_bkg_out, pad, padding_mode)
    branches = loop.run(record=record)
    im_, out, bpp, mse_in, mse_out, msim_in, msim_out, vi, vi_msim = evaluate(
        kern, loop.im_in, loop.im_s, loop.output_s, clamp, adv=False, msssim=eval_msssim)
    res = AttackResult(im_adv=im_, output_adv=out, output_s=loop.output_s, bpp_ori=loop.bpp_ori, bpp=bpp,
                       mse_in=mse_in, mse_out=mse_out, msim_in=msim_in, msim_out=msim_out, vi=vi, vi_msim=vi_msim,
                       noise=loop.noise, branches=branches)
    if loop.roi is not None:
        res.output_t = loop.output_t
        res.tar_mse = roi_mse(out, loop.output_t, loop.roi[:4])
    return res


def ifgsm_batch(kern: CodecKernels, im_s, steps=10, epsilon=16.0, momentum=False, clamp=True, x0=None):
    """The step loop of attack_ifgsm.attack_ifgsm (attack_ifgsm.py:392-423) per image; x0: the start point
    (the random start clamp(im_s + U(-eps, eps), 0, 1) of :377-380; default im_s, :382).
    Returns (im_adv, output_s)."""
    B, _, H, W = im_s.shape
    im_s = im_s.contiguous()
    output_s, _ = eval_forward(kern, im_s, clamp=True)
    eps = float(epsilon) / 255.0
    alpha = float(eps / steps)
    x = im_s.clone() if x0 is None else x0.contiguous().clone()
    gacc = torch.zeros_like(x)
    part = torch.empty(B * K.blocks_per_image(), device=x.device)
    grad4 = K.empty_nc4(B, 3, H, W, x.device)
    l1 = torch.empty(B, device=x.device)
    invN = float(1.0 / (3 * H * W))
    for _ in range(steps):
        y4, sa = kern.g_a(K.to_nc4(x), save=True)
        xh4, ss = kern.g_s(y4, save=True)
        call("ica_attack_loss", ptr(xh4), ptr(output_s), ptr(grad4), ptr(part), B, H, W, invN, 0, 1, stream())
        gx4 = kern.g_a_backward(kern.g_s_backward(grad4, ss), sa)
        if momentum:
            call("ica_l1_partial", ptr(gx4), ptr(part), B, H, W, stream())
            K.reduce_rows(part, B, 1.0, out=l1)
        call("ica_ifgsm_step", ptr(x), ptr(im_s), ptr(gx4), ptr(gacc), ptr(l1), B, H, W, alpha, eps, int(momentum),
             stream())
    return x, output_s
