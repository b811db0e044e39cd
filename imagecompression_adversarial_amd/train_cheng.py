"""Train-mode forward + RateDistortionLoss + backward of cheng2020-anchor on the HIP kernels: the inner piece of the
adversarial fine-tune (train.py --adv) for ``-m cheng2020`` (``/root/reference/train.py:249-366``
fine-tunes whatever ``coder.load_model`` builds, ``coder.py:88-136``).

    result = image_comp(batch_x)            train.py:349   train mode: y_hat = y + U(-1/2, 1/2), z likewise
    out_criterion = criterion(result, x)    train.py:351   RateDistortionLoss :37-96
    out_criterion["loss"].backward()        train.py:358-359

The chain (CompressAI Cheng2020Anchor = JointAutoregressiveHierarchicalPriors with residual transforms; the
oracle's restatement is ``oracle/codec.cheng_forward``):

  loss -> x_hat -> g_s (RB / RBU blocks: dgrad with the fused leaky-ReLU and IGDN backward epilogues, weight grads)
       -> y_hat <- context_prediction^T (masked 5x5)  <- entropy_parameters^T (1x1, leaky ReLU) <- GC bwd (scales,
          means)  -> h_s^T (k3 / subpel, leaky ReLU) -> z_tilde <- EB bwd -> h_a^T (k3, k3 s2, leaky ReLU)
       -> y -> g_a (RBS / RB blocks: GDN backward fused into the next conv's dgrad, weight grads)

Weight gradients are ``ica_wgrad`` GEMMs over pixels (k3 s1 / k3 s2 / k1 s2 / k1 s1 / k5 s1); the subpel convs
(rho-ordered rows, ``engine_cheng._rho_weight``) take theirs from the PixelUnshuffle view of the output gradient and
scatter the rows back to CompressAI order; the masked conv's gradient is its full 5x5 weight gradient (CompressAI
applies the mask to weight.data, outside autograd)
(``oracle/codec.context_prediction``). GDN / IGDN parameter gradients come from t = dL/dn (``ica_gdn_t``) of the
summed gradient the fused GDN backward saves, then the NonNegativeParametrizer chain (``train_engine
.gdn_param_grads``). All operands fp32 (the inner attack runs on the model's attack precision)."""
from __future__ import annotations

import math

import torch

from . import hip_ops as K
from .engine_cheng import Conv3, Subpel, context_mask, rho_perm
from .train_engine import gdn_param_grads


def _unshuffle_rho(g4):
    """[N, C/4, 2H, 2W, 4] (PixelShuffle output, nChw4c) -> [N, 4 C4, H, W, 4]: quad 4 c4 + 2 qy + qx, lane e holds
    output channel 4 c4 + e at sub-pixel (qy, qx) = rho row 16 c4 + 4 q + e (engine_cheng rho order)."""
    N, C4, H2, W2, _ = g4.shape
    H, W = H2 // 2, W2 // 2
    return g4.view(N, C4, H, 2, W, 2, 4).permute(0, 1, 3, 5, 2, 4, 6).reshape(N, 4 * C4, H, W, 4).contiguous()


def _conv(P, pre, stride=1, mask=None):
    return Conv3(P(f"{pre}.weight"), P(f"{pre}.bias"), stride, mask=mask)


def entropy_forward(P, y4, M, params4, noise_y=None):
    """The joint entropy model in train mode (cheng2020 and mbt2018, anchors/model.py:97-106): y_hat = y + u, the
    masked context model, entropy_parameters(cat(h_s params, ctx)) -> (scales, means), GaussianConditional.
    noise_y: None draws CompressAI's two independent U(-1/2, 1/2) tensors (y_hat = quantize(y, "noise") and the
    GaussianConditional's own requantisation of y); a pair (y_hat noise, likelihood noise) pins both; one tensor pins
    a draw shared by both (tests).  The masked conv zeroes its masked taps in the parameter itself, as CompressAI's
    MaskedConv2d.forward does (``weight.data *= mask``)."""
    B = y4.shape[0]
    shape = (B, M, y4.shape[2], y4.shape[3])
    if isinstance(noise_y, (tuple, list)):
        n_hat, n_lik = noise_y
    elif noise_y is None:
        n_hat = torch.empty(shape, device=y4.device).uniform_(-0.5, 0.5)
        n_lik = torch.empty(shape, device=y4.device).uniform_(-0.5, 0.5)
    else:
        n_hat = n_lik = noise_y
    ny4 = K.to_nc4(n_hat.contiguous())
    nl4 = ny4 if n_lik is n_hat else K.to_nc4(n_lik.contiguous())
    yh4 = y4 + ny4                                     # y_hat = quantize(y, "noise") (train mode)
    wctx = P("context_prediction.weight")
    wctx.mul_(context_mask(5).to(wctx.device))         # MaskedConv2d: weight.data *= mask (in place)
    ctxc = _conv(P, "context_prediction", mask=context_mask(5))
    ctx4 = ctxc.forward(yh4, K.EPI_BIAS)
    ep = [_conv(P, f"entropy_parameters.{i}") for i in (0, 2, 4)]
    t0 = torch.cat((params4, ctx4), dim=1)
    e0 = ep[0].forward(t0, K.EPI_LRELU)
    e1 = ep[1].forward(e0, K.EPI_LRELU)
    gp4 = ep[2].forward(e1, K.EPI_BIAS)
    c4 = (M + 3) // 4
    scales4, means4 = gp4[:, :c4].contiguous(), gp4[:, c4:].contiguous()
    yt4, ylik4, _ = K.gc_likelihood(y4, M, scales4, means4, True, nl4)
    return {"yh4": yh4, "ctxc": ctxc, "ep": ep, "t0": t0, "e0": e0, "e1": e1, "scales4": scales4,
            "means4": means4, "yt4": yt4, "ylik4": ylik4}


def train_forward(ck, P, x4, noise_y=None, noise_z=None):
    """The train-mode forward of cheng2020 (oracle/codec.cheng_forward, training=True) with every activation the
    backward reads.  ck: the model's fp32 ChengKernels; P(name): the detached parameter; noise_y / noise_z: NCHW
    U(-1/2, 1/2) quantisation noise (drawn when None)."""
    B = x4.shape[0]
    N = ck.N
    in_a = []
    y4, sa = ck.ga.forward(x4, save=True, inputs=in_a)
    ha = [_conv(P, f"h_a.{i}", 2 if i in (4, 8) else 1) for i in (0, 2, 4, 6, 8)]
    za = [y4]
    for j, c in enumerate(ha):
        za.append(c.forward(za[-1], K.EPI_LRELU if j < 4 else K.EPI_BIAS))
    z4 = za.pop()
    if noise_z is None:
        noise_z = torch.empty((B, N, z4.shape[2], z4.shape[3]), device=x4.device).uniform_(-0.5, 0.5)
    zt4, zlik4, _ = K.eb_likelihood(z4, N, ck.eb, True, K.to_nc4(noise_z.contiguous()))
    hs0, hs4, hs8 = (_conv(P, f"h_s.{i}") for i in (0, 4, 8))
    hs2 = Subpel(P("h_s.2.0.weight"), P("h_s.2.0.bias"))
    hs6 = Subpel(P("h_s.6.0.weight"), P("h_s.6.0.bias"))
    s0 = hs0.forward(zt4, K.EPI_LRELU)
    s1 = hs2.forward(s0, K.EPI_LRELU)
    s2 = hs4.forward(s1, K.EPI_LRELU)
    s3 = hs6.forward(s2, K.EPI_LRELU)
    params4 = hs8.forward(s3, K.EPI_BIAS)
    ent = entropy_forward(P, y4, N, params4, noise_y)
    yh4 = ent["yh4"]
    in_s = []
    xh4, ss = ck.gs.forward(yh4, save=True, inputs=in_s)
    out = {k: v for k, v in locals().items() if k not in ("ck", "P", "B", "N", "ent")}
    out.update(ent)
    return out


class ChengTrainStep:
    """One train-mode forward / loss / backward of a ``codec.Cheng2020Anchor`` with gradients written into the
    RDTrainer's flat buffer views (CompressAI parameter names)."""

    def __init__(self, trainer):
        self.tr = trainer
        self.perm = {}

    # ------------------------------------------------------------------ helpers
    def _p(self, name):
        return self.tr.params[name].detach()

    def _g(self, name):
        return self.tr.views[name]

    def _wb(self, g4, Cout, x4, Cin, KS, S, pre, mask=None):
        """Weight (k KS, stride S) and bias gradients of conv `pre` from its output gradient g4 and input x4."""
        w = self._g(f"{pre}.weight")
        if mask is None:
            K.wgrad(g4, Cout, x4, Cin, KS, S, w, tag=f"{pre}.wgrad")
        else:
            tmp = torch.empty_like(w)
            K.wgrad(g4, Cout, x4, Cin, KS, S, tmp, tag=f"{pre}.wgrad")
            w.copy_(tmp * mask.to(w.device))
        K.channel_sum(g4, Cout, self._g(f"{pre}.bias"))

    def _wb_subpel(self, gshuf4, C, x4, Cin, pre):
        """Subpel conv `pre` (Conv2d(Cin, 4C, 3) -> PixelShuffle(2)): gradients from the shuffled output gradient."""
        g_rho = _unshuffle_rho(gshuf4)
        R = g_rho.shape[1] * 4
        key = (C, g_rho.device)
        if key not in self.perm:
            idx = rho_perm(C, g_rho.device)
            ok = idx >= 0
            self.perm[key] = (idx[ok], torch.nonzero(ok).flatten())
        dst, src = self.perm[key]
        tmp = torch.empty((R, Cin, 3, 3), device=g_rho.device)
        K.wgrad(g_rho, R, x4, Cin, 3, 1, tmp, tag=f"{pre}.wgrad")
        tb = torch.empty(R, device=g_rho.device)
        K.channel_sum(g_rho, R, tb)
        self._g(f"{pre}.weight").index_copy_(0, dst, tmp.index_select(0, src))
        self._g(f"{pre}.bias").index_copy_(0, dst, tb.index_select(0, src))

    def _gdn(self, pre, g_sum, saved, C, inverse):
        yg, s = saved
        t = K.gdn_t(g_sum, yg, s, inverse)
        gdn_param_grads(self._p(f"{pre}.beta"), self._p(f"{pre}.gamma"), t, (yg, s), C, self._g(f"{pre}.beta"),
                        self._g(f"{pre}.gamma"))

    def context_backward(self, gy, ylik4, gscale, yt4, means4, scales4, M, ep, t0, e0, e1, params4, yh4, ctxc):
        """GaussianConditional (scales, means) -> entropy_parameters (1x1, leaky ReLU) -> the masked context model:
        weight gradients; dL/dy (GC) and dL/d(y_hat) (context) added into gy; returns dL/d(h_s output)."""
        gl_y = K.bpp_grad(ylik4, gscale)
        gv, gsig = K.gc_bwd(yt4 - means4, scales4, gl_y, M)
        gy.add_(gv)                                         # y_tilde = y + u: dL/dy += dL/dv
        ggp = torch.cat((gsig, -gv), dim=1)                 # d/d(means) = -d/dv
        self._wb(ggp, 2 * M, e1, ep[2].Cin, 1, 1, "entropy_parameters.4")
        g = K.lrelu_bwd(ep[2].dgrad(ggp), e1)
        self._wb(g, ep[1].Cout, e0, ep[1].Cin, 1, 1, "entropy_parameters.2")
        g = K.lrelu_bwd(ep[1].dgrad(g), e0)
        self._wb(g, ep[0].Cout, t0, ep[0].Cin, 1, 1, "entropy_parameters.0")
        g = ep[0].dgrad(g)
        cp = params4.shape[1]
        gparams, gctx = g[:, :cp].contiguous(), g[:, cp:].contiguous()
        # CompressAI masks the weight outside autograd: its gradient is the full 5x5 conv gradient
        self._wb(gctx, 2 * M, yh4, M, 5, 1, "context_prediction")
        gy.add_(ctxc.dgrad(gctx))
        return gparams

    # ------------------------------------------------------------------ transforms
    def g_a_backward(self, ga, gy4, saved, inputs):
        """g_a weight / bias / GDN gradients (no input gradient): ChengAnalysis.backward plus weight gradients."""
        N = ga.N
        self._wb(gy4, N, inputs[6], N, 3, 2, "g_a.6")
        g = ga.last.dgrad(gy4)
        g_sum = None
        for i in range(5, -1, -1):
            blk, sv, hin, pre = ga.blocks[i], saved[i], inputs[i], f"g_a.{i}"
            if blk[0] == "rb":
                _, c1, c2 = blk
                a1, a2 = sv
                gp2 = K.lrelu_bwd(g, a2)
                self._wb(gp2, N, a1, N, 3, 1, f"{pre}.conv2")
                gc1 = c2.dgrad(gp2, K.EPI_LRELU_BWD, saved=(a1, None))
                self._wb(gc1, N, hin, N, 3, 1, f"{pre}.conv1")
                _, _, _, _, gd = ga.blocks[i - 1]
                g_sum = torch.empty_like(g)
                g = c1.dgrad(gc1, K.EPI_GDN_BWD, gdn=gd, res=g, save_x=g_sum, saved=saved[i - 1][1:])
            else:
                _, c1, c2, sk, gd = blk
                a1 = sv[0]
                cin = 3 if i == 0 else N
                self._gdn(f"{pre}.gdn", g_sum, sv[1:], N, False)
                self._wb(g, N, a1, N, 3, 1, f"{pre}.conv2")
                self._wb(g_sum, N, hin, cin, 1, 2, f"{pre}.skip")
                gc1 = c2.dgrad(g, K.EPI_LRELU_BWD, saved=(a1, None))
                self._wb(gc1, N, hin, cin, 3, 2, f"{pre}.conv1")
                if i > 0:
                    r = sk.dgrad(g_sum)
                    g = c1.dgrad(gc1, K.EPI_BIAS, res=r)
                    del r

    def g_s_backward(self, gs, gx4, saved, inputs):
        """g_s weight / bias / IGDN gradients; returns dL/d(y_hat)."""
        N = gs.N
        self._wb_subpel(gx4, 3, inputs[7], N, "g_s.7.0")
        g = gs.last.dgrad(gx4)
        g_sum = None
        for i in range(6, -1, -1):
            blk, sv, hin, pre = gs.blocks[i], saved[i], inputs[i], f"g_s.{i}"
            if blk[0] == "rb":
                _, c1, c2 = blk
                a1, a2 = sv
                gp2 = K.lrelu_bwd(g, a2)
                self._wb(gp2, N, a1, N, 3, 1, f"{pre}.conv2")
                gc1 = c2.dgrad(gp2, K.EPI_LRELU_BWD, saved=(a1, None))
                self._wb(gc1, N, hin, N, 3, 1, f"{pre}.conv1")
                if i == 0:
                    g = c1.dgrad(gc1, K.EPI_BIAS, res=g)
                else:
                    _, _, _, _, gd = gs.blocks[i - 1]
                    g_sum = torch.empty_like(g)
                    g = c1.dgrad(gc1, K.EPI_IGDN_BWD, gdn=gd, res=g, save_x=g_sum, saved=saved[i - 1][1:])
            else:
                _, sp, cv, up, gd = blk
                a1 = sv[0]
                self._gdn(f"{pre}.igdn", g_sum, sv[1:], N, True)
                self._wb(g, N, a1, N, 3, 1, f"{pre}.conv")
                self._wb_subpel(g_sum, N, hin, N, f"{pre}.upsample.0")
                ga1 = cv.dgrad(g, K.EPI_LRELU_BWD, saved=(a1, None))
                self._wb_subpel(ga1, N, hin, N, f"{pre}.subpel_conv.0")
                part = sp.dgrad(ga1)
                g = up.dgrad(g_sum, res=part)
                del part
        return g

    # ------------------------------------------------------------------ step
    def step(self, x, noise_y=None, noise_z=None):
        tr = self.tr
        x = x.contiguous()
        B, _, H, W = x.shape
        ck = tr.net.kernels("fp32")
        N = ck.N
        tr.flat_grad.zero_()
        tr._attach_grads()
        x4 = K.to_nc4(x)
        npx = B * H * W
        bscale = 1.0 / (-math.log(2) * npx)
        gscale = bscale * tr.lamb_r

        f = train_forward(ck, self._p, x4, noise_y, noise_z)
        y4, sa, in_a, ha, za, zt4, zlik4 = (f[k] for k in ("y4", "sa", "in_a", "ha", "za", "zt4", "zlik4"))
        hs0, hs2, hs4, hs6, hs8, s0, s1, s2, s3 = (f[k] for k in ("hs0", "hs2", "hs4", "hs6", "hs8", "s0", "s1",
                                                                  "s2", "s3"))
        params4, yh4, ctxc, ep, t0, e0, e1 = (f[k] for k in ("params4", "yh4", "ctxc", "ep", "t0", "e0", "e1"))
        scales4, means4, yt4, ylik4, xh4, ss, in_s = (f[k] for k in ("scales4", "means4", "yt4", "ylik4", "xh4", "ss",
                                                                     "in_s"))
        del f

        # ---- loss (train.py:52-96) ----
        loss, bpp, dist, g4 = tr._loss(xh4, x, [ylik4, zlik4], bscale)

        # ---- backward ----
        gy = self.g_s_backward(ck.gs, g4, ss, in_s)        # dL/d(y_hat) from g_s
        del ss, in_s, g4
        gparams = self.context_backward(gy, ylik4, gscale, yt4, means4, scales4, N, ep, t0, e0, e1, params4, yh4, ctxc)
        # h_s backward
        self._wb(gparams, hs8.Cout, s3, hs8.Cin, 3, 1, "h_s.8")
        g = hs8.dgrad(gparams, K.EPI_LRELU_BWD, saved=(s3, None))
        self._wb_subpel(g, hs6.C, s2, hs6.Cin, "h_s.6.0")
        g = K.lrelu_bwd(hs6.dgrad(g), s2)
        self._wb(g, hs4.Cout, s1, hs4.Cin, 3, 1, "h_s.4")
        g = hs4.dgrad(g, K.EPI_LRELU_BWD, saved=(s1, None))
        self._wb_subpel(g, hs2.C, s0, hs2.Cin, "h_s.2.0")
        g = K.lrelu_bwd(hs2.dgrad(g), s0)
        self._wb(g, hs0.Cout, zt4, hs0.Cin, 3, 1, "h_s.0")
        gz = hs0.dgrad(g)
        gz.add_(tr._eb_backward(ck, zt4, zlik4, N, gscale))   # z_tilde = z + u
        # h_a backward: za = [y, a0, a2, a4, a6]; conv i maps za[j] -> za[j + 1] (z for the last)
        g = gz
        for j in range(4, -1, -1):
            c, pre = ha[j], f"h_a.{2 * j}"
            self._wb(g, c.Cout, za[j], c.Cin, 3, c.S, pre)
            if c.S == 2:
                g = c.dgrad(g)
                if j > 0:
                    g = K.lrelu_bwd(g, za[j])
            elif j > 0:
                g = c.dgrad(g, K.EPI_LRELU_BWD, saved=(za[j], None))
            else:
                g = c.dgrad(g)
        gy.add_(g)
        self.g_a_backward(ck.ga, gy, sa, in_a)
        return {"loss": loss, "bpp_loss": bpp, "distortion_loss": dist}
