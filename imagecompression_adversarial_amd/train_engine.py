"""Train-mode forward + RateDistortionLoss + backward of the bmshj2018 codecs on the HIP kernels (cheng2020-anchor:
train_cheng.ChengTrainStep; mbt2018: train_mbt.MbtTrainStep; both dispatched from RDTrainer.step).

This is the inner piece of the adversarial fine-tune:

    result = image_comp(batch_x)                       train.py:349   (train mode: +U(-1/2,1/2) noise)
    out_criterion = criterion(result, batch_x)          train.py:351   RateDistortionLoss :37-96
    out_criterion["loss"].backward()                    train.py:358-359

``RDTrainer.step`` runs the forward with the activations the backward needs,
evaluates ``lambda*255^2*MSE + bpp`` (or ``lambda*(1-MS-SSIM) + bpp``) and writes
the gradient of every main parameter (all but ``*.quantiles``) into ``p.grad``,
a view of one flat buffer (``flat_grad``) so data-parallel training needs a
single all-reduce.  No autograd graph is built; the chain is

  loss -> x_hat -> g_s (dgrad conv_down + IGDN-bwd epilogue, wgrad, IGDN params)
       -> y_tilde <- GaussianConditional bwd (y, scales) -> h_s (ReLU, k3/k5 dgrad+wgrad)
       -> z_tilde <- EntropyBottleneck bwd (z, 58 logistic-MLP params per channel) -> h_a
       -> |y| -> y -> g_a (dgrad conv_up + GDN-bwd epilogue, wgrad, GDN params)

Weight gradients are MFMA GEMMs over pixels (ica_wgrad); GDN parameter gradients
come from t = dL/dn, written by the GDN-bwd epilogue of the dgrad conv (save_t):
dbeta' = sum_p t, dgamma'[c][j] = sum_p t_c x_j^2, then the NonNegativeParametrizer
chain (ica_reparam_bwd).  Only the CompressAI parameter names of the bmshj2018
models are used, so a reference checkpoint / optimizer state maps 1:1.
"""
from __future__ import annotations

import math

import torch

from . import hip_ops as K
from . import msssim as MS

GAMMA_BOUND = 2.0 ** -18  # NonNegativeParametrizer(minimum=0): sqrt(0 + 2^-36)


def gdn_param_grads(raw_beta, raw_gamma, t4, saved, C, g_beta, g_gamma):
    """GDN/IGDN parameter grads from t = dL/dn (the GDN-bwd epilogue's save_t) and the layer's saved (y, s):
    dbeta' = sum_p t, dgamma'[c][j] = sum_p t_c x_j^2, then the NonNegativeParametrizer chain (utils/ops.py:62-89)
    back to the raw parameters, written into g_beta / g_gamma."""
    y4, s4 = saved
    dbeta_e = torch.empty(C, device=t4.device)
    K.channel_sum(t4, C, dbeta_e)
    xsq = K.gdn_xsq(y4, s4)
    dgamma_e = torch.empty(C * C, device=t4.device)
    K.wgrad(t4, C, xsq, C, 1, 1, dgamma_e)
    K.reparam_bwd(raw_beta, dbeta_e, g_beta, K.GDN_BETA_BOUND)
    K.reparam_bwd(raw_gamma, dgamma_e, g_gamma, GAMMA_BOUND)


def _row_major(saved):
    if any(getattr(saved, "split", ())):
        raise RuntimeError("parameter gradients need the forward's activations row-major (forward(..., split=False))")


def synthesis_backward(ex, g4, y_in4, saved, params, grads, prefix):
    """g_s backward (engine.Synthesis): the input gradient (returned) and the weight / bias / IGDN parameter
    gradients, written into grads[prefix + name] (CompressAI names: 0.weight, 1.beta, ...)."""
    _row_major(saved)
    N, M = ex.N, ex.M
    g, C = g4, 3
    for i in (3, 2, 1, 0):
        p = ex.convs[i]
        cin = M if i == 0 else N
        inp = y_in4 if i == 0 else saved[i - 1][0]
        K.wgrad(inp, cin, g, C, 5, 2, grads[f"{prefix}{2 * i}.weight"], tag=f"{prefix}{2 * i}.wgrad")
        K.channel_sum(g, C, grads[f"{prefix}{2 * i}.bias"])
        if i > 0:
            t = torch.empty_like(saved[i - 1][0])
            g, _, _ = K.conv_down(g, C, p.bwd, None, N, 5, 2, K.EPI_IGDN_BWD, ex.gdns[i - 1],
                                  saved=saved[i - 1], save_t=t, it=p.it_bwd)
            q = f"{prefix}{2 * i - 1}"
            gdn_param_grads(params[f"{q}.beta"], params[f"{q}.gamma"], t, saved[i - 1], N, grads[f"{q}.beta"],
                            grads[f"{q}.gamma"])
        else:
            g, _, _ = K.conv_down(g, C, p.bwd, None, M, 5, 2, K.EPI_BIAS)
        C = N
    return g


def analysis_backward(ex, gy4, x4, saved, params, grads, prefix, input_grad=False):
    """g_a backward (engine.Analysis): weight / bias / GDN parameter gradients into grads[prefix + name], and
    the input gradient (nChw4c, 3 channels) when input_grad."""
    _row_major(saved)
    N, M = ex.N, ex.M
    g, C = gy4, M
    for i in (3, 2, 1, 0):
        inp = x4 if i == 0 else saved[i - 1][0]
        cin = 3 if i == 0 else N
        K.wgrad(g, C, inp, cin, 5, 2, grads[f"{prefix}{2 * i}.weight"], tag=f"{prefix}{2 * i}.wgrad")
        K.channel_sum(g, C, grads[f"{prefix}{2 * i}.bias"])
        if i > 0:
            t = torch.empty_like(saved[i - 1][0])
            g, _, _ = K.conv_up(g, C, ex.convs[i].bwd, None, N, K.EPI_GDN_BWD, ex.gdns[i - 1],
                                saved=saved[i - 1], save_t=t, it=ex.convs[i].it_bwd)
            q = f"{prefix}{2 * i - 1}"
            gdn_param_grads(params[f"{q}.beta"], params[f"{q}.gamma"], t, saved[i - 1], N, grads[f"{q}.beta"],
                            grads[f"{q}.gamma"])
        C = N
    if input_grad:
        gx, _, _ = K.conv_up(g, N, ex.convs[0].bwd, None, 3, K.EPI_BIAS, prec=ex.convs[0].bwd_prec)
        return gx
    return None


class RDTrainer:
    """HIP train step for a ``codec.FactorizedPrior`` / ``codec.ScaleHyperprior``."""

    def __init__(self, net, metric: str = "mse", lmbda: float = 1e-2):
        if metric not in ("mse", "ms-ssim"):
            raise ValueError(f"metric {metric!r}: the HIP trainer supports mse and ms-ssim (lpips is out of scope)")
        self.net, self.metric, self.lmbda = net, metric, float(lmbda)
        self.kind = net.model_kind
        if self.kind not in ("factorized", "hyper", "cheng2020", "context", "debug"):
            raise NotImplementedError(f"the HIP trainer covers bmshj2018, mbt2018, cheng2020-anchor and the debug "
                                      f"model, not {self.kind!r}")
        self._joint = None   # cheng2020 / mbt2018 / ae_onelayer (train_cheng, train_mbt, train_debug)
        # train.py:77-83: lambda == 100 is the reference's "Inf mode", the rate term leaves the loss (lamb_r = 0)
        self.lamb_r = 0.0 if self.lmbda == 100 else 1.0
        if self.lamb_r == 0.0:
            print("[WARNING] Inf Mode")
        named = dict(net.named_parameters())
        self.names = sorted(n for n in named if not n.endswith(".quantiles"))
        self.params = {n: named[n] for n in self.names}
        dev = next(net.parameters()).device
        total = sum(self.params[n].numel() for n in self.names)
        self.flat_grad = torch.zeros(total, device=dev)
        self.views, off = {}, 0
        for n in self.names:
            p = self.params[n]
            self.views[n] = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()

    # ------------------------------------------------------------------ #
    def _attach_grads(self):
        for n in self.names:
            p = self.params[n]
            if p.grad is None or p.grad.data_ptr() != self.views[n].data_ptr():
                p.grad = self.views[n]

    def _g(self, name):
        return self.views[name]

    # ------------------------------------------------------------------ #
    def _g_s_backward(self, ex, g4, y_in4, saved):
        """Synthesis backward with weight / bias / IGDN grads; returns dL/d(g_s input)."""
        return synthesis_backward(ex, g4, y_in4, saved, self.params, self.views, "g_s.")

    def _g_a_backward(self, ex, gy4, x4, saved):
        """Analysis backward with weight / bias / GDN grads (no input gradient)."""
        analysis_backward(ex, gy4, x4, saved, self.params, self.views, "g_a.")

    def _eb_backward(self, ck, v4, lik4, C, scale):
        gl = K.bpp_grad(lik4, scale)
        gv, gprm = K.eb_bwd(v4, gl, ck.eb, C)
        names = [f"entropy_bottleneck.{n}" for n in K.PackedEB.NAMES[:14]]
        K.eb_param_scatter(gprm, [self.params[n].detach() for n in names], [self._g(n) for n in names], C)
        return gv

    def _loss(self, xh4, x, liks, bscale):
        """RateDistortionLoss (train.py:52-96, training=True: no clamp on x_hat): (loss, bpp, distortion, dL/dx_hat
        as nChw4c)."""
        B, _, H, W = x.shape
        bpp = sum(torch.log(l.clamp_min(1.0 / 65536)).sum() for l in liks) * bscale
        g4 = torch.zeros_like(xh4)
        if self.metric == "mse":
            dist = K.sqdiff_mean(K.from_nc4(xh4, 3), x).mean()
            K.mse_grad_(xh4, x, g4, self.lmbda * 255.0 ** 2 * 2.0 / (B * 3 * H * W))
            loss = self.lmbda * 255.0 ** 2 * dist + self.lamb_r * bpp
        else:
            xh = K.from_nc4(xh4, 3)
            v, gX, _ = MS.ms_ssim_value_and_grad(xh, x, torch.full((B,), -self.lmbda / B, device=x.device),
                                                 data_range=1.0, mode=0)
            dist = v.mean()
            g4 = K.to_nc4(gX)
            loss = self.lmbda * (1.0 - dist) + self.lamb_r * bpp
        return loss, bpp, dist, g4

    # ------------------------------------------------------------------ #
    def step(self, x: torch.Tensor, noise_y: torch.Tensor | None = None, noise_z: torch.Tensor | None = None):
        """One train-mode forward + loss + backward.  x: [B,3,H,W] on the device (H, W multiples of 64).
        noise_y / noise_z: optional NCHW U(-1/2,1/2) quantisation noise (drawn here when None).
        Returns {"loss", "bpp_loss", "distortion_loss"} as 0-d device tensors; grads in p.grad."""
        if self.kind in ("cheng2020", "context", "debug"):
            if self._joint is None:
                if self.kind == "cheng2020":
                    from .train_cheng import ChengTrainStep as Step
                elif self.kind == "debug":
                    from .train_debug import DebugTrainStep as Step
                else:
                    from .train_mbt import MbtTrainStep as Step
                self._joint = Step(self)
            return self._joint.step(x, noise_y, noise_z)
        x = x.contiguous()
        B, _, H, W = x.shape
        ck = self.net.kernels()
        N, M = ck.N, ck.M
        self.flat_grad.zero_()
        self._attach_grads()
        x4 = K.to_nc4(x)
        npx = B * H * W
        bscale = 1.0 / (-math.log(2) * npx)
        gscale = bscale * self.lamb_r   # d loss / d log-likelihood (0 in Inf mode)

        y4, sa = ck.ga.forward(x4, save=True, split=False)   # the wgrad kernels read row-major activations
        yshape = (B, M, H // 16, W // 16)
        if noise_y is None:
            noise_y = torch.empty(yshape, device=x.device).uniform_(-0.5, 0.5)
        ny4 = K.to_nc4(noise_y.contiguous())
        if self.kind == "factorized":
            yt4, ylik4, _ = K.eb_likelihood(y4, M, ck.eb, True, ny4)
            liks = [ylik4]
        else:
            ha, hs = ck.ha, ck.hs
            a4 = K.abs_(y4)
            z1, _, _ = K.conv_down(a4, M, ha.convs[0].fwd, ha.convs[0].bias, N, 3, 1, K.EPI_RELU)
            z2, _, _ = K.conv_down(z1, N, ha.convs[1].fwd, ha.convs[1].bias, N, 5, 2, K.EPI_RELU)
            z4, _, _ = K.conv_down(z2, N, ha.convs[2].fwd, ha.convs[2].bias, N, 5, 2, K.EPI_BIAS)
            if noise_z is None:
                noise_z = torch.empty((B, N, H // 64, W // 64), device=x.device).uniform_(-0.5, 0.5)
            zt4, zlik4, _ = K.eb_likelihood(z4, N, ck.eb, True, K.to_nc4(noise_z.contiguous()))
            s1, _, _ = K.conv_up(zt4, N, hs.convs[0].fwd, hs.convs[0].bias, N, K.EPI_RELU, it=hs.convs[0].it_fwd)
            s2, _, _ = K.conv_up(s1, N, hs.convs[1].fwd, hs.convs[1].bias, N, K.EPI_RELU, it=hs.convs[1].it_fwd)
            sig4, _, _ = K.conv_down(s2, N, hs.convs[2].fwd, hs.convs[2].bias, M, 3, 1, K.EPI_RELU)
            yt4, ylik4, _ = K.gc_likelihood(y4, M, sig4, None, True, ny4)
            liks = [ylik4, zlik4]
        xh4, ss = ck.gs.forward(yt4, save=True, split=False)
        loss, bpp, dist, g4 = self._loss(xh4, x, liks, bscale)

        # ---- backward ----
        gyt = self._g_s_backward(ck.gs, g4, yt4, ss)
        del ss, g4
        if self.kind == "factorized":
            gv = self._eb_backward(ck, yt4, ylik4, M, gscale)
            gy = gyt.add_(gv)
        else:
            gl_y = K.bpp_grad(ylik4, gscale)
            gy_gc, gsig = K.gc_bwd(yt4, sig4, gl_y, M)
            gy = gyt.add_(gy_gc)
            # h_s backward
            g = K.relu_bwd_(gsig, sig4)
            K.wgrad(g, M, s2, N, 3, 1, self._g("h_s.4.weight"))
            K.channel_sum(g, M, self._g("h_s.4.bias"))
            g, _, _ = K.conv_down(g, M, hs.convs[2].bwd, None, N, 3, 1, K.EPI_BIAS)
            K.relu_bwd_(g, s2)
            K.wgrad(s1, N, g, N, 5, 2, self._g("h_s.2.weight"))
            K.channel_sum(g, N, self._g("h_s.2.bias"))
            g, _, _ = K.conv_down(g, N, hs.convs[1].bwd, None, N, 5, 2, K.EPI_BIAS)
            K.relu_bwd_(g, s1)
            K.wgrad(zt4, N, g, N, 5, 2, self._g("h_s.0.weight"))
            K.channel_sum(g, N, self._g("h_s.0.bias"))
            gz, _, _ = K.conv_down(g, N, hs.convs[0].bwd, None, N, 5, 2, K.EPI_BIAS)
            # EntropyBottleneck backward (z_tilde = z + u)
            gz.add_(self._eb_backward(ck, zt4, zlik4, N, gscale))
            # h_a backward
            K.wgrad(gz, N, z2, N, 5, 2, self._g("h_a.4.weight"))
            K.channel_sum(gz, N, self._g("h_a.4.bias"))
            g, _, _ = K.conv_up(gz, N, ha.convs[2].bwd, None, N, K.EPI_BIAS, it=ha.convs[2].it_bwd)
            K.relu_bwd_(g, z2)
            K.wgrad(g, N, z1, N, 5, 2, self._g("h_a.2.weight"))
            K.channel_sum(g, N, self._g("h_a.2.bias"))
            g, _, _ = K.conv_up(g, N, ha.convs[1].bwd, None, N, K.EPI_BIAS, it=ha.convs[1].it_bwd)
            K.relu_bwd_(g, z1)
            K.wgrad(g, N, a4, M, 3, 1, self._g("h_a.0.weight"))
            K.channel_sum(g, N, self._g("h_a.0.bias"))
            g, _, _ = K.conv_down(g, N, ha.convs[0].bwd, None, M, 3, 1, K.EPI_BIAS)
            gy.add_(K.abs_bwd_(g, y4))
        self._g_a_backward(ck.ga, gy, x4, sa)
        return {"loss": loss, "bpp_loss": bpp, "distortion_loss": dist}
