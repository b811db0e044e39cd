"""Train-mode forward + RateDistortionLoss + backward of mbt2018 (CompressAI JointAutoregressiveHierarchicalPriors,
``-m context``) on the HIP kernels: the adversarial fine-tune's inner piece (train.py --adv, reference
``/root/reference/train.py:249-366``) for the context-model codec.  The oracle's restatement is
``oracle/codec.mbt_forward`` (training=True).

  loss -> x_hat -> g_s (bmshj2018 k5 s2 deconvs + IGDN: train_engine.synthesis_backward) -> y_hat
       <- context_prediction^T <- entropy_parameters^T <- GC bwd (scales, means)   (train_cheng.context_backward)
       -> h_s^T (deconv k5 s2, leaky ReLU; conv k3) -> z_tilde <- EB bwd -> h_a^T (conv k5 s2 / k3, leaky ReLU)
       -> y -> g_a (k5 s2 convs + GDN: train_engine.analysis_backward)

All operands fp32; the deconv weight gradients are ica_wgrad with the roles of input and output gradient swapped
(include/ica_hip.h)."""
from __future__ import annotations

import math

import torch

from . import hip_ops as K
from .train_cheng import ChengTrainStep, entropy_forward
from .train_engine import analysis_backward, synthesis_backward


def _it192(C):
    return 6 if C == 192 else 0


def train_forward(ck, P, x4, noise_y=None, noise_z=None):
    """mbt_forward (training=True) with the activations the backward reads.  ck: the model's fp32 CodecKernels;
    P(name): the detached parameter."""
    B = x4.shape[0]
    N, M = ck.N, ck.M
    y4, sa = ck.ga.forward(x4, save=True, split=False)
    pc = lambda pre, kind, s, **kw: K.PackedConv(P(f"{pre}.weight"), P(f"{pre}.bias"), kind, s, **kw)  # noqa: E731
    ha = [pc("h_a.0", "conv", 1), pc("h_a.2", "conv", 2, it_bwd=_it192(N)), pc("h_a.4", "conv", 2, it_bwd=_it192(N))]
    z0, _, _ = K.conv_down(y4, M, ha[0].fwd, ha[0].bias, N, 3, 1, K.EPI_LRELU)
    z1, _, _ = K.conv_down(z0, N, ha[1].fwd, ha[1].bias, N, 5, 2, K.EPI_LRELU)
    z4, _, _ = K.conv_down(z1, N, ha[2].fwd, ha[2].bias, N, 5, 2, K.EPI_BIAS)
    if noise_z is None:
        noise_z = torch.empty((B, N, z4.shape[2], z4.shape[3]), device=x4.device).uniform_(-0.5, 0.5)
    zt4, zlik4, _ = K.eb_likelihood(z4, N, ck.eb, True, K.to_nc4(noise_z.contiguous()))
    hs = ck.hs
    M3 = hs.M3
    s0, _, _ = K.conv_up(zt4, N, hs.convs[0].fwd, hs.convs[0].bias, M, K.EPI_LRELU, it=hs.convs[0].it_fwd)
    s1, _, _ = K.conv_up(s0, M, hs.convs[1].fwd, hs.convs[1].bias, M3, K.EPI_LRELU, it=hs.convs[1].it_fwd)
    params4, _, _ = K.conv_down(s1, M3, hs.convs[2].fwd, hs.convs[2].bias, 2 * M, 3, 1, K.EPI_BIAS)
    ent = entropy_forward(P, y4, M, params4, noise_y)
    xh4, ss = ck.gs.forward(ent["yh4"], save=True, split=False)
    out = {k: v for k, v in locals().items() if k not in ("ck", "P", "B", "pc", "ent")}
    out.update(ent)
    return out


class MbtTrainStep(ChengTrainStep):
    """One train-mode forward / loss / backward of a ``codec.JointAutoregressiveHierarchicalPriors``."""

    def step(self, x, noise_y=None, noise_z=None):
        tr = self.tr
        x = x.contiguous()
        B, _, H, W = x.shape
        ck = tr.net.kernels("fp32")
        N, M = ck.N, ck.M
        tr.flat_grad.zero_()
        tr._attach_grads()
        x4 = K.to_nc4(x)
        bscale = 1.0 / (-math.log(2) * B * H * W)
        gscale = bscale * tr.lamb_r
        f = train_forward(ck, self._p, x4, noise_y, noise_z)
        loss, bpp, dist, g4 = tr._loss(f["xh4"], x, [f["ylik4"], f["zlik4"]], bscale)

        gy = synthesis_backward(ck.gs, g4, f["yh4"], f["ss"], tr.params, tr.views, "g_s.")
        del g4
        gparams = self.context_backward(gy, f["ylik4"], gscale, f["yt4"], f["means4"], f["scales4"], M, f["ep"],
                                        f["t0"], f["e0"], f["e1"], f["params4"], f["yh4"], f["ctxc"])
        # h_s backward: conv k3 (3M/2 -> 2M), deconv k5 s2 (M -> 3M/2) + LReLU, deconv k5 s2 (N -> M) + LReLU
        hs, M3, s0, s1 = ck.hs, f["M3"], f["s0"], f["s1"]
        self._wb(gparams, 2 * M, s1, M3, 3, 1, "h_s.4")
        g, _, _ = K.conv_down(gparams, 2 * M, hs.convs[2].bwd, None, M3, 3, 1, K.EPI_BIAS)
        g = K.lrelu_bwd(g, s1)
        K.wgrad(s0, M, g, M3, 5, 2, self._g("h_s.2.weight"), tag="h_s.2.wgrad")
        K.channel_sum(g, M3, self._g("h_s.2.bias"))
        g, _, _ = K.conv_down(g, M3, hs.convs[1].bwd, None, M, 5, 2, K.EPI_BIAS)
        g = K.lrelu_bwd(g, s0)
        K.wgrad(f["zt4"], N, g, M, 5, 2, self._g("h_s.0.weight"), tag="h_s.0.wgrad")
        K.channel_sum(g, M, self._g("h_s.0.bias"))
        gz, _, _ = K.conv_down(g, M, hs.convs[0].bwd, None, N, 5, 2, K.EPI_BIAS)
        gz.add_(tr._eb_backward(ck, f["zt4"], f["zlik4"], N, gscale))   # z_tilde = z + u
        # h_a backward: conv k5 s2 (N -> N), LReLU, conv k5 s2, LReLU, conv k3 (M -> N)
        ha, z0, z1 = f["ha"], f["z0"], f["z1"]
        self._wb(gz, N, z1, N, 5, 2, "h_a.4")
        g, _, _ = K.conv_up(gz, N, ha[2].bwd, None, N, K.EPI_BIAS, it=ha[2].it_bwd)
        g = K.lrelu_bwd(g, z1)
        self._wb(g, N, z0, N, 5, 2, "h_a.2")
        g, _, _ = K.conv_up(g, N, ha[1].bwd, None, N, K.EPI_BIAS, it=ha[1].it_bwd)
        g = K.lrelu_bwd(g, z0)
        self._wb(g, N, f["y4"], M, 3, 1, "h_a.0")
        g, _, _ = K.conv_down(g, N, ha[0].bwd, None, M, 3, 1, K.EPI_BIAS)
        gy.add_(g)
        analysis_backward(ck.ga, gy, x4, f["sa"], tr.params, tr.views, "g_a.")
        return {"loss": loss, "bpp_loss": bpp, "distortion_loss": dist}
