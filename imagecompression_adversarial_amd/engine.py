"""Executors for the CompressAI transforms on the HIP kernels.

``CodecKernels`` holds the packed weight fragments of one model (built once per
weight version) and runs the fused layer chains:

  g_a forward   : conv_down[+GDN epilogue] x3 -> conv_down            (anchors/utils.py:112-119, utils/ops.py:83-97)
  g_s forward   : conv_up[+IGDN epilogue] x3 -> conv_up               (anchors/utils.py:122-130)
  g_s backward  : conv_down[dgrad + IGDN-bwd epilogue] x3 -> conv_down
  g_a backward  : conv_up[dgrad + GDN-bwd epilogue] x3 -> conv_up
  h_a / h_s     : conv k3 s1 / k5 s2 / deconv k5 s2 with ReLU epilogues (CompressAI ScaleHyperprior)
  entropy       : EntropyBottleneck + GaussianConditional likelihood kernels

All tensors are nChw4c device tensors (see hip_ops).  Input-gradient paths
only: the attack freezes the codec (the reference computes unused weight
gradients).
"""
from __future__ import annotations

import torch

from . import hip_ops as K


class CodecKernels:
    def __init__(self, sd: dict, model: str = "hyper"):
        self.model = model
        dev = sd["g_a.0.weight"].device
        if dev.type != "cuda":
            raise RuntimeError("CodecKernels needs the state dict on the HIP device")
        self.N = sd["g_a.0.weight"].shape[0]
        self.M = sd["g_a.6.weight"].shape[0]
        self.ga = [K.PackedConv(sd[f"g_a.{i}.weight"], sd[f"g_a.{i}.bias"], "conv", 2) for i in (0, 2, 4, 6)]
        self.gs = [K.PackedConv(sd[f"g_s.{i}.weight"], sd[f"g_s.{i}.bias"], "deconv", 2) for i in (0, 2, 4, 6)]
        self.ga_gdn = [K.PackedGDN(sd[f"g_a.{i}.beta"], sd[f"g_a.{i}.gamma"]) for i in (1, 3, 5)]
        self.gs_gdn = [K.PackedGDN(sd[f"g_s.{i}.beta"], sd[f"g_s.{i}.gamma"]) for i in (1, 3, 5)]
        if model == "hyper":
            self.ha = [K.PackedConv(sd["h_a.0.weight"], sd["h_a.0.bias"], "conv", 1),
                       K.PackedConv(sd["h_a.2.weight"], sd["h_a.2.bias"], "conv", 2),
                       K.PackedConv(sd["h_a.4.weight"], sd["h_a.4.bias"], "conv", 2)]
            self.hs = [K.PackedConv(sd["h_s.0.weight"], sd["h_s.0.bias"], "deconv", 2),
                       K.PackedConv(sd["h_s.2.weight"], sd["h_s.2.bias"], "deconv", 2),
                       K.PackedConv(sd["h_s.4.weight"], sd["h_s.4.bias"], "conv", 1)]
        eb = {n: sd[f"entropy_bottleneck.{n}"] for n in K.PackedEB.NAMES}
        self.eb = K.PackedEB(eb)

    # ------------------------------------------------------------------ g_a
    def g_a(self, x4, save=False):
        h, C, saved = x4, 3, []
        for i in range(3):
            p = self.ga[i]
            h, sx, ss = K.conv_down(h, C, p.fwd, p.bias, self.N, 5, 2, K.EPI_GDN, self.ga_gdn[i], save,
                                    tag=f"g_a.{2 * i}.fwd")
            saved.append((sx, ss))
            C = self.N
        p = self.ga[3]
        y, _, _ = K.conv_down(h, self.N, p.fwd, p.bias, self.M, 5, 2, K.EPI_BIAS, tag="g_a.6.fwd")
        return y, saved

    def g_a_backward(self, gy4, saved):
        g, C = gy4, self.M
        for i in (3, 2, 1):
            g, _, _ = K.conv_up(g, C, self.ga[i].bwd, None, self.N, K.EPI_GDN_BWD, self.ga_gdn[i - 1],
                                saved=saved[i - 1], tag=f"g_a.{2 * i}.dgrad")
            C = self.N
        gx, _, _ = K.conv_up(g, self.N, self.ga[0].bwd, None, 3, K.EPI_BIAS, tag="g_a.0.dgrad")
        return gx

    # ------------------------------------------------------------------ g_s
    def g_s(self, y4, save=False):
        h, C, saved = y4, self.M, []
        for i in range(3):
            p = self.gs[i]
            h, sx, ss = K.conv_up(h, C, p.fwd, p.bias, self.N, K.EPI_IGDN, self.gs_gdn[i], save,
                                  tag=f"g_s.{2 * i}.fwd")
            saved.append((sx, ss))
            C = self.N
        p = self.gs[3]
        xh, _, _ = K.conv_up(h, self.N, p.fwd, p.bias, 3, K.EPI_BIAS, tag="g_s.6.fwd")
        return xh, saved

    def g_s_backward(self, gx4, saved):
        g, C = gx4, 3
        for i in (3, 2, 1):
            g, _, _ = K.conv_down(g, C, self.gs[i].bwd, None, self.N, 5, 2, K.EPI_IGDN_BWD, self.gs_gdn[i - 1],
                                  saved=saved[i - 1], tag=f"g_s.{2 * i}.dgrad")
            C = self.N
        gy, _, _ = K.conv_down(g, self.N, self.gs[0].bwd, None, self.M, 5, 2, K.EPI_BIAS, tag="g_s.0.dgrad")
        return gy

    # ------------------------------------------------------------------ hyperprior
    def h_a(self, y4):
        a = K.abs_(y4)
        p0, p1, p2 = self.ha
        z, _, _ = K.conv_down(a, self.M, p0.fwd, p0.bias, self.N, 3, 1, K.EPI_RELU)
        z, _, _ = K.conv_down(z, self.N, p1.fwd, p1.bias, self.N, 5, 2, K.EPI_RELU)
        z, _, _ = K.conv_down(z, self.N, p2.fwd, p2.bias, self.N, 5, 2, K.EPI_BIAS)
        return z

    def h_s(self, z4):
        p0, p1, p2 = self.hs
        s, _, _ = K.conv_up(z4, self.N, p0.fwd, p0.bias, self.N, K.EPI_RELU)
        s, _, _ = K.conv_up(s, self.N, p1.fwd, p1.bias, self.N, K.EPI_RELU)
        s, _, _ = K.conv_down(s, self.N, p2.fwd, p2.bias, self.M, 3, 1, K.EPI_RELU)
        return s

    def forward(self, x4, training=False, noise_y4=None, noise_z4=None):
        """net(x) (anchors/balle.py:25-55): returns x_hat4, y4, likelihood tensors and per-image sum log p."""
        y4, _ = self.g_a(x4)
        if self.model == "factorized":
            yh, ylik, ysum = K.eb_likelihood(y4, self.M, self.eb, training, noise_y4)
            xh, _ = self.g_s(yh)
            return {"x_hat4": xh, "y4": y4, "lik4": {"y": ylik}, "sumlog": ysum}
        z4 = self.h_a(y4)
        zh, zlik, zsum = K.eb_likelihood(z4, self.N, self.eb, training, noise_z4)
        s4 = self.h_s(zh)
        yh, ylik, ysum = K.gc_likelihood(y4, self.M, s4, None, training, noise_y4)
        xh, _ = self.g_s(yh)
        return {"x_hat4": xh, "y4": y4, "z4": z4, "lik4": {"y": ylik, "z": zlik}, "sumlog": ysum + zsum}
