"""Executors for the CompressAI transforms on the HIP kernels.

Per-transform executors hold the packed weight fragments (built once per
weight version) and run the fused layer chains:

  Analysis  (g_a)  forward : conv_down[+GDN epilogue] x3 -> conv_down      (anchors/utils.py:112-119, utils/ops.py:83-97)
                   backward: conv_up[dgrad + GDN-bwd epilogue] x3 -> conv_up3 (Z-gather, 3 channels)
  Synthesis (g_s)  forward : conv_up[+IGDN epilogue] x3 -> conv_up3          (anchors/utils.py:122-130)
                   backward: conv_down[dgrad + IGDN-bwd epilogue] x3 -> conv_down
  HyperAnalysis / HyperSynthesis (h_a / h_s): conv k3 s1 / k5 s2, deconv k5 s2, ReLU epilogues
  entropy: EntropyBottleneck + GaussianConditional likelihood kernels

All tensors are nChw4c device tensors (see hip_ops).  Input-gradient paths
only: the attack freezes the codec (the reference computes unused weight
gradients).
"""
from __future__ import annotations

import torch

from . import hip_ops as K


def _P(sd, prefix, name):
    return sd[f"{prefix}.{name}" if prefix else name]


class Saved(list):
    """The per-layer (y, s) pairs a forward saves for its backward, and which levels (L0 = image ... L4 = latent)
    were stored parity-split (the backward must address them the same way)."""

    def __init__(self, items=(), split=(False,) * 5, exact=True):
        super().__init__(items)
        self.split = tuple(split)
        self.exact = exact   # every level exactly halves the one above (input sides multiples of 16)


def _layout_of(saved):
    """The forward's layout record; a plain list would lose it (and a split forward would be misread)."""
    if not isinstance(saved, Saved):
        raise TypeError("backward needs the forward's Saved record (keep its type when selecting rows)")
    return saved.split


def _lay(lv, a, b):
    """layout of a launch from level a to level b"""
    return (K.LAYOUT_IN if lv[a] else 0) | (K.LAYOUT_OUT if lv[b] else 0)


def _levels(split):
    """split (True / False / per-level (L1, L2, L3) flags) -> flags of L0..L4 (the image and the latent: never)"""
    if isinstance(split, (tuple, list)):
        s = tuple(bool(v) for v in split)
    else:
        s = (bool(split),) * 3
    return (False,) + s + (False,)


def _split_policy(convs):
    """Which inner levels (L1, L2, L3) of the k5 s2 stacks are stored parity-split.  Every conv
    kernel addresses that order (ica_conv_args.layout), so this is a measured choice per operand path: x6 and bf16
    store all three split (config 2: 1351 -> 1371 img-step/s; config 5: 390 -> 394, where the L1 conv_up launches
    gain 1.6 ms and the bf16 RGB-end kernels give back 0.7 of it; L1 row-major measured 393); the fp32 kernels are
    MFMA-bound and the split's address arithmetic cost them 0.5 % (779 -> 775), so fp32 stays row-major."""
    precs = {c.fwd_prec for c in convs} | {c.bwd_prec for c in convs}
    if precs & {K.PREC_X6, K.PREC_BF16}:
        return (True, True, True)
    return (False, False, False)


class Analysis:
    """g_a = conv(3,N)-GDN-conv(N,N)-GDN-conv(N,N)-GDN-conv(N,M), all k5 s2."""

    def __init__(self, sd: dict, prefix: str = "g_a", tag: str = "g_a", prec: int = K.PREC_FP32):
        self.tag = tag
        self.N = _P(sd, prefix, "0.weight").shape[0]
        self.M = _P(sd, prefix, "6.weight").shape[0]
        # C = 192 GDN layers (q6-8) run 6 row tiles per wave: convs 0-2 forward, convs 1-3 input-gradient
        g6 = 6 if self.N == 192 else 0
        self.convs = [K.PackedConv(_P(sd, prefix, f"{i}.weight"), _P(sd, prefix, f"{i}.bias"), "conv", 2, prec,
                                   it_fwd=g6 if i < 6 else 0, it_bwd=g6 if i > 0 else 0)
                      for i in (0, 2, 4, 6)]
        self.gdns = [K.PackedGDN(_P(sd, prefix, f"{i}.beta"), _P(sd, prefix, f"{i}.gamma")) for i in (1, 3, 5)]
        self.split = _split_policy(self.convs)

    def forward(self, x4, save=False, split=None):
        """split: which inner levels (L1, L2, L3) to store parity-split (True / False / per-level flags; default
        the operand path's policy), each only when its sides are even; the transform's output y and its input
        gradient stay row-major either way."""
        H, W = x4.shape[2], x4.shape[3]
        lv = _levels(self.split if split is None else split)
        lv = tuple(f and ((H + (1 << k) - 1) >> k) % 2 == 0 and ((W + (1 << k) - 1) >> k) % 2 == 0
                   for k, f in enumerate(lv))
        h, C, saved = x4, 3, Saved(split=lv, exact=H % 16 == 0 and W % 16 == 0)
        for i in range(3):   # layer i: level i -> level i + 1
            p = self.convs[i]
            h, sx, ss = K.conv_down(h, C, p.fwd, p.bias, self.N, 5, 2, K.EPI_GDN, self.gdns[i], save,
                                    tag=f"{self.tag}.{2 * i}.fwd", prec=p.fwd_prec, it=p.it_fwd,
                                    layout=_lay(lv, i, i + 1))
            saved.append((sx, ss))
            C = self.N
        p = self.convs[3]
        y, _, _ = K.conv_down(h, self.N, p.fwd, p.bias, self.M, 5, 2, K.EPI_BIAS, tag=f"{self.tag}.6.fwd",
                              prec=p.fwd_prec, layout=_lay(lv, 3, 4))
        return y, saved

    def backward(self, gy4, saved):
        lv = _layout_of(saved)
        if not saved.exact:
            # the input gradients are 2x transposed convs: an odd level (sides not multiples of 16) has no
            # exact transpose here (the attack pads its images to multiples of 64, coder.read_image)
            raise ValueError("g_a input gradient: image sides must be multiples of 16")
        g, C = gy4, self.M
        for i in (3, 2, 1):
            g, _, _ = K.conv_up(g, C, self.convs[i].bwd, None, self.N, K.EPI_GDN_BWD, self.gdns[i - 1],
                                saved=saved[i - 1], tag=f"{self.tag}.{2 * i}.dgrad", prec=self.convs[i].bwd_prec,
                                it=self.convs[i].it_bwd, layout=_lay(lv, i + 1, i))
            C = self.N
        gx, _, _ = K.conv_up(g, self.N, self.convs[0].bwd, None, 3, K.EPI_BIAS, tag=f"{self.tag}.0.dgrad",
                             prec=self.convs[0].bwd_prec, layout=_lay(lv, 1, 0))
        return gx


class Synthesis:
    """g_s = deconv(M,N)-IGDN-deconv(N,N)-IGDN-deconv(N,N)-IGDN-deconv(N,3), all k5 s2 op1."""

    def __init__(self, sd: dict, prefix: str = "g_s", tag: str = "g_s", prec: int = K.PREC_FP32):
        self.tag = tag
        self.M = _P(sd, prefix, "0.weight").shape[0]
        self.N = _P(sd, prefix, "0.weight").shape[1]
        # C = 192 IGDN layers (q6-8): deconvs 0-2 forward, deconvs 1-3 input-gradient (conv_down into N channels)
        g6 = 6 if self.N == 192 else 0
        self.convs = [K.PackedConv(_P(sd, prefix, f"{i}.weight"), _P(sd, prefix, f"{i}.bias"), "deconv", 2, prec,
                                   it_fwd=g6 if i < 6 else 0, it_bwd=g6 if i > 0 else 0)
                      for i in (0, 2, 4, 6)]
        self.gdns = [K.PackedGDN(_P(sd, prefix, f"{i}.beta"), _P(sd, prefix, f"{i}.gamma")) for i in (1, 3, 5)]
        self.split = _split_policy(self.convs)

    def forward(self, y4, save=False, split=None):
        """split: as Analysis.forward (the inner levels are 2x, 4x, 8x the latent sides: always even)."""
        lv = _levels(self.split if split is None else split)
        h, C, saved = y4, self.M, Saved(split=lv)
        for i in range(3):   # layer i: level 4 - i -> level 3 - i
            p = self.convs[i]
            h, sx, ss = K.conv_up(h, C, p.fwd, p.bias, self.N, K.EPI_IGDN, self.gdns[i], save,
                                  tag=f"{self.tag}.{2 * i}.fwd", prec=p.fwd_prec, it=p.it_fwd,
                                  layout=_lay(lv, 4 - i, 3 - i))
            saved.append((sx, ss))
            C = self.N
        p = self.convs[3]
        xh, _, _ = K.conv_up(h, self.N, p.fwd, p.bias, 3, K.EPI_BIAS, tag=f"{self.tag}.6.fwd", prec=p.fwd_prec,
                             layout=_lay(lv, 1, 0))
        return xh, saved

    def backward(self, gx4, saved):
        lv = _layout_of(saved)
        g, C = gx4, 3
        for i in (3, 2, 1):   # level 3 - i -> level 4 - i
            g, _, _ = K.conv_down(g, C, self.convs[i].bwd, None, self.N, 5, 2, K.EPI_IGDN_BWD, self.gdns[i - 1],
                                  saved=saved[i - 1], tag=f"{self.tag}.{2 * i}.dgrad", prec=self.convs[i].bwd_prec,
                                  it=self.convs[i].it_bwd, layout=_lay(lv, 3 - i, 4 - i))
            C = self.N
        gy, _, _ = K.conv_down(g, self.N, self.convs[0].bwd, None, self.M, 5, 2, K.EPI_BIAS,
                               tag=f"{self.tag}.0.dgrad", prec=self.convs[0].bwd_prec, layout=_lay(lv, 3, 4))
        return gy


class HyperAnalysis:
    """h_a = conv(M,N,k3,s1)-ReLU-conv(N,N)-ReLU-conv(N,N) applied to |y| (CompressAI ScaleHyperprior)."""

    def __init__(self, sd: dict, prefix: str = "h_a"):
        self.M = _P(sd, prefix, "0.weight").shape[1]
        self.N = _P(sd, prefix, "0.weight").shape[0]
        # q6-8 (N = 192): the k5 s2 input-gradients (conv_up into 192 channels, the fine-tune) run 6 row tiles
        r6 = 6 if self.N == 192 else 0
        self.convs = [K.PackedConv(_P(sd, prefix, "0.weight"), _P(sd, prefix, "0.bias"), "conv", 1),
                      K.PackedConv(_P(sd, prefix, "2.weight"), _P(sd, prefix, "2.bias"), "conv", 2, it_bwd=r6),
                      K.PackedConv(_P(sd, prefix, "4.weight"), _P(sd, prefix, "4.bias"), "conv", 2, it_bwd=r6)]

    def forward(self, y4, take_abs=True):
        a = K.abs_(y4) if take_abs else y4
        p0, p1, p2 = self.convs
        z, _, _ = K.conv_down(a, self.M, p0.fwd, p0.bias, self.N, 3, 1, K.EPI_RELU)
        z, _, _ = K.conv_down(z, self.N, p1.fwd, p1.bias, self.N, 5, 2, K.EPI_RELU)
        z, _, _ = K.conv_down(z, self.N, p2.fwd, p2.bias, self.N, 5, 2, K.EPI_BIAS)
        return z


class HyperSynthesis:
    """h_s = deconv(N,N)-ReLU-deconv(N,N)-ReLU-conv(N,M,k3,s1)-ReLU."""

    def __init__(self, sd: dict, prefix: str = "h_s"):
        self.N = _P(sd, prefix, "0.weight").shape[0]
        self.M = _P(sd, prefix, "4.weight").shape[0]
        r6 = 6 if self.N == 192 else 0   # q6-8: ReLU deconvs into 192 channels (6 row tiles)
        self.convs = [K.PackedConv(_P(sd, prefix, "0.weight"), _P(sd, prefix, "0.bias"), "deconv", 2, it_fwd=r6),
                      K.PackedConv(_P(sd, prefix, "2.weight"), _P(sd, prefix, "2.bias"), "deconv", 2, it_fwd=r6),
                      K.PackedConv(_P(sd, prefix, "4.weight"), _P(sd, prefix, "4.bias"), "conv", 1)]

    def forward(self, z4):
        p0, p1, p2 = self.convs
        s, _, _ = K.conv_up(z4, self.N, p0.fwd, p0.bias, self.N, K.EPI_RELU, it=p0.it_fwd)
        s, _, _ = K.conv_up(s, self.N, p1.fwd, p1.bias, self.N, K.EPI_RELU, it=p1.it_fwd)
        s, _, _ = K.conv_down(s, self.N, p2.fwd, p2.bias, self.M, 3, 1, K.EPI_RELU)
        return s


class MbtHyperAnalysis:
    """mbt2018 h_a = conv(M,N,k3,s1)-LReLU-conv(N,N,k5,s2)-LReLU-conv(N,N,k5,s2), applied to y itself
    (anchors/model.py:97 ``net.h_a(y)``; CompressAI JointAutoregressiveHierarchicalPriors)."""

    def __init__(self, sd: dict, prefix: str = "h_a"):
        self.M = _P(sd, prefix, "0.weight").shape[1]
        self.N = _P(sd, prefix, "0.weight").shape[0]
        self.convs = [K.PackedConv(_P(sd, prefix, "0.weight"), _P(sd, prefix, "0.bias"), "conv", 1),
                      K.PackedConv(_P(sd, prefix, "2.weight"), _P(sd, prefix, "2.bias"), "conv", 2),
                      K.PackedConv(_P(sd, prefix, "4.weight"), _P(sd, prefix, "4.bias"), "conv", 2)]

    def forward(self, y4):
        p0, p1, p2 = self.convs
        z, _, _ = K.conv_down(y4, self.M, p0.fwd, p0.bias, self.N, 3, 1, K.EPI_LRELU)
        z, _, _ = K.conv_down(z, self.N, p1.fwd, p1.bias, self.N, 5, 2, K.EPI_LRELU)
        z, _, _ = K.conv_down(z, self.N, p2.fwd, p2.bias, self.N, 5, 2, K.EPI_BIAS)
        return z


def _up_it(C):
    """Row tiles per wave for the k5 transposed convs (conv_up runs IT in {1, 4, 6})."""
    return 6 if C == 192 else (1 if C <= 32 else 4)


class MbtHyperSynthesis:
    """mbt2018 h_s = deconv(N,M)-LReLU-deconv(M,3M/2)-LReLU-conv(3M/2,2M,k3,s1): the hyper half of the
    (scales, means) parameters fed to entropy_parameters."""

    def __init__(self, sd: dict, prefix: str = "h_s"):
        self.N = _P(sd, prefix, "0.weight").shape[0]
        self.M = _P(sd, prefix, "0.weight").shape[1]
        self.M3 = _P(sd, prefix, "2.weight").shape[1]
        self.out_channels = _P(sd, prefix, "4.weight").shape[0]
        self.convs = [K.PackedConv(_P(sd, prefix, "0.weight"), _P(sd, prefix, "0.bias"), "deconv", 2,
                                   it_fwd=_up_it(self.M)),
                      K.PackedConv(_P(sd, prefix, "2.weight"), _P(sd, prefix, "2.bias"), "deconv", 2,
                                   it_fwd=_up_it(self.M3)),
                      K.PackedConv(_P(sd, prefix, "4.weight"), _P(sd, prefix, "4.bias"), "conv", 1)]

    def forward(self, z4):
        p0, p1, p2 = self.convs
        s, _, _ = K.conv_up(z4, self.N, p0.fwd, p0.bias, self.M, K.EPI_LRELU, it=p0.it_fwd)
        s, _, _ = K.conv_up(s, self.M, p1.fwd, p1.bias, self.M3, K.EPI_LRELU, it=p1.it_fwd)
        s, _, _ = K.conv_down(s, self.M3, p2.fwd, p2.bias, self.out_channels, 3, 1, K.EPI_BIAS)
        return s


class CodecKernels:
    """Whole-model executor from a CompressAI-format state dict (device tensors)."""

    def __init__(self, sd: dict, model: str = "hyper", precision: str = "fp32"):
        """precision 'x6': the k5 s2 g_a / g_s layers run the fp32-accurate bf16x6 kernels (ica_conv_x6.hip: exact
        3-way bf16 operand splits, six products, fp32 accumulate and fp32 epilogues / storage); 'fp32': fp32-operand
        MFMA everywhere; 'bf16': bf16-operand MFMA convs (fp32 accumulate, bf16 activations; BASELINE config 5,
        SURVEY §8f rank 1).  h_a / h_s and the entropy models stay fp32."""
        self.model = model
        if precision not in ("fp32", "bf16", "x6"):
            raise ValueError(f"precision {precision!r}: fp32 | x6 | bf16")
        self.precision = precision
        prec = {"fp32": K.PREC_FP32, "bf16": K.PREC_BF16, "x6": K.PREC_X6}[precision]
        if sd["g_a.0.weight"].device.type != "cuda":
            raise RuntimeError("CodecKernels needs the state dict on the HIP device")
        self.ga = Analysis(sd, prec=prec)
        self.gs = Synthesis(sd, prec=prec)
        self.N, self.M = self.ga.N, self.ga.M
        if model == "hyper":
            self.ha = HyperAnalysis(sd)
            self.hs = HyperSynthesis(sd)
        elif model == "context":   # mbt2018: masked 5x5 context model + 1x1 entropy_parameters stack
            from .engine_cheng import ChengContext, ChengEntropyParameters
            self.ha = MbtHyperAnalysis(sd)
            self.hs = MbtHyperSynthesis(sd)
            self.ctx = ChengContext(sd)
            self.ep = ChengEntropyParameters(sd)
        self.eb = K.PackedEB({n: sd[f"entropy_bottleneck.{n}"] for n in K.PackedEB.NAMES})

    # thin aliases used by the attack loop
    def g_a(self, x4, save=False):
        return self.ga.forward(x4, save)

    def g_a_backward(self, gy4, saved):
        return self.ga.backward(gy4, saved)

    def g_s(self, y4, save=False):
        return self.gs.forward(y4, save)

    def g_s_backward(self, gx4, saved):
        return self.gs.backward(gx4, saved)

    def _to_gs(self, yh4):
        """y_hat into g_s: bf16 activations on the bf16 path (rounded latents are exact in bf16 up to 256)."""
        return K.cast_nc4(yh4, torch.bfloat16) if self.precision == "bf16" else yh4

    def forward(self, x4, training=False, noise_y4=None, noise_z4=None):
        """net(x) (anchors/balle.py:25-55): x_hat4, y4, likelihood tensors and per-image sum log p."""
        y4, _ = self.ga.forward(x4)
        if self.precision == "bf16":   # the entropy models and h_a run fp32
            y4 = K.cast_nc4(y4, torch.float32)
        if self.model == "factorized":
            yh, ylik, ysum = K.eb_likelihood(y4, self.M, self.eb, training, noise_y4)
            xh, _ = self.gs.forward(self._to_gs(yh))
            return {"x_hat4": xh, "y4": y4, "y_hat4": yh, "lik4": {"y": ylik}, "sumlog": ysum}
        if self.model == "context":
            return self._forward_context(y4, training)
        z4 = self.ha.forward(y4)
        zh, zlik, zsum = K.eb_likelihood(z4, self.N, self.eb, training, noise_z4)
        s4 = self.hs.forward(zh)
        yh, ylik, ysum = K.gc_likelihood(y4, self.M, s4, None, training, noise_y4)
        xh, _ = self.gs.forward(self._to_gs(yh))
        return {"x_hat4": xh, "y4": y4, "y_hat4": yh, "z4": z4, "z_hat4": zh, "scales4": s4,
                "lik4": {"y": ylik, "z": zlik}, "sumlog": ysum + zsum}

    def _forward_context(self, y4, training):
        """entropy_estimator for MODEL == "context" (anchors/model.py:95-104) + g_s(y_hat), eval mode:
        y_hat = round(y) (quantize "dequantize", no means), params = h_s(z_hat), ctx = masked conv(y_hat),
        (scales, means) = entropy_parameters(cat(params, ctx)).chunk(2), GC likelihood with means."""
        if training:
            raise NotImplementedError("mbt2018 runs eval-mode forwards only (attack path)")
        M = self.M
        z4 = self.ha.forward(y4)
        zh, zlik, zsum = K.eb_likelihood(z4, self.N, self.eb, False, None)
        params = self.hs.forward(zh)
        y_hat4 = K.round_(y4)
        ctx = self.ctx.forward(y_hat4)
        gp = self.ep.forward(torch.cat((params, ctx), dim=1))   # channel concat of nChw4c tensors (M % 4 == 0)
        c4 = (M + 3) // 4
        scales4 = gp[:, :c4].contiguous()
        means4 = gp[:, c4:].contiguous()
        _, ylik, ysum = K.gc_likelihood(y4, M, scales4, means4, False, None)
        xh, _ = self.gs.forward(self._to_gs(y_hat4))
        return {"x_hat4": xh, "y4": y4, "y_hat4": y_hat4, "z4": z4, "z_hat4": zh, "scales4": scales4,
                "means4": means4, "lik4": {"y": ylik, "z": zlik}, "sumlog": ysum + zsum}
