"""Executor for the reference's "debug" model, ae_onelayer(N=3, M=192) (anchors/model.py:8-33, 60-68): g_a one
3x3 stride-1 conv (3 -> 192), g_s one 3x3 stride-1 transposed conv (192 -> 3), around CompressAI's mean-scale
hyperprior (mbt2018's h_a / h_s without the context model, N = 3).  Its forward reconstructs from the
unquantised latent (x_hat = g_s(y), anchors/model.py:30) and its attack runs on an unclamped input from a random
start (attack_rd.py:493-494, 514-515): clamp_input = False tells the attack loop (attack.AttackLoop).

Kernel mapping: both transforms are the k3 stride-1 conv_down of the cheng2020 engine (engine_cheng.Conv3); the
transposed conv is the same conv with the weight's channel axes swapped and its taps reversed.  The 3-channel
sides (the image into g_a, the image gradient into g_s's input gradient, z_hat into h_s.0) are carried as 16
channels, zero past the third, with zero weight columns: the 16-channel chunk kernels then run them unchanged,
and the zero channels contribute exact zeros.  fp32 operands (the layers are 3 wide on one side: no x6 packs)."""
from __future__ import annotations

import torch

from . import hip_ops as K
from .engine import MbtHyperAnalysis, MbtHyperSynthesis, _P
from .engine_cheng import Conv3

CP = 16   # channels the 3-channel sides are carried at


def pad_nc4(x4: torch.Tensor, C: int = CP) -> torch.Tensor:
    """An nChw4c tensor of <= 4 channels (one quad) as C channels, zero past the quad."""
    N, q, H, W, _ = x4.shape
    out = torch.zeros((N, K.c4(C), H, W, 4), dtype=x4.dtype, device=x4.device)
    out[:, :q].copy_(x4)
    return out


def _pad_dim(w: torch.Tensor, dim: int, n: int = CP) -> torch.Tensor:
    w = w.detach()
    shape = list(w.shape)
    shape[dim] = n
    out = torch.zeros(shape, dtype=w.dtype, device=w.device)
    out.narrow(dim, 0, w.shape[dim]).copy_(w)
    return out


class DebugAnalysis:
    """g_a = conv(3, M, kernel_size=3, stride=1) (anchors/model.py:13-15); the image carried at 16 channels."""

    def __init__(self, sd, prefix="g_a"):
        w = _P(sd, prefix, "0.weight")
        self.M = w.shape[0]
        self.conv = Conv3(_pad_dim(w, 1), _P(sd, prefix, "0.bias"))

    def forward(self, x4, save=False):
        return self.conv.forward(pad_nc4(x4), K.EPI_BIAS, tag="g_a.0.fwd"), None

    def backward(self, gy4, saved):
        return self.conv.dgrad(gy4, K.EPI_BIAS, tag="g_a.0.dgrad")[:, :1].contiguous()


class DebugSynthesis:
    """g_s = deconv(M, 3, kernel_size=3, stride=1) (anchors/model.py:17-19): ConvTranspose2d(padding 1) is the conv
    with weight[o][i] = W[i][o], taps reversed; its 3 outputs carried at 16 (zero weight rows and bias)."""

    def __init__(self, sd, prefix="g_s"):
        w = _P(sd, prefix, "0.weight")
        self.M = w.shape[0]
        wc = w.detach().transpose(0, 1).flip(-1, -2).contiguous()
        self.conv = Conv3(_pad_dim(wc, 0), _pad_dim(_P(sd, prefix, "0.bias"), 0))

    def forward(self, y4, save=False):
        return self.conv.forward(y4, K.EPI_BIAS, tag="g_s.0.fwd")[:, :1].contiguous(), None

    def backward(self, gx4, saved):
        return self.conv.dgrad(pad_nc4(gx4), K.EPI_BIAS, tag="g_s.0.dgrad")


class DebugHyperSynthesis:
    """mbt2018's h_s (MbtHyperSynthesis) on an N = 3 z_hat carried at 16 channels (h_s.0's weight zero-padded)."""

    def __init__(self, sd, prefix="h_s"):
        hs = {n: _P(sd, prefix, n) for n in ("0.weight", "0.bias", "2.weight", "2.bias", "4.weight", "4.bias")}
        hs["0.weight"] = _pad_dim(hs["0.weight"], 0)
        self.inner = MbtHyperSynthesis(hs, prefix="")
        self.out_channels = self.inner.out_channels

    def forward(self, z4):
        return self.inner.forward(pad_nc4(z4))


class DebugKernels:
    """CodecKernels-compatible executor for ae_onelayer (attack path + eval forward)."""

    model = "debug"
    clamp_input = False

    def __init__(self, sd: dict, precision: str = "fp32"):
        if sd["g_a.0.weight"].device.type != "cuda":
            raise RuntimeError("DebugKernels needs the state dict on the HIP device")
        if precision != "fp32":
            raise NotImplementedError(f"ae_onelayer runs fp32 operands, not {precision!r}")
        self.ga = DebugAnalysis(sd)
        self.gs = DebugSynthesis(sd)
        self.M = self.ga.M
        self.N = sd["h_a.0.weight"].shape[0]
        self.ha = MbtHyperAnalysis(sd)
        self.hs = DebugHyperSynthesis(sd)
        self.eb = K.PackedEB({n: sd[f"entropy_bottleneck.{n}"] for n in K.PackedEB.NAMES})

    def g_a(self, x4, save=False):
        return self.ga.forward(x4, save)

    def g_a_backward(self, gy4, saved):
        return self.ga.backward(gy4, saved)

    def g_s(self, y4, save=False):
        return self.gs.forward(y4, save)

    def g_s_backward(self, gx4, saved):
        return self.gs.backward(gx4, saved)

    def forward(self, x4, training=False, noise_y4=None, noise_z4=None):
        """ae_onelayer.forward (anchors/model.py:21-33), eval mode: likelihoods of the mean-scale hyperprior and
        x_hat = g_s(y)."""
        if training:
            raise NotImplementedError("ae_onelayer runs eval-mode forwards only (attack path)")
        y4, _ = self.ga.forward(x4)
        z4 = self.ha.forward(y4)
        zh, zlik, zsum = K.eb_likelihood(z4, self.N, self.eb, False, None)
        gp = self.hs.forward(zh)
        c4 = (self.M + 3) // 4
        scales4, means4 = gp[:, :c4].contiguous(), gp[:, c4:].contiguous()
        yh, ylik, ysum = K.gc_likelihood(y4, self.M, scales4, means4, False, None)
        xh, _ = self.gs.forward(y4)
        return {"x_hat4": xh, "y4": y4, "y_hat4": yh, "z4": z4, "z_hat4": zh, "scales4": scales4,
                "means4": means4, "lik4": {"y": ylik, "z": zlik}, "sumlog": ysum + zsum}
