"""Train-mode forward + RateDistortionLoss + backward of the reference's "debug" model, ae_onelayer(N=3, M=192)
(anchors/model.py:8-33; ``-m debug``), on the HIP kernels: the adversarial fine-tune's inner piece (train.py --adv,
``/root/reference/train.py:249-366`` fine-tunes whatever ``coder.load_model`` builds, ``coder.py:88-101``).  The
oracle's restatement is ``oracle/codec.debug_forward`` (training=True).

  loss -> x_hat = g_s(y) (the UNQUANTISED latent, anchors/model.py:30) -> y
       <- GC bwd (scales, means; y_tilde = y + u, the GaussianConditional's own draw)
       -> h_s^T (conv k3 (3M/2 -> 2M); deconv k5 s2 (M -> 3M/2) + LReLU; deconv k5 s2 (N -> M) + LReLU)
       -> z_tilde <- EB bwd -> h_a^T (conv k5 s2, LReLU, conv k5 s2, LReLU, conv k3 (M -> N)) -> y
       -> g_a (conv k3, 3 -> M): weight and bias gradients only

The 3-channel sides run as the eval executor runs them (engine_debug): the image and the g_s output gradient are
carried at 16 channels, zero past the third, and the N = 3 hyper layers' input gradients run on weights zero-padded
to 16 channels on their 3-wide sides (the 16-channel-chunk conv kernels; the zero channels contribute exact zeros and
are sliced off).  Weight gradients are ica_wgrad GEMMs over pixels on the unpadded tensors (any channel count); the
transposed convs take theirs with the roles of input and output gradient swapped (include/ica_hip.h).  fp32
operands throughout (ae_onelayer has no bf16 / x6 packs: engine_debug)."""
from __future__ import annotations

import math

import torch

from . import hip_ops as K
from .engine_debug import CP, _pad_dim, pad_nc4
from .engine_cheng import Conv3
from .train_cheng import ChengTrainStep


def _quad0(t4):
    """The first channel quad (channels 0-3) of a 16-channel nChw4c tensor: the N = 3 side, fourth lane zero."""
    return t4[:, :1].contiguous()


def train_forward(ck, P, x4, noise_y=None, noise_z=None):
    """debug_forward (training=True) with the activations the backward reads.  ck: the model's DebugKernels (fp32);
    P(name): the detached parameter; noise_y: the GaussianConditional's U(-1/2, 1/2) draw on y (NCHW, M channels),
    noise_z: the EntropyBottleneck's on z (N channels); drawn when None."""
    B, H, W = x4.shape[0], x4.shape[2], x4.shape[3]
    N, M = ck.N, ck.M
    xp4 = pad_nc4(x4)
    ga = Conv3(_pad_dim(P("g_a.0.weight"), 1), P("g_a.0.bias"), fwd_only=True)
    y4 = ga.forward(xp4, K.EPI_BIAS, tag="g_a.0.fwd")
    pc = lambda pre, s: K.PackedConv(P(f"{pre}.weight"), P(f"{pre}.bias"), "conv", s)  # noqa: E731
    ha = [pc("h_a.0", 1), pc("h_a.2", 2), pc("h_a.4", 2)]
    z0, _, _ = K.conv_down(y4, M, ha[0].fwd, ha[0].bias, N, 3, 1, K.EPI_LRELU)
    z1, _, _ = K.conv_down(z0, N, ha[1].fwd, ha[1].bias, N, 5, 2, K.EPI_LRELU)
    z4, _, _ = K.conv_down(z1, N, ha[2].fwd, ha[2].bias, N, 5, 2, K.EPI_BIAS)
    if noise_z is None:
        noise_z = torch.empty((B, N, z4.shape[2], z4.shape[3]), device=x4.device).uniform_(-0.5, 0.5)
    zt4, zlik4, _ = K.eb_likelihood(z4, N, ck.eb, True, K.to_nc4(noise_z.contiguous()))
    hs = ck.hs.inner                     # MbtHyperSynthesis on the 16-channel z (h_s.0 weight zero-padded)
    M3 = hs.M3
    s0, _, _ = K.conv_up(pad_nc4(zt4), CP, hs.convs[0].fwd, hs.convs[0].bias, M, K.EPI_LRELU, it=hs.convs[0].it_fwd)
    s1, _, _ = K.conv_up(s0, M, hs.convs[1].fwd, hs.convs[1].bias, M3, K.EPI_LRELU, it=hs.convs[1].it_fwd)
    params4, _, _ = K.conv_down(s1, M3, hs.convs[2].fwd, hs.convs[2].bias, 2 * M, 3, 1, K.EPI_BIAS)
    c4 = (M + 3) // 4
    scales4, means4 = params4[:, :c4].contiguous(), params4[:, c4:].contiguous()
    if noise_y is None:
        noise_y = torch.empty((B, M, H, W), device=x4.device).uniform_(-0.5, 0.5)
    yt4, ylik4, _ = K.gc_likelihood(y4, M, scales4, means4, True, K.to_nc4(noise_y.contiguous()))
    wc = P("g_s.0.weight").transpose(0, 1).flip(-1, -2).contiguous()   # ConvTranspose2d(pad 1) as a conv
    gs = Conv3(_pad_dim(wc, 0), _pad_dim(P("g_s.0.bias"), 0))
    xh4 = _quad0(gs.forward(y4, K.EPI_BIAS, tag="g_s.0.fwd"))          # x_hat = g_s(y)
    out = {k: v for k, v in locals().items() if k not in ("ck", "P", "B", "pc", "hs", "wc", "noise_y", "noise_z")}
    return out


class DebugTrainStep(ChengTrainStep):
    """One train-mode forward / loss / backward of a ``codec.AeOneLayer`` with gradients written into the
    RDTrainer's flat buffer views (CompressAI parameter names)."""

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

        # g_s = deconv(M, 3, k3, s1): its weight gradient is the conv view's, transposed back and taps reversed
        tmp = torch.empty((3, M, 3, 3), device=x.device)
        K.wgrad(g4, 3, f["y4"], M, 3, 1, tmp, tag="g_s.0.wgrad")
        self._g("g_s.0.weight").copy_(tmp.transpose(0, 1).flip(-1, -2))
        K.channel_sum(g4, 3, self._g("g_s.0.bias"))
        gy = f["gs"].dgrad(pad_nc4(g4), K.EPI_BIAS, tag="g_s.0.dgrad")
        del g4

        # GaussianConditional (y_tilde = y + u; likelihood of y_tilde - means at scales): dL/dy, dL/d(h_s output)
        gl_y = K.bpp_grad(f["ylik4"], gscale)
        gv, gsig = K.gc_bwd(f["yt4"] - f["means4"], f["scales4"], gl_y, M)
        gy.add_(gv)
        gparams = torch.cat((gsig, -gv), dim=1)             # (scales, means) = h_s(z_hat).chunk(2, 1)

        # h_s backward (the 16-channel z_hat of the forward; h_s.0's weight gradient on the 3 real channels)
        hs, M3, s0, s1, zt4 = ck.hs.inner, f["M3"], f["s0"], f["s1"], f["zt4"]
        self._wb(gparams, 2 * M, s1, M3, 3, 1, "h_s.4")
        g, _, _ = K.conv_down(gparams, 2 * M, hs.convs[2].bwd, None, M3, 3, 1, K.EPI_BIAS)
        g = K.lrelu_bwd(g, s1)
        K.wgrad(s0, M, g, M3, 5, 2, self._g("h_s.2.weight"), tag="h_s.2.wgrad")
        K.channel_sum(g, M3, self._g("h_s.2.bias"))
        g, _, _ = K.conv_down(g, M3, hs.convs[1].bwd, None, M, 5, 2, K.EPI_BIAS)
        g = K.lrelu_bwd(g, s0)
        K.wgrad(zt4, N, g, M, 5, 2, self._g("h_s.0.weight"), tag="h_s.0.wgrad")
        K.channel_sum(g, M, self._g("h_s.0.bias"))
        gz, _, _ = K.conv_down(g, M, hs.convs[0].bwd, None, CP, 5, 2, K.EPI_BIAS)
        gz = _quad0(gz)
        gz.add_(tr._eb_backward(ck, zt4, f["zlik4"], N, gscale))   # z_tilde = z + u

        # h_a backward: the N = 3 convs' input gradients on weights zero-padded to 16 on the 3-wide sides
        z0, z1 = f["z0"], f["z1"]
        pad2 = lambda pre: K.PackedConv(_pad_dim(_pad_dim(self._p(f"{pre}.weight"), 0), 1), None, "conv", 2)  # noqa: E731
        self._wb(gz, N, z1, N, 5, 2, "h_a.4")
        g, _, _ = K.conv_up(pad_nc4(gz), CP, pad2("h_a.4").bwd, None, CP, K.EPI_BIAS)
        g = K.lrelu_bwd(_quad0(g), z1)
        self._wb(g, N, z0, N, 5, 2, "h_a.2")
        g, _, _ = K.conv_up(pad_nc4(g), CP, pad2("h_a.2").bwd, None, CP, K.EPI_BIAS)
        g = K.lrelu_bwd(_quad0(g), z0)
        self._wb(g, N, f["y4"], M, 3, 1, "h_a.0")
        ha0 = K.PackedConv(_pad_dim(self._p("h_a.0.weight"), 0), None, "conv", 1)
        g, _, _ = K.conv_down(pad_nc4(g), CP, ha0.bwd, None, M, 3, 1, K.EPI_BIAS)
        gy.add_(g)

        # g_a = conv(3, M, k3, s1): weight and bias gradients (the image needs no gradient)
        self._wb(gy, M, x4, 3, 3, 1, "g_a.0")
        return {"loss": loss, "bpp_loss": bpp, "distortion_loss": dist}
