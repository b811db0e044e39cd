"""CPU fp32 restatement of the CompressAI codec math the reference attacks.

TEST INFRASTRUCTURE (see oracle/__init__.py).  Every function works on a plain
``params`` dict whose keys are CompressAI state-dict names (``g_a.0.weight``,
``g_a.1.gamma``, ``entropy_bottleneck._matrix0`` ...), so the same synthetic
state dict drives this oracle and the HIP package.

Reference anchors:
  * layer geometry ``conv``/``deconv``           anchors/utils.py:112-130
  * GDN / IGDN (same reparametrisation as CompressAI)  utils/ops.py:58-97
  * LowerBound/UpperBound pass-through gradients utils/ops.py:28-56
  * model composition (ScaleHyperprior forward)  anchors/balle.py:37-41, anchors/model.py:91-95
  * EntropyBottleneck likelihood formula        utils/metrics_compare/decode.py:35-41 (text)
  * GaussianConditional likelihood               visual_distribution.py:85-101, attack_rd.py:46 (0.11 floor)
  * bpp                                          attack_rd.py:303,419
  * cheng2020-anchor (CompressAI Cheng2020Anchor, built at anchors/model.py:76-77; composition
    anchors/model.py:97-106): restated from the public CompressAI layer definitions (SURVEY §8 a17 and
    Appendix A.7).  CompressAI is not vendored in /root/reference and not installed, so the
    architecture itself is PARITY UNPINNED beyond its primitives (conv geometry, GDN, bounds).
  * mbt2018 (CompressAI JointAutoregressiveHierarchicalPriors, built at anchors/model.py:74-75; composition
    anchors/model.py:95-104, the same entropy_estimator branch as cheng2020): bmshj2018 g_a / g_s with
    LeakyReLU hyper transforms.  Same status as cheng2020: restated from the public CompressAI definition,
    PARITY UNPINNED beyond its primitives.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------- #
# Quality -> (N, M) tables (CompressAI zoo)
# --------------------------------------------------------------------------- #
def model_channels(model: str, quality: int) -> tuple[int, int]:
    if model in ("factorized", "hyper"):
        return (128, 192) if quality <= 5 else (192, 320)
    if model == "context":
        return (192, 192) if quality <= 4 else (192, 320)
    if model == "cheng2020":
        n = 128 if quality <= 3 else 192
        return (n, n)
    if model == "debug":   # anchors/model.py:61-68: ae_onelayer(N=3, M=192) at every quality
        return (3, 192)
    raise ValueError(model)


# --------------------------------------------------------------------------- #
# Bounds with one-sided pass-through gradient (utils/ops.py:28-56)
# --------------------------------------------------------------------------- #
class LowBound(torch.autograd.Function):
    """utils/ops.py:28-41: fwd clamp(min=b); bwd g * ((x >= b) | (g < 0))."""

    @staticmethod
    def forward(ctx, x, b):
        ctx.save_for_backward(x)
        ctx.b = b
        return torch.clamp(x, min=b)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        keep = (x >= ctx.b) | (g < 0.0)
        return g * keep.float(), None


class UpBound(torch.autograd.Function):
    """utils/ops.py:43-56: fwd clamp(max=b); bwd g * ((x <= b) | (g > 0))."""

    @staticmethod
    def forward(ctx, x, b):
        ctx.save_for_backward(x)
        ctx.b = b
        return torch.clamp(x, max=b)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        keep = (x <= ctx.b) | (g > 0.0)
        return g * keep.float(), None


def bound01(x, lo=0.0, hi=1.0):
    """``Up_bound(Low_bound(x, lo), hi)`` as used at attack_rd.py:354,507,517."""
    return UpBound.apply(LowBound.apply(x, lo), hi)


# --------------------------------------------------------------------------- #
# GDN (utils/ops.py:58-97 == compressai.layers.GDN)
# --------------------------------------------------------------------------- #
REPARAM_OFFSET = 2.0 ** -18
PEDESTAL = REPARAM_OFFSET ** 2


def gdn_effective(beta, gamma, beta_min=1e-6):
    """NonNegativeParametrizer: LowerBound(x, sqrt(min + ped))**2 - ped (utils/ops.py:83-89)."""
    beta_bound = (beta_min + PEDESTAL) ** 0.5
    gamma_bound = REPARAM_OFFSET
    b = LowBound.apply(beta, beta_bound) ** 2 - PEDESTAL
    g = LowBound.apply(gamma, gamma_bound) ** 2 - PEDESTAL
    return b, g


def gdn(x, beta, gamma, inverse=False):
    """utils/ops.py:83-97: norm = conv1x1(x^2, gamma', beta'); y = x*rsqrt(norm) | x*sqrt(norm)."""
    C = x.shape[1]
    b, g = gdn_effective(beta, gamma)
    norm = F.conv2d(x ** 2, g.reshape(C, C, 1, 1), b)
    norm = torch.sqrt(norm) if inverse else torch.rsqrt(norm)
    return x * norm


def gdn_init(C, gamma_init=0.1):
    """Initial stored params: sqrt(max(x + ped, ped)) (utils/ops.py:71-81)."""
    beta = torch.sqrt(torch.ones(C) + PEDESTAL)
    gamma = torch.sqrt(gamma_init * torch.eye(C) + PEDESTAL)
    return beta, gamma


# --------------------------------------------------------------------------- #
# Conv geometry (anchors/utils.py:112-130)
# --------------------------------------------------------------------------- #
def conv(x, w, b, stride=2):
    k = w.shape[-1]
    return F.conv2d(x, w, b, stride=stride, padding=k // 2)


def deconv(x, w, b, stride=2):
    k = w.shape[-1]
    return F.conv_transpose2d(x, w, b, stride=stride, padding=k // 2, output_padding=stride - 1)


# --------------------------------------------------------------------------- #
# Transforms (CompressAI bmshj2018 g_a/g_s/h_a/h_s)
# --------------------------------------------------------------------------- #
def g_a(P, x, prefix="g_a"):
    for i in (0, 2, 4):
        x = conv(x, P[f"{prefix}.{i}.weight"], P[f"{prefix}.{i}.bias"])
        x = gdn(x, P[f"{prefix}.{i+1}.beta"], P[f"{prefix}.{i+1}.gamma"], inverse=False)
    return conv(x, P[f"{prefix}.6.weight"], P[f"{prefix}.6.bias"])


def g_s(P, y, prefix="g_s"):
    for i in (0, 2, 4):
        y = deconv(y, P[f"{prefix}.{i}.weight"], P[f"{prefix}.{i}.bias"])
        y = gdn(y, P[f"{prefix}.{i+1}.beta"], P[f"{prefix}.{i+1}.gamma"], inverse=True)
    return deconv(y, P[f"{prefix}.6.weight"], P[f"{prefix}.6.bias"])


def h_a(P, y):
    """h_a = conv3x3 s1 - ReLU - conv - ReLU - conv (A.2)."""
    z = F.relu(conv(y, P["h_a.0.weight"], P["h_a.0.bias"], stride=1))
    z = F.relu(conv(z, P["h_a.2.weight"], P["h_a.2.bias"]))
    return conv(z, P["h_a.4.weight"], P["h_a.4.bias"])


def h_s(P, z):
    """h_s = deconv - ReLU - deconv - ReLU - conv3x3 s1 - ReLU (A.2)."""
    s = F.relu(deconv(z, P["h_s.0.weight"], P["h_s.0.bias"]))
    s = F.relu(deconv(s, P["h_s.2.weight"], P["h_s.2.bias"]))
    return F.relu(conv(s, P["h_s.4.weight"], P["h_s.4.bias"], stride=1))


# --------------------------------------------------------------------------- #
# Entropy models
# --------------------------------------------------------------------------- #
EB_FILTERS = (3, 3, 3, 3)
LIKELIHOOD_BOUND = 1e-9
SCALE_BOUND = 0.11


def eb_logits_cumulative(P, v, prefix="entropy_bottleneck"):
    """v: [C, 1, L]; f_i(u) = softplus(H_i) u + b_i (+ tanh(a_i) tanh(.)) (A.3)."""
    logits = v
    for i in range(len(EB_FILTERS) + 1):
        logits = torch.matmul(F.softplus(P[f"{prefix}._matrix{i}"]), logits)
        logits = logits + P[f"{prefix}._bias{i}"]
        if i < len(EB_FILTERS):
            logits = logits + torch.tanh(P[f"{prefix}._factor{i}"]) * torch.tanh(logits)
    return logits


def eb_likelihood(P, v, prefix="entropy_bottleneck"):
    lower = eb_logits_cumulative(P, v - 0.5, prefix)
    upper = eb_logits_cumulative(P, v + 0.5, prefix)
    sign = -torch.sign(lower + upper)
    lik = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))
    # CompressAI likelihood_lower_bound = LowerBound(1e-9): clamp forward, one-sided pass-through backward
    # (identical rule to utils/ops.py:28-41)
    return LowBound.apply(lik, LIKELIHOOD_BOUND)


def entropy_bottleneck(P, z, training=False, noise=None, prefix="entropy_bottleneck"):
    """Returns (z_hat, z_likelihoods).  Eval: round(z - median) + median."""
    C = z.shape[1]
    v = z.transpose(0, 1).contiguous().reshape(C, 1, -1)
    med = P[f"{prefix}.quantiles"][:, :, 1:2]
    if training:
        if noise is None:
            noise = torch.empty_like(v).uniform_(-0.5, 0.5)
        else:
            noise = noise.transpose(0, 1).contiguous().reshape(C, 1, -1)
        out = v + noise
    else:
        out = torch.round(v - med) + med
    lik = eb_likelihood(P, out, prefix)
    shape = (C, z.shape[0]) + tuple(z.shape[2:])
    out = out.reshape(shape).transpose(0, 1).contiguous()
    lik = lik.reshape(shape).transpose(0, 1).contiguous()
    return out, lik


def eb_aux_loss(P, prefix="entropy_bottleneck"):
    """EntropyBottleneck.loss(): sum |F(quantiles) - target| (A.3)."""
    tail_mass = 1e-9
    t = math.log(2 / tail_mass - 1)
    target = torch.tensor([-t, 0.0, t])
    q = P[f"{prefix}.quantiles"]
    logits = eb_logits_cumulative({k: v.detach() for k, v in P.items()}, q, prefix)
    return torch.abs(logits - target).sum()


def _std_cumulative(x):
    return 0.5 * torch.erfc(-(2 ** -0.5) * x)


def gc_likelihood(y_hat, scales, means=None):
    values = y_hat - means if means is not None else y_hat
    # lower_bound_scale = LowerBound(0.11) and LowerBound(1e-9) on the likelihood:
    # same forward as a clamp, but the gradient passes where it would push the value up (g < 0)
    scales = LowBound.apply(scales, SCALE_BOUND)
    values = torch.abs(values)
    upper = _std_cumulative((0.5 - values) / scales)
    lower = _std_cumulative((-0.5 - values) / scales)
    return LowBound.apply(upper - lower, LIKELIHOOD_BOUND)


def gaussian_conditional(y, scales, means=None, training=False, noise=None):
    if training:
        if noise is None:
            noise = torch.empty_like(y).uniform_(-0.5, 0.5)
        y_hat = y + noise
    else:
        y_hat = torch.round(y - means) + means if means is not None else torch.round(y)
    return y_hat, gc_likelihood(y_hat, scales, means)


# --------------------------------------------------------------------------- #
# Full model forward (ScaleHyperprior / FactorizedPrior)
# --------------------------------------------------------------------------- #
def forward(P, x, model="hyper", training=False, noise_y=None, noise_z=None):
    """net(x) -> {"x_hat", "likelihoods": {"y", "z"}} (anchors/balle.py:25-55)."""
    if model == "cheng2020":
        return cheng_forward(P, x, training, noise_y, noise_z)
    if model == "debug":
        return debug_forward(P, x, training, noise_y, noise_z)
    if model == "context":
        return mbt_forward(P, x, training, noise_y, noise_z)
    y = g_a(P, x)
    if model == "factorized":
        y_hat, y_lik = entropy_bottleneck(P, y, training, noise_y)
        return {"x_hat": g_s(P, y_hat), "likelihoods": {"y": y_lik}}
    if model != "hyper":
        raise NotImplementedError(model)
    z = h_a(P, torch.abs(y))
    z_hat, z_lik = entropy_bottleneck(P, z, training, noise_z)
    scales = h_s(P, z_hat)
    y_hat, y_lik = gaussian_conditional(y, scales, None, training, noise_y)
    return {"x_hat": g_s(P, y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


# --------------------------------------------------------------------------- #
# cheng2020-anchor (CompressAI Cheng2020Anchor / JointAutoregressiveHierarchicalPriors)
# --------------------------------------------------------------------------- #
LRELU_SLOPE = 0.01  # nn.LeakyReLU() default


def lrelu(x):
    return F.leaky_relu(x, LRELU_SLOPE)


def conv_k(x, w, b, stride=1):
    """CompressAI conv3x3 / conv1x1: Conv2d(k, stride, padding=k//2)."""
    return F.conv2d(x, w, b, stride=stride, padding=w.shape[-1] // 2)


def subpel(x, w, b, r=2):
    """subpel_conv3x3: Conv2d(in, out*r^2, 3, padding=1) -> PixelShuffle(r)."""
    return F.pixel_shuffle(conv_k(x, w, b), r)


def rb_stride(P, pre, x):
    """ResidualBlockWithStride(stride=2): GDN(conv3x3(lrelu(conv3x3_s2(x)))) + conv1x1_s2(x)."""
    out = lrelu(conv_k(x, P[f"{pre}.conv1.weight"], P[f"{pre}.conv1.bias"], 2))
    out = conv_k(out, P[f"{pre}.conv2.weight"], P[f"{pre}.conv2.bias"])
    out = gdn(out, P[f"{pre}.gdn.beta"], P[f"{pre}.gdn.gamma"])
    return out + conv_k(x, P[f"{pre}.skip.weight"], P[f"{pre}.skip.bias"], 2)


def rb(P, pre, x):
    """ResidualBlock(N, N): lrelu(conv3x3(lrelu(conv3x3(x)))) + x."""
    out = lrelu(conv_k(x, P[f"{pre}.conv1.weight"], P[f"{pre}.conv1.bias"]))
    out = lrelu(conv_k(out, P[f"{pre}.conv2.weight"], P[f"{pre}.conv2.bias"]))
    return out + x


def rb_up(P, pre, x):
    """ResidualBlockUpsample(2): IGDN(conv3x3(lrelu(subpel(x)))) + subpel_upsample(x)."""
    out = lrelu(subpel(x, P[f"{pre}.subpel_conv.0.weight"], P[f"{pre}.subpel_conv.0.bias"]))
    out = conv_k(out, P[f"{pre}.conv.weight"], P[f"{pre}.conv.bias"])
    out = gdn(out, P[f"{pre}.igdn.beta"], P[f"{pre}.igdn.gamma"], inverse=True)
    return out + subpel(x, P[f"{pre}.upsample.0.weight"], P[f"{pre}.upsample.0.bias"])


def cheng_g_a(P, x):
    x = rb_stride(P, "g_a.0", x)
    x = rb(P, "g_a.1", x)
    x = rb_stride(P, "g_a.2", x)
    x = rb(P, "g_a.3", x)
    x = rb_stride(P, "g_a.4", x)
    x = rb(P, "g_a.5", x)
    return conv_k(x, P["g_a.6.weight"], P["g_a.6.bias"], 2)


def cheng_g_s(P, y):
    y = rb(P, "g_s.0", y)
    y = rb_up(P, "g_s.1", y)
    y = rb(P, "g_s.2", y)
    y = rb_up(P, "g_s.3", y)
    y = rb(P, "g_s.4", y)
    y = rb_up(P, "g_s.5", y)
    y = rb(P, "g_s.6", y)
    return subpel(y, P["g_s.7.0.weight"], P["g_s.7.0.bias"])


def cheng_h_a(P, y):
    z = lrelu(conv_k(y, P["h_a.0.weight"], P["h_a.0.bias"]))
    z = lrelu(conv_k(z, P["h_a.2.weight"], P["h_a.2.bias"]))
    z = lrelu(conv_k(z, P["h_a.4.weight"], P["h_a.4.bias"], 2))
    z = lrelu(conv_k(z, P["h_a.6.weight"], P["h_a.6.bias"]))
    return conv_k(z, P["h_a.8.weight"], P["h_a.8.bias"], 2)


def cheng_h_s(P, z):
    s = lrelu(conv_k(z, P["h_s.0.weight"], P["h_s.0.bias"]))
    s = lrelu(subpel(s, P["h_s.2.0.weight"], P["h_s.2.0.bias"]))
    s = lrelu(conv_k(s, P["h_s.4.weight"], P["h_s.4.bias"]))
    s = lrelu(subpel(s, P["h_s.6.0.weight"], P["h_s.6.0.bias"]))
    return conv_k(s, P["h_s.8.weight"], P["h_s.8.bias"])


def context_mask(k=5):
    """MaskedConv2d type 'A': zero the centre tap and everything after it in raster order."""
    m = torch.ones(k, k)
    m[k // 2, k // 2:] = 0
    m[k // 2 + 1:] = 0
    return m


def context_prediction(P, y_hat):
    """CompressAI's MaskedConv2d.forward: ``self.weight.data *= self.mask`` (in place, outside autograd), then the
    plain conv on the parameter, so the weight's gradient is the UNMASKED conv weight gradient (all 25 taps) and the
    masked taps' gradients enter clip_grad_norm_ (reference train.py:360)."""
    w = P["context_prediction.weight"]
    with torch.no_grad():
        w.mul_(context_mask(w.shape[-1]).to(w.dtype))
    return F.conv2d(y_hat, w, P["context_prediction.bias"], padding=w.shape[-1] // 2)


def joint_noise(noise_y):
    """Train-mode noise of the joint-prior models: (for y_hat = quantize(y, "noise"), for the GaussianConditional's
    own requantisation).  CompressAI draws the two independently (JointAutoregressiveHierarchicalPriors.forward);
    None draws both, a pair pins both, and one tensor pins a shared draw (the pinned mode of the round-5 tests)."""
    if isinstance(noise_y, (tuple, list)):
        return noise_y[0], noise_y[1]
    return noise_y, noise_y


def entropy_parameters(P, t):
    t = lrelu(conv_k(t, P["entropy_parameters.0.weight"], P["entropy_parameters.0.bias"]))
    t = lrelu(conv_k(t, P["entropy_parameters.2.weight"], P["entropy_parameters.2.bias"]))
    return conv_k(t, P["entropy_parameters.4.weight"], P["entropy_parameters.4.bias"])


def cheng_forward(P, x, training=False, noise_y=None, noise_z=None):
    """entropy_estimator for cheng2020 (anchors/model.py:97-106) + g_s(y_hat) (compressor :80-84)."""
    y = cheng_g_a(P, x)
    z = cheng_h_a(P, y)
    z_hat, z_lik = entropy_bottleneck(P, z, training, noise_z)
    params = cheng_h_s(P, z_hat)
    ny_hat, ny_lik = joint_noise(noise_y)
    if training:
        y_hat = y + (ny_hat if ny_hat is not None else torch.empty_like(y).uniform_(-0.5, 0.5))
    else:
        y_hat = torch.round(y)   # quantize(y, "dequantize") with means=None
    ctx = context_prediction(P, y_hat)
    gp = entropy_parameters(P, torch.cat((params, ctx), dim=1))
    scales, means = gp.chunk(2, 1)
    _, y_lik = gaussian_conditional(y, scales, means, training, ny_lik)
    return {"x_hat": cheng_g_s(P, y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


# --------------------------------------------------------------------------- #
# mbt2018 (CompressAI JointAutoregressiveHierarchicalPriors)
# --------------------------------------------------------------------------- #
def mbt_h_a(P, y):
    """h_a = conv3x3 s1 - LReLU - conv5x5 s2 - LReLU - conv5x5 s2 (on y, not |y|)."""
    z = lrelu(conv(y, P["h_a.0.weight"], P["h_a.0.bias"], stride=1))
    z = lrelu(conv(z, P["h_a.2.weight"], P["h_a.2.bias"]))
    return conv(z, P["h_a.4.weight"], P["h_a.4.bias"])


def mbt_h_s(P, z):
    """h_s = deconv(N,M) - LReLU - deconv(M,3M/2) - LReLU - conv3x3 s1 (3M/2 -> 2M)."""
    s = lrelu(deconv(z, P["h_s.0.weight"], P["h_s.0.bias"]))
    s = lrelu(deconv(s, P["h_s.2.weight"], P["h_s.2.bias"]))
    return conv(s, P["h_s.4.weight"], P["h_s.4.bias"], stride=1)


def mbt_forward(P, x, training=False, noise_y=None, noise_z=None):
    """entropy_estimator for MODEL == "context" (anchors/model.py:95-104) + g_s(y_hat) (compressor :80-84)."""
    y = g_a(P, x)
    z = mbt_h_a(P, y)
    z_hat, z_lik = entropy_bottleneck(P, z, training, noise_z)
    params = mbt_h_s(P, z_hat)
    ny_hat, ny_lik = joint_noise(noise_y)
    if training:
        y_hat = y + (ny_hat if ny_hat is not None else torch.empty_like(y).uniform_(-0.5, 0.5))
    else:
        y_hat = torch.round(y)
    ctx = context_prediction(P, y_hat)
    gp = entropy_parameters(P, torch.cat((params, ctx), dim=1))
    scales, means = gp.chunk(2, 1)
    _, y_lik = gaussian_conditional(y, scales, means, training, ny_lik)
    return {"x_hat": g_s(P, y_hat), "likelihoods": {"y": y_lik, "z": z_lik}}


# --------------------------------------------------------------------------- #
# ae_onelayer, the "debug" model (anchors/model.py:8-33): one 3x3 stride-1 conv each way around the
# MeanScaleHyperprior entropy model (CompressAI: mbt2018's h_a / h_s, no context model)
# --------------------------------------------------------------------------- #
def debug_g_a(P, x):
    """g_a = conv(3, M, kernel_size=3, stride=1) (anchors/model.py:13-15; anchors/utils.py:112-119)."""
    return conv(x, P["g_a.0.weight"], P["g_a.0.bias"], stride=1)


def debug_g_s(P, y):
    """g_s = deconv(M, 3, kernel_size=3, stride=1): ConvTranspose2d, padding 1, output_padding 0
    (anchors/model.py:17-19; anchors/utils.py:122-130)."""
    return deconv(y, P["g_s.0.weight"], P["g_s.0.bias"], stride=1)


def debug_forward(P, x, training=False, noise_y=None, noise_z=None):
    """ae_onelayer.forward (anchors/model.py:21-33): the likelihoods of the mean-scale hyperprior, and
    x_hat = g_s(y) -- of the UNQUANTISED latent (the reference's line 30; its y_hat is computed and unused)."""
    y = debug_g_a(P, x)
    z = mbt_h_a(P, y)
    z_hat, z_lik = entropy_bottleneck(P, z, training, noise_z)
    scales, means = mbt_h_s(P, z_hat).chunk(2, 1)
    _, y_lik = gaussian_conditional(y, scales, means, training, noise_y)
    return {"x_hat": debug_g_s(P, y), "likelihoods": {"y": y_lik, "z": z_lik}}


def transforms(P, x, model="hyper"):
    """g_s(g_a(x)) without quantisation (the attack's expensive branch, attack_rd.py:344-349)."""
    if model == "cheng2020":
        return cheng_g_s(P, cheng_g_a(P, x))
    if model == "debug":
        return debug_g_s(P, debug_g_a(P, x))
    return g_s(P, g_a(P, x))


def bpp(likelihoods: dict, num_pixels: int):
    """attack_rd.py:419 / self_ensemble.py:222: sum_k sum log p / (-ln2 * H*W)."""
    return sum(torch.log(l).sum() / (-math.log(2) * num_pixels) for l in likelihoods.values())


# --------------------------------------------------------------------------- #
# Synthetic weights in CompressAI naming (SURVEY 8d "Synthetic inputs")
# --------------------------------------------------------------------------- #
def _conv_init(gen, cout, cin, k, transposed=False):
    # PyTorch default: kaiming_uniform(a=sqrt(5)) -> U(-1/sqrt(fan_in), 1/sqrt(fan_in)).
    # nn.ConvTranspose2d computes fan_in from weight.size(1) * k * k = cout * k * k.
    shape = (cin, cout, k, k) if transposed else (cout, cin, k, k)
    fan_in = shape[1] * k * k
    bound = 1.0 / math.sqrt(fan_in)
    w = (torch.rand(shape, generator=gen) * 2 - 1) * bound
    b = (torch.rand(cout, generator=gen) * 2 - 1) * bound
    return w, b


def init_params(model="hyper", quality=3, seed=0, N=None, M=None):
    """Seeded synthetic state dict with CompressAI key names (random init, not pretrained)."""
    if N is None or M is None:
        N, M = model_channels(model, quality)
    gen = torch.Generator().manual_seed(seed)
    P = {}

    def cv(name, cout, cin, k, transposed=False):
        P[f"{name}.weight"], P[f"{name}.bias"] = _conv_init(gen, cout, cin, k, transposed)

    def gd(name, C):
        P[f"{name}.beta"], P[f"{name}.gamma"] = gdn_init(C)

    if model == "cheng2020":
        return _init_cheng(P, cv, gd, gen, N)
    if model == "debug":
        cv("g_a.0", M, 3, 3)
        cv("g_s.0", 3, M, 3, True)
        _init_mbt_hyper(cv, N, M)
        _init_eb(P, gen, N)
        return P
    cv("g_a.0", N, 3, 5); gd("g_a.1", N)
    cv("g_a.2", N, N, 5); gd("g_a.3", N)
    cv("g_a.4", N, N, 5); gd("g_a.5", N)
    cv("g_a.6", M, N, 5)
    cv("g_s.0", N, M, 5, True); gd("g_s.1", N)
    cv("g_s.2", N, N, 5, True); gd("g_s.3", N)
    cv("g_s.4", N, N, 5, True); gd("g_s.5", N)
    cv("g_s.6", 3, N, 5, True)
    eb_ch = M if model == "factorized" else N
    if model == "context":
        _init_mbt_hyper(cv, N, M)
        cv("context_prediction", 2 * M, M, 5)
        cv("entropy_parameters.0", M * 10 // 3, M * 12 // 3, 1)
        cv("entropy_parameters.2", M * 8 // 3, M * 10 // 3, 1)
        cv("entropy_parameters.4", M * 6 // 3, M * 8 // 3, 1)
    if model == "hyper":
        cv("h_a.0", N, M, 3)
        cv("h_a.2", N, N, 5)
        cv("h_a.4", N, N, 5)
        cv("h_s.0", N, N, 5, True)
        cv("h_s.2", N, N, 5, True)
        cv("h_s.4", M, N, 3)
    _init_eb(P, gen, eb_ch)
    return P


def _init_mbt_hyper(cv, N, M):
    """CompressAI MeanScaleHyperprior / mbt2018 h_a, h_s shapes."""
    cv("h_a.0", N, M, 3)
    cv("h_a.2", N, N, 5)
    cv("h_a.4", N, N, 5)
    cv("h_s.0", M, N, 5, True)
    cv("h_s.2", M * 3 // 2, M, 5, True)
    cv("h_s.4", M * 2, M * 3 // 2, 3)


def _init_cheng(P, cv, gd, gen, N):
    """Cheng2020Anchor(N) state-dict names / shapes (CompressAI), random init."""
    for i in (0, 2, 4):   # ResidualBlockWithStride
        cv(f"g_a.{i}.conv1", N, 3 if i == 0 else N, 3)
        cv(f"g_a.{i}.conv2", N, N, 3)
        gd(f"g_a.{i}.gdn", N)
        cv(f"g_a.{i}.skip", N, 3 if i == 0 else N, 1)
    for pre in ("g_a.1", "g_a.3", "g_a.5", "g_s.0", "g_s.2", "g_s.4", "g_s.6"):   # ResidualBlock
        cv(f"{pre}.conv1", N, N, 3)
        cv(f"{pre}.conv2", N, N, 3)
    cv("g_a.6", N, N, 3)
    for i in (1, 3, 5):   # ResidualBlockUpsample
        cv(f"g_s.{i}.subpel_conv.0", 4 * N, N, 3)
        cv(f"g_s.{i}.conv", N, N, 3)
        gd(f"g_s.{i}.igdn", N)
        cv(f"g_s.{i}.upsample.0", 4 * N, N, 3)
    cv("g_s.7.0", 12, N, 3)
    for i in (0, 2, 4, 6, 8):
        cv(f"h_a.{i}", N, N, 3)
    cv("h_s.0", N, N, 3)
    cv("h_s.2.0", 4 * N, N, 3)
    cv("h_s.4", N * 3 // 2, N, 3)
    cv("h_s.6.0", 4 * (N * 3 // 2), N * 3 // 2, 3)
    cv("h_s.8", 2 * N, N * 3 // 2, 3)
    cv("context_prediction", 2 * N, N, 5)
    cv("entropy_parameters.0", N * 10 // 3, N * 12 // 3, 1)
    cv("entropy_parameters.2", N * 8 // 3, N * 10 // 3, 1)
    cv("entropy_parameters.4", N * 6 // 3, N * 8 // 3, 1)
    _init_eb(P, gen, N)
    return P


def _init_eb(P, gen, eb_ch):
    # EntropyBottleneck(C, filters=(3,3,3,3), init_scale=10) (A.3)
    filters = (1,) + EB_FILTERS + (1,)
    scale = 10.0 ** (1 / (len(EB_FILTERS) + 1))
    for i in range(len(EB_FILTERS) + 1):
        init = math.log(math.expm1(1 / scale / filters[i + 1]))
        P[f"entropy_bottleneck._matrix{i}"] = torch.full((eb_ch, filters[i + 1], filters[i]), init)
        P[f"entropy_bottleneck._bias{i}"] = torch.rand((eb_ch, filters[i + 1], 1), generator=gen) - 0.5
        if i < len(EB_FILTERS):
            P[f"entropy_bottleneck._factor{i}"] = torch.zeros((eb_ch, filters[i + 1], 1))
    P["entropy_bottleneck.quantiles"] = torch.tensor([-10.0, 0.0, 10.0]).repeat(eb_ch, 1, 1)


def perturb_params(P, seed=1, gdn_scale=0.3, eb_scale=0.5):
    """Move GDN/EB parameters off their init so parity tests exercise non-trivial
    gamma (off-diagonal), beta and EB factor/matrix values.  Off-diagonal gamma
    entries are pushed both above and below the reparam lower bound."""
    gen = torch.Generator().manual_seed(seed)
    Q = dict(P)
    for k, v in P.items():
        if k.endswith(".gamma"):
            C = v.shape[0]
            d = (torch.rand((C, C), generator=gen) * 2 - 1) * (gdn_scale / math.sqrt(C))
            Q[k] = v + d.abs() * (torch.rand((C, C), generator=gen) > 0.3).float()
        elif k.endswith(".beta"):
            Q[k] = v + torch.rand(v.shape, generator=gen) * gdn_scale
        elif k.startswith("entropy_bottleneck._factor") or k.startswith("entropy_bottleneck._matrix"):
            Q[k] = v + (torch.rand(v.shape, generator=gen) * 2 - 1) * eb_scale
        elif k == "entropy_bottleneck.quantiles":
            Q[k] = v + (torch.rand(v.shape, generator=gen) * 2 - 1) * eb_scale
    return Q
