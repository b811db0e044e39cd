"""CompressAI-compatible codec modules running on the HIP kernels.

Replaces the un-vendored third-party surface the reference drives
(anchors/model.py:3-5, anchors/balle.py:7-8): ``bmshj2018_factorized`` /
``bmshj2018_hyperprior`` models with ``g_a``, ``g_s``, ``h_a``, ``h_s``,
``entropy_bottleneck``, ``gaussian_conditional``, ``forward(x) ->
{"x_hat", "likelihoods"}``, ``aux_loss()`` and CompressAI state-dict keys
(``g_a.0.weight``, ``g_a.1.beta``, ``g_a.1.gamma``, ``g_a.1.beta_reparam.pedestal``,
``entropy_bottleneck._matrix0``, ``entropy_bottleneck.quantiles``, ...).

``g_a`` / ``g_s`` are nn.Sequential containers (so parameters and indexing
look like CompressAI's) whose forward runs the fused HIP chain as one
autograd Function: forward saves the GDN activations, backward runs the fused
dgrad chain and, when the bmshj2018 g_a / g_s parameters require grad, their
weight / bias / GDN gradients on the HIP wgrad kernels.  The other transforms
(h_a / h_s, cheng2020) raise when asked for parameter gradients; the full-model
train step is train_engine.RDTrainer.
"""
from __future__ import annotations

import math
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import engine as E
from . import engine_cheng as EC
from . import engine_debug as ED
from . import hip_ops as K

# --------------------------------------------------------------------------- #
# Parametrizers (compressai.ops.parametrizers / bound_ops; utils/ops.py:58-97)
# --------------------------------------------------------------------------- #


class LowerBound(nn.Module):
    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound)


class NonNegativeParametrizer(nn.Module):
    def __init__(self, minimum: float = 0.0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        pedestal = self.reparam_offset ** 2
        self.register_buffer("pedestal", torch.Tensor([pedestal]))
        bound = (self.minimum + self.reparam_offset ** 2) ** 0.5
        self.lower_bound = LowerBound(bound)

    def init(self, x):
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))

    def forward(self, x):
        return self.lower_bound(x) ** 2 - self.pedestal


class GDN(nn.Module):
    """GDN / IGDN parameters (compressai.layers.GDN == utils/ops.py:58-97).  Inside g_a/g_s the
    normalisation runs fused in the producing conv's epilogue; stand-alone use is not supported."""

    def __init__(self, in_channels: int, inverse: bool = False, beta_min: float = 1e-6, gamma_init: float = 0.1):
        super().__init__()
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        self.beta = nn.Parameter(self.beta_reparam.init(torch.ones(in_channels)))
        self.gamma_reparam = NonNegativeParametrizer()
        self.gamma = nn.Parameter(self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels)))

    def forward(self, x):
        raise RuntimeError("GDN runs fused inside g_a/g_s on this backend; call the transform, not the layer")


def conv(in_channels, out_channels, kernel_size=5, stride=2):
    """anchors/utils.py:112-119."""
    return nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(in_channels, out_channels, kernel_size=5, stride=2):
    """anchors/utils.py:122-130."""
    return nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              output_padding=stride - 1, padding=kernel_size // 2)


# --------------------------------------------------------------------------- #
# Fused transforms
# --------------------------------------------------------------------------- #


def _state(module: nn.Module) -> dict:
    return {k: v for k, v in module.state_dict(keep_vars=True).items()}


def _key(module: nn.Module):
    return tuple((p.data_ptr(), p._version) for p in module.parameters())


class _TransformFn(torch.autograd.Function):
    """One fused HIP chain as an autograd node.  Backward: the input gradient, and, when the transform's
    parameters require grad, their gradients from the HIP wgrad / GDN-parameter kernels (the bmshj2018
    transforms; train_engine.analysis_backward / synthesis_backward)."""

    @staticmethod
    def forward(ctx, x, module, *params):
        ex = module._executor()
        need_x = ctx.needs_input_grad[0]
        need_w = any(ctx.needs_input_grad[2:])
        if need_w and not module._wgrad_ok:
            raise NotImplementedError(f"{type(module).__name__}: parameter gradients are computed for the bmshj2018 "
                                      "g_a / g_s only; freeze this transform with requires_grad_(False)")
        x4 = K.to_nc4(x.detach().contiguous())
        # parameter gradients read the saved activations row-major (the wgrad kernels)
        kw = {"split": False} if need_w and isinstance(ex, (E.Analysis, E.Synthesis)) else {}
        out4, saved = ex.forward(x4, save=need_x or need_w, **kw)
        ctx.ex, ctx.saved, ctx.cin, ctx.module = ex, saved, x.shape[1], module
        ctx.x4 = x4 if need_w else None
        ctx.need_x, ctx.need_w = need_x, need_w
        return K.from_nc4(out4, module.out_channels)

    @staticmethod
    def backward(ctx, gy):
        from . import train_engine as T
        g4 = K.to_nc4(gy.contiguous())
        module, ex = ctx.module, ctx.ex
        pgrads = (None,) * (len(ctx.needs_input_grad) - 2)
        gx = None
        if ctx.need_w:
            named = list(module.named_parameters())
            params = {n: p.detach() for n, p in named}
            grads = {n: torch.zeros_like(p) for n, p in named}
            if isinstance(module, AnalysisTransform):
                gx4 = T.analysis_backward(ex, g4, ctx.x4, ctx.saved, params, grads, "", input_grad=ctx.need_x)
            else:
                gx4 = T.synthesis_backward(ex, g4, ctx.x4, ctx.saved, params, grads, "")
            pgrads = tuple(grads[n] for n, _ in named)
            if ctx.need_x:
                gx = K.from_nc4(gx4, ctx.cin)
        elif ctx.need_x:
            gx = K.from_nc4(ex.backward(g4, ctx.saved), ctx.cin)
        ctx.saved = ctx.x4 = None
        return (gx, None) + pgrads


class _FusedSequential(nn.Sequential):
    _exec_cls = None
    _wgrad_ok = False   # parameter gradients through the module API (bmshj2018 g_a / g_s)

    def __init__(self, *layers):
        super().__init__(*layers)
        self._ex = None
        self._ex_key = None

    def _executor(self):
        k = _key(self)
        if self._ex is None or self._ex_key != k:
            self._ex = self._make_executor(_state(self))
            self._ex_key = k
        return self._ex

    def forward(self, x):
        if not torch.is_grad_enabled():
            out4, _ = self._executor().forward(K.to_nc4(x.detach().contiguous()), save=False)
            return K.from_nc4(out4, self.out_channels)
        return _TransformFn.apply(x, self, *self.parameters())


class AnalysisTransform(_FusedSequential):
    """g_a: conv(3,N)-GDN-conv(N,N)-GDN-conv(N,N)-GDN-conv(N,M) (CompressAI bmshj2018)."""
    _wgrad_ok = True

    def __init__(self, N, M):
        super().__init__(conv(3, N), GDN(N), conv(N, N), GDN(N), conv(N, N), GDN(N), conv(N, M))
        self.out_channels = M

    def _make_executor(self, sd):
        return E.Analysis(sd, prefix="")


class SynthesisTransform(_FusedSequential):
    """g_s: deconv(M,N)-IGDN-deconv(N,N)-IGDN-deconv(N,N)-IGDN-deconv(N,3)."""
    _wgrad_ok = True

    def __init__(self, N, M):
        super().__init__(deconv(M, N), GDN(N, inverse=True), deconv(N, N), GDN(N, inverse=True),
                         deconv(N, N), GDN(N, inverse=True), deconv(N, 3))
        self.out_channels = 3

    def _make_executor(self, sd):
        return E.Synthesis(sd, prefix="")


class _ForwardOnly(nn.Sequential):
    def __init__(self, *layers):
        super().__init__(*layers)
        self._ex = None
        self._ex_key = None

    def _executor(self):
        k = _key(self)
        if self._ex is None or self._ex_key != k:
            self._ex = self._make_executor(_state(self))
            self._ex_key = k
        return self._ex

    def forward(self, x):
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            # no silent gradient hole: a caller that trains through the module API (train.py:349-362) must
            # use the HIP trainer (train_engine.RDTrainer, train.py --adv), which covers these transforms
            raise NotImplementedError(f"{type(self).__name__} is forward-only on the module API; freeze it "
                                      "(requires_grad_(False)) or train with train_engine.RDTrainer")
        out4 = self._run(self._executor(), K.to_nc4(x.detach().contiguous()))
        return K.from_nc4(out4, self.out_channels)


class HyperAnalysisTransform(_ForwardOnly):
    """h_a = conv(M,N,3,1)-ReLU-conv(N,N)-ReLU-conv(N,N)."""

    def __init__(self, N, M):
        super().__init__(conv(M, N, stride=1, kernel_size=3), nn.ReLU(inplace=True), conv(N, N),
                         nn.ReLU(inplace=True), conv(N, N))
        self.out_channels = N

    def _make_executor(self, sd):
        return E.HyperAnalysis(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4, take_abs=False)


class HyperSynthesisTransform(_ForwardOnly):
    """h_s = deconv(N,N)-ReLU-deconv(N,N)-ReLU-conv(N,M,3,1)-ReLU."""

    def __init__(self, N, M):
        super().__init__(deconv(N, N), nn.ReLU(inplace=True), deconv(N, N), nn.ReLU(inplace=True),
                         conv(N, M, stride=1, kernel_size=3), nn.ReLU(inplace=True))
        self.out_channels = M

    def _make_executor(self, sd):
        return E.HyperSynthesis(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


class MbtHyperAnalysisTransform(_ForwardOnly):
    """mbt2018 h_a = conv(M,N,3,1)-LReLU-conv(N,N,5,2)-LReLU-conv(N,N,5,2)."""

    def __init__(self, N, M):
        super().__init__(conv(M, N, stride=1, kernel_size=3), nn.LeakyReLU(inplace=True),
                         conv(N, N, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                         conv(N, N, stride=2, kernel_size=5))
        self.out_channels = N

    def _make_executor(self, sd):
        return E.MbtHyperAnalysis(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


class MbtHyperSynthesisTransform(_ForwardOnly):
    """mbt2018 h_s = deconv(N,M)-LReLU-deconv(M,3M/2)-LReLU-conv(3M/2,2M,3,1)."""

    def __init__(self, N, M):
        super().__init__(deconv(N, M, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                         deconv(M, M * 3 // 2, stride=2, kernel_size=5), nn.LeakyReLU(inplace=True),
                         conv(M * 3 // 2, M * 2, stride=1, kernel_size=3))
        self.out_channels = 2 * M

    def _make_executor(self, sd):
        return E.MbtHyperSynthesis(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


# --------------------------------------------------------------------------- #
# cheng2020-anchor layers (compressai.layers)
# --------------------------------------------------------------------------- #
def conv3x3(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv1x1(in_ch, out_ch, stride=1):
    return nn.Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def subpel_conv3x3(in_ch, out_ch, r=1):
    return nn.Sequential(nn.Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), nn.PixelShuffle(r))


class _FusedOnly(nn.Module):
    def forward(self, x):
        raise RuntimeError(f"{type(self).__name__} runs fused inside its transform on this backend")


class ResidualBlockWithStride(_FusedOnly):
    def __init__(self, in_ch, out_ch, stride=2):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch, stride=stride)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.gdn = GDN(out_ch)
        self.skip = conv1x1(in_ch, out_ch, stride=stride) if (stride != 1 or in_ch != out_ch) else None


class ResidualBlockUpsample(_FusedOnly):
    def __init__(self, in_ch, out_ch, upsample=2):
        super().__init__()
        self.subpel_conv = subpel_conv3x3(in_ch, out_ch, upsample)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv = conv3x3(out_ch, out_ch)
        self.igdn = GDN(out_ch, inverse=True)
        self.upsample = subpel_conv3x3(in_ch, out_ch, upsample)


class ResidualBlock(_FusedOnly):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None


class ChengAnalysisTransform(_FusedSequential):
    def __init__(self, N):
        super().__init__(ResidualBlockWithStride(3, N, 2), ResidualBlock(N, N), ResidualBlockWithStride(N, N, 2),
                         ResidualBlock(N, N), ResidualBlockWithStride(N, N, 2), ResidualBlock(N, N),
                         conv3x3(N, N, stride=2))
        self.out_channels = N

    def _make_executor(self, sd):
        return EC.ChengAnalysis(sd, prefix="")


class ChengSynthesisTransform(_FusedSequential):
    def __init__(self, N):
        super().__init__(ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N),
                         ResidualBlockUpsample(N, N, 2), ResidualBlock(N, N), ResidualBlockUpsample(N, N, 2),
                         ResidualBlock(N, N), subpel_conv3x3(N, 3, 2))
        self.out_channels = 3

    def _make_executor(self, sd):
        return EC.ChengSynthesis(sd, prefix="")


class ChengHyperAnalysis(_ForwardOnly):
    def __init__(self, N):
        super().__init__(conv3x3(N, N), nn.LeakyReLU(inplace=True), conv3x3(N, N), nn.LeakyReLU(inplace=True),
                         conv3x3(N, N, stride=2), nn.LeakyReLU(inplace=True), conv3x3(N, N),
                         nn.LeakyReLU(inplace=True), conv3x3(N, N, stride=2))
        self.out_channels = N

    def _make_executor(self, sd):
        return EC.ChengHA(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


class ChengHyperSynthesis(_ForwardOnly):
    def __init__(self, N):
        super().__init__(conv3x3(N, N), nn.LeakyReLU(inplace=True), subpel_conv3x3(N, N, 2),
                         nn.LeakyReLU(inplace=True), conv3x3(N, N * 3 // 2), nn.LeakyReLU(inplace=True),
                         subpel_conv3x3(N * 3 // 2, N * 3 // 2, 2), nn.LeakyReLU(inplace=True),
                         conv3x3(N * 3 // 2, N * 2))
        self.out_channels = 2 * N

    def _make_executor(self, sd):
        return EC.ChengHS(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


class EntropyParameters(_ForwardOnly):
    def __init__(self, M):
        super().__init__(nn.Conv2d(M * 12 // 3, M * 10 // 3, 1), nn.LeakyReLU(inplace=True),
                         nn.Conv2d(M * 10 // 3, M * 8 // 3, 1), nn.LeakyReLU(inplace=True),
                         nn.Conv2d(M * 8 // 3, M * 6 // 3, 1))
        self.out_channels = M * 6 // 3

    def _make_executor(self, sd):
        return EC.ChengEntropyParameters(sd, prefix="")

    def _run(self, ex, x4):
        return ex.forward(x4)


class MaskedConv2d(nn.Conv2d):
    """compressai.layers.MaskedConv2d (type 'A' context model), forward on the HIP conv engine."""

    def __init__(self, *args, mask_type="A", **kwargs):
        super().__init__(*args, **kwargs)
        if mask_type not in ("A", "B"):
            raise ValueError(f'Invalid "mask_type" value "{mask_type}"')
        self.mask_type = mask_type
        self.register_buffer("mask", torch.ones_like(self.weight.data))
        _, _, h, w = self.mask.size()
        self.mask[:, :, h // 2, w // 2 + (mask_type == "B"):] = 0
        self.mask[:, :, h // 2 + 1:] = 0
        self._ex, self._ex_key = None, None

    def forward(self, x):
        if self.mask_type != "A":
            raise NotImplementedError("mask type B is not used by cheng2020 / mbt2018")
        self.weight.data *= self.mask   # as CompressAI's forward: the stored weight keeps its masked taps at zero
        k = (self.weight.data_ptr(), self.weight._version, self.bias.data_ptr(), self.bias._version)
        if self._ex is None or self._ex_key != k:
            self._ex = EC.ChengContext({"weight": self.weight.detach(), "bias": self.bias.detach()}, prefix="")
            self._ex_key = k
        return K.from_nc4(self._ex.forward(K.to_nc4(x.detach().contiguous())), self.out_channels)


# --------------------------------------------------------------------------- #
# Entropy models (compressai.entropy_models)
# --------------------------------------------------------------------------- #


class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound: float = 1e-9):
        super().__init__()
        self.use_likelihood_bound = likelihood_bound > 0
        self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    def _coder_tables(self):
        """Host coding tables from the `_quantized_cdf` / `_cdf_length` / `_offset` buffers (cached)."""
        from . import entropy_coding as EC_
        if self._offset.numel() == 0:
            raise ValueError("Entropy model is not updated: run update() first (CompressAI semantics)")
        k = tuple((b.data_ptr(), b._version) for b in (self._quantized_cdf, self._cdf_length, self._offset))
        if getattr(self, "_tab_key", None) != k:
            self._tab = EC_.Tables(self._quantized_cdf, self._cdf_length, self._offset)
            self._tab_key = k
        return self._tab

    def _set_tables(self, cdf, length, offset):
        dev = self._offset.device
        self._quantized_cdf = cdf.to(dev)
        self._cdf_length = length.to(dev)
        self._offset = offset.to(dev)

    def quantize(self, inputs, mode, means=None):
        """CompressAI EntropyModel.quantize ("noise" | "dequantize" | "symbols"); round = half-to-even."""
        if mode not in ("noise", "dequantize", "symbols"):
            raise ValueError(f'Invalid quantization mode: "{mode}"')
        if mode == "noise":
            return inputs + torch.empty_like(inputs).uniform_(-0.5, 0.5)
        outputs = inputs.clone()
        if means is not None:
            outputs -= means
        outputs = torch.round(outputs)
        if mode == "dequantize":
            if means is not None:
                outputs += means
            return outputs
        return outputs.int()


class EntropyBottleneck(EntropyModel):
    def __init__(self, channels, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3)):
        super().__init__()
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = math.log(math.expm1(1 / scale / filters[i + 1]))
            self.register_parameter(f"_matrix{i:d}",
                                    nn.Parameter(torch.full((channels, filters[i + 1], filters[i]), init)))
            self.register_parameter(f"_bias{i:d}",
                                    nn.Parameter(torch.empty(channels, filters[i + 1], 1).uniform_(-0.5, 0.5)))
            if i < len(self.filters):
                self.register_parameter(f"_factor{i:d}", nn.Parameter(torch.zeros(channels, filters[i + 1], 1)))
        self.quantiles = nn.Parameter(torch.Tensor([-self.init_scale, 0, self.init_scale]).repeat(channels, 1, 1))
        target = math.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))
        self._packed = None
        self._packed_key = None

    def _pack(self):
        names = K.PackedEB.NAMES
        k = tuple((getattr(self, n).data_ptr(), getattr(self, n)._version) for n in names)
        if self._packed is None or self._packed_key != k:
            self._packed = K.PackedEB({n: getattr(self, n) for n in names})
            self._packed_key = k
        return self._packed

    def _logits_cumulative(self, inputs, stop_gradient: bool):
        logits = inputs
        for i in range(len(self.filters) + 1):
            matrix = getattr(self, f"_matrix{i:d}")
            bias = getattr(self, f"_bias{i:d}")
            if stop_gradient:
                matrix, bias = matrix.detach(), bias.detach()
            logits = torch.matmul(F.softplus(matrix), logits) + bias
            if i < len(self.filters):
                factor = getattr(self, f"_factor{i:d}")
                if stop_gradient:
                    factor = factor.detach()
                logits = logits + torch.tanh(factor) * torch.tanh(logits)
        return logits

    def loss(self):
        """Aux loss on the quantiles (parameter-only, C x 3 values; train.py:364, adv_train.py:190)."""
        logits = self._logits_cumulative(self.quantiles, stop_gradient=True)
        return torch.abs(logits - self.target).sum()

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    def update(self, force: bool = False) -> bool:
        """EntropyBottleneck.update: the quantised CDF tables (entropy_coding.eb_tables)."""
        from . import entropy_coding as EC_
        if self._offset.numel() > 0 and not force:
            return False
        prm = {n: getattr(self, n) for n in K.PackedEB.NAMES if not n.startswith("quantiles")}
        self._set_tables(*EC_.eb_tables(prm, self.quantiles, len(self.filters)))
        return True

    def compress(self, x):
        """x [B, C, H, W] on the HIP device -> one rANS bitstream per image (symbols round(x - median))."""
        from . import entropy_coding as EC_
        tab = self._coder_tables()
        B, C, H, W = x.shape
        sym, idx = EC_.eb_symbols(K.to_nc4(x.detach().contiguous()), C, self._get_medians().detach().reshape(-1)
                                  .contiguous())
        return EC_.encode_batch(sym, idx, tab)

    def decompress(self, strings, size):
        from . import entropy_coding as EC_
        tab = self._coder_tables()
        H, W = int(size[0]), int(size[1])
        B, C = len(strings), self.channels
        dev = self.quantiles.device
        idx = EC_.eb_indexes(B, C, H, W, "cpu")
        sym = EC_.decode_batch(strings, idx, tab)
        med = self._get_medians().detach().reshape(-1).contiguous()
        return K.from_nc4(EC_.dequantize(sym, B, C, H, W, medians=med, device=dev), C)

    def forward(self, x, training=None):
        if training is None:
            training = self.training
        C = x.shape[1]
        noise4 = None
        if training:
            noise4 = K.to_nc4(torch.empty_like(x).uniform_(-0.5, 0.5))
        zh4, lik4, _ = K.eb_likelihood(K.to_nc4(x.detach().contiguous()), C, self._pack(), training, noise4)
        return K.from_nc4(zh4, C), K.from_nc4(lik4, C)


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table=None, scale_bound=0.11, tail_mass=1e-9):
        super().__init__()
        self.tail_mass = float(tail_mass)
        self.register_buffer("scale_table", torch.Tensor(tuple(scale_table) if scale_table else ()))
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]))
        self.lower_bound_scale = LowerBound(scale_bound)

    def update_scale_table(self, scale_table, force: bool = False) -> bool:
        if self._offset.numel() > 0 and not force:
            return False
        dev = self.scale_bound.device
        self.scale_table = torch.Tensor(tuple(float(v) for v in scale_table)).to(dev)
        self.update()
        return True

    def update(self):
        """GaussianConditional.update: one quantised CDF per scale_table entry (entropy_coding.gc_tables)."""
        from . import entropy_coding as EC_
        self._set_tables(*EC_.gc_tables(self.scale_table, self.tail_mass))

    def build_indexes(self, scales):
        from . import entropy_coding as EC_
        s4 = K.to_nc4(scales.detach().contiguous())
        B, C, H, W = scales.shape
        _, idx = EC_.gc_symbols(s4, C, s4, None, self.scale_table.to(scales.device).contiguous(),
                                float(self.scale_bound))
        return idx.view(B, C, H, W)

    def compress(self, inputs, indexes, means=None):
        from . import entropy_coding as EC_
        tab = self._coder_tables()
        B, C, H, W = inputs.shape
        y4 = K.to_nc4(inputs.detach().contiguous())
        m4 = K.to_nc4(means.detach().contiguous()) if means is not None else None
        sym, _ = EC_.gc_symbols(y4, C, y4, m4, self.scale_table.to(inputs.device).contiguous(),
                                float(self.scale_bound))
        return EC_.encode_batch(sym, indexes.reshape(B, -1).to(torch.int32), tab)

    def decompress(self, strings, indexes, dtype=torch.float, means=None):
        from . import entropy_coding as EC_
        tab = self._coder_tables()
        B, C, H, W = indexes.shape
        sym = EC_.decode_batch(strings, indexes.reshape(B, -1).to(torch.int32), tab)
        dev = indexes.device if indexes.is_cuda else self.scale_bound.device
        m4 = K.to_nc4(means.detach().contiguous()) if means is not None else None
        return K.from_nc4(EC_.dequantize(sym, B, C, H, W, means4=m4, device=dev), C).to(dtype)

    def forward(self, inputs, scales, means=None, training=None):
        if training is None:
            training = self.training
        C = inputs.shape[1]
        noise4 = K.to_nc4(torch.empty_like(inputs).uniform_(-0.5, 0.5)) if training else None
        m4 = K.to_nc4(means.detach().contiguous()) if means is not None else None
        yh4, lik4, _ = K.gc_likelihood(K.to_nc4(inputs.detach().contiguous()), C,
                                       K.to_nc4(scales.detach().contiguous()), m4, training, noise4)
        return K.from_nc4(yh4, C), K.from_nc4(lik4, C)


# --------------------------------------------------------------------------- #
# Models (CompressAI bmshj2018)
# --------------------------------------------------------------------------- #


class CompressionModel(nn.Module):
    def aux_loss(self):
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def load_state_dict(self, state_dict, strict=True):
        # CompressAI buffers with checkpoint-dependent sizes (anchors/utils.py:74-109)
        for name, mod in self.named_modules():
            if isinstance(mod, EntropyModel):
                for b in ("_offset", "_quantized_cdf", "_cdf_length", "scale_table"):
                    key = f"{name}.{b}"
                    if key in state_dict and hasattr(mod, b):
                        getattr(mod, b).resize_(state_dict[key].size())
        return super().load_state_dict(state_dict, strict=strict)

    def update(self, scale_table=None, force: bool = False) -> bool:
        """CompressionModel.update: build the entropy coders' CDF tables (required before compress())."""
        from . import entropy_coding as EC_
        if scale_table is None:
            scale_table = EC_.get_scale_table()
        updated = False
        for m in self.modules():
            if isinstance(m, EntropyBottleneck):
                updated |= m.update(force=force)
            elif isinstance(m, GaussianConditional):
                updated |= m.update_scale_table(scale_table, force=force)
        return updated

    def attack_precision(self, requested: str | None = None) -> str:
        """Conv operand precision of the attack engine: the request, else x6 (fp32-accurate bf16x6): the 5x5
        stride-2 transforms of bmshj2018 / mbt2018, and cheng2020's 3x3 convs (engine_cheng.ChengKernels lists which
        launches; the rest keep fp32 operands).  'bf16': bf16-operand convs (bmshj2018 / mbt2018: bf16 activations
        too; cheng2020: bf16 operands over fp32 activations on its k3 conv_downs)."""
        return requested or "x6"

    def kernels(self, precision: str = "fp32"):
        """Whole-model HIP executor (used by the attack engine).  precision 'bf16': bf16-operand g_a / g_s
        convs (bmshj2018 / mbt2018: BASELINE config 5; cheng2020: engine_cheng.ChengKernels).  One executor per
        precision, each valid for one weight
        version: the fine-tune's x6 inner attack and fp32 train step share a weight update without repacking
        each other's executor (train.py adv_step -> RDTrainer.step)."""
        key = tuple((p.data_ptr(), p._version) for p in self.parameters())
        cache = getattr(self, "_ck_cache", None)
        if cache is None or cache[0] != key:
            cache = (key, {})
            self._ck_cache = cache
        ex = cache[1].get(precision)
        if ex is None:
            sd = {k: v.detach() for k, v in self.state_dict().items()}
            if self.model_kind == "cheng2020":
                ex = EC.ChengKernels(sd, precision=precision)
            elif self.model_kind == "debug":
                ex = ED.DebugKernels(sd, precision=precision)
            else:
                ex = E.CodecKernels(sd, self.model_kind, precision=precision)
            cache[1][precision] = ex
        return ex


class FactorizedPrior(CompressionModel):
    model_kind = "factorized"

    def __init__(self, N, M, **kwargs):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(M)
        self.g_a = AnalysisTransform(N, M)
        self.g_s = SynthesisTransform(N, M)
        self.N, self.M = int(N), int(M)

    def forward(self, x):
        y = self.g_a(x)
        y_hat, y_likelihoods = self.entropy_bottleneck(y)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods}}

    def compress(self, x):
        """FactorizedPrior.compress: rANS bitstreams of round(g_a(x) - medians)."""
        with torch.no_grad():
            y = self.g_a(x)
            return {"strings": [self.entropy_bottleneck.compress(y)], "shape": y.size()[-2:]}

    def decompress(self, strings, shape):
        with torch.no_grad():
            y_hat = self.entropy_bottleneck.decompress(strings[0], shape)
            return {"x_hat": self.g_s(y_hat).clamp_(0, 1)}


class ScaleHyperprior(CompressionModel):
    model_kind = "hyper"

    def __init__(self, N, M, **kwargs):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.g_a = AnalysisTransform(N, M)
        self.g_s = SynthesisTransform(N, M)
        self.h_a = HyperAnalysisTransform(N, M)
        self.h_s = HyperSynthesisTransform(N, M)
        self.gaussian_conditional = GaussianConditional(None)
        self.N, self.M = int(N), int(M)

    def forward(self, x):
        y = self.g_a(x)
        z = self.h_a(torch.abs(y))
        z_hat, z_likelihoods = self.entropy_bottleneck(z)
        scales_hat = self.h_s(z_hat)
        y_hat, y_likelihoods = self.gaussian_conditional(y, scales_hat)
        x_hat = self.g_s(y_hat)
        return {"x_hat": x_hat, "likelihoods": {"y": y_likelihoods, "z": z_likelihoods}}

    def compress(self, x):
        """ScaleHyperprior.compress: z -> EB bitstreams, scales = h_s(z_hat), y -> GC bitstreams.  One HIP pass
        (g_a, h_a, symbols, h_s, symbols on nChw4c tensors), then rANS per image on host threads."""
        from . import entropy_coding as EC_
        eb, gc = self.entropy_bottleneck, self.gaussian_conditional
        ztab, ytab = eb._coder_tables(), gc._coder_tables()
        ck = self.kernels()
        with torch.no_grad():
            x4 = K.to_nc4(x.detach().contiguous())
            y4, _ = ck.ga.forward(x4)
            z4 = ck.ha.forward(y4)
            B, _, zh, zw, _ = z4.shape
            med = eb._get_medians().detach().reshape(-1).contiguous()
            zs, zi = EC_.eb_symbols(z4, self.N, med)
            z_hat4 = EC_.dequantize(zs, B, self.N, zh, zw, medians=med, device=x.device)
            s4 = ck.hs.forward(z_hat4)
            ys, yi = EC_.gc_symbols(y4, self.M, s4, None, gc.scale_table.to(x.device).contiguous(),
                                    float(gc.scale_bound))
            z_strings = EC_.encode_batch(zs, zi, ztab)
            y_strings = EC_.encode_batch(ys, yi, ytab)
        return {"strings": [y_strings, z_strings], "shape": torch.Size((zh, zw))}

    def decompress(self, strings, shape):
        from . import entropy_coding as EC_
        eb, gc = self.entropy_bottleneck, self.gaussian_conditional
        ytab = gc._coder_tables()
        ck = self.kernels()
        dev = self.entropy_bottleneck.quantiles.device
        with torch.no_grad():
            z_hat = eb.decompress(strings[1], shape)
            s4 = ck.hs.forward(K.to_nc4(z_hat))
            B, _, yh, yw, _ = s4.shape
            _, yi = EC_.gc_symbols(s4, self.M, s4, None, gc.scale_table.to(dev).contiguous(), float(gc.scale_bound))
            ys = EC_.decode_batch(strings[0], yi, ytab)
            y_hat4 = EC_.dequantize(ys, B, self.M, yh, yw, device=dev)
            xh4, _ = ck.gs.forward(ck._to_gs(y_hat4))
            return {"x_hat": K.from_nc4(xh4, 3).clamp_(0, 1)}


def _ar_coder(model):
    """The model's packed context-model coder (ar_coding.ArCoder), rebuilt when a parameter changes or when the
    GaussianConditional's scale table / bound (buffers, replaced by update_scale_table(force=True)) change: the coder
    emits indexes into that table."""
    from .ar_coding import ArCoder
    gc = model.gaussian_conditional
    key = (tuple((p.data_ptr(), p._version) for p in model.parameters()),
           gc.scale_table.data_ptr(), gc.scale_table._version, tuple(gc.scale_table.shape), float(gc.scale_bound))
    cache = getattr(model, "_ar_cache", None)
    if cache is None or cache[0] != key:
        sd = {k: v.detach() for k, v in model.state_dict().items()}
        cache = (key, ArCoder(sd, model.M, gc.scale_table.to(model.entropy_bottleneck.quantiles.device),
                              float(gc.scale_bound)))
        model._ar_cache = cache
    return cache[1]


def _ar_compress(model, x):
    """JointAutoregressiveHierarchicalPriors.compress: z -> EntropyBottleneck bitstreams, params = h_s(z_hat), y ->
    the autoregressive GaussianConditional bitstreams (ar_coding; position-major symbols, one stream per image)."""
    from . import entropy_coding as EC_
    B, _, H, W = x.shape
    if H % 64 or W % 64:
        raise ValueError(f"{H}x{W}: the context models code images whose sides are multiples of 64 "
                         "(y is then exactly 4x the hyper-latent grid)")
    eb, gc = model.entropy_bottleneck, model.gaussian_conditional
    ztab, ytab = eb._coder_tables(), gc._coder_tables()
    ck = model.kernels()
    with torch.no_grad():
        x4 = K.to_nc4(x.detach().contiguous())
        y4, _ = ck.ga.forward(x4)
        z4 = ck.ha.forward(y4)
        _, _, zh, zw, _ = z4.shape
        med = eb._get_medians().detach().reshape(-1).contiguous()
        zs, zi = EC_.eb_symbols(z4, model.N, med)
        z_hat4 = EC_.dequantize(zs, B, model.N, zh, zw, medians=med, device=x.device)
        params4 = ck.hs.forward(z_hat4)
        ys, yi, _ = _ar_coder(model).encode(y4, params4)
        z_strings = EC_.encode_batch(zs, zi, ztab)
        y_strings = EC_.encode_batch(ys, yi, ytab)
    return {"strings": [y_strings, z_strings], "shape": torch.Size((zh, zw))}


def _ar_decompress(model, strings, shape):
    """JointAutoregressiveHierarchicalPriors.decompress: z_hat, params = h_s(z_hat), y_hat position by position,
    x_hat = g_s(y_hat).clamp(0, 1)."""
    eb, gc = model.entropy_bottleneck, model.gaussian_conditional
    ytab = gc._coder_tables()
    ck = model.kernels()
    with torch.no_grad():
        z_hat = eb.decompress(strings[1], shape)
        params4 = ck.hs.forward(K.to_nc4(z_hat))
        y_hat4 = _ar_coder(model).decode(strings[0], params4, ytab)
        xh4, _ = ck.gs.forward(y_hat4)
        return {"x_hat": K.from_nc4(xh4, 3).clamp_(0, 1)}


def _train_values(model, x, train_forward):
    """The train-mode forward's values (random quantisation noise) of a joint-prior model; a call that would need
    gradients is refused (no silent gradient hole, as _ForwardOnly): train through train_engine.RDTrainer."""
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in model.parameters())):
        raise NotImplementedError(f"{type(model).__name__} is forward-only on the module API; freeze it "
                                  "(requires_grad_(False)) or train with train_engine.RDTrainer")
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    f = train_forward(model.kernels("fp32"), sd.__getitem__, K.to_nc4(x.detach().contiguous()))
    return {"x_hat": K.from_nc4(f["xh4"], 3),
            "likelihoods": {"y": K.from_nc4(f["ylik4"], model.M), "z": K.from_nc4(f["zlik4"], model.N)}}


class Cheng2020Anchor(CompressionModel):
    """compressai.models.Cheng2020Anchor (JointAutoregressiveHierarchicalPriors with residual transforms).
    Eval-mode forward (the attack path) and the train-mode forward's values; the fine-tune's gradients come from
    the HIP trainer (train_engine.RDTrainer -> train_cheng.ChengTrainStep, train.py --adv)."""
    model_kind = "cheng2020"

    def __init__(self, N=192, **kwargs):
        super().__init__()
        M = N
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.g_a = ChengAnalysisTransform(N)
        self.h_a = ChengHyperAnalysis(N)
        self.h_s = ChengHyperSynthesis(N)
        self.g_s = ChengSynthesisTransform(N)
        self.gaussian_conditional = GaussianConditional(None)
        self.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)
        self.entropy_parameters = EntropyParameters(M)
        self.N, self.M = int(N), int(M)

    def forward(self, x):
        if self.training:
            from .train_cheng import train_forward
            return _train_values(self, x, train_forward)
        res = self.kernels().forward(K.to_nc4(x.detach().contiguous()))
        return {"x_hat": K.from_nc4(res["x_hat4"], 3),
                "likelihoods": {"y": K.from_nc4(res["lik4"]["y"], self.M), "z": K.from_nc4(res["lik4"]["z"], self.N)}}

    def compress(self, x):
        return _ar_compress(self, x)

    def decompress(self, strings, shape):
        return _ar_decompress(self, strings, shape)


class DebugAnalysisTransform(_FusedSequential):
    """ae_onelayer g_a = conv(3, M, kernel_size=3, stride=1) (anchors/model.py:13-15)."""

    def __init__(self, M):
        super().__init__(conv(3, M, kernel_size=3, stride=1))
        self.out_channels = M

    def _make_executor(self, sd):
        return ED.DebugAnalysis(sd, prefix="")


class DebugSynthesisTransform(_FusedSequential):
    """ae_onelayer g_s = deconv(M, 3, kernel_size=3, stride=1) (anchors/model.py:17-19)."""

    def __init__(self, M):
        super().__init__(deconv(M, 3, kernel_size=3, stride=1))
        self.out_channels = 3

    def _make_executor(self, sd):
        return ED.DebugSynthesis(sd, prefix="")


class DebugHyperSynthesisTransform(MbtHyperSynthesisTransform):
    """mbt2018's h_s at N = 3 (z_hat carried at 16 channels, engine_debug.DebugHyperSynthesis)."""

    def _make_executor(self, sd):
        return ED.DebugHyperSynthesis(sd, prefix="")


class AeOneLayer(CompressionModel):
    """anchors/model.py:8-33 ae_onelayer(MeanScaleHyperprior): one 3x3 stride-1 conv each way around the mean-scale
    hyperprior; forward reconstructs from the unquantised latent.  No pretrained weights exist (anchors/model.py:62):
    random / user-supplied weights, eval forward, the attack path (fp32 operands), the train-mode forward's values;
    the fine-tune's gradients come from train_engine.RDTrainer -> train_debug.DebugTrainStep."""
    model_kind = "debug"

    def __init__(self, N=3, M=192, **kwargs):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.g_a = DebugAnalysisTransform(M)
        self.g_s = DebugSynthesisTransform(M)
        self.h_a = MbtHyperAnalysisTransform(N, M)
        self.h_s = DebugHyperSynthesisTransform(N, M)
        self.gaussian_conditional = GaussianConditional(None)
        self.N, self.M = int(N), int(M)

    def attack_precision(self, requested: str | None = None) -> str:
        return requested or "fp32"

    def forward(self, x):
        if self.training:
            from .train_debug import train_forward
            return _train_values(self, x, train_forward)
        res = self.kernels("fp32").forward(K.to_nc4(x.detach().contiguous()))
        return {"x_hat": K.from_nc4(res["x_hat4"], 3),
                "likelihoods": {"y": K.from_nc4(res["lik4"]["y"], self.M), "z": K.from_nc4(res["lik4"]["z"], self.N)}}


class JointAutoregressiveHierarchicalPriors(CompressionModel):
    """compressai.models.JointAutoregressiveHierarchicalPriors (mbt2018): bmshj2018 g_a / g_s, LReLU hyper
    transforms, masked 5x5 context model.  Eval-mode forward (the attack path, anchors/model.py:95-104) and the
    train-mode forward's values; the fine-tune's gradients come from train_engine.RDTrainer -> train_mbt."""
    model_kind = "context"

    def __init__(self, N=192, M=192, **kwargs):
        super().__init__()
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.g_a = AnalysisTransform(N, M)
        self.g_s = SynthesisTransform(N, M)
        self.h_a = MbtHyperAnalysisTransform(N, M)
        self.h_s = MbtHyperSynthesisTransform(N, M)
        self.gaussian_conditional = GaussianConditional(None)
        self.entropy_parameters = EntropyParameters(M)
        self.context_prediction = MaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)
        self.N, self.M = int(N), int(M)

    def forward(self, x):
        if self.training:
            from .train_mbt import train_forward
            return _train_values(self, x, train_forward)
        res = self.kernels().forward(K.to_nc4(x.detach().contiguous()))
        return {"x_hat": K.from_nc4(res["x_hat4"], 3),
                "likelihoods": {"y": K.from_nc4(res["lik4"]["y"], self.M), "z": K.from_nc4(res["lik4"]["z"], self.N)}}

    def compress(self, x):
        return _ar_compress(self, x)

    def decompress(self, strings, shape):
        return _ar_decompress(self, strings, shape)


# --------------------------------------------------------------------------- #
# Zoo constructors (compressai.zoo)
# --------------------------------------------------------------------------- #
_CFG = {
    "bmshj2018-factorized": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "bmshj2018-hyperprior": {q: ((128, 192) if q <= 5 else (192, 320)) for q in range(1, 9)},
    "mbt2018": {q: ((192, 192) if q <= 4 else (192, 320)) for q in range(1, 9)},
    "cheng2020-anchor": {q: (128 if q <= 3 else 192, None) for q in range(1, 7)},
}


def _load_pretrained(model, arch, quality, metric):
    """Pretrained zoo weights need a download the offline box cannot do (coder.py:96-101).
    A local CompressAI-format file is used when present: $TORCH_HOME/checkpoints/<arch>-<quality>-<metric>*.pth*"""
    import glob
    import os
    home = os.environ.get("TORCH_HOME", "./ckpts/torch/")
    pats = glob.glob(os.path.join(home, "checkpoints", f"{arch}-{quality}*"))
    if not pats:
        raise RuntimeError(f"pretrained {arch} q{quality} ({metric}) needs a network download; place the "
                           f"CompressAI checkpoint under {home}/checkpoints or pass -ckpt")
    sd = torch.load(pats[0], map_location="cpu", weights_only=True)
    model.load_state_dict(sd.get("state_dict", sd))
    return model


def bmshj2018_factorized(quality, metric="mse", pretrained=False, progress=True, **kwargs):
    N, M = _CFG["bmshj2018-factorized"][quality]
    m = FactorizedPrior(N, M)
    return _load_pretrained(m, "bmshj2018-factorized", quality, metric) if pretrained else m


def bmshj2018_hyperprior(quality, metric="mse", pretrained=False, progress=True, **kwargs):
    N, M = _CFG["bmshj2018-hyperprior"][quality]
    m = ScaleHyperprior(N, M)
    return _load_pretrained(m, "bmshj2018-hyperprior", quality, metric) if pretrained else m


def cheng2020_anchor(quality, metric="mse", pretrained=False, progress=True, **kwargs):
    if quality not in _CFG["cheng2020-anchor"]:
        raise ValueError(f"cheng2020-anchor quality {quality} not in 1..6")
    N, _ = _CFG["cheng2020-anchor"][quality]
    m = Cheng2020Anchor(N)
    return _load_pretrained(m, "cheng2020-anchor", quality, metric) if pretrained else m


def mbt2018(quality, metric="mse", pretrained=False, progress=True, **kwargs):
    if quality not in _CFG["mbt2018"]:
        raise ValueError(f"mbt2018 quality {quality} not in 1..8")
    N, M = _CFG["mbt2018"][quality]
    m = JointAutoregressiveHierarchicalPriors(N, M)
    return _load_pretrained(m, "mbt2018", quality, metric) if pretrained else m
