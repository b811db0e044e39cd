"""Real entropy coding for the bmshj2018 models: CompressAI's update() / compress() /
decompress() on libica_hip.

  tables    EntropyBottleneck.update / GaussianConditional.update: the pmf of every CDF row is computed once per
            weight version with the same float32 formulas CompressAI uses (host, CPU torch: deterministic, tiny);
            its 16-bit quantisation runs in C++ (ica_pmf_to_quantized_cdf).  The results fill the
            `_quantized_cdf` / `_offset` / `_cdf_length` buffers a CompressAI checkpoint carries
            (anchors/balle.py:57-72 restores them; loaded tables are used as they are).
  symbols   on the GPU straight from the nChw4c latents (ica_gc_symbols / ica_eb_symbols), copied to the host
            once per batch.
  rANS      ica_rans_encode / ica_rans_decode, one bitstream per image (CompressAI's stream format: a single
            sequential 64-bit rANS state), images of a batch on parallel host threads (ctypes drops the GIL).
  dequant   decoded symbols back into nChw4c latents on the GPU (ica_dequantize).

The context models (mbt2018, cheng2020) need CompressAI's autoregressive decoder, which is not built.
"""
from __future__ import annotations

import ctypes as C
import math
from concurrent.futures import ThreadPoolExecutor
from statistics import NormalDist

import numpy as np
import torch
import torch.nn.functional as F

from . import hip_ops as K
from ._lib import call, lib, ptr, stream

PRECISION = 16


def get_scale_table(lo=0.11, hi=256, levels=64):
    """compressai.models.utils.get_scale_table."""
    return torch.exp(torch.linspace(math.log(lo), math.log(hi), levels))


def pmf_to_quantized_cdf(pmf, precision=PRECISION) -> np.ndarray:
    p = np.ascontiguousarray(np.asarray(pmf, dtype=np.float32))
    out = np.zeros(p.size + 1, np.int32)
    rc = lib().ica_pmf_to_quantized_cdf(p.ctypes.data_as(C.c_void_p), int(p.size), int(precision),
                                        out.ctypes.data_as(C.c_void_p))
    if rc != 0:
        raise ValueError(f"pmf_to_quantized_cdf failed ({rc}): non-finite, negative or all-zero pmf")
    return out


def _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length) -> torch.Tensor:
    """EntropyModel._pmf_to_cdf: rows [pmf[:length], tail] -> int32 [rows, max_length + 2]."""
    cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
    for i, p in enumerate(pmf):
        prob = torch.cat((p[: int(pmf_length[i])], tail_mass[i]), dim=0)
        c = pmf_to_quantized_cdf(prob.numpy())
        cdf[i, : c.size] = torch.from_numpy(c)
    return cdf


def _logits_cumulative(params: dict, v: torch.Tensor, n_filters: int) -> torch.Tensor:
    logits = v
    for i in range(n_filters + 1):
        logits = torch.matmul(F.softplus(params[f"_matrix{i}"]), logits)
        logits = logits + params[f"_bias{i}"]
        if i < n_filters:
            logits = logits + torch.tanh(params[f"_factor{i}"]) * torch.tanh(logits)
    return logits


def eb_tables(params: dict, quantiles: torch.Tensor, n_filters: int = 4):
    """EntropyBottleneck.update on CPU float32: (quantized_cdf, cdf_length, offset)."""
    params = {k: v.detach().float().cpu() for k, v in params.items()}
    q = quantiles.detach().float().cpu()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lower = _logits_cumulative(params, samples - 0.5, n_filters)
    upper = _logits_cumulative(params, samples + 0.5, n_filters)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    cdf = _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-minima).int()


def gc_tables(scale_table: torch.Tensor, tail_mass: float = 1e-9):
    """GaussianConditional.update on CPU float32: (quantized_cdf, cdf_length, offset)."""
    scale_table = scale_table.detach().float().cpu()
    multiplier = -NormalDist().inv_cdf(tail_mass / 2)   # scipy.stats.norm.ppf in CompressAI
    pmf_center = torch.ceil(scale_table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(pmf_length.max())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    s = scale_table.unsqueeze(1)
    const = float(-(2 ** -0.5))
    upper = 0.5 * torch.erfc(const * ((0.5 - samples) / s))
    lower = 0.5 * torch.erfc(const * ((-0.5 - samples) / s))
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-pmf_center).int()


class Tables:
    """Host copies of one entropy model's coding tables (contiguous int32, what the C coder reads)."""

    def __init__(self, cdf: torch.Tensor, cdf_length: torch.Tensor, offset: torch.Tensor):
        self.cdf = np.ascontiguousarray(cdf.detach().cpu().numpy().astype(np.int32))
        self.sizes = np.ascontiguousarray(cdf_length.detach().cpu().numpy().reshape(-1).astype(np.int32))
        self.offsets = np.ascontiguousarray(offset.detach().cpu().numpy().reshape(-1).astype(np.int32))
        if self.cdf.ndim != 2 or self.cdf.shape[0] != self.sizes.size or self.sizes.size != self.offsets.size:
            raise ValueError("inconsistent entropy-coder tables (run update() first)")
        self.stride = self.cdf.shape[1]

    def _args(self):
        v = C.c_void_p
        return (self.cdf.ctypes.data_as(v), int(self.stride), self.sizes.ctypes.data_as(v),
                self.offsets.ctypes.data_as(v), int(self.sizes.size))


def _encode_one(sym: np.ndarray, idx: np.ndarray, tab: Tables) -> bytes:
    n = sym.size
    cap = 4 * (10 * n + 2)
    out = np.empty(cap, np.uint8)
    need = C.c_long(0)
    v = C.c_void_p
    r = lib().ica_rans_encode(sym.ctypes.data_as(v), idx.ctypes.data_as(v), n, *tab._args(), out.ctypes.data_as(v),
                              cap, C.byref(need))
    if r < 0:
        raise RuntimeError(f"ica_rans_encode failed ({r})")
    return out[:r].tobytes()


def _decode_one(data: bytes, idx: np.ndarray, tab: Tables) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8)
    out = np.empty(idx.size, np.int32)
    v = C.c_void_p
    rc = lib().ica_rans_decode(buf.ctypes.data_as(v), buf.size, idx.ctypes.data_as(v), idx.size, *tab._args(),
                               out.ctypes.data_as(v))
    if rc != 0:
        raise RuntimeError(f"ica_rans_decode failed ({rc}): truncated or corrupt bitstream")
    return out


def _pool(n):
    return ThreadPoolExecutor(max_workers=max(1, min(n, 16)))


def encode_batch(sym: torch.Tensor, idx: torch.Tensor, tab: Tables) -> list:
    """sym / idx: [B, n] int32 (device or host) -> one bitstream per image."""
    s = np.ascontiguousarray(sym.cpu().numpy())
    i = np.ascontiguousarray(idx.cpu().numpy())
    with _pool(s.shape[0]) as ex:
        return list(ex.map(lambda b: _encode_one(s[b], i[b], tab), range(s.shape[0])))


def decode_batch(strings, idx: torch.Tensor, tab: Tables) -> torch.Tensor:
    """strings: B bitstreams, idx: [B, n] int32 -> [B, n] int32 symbols (host)."""
    i = np.ascontiguousarray(idx.cpu().numpy())
    with _pool(len(strings)) as ex:
        rows = list(ex.map(lambda b: _decode_one(strings[b], i[b], tab), range(len(strings))))
    return torch.from_numpy(np.stack(rows, 0))


# --------------------------------------------------------------------------- #
# Device helpers (nChw4c latents <-> NCHW-ordered int32 symbols)
# --------------------------------------------------------------------------- #
def eb_symbols(z4, C_, medians):
    B, _, H, W, _ = z4.shape
    sym = torch.empty((B, C_ * H * W), dtype=torch.int32, device=z4.device)
    idx = torch.empty_like(sym)
    call("ica_eb_symbols", ptr(z4), ptr(medians), ptr(sym), ptr(idx), B, C_, H, W, stream())
    return sym, idx


def gc_symbols(y4, C_, scales4, means4, scale_table, bound=0.11):
    B, _, H, W, _ = y4.shape
    sym = torch.empty((B, C_ * H * W), dtype=torch.int32, device=y4.device)
    idx = torch.empty_like(sym)
    call("ica_gc_symbols", ptr(y4), ptr(scales4), ptr(means4), ptr(scale_table), int(scale_table.numel()),
         float(bound), ptr(sym), ptr(idx), B, C_, H, W, stream())
    return sym, idx


def eb_indexes(B, C_, H, W, device):
    return torch.arange(C_, dtype=torch.int32, device=device).view(1, C_, 1).expand(B, C_, H * W).reshape(B, -1)


def dequantize(sym, B, C_, H, W, means4=None, medians=None, device=None):
    sym = sym.to(device).contiguous()
    out4 = K.empty_nc4(B, C_, H, W, device)
    if C_ % 4:
        out4.zero_()
    call("ica_dequantize", ptr(sym), ptr(means4), ptr(medians), ptr(out4), B, C_, H, W, stream())
    return out4
