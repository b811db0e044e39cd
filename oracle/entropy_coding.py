"""CPU restatement of CompressAI's entropy coding: the quantised-CDF tables of
EntropyBottleneck.update / GaussianConditional.update, build_indexes, and the 64-bit rANS coder with 16-bit
frequencies and 4-bit bypass coding that EntropyModel.compress / decompress drive.

TEST INFRASTRUCTURE (see oracle/__init__.py).  CompressAI is not vendored in /root/reference and not
installed, so this follows its published algorithm (compressai/entropy_models/entropy_models.py, the C++
rans_interface / pmf_to_quantized_cdf, ryg_rans rans64.h); the reference's own footprint is the buffers its
checkpoints carry (`_quantized_cdf`, `_offset`, `_cdf_length`, `scale_table`; anchors/balle.py:57-72,
anchors/utils.py:74-109).  PARITY UNPINNED: no CompressAI bitstream or table fixture exists in the reference.
Pure-Python loops: small cases only.
"""
from __future__ import annotations

import math

import torch

PRECISION = 16
BYPASS_BITS = 4
BYPASS_MAX = (1 << BYPASS_BITS) - 1
RANS_L = 1 << 31
MASK64 = (1 << 64) - 1


def get_scale_table(lo=0.11, hi=256, levels=64):
    """compressai.models.utils get_scale_table."""
    return torch.exp(torch.linspace(math.log(lo), math.log(hi), levels))


def pmf_to_quantized_cdf(pmf, precision=PRECISION):
    """pmf (float32 values) -> cumulative frequencies summing to 2^precision, each slot >= 1."""
    f32 = [float(torch.tensor(p, dtype=torch.float32)) for p in pmf]
    one = float(1 << precision)
    cdf = [0] + [int(round_half_away(float(torch.tensor(p, dtype=torch.float32) * torch.tensor(one))))
                 for p in f32]
    total = sum(cdf)
    assert total > 0
    cdf = [((1 << precision) * v) // total for v in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = 1 << precision
    n = len(cdf) - 1
    for i in range(n):
        if cdf[i] == cdf[i + 1]:
            best_freq, best = None, -1
            for j in range(n):
                f = cdf[j + 1] - cdf[j]
                if f > 1 and (best_freq is None or f < best_freq):
                    best_freq, best = f, j
            assert best != -1
            if best < i:
                for j in range(best + 1, i + 1):
                    cdf[j] -= 1
            else:
                for j in range(i + 1, best + 1):
                    cdf[j] += 1
    return cdf


def round_half_away(v: float) -> float:
    """std::round (half away from zero)."""
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length):
    cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
    for i, p in enumerate(pmf):
        prob = torch.cat((p[: int(pmf_length[i])], tail_mass[i]), dim=0)
        c = pmf_to_quantized_cdf(prob.tolist())
        cdf[i, : len(c)] = torch.tensor(c, dtype=torch.int32)
    return cdf


def eb_tables(P, prefix="entropy_bottleneck", logits_cumulative=None):
    """EntropyBottleneck.update: (quantized_cdf, cdf_length, offset, medians) from the CDF MLP and quantiles."""
    from . import codec
    q = P[f"{prefix}.quantiles"].detach().float()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    offset = -minima
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lc = logits_cumulative or (lambda v: codec.eb_logits_cumulative(P, v, prefix))
    lower = lc(samples - 0.5)
    upper = lc(samples + 0.5)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    cdf = _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), offset.int(), medians


def gc_tables(scale_table, tail_mass=1e-9):
    """GaussianConditional.update: (quantized_cdf, cdf_length, offset)."""
    from statistics import NormalDist
    multiplier = -NormalDist().inv_cdf(tail_mass / 2)
    pmf_center = torch.ceil(scale_table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(pmf_length.max())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    s = scale_table.unsqueeze(1).float()
    cum = lambda x: 0.5 * torch.erfc(float(-(2 ** -0.5)) * x)   # noqa: E731
    upper = cum((0.5 - samples) / s)
    lower = cum((-0.5 - samples) / s)
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-pmf_center).int()


def build_indexes(scales, scale_table, bound=0.11):
    s = torch.clamp(scales, min=bound)
    idx = torch.full(scales.shape, len(scale_table) - 1, dtype=torch.int32)
    for v in scale_table[:-1]:
        idx -= (s <= v).int()
    return idx


# --------------------------------------------------------------------------- #
# rANS (ryg_rans rans64 + CompressAI bypass coding)
# --------------------------------------------------------------------------- #
def _expand(s, cdf, max_value, offset):
    value = s - offset
    raw = 0
    if value < 0:
        raw, value = -2 * value - 1, max_value
    elif value >= max_value:
        raw, value = 2 * (value - max_value), max_value
    seq = [(cdf[value], cdf[value + 1] - cdf[value], False)]
    if value == max_value:
        nb = 0
        while (raw >> (nb * BYPASS_BITS)) != 0:
            nb += 1
        v = nb
        while v >= BYPASS_MAX:
            seq.append((BYPASS_MAX, 0, True))
            v -= BYPASS_MAX
        seq.append((v, 0, True))
        for j in range(nb):
            seq.append(((raw >> (j * BYPASS_BITS)) & BYPASS_MAX, 0, True))
    return seq


def rans_encode(symbols, indexes, cdfs, cdf_sizes, offsets) -> bytes:
    syms = []
    for s, k in zip(symbols, indexes):
        syms.extend(_expand(int(s), [int(v) for v in cdfs[k]], int(cdf_sizes[k]) - 2, int(offsets[k])))
    x = RANS_L
    words = []   # emitted back to front
    for start, freq, bypass in reversed(syms):
        f = (1 << (PRECISION - BYPASS_BITS)) if bypass else freq
        x_max = ((RANS_L >> PRECISION) << 32) * f
        if x >= x_max:
            words.append(x & 0xFFFFFFFF)
            x >>= 32
        if bypass:
            x = (x << BYPASS_BITS) | start
        else:
            x = ((x // freq) << PRECISION) + (x % freq) + start
    words.append(x >> 32)
    words.append(x & 0xFFFFFFFF)
    words.reverse()
    return b"".join(w.to_bytes(4, "little") for w in words)


def rans_decode(data: bytes, indexes, cdfs, cdf_sizes, offsets):
    words = [int.from_bytes(data[i:i + 4], "little") for i in range(0, len(data), 4)]
    x = words[0] | (words[1] << 32)
    p = 2
    out = []
    mask = (1 << PRECISION) - 1

    def get_bits(nb):
        nonlocal x, p
        v = x & ((1 << nb) - 1)
        x >>= nb
        if x < RANS_L:
            x = ((x << 32) | words[p]) & MASK64
            p += 1
        return v

    for k in indexes:
        cdf = [int(v) for v in cdfs[k]]
        size = int(cdf_sizes[k])
        max_value = size - 2
        cum = x & mask
        s = next(i for i in range(size) if cdf[i] > cum) - 1
        x = (cdf[s + 1] - cdf[s]) * (x >> PRECISION) + (x & mask) - cdf[s]
        if x < RANS_L:
            x = ((x << 32) | words[p]) & MASK64
            p += 1
        value = s
        if value == max_value:
            v = get_bits(BYPASS_BITS)
            nb = v
            while v == BYPASS_MAX:
                v = get_bits(BYPASS_BITS)
                nb += v
            raw = 0
            for j in range(nb):
                raw |= get_bits(BYPASS_BITS) << (j * BYPASS_BITS)
            value = raw >> 1
            value = -value - 1 if raw & 1 else value + max_value
        out.append(value + int(offsets[k]))
    return out


def compress_ar_symbols(P, y, params, scale_table, bound=0.11):
    """JointAutoregressiveHierarchicalPriors._compress_ar (compressai/models/google.py; the context models the
    reference builds at anchors/model.py:74-77, entropy estimated at anchors/model.py:97-106), for every image of
    y [B, M, H, W] with params = h_s(z_hat) [B, 2M, H, W]: raster order; y_crop = the 5x5 window of the zero-padded
    y_hat; ctx = conv2d(y_crop, masked weight, bias); gaussian_params = entropy_parameters(cat(params, ctx));
    scales, means = chunk(2); index = build_indexes(scales); symbol = round(y - means); y_hat = symbol + means.
    Returns (symbols, indexes) [B, H W M] int32 in the bitstream's position-major order and y_hat [B, M, H, W].
    Pure-Python loop over positions: small latents only."""
    from .codec import context_mask, entropy_parameters
    B, M, H, W = y.shape
    w = P["context_prediction.weight"] * context_mask(P["context_prediction.weight"].shape[-1])
    pad = 2
    y_hat = torch.nn.functional.pad(y, (pad, pad, pad, pad))
    syms = torch.empty((B, H * W, M), dtype=torch.int32)
    idxs = torch.empty_like(syms)
    for h in range(H):
        for x in range(W):
            crop = y_hat[:, :, h:h + 5, x:x + 5]
            ctx = torch.nn.functional.conv2d(crop, w, P["context_prediction.bias"])
            gp = entropy_parameters(P, torch.cat((params[:, :, h:h + 1, x:x + 1], ctx), dim=1))
            scales, means = gp.chunk(2, 1)
            idx = build_indexes(scales, scale_table, bound).reshape(B, M)
            q = torch.round(crop[:, :, pad, pad] - means.reshape(B, M)).int()
            y_hat[:, :, h + pad, x + pad] = q.float() + means.reshape(B, M)
            syms[:, h * W + x] = q
            idxs[:, h * W + x] = idx.int()
    return syms.reshape(B, -1), idxs.reshape(B, -1), y_hat[:, :, pad:-pad, pad:-pad]
