"""Autoregressive coding of the context models' latents (mbt2018 / cheng2020): the compress() / decompress() of
CompressAI's JointAutoregressiveHierarchicalPriors (its _compress_ar / _decompress_ar; the models the reference
builds at anchors/model.py:74-77, whose y entropy model is the masked 5x5 context prediction of
anchors/model.py:97-106), on the HIP step kernel of csrc/ica_ar.hip.

encode(y4, params4): one launch; one workgroup per image walks the latent raster and emits the symbols / CDF rows
in the bitstream's position-major order, which the host rANS coder (ica_codec.hip) turns into one bitstream per
image.  decode(strings, params4): the next position's context needs the symbols just decoded, so every position is
one step launch (apply the previous position's symbols, emit this position's rows / means) and one host decode of
that position for every image (ica_rans_dec_step).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import hip_ops as K
from ._lib import ArArgs, call, lib, ptr, stream

# the type-A mask's causal taps of the 5x5 window, in the order of the packed context weight (ica_ar.hip)
CAUSAL_TAPS = [(ky, kx) for ky in range(2) for kx in range(5)] + [(2, 0), (2, 1)]


class ArCoder:
    """Packed context-model weights of one model (the state dict's context_prediction / entropy_parameters)."""

    def __init__(self, sd: dict, M: int, scale_table: torch.Tensor, scale_bound: float = 0.11):
        wc = sd["context_prediction.weight"].detach().float()
        if wc.shape[0] != 2 * M or wc.shape[1] != M or tuple(wc.shape[2:]) != (5, 5):
            raise ValueError(f"context_prediction weight {tuple(wc.shape)}: expected ({2 * M}, {M}, 5, 5)")
        self.M = M
        self.dev = wc.device
        # [2M][12][M] -> [2M][12 M]: k = tap * M + c (the masked taps never enter: type-A mask by construction)
        self.wc = torch.stack([wc[:, :, ky, kx] for ky, kx in CAUSAL_TAPS], 1).reshape(2 * M, 12 * M).contiguous()
        self.bc = sd["context_prediction.bias"].detach().float().contiguous()
        ws = [sd[f"entropy_parameters.{i}.weight"].detach().float() for i in (0, 2, 4)]
        self.bs = [sd[f"entropy_parameters.{i}.bias"].detach().float().contiguous() for i in (0, 2, 4)]
        self.ws = [w.reshape(w.shape[0], w.shape[1]).contiguous() for w in ws]
        self.E1, self.E2 = self.ws[0].shape[0], self.ws[1].shape[0]
        if self.ws[0].shape[1] != 4 * M or self.ws[2].shape[0] != 2 * M:
            raise ValueError("entropy_parameters: expected 4M -> E1 -> E2 -> 2M 1x1 convs")
        self.table = scale_table.detach().float().to(self.dev).contiguous()
        self.bound = float(scale_bound)

    def _args(self, B, H, W, y4=None, params4=None, yhat=None, sym=None, idx=None, sym_in=None, means=None):
        return ArArgs(ptr(y4), ptr(params4), ptr(yhat), ptr(sym), ptr(idx), ptr(sym_in), ptr(means), ptr(self.wc),
                      ptr(self.bc), ptr(self.ws[0]), ptr(self.bs[0]), ptr(self.ws[1]), ptr(self.bs[1]),
                      ptr(self.ws[2]), ptr(self.bs[2]), ptr(self.table), int(self.table.numel()), self.bound,
                      B, self.M, H, W, self.E1, self.E2)

    def _check(self, params4, B, H, W):
        if params4.dtype != torch.float32 or tuple(params4.shape) != (B, K.c4(2 * self.M), H, W, 4):
            raise ValueError(f"params4 {tuple(params4.shape)}: expected nChw4c ({B}, {K.c4(2 * self.M)}, {H}, {W}, 4)")

    def encode(self, y4: torch.Tensor, params4: torch.Tensor):
        """-> (symbols, indexes) [B, H W M] int32 (device, position-major) and y_hat4 (nChw4c)."""
        B, _, H, W, _ = y4.shape
        self._check(params4, B, H, W)
        M = self.M
        yhat = torch.zeros((B, M, H + 4, W + 4), device=y4.device)
        sym = torch.empty((B, H * W * M), dtype=torch.int32, device=y4.device)
        idx = torch.empty_like(sym)
        # the contiguous copies stay bound to locals while the launch that reads them is enqueued (ArArgs holds raw
        # pointers only)
        y4c, p4c = y4.contiguous(), params4.contiguous()
        a = self._args(B, H, W, y4=y4c, params4=p4c, yhat=yhat, sym=sym, idx=idx)
        call("ica_ar_step", C.c_void_p(C.addressof(a)), 0, H * W, 0, stream())
        return sym, idx, K.to_nc4(yhat[:, :, 2:H + 2, 2:W + 2].contiguous())

    def decode(self, strings, params4: torch.Tensor, tab) -> torch.Tensor:
        """strings: one bitstream per image; tab: the GaussianConditional's entropy_coding.Tables -> y_hat4."""
        B, _, H, W, _ = params4.shape
        self._check(params4, B, H, W)
        if len(strings) != B:
            raise ValueError(f"{len(strings)} bitstreams for {B} images")
        M, dev = self.M, params4.device
        yhat = torch.zeros((B, M, H + 4, W + 4), device=dev)
        idx = torch.empty((B, M), dtype=torch.int32, device=dev)
        means = torch.empty((B, M), device=dev)
        sym_in = torch.empty((B, M), dtype=torch.int32, device=dev)
        idx_h = torch.empty((B, M), dtype=torch.int32).pin_memory()
        sym_h = torch.empty((B, M), dtype=torch.int32).pin_memory()
        p4c = params4.contiguous()   # alive for all H*W+1 step launches that read it through ArArgs
        bufs = [np.frombuffer(s, np.uint8) for s in strings]
        decs = (C.c_void_p * B)()
        v = C.c_void_p
        try:
            for b, buf in enumerate(bufs):
                h = C.c_void_p()
                rc = lib().ica_rans_dec_open(buf.ctypes.data_as(v), buf.size, C.byref(h))
                if rc != 0:
                    raise RuntimeError(f"context-model bitstream {b} is malformed ({rc})")
                decs[b] = h
            a = self._args(B, H, W, params4=p4c, yhat=yhat, idx=idx, sym_in=sym_in, means=means)
            pa = C.c_void_p(C.addressof(a))
            bad = C.c_int(-1)
            for p in range(H * W + 1):
                call("ica_ar_step", pa, p, min(p + 1, H * W), 1, stream())
                if p == H * W:
                    break
                idx_h.copy_(idx)   # synchronous: the rows of position p
                rc = lib().ica_rans_dec_step(decs, B, idx_h.numpy().ctypes.data_as(v), M, *tab._args(),
                                             sym_h.numpy().ctypes.data_as(v), C.byref(bad))
                if rc != 0:
                    raise RuntimeError(f"ica_rans_dec_step failed ({rc}) on image {bad.value}, position {p}: "
                                       "truncated or corrupt bitstream")
                sym_in.copy_(sym_h, non_blocking=True)
        finally:
            for b in range(B):
                if decs[b]:
                    lib().ica_rans_dec_close(decs[b])
        return K.to_nc4(yhat[:, :, 2:H + 2, 2:W + 2].contiguous())
