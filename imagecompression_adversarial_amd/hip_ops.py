"""Typed host wrappers over the C ABI (torch tensors in, torch tensors out).

Internal activation layout is nChw4c, stored as a torch tensor of shape
[N, ceil(C/4), H, W, 4] (fp32, contiguous); the logical channel count travels
with it.  All launches go on torch's current HIP stream.
"""
from __future__ import annotations

import math

import torch

from ._lib import ConvArgs, call, lib, ptr, stream

EPI_BIAS, EPI_RELU, EPI_GDN, EPI_IGDN, EPI_GDN_BWD, EPI_IGDN_BWD, EPI_LRELU, EPI_LRELU_BWD = range(8)
FILL_PLAIN, FILL_LRELU_MASK, FILL_UNSHUFFLE = range(3)
ORDER_DOWN, ORDER_UP = 0, 1
ORDER_RGB5 = 2   # ica_pack_conv_weight_x6: dense tap-row pack of a k5 conv_down with <= 3 input channels
# parity-split tensors of an x6 k5 s2 launch (ica_conv_args.layout): the input x, the output-layout tensors
LAYOUT_IN, LAYOUT_OUT = 1, 2
GDN_BETA_BOUND = float((1e-6 + 2.0 ** -36) ** 0.5)  # NonNegativeParametrizer bound (utils/ops.py:67)


# Optional per-launch timing hook used by bench.py: {tag: [(ev0, ev1), ...]}.
# When set, every tagged conv launch is bracketed by HIP events recorded on
# the current stream (the stream the kernel runs on); no synchronisation.
EVENT_HOOK = None


def _ev_begin(tag, n):
    if EVENT_HOOK is None or tag is None:
        return None
    if LAUNCH_HOOK is not None:
        last_launch()   # consume the launch record: _ev_end sees only this tag's launches
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return (tag, e0, n)


def _ev_end(h, flops=None):
    """EVENT_HOOK[tag] gets (start event, end event, images in the launch)."""
    if h is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        EVENT_HOOK.setdefault(h[0], []).append((h[1], e1, h[2]))
        if flops is not None:
            FLOPS_HOOK[h[0]] = flops / max(h[2], 1)
        if LAUNCH_HOOK is not None:
            LAUNCH_HOOK.setdefault(h[0], set()).add(last_launch())


# kernels behind each tagged launch (filled while EVENT_HOOK and LAUNCH_HOOK are set): {tag: {(kernel, threads)}}
LAUNCH_HOOK = None


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the HIP sources the library is built from (csrc/*.hip, *.h, in name order):
    the revision stamp of a PMC traffic measurement."""
    import glob
    import hashlib
    import os
    h = hashlib.sha256()
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    for f in sorted(glob.glob(os.path.join(d, "*.hip")) + glob.glob(os.path.join(d, "*.h"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def last_launch():
    """(demangled kernel name, grid size in threads) of this thread's only kernel launch since the previous call
    (ica_last_launch, which consumes the record): the names and Grid_Size that rocprofv3 reports for the same
    dispatch.  None when there was no launch, ("<N launches>", 0) when there were several (no stamp matches that)."""
    import ctypes as C
    buf = C.create_string_buffer(512)
    thr = C.c_ulonglong(0)
    n = lib().ica_last_launch(buf, 512, C.byref(thr))
    if n <= 0:
        return None
    if n > 1:
        return f"<{n} launches>", 0
    return buf.value.decode(errors="replace"), int(thr.value)


# operand precision of each tagged conv launch (filled while EVENT_HOOK is set): what actually ran, small-grid
# fp32 fallbacks of x6 layers included
PREC_HOOK = {}


_PREC_SUFFIX = {0: "fp32", 1: "bf16", 2: "x6", 3: "b1"}   # PREC_FP32, PREC_BF16, PREC_X6, PREC_B1


def _prec_note(tag, prec):
    """Record the operands a tagged launch runs on; returns the tag to time it under: a tag first seen with other
    operands (e.g. the fine-tune's fp32 train step next to its x6 inner attack) is timed as 'tag[fp32]'."""
    if EVENT_HOOK is None or tag is None:
        return tag
    first = PREC_HOOK.setdefault(tag, prec)
    if first != prec:
        tag = f"{tag}[{_PREC_SUFFIX.get(prec, prec)}]"
        PREC_HOOK.setdefault(tag, prec)
    return tag


# algorithmic FLOPs PER IMAGE of each tagged ica_conv_ex launch (filled while EVENT_HOOK is set): 2*MAC of the
# conv (a transposed conv counts the MACs of the conv it differentiates) + the GDN channel GEMM if fused
FLOPS_HOOK = {}


def _dev_check(t: torch.Tensor, name="tensor"):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a HIP device tensor (no CPU fallback on the hot path)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def c4(C: int) -> int:
    return (C + 3) // 4


def empty_nc4(N, C, H, W, device, dtype=torch.float32):
    return torch.empty((N, c4(C), H, W, 4), dtype=dtype, device=device)


def cast_nc4(x4: torch.Tensor, dtype) -> torch.Tensor:
    """fp32 <-> bf16 copy of an nChw4c tensor (the ends of the bf16 conv path) on the HIP cast kernels."""
    if x4.dtype == dtype:
        return x4
    if not x4.is_cuda or not x4.is_contiguous():
        raise RuntimeError("cast_nc4 needs a contiguous HIP tensor")
    y = torch.empty(x4.shape, dtype=dtype, device=x4.device)
    if dtype == torch.bfloat16 and x4.dtype == torch.float32:
        call("ica_cast_f32_bf16", ptr(x4), ptr(y), x4.numel(), stream())
    elif dtype == torch.float32 and x4.dtype == torch.bfloat16:
        call("ica_cast_bf16_f32", ptr(x4), ptr(y), x4.numel(), stream())
    else:
        raise RuntimeError(f"cast_nc4 {x4.dtype} -> {dtype}")
    return y


def to_nc4(x: torch.Tensor) -> torch.Tensor:
    x = x.contiguous()
    _dev_check(x, "x")
    N, C, H, W = x.shape
    y = empty_nc4(N, C, H, W, x.device)
    call("ica_nchw_to_nc4", ptr(x), ptr(y), N, C, H, W, stream())
    return y


def from_nc4(x4: torch.Tensor, C: int) -> torch.Tensor:
    _dev_check(x4, "x4")
    N, _, H, W, _ = x4.shape
    y = torch.empty((N, C, H, W), dtype=torch.float32, device=x4.device)
    call("ica_nc4_to_nchw", ptr(x4), ptr(y), N, C, H, W, stream())
    return y


# --------------------------------------------------------------------------- #
# Weight packing
# --------------------------------------------------------------------------- #
def pack_conv(w: torch.Tensor, O: int, Cc: int, KS: int, so: int, sc: int, order: int, CC: int,
              flip: bool = False, it: int = 0) -> torch.Tensor:
    """Pack a conv weight viewed as W[o][c][ky][kx] (strides so, sc; k contiguous); flip reverses the taps;
    it = 32-channel row tiles per wave (0: the library default for O)."""
    w = w.detach().contiguous()
    _dev_check(w, "weight")
    n = int(lib().ica_pack_conv_weight_size(O, Cc, KS, CC, it))
    dst = torch.empty(n, dtype=torch.float32, device=w.device)
    call("ica_pack_conv_weight", ptr(w), ptr(dst), O, Cc, KS, so, sc, CC, order, int(flip), it, stream())
    return dst


def pack_conv_bf16(w: torch.Tensor, O: int, Cc: int, KS: int, so: int, sc: int, order: int, flip: bool = False,
                   it: int = 0) -> torch.Tensor:
    """bf16 fragments (prec=1 launches): the CC=16 fp32 fragment order, each element rounded to bf16."""
    w = w.detach().contiguous()
    _dev_check(w, "weight")
    n = int(lib().ica_pack_conv_weight_bf16_size(O, Cc, KS, it))
    dst = torch.empty(n, dtype=torch.bfloat16, device=w.device)
    call("ica_pack_conv_weight_bf16", ptr(w), ptr(dst), O, Cc, KS, so, sc, order, int(flip), it, stream())
    return dst


PREC_FP32, PREC_BF16, PREC_X6 = 0, 1, 2
# bf16 operands over fp32 activations: the k3 conv_downs (cheng2020 --precision bf16) on the hi plane of the x6 pack
# (RNE bf16 of activations and weights, fp32 accumulate, fp32 tensors; GDN epilogue GEMMs on the x6 gamma' pack)
PREC_B1 = 3


def x6_it(O: int) -> int:
    """Row tiles per wave of an x6 launch (the library default for O: 4 for 128 channels, 3 for 192)."""
    return int(lib().ica_conv_it(O))


def pack_conv_x6(w: torch.Tensor, O: int, Cc: int, KS: int, so: int, sc: int, order: int, it: int) -> torch.Tensor:
    """fp32-accurate bf16x6 fragments (prec=2 launches, ica_conv_x6.hip): three bf16 planes (hi, mid, lo: an exact
    split of each weight) of the CC=16 fragment order."""
    w = w.detach().contiguous()
    _dev_check(w, "weight")
    n = int(lib().ica_pack_conv_weight_x6_size(O, Cc, KS, it))
    dst = torch.empty(n, dtype=torch.bfloat16, device=w.device)
    call("ica_pack_conv_weight_x6", ptr(w), ptr(dst), O, Cc, KS, so, sc, order, it, stream())
    return dst


def x6_ok(O: int, C: int, it: int, kind: int) -> bool:
    """Shapes ica_conv_x6_dispatch (ica_conv_x6.hip) covers for a k5 s2 launch with O output / C input channels:
    kind 0 (conv_down): C >= 16, a multiple of 16; O = 128-multiples (IT 4: bias, GDN, IGDN_BWD) or 96-multiples
    (IT 3: bias only -- the only IT 3 conv_downs, g_a.6 forward and the g_s.0 input gradient, have no epilogue);
    kind 1 (conv_up): IT 4 only (O a 128-multiple) with C = 64, 128 or a 64-multiple.  No explicit-IT (C = 192 GDN)
    launch.  Anything else keeps the fp32 pack."""
    if it != 0 or C < 16 or C % 16:
        return False
    if kind == 0:
        return O % 128 == 0 or O % 96 == 0
    return O % 128 == 0 and (C in (64, 128) or C % 64 == 0)


def conv_cc(Cin: int) -> int:
    return 4 if Cin <= 4 else 16


def pack_up3(w_view: torch.Tensor, prec: int = 0) -> torch.Tensor:
    """Fragments for conv_up3 from a [Cin][3][5][5] transposed-conv weight view (prec 1: bf16, 2: x6)."""
    w = w_view.detach().contiguous()
    _dev_check(w, "weight")
    Cin = w.shape[0]
    n = int(lib().ica_pack_up3_size(Cin))
    if prec == PREC_X6:
        dst = torch.empty(3 * n, dtype=torch.bfloat16, device=w.device)
        call("ica_pack_up3_x6", ptr(w), ptr(dst), Cin, stream())
    elif prec:
        dst = torch.empty(n, dtype=torch.bfloat16, device=w.device)
        call("ica_pack_up3_bf16", ptr(w), ptr(dst), Cin, stream())
    else:
        dst = torch.empty(n, device=w.device)
        call("ica_pack_up3", ptr(w), ptr(dst), Cin, stream())
    return dst


class PackedConv:
    """Packed fragments for one conv layer, for both its forward and its dgrad.

    kind 'conv'   : nn.Conv2d weight [Cout][Cin][k][k]   fwd = conv_down, dgrad = conv_up
    kind 'deconv' : nn.ConvTranspose2d weight [Cin][Cout][k][k]  fwd = conv_up, dgrad = conv_down
    """

    def __init__(self, weight: torch.Tensor, bias, kind: str, stride: int, prec: int = PREC_FP32,
                 it_fwd: int = 0, it_bwd: int = 0):
        """prec=PREC_BF16 packs the k5 s2 layers as bf16 fragments (fwd_prec / bwd_prec record what each pack
        is): 16-channel chunks, 4-tap groups for an RGB conv input, the Z-gather pack for 3-channel outputs.
        it_fwd / it_bwd: 32-channel row tiles per wave of the forward / input-gradient launches (0 = the library
        default; 6 for the C = 192 GDN layers of bmshj2018 q6-8, whose epilogue needs all channels in one wave; the
        bf16 path has IT = 6 kernels for those GDN / IGDN layers and their input gradients too)."""
        self.it_fwd, self.it_bwd = it_fwd, it_bwd
        if prec == PREC_X6:
            self._init_x6(weight, bias, kind, stride)
            return
        self.kind = kind
        self.fwd_prec = self.bwd_prec = PREC_FP32
        self.stride = stride
        self.KS = weight.shape[-1]
        KK = self.KS * self.KS
        if kind == "conv":
            self.Cout, self.Cin = weight.shape[0], weight.shape[1]
            # forward: o = co, c = ci
            if prec == PREC_BF16 and self.KS == 5 and stride == 2 and (self.Cin >= 16 or self.Cin <= 4):
                # an RGB input into 128 channels: the dense tap-row pack of conv_rgb5_bf16 (ica_conv_ex routes those
                # launches there); other shapes keep the tap groups / 16-channel chunks
                rgb5 = self.Cin <= 3 and self.Cout == 128 and it_fwd in (0, 4)
                self.fwd = pack_conv_bf16(weight, self.Cout, self.Cin, 5, self.Cin * KK, KK,
                                          ORDER_RGB5 if rgb5 else ORDER_DOWN, it=it_fwd)
                self.fwd_prec = PREC_BF16
            else:
                self.fwd = pack_conv(weight, self.Cout, self.Cin, self.KS, self.Cin * KK, KK, ORDER_DOWN,
                                     conv_cc(self.Cin), it=it_fwd)
            # dgrad: k5 s2 -> conv_up (o = ci, c = co); k3 s1 -> conv_down with the taps reversed
            self.bwd = None
            if self.KS == 3 and stride == 1 and self.Cout % 16 == 0:
                self.bwd = pack_conv(weight, self.Cin, self.Cout, 3, KK, self.Cin * KK, ORDER_DOWN,
                                     conv_cc(self.Cout), flip=True)
            elif self.KS == 5 and stride == 2 and self.Cout % 16 == 0:
                if self.Cin == 3:   # input-gradient of the first conv: Z-gather kernel
                    self.bwd = pack_up3(weight, prec)
                    self.bwd_prec = prec
                elif prec == PREC_BF16:
                    self.bwd = pack_conv_bf16(weight, self.Cin, self.Cout, 5, KK, self.Cin * KK, ORDER_UP, it=it_bwd)
                    self.bwd_prec = PREC_BF16
                else:
                    self.bwd = pack_conv(weight, self.Cin, self.Cout, self.KS, KK, self.Cin * KK, ORDER_UP, 16,
                                         it=it_bwd)
        elif kind == "deconv":
            self.Cin, self.Cout = weight.shape[0], weight.shape[1]
            # forward (conv_up): o = co, c = ci
            if self.Cout == 3 and self.KS == 5:
                self.fwd = pack_up3(weight, prec)
                self.fwd_prec = prec
            elif prec == PREC_BF16 and self.KS == 5:
                self.fwd = pack_conv_bf16(weight, self.Cout, self.Cin, 5, KK, self.Cout * KK, ORDER_UP, it=it_fwd)
                self.fwd_prec = PREC_BF16
            else:
                self.fwd = pack_conv(weight, self.Cout, self.Cin, self.KS, KK, self.Cout * KK, ORDER_UP, 16,
                                     it=it_fwd)
            # dgrad (conv_down, stride 2): o = ci, c = co
            if prec == PREC_BF16 and self.KS == 5 and stride == 2 and (self.Cout >= 16 or self.Cout <= 4):
                rgb5 = self.Cout <= 3 and self.Cin == 128 and it_bwd in (0, 4)
                self.bwd = pack_conv_bf16(weight, self.Cin, self.Cout, 5, self.Cout * KK, KK,
                                          ORDER_RGB5 if rgb5 else ORDER_DOWN, it=it_bwd)
                self.bwd_prec = PREC_BF16
            else:
                self.bwd = pack_conv(weight, self.Cin, self.Cout, self.KS, self.Cout * KK, KK, ORDER_DOWN,
                                     conv_cc(self.Cout), it=it_bwd)
        else:
            raise ValueError(kind)
        self.bias = None if bias is None else bias.detach().contiguous()

    def _init_x6(self, weight, bias, kind, stride):
        """PREC_X6: the k5 s2 launches run on the bf16x6 kernels: >= 16 channels on both ends (conv_down_x6 /
        conv_up_x6) and the conv_downs whose input has <= 3 channels (g_a.0 forward, g_s.6 input gradient: conv_rgb5_x6
        with the 75 (tap, channel) pairs packed densely into 5 K steps) and the 3-channel transposed-conv outputs (x6 conv_up3).  Explicit 6-tile layers
        keep the fp32 packs."""
        fp = PackedConv(weight, bias, kind, stride, PREC_FP32, self.it_fwd, self.it_bwd)
        self.__dict__.update(fp.__dict__)
        if self.KS != 5 or stride != 2:
            return
        KK = 25
        rgb_ok = lambda O, C, it: it == 0 and C <= 3 and O == 128   # noqa: E731  (conv_rgb5_x6: one 128-row block)
        if kind == "conv" and self.Cin == 3 and self.Cout % 16 == 0:    # input gradient to RGB: x6 conv_up3
            self.bwd = pack_up3(weight, PREC_X6)
            self.bwd_prec = PREC_X6
        if kind == "deconv" and self.Cout == 3 and self.Cin % 16 == 0:  # g_s.6 forward to RGB: x6 conv_up3
            self.fwd = pack_up3(weight, PREC_X6)
            self.fwd_prec = PREC_X6
        if kind == "conv":
            if rgb_ok(self.Cout, self.Cin, self.it_fwd):   # forward from the RGB image: dense tap-row K
                self.fwd = pack_conv_x6(weight, self.Cout, self.Cin, 5, self.Cin * KK, KK, ORDER_RGB5, 4)
                self.fwd_prec = PREC_X6
            elif x6_ok(self.Cout, self.Cin, self.it_fwd, 0):  # forward conv_down: o = co, c = ci
                self.fwd = pack_conv_x6(weight, self.Cout, self.Cin, 5, self.Cin * KK, KK, ORDER_DOWN, x6_it(self.Cout))
                self.fwd_prec = PREC_X6
            if self.Cin != 3 and x6_ok(self.Cin, self.Cout, self.it_bwd, 1):   # dgrad conv_up: o = ci, c = co
                self.bwd = pack_conv_x6(weight, self.Cin, self.Cout, 5, KK, self.Cin * KK, ORDER_UP, x6_it(self.Cin))
                self.bwd_prec = PREC_X6
        else:
            if self.Cout != 3 and x6_ok(self.Cout, self.Cin, self.it_fwd, 1):  # forward conv_up: o = co, c = ci
                self.fwd = pack_conv_x6(weight, self.Cout, self.Cin, 5, KK, self.Cout * KK, ORDER_UP, x6_it(self.Cout))
                self.fwd_prec = PREC_X6
            if rgb_ok(self.Cin, self.Cout, self.it_bwd):   # dgrad from the RGB-sized gradient (view [ci][co])
                self.bwd = pack_conv_x6(weight, self.Cin, self.Cout, 5, self.Cout * KK, KK, ORDER_RGB5, 4)
                self.bwd_prec = PREC_X6
            elif x6_ok(self.Cin, self.Cout, self.it_bwd, 0):    # dgrad conv_down: o = ci, c = co
                self.bwd = pack_conv_x6(weight, self.Cin, self.Cout, 5, self.Cout * KK, KK, ORDER_DOWN, x6_it(self.Cin))
                self.bwd_prec = PREC_X6


class PackedGDN:
    def __init__(self, beta: torch.Tensor, gamma: torch.Tensor):
        C = beta.shape[0]
        self.C = C
        T = C // 32
        dev = beta.device
        beta = beta.detach().contiguous()
        gamma = gamma.detach().reshape(C, C).contiguous()
        self.gp = torch.empty(T * T * 64 * 16, device=dev)
        self.gpT = torch.empty(T * T * 64 * 16, device=dev)
        self.beta = torch.empty(C, device=dev)
        call("ica_pack_gdn", ptr(gamma), ptr(beta), ptr(self.gp), ptr(self.beta), C, 0, GDN_BETA_BOUND, stream())
        call("ica_pack_gdn", ptr(gamma), ptr(beta), ptr(self.gpT), ptr(self.beta), C, 1, GDN_BETA_BOUND, stream())
        self._src = (gamma, beta)
        self.gpb = self.gpbT = None
        self.gpx = self.gpxT = None

    def x6(self):
        """Three-plane bf16 splits of gamma' / gamma'^T for prec=2 epilogues (built once, on first use)."""
        if self.gpx is None:
            n = int(lib().ica_pack_gdn_x6_size(self.C))
            self.gpx = torch.empty(n // 2, dtype=torch.bfloat16, device=self.gp.device)
            self.gpxT = torch.empty_like(self.gpx)
            call("ica_pack_gdn_x6", ptr(self.gp), ptr(self.gpx), self.C, stream())
            call("ica_pack_gdn_x6", ptr(self.gpT), ptr(self.gpxT), self.C, stream())
        return self

    def bf16(self):
        """bf16x3 hi/lo fragments of gamma' / gamma'^T for prec=1 epilogues (built once, on first use)."""
        if self.gpb is None:
            gamma, beta = self._src
            T = self.C // 32
            self.gpb = torch.empty(T * T * 2048, dtype=torch.bfloat16, device=gamma.device)
            self.gpbT = torch.empty_like(self.gpb)
            call("ica_pack_gdn_bf16", ptr(gamma), ptr(beta), ptr(self.gpb), ptr(self.beta), self.C, 0,
                 GDN_BETA_BOUND, stream())
            call("ica_pack_gdn_bf16", ptr(gamma), ptr(beta), ptr(self.gpbT), ptr(self.beta), self.C, 1,
                 GDN_BETA_BOUND, stream())
        return self


# --------------------------------------------------------------------------- #
# Convolutions
# --------------------------------------------------------------------------- #
def conv_down(x4, Cin, wp, bias, Cout, KS, S, epi=EPI_BIAS, gdn: PackedGDN | None = None, save=False,
              saved=None, out=None, tag=None, save_t=None, prec=PREC_FP32, it=0, layout=0):
    """y = conv2d(x, W, stride S, pad KS//2) (+epilogue).  Returns (y4, save_x, save_s).
    save_t: optional nChw4c output of t = dL/dn for the GDN-bwd epilogues (GDN parameter gradients).
    prec=PREC_BF16: bf16-operand launch (wp from pack_conv_bf16; goes through ica_conv_ex).
    it: the row-tile count wp was packed with (0 = library default; explicit values go through ica_conv_ex).
    layout: parity-split tensors (LAYOUT_IN: x, LAYOUT_OUT: y and the saved / output-layout tensors; x6 only)."""
    N, _, H, W, _ = x4.shape
    tag = _prec_note(tag, prec)
    if prec in (PREC_BF16, PREC_X6) or it or layout:
        return _conv_prec(x4, Cin, wp, bias, Cout, KS, S, 0, epi, gdn, save, saved, out, tag, save_t, prec, it,
                          layout)
    Ho = (H + 2 * (KS // 2) - KS) // S + 1
    Wo = (W + 2 * (KS // 2) - KS) // S + 1
    y = out if out is not None else empty_nc4(N, Cout, Ho, Wo, x4.device)
    ss = None
    if save and epi in (EPI_GDN, EPI_IGDN):
        # backward needs (y, s): y = x*s is this layer's output (kept alive anyway as the next
        # layer's input), so only s is written; the bwd epilogue recovers x = y / s.
        ss = empty_nc4(N, Cout, Ho, Wo, x4.device)
    in_x = in_s = None
    if epi in (EPI_GDN_BWD, EPI_IGDN_BWD):
        in_x, in_s = saved
    ev = _ev_begin(tag, N)
    call("ica_conv_down", ptr(x4), ptr(y), ptr(wp), ptr(bias), N, Cin, H, W, Cout, Ho, Wo, KS, S, epi,
         ptr(None if gdn is None else (gdn.gpT if epi >= EPI_GDN_BWD else gdn.gp)),
         ptr(None if gdn is None else gdn.beta), None, ptr(ss), ptr(in_x), ptr(in_s), ptr(save_t), stream())
    _ev_end(ev)
    return y, (y if ss is not None else None), ss


def conv_up(x4, Cin, wp, bias, Cout, epi=EPI_BIAS, gdn: PackedGDN | None = None, save=False, saved=None,
            out=None, tag=None, save_t=None, prec=PREC_FP32, it=0, layout=0):
    """y = conv_transpose2d(x, W, stride 2, pad 2, output_padding 1) (+epilogue).  layout: as conv_down (the
    3-channel output of conv_up3 is always row-major)."""
    N, _, H, W, _ = x4.shape
    tag = _prec_note(tag, prec)
    if (prec in (PREC_BF16, PREC_X6) or it or layout) and Cout != 3:
        return _conv_prec(x4, Cin, wp, bias, Cout, 5, 2, 1, epi, gdn, save, saved, out, tag, save_t, prec, it,
                          layout)
    Ho, Wo = 2 * H, 2 * W
    y = out if out is not None else empty_nc4(N, Cout, Ho, Wo, x4.device)
    if Cout == 3:
        if epi != EPI_BIAS:
            raise RuntimeError("conv_up to 3 channels supports the bias epilogue only")
        ev = _ev_begin(tag, N)
        call({PREC_BF16: "ica_conv_up3_bf16", PREC_X6: "ica_conv_up3_x6"}.get(prec, "ica_conv_up3"), ptr(x4), ptr(y),
             ptr(wp), ptr(bias), N, Cin, H, W, int(layout), stream())
        _ev_end(ev)
        return y, None, None
    ss = None
    if save and epi in (EPI_GDN, EPI_IGDN):
        # backward needs (y, s): y = x*s is this layer's output (kept alive anyway as the next
        # layer's input), so only s is written; the bwd epilogue recovers x = y / s.
        ss = empty_nc4(N, Cout, Ho, Wo, x4.device)
    in_x = in_s = None
    if epi in (EPI_GDN_BWD, EPI_IGDN_BWD):
        in_x, in_s = saved
    ev = _ev_begin(tag, N)
    call("ica_conv_up", ptr(x4), ptr(y), ptr(wp), ptr(bias), N, Cin, H, W, Cout, Ho, Wo, epi,
         ptr(None if gdn is None else (gdn.gpT if epi >= EPI_GDN_BWD else gdn.gp)),
         ptr(None if gdn is None else gdn.beta), None, ptr(ss), ptr(in_x), ptr(in_s), ptr(save_t), stream())
    _ev_end(ev)
    return y, (y if ss is not None else None), ss


def _conv_prec(x4, Cin, wp, bias, Cout, KS, S, kind, epi, gdn, save, saved, out, tag, save_t, prec, it, layout=0):
    """conv_down / conv_up semantics (returns (y4, save_x, save_s)) through ica_conv_ex: bf16-operand launches and
    explicit row-tile counts."""
    N, _, H, W, _ = x4.shape
    Ho, Wo = ((H + 2 * (KS // 2) - KS) // S + 1, (W + 2 * (KS // 2) - KS) // S + 1) if kind == 0 else (2 * H, 2 * W)
    dt = torch.bfloat16 if prec == PREC_BF16 else torch.float32
    ss = empty_nc4(N, Cout, Ho, Wo, x4.device, dt) if (save and epi in (EPI_GDN, EPI_IGDN)) else None
    y = conv_ex(x4, Cin, wp, bias, Cout, KS, S, kind, epi, it, gdn, save_s=ss, saved=saved, save_t=save_t, out=out,
                tag=tag, prec=prec, layout=layout)
    return y, (y if ss is not None else None), ss


def conv_ex(x4, Cin, wp, bias, Cout, KS, S, kind=0, epi=EPI_BIAS, it=0, gdn: PackedGDN | None = None, res=None,
            save_x=None, save_s=None, saved=None, save_t=None, mask=None, fill_mode=FILL_PLAIN, ps=False,
            out=None, tag=None, alg_rows=None, prec=PREC_FP32, layout=0):
    """Generic conv launch (ica_conv_ex).  kind 0: conv2d(x, W, stride S, pad KS//2); kind 1: the stride-2
    transposed conv (dgrad of a stride-2 conv).  fill_mode 2 views x ([N, Cin/16, 2H, 2W, 4]) as the
    PixelUnshuffle(2) tensor [N, Cin/4, H, W, 4] in rho order; ps stores PixelShuffle(2) of the rho-ordered
    Cout rows (y: [N, Cout/16, 2Ho, 2Wo, 4]).  save_x / save_s / save_t: caller-allocated outputs."""
    N, C4x, H, W, _ = x4.shape
    if fill_mode == FILL_UNSHUFFLE:
        if Cin != 16 * C4x:
            raise RuntimeError("unshuffled conv input: Cin must be 16 * input channel groups")
        H, W = H // 2, W // 2
    if kind == 0:
        Ho = (H + 2 * (KS // 2) - KS) // S + 1
        Wo = (W + 2 * (KS // 2) - KS) // S + 1
    else:
        Ho, Wo = 2 * H, 2 * W
    dt = torch.bfloat16 if prec == PREC_BF16 else torch.float32   # bf16 path: bf16 activations
    if out is not None:
        y = out
    elif ps:
        y = torch.empty((N, Cout // 16, 2 * Ho, 2 * Wo, 4), dtype=dt, device=x4.device)
    else:
        y = empty_nc4(N, Cout, Ho, Wo, x4.device, dt)
    in_x = in_s = None
    if saved is not None:
        in_x, in_s = saved
    gp = None
    if gdn is not None:
        if prec == PREC_BF16:
            gdn.bf16()
            gp = gdn.gpbT if epi in (EPI_GDN_BWD, EPI_IGDN_BWD) else gdn.gpb
        elif prec in (PREC_X6, PREC_B1):   # x6 epilogue GEMMs (k5 s2 and, since round 4, the k3 s1 conv_downs)
            gdn.x6()
            gp = gdn.gpxT if epi in (EPI_GDN_BWD, EPI_IGDN_BWD) else gdn.gpx
        else:   # fp32 epilogues (fp32 operands)
            gp = gdn.gpT if epi in (EPI_GDN_BWD, EPI_IGDN_BWD) else gdn.gp
    a = ConvArgs(ptr(x4), ptr(y), ptr(wp), ptr(bias), ptr(gp), ptr(None if gdn is None else gdn.beta), ptr(save_x),
                 ptr(save_s), ptr(in_x), ptr(in_s), ptr(save_t), ptr(res), ptr(mask), N, Cin, H, W, Cout, Ho, Wo,
                 kind, KS, S, epi, it, fill_mode, int(bool(ps)), int(prec), int(layout))
    import ctypes
    tag = _prec_note(tag, prec)
    ev = _ev_begin(tag, N)
    call("ica_conv_ex", ctypes.c_void_p(ctypes.addressof(a)), stream())
    if ev is not None:
        px = N * (H * W if kind == 1 else Ho * Wo)
        # alg_rows: real (non-padding) rows of a rho-ordered subpel weight (4 * C)
        cin_alg = alg_rows if (fill_mode == FILL_UNSHUFFLE and alg_rows) else Cin
        cout_alg = alg_rows if (ps and alg_rows) else Cout
        fl = 2.0 * cin_alg * cout_alg * KS * KS * px
        if epi in (EPI_GDN, EPI_IGDN, EPI_GDN_BWD, EPI_IGDN_BWD):
            fl += 2.0 * Cout * Cout * N * Ho * Wo
        _ev_end(ev, fl)
    return y


def pack_up3k3_x6(w1: torch.Tensor, ws: torch.Tensor) -> torch.Tensor:
    """Fragments of conv_up3k3_x6 (three bf16 planes) from the conv1 [Cg][3][3][3] and skip [Cg][3][1][1] weights of
    cheng2020's g_a.0 (ResidualBlockWithStride(3, N))."""
    w1, ws = w1.detach().contiguous(), ws.detach().contiguous()
    _dev_check(w1, "weight")
    _dev_check(ws, "weight")
    Cg = w1.shape[0]
    if tuple(w1.shape) != (Cg, 3, 3, 3) or tuple(ws.shape) != (Cg, 3, 1, 1):
        raise RuntimeError("pack_up3k3_x6: conv1 [Cg][3][3][3] and skip [Cg][3][1][1] weights")
    dst = torch.empty(int(lib().ica_pack_up3k3_x6_size(Cg)) // 2, dtype=torch.bfloat16, device=w1.device)
    call("ica_pack_up3k3_x6", ptr(w1), ptr(ws), ptr(dst), Cg, stream())
    return dst


def conv_up3k3_x6(g1: torch.Tensor, gs: torch.Tensor, wp: torch.Tensor, Hout: int, Wout: int, tag=None):
    """dx = conv3x3_s2^T(g1) + conv1x1_s2^T(gs) for a 3-channel input (x6 operands, one pass; ica_conv_up3k3_x6).
    g1, gs: nChw4c [N][Cg/4][H][W][4] row-major; returns dx [N][1][Hout][Wout][4]."""
    for t, nm in ((g1, "g1"), (gs, "gs")):
        _dev_check(t, nm)
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError(f"conv_up3k3_x6: {nm} must be contiguous fp32 nChw4c")
    if g1.shape != gs.shape:
        raise RuntimeError("conv_up3k3_x6: g1 and gs shapes differ")
    N, C4, H, W, _ = g1.shape
    dx = empty_nc4(N, 3, Hout, Wout, g1.device)
    ev = _ev_begin(tag, N)
    call("ica_conv_up3k3_x6", ptr(g1), ptr(gs), ptr(wp), ptr(dx), N, 4 * C4, H, W, Hout, Wout, stream())
    _ev_end(ev, 2.0 * 4 * C4 * 3 * (9 + 1) * N * H * W)
    return dx


# --------------------------------------------------------------------------- #
# Reductions / elementwise
# --------------------------------------------------------------------------- #
def blocks_per_image() -> int:
    return int(lib().ica_elem_blocks_per_image())


def reduce_rows(part: torch.Tensor, B: int, scale: float = 1.0, out=None):
    nblk = part.numel() // B
    o = out if out is not None else torch.empty(B, device=part.device)
    call("ica_reduce_rows", ptr(part), ptr(o), B, nblk, float(scale), stream())
    return o


def abs_(x: torch.Tensor) -> torch.Tensor:
    y = torch.empty_like(x)
    call("ica_abs", ptr(x), ptr(y), x.numel(), stream())
    return y


def round_(x: torch.Tensor) -> torch.Tensor:
    y = torch.empty_like(x)
    call("ica_round", ptr(x), ptr(y), x.numel(), stream())
    return y


def clamp01(x: torch.Tensor) -> torch.Tensor:
    y = torch.empty_like(x)
    call("ica_clamp01", ptr(x), ptr(y), x.numel(), stream())
    return y


def sqdiff_mean(a: torch.Tensor, b: torch.Tensor, clamp_a=False) -> torch.Tensor:
    """Per-image mean((clamp?(a) - b)^2) over the trailing dims (deterministic)."""
    B = a.shape[0]
    length = a[0].numel()
    part = torch.empty(B * blocks_per_image(), device=a.device)
    call("ica_sqdiff_partial", ptr(a.contiguous()), ptr(b.contiguous()), ptr(part), B, length, int(clamp_a), stream())
    return reduce_rows(part, B, 1.0 / length)


class PackedEB:
    NAMES = ([f"_matrix{i}" for i in range(5)] + [f"_bias{i}" for i in range(5)]
             + [f"_factor{i}" for i in range(4)] + ["quantiles"])

    def __init__(self, tensors: dict):
        import ctypes as C
        ts = [tensors[n].detach().contiguous() for n in self.NAMES]
        for t in ts:
            _dev_check(t, "entropy_bottleneck param")
        self.C = ts[-1].shape[0]
        dev = ts[0].device
        self.prm = torch.empty(self.C * 58, device=dev)
        self.med = torch.empty(self.C, device=dev)
        arr = (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
        self._keep = ts
        # the host array of device pointers is consumed synchronously by the launcher
        call("ica_pack_eb", C.cast(arr, C.c_void_p), ptr(self.prm), ptr(self.med), self.C, stream())


def eb_likelihood(z4: torch.Tensor, C: int, eb: PackedEB, training=False, qnoise4=None):
    """EntropyBottleneck forward on nc4 z: returns (z_hat4, lik4, per-image sum log lik)."""
    N, _, H, W, _ = z4.shape
    zh = torch.empty_like(z4)
    lik = torch.empty_like(z4)
    part = torch.empty(N * blocks_per_image(), device=z4.device)
    call("ica_eb_likelihood", ptr(z4), ptr(eb.prm), ptr(eb.med), ptr(qnoise4), ptr(zh), ptr(lik), ptr(part), N, C, H,
         W, int(training), stream())
    return zh, lik, reduce_rows(part, N)


def gc_likelihood(y4: torch.Tensor, C: int, scales4: torch.Tensor, means4=None, training=False, qnoise4=None):
    N, _, H, W, _ = y4.shape
    yh = torch.empty_like(y4)
    lik = torch.empty_like(y4)
    part = torch.empty(N * blocks_per_image(), device=y4.device)
    call("ica_gc_likelihood", ptr(y4), ptr(scales4), ptr(means4), ptr(qnoise4), ptr(yh), ptr(lik), ptr(part), N, C,
         H, W, int(training), stream())
    return yh, lik, reduce_rows(part, N)


def bits_to_bpp(sumlog: torch.Tensor, num_pixels: int) -> torch.Tensor:
    return sumlog / (-math.log(2) * num_pixels)


# --------------------------------------------------------------------------- #
# Training-side wrappers (ica_train.hip)
# --------------------------------------------------------------------------- #
def wgrad(Sm4, A, Lg4, Bc, KS, S, out, accumulate=False, tag=None):
    """out[a][b][ky][kx] (+)= sum Sm[n][a][p] Lg[n][b][S p + k - KS//2]  (see include/ica_hip.h).
    tag: optional EVENT_HOOK tag (algorithmic FLOPs 2 * A * B * KS^2 * small-grid pixels)."""
    N, _, Hs, Ws, _ = Sm4.shape
    _, _, Hb, Wb, _ = Lg4.shape
    if out.numel() != A * Bc * KS * KS or not out.is_contiguous():
        raise RuntimeError("wgrad: output must be a contiguous [A][B][KS][KS] tensor")
    nsplit = int(lib().ica_wgrad_nsplit(A, Bc, N * Hs * ((Ws + 31) // 32)))
    ws = torch.empty(int(lib().ica_wgrad_ws_size(A, Bc, KS, nsplit)), device=Sm4.device)
    ev = _ev_begin(tag, N)
    call("ica_wgrad", ptr(Sm4), ptr(Lg4), ptr(ws), ptr(out), N, A, Bc, Hs, Ws, Hb, Wb, KS, S, KS // 2, nsplit,
         int(accumulate), stream())
    _ev_end(ev, 2.0 * A * Bc * KS * KS * N * Hs * Ws)
    return out


def channel_sum(x4, C, out, accumulate=False):
    N, _, H, W, _ = x4.shape
    call("ica_channel_sum", ptr(x4), ptr(out), N, C, H, W, int(accumulate), stream())
    return out


def relu_bwd_(g4, y4):
    call("ica_relu_bwd", ptr(g4), ptr(y4), g4.numel(), stream())
    return g4


def abs_bwd_(g4, x4):
    call("ica_abs_bwd", ptr(g4), ptr(x4), g4.numel(), stream())
    return g4


def lrelu_bwd(g4, a4):
    """g * lrelu'(a) into a new tensor (a: the saved leaky-ReLU output)."""
    out = torch.empty_like(g4)
    call("ica_lrelu_bwd", ptr(g4), ptr(a4), ptr(out), g4.numel(), stream())
    return out


def gdn_t(g4, y4, s4, inverse):
    """t = dL/dn of a GDN / IGDN layer from g = dL/dy and its saved (y, s) (ica_gdn_t)."""
    out = torch.empty_like(g4)
    call("ica_gdn_t", ptr(g4), ptr(y4), ptr(s4), ptr(out), g4.numel(), int(bool(inverse)), stream())
    return out


def gdn_xsq(y4, s4):
    out = torch.empty_like(y4)
    call("ica_gdn_xsq", ptr(y4), ptr(s4), ptr(out), y4.numel(), stream())
    return out


def reparam_bwd(p, gprime, gout, bound, accumulate=True):
    call("ica_reparam_bwd", ptr(p.detach().contiguous()), ptr(gprime.contiguous()), ptr(gout), p.numel(),
         float(bound), int(accumulate), stream())


def bpp_grad(lik4, scale):
    g = torch.empty_like(lik4)
    call("ica_bpp_grad", ptr(lik4), ptr(g), lik4.numel(), float(scale), stream())
    return g


def gc_bwd(yt4, sigma4, gl4, C):
    N, _, H, W, _ = yt4.shape
    gy, gs = torch.empty_like(yt4), torch.empty_like(yt4)
    call("ica_gc_bwd", ptr(yt4), ptr(sigma4), ptr(gl4), ptr(gy), ptr(gs), N, C, H, W, stream())
    return gy, gs


def eb_bwd(v4, gl4, eb: PackedEB, C):
    N, _, H, W, _ = v4.shape
    gv = torch.zeros_like(v4)
    gprm = torch.empty(C * 58, device=v4.device)
    call("ica_eb_bwd", ptr(v4), ptr(gl4), ptr(eb.prm), ptr(gv), ptr(gprm), N, C, H, W, stream())
    return gv, gprm


def eb_param_scatter(gprm, raw: list, graw: list, C):
    """Accumulate the 58-per-channel effective-parameter grads into the 14 raw EB parameter grads."""
    import ctypes as Cc
    for t in list(raw) + list(graw):
        if not t.is_contiguous():
            raise RuntimeError("entropy_bottleneck params/grads must be contiguous")
    ra = (Cc.c_void_p * 14)(*[t.data_ptr() for t in raw])
    ga = (Cc.c_void_p * 14)(*[t.data_ptr() for t in graw])
    call("ica_eb_param_scatter", ptr(gprm), Cc.cast(ra, Cc.c_void_p), Cc.cast(ga, Cc.c_void_p), C, stream())


def mse_grad_(xh4, x, g4, scale):
    B, _, H, W = x.shape
    call("ica_mse_grad", ptr(xh4), ptr(x.contiguous()), ptr(g4), B, H, W, float(scale), stream())
    return g4
