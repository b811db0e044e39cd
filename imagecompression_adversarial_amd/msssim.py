"""MS-SSIM on the HIP kernels (forward + backward), both reference variants.

  mode 0 ``ms_ssim``      == pytorch_msssim.ms_ssim(X, Y, data_range, size_average)
                             (attack_rd.py:336,362; self_ensemble.py:225,228)
  mode 1 ``torch_msssim`` == utils/torch_msssim.MS_SSIM(max_val)(X, Y)
                             (utils/torch_msssim.py:54-71; adv_train.py:92,170)

``ms_ssim_per_image`` returns one value per image (mean over channels), which is
what the per-image batched attack needs; ``size_average`` means over images.
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from ._lib import call, lib, ptr, stream

MS_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def _win_valid(ws=11, sigma=1.5):
    # pytorch_msssim._fspecial_gauss_1d, float32 on the host
    coords = torch.arange(ws, dtype=torch.float32) - ws // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    return (g / g.sum()).tolist()


def _win_same(ws):
    # utils/torch_msssim.py:8-10 gaussian(window_size, 1.5*ws/11)
    sigma = 1.5 * ws / 11
    g = torch.tensor([math.exp(-(x - ws // 2) ** 2 / float(2 * sigma ** 2)) for x in range(ws)])
    return (g / g.sum()).tolist()


def _carr(vals):
    return (C.c_float * len(vals))(*vals)


def _level_geometry(H, W, ws, mode):
    pad = ws // 2 if mode == 1 else 0
    return H + 2 * pad - ws + 1, W + 2 * pad - ws + 1


class _Pyramid:
    def __init__(self, X, Y, mode, data_range):
        assert X.shape == Y.shape and X.dim() == 4
        self.mode = mode
        B, Cc, H, W = X.shape
        self.B, self.C = B, Cc
        self.P = B * Cc
        self.C1 = (0.01 * data_range) ** 2
        self.C2 = (0.03 * data_range) ** 2
        if mode == 0:
            assert min(H, W) > (11 - 1) * 2 ** 4, "Image size should be larger than 160 (pytorch_msssim)"
        self.X, self.Y, self.HW, self.wins, self.pads = [X.contiguous()], [Y.contiguous()], [(H, W)], [], []
        for lvl in range(5):
            h, w = self.HW[-1]
            if mode == 0:
                ws, win = 11, _win_valid()
            else:
                ws = min(h, w, 11)
                win = _win_same(ws)
            self.wins.append((ws, _carr(win)))
            if lvl < 4:
                ph, pw = (h % 2, w % 2) if mode == 0 else (0, 0)
                self.pads.append((ph, pw))
                ho, wo = (h + 2 * ph - 2) // 2 + 1, (w + 2 * pw - 2) // 2 + 1
                xn = torch.empty((B, Cc, ho, wo), device=X.device)
                yn = torch.empty_like(xn)
                call("ica_avgpool2", ptr(self.X[-1]), ptr(xn), self.P, h, w, ph, pw, stream())
                call("ica_avgpool2", ptr(self.Y[-1]), ptr(yn), self.P, h, w, ph, pw, stream())
                self.X.append(xn)
                self.Y.append(yn)
                self.HW.append((ho, wo))
        self.nout = [float(math.prod(_level_geometry(h, w, ws, mode))) for (h, w), (ws, _) in zip(self.HW, self.wins)]

    def level(self, l, maps=None, wgt=None):
        h, w = self.HW[l]
        ws, win = self.wins[l]
        nblk = int(lib().ica_msssim_blocks(h, w, ws, self.mode))
        part = torch.empty(self.P * nblk * 2, device=self.X[0].device)
        out = torch.empty(self.P * 2, device=self.X[0].device)
        call("ica_msssim_level", ptr(self.X[l]), ptr(self.Y[l]), self.P, h, w, C.cast(win, C.c_void_p), ws, self.mode,
             float(self.C1), float(self.C2), ptr(part), ptr(out), ptr(maps), ptr(wgt), stream())
        return out

    def forward(self):
        self.lvl = torch.stack([self.level(l) for l in range(5)])  # [5][P*2]
        G = self.C if self.mode == 0 else self.P
        val = torch.empty(self.P // G, device=self.X[0].device)
        call("ica_msssim_combine", ptr(self.lvl), self.P, G, self.mode, None, ptr(val), None,
             C.cast(_carr(self.nout), C.c_void_p), stream())
        return val

    def backward(self, dval):
        """dval: upstream gradient per combine group; returns (dX, dY) at full resolution."""
        G = self.C if self.mode == 0 else self.P
        dev = self.X[0].device
        wgt = torch.empty(5 * self.P * 2, device=dev)
        val = torch.empty(self.P // G, device=dev)
        call("ica_msssim_combine", ptr(self.lvl), self.P, G, self.mode, ptr(dval.contiguous()), ptr(val), ptr(wgt),
             C.cast(_carr(self.nout), C.c_void_p), stream())
        gX = gY = None
        for l in range(4, -1, -1):
            h, w = self.HW[l]
            ws, win = self.wins[l]
            ho, wo = _level_geometry(h, w, ws, self.mode)
            maps = torch.empty(5 * self.P * ho * wo, device=dev)
            self.level(l, maps=maps, wgt=wgt[l * self.P * 2:(l + 1) * self.P * 2])
            gXl = torch.zeros((self.B, self.C, h, w), device=dev)
            gYl = torch.zeros_like(gXl)
            if gX is not None:
                ph, pw = self.pads[l]
                call("ica_avgpool2_bwd", ptr(gX), ptr(gXl), self.P, h, w, ph, pw, stream())
                call("ica_avgpool2_bwd", ptr(gY), ptr(gYl), self.P, h, w, ph, pw, stream())
            call("ica_msssim_level_bwd", ptr(self.X[l]), ptr(self.Y[l]), ptr(maps), self.P, h, w,
                 C.cast(win, C.c_void_p), ws, self.mode, ptr(gXl), ptr(gYl), stream())
            gX, gY = gXl, gYl
        return gX, gY


def ms_ssim_per_image(X, Y, data_range=1.0):
    return _Pyramid(X, Y, 0, data_range).forward()


def ms_ssim_value_and_grad(X, Y, dval, data_range=1.0, mode=0):
    """Returns (value[groups], dX, dY) for upstream dval[groups]."""
    pyr = _Pyramid(X, Y, mode, data_range)
    v = pyr.forward()
    gX, gY = pyr.backward(dval)
    return v, gX, gY


class _MSSSIMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Y, data_range, mode):
        pyr = _Pyramid(X.detach(), Y.detach(), mode, data_range)
        v = pyr.forward()
        ctx.pyr = pyr
        return v

    @staticmethod
    def backward(ctx, g):
        gX, gY = ctx.pyr.backward(g.contiguous())
        return gX, gY, None, None


def ms_ssim(X, Y, data_range=255, size_average=True):
    """Drop-in for pytorch_msssim.ms_ssim (5 levels, win 11, sigma 1.5)."""
    v = _MSSSIMFn.apply(X, Y, float(data_range), 0)
    return v.mean() if size_average else v


def torch_msssim(X, Y, max_val=1.0):
    """Drop-in for utils/torch_msssim.MS_SSIM(max_val)(X, Y) (batch-global)."""
    return _MSSSIMFn.apply(X, Y, float(max_val), 1)[0]
