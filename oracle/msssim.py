"""CPU fp32 restatements of the two MS-SSIM variants on the hot path.

TEST INFRASTRUCTURE (see oracle/__init__.py).

(i)  ``ms_ssim`` — pytorch_msssim.ms_ssim (third-party, unvendored; called at
     attack_rd.py:336,362, self_ensemble.py:225,228).  SURVEY Appendix A.5(i):
     separable 11-tap Gaussian (sigma 1.5), VALID conv, per-(N,C) means, ReLU on
     cs / ssim, avg_pool2d(2, padding=s%2).  Pinned against the reference's own
     independent NumPy MS-SSIM (utils/metrics_compare/msssim.py:119-178) through
     tests/golden/msssim_np.npz (tests/test_msssim_np_golden.py).
(ii) ``torch_msssim`` — utils/torch_msssim.py:26-71 (in-tree; used by
     adv_train.py:92,170).  2-D window min(H,W,11), sigma=1.5*ws/11, zero "same"
     padding, global mean per level, no ReLU, avg_pool2d(2,2).  Pinned by
     tests/golden (generated from the reference module itself).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

MS_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def gauss_1d(size=11, sigma=1.5):
    coords = torch.arange(size, dtype=torch.float32) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def _gfilter_valid(x, win):
    C = x.shape[1]
    w = win.reshape(1, 1, 1, -1).repeat(C, 1, 1, 1)
    x = F.conv2d(x, w.transpose(2, 3), groups=C)  # along H
    x = F.conv2d(x, w, groups=C)  # along W
    return x


def _ssim_pc(X, Y, win, data_range=1.0, K=(0.01, 0.03)):
    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1 = _gfilter_valid(X, win)
    mu2 = _gfilter_valid(Y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = _gfilter_valid(X * X, win) - mu1_sq
    s2 = _gfilter_valid(Y * Y, win) - mu2_sq
    s12 = _gfilter_valid(X * Y, win) - mu1_mu2
    cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
    ssim_map = ((2 * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    return torch.flatten(ssim_map, 2).mean(-1), torch.flatten(cs_map, 2).mean(-1)


def ms_ssim_per_image(X, Y, data_range=1.0, win_size=11, win_sigma=1.5):
    """pytorch_msssim.ms_ssim(..., size_average=False) -> [N] (mean over channels)."""
    assert min(X.shape[-2:]) > (win_size - 1) * 2 ** 4, "image too small for 5-level MS-SSIM"
    win = gauss_1d(win_size, win_sigma).to(X.dtype)   # float64 replays (fp32: unchanged)
    w = torch.tensor(MS_WEIGHTS, dtype=X.dtype)
    mcs = []
    for i in range(len(MS_WEIGHTS)):
        ssim_pc, cs = _ssim_pc(X, Y, win, data_range)
        if i < len(MS_WEIGHTS) - 1:
            mcs.append(torch.relu(cs))
            pad = [s % 2 for s in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=pad)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    ssim_pc = torch.relu(ssim_pc)
    stack = torch.stack(mcs + [ssim_pc], dim=0)
    val = torch.prod(stack ** w.view(-1, 1, 1), dim=0)
    return val.mean(1)


def ms_ssim(X, Y, data_range=1.0):
    """pytorch_msssim.ms_ssim(X, Y, data_range, size_average=True)."""
    return ms_ssim_per_image(X, Y, data_range).mean()


# ---- variant (ii): utils/torch_msssim.py ---------------------------------- #
def _gaussian_tm(window_size, sigma):
    g = torch.tensor([math.exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    return g / g.sum()


def _window_tm(window_size, sigma, channel):
    w1 = _gaussian_tm(window_size, sigma).unsqueeze(1)
    w2 = w1.mm(w1.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def _ssim_tm(img1, img2, max_val=1.0):
    """utils/torch_msssim.py:26-52 (note: (w, h) names are (H, W))."""
    _, c, w, h = img1.size()
    ws = min(w, h, 11)
    sigma = 1.5 * ws / 11
    window = _window_tm(ws, sigma, 3)
    p = ws // 2
    mu1 = F.conv2d(img1, window, padding=p, groups=3)
    mu2 = F.conv2d(img2, window, padding=p, groups=3)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, window, padding=p, groups=3) - mu1_sq
    s2 = F.conv2d(img2 * img2, window, padding=p, groups=3) - mu2_sq
    s12 = F.conv2d(img1 * img2, window, padding=p, groups=3) - mu1_mu2
    C1 = (0.01 * max_val) ** 2
    C2 = (0.03 * max_val) ** 2
    V1 = 2.0 * s12 + C2
    V2 = s1 + s2 + C2
    ssim_map = ((2 * mu1_mu2 + C1) * V1) / ((mu1_sq + mu2_sq + C1) * V2)
    mcs_map = V1 / V2
    return ssim_map.mean(), mcs_map.mean()


def torch_msssim(img1, img2, max_val=1.0, levels=5):
    """utils/torch_msssim.py:54-71: prod(mcs[0:4]**w[0:4]) * ssim[4]**w[4]."""
    weight = torch.tensor(MS_WEIGHTS)
    ms, mcs = [], []
    for _ in range(levels):
        s, c = _ssim_tm(img1, img2, max_val)
        ms.append(s)
        mcs.append(c)
        img1 = F.avg_pool2d(img1, kernel_size=2, stride=2)
        img2 = F.avg_pool2d(img2, kernel_size=2, stride=2)
    ms = torch.stack(ms)
    mcs = torch.stack(mcs)
    return torch.prod(mcs[: levels - 1] ** weight[: levels - 1]) * (ms[levels - 1] ** weight[levels - 1])
