"""GPU parity: each HIP kernel family vs the CPU oracle (fp32 torch) on seeded inputs.

Tolerances (fp32, stated): conv/deconv/GDN chains rel-max <= 2e-5 of the
tensor's max magnitude per layer, <= 1e-4 through the 8-layer fwd+bwd chain;
bounds/clamp masks and rounding bit-exact.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import codec
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda:0")


def rnd(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


@pytest.fixture(scope="module")
def K():
    from imagecompression_adversarial_amd import hip_ops
    return hip_ops


def test_layout_roundtrip(K):
    for C in (3, 8, 128, 192):
        x = rnd((2, C, 5, 7), C).to(dev())
        x4 = K.to_nc4(x)
        if C % 4:
            assert float(x4[:, -1, :, :, C % 4:].abs().max()) == 0.0
        assert torch.equal(K.from_nc4(x4, C), x)


@pytest.mark.parametrize("cin,cout,ks,s,hw", [
    (3, 128, 5, 2, (64, 96)), (128, 128, 5, 2, (32, 64)), (128, 192, 5, 2, (16, 32)),
    (192, 128, 3, 1, (8, 12)), (128, 128, 5, 2, (10, 14)), (3, 128, 5, 2, (20, 36)), (128, 192, 3, 1, (6, 10))])
def test_conv_down_vs_oracle(K, cin, cout, ks, s, hw):
    H, W = hw
    x = rnd((2, cin, H, W), 1)
    w = rnd((cout, cin, ks, ks), 2) * (1.0 / (cin * ks * ks) ** 0.5)
    b = rnd((cout,), 3) * 0.1
    ref = F.conv2d(x, w, b, stride=s, padding=ks // 2)
    p = K.PackedConv(w.to(dev()), b.to(dev()), "conv", s)
    y4, _, _ = K.conv_down(K.to_nc4(x.to(dev())), cin, p.fwd, p.bias, cout, ks, s, K.EPI_BIAS)
    y = K.from_nc4(y4, cout).cpu()
    assert y.shape == ref.shape
    assert rel_err(y, ref) < 2e-5
    yr4, _, _ = K.conv_down(K.to_nc4(x.to(dev())), cin, p.fwd, p.bias, cout, ks, s, K.EPI_RELU)
    assert rel_err(K.from_nc4(yr4, cout).cpu(), F.relu(ref)) < 2e-5


@pytest.mark.parametrize("cin,cout,hw", [(192, 128, (4, 6)), (128, 128, (8, 16)), (128, 3, (16, 24)),
                                         (128, 128, (5, 7)), (128, 3, (9, 13))])
def test_conv_up_vs_oracle(K, cin, cout, hw):
    H, W = hw
    x = rnd((2, cin, H, W), 4)
    w = rnd((cin, cout, 5, 5), 5) * (1.0 / (cout * 25) ** 0.5)
    b = rnd((cout,), 6) * 0.1
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=2, output_padding=1)
    p = K.PackedConv(w.to(dev()), b.to(dev()), "deconv", 2)
    y4, _, _ = K.conv_up(K.to_nc4(x.to(dev())), cin, p.fwd, p.bias, cout)
    y = K.from_nc4(y4, cout).cpu()
    assert y.shape == ref.shape
    assert rel_err(y, ref) < 2e-5


@pytest.mark.parametrize("cin,cout,hw", [(128, 3, (32, 48)), (128, 128, (16, 24)), (128, 192, (8, 12))])
def test_dgrad_paths(K, cin, cout, hw):
    """conv dgrad via conv_up and deconv dgrad via conv_down vs torch autograd."""
    H, W = hw
    # conv (cout <- cin) forward on [H, W]; its dgrad maps grad [H/2, W/2, cout] -> [H, W, cin]
    w = rnd((cout, cin, 5, 5), 7) * 0.05
    x = rnd((2, cin, H, W), 8).requires_grad_(True)
    y = F.conv2d(x, w, None, stride=2, padding=2)
    g = rnd(tuple(y.shape), 9)
    y.backward(g)
    if cout % 16 == 0:
        p = K.PackedConv(w.to(dev()), None, "conv", 2)
        gx4, _, _ = K.conv_up(K.to_nc4(g.to(dev())), cout, p.bwd, None, cin)
        assert rel_err(K.from_nc4(gx4, cin).cpu(), x.grad) < 2e-5
    # deconv (cin -> cout), weight [cin][cout]; dgrad maps [2H', 2W', cout] -> [H', W', cin]
    wt = rnd((cin, cout, 5, 5), 10) * 0.05
    xt = rnd((2, cin, H // 2, W // 2), 11).requires_grad_(True)
    yt = F.conv_transpose2d(xt, wt, None, stride=2, padding=2, output_padding=1)
    gt = rnd(tuple(yt.shape), 12)
    yt.backward(gt)
    p = K.PackedConv(wt.to(dev()), None, "deconv", 2)
    gx4, _, _ = K.conv_down(K.to_nc4(gt.to(dev())), cout, p.bwd, None, cin, 5, 2, K.EPI_BIAS)
    assert rel_err(K.from_nc4(gx4, cin).cpu(), xt.grad) < 2e-5


@pytest.mark.parametrize("hw", [(32, 48), (16, 24), (18, 70)])
def test_first_conv_dgrad_zgather(K, hw):
    """Input-gradient of conv 3->128 (k5 s2) through the Z-gather conv_up3 kernel."""
    H, W = hw
    w = rnd((128, 3, 5, 5), 17) * 0.1
    x = rnd((2, 3, 2 * H, 2 * W), 18).requires_grad_(True)
    y = F.conv2d(x, w, None, stride=2, padding=2)
    g = rnd(tuple(y.shape), 19)
    y.backward(g)
    p = K.PackedConv(w.to(dev()), None, "conv", 2)
    gx4, _, _ = K.conv_up(K.to_nc4(g.to(dev())), 128, p.bwd, None, 3)
    assert rel_err(K.from_nc4(gx4, 3).cpu(), x.grad) < 2e-5


@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_epilogues(K, inverse):
    """conv_down / conv_up + fused (I)GDN forward and backward vs oracle autograd."""
    C = 128
    P = codec.perturb_params(dict(zip(("a.beta", "a.gamma"), codec.gdn_init(C))), seed=5)
    beta, gamma = P["a.beta"], P["a.gamma"]
    gd = K.PackedGDN(beta.to(dev()), gamma.to(dev()))
    epi_f = K.EPI_IGDN if inverse else K.EPI_GDN
    epi_b = K.EPI_IGDN_BWD if inverse else K.EPI_GDN_BWD
    # forward through conv_down (k5 s2)
    x = rnd((2, C, 24, 40), 13)
    w = rnd((C, C, 5, 5), 14) * 0.02
    b = rnd((C,), 15) * 0.1
    pre = F.conv2d(x, w, b, stride=2, padding=2).requires_grad_(True)
    ref = codec.gdn(pre, beta, gamma, inverse)
    p = K.PackedConv(w.to(dev()), b.to(dev()), "conv", 2)
    y4, sx, ss = K.conv_down(K.to_nc4(x.to(dev())), C, p.fwd, p.bias, C, 5, 2, epi_f, gd, save=True)
    assert rel_err(K.from_nc4(y4, C).cpu(), ref.detach()) < 2e-5
    assert sx is y4  # saved pair is (GDN output y, s); backward recovers x = y / s
    # s = n^(-1/2) (GDN) or n^(1/2) (IGDN): y / s reproduces the pre-normalisation x
    assert rel_err((K.from_nc4(y4, C) / K.from_nc4(ss, C)).cpu(), pre.detach()) < 2e-5
    # backward epilogue: feed g through conv_up of an identity-free weight and compare with
    # autograd of gdn(pre) driven by the same upstream gradient
    g_up = rnd(tuple(ref.shape), 16)
    ref.backward(g_up)
    # conv_up with a delta weight would be identity-like; instead test via conv_down of a
    # 1x1-equivalent: run the epilogue on conv_up(dy) where dy is constructed so conv_up(dy) == g_up
    # -> use the dgrad of a deconv: conv_down(gt) with W chosen as a 5x5 delta at centre (k=2,2)
    wdel = torch.zeros(C, C, 5, 5)
    wdel[torch.arange(C), torch.arange(C), 2, 2] = 1.0
    # conv_down with stride 2 of an upsampled-by-2 grid picks the even samples: build gt on 2x grid
    gt = torch.zeros(2, C, 2 * g_up.shape[2], 2 * g_up.shape[3])
    gt[:, :, ::2, ::2] = g_up
    pd = K.PackedConv(wdel.to(dev()), None, "deconv", 2)  # dgrad = conv_down with W[o=ci][c=co]
    dx4, _, _ = K.conv_down(K.to_nc4(gt.to(dev())), C, pd.bwd, None, C, 5, 2, epi_b, gd, saved=(sx, ss))
    assert rel_err(K.from_nc4(dx4, C).cpu(), pre.grad) < 5e-5
    # same epilogue on conv_up: conv_up(x, W) with centre-delta on a half-res grid places x at even outputs
    half = torch.zeros(2, C, g_up.shape[2] // 2, g_up.shape[3] // 2)
    if g_up.shape[2] % 2 == 0 and g_up.shape[3] % 2 == 0:
        pu = K.PackedConv(wdel.to(dev()), None, "conv", 2)  # dgrad = conv_up with W[o=ci][c=co]
        gsub = torch.zeros_like(g_up)
        gsub[:, :, ::2, ::2] = g_up[:, :, ::2, ::2]
        half = g_up[:, :, ::2, ::2].contiguous()
        dx4u, _, _ = K.conv_up(K.to_nc4(half.to(dev())), C, pu.bwd, None, C, epi_b, gd, saved=(sx, ss))
        pre2 = pre.detach().clone().requires_grad_(True)
        codec.gdn(pre2, beta, gamma, inverse).backward(gsub)
        assert rel_err(K.from_nc4(dx4u, C).cpu(), pre2.grad) < 5e-5
