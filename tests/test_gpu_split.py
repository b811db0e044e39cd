"""Parity-split storage of the inner levels of the x6 k5 s2 stacks (ica_conv_args.layout).

The layout moves pixels, not arithmetic: every kernel runs the same instruction sequence on the same values, so
each launch, the g_a + g_s chain, its input gradient and whole attack steps must be BIT-IDENTICAL to the row-major
run (compared after undoing the split on the host).  Cases cover every x6 kernel that reads or writes the split
order: conv_down (PT = 2, PT = 1 and the small-grid kernel), conv_up (PT = 2 / PT = 1 / small grid, 128- and
192-channel inputs), the RGB-input conv (GDN forward, IGDN backward) and conv_up3."""
import pytest
import torch

from oracle import codec

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def split4(x4):
    """row-major nChw4c -> parity-split: the four (y & 1, x & 1) sub-planes of (H/2) x (W/2) pixels in turn"""
    N, C4, H, W, _ = x4.shape
    return x4.view(N, C4, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 5, 2, 4, 6).contiguous().view(N, C4, H, W, 4)


def merge4(xs):
    N, C4, H, W, _ = xs.shape
    return xs.view(N, C4, 2, 2, H // 2, W // 2, 4).permute(0, 1, 4, 2, 5, 3, 6).contiguous().view(N, C4, H, W, 4)


def _gen(seed):
    return torch.Generator(device=DEV).manual_seed(seed)


def _layers(C=128):
    from imagecompression_adversarial_amd import hip_ops as K
    g = _gen(0)
    r = lambda *s: torch.rand(s, generator=g, device=DEV) * 2 - 1   # noqa: E731
    gd = K.PackedGDN(torch.ones(C, device=DEV) * 1.01, (0.1 * torch.eye(C, device=DEV) + 0.001).sqrt())
    conv = K.PackedConv(r(C, C, 5, 5) * 0.02, r(C) * 0.1, "conv", 2, K.PREC_X6)
    deconv = K.PackedConv(r(C, C, 5, 5) * 0.02, r(C) * 0.1, "deconv", 2, K.PREC_X6)
    rgb = K.PackedConv(r(C, 3, 5, 5) * 0.1, r(C) * 0.1, "conv", 2, K.PREC_X6)
    rgbd = K.PackedConv(r(C, 3, 5, 5) * 0.1, r(3) * 0.1, "deconv", 2, K.PREC_X6)
    for p in (conv, deconv, rgb, rgbd):
        assert p.fwd_prec == K.PREC_X6 and p.bwd_prec == K.PREC_X6
    return gd, conv, deconv, rgb, rgbd


def _act(B, C, H, W, seed, lo=-1.0, hi=1.0):
    from imagecompression_adversarial_amd import hip_ops as K
    return K.empty_nc4(B, C, H, W, DEV).uniform_(lo, hi, generator=_gen(seed))


def _same(a, b):
    assert a.shape == b.shape
    assert torch.equal(a, b), float((a - b).abs().max())


# (B, H, W) of the conv_down OUTPUT: PT = 2 (>= 256 blocks), PT = 1, small grid (<= 32 x 32)
DOWN_SHAPES = [(8, 64, 128), (1, 32, 64), (2, 16, 16)]


@pytest.mark.parametrize("B,Ho,Wo", DOWN_SHAPES)
@pytest.mark.parametrize("lay_out", [True, False])
def test_conv_down_split(B, Ho, Wo, lay_out):
    from imagecompression_adversarial_amd import hip_ops as K
    gd, conv, deconv, _, _ = _layers()
    C = 128
    x = _act(B, C, 2 * Ho, 2 * Wo, 1)
    sy, ss = _act(B, C, Ho, Wo, 2, 0.0, 1.0), _act(B, C, Ho, Wo, 3, 0.5, 1.0)
    lay = K.LAYOUT_IN | (K.LAYOUT_OUT if lay_out else 0)
    out = merge4 if lay_out else (lambda t: t)
    sv = split4 if lay_out else (lambda t: t)
    # bias
    y0, _, _ = K.conv_down(x, C, conv.fwd, conv.bias, C, 5, 2, K.EPI_BIAS, prec=K.PREC_X6)
    y1, _, _ = K.conv_down(split4(x), C, conv.fwd, conv.bias, C, 5, 2, K.EPI_BIAS, prec=K.PREC_X6, layout=lay)
    _same(out(y1), y0)
    # GDN forward, saving s
    y0, _, s0 = K.conv_down(x, C, conv.fwd, conv.bias, C, 5, 2, K.EPI_GDN, gd, True, prec=K.PREC_X6)
    y1, _, s1 = K.conv_down(split4(x), C, conv.fwd, conv.bias, C, 5, 2, K.EPI_GDN, gd, True, prec=K.PREC_X6,
                            layout=lay)
    _same(out(y1), y0)
    _same(out(s1), s0)
    # IGDN backward (the g_s input gradient): saved (y, s) at the output level
    y0, _, _ = K.conv_down(x, C, deconv.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gd, saved=(sy, ss), prec=K.PREC_X6)
    y1, _, _ = K.conv_down(split4(x), C, deconv.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gd, saved=(sv(sy), sv(ss)),
                           prec=K.PREC_X6, layout=lay)
    _same(out(y1), y0)


# (B, H, W) of the conv_up INPUT: PT = 2, PT = 1 (round fill), small grid; Cin 128 and 192 (64-channel groups)
UP_SHAPES = [(4, 64, 128, 128), (4, 32, 48, 128), (2, 16, 16, 128), (2, 32, 48, 192)]


@pytest.mark.parametrize("B,H,W,Cin", UP_SHAPES)
@pytest.mark.parametrize("lay_in", [True, False])
def test_conv_up_split(B, H, W, Cin, lay_in):
    from imagecompression_adversarial_amd import hip_ops as K
    gd, _, _, _, _ = _layers()
    g = _gen(5)
    C = 128
    # conv weight [Cin][C]: its input gradient is the conv_up Cin -> C; deconv weight [Cin][C]: conv_up Cin -> C
    wc = K.PackedConv((torch.rand(Cin, C, 5, 5, generator=g, device=DEV) - 0.5) * 0.04, None, "conv", 2, K.PREC_X6)
    wd = K.PackedConv((torch.rand(Cin, C, 5, 5, generator=g, device=DEV) - 0.5) * 0.04,
                      torch.rand(C, generator=g, device=DEV) * 0.1, "deconv", 2, K.PREC_X6)
    assert wc.bwd_prec == K.PREC_X6 and wd.fwd_prec == K.PREC_X6
    x = _act(B, Cin, H, W, 6)
    sy, ss = _act(B, C, 2 * H, 2 * W, 7, 0.0, 1.0), _act(B, C, 2 * H, 2 * W, 8, 0.5, 1.0)
    lay = K.LAYOUT_OUT | (K.LAYOUT_IN if lay_in else 0)
    xin = split4(x) if lay_in else x
    y0, _, _ = K.conv_up(x, Cin, wd.fwd, wd.bias, C, K.EPI_BIAS, prec=K.PREC_X6)
    y1, _, _ = K.conv_up(xin, Cin, wd.fwd, wd.bias, C, K.EPI_BIAS, prec=K.PREC_X6, layout=lay)
    _same(merge4(y1), y0)
    y0, _, s0 = K.conv_up(x, Cin, wd.fwd, wd.bias, C, K.EPI_IGDN, gd, True, prec=K.PREC_X6)
    y1, _, s1 = K.conv_up(xin, Cin, wd.fwd, wd.bias, C, K.EPI_IGDN, gd, True, prec=K.PREC_X6, layout=lay)
    _same(merge4(y1), y0)
    _same(merge4(s1), s0)
    y0, _, _ = K.conv_up(x, Cin, wc.bwd, None, C, K.EPI_GDN_BWD, gd, saved=(sy, ss), prec=K.PREC_X6)
    y1, _, _ = K.conv_up(xin, Cin, wc.bwd, None, C, K.EPI_GDN_BWD, gd, saved=(split4(sy), split4(ss)),
                         prec=K.PREC_X6, layout=lay)
    _same(merge4(y1), y0)


@pytest.mark.parametrize("B,H,W", [(2, 64, 96), (1, 48, 40)])
def test_rgb_ends_split(B, H, W):
    """The image-side ends: the RGB-input conv writes the split order (GDN forward, IGDN backward reading split
    (y, s)); conv_up3 reads it."""
    from imagecompression_adversarial_amd import hip_ops as K
    gd, _, _, rgb, rgbd = _layers()
    C = 128
    x = _act(B, 3, H, W, 9, 0.0, 1.0)
    y0, _, s0 = K.conv_down(x, 3, rgb.fwd, rgb.bias, C, 5, 2, K.EPI_GDN, gd, True, prec=K.PREC_X6)
    y1, _, s1 = K.conv_down(x, 3, rgb.fwd, rgb.bias, C, 5, 2, K.EPI_GDN, gd, True, prec=K.PREC_X6,
                            layout=K.LAYOUT_OUT)
    _same(merge4(y1), y0)
    _same(merge4(s1), s0)
    sy, ss = _act(B, C, H // 2, W // 2, 10, 0.0, 1.0), _act(B, C, H // 2, W // 2, 11, 0.5, 1.0)
    g0, _, _ = K.conv_down(x, 3, rgbd.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gd, saved=(sy, ss), prec=K.PREC_X6)
    g1, _, _ = K.conv_down(x, 3, rgbd.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gd, saved=(split4(sy), split4(ss)),
                           prec=K.PREC_X6, layout=K.LAYOUT_OUT)
    _same(merge4(g1), g0)
    h = _act(B, C, H // 2, W // 2, 12)
    for wp, bias in ((rgbd.fwd, rgbd.bias), (rgb.bwd, None)):
        o0, _, _ = K.conv_up(h, C, wp, bias, 3, K.EPI_BIAS, prec=K.PREC_X6)
        o1, _, _ = K.conv_up(split4(h), C, wp, bias, 3, K.EPI_BIAS, prec=K.PREC_X6, layout=K.LAYOUT_IN)
        _same(o1, o0)


def test_split_rejected_outside_k5s2():
    """The split order is addressed by the k5 s2 launches (plain fill, no PixelShuffle) and needs even planes: a
    k3 s1 launch (cheng2020's convs) and an odd plane are refused, not silently misread."""
    from imagecompression_adversarial_amd import hip_ops as K
    g = _gen(13)
    w3 = (torch.rand(128, 128, 3, 3, generator=g, device=DEV) - 0.5) * 0.04
    p3 = K.PackedConv(w3, None, "conv", 1, K.PREC_FP32)
    x = _act(1, 128, 32, 32, 14)
    with pytest.raises(RuntimeError):
        K.conv_ex(x, 128, p3.fwd, None, 128, 3, 1, 0, K.EPI_BIAS, layout=K.LAYOUT_IN)
    w5 = (torch.rand(128, 128, 5, 5, generator=g, device=DEV) - 0.5) * 0.04
    for prec in (K.PREC_FP32, K.PREC_X6):
        p5 = K.PackedConv(w5, None, "conv", 2, prec)
        with pytest.raises(RuntimeError):   # 17 x 17 output: an odd plane cannot be split
            K.conv_down(_act(1, 128, 34, 34, 15), 128, p5.fwd, None, 128, 5, 2, K.EPI_BIAS, prec=p5.fwd_prec,
                        layout=K.LAYOUT_OUT)


def _kern(P, precision="x6"):
    from imagecompression_adversarial_amd.engine import CodecKernels
    return CodecKernels({k: v.to(DEV) for k, v in P.items()}, "hyper", precision=precision)


ALL = (False, True, True, True, False)


@pytest.mark.parametrize("precision,H,W,expect_split", [("x6", 128, 192, ALL), ("x6", 64, 96, ALL),
                                                        ("x6", 136, 200, (False, True, True, False, False)),
                                                        ("fp32", 128, 192, ALL), ("bf16", 128, 192, ALL),
                                                        ("fp32", 64, 64, ALL)])
def test_chain_split_bitexact(precision, H, W, expect_split):
    """g_a + g_s forward and input gradient with the inner levels split == row-major, bit for bit, on every
    operand path (the fp32 64 x 64 case runs the small-grid kernels).  136 x 200 has a 17 x 25 third level: the
    engine keeps that g_a level row-major (its input gradient is refused: no exact transpose through an odd
    level); g_s, at 2x / 4x / 8x the latent sides, still splits every level."""
    from imagecompression_adversarial_amd import hip_ops as K
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    ks, kr = _kern(P, precision), _kern(P, precision)
    ks.ga.split = ks.gs.split = True   # every inner level, whatever the path's default policy
    kr.ga.split = kr.gs.split = False
    g = torch.Generator().manual_seed(3)
    x = torch.rand((2, 3, H, W), generator=g).to(DEV)
    Ho, Wo = -(-H // 16) * 16, -(-W // 16) * 16   # g_s output: 16x the latent sides
    gout = (torch.rand((2, 3, Ho, Wo), generator=g) * 2 - 1).to(DEV)
    res = []
    for k in (ks, kr):
        y4, sa = k.g_a(K.to_nc4(x), save=True)
        xh4, ss = k.g_s(y4, save=True)
        gy4 = k.g_s_backward(K.to_nc4(gout), ss)
        if H % 16:   # no exact input gradient through an odd level
            with pytest.raises(ValueError):
                k.g_a_backward(gy4, sa)
            gx4 = gy4
        else:
            gx4 = k.g_a_backward(gy4, sa)
        res.append((y4, xh4, gx4, sa.split, ss.split))
    assert res[0][3] == expect_split and res[0][4] == ALL
    assert not any(res[1][3]) and not any(res[1][4])
    for a, b in zip(res[0][:3], res[1][:3]):
        _same(a, b)


def test_attack_split_bitexact():
    """Three attack steps (x6 engine) with split inner levels == row-major: same noise bits, same branches."""
    from imagecompression_adversarial_amd.attack import attack_batch
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    ks, kr = _kern(P), _kern(P)
    kr.ga.split = kr.gs.split = False
    x = torch.rand((2, 3, 128, 128), generator=torch.Generator().manual_seed(21)).to(DEV)
    a = attack_batch(ks, x, steps=3, eval_msssim=False, record=True)
    b = attack_batch(kr, x, steps=3, eval_msssim=False, record=True)
    assert a.branches == b.branches
    _same(a.noise, b.noise)
    _same(a.output_s, b.output_s)


def test_split_policy():
    """The default per-level choice (engine._split_policy): x6 and bf16 split L1-L3, fp32 none."""
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    for precision, want in (("x6", (True, True, True)), ("bf16", (True, True, True)), ("fp32", (False,) * 3)):
        k = _kern(P, precision)
        assert k.ga.split == want and k.gs.split == want, precision
