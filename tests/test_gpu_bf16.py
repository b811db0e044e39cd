"""GPU parity of the bf16-operand conv path (BASELINE config 5).

The bf16 path computes with bf16 conv operands (fp32 accumulate) and keeps its inter-layer activations,
saved GDN tensors and gradients as bf16 nChw4c (the image-domain ends stay fp32).  Two references:
  * "emulated bf16": the CPU oracle's fp32 conv applied to bf16-rounded operands (x.bfloat16().float(),
    w.bfloat16().float()).  fp32 outputs match it to accumulation-order noise (rel-max <= 2e-5); bf16 outputs
    to their final rounding (<= 4e-3: half a bf16 ulp of the largest element plus noise).
  * the fp32 oracle itself: rel-max <= 1e-2 per layer; GDN-backward epilogues (x = y/s and s read back
    as bf16) <= 1.5e-2; <= 3e-2 through the g_a+g_s chain and its input gradient (stated tolerance of the
    bf16 path).
The ROI attack at the config-5 tile size (2048x2048) is checked by size-independent properties against the
fp32 HIP path: L-inf box and [0,1] exact, reconstruction within 3e-2, same first-step branch.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import codec
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def bf(t):
    return t.bfloat16().float()


def nc4b(K, x):
    """CPU NCHW -> device bf16 nChw4c (the bf16 path's activation format)."""
    return K.to_nc4(x.to(DEV)).bfloat16()


def unb(K, y4, C):
    """device nChw4c (bf16 or fp32) -> CPU NCHW fp32."""
    return K.from_nc4(y4.float(), C).cpu()


@pytest.fixture(scope="module")
def K():
    from imagecompression_adversarial_amd import hip_ops
    return hip_ops


@pytest.mark.parametrize("cin,cout,hw", [(128, 128, (32, 64)), (128, 192, (16, 32)), (128, 128, (10, 14)),
                                         (192, 128, (12, 20))])
def test_conv_down_bf16(K, cin, cout, hw):
    H, W = hw
    x = rnd((2, cin, H, W), 1)
    w = rnd((cout, cin, 5, 5), 2) * (1.0 / (cin * 25) ** 0.5)
    b = rnd((cout,), 3) * 0.1
    emu = F.conv2d(bf(x), bf(w), b, stride=2, padding=2)
    ref = F.conv2d(x, w, b, stride=2, padding=2)
    p = K.PackedConv(w.to(DEV), b.to(DEV), "conv", 2, K.PREC_BF16)
    assert p.fwd_prec == K.PREC_BF16 and p.fwd.dtype == torch.bfloat16
    y4, _, _ = K.conv_down(nc4b(K, x), cin, p.fwd, p.bias, cout, 5, 2, K.EPI_BIAS, prec=p.fwd_prec)
    assert y4.dtype == torch.bfloat16
    y = unb(K, y4, cout)
    assert rel_err(y, emu) < 4e-3
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("cin,cout,hw", [(192, 128, (4, 6)), (128, 128, (8, 16)), (128, 128, (5, 7))])
def test_conv_up_bf16(K, cin, cout, hw):
    H, W = hw
    x = rnd((2, cin, H, W), 4)
    w = rnd((cin, cout, 5, 5), 5) * (1.0 / (cout * 25) ** 0.5)
    b = rnd((cout,), 6) * 0.1
    emu = F.conv_transpose2d(bf(x), bf(w), b, stride=2, padding=2, output_padding=1)
    p = K.PackedConv(w.to(DEV), b.to(DEV), "deconv", 2, K.PREC_BF16)
    assert p.fwd_prec == K.PREC_BF16
    y4, _, _ = K.conv_up(nc4b(K, x), cin, p.fwd, p.bias, cout, prec=p.fwd_prec)
    assert rel_err(unb(K, y4, cout), emu) < 4e-3


def _gdn_params(C, seed):
    beta = rnd((C,), seed, 0.5, 1.5)
    gamma = (0.1 * torch.eye(C) + 0.02 * rnd((C, C), seed + 1, 0, 1)).reshape(C, C, 1, 1)
    return beta, gamma


@pytest.mark.parametrize("C,cin", [(128, 128), (192, 192), (192, 320)])
@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_fwd_epilogues_bf16(K, inverse, C, cin):
    """GDN fused into conv_down (g_a) / IGDN into conv_up (g_s): emulated-bf16 conv, then fp32 GDN.  C = 192: the
    q6-8 layers (6 row tiles per wave, parameters read from global memory), incl. g_s.0's 320-channel input."""
    H, W = 16, 24
    if not inverse and cin != C:
        pytest.skip("g_a's GDN layers take N channels")
    it = 6 if C == 192 else 0
    x = rnd((2, cin, H, W), 11)
    beta, gamma = _gdn_params(C, 12)
    gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
    w = rnd((C, cin, 5, 5) if not inverse else (cin, C, 5, 5), 14) * (1.0 / (cin * 25) ** 0.5)
    b = rnd((C,), 15) * 0.1
    if not inverse:
        p = K.PackedConv(w.to(DEV), b.to(DEV), "conv", 2, K.PREC_BF16, it_fwd=it)
        y4, _, ss = K.conv_down(nc4b(K, x), cin, p.fwd, p.bias, C, 5, 2, K.EPI_GDN, gdn, True, prec=p.fwd_prec,
                                it=it)
        pre = F.conv2d(bf(x), bf(w), b, stride=2, padding=2)
    else:
        p = K.PackedConv(w.to(DEV), b.to(DEV), "deconv", 2, K.PREC_BF16, it_fwd=it)
        y4, _, ss = K.conv_up(nc4b(K, x), cin, p.fwd, p.bias, C, K.EPI_IGDN, gdn, True, prec=p.fwd_prec, it=it)
        pre = F.conv_transpose2d(bf(x), bf(w), b, stride=2, padding=2, output_padding=1)
    out = codec.gdn(pre, beta, gamma, inverse)
    assert rel_err(unb(K, y4, C), out) < 4e-3
    be, ge = codec.gdn_effective(beta, gamma)
    norm = F.conv2d(pre ** 2, ge.reshape(C, C, 1, 1), be)
    s_ref = torch.sqrt(norm) if inverse else torch.rsqrt(norm)
    assert rel_err(unb(K, ss, C), s_ref) < 4e-3


@pytest.mark.parametrize("C,cg", [(128, 128), (192, 192), (192, 320)])
@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_bwd_epilogues_bf16(K, inverse, C, cg):
    """Input-gradient kernels: g_a conv (conv_up + GDN_BWD of the previous GDN) and g_s deconv (conv_down +
    IGDN_BWD).  Reference: autograd of (I)GDN(a) with the upstream gradient = the emulated-bf16 transposed
    conv of g (the kernel's main loop on bf16 operands).  C = 192: the q6-8 layers (6 row tiles per wave), incl.
    g_a.6's input gradient from the 320-channel latent (cg: the gradient's channels)."""
    H, W = 16, 24
    if inverse and cg != C:
        pytest.skip("g_s's IGDN-backward layers take N-channel gradients")
    it = 6 if C == 192 else 0
    beta, gamma = _gdn_params(C, 21)
    gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
    if not inverse:   # layer input a at H x W (GDN output feeds a k5 s2 conv); g at H/2 x W/2
        w = rnd((cg, C, 5, 5), 24) * (1.0 / (C * 25) ** 0.5)
        a = rnd((1, C, H, W), 23)
        g = rnd((1, cg, H // 2, W // 2), 25)
        gy = F.conv_transpose2d(bf(g), bf(w), None, stride=2, padding=2, output_padding=1)
        p = K.PackedConv(w.to(DEV), None, "conv", 2, K.PREC_BF16, it_bwd=it)
    else:             # IGDN output feeds a k5 s2 op1 deconv; g at 2H x 2W
        w = rnd((C, C, 5, 5), 24) * (1.0 / (C * 25) ** 0.5)
        a = rnd((1, C, H, W), 23)
        g = rnd((1, C, 2 * H, 2 * W), 25)
        gy = F.conv2d(bf(g), bf(w), None, stride=2, padding=2)   # dgrad of the deconv (adjoint: same w)
        p = K.PackedConv(w.to(DEV), None, "deconv", 2, K.PREC_BF16, it_bwd=it)
    ad = a.clone().requires_grad_(True)
    yprev = codec.gdn(ad, beta, gamma, inverse)
    s = (yprev / a).detach()
    yprev.backward(gy)
    saved = (nc4b(K, yprev.detach()), nc4b(K, s))
    assert p.bwd_prec == K.PREC_BF16
    if not inverse:
        out4, _, _ = K.conv_up(nc4b(K, g), cg, p.bwd, None, C, K.EPI_GDN_BWD, gdn, saved=saved, prec=p.bwd_prec,
                               it=it)
    else:
        out4, _, _ = K.conv_down(nc4b(K, g), C, p.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gdn, saved=saved,
                                 prec=p.bwd_prec, it=it)
    assert rel_err(unb(K, out4, C), ad.grad) < 1.5e-2


@pytest.mark.parametrize("q", [3, 6])
def test_chain_bf16_vs_fp32(K, q):
    """hyper q3 g_a + g_s forward and input gradient in bf16 vs the fp32 oracle (config-5 path); q6: N = 192,
    M = 320 (attack_rd.py:706-715 sweeps every quality)."""
    from imagecompression_adversarial_amd.engine import CodecKernels
    P = codec.perturb_params(codec.init_params("hyper", q, seed=0), seed=1)
    N, M = codec.model_channels("hyper", q)
    kern = CodecKernels({k: v.to(DEV) for k, v in P.items()}, "hyper", precision="bf16")
    x = rnd((2, 3, 64, 96), 7, 0.0, 1.0)
    xr = x.clone().requires_grad_(True)
    y_ref = codec.g_a(P, xr)
    out_ref = codec.g_s(P, y_ref)
    gout = rnd(out_ref.shape, 9)
    (out_ref * gout).sum().backward()
    y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
    xh4, ss = kern.g_s(y4, save=True)
    assert xh4.dtype == torch.float32 and y4.dtype == torch.bfloat16
    xh = K.from_nc4(xh4, 3).cpu()
    assert rel_err(xh, out_ref.detach()) < 3e-2
    g4 = K.to_nc4(gout.to(DEV))
    gx4 = kern.g_a_backward(kern.g_s_backward(g4, ss), sa)
    gx = K.from_nc4(gx4, 3).cpu()
    assert rel_err(gx, xr.grad) < 3e-2
    assert rel_err(unb(K, y4, M), y_ref.detach()) < 3e-2
    if q == 6:   # every C = 192 GDN layer ran its IT = 6 bf16 kernel
        assert all(c.fwd_prec == K.PREC_BF16 for c in kern.ga.convs + kern.gs.convs)
        assert all(c.bwd_prec == K.PREC_BF16 for c in kern.ga.convs + kern.gs.convs)


@pytest.mark.parametrize("q", [3, 6])
@pytest.mark.parametrize("roi", [(256, 1536, 512, 1792)])
def test_roi_attack_2048_bf16_properties(roi, q):
    """Config-5 tile (2048x2048, ROI, targeted) on the bf16 path: exact invariants, and the first steps agree
    with the fp32 HIP path within the bf16 tolerance; q6: the N = 192 transforms."""
    from imagecompression_adversarial_amd.attack import attack_batch
    from imagecompression_adversarial_amd.engine import CodecKernels
    P = codec.perturb_params(codec.init_params("hyper", q, seed=0), seed=1)
    sd = {k: v.to(DEV) for k, v in P.items()}
    k16 = CodecKernels(sd, "hyper", precision="bf16")
    k32 = CodecKernels(sd, "hyper")
    x = rnd((1, 3, 2048, 2048), 31, 0.0, 1.0).to(DEV)
    t = rnd((1, 3, 2048, 2048), 32, 0.0, 1.0).to(DEV)
    kw = dict(steps=3, noise_thr=2e-5, target=t, roi=roi, la_tar=1.0, la_bkg_in=0.01, la_bkg_out=0.5,
              eval_msssim=False)
    r16 = attack_batch(k16, x, record=True, **kw)
    r32 = attack_batch(k32, x, record=True, **kw)
    eps = 16.0 / 255.0
    assert float((r16.im_adv - x).abs().max()) <= eps + 1e-6
    assert float(r16.im_adv.min()) >= 0.0 and float(r16.im_adv.max()) <= 1.0
    assert rel_err(r16.output_s.cpu(), r32.output_s.cpu()) < 3e-2
    assert rel_err(r16.output_t.cpu(), r32.output_t.cpu()) < 3e-2
    assert [bool(v) for v in r16.branches[0]] == [bool(v) for v in r32.branches[0]]


@pytest.mark.parametrize("C", [128, 192])
@pytest.mark.parametrize("hw", [(64, 96), (20, 36)])
def test_rgb_input_conv_bf16_tap_groups(K, hw, C):
    """g_a.0 forward (conv 3->C + GDN) on bf16 4-tap x 4-channel groups vs emulated bf16 (C = 192: 6 row tiles)."""
    H, W = hw
    it = 6 if C == 192 else 0
    x = rnd((2, 3, H, W), 41, 0.0, 1.0)
    w = rnd((C, 3, 5, 5), 42) * 0.1
    b = rnd((C,), 43) * 0.1
    beta, gamma = _gdn_params(C, 44)
    gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
    p = K.PackedConv(w.to(DEV), b.to(DEV), "conv", 2, K.PREC_BF16, it_fwd=it)
    assert p.fwd_prec == K.PREC_BF16
    y4, _, _ = K.conv_down(K.to_nc4(x.to(DEV)), 3, p.fwd, p.bias, C, 5, 2, K.EPI_GDN, gdn, True, prec=p.fwd_prec,
                           it=it)
    ref = codec.gdn(F.conv2d(bf(x), bf(w), b, stride=2, padding=2), beta, gamma, False)
    assert rel_err(unb(K, y4, C), ref) < 4e-3


@pytest.mark.parametrize("C", [128, 192])
@pytest.mark.parametrize("hw", [(16, 24), (9, 13)])
def test_rgb_output_deconv_bf16(K, hw, C):
    """g_s.6 forward (deconv C->3, Z-gather kernel) and its input-gradient (conv_down 3->C on tap groups,
    IGDN_BWD epilogue) on bf16 operands vs emulated bf16 (C = 192: 6 row tiles)."""
    H, W = hw
    it = 6 if C == 192 else 0
    x = rnd((2, C, H, W), 51)
    w = rnd((C, 3, 5, 5), 52) * (1.0 / (3 * 25) ** 0.5)
    b = rnd((3,), 53) * 0.1
    p = K.PackedConv(w.to(DEV), b.to(DEV), "deconv", 2, K.PREC_BF16, it_bwd=it)
    assert p.fwd_prec == K.PREC_BF16 and p.bwd_prec == K.PREC_BF16
    y4, _, _ = K.conv_up(nc4b(K, x), C, p.fwd, p.bias, 3, prec=p.fwd_prec)
    emu = F.conv_transpose2d(bf(x), bf(w), b, stride=2, padding=2, output_padding=1)
    assert rel_err(K.from_nc4(y4, 3).cpu(), emu) < 2e-5
    # input-gradient through the preceding IGDN
    beta, gamma = _gdn_params(C, 54)
    gdn = K.PackedGDN(beta.to(DEV), gamma.to(DEV))
    a = rnd((1, C, H, W), 55)
    g = rnd((1, 3, 2 * H, 2 * W), 56)
    ad = a.clone().requires_grad_(True)
    yprev = codec.gdn(ad, beta, gamma, True)
    s = (yprev / a).detach()
    yprev.backward(F.conv2d(bf(g), bf(w), None, stride=2, padding=2))
    saved = (nc4b(K, yprev.detach()), nc4b(K, s))
    out4, _, _ = K.conv_down(K.to_nc4(g.to(DEV)), 3, p.bwd, None, C, 5, 2, K.EPI_IGDN_BWD, gdn, saved=saved,
                             prec=p.bwd_prec, it=it)
    assert rel_err(unb(K, out4, C), ad.grad) < 1.5e-2


@pytest.mark.parametrize("hw", [(32, 48), (18, 26)])
def test_first_conv_dgrad_bf16(K, hw):
    """g_a.0 input-gradient (Z-gather transposed conv 128->3) on bf16 operands vs emulated bf16."""
    H, W = hw
    C = 128
    w = rnd((C, 3, 5, 5), 61) * 0.1
    g = rnd((2, C, H, W), 62)
    p = K.PackedConv(w.to(DEV), None, "conv", 2, K.PREC_BF16)
    assert p.bwd_prec == K.PREC_BF16
    out4, _, _ = K.conv_up(nc4b(K, g), C, p.bwd, None, 3, prec=p.bwd_prec)
    emu = F.conv_transpose2d(bf(g), bf(w), None, stride=2, padding=2, output_padding=1)
    assert rel_err(K.from_nc4(out4, 3).cpu(), emu) < 2e-5
