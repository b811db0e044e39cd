"""The fp32-accurate bf16x6 conv path (ica_conv_x6.hip; precision "x6"): every fp32 operand of the k5 s2 g_a / g_s
layers split exactly into three bf16 parts, six products per k step, fp32 accumulation / epilogues / storage.

Stated tolerances: the same as the fp32-MFMA path against the oracle (layer outputs rel <= 1e-4 of the tensor max,
the g_a + g_s input gradient rel <= 1e-3), and, against a float64 evaluation of the same chain, an error no larger
than 2x the fp32-MFMA path's own error (the accuracy claim: x6 is an fp32 computation, not a reduced-precision one).
Shapes cover partial tiles (64 x 96, 80 x 112 -> 5 x 7 latents) and the 192-channel ends (g_s.0 / the g_a.6
input-gradient read Cin = 192 in 64-channel LDS groups; g_a.6 / the g_s.0 input-gradient write 192 channels)."""
import pytest
import torch

from oracle import codec
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def _kern(P, precision):
    from imagecompression_adversarial_amd.engine import CodecKernels
    return CodecKernels({k: v.to(DEV) for k, v in P.items()}, "hyper", precision=precision)


def _chain(kern, x, gout):
    from imagecompression_adversarial_amd import hip_ops as K
    y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
    xh4, ss = kern.g_s(y4, save=True)
    gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4(gout.to(DEV)), ss), sa)
    return K.from_nc4(y4, 192).cpu(), K.from_nc4(xh4, 3).cpu(), K.from_nc4(gx4, 3).cpu()


@pytest.mark.parametrize("H,W", [(64, 96), (80, 112), (128, 192)])
def test_x6_chain_vs_oracle_and_float64(H, W):
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    kx6 = _kern(P, "x6")
    assert any(c.fwd_prec == 2 for c in kx6.ga.convs) and any(c.bwd_prec == 2 for c in kx6.gs.convs)
    k32 = _kern(P, "fp32")
    x = rnd((2, 3, H, W), 11)
    xr = x.clone().requires_grad_(True)
    y_ref = codec.g_a(P, xr)
    xh_ref = codec.g_s(P, y_ref)
    gout = rnd(xh_ref.shape, 12, -1, 1)
    (xh_ref * gout).sum().backward()
    y6, xh6, gx6 = _chain(kx6, x, gout)
    assert rel_err(y6, y_ref.detach()) < 1e-4
    assert rel_err(xh6, xh_ref.detach()) < 1e-4
    assert rel_err(gx6, xr.grad) < 1e-3
    # float64 evaluation of the same chain
    P64 = {k: v.double() for k, v in P.items()}
    x64 = x.double().requires_grad_(True)
    y64 = codec.g_a(P64, x64)
    xh64 = codec.g_s(P64, y64)
    (xh64 * gout.double()).sum().backward()
    y32, xh32, gx32 = _chain(k32, x, gout)
    for got6, got32, ref in ((y6, y32, y64), (xh6, xh32, xh64), (gx6, gx32, x64.grad)):
        e6 = float((got6.double() - ref.detach()).abs().max())
        e32 = float((got32.double() - ref.detach()).abs().max())
        # within 2x the fp32-MFMA path's own error, with an fp32-level floor of 2e-6 of the tensor max (~17 ulps):
        # the fp32 path's small-grid kernels (<= 64x64 outputs) split the tap sum over 4 waves, which can make its
        # error smaller than one sequential fp32 chain's
        assert e6 <= 2.0 * e32 + 2e-6 * float(ref.detach().abs().max()), (e6, e32)


def test_x6_attack_steps_match_fp32_path():
    """A few attack steps on x6 kernels follow the fp32-MFMA path (same branches; noise within the tolerance of
    the fp32 path vs the oracle)."""
    from imagecompression_adversarial_amd.attack import attack_batch
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    x = rnd((2, 3, 128, 128), 21).to(DEV)
    r6 = attack_batch(_kern(P, "x6"), x, steps=5, eval_msssim=False, record=True)
    r32 = attack_batch(_kern(P, "fp32"), x, steps=5, eval_msssim=False, record=True)
    assert r6.branches == r32.branches
    assert rel_err(r6.noise.cpu(), r32.noise.cpu()) < 2e-3
    assert rel_err(r6.output_s.cpu(), r32.output_s.cpu()) < 1e-4
