"""The benchmarked shapes themselves (BASELINE configs 2 and 3: 768x512 images) on the product default (x6
operands), so that every grid-size-dependent dispatch choice the bench takes is exercised under parity:
  * conv_down_x6 PT = 1 / PT = 2 (PT = 1 when the PT = 2 grid has fewer blocks than the 256 CUs: g_a.6 / the
    g_s.0 input gradient at 32x48 run 12 blocks per image, so B = 1 and B = 21 take PT = 1, B = 32 PT = 2);
  * conv_up_x6 PT = 1 when it fills the CU rounds better (32x48 inputs at B = 32: 384 -> 768 blocks);
  * the XCD-aware block remap over the >= 786k-thread grids of the 128x192 / 256x384 layers at B = 32.

Checks and stated tolerances:
  * hyper q3, B = 1, 512x768: g_a + g_s forward and the input gradient vs the CPU oracle (pinned to the
    reference layers by tests/golden) -- y / x_hat rel <= 1e-4 of the tensor max, input gradient rel <= 1e-3;
  * hyper q3, B = 1, 512x768: a 3-step attack vs the oracle -- identical branches, output_s rel <= 1e-4, noise
    rel <= 2e-3;
  * B = 32 vs images run alone (B = 1) and in a sub-batch (B = 21): y, x_hat and the input gradient BIT-EXACT
    per image (the batch-independence the speculative / compacted attack step relies on, attack.py _select);
  * branch compaction on x6 at B = 32 with mixed branches (sub-batches of 21 images): compacted == full-batch
    network step, bit for bit, over 3 steps;
  * cheng2020 q6 (config 3), B = 1, 512x768, x6: g_a + g_s forward vs the oracle (2e-4); forward and input
    gradient against float64, no worse than 2x the fp32 oracle's own error (+ 2e-6 of max).
"""
import pytest
import torch

from oracle import attack as oa
from oracle import codec
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
H, W = 512, 768


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


@pytest.fixture(scope="module")
def hyper3():
    from imagecompression_adversarial_amd.engine import CodecKernels
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * 40.0     # trained-scale latents (make_golden.py TRAJ100)
    return P, CodecKernels({k: v.to(DEV) for k, v in P.items()}, "hyper", precision="x6")


def _chain(kern, x, gout):
    from imagecompression_adversarial_amd import hip_ops as K
    y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
    xh4, ss = kern.g_s(y4, save=True)
    gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4(gout.to(DEV)), ss), sa)
    return K.from_nc4(y4, y4.shape[1] * 4), K.from_nc4(xh4, 3), K.from_nc4(gx4, 3)


def test_hyper_headline_chain_vs_oracle(hyper3):
    P, kern = hyper3
    torch.set_num_threads(16)
    x = rnd((1, 3, H, W), 41)
    xr = x.clone().requires_grad_(True)
    y_ref = codec.g_a(P, xr)
    xh_ref = codec.g_s(P, y_ref)
    gout = rnd(xh_ref.shape, 42, -1, 1)
    (xh_ref * gout).sum().backward()
    y, xh, gx = (t.cpu() for t in _chain(kern, x, gout))
    assert rel_err(y[:, :192], y_ref.detach()) < 1e-4
    assert rel_err(xh, xh_ref.detach()) < 1e-4
    assert rel_err(gx, xr.grad) < 1e-3


def test_hyper_headline_attack_vs_oracle(hyper3):
    from imagecompression_adversarial_amd.attack import attack_batch
    P, kern = hyper3
    torch.set_num_threads(16)
    x = rnd((1, 3, H, W), 43)
    res = attack_batch(kern, x.to(DEV), steps=3, eval_msssim=False, record=True)
    rec = []
    ref = oa.attack(P, x, steps=3, eval_msssim=False, record=rec)
    for i, br in enumerate(res.branches):
        assert [bool(v) for v in br] == [bool(v) for v in rec[i]["cheap"]], i
    assert rel_err(res.output_s.cpu(), ref.output_s) < 1e-4
    assert rel_err(res.noise.cpu(), ref.noise) < 2e-3


def test_hyper_headline_batch32_bitexact(hyper3):
    _, kern = hyper3
    x = rnd((32, 3, H, W), 44)
    gout = rnd((32, 3, H, W), 45, -1, 1)
    y32, xh32, gx32 = _chain(kern, x, gout)
    for idx in ([0], [31], list(range(5, 26))):   # B = 1 (PT = 1 everywhere) and B = 21 (PT = 1 below 256 blocks)
        y, xh, gx = _chain(kern, x[idx], gout[idx])
        assert torch.equal(y, y32[idx]), idx[:2]
        assert torch.equal(xh, xh32[idx]), idx[:2]
        assert torch.equal(gx, gx32[idx]), idx[:2]


def test_hyper_headline_compaction_bitexact(hyper3):
    """Images 0, 3, 6, ... start with a noise whose input distortion is above -noise (the cheap branch), the
    other 21 run the network: the compacted sub-batch step equals the full-batch step bit for bit."""
    from imagecompression_adversarial_amd.attack import AttackLoop
    _, kern = hyper3
    B = 32
    x = rnd((B, 3, H, W), 46).to(DEV)
    n0 = torch.zeros_like(x)
    n0[0::3] = rnd((11, 3, H, W), 47, -0.06, 0.06).to(DEV)
    loops = []
    for compact in (True, False):
        lp = AttackLoop(kern, x, steps=3, init_noise=n0)
        lp.compact = compact
        brs = [lp.step(i, census=True) for i in range(3)]
        loops.append((lp, brs))
    (a, ba), (b, bb) = loops
    assert ba == bb
    assert 0 < sum(ba[0]) < B, ba[0]      # mixed branches in the first step
    assert torch.equal(a.noise, b.noise) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)


def test_cheng_headline_chain_vs_oracle():
    """cheng2020's g_a + g_s at 512x768, forward vs the fp32 oracle (2e-4), and -- for the input gradient, whose
    13 leaky-ReLU residual blocks make it kink-sensitive at this size -- against a float64 evaluation of the same
    chain: the x6 path must be at least as accurate as the fp32 oracle itself, within 2x its error plus an fp32
    floor of 2e-6 of the tensor max.  (Measured: the fp32 oracle's input gradient is 2.6e-3 of max away from
    float64 at one leaky-ReLU kink (216, 648), the fp32 HIP path likewise, x6 1.3e-3; scripts/accuracy_diag.py.)"""
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd.engine_cheng import ChengKernels
    torch.set_num_threads(16)
    P = codec.perturb_params(codec.init_params("cheng2020", 6, seed=0), seed=1)
    kern = ChengKernels({k: v.to(DEV) for k, v in P.items()}, precision="x6")
    x = rnd((1, 3, H, W), 48)
    y4, sa = kern.g_a(K.to_nc4(x.to(DEV)), save=True)
    xh4, ss = kern.g_s(y4, save=True)
    got = [K.from_nc4(y4, 192).cpu(), K.from_nc4(xh4, 3).cpu()]
    gout = rnd(got[1].shape, 49, -1, 1)
    gx4 = kern.g_a_backward(kern.g_s_backward(K.to_nc4(gout.to(DEV)), ss), sa)
    got.append(K.from_nc4(gx4, 3).cpu())
    refs = {}
    for dt in (torch.float32, torch.float64):
        Pd = {k: v.to(dt) for k, v in P.items()}
        xr = x.to(dt).clone().requires_grad_(True)
        yr = codec.cheng_g_a(Pd, xr)
        xhr = codec.cheng_g_s(Pd, yr)
        xhr.backward(gout.to(dt))
        refs[dt] = (yr.detach(), xhr.detach(), xr.grad)
    assert rel_err(got[0], refs[torch.float32][0]) < 2e-4
    assert rel_err(got[1], refs[torch.float32][1]) < 2e-4
    for name, g, r32, r64 in zip(("y", "x_hat", "input grad"), got, refs[torch.float32], refs[torch.float64]):
        e6, e32 = rel_err(g, r64), rel_err(r32, r64)
        assert e6 <= 2.0 * e32 + 2e-6, (name, e6, e32)
