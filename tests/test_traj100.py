"""Long-horizon (100-step, config 1) attack parity against trajectories of the REFERENCE's own layers.

Fixture: tests/golden/traj100.npz (tests/golden/make_golden.py traj100): attack_rd.attack_ restated on
/root/reference's utils/ops.py Low_bound/Up_bound + GDN and anchors/utils.py conv/deconv, torch Adam and
MultiStepLR, 100 steps, one 256x256 image, hyper q1 widths, default -noise / -lr_attack / -e.  Two weight
scales: "t100a" (10 branch flips into the cheap branch) and "t100b" (hovers at the budget: 54 cheap steps).

Checks and stated tolerances:
  * the lr table (MultiStepLR stepped every steps//3, milestones 1/2/3 -> drops at i = 0, 33, 66) equals the
    reference's, value for value;
  * CPU oracle: identical branch sequence over all 100 steps, loss_i rel <= 1e-4, final noise within NOISE_MAX /
    NOISE_P999 (another CPU's fp32 reduction order, amplified by Adam; 0 on the generating platform), eval metrics
    rel <= 1e-3;
  * HIP path (-m gpu), on BOTH operand paths (fp32 MFMA and the default x6 = fp32-accurate bf16x6): pre-eval
    latents within 1e-5 of max|y| with rounding differences only at near-ties, the target equal to the reference
    decoder of the GPU's rounded latents within 1e-4; then, from the reference's target, an identical branch
    sequence for at least DIV_MIN[(tag, precision)] steps -- the step each path achieves, measured on MI355X and
    asserted as the bound (the branch at loss_i ~ -noise is discontinuous, so an fp32 reduction-order difference
    may flip a late step; the assertion message carries both branch strings); loss_i per step rel <= 1e-3 while
    the sequences agree; up to the first divergence the noise itself against the reference's
    (tests/golden/traj100_snap.npz, same run): at the snapshot steps within NOISE_MAX / NOISE_P999 (the spread of
    18 fp32 re-evaluations of the reference algorithm, x1.25), and per step the fingerprints sum|noise| /
    sum noise^2 / <noise, pattern> rel <= 1e-2 of their scale; the final noise (when all 100 agree) within the
    same bounds (for scale: the same algorithm in fp64 diverges from the fp32 reference's branch sequence at step
    32 / 40 and ends O(1) away); final mse_in within
    10 % of the reference's, VI within 1 dB, |noise_c| <= eps and im_in in [0, 1] exactly.
Measured on MI355X (round 3): both paths keep the reference's branch sequence for all 100 steps on both runs.
x6 ends further from the reference noise on t100b (max 4.8e-2, p99.9 1.3e-3; fp32 1.6e-2 / 3.9e-4) although its
per-step network gradient is as accurate as the fp32 ones: at the reference's own step-9 / 24 / 49 states the
gradient is within 4.3-4.8e-6 of max of a float64 evaluation for x6, 3.6e-6 for the fp32 HIP path and 2.8-3.3e-6
for the fp32 CPU oracle (scripts/accuracy_diag.py t100b) -- the difference is Adam's amplification of fp32-level
gradient noise where |g| ~ eps, which the fp64 run of the same algorithm shows at full strength.
"""
import os

import numpy as np
import pytest
import torch

from tests.conftest import REPO

FIX = os.path.join(REPO, "tests", "golden", "traj100.npz")
SNAP = os.path.join(REPO, "tests", "golden", "traj100_snap.npz")
TAGS = ("t100a", "t100b")
# Noise bounds, relative to max|noise_ref|: what fp32 rounding alone does to this trajectory.  18 fp32 re-evaluations
# of the reference algorithm on the CPU oracle (1 thread instead of 8, weights or the image moved by +-1 ulp;
# scripts/traj100_spread.py -> profiles/r03/traj100_spread.txt) keep all 100 branches but end up to 4.77e-2 (max)
# and 1.41e-2 (99.9th percentile) away from the reference's final noise; the bounds are 1.25x those.
NOISE_MAX, NOISE_P999 = 6e-2, 1.8e-2
# first step whose branch differs from the reference's (100 = none), as achieved on MI355X by each path
DIV_MIN = {("t100a", "fp32"): 100, ("t100b", "fp32"): 100, ("t100a", "x6"): 100, ("t100b", "x6"): 100}
# the HIP paths' own p99.9 bound, ~2-3x the largest p99.9 each path measured on MI355X over the snapshot steps and
# the final noise (rounds 3-4: t100a fp32 3.0e-5, x6 8.3e-5; t100b fp32 4.4e-4, x6 2.3e-3): the calibrated CPU
# bound NOISE_P999 above is ~10x looser than any path needs, so a several-fold loss of accuracy would pass it
P999_PATH = {("t100a", "fp32"): 1e-4, ("t100a", "x6"): 2e-4, ("t100b", "fp32"): 1e-3, ("t100b", "x6"): 5e-3}


@pytest.fixture(scope="module")
def t100():
    return np.load(FIX)


def _fingerprint_pattern():
    # tests/golden/make_golden.py fingerprint_pattern: U(-1, 1) from torch.Generator seed 977, the image's shape
    g = torch.Generator().manual_seed(977)
    return (torch.rand((1, 3, 256, 256), generator=g) * 2.0 - 1.0).numpy()


def _params(scale):
    from oracle import codec
    P = codec.perturb_params(codec.init_params("hyper", 1, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * float(scale)
    return P


def _image():
    g = torch.Generator().manual_seed(101)
    return torch.rand((1, 3, 256, 256), generator=g)


def test_lr_table_matches_reference(t100):
    from imagecompression_adversarial_amd.attack import _lr_table
    for tag in TAGS:
        assert _lr_table(100, 0.01) == [float(v) for v in t100[f"{tag}_lr"]]
    lr = _lr_table(100, 0.01)
    assert lr[0] == 0.01 and lr[1] == lr[33] and lr[34] == lr[66] and lr[67] == lr[99]
    assert lr[1] != lr[34] != lr[67]


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_traj100_vs_reference(t100, tag):
    from oracle import attack as oatt
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    P = _params(t100[f"{tag}_scale"])
    rec = []
    r = oatt.attack(P, _image(), steps=100, record=rec, eval_msssim=False)
    br = [int(bool(d["cheap"][0])) for d in rec]
    assert br == [int(v) for v in t100[f"{tag}_branch"]]
    li = np.array([float(d["loss_i"][0]) for d in rec])
    assert np.abs(li - t100[f"{tag}_loss_i"]).max() <= 1e-4 * np.abs(t100[f"{tag}_loss_i"]).max()
    # same-platform runs agree to ~1e-6; another CPU (ISA / thread split of the conv reductions) reorders fp32 sums
    # and Adam's 1/sqrt(v) amplifies that where |g| ~ eps, so the bound is the calibrated fp32 spread (NOISE_MAX / NOISE_P999)
    mx, p999 = _noise_close(r.noise.numpy(), t100[f"{tag}_noise"])
    assert mx <= NOISE_MAX and p999 <= NOISE_P999, (mx, p999)
    assert abs(float(r.eval.mse_in[0]) - float(t100[f"{tag}_mse_in"])) <= 1e-3 * float(t100[f"{tag}_mse_in"])
    assert abs(float(r.eval.mse_out[0]) - float(t100[f"{tag}_mse_out"])) <= 1e-3 * float(t100[f"{tag}_mse_out"])


def _noise_close(got, ref):
    d = np.abs(got - ref) / np.abs(ref).max()
    return float(d.max()), float(np.quantile(d, 0.999))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "x6"])
@pytest.mark.parametrize("tag", TAGS)
def test_hip_traj100_vs_reference(t100, tag, precision):
    from imagecompression_adversarial_amd.attack import AttackLoop, evaluate
    from imagecompression_adversarial_amd.engine import CodecKernels
    dev = torch.device("cuda:0")
    P = _params(t100[f"{tag}_scale"])
    kern = CodecKernels({k: v.to(dev) for k, v in P.items()}, "hyper", precision=precision)
    xs = _image().to(dev)
    loop = AttackLoop(kern, xs, steps=100)
    os_ref = t100[f"{tag}_output_s"]
    # pre-eval target clamp(g_s(round(g_a(x)))): round() is discontinuous, so a latent within fp32 noise of a
    # half-integer may round the other way (each such latent moves a ~30x30-pixel footprint).  Checked in
    # pieces: y vs the oracle (pinned to the reference layers) within 1e-5 of max|y|, every rounding
    # difference at a near-tie, and output_s == the oracle decoder applied to the GPU's rounded latents.
    from imagecompression_adversarial_amd import hip_ops as K
    from oracle import codec
    y4, _ = kern.g_a(K.to_nc4(xs))
    y_gpu = K.from_nc4(y4, 192).cpu()
    with torch.no_grad():
        y_ref = codec.g_a(P, _image())
        tol = 1e-5 * float(y_ref.abs().max())
        assert float((y_gpu - y_ref).abs().max()) <= tol
        flip = torch.round(y_gpu) != torch.round(y_ref)
        near = ((y_ref - torch.floor(y_ref)) - 0.5).abs() <= tol
        assert bool((~flip | near).all())
        os_gpu_round = torch.clamp(codec.g_s(P, torch.round(y_gpu)), 0, 1)
    assert float((loop.output_s.cpu() - os_gpu_round).abs().max()) <= 1e-4
    print(f"{tag}: {int(flip.sum())} latents round differently (near-ties)")
    if not bool(flip.any()):
        assert np.abs(loop.output_s.cpu().numpy() - os_ref).max() <= 1e-4
    # the trajectory is then run from the reference's own target, so it isolates the attack step
    loop.output_s.copy_(torch.from_numpy(os_ref).to(dev))
    eps = np.float32(16 / 255.0)
    snap = np.load(SNAP)
    snap_steps = [int(v) for v in snap["snap_steps"]]
    pat = torch.from_numpy(_fingerprint_pattern()).to(dev).double()
    br, li, fp, snaps = [], [], [], {}
    for i in range(100):
        br.append(loop.step(i, record_im_in=True, census=True)[0])
        li.append(float(loop.loss_i[0]))
        n = loop.noise.double()
        fp.append([float(n.abs().sum()), float((n * n).sum()), float((n * pat).sum())])
        if i in snap_steps:
            snaps[i] = loop.noise.cpu().numpy()
        im_in = loop.im_in
        assert float((im_in - xs).abs().max()) <= eps * (1 + 1e-6)
        assert float(im_in.min()) >= 0.0 and float(im_in.max()) <= 1.0
    ref_br = [int(v) for v in t100[f"{tag}_branch"]]
    div = next((i for i in range(100) if br[i] != ref_br[i]), 100)
    bstr = "".join("c" if b else "E" for b in br)
    rstr = "".join("c" if b else "E" for b in ref_br)
    print(f"{tag}/{precision}: branch sequence identical for {div}/100 steps")
    assert div >= DIV_MIN[(tag, precision)], (div, f"hip {bstr}", f"ref {rstr}")
    ref_li = t100[f"{tag}_loss_i"]
    for i in range(div):
        assert abs(li[i] - ref_li[i]) <= 1e-3 * max(abs(ref_li[i]), 1e-12), (i, li[i], ref_li[i])
    # the noise itself up to the first divergence: snapshots element-wise, every step through its fingerprints
    ref_fp = snap[f"{tag}_fp"]
    fp = np.array(fp)
    scale = np.abs(ref_fp[:div]).max(0) if div else np.ones(3)
    for i in range(div):
        rel = np.abs(fp[i] - ref_fp[i]) / scale
        assert (rel <= 1e-2).all(), (i, fp[i].tolist(), ref_fp[i].tolist())
    for k, i in enumerate(snap_steps):
        if i < div:
            mx, p999 = _noise_close(snaps[i], snap[f"{tag}_snap"][k])
            print(f"{tag}/{precision}: noise after step {i}: rel diff max {mx:.2e}, p99.9 {p999:.2e}")
            assert mx <= NOISE_MAX and p999 <= min(NOISE_P999, P999_PATH[(tag, precision)]), (i, mx, p999)
    if div == 100:
        # Adam's 1/sqrt(v) amplifies fp32 ordering differences where |g| ~ eps (NOISE_MAX / NOISE_P999 above; for
        # scale: the SAME algorithm in fp64 leaves the fp32 reference's branch sequence at step 32 (t100a) / 40
        # (t100b) and ends O(1) away, max 1.3 / 1.5, p99.9 0.95 / 0.99 of max|noise|)
        mx, p999 = _noise_close(loop.noise.cpu().numpy(), t100[f"{tag}_noise"])
        print(f"{tag}/{precision}: final noise rel diff max {mx:.2e}, p99.9 {p999:.2e}")
        assert mx <= NOISE_MAX and p999 <= min(NOISE_P999, P999_PATH[(tag, precision)]), (mx, p999)
    res = evaluate(kern, loop.im_in, loop.im_s, loop.output_s, msssim=False)
    mse_in, mse_out = float(res[3][0]), float(res[4][0])
    assert abs(mse_in - float(t100[f"{tag}_mse_in"])) <= 0.1 * float(t100[f"{tag}_mse_in"])
    vi = 10 * np.log10(mse_out / mse_in)
    assert abs(vi - float(t100[f"{tag}_vi"])) <= 1.0, (vi, float(t100[f"{tag}_vi"]))
