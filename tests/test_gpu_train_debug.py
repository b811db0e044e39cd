"""GPU parity of the adversarial fine-tune of the reference's "debug" model, ae_onelayer(N=3, M=192)
(anchors/model.py:8-33; reference train.py:249-366 fine-tunes whatever coder.load_model builds, coder.py:88-101), on
train_debug.DebugTrainStep, against the oracle's autograd of its restated forward (oracle/codec.debug_forward,
training=True) and oracle.attack.adv_train_step.  The hyperprior half is mbt2018's (CompressAI MeanScaleHyperprior),
restated from public CompressAI: parity unpinned beyond its primitives (oracle/codec.py header)."""
import pytest
import torch

from oracle import attack as oa
from oracle import codec as oc
from tests.conftest import rel_err
from tests.test_gpu_train_joint import _f64_with_path_kinks, rnd

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _net(P):
    from imagecompression_adversarial_amd.anchors import model as am
    net = am.init_model("debug", 3, "mse", pretrained=False)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items() if k in sd})
    net.load_state_dict(sd)
    return net.to(DEV).train()


@pytest.mark.parametrize("metric,H,W", [("mse", 64, 64), ("mse", 64, 128), ("ms-ssim", 192, 192)])
def test_debug_rd_backward_vs_float64(metric, H, W, monkeypatch):
    """Train-mode forward + RateDistortionLoss + backward of ae_onelayer against the float64 oracle evaluated with the
    HIP forward's own leaky-ReLU sides (h_a.0 / h_a.2 / h_s.0 / h_s.2; every sign disagreement a kink): loss values at
    1e-5, every main parameter's gradient (g_a / g_s, the N = 3 hyper layers, the EntropyBottleneck's filters)
    within 2e-4 of its max."""
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd.train import LAMBS
    from imagecompression_adversarial_amd.train_debug import train_forward
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    P = oc.perturb_params(oc.init_params("debug", 3, seed=0), seed=1)
    N, M = oc.model_channels("debug", 3)
    assert (N, M) == (3, 192)
    B = 2
    x = rnd((B, 3, H, W), 5)
    ny = rnd((B, M, H, W), 6, -0.5, 0.5)             # y is full resolution (stride-1 g_a)
    nz = rnd((B, N, H // 4, W // 4), 7, -0.5, 0.5)
    lmbda = LAMBS[metric][2]
    net = _net(P)
    tr = RDTrainer(net, metric, lmbda)
    got = tr.step(x.to(DEV), ny.to(DEV), nz.to(DEV))
    named = dict(net.named_parameters())
    f = train_forward(net.kernels("fp32"), lambda k: named[k].detach(), K.to_nc4(x.to(DEV)), ny.to(DEV), nz.to(DEV))
    masks = [(K.from_nc4(f[k], f[k].shape[1] * 4) > 0).cpu() for k in ("z0", "z1", "s0", "s1")]
    del f
    torch.cuda.synchronize()
    ref, grads, dis = _f64_with_path_kinks(P, x, ny, nz, metric, lmbda, masks, monkeypatch, "debug")
    for k in ("loss", "bpp_loss", "distortion_loss"):
        r = float(ref[k].detach())
        assert abs(float(got[k]) - r) <= 1e-5 * max(abs(r), 1.0), (k, float(got[k]), r)
    worst, checked = [], 0
    for k, g64 in grads.items():
        if k.endswith(".quantiles"):
            continue
        g = named[k].grad
        assert g is not None, k
        worst.append((rel_err(g.detach().cpu().double().reshape(g64.shape), g64), k))
        checked += 1
    worst.sort(reverse=True)
    print(f"largest sign disagreement {dis:.1e} of max; worst gradients:", [(f"{e:.1e}", k) for e, k in worst[:4]])
    assert checked == len(tr.names), (checked, len(tr.names))
    assert worst[0][0] < 2e-4, worst[:5]


def test_debug_train_forward_values():
    """The module API's train-mode forward: refused while parameters require grad (train through RDTrainer), values
    with frozen parameters: likelihoods in (0, 1], x_hat = g_s(y) equal to the eval forward's (no quantisation on the
    reconstruction path, anchors/model.py:30)."""
    P = oc.perturb_params(oc.init_params("debug", 3, seed=0), seed=1)
    net = _net(P)
    x = rnd((1, 3, 64, 64), 8).to(DEV)
    with pytest.raises(NotImplementedError):
        net(x)
    for p in net.parameters():
        p.requires_grad_(False)
    out = net(x)
    net.eval()
    ev = net(x)
    torch.cuda.synchronize()
    for v in out["likelihoods"].values():
        assert float(v.min()) > 0.0 and float(v.max()) <= 1.0
    assert out["x_hat"].shape == x.shape
    assert torch.equal(out["x_hat"], ev["x_hat"])


def test_debug_adv_train_two_steps():
    """Two outer steps of train.py --adv on ae_onelayer (one Adam state across them; the inner attack's random start
    drawn from the global CPU RNG on both sides, attack_rd.py:493-494) vs oracle.attack.adv_train_step.  The attack
    box is 1e-3/255 (the debug attack is ill-conditioned at fp32: tests/test_gpu_debug.py), so the two outer steps
    compare the RD step, clip_grad_norm_ and Adam: pre-clip gradient norm to 2e-5, loss values to 1e-4, and after
    the second Adam step the parameter moves in direction (cosine > 0.999) and median (1e-2 of a step)."""
    from types import SimpleNamespace
    from imagecompression_adversarial_amd import coder
    from imagecompression_adversarial_amd.train import LAMBS, adv_step
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    steps, B, H, W = 2, 2, 64, 64
    P = oc.perturb_params(oc.init_params("debug", 3, seed=0), seed=1)
    N, M = oc.model_channels("debug", 3)
    lr_train, metric = 1e-4, "mse"
    lmbda = LAMBS[metric][2]
    net = _net(P)
    opt, aux = coder.configure_optimizers(net, SimpleNamespace(adv=True, lr_train=lr_train))
    tr = RDTrainer(net, metric, lmbda)
    eps = 1e-3
    args = SimpleNamespace(steps=steps, epsilon=eps, noise=1e-4, lr_attack=0.01, att_metric="L2", clamp=True,
                           round_adv=False)
    state = {}
    named = dict(net.named_parameters())
    p0 = {k: v.detach().cpu().clone() for k, v in named.items()}
    for o in range(2):
        x = rnd((B, 3, H, W), 60 + o)
        ny = rnd((B, M, H, W), 70 + o, -0.5, 0.5)
        nz = rnd((B, N, H // 4, W // 4), 90 + o, -0.5, 0.5)
        torch.manual_seed(100 + o)
        out, adv = adv_step(net, tr, opt, aux, x.to(DEV), args, qnoise=(ny.to(DEV), nz.to(DEV)))
        torch.cuda.synchronize()
        torch.manual_seed(100 + o)
        Pn, ref_out, ref_aux, ref_adv = oa.adv_train_step(P, x, steps=steps, epsilon=eps, model="debug",
                                                           metric=metric, lmbda=lmbda, lr_train=lr_train, noise_y=ny,
                                                           noise_z=nz, state=state)
        gn, gr = float(out["grad_norm"]), float(ref_out["grad_norm"])
        ea = float((adv.cpu() - ref_adv).abs().max())
        print(f"outer step {o}: grad norm HIP {gn:.4f} oracle {gr:.4f}; adversarial batch max |d| {ea:.1e}; loss "
              f"{float(out['loss']):.6f} vs {ref_out['loss']:.6f}; aux {float(out['aux_loss']):.4f} vs {ref_aux:.4f}")
        assert ea <= 2 * eps / 255.0 + 1e-6, ea   # the two box corners, plus fp32 rounding of im_s + noise
        assert abs(gn - gr) <= 2e-5 * gr, (gn, gr)
        for k in ("loss", "bpp_loss", "distortion_loss"):
            assert abs(float(out[k]) - ref_out[k]) <= 1e-4 * max(abs(ref_out[k]), 1.0), k
        assert abs(float(out["aux_loss"]) - ref_aux) <= 1e-4 * max(abs(ref_aux), 1.0)
    mh, mo, dd = [], [], []
    for k, v in Pn.items():
        if k.endswith(".quantiles"):
            continue
        a = (named[k].detach().cpu().reshape(v.shape) - p0[k].reshape(v.shape)).flatten()
        b = (v - P[k].reshape(v.shape)).flatten()
        mh.append(a)
        mo.append(b)
        dd.append((a - b).abs() / lr_train)
    mh, mo, dd = torch.cat(mh).double(), torch.cat(mo).double(), torch.cat(dd).double()
    cos = float(mh @ mo / (mh.norm() * mo.norm()))
    med = float(dd.median())
    print(f"parameter moves after two steps: cosine {cos:.6f}, median |d| {med:.2e} steps, max {float(dd.max()):.2e}")
    assert cos > 0.999, cos
    assert med <= 1e-2, med
