"""GPU parity of the adversarial fine-tune of the joint-prior codecs (SURVEY §8 a15 for ``-m cheng2020`` and
``-m context`` = mbt2018; reference train.py:249-366 fine-tunes whatever coder.load_model builds) against the
oracle's autograd of its restated forwards (oracle/codec.cheng_forward / mbt_forward, training=True): the gradient of
every main parameter with fixed quantisation noise, and one whole outer step (inner attack, RD backward, clip, Adam,
aux Adam) against oracle.attack.adv_train_step.  Both architectures are restated from public CompressAI: parity
unpinned beyond their primitives (oracle/codec.py header)."""
import pytest
import torch

from oracle import attack as oa
from oracle import codec as oc
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def _net(P, q, model="cheng2020"):
    from imagecompression_adversarial_amd import codec
    net = codec.cheng2020_anchor(q) if model == "cheng2020" else codec.mbt2018(q)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items() if k in sd})
    net.load_state_dict(sd)
    return net.to(DEV).train()


def _path_masks(f, model="cheng2020"):
    """The side of zero of every leaky-ReLU output of the HIP train forward (train_cheng / train_mbt .train_forward's
    dict), NCHW bool on the CPU, in the order the oracle forward calls lrelu.  cheng2020: g_a (per block conv1
    [, conv2]), h_a (4), h_s (4), entropy_parameters (2), g_s (per block conv1 [, conv2] / subpel); mbt2018: h_a (2),
    h_s (2), entropy_parameters (2)."""
    from imagecompression_adversarial_amd import hip_ops as K
    if model == "context":
        return [(K.from_nc4(f[k], f[k].shape[1] * 4) > 0).cpu() for k in ("z0", "z1", "s0", "s1", "e0", "e1")]
    acts = []
    for blk in f["sa"]:
        acts += list(blk[:2]) if len(blk) == 2 else [blk[0]]
    acts += f["za"][1:] + [f["s0"], f["s1"], f["s2"], f["s3"], f["e0"], f["e1"]]
    for blk in f["ss"]:
        acts += list(blk[:2]) if len(blk) == 2 else [blk[0]]
    return [(K.from_nc4(t, t.shape[1] * 4) > 0).cpu() for t in acts]


def _f64_with_path_kinks(P, x, ny, nz, metric, lmbda, masks, monkeypatch, model="cheng2020"):
    """Loss values and parameter gradients of the float64 oracle train forward whose every leaky ReLU takes the HIP
    path's side of zero (masks, cheng_forward call order).  Asserts that every sign disagreement is a kink: a float64
    pre-activation within KINK_REL of its tensor's max of zero.  Returns (loss dict, grads, largest disagreement)."""
    from tests.f64_replay import KINK_REL
    queue = list(masks)
    worst = [0.0]

    def lrelu_path(a):
        m = queue.pop(0)[:, :a.shape[1]]   # the nChw4c padding channels (C % 4 != 0, e.g. 426 at N = 128)
        assert m.shape == a.shape, (m.shape, a.shape)
        dis = (a.detach() > 0) != m
        if bool(dis.any()):
            r = float(a.detach().abs()[dis].max() / a.detach().abs().max())
            worst[0] = max(worst[0], r)
            assert r < KINK_REL, f"sign disagreement at {r:.1e} of max: not a kink"
        return torch.where(m, a, a * oc.LRELU_SLOPE)

    P64 = {k: v.double().requires_grad_(True) for k, v in P.items()}
    monkeypatch.setattr(oc, "lrelu", lrelu_path)
    res = oc.forward(P64, x.double(), model, training=True, noise_y=ny.double(), noise_z=nz.double())
    assert not queue, len(queue)
    out = oa.rd_loss(res, x.double(), metric, lmbda)
    out["loss"].backward()
    monkeypatch.undo()
    return out, {k: v.grad for k, v in P64.items() if v.grad is not None}, worst[0]


@pytest.mark.parametrize("model,q,metric,H,W", [
    ("cheng2020", 6, "mse", 128, 128), ("cheng2020", 6, "ms-ssim", 192, 192), ("cheng2020", 2, "mse", 128, 192),
    ("context", 3, "mse", 128, 128), ("context", 6, "ms-ssim", 192, 192)])
def test_joint_rd_backward_vs_float64(model, q, metric, H, W, monkeypatch):
    """Train-mode forward + RateDistortionLoss + backward (train_cheng.ChengTrainStep / train_mbt.MbtTrainStep; mbt2018
    q6 has M = 320) against the float64 oracle (oracle/codec.cheng_forward / mbt_forward, training=True) evaluated
    with the HIP forward's own leaky-ReLU sides: every sign
    disagreement is a kink (< KINK_REL of the tensor max), loss values at 1e-5, every main parameter's gradient within
    2e-4 of its max.  (Against the plain fp32 oracle the leaky-ReLU layers' weight gradients differ by up to
    ~4e-3 of max at these shapes: each fp32 evaluation puts a few kink pre-activations on its own side, and the
    fp32 oracle itself is 1.2e-3 off float64 on g_s.4.conv1 at q2.)"""
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd.train import LAMBS
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    if model == "cheng2020":
        from imagecompression_adversarial_amd.train_cheng import train_forward
    else:
        from imagecompression_adversarial_amd.train_mbt import train_forward
    P = oc.perturb_params(oc.init_params(model, q, seed=0), seed=1)
    N, M = oc.model_channels(model, q)
    B = 2
    x = rnd((B, 3, H, W), 5)
    ny = rnd((B, M, H // 16, W // 16), 6, -0.5, 0.5)
    nz = rnd((B, N, H // 64, W // 64), 7, -0.5, 0.5)
    lmbda = LAMBS[metric][q - 1]
    net = _net(P, q, model)
    tr = RDTrainer(net, metric, lmbda)
    got = tr.step(x.to(DEV), ny.to(DEV), nz.to(DEV))
    named = dict(net.named_parameters())
    f = train_forward(net.kernels("fp32"), lambda k: named[k].detach(), K.to_nc4(x.to(DEV)), ny.to(DEV), nz.to(DEV))
    masks = _path_masks(f, model)
    del f
    torch.cuda.synchronize()
    ref, grads, dis = _f64_with_path_kinks(P, x, ny, nz, metric, lmbda, masks, monkeypatch, model)
    for k in ("loss", "bpp_loss", "distortion_loss"):
        r = float(ref[k].detach())
        assert abs(float(got[k]) - r) <= 1e-5 * max(abs(r), 1.0), k
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


@pytest.mark.parametrize("model", ["cheng2020", "context"])
def test_joint_train_forward_values(model):
    """The module API's train-mode forward: refused while parameters require grad (no silent gradient hole: train
    through RDTrainer), values with frozen parameters (its own random quantisation noise): likelihoods in (0, 1],
    a finite x_hat of the input's shape."""
    P = oc.perturb_params(oc.init_params(model, 6, seed=0), seed=1)
    net = _net(P, 6, model)
    x = rnd((1, 3, 64, 64), 8).to(DEV)
    with pytest.raises(NotImplementedError):
        net(x)
    for p in net.parameters():
        p.requires_grad_(False)
    out = net(x)
    torch.cuda.synchronize()
    for v in out["likelihoods"].values():
        assert float(v.min()) > 0.0 and float(v.max()) <= 1.0
    assert torch.isfinite(out["x_hat"]).all() and out["x_hat"].shape == x.shape


@pytest.mark.parametrize("model", ["cheng2020", "context"])
def test_joint_adv_train_step_vs_oracle(model):
    """One whole outer step of train.py --adv for cheng2020 / mbt2018 q6 (x6 inner attack, 4 inner steps, the cheng
    attack tests' input) vs oracle.attack.adv_train_step: branch sequence step by step; the adversarial batch at the
    cheng2020 attack tolerance (2e-3 of max, leaky-ReLU kinks: tests/test_gpu_cheng.py); loss values at 1e-4; the
    first Adam step's parameter moves with 99.9 % within 1e-2 of the step size and every one within 2 steps (sign
    flips of near-zero gradients)."""
    from types import SimpleNamespace
    from imagecompression_adversarial_amd import coder
    from imagecompression_adversarial_amd.train import LAMBS, adv_step
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    q, steps, B, H, W = 6, 4, 2, 64, 64
    P = oc.perturb_params(oc.init_params(model, q, seed=0), seed=1)
    N, M = oc.model_channels(model, q)
    x = rnd((B, 3, H, W), 34)
    ny = rnd((B, M, H // 16, W // 16), 42, -0.5, 0.5)
    nz = rnd((B, N, H // 64, W // 64), 43, -0.5, 0.5)
    lr_train, metric = 1e-4, "mse"
    lmbda = LAMBS[metric][q - 1]
    net = _net(P, q, model)
    opt, aux = coder.configure_optimizers(net, SimpleNamespace(adv=True, lr_train=lr_train))
    tr = RDTrainer(net, metric, lmbda)
    args = SimpleNamespace(steps=steps, epsilon=16.0, noise=1e-4, lr_attack=0.01, att_metric="L2", clamp=True,
                           round_adv=False)
    br = []
    out, batch_adv = adv_step(net, tr, opt, aux, x.to(DEV), args, qnoise=(ny.to(DEV), nz.to(DEV)), record=br)
    torch.cuda.synchronize()
    rec = []
    Pn, ref_out, ref_aux, ref_adv = oa.adv_train_step(P, x, steps=steps, model=model, metric=metric,
                                                       lmbda=lmbda, lr_train=lr_train, noise_y=ny, noise_z=nz,
                                                       record=rec)
    assert len(br) == len(rec) == steps
    for i in range(steps):
        assert [bool(v) for v in br[i]] == [bool(v) for v in rec[i]["cheap"]], i
    assert rel_err(batch_adv.cpu(), ref_adv) < 2e-3
    for k in ("loss", "bpp_loss", "distortion_loss"):
        assert abs(float(out[k]) - ref_out[k]) <= 1e-4 * max(abs(ref_out[k]), 1.0), k
    assert abs(float(out["aux_loss"]) - ref_aux) <= 1e-4 * max(abs(ref_aux), 1.0)
    named = dict(net.named_parameters())
    worst = []
    for k, v in Pn.items():
        stp = lr_train if not k.endswith(".quantiles") else 1e-3
        d = (named[k].detach().cpu().reshape(v.shape) - v).abs() / stp
        worst.append((float(d.max()), float(torch.quantile(d.flatten().double(), 0.999)) if d.numel() > 1 else 0.0, k))
    worst.sort(reverse=True)
    print("worst parameter moves (max, p99.9 in steps):", worst[:3])
    assert worst[0][0] <= 2.0, worst[:3]
    assert max(w[1] for w in worst) <= 1e-2, sorted(worst, key=lambda w: -w[1])[:3]


@pytest.mark.parametrize("model", ["cheng2020", "context"])
def test_joint_adv_train_two_steps_clipped(model):
    """Two outer steps of train.py --adv (one Adam state across them) vs oracle.attack.adv_train_step, with lambda
    large enough that clip_grad_norm_(1.0) is active (reference train.py:360): the pre-clip norm of every main gradient
    matches the oracle's to 2e-5 (measured 2-4e-6).  The masked context taps keep their gradient, as CompressAI's
    MaskedConv2d (it masks weight.data, outside autograd): their clipped gradient must equal the oracle's (1e-3 of its
    max) and be non-zero.  (Their share of the clipped norm is ~1e-6 here, printed: the norm alone could not tell.)
    Independent y_hat / likelihood noise per step (CompressAI's two draws).  After the second Adam step the parameter moves are compared in direction (cosine) and
    median: per element, Adam's m / sqrt(v) over two clipped gradients amplifies the fp32 oracle's own leaky-ReLU-kink
    gradient noise (up to ~4e-3 of max: test_joint_rd_backward_vs_float64) where the two steps' gradients cancel."""
    from types import SimpleNamespace
    from imagecompression_adversarial_amd import coder
    from imagecompression_adversarial_amd.train import adv_step
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    q, steps, B, H, W = 6, 2, 2, 64, 64
    P = oc.perturb_params(oc.init_params(model, q, seed=0), seed=1)
    N, M = oc.model_channels(model, q)
    lr_train, metric, lmbda = 1e-4, "mse", 2.0
    net = _net(P, q, model)
    opt, aux = coder.configure_optimizers(net, SimpleNamespace(adv=True, lr_train=lr_train))
    tr = RDTrainer(net, metric, lmbda)
    # a 1e-3/255 L-inf box: the inner attack runs, but its leaky-ReLU-kink sign flips (tests/test_gpu_cheng.py) cannot
    # move the batch by more than 8e-6, so the two outer steps compare the RD step, clip and Adam, not the attack
    eps = 1e-3
    args = SimpleNamespace(steps=steps, epsilon=eps, noise=1e-4, lr_attack=0.01, att_metric="L2", clamp=True,
                           round_adv=False)
    state = {}
    P0 = {k: v.clone() for k, v in P.items()}   # the oracle's eval forwards zero P's masked taps in place
    named0 = dict(net.named_parameters())
    p0 = {k: v.detach().cpu().clone() for k, v in named0.items()}
    for o in range(2):
        x = rnd((B, 3, H, W), 60 + o)
        ny = (rnd((B, M, H // 16, W // 16), 70 + o, -0.5, 0.5), rnd((B, M, H // 16, W // 16), 80 + o, -0.5, 0.5))
        nz = rnd((B, N, H // 64, W // 64), 90 + o, -0.5, 0.5)
        out, adv = adv_step(net, tr, opt, aux, x.to(DEV), args, qnoise=(tuple(t.to(DEV) for t in ny), nz.to(DEV)))
        torch.cuda.synchronize()
        Pn, ref_out, _, ref_adv = oa.adv_train_step(P, x, steps=steps, epsilon=eps, model=model, metric=metric,
                                                     lmbda=lmbda, lr_train=lr_train, noise_y=ny, noise_z=nz,
                                                     state=state)
        gn, gr = float(out["grad_norm"]), float(ref_out["grad_norm"])
        ea = rel_err(adv.cpu(), ref_adv)
        print(f"outer step {o}: grad norm HIP {gn:.4f} oracle {gr:.4f}; adversarial batch {ea:.1e}; loss "
              f"{float(out['loss']):.6f} vs {ref_out['loss']:.6f}")
        assert gr > 1.0, "clip_grad_norm_ inactive: raise lambda"
        assert ea < 1e-4, ea
        mask = 1 - oc.context_mask(5)
        gc = named0["context_prediction.weight"].grad.detach().cpu() * mask   # clipped: the total norm is now 1
        gco = state["Q"]["context_prediction.weight"].grad.detach() * mask
        print(f"  masked-tap share of the clipped gradient {float(gc.norm()):.3e}, vs oracle {rel_err(gc, gco):.1e}")
        assert float(gco.abs().max()) > 0 and rel_err(gc, gco) < 1e-3
        assert abs(gn - gr) <= 2e-5 * gr, (gn, gr)
        for k in ("loss", "bpp_loss", "distortion_loss"):
            assert abs(float(out[k]) - ref_out[k]) <= 1e-4 * max(abs(ref_out[k]), 1.0), k
    named = named0
    mh, mo, dd = [], [], []
    for k, v in Pn.items():
        if k.endswith(".quantiles"):
            continue
        a = (named[k].detach().cpu().reshape(v.shape) - p0[k].reshape(v.shape)).flatten()
        b = (v - P0[k].reshape(v.shape)).flatten()
        mh.append(a)
        mo.append(b)
        dd.append((a - b).abs() / lr_train)
    names = [k for k in Pn if not k.endswith(".quantiles")]
    per = sorted(((float(d.max()), float(m.abs().max()) / lr_train, float(o.abs().max()) / lr_train, k)
                  for d, m, o, k in zip(dd, mh, mo, names)), reverse=True)
    print("largest move differences (max |d|, max |HIP move|, max |oracle move|, in steps):", per[:4])
    mh, mo, dd = torch.cat(mh).double(), torch.cat(mo).double(), torch.cat(dd).double()
    cos = float(mh @ mo / (mh.norm() * mo.norm()))
    med = float(dd.median())
    print(f"parameter moves after two steps: cosine {cos:.6f}, median |d| {med:.2e} steps, p99 "
          f"{float(torch.quantile(dd[:1 << 24], 0.99)):.2e}")
    assert cos > 0.999, cos
    assert med <= 1e-2, med
    w = named["context_prediction.weight"].detach().cpu()
    assert float((w * (1 - oc.context_mask(5))).abs().max()) > 0, "the masked taps must move (unmasked gradient)"
