"""GPU parity of the adversarial fine-tune backward against the oracle's autograd:
train-mode forward with fixed quantisation noise, RateDistortionLoss (train.py:37-96), and the gradient
of every main parameter of bmshj2018-hyperprior / -factorized (CompressAI names)."""
import numpy as np
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


def _net(model, P):
    from imagecompression_adversarial_amd import codec
    net = codec.bmshj2018_hyperprior(3) if model == "hyper" else codec.bmshj2018_factorized(3)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items() if k in sd})
    net.load_state_dict(sd)
    return net.to(DEV).train()


def _oracle_grads(P, x, model, metric, lmbda, ny, nz):
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    res = oc.forward(Pr, x, model, training=True, noise_y=ny, noise_z=nz)
    out = oa.rd_loss(res, x, metric, lmbda)
    out["loss"].backward()
    return out, {k: v.grad for k, v in Pr.items() if v.grad is not None}


@pytest.mark.parametrize("model,metric,H,W", [("hyper", "mse", 128, 128), ("hyper", "ms-ssim", 192, 192),
                                              ("factorized", "mse", 128, 192)])
def test_rd_backward_vs_oracle(model, metric, H, W):
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    P = oc.perturb_params(oc.init_params(model, 3, seed=0), seed=1)
    B = 2
    x = rnd((B, 3, H, W), 5)
    N, M = 128, 192
    ny = rnd((B, M, H // 16, W // 16), 6, -0.5, 0.5)
    nz = rnd((B, N, H // 64, W // 64), 7, -0.5, 0.5) if model == "hyper" else None
    lmbda = 0.0130 if metric == "mse" else 8.73
    net = _net(model, P)
    tr = RDTrainer(net, metric, lmbda)
    got = tr.step(x.to(DEV), ny.to(DEV), None if nz is None else nz.to(DEV))
    torch.cuda.synchronize()
    ref, grads = _oracle_grads(P, x, model, metric, lmbda, ny, nz)
    for k in ("loss", "bpp_loss", "distortion_loss"):
        assert abs(float(got[k]) - float(ref[k])) <= 1e-4 * max(abs(float(ref[k])), 1.0), k
    named = dict(net.named_parameters())
    checked = 0
    worst = []
    for k, gref in grads.items():
        if k.endswith(".quantiles"):
            continue
        g = named[k].grad
        assert g is not None, k
        e = rel_err(g.detach().cpu().reshape(gref.shape), gref)
        worst.append((e, k))
        checked += 1
    worst.sort(reverse=True)
    assert checked == len(tr.names), (checked, len(tr.names))
    # fp32 with different reduction orders; entropy-model grads go through exp/tanh chains
    assert worst[0][0] < 2e-3, worst[:5]


def test_rd_backward_batch_sum_property():
    """Size-independent property at a bench-like shape: grads of a batch == mean of the two half-batch grads
    (the loss is a batch mean), which is exactly what the data-parallel all-reduce relies on."""
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    P = oc.perturb_params(oc.init_params("hyper", 3, seed=0), seed=1)
    net = _net("hyper", P)
    tr = RDTrainer(net, "mse", 0.0130)
    B, H, W = 4, 256, 256
    x = rnd((B, 3, H, W), 9).to(DEV)
    ny = rnd((B, 192, H // 16, W // 16), 10, -0.5, 0.5).to(DEV)
    nz = rnd((B, 128, H // 64, W // 64), 11, -0.5, 0.5).to(DEV)
    tr.step(x, ny, nz)
    full = tr.flat_grad.clone()
    tr.step(x[:2], ny[:2], nz[:2])
    a = tr.flat_grad.clone()
    tr.step(x[2:], ny[2:], nz[2:])
    b = tr.flat_grad.clone()
    torch.cuda.synchronize()
    assert rel_err(((a + b) / 2).cpu(), full.cpu()) < 1e-3
    assert torch.isfinite(full).all()
