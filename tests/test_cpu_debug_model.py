"""CPU checks of the "debug" model (ae_onelayer, anchors/model.py:8-33): the oracle restatement against plain
torch ops, the module's CompressAI state-dict surface against the oracle's synthetic init, the factory's
no-pretrained rule (anchors/model.py:62), and the oracle attack's debug semantics (attack_rd.py:493-494, 514-515)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import attack as oa
from oracle import codec as oc


def test_oracle_debug_transforms_are_one_conv_each():
    P = oc.init_params("debug", 3, seed=0)
    assert oc.model_channels("debug", 1) == oc.model_channels("debug", 8) == (3, 192)
    x = torch.rand(1, 3, 12, 20)
    y = oc.debug_g_a(P, x)
    assert torch.allclose(y, F.conv2d(x, P["g_a.0.weight"], P["g_a.0.bias"], padding=1))
    xh = oc.debug_g_s(P, y)
    assert xh.shape == x.shape
    assert torch.allclose(xh, F.conv_transpose2d(y, P["g_s.0.weight"], P["g_s.0.bias"], padding=1))
    r = oc.forward(P, x[:, :, :, :16], "debug")
    assert torch.equal(r["x_hat"], oc.debug_g_s(P, oc.debug_g_a(P, x[:, :, :, :16])))   # x_hat = g_s(y), no round
    assert r["likelihoods"]["z"].shape == (1, 3, 3, 4)


def test_debug_module_state_dict_matches_oracle():
    from imagecompression_adversarial_amd.anchors import model as am
    net = am.init_model("debug", 5, "mse", pretrained=False)
    sd = net.state_dict()
    P = oc.init_params("debug", 5, seed=0)
    for k, v in P.items():
        assert k in sd, k
        assert sd[k].numel() == v.numel(), k
    with pytest.raises(AssertionError):
        am.init_model("debug", 3, "mse", pretrained=True)


def test_oracle_debug_attack_unclamped_random_start():
    P = oc.init_params("debug", 3, seed=0)
    x = torch.rand(1, 3, 16, 16)
    x[:, :, :4] = 1.0
    torch.manual_seed(3)
    start = torch.empty(x.shape).uniform_(-1e-2, 1e-2)
    torch.manual_seed(3)
    r0 = oa.attack(P, x, steps=3, noise_thr=1e-4, model="debug", eval_msssim=False)
    r = oa.attack(P, x, steps=3, noise_thr=1e-4, model="debug", eval_msssim=False, init_noise=start)
    assert torch.equal(r0.noise, r.noise)       # the start is U(-sqrt(noise), sqrt(noise)) from the global RNG
    assert float((x + r.noise.clamp(-16 / 255, 16 / 255)).max()) > 1.0   # nothing clamps the input
    assert float(r.im_in.max()) > 1.0


def test_debug_model_trainer_accepted():
    """RDTrainer takes the debug model since round 6 (train_debug.DebugTrainStep; reference train.py:249-366 fine-tunes
    whatever coder.load_model builds): the flat gradient buffer covers every main parameter, the EB quantiles stay
    with the aux optimiser."""
    from imagecompression_adversarial_amd.anchors import model as am
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    net = am.init_model("debug", 3, "mse", pretrained=False)
    tr = RDTrainer(net, "mse", 0.0483)
    named = dict(net.named_parameters())
    assert set(tr.names) == {k for k in named if not k.endswith(".quantiles")}
    assert tr.flat_grad.numel() == sum(named[k].numel() for k in tr.names)
    assert "g_a.0.weight" in tr.names and "g_s.0.weight" in tr.names and "h_s.0.weight" in tr.names
