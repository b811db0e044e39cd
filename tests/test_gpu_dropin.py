"""GPU tests of the drop-in surface: CompressAI-compatible model objects (net(x), net.g_a /
net.g_s autograd, entropy modules), the utils mirror (ops bounds, torch_msssim.MS_SSIM) and
the attack_rd CLI, against the CPU oracle / golden vectors."""
import numpy as np
import pytest
import torch

from oracle import codec as oc
from oracle import msssim as oms
from tests.conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


@pytest.fixture(scope="module")
def net_and_params():
    from imagecompression_adversarial_amd import codec
    P = oc.perturb_params(oc.init_params("hyper", 3, seed=0), seed=1)
    net = codec.bmshj2018_hyperprior(3)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items()})
    net.load_state_dict(sd)
    return net.to(DEV).eval(), P


def test_model_forward_vs_oracle(net_and_params):
    net, P = net_and_params
    x = rnd((2, 3, 128, 192), 3)
    with torch.no_grad():
        out = net(x.to(DEV))
    ref = oc.forward(P, x)
    assert rel_err(out["x_hat"].cpu(), ref["x_hat"]) < 1e-4
    for k in ("y", "z"):
        assert rel_err(out["likelihoods"][k].cpu(), ref["likelihoods"][k]) < 1e-3
    bpp = oc.bpp({k: v.cpu() for k, v in out["likelihoods"].items()}, 128 * 192)
    assert abs(bpp.item() - oc.bpp(ref["likelihoods"], 128 * 192).item()) < 1e-3


def test_transform_autograd_vs_oracle(net_and_params):
    net, P = net_and_params
    for p in net.parameters():
        p.requires_grad_(False)
    x = rnd((1, 3, 64, 128), 4)
    xd = x.to(DEV).requires_grad_(True)
    y = net.g_a(xd)
    xh = net.g_s(y)
    loss = (xh * xh).mean() + 0.1 * y.abs().mean()
    loss.backward()
    xr = x.clone().requires_grad_(True)
    yr = oc.g_a(P, xr)
    xhr = oc.g_s(P, yr)
    ((xhr * xhr).mean() + 0.1 * yr.abs().mean()).backward()
    assert rel_err(y.detach().cpu(), yr.detach()) < 1e-4
    assert rel_err(xh.detach().cpu(), xhr.detach()) < 1e-4
    assert rel_err(xd.grad.cpu(), xr.grad) < 1e-3


def test_image_coder_tuple(net_and_params):
    from imagecompression_adversarial_amd.anchors import balle
    net, P = net_and_params
    ic = balle.Image_coder.__new__(balle.Image_coder)
    torch.nn.Module.__init__(ic)
    ic.MODEL, ic.net = "hyper", net
    x = rnd((1, 3, 64, 64), 5).to(DEV)
    with torch.no_grad():
        x_hat, y, z_hat, y_lik, z_lik = ic(x, False, False, False)
    assert x_hat.shape == x.shape and y.shape == (1, 192, 4, 4) and z_hat.shape == (1, 128, 1, 1)
    assert float(y_lik.min()) >= 1e-9 and float(z_lik.max()) <= 1.0


def test_ops_bounds_exact(golden):
    from imagecompression_adversarial_amd.utils import ops
    x = torch.tensor(golden["bounds_x"]).to(DEV)
    for tag, gval in (("gpos", 1.0), ("gneg", -1.0), ("gzero", 0.0)):
        xx = x.clone().requires_grad_(True)
        y = ops.Up_bound.apply(ops.Low_bound.apply(xx, 0.0), 1.0)
        y.backward(torch.full_like(y, gval))
        np.testing.assert_array_equal(y.detach().cpu().numpy(), golden["bounds_y"])
        np.testing.assert_array_equal(xx.grad.cpu().numpy(), golden[f"bounds_dx_{tag}"])


def test_torch_msssim_module_vs_golden(golden):
    from imagecompression_adversarial_amd.utils import torch_msssim
    a = rnd((1, 3, 192, 192), 31)
    b = torch.clamp(a + (rnd((1, 3, 192, 192), 32) - 0.5) * 0.2, 0, 1)
    bd = b.to(DEV).requires_grad_(True)
    v = torch_msssim.MS_SSIM(max_val=1.0)(a.to(DEV), bd)
    v.backward()
    assert abs(v.item() - float(golden["tmssim_val"])) < 2e-6
    assert rel_err(bd.grad.cpu(), golden["tmssim_grad"]) < 1e-3


def test_attack_rd_cli_runs(capsys):
    from imagecompression_adversarial_amd import attack_rd, coder
    args = coder.config().parse_args(["-m", "hyper", "-metric", "mse", "-q", "1", "-steps", "3",
                                      "-s", "synthetic:2x192x256", "--synthetic-weights", "--batch", "2"])
    out = attack_rd.main(args)
    txt = capsys.readouterr().out
    assert "AVG: hyper-mse-1" in txt and "synthetic_0" in txt and "synthetic_1" in txt
    assert out["bpp_ori"] > 0 and out["bpp"] > 0


def test_attack_rd_cli_targeted_roi(capsys, tmp_path, monkeypatch):
    """-t / --mask_loc (README 'attack with ROI'): runs end to end and writes the target-suffixed PNGs."""
    from imagecompression_adversarial_amd import attack_rd, coder
    monkeypatch.chdir(tmp_path)
    args = coder.config().parse_args(["-m", "hyper", "-metric", "mse", "-q", "3", "-steps", "3", "-t", "synthetic",
                                      "--mask_loc", "16", "96", "8", "64", "-la_bkg_in", "0.01",
                                      "-s", "synthetic:1x128x128", "--synthetic-weights"])
    out = attack_rd.main(args)
    txt = capsys.readouterr().out
    assert "-> synthetic" in txt and "AVG: hyper-mse-3" in txt
    assert out["bpp"] > 0
    assert any(p.name.endswith("_advin_synthetic.png") for p in tmp_path.iterdir())


def test_attack_rd_cli_bf16_targeted_roi(capsys, tmp_path, monkeypatch):
    """Config 5 through the CLI: -t / --mask_loc on the bf16 conv path (--precision bf16)."""
    from imagecompression_adversarial_amd import attack_rd, coder
    monkeypatch.chdir(tmp_path)
    args = coder.config().parse_args(["-m", "hyper", "-metric", "mse", "-q", "3", "-steps", "3", "-t", "synthetic",
                                      "--mask_loc", "64", "192", "64", "192", "--precision", "bf16",
                                      "-s", "synthetic:2x256x256", "--synthetic-weights", "--batch", "2"])
    out = attack_rd.main(args)
    txt = capsys.readouterr().out
    assert "-> synthetic" in txt and "AVG: hyper-mse-3" in txt
    assert out["bpp"] > 0


def test_cheng2020_cli_runs(capsys):
    from imagecompression_adversarial_amd import attack_rd, coder
    args = coder.config().parse_args(["-m", "cheng2020", "-metric", "ms-ssim", "-q", "6", "-steps", "2",
                                      "-s", "synthetic:2x192x192", "--synthetic-weights", "--batch", "2"])
    out = attack_rd.main(args)
    txt = capsys.readouterr().out
    assert "AVG: cheng2020-ms-ssim-6" in txt
    assert out["bpp_ori"] > 0


@pytest.mark.parametrize("q", [3, 6])
def test_transform_weight_grads_vs_oracle(q):
    """Module API with trainable transforms (train.py:349-362 through the INTEGRATION.md module swap):
    net.g_a / net.g_s forward + loss.backward() give every g_a / g_s parameter gradient and the input
    gradient, equal to oracle autograd (rel <= 2e-3 of each tensor's max; fp32 reduction order).
    Transforms without a HIP parameter-gradient path raise instead of returning nothing."""
    from imagecompression_adversarial_amd import codec
    P = oc.perturb_params(oc.init_params("hyper", q, seed=0), seed=1)
    net = codec.bmshj2018_hyperprior(q)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items()})
    net.load_state_dict(sd)
    net = net.to(DEV).train()
    x = rnd((2, 3, 64, 128), 12)
    xd = x.to(DEV).requires_grad_(True)
    y = net.g_a(xd)
    xh = net.g_s(y)
    loss = ((xh - xd.detach()) ** 2).mean() + 0.1 * y.abs().mean()
    loss.backward()
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xr = x.clone().requires_grad_(True)
    yr = oc.g_a(Pr, xr)
    xhr = oc.g_s(Pr, yr)
    (((xhr - x) ** 2).mean() + 0.1 * yr.abs().mean()).backward()
    named = dict(net.named_parameters())
    checked = 0
    for k, v in Pr.items():
        if not k.startswith(("g_a.", "g_s.")):
            continue
        g = named[k].grad
        assert g is not None, k
        assert rel_err(g.cpu().reshape(v.shape), v.grad) < 2e-3, k
        checked += 1
    assert checked == sum(1 for k in named if k.startswith(("g_a.", "g_s.")))
    assert rel_err(xd.grad.cpu(), xr.grad) < 1e-3
    with pytest.raises(NotImplementedError):
        net.h_a(torch.abs(y.detach()))
