"""The whole-batch network step of the attack loop as a HIP graph (attack.AttackLoop._network_graph): the replayed
steps must give the eager loop's bits exactly, per-image and batch-coupled (the fine-tune's inner attack, reference
train.py:342 -> attack_rd.py:332-379), for the targeted ROI attack (attack_cv / attack_rd -t --mask_loc) on the
bf16 path and for cheng2020 (x6 and bf16), and the graph must actually be used."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _run(kern, x, steps, coupled, graph, monkeypatch, **kw):
    from imagecompression_adversarial_amd import attack as A
    monkeypatch.setattr(A, "ATTACK_GRAPH", graph)
    loop = A.AttackLoop(kern, x, steps=steps, coupled=coupled, **kw)
    loop.run()
    torch.cuda.synchronize()
    return loop


@pytest.mark.parametrize("coupled", [False, True])
@pytest.mark.parametrize("q,H,W,B", [(1, 256, 256, 8), (3, 128, 192, 3)])
def test_graph_replay_same_bits(q, H, W, B, coupled, monkeypatch):
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd.engine import CodecKernels
    torch.manual_seed(0)
    net = models.bmshj2018_hyperprior(q)
    sd = {k: v.detach().to(DEV) for k, v in net.state_dict().items()}
    kern = CodecKernels(sd, "hyper", precision="x6")
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand((B, 3, H, W), generator=g, device=DEV)
    steps = 12
    eager = _run(kern, x, steps, coupled, False, monkeypatch)
    graph = _run(kern, x, steps, coupled, True, monkeypatch)
    assert eager.graph_replays == 0
    assert graph.graph_replays >= 1, graph.graph_replays
    print(f"graph replays {graph.graph_replays} of {steps} steps; expensive image-steps {graph.expensive_image_steps()}")
    assert torch.equal(eager.noise, graph.noise)
    assert torch.equal(eager.m, graph.m) and torch.equal(eager.v, graph.v)
    assert torch.equal(eager.census, graph.census)


def _same(eager, graph, steps):
    assert eager.graph_replays == 0
    assert graph.graph_replays >= 1, graph.graph_replays
    print(f"graph replays {graph.graph_replays} of {steps} steps; expensive image-steps {graph.expensive_image_steps()}")
    assert torch.equal(eager.noise, graph.noise)
    assert torch.equal(eager.m, graph.m) and torch.equal(eager.v, graph.v)
    assert torch.equal(eager.census, graph.census)


@pytest.mark.parametrize("precision", ["bf16", "x6"])
def test_graph_replay_same_bits_roi(precision, monkeypatch):
    """The targeted ROI attack (the config-5 mode: target reconstruction, ROI-weighted losses) replays its network step
    (ica_roi_loss included) with the eager loop's bits."""
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd.engine import CodecKernels
    torch.manual_seed(0)
    net = models.bmshj2018_hyperprior(3)
    sd = {k: v.detach().to(DEV) for k, v in net.state_dict().items()}
    kern = CodecKernels(sd, "hyper", precision=precision)
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.rand((2, 3, 256, 384), generator=g, device=DEV)
    kw = dict(target=torch.rand((2, 3, 256, 384), generator=g, device=DEV), roi=(96, 288, 64, 192), la_tar=1.0,
              la_bkg_in=1.0, la_bkg_out=1.0)
    steps = 8
    _same(_run(kern, x, steps, False, False, monkeypatch, **kw), _run(kern, x, steps, False, True, monkeypatch, **kw),
          steps)


@pytest.mark.parametrize("precision,q", [("x6", 6), ("bf16", 2)])
def test_graph_replay_same_bits_cheng(precision, q, monkeypatch):
    """cheng2020 (config 3's model) replays its network step with the eager loop's bits."""
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd.engine_cheng import ChengKernels
    torch.manual_seed(0)
    net = models.cheng2020_anchor(q)
    sd = {k: v.detach().to(DEV) for k, v in net.state_dict().items()}
    kern = ChengKernels(sd, precision=precision)
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.rand((2, 3, 128, 192), generator=g, device=DEV)
    steps = 6
    _same(_run(kern, x, steps, False, False, monkeypatch), _run(kern, x, steps, False, True, monkeypatch), steps)
