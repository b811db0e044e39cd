"""INTEGRATION.md §2's ctypes stub, executed verbatim: the reference-side binding a maintainer would add
(attack_rd.py:506-548 as raw C-ABI calls around the conv engine) reproduces AttackLoop.step bit for bit over
several steps, on both operand paths.  A stale snippet (wrong argtypes, wrong arity, wrong argument meaning)
fails here; tests/test_cpu_boundary.py checks its argtypes against include/ica_hip.h on the CPU."""
import os
import re

import pytest
import torch

from tests.conftest import REPO


def _snippet():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. C-ABI level"):]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["x6", "fp32"])
def test_integration_snippet_matches_attack_loop(precision, monkeypatch):
    from oracle import codec
    from imagecompression_adversarial_amd.attack import AttackLoop, _lr_table
    from imagecompression_adversarial_amd.engine import CodecKernels
    monkeypatch.chdir(REPO)
    ns = {}
    exec(compile(_snippet(), "INTEGRATION.md", "exec"), ns)
    dev = torch.device("cuda:0")
    P = codec.perturb_params(codec.init_params("hyper", 3, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * 40.0   # non-zero latents: both branches occur
    kern = CodecKernels({k: v.to(dev) for k, v in P.items()}, "hyper", precision=precision)
    g = torch.Generator().manual_seed(5)
    im_s = torch.rand((3, 3, 128, 192), generator=g).to(dev)
    steps = 6
    loop = AttackLoop(kern, im_s, steps=steps)
    loop.compact = False
    noise, m, v = loop.noise.clone(), loop.m.clone(), loop.v.clone()
    lrs = _lr_table(steps, 0.01)
    for i in range(steps):
        br = ns["attack_step"](i, kern, im_s, noise, m, v, loop.output_s, lrs[i])
        ref_br = loop.step(i, census=True)
        torch.cuda.synchronize()
        assert br.tolist() == ref_br, (i, br.tolist(), ref_br)
        assert torch.equal(noise, loop.noise), i
        assert torch.equal(m, loop.m) and torch.equal(v, loop.v), i
    assert float(noise.abs().max()) > 0
