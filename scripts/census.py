"""Branch census of the attack loop (FLOPs count only the expensive-branch image-steps).

    python scripts/census.py [--config 2|1] [--steps 1001] [--batch 32] > gpurun_out/census.json

Runs the whole attack_rd step loop on the HIP path and records, per step, how many images took the
expensive branch (loss_i <= -noise: g_a + g_s fwd + bwd) and the wall time of the loop.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=(1, 2))
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--compact", type=int, default=1)
    args = ap.parse_args()
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd.attack import AttackLoop
    from imagecompression_adversarial_amd.engine import CodecKernels
    dev = torch.device("cuda", 0)
    if args.config == 2:
        q, H, W, B, steps = 3, 512, 768, 32, 1001
    else:
        q, H, W, B, steps = 1, 256, 256, 1, 100
    B = args.batch or B
    steps = args.steps or steps
    torch.manual_seed(0)
    net = models.bmshj2018_hyperprior(q)
    sd = {k: v.detach().to(dev) for k, v in net.state_dict().items()}
    kern = CodecKernels(sd, "hyper")
    gen = torch.Generator(device=dev).manual_seed(0)
    im_s = torch.rand((B, 3, H, W), generator=gen, device=dev)
    loop = AttackLoop(kern, im_s, steps=steps)
    if hasattr(loop, "compact"):
        loop.compact = bool(args.compact)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    exp = []
    for i in range(steps):
        br = loop.step(i, census=True)
        exp.append(B - sum(br))
        if i % 100 == 0:
            print(f"step {i} expensive {exp[-1]} t {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"config": args.config, "B": B, "H": H, "W": W, "steps": steps, "wall_s": el,
                      "img_step_per_s": B * steps / el, "expensive_image_steps": sum(exp),
                      "expensive_frac": sum(exp) / (B * steps), "per_step_expensive": exp}))


if __name__ == "__main__":
    main()
