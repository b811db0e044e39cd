"""Drop-in for attack_ifgsm.py: I-FGSM / MI-FGSM (grad-sign + L-inf projection) on HIP.

attack_ifgsm   attack_ifgsm.py:364-438 (random_start=False, multi_start=1 path)
mifgsm_attack  attack_ifgsm.py:348-362  (fused into ica_ifgsm_step)
eval           attack_ifgsm.py:216-273  (no MS-SSIM)

    python -m imagecompression_adversarial_amd.attack_ifgsm -m hyper -q 3 -steps 10 -s synthetic:2x256x256 --synthetic-weights
"""
from __future__ import annotations

import time

import torch

from . import coder
from .attack import evaluate, ifgsm_batch
from .attack_rd import _sources


def attack_ifgsm(im_s, net, args, random_start=False, multi_start=1, momentum=False):
    """Returns (im_adv, output_adv, output_s, bpp_ori, bpp, mse_in, mse_out, vi) per batch (lists for vi)."""
    if random_start or multi_start > 1:
        raise NotImplementedError("random start (PGD) variant is not on the HIP path yet")
    kern = net.kernels()
    from .attack import eval_forward
    _, bpp_ori = eval_forward(kern, im_s, clamp=True)
    x, output_s = ifgsm_batch(kern, im_s, steps=args.steps, epsilon=args.epsilon, momentum=momentum)
    im_, out, bpp, mse_in, mse_out, _, _, vi, _ = evaluate(kern, x, im_s, output_s, clamp=args.clamp, msssim=False)
    return im_, out, output_s, bpp_ori, bpp, mse_in, mse_out, vi


def main(args):
    net = coder.load_model(args, training=False).to(args.device)
    for p in net.parameters():
        p.requires_grad_(False)
    for name, t, H, W in _sources(args.source):
        if t is None:
            t, H, W = coder.read_image(name)
        start = time.time()
        im_adv, output_adv, output_s, bpp_ori, bpp, mse_in, mse_out, vi = attack_ifgsm(
            t.to(args.device), net, args, momentum=True)
        print(name, float(bpp_ori[0]), float(bpp[0]), vi[0], "Time:", time.time() - start)


if __name__ == "__main__":
    main(coder.config().parse_args())
