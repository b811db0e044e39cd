"""Drop-in for train.py --adv: adversarial fine-tuning of the bmshj2018 codecs on the HIP engine,
data-parallel over RCCL (one process per GPU).

    python -m imagecompression_adversarial_amd.train --adv -m hyper -q 3 -metric mse -steps 300 \
        -s synthetic:8x256x256 --synthetic-weights -train_steps 20
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m imagecompression_adversarial_amd.train --adv ...        # 8 x (batch_size / 8) images

RateDistortionLoss  train.py:37-96  (values only; the backward is train_engine.RDTrainer)
adv_step            train.py:335-366: inner attack_ (batch-coupled) -> train-mode forward -> loss ->
                    backward -> clip_grad_norm_(1.0) -> Adam(lr_train) -> aux Adam(1e-3) on EB.loss()
train               train.py:254-500 (the --adv path; lambda table :255-258, noise ramp :338-339)

Deliberate differences: the data is an image glob with random 256x256 crops or a seeded
synthetic batch (no vimeo dataset offline); lpips / --recompress are out of scope; no test_epoch
(it needs the kodak/vimeo test split); checkpoints are written with the reference's dict keys.
"""
from __future__ import annotations

import math
import os
import time
from glob import glob

import torch

from . import coder
from . import dist as D
from . import hip_ops as K
from . import msssim as MS
from .attack import attack_batch
from .train_engine import RDTrainer

LAMBS = {
    "mse": [0.0018, 0.0035, 0.0067, 0.0130, 0.0250, 0.0483, 0.0932, 0.1800],
    "ms-ssim": [2.40, 4.58, 8.73, 16.64, 31.73, 60.50, 115.37, 220.00],
}


class RateDistortionLoss:
    """train.RateDistortionLoss (train.py:37-96) for mse / ms-ssim; values from an output dict."""

    def __init__(self, metric="mse", lmbda=1e-2):
        if metric not in ("mse", "ms-ssim"):
            raise ValueError(f"metric {metric!r} (lpips is out of scope)")
        self.metric, self.lmbda = metric, float(lmbda)

    def __call__(self, output, target, training=True):
        N, _, H, W = target.shape
        num_pixels = N * H * W
        out = {}
        bpp = 0.0
        for lik in output["likelihoods"].values():
            bpp = bpp + torch.log(torch.clamp(lik, min=1.0 / 65536)).sum() / (-math.log(2) * num_pixels)
        out["bpp_loss"] = bpp
        x_hat = output["x_hat"]
        if not training:
            x_hat = torch.clamp(x_hat, 0.0, 1.0)
            out["mse_loss"] = torch.mean((x_hat - target) ** 2)
            out["msim_loss"] = MS.ms_ssim(x_hat, target, data_range=1.0)
            out["psnr"] = -10.0 * math.log10(float(out["mse_loss"]))
            out["msim_dB"] = -10.0 * math.log10(1.0 - float(out["msim_loss"]))
            return out
        lamb_r = 0.0 if self.lmbda == 100 else 1.0   # train.py:77-83 "Inf Mode"
        if self.metric == "mse":
            out["distortion_loss"] = torch.mean((x_hat - target) ** 2)
            out["loss"] = self.lmbda * 255 ** 2 * out["distortion_loss"] + lamb_r * bpp
        else:
            out["distortion_loss"] = MS.ms_ssim(x_hat, target, data_range=1.0)
            out["loss"] = self.lmbda * (1 - out["distortion_loss"]) + lamb_r * bpp
        return out


def main_parameters(net):
    return [p for n, p in net.named_parameters() if not n.endswith(".quantiles")]


def adv_step(net, trainer: RDTrainer, optimizer, aux_optimizer, batch_x, args, group=None, world=1, qnoise=None,
             record=None):
    """One outer step of train.py:335-366 on this rank's shard.  The loss of the reference is a mean over the
    GLOBAL batch, so each rank's gradient and loss values (means over its shard) are weighted by
    B_local / B_global and summed over ranks: exact for uneven shards too (one flat all-reduce).
    qnoise: optional (noise_y, noise_z) train-mode quantisation noise for this shard (tests); record: an optional list
    that receives the inner attack's per-step branch census (one list of per-image cheap flags per step)."""
    batch_x = batch_x.detach().contiguous()
    B_local = batch_x.shape[0]
    if B_local == 0:
        raise ValueError("empty shard: the global batch must hold at least one image per rank")
    B_global = D.global_count(B_local, batch_x.device, group)
    for p in net.parameters():
        p.requires_grad_(False)
    # the inner attack runs on the attack engine's precision (x6 by default for bmshj2018: fp32-accurate)
    kern = net.kernels(net.attack_precision(getattr(args, "precision", None)))
    res = attack_batch(kern, batch_x, steps=args.steps, epsilon=args.epsilon, noise_thr=args.noise,
                       lr=args.lr_attack, att_metric=args.att_metric, clamp=args.clamp, eval_msssim=False,
                       coupled=True, group=group, record=record is not None)
    if record is not None:
        record.extend(res.branches)
    for p in net.parameters():
        p.requires_grad_(True)
    batch_adv = res.im_adv.detach()
    if getattr(args, "round_adv", False):   # adv_train.py:162-164 quantises the adversarial input
        batch_adv = torch.round(batch_adv * 255.0) / 255.0
    net.train()
    optimizer.zero_grad(set_to_none=False)
    aux_optimizer.zero_grad()
    out = trainer.step(batch_adv, *(qnoise or ()))
    if group is not None:
        w = B_local / B_global
        trainer.flat_grad.mul_(w)
        D.allreduce_sum_(trainer.flat_grad, group)
        keys = ("loss", "bpp_loss", "distortion_loss")
        vals = torch.stack([torch.as_tensor(out[k], device=batch_x.device, dtype=torch.float32).reshape(())
                            for k in keys]) * w
        D.allreduce_sum_(vals, group, kind="loss")
        out.update({k: vals[i] for i, k in enumerate(keys)})
    out["grad_norm"] = torch.nn.utils.clip_grad_norm_(main_parameters(net), 1.0).detach()
    optimizer.step()
    aux_loss = net.aux_loss()
    aux_loss.backward()
    aux_optimizer.step()
    out["aux_loss"] = aux_loss.detach()
    return out, batch_adv


def _batches(args, rank, world, device):
    """Yield this rank's shard of each global batch (batch_size images of 256x256 crops)."""
    g = torch.Generator().manual_seed(1234)
    src = args.source
    gb = int(src.split(":", 1)[1].split("x")[0]) if src.startswith("synthetic:") else args.batch_size
    if gb < world:
        raise ValueError(f"global batch {gb} < {world} ranks: every rank needs at least one image")
    if src.startswith("synthetic:"):
        B, H, W = (int(v) for v in src.split(":", 1)[1].split("x"))
        sl = D.shard_range(B, rank, world)
        while True:
            x = torch.rand((B, 3, H, W), generator=g)
            yield x[sl.start:sl.stop].to(device)
    files = sorted(glob(src))
    if not files:
        raise FileNotFoundError(src)
    crop = 256
    while True:
        idx = torch.randint(len(files), (args.batch_size,), generator=g).tolist()
        ims = []
        for i in idx:
            t, H, W = coder.read_image(files[i])
            t = t[:, :, :H, :W]
            if H < crop or W < crop:
                raise ValueError(f"{files[i]} smaller than the {crop}px crop")
            y0 = int(torch.randint(H - crop + 1, (1,), generator=g))
            x0 = int(torch.randint(W - crop + 1, (1,), generator=g))
            ims.append(t[:, :, y0:y0 + crop, x0:x0 + crop])
        x = torch.cat(ims, 0)
        sl = D.shard_range(x.shape[0], rank, world)
        yield x[sl.start:sl.stop].contiguous().to(device)


def save_checkpoint(state, filename):
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    torch.save(state, filename)


def train(args):
    rank, world, group = D.init_from_env()
    if world > 1:
        args.device = f"cuda:{torch.cuda.current_device()}"
    if not args.adv:
        raise NotImplementedError("only the adversarial fine-tune (--adv) runs on the HIP trainer")
    net, last_epoch, optimizer, aux_optimizer, lr_scheduler = coder.load_model(args, training=True)
    lamb = LAMBS[args.metric][args.quality - 1] if args.lamb is None else args.lamb
    trainer = RDTrainer(net, args.metric, lamb)
    noise_range = args.noise
    ckpt_dir = f"./ckpts/adv/{args.model}-{lamb}-{args.metric}-{args.noise}-{args.steps}"
    if rank == 0:
        print("Lambda:", lamb)
        print("Learning rate (training):", args.lr_train)
        print("Learning rate (adversarial):", args.lr_attack)
        print(args.batch_size, "adv examples in all", args.batch_size, f"({world} ranks)")
    data = _batches(args, rank, world, args.device)
    t = time.time()
    out = None
    for step in range(args.train_steps):
        if step <= 100:
            args.noise = noise_range * step / 100   # train.py:338-339
        batch_x = next(data)
        out, _ = adv_step(net, trainer, optimizer, aux_optimizer, batch_x, args, group, world)
        if rank == 0 and (step % 10 == 0 or step == args.train_steps - 1):
            print("step:", step, "loss:", float(out["loss"]), "distortion:", float(out["distortion_loss"]),
                  "rate:", float(out["bpp_loss"]), f"lr: {optimizer.param_groups[0]['lr']}",
                  "Epoch Time:", time.time() - t)
        if rank == 0 and args.save_every and step > 0 and step % args.save_every == 0:
            save_checkpoint({"epoch": last_epoch, "step": step, "state_dict": net.state_dict(),
                             "loss": float(out["loss"]), "optimizer": optimizer.state_dict(),
                             "aux_optimizer": aux_optimizer.state_dict(),
                             "lr_scheduler": lr_scheduler.state_dict()},
                            f"{ckpt_dir}/ckpt-{last_epoch}-{step}.pth.tar")
    return out


def config():
    p = coder.config()
    p.add_argument("-train_steps", dest="train_steps", type=int, default=2001,
                   help="outer steps (train.py returns at step 2000)")
    p.add_argument("--round-adv", dest="round_adv", action="store_true",
                   help="quantise the adversarial batch to uint8 levels (adv_train.py:162-164)")
    p.add_argument("--save-every", dest="save_every", type=int, default=100)
    return p


if __name__ == "__main__":
    train(config().parse_args())
