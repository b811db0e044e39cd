"""Drop-in for coder.py: shared CLI, image I/O, model loading.

config                coder.py:166-220 (same flags, same defaults)
read_image            coder.py:21-40   (PIL -> /255 (float64) -> float32, zero-pad to x64, NCHW)
write_image           coder.py:42-48   (np.round(x*255) -> uint8; round-half-to-even)
load_model            coder.py:88-147
configure_optimizers  coder.py:50-86
code                  coder.py:153-164
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .anchors import model as models

os.environ.setdefault("TORCH_HOME", "./ckpts/torch/")


def read_image(filename, padding=64):
    from PIL import Image
    img = np.array(Image.open(filename)) / 255.0
    C = 3
    if len(img.shape) < 3:
        print("[WARNING] automatically convert gray image to rgb format!")
        H, W = img.shape
        img = np.tile(img.reshape((H, W, 1)), (1, 1, 3))
    else:
        H, W, _ = img.shape
    H_PAD = int(padding * np.ceil(H / padding))
    W_PAD = int(padding * np.ceil(W / padding))
    im = np.zeros([H_PAD, W_PAD, 3], dtype="float32")
    im[:H, :W, :3] = img[:, :, :3]
    im = torch.FloatTensor(im).permute(2, 0, 1).contiguous().view(1, C, H_PAD, W_PAD)
    return im, H, W


def write_image(x, filename, H=None, W=None):
    from PIL import Image
    if H is None and W is None:
        H, W = x.shape[2:]
    x = np.round(x.data[0].cpu().numpy() * 255.0)
    x = x.astype("uint8").transpose(1, 2, 0)
    Image.fromarray(x[:H, :W, :]).save(filename)


def configure_optimizers(net, args):
    parameters = {n for n, p in net.named_parameters() if not n.endswith(".quantiles") and p.requires_grad}
    aux_parameters = {n for n, p in net.named_parameters() if n.endswith(".quantiles") and p.requires_grad}
    params_dict = dict(net.named_parameters())
    assert len(parameters & aux_parameters) == 0
    if not args.adv:
        assert len(parameters | aux_parameters) - len(params_dict.keys()) == 0
    optimizer = torch.optim.Adam((params_dict[n] for n in sorted(parameters)), lr=args.lr_train)
    aux_optimizer = torch.optim.Adam((params_dict[n] for n in sorted(aux_parameters)), lr=1e-3)
    return optimizer, aux_optimizer


def load_model(args, training):
    MODEL = args.model
    quality = args.quality
    arch_lists = ["factorized", "hyper", "context", "cheng2020", "debug"]
    assert MODEL in arch_lists, f"'{MODEL}' not in {arch_lists} for param '-m'"
    print("==================== NETWORK SETTINGS ===================")
    print("[ARCH]", MODEL, quality, args.metric)
    download = False
    if not args.checkpoint and not args.new:
        print("[CKPT] Download from CompressAI Model Zoo!")
        download = True
    elif not args.checkpoint:
        print("[CKPT] No Checkpoint Loaded!!!")
    if getattr(args, "synthetic_weights", False):
        download = False
        print("[CKPT] synthetic seeded weights (no zoo download available offline)")
    net = models.init_model(MODEL, quality=quality, metric=args.metric, pretrained=download)
    if getattr(args, "synthetic_weights", False):
        _synthetic_init(net, seed=0)
    net = net.to(args.device)
    checkpoint = None
    if args.checkpoint:
        print("[CKPT] Loading", args.checkpoint)
        checkpoint = torch.load(args.checkpoint, map_location=args.device, weights_only=True)
        if checkpoint.get("state_dict"):
            net.load_state_dict(checkpoint["state_dict"])
        else:
            # old version ckpts (coder.py:107-116): an anchors.balle.Image_coder state dict ("net."-prefixed
            # CompressAI names, CDF buffers of checkpoint-dependent size); converted and re-saved as
            # {"state_dict": ...} next to it (args.checkpoint + "new"), then loaded from there
            old = convert_old_checkpoint(checkpoint)
            torch.save({"state_dict": old}, args.checkpoint + "new")
            checkpoint = torch.load(args.checkpoint + "new", map_location=args.device, weights_only=True)
            net.load_state_dict(checkpoint["state_dict"])
    print("=========================================================")
    if training:
        last_epoch = 0
        optimizer, aux_optimizer = configure_optimizers(net, args)
        lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min", factor=0.5)
        if checkpoint is not None and "state_dict" in checkpoint:
            last_epoch = checkpoint["epoch"] + 1
            optimizer.load_state_dict(checkpoint["optimizer"])
            aux_optimizer.load_state_dict(checkpoint["aux_optimizer"])
            lr_scheduler.load_state_dict(checkpoint["lr_scheduler"])
        return net.train(), last_epoch, optimizer, aux_optimizer, lr_scheduler
    if checkpoint is not None and getattr(args, "eval", False):
        # evaluation of a training checkpoint (coder.py:138-146): report its epoch / step / learning rate
        last_epoch = checkpoint["epoch"]
        print("Trained epoch", last_epoch)
        if checkpoint.get("step"):
            print("Trained step", checkpoint["step"])
        optimizer, aux_optimizer = configure_optimizers(net, args)
        optimizer.load_state_dict(checkpoint["optimizer"])
        print(f"Learning rate: {optimizer.param_groups[0]['lr']}")
    return net.eval()


def convert_old_checkpoint(state_dict, prefix="net."):
    """anchors.balle.Image_coder.load_state_dict (anchors/balle.py:57-72) + net_old.net.state_dict()
    (coder.py:110-113): strip the wrapper's "net." prefix; the CDF buffers keep their checkpoint sizes (the
    model's load_state_dict resizes them, anchors/utils.py:74-109)."""
    if not state_dict or not all(k.startswith(prefix) for k in state_dict):
        raise KeyError(f"not an old-format (Image_coder) checkpoint: keys must start with {prefix!r}")
    return {k[len(prefix):]: v for k, v in state_dict.items()}


def _synthetic_init(net, seed=0):
    """Seeded CompressAI-default init (conv: PyTorch default; GDN beta=1, gamma=0.1 I; EB init)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith(".weight") or name.endswith(".bias"):
                mod = net.get_submodule(name.rsplit(".", 1)[0])
                w = mod.weight
                fan_in = w.shape[1] * w.shape[2] * w.shape[3]
                bound = 1.0 / fan_in ** 0.5
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * bound)
            elif "._bias" in name:
                p.copy_(torch.rand(p.shape, generator=g) - 0.5)


@torch.no_grad()
def code(args, net, input_file, out_file=None):
    net.eval()
    im, _, _ = read_image(input_file)
    result = net(im.to(args.device))
    if out_file:
        write_image(torch.clamp(result["x_hat"], min=0.0, max=1.0), out_file)
    return result


def config():
    p = argparse.ArgumentParser()
    p.add_argument("-device", type=str, default="cuda:0", help="dev id")
    p.add_argument("-lr_train", dest="lr_train", type=float, default=0.0001, help="train learning rate")
    p.add_argument("-lamb", dest="lamb", type=float, default=None, help="training lambda")
    p.add_argument("--eval", dest="eval", action="store_true", help="evaluation mode")
    p.add_argument("--adv", action="store_true", help="Adversarial training")
    p.add_argument("-batch_size", type=int, default=8, help="Batch size")
    p.add_argument("-cn", "--ckpt_num", type=int, help="load checkpoint by step number")
    p.add_argument("-l", "--lamb", type=float, default=6400.0, help="lambda")
    p.add_argument("-j", "--job", type=str, default="", help="job name")
    p.add_argument("--ctx", dest="context", action="store_true")
    p.add_argument("--no-ctx", dest="context", action="store_false")
    p.add_argument("--post", dest="post", action="store_true")
    p.add_argument("-itx", dest="iter_x", type=int, default=0, help="iter step updating x")
    p.add_argument("-ity", dest="iter_y", type=int, default=0, help="iter step updating y")
    p.add_argument("-m", dest="model", type=str, default="hyper",
                   help="compress model in 'factor','hyper','context','cheng2020','nonlocal'")
    p.add_argument("-metric", dest="metric", type=str, default="ms-ssim", help="mse or ms-ssim")
    p.add_argument("-q", dest="quality", type=int, default="3", help="quality in [1-8]")
    p.add_argument("--new", dest="new", action="store_true", help="train new model")
    p.add_argument("-padmode", dest="padding_mode", type=str, default="reflect", help="pad mode")
    p.add_argument("-steps", dest="steps", type=int, default=1001, help="attack iteration steps")
    p.add_argument("-random", dest="random", type=int, default=1, help="random start numbers")
    p.add_argument("-la", dest="lamb_attack", type=float, default=0.2, help="attack lambda")
    p.add_argument("-noise", dest="noise", type=float, default=0.0001, help="input noise threshold")
    p.add_argument("-lr_attack", dest="lr_attack", type=float, default=0.01, help="attack learning rate")
    p.add_argument("-s", dest="source", type=str, default="/workspace/ct/datasets/kodak/kodim*.png",
                   help="source input image (glob), or synthetic:<B>x<H>x<W>")
    p.add_argument("-t", dest="target", type=str, default=None, help="target image")
    p.add_argument("-ckpt", dest="checkpoint", type=str, default=None, help="local checkpoint dir")
    p.add_argument("--mask_loc", nargs="+", type=int, default=None)
    p.add_argument("-la_bkg_in", dest="lamb_bkg_in", type=float, default=1.0,
                   help="attack lambda of background area of input")
    p.add_argument("-la_bkg_out", dest="lamb_bkg_out", type=float, default=1.0,
                   help="attack lambda of background area of output")
    p.add_argument("-la_tar", dest="lamb_tar", type=float, default=1.0, help="attack lambda of target area")
    p.add_argument("-att_metric", dest="att_metric", type=str, default="L2", help="L1, L2, ms-ssim or lpips")
    p.add_argument("-e", dest="epsilon", type=float, default=16.0, help="noise max value epsilon")
    p.add_argument("-r", dest="rate", action="store_true", help="rate/distortion attack flag")
    p.add_argument("-p", dest="pad", type=int, default=None, help="padding size")
    p.add_argument("--log", dest="log", type=str, default="./logs/log.txt", help="log file")
    p.add_argument("--debug", dest="debug", action="store_true")
    p.add_argument("--no-clamp", dest="clamp", action="store_false")
    p.add_argument("-ssteps", dest="search_steps", type=int, default=20, help="binary search steps for CW")
    p.add_argument("-re", dest="recompress", type=int, default=None, help="recompress times")
    p.add_argument("--defend", action="store_true", help="defend mode")
    p.add_argument("--defend_m", dest="method", type=str, default="ensemble",
                   help="defend method in ['ensemble', 'resize']")
    p.add_argument("-degrade", dest="degrade", type=str, default=None, help="degrade method in ['deblur']")
    p.add_argument("--fintune", action="store_true")
    # backend extensions (not in the reference CLI)
    p.add_argument("--synthetic-weights", dest="synthetic_weights", action="store_true",
                   help="seeded CompressAI-init weights instead of the zoo download (offline)")
    p.add_argument("--batch", dest="batch", type=int, default=1,
                   help="attack this many same-size images per launch (per-image semantics preserved)")
    p.add_argument("--precision", dest="precision", type=str, default=None, choices=("x6", "fp32", "bf16"),
                   help="g_a/g_s conv operands: x6 (the default: fp32-accurate bf16x6 split-operand MFMA, error "
                        "vs float64 no larger than the fp32-operand path's), fp32 (fp32-operand MFMA; the debug "
                        "model's only one) or bf16 (bf16 operands, fp32 accumulate; BASELINE config 5; cheng2020: "
                        "over fp32 activations)")
    return p
