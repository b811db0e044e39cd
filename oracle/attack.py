"""CPU fp32 restatement of the attack step loops and the adversarial fine-tune step.

TEST INFRASTRUCTURE (see oracle/__init__.py).

  * ``attack``      attack_rd.attack_ (attack_rd.py:381-575) + attack_our (:332-379)
                    + self_ensemble.eval (self_ensemble.py:173-252).
                    ``coupled=False`` (default): each image of the batch is an
                    independent reference run (per-image loss_i, branch, loss);
                    ``coupled=True``: the batch-mean semantics train.py:342 uses.
  * ``ifgsm``       attack_ifgsm.attack_ifgsm / mifgsm_attack (attack_ifgsm.py:348-438).
  * ``rd_loss``     train.RateDistortionLoss (train.py:37-96).
  * ``adv_train_step``  train.py:335-366 (the working --adv path).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import torch

from . import codec
from .msssim import ms_ssim, ms_ssim_per_image


def lr_schedule(steps: int, lr: float):
    """MultiStepLR([1,2,3], gamma=0.33) stepped when i % (steps//3) == 0 (attack_rd.py:503,553)."""
    import warnings
    p = torch.zeros(1, requires_grad=True)
    opt = torch.optim.Adam([p], lr=lr)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
    out = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(steps):
            out.append(opt.param_groups[0]["lr"])
            if i % max(steps // 3, 1) == 0:
                sch.step()
    return out


def _per_image_mean(x):
    return x.flatten(1).mean(1)


def eval_batch(P, im_adv, im_s, output_s, model="hyper", clamp=True, adv=False, msssim=True):
    """self_ensemble.eval (self_ensemble.py:173-252), evaluated per image."""
    with torch.no_grad():
        im_ = torch.clamp(im_adv, 0.0, 1.0) if clamp else im_adv
        res = codec.forward(P, im_, model)
        out = torch.clamp(res["x_hat"], 0.0, 1.0) if clamp else res["x_hat"]
        H, W = im_adv.shape[2:]
        B = im_adv.shape[0]
        bpp = torch.stack([codec.bpp({k: v[b:b + 1] for k, v in res["likelihoods"].items()}, H * W)
                           for b in range(B)])
        mse_in = _per_image_mean((im_ - im_s) ** 2)
        mse_out = _per_image_mean((out - output_s) ** 2)
        if msssim:
            msim_in = ms_ssim_per_image(im_, im_s)
            msim_out = ms_ssim_per_image(out, output_s)
        else:
            msim_in = msim_out = torch.full((B,), float("nan"))
        vi, vi_msim = [], []
        for b in range(B):
            mi, mo = float(mse_in[b]), float(mse_out[b])
            v = vm = None
            if mi > 1e-20 and mo > 1e-20:
                v = 10.0 * math.log10(mo / mi)
                if not adv and msssim and float(msim_in[b]) < 0.9999:
                    vm = 10.0 * math.log10((1 - float(msim_out[b])) / (1 - float(msim_in[b])))
            vi.append(v)
            vi_msim.append(vm)
    return SimpleNamespace(im=im_, out=out, bpp=bpp, mse_in=mse_in, mse_out=mse_out,
                           msim_in=msim_in, msim_out=msim_out, vi=vi, vi_msim=vi_msim)


def _roi_masks(H, W, roi):
    x0, x1, y0, y1 = (0, W, 0, H) if roi is None else roi
    m = torch.zeros(1, 1, H, W)
    m[:, :, y0:y1, x0:x1] = 1.0     # attack_cv.py:159-161 (x = width, y = height)
    return m, 1.0 - m


def _masked_mean(e, m):
    """Per-image mean of e over the elements where m == 1 (3 channels each); 0 for an empty region."""
    cnt = 3.0 * m.sum()
    if float(cnt) == 0.0:
        return torch.zeros(e.shape[0], dtype=e.dtype)
    return (e * m).flatten(1).sum(1) / cnt


def attack(P, im_s, steps=1001, epsilon=16.0, noise_thr=1e-4, lr=0.01, att_metric="L2",
           clamp=True, model="hyper", coupled=False, init_noise=None, eval_msssim=True,
           record=None, target=None, roi=None, la_tar=1.0, la_bkg_in=1.0, la_bkg_out=1.0, expensive=None,
           adv=False, pad=None, padding_mode="reflect"):
    """attack_rd.attack_ restated (Adam on additive noise, L-inf box in the forward).

    record: optional list; per step appends dict(loss_i, branch) for trajectory tests.
    target / roi: the targeted / ROI attack (semantics as DESIGN.md states them;
    the reference's own masked loss (attack_data.py:219-221) multiplies scalar means by mask tensors, so
    its masked means are restated here as proper per-region means):
    expensive: optional f(im_in_subset, step) -> x_ replacing g_s(g_a(.)) in the expensive branch (the --adv
    attack through a defence, oracle.defend.adv_*); adv: the eval's args.adv (no vi_msim).
      loss_i = mean_tar((s - ii)^2) + la_bkg_in * mean_bkg((s - ii)^2)
      loss_o = la_tar * mean_tar((out_t - o)^2) + la_bkg_out * mean_bkg((out_s - o)^2)   (minimised)
    """
    B = im_s.shape[0]
    with torch.no_grad():
        H, W = im_s.shape[2:]
        if pad:   # attack_rd.py:389-419: padded pre-eval, cropped output_s, bits per unpadded pixel
            import torch.nn.functional as F
            res = codec.forward(P, F.pad(im_s, (pad, pad, pad, pad), mode=padding_mode), model)
            output_s = torch.clamp(res["x_hat"][:, :, pad:-pad, pad:-pad], 0.0, 1.0)
        else:
            res = codec.forward(P, im_s, model)
            output_s = torch.clamp(res["x_hat"], 0.0, 1.0) if clamp else res["x_hat"]
        bpp_ori = torch.stack([codec.bpp({k: v[b:b + 1] for k, v in res["likelihoods"].items()}, H * W)
                               for b in range(B)])
    noise_range = epsilon / 255.0
    if target is not None:
        return _attack_roi(P, im_s, output_s, bpp_ori, steps, noise_range, noise_thr, lr, clamp, model,
                           init_noise, eval_msssim, record, target, roi, la_tar, la_bkg_in, la_bkg_out)
    if init_noise is not None:
        noise = init_noise.clone()
    elif model == "debug":   # attack_rd.py:493-494: U(-sqrt(noise), sqrt(noise)) from the global RNG
        noise = torch.empty(im_s.shape).uniform_(-noise_thr ** 0.5, noise_thr ** 0.5).to(im_s.dtype)
    else:
        noise = torch.zeros_like(im_s)
    noise.requires_grad_(True)
    opt = torch.optim.Adam([noise], lr=lr)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
    im_in = None
    for i in range(steps):
        noise_c = codec.UpBound.apply(codec.LowBound.apply(noise, -noise_range), noise_range)
        if model == "debug":   # attack_rd.py:514-515: the debug model's input is not clamped to [0, 1]
            im_in = im_s + noise_c
        else:
            im_in = codec.UpBound.apply(codec.LowBound.apply(im_s + noise_c, 0.0), 1.0)
        if coupled:
            loss_i = torch.mean((im_s - im_in) ** 2)
            cheap = torch.full((B,), bool(loss_i > noise_thr))
            li_b = loss_i.expand(B)
        else:
            li_b = _per_image_mean((im_s - im_in) ** 2)
            cheap = li_b > noise_thr
        losses = torch.zeros((), dtype=im_s.dtype)
        if bool(cheap.any()):
            idx = cheap.nonzero().flatten()
            if att_metric == "L2":
                if coupled:
                    losses = losses + torch.mean((im_s - im_in) ** 2)
                else:
                    losses = losses + _per_image_mean((im_s[idx] - im_in[idx]) ** 2).sum()
            elif att_metric == "ms-ssim":
                if coupled:
                    losses = losses + (1.0 - ms_ssim(im_s, im_in))
                else:
                    losses = losses + (1.0 - ms_ssim_per_image(im_s[idx], im_in[idx])).sum()
            else:
                raise ValueError(att_metric)
        if bool((~cheap).any()):
            idx = (~cheap).nonzero().flatten()
            x_ = codec.transforms(P, im_in[idx], model) if expensive is None else expensive(im_in[idx], i)
            out = codec.bound01(x_) if clamp else x_
            if att_metric == "L2":
                if coupled:
                    losses = losses + (1.0 - torch.mean((output_s - out) * (output_s - out)))
                else:
                    d = output_s[idx] - out
                    losses = losses + (1.0 - _per_image_mean(d * d)).sum()
            else:
                if coupled:
                    losses = losses + ms_ssim(out, output_s)
                else:
                    losses = losses + ms_ssim_per_image(out, output_s[idx]).sum()
        if record is not None:
            record.append({"loss_i": li_b.detach().clone(), "cheap": cheap.clone(),
                           "lr": opt.param_groups[0]["lr"]})
        opt.zero_grad()
        losses.backward()
        opt.step()
        if i % max(steps // 3, 1) == 0:
            sch.step()
    im_in = im_in.detach()
    ev = eval_batch(P, im_in, im_s, output_s, model, clamp, adv=adv, msssim=eval_msssim)
    return SimpleNamespace(im_adv=ev.im, output_adv=ev.out, output_s=output_s, bpp_ori=bpp_ori,
                           bpp=ev.bpp, eval=ev, noise=noise.detach(), im_in=im_in)


def _attack_roi(P, im_s, output_s, bpp_ori, steps, noise_range, noise_thr, lr, clamp, model, init_noise,
                eval_msssim, record, target, roi, la_tar, la_bkg_in, la_bkg_out):
    B, _, H, W = im_s.shape
    with torch.no_grad():
        t = target.expand_as(im_s) if target.shape[0] == 1 else target
        output_t = torch.clamp(codec.forward(P, t, model)["x_hat"], 0.0, 1.0)
    m_tar, m_bkg = _roi_masks(H, W, roi)
    noise = torch.zeros_like(im_s) if init_noise is None else init_noise.clone()
    noise.requires_grad_(True)
    opt = torch.optim.Adam([noise], lr=lr)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [1, 2, 3], gamma=0.33)
    im_in = None
    for i in range(steps):
        noise_c = codec.UpBound.apply(codec.LowBound.apply(noise, -noise_range), noise_range)
        im_in = codec.UpBound.apply(codec.LowBound.apply(im_s + noise_c, 0.0), 1.0)
        d_in = (im_s - im_in) ** 2
        li_b = _masked_mean(d_in, m_tar) + la_bkg_in * _masked_mean(d_in, m_bkg)
        cheap = li_b > noise_thr
        losses = torch.zeros((), dtype=im_s.dtype)
        if bool(cheap.any()):
            losses = losses + li_b[cheap].sum()
        if bool((~cheap).any()):
            idx = (~cheap).nonzero().flatten()
            x_ = codec.transforms(P, im_in[idx], model)
            out = codec.bound01(x_) if clamp else x_
            lo = la_tar * _masked_mean((output_t[idx] - out) ** 2, m_tar) + \
                la_bkg_out * _masked_mean((output_s[idx] - out) ** 2, m_bkg)
            losses = losses + lo.sum()
        if record is not None:
            record.append({"loss_i": li_b.detach().clone(), "cheap": cheap.clone(), "lr": opt.param_groups[0]["lr"]})
        opt.zero_grad()
        losses.backward()
        opt.step()
        if i % max(steps // 3, 1) == 0:
            sch.step()
    im_in = im_in.detach()
    ev = eval_batch(P, im_in, im_s, output_s, model, clamp, adv=False, msssim=eval_msssim)
    x0, x1, y0, y1 = (0, W, 0, H) if roi is None else roi
    dd = (ev.out - output_t)[:, :, y0:y1, x0:x1]
    tar_mse = (dd * dd).flatten(1).mean(1)
    return SimpleNamespace(im_adv=ev.im, output_adv=ev.out, output_s=output_s, bpp_ori=bpp_ori, bpp=ev.bpp, eval=ev,
                           noise=noise.detach(), im_in=im_in, output_t=output_t, tar_mse=tar_mse)


def ifgsm(P, im_s, steps=10, epsilon=16.0, momentum=False, model="hyper", start_noise=None):
    """attack_ifgsm.attack_ifgsm (attack_ifgsm.py:364-438), per image.  start_noise: the U(-eps, eps) draw of
    the random (PGD) start, im_adv0 = clamp(im_s + start_noise, 0, 1) (:377-380); None: start at im_s."""
    with torch.no_grad():
        res = codec.forward(P, im_s, model)
        output_s = torch.clamp(res["x_hat"], 0.0, 1.0)
    eps = epsilon / 255.0
    if start_noise is not None:
        im_adv = torch.clamp(im_s + start_noise, 0, 1).detach().requires_grad_(True)
    else:
        im_adv = im_s.detach().clone().requires_grad_(True)
    g = torch.zeros_like(im_s)
    alpha = eps / steps
    for _ in range(steps):
        out = codec.transforms(P, im_adv, model)
        d = output_s - out
        loss = _per_image_mean(d * d).sum()
        grad, = torch.autograd.grad(loss, im_adv)
        with torch.no_grad():
            if momentum:
                l1 = grad.abs().flatten(1).sum(1).view(-1, 1, 1, 1)
                g = 1.0 * g + grad / l1
                nxt = torch.clamp(im_adv + alpha * torch.sign(g), 0, 1)
            else:
                nxt = im_adv + eps / steps * torch.sign(grad)
            nxt = torch.where(nxt > im_s + eps, im_s + eps, nxt)
            nxt = torch.where(nxt < im_s - eps, im_s - eps, nxt)
        im_adv = nxt.detach().requires_grad_(True)
    return im_adv.detach(), output_s


def rd_loss(out, target, metric="mse", lmbda=0.0067):
    """train.RateDistortionLoss.forward(training=True) (train.py:52-96), incl. the "Inf Mode" of
    lmbda == 100 (train.py:77-83: the rate term leaves the loss)."""
    N, _, H, W = target.shape
    num_pixels = N * H * W
    bpp = 0.0
    for lik in out["likelihoods"].values():
        lik = torch.clamp(lik, min=1.0 / 65536)
        bpp = bpp + torch.log(lik).sum() / (-math.log(2) * num_pixels)
    lamb_r = 0.0 if lmbda == 100 else 1.0
    if metric == "mse":
        d = torch.mean((out["x_hat"] - target) ** 2)
        loss = lmbda * 255 ** 2 * d + lamb_r * bpp
    elif metric == "ms-ssim":
        d = ms_ssim(out["x_hat"], target, data_range=1.0)
        loss = lmbda * (1 - d) + lamb_r * bpp
    else:
        raise ValueError(metric)
    return {"loss": loss, "bpp_loss": bpp, "distortion_loss": d}


def adv_train_step(P, batch_x, steps=300, noise_thr=1e-4, epsilon=16.0, lr_attack=0.01, att_metric="L2",
                   clamp=True, model="hyper", metric="mse", lmbda=0.0130, lr_train=1e-4, noise_y=None,
                   noise_z=None, record=None, state=None):
    """One outer step of train.py --adv (train.py:335-366): the batch-coupled inner attack (attack_rd.attack_
    on the whole batch, train.py:342), the train-mode forward of the adversarial batch with the given
    quantisation noise, RateDistortionLoss against that same batch (:349-351), backward,
    clip_grad_norm_(1.0) over the main parameters (:360), Adam(lr_train) (:361), then the aux loss of the
    EntropyBottleneck quantiles and its Adam(1e-3) (:363-366; coder.py:50-86 optimiser split).
    Returns (updated params dict, loss values (with the pre-clip gradient norm "grad_norm"), aux loss, the
    adversarial batch); record: the inner attack's per-step records (attack()).  state: a dict that carries the
    parameters and both Adam optimisers from one call to the next (several outer steps of one run; P is read on the
    first call only)."""
    r = attack(P, batch_x, steps=steps, epsilon=epsilon, noise_thr=noise_thr, lr=lr_attack, att_metric=att_metric,
               clamp=clamp, model=model, coupled=True, eval_msssim=False, record=record)
    batch_adv = r.im_adv.detach()
    main_names = sorted(k for k in P if not k.endswith(".quantiles"))
    aux_names = sorted(k for k in P if k.endswith(".quantiles"))
    if state is not None and "Q" in state:
        Q, opt, aux_opt = state["Q"], state["opt"], state["aux_opt"]
    else:
        Q = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
        opt = torch.optim.Adam([Q[k] for k in main_names], lr=lr_train)
        aux_opt = torch.optim.Adam([Q[k] for k in aux_names], lr=1e-3)
        if state is not None:
            state.update(Q=Q, opt=opt, aux_opt=aux_opt)
    res = codec.forward(Q, batch_adv, model, training=True, noise_y=noise_y, noise_z=noise_z)
    out = rd_loss(res, batch_adv, metric, lmbda)
    opt.zero_grad()
    aux_opt.zero_grad()
    out["loss"].backward()
    gn = torch.nn.utils.clip_grad_norm_([Q[k] for k in main_names], 1.0)
    opt.step()
    out["grad_norm"] = gn
    aux_loss = codec.eb_aux_loss(Q)
    aux_opt.zero_grad()
    aux_loss.backward()
    aux_opt.step()
    return ({k: v.detach() for k, v in Q.items()}, {k: float(v.detach()) for k, v in out.items()}, float(aux_loss.detach()),
            batch_adv)
