"""Drop-in for anchors/model.py: model factory and the functional entropy estimator.

init_model       anchors/model.py:60-78
compressor       anchors/model.py:80-84
entropy_estimator anchors/model.py:86-108
probe            anchors/model.py:110-131
"""
from __future__ import annotations

import torch

from .. import codec


def init_model(MODEL, quality, metric, pretrained=True):
    if MODEL == "factorized":
        return codec.bmshj2018_factorized(quality=quality, metric=metric, pretrained=pretrained)
    if MODEL == "hyper":
        return codec.bmshj2018_hyperprior(quality=quality, metric=metric, pretrained=pretrained)
    if MODEL == "cheng2020":
        return codec.cheng2020_anchor(quality=quality, metric=metric, pretrained=pretrained)
    if MODEL == "context":
        return codec.mbt2018(quality=quality, metric=metric, pretrained=pretrained)
    if MODEL == "debug":   # anchors/model.py:61-68: ae_onelayer(N=3, M=192) at every quality, never pretrained
        assert not pretrained, "No download-able model available!"
        return codec.AeOneLayer(N=3, M=192)
    raise AssertionError(f"'{MODEL}' not in ['factorized', 'hyper', 'context', 'cheng2020', 'debug']")


def compressor(x, net, MODEL):
    y = net.g_a(x)
    y_hat, z_hat, entropys = entropy_estimator(y, net, MODEL)
    x_hat = net.g_s(y_hat)
    return {"x_hat": x_hat, "y_hat": y_hat, "z_hat": z_hat, "likelihoods": entropys}


def entropy_estimator(y, net, MODEL):
    if MODEL == "factorized":
        y_hat, y_likelihoods = net.entropy_bottleneck(y)
        z_hat, z_likelihoods = 0, torch.Tensor([1.0])
    elif MODEL == "hyper":
        z = net.h_a(torch.abs(y))
        z_hat, z_likelihoods = net.entropy_bottleneck(z)
        scales_hat = net.h_s(z_hat)
        y_hat, y_likelihoods = net.gaussian_conditional(y, scales_hat)
    elif MODEL in ("context", "cheng2020"):
        z = net.h_a(y)
        z_hat, z_likelihoods = net.entropy_bottleneck(z)
        params = net.h_s(z_hat)
        y_hat = net.gaussian_conditional.quantize(y, "noise" if net.training else "dequantize")
        ctx_params = net.context_prediction(y_hat)
        gaussian_params = net.entropy_parameters(torch.cat((params, ctx_params), dim=1))
        scales_hat, means_hat = gaussian_params.chunk(2, 1)
        _, y_likelihoods = net.gaussian_conditional(y, scales_hat, means=means_hat)
    else:
        raise NotImplementedError(MODEL)
    return y_hat, z_hat, {"y": y_likelihoods, "z": z_likelihoods}


def probe(x, net, name="y_hat", MODEL="hyper"):
    if name == "y_hat":
        return net.g_a(x)
    if name == "z_hat":
        return net.h_a(net.g_a(x))
    if name == "scales_hat":
        return net.h_s(net.h_a(net.g_a(x)))
    if name == "means_hat":
        if MODEL in ("context", "cheng2020"):
            y = net.g_a(x)
            z = net.h_a(y)
            y_hat = net.gaussian_conditional.quantize(y, "noise" if net.training else "dequantize")
            z_hat, _ = net.entropy_bottleneck(z)
            params = net.h_s(z_hat)
            ctx_params = net.context_prediction(y_hat)
            gaussian_params = net.entropy_parameters(torch.cat((params, ctx_params), dim=1))
            _, means_hat = gaussian_params.chunk(2, 1)
            return means_hat
        return None
    raise ValueError(name)
