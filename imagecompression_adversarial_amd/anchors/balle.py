"""Drop-in for anchors/balle.py: Image_coder (tuple-returning wrapper, anchors/balle.py:12-72)."""
from __future__ import annotations

import torch

from . import model as models
from .utils import update_registered_buffers


class Image_coder(torch.nn.Module):
    def __init__(self, MODEL, quality, metric, pretrained=True):
        super().__init__()
        self.MODEL = MODEL
        self.net = models.init_model(MODEL, quality, metric, pretrained)

    def forward(self, x, TRAINING, CONTEXT, POSTPROCESS):
        """returns (x_hat, y, z_hat, y_likelihoods, z_likelihoods) (anchors/balle.py:25-55)."""
        self.net.train() if TRAINING else self.net.eval()
        y = self.net.g_a(x)
        y_hat, z_hat, lik = models.entropy_estimator(y, self.net, self.MODEL)
        x_hat = self.net.g_s(y_hat)
        return x_hat, y, z_hat, lik["y"], lik["z"]

    def load_state_dict(self, state_dict):
        update_registered_buffers(self.net.entropy_bottleneck, "net.entropy_bottleneck",
                                  ["_quantized_cdf", "_offset", "_cdf_length"], state_dict)
        if self.MODEL in ("hyper", "context", "cheng2020"):
            update_registered_buffers(self.net.gaussian_conditional, "net.gaussian_conditional",
                                      ["_quantized_cdf", "_offset", "_cdf_length", "scale_table"], state_dict)
        return super().load_state_dict(state_dict)
