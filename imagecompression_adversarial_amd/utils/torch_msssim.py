"""Drop-in for utils/torch_msssim.py (MS_SSIM module, 2-D window, same padding, global mean)
running on the HIP MS-SSIM kernels (utils/torch_msssim.py:18-76)."""
from __future__ import annotations

import torch

from .. import msssim as _ms


class MS_SSIM(torch.nn.Module):
    def __init__(self, size_average=True, max_val=255, device_id=0):
        super().__init__()
        self.size_average = size_average
        self.channel = 3
        self.max_val = max_val

    def ms_ssim(self, img1, img2, levels=5):
        assert levels == 5
        return _ms.torch_msssim(img1, img2, max_val=self.max_val)

    def forward(self, img1, img2, levels=5):
        return self.ms_ssim(img1, img2, levels)
