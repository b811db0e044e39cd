"""Drop-in for anchors/utils.py: conv/deconv geometry and dynamic buffer resize for checkpoints.

conv / deconv                 anchors/utils.py:112-130
update_registered_buffers     anchors/utils.py:74-109
"""
from __future__ import annotations

import torch

from ..codec import conv, deconv  # noqa: F401  (same geometry; used by the fused transforms)


def find_named_buffer(module, query):
    return next((b for n, b in module.named_buffers() if n == query), None)


def update_registered_buffers(module, module_name, buffer_names, state_dict, policy="resize_if_empty",
                              dtype=torch.int):
    valid = [n for n, _ in module.named_buffers()]
    for name in buffer_names:
        if name not in valid:
            raise ValueError(f'Invalid buffer name "{name}"')
    for name in buffer_names:
        new_size = state_dict[f"{module_name}.{name}"].size()
        buf = find_named_buffer(module, name)
        if policy in ("resize_if_empty", "resize"):
            if buf is None:
                raise RuntimeError(f'buffer "{name}" was not registered')
            if policy == "resize" or buf.numel() == 0:
                buf.resize_(new_size)
        elif policy == "register":
            if buf is not None:
                raise RuntimeError(f'buffer "{name}" was already registered')
            module.register_buffer(name, torch.empty(new_size, dtype=dtype).fill_(0))
        else:
            raise ValueError(f'Invalid policy "{policy}"')
