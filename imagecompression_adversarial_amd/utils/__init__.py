"""Mirror of the reference's ``utils`` package (utils/ops.py, utils/torch_msssim.py)."""
