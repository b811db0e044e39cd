"""Process-per-GPU data parallelism for the two paths that shard.

* Attack (attack_rd / bench): images are independent -> each rank attacks its own
  shard, no collective on the data path (``shard_range``).
* Adversarial fine-tune (train.py --adv): each rank runs the inner attack and the
  train-mode backward on its shard, then ONE all-reduce (mean) of the flat
  gradient buffer (19.4 MiB fp32 for hyper q1-5) over RCCL/xGMI, then identical
  clip + Adam on every rank.  The batch-coupled inner attack adds one 4-byte
  all-reduce per inner step (``couple_loss_i``).

Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...``
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment).  Backend "nccl"
is RCCL on ROCm; "gloo" is used for the CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


# Optional timing hook (bench.py --config 4): {"grad": [(ev0, ev1), ...], "couple": [...]}, HIP events recorded on the
# issuing stream around each collective of the fine-tune (no synchronisation)
COLL_HOOK = None


def _timed(kind, fn):
    if COLL_HOOK is None or not torch.cuda.is_available():
        return fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = fn()
    e1.record()
    COLL_HOOK.setdefault(kind, []).append((e0, e1))
    return r


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init_from_env(backend: str | None = None):
    """Initialise the default process group when WORLD_SIZE > 1; returns (rank, world, group|None)."""
    world, rank, local = env_world()
    if world <= 1:
        return 0, 1, None
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=rank, world_size=world)
    return dist.get_rank(), dist.get_world_size(), dist.group.WORLD


def shard_range(n: int, rank: int, world: int) -> range:
    """Contiguous, balanced shard of n items for this rank (sizes differ by at most 1)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return range(lo, hi)


def allreduce_mean_(t: torch.Tensor, group=None, world: int | None = None) -> torch.Tensor:
    """In-place mean over ranks (SUM then scale: gloo has no AVG).  One collective for the whole buffer."""
    if group is None:
        return t
    if world is None:
        world = dist.get_world_size(group)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    t.div_(world)
    return t


def allreduce_sum_(t: torch.Tensor, group=None, kind: str = "grad") -> torch.Tensor:
    """In-place sum over ranks (one collective for the whole buffer); `kind` names it in COLL_HOOK."""
    if group is not None:
        _timed(kind, lambda: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group))
    return t


def couple_loss_i(loss_i: torch.Tensor, B_global: int, group=None) -> torch.Tensor:
    """Batch-coupled attack semantics: every entry of loss_i (per-image input MSEs of this rank's shard)
    becomes the mean over the global batch (attack_rd.py:333 applied to the whole batch)."""
    tot = loss_i.sum().reshape(1)
    if group is not None:
        _timed("couple", lambda: dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group))
    loss_i.copy_((tot / B_global).expand(loss_i.shape[0]))
    return loss_i


def global_count(n_local: int, device, group=None) -> int:
    if group is None:
        return n_local
    t = torch.tensor([float(n_local)], device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())
