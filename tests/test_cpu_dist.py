"""world_size-2 gloo tests (CPU) of the data-parallel pieces of the adversarial fine-tune and the
sharded attack: gradient all-reduce-mean, batch-coupled loss_i, shard ranges,
and that clip + Adam after the all-reduce keep the replicas bit-identical."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from imagecompression_adversarial_amd import dist as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, group = D.init_from_env("gloo")
        assert (r, w) == (rank, world)
        out = {}
        # 1. gradient mean
        g = torch.arange(6, dtype=torch.float32) * (rank + 1)
        D.allreduce_mean_(g, group, w)
        out["grad"] = g.tolist()
        # 2. coupled loss_i: shard of a global batch of 5 per-image losses (3 on rank 0, 2 on rank 1)
        glob_l = torch.tensor([1e-4, 3e-4, 2e-4, 5e-5, 7e-4])
        sl = D.shard_range(5, rank, w)
        li = glob_l[sl.start:sl.stop].clone()
        Bg = D.global_count(li.shape[0], "cpu", group)
        D.couple_loss_i(li, Bg, group)
        out["Bg"] = Bg
        out["loss_i"] = li.tolist()
        # 3. replicas stay identical: per-rank grads -> mean -> clip -> Adam
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.randn(10)), torch.nn.Parameter(torch.randn(3, 4))]
        opt = torch.optim.Adam(params, lr=1e-2)
        flat = torch.zeros(22)
        params[0].grad = flat[:10].view(10)
        params[1].grad = flat[10:].view(3, 4)
        for step in range(3):
            gen = torch.Generator().manual_seed(100 * rank + step)
            flat.copy_(torch.randn(22, generator=gen) * 5)
            D.allreduce_mean_(flat, group, w)
            torch.nn.utils.clip_grad_norm_(params, 1.0)
            opt.step()
        out["params"] = torch.cat([p.detach().flatten() for p in params]).tolist()
        # 4. the N > 1 bench line's per-rank evidence (bench._rank_stats): gathered before the MAX
        import bench
        out["ranks"] = bench._rank_stats(dist, torch.device("cpu"), 1.0 + rank, 10.0 * (rank + 1), w,
                                         extra=0.25 * rank)
        q.put((rank, out))
    except Exception as e:  # surface failures to the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert "error" not in res[r], res[r]
    exp = (torch.arange(6, dtype=torch.float32) * 1.5).tolist()
    assert res[0]["grad"] == exp and res[1]["grad"] == exp
    assert res[0]["Bg"] == 5 and res[1]["Bg"] == 5
    mean = float(torch.tensor([1e-4, 3e-4, 2e-4, 5e-5, 7e-4]).sum() / 5)
    assert len(res[0]["loss_i"]) + len(res[1]["loss_i"]) == 5
    for r in (0, 1):
        assert all(abs(v - mean) < 1e-10 for v in res[r]["loss_i"])
    assert res[0]["params"] == res[1]["params"]
    rk = res[0]["ranks"]
    assert rk == res[1]["ranks"]
    assert rk["backend"] == "gloo" and rk["world_size"] == 2
    assert rk["rank_elapsed_s"] == [1.0, 2.0] and rk["rank_value"] == [10.0, 10.0]
    assert rk["elapsed_min_s"] == 1.0 and rk["elapsed_max_s"] == 2.0 and rk["imbalance"] == 1.0
    assert rk["rank_extra"] == [0.0, 0.25] and rk["rank_device"] == [-1, -1]


def test_rank_stats_single_process():
    import bench
    rk = bench._rank_stats(None, torch.device("cpu"), 2.0, 64.0, 1)
    assert rk["backend"] is None and rk["world_size"] == 1
    assert rk["rank_value"] == [32.0] and rk["imbalance"] == 0.0


@pytest.mark.parametrize("n,world", [(32, 8), (5, 2), (7, 3), (1, 4)])
def test_shard_range_partition(n, world):
    seen = []
    for r in range(world):
        sl = D.shard_range(n, r, world)
        seen.extend(sl)
        assert len(sl) in (n // world, n // world + 1)
    assert seen == list(range(n))
