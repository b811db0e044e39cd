"""Benchmark: attack-step·images/s on Balle2018-hyperprior q3, 512x768 (BASELINE.json configs[1]);
``--model cheng2020`` measures configs[2]'s per-GPU shard (cheng2020-anchor q6, 32 images of 768x512);
``--config 5`` measures configs[4]'s per-GPU shard: the targeted ROI attack on 2048x2048 tiles on the
bf16-operand MFMA conv path (8 tiles per GPU, target = a second synthetic image, ROI = the centre box).

One "step" = one attack_rd.attack_ iteration over the per-GPU batch: L-inf box
+ input clamp, per-image branch (loss_i > -noise: input loss only, attack_rd.py:334-338), g_a + g_s forward,
loss, g_s + g_a input-gradient backward for the images in the network branch (compacted sub-batch), Adam
on the noise (attack_rd.py:506-559) — every kernel on HIP, inputs resident in HBM.  The line carries the
branch census of the timed steps and (N = 1, hyperprior) of one whole 1001-step run with its wall time.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, weak scaling)

Images shard across GPUs (each rank attacks its own images; no collective on
the data path).  A single scalar MAX all-reduce of the elapsed time is the only
collective.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "attack-step·images/sec, Balle2018-hyper 768×512 1001-step PGD, 1/2/4/8 GPU"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: Peak BF16 MFMA, dense (no sparsity)


def layer_flops(tag, N, M, H, W, B):
    """Algorithmic FLOPs of one launch of a tagged conv kernel (2*MAC, padding not counted).  A '[prec]' suffix
    (hip_ops: the same layer run on other operands, e.g. the fine-tune's fp32 train step) does the same work."""
    name, kind = tag.split("[", 1)[0].rsplit(".", 1)
    lay = {  # (conv type, Cin, Cout, output resolution divisor, gdn channels in epilogue)
        "g_a.0": ("down", 3, N, 2, N), "g_a.2": ("down", N, N, 4, N), "g_a.4": ("down", N, N, 8, N),
        "g_a.6": ("down", N, M, 16, 0),
        "g_s.0": ("up", M, N, 8, N), "g_s.2": ("up", N, N, 4, N), "g_s.4": ("up", N, N, 2, N),
        "g_s.6": ("up", N, 3, 1, 0),
    }[name]
    typ, cin, cout, div, gdn = lay
    out_px = (H // div) * (W // div)
    conv_macs = cin * cout * 25 * out_px / (4 if typ == "up" else 1)
    if kind == "fwd":
        macs = conv_macs + gdn * gdn * out_px
    else:  # dgrad: same conv MACs; GDN-bwd epilogue (one C x C GEMM) at the layer-input resolution
        in_px = out_px * 4 if typ == "down" else out_px // 4
        has_gdn = name not in ("g_a.0", "g_s.0")
        macs = conv_macs + (N * N * in_px if has_gdn else 0)
    return 2.0 * macs * B


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(H, W, quality, seconds, model="hyper", big_batch=32):
    """The CPU oracle (PyTorch-CPU fp32 restatement, kind 'port') timed on this host, bounded to ~`seconds` of
    CPU work per variant:
      * value: one reference attack step on ONE image (the reference attacks one image per call,
        attack_rd.py:646-670), weight gradients computed as the reference does (params require grad);
      * variants: the same step without the unused weight gradients (dgrad only), and one step of a
        ``big_batch``-image batch (the GPU workload's per-GPU batch) with weight gradients."""
    from oracle import codec
    # the box's CPU share (OMP_NUM_THREADS is set to it there); never oversubscribe
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0)))))
    P = codec.init_params(model, quality, seed=0)
    eps = 16 / 255.0

    def make(B, wgrad):
        for v in P.values():
            v.requires_grad_(wgrad)
        g = torch.Generator().manual_seed(0)
        im_s = torch.rand((B, 3, H, W), generator=g)
        with torch.no_grad():
            os_ = torch.clamp(codec.forward(P, im_s[:1], model)["x_hat"], 0, 1).expand(B, -1, -1, -1)
        noise = torch.zeros_like(im_s).requires_grad_(True)
        opt = torch.optim.Adam([noise], lr=0.01)

        def one():
            nc = codec.bound01(noise, -eps, eps)
            im_in = codec.bound01(im_s + nc)
            li = torch.mean((im_s - im_in) ** 2)
            o = codec.bound01(codec.transforms(P, im_in, model))
            loss = 1.0 - torch.mean((os_ - o) ** 2) if li <= 1e-4 else li
            opt.zero_grad()
            for v in P.values():
                v.grad = None
            loss.backward()
            opt.step()
        return one

    def timed(one, B, budget, max_steps=50):
        one()
        t0 = time.perf_counter()
        n = 0
        while True:
            one()
            n += 1
            el = time.perf_counter() - t0
            if el > budget or n >= max_steps:
                break
        return B * n / el, n, el

    v1, n1, e1 = timed(make(1, True), 1, seconds)
    vd, nd, ed = timed(make(1, False), 1, seconds * 0.6)
    one_b = make(big_batch, True)
    t0 = time.perf_counter()
    one_b()
    eb = time.perf_counter() - t0
    vb = big_batch / eb
    return {"value": v1, "unit": "attack-step·images/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"oracle attack step (fwd+bwd incl. weight grads as the reference), 1 image {W}x{H}, "
                      f"{model} q{quality}, {n1} timed steps after 1 warm-up ({e1:.1f} s)",
            "variants": {"b1_dgrad_only": {"value": vd, "sample": f"{nd} steps ({ed:.1f} s), no weight grads"},
                         f"b{big_batch}_with_wgrad": {"value": vb,
                                                      "sample": f"1 step of {big_batch} images ({eb:.1f} s)"}}}


X6_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6.0   # fp32-equivalent ceiling of six bf16 MFMAs per fp32 k-step


def _tag_prec(kern):
    """Operand precision of each tagged conv launch (0 fp32 MFMA, 1 bf16, 2 bf16x6 fp32-accurate)."""
    out = {}
    for tr, pre in ((kern.ga, "g_a"), (kern.gs, "g_s")):
        for i, p in enumerate(tr.convs):
            out[f"{pre}.{2 * i}.fwd"] = p.fwd_prec
            out[f"{pre}.{2 * i}.dgrad"] = p.bwd_prec
    return out


_PREC_NAME = {0: "fp32", 1: "bf16", 2: "x6", 3: "bf16 (fp32 activations)"}


def _peak(prec):
    return {1: BF16_MFMA_PEAK_TFLOPS, 2: X6_PEAK_TFLOPS, 3: BF16_MFMA_PEAK_TFLOPS}.get(prec, FP32_MFMA_PEAK_TFLOPS)


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("ICA_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev, dist


def _rank_stats(dist, dev, el, units, world, extra=None):
    """Per-rank evidence for the N > 1 line (the driver's 8-GPU run): the backend and world size the process group
    actually initialised, every rank's own elapsed time over the timed steps (gathered BEFORE the MAX that sets
    `value`), its device and work units, and the spread.  `extra` (per rank, float): e.g. the fine-tune's
    all-reduce milliseconds per outer step."""
    vals = [float(el), float(units), float(dev.index if dev.index is not None else -1), float(extra or 0.0)]
    if dist is None:
        rows = [vals]
        backend, ws = None, 1
    else:
        backend = str(dist.get_backend())
        # gloo gathers host tensors (its CUDA support covers all_reduce / broadcast only)
        t = torch.tensor(vals, device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rows = [p.tolist() for p in parts]
        ws = dist.get_world_size()
    els = [r[0] for r in rows]
    out = {"backend": backend, "world_size": ws,
           "rank_elapsed_s": [round(e, 4) for e in els],
           "rank_value": [round(r[1] / r[0], 3) if r[0] > 0 else None for r in rows],
           "rank_device": [int(r[2]) for r in rows],
           "elapsed_min_s": round(min(els), 4), "elapsed_max_s": round(max(els), 4),
           "imbalance": round(max(els) / min(els) - 1.0, 4) if min(els) > 0 else None}
    if extra is not None:
        out["rank_extra"] = [round(r[3], 4) for r in rows]
    return out


def _kernel_table(hook, flops_img):
    tot_ms = {tag: sum(a.elapsed_time(b) for a, b, _ in evs) for tag, evs in hook.items()}
    tot_fl = {tag: sum(flops_img[tag] * n for _, _, n in evs) for tag, evs in hook.items()}
    return tot_ms, tot_fl


def _launch_table(launches, rank):
    """{tag: [[kernel, grid_threads], ...]} of the timed launches; written to $ICA_LAUNCH_TABLE (rank 0) for
    scripts/pmc_traffic.py, which matches PMC rows to tags through it."""
    table = {t: sorted([list(k) for k in v if k]) for t, v in (launches or {}).items()}
    path = os.environ.get("ICA_LAUNCH_TABLE")
    if path and rank == 0:
        with open(path, "w") as f:
            json.dump(table, f, indent=1)
    return table


def _traffic(tfile, dom, table):
    """HBM bytes per launch of the dominant tag from the committed PMC file, reported only when its stamp (kernel,
    grid, source hash: scripts/pmc_traffic.py) matches the launch just timed; otherwise None and the reason."""
    from imagecompression_adversarial_amd import hip_ops as K
    if not tfile:
        return None, "no PMC traffic file for this configuration"
    tf = os.path.join(REPO, "profiles", tfile)
    if not os.path.exists(tf):
        return None, f"profiles/{tfile} absent"
    try:
        e = json.load(open(tf)).get(dom)
    except (OSError, ValueError):
        return None, f"profiles/{tfile} unreadable"
    if not isinstance(e, dict):
        return None, f"profiles/{tfile} has no stamped entry for {dom}"
    launched = table.get(dom, [])
    if len(launched) != 1:
        return None, f"{dom} ran {len(launched)} distinct kernels / grids in the timed steps"
    kern, grid = launched[0]
    src = K.source_hash()
    if e.get("kernel") != kern or e.get("grid") != grid or e.get("src") != src:
        return None, (f"stale: profiles/{tfile} measured {e.get('kernel')} grid {e.get('grid')} src {e.get('src')}; "
                      f"timed {kern} grid {grid} src {src}")
    return e["bytes"], f"profiles/{tfile}: {kern}, grid {grid}, src {src}"


def cpu_baseline_finetune(q, metric, lmbda, B, H, W, inner):
    """configs[3] on the CPU oracle (oracle.attack.adv_train_step: coupled inner attack + train-mode RD step + clip +
    Adam + aux Adam).  Not bounded by --cpu-seconds: it always times a warm-up outer step and one outer step each with
    1 and 3 inner steps, on the bench's batch (≈10-20 s on 16 cores); the inner-step time is their difference / 2, the
    rest is the train step, and the rate is an EXTRAPOLATION to an outer step with `inner` inner steps (the same
    accounting as the GPU value: inner image-steps per second of whole outer steps)."""
    from oracle import attack as oa
    from oracle import codec
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0)))))
    P = codec.init_params("hyper", q, seed=0)
    g = torch.Generator().manual_seed(0)
    x = torch.rand((B, 3, H, W), generator=g)
    N, M = codec.model_channels("hyper", q)

    def outer(k):
        ny = torch.rand((B, M, H // 16, W // 16), generator=g) - 0.5
        nz = torch.rand((B, N, H // 64, W // 64), generator=g) - 0.5
        t0 = time.perf_counter()
        oa.adv_train_step(P, x, steps=k, model="hyper", metric=metric, lmbda=lmbda, noise_y=ny, noise_z=nz)
        return time.perf_counter() - t0
    outer(1)   # warm-up
    t1, t3 = outer(1), outer(3)
    t_inner = max((t3 - t1) / 2, 1e-9)
    t_train = max(t1 - t_inner, 0.0)
    t_outer = inner * t_inner + t_train
    return {"value": B * inner / t_outer, "unit": "attack-step·images/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"oracle adv_train_step (train.py:335-366) on {B} x {W}x{H}, hyper q{q}, {metric}: outer steps "
                      f"with 1 and 3 inner steps timed ({t1:.1f} s, {t3:.1f} s): {t_inner:.2f} s per inner step, "
                      f"{t_train:.2f} s train step, extrapolated to {inner} inner steps per outer step "
                      f"({t_outer:.0f} s)"}


def bench_finetune(args):
    """configs[3]: train.py --adv (train.py:335-366) outer steps on this rank's shard: the batch-coupled
    300-step inner attack (a 4-byte all-reduce per inner step), the train-mode RD forward / backward with
    every weight gradient, one flat gradient all-reduce (RCCL over xGMI), clip + Adam + aux Adam.
    Weak scaling: 8 images of 256x256 per GPU (train.py's batch of 8 per rank), hyper q1, ms-ssim
    (the README's fine-tune command), lambda from the train.py table."""
    from types import SimpleNamespace
    world, rank, dev, dist = _dist_env()
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd import coder
    from imagecompression_adversarial_amd import dist as D
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd.train import LAMBS, adv_step
    from imagecompression_adversarial_amd.train_engine import RDTrainer
    q, metric = (args.quality or 1), "ms-ssim"
    B, H, W, inner = 8, 256, 256, 300
    torch.manual_seed(0)
    net = models.bmshj2018_hyperprior(q)
    coder._synthetic_init(net, seed=0)
    net = net.to(dev).train()
    opt, aux = coder.configure_optimizers(net, SimpleNamespace(adv=True, lr_train=1e-4))
    lmbda = LAMBS[metric][q - 1]
    tr = RDTrainer(net, metric, lmbda)
    group = dist.group.WORLD if dist else None
    fprec = net.attack_precision(args.precision)
    fargs = SimpleNamespace(steps=inner, epsilon=16.0, noise=1e-4, lr_attack=0.01, att_metric="L2", clamp=True,
                            round_adv=False, precision=fprec)
    gen = torch.Generator(device=dev).manual_seed(rank)
    xs = [torch.rand((B, 3, H, W), generator=gen, device=dev) for _ in range(args.warmup + args.steps)]
    for i in range(args.warmup):
        adv_step(net, tr, opt, aux, xs[i], fargs, group, world)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    D.COLL_HOOK = {} if dist else None
    from imagecompression_adversarial_amd import attack as A
    g0 = dict(A.GRAPH_STATS)
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        adv_step(net, tr, opt, aux, xs[i], fargs, group, world)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    coll, D.COLL_HOOK = D.COLL_HOOK, None
    # all-reduce time per outer step (HIP events around each collective on the issuing stream)
    coll_ms = {k: sum(a.elapsed_time(b) for a, b in v) / args.steps for k, v in (coll or {}).items()}
    replays = A.GRAPH_STATS["replays"] - g0["replays"]
    captures = A.GRAPH_STATS["captures"] - g0["captures"]
    # Per-kernel times: the timed outer steps replay the inner attack's network step as a HIP graph (one launch per
    # inner step; its kernels carry no events), so ONE more outer step runs right after them with the graph off and
    # every tagged launch bracketed by HIP events: per-launch times, launch counts and the launch table of a whole
    # outer step (the roofline and the PMC stamps refer to these launches, which run the same kernels on the same
    # shapes as the replays).
    graph_on, A.ATTACK_GRAPH = A.ATTACK_GRAPH, False
    K.EVENT_HOOK = {}
    K.FLOPS_HOOK = {}
    K.PREC_HOOK = {}
    K.LAUNCH_HOOK = {}
    adv_step(net, tr, opt, aux, xs[args.warmup], fargs, group, world)
    torch.cuda.synchronize()
    A.ATTACK_GRAPH = graph_on
    hook, K.EVENT_HOOK = K.EVENT_HOOK, None
    table = _launch_table(K.LAUNCH_HOOK, rank)
    K.LAUNCH_HOOK = None
    ranks = _rank_stats(dist, dev, el, B * inner * args.steps, world, extra=coll_ms.get("grad", 0.0) if dist else None)
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    N, M = net.N, net.M
    flops_img = {t: (K.FLOPS_HOOK[t] if t in K.FLOPS_HOOK else layer_flops(t, N, M, H, W, 1)) for t in hook}
    tot_ms, tot_fl = _kernel_table(hook, flops_img)   # one eager outer step
    est_ms = dict(tot_ms)
    dom = max(est_ms, key=est_ms.get)
    wg = [t for t in tot_ms if t.endswith(".wgrad")]
    wdom = max(wg, key=tot_ms.get) if wg else None

    def roof(tag):
        if tag is None:
            return None
        ach = tot_fl[tag] / (tot_ms[tag] * 1e-3) / 1e12
        pk = _peak(K.PREC_HOOK.get(tag, 0))   # the operands that tag's launches ran on
        traffic, tnote = _traffic("pmc_traffic_c4.json", tag, table)
        return {"bound": "mfma", "kernel": tag, "achieved": round(ach, 2), "peak": pk,
                "unit": "TFLOP/s", "frac": round(ach / pk, 4), "traffic": traffic, "traffic_source": tnote,
                "operands": _PREC_NAME[K.PREC_HOOK.get(tag, 0)],
                "launch_ms": round(tot_ms[tag] / len(hook[tag]), 4),
                "flops_per_launch": tot_fl[tag] / len(hook[tag])}
    ms_outer = el / args.steps * 1e3
    value = B * world * inner * args.steps / el
    if rank == 0:
        out = {
            "metric": "attack-step·images/sec, train.py --adv fine-tune (configs[3]): inner attack image-steps per "
                      "second over whole outer steps (inner attack + RD train step + grad all-reduce + Adam)",
            "value": round(value, 3), "unit": "attack-step·images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_outer, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("f32 (inner attack: fp32-accurate x6 operands on the large layers, fp32 MFMA on the small-grid "
                      "ones; train step fp32 MFMA)" if fprec == "x6" else "f32"),
            "data": "synthetic (torch.rand 256x256 crops, seeded CompressAI-init weights)",
            "config": {"workload": f"train.py --adv -m hyper -q {q} -metric {metric} -steps {inner} -lamb {lmbda}, "
                                   f"{B} images/GPU of {W}x{H}, one outer step per timed step",
                       "per_gpu_batch": B, "global_batch": B * world, "height": H, "width": W,
                       "parallelism": f"data-parallel x{world}, one flat grad all-reduce per outer step"},
            "outer_steps_per_s": round(args.steps / el, 4),
            "distributed": dict(ranks, **({"allreduce_ms_per_outer_step": {k: round(v, 4) for k, v in coll_ms.items()},
                                           "rank_extra_is": "flat-gradient all-reduce ms per outer step"}
                                          if dist else {})),
            "roofline": roof(dom), "wgrad_roofline": roof(wdom),
            "per_kernel_ms_total_per_outer_step": {k: round(v, 3) for k, v in sorted(est_ms.items())},
            "attack_graph": {"captures_per_outer_step": round(captures / args.steps, 3),
                             "replays_per_outer_step": round(replays / args.steps, 3),
                             "note": "timed steps replay the inner network step as a HIP graph; per-kernel times, "
                                     "roofline and launch table from one eager outer step run after them"},
            "cpu_baseline": (None if world > 1 or args.no_cpu_baseline else
                             cpu_baseline_finetune(q, metric, lmbda, B, H, W, inner)),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=768)
    ap.add_argument("--quality", type=int, default=None, help="default 3 (hyper) / 6 (cheng2020)")
    ap.add_argument("--model", default="hyper", choices=("hyper", "cheng2020"))
    ap.add_argument("--precision", default=None, choices=("fp32", "x6", "bf16"),
                    help="conv operand precision of g_a/g_s: x6 (default: fp32-accurate bf16x6 split-operand "
                         "MFMA), fp32 (fp32-operand MFMA; cheng2020 default), bf16 (config 5 default)")
    ap.add_argument("--config", type=int, default=None, choices=(2, 3, 4, 5),
                    help="BASELINE.json configs[k-1] per-GPU shard: 2 hyper q3 fp32 (default), 3 cheng2020 q6, "
                         "4 train.py --adv fine-tune outer steps (8 x 256^2 per GPU, 300 inner steps, RCCL grad "
                         "all-reduce), 5 targeted ROI hyper q3 2048x2048 bf16")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mixed", type=float, default=None, metavar="SCALE",
                    help="also time one whole 1001-step run with g_a's last weight scaled by SCALE (40: O(1) latents "
                         "as a trained codec has, so the run hovers at the -noise budget and both branches occur; "
                         "make_golden.py TRAJ100) and report its branch census, rate and host branch-read cost "
                         "next to the (unchanged, all-network-branch) headline")
    ap.add_argument("--full-run", dest="full_run", type=int, default=None,
                    help="1: also run the whole 1001-step loop once (wall time + branch census of the full run); "
                         "default 1 for the hyperprior configs at N = 1, 0 for cheng2020 (~7 min)")
    args = ap.parse_args()

    if args.config == 4:
        return bench_finetune(args)
    roi_mode = False
    if args.full_run is None:
        args.full_run = int(args.config != 3 and args.model != "cheng2020")
    if args.config == 3:
        args.model = "cheng2020"
    elif args.config == 5:
        roi_mode = True
        args.height = args.width = 2048
        if args.batch == 32:
            args.batch = 8
        if args.precision is None:
            args.precision = "bf16"
    if args.precision is None:   # the attack engine's default: x6 (fp32-accurate)
        args.precision = "x6"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ICA_BENCH_DIST_BACKEND=gloo rehearses the N>1 path with every rank on the box's GPUs modulo their
    # count (one-GPU boxes); the driver's multi-GPU runs use the default, RCCL with one GPU per rank
    backend = os.environ.get("ICA_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from imagecompression_adversarial_amd import attack as A
    from imagecompression_adversarial_amd import codec as models
    from imagecompression_adversarial_amd import hip_ops as K
    from imagecompression_adversarial_amd.attack import AttackLoop
    # the timed steps run the product path: the whole-batch network step replayed as a HIP graph (attack.py; also
    # for the ROI attack), no timing hooks.  ICA_BENCH_GRAPH=0 times them eager (A/B).  Per-kernel times, the
    # roofline and the launch table come from a profiling pass right after the timed region: the same number of
    # eager steps with every tagged launch bracketed by HIP events.
    A.ATTACK_GRAPH = A.ATTACK_GRAPH and os.environ.get("ICA_BENCH_GRAPH", "1") != "0"
    from imagecompression_adversarial_amd.engine import CodecKernels
    from imagecompression_adversarial_amd.engine_cheng import ChengKernels

    H, W, B = args.height, args.width, args.batch
    model = args.model
    if args.quality is None:
        args.quality = 6 if model == "cheng2020" else 3
    # random-init CompressAI-architecture weights (seed 0; no checkpoints offline), product modules
    torch.manual_seed(0)
    net = models.cheng2020_anchor(args.quality) if model == "cheng2020" else models.bmshj2018_hyperprior(args.quality)
    sd = {k: v.detach().to(dev) for k, v in net.state_dict().items()}
    kern = (ChengKernels(sd, precision=args.precision) if model == "cheng2020"
            else CodecKernels(sd, "hyper", precision=args.precision))
    N, M = kern.N, kern.M
    gen = torch.Generator(device=dev).manual_seed(rank)
    im_s = torch.rand((B, 3, H, W), generator=gen, device=dev)
    roi_kw = {}
    if roi_mode:   # README "attack with ROI": -t target, --mask_loc x0 x1 y0 y1 (centre box), la_* defaults
        roi_kw = dict(target=torch.rand((B, 3, H, W), generator=gen, device=dev),
                      roi=(W // 4, 3 * W // 4, H // 4, 3 * H // 4), la_tar=1.0, la_bkg_in=1.0, la_bkg_out=1.0)
    loop = AttackLoop(kern, im_s, steps=1001, **roi_kw)

    for i in range(args.warmup):
        loop.step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    exp0, rep0 = loop.expensive_image_steps(), loop.graph_replays
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        loop.step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    exp_steps = loop.expensive_image_steps() - exp0   # image-steps of the timed window that ran the network
    graph_replays = loop.graph_replays - rep0
    # profiling pass: as many eager steps, every tagged launch timed by HIP events on its stream
    graph_ok, loop.graph_ok = loop.graph_ok, False
    K.EVENT_HOOK = {}
    K.PREC_HOOK = {}
    K.FLOPS_HOOK = {}
    K.LAUNCH_HOOK = {}
    exp1 = loop.expensive_image_steps()
    for j in range(args.steps):
        loop.step(min(args.warmup + args.steps + j, 1000))
    torch.cuda.synchronize()
    loop.graph_ok = graph_ok
    prof_exp = loop.expensive_image_steps() - exp1
    hook, K.EVENT_HOOK = K.EVENT_HOOK, None
    table = _launch_table(K.LAUNCH_HOOK, rank)
    K.LAUNCH_HOOK = None
    ranks = _rank_stats(dist, dev, el, B * args.steps, world)
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # per-kernel durations (HIP events on the launch stream) and algorithmic FLOPs of every launch: a launch
    # covers the images of its (compacted) batch, so the FLOPs are per-image FLOPs x the launch's images
    if model == "cheng2020":   # per-image algorithmic FLOPs recorded by hip_ops.conv_ex
        flops_img = dict(K.FLOPS_HOOK)
    else:
        flops_img = {t: layer_flops(t, N, M, H, W, 1) for t in hook}
    tot_ms = {tag: sum(a.elapsed_time(b) for a, b, _ in evs) for tag, evs in hook.items()}
    tot_fl = {tag: sum(flops_img[tag] * n for _, _, n in evs) for tag, evs in hook.items()}
    per_tag = {tag: tot_ms[tag] / len(hook[tag]) for tag in hook}
    dom = max(tot_ms, key=tot_ms.get) if tot_ms else None
    dom_ms = per_tag[dom] if dom else 0.0
    dom_flops = tot_fl[dom] / len(hook[dom]) if dom else 0.0
    achieved = tot_fl[dom] / (tot_ms[dom] * 1e-3) / 1e12 if dom else 0.0
    tag_prec = (dict(K.PREC_HOOK) or _tag_prec(kern)) if model == "hyper" else dict(K.PREC_HOOK)
    peak = _peak(tag_prec.get(dom, 0))
    # HBM bytes per launch of the dominant kernel from the committed PMC passes of the same shapes
    # (scripts/gpu_pmc.sh + scripts/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE per the gfx950 correction), only
    # when the file's stamp names the kernel, grid and sources just timed
    tfile = None
    if args.precision == "x6" and not roi_mode and (H, W, B) == (512, 768, 32) and model == "hyper":
        tfile = "pmc_traffic_x6.json"
    elif args.precision == "fp32" and not roi_mode and (H, W, B) == (512, 768, 32) and model == "hyper":
        tfile = "pmc_traffic.json"
    elif args.precision == "bf16" and (H, W, B) == (2048, 2048, 8):
        tfile = "pmc_traffic_c5.json"
    elif args.precision == "x6" and not roi_mode and (H, W, B) == (512, 768, 32) and model == "cheng2020":
        tfile = "pmc_traffic_c3x6.json"
    traffic, traffic_note = _traffic(tfile, dom, table) if dom else (None, "no tagged launch")
    # network FLOPs per timed step, weighted by the branches actually taken (a cheap-branch
    # image-step runs no network and counts 0): the launches only covered the expensive images
    total_flops = sum(tot_fl.values()) / args.steps
    ms_step = el / args.steps * 1e3
    value = B * world * args.steps / el

    # the whole 1001-step loop once (N == 1): wall time, img-step/s and the branch census of the full run
    full = None
    if world == 1 and args.full_run:
        loop2 = AttackLoop(kern, im_s, steps=1001, **roi_kw)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(1001):
            loop2.step(i)
        torch.cuda.synchronize()
        fe = time.perf_counter() - t1
        fx = loop2.expensive_image_steps()
        full = {"steps": 1001, "wall_s": round(fe, 3), "value": round(B * 1001 / fe, 3),
                "expensive_image_steps": fx, "image_steps": B * 1001,
                "expensive_frac": round(fx / (B * 1001), 4)}
        del loop2

    # mixed branches (N == 1, hyperprior): trained-scale latents, one whole 1001-step run
    mixed = None
    if world == 1 and args.mixed and model == "hyper":
        sd2 = dict(sd)
        sd2["g_a.6.weight"] = sd["g_a.6.weight"] * float(args.mixed)
        kern2 = CodecKernels(sd2, "hyper", precision=args.precision)
        loop3 = AttackLoop(kern2, im_s, steps=1001, **roi_kw)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(1001):
            loop3.step(i)
        torch.cuda.synchronize()
        fe = time.perf_counter() - t1
        fx = loop3.expensive_image_steps()
        mixed = {"weight_scale": args.mixed, "steps": 1001, "wall_s": round(fe, 3),
                 "value": round(B * 1001 / fe, 3), "expensive_image_steps": fx, "image_steps": B * 1001,
                 "expensive_frac": round(fx / (B * 1001), 4),
                 "steps_waiting_for_branch_read": loop3.sync_steps,
                 "branch_read_wait_s": round(loop3.sync_wait_s, 3),
                 "ms_per_step": round(fe / 1001 * 1e3, 3)}
        del loop3, kern2

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # cheng2020 and the 2048x2048 tiles take seconds per image-step on the CPU: their batch variant is 4 / 2
            # images, not the GPU's batch (the sample stays at ~1 min of CPU work)
            cpu = cpu_baseline(H, W, args.quality, args.cpu_seconds, model,
                               big_batch=4 if model == "cheng2020" else (2 if roi_mode else 32))
        metric = METRIC if model == "hyper" else \
            "attack-step·images/sec, Cheng2020-anchor q6 768×512 (configs[2] per-GPU shard)"
        if roi_mode:
            metric = "attack-step·images/sec, targeted ROI attack Balle2018-hyper 2048×2048 bf16 (configs[4] per-GPU shard)"
        name = "hyper" if model == "hyper" else "cheng2020"
        out = {
            "metric": metric, "value": round(value, 3), "unit": "attack-step·images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": {"bf16": ("bf16 operands, f32 accumulate" if model == "hyper" else
                               "bf16 operands over f32 activations on the k3 conv_downs, f32 accumulate"),
                      "x6": "f32 (fp32-accurate: exact 3-way bf16 operand splits, 6 MFMA products, f32 accumulate)",
                      }.get(args.precision, "f32"),
            "data": "synthetic (torch.rand images, seeded CompressAI-init weights)",
            "config": {"workload": (f"attack_rd -m {name} -q {args.quality} -att_metric L2 -noise 1e-4"
                                    + (f" -t <target> --mask_loc {W // 4} {3 * W // 4} {H // 4} {3 * H // 4}"
                                       if roi_mode else "")
                                    + f", {B} images/GPU of {W}x{H}, steps of the 1001-step loop, "
                                      f"{args.precision} conv operands"),
                       "per_gpu_batch": B, "global_batch": B * world, "height": H, "width": W,
                       "parallelism": f"image-shard x{world} (no data-path collective)"},
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2),
                         "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": traffic_note,
                         "launch_ms": round(dom_ms, 4), "flops_per_launch": dom_flops},
            "branch_census": {"expensive_image_steps": exp_steps, "image_steps": B * args.steps,
                              "expensive_frac": round(exp_steps / (B * args.steps), 4)},
            "timing": {"timed_steps": ("network step replayed as a HIP graph (product default)" if graph_replays
                                       else "eager"),
                       "graph_replays": graph_replays,
                       "per_kernel_source": f"profiling pass: {args.steps} eager steps right after the timed region, "
                                            "every tagged launch bracketed by HIP events on its stream",
                       "profiling_pass_expensive_image_steps": prof_exp},
            "distributed": ranks,
            "full_run": full,
            "mixed_branch_run": mixed,
            "step_gflop_per_image": round(total_flops / B / 1e9, 2),
            "step_tflops": round(total_flops / (ms_step * 1e-3) / 1e12, 2),
            "step_roofline_frac": round(total_flops / (ms_step * 1e-3) / 1e12 /
                                        _peak({"bf16": 1, "x6": 2}.get(args.precision, 0)),
                                        4),
            "per_kernel_ms": {k: round(v, 4) for k, v in sorted(per_tag.items())},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
