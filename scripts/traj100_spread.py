"""How far fp32 rounding alone moves the 100-step traj100 trajectories (tests/golden/traj100.npz), measured on the
CPU oracle (the reference's algorithm restated; the checker, not the product):
  * the same run with weights / input image perturbed by one fp32 ulp (random sign per element, several seeds);
  * the same run on 1 thread vs the default thread count (another fp32 summation order).
For each variant: the first step whose branch differs from the reference's, and the final-noise difference
(max and 99.9th percentile of |noise - noise_ref| / max|noise_ref|).  This calibrates the bounds of
tests/test_traj100.py: a HIP path whose trajectory stays inside this spread is as close to the reference as
another fp32 evaluation of the same algorithm.

    python scripts/traj100_spread.py [n_seeds] > profiles/r03/traj100_spread.txt
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import attack as oatt  # noqa: E402
from oracle import codec  # noqa: E402


def params(scale):
    P = codec.perturb_params(codec.init_params("hyper", 1, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * float(scale)
    return P


def image():
    g = torch.Generator().manual_seed(101)
    return torch.rand((1, 3, 256, 256), generator=g)


def ulp_perturb(t, seed):
    g = torch.Generator().manual_seed(seed)
    sign = torch.randint(0, 2, t.shape, generator=g).to(torch.int32) * 2 - 1
    bits = t.contiguous().view(torch.int32)
    out = (bits + sign * (bits != 0).to(torch.int32)).view(torch.float32)
    return out


def run(P, x, nthreads=None):
    if nthreads:
        torch.set_num_threads(nthreads)
    rec = []
    r = oatt.attack(P, x, steps=100, record=rec, eval_msssim=False)
    br = [int(bool(d["cheap"][0])) for d in rec]
    return br, r.noise.numpy()


def main():
    nseed = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    t100 = np.load(os.path.join(REPO, "tests", "golden", "traj100.npz"))
    default_threads = min(8, os.cpu_count() or 1)
    for tag in ("t100a", "t100b"):
        ref_br = [int(v) for v in t100[f"{tag}_branch"]]
        ref_n = t100[f"{tag}_noise"]
        scale = np.abs(ref_n).max()

        def report(name, br, nz):
            div = next((i for i in range(100) if br[i] != ref_br[i]), 100)
            d = np.abs(nz - ref_n) / scale
            print(f"{tag} {name:28s} branch identical {div:3d}/100  final noise max {d.max():.3e}  "
                  f"p99.9 {np.quantile(d, 0.999):.3e}", flush=True)

        P0, x0 = params(t100[f"{tag}_scale"]), image()
        report("oracle, default threads", *run(P0, x0, default_threads))
        report("oracle, 1 thread", *run(P0, x0, 1))
        torch.set_num_threads(default_threads)
        for s in range(nseed):
            Pp = {k: ulp_perturb(v, 1000 + 17 * s + i) for i, (k, v) in enumerate(sorted(P0.items()))}
            report(f"weights +-1 ulp (seed {s})", *run(Pp, x0))
            report(f"image +-1 ulp (seed {s})", *run(P0, ulp_perturb(x0, 5000 + s)))


if __name__ == "__main__":
    main()
