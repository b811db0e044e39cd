"""The attack_rd CLI sharded over torchrun ranks on the HIP path (SURVEY §8e attack row): two ranks (gloo
process group, both on the box's GPU) print the same per-image lines and AVG line as one process, and the
targeted mode's PNGs (-t) are byte-identical.  Per-image semantics make every image's attack independent of
which rank runs it, so the comparison is exact (wall-clock fields aside)."""
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import REPO
from tests.test_cpu_attack_cli import _strip_time

pytestmark = pytest.mark.gpu

CLI = ["-m", "imagecompression_adversarial_amd.attack_rd", "-m", "hyper", "-q", "3", "-s", "synthetic:3x64x64",
       "--synthetic-weights", "-steps", "3", "-t", "synthetic"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, cwd):
    env = dict(os.environ, PYTHONPATH=REPO, ICA_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _result_lines(out):
    return [ln for ln in _strip_time(out) if ln.startswith(("synthetic_", "AVG:"))]


def test_two_rank_cli_matches_one_rank(tmp_path):
    d1, d2 = tmp_path / "one", tmp_path / "two"
    d1.mkdir()
    d2.mkdir()
    one = _run([sys.executable] + CLI, str(d1))
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port())] + CLI, str(d2))
    l1, l2 = _result_lines(one), _result_lines(two)
    assert len(l1) == 4 and l1 == l2, (l1, l2)
    pngs = sorted(os.listdir(d1))
    assert len(pngs) == 9 and pngs == sorted(os.listdir(d2))
    for f in pngs:
        assert (d1 / f).read_bytes() == (d2 / f).read_bytes(), f


def test_debug_model_cli(tmp_path):
    """attack_rd -m debug (ae_onelayer, anchors/model.py:61-68) end to end on the HIP path: seeded synthetic weights
    (the model has none to download), per-image lines and the AVG line."""
    cli = ["-m", "imagecompression_adversarial_amd.attack_rd", "-m", "debug", "-q", "3", "-s", "synthetic:2x64x64",
           "--synthetic-weights", "-steps", "3"]
    out = _run([sys.executable] + cli, str(tmp_path))
    lines = _result_lines(out)
    assert len(lines) == 3 and lines[-1].startswith("AVG:"), out[-2000:]
