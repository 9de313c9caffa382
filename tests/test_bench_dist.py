"""bench.py's N>1 path, executed end to end on one GPU.

`bench.py --gpus 2` relaunches itself under torch.distributed.run; with
`--dist-backend gloo` every transfer (band gather, ReSTIR halo exchange) is
staged through host memory, and RT0_BENCH_DEVICE=0 puts both ranks on the one
device of a one-GPU box.  Everything else -- the band split, band-packed
accumulators, round-robin ReSTIR bands, the event ordering between librt0's
stream and torch's, the gather's reorder -- is the code the 8-GPU RCCL run
executes.  Rank 0's gathered image must equal the N=1 image bit for bit
(pixels are independent in progressive mode; sharded ReSTIR reads only the
exchanged halo rows, which hold the same values as the whole image's).  C5
adds the triangle model: each rank's light-sampling kernel queues its own
occlusion walks.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def run_bench(tmp_path, config, gpus, extra=()):
    img = tmp_path / ("%s_n%d.npy" % (config, gpus))
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--config", config, "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--save-image", str(img)] + list(extra)
    env = dict(os.environ, RT0_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    if r.returncode != 0:  # the ranks' own tracebacks, not torch.distributed.run's summary
        lines = [l for l in r.stderr.splitlines() if l.startswith("[rank") or "Error" in l]
        raise AssertionError("bench.py --gpus %d failed:\n%s" % (gpus, "\n".join(lines[-40:]) or r.stderr[-3000:]))
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), np.load(img)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c3", "c5"])
def test_bench_two_ranks_match_one(tmp_path, gpu_required, config):
    one, a = run_bench(tmp_path, config, 1)
    two, b = run_bench(tmp_path, config, 2, ["--dist-backend", "gloo", "--scaling", "strong"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["dist_backend"] == "gloo"
    assert a.shape == b.shape
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.0
    assert np.array_equal(a, b), np.abs(a - b).max()


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c4"])
def test_bench_weak_scaling_two_ranks(tmp_path, gpu_required, config):
    """The default N>1 step of a progressive workload (weak scaling): N x spp
    passes, each rank rendering its rows for all of them -- the gathered image
    equals one rank rendering 2 x spp passes, bit for bit, and the line says
    "weak" with the samples of the whole job."""
    spp = 4
    one, a = run_bench(tmp_path, config, 1, ["--spp", str(2 * spp)])
    two, b = run_bench(tmp_path, config, 2, ["--dist-backend", "gloo", "--spp", str(spp)])
    assert two["scaling"] == "weak" and two["config"]["spp"] == 2 * spp == one["config"]["spp"]
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.0
    assert np.array_equal(a, b), np.abs(a - b).max()
