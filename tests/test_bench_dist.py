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


def run_bench(tmp_path, config, gpus, extra=(), tag=""):
    img = tmp_path / ("%s_n%d%s.npy" % (config, gpus, tag))
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--config", config, "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--save-image", str(img)] + list(extra)
    env = dict(os.environ, RT0_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    if r.returncode != 0:  # the ranks' own tracebacks, not torch.distributed.run's summary
        lines = [l for l in r.stderr.splitlines() if l.startswith("[rank") or "Error" in l]
        raise AssertionError("bench.py --gpus %d failed:\n%s" % (gpus, "\n".join(lines[-40:]) or r.stderr[-3000:]))
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    sec = tmp_path / ("%s_n%d%s_secondary.npy" % (config, gpus, tag))
    out = json.loads(line)
    out["_secondary_image"] = np.load(sec) if sec.exists() else None
    return out, np.load(img)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c3", "c5"])
def test_bench_two_ranks_match_one(tmp_path, gpu_required, config):
    one, a = run_bench(tmp_path, config, 1)
    two, b = run_bench(tmp_path, config, 2, ["--dist-backend", "gloo"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["dist_backend"] == "gloo"
    assert a.shape == b.shape
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.0
    assert two["scaling"] == "strong"
    assert np.array_equal(a, b), np.abs(a - b).max()


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c4"])
def test_bench_both_scalings_two_ranks(tmp_path, gpu_required, config):
    """At N>1 a progressive workload's line carries both jobs: its default
    (C2 strong: BASELINE's fixed 1024^2 job split N ways; C4 weak: N x spp
    passes, each rank its rows of all of them) as `value`, and the other one
    as secondary_<mode>_Msamples_s.  Both gathered images equal one rank's
    render of the same job bit for bit (spp and 2 x spp passes)."""
    spp = 4
    one, a = run_bench(tmp_path, config, 1, ["--spp", str(spp)])
    one2, a2 = run_bench(tmp_path, config, 1, ["--spp", str(2 * spp)], tag="x2")
    two, b = run_bench(tmp_path, config, 2, ["--dist-backend", "gloo", "--spp", str(spp)])
    default = {"c2": "strong", "c4": "weak"}[config]
    other = "weak" if default == "strong" else "strong"
    assert two["scaling"] == default, two["scaling"]
    assert two["value"] > 0 and two["secondary_%s_Msamples_s" % other] > 0
    assert "job" in two["config"] and "secondary_job" in two["config"]
    assert two["config"]["spp"] == (spp if default == "strong" else 2 * spp)
    b2 = two["_secondary_image"]
    assert b2 is not None
    strong_img, weak_img = (b, b2) if default == "strong" else (b2, b)
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.0
    assert np.array_equal(a, strong_img), np.abs(a - strong_img).max()
    assert np.array_equal(a2, weak_img), np.abs(a2 - weak_img).max()
