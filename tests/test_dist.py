"""The N>1 path on CPU: world_size-2/3 gloo process groups run the same
band pack -> gather -> unpack code bench.py runs over RCCL, with accumulators
whose owned bands hold rank-specific values; rank 0 must reassemble the
exact image (bitwise)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rt0.shard as shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _expected(H, W, band):
    img = torch.arange(H * W * 4, dtype=torch.float32).reshape(H, W, 4)
    return img


def _worker(rank, world, port, H, W, band, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _expected(H, W, band)
        acc = torch.zeros_like(full)
        nb = H // band
        for b in shard.owned_bands(rank, world, nb):
            acc[b * band:(b + 1) * band] = full[b * band:(b + 1) * band]
        img = shard.gather_image(acc, rank, world, band)
        if rank == 0:
            q.put(bool(torch.equal(img, full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 64), (3, 80)])
def test_band_gather_reassembles_image(world, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, 24, 16, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def test_band_ownership_partitions_rows():
    for world in (1, 2, 3, 4, 8):
        nb = 64
        seen = sorted(b for r in range(world) for b in shard.owned_bands(r, world, nb))
        assert seen == list(range(nb))
