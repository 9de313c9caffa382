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


def test_gather_pads_a_partial_last_band():
    """Contiguous-block sharding (ReSTIR) uses bands that need not divide H."""
    H, W, world = 40, 8, 3
    band = shard.block_band(H, world)
    full = _expected(H, W, band)
    parts = []
    for rank in range(world):
        lo, hi = shard.block_rows(rank, band, H)
        acc = torch.zeros_like(full)
        acc[lo:hi] = full[lo:hi]
        parts.append(acc)
    # single-process check of pack/unpack with padding (gather_image's local part)
    pad = (-H) % band
    padded = [torch.cat([p, p.new_zeros((pad, W, 4))]) for p in parts]
    sends = [shard.pack(p, r, world, band) for r, p in enumerate(padded)]
    img = shard.unpack(sends, world, band, torch.zeros_like(padded[0]))[:H]
    assert torch.equal(img, full)


def _halo_cases():
    """(H, world, band, halo): contiguous blocks (band = block_band) and
    round-robin bands (interleaved_band, several per rank)."""
    for H, world, halo in ((96, 3, 24), (1080, 8, 24), (40, 3, 16), (64, 8, 16)):
        yield H, world, shard.block_band(H, world), halo
    for H, world, halo in ((192, 2, 24), (1080, 8, 24), (4096, 8, 24), (200, 3, 16), (1080, 3, 24)):
        yield H, world, shard.interleaved_band(H, world, halo=halo), halo
    # bench.py's four bands per rank (C5 at N=8: 128-row bands)
    for H, world, halo in ((4096, 8, 24), (4096, 4, 24), (2048, 2, 24)):
        yield H, world, shard.interleaved_band(H, world, per_rank=4, halo=halo), halo


def test_cost_cuts_equal_cost_blocks():
    """shard.cost_cuts: contiguous blocks of equal measured cost, aligned to
    16 rows, every block non-empty, covering the image."""
    cuts = shard.cost_cuts([1, 1, 1, 1, 4, 4, 1, 1], 512, 4096, 4)
    assert cuts == [0, 1792, 2432, 2880, 4096]
    assert shard.cost_cuts([1.0] * 64, 64, 4096, 8) == [512 * k for k in range(9)]
    # a cost spike in one band: blocks stay >= 16 rows and in order
    c = shard.cost_cuts([0.0] * 10 + [100.0] + [0.0] * 53, 64, 4096, 8)
    assert c[0] == 0 and c[-1] == 4096 and all(b - a >= 16 and a % 16 == 0 for a, b in zip(c, c[1:]))


def test_halo_plan_pairs_sends_with_recvs():
    for H, world, band, halo in _halo_cases():
        plans = {r: shard.halo_plan(r, world, band, H, min(halo, band)) for r in range(world)}
        for r, plan in plans.items():
            own = shard.owned_band_rows(r, world, band, H)
            for kind, peer, r0, r1 in plan:
                other = "recv" if kind == "send" else "send"
                # the transfers between two ranks pair up in posting order
                mine = [p[2:] for p in plan if p[0] == kind and p[1] == peer]
                theirs = [p[2:] for p in plans[peer] if p[0] == other and p[1] == r]
                assert mine == theirs
                inside = [lo <= r0 < r1 <= hi for lo, hi in own]
                if kind == "send":
                    assert any(inside)  # only own rows leave a rank
                else:
                    assert all(r1 <= lo or r0 >= hi for lo, hi in own)  # received rows are not own rows
            # every row within `halo` of an own band is own or received
            got = set(y for lo, hi in own for y in range(lo, hi))
            got |= set(y for k, _, r0, r1 in plan if k == "recv" for y in range(r0, r1))
            need = set(y for lo, hi in own for y in range(max(0, lo - halo), min(H, hi + halo)))
            assert need <= got, (H, world, band, halo, r)


def _halo_worker(rank, world, port, H, W, halo, q, band=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        band = band or shard.block_band(H, world)
        own = shard.owned_band_rows(rank, world, band, H)
        full = [_expected(H, W, band) + k * 1e6 for k in range(2)]
        planes = [torch.full_like(f, -1.0) for f in full]
        for p, f in zip(planes, full):
            for lo, hi in own:
                p[lo:hi] = f[lo:hi]
        shard.exchange_halo(planes, rank, world, band, halo)
        valid = torch.zeros(H, dtype=torch.bool)
        for lo, hi in own:
            valid[max(0, lo - halo):min(H, hi + halo)] = True
        ok = all(torch.equal(p[valid], f[valid]) for p, f in zip(planes, full))
        # rows beyond the halos are untouched
        ok = ok and all(bool((p[~valid] == -1).all()) for p in planes)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,halo,band", [(2, 64, 16, None), (3, 96, 24, None), (2, 192, 24, 48), (3, 200, 16, 32)])
def test_restir_halo_exchange_over_gloo(world, H, halo, band):
    """The point-to-point halo exchange of sharded ReSTIR (the RCCL code path
    on GPUs) delivers exactly the neighbours' rows on every rank: contiguous
    blocks (band None) and round-robin bands."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, H, 12, halo, q, band)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def _worker_compact(rank, world, port, H, W, band, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _expected(H, W, band)
        g = shard.BandGather(H, W, rank, world, band, "cpu")
        nb = (H + band - 1) // band
        # what a shard renders into its band-packed accumulator: its bands in order
        for j, b in enumerate(shard.owned_bands(rank, world, nb)):
            rows = full[b * band:(b + 1) * band]
            g.acc[j * band:j * band + rows.shape[0]] = rows
        for _ in range(2):  # the buffers are reused step after step
            img = g.gather()
        if rank == 0:
            q.put(bool(torch.equal(img, full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 64), (3, 80), (4, 64)])
def test_band_packed_gather_reassembles_image(world, H):
    """bench.py's multi-GPU step: band-packed accumulators -> one gather -> one
    index_copy_ on rank 0 == the full image, bitwise (uneven ownership too)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_compact, args=(r, world, port, H, 24, 16, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def _worker_block(rank, world, port, H, W, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        band = shard.block_band(H, world)
        full = _expected(H, W, band)
        g = shard.BandGather(H, W, rank, world, band, "cpu")
        # bench.py's ReSTIR layout: a full-size accumulator padded to world x band
        # rows, only this rank's block rendered; the block is the send buffer
        acc = torch.zeros((world * band, W, 4))
        lo, hi = shard.block_rows(rank, band, H)
        acc[lo:hi] = full[lo:hi]
        for _ in range(2):
            img = g.gather(acc[rank * band:(rank + 1) * band])
        if rank == 0:
            q.put(bool(torch.equal(img, full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 64), (3, 80)])
def test_block_gather_reassembles_image(world, H):
    """bench.py's sharded-ReSTIR step end: contiguous row blocks (a short last
    block included) -> one gather into the preallocated buffer == the image."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_block, args=(r, world, port, H, 12, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


def _restir_gather_worker(rank, world, port, H, W, q):
    """bench.py's Restir gather at N > 1: the rank's round-robin bands of a
    full-size (band-padded) accumulator packed with one index_select into a
    send buffer of the gather's row count, then BandGather."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        band = shard.interleaved_band(H, world)
        nb = (H + band - 1) // band
        full = _expected(H, W, band)
        acc = torch.full((nb * band, W, 4), -1.0)
        own = shard.owned_band_rows(rank, world, band, H)
        for lo, hi in own:
            acc[lo:hi] = full[lo:hi]
        g = shard.BandGather(H, W, rank, world, band, "cpu")
        rows = torch.tensor([y for lo, _ in own for y in range(lo, lo + band)], dtype=torch.long)
        send_buf = torch.zeros((g.rows, W, 4))
        torch.index_select(acc, 0, rows, out=send_buf[:len(rows)])
        img = g.gather(send_buf)
        q.put((rank, True if rank != 0 else bool(torch.equal(img, full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 200), (3, 1080), (4, 512)])
def test_restir_round_robin_gather_over_gloo(world, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_restir_gather_worker, args=(r, world, port, H, 6, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res
