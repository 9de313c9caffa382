"""Multi-GPU pixel sharding: 16-row bands dealt round-robin over ranks, one
gather of the HDR accumulator bands to rank 0 (RCCL over xGMI with the "nccl"
backend; gloo on CPU for tests).

Why bands: Cornell cost varies strongly by image region (the light and the
boxes), so contiguous halves would load-balance badly; 16-row bands dealt
round-robin give every rank a statistically equal slice, and each band is a
whole number of 16x16 workgroup tiles.  Pixels are independent in progressive
mode without ReSTIR (raytracer.glsl:2120, 2168), so the only exchange is the
final gather: (N-1)/N of W*H*16 bytes, each peer sending its own slice to
rank 0 over its own xGMI link.
"""


def owned_bands(rank, world, n_bands):
    return [b for b in range(n_bands) if b % world == rank]


def pack(acc, rank, world, band):
    """acc: [H, W, 4] tensor (full image, only owned bands valid) ->
    [max_owned, band, W, 4] contiguous send buffer (zero-padded)."""
    import torch
    H, W = acc.shape[0], acc.shape[1]
    nb = (H + band - 1) // band
    own = owned_bands(rank, world, nb)
    max_owned = (nb + world - 1) // world
    send = torch.zeros((max_owned, band, W, acc.shape[2]), dtype=acc.dtype, device=acc.device)
    if own:
        idx = torch.tensor(own, device=acc.device)
        send[:len(own)] = acc.view(nb, band, W, acc.shape[2]).index_select(0, idx)
    return send


def unpack(gathered, world, band, image):
    """gathered[src] = pack() of rank src -> writes every band into image [H, W, 4]."""
    import torch
    H, W = image.shape[0], image.shape[1]
    nb = (H + band - 1) // band
    view = image.view(nb, band, W, image.shape[2])
    for src in range(world):
        own = owned_bands(src, world, nb)
        if own:
            view[torch.tensor(own, device=image.device)] = gathered[src][:len(own)]
    return image


def gather_image(acc, rank, world, band, image=None, bufs=None):
    """Collective: every rank passes its accumulator; rank 0 returns the
    assembled [H, W, 4] image (others return None).  A partial last band is
    padded for the transfer."""
    import torch
    import torch.distributed as dist
    H = acc.shape[0]
    pad = (-H) % band
    if pad:
        acc = torch.cat([acc, acc.new_zeros((pad,) + tuple(acc.shape[1:]))])
    send = pack(acc, rank, world, band)
    if rank == 0:
        bufs = bufs if bufs is not None else [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, bufs, dst=0)
        full = torch.zeros_like(acc) if (image is None or pad) else image
        full = unpack(bufs, world, band, full)
        if pad:
            if image is None:
                return full[:H].clone()
            image.copy_(full[:H])
            return image
        return full
    dist.gather(send, None, dst=0)
    return None


class StreamOrder:
    """Orders librt0's stream (rt0_device_accum) against torch's current stream
    with events, so that a producer on one and a consumer on the other need no
    host synchronisation: torch_after_rt0() before torch work that reads what
    librt0 wrote (exchanges, gathers), rt0_after_torch() before a librt0
    launch that reads what torch wrote (a zeroed accumulator, received halo
    rows).  Also times a torch-stream interval (begin/end_timing)."""

    def __init__(self, renderer, device):
        import torch
        _, stream = renderer.device_accum()
        self.torch = torch
        self.ext = torch.cuda.ExternalStream(stream, device=device)
        self.ev_rt0 = torch.cuda.Event()
        self.ev_torch = torch.cuda.Event()
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t1 = torch.cuda.Event(enable_timing=True)

    def torch_after_rt0(self):
        self.ev_rt0.record(self.ext)
        self.torch.cuda.current_stream().wait_event(self.ev_rt0)

    def rt0_after_torch(self):
        self.ev_torch.record(self.torch.cuda.current_stream())
        self.ext.wait_event(self.ev_torch)

    def begin_timing(self):
        self.t0.record()
        return self.t0

    def end_timing(self, ev=None):
        self.t1.record()

    def elapsed_ms(self):
        """t0 -> t1 on torch's stream (waits for t1)."""
        self.t1.synchronize()
        return self.t0.elapsed_time(self.t1)


class BandGather:
    """The per-step gather for band-packed accumulators (rt0_set_accum_buffer_compact):
    every rank renders straight into a [rows, W, 4] buffer holding only its
    bands, which is the send buffer as it stands; rank 0 receives every rank's
    buffer into one preallocated [world, rows, W, 4] tensor (the gather's
    output list is views of it) and scatters the bands into the image with one
    index_copy_ over cached indices.  No packing, no per-step allocation or
    host->device index upload.

    With band = block_band(H, world) every rank owns one contiguous row block
    (sharded ReSTIR); `send` then passes that block of a full-size accumulator.

    staged=True (a gloo process group, which moves host tensors only): the
    send buffer is copied to host memory, gathered there, and rank 0 copies
    the received buffers back to the device -- the same layout and reorder,
    so the assembled image is identical."""

    def __init__(self, H, W, rank, world, band, device, channels=4, staged=False):
        import torch
        self.H, self.W, self.rank, self.world, self.band = H, W, rank, world, band
        self.staged = staged
        self.nb = (H + band - 1) // band
        self.max_owned = (self.nb + world - 1) // world
        self.rows = self.max_owned * band  # every rank's buffer has this many rows (RCCL needs equal sizes)
        self.acc = torch.zeros((self.rows, W, channels), dtype=torch.float32, device=device)
        if rank == 0:
            self.recv = torch.empty((world, self.rows, W, channels), dtype=torch.float32, device=device)
            self.bufs = list(self.recv.unbind(0))  # views: the gather writes straight into recv
            src_slot, dst_band = [], []
            for s in range(world):
                for j, b in enumerate(owned_bands(s, world, self.nb)):
                    src_slot.append(s * self.max_owned + j)
                    dst_band.append(b)
            self.src = torch.tensor(src_slot, device=device)
            self.dst = torch.tensor(dst_band, device=device)
            self.image = torch.zeros((self.nb * band, W, channels), dtype=torch.float32, device=device)
            if staged:
                self.recv_host = torch.empty((world, self.rows, W, channels), dtype=torch.float32)
                self.bufs_host = list(self.recv_host.unbind(0))

    def gather(self, send=None):
        """Collective; rank 0 returns the assembled [H, W, 4] image (a view of a
        persistent buffer), the other ranks None.  send defaults to self.acc."""
        import torch.distributed as dist
        send = self.acc if send is None else send
        if self.staged:
            send = send.cpu()
        if self.rank != 0:
            dist.gather(send, None, dst=0)
            return None
        if self.staged:
            dist.gather(send, self.bufs_host, dst=0)
            self.recv.copy_(self.recv_host)
        else:
            dist.gather(send, self.bufs, dst=0)
        bands = self.recv.view(self.world * self.max_owned, self.band, self.W, -1)
        img = self.image.view(self.nb, self.band, self.W, -1)
        img.index_copy_(0, self.dst, bands.index_select(0, self.src))
        return self.image[:self.H]


# ------------------------------------------------------------- sharded ReSTIR
# ReSTIR's spatial pass reads the previous pass's reservoirs up to ~16 px away
# (raytracer.glsl:1726-1760) and the temporal pass reads the history at a
# reprojected position (1485-1523).  A ReSTIR shard owns the row bands b with
# b % world == rank: ONE contiguous block when band = block_band(H, world), or
# several bands dealt round-robin (interleaved_band) so that the expensive
# rows of a scene are spread over all ranks.  After every pass each band
# boundary between two ranks swaps `halo` rows of the newest reservoir planes
# (halo <= band, so a halo reaches into the neighbouring band only): one
# batched point-to-point exchange per pass, 2 x halo x W x 32 B per boundary
# (SURVEY 8e).  The history planes are earlier "newest" planes, so their halos
# are already in place.  librt0 counts any fetch outside the own bands + halo
# (Renderer.halo_misses): zero means the sharded render equals the unsharded
# one bit for bit.

def block_band(height, world):
    """Rows per shard for contiguous blocks: ceil(H / world) rounded up to the
    16-row workgroup tile."""
    return ((height + world - 1) // world + 15) // 16 * 16


def interleaved_band(height, world, per_rank=2, halo=24):
    """Band height for `per_rank` round-robin bands per shard: the load balance
    of a scene whose cost varies by row (sky vs geometry) against one halo
    exchange per band boundary.  At least 2 x `halo` rows (the halos of a
    band's two boundaries stay within the neighbouring band and do not
    overlap) and a multiple of 16."""
    b = block_band(height, world * per_rank)
    return max(b, (2 * halo + 15) // 16 * 16)


def cost_cuts(band_cost, band_rows, height, world, align=16):
    """Row cuts [0, c1, ..., height] of `world` contiguous blocks of equal
    measured cost: band_cost[b] is the time of rows [b * band_rows, (b + 1) *
    band_rows) (a previous pass, or a calibration render); the cost inside a
    band is taken as uniform and each cut is rounded to `align` rows (the
    workgroup tile) and kept at least `align` rows after the previous one."""
    import bisect
    pre = [0.0]
    for c in band_cost:
        pre.append(pre[-1] + max(c, 0.0))
    total = pre[-1]
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        b = min(len(band_cost) - 1, max(0, bisect.bisect_right(pre, target) - 1))
        frac = (target - pre[b]) / band_cost[b] if band_cost[b] > 0 else 0.0
        y = int(round((b + frac) * band_rows / align)) * align
        y = max(cuts[-1] + align, min(y, height - (world - k) * align))
        cuts.append(y)
    cuts.append(height)
    return cuts


def block_rows(rank, band, height):
    """Rows of the contiguous block of `rank` (band = block_band)."""
    lo = min(height, rank * band)
    return lo, min(height, lo + band)


def owned_band_rows(rank, world, band, height):
    """[(lo, hi)] of the bands of `rank`, top to bottom in row order."""
    nb = (height + band - 1) // band
    return [(b * band, min(height, (b + 1) * band)) for b in range(rank, nb, world)]


def halo_plan(rank, world, band, height, halo):
    """Point-to-point transfers of one halo exchange for `rank`:
    [("send"|"recv", peer, row0, row1)], band boundaries in row order, so that
    the transfers between any two ranks are posted in the same order on both
    sides.  Every send has the matching recv on the peer with the same rows."""
    if halo <= 0 or world <= 1:
        return []
    if halo > band:
        raise ValueError("halo (%d rows) larger than a shard's band (%d rows)" % (halo, band))
    nb = (height + band - 1) // band
    plan = []
    for b in range(nb - 1):  # the boundary between bands b and b + 1, at row y
        lower, upper = b % world, (b + 1) % world
        if lower == upper or rank not in (lower, upper):
            continue
        y = (b + 1) * band
        below = min(halo, band)  # rows of band b next to y
        above = min(halo, min(height, y + band) - y)  # rows of band b + 1 next to y
        if rank == lower:
            plan.append(("send", upper, y - below, y))
            plan.append(("recv", upper, y, y + above))
        else:
            plan.append(("recv", lower, y - below, y))
            plan.append(("send", lower, y, y + above))
    return plan


def exchange_halo(planes, rank, world, band, halo, staged=False):
    """Collective over torch.distributed (RCCL on GPUs, gloo on CPU): planes is
    a list of [H, W, 4] tensors, fresh in this rank's block; afterwards the
    halo rows hold the neighbours' rows.  staged=True (gloo with device
    planes): sent rows are copied to host buffers first and received rows
    copied back to the device afterwards."""
    import torch.distributed as dist
    height = planes[0].shape[0]
    ops, back = [], []
    for p in planes:
        for kind, peer, r0, r1 in halo_plan(rank, world, band, height, halo):
            rows = p[r0:r1]
            if staged and rows.is_cuda:
                host = rows.cpu() if kind == "send" else rows.new_empty(rows.shape, device="cpu")
                if kind == "recv":
                    back.append((rows, host))
                rows = host
            fn = dist.isend if kind == "send" else dist.irecv
            ops.append(dist.P2POp(fn, rows, peer))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for dev_rows, host in back:
        dev_rows.copy_(host)


def exchange_halo_local(planes_by_rank, band, halo):
    """The same exchange between shards living in one process (tests, or
    several shards on one device): planes_by_rank[rank] = list of planes."""
    world = len(planes_by_rank)
    height = planes_by_rank[0][0].shape[0]
    for rank in range(world):
        for kind, peer, r0, r1 in halo_plan(rank, world, band, height, halo):
            if kind == "recv":
                for dst, src in zip(planes_by_rank[rank], planes_by_rank[peer]):
                    dst[r0:r1].copy_(src[r0:r1])


class RestirShard:
    """One rank's sharded ReSTIR renderer state: torch-owned reservoir planes
    handed to librt0, so that the halo rows can be exchanged as tensors."""

    def __init__(self, renderer, rank, world, height, width, device, halo=24, band=None, staged=False, order=None):
        import torch
        self.r = renderer
        self.rank, self.world, self.halo, self.staged = rank, world, halo, staged
        self.order = order or StreamOrder(renderer, device)
        self.band = band or block_band(height, world)  # default: one contiguous block
        # four interleaved main/aux pairs (rt0_set_restir_buffers): texel (y, x)
        # of a pair = its main then its aux RGBA32F, so a row range of a pair
        # tensor is both planes' rows
        self.pairs = torch.zeros((4, height, width, 2, 4), dtype=torch.float32, device=device)
        renderer.set_restir_buffers([self.pairs[k, :, :, j].data_ptr() for k in range(4) for j in range(2)])
        self.by_ptr = {self.pairs[k, :, :, 0].data_ptr(): k for k in range(4)}
        renderer.set_shard(rank, world, self.band)
        renderer.set_halo(halo)
        torch.cuda.synchronize(device)

    def newest(self):
        """The pair tensor (H, W, 2, 4) of the newest reservoir planes."""
        m, _ = self.r.device_restir(0)
        return [self.pairs[self.by_ptr[m]]]

    def render(self, first, n, exchange=None):
        """Passes first..first+n-1, one launch each, halo exchange after each
        (exchange(planes) defaults to exchange_halo over torch.distributed).
        The launches are asynchronous on librt0's stream; each exchange waits
        for its pass and the next pass for the exchange through events (no host
        synchronisation per pass).  Raises if any fetch fell outside block + halo."""
        for k in range(first, first + n):
            self.r.render_async(k, 1)
            planes = self.newest()
            self.order.torch_after_rt0()
            if exchange is None:
                exchange_halo(planes, self.rank, self.world, self.band, self.halo, staged=self.staged)
            else:
                exchange(planes)
            self.order.rt0_after_torch()
        miss = self.r.halo_misses()
        if miss:
            raise RuntimeError("sharded ReSTIR: %d reservoir fetches fell outside the %d-row halo; "
                               "raise the halo" % (miss, self.halo))
