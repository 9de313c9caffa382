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
    assembled [H, W, 4] image (others return None).  H must be a multiple of band."""
    import torch
    import torch.distributed as dist
    if acc.shape[0] % band:
        raise ValueError("image height must be a multiple of the band height")
    send = pack(acc, rank, world, band)
    if rank == 0:
        bufs = bufs if bufs is not None else [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, bufs, dst=0)
        image = image if image is not None else torch.zeros_like(acc)
        return unpack(bufs, world, band, image)
    dist.gather(send, None, dst=0)
    return None
