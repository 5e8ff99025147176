"""Multi-GPU sharding of the icon path.  One process per GPU.

Two shapes of parallelism, both over ``torch.distributed`` (backend ``nccl`` =
RCCL on ROCm; ``gloo`` for CPU tests):

* **Image-parallel** (BASELINE configs 2-4): :func:`shard_range` gives each
  rank a contiguous range of images; every rank computes its icons locally.
  There is no data-path collective — the icon of an image never depends on
  another image (``ClassifierProcessor._get_img_batch`` is a per-image loop,
  ``classifying_tools.py:311-321``).

* **Tiled single image** (config 5, e.g. 65536 x 65536 RGB at depth 8):
  :class:`TiledHaar` splits the rows into bands.  Because an icon pixel is a
  non-overlapping 2^D x 2^D block sum, bands whose boundaries are
  multiples of 2^D need **no halo**: each rank computes its icon slab and one
  ``all_gather`` assembles the icon (24.6 KB per rank for config 5 on 8 GPUs).
  For an existing, unaligned partition a rank's last icon row straddles into
  the next rank's band: ONE point-to-point exchange of fewer than 2^D rows
  (``batch_isend_irecv`` -> ``ncclSend``/``ncclRecv`` over xGMI) replaces the
  reference-style per-level one-row halo, because all D levels are computed
  from the original rows at once.  Padding (``data_loader.py:66-117``) only
  touches the last band and stays local.

The per-band computation is the product HIP path (``wicca_haar_ll_u8`` on
device pointers).  ``compute=`` exists so the CPU tests can drive the same
sharding and exchange logic under ``gloo`` with an injected checker.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

from . import _lib


def shard_range(n: int, world: int, rank: int) -> range:
    """Contiguous, balanced share of ``n`` items for ``rank`` of ``world``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def aligned_bands(H: int, world: int, depth: int) -> list[tuple[int, int]]:
    """Row bands whose boundaries are multiples of 2^depth (halo-free).

    Icon rows are split as evenly as possible; the last band also carries the
    image's final partial block (its padding stays local).
    """
    r = 1 << max(depth, 0)
    oh = -(-H // r)
    bands = []
    for k in range(world):
        rows = shard_range(oh, world, k)
        bands.append((min(rows.start * r, H), min(rows.stop * r, H)))
    return bands


def owned_icon_rows(y0: int, y1: int, H: int, depth: int) -> range:
    """Icon rows whose block starts inside band [y0, y1)."""
    r = 1 << depth
    oh = -(-H // r)
    return range(min(-(-y0 // r), oh), min(-(-y1 // r), oh))


def halo_rows(y1: int, H: int, depth: int) -> int:
    """Rows a band ending at y1 needs from the next band (0 if aligned)."""
    r = 1 << depth
    return min(-(-y1 // r) * r, H) - y1


class TiledHaar:
    """Icon of one image whose rows are sharded over the ranks of ``group``.

    Every rank calls :meth:`__call__` (collective) with its band — a
    ``(rows, W, C)`` uint8 tensor holding image rows ``[y0, y0 + rows)`` — and
    gets back the full ``(ceil(H/2^D), ceil(W/2^D), C)`` icon.
    """

    def __init__(self, depth: int, border_type: int = 1, border_constant: int = 0,
                 group=None, compute: Optional[Callable] = None):
        if depth < 1:
            raise ValueError("tiling needs depth >= 1")
        self.depth = depth
        self.border_type = border_type
        self.border_constant = border_constant
        self.group = group
        self._compute = compute

    # ---------------- per-band icon rows (product path: HIP) ----------------
    def _icon_rows(self, rows, torch):
        """Icon of a row block (rows, W, C) — as if it were a whole image."""
        if self._compute is not None:
            return self._compute(rows, self.depth, self.border_type, self.border_constant)
        if not rows.is_cuda:
            raise RuntimeError("TiledHaar computes on device tensors (HIP); got a CPU tensor")
        rows = rows.contiguous()
        h, W, C = rows.shape
        r = 1 << self.depth
        out = torch.empty((-(-h // r), -(-W // r), C), dtype=torch.uint8, device=rows.device)
        lib = _lib.load()
        stream = torch.cuda.current_stream(rows.device).cuda_stream
        _lib.check(lib.wicca_haar_ll_u8(
            ctypes.c_void_p(rows.data_ptr()), h, W, C, W * C, self.depth, self.border_type,
            self.border_constant, ctypes.c_void_p(out.data_ptr()), out.shape[1] * C, 1, 1,
            rows.device.index if rows.device.index is not None else -1,
            ctypes.c_void_p(stream) if stream else None))
        return out

    def _bounds(self, band, y0: int):
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        b = torch.tensor([y0, y0 + band.shape[0]], dtype=torch.int64, device=band.device)
        allb = [torch.empty_like(b) for _ in range(world)]
        dist.all_gather(allb, b, group=self.group)
        return [tuple(int(v) for v in t.tolist()) for t in allb]

    def _peer(self, rank: int) -> int:
        import torch.distributed as dist
        return dist.get_global_rank(self.group, rank) if self.group is not None else rank

    def slab(self, band, y0: int, H: int, bounds: list[tuple[int, int]]):
        """This rank's icon rows (exchanges a halo when the partition is unaligned)."""
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        rows_here = band.shape[0]
        y1 = y0 + rows_here
        if bounds[rank] != (y0, y1):
            raise ValueError(f"rank {rank}: band ({y0}, {y1}) != bounds {bounds[rank]}")
        for k in range(1, world):
            if bounds[k][0] != bounds[k - 1][1]:
                raise ValueError("bands must be contiguous and ordered by rank")
        r = 1 << self.depth
        need = halo_rows(y1, H, self.depth)                        # rows received from rank+1
        give = halo_rows(y0, H, self.depth) if rank > 0 else 0     # rows sent to rank-1
        if need and (rank + 1 >= world or bounds[rank + 1][1] - bounds[rank + 1][0] < need):
            raise ValueError("next band is shorter than the halo it must provide")
        if give > rows_here:
            raise ValueError("band is shorter than the halo it must provide")
        halo = None
        if need or give:
            ops = []
            if give:
                ops.append(dist.P2POp(dist.isend, band[:give].contiguous(), self._peer(rank - 1),
                                      self.group))
            if need:
                halo = torch.empty((need,) + tuple(band.shape[1:]), dtype=band.dtype,
                                   device=band.device)
                ops.append(dist.P2POp(dist.irecv, halo, self._peer(rank + 1), self.group))
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        icon_rows = owned_icon_rows(y0, y1, H, self.depth)
        if len(icon_rows) == 0:
            return band.new_empty((0, -(-band.shape[1] // r), band.shape[2]))
        first = icon_rows.start * r - y0                 # local row of the first owned block
        full_end = (y1 // r) * r - y0 if need else rows_here
        parts = []
        if full_end > first:
            parts.append(self._icon_rows(band[first:full_end], torch))
        if need:  # the straddling icon row: tail of this band + halo
            tail = torch.cat([band[(y1 // r) * r - y0:], halo], dim=0)
            parts.append(self._icon_rows(tail, torch))
        return parts[0] if len(parts) == 1 else torch.cat(parts, dim=0)

    def gather(self, slab, H: int, bounds: list[tuple[int, int]]):
        """All-gather the slabs (one collective) into the full icon on every rank."""
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        counts = [len(owned_icon_rows(a, b, H, self.depth)) for a, b in bounds]
        mx = max(counts)
        if slab.shape[0] == mx:
            padded = slab.contiguous()
        else:
            padded = slab.new_zeros((mx,) + tuple(slab.shape[1:]))
            padded[:slab.shape[0]] = slab
        out = padded.new_empty((world * mx,) + tuple(slab.shape[1:]))
        dist.all_gather_into_tensor(out, padded, group=self.group)
        if all(c == mx for c in counts):
            return out
        return torch.cat([out[k * mx:k * mx + n] for k, n in enumerate(counts)], dim=0)

    def __call__(self, band, y0: int, H: int, bounds: Optional[list[tuple[int, int]]] = None):
        """Full icon on every rank.  ``bounds`` (every rank's band) may be given
        when the partition is known, e.g. :func:`aligned_bands`; otherwise it is
        all-gathered."""
        if bounds is None:
            bounds = self._bounds(band, y0)
        return self.gather(self.slab(band, y0, H, bounds), H, bounds)
