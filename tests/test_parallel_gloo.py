"""Multi-process (world_size 2 and 3, gloo, CPU) tests of the sharding logic.

The per-band icon is computed by an injected checker (the CPU oracle) so the
band partition, the halo exchange (batch_isend_irecv) and the slab all-gather
of wicca_amd.parallel.TiledHaar run exactly as on GPUs, minus the HIP call.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from wicca_amd.parallel import (TiledHaar, aligned_bands, halo_rows,  # noqa: E402
                                owned_icon_rows, shard_range)


def _oracle_compute(rows, depth, border, k):
    from oracle import c_oracle
    u8, _ = c_oracle.ll_f32_levels(rows.numpy(), depth, border, k)
    return torch.from_numpy(u8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cases, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import c_oracle
        for (H, W, C, D, border, k, cuts, seed) in cases:
            img = np.random.default_rng(seed).integers(0, 256, (H, W, C), dtype=np.uint8)
            ref = c_oracle.ll_f32_levels(img, D, border, k)[0]
            bounds = aligned_bands(H, world, D) if cuts is None else cuts
            y0, y1 = bounds[rank]
            band = torch.from_numpy(img[y0:y1].copy())
            th = TiledHaar(D, border, k, compute=_oracle_compute)
            # explicit bounds and all-gathered bounds must agree
            full = th(band, y0, H, bounds if cuts is None else None)
            if not np.array_equal(full.numpy(), ref):
                errq.put(f"rank {rank}: mismatch for {(H, W, C, D, border, k, cuts)}")
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")


def _run(world, cases):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    errors = []
    while not errq.empty():
        errors.append(errq.get())
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not errors, errors


def test_shard_range_partitions():
    for n in (0, 1, 7, 128, 1024):
        for world in (1, 2, 3, 8):
            got = [i for r in range(world) for i in shard_range(n, world, r)]
            assert got == list(range(n))
            sizes = [len(shard_range(n, world, r)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def test_aligned_bands_are_halo_free():
    for H, world, D in [(65536, 8, 8), (4320, 8, 5), (4321, 3, 5), (100, 2, 3), (7, 4, 1)]:
        b = aligned_bands(H, world, D)
        assert b[0][0] == 0 and b[-1][1] == H
        for (a0, a1), (c0, _) in zip(b, b[1:]):
            assert a1 == c0
        for (_, y1) in b:
            assert halo_rows(y1, H, D) == 0
        owned = [i for (y0, y1) in b for i in owned_icon_rows(y0, y1, H, D)]
        assert owned == list(range(-(-H // (1 << D))))


def test_tiled_world2_aligned_and_halo():
    cases = [
        (256, 96, 3, 5, 1, 0, None, 1),                       # aligned, no halo
        (203, 70, 3, 4, 1, 0, None, 2),                       # aligned, padded last band
        (203, 70, 3, 4, 0, 99, None, 3),                      # CONSTANT border
        (100, 40, 3, 3, 1, 0, [(0, 45), (45, 100)], 4),       # unaligned: 3-row halo
        (100, 40, 4, 3, 0, 7, [(0, 45), (45, 100)], 5),
        (64, 33, 1, 2, 1, 0, [(0, 31), (31, 64)], 6),          # C=1, aligned image
    ]
    _run(2, cases)


def test_tiled_world3_halo_chain():
    cases = [
        (300, 50, 3, 4, 1, 0, [(0, 90), (90, 211), (211, 300)], 7),
        (300, 50, 3, 4, 0, 255, [(0, 90), (90, 211), (211, 300)], 8),
        (1030, 20, 3, 8, 1, 0, None, 9),
    ]
    _run(3, cases)
