"""GPU image decode: the reference's ``load_image``.

``/root/reference/wicca/data_loader.py:31-63`` reads every file with
``cv2.imread`` (BGR) and converts it to RGB.  Here JPEG files are decoded on
the GPU (``wicca_amd/csrc/jpeg.hip``), restating libjpeg-turbo's default
arithmetic bit for bit (checked against Pillow 12.2.0 / libjpeg-turbo
3.1.4.1, ``tests/test_gpu_jpeg.py``), EXIF orientation applied as
``cv2.imread`` does; PNG, BMP (RLE included), TIFF and GIF files (the other
formats ``ClassifierProcessor`` counts, ``classifying_tools.py:162``) and
binary PGM / PPM are inflated / copied on host threads and converted to RGB
on the GPU
(``wicca_amd/csrc/raster.hip``, ``tests/test_gpu_raster.py``).  The entry
points sniff each file (``wicca_image_*``), so a batch may mix formats.

:func:`load_image` keeps the reference's contract: empty path ->
``ValueError("File path cannot be empty")``; any failure -> prints
``Error loading image {path}: Image didn't found. Please check your input.``
(``cv2.imread`` returns None for every file it cannot read and
``validate_image`` then raises that message, validation.py:94-95) and
returns ``None``; ``WICCA_LOAD_DETAIL=1`` prints the decoder's own reason
instead.  Files no decoder here handles (arithmetic-coded JPEG,
JPEG-compressed TIFF, plain PBM, 16-bit PNM, ...) fail that way too — there is no CPU fallback behind it.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib


_READ_POOL = None


def _read_pool():
    global _READ_POOL
    if _READ_POOL is None:
        import os
        from concurrent.futures import ThreadPoolExecutor
        _READ_POOL = ThreadPoolExecutor(min(16, len(os.sched_getaffinity(0))), thread_name_prefix="wicca-read")
    return _READ_POOL


class _BufferPool:
    """Recycled read buffers (1 MiB granules, at most WICCA_READ_POOL_MB idle,
    default 1024): a fresh np.empty per 10 MB file was mapped and page-faulted
    by 16 threads at once and unmapped again after the batch (TLB shootdowns
    across every CPU the process ran on), and the StagePlan's host issue of a
    batch took 10 to 34 ms from one batch to the next (tools/
    plan_variance_probe.py).  Only callers that hand the buffers back
    (:func:`release_buffers`, the stage plan's asynchronous calls) use it."""

    def __init__(self):
        import os
        import threading
        self._lock = threading.Lock()
        self._idle: dict[int, list] = {}
        self._bytes = 0
        self._cap = int(os.environ.get("WICCA_READ_POOL_MB", "1024")) << 20

    def take(self, n: int) -> np.ndarray:
        size = max(1, (n + (1 << 20) - 1) >> 20) << 20
        with self._lock:
            lst = self._idle.get(size)
            if lst:
                self._bytes -= size
                return lst.pop()
        return np.empty(size, np.uint8)

    def give(self, buf: np.ndarray) -> None:
        size = buf.nbytes
        with self._lock:
            if self._bytes + size <= self._cap:
                self._idle.setdefault(size, []).append(buf)
                self._bytes += size


_BUFFERS = _BufferPool()


def _read_into(p: str, pooled: bool) -> np.ndarray:
    import os
    with open(p, "rb", buffering=0) as f:
        n = os.fstat(f.fileno()).st_size
        buf = _BUFFERS.take(n) if pooled else np.empty(n, np.uint8)
        got = 0
        mv = memoryview(buf)
        while got < n:  # a file cut while it is read ends short, as cv2.imread reads it
            k = f.readinto(mv[got:])
            if not k:
                break
            got += k
    return buf[:got]


def _read_one(p: str) -> np.ndarray:
    return _read_into(p, False)


def _read_pooled(p: str) -> np.ndarray:
    return _read_into(p, True)


def release_buffers(blobs) -> None:
    """Hand the buffers of :func:`read_files` (pooled=True) back for reuse;
    the caller must be done with them (and with every view of them)."""
    for b in blobs:
        base = b.base if isinstance(b, np.ndarray) and b.base is not None else None
        if isinstance(base, np.ndarray) and base.ndim == 1 and base.nbytes % (1 << 20) == 0:
            _BUFFERS.give(base)


def _map_one(p: str) -> np.ndarray:
    import mmap
    import os
    with open(p, "rb") as f:
        if os.fstat(f.fileno()).st_size == 0:
            return np.empty(0, np.uint8)
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    return np.frombuffer(mm, np.uint8)


def read_files(paths: Sequence[str], pooled: bool = False, mapped: bool = False) -> list:
    """Each file's bytes as a uint8 array, read into memory of its own by a
    pool of threads (serial f.read() of 25 x 10 MB files took longer than the
    whole GPU stage of the batch).  mapped=True (the stage plan's default) or
    WICCA_READ_MMAP=1 maps the files instead (no copy; WICCA_READ_MMAP=0 forces
    copies), at a price: a file truncated or rewritten while it is mapped
    raises SIGBUS when the decoder touches the missing pages, where a copy
    (and cv2.imread) sees a short file."""
    import os
    for p in paths:
        if not p:
            raise ValueError("File path cannot be empty")
    if not paths:
        raise ValueError("need at least one array to stack")
    env = os.environ.get("WICCA_READ_MMAP")
    mapped = env == "1" or (mapped and env != "0")
    one = _map_one if mapped else _read_pooled if pooled else _read_one
    if len(paths) == 1:
        return [one(paths[0])]
    return list(_read_pool().map(one, paths))


def _buffers(blobs: Sequence[bytes]):
    n = len(blobs)
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    ptrs = (ctypes.c_void_p * n)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * n)(*[k.size for k in keep])
    return keep, ptrs, sizes


def info(data: bytes, apply_orientation: bool = True) -> tuple[int, int, int, int]:
    """(height, width, components, exif_orientation) of a JPEG file's bytes."""
    arr = np.frombuffer(data, np.uint8)
    h, w = ctypes.c_int64(), ctypes.c_int64()
    c, o = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.load().wicca_jpeg_info(arr.ctypes.data, arr.size, int(apply_orientation),
                                           ctypes.byref(h), ctypes.byref(w), ctypes.byref(c),
                                           ctypes.byref(o)))
    return h.value, w.value, c.value, o.value


KINDS = {1: "jpeg", 2: "png", 3: "bmp", 4: "tiff", 5: "gif", 6: "pnm"}


def image_info(data: bytes, apply_orientation: bool = True) -> tuple[int, int, str]:
    """(height, width, format) of a JPEG, PNG, BMP, TIFF, GIF or PNM file's bytes
    (format "jpeg" / "png" / "bmp" / "tiff" / "gif" / "pnm"; JPEG sizes after EXIF
    orientation)."""
    arr = np.frombuffer(data, np.uint8)
    h, w = ctypes.c_int64(), ctypes.c_int64()
    k = ctypes.c_int()
    _lib.check(_lib.load().wicca_image_info(arr.ctypes.data, arr.size, int(apply_orientation),
                                            ctypes.byref(h), ctypes.byref(w), ctypes.byref(k)))
    return h.value, w.value, KINDS[k.value]


# what the reference prints for any file cv2.imread cannot read (validation.py:94-95)
_UNREADABLE = "Image didn't found. Please check your input."


def _load_error(detail: str) -> str:
    import os
    return detail if os.environ.get("WICCA_LOAD_DETAIL") == "1" else _UNREADABLE


def _slot_error(data: bytes) -> str:
    """The parser's message for one file (re-parsed; host only)."""
    try:
        image_info(data)
    except Exception as e:  # the message of the C ABI's failure
        return str(e)
    return "decode failed"


def decode_batch(blobs: Sequence[bytes], apply_orientation: bool = True,
                 device: int | None = None, errors: str = "raise") -> list[np.ndarray | None]:
    """RGB (H, W, 3) uint8 arrays of JPEG / PNG / BMP / TIFF / GIF files, decoded in one GPU pass.

    errors="raise": the first file that does not parse raises (nothing is
    decoded); errors="none": such a file gives None in its slot and the others
    decode (load_image's per-file contract, data_loader.py:61-63).
    """
    if errors not in ("raise", "none"):
        raise ValueError("errors must be 'raise' or 'none'")
    if not blobs:
        return []
    n = len(blobs)
    outs: list[np.ndarray | None] = []
    for b in blobs:
        try:
            h, w, _ = image_info(b, apply_orientation)
        except (ValueError, NotImplementedError):
            if errors == "raise":
                raise
            outs.append(None)
            continue
        outs.append(np.empty((h, w, 3), np.uint8))
    keep, ptrs, sizes = _buffers(blobs)
    # slots that failed to parse get a 1-pixel placeholder (never written)
    holder = np.empty(3, np.uint8)
    dsts = (ctypes.c_void_p * n)(*[o.ctypes.data if o is not None else holder.ctypes.data for o in outs])
    pitches = (ctypes.c_int64 * n)(*[o.shape[1] * 3 if o is not None else 3 for o in outs])
    status = (ctypes.c_int * n)() if errors == "none" else None
    _lib.check(_lib.load().wicca_image_decode_u8(ptrs, sizes, n, dsts, pitches, int(apply_orientation),
                                                 0, -1 if device is None else int(device), None, status))
    del keep
    if status is not None:
        for i in range(n):
            if status[i] != 0:
                outs[i] = None
    return outs


def decode_batches(batches, apply_orientation: bool = True, device: int = 0, depth: int = 2):
    """Pipelined GPU decode of a stream of batches of image files (a data
    loader's loop): yields, per batch of file bytes, a list of device RGB
    ``torch.uint8`` tensors (H, W, 3).  Up to ``depth`` all-JPEG batches are
    in flight (``wicca_jpeg_decode_u8_async``): batch k+1's parse, de-stuffing
    and PCIe transfer overlap batch k's device decode; a batch holding PNG /
    BMP / TIFF / GIF files is decoded before it is queued.  Each yielded batch
    is complete (its ``wicca_jpeg_wait`` returned); files that do not parse
    raise."""
    import collections
    if depth < 1:
        raise ValueError("depth must be >= 1")
    lib = _lib.load()
    pending = collections.deque()

    def finish():
        ticket, outs, keep = pending.popleft()
        _lib.check(lib.wicca_jpeg_wait(ticket))
        del keep
        return outs

    try:
        yield from _decode_batches_loop(batches, apply_orientation, device, depth, lib, pending, finish)
    finally:  # an exception or an abandoned generator still waits for what is in flight
        while pending:
            item = pending.popleft()  # its outputs and file bytes stay alive until the wait returns
            lib.wicca_jpeg_wait(item[0])
            del item


def _decode_batches_loop(batches, apply_orientation, device, depth, lib, pending, finish):
    import torch
    for blobs in batches:
        blobs = list(blobs)
        outs = []
        all_jpeg = True
        for b in blobs:
            h, w, kind = image_info(b, apply_orientation)
            all_jpeg = all_jpeg and kind == "jpeg"
            outs.append(torch.empty((h, w, 3), dtype=torch.uint8, device=f"cuda:{device}"))
        n = len(blobs)
        keep, ptrs, sizes = _buffers(blobs)
        dsts = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
        pitches = (ctypes.c_int64 * n)(*[o.shape[1] * 3 for o in outs])
        if len(pending) >= depth:
            yield finish()
        ticket = ctypes.c_int64(0)
        # the library writes the outputs from a stream of its own: the caching
        # allocator may have handed out blocks that kernels queued on torch's
        # current stream still read, so that stream is drained first
        torch.cuda.current_stream(device).synchronize()
        if all_jpeg:
            _lib.check(lib.wicca_jpeg_decode_u8_async(ptrs, sizes, n, dsts, pitches, int(apply_orientation),
                                                      int(device), ctypes.byref(ticket)))
        else:  # PNG / BMP / TIFF / GIF in the batch: decoded before the call returns (ticket 0)
            torch.cuda.synchronize(device)  # the outputs' allocation is ordered before the library's stream
            _lib.check(lib.wicca_image_decode_u8(ptrs, sizes, n, dsts, pitches, int(apply_orientation), 1,
                                                 int(device), None, None))
        pending.append((ticket.value, outs, (keep, blobs)))
    while pending:
        yield finish()


def decode(data: bytes, apply_orientation: bool = True, device: int | None = None) -> np.ndarray:
    """RGB (H, W, 3) uint8 array of one JPEG / PNG / BMP / TIFF / GIF file's bytes."""
    return decode_batch([data], apply_orientation, device)[0]


def load_image(file_path: str) -> np.ndarray | None:
    """``wicca.data_loader.load_image`` (data_loader.py:31-63) with the decode on the GPU."""
    if not file_path:
        raise ValueError("File path cannot be empty")
    _lib.load()  # a missing or unloadable library raises here, never as a per-file None
    try:
        with open(file_path, "rb") as f:
            data = f.read()
        return decode(data)
    except (OSError, ValueError, NotImplementedError) as e:
        # an unreadable / corrupt / unsupported file: the reference prints and
        # returns None (data_loader.py:61-63); a missing library, a HIP error
        # or an exhausted device still raise (they are not file problems)
        print(f"Error loading image {file_path}: {_load_error(str(e))}")
        return None


def get_img_batch(file_paths: Sequence[str], shape, transform_depth: int, interpolation: int = 3,
                  border_type: int = 1, border_constant: int = 0, device: int | None = None,
                  devices: Sequence[int] | None = None, errors: str = "raise") -> tuple[np.ndarray, np.ndarray]:
    """``ClassifierProcessor._get_img_batch`` (classifying_tools.py:297-323)
    from file paths: GPU decode + resize + icon + icon resize; only the
    compressed files cross PCIe.  Returns ``(batch_images, batch_icons)``.
    With ``devices`` (several ids) the files are split over those GPUs,
    balanced by file size, one host thread each.

    errors="raise" (the reference: an unreadable file makes load_image return
    None and cv2.resize then raises, aborting the batch): the first file that
    does not parse raises.  errors="zero": that file alone fails — its slots
    are zero images, the error is printed as load_image prints it, and the
    batch's other files are processed."""
    from .coder import _border_value, _depth_index
    blobs = read_files(file_paths)
    out_w, out_h = int(shape[0]), int(shape[1])
    n = len(blobs)
    resized = _lib.pinned_empty((n, out_h, out_w, 3))  # DMA targets (wicca_host_alloc)
    icons = _lib.pinned_empty((n, out_h, out_w, 3))
    if errors not in ("raise", "zero"):
        raise ValueError("errors must be 'raise' or 'zero'")
    keep, ptrs, sizes = _buffers(blobs)
    k = _border_value(border_constant) if int(border_type) == 0 else 0
    lib = _lib.load()
    status = (ctypes.c_int * n)() if errors == "zero" else None
    if devices is not None and len(devices) > 1:
        devs = (ctypes.c_int * len(devices))(*devices)
        _lib.check(lib.wicca_image_icon_stage_multi_gpu(
            ptrs, sizes, n, _depth_index(transform_depth), int(border_type), k, out_w, out_h,
            int(interpolation), resized.ctypes.data, icons.ctypes.data, devs, len(devices), status))
    else:
        dev = devices[0] if devices else (-1 if device is None else int(device))
        _lib.check(lib.wicca_image_icon_stage_u8(
            ptrs, sizes, n, _depth_index(transform_depth), int(border_type), k, out_w, out_h,
            int(interpolation), resized.ctypes.data, icons.ctypes.data, dev, status))
    del keep
    if status is not None:
        for i in range(n):
            if status[i] != 0:  # as load_image reports it (data_loader.py:61-63)
                print(f"Error loading image {file_paths[i]}: {_load_error(_slot_error(blobs[i]))}")
    return resized, icons


def get_img_batches(batches, shape, transform_depth: int, interpolation: int = 3, border_type: int = 1,
                    border_constant: int = 0, device: int | None = None, depth: int = 2):
    """``get_img_batch`` over a stream of batches of file paths (the loop of
    ``ClassifierProcessor._classify``, classifying_tools.py:339-345):
    yields ``(batch_images, batch_icons)`` per batch, with up to ``depth``
    batches in flight (``wicca_image_icon_stage_async``) so that batch k+1's
    file parse, de-stuffing and PCIe transfer overlap batch k's device decode
    and stage.  Same outputs as ``get_img_batch`` (errors="raise")."""
    import collections
    from .coder import _border_value, _depth_index
    if depth < 1:
        raise ValueError("depth must be >= 1")
    lib = _lib.load()
    out_w, out_h = int(shape[0]), int(shape[1])
    k = _border_value(border_constant) if int(border_type) == 0 else 0
    dev = -1 if device is None else int(device)
    pending = collections.deque()

    def finish():
        ticket, res, ico, keep = pending.popleft()
        _lib.check(lib.wicca_image_stage_wait(ticket))
        del keep
        return res, ico

    try:
        for paths in batches:
            blobs = read_files(paths)
            n = len(blobs)
            res = np.empty((n, out_h, out_w, 3), np.uint8)
            ico = np.empty((n, out_h, out_w, 3), np.uint8)
            keep, ptrs, sizes = _buffers(blobs)
            if len(pending) >= depth:
                yield finish()
            ticket = ctypes.c_int64(0)
            _lib.check(lib.wicca_image_icon_stage_async(ptrs, sizes, n, _depth_index(transform_depth),
                                                        int(border_type), k, out_w, out_h, int(interpolation),
                                                        res.ctypes.data, ico.ctypes.data, dev,
                                                        ctypes.byref(ticket)))
            pending.append((ticket.value, res, ico, (keep, blobs)))
        while pending:
            yield finish()
    finally:  # an exception or an abandoned generator still waits for what is in flight
        while pending:
            item = pending.popleft()  # the output arrays it writes stay alive until the wait returns
            lib.wicca_image_stage_wait(item[0])
            del item
