"""The stage plan: ``ClassifierProcessor``'s whole (classifier x depth) matrix
of ``_get_img_batch`` computed ONCE per file.

The reference recomputes the per-file stage for every classifier and every
depth: ``process_classifiers`` loops over the depths
(``/root/reference/wicca/classifying_tools.py:546-551``), ``_parallel_proc``
submits one pool task per classifier (``:414-419``), each task's ``_classify``
walks the folder in batches (``:339-346``), and ``_get_img_batch`` decodes,
resizes, icons and resizes again every file of the batch (``:312-318``).  With
the demo's 14 classifiers and 5 depths every file is decoded 70 times.

:class:`StagePlan` is shared by those pool threads.  The first request for a
batch computes, in one native call (``wicca_image_stage_plan_u8``), the
outputs of every (shape, depth) pair the plan was given: each file is decoded
into HBM once, read once for the icons of all depths and once for the
INTER_AREA source resizes of all shapes, and every icon is resized to every
shape.  Later requests for the same batch — the other classifiers, the later
depths — are served from host memory.  A request for a pair the plan was not
given falls back to the per-call file stage (:func:`wicca_amd.get_img_batch`),
so the plan is never wrong, only sometimes not faster.

Drop-in (``ClassifierProcessor`` itself unchanged; a subclass or a
monkeypatch of one method)::

    plan = StagePlan([c[SHAPE] for c in classifiers.values()], proc.depth,
                     interpolation=proc.interpolation)
    proc._get_img_batch = lambda paths, shape: plan.get_img_batch(paths, shape, proc.depth)

(``proc.depth`` is the int ``process_classifiers`` sets before each depth's
pool, ``classifying_tools.py:546-547``.)

Every output is the bytes :func:`wicca_amd.get_img_batch` gives for that
(shape, depth) (``tests/test_gpu_plan.py``).
"""
from __future__ import annotations

import collections
import ctypes
import threading
from typing import Iterable, Sequence

import numpy as np

from . import _lib

Shape = tuple  # (width, height): cv2.resize's dsize order, as classifier[SHAPE]


def _norm_shape(shape) -> tuple[int, int]:
    w, h = int(shape[0]), int(shape[1])
    return (w, h)


def _norm_depths(depths) -> tuple[int, ...]:
    from .coder import _depth_index
    if isinstance(depths, (tuple, list, range)):
        out = []
        for d in depths:
            d = _depth_index(d)
            if d not in out:
                out.append(d)
        return tuple(out)
    return (_depth_index(depths),)


def _read(paths: Sequence, pooled: bool = False, mapped: bool = False) -> list:
    from .jpeg import read_files
    return read_files(paths, pooled=pooled, mapped=mapped)


def _matrix_args(file_paths, shapes, depths, interpolation, border_type, border_constant, device, pooled=False,
                 after_read=None, mapped=False):
    from .coder import _border_value
    shp = []
    for s in shapes:
        s = _norm_shape(s)
        if s not in shp:
            shp.append(s)
    if not shp:
        raise ValueError("need at least one shape")
    dep = _norm_depths(depths)
    if not dep:
        raise ValueError("need at least one depth")
    blobs = _read(file_paths, pooled, mapped)
    if after_read is not None:
        after_read()
    n = len(blobs)
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    # pinned host outputs: the device-to-host copies run by DMA, not as blit
    # kernels sharing the GPU with the plan's kernels (and, asynchronously,
    # without holding the host)
    resized = [_lib.pinned_empty((n, h, w, 3)) for (w, h) in shp]
    icons = [[_lib.pinned_empty((n, h, w, 3)) for _ in dep] for (w, h) in shp]
    k = _border_value(border_constant) if int(border_type) == 0 else 0
    args = ((ctypes.c_void_p * n)(*[b.ctypes.data for b in keep]), (ctypes.c_int64 * n)(*[b.size for b in keep]), n,
            (ctypes.c_int64 * (2 * len(shp)))(*[v for s in shp for v in s]), len(shp),
            (ctypes.c_int * len(dep))(*dep), len(dep), int(border_type), k, int(interpolation),
            (ctypes.c_void_p * len(shp))(*[r.ctypes.data for r in resized]),
            (ctypes.c_void_p * (len(shp) * len(dep)))(*[a.ctypes.data for row in icons for a in row]),
            -1 if device is None else int(device))
    out = {}
    for si, s in enumerate(shp):
        for di, d in enumerate(dep):
            out[(s, d)] = (resized[si], icons[si][di])
    return blobs, keep, args, out


class MatrixCall:
    """An issued :func:`get_img_matrix_async`; :meth:`wait` gives the matrix."""

    def __init__(self, ticket: int, keep, out: dict):
        self._ticket = ticket
        self._keep = keep  # the file bytes and argument arrays, alive until the wait
        self._out = out

    def wait(self) -> dict:
        if self._ticket is not None:
            ticket, self._ticket = self._ticket, None
            try:
                _lib.check(_lib.load().wicca_image_stage_plan_wait(ticket))
                # the native side is done with the file bytes: their read
                # buffers go back to the pool (only after a clean wait)
                from .jpeg import release_buffers
                blobs, self._keep = self._keep[0], None
                release_buffers(blobs)
            finally:
                self._keep = None
        return self._out

    def __del__(self):
        if getattr(self, "_ticket", None) is not None:  # dropped unwaited: the native side must be done with the arrays
            try:
                _lib.load().wicca_image_stage_plan_wait(self._ticket)
            except Exception:
                pass


def get_img_matrix_async(file_paths: Sequence, shapes: Iterable, depths, interpolation: int = 3,
                         border_type: int = 1, border_constant: int = 0,
                         device: int | None = None, _after_read=None, _issue_gate=None,
                         _mapped: bool = False) -> MatrixCall:
    """:func:`get_img_matrix` (errors "raise") without waiting for the device:
    the batch's host work, decode, plan kernels and output copies are queued
    (``wicca_image_stage_plan_async``) and its kernels run after the previous
    asynchronous call's, so a loop that issues batch k+1 before waiting for
    batch k overlaps k+1's host work and k's output copies with the kernels.
    (StagePlan's hooks: ``_after_read()`` once the files are read,
    ``_issue_gate`` = (enter, leave) around the native issue, ``_mapped``:
    the files memory-mapped instead of copied.)"""
    import os
    import time
    timing = os.environ.get("WICCA_ISSUE_TIMING") is not None
    marks = [time.perf_counter()]

    def after_read():
        marks.append(time.perf_counter())
        if _after_read is not None:
            _after_read()
    blobs, keep, args, out = _matrix_args(file_paths, shapes, depths, interpolation, border_type,
                                          border_constant, device, pooled=True, after_read=after_read,
                                          mapped=_mapped)
    if args[2] == 0:
        return MatrixCall(None, None, out)
    ticket = ctypes.c_int64(0)
    marks.append(time.perf_counter())
    if _issue_gate is not None:
        _issue_gate[0]()
    marks.append(time.perf_counter())
    try:
        _lib.check(_lib.load().wicca_image_stage_plan_async(*args, ctypes.byref(ticket)))
    finally:
        if _issue_gate is not None:
            _issue_gate[1]()
    if timing:  # WICCA_ISSUE_TIMING: the Python side of the issue (the native side prints its own phases)
        marks.append(time.perf_counter())
        d = [1e3 * (b - a) for a, b in zip(marks, marks[1:])]
        if len(d) == 4:
            import sys
            print(f"[wicca plan py] read {d[0]:.2f}, outputs + args {d[1]:.2f}, gate wait {d[2]:.2f}, "
                  f"native call {d[3]:.2f} ms", file=sys.stderr, flush=True)
    return MatrixCall(ticket.value, (blobs, keep, args), out)


def get_img_matrix(file_paths: Sequence, shapes: Iterable, depths, interpolation: int = 3, border_type: int = 1,
                   border_constant: int = 0, device: int | None = None,
                   errors: str = "raise") -> dict:
    """``_get_img_batch(file_paths, shape)`` at ``self.depth = depth`` for every
    (shape, depth) pair, from one native call: ``{(shape, depth): (batch_images,
    batch_icons)}`` with ``shape = (width, height)``.  errors: as
    :func:`wicca_amd.get_img_batch` ("raise" or "zero").  With "raise" the call
    goes through the asynchronous entry (issue, then wait): concurrent calls'
    kernels then queue on the device one after another while their host work
    overlaps, instead of contending for the GPU."""
    from .jpeg import _load_error, _slot_error
    if errors not in ("raise", "zero"):
        raise ValueError("errors must be 'raise' or 'zero'")
    if errors == "raise":
        return get_img_matrix_async(file_paths, shapes, depths, interpolation, border_type, border_constant,
                                    device).wait()
    blobs, keep, args, out = _matrix_args(file_paths, shapes, depths, interpolation, border_type,
                                          border_constant, device)
    n = args[2]
    status = (ctypes.c_int * n)()
    _lib.check(_lib.load().wicca_image_stage_plan_u8(*args, status))
    del keep
    for i in range(n):
        if status[i] != 0:  # as load_image reports it (data_loader.py:61-63)
            print(f"Error loading image {file_paths[i]}: {_load_error(_slot_error(blobs[i]))}")
    return out


class _Entry:
    __slots__ = ("event", "result", "error", "nbytes", "served")

    def __init__(self):
        self.event = threading.Event()
        self.result = None
        self.error = None
        self.nbytes = 0
        self.served = collections.Counter()


class StagePlan:
    """Shared, thread-safe cache of the stage matrix, keyed by batch.

    shapes: the classifiers' input shapes, one per classifier (repeats count:
        a (shape, depth) pair is expected once per classifier with that shape,
        and a batch is dropped once every expected request was served);
    depths: int / tuple / list / range (``normalize_depth``'s forms);
    batches: optional, the folder's batches in ``_classify``'s order
        (``os.listdir`` in steps of ``batch_size``): when a batch is first
        requested the next one starts computing in the background (at most
        ``ahead`` of them at a time), so its host work and PCIe transfers
        overlap the requested batch's device work and the classifiers'
        inference;
    devices: optional GPU ids; batch k of ``batches`` (or the k-th new batch)
        runs on ``devices[k % len(devices)]``;
    cache_bytes: the most host memory the cached outputs may hold (default: a
        quarter of the host's memory, at most 32 GiB).  ``process_classifiers``
        runs the depths one after another over the whole folder
        (classifying_tools.py:546-551), so a batch computed for every depth
        stays cached until the last depth reaches it; when the folder's outputs
        for all depths do not fit (known up front from ``batches``, or found
        when the cap first forces an eviction), the plan computes each batch
        per depth instead -- every shape of that depth from one decode, the
        14x saving across classifiers kept -- and the working set is a few
        batches of one depth;
    mapped_files: True (default) memory-maps the batch's files instead of
        copying them out of the page cache: 25 x 10 MB copies took 4-17 ms
        per batch on the host, and with them the loop's issue chain (read +
        parse / de-stuffing / uploads ~7 ms) outran the device's ~11 ms per
        batch now and then -- steady 12.5-16 ms per batch, against 12.1-12.6
        mapped (profiles/r06ze_*, r06zf_*).  A file truncated while its
        batch is being decoded faults (SIGBUS) on the pages past its new end:
        the library's reads of file bytes run under a SIGBUS guard, so the
        batch then fails with an error, as a short file would fail its slot
        under cv2.imread -- except uncompressed BMP / PNM rows, which the HIP
        runtime copies straight from the mapping.  Pass False for folders that
        may change during the run (WICCA_READ_MMAP=0 forces copies everywhere);
    copy: True (default) hands each request its own writable arrays, as the
        reference's ``np.stack`` does; False hands every classifier the one
        cached pair, READ-ONLY (a classifier writing into its batch raises
        instead of corrupting the others' input) -- Keras' ``preprocess_input``
        converts uint8 batches to new float arrays, so the demo's classifiers
        never write into them.  The private copies are ~665 MB of host memcpy
        per 25 x 8K batch of the demo (14 classifiers x 5 depths), more than
        the GPU's work on the batch.
    """

    def __init__(self, shapes: Iterable, depths, interpolation: int = 3, border_type: int = 1,
                 border_constant: int = 0, *, batches: Sequence[Sequence] | None = None,
                 device: int | None = None, devices: Sequence[int] | None = None, errors: str = "raise",
                 cache_bytes: int | None = None, copy: bool = True, ahead: int = 2, mapped_files: bool = True):
        self.expected = collections.Counter(_norm_shape(s) for s in shapes)
        if not self.expected:
            raise ValueError("need at least one shape")
        self.shapes = list(self.expected)
        self.depths = _norm_depths(depths)
        self.interpolation = int(interpolation)
        self.border_type = int(border_type)
        self.border_constant = border_constant
        self.device = device
        self.devices = list(devices) if devices else None
        self.errors = errors
        self.cache_bytes = int(cache_bytes) if cache_bytes is not None else _default_cache_bytes()
        self.copy = copy
        self.mapped_files = bool(mapped_files)
        self.ahead = max(0, int(ahead))
        self._order = {}
        self._batches = [list(b) for b in batches] if batches is not None else None
        # per_depth: entries are (batch, depth) -- see cache_bytes
        self.per_depth = False
        if self._batches is not None:
            for i, b in enumerate(self._batches):
                self._order.setdefault(self._key(b), i)
            files = sum(len(b) for b in self._batches)
            self.per_depth = files * self._file_bytes(len(self.depths)) > self.cache_bytes
        self._lock = threading.Lock()
        self._entries: collections.OrderedDict = collections.OrderedDict()
        self._bytes = 0
        self._new = 0
        self._prefetch: list = []
        self._retired = set()  # batches every expected request was served from (never prefetched again)
        self._matrix = get_img_matrix  # the native call (tests inject a stand-in)
        self.stats = collections.Counter()
        # native issues in the order the computations started (tickets): the
        # next batch starts (and reads its files) once this batch's files are
        # read, so its read overlaps this batch's native issue, and issues
        # after it
        self._gate = threading.Condition()
        self._ticket_next = 0
        self._ticket_turn = 0

    @staticmethod
    def _key(paths) -> tuple:
        return tuple(str(p) for p in paths)

    def _file_bytes(self, n_depths: int) -> int:
        """Output bytes per file: each shape's resized image and its icons."""
        return sum(w * h * 3 for (w, h) in self.shapes) * (1 + n_depths)

    def _device_for(self, key) -> int | None:
        if not self.devices:
            return self.device
        idx = self._order.get(key[0])
        if idx is None:
            idx = self._new
            self._new += 1
        return self.devices[idx % len(self.devices)]

    def _compute(self, key, entry: _Entry, device, issued=None) -> None:
        """Compute `entry`; `issued()` runs once the batch's files are read
        (the asynchronous native path) or its native work is queued: the
        owner starts the next batch's prefetch there.  The native issues go
        in ticket order (a batch's kernels before the next one's), so the
        next batch's file reads overlap this batch's parse, de-stuffing and
        uploads, not its kernels' order."""
        paths, depth = key
        depths = self.depths if depth is None else (depth,)
        native = self._matrix is get_img_matrix and self.errors == "raise"
        if native:
            with self._gate:
                my = self._ticket_next
                self._ticket_next += 1
        gate = {"entered": False, "left": not native}

        def enter():
            with self._gate:
                while self._ticket_turn != my:
                    self._gate.wait()
            gate["entered"] = True

        def leave():
            if not gate["left"]:
                gate["left"] = True
                with self._gate:
                    self._ticket_turn += 1
                    self._gate.notify_all()

        def after_read():
            nonlocal issued
            if issued is not None:
                cb, issued = issued, None
                cb()
        try:
            if native:
                call = get_img_matrix_async(list(paths), self.shapes, depths, self.interpolation, self.border_type,
                                            self.border_constant, device, _after_read=after_read,
                                            _issue_gate=(enter, leave), _mapped=self.mapped_files)
                after_read()  # (no files: nothing was read)
                entry.result = call.wait()
            else:
                if issued is not None:
                    issued()
                    issued = None
                entry.result = self._matrix(list(paths), self.shapes, depths, self.interpolation,
                                            self.border_type, self.border_constant, device, self.errors)
            if not self.copy:  # shared by every requester: read-only
                for pair in entry.result.values():
                    for a in pair:
                        a.flags.writeable = False
            # a shape's resized images are shared by its depths: count each array once
            entry.nbytes = sum({id(a): a.nbytes for pair in entry.result.values() for a in pair}.values())
        except BaseException as e:  # the requesters waiting now see the failure ...
            entry.error = e
        finally:
            if not gate["left"]:  # this ticket's turn passes even when it never issued
                if not gate["entered"]:
                    enter()
                leave()
            if issued is not None:  # the issue failed: the prefetch still starts
                try:
                    issued()
                except BaseException:
                    pass
            with self._lock:
                self.stats["computed"] += 1
                if self._entries.get(key) is entry:
                    if entry.error is not None:  # ... later ones compute the batch again
                        del self._entries[key]
                        self.stats["failed"] += 1
                    else:
                        self._bytes += entry.nbytes
                        self._trim(keep=key)
            entry.event.set()

    def _trim(self, keep) -> None:
        # lock held: drop least recently used finished batches above the cap
        for k in list(self._entries):
            if self._bytes <= self.cache_bytes:
                break
            e = self._entries[k]
            if k == keep or not e.event.is_set():
                continue
            del self._entries[k]
            self._bytes -= e.nbytes if e.result is not None else 0
            self.stats["evicted"] += 1
            if not self.per_depth:  # the folder does not fit for every depth: one depth at a time from now
                self.per_depth = True
                self.stats["per_depth"] += 1

    def _start_prefetch(self, key) -> None:
        # the batch after `key` starts now, while `key` itself is still being
        # computed: its host work (read, parse, de-stuffing, PCIe upload)
        # overlaps the other's device work; at most `ahead` background batches
        idx = self._order.get(key[0])
        if idx is None or idx + 1 >= len(self._batches):
            return
        nxt = (self._key(self._batches[idx + 1]), key[1])
        with self._lock:
            self._prefetch = [t for t in self._prefetch if t.is_alive()]
            if nxt in self._entries or nxt in self._retired or len(self._prefetch) >= self.ahead:
                return
            entry = _Entry()
            self._entries[nxt] = entry
            dev = self._device_for(nxt)
            t = threading.Thread(target=self._compute, args=(nxt, entry, dev), daemon=True)
            self._prefetch.append(t)
            self.stats["prefetched"] += 1
        t.start()

    def entry(self, file_paths, depth=None) -> _Entry:
        """The (computed) cache entry of a batch (of ``depth`` when the plan
        runs per depth); computes it on first use."""
        with self._lock:
            pk = self._key(file_paths)
            key = (pk, None)  # a batch computed for every depth serves any of them
            entry = self._entries.get(key)
            if entry is None and self.per_depth:
                key = (pk, depth if depth is not None else self.depths[0])
                entry = self._entries.get(key)
            owner = entry is None
            if owner:
                entry = _Entry()
                self._entries[key] = entry
                dev = self._device_for(key)
                self.stats["misses"] += 1
            else:
                self._entries.move_to_end(key)
                self.stats["hits"] += 1
        prefetch = (lambda: self._start_prefetch(key)) if self._batches is not None else None
        if owner:
            self._compute(key, entry, dev, issued=prefetch)
        else:
            if prefetch is not None:
                prefetch()
            entry.event.wait()
        return entry

    def get_img_batch(self, file_paths, shape, transform_depth) -> tuple[np.ndarray, np.ndarray]:
        """``ClassifierProcessor._get_img_batch(file_paths, shape)`` at
        ``self.depth = transform_depth`` (classifying_tools.py:297-323)."""
        from .coder import _depth_index
        s = _norm_shape(shape)
        d = _depth_index(transform_depth)
        if s not in self.expected or d not in self.depths:  # not planned: the per-call stage
            from .jpeg import get_img_batch
            self.stats["unplanned"] += 1
            return get_img_batch(list(file_paths), s, d, self.interpolation, self.border_type,
                                 self.border_constant, self.device, errors=self.errors)
        entry = self.entry(file_paths, d)
        if entry.error is not None:
            raise entry.error
        images, icons = entry.result[(s, d)]
        out = (images.copy(), icons.copy()) if self.copy else (images, icons)
        with self._lock:
            key = next((k for k in ((self._key(file_paths), d), (self._key(file_paths), None))
                        if self._entries.get(k) is entry), None)
            entry.served[(s, d)] += 1
            depths = self.depths if key is None or key[1] is None else (key[1],)
            done = all(entry.served[(sh, dd)] >= self.expected[sh] for sh in self.expected for dd in depths)
            if done and key is not None:
                del self._entries[key]
                self._bytes -= entry.nbytes
                self._retired.add(key)
                self.stats["retired"] += 1
        return out

    def cached_batches(self) -> int:
        with self._lock:
            return len(self._entries)

    def cached_bytes(self) -> int:
        with self._lock:
            return self._bytes

    def close(self) -> None:
        """Wait for a background batch and drop the cache."""
        for t in list(self._prefetch):
            t.join()
        self._prefetch = []
        with self._lock:
            self._entries.clear()
            self._retired.clear()
            self._bytes = 0


def _default_cache_bytes() -> int:
    """A quarter of the host's physical memory, at most 32 GiB."""
    try:
        import os
        total = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError, AttributeError):
        total = 16 << 30
    return int(min(32 << 30, total // 4))


def folder_batches(folder, batch_size: int = 25) -> list[list]:
    """``_classify``'s batches of a folder: ``os.listdir`` order in steps of
    ``batch_size`` (classifying_tools.py:335-340), as full paths."""
    import os
    names = os.listdir(folder)
    return [[os.path.join(str(folder), f) for f in names[i:i + batch_size]]
            for i in range(0, len(names), batch_size)]
