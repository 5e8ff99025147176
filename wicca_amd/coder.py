"""Drop-in wavelet coder: ``HaarCoder.get_small_copy`` on MI355X.

Mirrors the reference's plugin interface (``/root/reference/wicca/wavelet_coder.py``):

* :class:`WaveletCoder` — the abstract plugin type (reference ``:26-38``),
* :class:`HaarCoder` — its Haar implementation (reference ``:41-67``), same
  constructor, same ``_ONE_STEP_RATIO``, same ``get_small_copy`` signature,
  argument meaning, return type and exceptions.

``ClassifierProcessor(wavelet_coder=HaarCoder())`` (reference
``classifying_tools.py:116, :144``) and the visualisation helpers
(``visualization.py:91-94, :138-141``, keyword call) use it unchanged.

Every icon is computed by the HIP engine (``libwicca_hip.so`` through the C ABI
in ``include/wicca_haar.h``).  There is no CPU fallback: without the library or
a GPU the call raises.

Extra entry points beyond the reference interface:

* :meth:`HaarCoder.get_small_copies` — ragged batch, one kernel launch (the
  icon stage of ``ClassifierProcessor._get_img_batch``,
  ``classifying_tools.py:297-323``),
* :meth:`HaarCoder.get_small_copy_multi` — several depths from one upload
  (the depth loop of ``process_classifiers``, ``classifying_tools.py:546-551``),
* :meth:`HaarCoder.get_ll_plane` — the float32 ``low_left`` plane before
  quantisation (``wavelet_coder.py:61-65``).
"""
from __future__ import annotations

import ctypes
import operator
import threading
from abc import ABC, abstractmethod
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from .validation import (MSG_2D_INDEX, MSG_NDIM, MSG_NOT_ARRAY, validate_image)

# OpenCV border constants (cv2.BORDER_*); numbering as documented by OpenCV.
BORDER_CONSTANT = 0
BORDER_REPLICATE = 1
BORDER_REFLECT = 2
BORDER_WRAP = 3
BORDER_REFLECT_101 = 4
_HOST_PAD_MODES = {BORDER_REFLECT: "symmetric", BORDER_WRAP: "wrap", BORDER_REFLECT_101: "reflect"}


class WaveletCoder(ABC):
    """Abstract image compressor based on multi-resolution analysis.

    Reference: ``wicca/wavelet_coder.py:26-38``.
    """

    @abstractmethod
    def get_small_copy(self, image: np.ndarray, transform_depth: int,
                       border_type: int = BORDER_REPLICATE,
                       border_constant: int = 0) -> np.ndarray:
        """Resize the image using wavelet transform."""


def _depth_index(transform_depth) -> int:
    # The reference iterates ``range(transform_depth)`` (wavelet_coder.py:61),
    # which accepts anything with __index__ and raises TypeError otherwise.
    try:
        return operator.index(transform_depth)
    except TypeError:
        raise TypeError(f"'{type(transform_depth).__name__}' object cannot be "
                        "interpreted as an integer") from None


def _border_value(border_constant) -> int:
    # OpenCV saturate_cast<uchar> of the border scalar (round, then clamp).
    v = float(border_constant)
    return int(min(255, max(0, np.rint(v))))


def _pad_amounts(rows: int, cols: int, depth: int) -> tuple[int, int]:
    # wicca/data_loader.py:107-110
    if depth <= 0:
        return 0, 0
    ratio = 1 << depth
    return (-rows) % ratio, (-cols) % ratio


def _as_hwc(image: np.ndarray) -> np.ndarray:
    """An (H, W, C) view whose pixels are contiguous (rows may be strided), or a copy."""
    img = image if image.ndim == 3 else image[:, :, None]
    H, W, C = img.shape
    s0, s1, s2 = img.strides
    if (C == 1 or s2 == 1) and s1 == C and s0 >= W * C:
        return img
    return np.ascontiguousarray(img)


class _Binding:
    """One thread's device slot; returned to the binder when the thread ends
    (CPython drops a thread's ``threading.local`` values at thread exit)."""

    __slots__ = ("binder", "slot")

    def __init__(self, binder: "DeviceBinder", slot: int):
        self.binder = binder
        self.slot = slot

    def __del__(self):
        try:
            self.binder._release(self.slot)
        except Exception:  # interpreter shutdown
            pass


class DeviceBinder:
    """Thread -> device assignment for one shared coder.

    ``ClassifierProcessor`` hands ONE coder to a ``ThreadPoolExecutor`` with a
    worker per classifier (``classifying_tools.py:144, 414-419``; a new pool per
    depth, ``:546-551``), and every worker calls ``get_small_copy``
    (``:317``).  The first call on a thread binds it to the slot of
    ``devices`` with the fewest live threads (ties: the slot bound least often,
    then the lowest); the binding lasts for the thread's life, and its slot is
    released when the thread ends, so each new pool spreads over every GPU
    again.  ``devices`` may repeat an id (e.g. ``[0] * 8`` to exercise the
    assignment on a one-GPU box).
    """

    def __init__(self, devices: Sequence[int] | None = None):
        self._given = None if devices is None else [int(d) for d in devices]
        if self._given is not None and not self._given:
            raise ValueError("devices must not be empty")
        self._devices: list[int] | None = self._given
        self._lock = threading.Lock()
        self._local = threading.local()
        self._live: list[int] = []
        self._total: list[int] = []
        self.history: list[tuple[int, int, int]] = []  # (thread ident, slot, device)

    @property
    def devices(self) -> list[int]:
        if self._devices is None:
            with self._lock:
                if self._devices is None:
                    self._devices = self._default_devices()
        return self._devices

    @staticmethod
    def _default_devices() -> list[int]:
        # One rank of a multi-process launch (torch.distributed.run sets
        # LOCAL_WORLD_SIZE) owns the device it made current: -1 follows it.
        # No device visible: -1 too, so the C call raises NODEVICE.
        import os
        if int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1) > 1:
            return [-1]
        n = _lib.device_count()
        return list(range(n)) if n > 0 else [-1]

    def device(self) -> int:
        b = getattr(self._local, "binding", None)
        if b is None:
            devs = self.devices
            with self._lock:
                if len(self._live) != len(devs):
                    self._live = [0] * len(devs)
                    self._total = [0] * len(devs)
                slot = min(range(len(devs)), key=lambda i: (self._live[i], self._total[i], i))
                self._live[slot] += 1
                self._total[slot] += 1
                self.history.append((threading.get_ident(), slot, devs[slot]))
            b = _Binding(self, slot)
            self._local.binding = b
        return self._devices[b.slot]  # type: ignore[index]

    def _release(self, slot: int) -> None:
        with self._lock:
            if slot < len(self._live) and self._live[slot] > 0:
                self._live[slot] -= 1

    def live_counts(self) -> list[int]:
        """Live threads bound to each slot."""
        with self._lock:
            return list(self._live)


class HaarCoder(WaveletCoder):
    """The simplified image compressor based on the Haar wavelet, on MI355X.

    Reference: ``wicca/wavelet_coder.py:41-67``.

    Args:
        device: ``"auto"`` (default): every calling thread is bound, on its
            first call, to the least-loaded of ``devices`` (all visible GPUs
            unless given) — one shared coder spreads ``ClassifierProcessor``'s
            worker threads over the node (:class:`DeviceBinder`).  An int: that
            HIP device for every call.  ``None``: the calling thread's current
            HIP device.
        devices: the device ids ``"auto"`` binds threads to.
    """

    def __init__(self, device: int | str | None = "auto", devices: Sequence[int] | None = None):
        super().__init__()
        self._ONE_STEP_RATIO = 2
        self._binder: DeviceBinder | None = None
        if isinstance(device, str):
            if device != "auto":
                raise ValueError(f"device must be an int, None or 'auto', not {device!r}")
            self._binder = DeviceBinder(devices)
            self.device = -1
        else:
            if devices is not None:
                raise ValueError("devices= is only used with device='auto'")
            self.device = -1 if device is None else int(device)
        self._lib = _lib.load()

    @property
    def binder(self) -> DeviceBinder | None:
        """The thread -> device assignment (``device="auto"``), else None."""
        return getattr(self, "_binder", None)

    def _dev(self) -> int:
        """The device of this call: the thread's binding, or the fixed id."""
        b = getattr(self, "_binder", None)
        return b.device() if b is not None else self.device

    # ------------------------------------------------------------------ #
    # reference interface
    # ------------------------------------------------------------------ #
    def get_small_copy(self, image: np.ndarray, transform_depth: int,
                       border_type: int = BORDER_REPLICATE,
                       border_constant: int = 0) -> np.ndarray:
        """The 2^D-times smaller LL ("icon") copy of ``image``.

        Same contract as the reference (``wavelet_coder.py:50-67``): uint8
        (H, W, C) in, fresh C-contiguous uint8 (ceil(H/2^D), ceil(W/2^D), C)
        out, bottom/right padding per ``border_type`` / ``border_constant``.
        """
        img, depth, border, k = self._prepare(image, transform_depth, border_type,
                                              border_constant)
        if depth <= 0:
            return self._copy(img, image.ndim)
        H, W, C = img.shape
        oh, ow = -(-H // (1 << depth)), -(-W // (1 << depth))
        out = np.empty((oh, ow, C), np.uint8)
        _lib.check(self._lib.wicca_haar_ll_u8(
            img.ctypes.data, H, W, C, img.strides[0], depth, border, k,
            out.ctypes.data, ow * C, 0, 0, self._dev(), None))
        return out

    # ------------------------------------------------------------------ #
    # extensions
    # ------------------------------------------------------------------ #
    def get_ll_plane(self, image: np.ndarray, transform_depth: int,
                     border_type: int = BORDER_REPLICATE,
                     border_constant: int = 0) -> np.ndarray:
        """The float32 ``low_left`` plane before ``clip``/``astype`` (reference
        ``wavelet_coder.py:61-67``), bit-identical to the reference's."""
        img, depth, border, k = self._prepare(image, transform_depth, border_type,
                                              border_constant)
        H, W, C = img.shape
        if depth <= 0:
            oh, ow = H, W
        else:
            oh, ow = -(-H // (1 << depth)), -(-W // (1 << depth))
        out = np.empty((oh, ow, C), np.float32)
        _lib.check(self._lib.wicca_haar_ll_f32(
            img.ctypes.data, H, W, C, img.strides[0], depth, border, k,
            out.ctypes.data, ow * C * 4, 0, 0, self._dev(), None))
        return out[:, :, 0] if image.ndim == 2 else out

    def get_small_copies(self, images: Sequence[np.ndarray], transform_depth: int,
                         border_type: int = BORDER_REPLICATE,
                         border_constant: int = 0,
                         devices: Sequence[int] | None = None) -> list[np.ndarray]:
        """Icons of a ragged batch of images, one kernel launch per channel count.

        Equivalent to ``[self.get_small_copy(im, d, ...) for im in images]``
        (each image validated exactly like the single-image call).  With
        ``devices`` (several device ids), the batch is split image-parallel
        over those GPUs, one host thread each
        (``wicca_haar_ll_u8_batch_multi_gpu``).
        """
        prepared = [self._prepare(im, transform_depth, border_type, border_constant)
                    for im in images]
        outs: list[np.ndarray | None] = [None] * len(prepared)
        groups: dict[int, list[int]] = {}
        for i, (img, depth, border, k) in enumerate(prepared):
            if depth <= 0:
                outs[i] = self._copy(img, images[i].ndim)
            else:
                groups.setdefault(img.shape[2], []).append(i)
        for C, idx in groups.items():
            descs = (_lib.ImageDesc * len(idx))()
            keep = []
            for j, i in enumerate(idx):
                img, depth, border, k = prepared[i]
                H, W, _ = img.shape
                oh, ow = -(-H // (1 << depth)), -(-W // (1 << depth))
                out = np.empty((oh, ow, C), np.uint8)
                outs[i] = out
                keep.append(img)
                descs[j] = _lib.ImageDesc(img.ctypes.data, out.ctypes.data, H, W,
                                          img.strides[0], ow * C)
            # _prepare gives every member the caller's border and constant
            # (host-padded exotic borders come back as REPLICATE, needing none)
            _, depth, border, k = prepared[idx[0]]
            assert all(prepared[i][2:] == (border, k) for i in idx)
            if devices is not None and len(devices) > 1:
                devs = (ctypes.c_int * len(devices))(*devices)
                _lib.check(self._lib.wicca_haar_ll_u8_batch_multi_gpu(
                    descs, len(idx), C, depth, border, k, devs, len(devices)))
            else:
                dev = devices[0] if devices else self._dev()
                _lib.check(self._lib.wicca_haar_ll_u8_batch(descs, len(idx), C, depth, border, k,
                                                            0, 0, dev, None))
            del keep
        return outs  # type: ignore[return-value]

    def icon_stage(self, images: Sequence[np.ndarray], transform_depth: int, shape,
                   interpolation: int = 3, border_type: int = BORDER_REPLICATE,
                   border_constant: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """``ClassifierProcessor._get_img_batch`` (classifying_tools.py:297-323)
        for already-decoded images, each uploaded once:

        ``(np.stack([cv2.resize(im, shape, interpolation) for im in images]),
        np.stack([cv2.resize(self.get_small_copy(im, d), shape, interpolation)
        for im in images]))`` — INTER_NEAREST / INTER_LINEAR / INTER_AREA
        (the demo's), computed on the GPU (``wicca_icon_stage_u8``).
        """
        if int(border_type) not in (BORDER_CONSTANT, BORDER_REPLICATE):
            raise ValueError("icon_stage pads with BORDER_CONSTANT or BORDER_REPLICATE")
        prepared = [self._prepare(im, transform_depth, border_type, border_constant)
                    for im in images]
        if not prepared:
            raise ValueError("need at least one array to stack")
        out_w, out_h = int(shape[0]), int(shape[1])
        Cs = {img.shape[2] for img, _, _, _ in prepared}
        if len(Cs) != 1:
            raise ValueError("all input arrays must have the same shape")
        C = Cs.pop()
        _, depth, border, k = prepared[0]
        n = len(prepared)
        descs = (_lib.ImageDesc * n)()
        keep = []
        for i, (img, _, _, _) in enumerate(prepared):
            keep.append(img)
            descs[i] = _lib.ImageDesc(img.ctypes.data, None, img.shape[0], img.shape[1],
                                      img.strides[0], 0)
        resized = np.empty((n, out_h, out_w, C), np.uint8)
        icons = np.empty((n, out_h, out_w, C), np.uint8)
        _lib.check(self._lib.wicca_icon_stage_u8(descs, n, C, depth, border, k, out_w, out_h,
                                                 int(interpolation), resized.ctypes.data,
                                                 icons.ctypes.data, self._dev()))
        del keep
        if C == 1:  # cv2.resize returns single-channel images as 2-D arrays
            return resized[..., 0].copy(), icons[..., 0].copy()
        return resized, icons

    def get_small_copy_multi(self, image: np.ndarray, transform_depths: Iterable[int],
                             border_type: int = BORDER_REPLICATE,
                             border_constant: int = 0) -> dict[int, np.ndarray]:
        """``{d: self.get_small_copy(image, d, ...)}`` for every depth, one upload."""
        depths = [_depth_index(d) for d in transform_depths]
        if not depths:
            return {}
        if border_type in _HOST_PAD_MODES:
            return {d: self.get_small_copy(image, d, border_type, border_constant)
                    for d in depths}
        prepared = [self._prepare(image, d, border_type, border_constant) for d in depths]
        result: dict[int, np.ndarray] = {}
        dev_depths = [p[1] for p in prepared if p[1] >= 1]
        for (img, d, _, _) in prepared:
            if d <= 0:
                result[d] = self._copy(img, image.ndim)
        if dev_depths:
            # one image, the caller's border and constant for every depth (the
            # C side pads each depth on its own)
            img, _, border, k = prepared[0]
            H, W, C = img.shape
            outs = []
            for d in dev_depths:
                oh, ow = -(-H // (1 << d)), -(-W // (1 << d))
                outs.append(np.empty((oh, ow, C), np.uint8))
            n = len(dev_depths)
            c_depths = (ctypes.c_int * n)(*dev_depths)
            c_dsts = (ctypes.c_void_p * n)(*[o.ctypes.data for o in outs])
            c_pitch = (ctypes.c_int64 * n)(*[o.shape[1] * C for o in outs])
            _lib.check(self._lib.wicca_haar_ll_u8_multi(
                img.ctypes.data, H, W, C, img.strides[0], c_depths, n, border, k,
                c_dsts, c_pitch, 0, 0, self._dev(), None))
            for d, o in zip(dev_depths, outs):
                result[d] = o
        return result

    # ------------------------------------------------------------------ #
    # helpers
    # ------------------------------------------------------------------ #
    def _prepare(self, image, transform_depth, border_type, border_constant):
        """Reference checks in reference order; returns (hwc, depth, border, k).

        Order: validate_image (wavelet_coder.py:56) -> ratio (:58) ->
        get_padded_copy checks (data_loader.py:96-105) -> padding -> level
        loop (wavelet_coder.py:61-62, where 2-D planes raise IndexError).
        """
        validate_image(image)
        if not isinstance(image, np.ndarray):
            raise ValueError(MSG_NOT_ARRAY)
        if image.ndim not in (2, 3):
            raise ValueError(MSG_NDIM)
        depth = _depth_index(transform_depth)
        rows, cols = image.shape[0], image.shape[1]
        add_r, add_c = _pad_amounts(rows, cols, depth)
        padded = add_r or add_c
        border = int(border_type)
        if padded and border not in (BORDER_CONSTANT, BORDER_REPLICATE) \
                and border not in _HOST_PAD_MODES:
            raise ValueError(f"Unsupported border type {border_type}")
        # OpenCV returns a 2-D plane for padded (H, W, 1) input; the reference
        # then fails in the level loop on low_left[::2, :, :].
        if depth >= 1 and (image.ndim == 2 or (padded and image.shape[2] == 1)):
            raise IndexError(MSG_2D_INDEX)
        k = _border_value(border_constant) if border == BORDER_CONSTANT else 0
        img = _as_hwc(image)
        # The caller's CONSTANT / REPLICATE border and constant are carried
        # through whether or not THIS image needs padding (the kernels add
        # nothing when it does not), so every member of a batch or depth list
        # launches with the same border as the reference's per-image call.
        # Other border types are materialised on the host; the launch then sees
        # an image that needs no padding, under REPLICATE.
        if border not in (BORDER_CONSTANT, BORDER_REPLICATE):
            if padded:
                img = np.pad(img, [(0, add_r), (0, add_c), (0, 0)],
                             mode=_HOST_PAD_MODES[border])
            border, k = BORDER_REPLICATE, 0
        return img, depth, border, k

    def _copy(self, img: np.ndarray, ndim: int) -> np.ndarray:
        """Depth <= 0: the loop runs zero times; a fresh uint8 copy (device round trip)."""
        H, W, C = img.shape
        out = np.empty((H, W, C), np.uint8)
        _lib.check(self._lib.wicca_haar_ll_u8(
            img.ctypes.data, H, W, C, img.strides[0], 0, BORDER_REPLICATE, 0,
            out.ctypes.data, W * C, 0, 0, self._dev(), None))
        return out[:, :, 0].copy() if ndim == 2 else out
