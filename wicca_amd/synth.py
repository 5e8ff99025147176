"""Deterministic synthetic images (host restatement of the device generator).

Byte ``b`` (row-major ``y*W*C + x*C + c``) of image ``i`` is

    key  = mix64(seed * 0x100000001B3 + i)
    word = mix64(key + (b >> 3))
    byte = (word >> (8 * (b & 7))) & 0xFF

with ``mix64`` the splitmix64 finaliser.  The HIP kernel ``synth_u8_kernel``
(``wicca_amd/csrc/haar_ll.hip``) computes the same bytes on device, so the
benchmark never moves images over PCIe and any image it used can be
regenerated here for a spot check ("Synthetic inputs").
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def image_key(seed: int, index: int) -> np.uint64:
    with np.errstate(over="ignore"):
        z = np.uint64((seed * 0x100000001B3 + index) & 0xFFFFFFFFFFFFFFFF)
        return _mix64(np.array([z], np.uint64))[0]


def synth_rows(seed: int, index: int, first_row: int, rows: int, W: int, C: int) -> np.ndarray:
    """Rows ``[first_row, first_row + rows)`` of synthetic image ``index``."""
    b0 = first_row * W * C
    nbytes = rows * W * C
    w0, w1 = b0 // 8, (b0 + nbytes + 7) // 8
    with np.errstate(over="ignore"):
        words = _mix64(image_key(seed, index) + np.arange(w0, w1, dtype=np.uint64))
    raw = words.astype("<u8").view(np.uint8)[b0 - 8 * w0:b0 - 8 * w0 + nbytes]
    return raw.reshape(rows, W, C).copy()


def synth_image(seed: int, index: int, H: int, W: int, C: int) -> np.ndarray:
    """Image ``index`` of the synthetic stream ``seed`` as an (H, W, C) uint8 array."""
    nbytes = H * W * C
    nwords = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        words = _mix64(image_key(seed, index) + np.arange(nwords, dtype=np.uint64))
    out = words.astype("<u8").view(np.uint8)[:nbytes]
    return out.reshape(H, W, C).copy()
