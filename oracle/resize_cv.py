"""CPU restatement of ``cv2.resize`` for uint8 HWC images — TEST INFRASTRUCTURE.

The reference resizes twice per image on its caller path
(``/root/reference/wicca/classifying_tools.py:315`` the source image and
``:318`` the icon), with ``interpolation=self.interpolation`` (the demo passes
``cv2.INTER_AREA``, ``demo.ipynb`` cell "interpolation=cv2.INTER_AREA").  The
arithmetic lives in OpenCV (opencv-python 4.12.0.88, ``requirements.txt:91``),
which is NOT installed here and ships no fixture in the reference, so this
module restates OpenCV's published ``imgproc/src/resize.cpp`` algorithm
(``cv::resize`` -> ``cv::hal::resize``) and is **parity unpinned**: nothing in
this container can confirm it against an OpenCV binary.  It is the checker the
GPU path (``wicca_amd/csrc/resize.hip``) is tested against, bit for bit; the
product path never imports it.

Restated behaviour (uint8, 1-4 channels, ``dsize = (width, height)``):

* ``dsize == ssize``: a copy.
* single-channel results are 2-D arrays, whether the input was (H, W) or
  (H, W, 1) (OpenCV's Python binding).
* ``inv_scale = dsize / ssize`` (double), ``scale = 1 / inv_scale``.
* INTER_NEAREST: ``sx = min(floor(dx * (1 / inv_scale_x)), W - 1)``, same for y.
* INTER_LINEAR with both scales exactly 2: treated as INTER_AREA.
* INTER_AREA with both scales >= 1:
    - integer scales (``is_area_fast``): 2x2 with C in {1, 3, 4} averages as
      ``(a + b + c + d + 2) >> 2``; otherwise ``round_half_even(float(sum) *
      float(1 / (kx * ky)))``;
    - otherwise the area tables of ``computeResizeAreaTab`` (double) and the
      float accumulation of ``ResizeArea_Invoker``: per source row, ``buf`` =
      sequential ``buf + float(S) * alpha`` over the row's table entries;
      per destination row, ``sum = beta * buf`` for its first source row then
      ``sum = sum + beta * buf``; output ``round_half_even(sum)`` (cvRound)
      saturated to uint8.  No fused multiply-add (OpenCV's x86 baseline).
* INTER_AREA with a scale < 1, and INTER_LINEAR: the fixed-point bilinear
  path (``INTER_RESIZE_COEF_BITS = 11``): per column ``sx`` and ``fx`` (the
  "area" variant ``sx = floor(dx * scale)``, ``fx = (dx + 1) - (sx + 1) *
  inv_scale`` folded to its fraction, or the linear ``fx = (dx + 0.5) * scale
  - 0.5``), coefficients ``cvRound((1 - fx) * 2048)``, ``cvRound(fx * 2048)``
  in float; horizontal ``S[sx] * a0 + S[sx + C] * a1`` (int) left of
  ``xmax`` (the first column whose ``sx + 1 >= W``, which uses ``S[W-1] *
  2048``); vertical ``(((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) +
  2) >> 2`` (``VResizeLinear<uchar, int, short, ...>``) over rows ``sy`` and
  ``sy + 1`` clamped to the image.
"""
from __future__ import annotations

import math

import numpy as np

INTER_NEAREST = 0
INTER_LINEAR = 1
INTER_AREA = 3
SUPPORTED = (INTER_NEAREST, INTER_LINEAR, INTER_AREA)
_COEF_SCALE = 2048  # 1 << INTER_RESIZE_COEF_BITS
_F32 = np.float32


def _round_f32(x) -> np.ndarray:
    """cvRound of float32 values (round half to even), as int64."""
    return np.rint(np.asarray(x, _F32)).astype(np.int64)


def _area_tab(ssize: int, dsize: int, scale: float):
    """computeResizeAreaTab (resize.cpp): per destination index, its source
    indices and float32 weights in accumulation order."""
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        ent = []
        if sx1 - fsx1 > 1e-3:
            ent.append((sx1 - 1, _F32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            ent.append((sx, _F32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            ent.append((sx2, _F32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        tab.append(ent)
    return tab


def _padded_tab(tab):
    """(idx, w) arrays of shape (n, kmax); missing entries weigh 0.0 at index 0
    (adding float(S) * 0.0 = +0.0 never changes a float32 sum)."""
    kmax = max(len(t) for t in tab)
    idx = np.zeros((len(tab), kmax), np.int64)
    w = np.zeros((len(tab), kmax), _F32)
    cnt = np.array([len(t) for t in tab])
    for i, t in enumerate(tab):
        for k, (s, a) in enumerate(t):
            idx[i, k] = s
            w[i, k] = a
    return idx, w, cnt


def _resize_area_general(img, dw, dh, scale_x, scale_y):
    H, W, C = img.shape
    xi, xw, _ = _padded_tab(_area_tab(W, dw, scale_x))
    ytab = _area_tab(H, dh, scale_y)
    src = img.astype(_F32)
    out = np.empty((dh, dw, C), np.uint8)
    with np.errstate(over="ignore"):
        for dy, rows in enumerate(ytab):
            acc = None
            for sy, beta in rows:
                row = src[sy]                                  # (W, C)
                buf = np.zeros((dw, C), _F32)
                for k in range(xi.shape[1]):                    # sequential per column
                    buf = (buf + row[xi[:, k]] * xw[:, k, None]).astype(_F32)
                term = (_F32(beta) * buf).astype(_F32)
                acc = term if acc is None else (acc + term).astype(_F32)
            out[dy] = np.clip(_round_f32(acc), 0, 255)
    return out


def _resize_area_fast(img, kx, ky):
    H, W, C = img.shape
    dh, dw = H // ky, W // kx
    blocks = img[:dh * ky, :dw * kx].reshape(dh, ky, dw, kx, C).astype(np.int64)
    s = blocks.sum(axis=(1, 3))
    if kx == 2 and ky == 2 and C in (1, 3, 4):
        return ((s + 2) >> 2).astype(np.uint8)
    scale = _F32(1.0) / _F32(kx * ky)
    return np.clip(_round_f32(s.astype(_F32) * scale), 0, 255).astype(np.uint8)


def _linear_coeffs(ssize, dsize, scale, inv_scale, area_mode):
    """Per destination index: (sx, a0, a1, past_edge) of the fixed-point path."""
    d = np.arange(dsize)
    if area_mode:
        s = np.floor(d * scale).astype(np.int64)
        f = ((d + 1) - (s + 1) * inv_scale).astype(_F32)
        f = np.where(f <= 0, _F32(0), (f - np.floor(f)).astype(_F32)).astype(_F32)
    else:
        f = ((d + 0.5) * scale - 0.5).astype(_F32)
        s = np.floor(f).astype(np.int64)
        f = (f - s.astype(_F32)).astype(_F32)
    neg = s < 0
    f = np.where(neg, _F32(0), f).astype(_F32)
    s = np.where(neg, 0, s)
    edge = s + 1 >= ssize                       # xmax: S[sx] * ONE from here on
    f = np.where(s >= ssize - 1, _F32(0), f).astype(_F32)
    s = np.where(s >= ssize - 1, ssize - 1, s)
    a0 = _round_f32((_F32(1) - f) * _F32(_COEF_SCALE))
    a1 = _round_f32(f * _F32(_COEF_SCALE))
    return s, a0, a1, edge


def _resize_linear_fixed(img, dw, dh, sx_, ix_, sy_, iy_, area_mode):
    H, W, C = img.shape
    sx, a0, a1, edge = _linear_coeffs(W, dw, sx_, ix_, area_mode)
    # vertical coefficients (no edge folding on y: rows are clamped instead)
    d = np.arange(dh)
    if area_mode:
        sy = np.floor(d * sy_).astype(np.int64)
        fy = ((d + 1) - (sy + 1) * iy_).astype(_F32)
        fy = np.where(fy <= 0, _F32(0), (fy - np.floor(fy)).astype(_F32)).astype(_F32)
    else:
        fy = ((d + 0.5) * sy_ - 0.5).astype(_F32)
        sy = np.floor(fy).astype(np.int64)
        fy = (fy - sy.astype(_F32)).astype(_F32)
    b0 = _round_f32((_F32(1) - fy) * _F32(_COEF_SCALE))
    b1 = _round_f32(fy * _F32(_COEF_SCALE))
    r0 = np.clip(sy, 0, H - 1)
    r1 = np.clip(sy + 1, 0, H - 1)
    S = img.astype(np.int64)
    x1 = np.minimum(sx + 1, W - 1)

    def hres(rows):                              # (dh, W, C) -> (dh, dw, C)
        two = rows[:, sx, :] * a0[None, :, None] + rows[:, x1, :] * a1[None, :, None]
        one = rows[:, sx, :] * _COEF_SCALE
        return np.where(edge[None, :, None], one, two)

    h0, h1 = hres(S[r0]), hres(S[r1])
    v = (((b0[:, None, None] * (h0 >> 4)) >> 16) + ((b1[:, None, None] * (h1 >> 4)) >> 16) + 2) >> 2
    return v.astype(np.uint8)


def resize(image: np.ndarray, dsize, interpolation: int = INTER_AREA) -> np.ndarray:
    """``cv2.resize(image, dsize, interpolation=...)`` for uint8 (H, W[, C]) images."""
    img = np.asarray(image)
    two_d = img.ndim == 2
    if two_d:
        img = img[:, :, None]
    if img.dtype != np.uint8 or img.ndim != 3 or not 1 <= img.shape[2] <= 4:
        raise ValueError("uint8 images with 1-4 channels")
    if interpolation not in SUPPORTED:
        raise NotImplementedError(f"interpolation {interpolation}")
    dw, dh = int(dsize[0]), int(dsize[1])
    H, W, C = img.shape
    if dw <= 0 or dh <= 0 or H == 0 or W == 0:
        raise ValueError("empty size")
    if (dw, dh) == (W, H):
        out = img.copy()
    else:
        ix, iy = dw / W, dh / H
        scx, scy = 1.0 / ix, 1.0 / iy
        if interpolation == INTER_NEAREST:
            fx, fy = 1.0 / ix, 1.0 / iy
            xs = np.minimum(np.floor(np.arange(dw) * fx).astype(np.int64), W - 1)
            ys = np.minimum(np.floor(np.arange(dh) * fy).astype(np.int64), H - 1)
            out = img[ys][:, xs]
        else:
            kx, ky = int(round(scx)), int(round(scy))
            fast = abs(scx - kx) < np.finfo(float).eps and abs(scy - ky) < np.finfo(float).eps
            interp = interpolation
            if interp == INTER_LINEAR and fast and kx == 2 and ky == 2:
                interp = INTER_AREA
            if interp == INTER_AREA and scx >= 1 and scy >= 1:
                out = (_resize_area_fast(img, kx, ky) if fast
                       else _resize_area_general(img, dw, dh, scx, scy))
            else:
                out = _resize_linear_fixed(img, dw, dh, scx, ix, scy, iy, interp == INTER_AREA)
    out = np.ascontiguousarray(out)
    # OpenCV returns single-channel images as 2-D arrays, (H, W, 1) input included
    return np.ascontiguousarray(out[:, :, 0]) if out.shape[2] == 1 else out
