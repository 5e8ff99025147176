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
* INTER_CUBIC / INTER_LANCZOS4 (``resizeGeneric_`` with ``HResizeCubic`` /
  ``HResizeLanczos4`` and ``VResizeCubic`` / ``VResizeLanczos4``, uchar
  fixed point): per destination index ``f = float((d + 0.5) * scale - 0.5)``,
  ``s = floor(f)``, ``f -= s`` (never clamped for these two), coefficients
  ``interpolateCubic`` (A = -0.75, float32) or ``interpolateLanczos4``
  (double sin / cos, float32 sums, the 1e-6 special case) scaled by 2048 and
  rounded to short; horizontal ``sum_j a_j * S[clamp(s - K/2 + 1 + j)]``
  (int, replicated borders), vertical over rows ``clamp(sy - K/2 + 1 + k)``:
  Lanczos ``(sum + 2^21) >> 22`` (int); cubic the same for the row's tail,
  but OpenCV's 128-bit SIMD path (``VResizeCubicVec_32s8u``) for the first
  ``8 * floor(dw * C / 8)`` bytes of every row: float32 ``S_k * (b_k *
  2^-22)`` summed as ``S0*b0 + (S1*b1 + (S2*b2 + S3*b3))``, rounded half to
  even, saturated.
* INTER_LINEAR_EXACT (``resize_bitExact<uchar, interpolationLinear>``,
  softdouble geometry, 8.8 fixed point): both scales exactly 2 with C != 2
  goes to INTER_AREA; otherwise per destination index ``f = scale * (d +
  0.5) - 0.5`` (double), ``i = floor(f)``: ``i < 0`` (or a 1-pixel source)
  replicates the first sample, ``i >= size - 1`` the last, else weights
  ``c1 = round_half_even((f - i) * 256)``, ``c0 = 256 - c1``; horizontal
  ``c0 * S[i] + c1 * S[i + 1]`` (u16, first/last sample ``* 256`` outside),
  vertical ``(c0 * h[i] + c1 * h[i + 1] + 2^15) >> 16``, border rows
  ``(h + 128) >> 8``.
* INTER_NEAREST_EXACT (``resizeNN_bitexact``): ``ifx = ((W << 16) + dw / 2)
  / dw``, ``ifx0 = ifx / 2 - W % 2``, ``sx = min((ifx * dx + ifx0) >> 16, W - 1)``
  (integers), same for y.
"""
from __future__ import annotations

import math

import numpy as np

INTER_NEAREST = 0
INTER_LINEAR = 1
INTER_CUBIC = 2
INTER_AREA = 3
INTER_LANCZOS4 = 4
INTER_LINEAR_EXACT = 5
INTER_NEAREST_EXACT = 6
SUPPORTED = (INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA, INTER_LANCZOS4, INTER_LINEAR_EXACT,
             INTER_NEAREST_EXACT)
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


# --------------------------------------------------------------------------
# INTER_CUBIC / INTER_LANCZOS4 (resizeGeneric_, uchar fixed point)
# --------------------------------------------------------------------------
def _f32(v) -> np.float32:
    return np.float32(v)


def cubic_coeffs(x) -> list:
    """interpolateCubic (resize.cpp), float32 in the source's operation order."""
    x = _f32(x)
    A = _f32(-0.75)
    x1 = _f32(x + _f32(1))
    c0 = _f32(_f32(_f32(_f32(_f32(_f32(A * x1) - _f32(_f32(5) * A)) * x1) + _f32(_f32(8) * A)) * x1) - _f32(_f32(4) * A))
    c1 = _f32(_f32(_f32(_f32(_f32(_f32(A + _f32(2)) * x) - _f32(A + _f32(3))) * x) * x) + _f32(1))
    om = _f32(_f32(1) - x)
    c2 = _f32(_f32(_f32(_f32(_f32(_f32(A + _f32(2)) * om) - _f32(A + _f32(3))) * om) * om) + _f32(1))
    c3 = _f32(_f32(_f32(_f32(1) - c0) - c1) - c2)
    return [c0, c1, c2, c3]


_S45 = 0.70710678118654752440084436210485
_LCS = ((1, 0), (-_S45, -_S45), (0, 1), (_S45, -_S45), (-1, 0), (_S45, _S45), (0, -1), (-_S45, _S45))


def lanczos4_coeffs(x) -> list:
    """interpolateLanczos4 (resize.cpp): double sin / cos of -(x + 3) * pi / 4
    (C libm, as OpenCV calls std::sin / std::cos), float32 coefficients and
    sum, 1e30 for the zero tap (x + 3 - i == 0)."""
    x = _f32(x)
    x3 = _f32(x + _f32(3))
    y0 = float(-x3) * math.pi * 0.25
    s0, c0 = math.sin(y0), math.cos(y0)
    co, tot = [], _f32(0)
    for i in range(8):
        yi = _f32(x3 - _f32(i))
        if abs(yi) >= _f32(1e-6):
            y = float(-yi) * math.pi * 0.25
            c = _f32((_LCS[i][0] * s0 + _LCS[i][1] * c0) / (y * y))
        else:
            c = _f32(1e30)
        co.append(c)
        tot = _f32(tot + c)
    tot = _f32(_f32(1) / tot)
    return [_f32(c * tot) for c in co]


def _short_coef(c) -> int:
    """saturate_cast<short>(c * INTER_RESIZE_COEF_SCALE) of a float32 c."""
    v = int(np.rint(_f32(c * _f32(_COEF_SCALE))))
    return max(-32768, min(32767, v))


def kernel_tables(ssize: int, dsize: int, scale: float, K: int):
    """(offsets, short coefficients (dsize, K)) of the cubic (K = 4) or
    Lanczos-4 (K = 8) path for one axis."""
    ofs = np.empty(dsize, np.int64)
    co = np.empty((dsize, K), np.int64)
    fn = cubic_coeffs if K == 4 else lanczos4_coeffs
    for d in range(dsize):
        f = _f32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = _f32(f - _f32(s))
        ofs[d] = s
        co[d] = [_short_coef(c) for c in fn(f)]
    return ofs, co


def _resize_kernel(img, dw, dh, scx, scy, K):
    H, W, C = img.shape
    xo, xa = kernel_tables(W, dw, scx, K)
    yo, yb = kernel_tables(H, dh, scy, K)
    S = img.astype(np.int64)
    taps = np.clip(xo[:, None] - (K // 2 - 1) + np.arange(K)[None, :], 0, W - 1)     # (dw, K)
    rows = np.clip(yo[:, None] - (K // 2 - 1) + np.arange(K)[None, :], 0, H - 1)     # (dh, K)
    # horizontal: h[r, dx, c] = sum_j a[dx, j] * S[r, taps[dx, j], c]
    h = np.einsum("rdjc,dj->rdc", S[:, taps, :], xa)                                  # (H, dw, C)
    hv = h[rows]                                                                       # (dh, K, dw, C)
    n_el = dw * C
    out = np.empty((dh, dw * C), np.uint8)
    for dy in range(dh):
        Hk = hv[dy].reshape(K, n_el)
        b = yb[dy]
        isum = (Hk * b[:, None]).sum(axis=0)
        iv = np.clip((isum + (1 << 21)) >> 22, 0, 255)
        if K == 4:  # VResizeCubicVec_32s8u: the first 8 * floor(n_el / 8) bytes in float32
            vec = (n_el // 8) * 8
            bf = [_f32(_f32(int(bk)) * _f32(1.0 / (2048 * 2048))) for bk in b]
            Sf = Hk[:, :vec].astype(np.float32)
            t = (Sf[3] * bf[3]).astype(np.float32)
            t = ((Sf[2] * bf[2]).astype(np.float32) + t).astype(np.float32)
            t = ((Sf[1] * bf[1]).astype(np.float32) + t).astype(np.float32)
            t = ((Sf[0] * bf[0]).astype(np.float32) + t).astype(np.float32)
            iv[:vec] = np.clip(np.rint(t).astype(np.int64), 0, 255)
        out[dy] = iv
    return out.reshape(dh, dw, C)


# --------------------------------------------------------------------------
# INTER_LINEAR_EXACT (resize_bitExact<uchar, interpolationLinear<uchar>>)
# --------------------------------------------------------------------------
def linear_exact_tables(ssize: int, dsize: int, inv_scale: float):
    """(offsets, c1 in 1/256 units, min, max) of interpolationLinear."""
    scale = 1.0 / inv_scale
    ofs = np.zeros(dsize, np.int64)
    c1 = np.zeros(dsize, np.int64)
    lo, hi = 0, dsize
    for d in range(dsize):
        f = scale * (d + 0.5) - 0.5
        i = math.floor(f)
        if i >= 0 and ssize > 1:
            if i < ssize - 1:
                ofs[d] = i
                c1[d] = round((f - i) * 256)          # cvRound(softdouble): half to even
            else:
                ofs[d] = ssize - 1
                hi = min(hi, d)
        else:
            lo = max(lo, d + 1)
    return ofs, c1, lo, hi


def _resize_linear_exact(img, dw, dh, ix, iy):
    H, W, C = img.shape
    xo, xc, xlo, xhi = linear_exact_tables(W, dw, ix)
    yo, yc, ylo, yhi = linear_exact_tables(H, dh, iy)
    S = img.astype(np.int64)
    d = np.arange(dw)
    mid = (d >= xlo) & (d < xhi)
    x0 = np.where(mid, xo, 0)
    x1 = np.minimum(x0 + 1, W - 1)
    c1 = np.where(mid, xc, 0)[None, :, None]
    first = S[:, :1, :] * 256
    last = S[:, W - 1:W, :] * 256
    h = (256 - c1) * S[:, x0, :] + c1 * S[:, x1, :]                        # (H, dw, C)
    h = np.where((d < xlo)[None, :, None], first, h)
    h = np.where((d >= xhi)[None, :, None] & ~(d < xlo)[None, :, None], last, h)
    out = np.empty((dh, dw, C), np.uint8)
    for dy in range(dh):
        if dy < ylo:
            v = (h[0] + 128) >> 8
        elif dy >= yhi:
            v = (h[H - 1] + 128) >> 8
        else:
            r = yo[dy]
            v = ((256 - yc[dy]) * h[r] + yc[dy] * h[r + 1] + (1 << 15)) >> 16
        out[dy] = np.clip(v, 0, 255)
    return out


def nearest_exact_index(ssize: int, dsize: int) -> np.ndarray:
    """resizeNN_bitexact's 16-bit fixed-point source indices (clamped at 0 too)."""
    ifx = ((ssize << 16) + dsize // 2) // dsize
    ifx0 = ifx // 2 - ssize % 2
    s = (ifx * np.arange(dsize, dtype=np.int64) + ifx0) >> 16
    return np.clip(s, 0, ssize - 1)


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
        kx, ky = int(round(scx)), int(round(scy))
        fast = abs(scx - kx) < np.finfo(float).eps and abs(scy - ky) < np.finfo(float).eps
        interp = interpolation
        if interp == INTER_LINEAR_EXACT and fast and kx == 2 and ky == 2 and C != 2:
            interp = INTER_AREA  # resize.cpp: area (fast) equals bit-exact linear here
        if interp == INTER_NEAREST:
            fx, fy = 1.0 / ix, 1.0 / iy
            xs = np.minimum(np.floor(np.arange(dw) * fx).astype(np.int64), W - 1)
            ys = np.minimum(np.floor(np.arange(dh) * fy).astype(np.int64), H - 1)
            out = img[ys][:, xs]
        elif interp == INTER_NEAREST_EXACT:
            out = img[nearest_exact_index(H, dh)][:, nearest_exact_index(W, dw)]
        elif interp == INTER_LINEAR_EXACT:
            out = _resize_linear_exact(img, dw, dh, ix, iy)
        elif interp in (INTER_CUBIC, INTER_LANCZOS4):
            out = _resize_kernel(img, dw, dh, scx, scy, 4 if interp == INTER_CUBIC else 8)
        else:
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
