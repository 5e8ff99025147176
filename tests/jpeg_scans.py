"""Test helper: re-code a baseline JPEG file as a MULTI-SCAN sequential file,
one non-interleaved scan per component (ITU-T T.81 B.2.3, A.2.2), from the
quantised coefficients of the original.  Pillow's encoder only writes one
interleaved scan, so this is how the tests obtain files that exercise the
host decoder's sequential multi-scan path.  The entropy coder uses the
typical Huffman tables of T.81 Annex K (K.3).  Test infrastructure only.
"""
from __future__ import annotations

import ctypes

import numpy as np

# T.81 Table K.3 / K.4 (DC) and K.5 / K.6 (AC): BITS (counts per length 1..16) and HUFFVAL
_DC_L_BITS = [0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0]
_DC_C_BITS = [0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0]
_DC_VALS = list(range(12))
_AC_L_BITS = [0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7D]
_AC_L_VALS = bytes.fromhex(
    "01020300041105122131410613516107227114328191a1082342b1c11552d1f02433627282090a161718191a25262728"
    "292a3435363738393a434445464748494a535455565758595a636465666768696a737475767778797a83848586878889"
    "8a92939495969798999aa2a3a4a5a6a7a8a9aab2b3b4b5b6b7b8b9bac2c3c4c5c6c7c8c9cad2d3d4d5d6d7d8d9dae1e2"
    "e3e4e5e6e7e8e9eaf1f2f3f4f5f6f7f8f9fa")
_AC_C_BITS = [0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77]
_AC_C_VALS = bytes.fromhex(
    "000102031104052131061241510761711322328108144291a1b1c109233352f0156272d10a162434e125f11718191a26"
    "2728292a35363738393a434445464748494a535455565758595a636465666768696a737475767778797a828384858687"
    "88898a92939495969798999aa2a3a4a5a6a7a8a9aab2b3b4b5b6b7b8b9bac2c3c4c5c6c7c8c9cad2d3d4d5d6d7d8d9da"
    "e2e3e4e5e6e7e8e9eaf2f3f4f5f6f7f8f9fa")

_ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,
           7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
           39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


def _codes(bits, vals):
    """symbol -> (code, length) of a canonical table (T.81 C.2)."""
    out, code, k = {}, 0, 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            out[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)  # byte stuffing
                self.acc = self.n = 0

    def flush(self):
        while self.n:
            self.put(1, 1)  # pad with 1 bits (T.81 F.1.2.3)
        return bytes(self.out)


def _size(v):
    return int(abs(int(v))).bit_length()


def _vbits(v, s):
    return int(v) if v >= 0 else int(v) + (1 << s) - 1


def _segments(data: bytes):
    """(marker, payload) of the segments before the first SOS."""
    out, p = [], 2
    while p + 4 <= len(data):
        assert data[p] == 0xFF
        m = data[p + 1]
        ln = (data[p + 2] << 8) | data[p + 3]
        out.append((m, data[p + 4:p + 2 + ln]))
        if m == 0xDA:
            break
        p += 2 + ln
    return out


def _seg(m, payload):
    return bytes([0xFF, m, (len(payload) + 2) >> 8, (len(payload) + 2) & 255]) + payload


def split_scans(baseline: bytes, coefs: np.ndarray, order=None, restart: int = 0) -> bytes:
    """The same image as one sequential scan per component (in `order`,
    default SOF order), from `coefs` (the engine's layout: components back to
    back, bw x bh MCU-padded blocks of 64 int16 in natural order); with
    `restart` > 0 a DRI of that many MCUs (= blocks in a one-component scan)
    and RSTn markers between the intervals (T.81 E.1.4)."""
    segs = _segments(baseline)
    sof = next(p for m, p in segs if m in (0xC0, 0xC1))
    H, W, nc = (sof[1] << 8) | sof[2], (sof[3] << 8) | sof[4], sof[5]
    comps = [(sof[6 + 3 * c], sof[7 + 3 * c] >> 4, sof[7 + 3 * c] & 15) for c in range(nc)]
    hmax = max(h for _, h, _ in comps) if nc > 1 else 1
    vmax = max(v for _, _, v in comps) if nc > 1 else 1
    mcux = -(-W // (8 * hmax))
    mcuy = -(-H // (8 * vmax))
    geo, off = [], 0
    for cid, h, v in comps:
        if nc == 1:
            h = v = 1
        bw, bh = mcux * h, mcuy * v
        dw, dh = -(-W * h // hmax), -(-H * v // vmax)
        geo.append((cid, bw, bh, -(-dw // 8), -(-dh // 8), off))
        off += bw * bh
    blocks = coefs.reshape(-1, 64)
    out = bytearray(b"\xff\xd8")
    for m, p in segs:
        if m in (0xC4, 0xDA, 0xDD):  # own tables, no restart interval
            continue
        out += _seg(m, p)
    dht = bytearray()
    for tc_th, bits, vals in ((0x00, _DC_L_BITS, _DC_VALS), (0x01, _DC_C_BITS, _DC_VALS),
                              (0x10, _AC_L_BITS, _AC_L_VALS), (0x11, _AC_C_BITS, _AC_C_VALS)):
        dht += bytes([tc_th]) + bytes(bits) + bytes(vals)
    out += _seg(0xC4, bytes(dht))
    if restart:
        out += _seg(0xDD, bytes([restart >> 8, restart & 255]))
    tabs = [(_codes(_DC_L_BITS, _DC_VALS), _codes(_AC_L_BITS, _AC_L_VALS)),
            (_codes(_DC_C_BITS, _DC_VALS), _codes(_AC_C_BITS, _AC_C_VALS))]
    for c in (order if order is not None else range(nc)):
        cid, bw, bh, wb, hb, base = geo[c]
        t = 0 if c == 0 else 1
        dc_t, ac_t = tabs[t]
        out += _seg(0xDA, bytes([1, cid, (t << 4) | t, 0, 63, 0]))
        bw_ = _Bits()
        pred = 0
        for i in range(hb * wb):
            if restart and i and i % restart == 0:  # byte-align, marker, reset the DC predictor
                out += bw_.flush() + bytes([0xFF, 0xD0 + (i // restart - 1) % 8])
                bw_ = _Bits()
                pred = 0
            by, bx = divmod(i, wb)
            blk = blocks[base + by * bw + bx]
            zz = [int(blk[_ZIGZAG[k]]) for k in range(64)]
            diff = zz[0] - pred
            pred = zz[0]
            s = _size(diff)
            bw_.put(*dc_t[s])
            if s:
                bw_.put(_vbits(diff, s), s)
            run = 0
            for k in range(1, 64):
                v = zz[k]
                if v == 0:
                    run += 1
                    continue
                while run > 15:
                    bw_.put(*ac_t[0xF0])
                    run -= 16
                s = _size(v)
                bw_.put(*ac_t[(run << 4) | s])
                bw_.put(_vbits(v, s), s)
                run = 0
            if run:
                bw_.put(*ac_t[0x00])
        out += bw_.flush()
    out += b"\xff\xd9"
    return bytes(out)


def coefficients(data: bytes, force: int) -> np.ndarray:
    """The host entropy decoder's quantised coefficients of a file through
    wicca_jpeg_host_coefficients (no GPU)."""
    from wicca_amd import _lib
    arr = np.frombuffer(data, np.uint8)
    lib = _lib.load()
    nb = ctypes.c_int64()
    assert lib.wicca_jpeg_host_coefficients(arr.ctypes.data, arr.size, force, None, 0, ctypes.byref(nb)) == 0
    out = np.empty(nb.value * 64, np.int16)
    rc = lib.wicca_jpeg_host_coefficients(arr.ctypes.data, arr.size, force, out.ctypes.data, nb.value,
                                          ctypes.byref(nb))
    assert rc == 0, _lib.last_error()
    return out


def gray_file(coefs: np.ndarray, qt, W: int, H: int, restart: int = 0) -> bytes:
    """A baseline one-component JPEG holding exactly `coefs` (bh x bw blocks
    of 64 int16 quantised coefficients, natural order; bw = ceil(W/8)) and the
    quantisation table `qt` (64 values, natural order; 16-bit precision when
    any exceeds 255).  AC values within +-1023 and DC differences within
    +-2047 (the T.81 K.3 / K.5 tables).  For IDCT parity probes."""
    return coef_file([(coefs, qt)], W, H, restart)


def coef_file(comps, W: int, H: int, restart: int = 0) -> bytes:
    """gray_file for 1 or 3 components at 4:4:4 (interleaved MCUs of one
    block per component): `comps` = [(coefs, qt), ...], table i for
    component i."""
    bw, bh = -(-W // 8), -(-H // 8)
    nc = len(comps)
    blocks = [np.asarray(c).reshape(bh * bw, 64) for c, _ in comps]
    dqt = bytearray()
    for i, (_, qt) in enumerate(comps):
        qt = [int(q) for q in qt]
        wide = max(qt) > 255
        zq = [qt[_ZIGZAG[k]] for k in range(64)]
        dqt += bytes([(0x10 if wide else 0x00) | i]) + (b"".join(q.to_bytes(2, "big") for q in zq) if wide
                                                        else bytes(zq))
    out = bytearray(b"\xff\xd8")
    out += _seg(0xDB, bytes(dqt))
    out += _seg(0xC0, bytes([8, H >> 8, H & 255, W >> 8, W & 255, nc]) +
                b"".join(bytes([i + 1, 0x11, i]) for i in range(nc)))
    out += _seg(0xC4, bytes([0x00]) + bytes(_DC_L_BITS) + bytes(_DC_VALS) + bytes([0x10]) + bytes(_AC_L_BITS) +
                _AC_L_VALS)
    if restart:
        out += _seg(0xDD, bytes([restart >> 8, restart & 255]))
    out += _seg(0xDA, bytes([nc]) + b"".join(bytes([i + 1, 0x00]) for i in range(nc)) + bytes([0, 63, 0]))
    dc_t, ac_t = _codes(_DC_L_BITS, _DC_VALS), _codes(_AC_L_BITS, _AC_L_VALS)
    bits = _Bits()
    pred = [0] * nc
    for i in range(bh * bw):
        if restart and i and i % restart == 0:
            out += bits.flush() + bytes([0xFF, 0xD0 + (i // restart - 1) % 8])
            bits = _Bits()
            pred = [0] * nc
        for c in range(nc):
            zz = [int(blocks[c][i][_ZIGZAG[k]]) for k in range(64)]
            diff = zz[0] - pred[c]
            pred[c] = zz[0]
            s = _size(diff)
            assert s <= 11, "DC difference outside +-2047"
            bits.put(*dc_t[s])
            if s:
                bits.put(_vbits(diff, s), s)
            run = 0
            for k in range(1, 64):
                v = zz[k]
                if v == 0:
                    run += 1
                    continue
                while run > 15:
                    bits.put(*ac_t[0xF0])
                    run -= 16
                s = _size(v)
                assert s <= 10, "AC value outside +-1023"
                bits.put(*ac_t[(run << 4) | s])
                bits.put(_vbits(v, s), s)
                run = 0
            if run:
                bits.put(*ac_t[0x00])
    out += bits.flush() + b"\xff\xd9"
    return bytes(out)
