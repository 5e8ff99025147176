"""Generate golden vectors from the REFERENCE HaarCoder (run in the survey container only).

    python tests/golden/make_golden.py            # writes tests/golden/{cases.json,arrays.npz}

The reference (``/root/reference/wicca``, read-only, GPL-3.0) is imported
unmodified; nothing from it is copied into the repository — only the
input/output vectors it produced.  Its modules import ``cv2`` at module scope
(``wavelet_coder.py:19``, ``data_loader.py:20``) and opencv-python 4.12.0.88 is
not installed here, so a minimal stand-in module is placed in
``sys.modules["cv2"]`` first.  It supplies only what the hot path touches:

* ``BORDER_CONSTANT = 0``, ``BORDER_REPLICATE = 1`` (OpenCV's documented values),
* ``copyMakeBorder`` — bottom/right padding via ``np.pad`` (``edge`` /
  ``constant``), returning a 2-D array for (H, W, 1) input as OpenCV does.

All arithmetic (widening, level loop, clip, cast) and all validation is the
reference's own code on numpy 2.2.6 (the version pinned by the reference's
``requirements.txt:78``).  Only the padding step of padded cases runs through
the stand-in, so the border behaviour is pinned to OpenCV's *documented*
semantics, not to an OpenCV binary ("parity unpinned" for that step).

The float32 plane before quantisation is captured by wrapping the ``np``
module object seen by ``wicca.wavelet_coder`` so that ``np.clip`` records its
argument (``wavelet_coder.py:67``) — the reference code itself is unchanged.

Large inputs are not stored: they are regenerated from
``wicca_amd.synth.synth_image(seed, index, H, W, C)`` and only the SHA-256 of
the reference's output is recorded.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = "/root/reference"


def _install_cv2_standin() -> None:
    cv2 = types.ModuleType("cv2")
    cv2.BORDER_CONSTANT = 0
    cv2.BORDER_REPLICATE = 1

    def copyMakeBorder(src, top, bottom, left, right, borderType, dst=None, value=None):
        img = src[:, :, 0] if (src.ndim == 3 and src.shape[2] == 1) else src
        widths = [(top, bottom), (left, right)] + ([(0, 0)] if img.ndim == 3 else [])
        if borderType == cv2.BORDER_REPLICATE:
            return np.pad(img, widths, mode="edge")
        if borderType == cv2.BORDER_CONSTANT:
            v = value[0] if isinstance(value, (list, tuple)) else value
            return np.pad(img, widths, mode="constant", constant_values=v)
        raise NotImplementedError(f"stand-in supports REPLICATE/CONSTANT only, got {borderType}")

    cv2.copyMakeBorder = copyMakeBorder
    sys.modules["cv2"] = cv2


class _ClipRecorder(types.ModuleType):
    """Delegates to numpy; remembers the argument of the last np.clip call."""

    def __init__(self):
        super().__init__("np_recorder")
        self.last = None

    def __getattr__(self, name):
        return getattr(np, name)

    def clip(self, a, *args, **kwargs):
        self.last = np.array(a, copy=True)
        return np.clip(a, *args, **kwargs)


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main() -> None:
    _install_cv2_standin()
    sys.path.insert(0, REFERENCE)
    import wicca.wavelet_coder as wc  # noqa: E402  (reference, unmodified)

    sys.path.insert(0, REPO)
    from wicca_amd.synth import synth_image  # noqa: E402

    rec = _ClipRecorder()
    wc.np = rec
    coder = wc.HaarCoder()

    cases: list[dict] = []
    arrays: dict[str, np.ndarray] = {}
    rng = np.random.default_rng(20250919)

    def run(name, image, depth, border=1, k=0, store_input=True, synth=None,
            store_f32=True, positional=False):
        entry = {"name": name, "depth": depth, "border_type": border, "border_constant": k}
        if synth is not None:
            entry["synth"] = synth
        if isinstance(image, np.ndarray):
            entry["shape"] = list(image.shape)
            entry["dtype"] = str(image.dtype)
            entry["strides"] = list(image.strides)
        if store_input and isinstance(image, np.ndarray):
            base = image if image.flags.c_contiguous else np.ascontiguousarray(image)
            arrays[f"{name}__in"] = base
            entry["input_contiguous"] = bool(image.flags.c_contiguous)
        rec.last = None
        try:
            if positional:
                out = coder.get_small_copy(image, depth)
            else:
                out = coder.get_small_copy(image, depth, border_type=border, border_constant=k)
        except Exception as e:  # record the reference's failure
            entry["error"] = {"type": type(e).__name__, "message": str(e)}
            cases.append(entry)
            return
        entry["out_shape"] = list(out.shape)
        entry["out_dtype"] = str(out.dtype)
        entry["out_sha256"] = _sha(out)
        entry["out_c_contiguous"] = bool(out.flags.c_contiguous)
        if isinstance(image, np.ndarray):
            entry["out_shares_memory"] = bool(np.shares_memory(out, image))
        if out.size <= 1 << 16:
            arrays[f"{name}__out"] = out
        if store_f32 and rec.last is not None and rec.last.size <= 1 << 16:
            arrays[f"{name}__f32"] = rec.last.astype(np.float32)
            entry["has_f32"] = True
        cases.append(entry)

    # 1. random HWC images, C in {1,3,4}, aligned and unaligned, depth 0..10
    shapes = [(64, 64, 3), (37, 53, 3), (33, 17, 1), (32, 48, 1), (16, 16, 4),
              (29, 31, 4), (5, 7, 3), (1, 1, 3), (128, 96, 3), (45, 130, 2),
              (64, 256, 1)]
    for sh in shapes:
        img = rng.integers(0, 256, sh, dtype=np.uint8)
        for d in range(0, 11):
            if d >= 9 and sh[0] * sh[1] > 64 * 64:
                continue
            tag = "x".join(map(str, sh))
            run(f"rand_{tag}_d{d}_rep", img, d, border=1)
            if d in (1, 3, 5, 9):
                for k in (0, 7, 255):
                    run(f"rand_{tag}_d{d}_const{k}", img, d, border=0, k=k)

    # 2. wide / tall edge shapes crossing the kernel's 4096-pixel segments
    for sh, d in [((3, 4100, 3), 2), ((9, 4097, 1), 3), ((2, 8200, 3), 1),
                  ((40, 4608, 3), 5), ((17, 300, 3), 8), ((300, 5, 3), 8),
                  ((257, 520, 3), 8), ((520, 257, 1), 7)]:
        img = rng.integers(0, 256, sh, dtype=np.uint8)
        tag = "x".join(map(str, sh))
        run(f"edge_{tag}_d{d}_rep", img, d, border=1, store_f32=False)
        run(f"edge_{tag}_d{d}_const9", img, d, border=0, k=9, store_f32=False)

    # 3. adversarial depth >= 9: 255 everywhere but one 254 per 512x512 block
    adv = np.full((512, 512, 3), 255, np.uint8)
    adv[100, 200, 1] = 254
    for d in (9, 10):
        run(f"adv_512x512x3_d{d}_rep", adv, d, border=1)
        run(f"adv_512x512x3_d{d}_const255", adv, d, border=0, k=255)
    adv2 = np.full((1024, 1024, 1), 255, np.uint8)
    adv2[::512, ::512, 0] = 254
    run("adv_1024x1024x1_d10_rep", adv2, 10, border=1)
    run("adv_1024x1024x1_d11_rep", adv2, 11, border=1)

    # 4. extreme values
    for val in (0, 255):
        run(f"flat{val}_70x90x3_d4_rep", np.full((70, 90, 3), val, np.uint8), 4)

    # 5. strided (non-contiguous) views
    big = rng.integers(0, 256, (96, 120, 3), dtype=np.uint8)
    run("strided_rows_d2", big[::2], 2)
    run("strided_cols_d3", big[:, ::3], 3)
    run("strided_crop_d1", big[5:67, 7:101], 1)
    run("strided_chan_d2", big[:, :, ::-1], 2)
    run("strided_chan1_d2", big[:, :, 1:2], 2)

    # 6. negative depth: loop runs zero times, returns a copy
    img = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    run("neg_depth_-1", img, -1)
    run("neg_depth_-3", img, -3)
    run("positional_d2", img, 2, positional=True)

    # 7. error cases (type and message)
    run("err_none", None, 2, store_input=False)
    run("err_empty_rows", np.zeros((0, 5, 3), np.uint8), 2)
    run("err_empty_cols", np.zeros((5, 0, 3), np.uint8), 2)
    run("err_empty_chan", np.zeros((5, 5, 0), np.uint8), 2)
    run("err_float32", np.zeros((8, 8, 3), np.float32), 2)
    run("err_uint16", np.zeros((8, 8, 3), np.uint16), 2)
    run("err_list", [[1, 2], [3, 4]], 2, store_input=False)
    run("err_4d", np.zeros((4, 4, 3, 1), np.uint8), 1)
    run("err_1d", np.zeros((8,), np.uint8), 1)
    run("err_2d_gray_d1", rng.integers(0, 256, (8, 8), dtype=np.uint8), 1)
    run("ok_2d_gray_d0", rng.integers(0, 256, (8, 8), dtype=np.uint8), 0)
    run("err_hw1_padded_d2", rng.integers(0, 256, (6, 8, 1), dtype=np.uint8), 2)
    run("ok_hw1_aligned_d2", rng.integers(0, 256, (8, 8, 1), dtype=np.uint8), 2)

    # 8. BASELINE configs through the synthetic generator (hash only)
    #    config 1: one 2048x2048 grayscale image, depth 1 (as (H, W, 1))
    img = synth_image(1234, 0, 2048, 2048, 1)
    run("cfg1_2048x2048x1_d1", img, 1, store_input=False,
        synth={"seed": 1234, "index": 0}, store_f32=False)
    #    config 2/3 shapes, one image each, at the configured depths
    img = synth_image(0, 0, 2160, 3840, 3)
    run("cfg2_4k_d3", img, 3, store_input=False, synth={"seed": 0, "index": 0}, store_f32=False)
    img = synth_image(0, 1, 4320, 7680, 3)
    for d in range(1, 7):
        run(f"cfg3_8k_d{d}", img, d, store_input=False, synth={"seed": 0, "index": 1},
            store_f32=False)

    # 9. batch / depth-list groups whose members differ in alignment: the
    #    reference pads each image (and each depth) on its own, so a CONSTANT
    #    border must reach every unaligned member even when the first member
    #    needs no padding.  "group" names the batch / depth list a case belongs
    #    to; its members are listed in order.
    for k, d in ((77, 3), (0, 3), (200, 5)):
        members = [(64, 64, 3), (61, 59, 3), (32, 40, 3), (45, 130, 3), (64, 63, 3)]
        if d == 5:
            members = [(64, 96, 3), (70, 33, 3), (128, 32, 3), (97, 100, 3)]
        for j, sh in enumerate(members):
            img = rng.integers(0, 256, sh, dtype=np.uint8)
            run(f"group_batch_const{k}_d{d}_m{j}", img, d, border=0, k=k)
            cases[-1]["group"] = f"batch_const{k}_d{d}"
    for sh, k, depths in (((62, 62, 3), 77, (1, 3)), ((48, 40, 3), 5, (2, 3, 4, 5)),
                          ((64, 72, 4), 250, (3, 4, 6)), ((62, 62, 3), 77, (3, 1))):
        img = rng.integers(0, 256, sh, dtype=np.uint8)
        tag = "x".join(map(str, sh)) + "_" + "".join(map(str, depths))
        for d in depths:
            run(f"group_multi_{tag}_const{k}_d{d}", img, d, border=0, k=k)
            cases[-1]["group"] = f"multi_{tag}_const{k}"

    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "Todmount/wicca @ 2025-09-19 (wicca/wavelet_coder.py:50-67)",
                   "numpy": np.__version__,
                   "cases": cases}, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "arrays.npz"), **arrays)
    print(f"{len(cases)} cases, {len(arrays)} arrays")


if __name__ == "__main__":
    main()
