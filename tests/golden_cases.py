"""Loader for the reference golden vectors in tests/golden (see make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_CACHE: dict = {}


def load():
    if not _CACHE:
        with open(os.path.join(HERE, "cases.json")) as f:
            _CACHE["meta"] = json.load(f)
        _CACHE["arrays"] = np.load(os.path.join(HERE, "arrays.npz"), allow_pickle=False)
    return _CACHE["meta"], _CACHE["arrays"]


def cases(kind: str = "ok", max_pixels: int | None = None):
    meta, _ = load()
    out = []
    for c in meta["cases"]:
        is_err = "error" in c
        if kind == "ok" and is_err:
            continue
        if kind == "error" and not is_err:
            continue
        if max_pixels is not None and "shape" in c and np.prod(c["shape"][:2]) > max_pixels:
            continue
        out.append(c)
    return out


def input_of(case):
    """The exact input the reference saw (regenerated for synthetic cases)."""
    _, arrays = load()
    if "synth" in case:
        from wicca_amd.synth import synth_image
        H, W, C = case["shape"]
        return synth_image(case["synth"]["seed"], case["synth"]["index"], H, W, C)
    key = case["name"] + "__in"
    if key not in arrays:
        return None
    img = arrays[key]
    # rebuild the non-contiguous view the reference received
    if not case.get("input_contiguous", True):
        name = case["name"]
        if name == "strided_chan_d2":
            base = np.empty(img.shape, np.uint8)
            base[:, :, ::-1] = img
            img = base[:, :, ::-1]
        else:
            pad = np.zeros((img.shape[0] * 2 + 3, img.shape[1] * 3 + 5, img.shape[2]), np.uint8)
            pad[1:1 + 2 * img.shape[0]:2, 2:2 + 3 * img.shape[1]:3] = img
            img = pad[1:1 + 2 * img.shape[0]:2, 2:2 + 3 * img.shape[1]:3]
    return img


def expected_of(case):
    _, arrays = load()
    key = case["name"] + "__out"
    return arrays[key] if key in arrays else None


def f32_of(case):
    _, arrays = load()
    key = case["name"] + "__f32"
    return arrays[key] if key in arrays else None


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def groups(prefix: str):
    """{group name: [cases in order]} for batch ("batch_") or depth-list
    ("multi_") groups (make_golden.py section 9)."""
    out: dict = {}
    for c in cases("ok"):
        g = c.get("group")
        if g and g.startswith(prefix):
            out.setdefault(g, []).append(c)
    return out
