"""Depth-list semantics of the icon stage.

Mirrors ``normalize_depth`` (reference ``wicca/normalization.py:23-55``):
``ClassifierProcessor`` normalises its ``depth`` argument to a tuple and runs
the coder once per element (``classifying_tools.py:546-551``);
``HaarCoder.get_small_copy_multi(image, normalize_depth(depth))`` serves that
loop from one read.  Same accepted forms, same ValueError messages (pinned by
``tests/golden/normalize_depth.json``, produced by the reference itself).
"""
from __future__ import annotations

from typing import Union

Depth = Union[int, tuple, list, range]

MSG_NONE = "Depth must be provided"
MSG_FORM = "Depth must be a positive integer, tuple, list, or range"
MSG_ELEMS = "All depths must be integers greater than 0"


def normalize_depth(depth: Depth) -> tuple:
    """A positive int becomes a 1-tuple; a tuple / list / range becomes a tuple
    whose elements must all be ints > 0 (bool counts as int, as in Python)."""
    if depth is None:
        raise ValueError(MSG_NONE)
    if isinstance(depth, int) and depth > 0:
        return (depth,)
    if not isinstance(depth, (tuple, list, range)):
        raise ValueError(MSG_FORM)
    out = tuple(depth)
    for x in out:
        if not (isinstance(x, int) and x > 0):
            raise ValueError(MSG_ELEMS)
    return out
