"""Golden vectors for the depth-list semantics (run in the survey container only).

    python tests/golden/make_normalize_golden.py   # writes tests/golden/normalize_depth.json

Imports the REFERENCE ``wicca.normalization.normalize_depth``
(``/root/reference/wicca/normalization.py:23-55``, unmodified; its imports
need neither cv2 nor tensorflow) and records, for each input, the returned
tuple or the exception type and message.  Only these input/output pairs are
stored.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REFERENCE = "/root/reference"

# (label, python expression of the input) — evaluated here and in the test
CASES = [
    ("int", "3"), ("one", "1"), ("zero", "0"), ("negative", "-2"), ("none", "None"),
    ("tuple", "(1, 2, 3)"), ("list", "[4, 2]"), ("range", "range(1, 7)"),
    ("empty_tuple", "()"), ("empty_list", "[]"), ("tuple_with_zero", "(1, 0)"),
    ("list_with_str", "[1, 'a']"), ("float", "2.5"), ("str", "'3'"), ("bool", "True"),
    ("tuple_of_bools", "(True, 2)"), ("nested", "[(1, 2)]"), ("float_in_list", "[1.0]"),
    ("large", "(9, 12)"), ("set", "{1, 2}"),
]


def main() -> None:
    sys.path.insert(0, REFERENCE)
    from wicca.normalization import normalize_depth  # reference, unmodified

    out = []
    for label, expr in CASES:
        entry = {"name": label, "input": expr}
        try:
            entry["output"] = list(normalize_depth(eval(expr)))  # noqa: S307 (fixed literals)
        except Exception as e:  # noqa: BLE001 — the reference's exception is the vector
            entry["error"] = type(e).__name__
            entry["message"] = str(e)
        out.append(entry)
    with open(os.path.join(HERE, "normalize_depth.json"), "w") as f:
        json.dump({"source": "reference wicca/normalization.py:23-55", "cases": out}, f, indent=1)
    print(f"{len(out)} cases")


if __name__ == "__main__":
    main()
