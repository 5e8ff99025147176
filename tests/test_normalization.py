"""normalize_depth against the reference's own outputs (tests/golden/normalize_depth.json)."""
import json
import os

import pytest

from wicca_amd import normalize_depth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "normalize_depth.json")
CASES = json.load(open(GOLDEN))["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_normalize_depth_matches_reference(case):
    value = eval(case["input"])  # noqa: S307 — fixed literals written by the generator
    if "error" in case:
        with pytest.raises(ValueError) as ei:
            normalize_depth(value)
        assert type(ei.value).__name__ == case["error"]
        assert str(ei.value) == case["message"]
    else:
        out = normalize_depth(value)
        assert isinstance(out, tuple)
        assert list(out) == case["output"]
        assert [type(x) for x in out] == [type(x) for x in case["output"]]
