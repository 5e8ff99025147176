"""Host-side contract of the drop-in HaarCoder, checked without a GPU.

Every error the reference raises (tests/golden error cases) is raised by
wicca_amd.HaarCoder before any device work, with the same type and text.
"""
import inspect

import numpy as np
import pytest

import golden_cases as G
from oracle import c_oracle
from wicca_amd import BORDER_REPLICATE, HaarCoder, WaveletCoder
from wicca_amd.coder import _as_hwc, _pad_amounts

ERR = G.cases("error")


@pytest.fixture(scope="module")
def host_coder():
    return HaarCoder()  # constructing loads the library; no device call


def _input(case):
    if "shape" in case:
        return G.input_of(case)
    return None if case["name"] == "err_none" else [[1, 2], [3, 4]]


@pytest.mark.parametrize("case", ERR, ids=[c["name"] for c in ERR])
def test_errors_match_reference(host_coder, case):
    img = _input(case)
    with pytest.raises(Exception) as ei:
        host_coder.get_small_copy(img, case["depth"], case["border_type"],
                                  case["border_constant"])
    assert type(ei.value).__name__ == case["error"]["type"]
    assert str(ei.value) == case["error"]["message"]


def test_signature_matches_reference():
    sig = inspect.signature(HaarCoder.get_small_copy)
    assert list(sig.parameters) == ["self", "image", "transform_depth", "border_type",
                                    "border_constant"]
    assert sig.parameters["border_type"].default == BORDER_REPLICATE == 1
    assert sig.parameters["border_constant"].default == 0
    assert issubclass(HaarCoder, WaveletCoder)
    assert HaarCoder()._ONE_STEP_RATIO == 2


def test_non_integer_depth_raises_type_error(host_coder):
    with pytest.raises(TypeError):
        host_coder.get_small_copy(np.zeros((8, 8, 3), np.uint8), 2.0)


@pytest.mark.parametrize("H,W,d", [(4320, 7680, 1), (4320, 7680, 6), (2160, 3840, 3),
                                   (37, 53, 5), (1, 1, 8), (65536, 65536, 8)])
def test_pad_rule_matches_oracle(H, W, d):
    ar, ac = _pad_amounts(H, W, d)
    oh, ow = c_oracle.icon_shape(H, W, d)
    assert (H + ar) >> d == oh and (W + ac) >> d == ow


def test_hwc_view_keeps_strided_rows_without_copy():
    base = np.zeros((40, 50, 3), np.uint8)
    view = base[::2]
    v = _as_hwc(view)
    assert np.shares_memory(v, base) and v.strides[0] == 2 * 50 * 3
    assert not np.shares_memory(_as_hwc(base[:, ::2]), base)
    gray = np.zeros((6, 8), np.uint8)
    assert _as_hwc(gray).shape == (6, 8, 1)
