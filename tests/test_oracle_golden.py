"""The CPU oracle reproduces the reference's golden vectors bit for bit (no GPU).

Pins oracle/haar_numpy.py (NumPy restatement, also the CPU baseline) and
oracle/haar_oracle.c (float32 per-level emulation and exact integer block
sums) against outputs of the reference HaarCoder itself
(tests/golden/make_golden.py).
"""
import numpy as np
import pytest

import golden_cases as G
from oracle import c_oracle, haar_numpy

OK = G.cases("ok")
ERR = G.cases("error")


def _ids(cs):
    return [c["name"] for c in cs]


@pytest.mark.parametrize("case", OK,
                         ids=lambda c: c["name"])
def test_numpy_port_matches_reference(case):
    img = G.input_of(case)
    out = haar_numpy.get_small_copy(img, case["depth"], case["border_type"],
                                    case["border_constant"])
    assert list(out.shape) == case["out_shape"]
    assert G.sha(out) == case["out_sha256"]
    f32 = G.f32_of(case)
    if f32 is not None:
        plane = haar_numpy.get_small_copy_f32(img, case["depth"], case["border_type"],
                                              case["border_constant"])
        assert np.array_equal(plane.view(np.uint32), f32.view(np.uint32))


@pytest.mark.parametrize("case", [c for c in OK if len(c.get("shape", [])) == 3
                                  and c["depth"] >= 1 and np.prod(c["shape"]) <= 3_000_000],
                         ids=lambda c: c["name"])
def test_c_oracle_matches_reference(case):
    img = np.ascontiguousarray(G.input_of(case))
    d, b, k = case["depth"], case["border_type"], case["border_constant"]
    u8, f = c_oracle.ll_f32_levels(img, d, b, k)
    assert G.sha(u8) == case["out_sha256"]
    f32 = G.f32_of(case)
    if f32 is not None:
        assert np.array_equal(f.view(np.uint32), f32.view(np.uint32))
    if d <= 8:
        u8i, s = c_oracle.ll_int_block(img, d, b, k)
        assert G.sha(u8i) == case["out_sha256"]
        # the float plane is exactly S / 4^D for D <= 8
        assert np.array_equal(f, (s.astype(np.float64) / 4.0 ** d).astype(np.float32))


@pytest.mark.parametrize("case", ERR, ids=_ids(ERR))
def test_numpy_port_errors_match_reference(case):
    img = G.input_of(case) if "shape" in case else (
        None if case["name"] == "err_none" else [[1, 2], [3, 4]])
    with pytest.raises(Exception) as ei:
        haar_numpy.get_small_copy(img, case["depth"], case["border_type"],
                                  case["border_constant"])
    assert type(ei.value).__name__ == case["error"]["type"]
    assert str(ei.value) == case["error"]["message"]


def test_depth9_adversarial_rounding_is_the_references():
    """Depth >= 9: float32 rounding makes the reference differ from floor(S/4^D)."""
    case = next(c for c in OK if c["name"] == "adv_512x512x3_d9_rep")
    img = G.input_of(case)
    exact = int(img.astype(np.int64).sum(axis=(0, 1))[1]) // (512 * 512)
    assert exact == 254
    assert G.expected_of(case)[0, 0, 1] == 255
    assert c_oracle.ll_f32_levels(img, 9)[0][0, 0, 1] == 255


def test_synth_host_matches_c_oracle():
    from wicca_amd.synth import synth_image
    for seed, idx, shape in [(0, 0, (7, 9, 3)), (1234, 5, (3, 17, 1)), (2**40 + 3, 2, (4, 5, 4))]:
        a = synth_image(seed, idx, *shape)
        b = c_oracle.synth_u8(1, *shape, seed, idx)[0]
        assert np.array_equal(a, b)


def test_synth_rows_is_a_slice_of_synth_image():
    from wicca_amd.synth import synth_image, synth_rows
    img = synth_image(3, 1, 11, 7, 3)
    for a, b in ((0, 11), (1, 2), (3, 9), (10, 11)):
        assert np.array_equal(synth_rows(3, 1, a, b - a, 7, 3), img[a:b])
