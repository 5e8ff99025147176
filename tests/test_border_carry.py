"""CPU: the host layer hands the caller's border and constant to every launch.

Regression for the round-1 defect where a batch (or depth list) whose first
member needed no padding launched with REPLICATE / k=0, so later unaligned
members were padded wrongly (reference: data_loader.py:107-117 pads each
image with the caller's border).  The C ABI is replaced by a recorder, so
this runs without a GPU.
"""
import numpy as np

from wicca_amd import HaarCoder, _lib


class _Recorder:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def fn(*args):
            self.calls.append((name, args))
            return 0
        return fn


def _coder():
    c = HaarCoder.__new__(HaarCoder)
    c._ONE_STEP_RATIO = 2
    c.device = -1
    c._lib = _Recorder()
    return c


def test_batch_constant_first_member_aligned():
    c = _coder()
    imgs = [np.zeros((64, 64, 3), np.uint8), np.zeros((61, 59, 3), np.uint8)]
    c.get_small_copies(imgs, 3, 0, 77)
    (name, args), = c._lib.calls
    assert name == "wicca_haar_ll_u8_batch"
    assert args[3:6] == (3, 0, 77)  # depth, border, k
    c = _coder()
    c.get_small_copies(imgs, 3, 0, 77, devices=[0, 1])
    (name, args), = c._lib.calls
    assert name == "wicca_haar_ll_u8_batch_multi_gpu"
    assert args[3:6] == (3, 0, 77)


def test_multi_constant_smallest_depth_aligned():
    c = _coder()
    c.get_small_copy_multi(np.zeros((62, 62, 3), np.uint8), [1, 3], 0, 77)
    (name, args), = c._lib.calls
    assert name == "wicca_haar_ll_u8_multi"
    assert args[7:9] == (0, 77)  # border, k


def test_single_aligned_keeps_constant():
    c = _coder()
    c.get_small_copy(np.zeros((64, 64, 3), np.uint8), 3, 0, 300)
    (name, args), = c._lib.calls
    assert args[6:8] == (0, 255)  # saturated like OpenCV's scalar


def test_exotic_border_batch_is_host_padded_replicate():
    c = _coder()
    imgs = [np.zeros((64, 64, 3), np.uint8), np.zeros((61, 59, 3), np.uint8)]
    c.get_small_copies(imgs, 3, 2, 0)
    (name, args), = c._lib.calls
    assert args[4:6] == (1, 0)
    descs = args[0]
    assert (descs[1].height, descs[1].width) == (64, 64)  # padded on the host


def test_unknown_border_on_aligned_image_is_accepted():
    # reference: no padding needed -> cv2 is never called with the border
    c = _coder()
    c.get_small_copy(np.zeros((64, 64, 3), np.uint8), 3, 7, 0)
    (name, args), = c._lib.calls
    assert args[6] == 1
