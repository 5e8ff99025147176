"""Input contract of the icon path (mirror of ``wicca/validation.py:80-101``).

Same checks, same order, same exception types and messages as the
reference's ``validate_image``.  The reference's final ``np.max(image) > 255``
test can never fire for uint8 data and costs a full read of the
image, so it is not repeated here.
"""
from __future__ import annotations

import numpy as np

MSG_NONE = "Image didn't found. Please check your input."
MSG_EMPTY = "Image is empty"
MSG_DTYPE = "Image must be of type uint8"
MSG_NDIM = "Image must be 2D or 3D array"
MSG_NOT_ARRAY = "Image must be a numpy array"
MSG_2D_INDEX = "too many indices for array: array is 2-dimensional, but 3 were indexed"


def validate_image(image) -> None:
    """Raise ``ValueError`` for a missing, empty or non-uint8 image.

    Reference: ``wicca/validation.py:93-99``.  Like the reference, an object
    without ``.shape`` raises ``AttributeError`` and a 1-D array raises
    ``IndexError`` from ``shape[1]``.
    """
    if image is None:
        raise ValueError(MSG_NONE)
    if image.shape[0] == 0 or image.shape[1] == 0 or image.size == 0:
        raise ValueError(MSG_EMPTY)
    if image.dtype != np.uint8:
        raise ValueError(MSG_DTYPE)
