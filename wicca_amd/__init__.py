"""wicca_amd — MI355X-native Haar LL ("icon") engine for Todmount/wicca.

Drop-in for the reference's one hot path, ``HaarCoder.get_small_copy``
(``wicca/wavelet_coder.py:50-67``), computed by hand-written gfx950 HIP
kernels behind the C ABI in ``include/wicca_haar.h``.

    from wicca_amd import HaarCoder
    coder = HaarCoder()
    icon = coder.get_small_copy(image, transform_depth=5)
"""
from .coder import (BORDER_CONSTANT, BORDER_REFLECT, BORDER_REFLECT_101, BORDER_REPLICATE,
                    BORDER_WRAP, HaarCoder, WaveletCoder)
from .normalization import normalize_depth
from .jpeg import get_img_batch, get_img_batches, load_image
from .plan import StagePlan, folder_batches, get_img_matrix
from .resize import (INTER_AREA, INTER_CUBIC, INTER_LANCZOS4, INTER_LINEAR, INTER_LINEAR_EXACT, INTER_NEAREST,
                     INTER_NEAREST_EXACT, resize)
from .validation import validate_image

__all__ = ["HaarCoder", "WaveletCoder", "validate_image", "normalize_depth", "BORDER_CONSTANT", "BORDER_REPLICATE",
           "BORDER_REFLECT", "BORDER_WRAP", "BORDER_REFLECT_101", "resize", "INTER_NEAREST",
           "INTER_LINEAR", "INTER_AREA", "INTER_CUBIC", "INTER_LANCZOS4", "INTER_LINEAR_EXACT",
           "INTER_NEAREST_EXACT", "load_image", "get_img_batch", "get_img_batches", "StagePlan", "get_img_matrix",
           "folder_batches"]
__version__ = "0.2.0"
