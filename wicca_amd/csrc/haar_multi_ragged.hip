// haar_multi_ragged.hip — K5 over a ragged batch (per-image descriptors), the
// multi-depth icons of the file stage's decoded RGB images (SURVEY 8f item 1;
// see haar_multi_impl.h).  C = 3 only: decoded files are always RGB.
#include "haar_multi_impl.h"

namespace wicca {
#if WICCA_MULTI_D1
template hipError_t launch_multi_ragged_dc<1, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
#endif
template hipError_t launch_multi_ragged_dc<2, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_ragged_dc<3, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_ragged_dc<4, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_ragged_dc<5, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_ragged_dc<6, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_ragged_dc<7, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
}  // namespace wicca
