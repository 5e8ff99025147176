// haar_multi_d34.hip — K5 instantiations for DMIN in {3, 4} (see haar_multi_impl.h).
#include "haar_multi_impl.h"

namespace wicca {
template hipError_t launch_multi_dc<3, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<3, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<3, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<3, 4>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<4, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<4, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<4, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<4, 4>(int, const MultiParams&, int64_t, hipStream_t);
}  // namespace wicca
