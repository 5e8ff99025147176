// haar_multi_d57.hip — K5 instantiations for DMIN in {5, 6, 7} (see haar_multi_impl.h).
#include "haar_multi_impl.h"

namespace wicca {
template hipError_t launch_multi_dc<5, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<5, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<5, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<5, 4>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<6, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<6, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<6, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<6, 4>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<7, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<7, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<7, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<7, 4>(int, const MultiParams&, int64_t, hipStream_t);
}  // namespace wicca
