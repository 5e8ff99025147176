// haar_multi_d12.hip — K5 instantiations for DMIN in {1, 2} (see haar_multi_impl.h).
#include "haar_multi_impl.h"

namespace wicca {
#if WICCA_MULTI_D1
template hipError_t launch_multi_dc<1, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<1, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<1, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<1, 4>(int, const MultiParams&, int64_t, hipStream_t);
#endif
template hipError_t launch_multi_dc<2, 1>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<2, 2>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<2, 3>(int, const MultiParams&, int64_t, hipStream_t);
template hipError_t launch_multi_dc<2, 4>(int, const MultiParams&, int64_t, hipStream_t);
}  // namespace wicca
