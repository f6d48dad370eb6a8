// nlh_fast_e15_16.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (15,2), (16,2), (15,1), (16,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<15, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<15, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<16, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<16, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<15, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<15, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<16, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<16, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
