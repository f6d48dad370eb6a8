// nlh_fast_e13_14.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (13,2), (14,2), (13,1), (14,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<13, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<13, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<14, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<14, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<13, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<13, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<14, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<14, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
