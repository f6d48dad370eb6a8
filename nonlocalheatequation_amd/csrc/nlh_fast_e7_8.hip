// nlh_fast_e7_8.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (7,2), (8,2), (7,4), (8,4), (7,1), (8,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<7, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<7, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<7, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<7, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<7, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<7, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<8, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
