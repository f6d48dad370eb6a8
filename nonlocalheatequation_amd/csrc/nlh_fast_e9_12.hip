// nlh_fast_e9_12.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (9,2), (10,2), (11,2), (12,2), (9,1), (10,1), (11,1), (12,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<9, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<9, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<10, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<10, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<11, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<11, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<12, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<12, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<9, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<9, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<10, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<10, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<11, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<11, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<12, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<12, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
