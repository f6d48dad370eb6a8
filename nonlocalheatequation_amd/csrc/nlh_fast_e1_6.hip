// nlh_fast_e1_6.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (1,2), (2,2), (3,2), (4,2), (5,2), (6,2), (1,4), (2,4), (3,4), (4,4), (5,4), (6,4), (1,1), (2,1), (3,1), (4,1), (5,1), (6,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<1, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<1, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 2, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 2, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<1, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<1, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 4, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 4, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<1, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<1, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<2, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<3, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<4, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<5, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<6, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
