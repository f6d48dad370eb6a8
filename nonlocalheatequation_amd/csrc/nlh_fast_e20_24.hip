// nlh_fast_e20_24.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (20,1), (24,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<20, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<20, 1, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<24, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<24, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
