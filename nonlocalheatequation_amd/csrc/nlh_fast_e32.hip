// nlh_fast_e32.hip -- explicit instantiations of the fast kernel (nlh_fast.h) for
// (E, R) = (32,1).  Split per horizon range so the
// fully unrolled kernels compile in parallel.
#include "nlh_fast.h"

namespace nlh {
template int launch_fast_er<32, 1, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_fast_er<32, 1, false>(const RectList &, const StepConst &, hipStream_t);
}  // namespace nlh
