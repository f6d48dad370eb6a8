// nlh_wide_rt.hip -- instantiation unit of the run-time-horizon large-eps
// kernel k_wide_rt (nlh_wide_rt.h; J = 1, eps 49 .. 64).
#include "nlh_wide_rt.h"

namespace nlh {
template int launch_wide_rt_t<true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_rt_t<false>(const RectList &, const StepConst &, hipStream_t);

int wide_rt_blocks_per_cu() { return wide_rt_blocks_per_cu_t<false>(); }
}  // namespace nlh
