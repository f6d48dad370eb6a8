// nlh_wide_e37_40.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 37..40 (8-row chunks); split per horizon range so
// the unrolled kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<37, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<37, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<37>();
template int launch_wide_e<38, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<38, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<38>();
template int launch_wide_e<39, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<39, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<39>();
template int launch_wide_e<40, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<40, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<40>();
}  // namespace nlh
