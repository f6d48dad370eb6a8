// nlh_wide_e17_20.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 17..20; split per horizon range so the unrolled
// kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<17, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<17, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<18, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<18, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<19, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<19, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<20, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<20, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<17>();
template int wide_blocks_per_cu_e<18>();
template int wide_blocks_per_cu_e<19>();
template int wide_blocks_per_cu_e<20>();
}  // namespace nlh
