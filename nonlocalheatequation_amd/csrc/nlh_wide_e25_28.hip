// nlh_wide_e25_28.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 25..28; split per horizon range so the unrolled
// kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<25, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<25, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<26, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<26, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<27, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<27, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<28, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<28, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<25>();
template int wide_blocks_per_cu_e<26>();
template int wide_blocks_per_cu_e<27>();
template int wide_blocks_per_cu_e<28>();
}  // namespace nlh
