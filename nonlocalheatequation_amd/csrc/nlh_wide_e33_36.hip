// nlh_wide_e33_36.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 33..36 (8-row chunks); split per horizon range so
// the unrolled kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<33, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<33, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<33>();
template int launch_wide_e<34, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<34, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<34>();
template int launch_wide_e<35, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<35, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<35>();
template int launch_wide_e<36, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<36, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<36>();
}  // namespace nlh
