// nlh_wide_e41_44.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 41..44 (8-row chunks); split per horizon range so
// the unrolled kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<41, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<41, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<41>();
template int launch_wide_e<42, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<42, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<42>();
template int launch_wide_e<43, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<43, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<43>();
template int launch_wide_e<44, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<44, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<44>();
}  // namespace nlh
