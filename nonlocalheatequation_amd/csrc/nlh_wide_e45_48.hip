// nlh_wide_e45_48.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 45..48 (8-row chunks); split per horizon range so
// the unrolled kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<45, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<45, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<45>();
template int launch_wide_e<46, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<46, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<46>();
template int launch_wide_e<47, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<47, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<47>();
template int launch_wide_e<48, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<48, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<48>();
}  // namespace nlh
