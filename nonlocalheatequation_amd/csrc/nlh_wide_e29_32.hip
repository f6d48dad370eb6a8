// nlh_wide_e29_32.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 29..32; split per horizon range so the unrolled
// kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<29, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<29, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<30, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<30, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<31, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<31, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<32, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<32, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<29>();
template int wide_blocks_per_cu_e<30>();
template int wide_blocks_per_cu_e<31>();
template int wide_blocks_per_cu_e<32>();
}  // namespace nlh
