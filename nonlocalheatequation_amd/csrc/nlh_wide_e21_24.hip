// nlh_wide_e21_24.hip -- explicit instantiations of the large-horizon kernel
// k_wide (nlh_wide.h) for E = 21..24; split per horizon range so the unrolled
// kernels compile in parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<21, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<21, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<22, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<22, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<23, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<23, false>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<24, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<24, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<21>();
template int wide_blocks_per_cu_e<22>();
template int wide_blocks_per_cu_e<23>();
template int wide_blocks_per_cu_e<24>();
}  // namespace nlh
