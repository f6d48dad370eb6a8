// nlh_wide_e53_54.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 53..54 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<53, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<53, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<53>();
template int launch_wide_e<54, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<54, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<54>();
}  // namespace nlh
