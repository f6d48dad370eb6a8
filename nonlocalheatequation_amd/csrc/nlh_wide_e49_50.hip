// nlh_wide_e49_50.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 49..50 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<49, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<49, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<49>();
template int launch_wide_e<50, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<50, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<50>();
}  // namespace nlh
