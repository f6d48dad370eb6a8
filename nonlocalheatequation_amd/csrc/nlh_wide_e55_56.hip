// nlh_wide_e55_56.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 55..56 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<55, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<55, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<55>();
template int launch_wide_e<56, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<56, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<56>();
}  // namespace nlh
