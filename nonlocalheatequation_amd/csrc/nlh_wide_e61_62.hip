// nlh_wide_e61_62.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 61..62 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<61, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<61, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<61>();
template int launch_wide_e<62, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<62, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<62>();
}  // namespace nlh
