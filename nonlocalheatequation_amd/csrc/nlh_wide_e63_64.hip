// nlh_wide_e63_64.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 63..64 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<63, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<63, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<63>();
template int launch_wide_e<64, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<64, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<64>();
}  // namespace nlh
