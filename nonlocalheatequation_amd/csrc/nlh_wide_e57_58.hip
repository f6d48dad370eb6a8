// nlh_wide_e57_58.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 57..58 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<57, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<57, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<57>();
template int launch_wide_e<58, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<58, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<58>();
}  // namespace nlh
