// nlh_wide_e59_60.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 59..60 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<59, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<59, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<59>();
template int launch_wide_e<60, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<60, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<60>();
}  // namespace nlh
