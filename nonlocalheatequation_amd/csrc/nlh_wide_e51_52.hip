// nlh_wide_e51_52.hip -- explicit instantiations of the large-horizon kernel k_wide
// (nlh_wide.h) for E = 51..52 (8-row chunks, accumulators partly in AGPRs,
// one wave per SIMD); two horizons per unit so the unrolled kernels compile in
// parallel.
#include "nlh_wide.h"

namespace nlh {
template int launch_wide_e<51, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<51, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<51>();
template int launch_wide_e<52, true>(const RectList &, const StepConst &, hipStream_t);
template int launch_wide_e<52, false>(const RectList &, const StepConst &, hipStream_t);
template int wide_blocks_per_cu_e<52>();
}  // namespace nlh
