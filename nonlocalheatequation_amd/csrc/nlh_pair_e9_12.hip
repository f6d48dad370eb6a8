// nlh_pair_e9_12.hip -- explicit instantiations of the two-step pass (nlh_pair.h)
// for E = 9..12; split per horizon range so the unrolled kernels compile in parallel.
#include "nlh_pair.h"

namespace nlh {
template int launch_pair_e<9>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<9>(int);
template int launch_pair_e<10>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<10>(int);
template int launch_pair_e<11>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<11>(int);
template int launch_pair_e<12>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<12>(int);
}  // namespace nlh
