// nlh_pair_e1_4.hip -- explicit instantiations of the two-step pass (nlh_pair.h)
// for E = 1..4; split per horizon range so the unrolled kernels compile in parallel.
#include "nlh_pair.h"

namespace nlh {
template int launch_pair_e<1>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<1>(int);
template int launch_pair_e<2>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<2>(int);
template int launch_pair_e<3>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<3>(int);
template int launch_pair_e<4>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<4>(int);
}  // namespace nlh
