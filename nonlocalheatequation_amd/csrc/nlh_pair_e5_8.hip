// nlh_pair_e5_8.hip -- explicit instantiations of the two-step pass (nlh_pair.h)
// for E = 5..8; split per horizon range so the unrolled kernels compile in parallel.
#include "nlh_pair.h"

namespace nlh {
template int launch_pair_e<5>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<5>(int);
template int launch_pair_e<6>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<6>(int);
template int launch_pair_e<7>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<7>(int);
template int launch_pair_e<8>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<8>(int);
}  // namespace nlh
