// nlh_pair_e13_16.hip -- explicit instantiations of the two-step pass (nlh_pair.h)
// for E = 13..16; split per horizon range so the unrolled kernels compile in parallel.
#include "nlh_pair.h"

namespace nlh {
template int launch_pair_e<13>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<13>(int);
template int launch_pair_e<14>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<14>(int);
template int launch_pair_e<15>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<15>(int);
template int launch_pair_e<16>(const RectList &, const StepConst &, int, hipStream_t);
template int pair_blocks_per_cu_e<16>(int);
}  // namespace nlh
