// k_pc_bs512.hip — K3 instantiations for 512-lane workgroups (split for parallel builds).
#include "k_pc.cuh"

namespace vsiq {
template bool launch_pc_bs<true, true, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, true, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
}  // namespace vsiq
