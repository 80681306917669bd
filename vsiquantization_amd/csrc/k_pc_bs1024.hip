// k_pc_bs1024.hip — K3 instantiations for 1024-lane workgroups (split for parallel builds).
#include "k_pc.cuh"

namespace vsiq {
template bool launch_pc_bs<true, true, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, true, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
}  // namespace vsiq
