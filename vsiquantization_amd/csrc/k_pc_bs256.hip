// k_pc_bs256.hip — K3 instantiations for 256-lane workgroups (split for parallel builds).
#include "k_pc.cuh"

namespace vsiq {
template bool launch_pc_bs<true, true, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, true, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<true, false, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
template bool launch_pc_bs<false, false, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
}  // namespace vsiq
