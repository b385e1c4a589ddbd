// SPDX-License-Identifier: MIT
// Explicit instantiation of the fused kernel's launcher for double (its own translation unit, so the
// heavy kernel instantiations of fused.hpp compile in parallel with the rest of libgs_hip.so).
#include "../kernels.hpp"

namespace gsk {
template bool launch_fused<double>(const typename Vec2<double>::type*, typename Vec2<double>::type*,
                               const Geom&, const gs::Params&, int, int64_t, hipStream_t, int,
                               int, int, int, int, int, int, int, bool,
                               const GateLaunch*);
template int fused_gated_occupancy<double>(int, int, bool);
}  // namespace gsk
