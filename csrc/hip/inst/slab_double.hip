// SPDX-License-Identifier: MIT
// Explicit instantiation of the overlap shell's launcher (slab.hpp) for double (own translation unit).
#include "../kernels.hpp"

namespace gsk {
template bool launch_shell<double>(const void*, void*, const Geom&, const gs::Params&, int, int64_t,
                               int, int, hipStream_t);
}  // namespace gsk
