// odd_k912.hip — gf_odd kernel instances for K = 9..kOddMaxK (12) inputs
// (odd_impl.h), in their own unit so the build compiles them in parallel.
#include "odd_impl.h"

namespace hbec {

const void* odd_kernel_k912(int k, int r, int mode, bool plan, bool mirror, bool variant, bool list) {
    return odd_kernel_range<9, kOddMaxK>(k, r, mode, plan, mirror, variant, list);
}

}  // namespace hbec
