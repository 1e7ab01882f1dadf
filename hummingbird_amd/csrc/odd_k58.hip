// odd_k58.hip — gf_odd kernel instances for K = 5..8 inputs (odd_impl.h).
#include "odd_impl.h"

namespace hbec {

const void* odd_kernel_k58(int k, int r, int mode, bool plan, bool mirror, bool variant, bool list) {
    return odd_kernel_range<5, 8>(k, r, mode, plan, mirror, variant, list);
}

}  // namespace hbec
