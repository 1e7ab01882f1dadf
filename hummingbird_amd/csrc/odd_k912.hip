// odd_k912.hip — gf_odd kernel instances for K = 9..12 inputs (odd_impl.h),
// built when HBEC_ODD_MAXK >= 12 (kernels.h); empty otherwise.
#include "odd_impl.h"

namespace hbec {

const void* odd_kernel_k912(int k, int r, int mode, bool plan, bool mirror) {
    return odd_kernel_range<9, (HBEC_ODD_MAXK >= 12 ? 12 : 8)>(k, r, mode, plan, mirror);
}

}  // namespace hbec
