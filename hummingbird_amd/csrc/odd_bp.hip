// odd_bp.hip — bit-plane record kernels (gf_odd_rec<K, R, 0, XS>, odd_impl.h):
// one instance per compiled encode schedule of xor_sched.h, in their own unit
// so the build compiles them in parallel with the table kernels.
#include <utility>

#include "odd_impl.h"

namespace hbec {

template <int... I>
static const void* odd_bp_pick(int xs, bool list, std::integer_sequence<int, I...>) {
    static const void* const fns[] = {(const void*)&gf_odd_rec<XorNet<I>::K, XorNet<I>::R, kOddApply, I>...};
    static const void* const lfns[] = {(const void*)&gf_odd_rec<XorNet<I>::K, XorNet<I>::R, kOddApply, I, true>...};
    return xs >= 0 && xs < (int)sizeof...(I) ? (list ? lfns[xs] : fns[xs]) : nullptr;
}

template <int... I>
static const void* odd_bp_verify_pick(int xs, std::integer_sequence<int, I...>) {
    static const void* const fns[] = {(const void*)&gf_odd_rec<XorNet<I>::K, XorNet<I>::R, kOddVerify, I>...};
    return xs >= 0 && xs < (int)sizeof...(I) ? fns[xs] : nullptr;
}

const void* odd_kernel_bp(int xs, int mode, bool list) {
    if (mode == kOddVerify)
        return list ? nullptr : odd_bp_verify_pick(xs, std::make_integer_sequence<int, kXorShapeCount>{});
    return mode == kOddApply ? odd_bp_pick(xs, list, std::make_integer_sequence<int, kXorShapeCount>{}) : nullptr;
}

}  // namespace hbec
