// internal.h — helpers shared by the libhbec translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/hbec.h"

namespace hbec {

// Record a thread-local error message and return code.
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Queue out[r] (^)= XOR_c coeffs[r][c] * in[c] over n_obj strided objects.
int apply_views(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                uint64_t n_obj, uint64_t shard_len, hipStream_t stream);

}  // namespace hbec
