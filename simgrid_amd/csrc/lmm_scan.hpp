// lmm_scan.hpp — hipCUB-backed device primitives (lmm_scan.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lmmdev {

hipError_t scan_i64(void* tmp, size_t& tmp_bytes, const int64_t* in, int64_t* out, int64_t n, hipStream_t s);
hipError_t scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s);
hipError_t sort_pairs_i32(void* tmp, size_t& tmp_bytes, const int32_t* keys_in, int32_t* keys_out,
                          const int32_t* vals_in, int32_t* vals_out, int64_t n, int end_bit, hipStream_t s);

hipError_t sort_pairs_u64_i32(void* tmp, size_t& tmp_bytes, const unsigned long long* keys_in,
                              unsigned long long* keys_out, const int32_t* vals_in, int32_t* vals_out, int64_t n,
                              int end_bit, hipStream_t s);

}  // namespace lmmdev
