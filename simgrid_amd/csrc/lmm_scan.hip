// lmm_scan.hip — device-wide primitives for the resident flatten (lmm_resident_kernels.hpp): exclusive
// prefix sums and a stable key/value radix sort, from hipCUB (rocPRIM underneath, tuned for gfx9).
// Kept in their own translation unit so the hipCUB templates do not slow down lmm_hip.hip's build.
// Every call takes caller-owned scratch: `tmp`/`tmp_bytes` from a previous size query
// (tmp == nullptr), as hipCUB does.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "lmm_scan.hpp"

namespace lmmdev {

hipError_t scan_i64(void* tmp, size_t& tmp_bytes, const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, s);
}

hipError_t scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, s);
}

// Stable: equal keys keep their input order (the CSC of a constraint lists its elements in CSR order,
// i.e. by ascending variable, as the host counting sort of lmmhip_upload does).
hipError_t sort_pairs_i32(void* tmp, size_t& tmp_bytes, const int32_t* keys_in, int32_t* keys_out,
                          const int32_t* vals_in, int32_t* vals_out, int64_t n, int end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit, s);
}

hipError_t sort_pairs_u64_i32(void* tmp, size_t& tmp_bytes, const unsigned long long* keys_in,
                              unsigned long long* keys_out, const int32_t* vals_in, int32_t* vals_out, int64_t n,
                              int end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit, s);
}

}  // namespace lmmdev
