// TEST SUPPORT ONLY (tests/test_gpu_engines.py::test_persistent_rendezvous_deadline_falls_back_fast): a kernel
// that holds part of the chip for a given wall-clock time, launched by another process (tests/c/occupy_run.py:
// its hardware queue is its own, so the hold overlaps the test's persistent solve), so that the solve's grid
// cannot become co-resident.  Built into tests/c/libocc.so by __graft_entry__.build().
#include <hip/hip_runtime.h>

// 1024 threads (16 waves, four per SIMD) and 64 KB of LDS per workgroup: a CU running one has no room left for
// a persistent workgroup (1024 threads at 128 VGPRs, ~130 KB of LDS).  Each workgroup marks its slot of the
// mapped array `started` when it runs, then sleeps until `ticks` (100 MHz wall clock) have passed.
__global__ void __launch_bounds__(1024) occ_spin(long long ticks, int* started) {
  __shared__ int pad[16384];
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0)
    __hip_atomic_store(&started[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  pad[threadIdx.x] = int(t0);
  while (wall_clock64() - t0 < ticks)
    __builtin_amdgcn_s_sleep(16);
  __syncthreads();
  if (pad[(threadIdx.x + 1) & 1023] == 0x7fffffff && started)  // (keeps the LDS allocation)
    __hip_atomic_store(&started[blockIdx.x], 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" {
// Queue `blocks` spinning workgroups of `seconds` on `stream`; `started` is a mapped host array of `blocks` ints
// (hipHostMalloc'd by occ_alloc), zeroed here.  Returns 0 or the HIP error.
int occ_alloc(int n, int** host, int** dev) {
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(host), sizeof(int) * size_t(n), hipHostMallocMapped);
  if (e == hipSuccess)
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0);
  return int(e);
}
int occ_free(int* host) { return int(hipHostFree(host)); }
int occ_launch(void* stream, int blocks, double seconds, int* host, int* dev) {
  for (int i = 0; i < blocks; i++)
    host[i] = 0;
  const long long ticks = static_cast<long long>(seconds * 1e8);
  hipLaunchKernelGGL(occ_spin, dim3(blocks), dim3(1024), 0, static_cast<hipStream_t>(stream), ticks, dev);
  return int(hipGetLastError());
}
int occ_sync(void) { return int(hipDeviceSynchronize()); }
int occ_cus(void) {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev))
    return -1;
  return n;
}
}
