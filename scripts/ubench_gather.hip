// Calibration micro-benchmark for the LMM kernels' access patterns on MI355X:
//   random gathers of 1/2/4/8 B from tables of 1-80 MB (the per-constraint state the round kernels
//   read per element), group-per-row shapes, and random fp64 / int32 atomics (the decrement pushes).
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_gather.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <class T>
__global__ void gather(const int* __restrict__ idx, const T* __restrict__ tab, long n, double* out) {
  double acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += (double)tab[idx[i]];
  if (acc == 12345.678)
    out[0] = acc;
}

__global__ void stream_idx(const int4* __restrict__ idx, long n4, double* out) {
  long acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    int4 v = idx[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234567)
    out[0] = (double)acc;
}

__global__ void atomics_f64(const int* __restrict__ idx, double* tab, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    unsafeAtomicAdd(&tab[idx[i]], 1.0);
}
__global__ void atomics_i32(const int* __restrict__ idx, int* tab, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    atomicAdd(&tab[idx[i]], 1);
}
__global__ void scatter_u8(const int* __restrict__ idx, unsigned char* tab, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    tab[idx[i]] = 1;
}

int main() {
  const long n = 80'000'000;
  std::vector<int> h(n);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  int* d_idx;
  double* out;
  CHK(hipMalloc(&d_idx, n * 4));
  CHK(hipMalloc(&out, 8));
  void* tab;
  CHK(hipMalloc(&tab, 80'000'000L * 8));
  CHK(hipMemset(tab, 0, 80'000'000L * 8));
  auto time = [&](auto launch) {
    launch();
    CHK(hipEventRecord(a));
    for (int r = 0; r < 3; r++)
      launch();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
  };
  const int grid = 2048 * 4, block = 256;
  {
    float ms = time([&] { stream_idx<<<grid, block>>>((const int4*)d_idx, n / 4, out); });
    printf("stream int32 idx: %.3f ms  %.1f GB/s\n", ms, n * 4 / ms / 1e6);
  }
  for (long tabn : {1'000'000L, 4'000'000L, 10'000'000L}) {
    srand(1);
    for (long i = 0; i < n; i++)
      h[i] = (int)(((unsigned long)rand() * 2654435761UL) % tabn);
    CHK(hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice));
    float m8 = time([&] { gather<double><<<grid, block>>>(d_idx, (double*)tab, n, out); });
    float m4 = time([&] { gather<float><<<grid, block>>>(d_idx, (float*)tab, n, out); });
    float m2 = time([&] { gather<unsigned short><<<grid, block>>>(d_idx, (unsigned short*)tab, n, out); });
    float m1 = time([&] { gather<unsigned char><<<grid, block>>>(d_idx, (unsigned char*)tab, n, out); });
    printf("table %8ld entries: gather8 %.3f ms (%.2e/s, tab %.0f MB) gather4 %.3f gather2 %.3f gather1 %.3f ms\n",
           tabn, m8, n / m8 * 1e3, tabn * 8 / 1e6, m4, m2, m1);
    float mf = time([&] { atomics_f64<<<grid, block>>>(d_idx, (double*)tab, n); });
    float mi = time([&] { atomics_i32<<<grid, block>>>(d_idx, (int*)tab, n); });
    float ms = time([&] { scatter_u8<<<grid, block>>>(d_idx, (unsigned char*)tab, n); });
    printf("                         atomic f64 %.3f ms (%.2e/s)  atomic i32 %.3f ms  scatter u8 %.3f ms\n", mf,
           n / mf * 1e3, mi, ms);
  }
  return 0;
}
