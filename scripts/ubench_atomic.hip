// Micro-benchmark for the decrement push of mm_saturate: how should three per-element
// accumulations (remaining, usage, fixed-element count) into random constraints be issued?
//   A  three arrays, one lane per element issues 3 atomics (f64, f64, i32)     — the v3 layout
//   B  one 32-B record per constraint, 4 lanes per element, 3 of them issue one f64 atomic each in
//      the SAME wave instruction (same 64-B line -> one memory-side request?)
//   C  one 32-B record per constraint, one lane per element issues 3 f64 atomics
//   D  plain scattered 8-B stores (no atomics), for scale
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_atomic.hip -o scripts/ubench_atomic
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

__global__ void push_a(const int* __restrict__ idx, const double* __restrict__ w, long n, double* drem,
                       double* duse, int* dcnt) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = idx[i];
    const double x = w[i];
    atomicAdd(&dcnt[c], 1);
    unsafeAtomicAdd(&drem[c], x * 0.5);
    unsafeAtomicAdd(&duse[c], x);
  }
}

// 4 lanes per element; lane q in {0,1,2} adds to field q of the 32-B record
__global__ void push_b(const int* __restrict__ idx, const double* __restrict__ w, long n, double* rec) {
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int q = threadIdx.x & 3;
  for (long t = tid; t < 4 * n; t += (long)gridDim.x * blockDim.x) {
    const long i = t >> 2;
    const int c = idx[i];
    const double x = w[i];
    const double v = q == 0 ? x * 0.5 : q == 1 ? x : 1.0;
    if (q < 3)
      unsafeAtomicAdd(&rec[4 * long(c) + q], v);
  }
}

__global__ void push_c(const int* __restrict__ idx, const double* __restrict__ w, long n, double* rec) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = idx[i];
    const double x = w[i];
    unsafeAtomicAdd(&rec[4 * long(c)], x * 0.5);
    unsafeAtomicAdd(&rec[4 * long(c) + 1], x);
    unsafeAtomicAdd(&rec[4 * long(c) + 2], 1.0);
  }
}

// 2 lanes per element, each adds a 16-B pair? (f64 only has 8-B atomics): lanes 0/1 -> fields 0/1
__global__ void push_b2(const int* __restrict__ idx, const double* __restrict__ w, long n, double* rec) {
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int q = threadIdx.x & 1;
  for (long t = tid; t < 2 * n; t += (long)gridDim.x * blockDim.x) {
    const long i = t >> 1;
    const int c = idx[i];
    const double x = w[i];
    unsafeAtomicAdd(&rec[2 * long(c) + q], q ? x : x * 0.5);
  }
}

// B as the product issues it (u64 fixed-point adds, agent scope), and E: the same into a per-XCD replica of the
// records with WORKGROUP-scope atomics (performed in the XCD's own L2?), replicas summed afterwards.
__device__ __forceinline__ unsigned xcc_id_() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v & 7u;
}
template <int kScope>
__global__ void push_u64(const int* __restrict__ idx, const double* __restrict__ w, long n, unsigned long long* rec,
                         long nc) {
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int q = threadIdx.x & 3;
  unsigned long long* base = kScope == __HIP_MEMORY_SCOPE_WORKGROUP ? rec + 4 * nc * long(xcc_id_()) : rec;
  for (long t = tid; t < 4 * n; t += (long)gridDim.x * blockDim.x) {
    const long i = t >> 2;
    const int c = idx[i];
    const double x = w[i];
    const unsigned long long v = q == 0 ? (unsigned long long)(x * 1024) : q == 1 ? (unsigned long long)(x * 4096) : 1ull;
    if (q < 3)
      __hip_atomic_fetch_add(&base[4 * long(c) + q], v, __ATOMIC_RELAXED, kScope);
  }
}
__global__ void sum_cnt(const unsigned long long* rec, long nc, int nrep, unsigned long long* out) {
  unsigned long long s = 0;
  for (long c = blockIdx.x * (long)blockDim.x + threadIdx.x; c < nc; c += (long)gridDim.x * blockDim.x)
    for (int r = 0; r < nrep; r++)
      s += rec[4 * nc * r + 4 * c + 2];
  atomicAdd(out, s);
}

__global__ void store_d(const int* __restrict__ idx, const double* __restrict__ w, long n, double* tab) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    tab[idx[i]] = w[i];
}

// the claim pattern of saturate_one: returning CAS on a random int
__global__ void claim(const int* __restrict__ idx, long n, int* st, int* out) {
  int got = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int v = idx[i];
    if (st[v] == 0 && atomicCAS(&st[v], 0, 1) == 0)
      got++;
  }
  if (got == -1)
    out[0] = got;
}

int main() {
  const long n = 30'000'000;
  const long nc = 1'000'000;
  std::vector<int> h(n);
  std::vector<double> hw(n);
  srand(7);
  for (long i = 0; i < n; i++) {
    h[i] = (int)(((unsigned long)rand() * 2654435761UL) % nc);
    hw[i] = 1.0 + (rand() % 1000) * 1e-3;
  }
  int* d_idx;
  double* d_w;
  CHK(hipMalloc(&d_idx, n * 4));
  CHK(hipMalloc(&d_w, n * 8));
  CHK(hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_w, hw.data(), n * 8, hipMemcpyHostToDevice));
  double *drem, *duse, *rec;
  int *dcnt, *st, *out;
  CHK(hipMalloc(&drem, nc * 8));
  CHK(hipMalloc(&duse, nc * 8));
  CHK(hipMalloc(&dcnt, nc * 4));
  CHK(hipMalloc(&rec, nc * 32));
  CHK(hipMalloc(&st, 10'000'000 * 4));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(drem, 0, nc * 8));
  CHK(hipMemset(duse, 0, nc * 8));
  CHK(hipMemset(dcnt, 0, nc * 4));
  CHK(hipMemset(rec, 0, nc * 32));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
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
  const int block = 256;
  for (int grid : {1024, 2048, 8192}) {
    float ta = time([&] { push_a<<<grid, block>>>(d_idx, d_w, n, drem, duse, dcnt); });
    float tb = time([&] { push_b<<<grid, block>>>(d_idx, d_w, n, rec); });
    float tc = time([&] { push_c<<<grid, block>>>(d_idx, d_w, n, rec); });
    float tb2 = time([&] { push_b2<<<grid, block>>>(d_idx, d_w, n, rec); });
    float td = time([&] { store_d<<<grid, block>>>(d_idx, d_w, n, drem); });
    printf("grid %5d  %ld elems -> %ld cnsts: A 3 arrays %.3f ms (%.2e el/s)  B 4-lane record %.3f ms (%.2e el/s)"
           "  C 1-lane record %.3f ms  B2 2-lane pair %.3f ms  D plain store %.3f ms\n",
           grid, n, nc, ta, n / ta * 1e3, tb, n / tb * 1e3, tc, tb2, td);
  }
  {
    unsigned long long *rep, *cnt;
    CHK(hipMalloc(&rep, 8 * nc * 32));
    CHK(hipMalloc(&cnt, 8));
    for (int grid : {2048, 8192}) {
      CHK(hipMemset(rep, 0, 8 * nc * 32));
      float tf = time([&] { push_u64<__HIP_MEMORY_SCOPE_AGENT><<<grid, block>>>(d_idx, d_w, n, rep, nc); });
      CHK(hipMemset(cnt, 0, 8));
      sum_cnt<<<1024, 256>>>(rep, nc, 1, cnt);
      unsigned long long hf = 0;
      CHK(hipMemcpy(&hf, cnt, 8, hipMemcpyDeviceToHost));
      CHK(hipMemset(rep, 0, 8 * nc * 32));
      float te = time([&] { push_u64<__HIP_MEMORY_SCOPE_WORKGROUP><<<grid, block>>>(d_idx, d_w, n, rep, nc); });
      CHK(hipMemset(cnt, 0, 8));
      sum_cnt<<<1024, 256>>>(rep, nc, 8, cnt);
      unsigned long long he = 0;
      CHK(hipMemcpy(&he, cnt, 8, hipMemcpyDeviceToHost));
      printf("grid %5d u64 quad pushes: agent scope %.3f ms (%.2e el/s, count %llu / %ld)  workgroup scope into"
             " per-XCD replicas %.3f ms (%.2e el/s, count %llu / %ld)\n",
             grid, tf, n / tf * 1e3, hf, 4 * n, te, n / te * 1e3, he, 4 * n);
    }
  }
  {
    std::vector<int> hv(n);
    for (long i = 0; i < n; i++)
      hv[i] = (int)(((unsigned long)rand() * 2654435761UL) % 10'000'000L);
    CHK(hipMemcpy(d_idx, hv.data(), n * 4, hipMemcpyHostToDevice));
    float tcl = time([&] {
      (void)hipMemsetAsync(st, 0, 10'000'000 * 4);
      claim<<<2048, block>>>(d_idx, n, st, out);
    });
    printf("claim (load + CAS on 1e7 ints, incl. memset): %.3f ms (%.2e/s)\n", tcl, n / tcl * 1e3);
  }
  return 0;
}
