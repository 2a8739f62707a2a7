// lmm_hip.hip — MI355X (gfx950, CDNA4) kernels of the LMM solver + the C ABI of include/lmm/lmm_hip.h.
//
// The reference solves with two sequential CPU algorithms over boost::intrusive lists:
//   * System::lmm_solve (src/kernel/lmm/maxmin.cpp:502-693): progressive filling — repeatedly find
//     the constraint(s) with the globally smallest remaining/usage ratio (exact == ties,
//     maxmin.cpp:397-409), fix their active variables at that level (or at their bound,
//     maxmin.cpp:563-595), and update every constraint those variables touch (maxmin.cpp:601-659).
//   * FairBottleneck::bottleneck_solve (fair_bottleneck.cpp:23-153): Jacobi rounds of three sweeps.
//
// maxmin on the device — "local-minimum parallel progressive filling" (DESIGN.md §3).  Ratios never
// decrease, so a constraint whose ratio is <= the ratio of every constraint sharing an unfixed
// variable with it saturates at exactly its current ratio in the sequential order too.  One round:
//   mm_vote<G>   G lanes per alive variable (compacted rows): find the constraint(s) of minimal
//                ratio through 16-bit monotone keys (round-down of the ratio: a 2 MB table per 10^6
//                constraints that stays in L2), resolve key ties exactly in fp64, and cast one
//                atomic "vote" for the minimal constraint(s).  A bounded variable whose level
//                bound*penalty is below that minimum votes for nothing (maxmin.cpp:563-595).
//   mm_fix       one thread per alive variable: its constraint is a local minimum iff every alive
//                element voted for it (votes == alive element count); fix the variable at
//                ratio/penalty (or at its bound) and push w*x, w/p and count decrements with atomics.
//   mm_update    one thread per constraint: apply the decrements, clamp (surf_interface.hpp:34-44;
//                clamping a sum of non-negative decrements == clamping after each one), drop
//                saturated constraints (maxmin.cpp:608-623), refresh ratio and key; FATPIPE usage is
//                recomputed as the max over still-unfixed elements (maxmin.cpp:625-658).
// Every 16 rounds the alive rows are compacted (order preserving) so later rounds stream only live data.
//
// fair bottleneck — the reference's rounds are already bulk-synchronous; one round = three launches
// mirroring fair_bottleneck.cpp:65-87, :89-105 and :107-144.
//
// All arithmetic is fp64; device code is compiled with -ffp-contract=off so every a*b+c rounds like the
// reference (the FairBottleneck `value == bound` test is exact).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lmm/lmm_hip.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess)                                                                               \
      return fail(LMMHIP_E_HIP, std::string(#expr " -> ") + hipGetErrorString(e_) + " @" + __FILE__ + \
                                    ":" + std::to_string(__LINE__));                                    \
  } while (0)

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxBlocks = 2048;       // 256 CUs x 8 resident 256-thread blocks; grid-stride beyond
constexpr int kRowsPerThread = 8;      // compaction chunking
constexpr int kCompactRows = kBlock * kRowsPerThread;
constexpr unsigned kDeadKey = 0xFFFFu;  // > every key of a finite positive ratio (<= 0x7F80)
constexpr int kDrop = -1, kBound = -2;
constexpr int kTieBit = 1 << 30;

// control block words
enum : int {
  CTL_DONE = 0,
  CTL_ROUNDS = 1,
  CTL_ANY0 = 2,  // + parity
  CTL_NROWS = 4, // + buffer (3 buffers)
  CTL_NELEM = 8, // + buffer
  CTL_WORDS = 16
};

struct Dev {
  int32_t nV, nC;
  int64_t nnz;
  // structure (uploaded once)
  const uint32_t* var_ptr;   // [nV+1] CSR row offsets (variable-major)
  const int32_t* csr_c;      // [nnz]
  const double* csr_w;       // [nnz]
  const uint32_t* cnst_ptr;  // [nC+1] CSC offsets (constraint-major)
  const int32_t* csc_v;      // [nnz]
  const double* csc_w;       // [nnz]
  const double* pen;         // [nV]
  const double* vbound;      // [nV]
  const double* cbound;      // [nC]
  const uint8_t* cflags;     // [nC] bit0 FATPIPE, bit1 zero-weight enabled element
  // per-variable state
  double* x;       // [nV] values (output)
  int32_t* fixr;   // [nV] round in which the variable left the alive set (measurement only)
  double* vtmp;    // [nV] fair bottleneck: mu
  uint8_t* vst;    // [nV] fair bottleneck: 1 listed / 0 not
  // per-constraint state
  double* ratio;   // [nC] remaining/usage, +inf when out of the light table
  uint16_t* key;   // [nC] round-down 16-bit key of ratio, kDeadKey when out
  double* rem;     // [nC]
  double* use;     // [nC]
  double* drem;    // [nC] atomic accumulators (SHARED constraints)
  double* duse;    // [nC]
  int32_t* acnt;   // [nC] alive (unfixed) elements
  int32_t* dcnt;   // [nC] atomic accumulator of fixed elements
  int32_t* votes;  // [nC]
  // alive-row buffers: 0 = the original CSR (identity ids), 1/2 = compaction targets
  const int32_t* cvar[3];
  const uint32_t* crow[3];
  const int32_t* ccol[3];
  uint8_t* valive[3];
  int32_t* vinfo;  // [nV] per-row result of mm_vote
  int32_t* bsum;   // compaction scratch: per-block rows / elems (2 x blocks)
  int32_t* ctl;    // control words
};

__device__ __forceinline__ double dinf() { return __builtin_huge_val(); }

// 16-bit monotone key: round the ratio down to f32, keep the upper 16 bits (sign, exponent, 7 bits
// of mantissa).  Monotone non-decreasing, so key(a) < key(b) => a < b; equal keys need the exact
// fp64 comparison.
__device__ __forceinline__ uint16_t ratio_key(double r) {
  float f = __double2float_rd(r);
  return uint16_t(__float_as_uint(f) >> 16);
}

template <int W> __device__ __forceinline__ double grp_min(double v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1)
    v = fmin(v, __shfl_xor(v, o, W));
  return v;
}
template <int W> __device__ __forceinline__ unsigned grp_umin(unsigned v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1)
    v = min(v, (unsigned)__shfl_xor((int)v, o, W));
  return v;
}
template <int W> __device__ __forceinline__ int grp_imax(int v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1)
    v = max(v, __shfl_xor(v, o, W));
  return v;
}
template <int W> __device__ __forceinline__ int grp_isum(int v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1)
    v += __shfl_xor(v, o, W);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v = fmin(v, __shfl_xor(v, o, kWave));
  return v;
}

// =============================================================================================
// maxmin (System::lmm_solve)
// =============================================================================================

// Init, one wave per constraint: maxmin.cpp:520-555.  remaining = bound; skipped when
// bound <= bound*prec; usage = sum (SHARED) or max (FATPIPE) of w/p over the active elements.
__global__ void __launch_bounds__(kBlock) mm_init_cnsts(Dev s, double prec) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  int any = 0;
  for (int64_t c = int64_t(blockIdx.x) * wpb + threadIdx.x / kWave; c < s.nC; c += int64_t(gridDim.x) * wpb) {
    const uint32_t b = s.cnst_ptr[c], e = s.cnst_ptr[c + 1];
    const bool fat = s.cflags[c] & 1;
    double acc = 0.0;
    for (uint32_t j = b + lane; j < e; j += kWave) {
      double u = s.csc_w[j] / s.pen[s.csc_v[j]];
      acc = fat ? fmax(acc, u) : acc + u;
    }
    acc = fat ? wave_max(acc) : wave_sum(acc);
    if (lane == 0) {
      const double bound = s.cbound[c];
      const bool part = bound > bound * prec;
      const double usage = part ? acc : 0.0;
      s.rem[c] = bound;
      s.use[c] = usage;
      s.drem[c] = 0.0;
      s.duse[c] = 0.0;
      s.acnt[c] = int32_t(e - b);
      s.dcnt[c] = 0;
      s.votes[c] = 0;
      const bool alive = part && usage > 0;
      const double r = bound / usage;
      s.ratio[c] = alive ? r : dinf();
      s.key[c] = alive ? ratio_key(r) : uint16_t(kDeadKey);
      any |= alive;
    }
  }
  if (any)
    s.ctl[CTL_ANY0] = 1;
}

__global__ void __launch_bounds__(kBlock) mm_init_vars(Dev s) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock) {
    s.x[v] = 0.0;
    s.fixr[v] = -1;
    s.valive[0][v] = 1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.ctl[CTL_NROWS + 0] = s.nV;
    s.ctl[CTL_NELEM + 0] = int32_t(s.nnz);
  }
}

// Round phase 1 — vote.  G lanes per alive row; all loops are wave-uniform so the group shuffles
// always see their whole group.
template <int G> __global__ void __launch_bounds__(kBlock) mm_vote(Dev s, int buf, int par) {
  if (s.ctl[CTL_DONE])
    return;
  if (!s.ctl[CTL_ANY0 + par]) {  // no constraint left in the light table: maxmin.cpp:680
    s.ctl[CTL_DONE] = 1;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_ANY0 + (par ^ 1)] = 0;
  const int64_t nrows = s.ctl[CTL_NROWS + buf];
  const int32_t* __restrict__ cvar = s.cvar[buf];
  const uint32_t* __restrict__ crow = s.crow[buf];
  const int32_t* __restrict__ ccol = s.ccol[buf];
  const uint8_t* __restrict__ valive = s.valive[buf];
  const uint16_t* __restrict__ key = s.key;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane & (G - 1);
  constexpr int kGpw = kWave / G;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  for (int64_t base = wave * kGpw; base < nrows; base += nwaves * kGpw) {
    const int64_t row = base + lane / G;
    const bool valid = row < nrows && valive[row];
    uint32_t b = 0, e = 0;
    if (valid) {
      b = crow[row];
      e = crow[row + 1];
    }
    // pass 1: minimal key over the row
    unsigned mk = kDeadKey;
    for (uint32_t j = b + g; j < e; j += G)
      mk = min(mk, (unsigned)key[ccol[j]]);
    mk = grp_umin<G>(mk);
    // pass 2: how many elements share it
    int nmin = 0;
    for (uint32_t j = b + g; j < e; j += G)
      nmin += key[ccol[j]] == mk;
    nmin = grp_isum<G>(nmin);
    int v = valid ? cvar[row] : 0;
    const double vb = valid ? s.vbound[v] : -1.0;
    const bool live = valid && mk != kDeadKey;
    // exact minimum only when the key is ambiguous or a bound has to be compared
    double minr = dinf();
    if (live && (nmin > 1 || vb > 0))
      for (uint32_t j = b + g; j < e; j += G) {
        const int32_t c = ccol[j];
        if (key[c] == mk)
          minr = fmin(minr, s.ratio[c]);
      }
    minr = grp_min<G>(minr);
    const double lb = vb > 0 ? vb * s.pen[v] : dinf();
    const bool bounded = live && vb > 0 && lb < minr;
    int first = INT_MAX, last = -1;
    if (live && !bounded)
      for (uint32_t j = b + g; j < e; j += G) {
        const int32_t c = ccol[j];
        if (key[c] == mk && (nmin == 1 || s.ratio[c] == minr)) {
          atomicAdd(&s.votes[c], 1);
          first = min(first, c);
          last = max(last, c);
        }
      }
    first = -grp_imax<G>(-first);
    last = grp_imax<G>(last);
    if (valid && g == 0) {
      int code;
      if (!live)
        code = kDrop;
      else if (bounded)
        code = kBound;
      else
        code = first | (last != first ? kTieBit : 0);
      s.vinfo[row] = code;
    }
  }
}

// Round phase 2 — fix.  maxmin.cpp:580-595 (value) and :601-606 (decrements).
__global__ void __launch_bounds__(kBlock) mm_fix(Dev s, int buf, int round) {
  if (s.ctl[CTL_DONE])
    return;
  const int64_t nrows = s.ctl[CTL_NROWS + buf];
  const int32_t* __restrict__ cvar = s.cvar[buf];
  uint8_t* valive = s.valive[buf];
  for (int64_t row = int64_t(blockIdx.x) * kBlock + threadIdx.x; row < nrows; row += int64_t(gridDim.x) * kBlock) {
    if (!valive[row])
      continue;
    const int code = s.vinfo[row];
    const int v = cvar[row];
    if (code == kDrop) {  // every constraint of v left the light table: v stays at 0
      valive[row] = 0;
      s.fixr[v] = round;
      continue;
    }
    const double p = s.pen[v];
    double xv = 0.0;
    bool fix = false;
    if (code == kBound) {
      xv = s.vbound[v];
      fix = true;
    } else {
      const int c = code & (kTieBit - 1);
      if (s.votes[c] == s.acnt[c]) {
        fix = true;
        xv = s.ratio[c] / p;
      } else if (code & kTieBit) {  // several minimal constraints: any of them saturating fixes v
        const double r = s.ratio[c];
        for (uint32_t j = s.var_ptr[v]; j < s.var_ptr[v + 1] && !fix; j++) {
          const int32_t c2 = s.csr_c[j];
          if (c2 != c && s.ratio[c2] == r && s.votes[c2] == s.acnt[c2]) {
            fix = true;
            xv = r / p;
          }
        }
      }
    }
    if (!fix)
      continue;
    s.x[v] = xv;
    valive[row] = 0;
    s.fixr[v] = round;
    for (uint32_t j = s.var_ptr[v]; j < s.var_ptr[v + 1]; j++) {
      const int32_t c = s.csr_c[j];
      if (s.key[c] == kDeadKey)
        continue;
      atomicAdd(&s.dcnt[c], 1);
      if (!(s.cflags[c] & 1)) {
        const double w = s.csr_w[j];
        unsafeAtomicAdd(&s.drem[c], w * xv);
        unsafeAtomicAdd(&s.duse[c], w / p);
      }
    }
  }
}

// Round phase 3 — constraint update.  maxmin.cpp:603-658.
__global__ void __launch_bounds__(kBlock) mm_update(Dev s, int par, double prec) {
  if (s.ctl[CTL_DONE])
    return;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_ROUNDS] += 1;
  int any = 0;
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < s.nC; c += int64_t(gridDim.x) * kBlock) {
    if (s.key[c] == kDeadKey)
      continue;
    s.votes[c] = 0;
    const int dc = s.dcnt[c];
    if (!dc) {  // untouched: ratio unchanged
      any = 1;
      continue;
    }
    s.dcnt[c] = 0;
    s.acnt[c] -= dc;
    const double bound = s.cbound[c];
    double rem = s.rem[c], use;
    if (!(s.cflags[c] & 1)) {
      use = s.use[c] - s.duse[c];
      rem -= s.drem[c];
      s.drem[c] = 0.0;
      s.duse[c] = 0.0;
      if (rem < bound * prec)
        rem = 0.0;
      if (use < prec)
        use = 0.0;
    } else {  // FATPIPE: usage = max w/p over enabled elements whose variable is still at 0
      use = 0.0;
      for (uint32_t j = s.cnst_ptr[c]; j < s.cnst_ptr[c + 1]; j++) {
        const int32_t v = s.csc_v[j];
        if (s.x[v] > 0)
          continue;
        use = fmax(use, s.csc_w[j] / s.pen[v]);
      }
    }
    s.rem[c] = rem;
    s.use[c] = use;
    if (!(use > prec) || !(rem > bound * prec)) {
      s.ratio[c] = dinf();
      s.key[c] = kDeadKey;
    } else {
      const double r = rem / use;
      s.ratio[c] = r;
      s.key[c] = ratio_key(r);
      any = 1;
    }
  }
  if (any)
    s.ctl[CTL_ANY0 + (par ^ 1)] = 1;
}

// ---- order-preserving compaction of the alive rows: count / scan / write ----
__device__ __forceinline__ void block_scan2(int& a, int& b, int* sh) {  // exclusive, kBlock threads
  const int t = threadIdx.x;
  sh[t] = a;
  sh[kBlock + t] = b;
  __syncthreads();
  for (int o = 1; o < kBlock; o <<= 1) {
    int xa = t >= o ? sh[t - o] : 0, xb = t >= o ? sh[kBlock + t - o] : 0;
    __syncthreads();
    sh[t] += xa;
    sh[kBlock + t] += xb;
    __syncthreads();
  }
  a = sh[t] - a;  // exclusive
  b = sh[kBlock + t] - b;
  __syncthreads();
}

__global__ void __launch_bounds__(kBlock) cmp_count(Dev s, int in) {
  __shared__ int sh[2 * kBlock];
  const int64_t nrows = s.ctl[CTL_NROWS + in];
  const int64_t r0 = int64_t(blockIdx.x) * kCompactRows + int64_t(threadIdx.x) * kRowsPerThread;
  int nr = 0, ne = 0;
  for (int k = 0; k < kRowsPerThread; k++) {
    const int64_t row = r0 + k;
    if (row < nrows && s.valive[in][row]) {
      nr++;
      ne += int(s.crow[in][row + 1] - s.crow[in][row]);
    }
  }
  int a = nr, b = ne;
  block_scan2(a, b, sh);
  if (threadIdx.x == kBlock - 1) {
    s.bsum[2 * blockIdx.x] = a + nr;
    s.bsum[2 * blockIdx.x + 1] = b + ne;
  }
}

__global__ void __launch_bounds__(1024) cmp_scan(Dev s, int nblk, int out) {
  __shared__ int sa[1024], sb[1024];
  const int t = threadIdx.x;
  const int per = (nblk + 1023) / 1024;
  int a = 0, b = 0;
  for (int i = t * per; i < (t + 1) * per && i < nblk; i++) {
    a += s.bsum[2 * i];
    b += s.bsum[2 * i + 1];
  }
  sa[t] = a;
  sb[t] = b;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int xa = t >= o ? sa[t - o] : 0, xb = t >= o ? sb[t - o] : 0;
    __syncthreads();
    sa[t] += xa;
    sb[t] += xb;
    __syncthreads();
  }
  int ra = sa[t] - a, rb = sb[t] - b;  // exclusive base of this thread's segment
  for (int i = t * per; i < (t + 1) * per && i < nblk; i++) {
    const int ca = s.bsum[2 * i], cb = s.bsum[2 * i + 1];
    s.bsum[2 * i] = ra;
    s.bsum[2 * i + 1] = rb;
    ra += ca;
    rb += cb;
  }
  if (t == 1023) {
    s.ctl[CTL_NROWS + out] = sa[t];
    s.ctl[CTL_NELEM + out] = sb[t];
    const_cast<uint32_t*>(s.crow[out])[sa[t]] = uint32_t(sb[t]);
  }
}

__global__ void __launch_bounds__(kBlock) cmp_write(Dev s, int in, int out) {
  __shared__ int sh[2 * kBlock];
  const int64_t nrows = s.ctl[CTL_NROWS + in];
  const int64_t r0 = int64_t(blockIdx.x) * kCompactRows + int64_t(threadIdx.x) * kRowsPerThread;
  int nr = 0, ne = 0;
  for (int k = 0; k < kRowsPerThread; k++) {
    const int64_t row = r0 + k;
    if (row < nrows && s.valive[in][row]) {
      nr++;
      ne += int(s.crow[in][row + 1] - s.crow[in][row]);
    }
  }
  int pr = nr, pe = ne;
  block_scan2(pr, pe, sh);
  pr += s.bsum[2 * blockIdx.x];
  pe += s.bsum[2 * blockIdx.x + 1];
  int32_t* ovar = const_cast<int32_t*>(s.cvar[out]);
  uint32_t* orow = const_cast<uint32_t*>(s.crow[out]);
  int32_t* ocol = const_cast<int32_t*>(s.ccol[out]);
  for (int k = 0; k < kRowsPerThread; k++) {
    const int64_t row = r0 + k;
    if (row < nrows && s.valive[in][row]) {
      const uint32_t b = s.crow[in][row], e = s.crow[in][row + 1];
      ovar[pr] = s.cvar[in][row];
      orow[pr] = uint32_t(pe);
      s.valive[out][pr] = 1;
      for (uint32_t j = b; j < e; j++)
        ocol[pe++] = s.ccol[in][j];
      pr++;
    }
  }
}

// =============================================================================================
// FairBottleneck::bottleneck_solve
// =============================================================================================

__global__ void __launch_bounds__(kBlock) fb_init(Dev s) {
  const int64_t n = s.nV > s.nC ? s.nV : s.nC;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    if (i < s.nV) {  // fair_bottleneck.cpp:29-41 (only listed variables are flattened)
      s.x[i] = 0.0;
      s.vtmp[i] = 0.0;
      s.vst[i] = 1;
      s.fixr[i] = -1;
    }
    if (i < s.nC) {  // :44-50
      s.rem[i] = s.cbound[i];
      s.use[i] = 0.0;
      s.ratio[i] = 0.0;  // 0 = in the constraint list, +inf = erased
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_ANY0] = s.nV > 0;
}

// :65-87 — usage = remaining / (number of listed variables with w > 0), FATPIPE -> 1.
__global__ void __launch_bounds__(kBlock) fb_cnst_share(Dev s, int par) {
  if (s.ctl[CTL_DONE])
    return;
  if (!s.ctl[CTL_ANY0 + par]) {
    s.ctl[CTL_DONE] = 1;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.ctl[CTL_ANY0 + (par ^ 1)] = 0;
    s.ctl[CTL_ROUNDS] += 1;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int64_t c = int64_t(blockIdx.x) * wpb + threadIdx.x / kWave; c < s.nC; c += int64_t(gridDim.x) * wpb) {
    if (s.ratio[c] != 0.0)
      continue;
    int nb = 0;
    for (uint32_t j = s.cnst_ptr[c] + lane; j < s.cnst_ptr[c + 1]; j += kWave)
      nb += s.vst[s.csc_v[j]];
    nb = grp_isum<kWave>(nb);
    if (lane == 0) {
      if (nb > 0 && (s.cflags[c] & 1))
        nb = 1;
      if (nb == 0) {
        s.rem[c] = 0.0;
        s.use[c] = 0.0;
        s.ratio[c] = dinf();
      } else {
        s.use[c] = s.rem[c] / nb;
      }
    }
  }
}

// :89-105 — per listed variable: mu = min(usage/w, bound - value); value += mu; exact
// `value == bound` drops it from the list.
__global__ void __launch_bounds__(kBlock) fb_var_inc(Dev s, int par, int round) {
  if (s.ctl[CTL_DONE])
    return;
  int any = 0;
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock) {
    if (!s.vst[v])
      continue;
    double inc = DBL_MAX;
    for (uint32_t j = s.var_ptr[v]; j < s.var_ptr[v + 1]; j++)
      inc = fmin(inc, s.use[s.csr_c[j]] / s.csr_w[j]);
    const double vb = s.vbound[v];
    double x = s.x[v];
    if (vb > 0)
      inc = fmin(inc, vb - x);
    s.vtmp[v] = inc;
    x += inc;
    s.x[v] = x;
    if (x == vb)
      s.vst[v] = 0;
    else
      any = 1;
    s.fixr[v] = round;  // last round in which v was listed
  }
  if (any)
    s.ctl[CTL_ANY0 + (par ^ 1)] = 1;
}

// :107-144 — remaining -= sum w*mu over ALL enabled elements (stale mu of variables that already
// left the list included), FATPIPE: remaining -= min(usage, min w*mu); remaining <= 0 erases the
// constraint and every listed variable on it.
__global__ void __launch_bounds__(kBlock) fb_cnst_update(Dev s, double prec) {
  if (s.ctl[CTL_DONE])
    return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int64_t c = int64_t(blockIdx.x) * wpb + threadIdx.x / kWave; c < s.nC; c += int64_t(gridDim.x) * wpb) {
    if (s.ratio[c] != 0.0)
      continue;
    const uint32_t b = s.cnst_ptr[c], e = s.cnst_ptr[c + 1];
    const bool fat = s.cflags[c] & 1;
    double acc = fat ? dinf() : 0.0;
    for (uint32_t j = b + lane; j < e; j += kWave) {
      const double d = s.csc_w[j] * s.vtmp[s.csc_v[j]];
      acc = fat ? fmin(acc, d) : acc + d;
    }
    acc = fat ? wave_min(acc) : wave_sum(acc);
    double rem = s.rem[c];
    if (!fat) {
      rem -= acc;
    } else {
      double u = s.use[c];
      if (s.cflags[c] & 2)
        u = fmin(u, 0.0);
      u = fmin(u, acc);
      s.use[c] = u;
      rem -= u;
    }
    if (rem < prec)
      rem = 0.0;
    const bool erase = rem <= 0.0;
    if (lane == 0) {
      s.rem[c] = rem;
      if (erase)
        s.ratio[c] = dinf();
    }
    if (erase)
      for (uint32_t j = b + lane; j < e; j += kWave)
        s.vst[s.csc_v[j]] = 0;
  }
}

int grid_for(int64_t n, int per_block) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1)
    g = 1;
  if (g > kMaxBlocks)
    g = kMaxBlocks;
  return int(g);
}

}  // namespace

// =============================================================================================
// context + C ABI
// =============================================================================================
struct lmmhip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Dev d{};
  std::vector<void*> allocs;  // owned device allocations
  int32_t* h_ctl = nullptr;   // pinned mirror of the control words
  bool uploaded = false;
  bool profiling = false;
  int group = 8;  // lanes per row in mm_vote (power of two >= mean row length, <= 64)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // per-launch event pairs (profiling mode): recorded without synchronising, resolved after the
  // solve, so the timed launch sequence is not serialised by the measurement.
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  std::vector<int> launch_slot, launch_round;
  std::vector<float> launch_ms;
  lmmhip_stats stats{};
};

static void free_all(lmmhip_ctx* c) {
  for (void* p : c->allocs)
    (void)hipFree(p);
  c->allocs.clear();
  c->d = Dev{};
  c->uploaded = false;
}

template <class T> static int dalloc(lmmhip_ctx* c, T** out, int64_t n) {
  void* p = nullptr;
  size_t bytes = size_t(n > 0 ? n : 1) * sizeof(T);
  HIPCHK(hipMalloc(&p, bytes));
  c->allocs.push_back(p);
  *out = static_cast<T*>(p);
  return 0;
}

extern "C" {

const char* lmmhip_last_error(void) { return g_err.c_str(); }

int lmmhip_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_err = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    return 0;
  }
  return n;
}

int lmmhip_ctx_create(int device, lmmhip_ctx** out) {
  if (!out)
    return fail(LMMHIP_E_ARG, "null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(LMMHIP_E_NODEVICE, "no HIP device visible (the MI355X path has no CPU fallback)");
  auto* c = new lmmhip_ctx;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess)
      device = 0;
  }
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess)
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&c->h_ctl, CTL_WORDS * sizeof(int32_t), hipHostMallocDefault);
  if (e == hipSuccess)
    e = hipEventCreate(&c->ev0);
  if (e == hipSuccess)
    e = hipEventCreate(&c->ev1);
  if (e != hipSuccess) {
    delete c;
    return fail(LMMHIP_E_HIP, std::string("context creation: ") + hipGetErrorString(e));
  }
  *out = c;
  return 0;
}

int lmmhip_ctx_destroy(lmmhip_ctx* c) {
  if (!c)
    return 0;
  (void)hipSetDevice(c->device);
  if (c->stream)
    (void)hipStreamSynchronize(c->stream);
  free_all(c);
  if (c->h_ctl)
    (void)hipHostFree(c->h_ctl);
  if (c->ev0)
    (void)hipEventDestroy(c->ev0);
  if (c->ev1)
    (void)hipEventDestroy(c->ev1);
  for (hipEvent_t ev : c->pool)
    (void)hipEventDestroy(ev);
  if (c->stream)
    (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int lmmhip_upload(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, const int64_t* var_ptr,
                  const int32_t* cnst_idx, const double* weight, const double* penalty, const double* var_bound,
                  const double* cnst_bound, const uint8_t* cnst_flags) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (nV < 0 || nC < 0 || nnz < 0 || nV >= (1 << 30) || nC >= (1 << 30) || nnz > INT32_MAX)
    return fail(LMMHIP_E_ARG, "sizes out of range");
  if (nV > 0 && (!var_ptr || !penalty || !var_bound))
    return fail(LMMHIP_E_ARG, "null variable arrays");
  if (nC > 0 && (!cnst_bound || !cnst_flags))
    return fail(LMMHIP_E_ARG, "null constraint arrays");
  if (nnz > 0 && (!cnst_idx || !weight))
    return fail(LMMHIP_E_ARG, "null element arrays");
  if (nV > 0 && (var_ptr[0] != 0 || var_ptr[nV] != nnz))
    return fail(LMMHIP_E_ARG, "var_ptr must start at 0 and end at nnz");
  // host-side validation + 32-bit offsets + CSC (constraint-major) mirror by a stable counting sort
  std::vector<uint32_t> vp32(static_cast<size_t>(nV) + 1, 0);
  for (int64_t v = 0; v < nV; v++) {
    if (var_ptr[v + 1] < var_ptr[v])
      return fail(LMMHIP_E_ARG, "var_ptr not monotone");
    vp32[size_t(v) + 1] = uint32_t(var_ptr[v + 1]);
  }
  std::vector<uint32_t> cptr(static_cast<size_t>(nC) + 1, 0);
  for (int64_t j = 0; j < nnz; j++) {
    int32_t k = cnst_idx[j];
    if (k < 0 || k >= nC)
      return fail(LMMHIP_E_ARG, "cnst_idx out of range");
    if (!(weight[j] > 0))
      return fail(LMMHIP_E_ARG, "element weights must be > 0 (only active elements are flattened)");
    cptr[size_t(k) + 1]++;
  }
  for (int64_t v = 0; v < nV; v++)
    if (!(penalty[v] > 0))
      return fail(LMMHIP_E_ARG, "penalties must be > 0 (only enabled variables are flattened)");
  for (int64_t k = 0; k < nC; k++)
    cptr[size_t(k) + 1] += cptr[size_t(k)];
  std::vector<int32_t> cv(static_cast<size_t>(nnz));
  std::vector<double> cw(static_cast<size_t>(nnz));
  {
    std::vector<uint32_t> cur(cptr.begin(), cptr.end() - 1);
    for (int64_t v = 0; v < nV; v++)
      for (int64_t j = var_ptr[v]; j < var_ptr[v + 1]; j++) {
        uint32_t pos = cur[size_t(cnst_idx[j])]++;
        cv[pos] = int32_t(v);
        cw[pos] = weight[j];
      }
  }
  std::vector<int32_t> iota(static_cast<size_t>(nV));
  for (int64_t v = 0; v < nV; v++)
    iota[size_t(v)] = int32_t(v);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  free_all(c);
  Dev& d = c->d;
  d.nV = int32_t(nV);
  d.nC = int32_t(nC);
  d.nnz = nnz;
  uint32_t *vp, *cp, *crow1, *crow2;
  int32_t *csr_c, *csc_v, *cvar0, *cvar1, *cvar2, *ccol1, *ccol2;
  double *csr_w, *csc_w, *pen, *vb, *cb;
  uint8_t* cf;
  const int64_t nblk = (nV + kCompactRows - 1) / kCompactRows + 1;
  int rc = 0;
  rc |= dalloc(c, &vp, nV + 1);
  rc |= dalloc(c, &csr_c, nnz);
  rc |= dalloc(c, &csr_w, nnz);
  rc |= dalloc(c, &cp, nC + 1);
  rc |= dalloc(c, &csc_v, nnz);
  rc |= dalloc(c, &csc_w, nnz);
  rc |= dalloc(c, &pen, nV);
  rc |= dalloc(c, &vb, nV);
  rc |= dalloc(c, &cb, nC);
  rc |= dalloc(c, &cf, nC);
  rc |= dalloc(c, &d.x, nV);
  rc |= dalloc(c, &d.fixr, nV);
  rc |= dalloc(c, &d.vtmp, nV);
  rc |= dalloc(c, &d.vst, nV);
  rc |= dalloc(c, &d.ratio, nC);
  rc |= dalloc(c, &d.key, nC);
  rc |= dalloc(c, &d.rem, nC);
  rc |= dalloc(c, &d.use, nC);
  rc |= dalloc(c, &d.drem, nC);
  rc |= dalloc(c, &d.duse, nC);
  rc |= dalloc(c, &d.acnt, nC);
  rc |= dalloc(c, &d.dcnt, nC);
  rc |= dalloc(c, &d.votes, nC);
  rc |= dalloc(c, &cvar0, nV);
  rc |= dalloc(c, &cvar1, nV);
  rc |= dalloc(c, &cvar2, nV);
  rc |= dalloc(c, &crow1, nV + 1);
  rc |= dalloc(c, &crow2, nV + 1);
  rc |= dalloc(c, &ccol1, nnz);
  rc |= dalloc(c, &ccol2, nnz);
  for (int b = 0; b < 3; b++)
    rc |= dalloc(c, &d.valive[b], nV);
  rc |= dalloc(c, &d.vinfo, nV);
  rc |= dalloc(c, &d.bsum, 2 * nblk);
  rc |= dalloc(c, &d.ctl, CTL_WORDS);
  if (rc) {
    free_all(c);
    return LMMHIP_E_HIP;
  }
  HIPCHK(hipMemcpyAsync(vp, vp32.data(), sizeof(uint32_t) * (nV + 1), hipMemcpyHostToDevice, c->stream));
  if (nnz > 0) {
    HIPCHK(hipMemcpyAsync(csr_c, cnst_idx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csr_w, weight, sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csc_v, cv.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csc_w, cw.data(), sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipMemcpyAsync(cp, cptr.data(), sizeof(uint32_t) * (nC + 1), hipMemcpyHostToDevice, c->stream));
  if (nV > 0) {
    HIPCHK(hipMemcpyAsync(pen, penalty, sizeof(double) * nV, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(vb, var_bound, sizeof(double) * nV, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(cvar0, iota.data(), sizeof(int32_t) * nV, hipMemcpyHostToDevice, c->stream));
  }
  if (nC > 0) {
    HIPCHK(hipMemcpyAsync(cb, cnst_bound, sizeof(double) * nC, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(cf, cnst_flags, sizeof(uint8_t) * nC, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));  // host staging vectors die at return
  d.var_ptr = vp;
  d.csr_c = csr_c;
  d.csr_w = csr_w;
  d.cnst_ptr = cp;
  d.csc_v = csc_v;
  d.csc_w = csc_w;
  d.pen = pen;
  d.vbound = vb;
  d.cbound = cb;
  d.cflags = cf;
  d.cvar[0] = cvar0;
  d.crow[0] = vp;
  d.ccol[0] = csr_c;
  d.cvar[1] = cvar1;
  d.crow[1] = crow1;
  d.ccol[1] = ccol1;
  d.cvar[2] = cvar2;
  d.crow[2] = crow2;
  d.ccol[2] = ccol2;
  const double mean = nV > 0 ? double(nnz) / double(nV) : 1.0;
  c->group = mean <= 4 ? 4 : mean <= 8 ? 8 : mean <= 16 ? 16 : mean <= 32 ? 32 : 64;
  c->uploaded = true;
  c->stats = lmmhip_stats{};
  c->stats.n_var = nV;
  c->stats.n_cnst = nC;
  c->stats.nnz = nnz;
  return 0;
}

int lmmhip_update_vars(lmmhip_ctx* c, const double* penalty, const double* var_bound) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  HIPCHK(hipSetDevice(c->device));
  if (penalty && c->d.nV)
    HIPCHK(hipMemcpyAsync((void*)c->d.pen, penalty, sizeof(double) * c->d.nV, hipMemcpyHostToDevice, c->stream));
  if (var_bound && c->d.nV)
    HIPCHK(
        hipMemcpyAsync((void*)c->d.vbound, var_bound, sizeof(double) * c->d.nV, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_update_cnsts(lmmhip_ctx* c, const double* cnst_bound) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  HIPCHK(hipSetDevice(c->device));
  if (cnst_bound && c->d.nC)
    HIPCHK(
        hipMemcpyAsync((void*)c->d.cbound, cnst_bound, sizeof(double) * c->d.nC, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_set_profiling(lmmhip_ctx* c, int on) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  c->profiling = on != 0;
  return 0;
}

static int solve_maxmin(lmmhip_ctx* c, double prec);
static int solve_fair(lmmhip_ctx* c, double prec);
static int resolve_profile(lmmhip_ctx* c);

int lmmhip_solve(lmmhip_ctx* c, int kind, double precision) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "solve before upload");
  if (kind != LMMHIP_KIND_MAXMIN && kind != LMMHIP_KIND_FAIR_BOTTLENECK)
    return fail(LMMHIP_E_ARG, "unknown solver kind");
  HIPCHK(hipSetDevice(c->device));
  for (int i = 0; i < 8; i++) {
    c->stats.kernel_ms[i] = 0;
    c->stats.kernel_launches[i] = 0;
  }
  c->pool_used = 0;
  c->launch_slot.clear();
  c->launch_round.clear();
  c->launch_ms.clear();
  HIPCHK(hipMemsetAsync(c->d.ctl, 0, CTL_WORDS * sizeof(int32_t), c->stream));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  int rc = kind == LMMHIP_KIND_MAXMIN ? solve_maxmin(c, precision) : solve_fair(c, precision);
  if (rc)
    return rc;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  HIPCHK(hipEventSynchronize(c->ev1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->stats.device_ms = ms;
  c->stats.rounds = c->h_ctl[CTL_ROUNDS];
  if (c->profiling)
    return resolve_profile(c);
  return 0;
}

// Launch helper.  In profiling mode every launch is bracketed by two events from a pool (no host
// synchronisation); their elapsed times are resolved once the solve has finished.
static int prof_event(lmmhip_ctx* c, hipEvent_t* out) {
  if (c->pool_used == c->pool.size()) {
    hipEvent_t ev;
    HIPCHK(hipEventCreate(&ev));
    c->pool.push_back(ev);
  }
  *out = c->pool[c->pool_used++];
  return 0;
}

#define LAUNCH(slot, round, kern, grid, block, ...)                                 \
  do {                                                                              \
    hipEvent_t e0_ = nullptr, e1_ = nullptr;                                        \
    if (c->profiling) {                                                             \
      if (int rc_ = prof_event(c, &e0_))                                            \
        return rc_;                                                                 \
      HIPCHK(hipEventRecord(e0_, c->stream));                                       \
    }                                                                               \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, c->stream, __VA_ARGS__);  \
    HIPCHK(hipGetLastError());                                                      \
    if (c->profiling) {                                                             \
      if (int rc_ = prof_event(c, &e1_))                                            \
        return rc_;                                                                 \
      HIPCHK(hipEventRecord(e1_, c->stream));                                       \
      c->launch_slot.push_back(slot);                                               \
      c->launch_round.push_back(int(round));                                        \
    }                                                                               \
    c->stats.kernel_launches[slot] += 1;                                            \
  } while (0)

static int resolve_profile(lmmhip_ctx* c) {
  c->launch_ms.assign(c->launch_slot.size(), 0.f);
  for (size_t i = 0; i < c->launch_slot.size(); i++) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->pool[2 * i], c->pool[2 * i + 1]));
    c->launch_ms[i] = ms;
    c->stats.kernel_ms[c->launch_slot[i]] += ms;
  }
  return 0;
}

static int poll_ctl(lmmhip_ctx* c) {
  HIPCHK(hipMemcpyAsync(c->h_ctl, c->d.ctl, CTL_WORDS * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

static int launch_vote(lmmhip_ctx* c, int64_t r, int64_t nrows, int buf, int par) {
  const Dev& d = c->d;
  const int G = c->group;
  const int grid = grid_for(nrows * G, kBlock);
  switch (G) {
  case 4:
    LAUNCH(2, r, mm_vote<4>, grid, kBlock, d, buf, par);
    break;
  case 8:
    LAUNCH(2, r, mm_vote<8>, grid, kBlock, d, buf, par);
    break;
  case 16:
    LAUNCH(2, r, mm_vote<16>, grid, kBlock, d, buf, par);
    break;
  case 32:
    LAUNCH(2, r, mm_vote<32>, grid, kBlock, d, buf, par);
    break;
  default:
    LAUNCH(2, r, mm_vote<64>, grid, kBlock, d, buf, par);
    break;
  }
  return 0;
}

// Slots: 0 mm_init_cnsts, 1 mm_init_vars, 2 mm_vote, 3 mm_fix, 4 mm_update, 5 compaction.
static int solve_maxmin(lmmhip_ctx* c, double prec) {
  Dev& d = c->d;
  const int gC4 = grid_for(d.nC, kBlock / kWave);
  const int gC = grid_for(d.nC, kBlock);
  LAUNCH(0, -1, mm_init_cnsts, gC4, kBlock, d, prec);
  LAUNCH(1, -1, mm_init_vars, grid_for(d.nV, kBlock), kBlock, d);
  // Every round fixes at least one variable (progress), so nV + 2 rounds bound it.
  const int64_t max_rounds = int64_t(d.nV) + 2;
  int64_t r = 0, last_compact = 0, nrows = d.nV;
  int buf = 0, chunk = 2;
  for (;;) {
    const int gR = grid_for(nrows, kBlock);
    for (int k = 0; k < chunk; k++, r++) {
      const int par = int(r & 1);
      if (int rc = launch_vote(c, r, nrows, buf, par))
        return rc;
      LAUNCH(3, r, mm_fix, gR, kBlock, d, buf, int(r));
      LAUNCH(4, r, mm_update, gC, kBlock, d, par, prec);
    }
    if (int rc = poll_ctl(c))
      return rc;
    if (c->h_ctl[CTL_DONE])
      break;
    if (r > max_rounds)
      return fail(LMMHIP_E_NOCONVERGE, "maxmin round guard tripped");
    if (r - last_compact >= 16 && nrows > 4096) {  // order-preserving compaction of the alive rows
      const int out = buf == 1 ? 2 : 1;
      const int nblk = int((nrows + kCompactRows - 1) / kCompactRows);
      LAUNCH(5, r, cmp_count, nblk, kBlock, d, buf);
      LAUNCH(5, r, cmp_scan, 1, 1024, d, nblk, out);
      LAUNCH(5, r, cmp_write, nblk, kBlock, d, buf, out);
      if (int rc = poll_ctl(c))
        return rc;
      nrows = c->h_ctl[CTL_NROWS + out];
      buf = out;
      last_compact = r;
    }
    if (chunk < 16)
      chunk *= 2;
  }
  return 0;
}

static int solve_fair(lmmhip_ctx* c, double prec) {
  Dev& d = c->d;
  const int gC4 = grid_for(d.nC, kBlock / kWave);
  const int gVC = grid_for(std::max(d.nV, d.nC), kBlock);
  const int gV = grid_for(d.nV, kBlock);
  LAUNCH(0, -1, fb_init, gVC, kBlock, d);
  // The reference's rounds are not bounded by the system size (FATPIPE remaining can shrink
  // geometrically: millions of rounds on 60-variable systems); give up past this budget.
  const int64_t max_rounds = 64 * (int64_t(d.nV) + int64_t(d.nC)) + 4096;
  int64_t r = 0;
  int chunk = 4;
  for (;;) {
    for (int k = 0; k < chunk; k++, r++) {
      const int par = int(r & 1);
      LAUNCH(2, r, fb_cnst_share, gC4, kBlock, d, par);
      LAUNCH(3, r, fb_var_inc, gV, kBlock, d, par, int(r));
      LAUNCH(4, r, fb_cnst_update, gC4, kBlock, d, prec);
    }
    if (int rc = poll_ctl(c))
      return rc;
    if (c->h_ctl[CTL_DONE])
      break;
    if (r > max_rounds)
      return fail(LMMHIP_E_NOCONVERGE, "fair-bottleneck round guard tripped");
    if (chunk < 64)
      chunk *= 2;
  }
  return 0;
}

int lmmhip_launch_profile(lmmhip_ctx* c, int* slot, int* round, float* ms, int cap) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  int n = int(c->launch_ms.size());
  for (int i = 0; i < n && i < cap; i++) {
    slot[i] = c->launch_slot[size_t(i)];
    round[i] = c->launch_round[size_t(i)];
    ms[i] = c->launch_ms[size_t(i)];
  }
  return n;
}

int lmmhip_round_profile(lmmhip_ctx* c, int64_t* alive_vars, int64_t* alive_elems, int cap) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  const int64_t nV = c->d.nV;
  std::vector<int32_t> fr(size_t(nV > 0 ? nV : 1));
  std::vector<uint32_t> vp(size_t(nV) + 1);
  HIPCHK(hipSetDevice(c->device));
  if (nV) {
    HIPCHK(hipMemcpyAsync(fr.data(), c->d.fixr, sizeof(int32_t) * nV, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(vp.data(), c->d.var_ptr, sizeof(uint32_t) * (nV + 1), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  const int R = int(c->stats.rounds);
  // a variable is alive in rounds 0..fixr (inclusive); -1 = never processed
  std::vector<int64_t> dv(size_t(R) + 2, 0), de(size_t(R) + 2, 0);
  for (int64_t v = 0; v < nV; v++) {
    int f = fr[size_t(v)];
    if (f < 0)
      continue;
    if (f > R)
      f = R;
    dv[size_t(f)] += 1;
    de[size_t(f)] += vp[size_t(v) + 1] - vp[size_t(v)];
  }
  int64_t av = 0, ae = 0;
  for (int r = R; r >= 0; r--) {  // suffix sums
    av += dv[size_t(r)];
    ae += de[size_t(r)];
    if (r < cap) {
      alive_vars[r] = av;
      alive_elems[r] = ae;
    }
  }
  return R;
}

int lmmhip_get_values(lmmhip_ctx* c, double* out) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  if (!out && c->d.nV)
    return fail(LMMHIP_E_ARG, "null output");
  HIPCHK(hipSetDevice(c->device));
  if (c->d.nV)
    HIPCHK(hipMemcpyAsync(out, c->d.x, sizeof(double) * c->d.nV, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_values_device_ptr(lmmhip_ctx* c, const double** dptr) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  *dptr = c->d.x;
  return 0;
}

int lmmhip_get_stats(lmmhip_ctx* c, lmmhip_stats* out) {
  if (!c || !out)
    return fail(LMMHIP_E_ARG, "null argument");
  *out = c->stats;
  return 0;
}

}  // extern "C"
