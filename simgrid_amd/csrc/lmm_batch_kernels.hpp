// lmm_batch_kernels.hpp — many small independent max-min systems, one workgroup per system, the whole
// system in LDS (config C3: 4096 maxmin_bench "medium" systems,
// teshsuite/surf/maxmin_bench/maxmin_bench.cpp:37-116).
//
// The uploaded system is a disjoint union declared block-diagonal by lmmhip_set_batch: system i owns
// the dense variables [var_off[i], var_off[i+1]) and constraints [cnst_off[i], cnst_off[i+1]).  A
// workgroup stages one system's structure in LDS (16-bit local indices) and runs the same local-minimum
// progressive filling as the global engines (lmm_maxmin_kernels.hpp; maxmin.cpp:509-680) with every round
// inside the workgroup — no grid-wide synchronisation, no host round-trip:
//   init     usage = sum / max of w/p over the constraint's elements, thread per constraint, sequential in
//            CSC order like the reference's loop (maxmin.cpp:520-555)
//   round:   V  kG lanes per variable: exact minimum ratio over its live constraints (ties: smallest id);
//               a variable whose bound*penalty is below it is fixed at its bound (maxmin.cpp:563-595);
//               each live variable marks the constraints it blocks (votes elsewhere / bound fix), so a live
//               constraint left unmarked is a local minimum (ready: every live element votes for it)
//            S  kG lanes per variable voting for a ready constraint: x = ratio / penalty (maxmin.cpp:583);
//               its decrements go to its other live constraints as fixed-point integers (LDS atomics)
//            U  thread per constraint: the update of update_groups (clamps, FATPIPE recompute, saturation)
// Decrements are fixed-point integers (CstRec): results do not depend on the order of the LDS atomics.
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

constexpr int kBB = 256;  // threads per workgroup
constexpr int kG = 4;     // lanes per variable (vote, saturation) and per constraint (ready test)
constexpr int kSatW = 4;  // weights per lane prefetched by the saturation (rows up to kG * kSatW elements)

// LDS bytes of a workgroup for systems of at most nv variables, nc constraints and nnz elements
__host__ __device__ inline size_t batch_lds_bytes(int nv, int nc, int nnz) {
  size_t b = sizeof(double) * (4 * size_t(nc) + 3 * size_t(nv)) +                 // cnst / var state
             sizeof(unsigned long long) * 3 * size_t(nc) +                         // decrement records
             sizeof(int32_t) * size_t(nc) +                                        // scale exponents
             sizeof(uint16_t) * (size_t(nv) + 1 + size_t(nc) + 1 + 2 * size_t(nnz) + size_t(nv)) +
             3 * size_t(nc) + size_t(nv);
  return (b + 15) / 16 * 16;
}

__global__ void __launch_bounds__(kBB, 8) mm_batch_lds(Dev s, const int64_t* __restrict__ var_off,
                                                   const int64_t* __restrict__ cnst_off, int64_t nsys, double prec,
                                                   int max_nv, int max_nc, int max_nnz, int32_t* block_rounds) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  double* c_rem = reinterpret_cast<double*>(lds);
  double* c_use = c_rem + max_nc;
  double* c_rat = c_use + max_nc;
  double* c_bnd = c_rat + max_nc;
  double* v_x = c_bnd + max_nc;
  double* v_pen = v_x + max_nv;
  double* v_vb = v_pen + max_nv;
  unsigned long long* c_q = reinterpret_cast<unsigned long long*>(v_vb + max_nv);  // [3 * max_nc]
  int32_t* c_exp = reinterpret_cast<int32_t*>(c_q + 3 * max_nc);
  uint16_t* l_vp = reinterpret_cast<uint16_t*>(c_exp + max_nc);  // [max_nv + 1] CSR offsets
  uint16_t* l_cp = l_vp + (max_nv + 1);                           // [max_nc + 1] CSC offsets
  uint16_t* l_cc = l_cp + (max_nc + 1);                           // [max_nnz] CSR local constraint
  uint16_t* l_cv = l_cc + max_nnz;                                // [max_nnz] CSC local variable
  uint16_t* v_vote = l_cv + max_nnz;                              // [max_nv]
  uint8_t* c_st = reinterpret_cast<uint8_t*>(v_vote + max_nv);    // 0 live, 1 out
  uint8_t* c_fl = c_st + max_nc;                                  // FATPIPE
  uint8_t* c_nr = c_fl + max_nc;  // 1 = blocked this round: a live variable on it votes elsewhere or hit its bound
  uint8_t* v_st = c_nr + max_nc;  // 0 live, 1 done
  int rounds_max = 0;
  for (int64_t sy = blockIdx.x; sy < nsys; sy += gridDim.x) {
    const int64_t vb = var_off[sy], cb = cnst_off[sy];
    const int nv = int(var_off[sy + 1] - vb), nc = int(cnst_off[sy + 1] - cb);
    const uint32_t eb = s.var_ptr[vb], kb = s.cnst_ptr[cb];
    const int ne = int(s.var_ptr[vb + nv] - eb);
    // ---- stage the system ----
    for (int i = threadIdx.x; i <= nv; i += kBB)
      l_vp[i] = uint16_t(s.var_ptr[vb + i] - eb);
    for (int i = threadIdx.x; i <= nc; i += kBB)
      l_cp[i] = uint16_t(s.cnst_ptr[cb + i] - kb);
    for (int j = threadIdx.x; j < ne; j += kBB) {
      l_cc[j] = uint16_t(s.csr_c[eb + j] - cb);
      l_cv[j] = uint16_t(s.csc_v[kb + j] - vb);
    }
    for (int v = threadIdx.x; v < nv; v += kBB) {
      v_x[v] = 0.0;
      v_st[v] = 0;
      v_pen[v] = s.pen[vb + v];
      v_vb[v] = s.vbound[vb + v];
    }
    __syncthreads();
    // ---- init: maxmin.cpp:520-555, thread per constraint: usage = sum (FATPIPE: max) of w/p over its
    // elements in CSC order, one addition after the other like the reference's loop ----
    for (int c = threadIdx.x; c < nc; c += kBB) {
      const int b = l_cp[c], e = l_cp[c + 1];
      const bool fat = s.cflags[cb + c] & 1;
      double acc = 0.0;
      for (int k0 = b; k0 < e; k0 += 4) {  // four loads in flight, added in CSC order
        double u[4];
#pragma unroll
        for (int i = 0; i < 4; i++)
          u[i] = k0 + i < e ? s.csc_u[kb + k0 + i] : 0.0;
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (k0 + i < e)
            acc = fat ? fmax(acc, u[i]) : acc + u[i];
      }
      const double bound = s.cbound[cb + c];
      const bool part = bound > bound * prec;
      const double usage = part ? acc : 0.0;
      const bool alive = part && usage > 0;
      c_rem[c] = bound;
      c_use[c] = usage;
      c_bnd[c] = bound;
      c_rat[c] = alive ? bound / usage : dinf();
      c_exp[c] = cexp_pack(alive ? dec_scale(bound) : 0, alive ? dec_scale(usage) : 0, fat, !alive);
      c_q[3 * c] = c_q[3 * c + 1] = c_q[3 * c + 2] = 0;
      c_st[c] = alive ? 0 : 1;
      c_fl[c] = fat;
      c_nr[c] = 0;
    }
    __syncthreads();
    int round = 0;
    for (;; round++) {
      // ---- V: votes and bound fixes, G lanes per variable; every live variable marks the constraints it
      // blocks (c_nr): the ones it does not vote for, or all of them when it is fixed at its bound.  A
      // live constraint nothing blocks is a local minimum: it saturates in S (ready test, maxmin.cpp:578) ----
      for (int v = threadIdx.x / kG; v < nv; v += kBB / kG) {  // uniform within each G-lane group
        const int g = threadIdx.x & (kG - 1);
        const bool in = v_st[v] == 0;
        double minr = dinf();
        int t = 0xFFFF;
        const int jb = in ? l_vp[v] : 0, je = in ? l_vp[v + 1] : 0;
        for (int j = jb + g; j < je; j += kG) {
          const int c = l_cc[j];
          const double r = c_rat[c];  // +inf once c left the light table
          if (r < minr || (r == minr && c < t)) {
            minr = r;
            t = c;
          }
        }
#pragma unroll
        for (int o = 1; o < kG; o <<= 1) {  // (min ratio, smallest id) over the group
          const double r2 = __shfl_xor(minr, o, kWave);
          const int t2 = __shfl_xor(t, o, kWave);
          if (r2 < minr || (r2 == minr && t2 < t)) {
            minr = r2;
            t = t2;
          }
        }
        if (!in)
          continue;
        const double vbd = v_vb[v], p = v_pen[v];
        if (!(minr < dinf())) {  // every constraint of v left the light table: v stays at 0
          if (g == 0)
            v_st[v] = 1;
        } else if (vbd > 0 && vbd * p < minr) {  // maxmin.cpp:587-589
          if (g == 0) {
            v_x[v] = vbd;
            v_st[v] = 1;
          }
          for (int j = jb + g; j < je; j += kG) {
            const int c = l_cc[j];
            c_nr[c] = 1;
            const double w = s.csr_w[eb + j];
            if (c_st[c] == 1)
              continue;
            atomicAdd(&c_q[3 * c + 2], 1ull);
            if (!c_fl[c]) {
              atomicAdd(&c_q[3 * c], dec_q(w * vbd, cexp_rem(c_exp[c])));
              atomicAdd(&c_q[3 * c + 1], dec_q(w / p, cexp_use(c_exp[c])));
            }
          }
        } else {
          if (g == 0)
            v_vote[v] = uint16_t(t);
          for (int j = jb + g; j < je; j += kG) {
            const int c = l_cc[j];
            if (c != t)
              c_nr[c] = 1;
          }
        }
      }
      __syncthreads();
      // ---- S: saturation of the unblocked constraints' variables, G lanes per variable ----
      for (int v = threadIdx.x / kG; v < nv; v += kBB / kG) {
        const int g = threadIdx.x & (kG - 1);
        if (v_st[v] != 0)
          continue;
        const int t = v_vote[v];
        if (c_nr[t])  // (t is live: v voted for it this round)
          continue;
        const double p = v_pen[v];
        const double x = c_rat[t] / p;
        const int jb = l_vp[v] + g, je = l_vp[v + 1];
        double wv[kSatW];  // the group's weights, loads in flight together
#pragma unroll
        for (int i = 0; i < kSatW; i++)
          wv[i] = jb + i * kG < je ? s.csr_w[eb + jb + i * kG] : 0.0;
        if (g == 0) {
          v_x[v] = x;
          v_st[v] = 1;
        }
        for (int j = jb, i = 0; j < je; j += kG, i++) {
          const int c = l_cc[j];
          double w = 0.0;
#pragma unroll
          for (int k = 0; k < kSatW; k++)
            w = i == k ? wv[k] : w;
          if (i >= kSatW)
            w = s.csr_w[eb + j];
          if (c == t || c_st[c] == 1)
            continue;
          atomicAdd(&c_q[3 * c + 2], 1ull);
          if (!c_fl[c]) {
            atomicAdd(&c_q[3 * c], dec_q(w * x, cexp_rem(c_exp[c])));
            atomicAdd(&c_q[3 * c + 1], dec_q(w / p, cexp_use(c_exp[c])));
          }
        }
      }
      __syncthreads();
      // ---- U: constraint update (update_groups' arithmetic); unblocked live constraints saturated ----
      int alive = 0;
      for (int c = threadIdx.x; c < nc; c += kBB) {
        if (c_st[c] == 1)
          continue;
        if (!c_nr[c]) {  // saturated (maxmin.cpp:608-615)
          c_st[c] = 1;
          c_rat[c] = dinf();
          continue;
        }
        c_nr[c] = 0;
        const unsigned long long qz = c_q[3 * c + 2];
        if (qz == 0) {
          alive = 1;
          continue;
        }
        const unsigned long long qx = c_q[3 * c], qy = c_q[3 * c + 1];
        c_q[3 * c] = c_q[3 * c + 1] = c_q[3 * c + 2] = 0;
        const double bound = c_bnd[c];
        double rem = c_rem[c], use;
        if (!c_fl[c]) {
          const int32_t ce = c_exp[c];
          use = c_use[c] - dec_val(qy, cexp_use(ce));
          rem -= dec_val(qx, cexp_rem(ce));
          if (rem < bound * prec)
            rem = 0.0;
          if (use < prec)
            use = 0.0;
        } else {  // FATPIPE: max w/p over the elements whose variable is still at 0 (maxmin.cpp:625-658)
          use = 0.0;
          for (int k = l_cp[c]; k < l_cp[c + 1]; k++)
            if (!(v_x[l_cv[k]] > 0))
              use = fmax(use, s.csc_u[kb + k]);
        }
        c_rem[c] = rem;
        c_use[c] = use;
        if (!(use > prec) || !(rem > bound * prec)) {
          c_st[c] = 1;
          c_rat[c] = dinf();
        } else {
          c_rat[c] = rem / use;
          alive = 1;
        }
      }
      if (!__syncthreads_or(alive))  // light table empty (maxmin.cpp:680)
        break;
      if (round > nv + 2) {  // every round fixes >= 1 variable: the invariant broke
        rounds_max = -1;
        break;
      }
    }
    if (rounds_max < 0) {  // guard tripped: report it (mm_batch_rounds -> CTL_ERR = 2) and stop this block
      if (threadIdx.x == 0)
        block_rounds[blockIdx.x] = -1;
      return;
    }
    rounds_max = round + 1 > rounds_max ? round + 1 : rounds_max;
    for (int v = threadIdx.x; v < nv; v += kBB)
      s.x[vb + v] = v_x[v];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    block_rounds[blockIdx.x] = rounds_max;
}

// Block-diagonal check of the declared batch: every element of system i's variables is on one of system
// i's constraints (*bad = 1 otherwise).
__global__ void __launch_bounds__(kBlock) mm_batch_check(Dev s, const int64_t* var_off, const int64_t* cnst_off,
                                                         int64_t nsys, int32_t* bad) {
  for (int64_t sy = blockIdx.x; sy < nsys; sy += gridDim.x) {
    const int64_t cb = cnst_off[sy], ce = cnst_off[sy + 1];
    for (uint32_t j = s.var_ptr[var_off[sy]] + threadIdx.x; j < s.var_ptr[var_off[sy + 1]]; j += kBlock)
      if (s.csr_c[j] < cb || s.csr_c[j] >= ce)
        *bad = 1;
  }
}

__global__ void __launch_bounds__(kBlock) mm_batch_rounds(const int32_t* block_rounds, int n, int32_t* ctl) {
  int m = 0, err = 0;
  for (int i = threadIdx.x; i < n; i += kBlock) {
    m = block_rounds[i] > m ? block_rounds[i] : m;
    err |= block_rounds[i] < 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int t = __shfl_xor(m, o, kWave);
    m = t > m ? t : m;
    err |= __shfl_xor(err, o, kWave);
  }
  __shared__ int wm[kBlock / kWave], we[kBlock / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0) {
    wm[threadIdx.x / kWave] = m;
    we[threadIdx.x / kWave] = err;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kBlock / kWave; i++) {
      m = wm[i] > m ? wm[i] : m;
      err |= we[i];
    }
    ctl[CTL_ROUNDS] = m;
    ctl[CTL_LASTR] = m - 1;
    ctl[CTL_ERR] = err ? 2 : 0;  // 2 = round guard (a block's system stopped after nv + 2 rounds)
  }
}

}  // namespace lmmdev
