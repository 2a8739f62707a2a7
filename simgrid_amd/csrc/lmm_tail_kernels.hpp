// lmm_tail_kernels.hpp — hand-off of a max-min solve's tail to a compacted system (gfx950; included by
// lmm_hip.hip).  DESIGN.md §6, "Round 5: the tail hand-off".
//
// Late in a large solve (C2: the last ~60 of 214 rounds) few variables and constraints are left, but every
// round of the multi-launch engine still passes over the whole system's constraint arrays (the update, the
// changed-constraint bitmap every vote workgroup copies into LDS, the saturation's segment prefix) and pays the
// same dependent-latency chains: 60-90 us per round for work worth a few.  At a poll whose alive-row count is
// below LMMHIP_TAIL_ROWS, the solve's remaining system — the alive constraints (key not dead) and the alive
// variables (vstate 0) with their elements on alive constraints — is copied into a child context as a system of
// its own, with its state: remaining, usage, ratio, bound, the decrement scales (cexp) and key of every alive
// constraint, values 0 for the variables.  The child then continues progressive filling from that state with
// the engine its size calls for (mm_init_cont instead of mm_init_cnsts: the constraint state is not recomputed)
// and its values are scattered back.
//
// Why the result is the same bits: a vote is the lexicographic minimum of (ratio, constraint id) over the
// variable's alive constraints whatever engine computed it (the persistent votes of the round engine are kept
// exact by their floors, lmm_maxmin_kernels.hpp), so the child's first round — every variable votes — takes the
// votes the next round of the parent would have had; constraint ids keep their order (an order-preserving
// renumbering: ties break the same way), variable order does not matter (claims go by constraint, decrements are
// fixed-point sums, FATPIPE usage a max).  The decrements keep each constraint's scales, the clamps its original
// bound.  Elements on dead constraints are dropped: a vote skips them and a push to them is skipped.  An alive
// variable with no alive constraint left is dropped at 0, as the parent's next vote would.
#pragma once
#include "lmm_maxmin_kernels.hpp"

namespace lmmdev {

// Alive-constraint flags (1 / 0) for the order-preserving renumbering (an exclusive scan follows); cf[nC] = 0.
__global__ void __launch_bounds__(kBlock) tl_cflag(Dev s, int64_t* cf) {
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c <= s.nC; c += int64_t(gridDim.x) * kBlock)
    cf[c] = c < s.nC && s.key[c] != kDeadKey ? 1 : 0;
}

// Per row of the alive-row buffer in use (nh: the host's bound of its rows): the row's elements on alive
// constraints (rl) and whether it stays (rf: an alive variable with at least one).  rl[nh] = rf[nh] = 0.
__global__ void __launch_bounds__(kBlock) tl_rowlen(Dev s, int64_t nh, const int64_t* cf, int64_t* rl,
                                                     int64_t* rf) {
  const int buf = s.ctl[CTL_BUF];
  const int64_t nrows = s.ctl[CTL_NROWS + buf];
  for (int64_t row = int64_t(blockIdx.x) * kBlock + threadIdx.x; row <= nh; row += int64_t(gridDim.x) * kBlock) {
    int64_t n = 0;
    if (row < nh && row < nrows && !s.ctl[CTL_DONE]) {
      const int v = rvar(s.cvar[buf][row]);
      if (s.vstate[v] == 0) {
        const uint32_t b = s.var_ptr[v], e = s.var_ptr[v + 1];
        for (uint32_t j0 = b; j0 < e; j0 += 8) {  // the row's constraint flags, 8 gathers in flight
          int64_t f[8];
#pragma unroll
          for (int u = 0; u < 8; u++)
            f[u] = j0 + u < e ? cf[s.csr_c[j0 + u]] : 0;
#pragma unroll
          for (int u = 0; u < 8; u++)
            n += f[u];
        }
      }
    }
    rl[row] = n;
    rf[row] = n > 0;
  }
}

// The child's rows (t: the child system's Dev): CSR offsets, renumbered constraint ids and weights, penalty,
// bound, the identity row ids of its buffer 0, the parent id of each child variable (vmap), and the (constraint,
// element) sort pairs of the CSC transpose.  cmap / rlo / rvo: exclusive scans of tl_cflag / tl_rowlen.
__global__ void __launch_bounds__(kBlock) tl_rows(Dev s, Dev t, int64_t nh, const int64_t* cmap, const int64_t* cf,
                                                  const int64_t* rlo, const int64_t* rvo, uint32_t* vp, int32_t* csr_c,
                                                  double* csr_w, double* pen, double* vb, int32_t* cvar0, int32_t* vmap,
                                                  uint32_t* skey, unsigned long long* sval) {
  const int buf = s.ctl[CTL_BUF];
  for (int64_t row = int64_t(blockIdx.x) * kBlock + threadIdx.x; row < nh; row += int64_t(gridDim.x) * kBlock) {
    const int64_t vn = rvo[row];
    if (rvo[row + 1] == vn)  // not kept
      continue;
    const int v = rvar(s.cvar[buf][row]);
    int64_t k = rlo[row];
    vp[vn] = uint32_t(k);
    pen[vn] = s.pen[v];
    vb[vn] = s.vbound[v];
    cvar0[vn] = int32_t(vn);
    vmap[vn] = v;
    for (uint32_t j = s.var_ptr[v]; j < s.var_ptr[v + 1]; j++) {
      const int32_t c = s.csr_c[j];
      if (!cf[c])
        continue;
      const uint32_t cn = uint32_t(cmap[c]);
      csr_c[k] = int32_t(cn);
      csr_w[k] = s.csr_w[j];
      skey[k] = cn;
      sval[k] = (unsigned long long)uint32_t(k) | ((unsigned long long)uint32_t(vn) << 32);
      k++;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    vp[t.nV] = uint32_t(t.nnz);
}

// CSC of the child from the sorted pairs (a stable radix sort: each column keeps its elements in row order), and
// the column offsets from the sorted keys (every column, empty ones included).
__global__ void __launch_bounds__(kBlock) tl_csc(int64_t nnz, int64_t nc, const uint32_t* sk,
                                                 const unsigned long long* sv, const double* csr_w, int32_t* csc_v,
                                                 double* csc_w, uint32_t* cptr) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nnz; i += int64_t(gridDim.x) * kBlock) {
    const unsigned long long x = sv[i];
    csc_v[i] = int32_t(uint32_t(x >> 32));
    csc_w[i] = csr_w[uint32_t(x)];
    const int64_t k = sk[i], prev = i == 0 ? -1 : int64_t(sk[i - 1]);
    for (int64_t c = prev + 1; c <= k; c++)
      cptr[c] = uint32_t(i);
    if (i == nnz - 1)
      for (int64_t c = k + 1; c <= nc; c++)
        cptr[c] = uint32_t(nnz);
  }
  if (nnz == 0 && blockIdx.x == 0)
    for (int64_t c = threadIdx.x; c <= nc; c += kBlock)
      cptr[c] = 0;
}

// The alive constraints' bound, flags and solve state into the child (t): the record (remaining, usage, ratio,
// bound; empty decrements), the decrement scales and liveness (cexp) and the 16-bit key.
__global__ void __launch_bounds__(kBlock) tl_cnsts(Dev s, Dev t, const int64_t* cmap, const int64_t* cf, double* cb,
                                                   uint8_t* cfl) {
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < s.nC; c += int64_t(gridDim.x) * kBlock) {
    if (!cf[c])
      continue;
    const int64_t cn = cmap[c];
    cb[cn] = s.cbound[c];
    cfl[cn] = s.cflags[c];
    CstRec r = s.cst[c];
    r.drem = r.duse = r.dcnt = 0;
    t.cst[cn] = r;
    t.cexp[cn] = s.cexp[c];
    t.key[cn] = s.key[c];
  }
}

// A continued solve's init (instead of mm_init_cnsts: remaining, usage, ratio, scales and keys are the handed-off
// state): no element votes yet, no change stamp, no touch; the frontier engine's 32-bit key from the ratio.
__global__ void __launch_bounds__(kBlock) mm_init_cont(Dev s) {
  int alive = 0;
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < s.nC; c += int64_t(gridDim.x) * kBlock) {
    const bool a = s.key[c] != kDeadKey;
    s.nvote[c] = int32_t(s.cnst_ptr[c + 1] - s.cnst_ptr[c]);
    s.chg[c] = uint16_t(0xFFFF);
    s.ctouch[c] = 0;
    if (s.key32)
      s.key32[c] = a ? ratio_key32(s.cst[c].ratio) : kDead32;
    alive += a;
  }
  alive = grp_isum<kWave>(alive);
  if ((threadIdx.x & (kWave - 1)) == 0 && alive)
    atomicAdd(&s.ctl[CTL_ALIVE_C], alive);
}

// The child's values back into the parent's variables; fixed ones get their round in the parent's numbering.
__global__ void __launch_bounds__(kBlock) tl_scatter(Dev s, Dev t, const int32_t* vmap, int32_t r0) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < t.nV; v += int64_t(gridDim.x) * kBlock) {
    const int32_t p = vmap[v];
    s.x[p] = t.x[v];
    const int32_t st = t.vstate[v];
    s.vstate[p] = st ? r0 + st : 0;
  }
}

}  // namespace lmmdev
