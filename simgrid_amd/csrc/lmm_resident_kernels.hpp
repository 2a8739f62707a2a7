// lmm_resident_kernels.hpp — device-resident System mirror and its delta log.
//
// The host System (lmm_system.cpp) keeps the reference's bookkeeping (maxmin.cpp:205-323, 703-888:
// expand / expand_add / variable_free / update_* and the concurrency staging).  Instead of flattening
// the active part of the system on the host before every solve (O(nnz) host work + a full PCIe upload),
// resident mode mirrors the host's element / variable / constraint records in HBM, ships only the
// records a mutation touched (the delta log: rs_apply_*), and rebuilds the solver's CSR / CSC on the
// device with the exact selection rules of System::flatten_maxmin (lmm_system.cpp, which follows
// lmm_solve's init, maxmin.cpp:509-540):
//   * a variable is a member iff it has an enabled element with w > 0 on a listed constraint (active
//     set, or the modified set in selective mode) with bound > bound * prec;
//   * listed constraint c, in list order, is flattened iff a member has an enabled element with w > 0
//     on it (whatever its bound: the solver's init applies the bound test, so a bound crossing it keeps
//     the structure unless it changes the member set -- rs_cross_check);
//   * a member's CSR row is its slab in slot order, keeping the elements with w > 0 on a flattened
//     constraint;
//   * every variable with an enabled element on a listed constraint has its value reset to 0;
//   * dense constraint ids follow the list order, dense variable ids ascending variable ids, and the
//     CSC lists a constraint's elements in CSR order (stable radix sort) — the very arrays the host
//     path uploads, so both paths give bit-identical solves (tests/test_gpu_resident.py).
// All kernels are element-wise / per-slab streams (HBM-bound, no atomics on the hot arrays except the
// per-constraint degree counts).
#pragma once

#include "lmm_dev.hpp"

namespace lmmdev {

// Resident mirror (host ids; capacities grow on demand, contents survive growth).
struct ResDev {
  int32_t* e_cnst;   // [capE] constraint of element slot e
  double* e_w;       // [capE] consumption weight
  uint8_t* e_fl;     // [capE] bit0: in its constraint's enabled list
  int64_t* v_ebase;  // [capV] first element slot of the variable's slab
  int32_t* v_n;      // [capV] elements in use; -1 = dead variable (lmm_system.cpp; loops `i < n` skip it, rs_apply_v validates it)
  double* v_pen;     // [capV] sharing penalty
  double* v_bound;   // [capV] bound (-1 = none)
  double* c_bound;   // [capC]
  uint8_t* c_fl;     // [capC] bit0: FATPIPE
};

constexpr uint8_t kResElemEnabled = 1;
constexpr uint8_t kResCnstFatpipe = 1;

constexpr int kRsU = 8;  // slab elements per unrolled step of the flatten passes (their gathers in flight)

__global__ void __launch_bounds__(kBlock)
    rs_apply_e(int64_t n, const int64_t* __restrict__ id, const int32_t* __restrict__ cn,
               const double* __restrict__ w, const uint8_t* __restrict__ fl, ResDev r) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int64_t e = id[i];
    r.e_cnst[e] = cn[i];
    r.e_w[e] = w[i];
    r.e_fl[e] = fl[i];
  }
}

// Structural-change flags of a delta batch (read by lmmhip_res_flatten's refresh path): bit0 = the
// system's structure may have changed (slab moved / resized, or more part-test crossings than the
// crossing list holds), bit1 = a penalty changed (per-element usage w/p is stale).  A constraint bound
// that crosses the "part" test at the last flatten's precision is appended to the crossing list
// instead (rs_apply_c): the flattened structure only changes when the crossing changes the member set,
// which rs_cross_check decides on the device.
constexpr int kResStruct = 1, kResPenalty = 2;
constexpr int kResCrossCap = 4096;  // crossing-list capacity (ids since the last flatten)

__global__ void __launch_bounds__(kBlock)
    rs_apply_v(int64_t n, const int32_t* __restrict__ id, const int64_t* __restrict__ eb,
               const int32_t* __restrict__ ne, const double* __restrict__ pen, const double* __restrict__ bnd,
               ResDev r, int32_t* dirty) {
  int f = 0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t v = id[i];
    if (r.v_ebase[v] != eb[i] || r.v_n[v] != ne[i])
      f |= kResStruct;
    if (r.v_pen[v] != pen[i])
      f |= kResPenalty;
    r.v_ebase[v] = eb[i];
    r.v_n[v] = ne[i];
    r.v_pen[v] = pen[i];
    r.v_bound[v] = bnd[i];
  }
  if (f)
    atomicOr(dirty, f);
}

__global__ void __launch_bounds__(kBlock)
    rs_apply_c(int64_t n, const int32_t* __restrict__ id, const double* __restrict__ b,
               const uint8_t* __restrict__ fl, ResDev r, double prec, int32_t* dirty, int32_t* xn, int32_t* xlist) {
  int f = 0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const double ob = r.c_bound[id[i]], nb = b[i];
    if ((ob > ob * prec) != (nb > nb * prec)) {
      const int32_t k = atomicAdd(xn, 1);
      if (k >= 0 && k < kResCrossCap)  // (k < 0: the count wrapped after 2^31 crossings without a flatten)
        xlist[k] = id[i];
      else
        f |= kResStruct;
    }
    r.c_bound[id[i]] = nb;
    r.c_fl[id[i]] = fl[i];
  }
  if (f)
    atomicOr(dirty, f);
}

// pos[c] = list position of listed constraint c (pos pre-set to -1); lpart[i] = bound > bound * prec
// (maxmin.cpp:523-525).  lany[i] (int64, scanned later) is cleared here.
// FairBottleneck (fair_bottleneck.cpp:29-50) lists every active constraint without a bound test; lzero
// (cleared here) then marks the ones with an enabled zero-weight element (cflags bit1).
__global__ void __launch_bounds__(kBlock)
    rs_pos(int64_t nl, const int32_t* __restrict__ list, ResDev r, double prec, int fair, int32_t* pos,
           uint8_t* lpart, int64_t* lany, uint8_t* lzero, uint8_t* cls) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i <= nl; i += int64_t(gridDim.x) * kBlock) {
    lany[i] = 0;
    if (i == nl)
      break;
    lzero[i] = 0;
    const int32_t c = list[i];
    pos[c] = int32_t(i);
    const double b = r.c_bound[c];
    lpart[i] = fair ? 1 : b > b * prec;
    if (cls)  // max-min: class of constraint c by id (0 = not listed, 1 = listed, 2 = listed and part)
      cls[c] = uint8_t(1 + lpart[i]);
  }
}

// Per variable slot: value reset (enabled element on a listed constraint, maxmin.cpp:509-514) and
// membership (such an element with w > 0 on a part constraint, :527-538).  Marks the constraints a
// member has an enabled element of w > 0 on, part or not (System::flatten_maxmin's superset rule:
// lanyc by constraint id, plain stores of 1: the race is benign; rs_lany_list puts them in list order),
// and, for a non-member, the listed constraints it has such an element on (outc: a bound of one of
// those crossing the part test would make it a member -- rs_cross_check).  One gather per element, of
// the 1-byte class cls[c] written by rs_pos; the second pass over the slab (a member's non-part or a
// non-member's listed constraints) only runs for the few slabs that have such an element.  The row
// length is the number of marked elements unless a member also has a disabled element of weight > 0
// (System::flatten_maxmin takes every element of a member whose constraint is marked, enabled or not):
// *mixed then asks rs_rowlen for the full count.
__global__ void __launch_bounds__(kBlock)
    rs_mark(int64_t nv, ResDev r, const uint8_t* __restrict__ cls, uint8_t* lanyc, uint8_t* outc, uint8_t* vrst,
            int64_t* vm, int64_t* rl, int32_t* mixed) {
  bool mix = false;
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v <= nv; v += int64_t(gridDim.x) * kBlock) {
    if (v == nv) {
      vm[v] = 0;  // scan sentinels
      rl[v] = 0;
      break;
    }
    uint8_t rst = 0;
    int64_t cnt = 0, cnt1 = 0;  // enabled w > 0 elements on part / on listed non-part constraints
    bool dis = false;
    const int64_t b = r.v_ebase[v];
    const int n = r.v_n[v];
    for (int i0 = 0; i0 < n; i0 += kRsU) {  // kRsU elements' loads in flight together
      int32_t p[kRsU];
      uint8_t fl[kRsU], k[kRsU];
      double w[kRsU];
#pragma unroll
      for (int u = 0; u < kRsU; u++) {
        p[u] = i0 + u < n ? r.e_cnst[b + i0 + u] : -1;
        fl[u] = i0 + u < n ? r.e_fl[b + i0 + u] : 0;
        w[u] = i0 + u < n ? r.e_w[b + i0 + u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kRsU; u++)
        if (!(fl[u] & kResElemEnabled)) {
          dis |= p[u] >= 0 && w[u] > 0;
          p[u] = -1;
        }
#pragma unroll
      for (int u = 0; u < kRsU; u++)
        k[u] = p[u] >= 0 ? cls[p[u]] : 0;
#pragma unroll
      for (int u = 0; u < kRsU; u++) {
        if (!k[u])
          continue;
        rst = 1;
        if (w[u] > 0) {
          if (k[u] == 2) {
            cnt++;
            lanyc[p[u]] = 1;
          } else {
            cnt1++;
          }
        }
      }
    }
    if (cnt1) {  // listed non-part constraints: in the flat when v is a member, else v is one of their outsiders
      uint8_t* mark = cnt ? lanyc : outc;
      for (int i = 0; i < n; i++) {
        const int32_t p = r.e_cnst[b + i];
        if ((r.e_fl[b + i] & kResElemEnabled) && r.e_w[b + i] > 0 && cls[p] == 1)
          mark[p] = 1;
      }
    }
    vrst[v] = rst;
    vm[v] = cnt > 0;
    rl[v] = cnt > 0 ? cnt + cnt1 : 0;
    mix |= cnt > 0 && dis;
  }
  if (mix)
    atomicOr(mixed, 1);
}

// lany[i] = lanyc[list[i]] (max-min: rs_mark marks by constraint id).
__global__ void __launch_bounds__(kBlock)
    rs_lany_list(int64_t nl, const int32_t* __restrict__ list, const uint8_t* __restrict__ lanyc, int64_t* lany) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nl; i += int64_t(gridDim.x) * kBlock)
    lany[i] = lanyc[list[i]];
}

// posd[c] = dense id of listed constraint c when it is marked (lany), else left at -1.
__global__ void __launch_bounds__(kBlock)
    rs_posd(int64_t nl, const int32_t* __restrict__ list, const int64_t* __restrict__ lany,
            const int64_t* __restrict__ dcl, int32_t* posd) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nl; i += int64_t(gridDim.x) * kBlock)
    if (lany[i])
      posd[list[i]] = int32_t(dcl[i]);
}

// Max-min row lengths when a member has a disabled element (*mixed, from rs_mark; otherwise nothing to do):
// elements with w > 0 on a marked constraint, in slot order, no enabled-list test (System::flatten_maxmin).
// The CSC offsets come from the sorted constraint ids (rs_cptr_sorted), not from degree atomics.
__global__ void __launch_bounds__(kBlock)
    rs_rowlen(int64_t nv, ResDev r, const int32_t* __restrict__ posd, const int64_t* __restrict__ vm, int64_t* rl,
              const int32_t* __restrict__ mixed) {
  if (!*mixed)
    return;
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nv; v += int64_t(gridDim.x) * kBlock) {
    int64_t cnt = 0;
    if (vm[v]) {
      const int64_t b = r.v_ebase[v];
      const int n = r.v_n[v];
      for (int i0 = 0; i0 < n; i0 += kRsU) {  // kRsU elements' loads in flight together
        int32_t p[kRsU];
#pragma unroll
        for (int u = 0; u < kRsU; u++)
          p[u] = i0 + u < n ? r.e_cnst[b + i0 + u] : -1;
#pragma unroll
        for (int u = 0; u < kRsU; u++)
          p[u] = p[u] >= 0 ? posd[p[u]] : -1;
#pragma unroll
        for (int u = 0; u < kRsU; u++)
          if (p[u] >= 0 && r.e_w[b + i0 + u] > 0)
            cnt++;
      }
    }
    rl[v] = cnt;
  }
}

// CSC offsets from the stably sorted dense constraint ids sk[0..nnz): element j starts constraint sk[j] and
// every empty one between it and the previous element's constraint; the last element closes the rest.
__global__ void __launch_bounds__(kBlock)
    rs_cptr_sorted(int64_t nnz, int64_t nc, const int32_t* __restrict__ sk, uint32_t* cptr) {
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < nnz; j += int64_t(gridDim.x) * kBlock) {
    const int64_t k = sk[j], prev = j == 0 ? -1 : sk[j - 1];
    for (int64_t c = prev + 1; c <= k; c++)
      cptr[c] = uint32_t(j);
    if (j == nnz - 1)
      for (int64_t c = k + 1; c <= nc; c++)
        cptr[c] = uint32_t(nnz);
  }
}

// FairBottleneck membership pass (System::flatten_fair, fair_bottleneck.cpp:29-50), per variable slot:
// every live variable is reset (vrst = 1), to 1.0 when it has a positive penalty and no non-zero weight
// (vrst = 3); constraints with an enabled element of weight > 0 are listed (lany), those with an
// enabled zero-weight one get the FATPIPE quirk flag (lzero); membership itself needs the final lany
// and is decided by rs_rowlen_fair.  A penalised variable with non-zero but no positive weight is the
// host's "negative consumption weights" error (*err).
__global__ void __launch_bounds__(kBlock)
    rs_mark_fair(int64_t nv, ResDev r, const int32_t* __restrict__ pos, int64_t* lany, uint8_t* lzero,
                 uint8_t* vrst, int64_t* vm, int32_t* err) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v <= nv; v += int64_t(gridDim.x) * kBlock) {
    if (v == nv) {
      vm[v] = 0;
      break;
    }
    const int n = r.v_n[v];
    const int64_t b = r.v_ebase[v];
    bool nz = false, posw = false;
    for (int i = 0; i < n; i++) {
      const double w = r.e_w[b + i];
      nz |= w != 0.0;
      posw |= w > 0.0;
      if (!(r.e_fl[b + i] & kResElemEnabled))
        continue;
      const int32_t p = pos[r.e_cnst[b + i]];
      if (p < 0)
        continue;
      if (w > 0)
        lany[p] = 1;
      else if (w == 0.0)
        lzero[p] = 1;
    }
    const bool pen = r.v_pen[v] > 0.0;
    vrst[v] = n < 0 ? 0 : (pen && !nz) ? 3 : 1;
    vm[v] = 0;
    if (n >= 0 && pen && nz && !posw)
      atomicOr(err, 1);
  }
}

// Row lengths + membership (live, penalty > 0, an element of weight > 0 on a listed constraint).
__global__ void __launch_bounds__(kBlock)
    rs_rowlen_fair(int64_t nv, ResDev r, const int32_t* __restrict__ pos, const int64_t* __restrict__ lany,
                   const int64_t* __restrict__ dcl, int64_t* vm, int64_t* rl, int64_t* cdeg) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v <= nv; v += int64_t(gridDim.x) * kBlock) {
    if (v == nv) {
      rl[v] = 0;
      break;
    }
    int64_t cnt = 0;
    if (r.v_pen[v] > 0.0) {
      const int64_t b = r.v_ebase[v];
      const int n = r.v_n[v];
      for (int i = 0; i < n; i++) {
        const int32_t p = pos[r.e_cnst[b + i]];
        if (p >= 0 && lany[p] && r.e_w[b + i] > 0) {
          cnt++;
          atomicAdd(reinterpret_cast<unsigned long long*>(cdeg + dcl[p]), 1ull);
        }
      }
    }
    rl[v] = cnt;
    vm[v] = cnt > 0;
  }
}

// Dense constraint records in list order (fair: cflags bit1 = enabled zero-weight element).
__global__ void __launch_bounds__(kBlock)
    rs_cmeta(int64_t nl, const int32_t* __restrict__ list, ResDev r, const int64_t* __restrict__ lany,
             const int64_t* __restrict__ dcl, const uint8_t* __restrict__ lzero, double* cbound, uint8_t* cflags) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nl; i += int64_t(gridDim.x) * kBlock) {
    if (!lany[i])
      continue;
    const int32_t c = list[i];
    cbound[dcl[i]] = r.c_bound[c];
    cflags[dcl[i]] = uint8_t(((r.c_fl[c] & kResCnstFatpipe) ? 1 : 0) | (lzero && lzero[i] ? 2 : 0));
  }
}

// FairBottleneck CSC chunks (lmm_fb_kernels.hpp): nck[j] chunks of kChunk elements per constraint.
__global__ void __launch_bounds__(kBlock)
    rs_nchunks(int64_t nc, const int64_t* __restrict__ cdeg, int chunk, int64_t* nck) {
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j <= nc; j += int64_t(gridDim.x) * kBlock)
    nck[j] = j < nc ? (cdeg[j] + chunk - 1) / chunk : 0;
}

__global__ void __launch_bounds__(kBlock)
    rs_chunks(int64_t nc, const int64_t* __restrict__ cptr, const int64_t* __restrict__ nck,
              const int64_t* __restrict__ cch, int chunk, int32_t* c_ch, int32_t* ch_cnst, uint32_t* ch_beg) {
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j <= nc; j += int64_t(gridDim.x) * kBlock) {
    c_ch[j] = int32_t(cch[j]);
    if (j == nc)
      break;
    for (int64_t k = 0; k < nck[j]; k++) {
      ch_cnst[cch[j] + k] = int32_t(j);
      ch_beg[cch[j] + k] = uint32_t(cptr[j] + k * chunk);
    }
  }
}

// Per dense row: its CSR range and penalty in one 16-B record, so that rs_csc reads them with ONE gather per
// element (the per-element usage, penalty and row of the CSC come out of the transpose itself).
struct alignas(16) RowPen {
  uint32_t rb, re;
  double pen;
};

// Per CSR element: its weight and dense row in one 16-B record, so that rs_csc gathers both with one load.
struct alignas(16) WRow {
  double w;
  int32_t v, pad;
};

// CSR rows, per-variable arrays and the dense -> slot map.
__global__ void __launch_bounds__(kBlock)
    rs_write(int64_t nv, ResDev r, const int32_t* __restrict__ posd, const int64_t* __restrict__ vm,
             const int64_t* __restrict__ dv, const int64_t* __restrict__ ro, uint32_t* var_ptr, int32_t* csr_c,
             double* csr_w, double* pen, double* vbound, int32_t* cvar0, WRow* wrow, int32_t* kidx,
             RowPen* rowpen) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nv; v += int64_t(gridDim.x) * kBlock) {
    if (!vm[v])
      continue;
    const int64_t i = dv[v];
    int64_t k = ro[v];
    var_ptr[i] = uint32_t(k);
    pen[i] = r.v_pen[v];
    vbound[i] = r.v_bound[v];
    cvar0[i] = int32_t(i);
    const int64_t b = r.v_ebase[v];
    const int n = r.v_n[v];
    for (int j0 = 0; j0 < n; j0 += kRsU) {  // kRsU elements' loads in flight together, slab order kept
      int32_t p[kRsU];
      double w[kRsU];
#pragma unroll
      for (int u = 0; u < kRsU; u++) {
        p[u] = j0 + u < n ? r.e_cnst[b + j0 + u] : -1;
        w[u] = j0 + u < n ? r.e_w[b + j0 + u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kRsU; u++)
        p[u] = p[u] >= 0 && w[u] > 0 ? posd[p[u]] : -1;
#pragma unroll
      for (int u = 0; u < kRsU; u++)
        if (p[u] >= 0) {
          csr_c[k] = p[u];
          csr_w[k] = w[u];
          wrow[k] = WRow{w[u], int32_t(i), 0};
          kidx[k] = int32_t(k);
          k++;
        }
    }
    rowpen[i] = RowPen{uint32_t(ro[v]), uint32_t(k), r.v_pen[v]};
  }
}

// Refresh path (no structural change since the last flatten): the dense per-variable arrays only.
__global__ void __launch_bounds__(kBlock)
    rs_refresh_v(int64_t nv, ResDev r, const int64_t* __restrict__ vm, const int64_t* __restrict__ dv, double* pen,
                 double* vbound) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nv; v += int64_t(gridDim.x) * kBlock) {
    if (!vm[v])
      continue;
    pen[dv[v]] = r.v_pen[v];
    vbound[dv[v]] = r.v_bound[v];
  }
}

// Refresh path with part-test crossings (rs_apply_c's list, after rs_cmeta rewrote the dense bounds): does
// a crossing change the member set?  One workgroup per crossing constraint c (block-uniform branches):
//   * c not listed at the last flatten (cls 0): its bound plays no part;
//   * c passes the part test now: a non-member with an enabled element of w > 0 on c (outc, rs_mark) would
//     become a member -> structural;
//   * c fails it now: each member on c (its CSC column) must keep an element on a constraint that still
//     passes it, else it leaves the member set -> structural.  The dense rows are the members' enabled
//     elements of w > 0 on flattened constraints (the host skips this check when a member also has a
//     disabled one, rs_mark's *mixed), and the dense bounds are current, so several crossings since the
//     last flatten are judged together.
// Otherwise the member set, hence the flattened constraints (listed ones a member has such an element on)
// and the rows, are what a full flatten would build, and only the bounds changed.
__global__ void __launch_bounds__(kBlock)
    rs_cross_check(int32_t nx, const int32_t* __restrict__ xlist, ResDev r, double prec,
                   const uint8_t* __restrict__ cls, const uint8_t* __restrict__ outc, const int32_t* __restrict__ posd,
                   const uint32_t* __restrict__ cnst_ptr, const int32_t* __restrict__ csc_v,
                   const uint32_t* __restrict__ var_ptr, const int32_t* __restrict__ csr_c,
                   const double* __restrict__ cbound, int32_t* dirty) {
  for (int32_t i = blockIdx.x; i < nx; i += gridDim.x) {
    const int32_t c = xlist[i];
    if (cls[c] == 0)
      continue;
    const double b = r.c_bound[c];
    if (b > b * prec) {
      if (threadIdx.x == 0 && outc[c])
        atomicOr(dirty, kResStruct);
      continue;
    }
    const int32_t dc = posd[c];
    if (dc < 0)
      continue;
    bool lost = false;
    for (uint32_t j = cnst_ptr[dc] + threadIdx.x; j < cnst_ptr[dc + 1]; j += kBlock) {
      const int32_t v = csc_v[j];
      bool keep = false;
      for (uint32_t k = var_ptr[v]; k < var_ptr[v + 1] && !keep; k++) {
        const double cb = cbound[csr_c[k]];
        keep = cb > cb * prec;
      }
      lost |= !keep;
    }
    if (lost)
      atomicOr(dirty, kResStruct);
  }
}

// The CSC in CSR order (the sort's values sk), plus what mm_elem_usage would gather per element afterwards:
// usage w / penalty, the penalty and the variable's CSR row (the same division: identical bits).
__global__ void __launch_bounds__(kBlock)
    rs_csc(int64_t nnz, const int32_t* __restrict__ sk, const WRow* __restrict__ wrow,
           const RowPen* __restrict__ rowpen, int32_t* csc_v, double* csc_w, double* csc_u, double* csc_p,
           unsigned long long* csc_row, int32_t* c2c) {
  // kCscU elements per thread per step, their two dependent gathers (record, then row) in flight together
  constexpr int kCscU = 4;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t j0 = int64_t(blockIdx.x) * kBlock + threadIdx.x; j0 < nnz; j0 += kCscU * stride) {
    int32_t k[kCscU];
    WRow e[kCscU];
    RowPen rp[kCscU];
#pragma unroll
    for (int u = 0; u < kCscU; u++)
      k[u] = j0 + u * stride < nnz ? sk[j0 + u * stride] : -1;
#pragma unroll
    for (int u = 0; u < kCscU; u++)
      e[u] = k[u] >= 0 ? wrow[k[u]] : WRow{0.0, -1, 0};
#pragma unroll
    for (int u = 0; u < kCscU; u++)
      rp[u] = e[u].v >= 0 ? rowpen[e[u].v] : RowPen{0, 0, 1.0};
#pragma unroll
    for (int u = 0; u < kCscU; u++) {
      const int64_t j = j0 + u * stride;
      if (j >= nnz)
        break;
      csc_v[j] = e[u].v;
      csc_w[j] = e[u].w;
      csc_u[j] = e[u].w / rp[u].pen;
      csc_p[j] = rp[u].pen;
      csc_row[j] = (unsigned long long)rp[u].rb | ((unsigned long long)rp[u].re << 32);
      if (c2c)  // the inverse map, CSR element -> CSC position (the refresh path's per-variable updates)
        c2c[k[u]] = int32_t(j);
    }
  }
}

// Refresh path with a list of the variables the delta batches since the last flatten touched (lmmhip_res_apply):
// their dense penalty and bound, and — penalties moved — the usage w / penalty and penalty of each of their CSC
// elements, through the CSR -> CSC map rs_csc kept (the same division as mm_elem_usage: identical bits).  Work
// proportional to the changed variables instead of to the whole system.
__global__ void __launch_bounds__(kBlock)
    rs_refresh_vl(int64_t n, const int32_t* __restrict__ list, ResDev r, const int64_t* __restrict__ vm,
                  const int64_t* __restrict__ dv, double* pen, double* vbound, const uint32_t* __restrict__ var_ptr,
                  const int32_t* __restrict__ c2c, const double* __restrict__ csc_w, double* csc_u, double* csc_p,
                  int usage) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t v = list[i];
    if (!vm[v])
      continue;
    const int64_t d = dv[v];
    const double p = r.v_pen[v];
    pen[d] = p;
    vbound[d] = r.v_bound[v];
    if (!usage)
      continue;
    for (uint32_t k = var_ptr[d]; k < var_ptr[d + 1]; k++) {
      const int32_t j = c2c[k];
      csc_u[j] = csc_w[j] / p;
      csc_p[j] = p;
    }
  }
}

__global__ void __launch_bounds__(kBlock) rs_ptr32(int64_t n, const int64_t* __restrict__ in, uint32_t* out) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i <= n; i += int64_t(gridDim.x) * kBlock)
    out[i] = uint32_t(in[i]);
}

// The sliced fetch (lmmhip_res_values_sliced): ONE array, per variable slot the value the host writes back (as
// rs_values: the solved value of a member, 1.0 / 0 for a reset non-member) and, for the slots the host must leave
// alone (vrst 0), kValKeep — a signalling-NaN payload no arithmetic produces — instead of a separate flag array.
__global__ void __launch_bounds__(kBlock)
    rs_values_mark(int64_t nv, const int64_t* __restrict__ vm, const int64_t* __restrict__ dv,
                   const uint8_t* __restrict__ vrst, const double* __restrict__ x, unsigned long long* out) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nv; v += int64_t(gridDim.x) * kBlock) {
    const uint8_t r = vrst[v];
    const double val = vm[v] ? x[dv[v]] : r == 3 ? 1.0 : 0.0;
    out[v] = r ? (unsigned long long)__double_as_longlong(val) : kValKeep;
  }
}

// Per variable slot after the solve: the solved value of a member, 0 for the others (only slots with
// vrst set are written back by the host); rst_out (optional) receives a copy of the reset flags.
__global__ void __launch_bounds__(kBlock)
    rs_values(int64_t nv, const int64_t* __restrict__ vm, const int64_t* __restrict__ dv,
              const uint8_t* __restrict__ vrst, const double* __restrict__ x, double* out, uint8_t* rst_out) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nv; v += int64_t(gridDim.x) * kBlock) {
    const uint8_t r = vrst[v];
    out[v] = vm[v] ? x[dv[v]] : r == 3 ? 1.0 : 0.0;
    if (rst_out)
      rst_out[v] = r;
  }
}

}  // namespace lmmdev
