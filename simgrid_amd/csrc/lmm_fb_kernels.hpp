// lmm_fb_kernels.hpp — FairBottleneck::bottleneck_solve on gfx950 (included by lmm_hip.hip).
//
// One reference round (fair_bottleneck.cpp:59-145) is Jacobi-style: every constraint's share is
// computed before any variable moves, every variable's increment before any constraint is updated.
// The device round is the same phases:
//   phase 0  fb_pack_vst, fbk_count, fbk_nb   listed-variable count per constraint -> xnb
//   phase 1  fbk_share, fb_var_inc            shares, increments mu
//            fbk_acc, fbk_accc                (one context) increments w*mu in CSC order, FATPIPE minima
//   phase 2  fbk_update_seq, fbk_unlist       remaining (the reference's element-by-element chain), erasure,
//                                             delisting
// A variable-sharded solve (multi.py) runs the same kernels for its variables plus the constraint-owner
// kernels below (fbo_*), with the exchanges between the phases described there.
// Element work is cut into CSC chunks of at most kFbChunk elements (one wave each), so a constraint
// with 10^6 elements (a CPU under thousands of flows, C5) spreads over the chip instead of
// serialising one wave; per-chunk partials are combined per constraint in chunk order, so every
// reduction is deterministic.
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

constexpr int kFbChunk = 1024;

__global__ void __launch_bounds__(kBlock) fb_init(Dev s) {
  const int64_t n = s.nV > s.nC ? s.nV : s.nC;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    if (i < s.nV) {  // fair_bottleneck.cpp:29-41 (only listed variables are flattened)
      s.x[i] = 0.0;
      s.vtmp[i] = 0.0;
      if (s.mu_p)
        s.mu_p[i] = 0.0;
      s.vst[i] = 1;
      s.fixr[i] = -1;
    }
    if (i < s.nC) {  // :44-50
      s.rem[i] = s.cbound[i];
      s.use[i] = 0.0;
      s.ratio[i] = 0.0;  // 0 = in the constraint list, +inf = erased
      s.erased[i] = 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_ANY0] = s.nV > 0;
}

__device__ __forceinline__ uint32_t chunk_end(const Dev& s, int q, int c) {
  const uint32_t e = s.ch_beg[q] + kFbChunk, ce = s.cnst_ptr[c + 1];
  return e < ce ? e : ce;
}

// The listed flags packed 32 per word (vstb) before the count: its gathers then hit a table of nV / 8 bytes
// (1.25 MB at C5's 10^7 flows: resident in every XCD's L2) instead of the nV-byte flags.
__global__ void __launch_bounds__(kBlock) fb_pack_vst(Dev s) {
  if (s.ctl[CTL_DONE])
    return;
  const int64_t nw = (int64_t(s.nV) + 31) / 32;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nw; i += int64_t(gridDim.x) * kBlock) {
    uint32_t m = 0;
    const int64_t v0 = i * 32;
    if (v0 + 32 <= s.nV) {
      const uint4 a = reinterpret_cast<const uint4*>(s.vst + v0)[0], b = reinterpret_cast<const uint4*>(s.vst + v0)[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < 32; k++)
        m |= uint32_t(((w[k >> 2] >> (8 * (k & 3))) & 0xFF) != 0) << k;
    } else {
      for (int k = 0; v0 + k < s.nV; k++)
        m |= uint32_t(s.vst[v0 + k] != 0) << k;
    }
    s.vstb[i] = m;
  }
}

// :67-74 — listed variables (w > 0: every flattened element) of each chunk of a listed constraint.  all = 1
// (round 0: fair_bottleneck.cpp:29-41 lists every flattened variable): the chunk's length, nothing gathered.
__global__ void __launch_bounds__(kBlock) fbk_count(Dev s, int all) {
  if (s.ctl[CTL_DONE])
    return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int q = blockIdx.x * wpb + threadIdx.x / kWave; q < s.nch; q += gridDim.x * wpb) {
    const int c = s.ch_cnst[q];
    int nb = 0;
    if (all) {
      if (lane == 0)
        s.pcnt[q] = int(chunk_end(s, q, c) - s.ch_beg[q]);
      continue;
    }
    if (s.ratio[c] == 0.0) {
      const uint32_t e = chunk_end(s, q, c);
      for (uint32_t j0 = s.ch_beg[q] + lane; j0 < e; j0 += 4 * kWave) {  // 4 gathers in flight per lane
        int32_t vv[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
          vv[k] = j0 + k * kWave < e ? s.csc_v[j0 + k * kWave] : -1;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (vv[k] >= 0)
            nb += (s.vstb[vv[k] >> 5] >> (vv[k] & 31)) & 1;
      }
    }
    nb = grp_isum<kWave>(nb);
    if (lane == 0)
      s.pcnt[q] = nb;
  }
}

// per constraint: chunk counts -> xnb[c]; xnb[nC] = "a variable of this shard is still listed"
__global__ void __launch_bounds__(kBlock) fbk_nb(Dev s, int par) {
  if (s.ctl[CTL_DONE])
    return;
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < s.nC; c += gridDim.x * kBlock) {
    int nb = 0;
    for (int q = s.c_ch[c]; q < s.c_ch[c + 1]; q++)
      nb += s.pcnt[q];
    s.xnb[c] = nb;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.xnb[s.nC] = s.ctl[CTL_ANY0 + par];
}

// Per-wave sum of work counter k into one of its kFbwSlots slots (one atomic per wave, the waves spread over the slots;
// lmmhip_fb_work sums them).
__device__ __forceinline__ void fb_work_add(const Dev& s, int k, unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v += __shfl_xor(v, o, kWave);
  const int slot = int((blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave) & (kFbwSlots - 1));
  if ((threadIdx.x & (kWave - 1)) == 0 && v)
    atomicAdd(reinterpret_cast<unsigned long long*>(s.ctl + CTL_FBW_AT) + k * kFbwSlots + slot, v);
}

// :65-87 — usage = remaining / nb (FATPIPE: nb -> 1); nb == 0 erases the constraint.  xnb holds the
// counts of every shard; xnb[nC] == 0 means no variable is listed anywhere: the solve is over (:145).
__global__ void __launch_bounds__(kBlock) fbk_share(Dev s, int par) {
  if (s.ctl[CTL_DONE])
    return;
  if (s.xnb[s.nC] == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      s.ctl[CTL_DONE] = 1;
      if (s.hprog)  // the host's pacing words (solve_fair_rounds)
        __hip_atomic_store(s.hprog + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.ctl[CTL_ANY0 + (par ^ 1)] = 0;
    s.ctl[CTL_ROUNDS] += 1;
    if (s.hprog)
      __hip_atomic_store(s.hprog, s.ctl[CTL_ROUNDS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  unsigned long long ne = 0, nc = 0;  // this round's listed constraints and their elements (measurement)
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < s.nC; c += gridDim.x * kBlock) {
    if (s.ratio[c] != 0.0)
      continue;
    ne += s.cnst_ptr[c + 1] - s.cnst_ptr[c];
    nc += 1;
    int nb = s.xnb[c];
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
  fb_work_add(s, 0, ne);
  fb_work_add(s, 2, nc);
}

// :89-105 — per listed variable: mu = min(usage/w, bound - value); value += mu; exact
// `value == bound` drops it from the list.
// :89-105 once the minimum of usage / w over the row is known: bound, value, exact `value == bound` delisting.
__device__ __forceinline__ int var_inc_finish(const Dev& s, int64_t v, double inc, int round) {
  const double vb = s.vbound[v];
  double x = s.x[v];
  if (vb > 0)
    inc = fmin(inc, vb - x);
  s.vtmp[v] = inc;
  if (s.mu_p)
    s.mu_p[s.vperm[v]] = inc;  // (one scattered store per listed variable: the chains then gather with locality)
  x += inc;
  s.x[v] = x;
  s.fixr[v] = round;  // last round in which v was listed
  if (x == vb) {
    s.vst[v] = 0;
    return 0;
  }
  return 1;
}

// Wave-cooperative (waves with at least 16 listed rows): a wave takes 64 consecutive variables, whose rows are one contiguous CSR range; the lanes
// read that range coalesced (the u-th element of 64 rows per load touched ~64 lines) and min-reduce each
// element's usage / w into its row's slot in LDS (64-bit atomic min of the non-negative doubles' bits: the
// same minimum as a sequential fmin).
__global__ void __launch_bounds__(kBlock) fb_var_inc(Dev s, int par, int round) {
  if (s.ctl[CTL_DONE])
    return;
  __shared__ unsigned long long mn[kBlock];
  __shared__ uint32_t rb[kBlock];
  __shared__ uint8_t rl[kBlock];
  const int lane = threadIdx.x & (kWave - 1);
  unsigned long long* wmn = mn + (threadIdx.x - lane);
  uint32_t* wrb = rb + (threadIdx.x - lane);
  uint8_t* wrl = rl + (threadIdx.x - lane);
  const unsigned long long kMaxBits = (unsigned long long)__double_as_longlong(DBL_MAX);
  int any = 0;
  unsigned long long nvl = 0;  // listed variables seen by this lane (measurement)
  for (int64_t base = int64_t(blockIdx.x) * kBlock + (threadIdx.x - lane); base < s.nV;
       base += int64_t(gridDim.x) * kBlock) {  // wave-uniform
    const int64_t v = base + lane;
    const bool in = v < s.nV;
    const bool listed = in && s.vst[v];
    const uint32_t b = in ? s.var_ptr[v] : 0u, e = in ? s.var_ptr[v + 1] : 0u;
    const int nlisted = __popcll(__ballot(listed));
    nvl += listed;
    if (nlisted == 0)
      continue;
    if (nlisted < kWave / 4) {  // few listed rows (late rounds): each listed lane reads its own row
      if (!listed)
        continue;
      double inc = DBL_MAX;
      for (uint32_t j0 = b; j0 < e; j0 += 4) {  // 4 elements' loads in flight together
        int32_t cc[4];
        double ww[4], uu[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          cc[k] = j0 + k < e ? s.csr_c[j0 + k] : -1;
          ww[k] = j0 + k < e ? s.csr_w[j0 + k] : 1.0;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          uu[k] = cc[k] >= 0 ? s.use[cc[k]] : 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (cc[k] >= 0)
            inc = fmin(inc, uu[k] / ww[k] + 0.0);
      }
      any |= var_inc_finish(s, v, inc, round);
      continue;
    }
    const int last = int(s.nV - 1 - base < kWave - 1 ? s.nV - 1 - base : kWave - 1);
    const uint32_t B = __shfl(b, 0, kWave), E = __shfl(e, last, kWave);
    wmn[lane] = kMaxBits;
    wrb[lane] = in ? b : 0xFFFFFFFFu;  // (lanes past nV never own an element)
    wrl[lane] = listed;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t f0 = B; f0 < E; f0 += 2 * kWave) {  // wave-uniform, 2 loads per array in flight
      int32_t cc[2];
      double ww[2], uu[2];
      int ow[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const uint32_t f = f0 + u * kWave + lane;
        cc[u] = f < E ? s.csr_c[f] : -1;
        ww[u] = f < E ? s.csr_w[f] : 1.0;
        int o = 0;  // owner: the last lane whose row starts at or before f
#pragma unroll
        for (int st = kWave / 2; st > 0; st >>= 1)
          if (wrb[o + st] <= f)
            o += st;
        ow[u] = o;
        if (cc[u] >= 0 && !wrl[o])
          cc[u] = -1;
      }
#pragma unroll
      for (int u = 0; u < 2; u++)
        uu[u] = cc[u] >= 0 ? s.use[cc[u]] : 0.0;
#pragma unroll
      for (int u = 0; u < 2; u++)
        if (cc[u] >= 0)
          atomicMin(&wmn[ow[u]], (unsigned long long)__double_as_longlong(uu[u] / ww[u] + 0.0));
    }
    __builtin_amdgcn_wave_barrier();
    if (listed)
      any |= var_inc_finish(s, v, __longlong_as_double((long long)wmn[lane]), round);
    __builtin_amdgcn_wave_barrier();
  }
  if (__syncthreads_or(any) && threadIdx.x == 0)  // (one store per workgroup on the flag word, not one per wave)
    s.ctl[CTL_ANY0 + (par ^ 1)] = 1;
  fb_work_add(s, 1, nvl);
}

// mu of CSC element j (variable v): from the locality-ordered copy when there is one (fb_perm).
__device__ __forceinline__ double fb_mu(const Dev& s, uint32_t j, int32_t v) {
  return s.mu_p ? s.mu_p[s.csc_vp[j]] : s.vtmp[v];
}

// Locality order of the mu gathers (one context, once per upload): a flow's elements sit on its route's links,
// so sorting the variables by their row's first and last constraint (source-side and destination-side links)
// puts the flows a link carries in few runs; the chains, which must visit a link's elements in the reference's
// order, then gather mu from a few regions instead of one line per element.  Values never move: only the
// copy of mu the chains read (mu_p) and the element -> position map (csc_vp) use the order.
__global__ void __launch_bounds__(kBlock) fbp_keys(Dev s, unsigned long long* key, int32_t* val) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock) {
    const uint32_t b = s.var_ptr[v], e = s.var_ptr[v + 1];
    key[v] = b < e ? (unsigned long long)uint32_t(s.csr_c[b]) * uint64_t(s.nC) + uint32_t(s.csr_c[e - 1])
                   : ~0ull;
    val[v] = int32_t(v);
  }
}
__global__ void __launch_bounds__(kBlock) fbp_inv(Dev s, const int32_t* order) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < s.nV; i += int64_t(gridDim.x) * kBlock)
    s.vperm[order[i]] = int32_t(i);
}
__global__ void __launch_bounds__(kBlock) fbp_csc(Dev s) {
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < s.nnz; j += int64_t(gridDim.x) * kBlock)
    s.csc_vp[j] = s.vperm[s.csc_v[j]];
}

// :107-127 — per chunk of a listed constraint.  FATPIPE: min of w*mu over ALL its elements (the stale mu of
// variables that already left the list included) -> pacc.  Shared: the increments w * mu in CSC order into
// fbd (element-parallel, all gathers of the round spread over the chip), which fbk_update_seq then chains
// one at a time; only the elements of variables listed this round are rewritten: a delisted variable's mu
// (vtmp) no longer moves, so its increment written in its last listed round still holds (every variable is
// listed in round 0, a listed constraint was listed in every earlier round); vstb = the flags before
// fb_var_inc.
// Shared constraints shorter than `longmin` elements take their increments in fbk_update_seq itself (fb_chain_pull);
// only the long ones, whose chains are the round's critical path, get them precomputed here.
__global__ void __launch_bounds__(kBlock) fbk_acc(Dev s, int all, uint32_t longmin) {  // all: round 0, every variable listed
  if (s.ctl[CTL_DONE])
    return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int q = blockIdx.x * wpb + threadIdx.x / kWave; q < s.nch; q += gridDim.x * wpb) {
    const int c = s.ch_cnst[q];
    const bool fat = s.cflags[c] & 1;
    if (s.ratio[c] != 0.0)
      continue;
    if (!fat && s.cnst_ptr[c + 1] - s.cnst_ptr[c] < longmin)
      continue;
    if (!fat) {
      const uint32_t e = chunk_end(s, q, c);
      for (uint32_t j0 = s.ch_beg[q] + lane; j0 < e; j0 += 4 * kWave) {  // 4 gathers in flight per lane
        int32_t vv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t j = j0 + k * kWave;
          vv[k] = j < e ? s.csc_v[j] : -1;
        }
        if (!all) {
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (vv[k] >= 0 && !((s.vstb[vv[k] >> 5] >> (vv[k] & 31)) & 1))
              vv[k] = -1;
        }
        double dv[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
          dv[k] = vv[k] >= 0 ? s.csc_w[j0 + k * kWave] * fb_mu(s, j0 + k * kWave, vv[k]) : 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (vv[k] >= 0)
            s.fbd[j0 + k * kWave] = dv[k];
      }
      continue;
    }
    double acc = dinf();
    for (uint32_t j = s.ch_beg[q] + lane, e = chunk_end(s, q, c); j < e; j += kWave)
      acc = fmin(acc, s.csc_w[j] * fb_mu(s, j, s.csc_v[j]));
    acc = wave_min(acc);
    if (lane == 0)
      s.pacc[q] = acc;
  }
}

// per FATPIPE constraint: chunk minima in chunk order -> xmin
__global__ void __launch_bounds__(kBlock) fbk_accc(Dev s) {
  if (s.ctl[CTL_DONE])
    return;
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < s.nC; c += gridDim.x * kBlock) {
    double mn = dinf();
    if (s.ratio[c] == 0.0 && (s.cflags[c] & 1))
      for (int q = s.c_ch[c]; q < s.c_ch[c + 1]; q++)
        mn = fmin(mn, s.pacc[q]);
    s.xmin[c] = mn;
  }
}

// :118-125 — FATPIPE: usage = min(usage, w * mu over the enabled elements) (an enabled zero-weight element,
// cflags bit1, gives 0), remaining -= usage, clamped (double_update, surf_interface.hpp:34-44)
__device__ __forceinline__ double fb_fat_update(const Dev& s, int64_t c, double rem, double elem_min, double prec,
                                                double* use_out) {
  double u = s.use[c];
  if (s.cflags[c] & 2)
    u = fmin(u, 0.0);
  u = fmin(u, elem_min);
  *use_out = u;
  rem -= u;
  if (rem < prec)
    rem = 0.0;
  return rem;
}

// :110-116 — a shared constraint's remaining takes its elements' increments w * mu ONE AT A TIME in the
// CSC order (fbd[cb..ce)), each step a double_update (surf_interface.hpp:34-44) — the reference's own loop
// operation for operation, so with the CSC in enabled_element_set_ order the result is bit-identical.  Not
// an order-free sum: the saturating constraint's remaining ends a few ulps of its bound away from 0, and
// whether that residue is below the precision (erasure, :129) depends on the rounding of this exact chain —
// a tree sum is more accurate and erases constraints the reference keeps (C5 at 1e6 flows: 28 of them in
// round 0, a different fixed point for 12 % of the flows).  Called by a whole wave; the result is lane 0's.
//
// The chain is the critical path (C5's global dragonfly links hold ~1.6e5 elements), so it is fed without
// waiting: the lanes stream kSeqP x 64 increments into LDS (`d`, kSeqP * 64 doubles of this wave) and issue
// the loads of the next kSeqP x 64 before lane 0 chains the current ones.  And when every increment of a
// batch is >= 0 the clamp is taken once at its end: fl(r - d) <= r for d >= 0, so the unclamped remaining
// only decreases; the clamped chain equals it until its first value below the precision and is 0 from there
// on (0 - d < precision), i.e. the clamped result is 0 exactly when the unclamped end value is below the
// precision, and that end value otherwise.  A batch holding a negative (or NaN) increment takes the clamp
// at every step.
constexpr int kSeqP = 8;  // 64-element blocks per batch

// Lane 0: the n increments of one batch (d, in LDS) chained into rem, one double_update per element — the
// reference's loop; a batch of non-negative increments takes the clamp once at its end (same value, see above).
// (The wave-parallel fb_chain_scan below takes non-negative batches; this loop is its fallback.)
__device__ __forceinline__ double fb_chain_batch(const double* d, int n, double rem, double prec, bool nonneg) {
  if (nonneg) {
    for (int k = 0; k < n; k++)
      rem -= d[k];
    if (rem < prec)
      rem = 0.0;
  } else {
    for (int k = 0; k < n; k++) {
      rem -= d[k];
      if (rem < prec)
        rem = 0.0;
    }
  }
  return rem;
}

// The same non-negative batch chained by the whole wave, exactly.  While the running value x stays in one
// binade [2^e, 2^(e+1)) its grid is u = 2^(e-52) and x is a multiple of u, so fl(x - d) = x - u * rint(d / u)
// unless d / u is a tie (xx.5: the result's parity would decide) or the result leaves the binade: the chain is
// then x - u * (a prefix sum of integers), and the wave finds the first step that leaves the binade (prefix >= M
// = (x - 2^e) / u: the result could round onto the coarser grid below) or is a tie with one int64 scan, takes
// that step as the fp64 subtraction it is, and goes on from there.  Once x < prec the clamped chain is 0 (the
// values only decrease).  Identical, bit for bit, to lane 0's sequential loop; after kScanExits such steps in a
// batch (the value falls through binades element by element near the end of a saturating chain) the rest goes
// back to that loop: *k = the first increment not yet applied.  Needs prec > 0 and every d >= 0.
constexpr int kScanExits = 12;
__device__ __forceinline__ double fb_chain_scan(const double* d, int n, double x, double prec, int lane, int* k_out) {
  constexpr int kPer = kSeqP;  // increments per lane: lane l holds [l * kPer, (l + 1) * kPer)
  double dv[kPer];
  const double2* d2 = reinterpret_cast<const double2*>(d + lane * kPer);
#pragma unroll
  for (int t = 0; t < kPer / 2; t++) {
    const double2 v = d2[t];
    dv[2 * t] = v.x;
    dv[2 * t + 1] = v.y;
  }
  int k = 0, exits = 0;
  while (k < n) {  // wave-uniform (x, k identical on every lane)
    if (!(x >= prec)) {  // every later value is below the precision too: the clamped chain is 0
      k = n;
      x = 0.0;
      break;
    }
    if (x < 0x1p-1022 || exits >= kScanExits)  // subnormal grid / many binade steps: lane 0's loop
      break;
    const int e = __builtin_amdgcn_frexp_exp(x) - 1;  // x in [2^e, 2^(e+1))
    const long long M = (long long)(__builtin_amdgcn_ldexp(x, 52 - e) - 0x1p52);  // (x - 2^e) / u, exact
    long long run = 0, incl[kPer];
    bool tie[kPer];
#pragma unroll
    for (int t = 0; t < kPer; t++) {
      const int j = lane * kPer + t;
      long long q = 0;
      tie[t] = false;
      if (j >= k && j < n) {
        const double sc = __builtin_amdgcn_ldexp(dv[t], 52 - e);  // d / u, exact
        if (!(sc < 0x1p52)) {
          q = 1ll << 52;  // > M: leaves the binade
        } else {
          const double f = __builtin_floor(sc), fr = sc - f;
          tie[t] = fr == 0.5;
          q = (long long)f + (fr > 0.5 ? 1 : 0);
        }
      }
      run += q;
      incl[t] = run;
    }
    long long ex = run;  // exclusive wave scan of the lane totals
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const long long y = __shfl_up(ex, o, kWave);
      if (lane >= o)
        ex += y;
    }
    ex -= run;
    int first = -1;
    long long before = 0;
#pragma unroll
    for (int t = kPer - 1; t >= 0; t--) {  // this lane's first step that must be taken in fp64
      const int j = lane * kPer + t;
      if (j >= k && j < n && (tie[t] || ex + incl[t] >= M)) {
        first = j;
        before = ex + (t ? incl[t - 1] : 0);
      }
    }
    const unsigned long long m = __ballot(first >= 0);
    const double u = __builtin_amdgcn_ldexp(1.0, e - 52);
    if (!m) {  // the whole rest stays in the binade
      const long long tot = __shfl(ex + run, kWave - 1, kWave);
      x -= double(tot) * u;  // exact: a multiple of u in [2^e + u, 2^(e+1))
      k = n;
      break;
    }
    const int src = __ffsll((long long)m) - 1;
    const int js = __shfl(first, src, kWave);
    const long long pb = __shfl(before, src, kWave);
    x -= double(pb) * u;  // exact (pb < M)
    x -= d[js];           // the step itself, as the sequential loop takes it
    k = js + 1;
    exits++;
  }
  if (k >= n && x < prec)  // the batch's end clamp
    x = 0.0;
  *k_out = k;
  return x;
}

// One batch of the chain (d: this wave's LDS slots; the result is on every lane).
__device__ __forceinline__ double fb_chain_step(const double* d, int n, double rem, double prec, bool nonneg,
                                                int lane) {
  int k = 0;
  if (nonneg && prec > 0.0)
    rem = fb_chain_scan(d, n, rem, prec, lane, &k);
  // (after a partial scan: one clamp per step — the same value for non-negative increments, and it reads exactly
  // the n - k slots left, where the batched loop reads whole groups from an aligned start)
  if (k < n && lane == 0)
    rem = fb_chain_batch(d + k, n - k, rem, prec, nonneg && k == 0);
  rem = __shfl(rem, 0, kWave);
  __builtin_amdgcn_wave_barrier();
  return rem;
}

// The increments stream in kChainD batches ahead of the chain (kChainD x kSeqP doubles per lane in flight): with
// the batch itself chained wave-parallel (fb_chain_scan), the memory latency per batch is what is left to hide.
constexpr int kChainD = 4;
__device__ __forceinline__ double fb_chain(const double* __restrict__ fbd, uint32_t cb, uint32_t ce, double rem,
                                           double prec, double* d, int lane) {
  constexpr uint32_t kB = kSeqP * kWave;
  double nx[kChainD][kSeqP];
#pragma unroll
  for (int t = 0; t < kChainD; t++)
#pragma unroll
    for (int p = 0; p < kSeqP; p++) {
      const uint32_t j = cb + t * kB + p * kWave + lane;
      nx[t][p] = j < ce ? fbd[j] : 0.0;
    }
  for (uint32_t base = cb; base < ce; base += kChainD * kB) {  // wave-uniform
#pragma unroll
    for (int t = 0; t < kChainD; t++) {
      const uint32_t b0 = base + t * kB;
      if (b0 >= ce)  // wave-uniform
        break;
      bool nonneg = true;
#pragma unroll
      for (int p = 0; p < kSeqP; p++) {
        d[p * kWave + lane] = nx[t][p];
        nonneg &= nx[t][p] >= 0.0;
      }
      nonneg = __all(nonneg);
#pragma unroll
      for (int p = 0; p < kSeqP; p++) {  // the batch kChainD ahead
        const uint32_t j = b0 + kChainD * kB + p * kWave + lane;
        nx[t][p] = j < ce ? fbd[j] : 0.0;
      }
      __builtin_amdgcn_wave_barrier();
      rem = fb_chain_step(d, int(ce - b0 < kB ? ce - b0 : kB), rem, prec, nonneg, lane);
    }
  }
  return rem;
}

// fb_chain with the increments computed on the fly, w * mu for EVERY element of the constraint (a delisted
// variable's mu, vtmp, is the one of its last listed round: the same product fbk_acc would have kept in fbd):
// the element loads run two batches ahead and the mu gathers one batch ahead of the chain.
__device__ __forceinline__ double fb_chain_pull(const Dev& s, uint32_t cb, uint32_t ce, double rem, double prec,
                                                double* d, int lane) {
  int32_t ix[kSeqP];
  double ww[kSeqP], vt[kSeqP];
  const int32_t* __restrict__ cv = s.mu_p ? s.csc_vp : s.csc_v;  // (mu gathered in the locality order)
  const double* __restrict__ mu = s.mu_p ? s.mu_p : s.vtmp;
#pragma unroll
  for (int p = 0; p < kSeqP; p++) {  // batch 0: elements, then their mu
    const uint32_t j = cb + p * kWave + lane;
    ix[p] = j < ce ? cv[j] : -1;
    ww[p] = j < ce ? s.csc_w[j] : 0.0;
  }
#pragma unroll
  for (int p = 0; p < kSeqP; p++)
    vt[p] = ix[p] >= 0 ? mu[ix[p]] : 0.0;
#pragma unroll
  for (int p = 0; p < kSeqP; p++) {  // batch 1's elements
    const uint32_t j = cb + kSeqP * kWave + p * kWave + lane;
    ix[p] = j < ce ? cv[j] : -1;
  }
  for (uint32_t base = cb; base < ce; base += kSeqP * kWave) {  // wave-uniform
    bool nonneg = true;
#pragma unroll
    for (int p = 0; p < kSeqP; p++) {
      const double x = ww[p] * vt[p];  // (0 * 0 past the end: r - 0 == r)
      d[p * kWave + lane] = x;
      nonneg &= x >= 0.0;
    }
    nonneg = __all(nonneg);
    const uint32_t nb = base + kSeqP * kWave, nb2 = nb + kSeqP * kWave;
#pragma unroll
    for (int p = 0; p < kSeqP; p++) {  // next batch: mu gathers (its elements arrived) and weights
      const uint32_t j = nb + p * kWave + lane;
      vt[p] = ix[p] >= 0 ? mu[ix[p]] : 0.0;
      ww[p] = j < ce ? s.csc_w[j] : 0.0;
    }
#pragma unroll
    for (int p = 0; p < kSeqP; p++) {  // the batch after: elements
      const uint32_t j = nb2 + p * kWave + lane;
      ix[p] = j < ce ? cv[j] : -1;
    }
    __builtin_amdgcn_wave_barrier();
    rem = fb_chain_step(d, int(ce - base < uint32_t(kSeqP * kWave) ? ce - base : uint32_t(kSeqP * kWave)), rem, prec,
                        nonneg, lane);
  }
  return rem;
}

// Long shared constraints (>= longmin elements, C5's global dragonfly links with up to 1.6e5): their chains
// are the round's critical path, so each gets a whole workgroup (`fb_long_chain`) instead of one wave:
// fb_chain_scan's argument over steps of kBlock x 8 = 2048 increments, the int64 prefix a block-wide scan.
// The list (fb_long[0] = count, then the constraint ids) is built once per solve by fb_long_list.
__global__ void __launch_bounds__(kBlock) fb_long_list(Dev s, uint32_t longmin) {
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < s.nC; c += int64_t(gridDim.x) * kBlock)
    if (!(s.cflags[c] & 1) && s.cnst_ptr[c + 1] - s.cnst_ptr[c] >= longmin)
      s.fb_long[1 + atomicAdd(&s.fb_long[0], 1)] = int32_t(c);
}

constexpr int kLongBlocks = 128;  // workgroups of fbk_update_seq that take the long constraints (default)

// Block-wide (kBlock threads) exclusive scan of an int64 per thread; *tot = the block total.
__device__ __forceinline__ long long fb_block_scan64(long long v, long long* ws, long long* tot) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  long long incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const long long y = __shfl_up(incl, o, kWave);
    if (lane >= o)
      incl += y;
  }
  if (lane == kWave - 1)
    ws[w] = incl;
  __syncthreads();
  long long off = 0, t = 0;
#pragma unroll
  for (int i = 0; i < kBlock / kWave; i++) {
    off += i < w ? ws[i] : 0;
    t += ws[i];
  }
  __syncthreads();
  *tot = t;
  return off + incl - v;
}

// Block-wide minimum of an int per thread.
__device__ __forceinline__ int fb_block_min(int v, int* wi) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1)
    v = min(v, __shfl_xor(v, o, kWave));
  if (lane == 0)
    wi[w] = v;
  __syncthreads();
  int m = wi[0];
#pragma unroll
  for (int i = 1; i < kBlock / kWave; i++)
    m = min(m, wi[i]);
  __syncthreads();
  return m;
}

// The chain of long shared constraint c by the whole workgroup (sh: kBlock * kSeqP doubles of LDS).  Bit for
// bit the reference's loop, as fb_chain: non-negative steps are chained by the binade scan (exits and ties as
// fp64 steps, the end clamp once per step), anything else by thread 0 one double_update at a time.
__device__ void fb_long_chain(const Dev& s, int32_t c, double prec, double* sh) {
  __shared__ long long ws[kBlock / kWave];
  __shared__ int wi[kBlock / kWave];
  __shared__ double bx[2];
  constexpr int P = kSeqP;
  constexpr uint32_t kS = uint32_t(kBlock) * P;
  const int tid = threadIdx.x;
  const uint32_t cb = s.cnst_ptr[c], ce = s.cnst_ptr[c + 1];
  double x = s.rem[c];
  double nx[P];
#pragma unroll
  for (int t = 0; t < P; t++) {  // coalesced: element t * kBlock + tid of the step
    const uint32_t j = cb + t * kBlock + tid;
    nx[t] = j < ce ? s.fbd[j] : 0.0;
  }
  for (uint32_t base = cb; base < ce; base += kS) {  // block-uniform
    const int n = int(ce - base < kS ? ce - base : kS);
    bool nonneg = true;
#pragma unroll
    for (int t = 0; t < P; t++) {
      sh[t * kBlock + tid] = nx[t];
      nonneg &= nx[t] >= 0.0;
    }
#pragma unroll
    for (int t = 0; t < P; t++) {  // the next step's increments, in flight during this one
      const uint32_t j = base + kS + t * kBlock + tid;
      nx[t] = j < ce ? s.fbd[j] : 0.0;
    }
    nonneg = __syncthreads_and(nonneg);  // (also: sh written)
    double dv[P];
#pragma unroll
    for (int t = 0; t < P; t++)
      dv[t] = sh[tid * P + t];  // this thread's P consecutive increments
    int k = 0;
    if (nonneg && prec > 0.0) {
      int exits = 0;
      while (k < n) {  // block-uniform
        if (!(x >= prec)) {
          k = n;
          x = 0.0;
          break;
        }
        if (x < 0x1p-1022 || exits >= kScanExits)
          break;
        const int e = __builtin_amdgcn_frexp_exp(x) - 1;
        const long long M = (long long)(__builtin_amdgcn_ldexp(x, 52 - e) - 0x1p52);
        long long run = 0, incl[P];
        bool tie[P];
#pragma unroll
        for (int t = 0; t < P; t++) {
          const int j = tid * P + t;
          long long q = 0;
          tie[t] = false;
          if (j >= k && j < n) {
            const double sc = __builtin_amdgcn_ldexp(dv[t], 52 - e);
            if (!(sc < 0x1p52)) {
              q = 1ll << 52;
            } else {
              const double f = __builtin_floor(sc), fr = sc - f;
              tie[t] = fr == 0.5;
              q = (long long)f + (fr > 0.5 ? 1 : 0);
            }
          }
          run += q;
          incl[t] = run;
        }
        long long tot;
        const long long ex = fb_block_scan64(run, ws, &tot);
        int first = INT_MAX;
#pragma unroll
        for (int t = P - 1; t >= 0; t--) {
          const int j = tid * P + t;
          if (j >= k && j < n && (tie[t] || ex + incl[t] >= M))
            first = j;
        }
        const int js = fb_block_min(first, wi);
        const double u = __builtin_amdgcn_ldexp(1.0, e - 52);
        if (js == INT_MAX) {
          x -= double(tot) * u;  // exact
          k = n;
          break;
        }
        if (first == js) {  // the owner of the step publishes the prefix before it
          const int t = js - tid * P;
          long long pb = ex;
#pragma unroll
          for (int i = 0; i < P; i++)
            if (i < t)
              pb = ex + incl[i];
          bx[0] = double(pb);
        }
        __syncthreads();
        x -= bx[0] * u;  // exact (the prefix is below M < 2^52)
        x -= sh[js];     // the step itself
        __syncthreads();  // (bx reused)
        k = js + 1;
        exits++;
      }
      if (k >= n && x < prec)
        x = 0.0;
    }
    if (k < n) {  // thread 0, one double_update at a time (as fb_chain_batch)
      if (tid == 0)
        bx[1] = fb_chain_batch(sh + k, n - k, x, prec, nonneg && k == 0);
      __syncthreads();
      x = bx[1];
    }
    __syncthreads();  // sh is rewritten by the next step
  }
  if (tid == 0) {
    s.erased[c] = 0;
    s.rem[c] = x;
    if (x <= 0.0) {
      s.ratio[c] = dinf();
      s.erased[c] = 1;
    }
  }
}

// :107-140 for ONE context.  Workgroups [0, kLongBlocks) take the long shared constraints of fb_long, one whole
// workgroup each (fb_long_chain, from fbk_acc's increments in fbd); the others one wave per listed constraint:
// shorter shared ones through fb_chain_pull, FATPIPE ones from the chunk minima (fbk_accc); remaining <= 0
// erases the constraint (:129).
// nlb: the workgroups that take the long chains (list entries b, b + nlb, ...).  Round 5 measured taking them
// longest first from a queue (LMMHIP_FB_LPT): 8.38 vs 8.35-8.37 ms on C5, removed in round 6.  Round 6 measured the
// constraint's ratio / remaining loaded with its flags before the erased-flag store, with fb_var_inc's bound / value
// loaded with the listed flags: 8.40-8.41 against 8.36-8.37, not kept.
__global__ void __launch_bounds__(kBlock) fbk_update_seq(Dev s, double prec, uint32_t longmin, int nlb) {
  if (s.ctl[CTL_DONE])
    return;
  __shared__ __attribute__((aligned(16))) double dl[kBlock / kWave][kSeqP * kWave];
  if (int(blockIdx.x) < nlb) {
    const int nl = s.fb_long[0];
    for (int i = blockIdx.x; i < nl; i += nlb) {  // block-uniform
      const int32_t c = s.fb_long[1 + i];
      if (s.ratio[c] != 0.0) {
        if (threadIdx.x == 0)
          s.erased[c] = 0;
        continue;
      }
      fb_long_chain(s, c, prec, &dl[0][0]);
    }
    return;
  }
  const int lane = threadIdx.x & (kWave - 1);
  double* d = dl[threadIdx.x / kWave];
  for (int64_t c = (int64_t(blockIdx.x - nlb) * kBlock + threadIdx.x) / kWave; c < s.nC;
       c += int64_t(gridDim.x - nlb) * (kBlock / kWave)) {  // wave-uniform
    const bool fat = s.cflags[c] & 1;
    const uint32_t cb = s.cnst_ptr[c], ce = s.cnst_ptr[c + 1];
    if (!fat && ce - cb >= longmin)  // a long constraint: its workgroup writes everything
      continue;
    if (lane == 0)
      s.erased[c] = 0;
    if (s.ratio[c] != 0.0)
      continue;
    double rem = s.rem[c];
    if (fat) {
      double u;
      rem = fb_fat_update(s, c, rem, s.xmin[c], prec, &u);
      if (lane == 0)
        s.use[c] = u;
    } else {
      rem = fb_chain_pull(s, cb, ce, rem, prec, d, lane);
    }
    if (lane == 0) {
      s.rem[c] = rem;
      if (rem <= 0.0) {
        s.ratio[c] = dinf();
        s.erased[c] = 1;
      }
    }
  }
}

// ---- variable-sharded solve, constraint owners (simgrid_amd/multi.py FbShardPlan) ----
// Every shard holds a block of the variables (CSR rows, and a CSC of ALL constraints restricted to them:
// counts, delisting) and OWNS a block of the constraints: their full element lists in the reference's
// enabled_element_set_ order, with each element's variable given as its position in the gathered mu
// vector.  A round is four phases, the caller exchanging between them:
//   0  counts of the shard's listed variables per constraint      -> xnb      all-reduce SUM (integers: exact)
//   1  shares (replicated constraint state), the shard's mu      -> xmu      all-gather
//   2  owned constraints: increments from the gathered mu, the    -> xrem     all-gather
//      reference's per-element double_update chain (fb_chain)
//   3  remaining of every listed constraint from xrem, erasure, delisting of the shard's variables
// Every floating-point operation is the one-context solve's, on the same operands in the same order, so the
// result is bit-identical to it (and to the reference) whatever the number of shards.
struct FbOwner {
  int32_t nc;             // owned constraints
  int32_t nch;            // their chunks (kFbChunk elements)
  int64_t mu_off;         // position of this shard's first variable in xmu
  const int32_t* oc;      // [nc] global id of each owned constraint
  const uint32_t* optr;   // [nc+1] element offsets
  const int32_t* ovar;    // [onnz] position of the element's variable in xmu
  const double* ow;       // [onnz] weight
  const int32_t* och_o;   // [nch] owned-constraint index of each chunk
  const uint32_t* och_b;  // [nch] first element of each chunk
  const int32_t* cpos;    // [nC] position of each constraint's remaining in xrem
  double* fbd;            // [onnz] increments w * mu (owned CSC order)
  double* xmu;            // gathered mu (caller's buffer)
  double* xrem;           // gathered remaining (caller's buffer)
};

// phase 1 tail: this shard's mu into its block of the gathered vector (a delisted variable keeps its
// last mu: its increment still counts, fair_bottleneck.cpp:111-116)
__global__ void __launch_bounds__(kBlock) fbo_put_mu(Dev s, FbOwner o) {
  if (s.ctl[CTL_DONE])
    return;
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock)
    o.xmu[o.mu_off + v] = s.vtmp[v];
}

// phase 1 tail, multi-process delta exchange (multi.py _fb_rounds): the (position in xmu, mu) pairs of this
// shard's variables listed at the round's start (vstb; every variable in round 0) — the only mu values that
// changed this round: a delisted variable's mu is constant (fair_bottleneck.cpp:89-105 runs over the list
// only).  Appended in any order (one atomic per wave on *cnt, zeroed by the caller); the receiving ranks
// scatter them into their copy of xmu.
__global__ void __launch_bounds__(kBlock) fbo_pack_mu(Dev s, FbOwner o, int all, int32_t* pos, double* mu,
                                                      int32_t* cnt) {
  if (s.ctl[CTL_DONE])
    return;
  for (int64_t b = int64_t(blockIdx.x) * kBlock; b < s.nV; b += int64_t(gridDim.x) * kBlock) {  // wave-uniform
    const int64_t v = b + threadIdx.x;
    const bool listed = v < s.nV && (all || ((s.vstb[v >> 5] >> (v & 31)) & 1u));
    const int k = wave_append(listed, cnt);
    if (listed) {
      pos[k] = int32_t(o.mu_off + v);
      mu[k] = s.vtmp[v];
    }
  }
}

// phase 2a: increments of the owned listed constraints' elements (every element: the gathered mu of a
// delisted variable is its last one), one wave per chunk
__global__ void __launch_bounds__(kBlock) fbo_acc(Dev s, FbOwner o) {
  if (s.ctl[CTL_DONE])
    return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int q = blockIdx.x * wpb + threadIdx.x / kWave; q < o.nch; q += gridDim.x * wpb) {
    const int i = o.och_o[q];
    if (s.ratio[o.oc[i]] != 0.0)
      continue;
    const uint32_t b = o.och_b[q], ce = o.optr[i + 1];
    const uint32_t e = b + kFbChunk < ce ? b + kFbChunk : ce;
    for (uint32_t j0 = b + lane; j0 < e; j0 += 4 * kWave) {  // 4 gathers in flight per lane
      int32_t vv[4];
#pragma unroll
      for (int k = 0; k < 4; k++)
        vv[k] = j0 + k * kWave < e ? o.ovar[j0 + k * kWave] : -1;
      double dv[4];
#pragma unroll
      for (int k = 0; k < 4; k++)
        dv[k] = vv[k] >= 0 ? o.ow[j0 + k * kWave] * o.xmu[vv[k]] : 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (vv[k] >= 0)
          o.fbd[j0 + k * kWave] = dv[k];
    }
  }
}

// phase 2b: one wave per owned constraint: its new remaining (listed: the chain / FATPIPE update; else
// unchanged) into xrem
__global__ void __launch_bounds__(kBlock) fbo_chain(Dev s, FbOwner o, double prec) {
  if (s.ctl[CTL_DONE])
    return;
  __shared__ __attribute__((aligned(16))) double dl[kBlock / kWave][kSeqP * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  double* d = dl[threadIdx.x / kWave];
  for (int64_t i = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; i < o.nc;
       i += int64_t(gridDim.x) * (kBlock / kWave)) {  // wave-uniform
    const int c = o.oc[i];
    double rem = s.rem[c];
    if (s.ratio[c] == 0.0) {
      const uint32_t cb = o.optr[i], ce = o.optr[i + 1];
      if (s.cflags[c] & 1) {  // :118-125, the minimum over every element (chunk order irrelevant: fmin)
        double mn = dinf();
        for (uint32_t j = cb + lane; j < ce; j += kWave)
          mn = fmin(mn, o.fbd[j]);
        double u;
        rem = fb_fat_update(s, c, rem, wave_min(mn), prec, &u);
      } else {
        rem = fb_chain(o.fbd, cb, ce, rem, prec, d, lane);
      }
    }
    if (lane == 0)
      o.xrem[o.cpos[c]] = rem;
  }
}

// phase 3a: every listed constraint takes its owner's remaining; remaining <= 0 erases it (:129-131)
__global__ void __launch_bounds__(kBlock) fbo_apply(Dev s, FbOwner o) {
  if (s.ctl[CTL_DONE])
    return;
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < s.nC; c += gridDim.x * kBlock) {
    s.erased[c] = 0;
    if (s.ratio[c] != 0.0)
      continue;
    const double rem = o.xrem[o.cpos[c]];
    s.rem[c] = rem;
    if (rem <= 0.0) {
      s.ratio[c] = dinf();
      s.erased[c] = 1;
    }
  }
}

// :132-139 — the listed variables of an erased constraint leave the list
__global__ void __launch_bounds__(kBlock) fbk_unlist(Dev s, int bits) {
  if (s.ctl[CTL_DONE])
    return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wpb = kBlock / kWave;
  for (int q = blockIdx.x * wpb + threadIdx.x / kWave; q < s.nch; q += gridDim.x * wpb) {
    const int c = s.ch_cnst[q];
    if (!s.erased[c])
      continue;
    // bits (rounds > 0): skip the variables the round-start flags (vstb, resident in L2) already show delisted —
    // a variable leaves one time but sits on several erased constraints, and a random byte store costs a
    // partial-line write where the flag test is an L2 hit
    for (uint32_t j = s.ch_beg[q] + lane, e = chunk_end(s, q, c); j < e; j += kWave) {
      const int32_t v = s.csc_v[j];
      if (!bits || ((s.vstb[v >> 5] >> (v & 31)) & 1))
        s.vst[v] = 0;
    }
  }
}

}  // namespace lmmdev
