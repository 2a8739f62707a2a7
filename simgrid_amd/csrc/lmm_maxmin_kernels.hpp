// lmm_maxmin_kernels.hpp — System::lmm_solve on gfx950 (included by lmm_hip.hip).
//
// Local-minimum parallel progressive filling with persistent votes:
//   every alive variable votes for ONE constraint of minimal ratio among its constraints (ties:
//   smallest id — the smallest-id constraint of the global-minimum set then always collects every
//   vote, so each round makes progress).  Ratios never decrease, so a vote stays valid until the
//   voted constraint's ratio changes: only variables whose target changed in the previous round are
//   re-evaluated.  A constraint is a local minimum ("ready") iff every alive element votes for it.
//
// Round r (4 launches):
//   mm_vote<G>   re-evaluate the variables whose target changed in round r-1 (G lanes per row):
//                minimal 16-bit key over the row, exact fp64 only on key ties / bound checks; move
//                the vote; a variable whose level bound*penalty is below its minimum is fixed at its
//                bound right here (maxmin.cpp:563-595); a variable with no alive constraint drops.
//   mm_ready     one thread per constraint: no alive element votes elsewhere (nvote == 0) -> ready list.
//   mm_saturate  K waves per ready constraint: claim its alive variables, fix them at ratio/penalty
//                (maxmin.cpp:583), push w*x, w/p and count decrements (maxmin.cpp:601-606) and flag the
//                receiving constraints (ctouch).  (The persistent engine fuses the two: sat_block.)
//   mm_update    one thread per constraint: apply decrements, clamp (surf_interface.hpp:34-44 —
//                clamping a sum of non-negative decrements == clamping after each one), drop
//                saturated constraints (maxmin.cpp:608-623), refresh ratio, key and change stamp;
//                FATPIPE usage is recomputed over the still-unfixed elements (maxmin.cpp:625-658).
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

// Per-element usage w / penalty of every CSC element (maxmin.cpp:531-533's summand), computed at upload
// and whenever the penalties change, so the per-solve init streams it instead of gathering pen[v].
// Per CSC element: usage w / penalty and the penalty (with every penalty change), and — rows = 1, with every
// structure change — its variable's CSR row.
__global__ void __launch_bounds__(kBlock) mm_elem_usage(Dev s, int rows) {
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < s.nnz; j += int64_t(gridDim.x) * kBlock) {
    const int32_t v = s.csc_v[j];
    const double p = s.pen[v];
    s.csc_u[j] = s.csc_w[j] / p;
    s.csc_p[j] = p;
    if (rows)
      s.csc_row[j] = (unsigned long long)s.var_ptr[v] | ((unsigned long long)s.var_ptr[v + 1] << 32);
  }
}

// cdup (zeroed before): constraints holding two elements of one variable; every constraint of a row longer
// than 64 elements is flagged without the pairwise test.
__global__ void __launch_bounds__(kBlock) mm_dup_check(Dev s) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock) {
    const uint32_t b = s.var_ptr[v], e = s.var_ptr[v + 1];
    if (e - b > 64) {
      for (uint32_t i = b; i < e; i++)
        s.cdup[s.csr_c[i]] = 1;
      continue;
    }
    if (e - b <= 16) {  // the row in registers, its loads in flight together
      int32_t cc[16];
#pragma unroll
      for (int i = 0; i < 16; i++)
        cc[i] = b + i < e ? s.csr_c[b + i] : -1 - i;
#pragma unroll
      for (int i = 0; i < 16; i++)
#pragma unroll
        for (int j = i + 1; j < 16; j++)
          if (cc[i] >= 0 && cc[i] == cc[j])
            s.cdup[cc[i]] = 1;
      continue;
    }
    for (uint32_t i = b; i < e; i++)
      for (uint32_t j = i + 1; j < e; j++)
        if (s.csr_c[i] == s.csr_c[j])
          s.cdup[s.csr_c[i]] = 1;
  }
}

// Init, one wave per constraint: maxmin.cpp:520-555.  remaining = bound; skipped when
// bound <= bound*prec; usage = sum (SHARED) or max (FATPIPE) of w/p over the active elements.
// Waves `wave`, `wave + nwaves`, ... of the grid; returns (on lane 0) the constraints made alive.
// One group of kInitG lanes per constraint (kWave / kInitG constraints per wave at a time: a wave used to take its
// ~120 constraints of C2 one after the other, each a dependent chain of loads — 377 us per solve).
constexpr int kInitG = 16;
__device__ __forceinline__ int init_cnsts_waves(const Dev& s, double prec, int64_t wave, int64_t nwaves) {
  const int lane = threadIdx.x & (kWave - 1), gl = lane & (kInitG - 1);
  constexpr int kGpw = kWave / kInitG;
  int alive_cnt = 0;
  for (int64_t c = wave * kGpw + lane / kInitG; c < s.nC; c += nwaves * kGpw) {  // group-uniform
    const uint32_t b = s.cnst_ptr[c], e = s.cnst_ptr[c + 1];
    const bool fat = s.cflags[c] & 1;
    double acc = 0.0;
    // four loads in flight per lane, accumulated in a fixed order (a missing term adds 0.0 / max's 0.0 to a
    // non-negative acc), so every engine computes the same bits
    for (uint32_t j0 = b + gl; j0 < e; j0 += 4 * kInitG) {
      double u[4];
#pragma unroll
      for (int k = 0; k < 4; k++)
        u[k] = j0 + k * kInitG < e ? s.csc_u[j0 + k * kInitG] : 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++)
        acc = fat ? fmax(acc, u[k]) : acc + u[k];
    }
#pragma unroll
    for (int o = kInitG / 2; o > 0; o >>= 1) {
      const double y = __shfl_xor(acc, o, kInitG);
      acc = fat ? fmax(acc, y) : acc + y;
    }
    if (gl == 0) {
      const double bound = s.cbound[c];
      const bool part = bound > bound * prec;
      const double usage = part ? acc : 0.0;
      const bool alive = part && usage > 0;
      const double r = bound / usage;
      CstRec rec;
      rec.drem = rec.duse = rec.dcnt = 0;
      rec.pad = 0;
      s.ctouch[c] = 0;
      rec.rem = bound;
      rec.use = usage;
      rec.ratio = alive ? r : dinf();
      rec.bound = bound;
      s.cst[c] = rec;
      // fixed-point scales of this solve's decrements (CstRec): a round never removes more than the
      // remaining (<= bound) or the usage (<= initial usage) from a constraint
      s.cexp[c] = cexp_pack(alive ? dec_scale(bound) : 0, alive ? dec_scale(usage) : 0, fat, !alive);
      s.nvote[c] = int32_t(e - b);  // no element votes yet
      s.chg[c] = uint16_t(0xFFFF);
      s.key[c] = alive ? ratio_key(r) : uint16_t(kDeadKey);
      if (s.key32)  // (frontier engine)
        s.key32[c] = alive ? ratio_key32(r) : kDead32;
      alive_cnt += alive;
    }
  }
  return alive_cnt;
}

// (Round 6: the per-wave count of alive constraints this kernel used to add into one control word — read by nobody —
// was 8,192 atomics on one address per solve, serialised in the memory-side unit after the grid's short work: the
// whole 74-us init of C4 and ~70 us of C2's.)
__global__ void __launch_bounds__(kBlock) mm_init_cnsts(Dev s, double prec) {
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  init_cnsts_waves(s, prec, wave, int64_t(gridDim.x) * (kBlock / kWave));
}

// kRec: also the packed row records of buffer 0 (the multi-launch engine's init only).
template <bool kRec = false>
__device__ __forceinline__ void init_vars_range(const Dev& s, int64_t t, int64_t nthreads) {
  for (int64_t v = t; v < s.nV; v += nthreads) {
    s.x[v] = 0.0;
    s.vstate[v] = 0;
    s.rtgt[0][v] = kUnvoted;
    const int32_t cv = int32_t(v) | (s.vbound[v] > 0 ? int32_t(0x80000000u) : 0);
    const_cast<int32_t*>(s.cvar[0])[v] = cv;
    if (kRec && s.crec[0])
      s.crec[0][v] = make_uint2(uint32_t(cv), s.var_ptr[v]);
  }
}

__global__ void __launch_bounds__(kBlock) mm_init_vars(Dev s) {
  init_vars_range<true>(s, int64_t(blockIdx.x) * kBlock + threadIdx.x, int64_t(gridDim.x) * kBlock);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.ctl[CTL_NROWS + 0] = s.nV;
    s.ctl[CTL_NELEM + 0] = int32_t(s.nnz);
    if (s.crec[0])
      s.crec[0][s.nV] = make_uint2(0u, s.var_ptr[s.nV]);
  }
}

// The floor of a row that voted for a constraint of key mk: while the target's key stays strictly below
// it, the vote stands even if the target's ratio moved (keys never decrease).  It is the min key over the
// row's OTHER constraints (sk) and, for a bounded variable, the key of its level bound * penalty (key[t] <
// key(b*p) implies ratio[t] < b*p: the bound test of maxmin.cpp:587 stays false).  0 marks a "sensitive"
// row whose vote depends on the target's exact ratio (a key-level tie with another constraint or with the
// bound level), re-evaluated whenever the target is touched.
// Ready constraints without the mm_ready pass (LMMHIP_RDQ): a constraint whose count of elements voting
// elsewhere reaches 0 is ready in the round the count gets there.  The update (the fixed variables' elements
// leaving it) lists such constraints in its workgroup's segment (useg / ucnt: mm_ready's output format, LDS
// appends, no global atomics); the vote (a moving vote's atomicSub, made returning) queues the ones it makes
// ready (rdq, one entry per constraint and round through the rqst stamps, which the update sets too).
// mm_saturate_q re-checks every entry after the vote (alive, nothing voting elsewhere).
constexpr int kUSeg = 1024;  // update candidates per workgroup segment (>= the constraints a workgroup updates)
// (Round 6 measured the update's candidates appended to 8 lists — one returning add per workgroup on the list of its
// XCD — so that the saturation reads 8 lengths instead of a prefix of ~1,024 segment counts: the saturation gained
// ~4 us per round, the update lost 7-8 us to the adds at its end; C2 24.31 ms against 23.62, removed.)
__device__ __forceinline__ void rdq_push(const Dev& s, int32_t c, int qround) {
  if (atomicExch(&s.rqst[c], qround) != qround) {
    const int q = qround & 1;
    s.rdq[q][atomicAdd(&s.ctl[CTL_RDQ0 + q], 1)] = c;
  }
}
// The vote's queue through the workgroup (round 6): a constraint a re-vote made ready goes to an LDS list, and the
// workgroup reserves its range of the global queue with ONE add at its end (rdq_flush_lds).  The round anatomy
// (profiles/r06_c2_round_anatomy.json) found the queue's one counter word the longest wait of the tail's votes: per
// lane (round 5), then per wave, every queued constraint or wave was a returning add on that one word, ~10-13 ns
// each at the memory side, queued behind each other (11-17 us of a 27-us vote in round 200).  Past kRqCap
// entries a workgroup queues directly (the old path).  The queue's order does not matter: the saturation of one
// round's ready constraints commutes (no shared alive variable, fixed-point integer decrements).
constexpr int kRqCap = 2048;
// (Round 6 measured the workgroup's list written to a segment of its own — plain stores, read by the saturation after
// the update's segments — instead of the one returning add per workgroup: C2 23.59-23.60 ms against 23.48-23.58.)
struct RdqLds {
  int n, base;
  int32_t buf[kRqCap];
};
__device__ __forceinline__ void rdq_push_lds(const Dev& s, int32_t c, int qround, RdqLds* L) {
  if (c >= 0 && atomicExch(&s.rqst[c], qround) != qround) {
    const int pos = atomicAdd(&L->n, 1);  // (LDS)
    if (pos < kRqCap) {
      L->buf[pos] = c;
    } else {
      const int q = qround & 1;
      s.rdq[q][atomicAdd(&s.ctl[CTL_RDQ0 + q], 1)] = c;
    }
  }
}
// (every thread of the workgroup, after its last push)
__device__ __forceinline__ void rdq_flush_lds(const Dev& s, int qround, RdqLds* L) {
  __syncthreads();
  const int n = L->n < kRqCap ? L->n : kRqCap;
  const int q = qround & 1;
  if (threadIdx.x == 0)
    L->base = n ? atomicAdd(&s.ctl[CTL_RDQ0 + q], n) : 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    s.rdq[q][L->base + i] = L->buf[i];
}

__device__ __forceinline__ unsigned row_floor(unsigned sk, unsigned mk, double vb, double p) {
  unsigned fl = sk;
  if (vb > 0)
    fl = min(fl, (unsigned)ratio_key(vb * p));
  return fl <= mk ? 0u : fl;
}

// FATPIPE constraints (maxmin.cpp:625-658): usage = max of w/p over the unfixed elements.  A fixed element
// pushes its w/p into the record's duse slot with an unsigned max of the (non-negative) double's bits;
// mm_update recomputes the max over the CSC only when a removed element reached the current usage — the
// max over the remaining elements is unchanged otherwise.
__device__ __forceinline__ unsigned long long fat_bits(double u) { return (unsigned long long)__double_as_longlong(u); }

// Decrements of a fixed variable's element j (maxmin.cpp:601-606) into the constraint's record, as
// fixed-point integers (CstRec); FATPIPE constraints get the count and the removed w/p (fat_bits).  One lane
// issues them all (rare path: bound fixes in the vote).
__device__ __forceinline__ void push_decrement(const Dev& s, uint32_t j, double xv, double p) {
  const int32_t c = s.csr_c[j];
  const int32_t ce = s.cexp[c];
  if (ce & kCexpDead)
    return;
  unsigned long long* r = &s.cst[c].drem;
  s.ctouch[c] = 1;  // receives decrements this round (mm_update reads its record)
  atomicAdd(&r[2], 1ull);  // fixed elements leaving c (mm_update subtracts them from nvote)
  const double w = s.csr_w[j];
  if (!(ce & kCexpFat)) {
    atomicAdd(&r[0], dec_q(w * xv, cexp_rem(ce)));
    atomicAdd(&r[1], dec_q(w / p, cexp_use(ce)));
  } else {
    atomicMax(&r[1], fat_bits(w / p));
  }
}

// Round phase 1 — (re-)vote.  G lanes per alive row; loops are wave-uniform so the group shuffles
// always see their whole group.
template <int G> __global__ void __launch_bounds__(kBlock) mm_vote(Dev s, int round) {
  if (s.ctl[CTL_DONE])  // light table empty (maxmin.cpp:680), detected by mm_done
    return;
  const int buf = s.ctl[CTL_BUF];
  __shared__ int st_rows, st_elems;  // profiling counters (LDS, one store per block)
  if (s.vstat && threadIdx.x == 0)
    st_rows = st_elems = 0;
  if (s.vstat)
    __syncthreads();
  const int64_t nrows = s.ctl[CTL_NROWS + buf];
  const int32_t* __restrict__ cvar = s.cvar[buf];
  const uint32_t* __restrict__ crow = s.crow[buf];
  const int32_t* __restrict__ ccol = s.ccol[buf];
  const uint16_t* __restrict__ key = s.key;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane & (G - 1);
  constexpr int kGpw = kWave / G;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  // One lane per row decides whether the row needs work (its target changed last round); the rows
  // that do are then processed kGpw at a time (one G-lane group each), so a wave only pays for the
  // rows that need it.
  int32_t* __restrict__ rtgt = s.rtgt[buf];
  const uint16_t prev = uint16_t(round - 1);
  for (int64_t base = wave * kWave; base < nrows; base += nwaves * kWave) {
    const int64_t lrow = base + lane;
    const int lt = lrow < nrows ? rtgt[lrow] : kRetired;  // streamed, row-aligned
    // re-vote when the target changed last round, unless it is still strictly below every other
    // constraint of the row (their keys only grow): then the vote stands (skey)
    const bool lneed = lt == kUnvoted || (lt >= 0 && s.chg[lt] == prev && !(key[lt] < s.skey[buf][lrow]));
    unsigned long long mask = __ballot(lneed);
    while (mask) {  // wave-uniform
      unsigned long long m = mask;
      for (int i = 0; i < lane / G; i++)
        m &= m - 1;
      const int pos = m ? __ffsll((long long)m) - 1 : -1;
      for (int i = 0; i < kGpw; i++)
        mask &= mask - 1;
      const int src = pos < 0 ? 0 : pos;
      const int t = __shfl(lt, src, kWave);
      const int64_t row = base + src;
      const int v = pos >= 0 ? rvar(cvar[row]) : 0;
      bool need = pos >= 0;
      if (need && s.vstate[v] != 0) {  // fixed by mm_saturate since: retire the row
        if (g == 0)
          rtgt[row] = kRetired;
        need = false;
      }
      uint32_t b = 0, e = 0;
      if (need) {
        b = crow[row];
        e = crow[row + 1];
        if (s.vstat && g == 0) {
          atomicAdd(&st_rows, 1);
          atomicAdd(&st_elems, int(e - b));
        }
      }
      // the lane's first element stays in registers; rows longer than G loop over the rest
      const uint32_t j0 = b + g;
      const bool h0 = j0 < e;
      const int32_t c0 = h0 ? ccol[j0] : -1;
      const unsigned k0 = h0 ? key[c0] : kDeadKey;
      unsigned mk = k0;
      for (uint32_t j = j0 + G; j < e; j += G)
        mk = min(mk, (unsigned)key[ccol[j]]);
      mk = grp_umin<G>(mk);
      int nmin = h0 && k0 == mk;
      for (uint32_t j = j0 + G; j < e; j += G)
        nmin += key[ccol[j]] == mk;
      nmin = grp_isum<G>(nmin);
      const double vb = need ? s.vbound[v] : -1.0;
      const bool live = need && mk != kDeadKey;
      double minr = dinf();
      if (live && (nmin > 1 || vb > 0)) {
        if (h0 && k0 == mk)
          minr = s.cst[c0].ratio;
        for (uint32_t j = j0 + G; j < e; j += G) {
          const int32_t c = ccol[j];
          if (key[c] == mk)
            minr = fmin(minr, s.cst[c].ratio);
        }
      }
      minr = grp_min<G>(minr);
      const double p = need ? s.pen[v] : 1.0;
      const bool bounded = live && vb > 0 && vb * p < minr;
      int newt = INT_MAX;
      if (live && !bounded) {
        if (h0 && k0 == mk && (nmin == 1 || s.cst[c0].ratio == minr))
          newt = c0;
        for (uint32_t j = j0 + G; j < e; j += G) {
          const int32_t c = ccol[j];
          if (key[c] == mk && (nmin == 1 || s.cst[c].ratio == minr))
            newt = min(newt, c);
        }
      }
      newt = grp_imin<G>(newt);
      unsigned sk = h0 && c0 != newt ? k0 : kDeadKey;  // min key over the other constraints
      for (uint32_t j = j0 + G; j < e; j += G) {
        const int32_t c = ccol[j];
        if (c != newt)
          sk = min(sk, (unsigned)key[c]);
      }
      sk = grp_umin<G>(sk);
      if (live && !bounded && g == 0)  // the row's floor, 0 = "sensitive" (see vote_row)
        s.skey[buf][row] = uint16_t(row_floor(sk, mk, vb, p));
      int mult_new = h0 && c0 == newt, mult_old = h0 && c0 == t;
      for (uint32_t j = j0 + G; j < e; j += G) {
        const int32_t c = ccol[j];
        mult_new += c == newt;
        mult_old += c == t;
      }
      mult_new = grp_isum<G>(mult_new);
      mult_old = grp_isum<G>(mult_old);
      if (need && !live) {  // every constraint of v left the light table: v stays at 0
        if (g == 0) {
          s.vstate[v] = round + 1;  // fixed / dropped in this round
          rtgt[row] = kRetired;
        }
      } else if (bounded) {  // fixed at its bound (maxmin.cpp:587-589)
        if (g == 0) {
          s.vstate[v] = round + 1;  // fixed / dropped in this round
          s.x[v] = vb;
          rtgt[row] = kRetired;
          if (t >= 0 && key[t] != kDeadKey)
            atomicAdd(&s.nvote[t], mult_old);
        }
        for (uint32_t j = s.var_ptr[v] + g; j < s.var_ptr[v + 1]; j += G)
          push_decrement(s, j, vb, p);
      } else if (live && newt != t && g == 0) {
        if (t >= 0 && key[t] != kDeadKey)
          atomicAdd(&s.nvote[t], mult_old);
        atomicSub(&s.nvote[newt], mult_new);
        rtgt[row] = newt;
      }
    }
  }
  if (s.vstat) {
    __syncthreads();
    if (threadIdx.x == 0 && round < kStatRounds && blockIdx.x < kMaxBlocks) {
      s.vstat[2 * (int64_t(round) * kMaxBlocks + blockIdx.x)] = st_rows;
      s.vstat[2 * (int64_t(round) * kMaxBlocks + blockIdx.x) + 1] = st_elems;
    }
  }
}

// Alive-constraint list: built at init (from_all: every constraint id into list 0), then re-compacted from the
// list in use (ctl CTL_CB) into the other one (order not preserved; mm_flip switches).  One contiguous range
// per block: count, ONE atomic per block for its output range, write (a counter per 256 entries cost ~44 us
// of contended atomics on C2).
__global__ void __launch_bounds__(kBlock) mm_clist(Dev s, int from_all) {
  if (!from_all && s.ctl[CTL_DONE])
    return;
  __shared__ int wsum[kBlock / kWave];
  __shared__ int base_sh;
  const int in = from_all ? 0 : s.ctl[CTL_CB], out = from_all ? 0 : in ^ 1;
  const int64_t n = from_all ? s.nC : s.ctl[CTL_NCL0 + in];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = int64_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int cnt = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const int32_t c = from_all ? int32_t(i) : s.clist[in][i];
    cnt += s.key[c] != kDeadKey;
  }
  cnt = grp_isum<kWave>(cnt);
  if (lane == 0)
    wsum[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int k = 0; k < kBlock / kWave; k++)
      t += wsum[k];
    base_sh = t ? atomicAdd(&s.ctl[CTL_NCL0 + out], t) : 0;
  }
  __syncthreads();
  int pos = base_sh;
  for (int64_t b0 = lo; b0 < hi; b0 += kBlock) {  // block-uniform
    const int64_t i = b0 + threadIdx.x;
    int32_t c = -1;
    if (i < hi)
      c = from_all ? int32_t(i) : s.clist[in][i];
    const bool alive = c >= 0 && s.key[c] != kDeadKey;
    const unsigned long long m = __ballot(alive);
    __syncthreads();
    if (lane == 0)
      wsum[w] = __popcll(m);
    __syncthreads();
    int off = pos, tot = 0;
    for (int k = 0; k < kBlock / kWave; k++) {
      off += k < w ? wsum[k] : 0;
      tot += wsum[k];
    }
    if (alive)
      s.clist[out][off + __popcll(m & ((1ull << lane) - 1))] = c;
    pos += tot;
  }
}

// The control words into a pinned host slot, written by the GPU itself (mapped memory, system-scope release):
// a copy-engine transfer on the stream cost a 20-40 us gap before the next kernel at every poll (~1 ms per C2
// solve in the rocprofv3 trace).
__global__ void mm_ctl_out(Dev s, int32_t* dst) {
  const int i = threadIdx.x;
  if (i < CTL_WORDS)
    __hip_atomic_store(dst + i, s.ctl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// After a list re-compaction and / or a row compaction: switch the buffers in use (one thread).
__global__ void mm_flip(Dev s, int clist, int rows) {
  if (s.ctl[CTL_DONE])
    return;
  if (clist) {
    const int in = s.ctl[CTL_CB];
    s.ctl[CTL_CB] = in ^ 1;
    s.ctl[CTL_NCL0 + in] = 0;  // the old list's counter: the next re-compaction's output
  }
  if (rows && s.ctl[CTL_CMPGO]) {
    const int in = s.ctl[CTL_BUF];
    s.ctl[CTL_BUF] = in == 1 ? 2 : 1;
  }
}

// Lane-per-row variant of mm_vote for short rows (mean length <= 8).  The filter pass streams the
// row targets (one lane per row, kFilt rows in flight per lane) and queues the rows that need a
// re-vote in LDS; each full queue of kBlock rows is then resolved one lane per row, with up to kReg
// independent gathers in flight, so the rare slow rows no longer stall whole waves of fast ones.
#ifndef LMM_KFILT
#define LMM_KFILT 8
#endif
constexpr int kFilt = LMM_KFILT;  // rows per lane per filter step (their loads in flight together; build knob)

// Re-vote of one row, one lane: the first R elements in registers (their loads in flight together), longer
// rows loop over the rest.  Every load indexed by the row or its variable is issued at once.
// kRec: the row's variable and CSR range from the packed records (crec; the multi-launch engine's short-row
// vote only — other instantiations, e.g. the persistent kernel, keep their register budget).
// (LMM_ANAT: `an` = record the dependent levels into aa.lv[0..5]: row record, variable state, row elements, keys,
// exact ratios, the vote's stores and atomics)
#if LMM_ANAT
#define VR_ANAT_PARAMS , bool an = false, AnatAcc* aa = nullptr
#define VR_LVL(i, dep)       \
  do {                       \
    if (an)                  \
      ANAT_LVL(*aa, i, dep); \
  } while (0)
#else
#define VR_ANAT_PARAMS
#define VR_LVL(i, dep) \
  do {                 \
  } while (0)
#endif
// kRdq: a constraint this re-vote made ready (nothing votes elsewhere any more) is returned in *rdq_c for the
// caller's workgroup-wide queueing (rdq_push_lds), or queued here when rdq_c is null.
template <int R, bool kRec = false, bool kRdq = false>
__device__ __forceinline__ void vote_row(const Dev& s, int buf, int round, int64_t row, int* st_rows,
                                         int* st_elems, const uint16_t* __restrict__ key, int* rdq_c = nullptr
                                         VR_ANAT_PARAMS) {
#if LMM_ANAT
  if (an)
    aa->at = anat_now();
#endif
  const int32_t* __restrict__ cvar = s.cvar[buf];
  const uint32_t* __restrict__ crow = s.crow[buf];
  const int32_t* __restrict__ ccol = s.ccol[buf];
  int32_t* __restrict__ rtgt = s.rtgt[buf];
  uint16_t* __restrict__ skey = s.skey[buf];
  // (key: s.key, or its copy in LDS — persistent engine, small systems)
  const int t = rtgt[row];
  int32_t cv;
  uint32_t b, e;
  if (kRec) {  // (the row's variable and CSR range from one 8-B record and its successor)
    const uint2 r0 = s.crec[buf][row], r1 = s.crec[buf][row + 1];
    cv = int32_t(r0.x);
    b = r0.y;
    e = r1.y;
  } else {
    cv = cvar[row];
    b = crow[row];
    e = crow[row + 1];
  }
  VR_LVL(0, b + e + uint32_t(t) + uint32_t(cv));
  const int v = rvar(cv);
  const int32_t vst = s.vstate[v];
  const bool bnd = rbounded(cv);
  const double vb = bnd ? s.vbound[v] : -1.0;
  const double p = bnd ? s.pen[v] : 1.0;  // read below only when vb > 0
  VR_LVL(1, vst);
  // (the row's gathers wait for the variable's state: a fixed variable's row — every variable once, when
  // its saturated target dies — retires without them; measured cheaper on C2 than issuing them early)
  if (vst != 0) {  // fixed by a saturation since: retire the row
    rtgt[row] = kRetired;
    return;
  }
  if (s.vstat) {
    atomicAdd(st_rows, 1);
    atomicAdd(st_elems, int(e - b));
  }
  int32_t cc[R];
  unsigned kk[R];
#pragma unroll
  for (int i = 0; i < R; i++)
    cc[i] = b + i < e ? ccol[b + i] : -1;
#if LMM_ANAT
  {
    int32_t ccs = 0;
#pragma unroll
    for (int i = 0; i < R; i++)
      ccs += cc[i];
    VR_LVL(2, ccs);
  }
#endif
#pragma unroll
  for (int i = 0; i < R; i++)
    kk[i] = cc[i] >= 0 ? key[cc[i]] : kDeadKey;
  const unsigned kt = t >= 0 ? key[t] : kDeadKey;
  // Elements beyond the first R: three passes (min key; count / old multiplicity / candidate; the other
  // keys / new multiplicity), plus the exact-ratio pass on key ties or bounded variables, each with its
  // loads unrolled so that they are in flight together.
  unsigned mk = kDeadKey;
#pragma unroll
  for (int i = 0; i < R; i++)
    mk = min(mk, kk[i]);
#pragma unroll 4
  for (uint32_t j = b + R; j < e; j++)
    mk = min(mk, (unsigned)key[ccol[j]]);
  VR_LVL(3, mk + kt);
  if (mk == kDeadKey) {  // every constraint of v left the light table: v stays at 0
    s.vstate[v] = round + 1;  // fixed / dropped in this round
    rtgt[row] = kRetired;
    return;
  }
  int nmin = 0, mult_old = 0, newt = INT_MAX;  // newt: the smallest id at the minimal key
#pragma unroll
  for (int i = 0; i < R; i++) {
    nmin += kk[i] == mk;
    mult_old += cc[i] == t;
    if (kk[i] == mk)
      newt = min(newt, cc[i]);
  }
#pragma unroll 4
  for (uint32_t j = b + R; j < e; j++) {
    const int32_t c = ccol[j];
    const unsigned k = key[c];
    nmin += k == mk;
    mult_old += c == t;
    if (k == mk)
      newt = min(newt, c);
  }
  double minr = dinf();
  if (nmin > 1 || vb > 0) {  // exact ratios at the minimal key: lexicographic min of (ratio, id)
    newt = INT_MAX;
    // the tied constraints' ratios: all loads issued before the first compare (one dependent level: a compare right
    // after each conditional load waits for the loads one at a time).  Not in the persistent kernel (kRec = kRdq =
    // false), whose 128-VGPR budget the ratios array exceeds (47 VGPRs spilled).
    constexpr bool kTieLd = kRec || kRdq;
    double rr[kTieLd ? R : 1];
    if (kTieLd) {
#pragma unroll
      for (int i = 0; i < R; i++)
        rr[kTieLd ? i : 0] = kk[i] == mk ? s.cst[cc[i]].ratio : dinf();
    }
#pragma unroll
    for (int i = 0; i < R; i++)
      if (kk[i] == mk) {
        const double r = kTieLd ? rr[kTieLd ? i : 0] : s.cst[cc[i]].ratio;
        if (r < minr || (r == minr && cc[i] < newt)) {
          minr = r;
          newt = cc[i];
        }
      }
    for (uint32_t j = b + R; j < e; j++) {
      const int32_t c = ccol[j];
      if (key[c] == mk) {
        const double r = s.cst[c].ratio;
        if (r < minr || (r == minr && c < newt)) {
          minr = r;
          newt = c;
        }
      }
    }
  }
  VR_LVL(4, minr + double(newt));
  if (vb > 0 && vb * p < minr) {  // fixed at its bound (maxmin.cpp:587-589)
    s.vstate[v] = round + 1;  // fixed / dropped in this round
    s.x[v] = vb;
    rtgt[row] = kRetired;
    if (t >= 0 && kt != kDeadKey)
      atomicAdd(&s.nvote[t], mult_old);
    for (uint32_t j = s.var_ptr[v]; j < s.var_ptr[v + 1]; j++)
      push_decrement(s, j, vb, p);
    return;
  }
  unsigned sk = kDeadKey;  // min key over the other constraints of the row
  int mult_new = 0;
#pragma unroll
  for (int i = 0; i < R; i++) {
    if (cc[i] != newt)
      sk = min(sk, kk[i]);
    mult_new += cc[i] == newt;
  }
#pragma unroll 4
  for (uint32_t j = b + R; j < e; j++) {
    const int32_t c = ccol[j];
    const unsigned k = key[c];
    if (c != newt)
      sk = min(sk, k);
    mult_new += c == newt;
  }
  skey[row] = uint16_t(row_floor(sk, mk, vb, p));
  if (newt == t)
    return;
  if (t >= 0 && kt != kDeadKey)
    atomicAdd(&s.nvote[t], mult_old);
  if (kRdq) {
    const int old = atomicSub(&s.nvote[newt], mult_new);
    if (old == mult_new) {  // nothing votes elsewhere any more: ready
      if (rdq_c)
        *rdq_c = newt;
      else
        rdq_push(s, newt, round);
    }
    VR_LVL(5, old);
  } else {
    atomicSub(&s.nvote[newt], mult_new);
  }
  rtgt[row] = newt;
}

// Filter + re-vote of the rows [lo, hi) of buffer `buf` by the calling workgroup, every wave on its own
// contiguous share of 64-row groups with no workgroup barrier: a wave streams F rows per lane at a time
// (targets and floors, loads in flight together), tests the target against the changed-constraint bitmap
// (kBits: in LDS, built by mm_update — a set bit means the target's KEY changed or it died last round;
// otherwise the 16-bit change stamps), gathers the target's key for those rows, and queues the rows whose
// vote may move in its own LDS queue `qw` (2 x 64 entries); every full 64 are resolved one lane per row
// (vote_row) right away, so one wave's dependent gathers overlap the other waves' streaming.
// A row re-votes when it never voted, when its target's key changed or it died and the key is no longer
// strictly below the row's floor (skey: its other keys only grow), or — sensitive rows (skey 0) — when its
// target was touched at all (chg stamp).  Returns the rows this wave queued (lane-uniform).
// kDiag (measurement only, LMMHIP_VOTE_DIAG): 1 = the filter alone (rows queued, none resolved), with
// per-round counters of target-changed / sensitive / queued rows in vstat's kDiagSlot.
constexpr int kQW = 2 * kWave;  // per-wave queue capacity
constexpr int kDiagSlot = kMaxBlocks - 4;  // vstat block slots kDiagSlot.. hold the vote diagnostics (kDiag)

// The wave's row range [wlo, whi) of the workgroup's rows [lo, hi).
__device__ __forceinline__ void vote_wave_range(int64_t lo, int64_t hi, int64_t& wlo, int64_t& whi) {
  const int w = threadIdx.x / kWave, nw = blockDim.x / kWave;
  const int64_t ngr = (hi - lo + kWave - 1) / kWave;
  const int64_t gpw = (ngr + nw - 1) / nw;
  wlo = lo + int64_t(w) * gpw * kWave;
  whi = wlo + gpw * kWave < hi ? wlo + gpw * kWave : hi;
}

// kPre: the targets and floors of the wave's first filter step were loaded by the caller (tt0 / sk0, issued before
// the bitmap copy, so that their latency overlaps it).
// LMM_ANAT: `an` = stamp the filter steps and re-vote batches of this wave into aa (lv[6] filter loads, lv[7] filter
// gathers, lv[8] re-vote batches; w[0] steps, w[1] batches) and vote_row's levels into ar.
#if LMM_ANAT
#define VW_ANAT_PARAMS , bool an = false, AnatAcc* aa = nullptr, AnatAcc* ar = nullptr, unsigned* wcnt = nullptr
#else
#define VW_ANAT_PARAMS
#endif
template <bool kBits, int R, int F, int kDiag, bool kRec = false, bool kRdq = false, bool kPre = false>
__device__ __forceinline__ int vote_waves(const Dev& s, int buf, int round, int64_t lo, int64_t hi,
                                          const uint64_t* bits, int* qw, int* st_rows, int* st_elems,
                                          const uint16_t* __restrict__ key, const int* tt0 = nullptr,
                                          const unsigned* sk0 = nullptr, RdqLds* rql = nullptr VW_ANAT_PARAMS) {
  const int lane = threadIdx.x & (kWave - 1);
  int64_t wlo, whi;
  vote_wave_range(lo, hi, wlo, whi);
  const int32_t* __restrict__ rtgt = s.rtgt[buf];
  const uint16_t* __restrict__ skey = s.skey[buf];
  const uint16_t prev = uint16_t(round - 1);
  const unsigned long long below = (1ull << lane) - 1;
  int qn = 0, nq = 0;
  int dg[4] = {0, 0, 0, 0};  // kDiag 1: target-changed / sensitive / queued / queued sensitive rows of this lane
  for (int64_t base = wlo; base < whi; base += int64_t(F) * kWave) {  // wave-uniform
    int tt[F];
    unsigned sk[F];
#if LMM_ANAT
    if (an) {
      aa->at = anat_now();
      wcnt[0]++;
    }
#endif
    if (kPre && base == wlo) {  // wave-uniform
#pragma unroll
      for (int u = 0; u < F; u++) {
        tt[u] = tt0[u];
        sk[u] = sk0[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < F; u++) {
        const int64_t row = base + u * kWave + lane;
        tt[u] = row < whi ? rtgt[row] : kRetired;
        sk[u] = row < whi ? unsigned(skey[row]) : 1u;
      }
    }
#if LMM_ANAT
    if (an) {
      int ts = 0;
#pragma unroll
      for (int u = 0; u < F; u++)
        ts += tt[u] + int(sk[u]);
      ANAT_LVL(*aa, 6, ts);
    }
#endif
    bool ch[F];
#pragma unroll
    for (int u = 0; u < F; u++) {
      if (kBits)
        ch[u] = tt[u] >= 0 && ((bits[tt[u] >> 6] >> (tt[u] & 63)) & 1);
      else
        ch[u] = tt[u] >= 0 && s.chg[tt[u]] == prev;
    }
    unsigned kt[F], cg[F];
#pragma unroll
    for (int u = 0; u < F; u++) {  // target key (changed targets) / stamp (sensitive rows), together
      kt[u] = ch[u] ? key[tt[u]] : 0u;
      cg[u] = (kBits && !ch[u] && tt[u] >= 0 && sk[u] == 0) ? unsigned(s.chg[tt[u]]) : 0x10000u;
    }
#if LMM_ANAT
    if (an) {
      unsigned ks = 0;
#pragma unroll
      for (int u = 0; u < F; u++)
        ks += kt[u] + cg[u];
      ANAT_LVL(*aa, 7, ks);
    }
#endif
    unsigned needm = 0;
#pragma unroll
    for (int u = 0; u < F; u++) {
      bool need = tt[u] == kUnvoted;  // (rows >= whi carry kRetired)
      if (ch[u])
        need = !(kt[u] < sk[u]);
      else if (kBits && cg[u] == prev)
        need = true;
      needm |= unsigned(need) << u;
      if (kDiag == 1) {
        dg[0] += ch[u];
        dg[1] += tt[u] >= 0 && sk[u] == 0;
        dg[2] += need;
        if (need && tt[u] >= 0) {  // the targets whose voters need a re-vote (mm_vote_diagcount)
          atomicOr(reinterpret_cast<unsigned long long*>(&s.flagbits[tt[u] >> 6]), 1ull << (tt[u] & 63));
          dg[3] += sk[u] == 0;
        }
      }
    }
#pragma unroll 1
    for (int u = 0; u < F; u++) {
      const bool need = (needm >> u) & 1;
      const unsigned long long m = __ballot(need);
      if (need)
        qw[qn + __popcll(m & below)] = int(base + u * kWave + lane);
      qn += __popcll(m);
      if (qn >= kWave) {  // wave-uniform: resolve the newest 64
        __builtin_amdgcn_wave_barrier();
        qn -= kWave;
        nq += kWave;
        const int row = qw[qn + lane];
        __builtin_amdgcn_wave_barrier();
        int pc = -1;  // (kRdq) a constraint this lane's re-vote made ready
#if LMM_ANAT
        if (an) {
          aa->at = anat_now();
          wcnt[1]++;
        }
        if (kDiag == 0)
          vote_row<R, kRec, kRdq>(s, buf, round, row, st_rows, st_elems, key, &pc, an, ar);
        if (kRdq && kDiag == 0)
          rdq_push_lds(s, pc, round, rql);
        if (an)
          ANAT_LVL(*aa, 8, 0u);
#else
        if (kDiag == 0)
          vote_row<R, kRec, kRdq>(s, buf, round, row, st_rows, st_elems, key, &pc);
        if (kRdq && kDiag == 0)
          rdq_push_lds(s, pc, round, rql);
#endif
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#if LMM_ANAT
  if (an && qn > 0) {
    aa->at = anat_now();
    wcnt[1]++;
  }
  int pc = -1;
  if (kDiag == 0 && lane < qn)
    vote_row<R, kRec, kRdq>(s, buf, round, qw[lane], st_rows, st_elems, key, &pc, an, ar);
  __builtin_amdgcn_wave_barrier();
  if (kRdq && kDiag == 0)
    rdq_push_lds(s, pc, round, rql);
  if (an && qn > 0)
    ANAT_LVL(*aa, 8, 0u);
#else
  int pc = -1;
  if (kDiag == 0 && lane < qn)
    vote_row<R, kRec, kRdq>(s, buf, round, qw[lane], st_rows, st_elems, key, &pc);
  if (kRdq && kDiag == 0)
    rdq_push_lds(s, pc, round, rql);
#endif
  if (kDiag == 1 && s.vstat && round < kStatRounds) {
    int32_t* d = s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot);
    for (int k = 0; k < 4; k++) {
      const int t = grp_isum<kWave>(dg[k]);
      if (lane == 0 && t)
        atomicAdd(&d[k == 3 ? 6 : k], t);
    }
  }
  return nq + qn;
}

constexpr int kBitWords = 17408;  // LDS bitmap capacity of the multi-launch vote: 1,114,112 constraints

// The changed-constraint bitmap into LDS (16 B per thread per step).
#ifndef LMM_BITS_UNROLL
#define LMM_BITS_UNROLL 2  // steps with their loads in flight together (build knob, measurement)
#endif
// Every CU copies the same ~125 KB at the start of every vote; starting each workgroup's copy at its own offset
// lets an XCD's CUs miss on different lines of the freshly written bitmap instead of all waiting on the same
// ones: C2 25.50-25.59 ms (2 loads in flight) / 25.56-25.59 (1) against 25.76-25.88 without (same box; 2 loads
// in flight alone: 25.85); on a second box 25.30-25.31 against 25.45-25.50, 4 in flight 26.75 (stress 28.29
// vs 28.56).  Build knob LMM_BITS_STAGGER=0: the plain copy.
#ifndef LMM_BITS_STAGGER
#define LMM_BITS_STAGGER 1
#endif
// (the multi-launch vote instantiates the staggered copy; the persistent kernel keeps the plain one, whose
// registers it cannot spare at its 128-VGPR budget)
template <int B, bool kStagger = false, int kU = 1>
__device__ __forceinline__ void load_bits(const Dev& s, uint64_t* bits) {
  const int n16 = (s.nC + 127) / 128;
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(s.chgbits);
  uint4* dst = reinterpret_cast<uint4*>(bits);
  const int off = kStagger && n16 > 0 ? int((int64_t(blockIdx.x) * 4099 * B) % n16) : 0;
  for (int i0 = threadIdx.x; i0 < n16; i0 += kU * B) {
    uint4 t[kU];
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (i0 + u * B < n16) {
        const int i = kStagger ? (i0 + u * B + off) % n16 : i0 + u * B;
        t[u] = src[i];
      }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (i0 + u * B < n16) {
        const int i = kStagger ? (i0 + u * B + off) % n16 : i0 + u * B;
        dst[i] = t[u];
      }
  }
}

// Vote diagnostics (measurement only): the constraints flagged by the filter pass (targets of queued rows,
// flagbits) -> their count and the sum of their CSC degrees and voters' share, per round; clears the flags.
__global__ void __launch_bounds__(kBlock) mm_vote_diagcount(Dev s, int round) {
  int nf = 0, deg = 0;
  for (int64_t w = int64_t(blockIdx.x) * kBlock + threadIdx.x; w < (s.nC + 63) / 64; w += int64_t(gridDim.x) * kBlock) {
    unsigned long long m = s.flagbits[w];
    s.flagbits[w] = 0;
    while (m) {
      const int b = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int64_t c = w * 64 + b;
      nf++;
      deg += int(s.cnst_ptr[c + 1] - s.cnst_ptr[c]);
    }
  }
  nf = grp_isum<kWave>(nf);
  deg = grp_isum<kWave>(deg);
  if ((threadIdx.x & (kWave - 1)) == 0 && s.vstat && round < kStatRounds) {
    int32_t* d = s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot);
    atomicAdd(&d[4], nf);
    atomicAdd(&d[5], deg);
  }
}

// Multi-launch engine, short rows (mean length <= 8): one 1024-thread workgroup per CU (the bitmap takes up
// to kBitWords * 8 B of LDS), one contiguous chunk of rows per workgroup.
constexpr int kVBlock = 1024;
// LMM_VOTE_PRE: the first filter step's loads issued before the bitmap copy (build knob, measurement).  Round 5, same
// box: 24.313 / 24.390 ms against 24.340 / 24.309 without (neutral: the copy is not the vote's critical path); off.
#ifndef LMM_VOTE_PRE
#define LMM_VOTE_PRE 0
#endif
template <int B, bool kBits, int kDiag = 0, bool kRec = false, bool kRdq = false>
__global__ void __launch_bounds__(B) mm_vote_lane(Dev s, int round) {
#if LMM_ANAT
  unsigned long long* arec = kDiag == 0 ? anat_rec(s, anat_slot(s, round), ANAT_VOTE) : nullptr;
  const bool an = arec != nullptr;
  AnatAcc aa{}, ar{};
  unsigned wcnt[2] = {0, 0};
  const unsigned long long t_in = an ? anat_now() : 0;
#endif
  if (s.ctl[CTL_DONE])
    return;
  const int buf = s.ctl[CTL_BUF];
  __shared__ int st_rows, st_elems;
  __shared__ int q[(B / kWave) * kQW];  // per-wave queues of rows to re-vote
  __shared__ __attribute__((aligned(16))) uint64_t bits[kBits ? kBitWords : 2];
  __shared__ RdqLds rql;  // (kRdq) the constraints this workgroup's re-votes made ready
  if (threadIdx.x == 0) {
    st_rows = st_elems = 0;
    rql.n = 0;
  }
  const int64_t nrows = s.ctl[CTL_NROWS + buf];
  const int64_t per = ((nrows + gridDim.x - 1) / gridDim.x + kWave - 1) / kWave * kWave;  // rows per workgroup
  const int64_t lo = int64_t(blockIdx.x) * per;
  const int64_t hi = lo + per < nrows ? lo + per : nrows;
  constexpr bool kPre = LMM_VOTE_PRE != 0 && kBits && kDiag == 0;
  int tt0[kPre ? kFilt : 1];
  unsigned sk0[kPre ? kFilt : 1];
  if (kPre) {  // the wave's first filter step, in flight during the bitmap copy
    int64_t wlo, whi;
    vote_wave_range(lo, hi, wlo, whi);
#pragma unroll
    for (int u = 0; u < (kPre ? kFilt : 1); u++) {
      const int64_t row = wlo + u * kWave + (threadIdx.x & (kWave - 1));
      tt0[u] = row < whi ? s.rtgt[buf][row] : kRetired;
      sk0[u] = row < whi ? unsigned(s.skey[buf][row]) : 1u;
    }
  }
  if (kBits)
    load_bits<B, LMM_BITS_STAGGER != 0, LMM_BITS_UNROLL>(s, bits);
  __syncthreads();
#if LMM_ANAT
  const unsigned long long t_bits = an ? anat_now() : 0;
#endif
  if (kDiag == 2) {  // measurement only: the bitmap load alone, and the changed-constraint count
    if (kBits && blockIdx.x == 0 && s.vstat && round < kStatRounds) {
      int pc = 0;
      for (int i = threadIdx.x; i < (s.nC + 63) / 64; i += B)
        pc += __popcll(bits[i]);
      atomicAdd(s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot) + 3, pc);
    }
    if (threadIdx.x == 0 && bits[1] == 0x5a5a5a5a5a5a5a5aull)  // keeps the load
      s.ctl[CTL_WORDS - 1] = 1;
    return;
  }
#if LMM_ANAT
  int nq = 0;
  if (lo < hi)
    nq = vote_waves<kBits, 8, kFilt, kDiag, kRec, kRdq, kPre>(s, buf, round, lo, hi, bits,
                                                              q + (threadIdx.x / kWave) * kQW, &st_rows, &st_elems,
                                                              s.key, tt0, sk0, &rql, an, &aa, &ar, wcnt);
  if (kRdq && kDiag == 0)
    rdq_flush_lds(s, round, &rql);
  if (an) {  // the wave's record (vote_row's levels: the slowest lane of the wave)
    const unsigned long long t_out = anat_now();
    unsigned lv[6];
#pragma unroll
    for (int i = 0; i < 6; i++)
      lv[i] = anat_wmax(ar.lv[i]);
    int64_t wlo, whi;
    vote_wave_range(lo, hi, wlo, whi);
    if ((threadIdx.x & (kWave - 1)) == 0) {
      arec[0] = t_in;
      arec[1] = t_out;
      arec[2] = blockIdx.x;
      arec[3] = t_bits;
      arec[4] = wcnt[0];
      arec[5] = aa.lv[6];
      arec[6] = aa.lv[7];
      arec[7] = wcnt[1];
      arec[8] = aa.lv[8];
#pragma unroll
      for (int i = 0; i < 6; i++)
        arec[9 + i] = lv[i];
      arec[15] = unsigned(nq);
      arec[16] = whi > wlo ? unsigned(whi - wlo) : 0u;
    }
  }
#else
  if (lo < hi)
    vote_waves<kBits, 8, kFilt, kDiag, kRec, kRdq, kPre>(s, buf, round, lo, hi, bits, q + (threadIdx.x / kWave) * kQW,
                                                         &st_rows, &st_elems, s.key, tt0, sk0, &rql);
  if (kRdq && kDiag == 0)
    rdq_flush_lds(s, round, &rql);
#endif
  if (s.vstat && kDiag == 0) {
    __syncthreads();
    if (threadIdx.x == 0 && round < kStatRounds && blockIdx.x < kMaxBlocks) {
      s.vstat[2 * (int64_t(round) * kMaxBlocks + blockIdx.x)] = st_rows;
      s.vstat[2 * (int64_t(round) * kMaxBlocks + blockIdx.x) + 1] = st_elems;
    }
  }
}

// Round phase 2 — ready list: alive constraints every alive element votes for.  Block b scans one
// contiguous chunk of the alive-constraint list and writes its ready constraints into its own segment
// of `ready` (LDS counter, no global atomic); bready[b] = segment length.
__device__ __forceinline__ int64_t chunk_of(int64_t n, int nblocks) { return (n + nblocks - 1) / nblocks; }

__global__ void __launch_bounds__(kBlock) mm_ready(Dev s) {
  if (s.ctl[CTL_DONE])
    return;
  const int cb = s.ctl[CTL_CB];
  __shared__ int cnt;
  if (threadIdx.x == 0)
    cnt = 0;
  __syncthreads();
  const int64_t n = s.ctl[CTL_NCL0 + cb];
  const int64_t chunk = chunk_of(n, gridDim.x);
  const int64_t lo = int64_t(blockIdx.x) * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const int32_t c = s.clist[cb][i];
    if (s.key[c] != kDeadKey && s.nvote[c] == 0)
      s.ready[lo + atomicAdd(&cnt, 1)] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    s.bready[blockIdx.x] = cnt;
}


// Round phase 3 — saturation of the ready constraints (maxmin.cpp:578-606): sat_block for the persistent
// engine (ready test fused in), mm_saturate over mm_ready's list for the multi-launch engine.

// Round phase 3 — saturate the ready constraints: maxmin.cpp:578-606.
// K waves per ready constraint c (K = the host's estimate of c's 64-element CSC chunks), wave k taking
// chunks k, k + K, ...  Per chunk: lanes claim the alive variables (atomicCAS: a duplicate element
// claims once, also across the waves of c), fix them at ratio/penalty; then the claimed variables'
// CSR elements are flattened over the wave (wave prefix of the row lengths in LDS, owner lane found by
// binary search), kSatU x kWave elements at a time so that their gathers are in flight together, and
// each element's three pushes are issued by a quad of lanes into the constraint's 32-B record (ONE
// atomic request per element; scripts/ubench_atomic.hip).  Decrements to c itself are skipped: c
// leaves the light table (every alive variable on it is fixed, usage -> 0, maxmin.cpp:608-615).
// c's ratio is left in place (the other waves of c read it; the dead key hides it from later readers).
#ifndef LMM_KSATU
#define LMM_KSATU 4  // (build knob, measurement)
#endif
constexpr int kSatU = LMM_KSATU;

// (LMM_ANAT: `an` = stamp the chunk's dependent levels into aa: lv[1] CSC element loads, lv[2] variable states and
// claims, lv[3] the claimed rows' elements, lv[4] their constraints' words, lv[5] the pushes; wc[1] chunks, wc[2]
// fixed variables, wc[3] pushed elements)
#if LMM_ANAT
#define SC_ANAT_PARAMS , bool an = false, AnatAcc* aa = nullptr, unsigned* wc = nullptr
#define SC_ANAT_ARGS , an, aa, wc
#define SC_LVL(i, dep)       \
  do {                       \
    if (an)                  \
      ANAT_LVL(*aa, i, dep); \
  } while (0)
#else
#define SC_ANAT_PARAMS
#define SC_ANAT_ARGS
#define SC_LVL(i, dep) \
  do {                 \
  } while (0)
#endif
__device__ __forceinline__ void saturate_chunk(const Dev& s, int32_t c, double r, uint32_t j0, uint32_t ce,
                                               int round, int lane, int* pre, bool dup SC_ANAT_PARAMS) {
#if LMM_ANAT
  if (an) {
    aa->at = anat_now();
    wc[1]++;
  }
#endif
  const int q = lane & 3;
  const uint32_t j = j0 + lane;
  int32_t lv = -1;
  double lp = 1.0, lx = 0.0;
  uint32_t rb = 0, re = 0;
  if (j < ce) {
    // the variable's penalty and CSR row come with the element (coalesced, csc_p / csc_row): no gather after
    // the claim (round 3; gathering them there cost C2 one more dependent random read per fixed variable)
    lv = s.csc_v[j];
    lp = s.csc_p[j];
    const unsigned long long row = s.csc_row[j];
    rb = uint32_t(row);
    re = uint32_t(row >> 32);
  }
  SC_LVL(1, uint32_t(lv) + rb + re);
  if (j < ce) {
    if (s.vstate[lv] != 0)
      lv = -1;
    else if (!dup)
      s.vstate[lv] = round + 1;
    else if (atomicCAS(&s.vstate[lv], 0, round + 1) != 0)
      lv = -1;
  }
  int len = 0;
  if (lv >= 0) {
    lx = r / lp;
    s.x[lv] = lx;
    len = int(re - rb);
  } else {
    rb = re = 0;
  }
#if LMM_ANAT
  if (an) {
    ANAT_LVL(*aa, 2, lv);
    wc[2] += unsigned(__popcll(__ballot(lv >= 0)));
  }
#endif
  int incl = len;  // inclusive wave scan of the row lengths
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int t = __shfl_up(incl, o, kWave);
    if (lane >= o)
      incl += t;
  }
  const int total = __shfl(incl, kWave - 1, kWave);
  pre[lane] = incl - len;  // exclusive prefix (non-decreasing in lane)
  __builtin_amdgcn_wave_barrier();
  for (int f0 = 0; f0 < total; f0 += kSatU * kWave) {  // wave-uniform
    int32_t cc[kSatU];
    uint32_t kk[kSatU];
    int ol[kSatU];
    double ww[kSatU];
#pragma unroll
    for (int u = 0; u < kSatU; u++) {  // owner lanes and element indices, then independent gathers
      const int f = f0 + u * kWave + lane;
      int o = 0;  // owner lane: last lane with pre <= f
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1)
        if (pre[o + step] <= f)
          o += step;
      ol[u] = o;
      kk[u] = uint32_t(__shfl(int(rb), o, kWave)) + uint32_t(f - pre[o]);
      cc[u] = f < total ? s.csr_c[kk[u]] : -1;
      ww[u] = f < total ? s.csr_w[kk[u]] : 0.0;  // with the constraint id: one round trip
    }
#if LMM_ANAT
    if (an) {
      double sw = 0.0;
#pragma unroll
      for (int u = 0; u < kSatU; u++)
        sw += ww[u] + double(cc[u]);
      ANAT_LVL(*aa, 3, sw);
    }
#endif
    long long a0[kSatU], a1[kSatU];  // fixed-point decrements (CstRec)
    bool fat[kSatU];
#pragma unroll
    for (int u = 0; u < kSatU; u++) {
      const double ox = __shfl(lx, ol[u], kWave);
      const double op = __shfl(lp, ol[u], kWave);
      fat[u] = false;
      a0[u] = a1[u] = 0;
      const int32_t ce = cc[u] >= 0 ? s.cexp[cc[u]] : kCexpDead;  // scales, policy and liveness in one word
      if (cc[u] >= 0 && (cc[u] == c || (ce & kCexpDead)))
        cc[u] = -1;
      if (cc[u] >= 0) {
        s.ctouch[cc[u]] = 1;  // receives decrements this round (mm_update reads its record)
        fat[u] = ce & kCexpFat;
        const double w = ww[u];
        a0[u] = (long long)dec_q(w * ox, cexp_rem(ce));
        a1[u] = fat[u] ? (long long)fat_bits(w / op) : (long long)dec_q(w / op, cexp_use(ce));
      }
    }
#if LMM_ANAT
    if (an) {
      long long sa = 0;
#pragma unroll
      for (int u = 0; u < kSatU; u++) {
        sa += a0[u] + a1[u];
        wc[3] += unsigned(__popcll(__ballot(cc[u] >= 0)));
      }
      ANAT_LVL(*aa, 4, sa);
    }
#endif
#pragma unroll
    for (int u = 0; u < kSatU; u++) {
      const int nel = total - f0 - u * kWave;
#pragma unroll
      for (int t = 0; t < kWave / 16; t++) {
        if (t * 16 >= nel)
          break;
        const int e = t * 16 + (lane >> 2);
        const int ec = __shfl(cc[u], e, kWave);
        const int ef = __shfl(int(fat[u]), e, kWave);
        const long long e0 = __shfl(a0[u], e, kWave);
        const long long e1 = __shfl(a1[u], e, kWave);
        if (ec >= 0 && q < 3 && (!ef || q == 2))
          atomicAdd(&s.cst[ec].drem + q, (unsigned long long)(q == 0 ? e0 : q == 1 ? e1 : 1ll));
        if (ec >= 0 && ef && q == 1)  // FATPIPE: the removed w/p (fat_bits)
          atomicMax(&s.cst[ec].duse, (unsigned long long)e1);
      }
    }
    SC_LVL(5, 0u);
  }
  __builtin_amdgcn_wave_barrier();
}

// Ready test + saturation, block-cooperative.  In pass p, wave w of workgroup b tests the 64 constraints of
// group (p * NBW + w) * grid + b (consecutive groups on different workgroups, so the ready constraints spread
// over the chip; lanes stay coalesced); entries are list positions (cl) or identity ids (cl == nullptr).  The
// ready ones of all the workgroup's passes are collected in LDS with the prefix of their 64-element CSC
// chunks (up to CAP at a time), then the workgroup's waves take the chunks round-robin: a high-degree
// constraint (a fat-tree core link) spreads over the waves instead of serialising one, and the saturation
// chains of many constraints run side by side.  Ready constraints share no alive variable (each alive
// variable votes for exactly one), so claims never race between them.  c leaves the light table:
// ctouch[c] = 2 tells mm_update (the owner of key / chg) to retire it; c's ratio is left in place.
template <int NB, int CAP> struct SatLds {
  int32_t rc[CAP];      // collected ready constraints
  int32_t rr[CAP + 1];  // exclusive prefix of their chunk counts
  int wa[NB / kWave], wb[NB / kWave];
  int na, nb;           // collected constraints / chunks
  int pre[NB / kWave][kWave];  // saturate_chunk's per-wave row-length prefix
};

template <int NB, int CAP>
__device__ __forceinline__ void sat_flush(const Dev& s, int round, SatLds<NB, CAP>& L) {
  constexpr int NBW = NB / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int ta = L.na, tb = L.nb;
  for (int g = w; g < tb; g += NBW) {  // wave-uniform
    int k = 0;  // last collected entry whose first chunk is <= g
#pragma unroll
    for (int step = CAP / 2; step > 0; step >>= 1)
      if (k + step < ta && L.rr[k + step] <= g)
        k += step;
    const int32_t cc = L.rc[k];
    const int ch = g - L.rr[k];
    const double r = ld_rlx(&s.cst[cc].ratio);  // wave-uniform address: keep it off the scalar cache
    saturate_chunk(s, cc, r, s.cnst_ptr[cc] + uint32_t(ch) * kWave, s.cnst_ptr[cc + 1], round, lane, L.pre[w],
                   s.cdup[cc] != 0);
    if (ch == 0 && lane == 0)
      s.ctouch[cc] = 2;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    L.na = L.nb = 0;
  __syncthreads();
}

// Returns whether the workgroup found a ready constraint.
template <int NB, int CAP>
__device__ __forceinline__ bool sat_block(const Dev& s, int round, const int32_t* __restrict__ cl, int64_t n,
                                          SatLds<NB, CAP>& L) {
  static_assert(CAP >= NB, "one pass must fit");
  constexpr int NBW = NB / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (threadIdx.x == 0)
    L.na = L.nb = 0;
  __syncthreads();
  bool any = false;
  for (int64_t p = 0; p * NB * gridDim.x < n; p++) {  // workgroup-uniform
    const int64_t i = ((p * NBW + w) * gridDim.x + blockIdx.x) * kWave + lane;
    int32_t c = -1;
    if (i < n)
      c = cl ? cl[i] : int32_t(i);
    const bool rdy = c >= 0 && s.key[c] != kDeadKey && s.nvote[c] == 0;
    const int nch = rdy ? int((s.cnst_ptr[c + 1] - s.cnst_ptr[c] + kWave - 1) / kWave) : 0;
    int ia = rdy, ib = nch;  // block exclusive scans of (ready, chunks)
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int xa = __shfl_up(ia, o, kWave), xb = __shfl_up(ib, o, kWave);
      if (lane >= o) {
        ia += xa;
        ib += xb;
      }
    }
    if (lane == kWave - 1) {
      L.wa[w] = ia;
      L.wb[w] = ib;
    }
    __syncthreads();
    int oa = L.na, ob = L.nb, ta = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < NBW; k++) {
      oa += k < w ? L.wa[k] : 0;
      ob += k < w ? L.wb[k] : 0;
      ta += L.wa[k];
      tb += L.wb[k];
    }
    if (rdy) {
      L.rc[oa + ia - 1] = c;
      L.rr[oa + ia - 1] = ob + ib - nch;
    }
    any |= ta > 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      L.na += ta;
      L.nb += tb;
    }
    __syncthreads();
    if (L.na > CAP - NB)  // workgroup-uniform: the next pass might not fit
      sat_flush<NB, CAP>(s, round, L);
  }
  if (L.na)
    sat_flush<NB, CAP>(s, round, L);
  return any;
}

// Multi-launch engine: saturation of mm_ready's list, K waves per ready constraint (chunks k, k + K, ...)
// spread evenly over the whole grid — the ready list is global here, so the work balances across workgroups.
template <int K> __device__ __forceinline__ void saturate_one(const Dev& s, int32_t c, int k, int round, int lane,
                                                              int* pre) {
  const double r = ld_rlx(&s.cst[c].ratio);  // wave-uniform address: keep it off the scalar cache
  const uint32_t ce = s.cnst_ptr[c + 1];
  const bool dup = s.cdup[c] != 0;
  for (uint32_t base = s.cnst_ptr[c] + uint32_t(k) * kWave; base < ce; base += K * kWave)  // wave-uniform
    saturate_chunk(s, c, r, base, ce, round, lane, pre, dup);
  if (k == 0 && lane == 0)  // c leaves the light table: mm_update (the owner of key / chg) retires it
    s.ctouch[c] = 2;
}
// (the same with the constraint's ratio, CSC range and duplicate flag already loaded)
template <int K> __device__ __forceinline__ void saturate_one_pre(const Dev& s, int32_t c, int k, int round, int lane,
                                                                  int* pre, double r, uint32_t cb, uint32_t ce,
                                                                  bool dup SC_ANAT_PARAMS) {
  for (uint32_t base = cb + uint32_t(k) * kWave; base < ce; base += K * kWave)  // wave-uniform
    saturate_chunk(s, c, r, base, ce, round, lane, pre, dup SC_ANAT_ARGS);
  if (k == 0 && lane == 0)
    s.ctouch[c] = 2;
}

// K waves per ready constraint: every block rebuilds the exclusive prefix of the per-segment ready
// counts in LDS (parallel: 8 segments per thread, wave shuffles, one LDS exchange) and maps its waves
// onto the ready list by binary search.
template <int K> __global__ void __launch_bounds__(kBlock) mm_saturate(Dev s, int round, int ready_blocks) {
  if (s.ctl[CTL_DONE])
    return;
  const int cb = s.ctl[CTL_CB];
  __shared__ int pre[kMaxBlocks + 1];
  __shared__ int wsum[kBlock / kWave];
  __shared__ int wpre[kBlock / kWave][kWave];  // per-wave row-length prefix (saturate_chunk)
  constexpr int kPer = kMaxBlocks / kBlock;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int loc[kPer];
  int sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int seg = threadIdx.x * kPer + k;
    loc[k] = seg < ready_blocks ? s.bready[seg] : 0;
    sum += loc[k];
  }
  int incl = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int t = __shfl_up(incl, o, kWave);
    if (lane >= o)
      incl += t;
  }
  if (lane == kWave - 1)
    wsum[w] = incl;
  __syncthreads();
  int acc = incl - sum, total = 0;
#pragma unroll
  for (int i = 0; i < kBlock / kWave; i++) {
    acc += i < w ? wsum[i] : 0;
    total += wsum[i];
  }
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    pre[threadIdx.x * kPer + k] = acc;
    acc += loc[k];
  }
  __syncthreads();
  if (total && blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_LASTR] = round;  // plain store: this round fixes variables
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  const int64_t chunk = chunk_of(s.ctl[CTL_NCL0 + cb], ready_blocks);
  for (int64_t g = wave; g < int64_t(total) * K; g += nwaves) {
    const int64_t i = g / K;
    const int k = int(g % K);
    int lo = 0;  // last segment with pre[seg] <= i
#pragma unroll
    for (int step = kMaxBlocks / 2; step > 0; step >>= 1)
      if (lo + step < ready_blocks && pre[lo + step] <= i)
        lo += step;
    saturate_one<K>(s, s.ready[lo * chunk + (i - pre[lo])], k, round, lane, wpre[w]);
  }
}


// Saturation without the mm_ready pass (LMMHIP_RDQ): the update's per-workgroup candidate segments (ublocks of
// them, mm_saturate's prefix and binary search over their counts) then the vote's queue; K waves per entry;
// an entry is saturated when it is still alive with nothing voting elsewhere (every vote of the round is in).
// Block 0 empties the other parity's vote queue, which the next round's vote fills.
// A candidate's ratio, CSC range and duplicate flag are loaded with its key and vote count (round 5, same box, two
// passes, profiles/r05_ab_c2_spec2.json: C2 24.285-24.293 ms against 24.309-24.340 without).  LMM_SATQ_PIPE (build
// knob): the next task's candidate state loaded ahead (round 6).  Also measured in round 6 and removed: a batched form
// (a wave's 64 tasks' states in one load, the ready tasks' first chunks 2 / 4 at a time, the claimed variables gathered
// in LDS and pushed 64 at a time; with 64- or 32-element chunks): 23.54-23.68 ms against 23.53 on the same box.
#ifndef LMM_SATQ_PIPE
#define LMM_SATQ_PIPE 1
#endif
template <int K> __global__ void __launch_bounds__(kBlock) mm_saturate_q(Dev s, int round, int ublocks) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_SAT);
  const bool an = arec != nullptr;
  AnatAcc aa_s{};
  AnatAcc* aa = &aa_s;
  unsigned wc[4] = {0, 0, 0, 0};  // candidates, chunks, fixed variables, pushed elements
  const unsigned long long t_in = an ? anat_now() : 0;
#endif
  if (s.ctl[CTL_DONE])
    return;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_RDQ0 + ((round + 1) & 1)] = 0;
  __shared__ int wpre[kBlock / kWave][kWave];  // per-wave row-length prefix (saturate_chunk)
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  __shared__ int pre[kMaxBlocks + 1];
  __shared__ int wsum[kBlock / kWave];
  constexpr int kPer = kMaxBlocks / kBlock;
  int loc[kPer];
  int sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int seg = threadIdx.x * kPer + k;
    loc[k] = seg < ublocks ? s.ucnt[seg] : 0;
    sum += loc[k];
  }
  int incl = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int t = __shfl_up(incl, o, kWave);
    if (lane >= o)
      incl += t;
  }
  if (lane == kWave - 1)
    wsum[w] = incl;
  __syncthreads();
  int acc = incl - sum, total = 0;
#pragma unroll
  for (int i = 0; i < kBlock / kWave; i++) {
    acc += i < w ? wsum[i] : 0;
    total += wsum[i];
  }
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    pre[threadIdx.x * kPer + k] = acc;
    acc += loc[k];
  }
  __syncthreads();
#if LMM_ANAT
  const unsigned long long t_pre = an ? anat_now() : 0;
#endif
  const int nq = s.ctl[CTL_RDQ0 + (round & 1)];
  const int32_t* __restrict__ q = s.rdq[round & 1];
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  const int64_t T = (int64_t(total) + nq) * K;  // tasks: (candidate, wave k of its K)
  auto cand_of = [&](int64_t g) -> int32_t {   // the candidate of task g: the update's segments, then the vote's queue
    const int64_t i = g / K;
    if (i >= total)
      return q[i - total];
    int lo = 0;  // last segment with pre[seg] <= i
#pragma unroll
    for (int step = kMaxBlocks / 2; step > 0; step >>= 1)
      if (lo + step < ublocks && pre[lo + step] <= i)
        lo += step;
    return s.useg[int64_t(lo) * kUSeg + (i - pre[lo])];
  };
#if LMM_SATQ_PIPE
  // Software-pipelined over the wave's tasks (round 6): the next task's candidate state (key, vote count, ratio, CSC
  // range, duplicate flag) and the candidate id of the task after it are loaded before this task's chunks, so a task
  // starts with its CSC element loads instead of two dependent levels (candidate id, then its state).  The round
  // anatomy (profiles/r06_c2_round_anatomy.json) shows a tail-round wave running ~9 tasks one after the other.
  struct CandSt {
    int32_t c;
    unsigned kc;
    int nv;
    double r;
    uint32_t cb, ce;
    bool dup;
  };
  auto state_of = [&](int32_t c) -> CandSt {
    CandSt x;
    x.c = c;
    if (c < 0) {
      x.kc = kDeadKey;
      x.nv = 1;
      x.r = 0.0;
      x.cb = x.ce = 0;
      x.dup = false;
      return x;
    }
    x.kc = s.key[c];
    x.nv = s.nvote[c];
    x.r = ld_rlx(&s.cst[c].ratio);
    x.cb = s.cnst_ptr[c];
    x.ce = s.cnst_ptr[c + 1];
    x.dup = s.cdup[c] != 0;
    return x;
  };
  CandSt cur = state_of(wave < T ? cand_of(wave) : -1);
  int32_t cnext = wave + nwaves < T ? cand_of(wave + nwaves) : -1;
  for (int64_t g = wave; g < T; g += nwaves) {  // wave-uniform
    const int k = int(g % K);
#if LMM_ANAT
    if (an) {
      aa->at = anat_now();
      wc[0]++;
    }
#endif
    SC_LVL(6, cur.r + double(cur.kc + unsigned(cur.nv) + cur.cb + cur.ce + unsigned(cur.dup)));
    const CandSt nxt = state_of(cnext);  // (issued before this task's chunk loads)
    cnext = g + 2 * nwaves < T ? cand_of(g + 2 * nwaves) : -1;
    if (cur.kc != kDeadKey && cur.nv == 0) {  // (the round's CTL_LASTR: mm_update, from the constraints saturated here)
      saturate_one_pre<K>(s, cur.c, k, round, lane, wpre[w], cur.r, cur.cb, cur.ce, cur.dup SC_ANAT_ARGS);
    }
    cur = nxt;
  }
#else
  for (int64_t g = wave; g < T; g += nwaves) {  // wave-uniform
    const int k = int(g % K);
#if LMM_ANAT
    if (an) {
      aa->at = anat_now();
      wc[0]++;
    }
#endif
    const int32_t c = cand_of(g);
    SC_LVL(0, c);
    // the constraint's ratio, CSC range and duplicate flag loaded with its key and count (one dependent level less;
    // a candidate that is not ready discards them)
    const unsigned kc = s.key[c];
    const int nv = s.nvote[c];
    const double r = ld_rlx(&s.cst[c].ratio);
    const uint32_t cb = s.cnst_ptr[c], cend = s.cnst_ptr[c + 1];
    const bool dup = s.cdup[c] != 0;
    SC_LVL(6, r + double(kc + unsigned(nv) + cb + cend + unsigned(dup)));
    if (kc == kDeadKey || nv != 0)
      continue;
    saturate_one_pre<K>(s, c, k, round, lane, wpre[w], r, cb, cend, dup SC_ANAT_ARGS);
  }
#endif
#if LMM_ANAT
  if (an && lane == 0) {
    arec[0] = t_in;
    arec[1] = anat_now();
    arec[2] = blockIdx.x;
    arec[3] = t_pre;
    for (int f = 0; f < 7; f++)
      arec[4 + f] = aa->lv[f];
    for (int f = 0; f < 4; f++)
      arec[11 + f] = wc[f];
  }
#endif
}

// Round phase 4 — constraint update: maxmin.cpp:603-658, one wave = 64 consecutive constraints (identity
// order), so the changed-constraint bitmap the next vote reads is one ballot per wave.  A bit is set when
// the constraint's 16-bit KEY changed or it left the light table (the only events that can move a
// non-sensitive vote, vote_row); chg[c] = round marks every touched constraint (sensitive rows).
// FATPIPE usage is recomputed wave-cooperatively: max w/p over the elements whose variable is still at
// 0 (maxmin.cpp:625-658), 64 elements per step.  Returns (per lane) alive constraints; *touch = some
// constraint of the wave was touched.
// K groups of 64 constraints (base0 + k * stride) at once: every load of the K groups (key and touch
// flag, then — touched constraints only — record, flags, scale, votes) is issued before any of them is
// used, so a wave keeps K times the memory requests in flight.
// (LMM_ANAT: `an` = stamp the steps into aa: lv[0] keys and touch flags, lv[1] touched records, lv[2] the rest;
// wc[0] steps, wc[1] touched constraints)
template <int K, bool kRdq = false>
__device__ __forceinline__ int update_groups(const Dev& s, int64_t base0, int64_t stride, int round, double prec,
                                             bool* touch, int* ucnt_sh = nullptr, int32_t* ulist = nullptr
#if LMM_ANAT
                                             , bool an = false, AnatAcc* aa = nullptr, unsigned* wc = nullptr
#endif
) {
  const int lane = threadIdx.x & (kWave - 1);
#if LMM_ANAT
  if (an) {
    aa->at = anat_now();
    wc[0]++;
  }
#endif
  unsigned okey[K], tf[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int64_t c = base0 + k * stride + lane;
    okey[k] = c < s.nC ? unsigned(s.key[c]) : kDeadKey;
    tf[k] = c < s.nC ? unsigned(s.ctouch[c]) : 0u;  // 1 = received decrements, 2 = saturated this round
  }
#if LMM_ANAT
  if (an) {
    unsigned ks = 0;
#pragma unroll
    for (int k = 0; k < K; k++)
      ks += okey[k] + tf[k];
    ANAT_LVL(*aa, 0, ks);
  }
#endif
  unsigned long long qx[K], qy[K], qz[K];
  double rem[K], use[K], bnd[K];
  int32_t ce[K], nv[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int64_t c = base0 + k * stride + lane;
    qx[k] = qy[k] = qz[k] = 0;
    rem[k] = use[k] = bnd[k] = 0.0;
    ce[k] = nv[k] = 0;
    if (okey[k] != kDeadKey && tf[k] == 1) {  // an untouched constraint keeps its record as it is
      const CstRec* rec = s.cst + c;
      qx[k] = rec->drem;
      qy[k] = rec->duse;
      qz[k] = rec->dcnt;
      rem[k] = rec->rem;
      use[k] = rec->use;
      bnd[k] = rec->bound;
      ce[k] = s.cexp[c];
      nv[k] = s.nvote[c];
    }
  }
#if LMM_ANAT
  if (an) {
    double rs = 0.0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      rs += rem[k] + use[k] + bnd[k] + double(qx[k] + qy[k] + qz[k]) + double(ce[k] + nv[k]);
      wc[1] += unsigned(__popcll(__ballot(okey[k] != kDeadKey && tf[k] == 1)));
    }
    ANAT_LVL(*aa, 1, rs);
  }
#endif
  int alive = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int64_t gbase = base0 + k * stride;
    if (gbase >= s.nC)  // wave-uniform
      break;
    const int64_t c = gbase + lane;
    const bool live0 = okey[k] != kDeadKey;
    const bool sat = live0 && tf[k] == 2;
    const bool live = live0 && !sat;
    const bool tch = live && tf[k] == 1;
    const bool fat = tch && (ce[k] & kCexpFat);
    // FATPIPE: recompute only when a removed element reached the usage (fat_bits in duse)
    const bool fre = fat && !(__longlong_as_double((long long)qy[k]) < use[k]);
    double fuse = use[k];
    unsigned long long fm = __ballot(fre);
    while (fm) {  // wave-uniform: FATPIPE usage over the still-unfixed elements (maxmin.cpp:625-658)
      const int l = __ffsll((long long)fm) - 1;
      fm &= fm - 1;
      const int64_t cl = gbase + l;
      const uint32_t b = s.cnst_ptr[cl], e = s.cnst_ptr[cl + 1];
      double m = 0.0;
      // (the element's w/p loaded with its variable: no branch between a load and the next one)
      for (uint32_t j = b + lane; j < e; j += kWave) {
        const double u = s.csc_u[j];
        m = !(s.x[s.csc_v[j]] > 0) ? fmax(m, u) : m;
      }
      m = wave_max(m);
      if (lane == l)
        fuse = m;
    }
    bool changed = false;
    CstRec* rec = s.cst + c;
    if (sat) {
      *touch = true;  // (a saturation this round: the round's CTL_LASTR, set here instead of by every ready task)
      s.key[c] = kDeadKey;
      s.cexp[c] = kCexpDead;
      s.chg[c] = uint16_t(round);
      s.ctouch[c] = 0;
      rec->ratio = dinf();
      changed = true;
    } else if (live) {
      if (!tch) {
        alive++;
      } else {
        *touch = true;
        s.ctouch[c] = 0;
        rec->drem = rec->duse = rec->dcnt = 0;
        const int nvn = nv[k] - int(qz[k]);
        s.nvote[c] = nvn;
        s.chg[c] = uint16_t(round);
        double r0 = rem[k], u0;
        if (!fat) {
          u0 = use[k] - dec_val(qy[k], cexp_use(ce[k]));
          r0 -= dec_val(qx[k], cexp_rem(ce[k]));
          if (r0 < bnd[k] * prec)
            r0 = 0.0;
          if (u0 < prec)
            u0 = 0.0;
        } else {
          u0 = fuse;
        }
        rec->rem = r0;
        rec->use = u0;
        if (!(u0 > prec) || !(r0 > bnd[k] * prec)) {
          rec->ratio = dinf();
          s.key[c] = kDeadKey;
          s.cexp[c] = kCexpDead;
          changed = true;
        } else {
          const double r = r0 / u0;
          rec->ratio = r;
          const unsigned nk = ratio_key(r);
          s.key[c] = uint16_t(nk);
          changed = nk != okey[k];
          alive++;
          if (kRdq && nvn == 0) {  // its last elements voting elsewhere left with fixed variables: ready next
            const int slot = atomicAdd(ucnt_sh, 1);  // round (the stamp keeps the vote from queueing it too)
            ulist[slot] = int32_t(c);
            s.rqst[c] = round + 1;
          }
        }
      }
    }
    const unsigned long long word = __ballot(changed);
    if (lane == 0)
      s.chgbits[gbase >> 6] = word;
  }
#if LMM_ANAT
  if (an)
    ANAT_LVL(*aa, 2, alive);
#endif
  return alive;
}

// balive[block] = constraints of the block's range still in the light table (read by mm_done; plain
// stores, no global atomic).
// groups of 64 constraints per wave step, their loads in flight together (build knob, measurement).  Round 5, same
// box, two passes (scripts/gpu_r05_updk.sh, profiles/r05_ab_c2_updk.json): 4 -> C2 24.35-24.36 ms against
// 24.40-24.42 with 2 and 24.54-24.58 with 1 (at C2 a thread of the 1,024 update workgroups owns ~4 constraints:
// with 4 groups every load of the round's update is issued at once)
#ifndef LMM_UPD_K
#define LMM_UPD_K 4
#endif
template <bool kRdq = false> __global__ void __launch_bounds__(kBlock) mm_update(Dev s, int round, double prec) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_UPD);
  const bool an = arec != nullptr;
  AnatAcc aa{};
  unsigned wc[2] = {0, 0};
  const unsigned long long t_in = an ? anat_now() : 0;
#endif
  if (s.ctl[CTL_DONE])
    return;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_ROUNDS] += 1;
  __shared__ int alive_cnt, ucnt_sh;
  __shared__ int32_t ulist[kRdq ? kUSeg : 1];
  if (threadIdx.x == 0)
    alive_cnt = ucnt_sh = 0;
  __syncthreads();
  int alive = 0;
  bool any_touch = false;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t base = (int64_t(blockIdx.x) * kBlock + threadIdx.x) & ~int64_t(kWave - 1); base < s.nC;
       base += LMM_UPD_K * stride)  // wave-uniform; LMM_UPD_K groups of 64 constraints per step, loads in flight together
#if LMM_ANAT
    alive += update_groups<LMM_UPD_K, kRdq>(s, base, stride, round, prec, &any_touch, &ucnt_sh, ulist, an, &aa, wc);
  const unsigned long long t_loop = an ? anat_now() : 0;
#else
    alive += update_groups<LMM_UPD_K, kRdq>(s, base, stride, round, prec, &any_touch, &ucnt_sh, ulist);
#endif
  if (alive)
    atomicAdd(&alive_cnt, alive);
  __syncthreads();
  if (threadIdx.x == 0)
    s.balive[blockIdx.x] = alive_cnt;
  if (kRdq) {  // the workgroup's ready candidates for the next round into its segment
    const int n = ucnt_sh;
    for (int i = threadIdx.x; i < n; i += kBlock)
      s.useg[int64_t(blockIdx.x) * kUSeg + i] = ulist[i];
    if (threadIdx.x == 0)
      s.ucnt[blockIdx.x] = n;
  }
  if (__syncthreads_or(any_touch) && threadIdx.x == 0)
    s.ctl[CTL_LASTR] = round;  // plain store: the last round that changed a constraint
#if LMM_ANAT
  if (an && (threadIdx.x & (kWave - 1)) == 0) {
    arec[0] = t_in;
    arec[1] = anat_now();
    arec[2] = blockIdx.x;
    arec[3] = t_loop;
    for (int f = 0; f < 3; f++)
      arec[4 + f] = aa.lv[f];
    arec[7] = wc[0];
    arec[8] = wc[1];
  }
#endif
}

// Saturated set of the solved system: sat(c) = NOT double_positive(bound - U_c,
// bound * prec) with U_c = Constraint::get_usage() (maxmin.cpp:948-961: sum, or max for FATPIPE, of
// w * x over the enabled elements of weight > 0 — exactly the flattened CSC of c).  One wave per
// constraint.  FairBottleneck: sat(c) = c was erased (fair_bottleneck.cpp:129-140, ratio = +inf).
__global__ void __launch_bounds__(kBlock) mm_saturated(Dev s, double prec, int fair, uint8_t* out) {
  const int lane = threadIdx.x & (kWave - 1);
  for (int64_t c = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; c < s.nC;
       c += int64_t(gridDim.x) * (kBlock / kWave)) {
    if (fair) {
      if (lane == 0)
        out[c] = s.ratio[c] != 0.0;
      continue;
    }
    const bool fat = s.cflags[c] & 1;
    double u = 0.0;
    for (uint32_t j = s.cnst_ptr[c] + lane; j < s.cnst_ptr[c + 1]; j += kWave) {
      const double t = s.csc_w[j] * s.x[s.csc_v[j]];
      u = fat ? fmax(u, t) : u + t;
    }
    u = fat ? wave_max(u) : wave_sum(u);
    if (lane == 0) {
      const double b = s.cbound[c];
      out[c] = !((b - u) > b * prec);
    }
  }
}

// Variables of the solved system in the caller's id space: dense index d -> host slot (resident
// flatten: dv = exclusive scan of the membership mask vm), written at out[d] (ascending slots).
__global__ void __launch_bounds__(kBlock) rs_touched(int64_t nslots, const int64_t* vm, const int64_t* dv,
                                                     int32_t* out) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < nslots; v += int64_t(gridDim.x) * kBlock)
    if (vm[v])
      out[dv[v]] = int32_t(v);
}

// Termination (maxmin.cpp:680): no constraint left in the light table after the last update.
__global__ void __launch_bounds__(kBlock) mm_done(Dev s, int update_blocks) {
  int a = 0;
  for (int b = threadIdx.x; b < update_blocks; b += kBlock)
    a += s.balive[b];
  a = grp_isum<kWave>(a);
  __shared__ int w[kBlock / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0)
    w[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x == 0 && w[0] + w[1] + w[2] + w[3] == 0)
    s.ctl[CTL_DONE] = 1;
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
  a = sh[t] - a;
  b = sh[kBlock + t] - b;
  __syncthreads();
}

__device__ __forceinline__ bool row_alive(const Dev& s, int in, int64_t row) {
  return s.vstate[rvar(s.cvar[in][row])] == 0;
}

__global__ void __launch_bounds__(kBlock) cmp_count(Dev s) {
  if (s.ctl[CTL_DONE])
    return;
  const int in = s.ctl[CTL_BUF];
  __shared__ int sh[2 * kBlock];
  const int64_t nrows = s.ctl[CTL_NROWS + in];
  const int64_t r0 = int64_t(blockIdx.x) * kCompactRows + int64_t(threadIdx.x) * kRowsPerThread;
  // the thread's rows' loads issued together (ids, then states and row bounds), not one row's chain after another
  int32_t cv[kRowsPerThread];
#pragma unroll
  for (int k = 0; k < kRowsPerThread; k++)
    cv[k] = r0 + k < nrows ? s.cvar[in][r0 + k] : -1;
  bool al[kRowsPerThread];
  uint32_t rb[kRowsPerThread + 1];
#pragma unroll
  for (int k = 0; k < kRowsPerThread; k++)
    al[k] = r0 + k < nrows && s.vstate[rvar(cv[k])] == 0;
#pragma unroll
  for (int k = 0; k <= kRowsPerThread; k++)
    rb[k] = r0 + k <= nrows ? s.crow[in][r0 + k] : 0u;
  int nr = 0, ne = 0;
#pragma unroll
  for (int k = 0; k < kRowsPerThread; k++)
    if (al[k]) {
      nr++;
      ne += int(rb[k + 1] - rb[k]);
    }
  int a = nr, b = ne;
  block_scan2(a, b, sh);
  if (threadIdx.x == kBlock - 1) {
    s.bsum[2 * blockIdx.x] = a + nr;
    s.bsum[2 * blockIdx.x + 1] = b + ne;
  }
}

// Exclusive scan of the per-block counts, totals into the output buffer's words, and the decision: rewrite
// only when fewer than pct % of the scanned rows are alive (CTL_CMPGO).
__global__ void __launch_bounds__(1024) cmp_scan(Dev s, int nblk, int pct) {
  if (s.ctl[CTL_DONE])
    return;
  const int in = s.ctl[CTL_BUF], out = in == 1 ? 2 : 1;
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
    const int go = int64_t(sa[t]) * 100 < int64_t(s.ctl[CTL_NROWS + in]) * pct;
    s.ctl[CTL_CMPGO] = go;
    if (go) {
      s.ctl[CTL_NROWS + out] = sa[t];
      s.ctl[CTL_NELEM + out] = sb[t];
      const_cast<uint32_t*>(s.crow[out])[sa[t]] = uint32_t(sb[t]);
      if (s.crec[out])
        s.crec[out][sa[t]] = make_uint2(0u, uint32_t(sb[t]));
    }
  }
}

// Exclusive block scan of two counters (wave shuffles + one LDS exchange); ta/tb = block totals.
__device__ __forceinline__ void block_scan_pair(int& a, int& b, int& ta, int& tb) {
  __shared__ int wa[kBlock / kWave], wb[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int ia = a, ib = b;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int xa = __shfl_up(ia, o, kWave), xb = __shfl_up(ib, o, kWave);
    if (lane >= o) {
      ia += xa;
      ib += xb;
    }
  }
  if (lane == kWave - 1) {
    wa[w] = ia;
    wb[w] = ib;
  }
  __syncthreads();
  int oa = 0, ob = 0;
  ta = tb = 0;
#pragma unroll
  for (int i = 0; i < kBlock / kWave; i++) {
    oa += i < w ? wa[i] : 0;
    ob += i < w ? wb[i] : 0;
    ta += wa[i];
    tb += wb[i];
  }
  __syncthreads();
  a = oa + ia - a;
  b = ob + ib - b;
}

// Rows of a block are visited k-major (row = base + k * kBlock + thread) so that neighbouring lanes
// read and write neighbouring rows; the output keeps the input order.
__global__ void __launch_bounds__(kBlock) cmp_write(Dev s) {
  if (s.ctl[CTL_DONE] || !s.ctl[CTL_CMPGO])
    return;
  const int in = s.ctl[CTL_BUF], out = in == 1 ? 2 : 1;
  const int64_t nrows = s.ctl[CTL_NROWS + in];
  const int64_t base = int64_t(blockIdx.x) * kCompactRows;
  int pr = s.bsum[2 * blockIdx.x], pe = s.bsum[2 * blockIdx.x + 1];
  const int32_t* __restrict__ icol = s.ccol[in];
  int32_t* ovar = const_cast<int32_t*>(s.cvar[out]);
  uint32_t* orow = const_cast<uint32_t*>(s.crow[out]);
  int32_t* __restrict__ ocol = const_cast<int32_t*>(s.ccol[out]);
  __shared__ int sh_pre[kBlock];
  __shared__ uint32_t sh_beg[kBlock];
  for (int k = 0; k < kRowsPerThread; k++) {
    const int64_t row = base + int64_t(k) * kBlock + threadIdx.x;
    int32_t v = 0;  // (bounded flag kept)
    bool al = false;
    uint32_t b = 0, e = 0;
    if (row < nrows) {
      v = s.cvar[in][row];
      al = s.vstate[rvar(v)] == 0;
      if (al) {
        b = s.crow[in][row];
        e = s.crow[in][row + 1];
      }
    }
    int xr = al, xe = int(e - b), tr, te;
    block_scan_pair(xr, xe, tr, te);
    if (al) {
      const int o = pr + xr;
      ovar[o] = v;
      if (s.crec[out])
        s.crec[out][o] = make_uint2(uint32_t(v), uint32_t(pe + xe));
      s.rtgt[out][o] = s.rtgt[in][row];
      s.skey[out][o] = s.skey[in][row];
      orow[o] = uint32_t(pe + xe);
    }
    // the step's elements land in one contiguous output range [pe, pe + te): copied by the whole block,
    // element f from the row whose exclusive prefix is the last one <= f (coalesced stores, the loads
    // follow the rows in order) instead of one row per thread
    sh_pre[threadIdx.x] = xe;
    sh_beg[threadIdx.x] = b;
    __syncthreads();
    for (int f = threadIdx.x; f < te; f += kBlock) {
      // the last row whose prefix is <= f: it holds f (a dead / empty row shares its prefix with the next
      // row, so the last one with that prefix is never empty while f < te)
      int r = 0;
#pragma unroll
      for (int st = kBlock / 2; st > 0; st >>= 1)
        if (r + st < kBlock && sh_pre[r + st] <= f)
          r += st;
      ocol[pe + f] = icol[sh_beg[r] + uint32_t(f - sh_pre[r])];
    }
    __syncthreads();
    pr += tr;
    pe += te;
  }
}

}  // namespace lmmdev
