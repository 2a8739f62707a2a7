// lmm_frontier_kernels.hpp — System::lmm_solve, "frontier" engine (gfx950; included by lmm_hip.hip).
//
// The same local-minimum progressive filling as lmm_maxmin_kernels.hpp (every alive variable
// votes for the smallest-id constraint of minimal ratio among its constraints; a constraint every alive
// element votes for is a local minimum and saturates), with every round's work proportional to what CHANGED
// instead of to what is still alive.  The multi-launch engine streams every alive row each round to find the
// votes that may move (9e6 rows and ~3.6e6 random key gathers per C2 round); here each vote is registered
// where it can be invalidated — at its target constraint:
//
//   vslot[j]  (u32, per CSC element j of constraint c): the vote floor of j's variable when that variable
//             votes for c through one of its elements on c, kNoVoter otherwise.  The floor (row_floor32) is
//             the min 32-bit key (ratio_key32) over the variable's other constraints (and of its bound level):
//             while c's key stays strictly below it the vote stands, because keys never decrease; 0 =
//             "sensitive", the vote depends on c's exact ratio (a tie within 2^-24).
//   minfl[c]  (u32): a lower bound of the floors registered at c (kNoVoter: none).
//
// So a vote can only move when its target was touched in the last update and the target's new key reached
// the floor: the update pass, which owns every touched constraint anyway, reads the slots of exactly the
// touched constraints whose new key reached minfl and queues those voters.  Round r (3 launches):
//
//   fr_vote    re-vote the queued variables (one lane each, the row in registers): new target and floor,
//              slot + minfl at the new target, vote counts moved; bound fixes (maxmin.cpp:587-589) and
//              variables whose every constraint left the light table as in mm_vote.  Round 0 (fr_vote_all)
//              votes every variable.
//   fr_sat     ready test (alive, nvote == 0) fused with the saturation of the ready constraints (their CSC
//              chunks shared by the workgroup's waves, saturate_chunk: maxmin.cpp:578-606); constraints of
//              more than kFrBigCh chunks go to a list that fr_sat_big spreads over the whole grid.
//   fr_update  constraint update (maxmin.cpp:603-658, as mm_update) + the slot scan of the touched
//              constraints whose key reached minfl -> the workgroup's segment of the re-vote queue.
//
// The decisions are exactly those of the other engines (same votes before every saturation, same ready
// sets, integer / fixed-point atomics only): results are bit-identical to them (tests/test_gpu_engines.py).
// Work per C2 round: the touched constraints' records and slots, the re-voted rows, the saturated
// constraints' elements — no pass over the alive rows, no compaction.
#pragma once
#include "lmm_maxmin_kernels.hpp"

namespace lmmdev {

constexpr int kFB = 256;                 // threads per workgroup = constraints per workgroup (update, saturation)
constexpr uint32_t kNoVoter = 0xFFFFFFFFu;  // vslot: no vote registered at this element; minfl: none at all
constexpr int kFrBigCh = 16;             // constraints of more CSC chunks than this saturate in fr_sat_big
constexpr int kFrBigWaves = 16;          // waves per big constraint in fr_sat_big
constexpr int kFVS = 4;                  // fr_update segments (workgroups) per fr_vote workgroup

// CSR element -> (constraint, CSC position) pairs (csr_cs), once per uploaded structure: one wave per
// constraint, each CSC element finds its CSR element in its variable's row (csc_row); the k-th element of a
// variable on a constraint maps to the k-th (duplicates: cdup).  Also the largest CSC degree (into *maxdeg).
__global__ void __launch_bounds__(kBlock) fr_c2s(Dev s, int2* cs, int32_t* maxdeg) {
  const int lane = threadIdx.x & (kWave - 1);
  int md = 0;
  for (int64_t c = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; c < s.nC;
       c += int64_t(gridDim.x) * (kBlock / kWave)) {
    const uint32_t b = s.cnst_ptr[c], e = s.cnst_ptr[c + 1];
    md = max(md, int(e - b));
    const bool dup = s.cdup[c] != 0;
    // A constraint with a duplicate element: the k-th occurrence of a variable is found by counting the earlier
    // ones.  When the column lists its variables in ascending order (the CSC built in CSR order: every upload
    // path of a max-min system) equal ids are adjacent and only the run before j is scanned; otherwise every
    // earlier element (O(degree^2) for the column, ADVICE r04: one duplicate on a core link made that seconds).
    bool sorted_col = true;
    if (dup) {
      bool desc = false;
      for (uint32_t j = b + 1 + lane; j < e; j += kWave)
        desc |= s.csc_v[j - 1] > s.csc_v[j];
      sorted_col = __ballot(desc) == 0;
    }
    for (uint32_t j = b + lane; j < e; j += kWave) {
      const int32_t v = s.csc_v[j];
      const unsigned long long row = s.csc_row[j];
      int occ = 0;
      if (dup && sorted_col)
        for (uint32_t i = j; i > b && s.csc_v[i - 1] == v; i--)
          occ++;
      else if (dup)
        for (uint32_t i = b; i < j; i++)
          occ += s.csc_v[i] == v;
      for (uint32_t k = uint32_t(row); k < uint32_t(row >> 32); k++)
        if (s.csr_c[k] == int32_t(c) && occ-- == 0) {
          cs[k] = make_int2(int32_t(c), int32_t(j));
          break;
        }
    }
  }
  md = -grp_imin<kWave>(-md);
  if (lane == 0 && md)
    atomicMax(maxdeg, md);
}

// Per-solve variable state (mm_init_vars) + the (bound, penalty) record the re-votes read in one line.
// (with the slots' and floors' kNoVoter fill: two copy-engine fills and their launch gaps less per solve)
__global__ void __launch_bounds__(kBlock) fr_init_vars(Dev s) {
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += stride) {
    s.x[v] = 0.0;
    s.vstate[v] = 0;
    s.rtgt[0][v] = kUnvoted;
    s.pvb[v] = make_double2(s.vbound[v], s.pen[v]);
  }
  uint4* vs4 = reinterpret_cast<uint4*>(s.vslot);  // (scratch allocations: 256-B aligned)
  const uint4 none = make_uint4(kNoVoter, kNoVoter, kNoVoter, kNoVoter);
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < s.nnz / 4; j += stride)
    vs4[j] = none;
  for (int64_t j = (s.nnz & ~int64_t(3)) + int64_t(blockIdx.x) * kBlock + threadIdx.x; j < s.nnz; j += stride)
    s.vslot[j] = kNoVoter;
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < s.nC; c += stride)
    s.minfl[c] = kNoVoter;
}

// Diagnostic counters (profiling mode only, vstat's kDiagSlot words of each round): 0 touched constraints,
// 1 scanned constraints, 2 scanned slots, 3 queued votes, 4 moved votes, 5 ready constraints, 6 re-votes,
// 7 bound fixes.
__device__ __forceinline__ void fr_diag(const Dev& s, int round, int k, bool pred) {
  if (!s.vstat || round >= kStatRounds)
    return;
  const unsigned long long m = __ballot(pred);
  if (m && (threadIdx.x & (kWave - 1)) == __ffsll((long long)m) - 1)
    atomicAdd(s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot) + k, __popcll(m));
}
__device__ __forceinline__ void fr_diag_n(const Dev& s, int round, int k, int n) {
  if (!s.vstat || round >= kStatRounds)
    return;
  n = grp_isum<kWave>(n);
  if ((threadIdx.x & (kWave - 1)) == 0 && n)
    atomicAdd(s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot) + k, n);
}

// Re-vote of variable v (one lane): t = its current target (kUnvoted in round 0), [b, e) its CSR row.  The
// first R elements stay in registers with their loads in flight together; longer rows loop over the rest.
// The arithmetic and the decisions are vote_row's (lmm_maxmin_kernels.hpp).
// Outcome of fr_revote (diagnostics): the vote stayed, moved, was fixed at its bound, or dropped.
enum : int { FR_STAY = 0, FR_MOVE = 1, FR_BOUND = 2, FR_DROP = 3 };

// The floor of a vote for a constraint of key mk (row_floor with 32-bit keys): min key over the row's other
// constraints and, bounded, the key of the level bound * penalty; 0 = sensitive (a key-level tie).
__device__ __forceinline__ uint32_t row_floor32(uint32_t sk, uint32_t mk, double vb, double p) {
  uint32_t fl = sk;
  if (vb > 0)
    fl = min(fl, ratio_key32(vb * p));
  return fl <= mk ? 0u : fl;
}

// (LMM_ANAT: `an` = the dependent levels into ar->lv: 1 row (csr_cs) + bound / penalty, 2 keys + floors, 3 the rest of
// the row + exact ratios, 4 the vote's stores and atomics issued)
template <int R, bool kMinfl = true, bool kEarly = true>
__device__ __forceinline__ int fr_revote(const Dev& s, int v, int t, uint32_t b, uint32_t e, int round
#if LMM_ANAT
                                         , bool an = false, AnatAcc* ar = nullptr
#endif
) {
#if LMM_ANAT
#define FV_LVL(i, dep)       \
  do {                       \
    if (an)                  \
      ANAT_LVL(*ar, i, dep); \
  } while (0)
#else
#define FV_LVL(i, dep) \
  do {                 \
  } while (0)
#endif
  const uint32_t* __restrict__ key = s.key32;
  // (a queued variable is alive: votes are registered only by alive variables, and the slot of a variable
  // fixed since — at its bound, by fr_revote — was cleared when it was queued)
  const double2 bp = s.pvb[v];
  const double vb = bp.x, p = bp.y;
  int32_t cc[R];
  uint32_t sl[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    const int2 x = b + i < e ? s.csr_cs[b + i] : make_int2(-1, 0);
    cc[i] = x.x;
    sl[i] = uint32_t(x.y);
  }
#if LMM_ANAT
  if (an) {
    int sc = 0;
#pragma unroll
    for (int i = 0; i < R; i++)
      sc += cc[i] + int(sl[i]);
    FV_LVL(1, vb + p + double(sc));
  }
#endif
  uint32_t kk[R], mf[R];  // keys and registered floors of the row's constraints, their loads in flight together
#pragma unroll
  for (int i = 0; i < R; i++) {
    kk[i] = cc[i] >= 0 ? key[cc[i]] : kDead32;
    mf[i] = kMinfl && kEarly && cc[i] >= 0 ? s.minfl[cc[i]] : 0u;
  }
#if LMM_ANAT
  if (an) {
    uint32_t sk0 = 0;
#pragma unroll
    for (int i = 0; i < R; i++)
      sk0 += kk[i] + mf[i];
    FV_LVL(2, sk0);
  }
#endif
  uint32_t mk = kDead32;
#pragma unroll
  for (int i = 0; i < R; i++)
    mk = min(mk, kk[i]);
#pragma unroll 4
  for (uint32_t j = b + R; j < e; j++)
    mk = min(mk, key[s.csr_cs[j].x]);
  if (mk == kDead32) {  // every constraint of v left the light table: v stays at 0
    s.vstate[v] = round + 1;
    return FR_DROP;
  }
  int nmin = 0, mult_old = 0, newt = INT_MAX;
  uint32_t kt = kDead32;
#pragma unroll
  for (int i = 0; i < R; i++) {
    nmin += kk[i] == mk;
    if (cc[i] == t) {
      mult_old++;
      kt = kk[i];
    }
    if (kk[i] == mk)
      newt = min(newt, cc[i]);
  }
#pragma unroll 4
  for (uint32_t j = b + R; j < e; j++) {
    const int32_t c = s.csr_cs[j].x;
    const uint32_t k = key[c];
    nmin += k == mk;
    if (c == t) {
      mult_old++;
      kt = k;
    }
    if (k == mk)
      newt = min(newt, c);
  }
  double minr = dinf();
  if (nmin > 1 || vb > 0) {  // exact ratios at the minimal key: lexicographic min of (ratio, id)
    newt = INT_MAX;
    double rr[R];  // the tied constraints' ratios, all loads issued before the first compare (one dependent level:
                   // a compare right after each conditional load waited for the loads one at a time)
#pragma unroll
    for (int i = 0; i < R; i++)
      rr[i] = kk[i] == mk ? s.cst[cc[i]].ratio : dinf();
#pragma unroll
    for (int i = 0; i < R; i++)
      if (kk[i] == mk && (rr[i] < minr || (rr[i] == minr && cc[i] < newt))) {
        minr = rr[i];
        newt = cc[i];
      }
    for (uint32_t j = b + R; j < e; j++) {
      const int32_t c = s.csr_cs[j].x;
      if (key[c] == mk) {
        const double r = s.cst[c].ratio;
        if (r < minr || (r == minr && c < newt)) {
          minr = r;
          newt = c;
        }
      }
    }
  }
  FV_LVL(3, minr + double(newt + nmin));
  if (vb > 0 && vb * p < minr) {  // fixed at its bound (maxmin.cpp:587-589)
    s.vstate[v] = round + 1;
    s.x[v] = vb;
    if (t >= 0 && kt != kDead32)
      atomicAdd(&s.nvote[t], mult_old);
    for (uint32_t j = b; j < e; j++)
      push_decrement(s, j, vb, p);
    return FR_BOUND;
  }
  uint32_t sk = kDead32;  // min key over the other constraints of the row
  int mult_new = 0;
  uint32_t slot = 0xFFFFFFFFu;  // CSC position of one of v's elements on newt (the smallest)
  uint32_t mfn = kNoVoter;      // newt's minfl as read with the keys (only decreases within this launch)
#pragma unroll
  for (int i = 0; i < R; i++) {
    if (cc[i] != newt) {
      sk = min(sk, kk[i]);
    } else {
      mult_new++;
      slot = min(slot, sl[i]);
      mfn = kEarly ? mf[i] : kNoVoter;
    }
  }
  for (uint32_t j = b + R; j < e; j++) {
    const int2 x = s.csr_cs[j];
    if (x.x != newt) {
      sk = min(sk, key[x.x]);
    } else {
      mult_new++;
      slot = min(slot, uint32_t(x.y));
      mfn = kNoVoter;  // (read with the keys only for the first R elements: always take the atomic)
    }
  }
  // (a floor of kDead32 — no other alive constraint, unbounded — is stored as kDead32 - 1: the vote then
  // moves only when newt itself dies, exactly as before)
  const uint32_t fl = min(row_floor32(sk, mk, vb, p), kNoVoter - 1u);
  if (kMinfl && !kEarly)  // (loaded before the slot's store: a load issued after a store waits for it)
    mfn = s.minfl[newt];
  s.vslot[slot] = fl;
  if (kMinfl && fl < mfn)
    atomicMin(&s.minfl[newt], fl);
  if (newt == t) {
    FV_LVL(4, 0u);
    return FR_STAY;
  }
  if (t >= 0 && kt != kDead32)
    atomicAdd(&s.nvote[t], mult_old);
  atomicSub(&s.nvote[newt], mult_new);
  s.rtgt[0][v] = newt;
  FV_LVL(4, 0u);
  return FR_MOVE;
}

// Round 0: every variable votes (the floors' per-constraint minima come after, from fr_minfl_all).
__global__ void __launch_bounds__(kBlock) fr_vote_all(Dev s) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock)
    fr_revote<8, false>(s, int(v), kUnvoted, s.var_ptr[v], s.var_ptr[v + 1], 0);
}

// After round 0's vote: minfl[c] = min of the floors registered in c's slots, 16 lanes per constraint (four
// constraints per wave; one segmented pass over the slots instead of ~nV atomics).
__global__ void __launch_bounds__(kBlock) fr_minfl_all(Dev s) {
  const int lane = threadIdx.x & (kWave - 1), gl = lane & 15;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  for (int64_t c = wave * 4 + lane / 16; c < s.nC; c += nwaves * 4) {  // group-uniform
    const uint32_t b = s.cnst_ptr[c], e = s.cnst_ptr[c + 1];
    uint32_t m = kNoVoter;
    for (uint32_t j = b + gl; j < e; j += 64) {
      uint32_t f[4];
#pragma unroll
      for (int k = 0; k < 4; k++)
        f[k] = j + 16 * k < e ? s.vslot[j + 16 * k] : kNoVoter;
#pragma unroll
      for (int k = 0; k < 4; k++)
        m = min(m, f[k]);
    }
    m = grp_umin<16>(m);
    if (gl == 0)
      s.minfl[c] = m;
  }
}

// Rounds >= 1: the variables fr_update queued in workgroup b's segment (the CSC range of its constraints).
// Also the termination test (maxmin.cpp:680): no constraint alive after the last update -> CTL_DONE.
// fr_vote_blk: the work of workgroup vb.
template <int R>
__device__ __forceinline__ void fr_vote_blk(const Dev& s, int round, int spb, int vb
#if LMM_ANAT
                                            , bool an = false, AnatAcc* aa = nullptr, AnatAcc* ar = nullptr,
                                            unsigned* wc = nullptr
#endif
) {
  // spb (<= kFVS) consecutive segments per workgroup: on C2 ~170 queued rows, one pass, and the launch's
  // workgroups resident at once; small systems keep one segment per workgroup (more workgroups)
  const int64_t nseg = (int64_t(s.nC) + kFB - 1) / kFB;
  int n[kFVS], pre[kFVS + 1];
  uint32_t seg[kFVS];
  pre[0] = 0;
#pragma unroll
  for (int k = 0; k < kFVS; k++) {
    const int64_t sg = int64_t(vb) * spb + k;
    n[k] = k < spb && sg < nseg ? s.fq_n[sg] : 0;
    seg[k] = k < spb && sg < nseg ? s.cnst_ptr[sg * kFB] : 0u;
    pre[k + 1] = pre[k] + n[k];
  }
#if LMM_ANAT
  if (an) {
    ANAT_LVL(*aa, 0, pre[kFVS] + int(seg[0]));
    wc[0] = unsigned(pre[kFVS]);
  }
#endif
  for (int i = threadIdx.x; i < pre[kFVS]; i += kFB) {
    int k = 0;
#pragma unroll
    for (int q = 1; q < kFVS; q++)
      k += i >= pre[q];
    const uint32_t at = seg[k] + uint32_t(i - pre[k]);
#if LMM_ANAT
    if (an) {
      ar->at = anat_now();
      wc[1]++;
    }
#endif
    const unsigned long long a = s.fq_a[at], rw = s.fq_b[at];
#if LMM_ANAT
    if (an)
      ANAT_LVL(*ar, 0, a + rw);
    const int o = fr_revote<R, true, false>(s, int(uint32_t(a)), int(uint32_t(a >> 32)), uint32_t(rw),
                                             uint32_t(rw >> 32), round, an, ar);
#else
    const int o = fr_revote<R, true, false>(s, int(uint32_t(a)), int(uint32_t(a >> 32)), uint32_t(rw),
                                             uint32_t(rw >> 32), round);
#endif
    if (s.vstat) {
      fr_diag(s, round, 6, true);
      fr_diag(s, round, 4, o == FR_MOVE);
      fr_diag(s, round, 7, o == FR_BOUND);
    }
  }
}

template <int R = 8> __global__ void __launch_bounds__(kFB) fr_vote(Dev s, int round, int spb) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_VOTE);
  const bool an = arec != nullptr;
  AnatAcc aa{}, ar{};
  unsigned wc[2] = {0, 0};  // queued rows of the workgroup, this lane's re-votes
  const unsigned long long t_in = an ? anat_now() : 0;
  aa.at = t_in;
#endif
  if (s.ctl[CTL_DONE])
    return;
  if (s.ctl[CTL_PALIVE0 + ((round - 1) & 1)] == 0) {  // written by the last fr_update
    if (blockIdx.x == 0 && threadIdx.x == 0)
      s.ctl[CTL_DONE] = 1;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_PALIVE0 + (round & 1)] = 0;  // this round's fr_update raises it
#if LMM_ANAT
  fr_vote_blk<R>(s, round, spb, blockIdx.x, an, &aa, &ar, wc);
  if (an) {  // the wave's record: queue-count level (lane 0), the re-vote levels of its slowest lane
    const unsigned long long t_out = anat_now();
    unsigned lv[5];
#pragma unroll
    for (int i = 0; i < 5; i++)
      lv[i] = anat_wmax(ar.lv[i]);
    const unsigned nre = anat_wmax(wc[1]);
    if ((threadIdx.x & (kWave - 1)) == 0) {
      arec[0] = t_in;
      arec[1] = t_out;
      arec[2] = blockIdx.x;
      arec[3] = aa.lv[0];
      for (int i = 0; i < 5; i++)
        arec[4 + i] = lv[i];
      arec[9] = nre;
      arec[10] = wc[0];
    }
  }
#else
  fr_vote_blk<R>(s, round, spb, blockIdx.x);
#endif
}

// Saturation of one 64-element CSC chunk of ready constraint c: saturate_chunk's decisions and arithmetic
// (maxmin.cpp:578-606), with the loads of the chunk issued before its stores and atomics — the claim and the
// value are stored last (a wave's loads wait for its older stores / atomics): CSC elements -> variable states
// -> the claimed rows' elements (kFrSatU x 64 in flight) -> their constraints' packed words, then the
// decrement pushes and the variables' states.  Deferring the claim is safe: ready constraints share no alive
// variable, and a variable appears once in c's CSC unless c has a duplicate element (cdup: claimed by
// atomicCAS, as before).
constexpr int kFrSatU = 8;
// (Round 6, measured and removed: the pushes of a chunk's passes kept in LDS and issued after all its loads, so that a
// second pass's loads do not wait for the first pass's atomics — C4 3.27 ms against 3.14-3.19 without, same box; and
// the pushes aggregated per constraint in a per-wave LDS hash table (CAS-probed slots, 64-bit LDS adds, one global
// atomic per distinct constraint and pass) against the hot-address serialisation of a saturating host link's flows,
// whose other links repeat ~50 times in a chunk — C4 3.63 ms against 3.12: the table's probing and flush cost more;
// and 16 claimed-row elements per lane per pass instead of 8, a C4 chunk's pushes in one pass — 3.28 against 3.12.)

// (LMM_ANAT: `an` = the chunk's dependent levels into aa->lv: 2 CSC elements + variable states, 3 the claimed rows'
// elements, 4 their constraints' words, 5 the pushes issued, 6 the claims / values stored; wc[1] chunks, wc[2] fixed
// variables, wc[3] pushed elements)
__device__ __forceinline__ void fr_sat_chunk(const Dev& s, int32_t c, double r, uint32_t j0, uint32_t cend,
                                             int round, int lane, int* pre, bool dup
#if LMM_ANAT
                                             , bool an = false, AnatAcc* aa = nullptr, unsigned* wc = nullptr
#endif
) {
#if LMM_ANAT
  if (an) {
    aa->at = anat_now();
    wc[1]++;
  }
#define FS_LVL(i, dep)       \
  do {                       \
    if (an)                  \
      ANAT_LVL(*aa, i, dep); \
  } while (0)
#else
#define FS_LVL(i, dep) \
  do {                 \
  } while (0)
#endif
  const int q = lane & 3;
  const uint32_t j = j0 + lane;
  int32_t lv = -1;
  double lp = 1.0, lx = 0.0;
  uint32_t rb = 0, re = 0;
  if (j < cend) {
    lv = s.csc_v[j];
    lp = s.csc_p[j];
    const unsigned long long row = s.csc_row[j];
    rb = uint32_t(row);
    re = uint32_t(row >> 32);
    if (s.vstate[lv] != 0)
      lv = -1;
    else if (dup && atomicCAS(&s.vstate[lv], 0, round + 1) != 0)
      lv = -1;
  }
  int len = 0;
  if (lv >= 0) {
    lx = r / lp;
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
  for (int f0 = 0; f0 < total; f0 += kFrSatU * kWave) {  // wave-uniform (one pass up to 512 elements)
    int32_t cc[kFrSatU];
    int ol[kFrSatU];
    double ww[kFrSatU];
#pragma unroll
    for (int u = 0; u < kFrSatU; u++) {
      const int f = f0 + u * kWave + lane;
      int o = 0;  // owner lane: last lane with pre <= f
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1)
        if (pre[o + step] <= f)
          o += step;
      ol[u] = o;
      const uint32_t k = uint32_t(__shfl(int(rb), o, kWave)) + uint32_t(f - pre[o]);
      cc[u] = f < total ? s.csr_c[k] : -1;
      ww[u] = f < total ? s.csr_w[k] : 0.0;
    }
#if LMM_ANAT
    if (an) {
      double sw = 0.0;
#pragma unroll
      for (int u = 0; u < kFrSatU; u++) {
        sw += ww[u] + double(cc[u]);
        wc[3] += unsigned(__popcll(__ballot(cc[u] >= 0)));
      }
      ANAT_LVL(*aa, 3, sw);
    }
#endif
    int32_t cx[kFrSatU];
#pragma unroll
    for (int u = 0; u < kFrSatU; u++)
      cx[u] = cc[u] >= 0 ? s.cexp[cc[u]] : kCexpDead;  // scales, policy and liveness in one word
#if LMM_ANAT
    if (an) {
      int32_t sx = 0;
#pragma unroll
      for (int u = 0; u < kFrSatU; u++)
        sx += cx[u];
      ANAT_LVL(*aa, 4, sx);
    }
#endif
#pragma unroll
    for (int u = 0; u < kFrSatU; u++) {
      const double ox = __shfl(lx, ol[u], kWave);
      const double op = __shfl(lp, ol[u], kWave);
      bool fat = false;
      long long a0 = 0, a1 = 0;  // fixed-point decrements (CstRec)
      int32_t tc = cc[u];
      if (tc >= 0 && (tc == c || (cx[u] & kCexpDead)))
        tc = -1;
      if (tc >= 0) {
        s.ctouch[tc] = 1;  // receives decrements this round (fr_update reads its record)
        fat = cx[u] & kCexpFat;
        a0 = (long long)dec_q(ww[u] * ox, cexp_rem(cx[u]));
        a1 = fat ? (long long)fat_bits(ww[u] / op) : (long long)dec_q(ww[u] / op, cexp_use(cx[u]));
      }
      const int nel = total - f0 - u * kWave;
#pragma unroll
      for (int t = 0; t < kWave / 16; t++) {  // each element's pushes by a quad of lanes: one atomic request
        if (t * 16 >= nel)
          break;
        const int e = t * 16 + (lane >> 2);
        const int ec = __shfl(tc, e, kWave);
        const int ef = __shfl(int(fat), e, kWave);
        const long long e0 = __shfl(a0, e, kWave);
        const long long e1 = __shfl(a1, e, kWave);
        if (ec >= 0 && q < 3 && (!ef || q == 2))
          atomicAdd(&s.cst[ec].drem + q, (unsigned long long)(q == 0 ? e0 : q == 1 ? e1 : 1ll));
        if (ec >= 0 && ef && q == 1)  // FATPIPE: the removed w/p (fat_bits)
          atomicMax(&s.cst[ec].duse, (unsigned long long)e1);
      }
    }
    FS_LVL(5, 0u);
  }
  if (lv >= 0) {  // the claim and the value, last
    if (!dup)
      s.vstate[lv] = round + 1;
    s.x[lv] = lx;
  }
  __builtin_amdgcn_wave_barrier();
  FS_LVL(6, 0u);
}

// The collected ready constraints' chunks, round-robin over the workgroup's waves (sat_flush with fr_sat_chunk).
#if LMM_ANAT
#define FR_ANAT_PARAMS , bool an = false, AnatAcc* aa = nullptr, unsigned* wc = nullptr
#define FR_ANAT_ARGS , an, aa, wc
#else
#define FR_ANAT_PARAMS
#define FR_ANAT_ARGS
#endif
// The ready constraints a saturation workgroup collected, with their CSC chunk prefix and — loaded by the ready test
// itself (round 6) — their CSC range, ratio and duplicate flag, so that a chunk's first loads are its CSC elements.
template <int NB> struct FrSatLds {
  int32_t rc[NB];      // collected ready constraints
  int32_t rr[NB + 1];  // exclusive prefix of their chunk counts
  uint32_t rb[NB], re[NB];
  double rt[NB];
  uint8_t rd[NB];
  int wa[NB / kWave], wb[NB / kWave];
  int na, nb;
  int pre[NB / kWave][kWave];  // fr_sat_chunk's per-wave row-length prefix
};

template <int NB>
__device__ __forceinline__ void fr_flush(const Dev& s, int round, FrSatLds<NB>& L FR_ANAT_PARAMS) {
  constexpr int NBW = NB / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int ta = L.na, tb = L.nb;
  for (int g = w; g < tb; g += NBW) {  // wave-uniform
    int k = 0;  // last collected entry whose first chunk is <= g
#pragma unroll
    for (int step = NB / 2; step > 0; step >>= 1)
      if (k + step < ta && L.rr[k + step] <= g)
        k += step;
    const int32_t cc = L.rc[k];
    const int ch = g - L.rr[k];
    const double r = L.rt[k];
    fr_sat_chunk(s, cc, r, L.rb[k] + uint32_t(ch) * kWave, L.re[k], round, lane, L.pre[w], L.rd[k] != 0 FR_ANAT_ARGS);
    if (ch == 0 && lane == 0)
      s.ctouch[cc] = 2;
  }
}

// Ready test + saturation: workgroup b tests its kFS constraints; the ready ones are collected in LDS with
// the prefix of their 64-element CSC chunks and the workgroup's 16 waves take the chunks round-robin
// (fr_flush).  A constraint of more than kFrBigCh chunks is listed for fr_sat_big instead.
constexpr int kFS = 1024;

template <int NB>
__device__ __forceinline__ void fr_sat_blk(const Dev& s, int round, int bigch, int vb, FrSatLds<NB>& L
                                           FR_ANAT_PARAMS) {
  constexpr int NBW = NB / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int64_t c = int64_t(vb) * NB + threadIdx.x;
  bool rdy = false;
  int nch = 0;
  // every load of the ready test in one dependent level (round 6; the short-circuit test took three: key, then vote
  // count, then CSC range), and — in the 256-thread workgroups of the small systems, where the extra lines are few —
  // the ratio and duplicate flag with them (coalesced: one constraint per lane)
  uint32_t kc = kDead32, cb = 0, ce = 0;
  int nv = 1;
  double rt = 0.0;
  bool dp = false;
  if (c < s.nC) {
    kc = s.key32[c];
    nv = s.nvote[c];
    cb = s.cnst_ptr[c];
    ce = s.cnst_ptr[c + 1];
    if (NB == 256) {
      rt = s.cst[c].ratio;
      dp = s.cdup[c] != 0;
    }
  }
  if (kc != kDead32 && nv == 0) {
    rdy = true;
    if (NB != 256) {
      rt = s.cst[c].ratio;
      dp = s.cdup[c] != 0;
    }
    nch = int((ce - cb + kWave - 1) / kWave);
    if (s.vstat)
      atomicAdd(s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot) + 5, 1);
    if (nch > bigch) {  // rare (fat-tree core links): spread over the grid by fr_sat_big
      s.ready[atomicAdd(&s.ctl[CTL_NREADY], 1)] = int32_t(c);
      rdy = false;
      nch = 0;
    }
  }
  int ia = rdy, ib = nch;  // wave inclusive scans of (ready, chunks)
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
  int oa = 0, ob = 0, ta = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < NBW; k++) {
    oa += k < w ? L.wa[k] : 0;
    ob += k < w ? L.wb[k] : 0;
    ta += L.wa[k];
    tb += L.wb[k];
  }
  if (rdy) {
    const int k = oa + ia - 1;
    L.rc[k] = int32_t(c);
    L.rr[k] = ob + ib - nch;
    L.rb[k] = cb;
    L.re[k] = ce;
    L.rt[k] = rt;
    L.rd[k] = uint8_t(dp);
  }
  if (threadIdx.x == 0) {
    L.na = ta;
    L.nb = tb;
    if (ta)
      s.ctl[CTL_LASTR] = round;  // plain store: this round fixes variables
  }
  __syncthreads();
#if LMM_ANAT
  if (an) {  // the ready test and the workgroup's collection, then the chunks
    ANAT_LVL(*aa, 0, ta);
    wc[0] = unsigned(tb);
  }
#endif
  if (ta)  // workgroup-uniform
    fr_flush<NB>(s, round, L FR_ANAT_ARGS);
}

template <int kFS> __global__ void __launch_bounds__(kFS) fr_sat(Dev s, int round, int bigch) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_SAT);
  const bool an = arec != nullptr;
  AnatAcc aa{};
  unsigned wc[4] = {0, 0, 0, 0};  // the workgroup's chunks, this wave's chunks, fixed variables, pushed elements
  const unsigned long long t_in = an ? anat_now() : 0;
  aa.at = t_in;
#endif
  if (s.ctl[CTL_DONE])
    return;
  __shared__ FrSatLds<kFS> L;
#if LMM_ANAT
  fr_sat_blk<kFS>(s, round, bigch, blockIdx.x, L, an, &aa, wc);
  if (an && (threadIdx.x & (kWave - 1)) == 0) {
    arec[0] = t_in;
    arec[1] = anat_now();
    arec[2] = blockIdx.x;
    for (int i = 0; i < 7; i++)
      arec[3 + i] = aa.lv[i];
    for (int i = 0; i < 4; i++)
      arec[10 + i] = wc[i];
  }
#else
  fr_sat_blk<kFS>(s, round, bigch, blockIdx.x, L);
#endif
}

// The big ready constraints listed by fr_sat (count CTL_NREADY, reset by fr_update): kFrBigWaves waves per
// constraint over the whole grid, wave k taking chunks k, k + kFrBigWaves, ...
// (the grid's waves over the list: wave / nwaves; wpre = the calling wave's 64-int LDS scratch)
__device__ __forceinline__ void fr_sat_big_waves(const Dev& s, int round, int bigw, int nb, int64_t wave,
                                                 int64_t nwaves, int* wpre FR_ANAT_PARAMS) {
  const int lane = threadIdx.x & (kWave - 1);
  for (int64_t g = wave; g < int64_t(nb) * bigw; g += nwaves) {
    const int32_t c = s.ready[g / bigw];
    const int k = int(g % bigw);
    const double r = ld_rlx(&s.cst[c].ratio);
    const uint32_t ce = s.cnst_ptr[c + 1];
    const bool dup = s.cdup[c] != 0;
    for (uint32_t base = s.cnst_ptr[c] + uint32_t(k) * kWave; base < ce; base += uint32_t(bigw) * kWave)
      fr_sat_chunk(s, c, r, base, ce, round, lane, wpre, dup FR_ANAT_ARGS);
    if (k == 0 && lane == 0)
      s.ctouch[c] = 2;
  }
}

__global__ void __launch_bounds__(kBlock) fr_sat_big(Dev s, int round, int bigw) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_SATB);
  const bool an = arec != nullptr;
  AnatAcc aa{};
  unsigned wc[4] = {0, 0, 0, 0};
  const unsigned long long t_in = an ? anat_now() : 0;
  aa.at = t_in;
#endif
  if (s.ctl[CTL_DONE])
    return;
  const int nb = s.ctl[CTL_NREADY];
#if LMM_ANAT
  if (an && (threadIdx.x & (kWave - 1)) == 0) {
    arec[0] = t_in;
    arec[1] = anat_now();
    arec[2] = blockIdx.x;
    arec[10] = unsigned(nb);
  }
#endif
  if (nb == 0)
    return;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    s.ctl[CTL_LASTR] = round;
  __shared__ int wpre[kBlock / kWave][kWave];
  const int w = threadIdx.x / kWave;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
#if LMM_ANAT
  fr_sat_big_waves(s, round, bigw, nb, wave, nwaves, wpre[w], an, &aa, wc);
  if (an && (threadIdx.x & (kWave - 1)) == 0) {
    arec[1] = anat_now();
    for (int i = 0; i < 7; i++)
      arec[3 + i] = aa.lv[i];
    for (int i = 1; i < 4; i++)
      arec[10 + i] = wc[i];
  }
#else
  fr_sat_big_waves(s, round, bigw, nb, wave, nwaves, wpre[w]);
#endif
}

// Constraint update (maxmin.cpp:603-658; the arithmetic of update_groups) + slot scan.  Workgroup b owns
// constraints [b * kFB, (b + 1) * kFB), one per thread.  A touched constraint whose new key reached its minfl
// (or that left the light table) has its slots read — all such constraints of a wave flattened over the wave,
// kFrScanU x 64 slots in flight — and the voters whose floor the key reached are queued for fr_vote in the
// workgroup's segment (fq_a: variable | old target << 32, fq_b: CSR row), their slots cleared; minfl becomes
// the min floor of the voters that stay.
// Every load of the pass is issued before its first store (a wave's loads wait for its older stores and
// atomics, MI355X_MICROARCH.md `s_waitcnt vmcnt`): constraint state -> slots -> queued variables' rows, then
// the stores of the new state, the queue and the cleared slots.
constexpr int kFrScanU = 8;

struct FrUpdLds {
  int qn;
  int pre[kFB / kWave][kWave];
  uint32_t mf[kFB];
};

// (LMM_ANAT: `an` = the levels into aa->lv: 0 keys + touch flags, 1 touched records, 2 arithmetic + scan prefix +
// barrier, 3 slots, 4 queued voters' variable and row, 5 stores + barriers; wc[0] scanned slots)
// spec (round 6, small systems): a constraint's record, scales, votes, floor and CSC range are loaded with its key and
// touch flag whether or not it was touched (coalesced, one constraint per lane), one dependent level instead of two.
__device__ __forceinline__ void fr_update_blk(const Dev& s, int round, double prec, int vb, FrUpdLds& U, bool spec
                                              FR_ANAT_PARAMS) {
  int& qn = U.qn;
  auto& pre = U.pre;
  uint32_t* mf = U.mf;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (threadIdx.x == 0)
    qn = 0;
  if (vb == 0 && threadIdx.x == 0) {
    s.ctl[CTL_ROUNDS] += 1;
    s.ctl[CTL_NREADY] = 0;  // fr_sat_big's list of the next round
  }
  const int64_t gbase = int64_t(vb) * kFB + int64_t(w) * kWave;
  const int64_t c = gbase + lane;
  const bool in = c < s.nC;
  const uint32_t okey = in ? s.key32[c] : kDead32;
  const unsigned tf = in ? unsigned(s.ctouch[c]) : 0u;  // 1 = received decrements, 2 = saturated this round
#if LMM_ANAT
  if (an)
    ANAT_LVL(*aa, 0, okey + tf);
#endif
  const bool live0 = okey != kDead32;
  const bool sat = live0 && tf == 2;
  const bool live = live0 && !sat;
  const bool tch = live && tf == 1;
  unsigned long long qx = 0, qy = 0, qz = 0;
  double rem = 0.0, use = 0.0, bnd = 0.0;
  int32_t ce = 0, nv = 0;
  uint32_t mfl = kNoVoter;
  uint32_t cb = 0, cend = 0;
  if (spec ? in : tch) {
    const CstRec* rec = s.cst + c;
    qx = rec->drem;
    qy = rec->duse;
    qz = rec->dcnt;
    rem = rec->rem;
    use = rec->use;
    bnd = rec->bound;
    ce = s.cexp[c];
    nv = s.nvote[c];
    mfl = s.minfl[c];
    cb = s.cnst_ptr[c];
    cend = s.cnst_ptr[c + 1];
  }
#if LMM_ANAT
  if (an)
    ANAT_LVL(*aa, 1, rem + use + bnd + double(qx + qy + qz) + double(ce + nv + int(mfl + cb + cend)));
#endif
  const bool fat = tch && (ce & kCexpFat);
  // FATPIPE: recompute only when a removed element reached the usage (fat_bits in duse)
  const bool fre = fat && !(__longlong_as_double((long long)qy) < use);
  double fuse = use;
  unsigned long long fm = __ballot(fre);
  while (fm) {  // wave-uniform: FATPIPE usage over the still-unfixed elements (maxmin.cpp:625-658)
    const int l = __ffsll((long long)fm) - 1;
    fm &= fm - 1;
    const int64_t cl = gbase + l;
    const uint32_t b = s.cnst_ptr[cl], e = s.cnst_ptr[cl + 1];
    double m = 0.0;
    // (the element's w/p loaded with its variable: no branch between a load and the next one)
#pragma unroll 4
    for (uint32_t j = b + lane; j < e; j += kWave) {
      const double u = s.csc_u[j];
      m = !(s.x[s.csc_v[j]] > 0) ? fmax(m, u) : m;
    }
    m = wave_max(m);
    if (lane == l)
      fuse = m;
  }
  // the new state, in registers (stored after the scan's loads)
  uint32_t nk = okey;
  bool alive = false;
  double r0 = rem, u0 = use, rnew = 0.0;
  if (sat) {
    nk = kDead32;
  } else if (live) {
    if (!tch) {
      alive = true;
    } else {
      if (!fat) {
        u0 = use - dec_val(qy, cexp_use(ce));
        r0 -= dec_val(qx, cexp_rem(ce));
        if (r0 < bnd * prec)
          r0 = 0.0;
        if (u0 < prec)
          u0 = 0.0;
      } else {
        u0 = fuse;
      }
      if (!(u0 > prec) || !(r0 > bnd * prec)) {
        nk = kDead32;
        rnew = dinf();
      } else {
        rnew = r0 / u0;
        nk = ratio_key32(rnew);
        alive = true;
      }
    }
  }
  // ---- slot scan of the touched constraints whose key reached a registered floor ----
  const bool scan = tch && mfl != kNoVoter && nk >= mfl;
  const int len = scan ? int(cend - cb) : 0;
  if (s.vstat) {
    fr_diag(s, round, 0, tch);
    fr_diag(s, round, 1, scan);
    fr_diag_n(s, round, 2, len);
  }
  int incl = len;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if (lane >= o)
      incl += x;
  }
  const int total = __shfl(incl, kWave - 1, kWave);
  pre[w][lane] = incl - len;
  mf[threadIdx.x] = kNoVoter;
  __syncthreads();  // (qn, pre, mf)
#if LMM_ANAT
  if (an) {
    ANAT_LVL(*aa, 2, total);
    wc[0] = unsigned(total);
  }
#endif
  const uint32_t seg = s.cnst_ptr[int64_t(vb) * kFB];
  for (int f0 = 0; f0 < total; f0 += kFrScanU * kWave) {  // wave-uniform (one pass up to 512 slots)
    int ol[kFrScanU];
    uint32_t jj[kFrScanU];
    uint32_t fl[kFrScanU];
#pragma unroll
    for (int u = 0; u < kFrScanU; u++) {
      const int f = f0 + u * kWave + lane;
      int o = 0;  // owner lane: last lane with pre <= f
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1)
        if (pre[w][o + step] <= f)
          o += step;
      ol[u] = o;
      jj[u] = uint32_t(__shfl(int(cb), o, kWave)) + uint32_t(f - pre[w][o]);
      fl[u] = f < total ? s.vslot[jj[u]] : kNoVoter;
    }
#if LMM_ANAT
    if (an) {
      uint32_t sf = 0;
#pragma unroll
      for (int u = 0; u < kFrScanU; u++)
        sf += fl[u];
      ANAT_LVL(*aa, 3, sf);
    }
#endif
    bool q[kFrScanU];
    int32_t qv[kFrScanU];
    unsigned long long qr[kFrScanU];
#pragma unroll
    for (int u = 0; u < kFrScanU; u++) {  // the queued voters' variable and row, loads in flight together
      const uint32_t okk = uint32_t(__shfl(int(nk), ol[u], kWave));
      q[u] = fl[u] != kNoVoter && fl[u] <= okk;
      if (fl[u] != kNoVoter && !q[u])
        atomicMin(&mf[w * kWave + ol[u]], fl[u]);
      qv[u] = q[u] ? s.csc_v[jj[u]] : 0;
      qr[u] = q[u] ? s.csc_row[jj[u]] : 0ull;
    }
#if LMM_ANAT
    if (an) {
      unsigned long long sq = 0;
#pragma unroll
      for (int u = 0; u < kFrScanU; u++)
        sq += qr[u] + unsigned(qv[u]);
      ANAT_LVL(*aa, 4, sq);
    }
#endif
#pragma unroll
    for (int u = 0; u < kFrScanU; u++) {
      const unsigned long long m = __ballot(q[u]);
      if (!m)
        continue;
      if (s.vstat && lane == 0)
        atomicAdd(s.vstat + 2 * (int64_t(round) * kMaxBlocks + kDiagSlot) + 3, __popcll(m));
      int base = 0;
      if (lane == 0)
        base = atomicAdd(&qn, __popcll(m));
      base = __shfl(base, 0, kWave);
      if (q[u]) {
        const int pos = base + __popcll(m & ((1ull << lane) - 1));
        s.fq_a[seg + pos] = (unsigned long long)uint32_t(qv[u]) | ((unsigned long long)uint32_t(gbase + ol[u]) << 32);
        s.fq_b[seg + pos] = qr[u];
        s.vslot[jj[u]] = kNoVoter;
      }
    }
  }
  // ---- the stores of the new state ----
  if (sat) {
    s.key32[c] = kDead32;
    s.cexp[c] = kCexpDead;
    s.ctouch[c] = 0;
    s.cst[c].ratio = dinf();
  } else if (tch) {
    CstRec* rec = s.cst + c;
    s.ctouch[c] = 0;
    rec->drem = rec->duse = rec->dcnt = 0;
    s.nvote[c] = nv - int(qz);
    rec->rem = r0;
    rec->use = u0;
    rec->ratio = rnew;
    s.key32[c] = nk;
    if (nk == kDead32)
      s.cexp[c] = kCexpDead;
  }
  __syncthreads();  // (mf, qn)
  if (scan)
    s.minfl[c] = mf[threadIdx.x];
  const bool any_alive = __syncthreads_or(alive);
  if (threadIdx.x == 0) {
    s.fq_n[vb] = qn;
    if (any_alive) {
      s.ctl[CTL_PALIVE0 + (round & 1)] = 1;
    }
  }
  if (__syncthreads_or(tch || sat) && threadIdx.x == 0)
    s.ctl[CTL_LASTR] = round;  // plain store: the last round that changed a constraint
#if LMM_ANAT
  if (an)
    ANAT_LVL(*aa, 5, 0u);
#endif
}

__global__ void __launch_bounds__(kFB) fr_update(Dev s, int round, double prec, int spec) {
#if LMM_ANAT
  unsigned long long* arec = anat_rec(s, anat_slot(s, round), ANAT_UPD);
  const bool an = arec != nullptr;
  AnatAcc aa{};
  unsigned wc[1] = {0};
  const unsigned long long t_in = an ? anat_now() : 0;
  aa.at = t_in;
#endif
  if (s.ctl[CTL_DONE])
    return;
  __shared__ FrUpdLds U;
#if LMM_ANAT
  fr_update_blk(s, round, prec, blockIdx.x, U, spec != 0, an, &aa, wc);
  if (an && (threadIdx.x & (kWave - 1)) == 0) {
    arec[0] = t_in;
    arec[1] = anat_now();
    arec[2] = blockIdx.x;
    for (int i = 0; i < 6; i++)
      arec[3 + i] = aa.lv[i];
    arec[9] = wc[0];
  }
#else
  fr_update_blk(s, round, prec, blockIdx.x, U, spec != 0);
#endif
}

}  // namespace lmmdev
