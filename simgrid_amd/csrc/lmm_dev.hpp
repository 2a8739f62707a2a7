// lmm_dev.hpp — device-side layout and helpers shared by the LMM kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdint>

namespace lmmdev {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxBlocks = 2048;       // 256 CUs x 8 resident 256-thread blocks; grid-stride beyond
constexpr int kRowsPerThread = 8;      // compaction chunking
constexpr int kCompactRows = kBlock * kRowsPerThread;
constexpr unsigned kDeadKey = 0xFFFFu;  // > every key of a finite positive ratio (<= 0x7F80)

// control block words (int32, zeroed at the start of every solve)
enum : int {
  CTL_DONE = 0,
  CTL_ROUNDS = 1,
  CTL_ANY0 = 2,      // fair bottleneck: "some variable still listed", per round parity (2 words)
  CTL_NROWS = 4,     // alive-row buffer sizes (3 buffers)
  CTL_NELEM = 7,     // alive-row buffer element counts (3 buffers)
  CTL_ALIVE_C = 10,  // (unused since round 6)
  CTL_NREADY = 11,   // maxmin: ready-list length of the current round
  CTL_RDQ0 = 12,     // multi-launch maxmin: the vote's ready-queue lengths, per round parity (2 words; rdq)
  CTL_NCL0 = 14,     // maxmin: alive-constraint list lengths (2 buffers)
  CTL_LASTR = 16,    // maxmin: last round that fixed a variable (+1 = rounds)
  CTL_PALIVE0 = 17,  // persistent maxmin: constraints alive after round r's update, per round parity (2 words)
  CTL_ERR = 19,      // persistent kernels: 1 = grid-barrier timeout, 2 = round guard
  CTL_RESEVAL = 20,  // persistent maxmin (profiling): rows re-evaluated by the vote, summed over the solve
  // multi-launch maxmin: the buffers in use live on the device, so a compaction needs no host round trip
  CTL_BUF = 21,    // alive-row buffer of the next vote (0 = the CSR, 1 / 2 = compaction targets)
  CTL_CB = 22,     // alive-constraint list in use (0 / 1)
  CTL_CMPGO = 23,  // the last compaction count found the rewrite worth it (cmp_scan -> cmp_write, mm_flip)
  // fair bottleneck: the reference's work summed over the rounds, three uint64 counters —
  // elements of the listed constraints, listed variables, listed constraints — each spread over kFbwSlots uint64
  // slots after the control words (CTL_FBW_AT; round 6: one counter word took one atomic per wave, 8,192 per
  // fb_var_inc launch, ~11 ns each on one address, drained after the grid's last wave)
  CTL_FBW = 24,
  CTL_WORDS = 32
};
constexpr int kFbwSlots = 64;
constexpr int CTL_FBW_AT = CTL_WORDS;                    // first int32 word of the [3][kFbwSlots] uint64 slots
constexpr int CTL_ALLOC = CTL_WORDS + 2 * 3 * kFbwSlots;  // int32 words of the control buffer

// maxmin per-constraint state, one 64-B line per constraint (array-of-structs): a constraint touched
// in a round dirties ONE line instead of one line in each of eight arrays (mm_update's write-back
// at the kernel boundary), and the first three fields are the decrement record: the three pushes of
// one element, issued by the 4 lanes of a quad in ONE wave instruction, are one memory-side atomic
// request (scripts/ubench_atomic.hip: 2.9x the rate of three separate arrays).
//
// Determinism: the decrements are summed as 64-bit FIXED-POINT integers (w*x scaled by 2^srem, w/p by
// 2^suse, per-constraint powers of two chosen at init so that a round's sum stays below 2^61, see
// dec_scale), so the sum is the same whatever order the atomics land in: a solve is bit-reproducible
// run to run, like the reference's sequential loop (maxmin.cpp:601-606).  Each term is rounded once
// to 2^-61 of the constraint's bound / initial usage (256x finer than one fp64 ulp of it).
struct alignas(64) CstRec {
  unsigned long long drem, duse, dcnt;  // fixed-point decrements pushed this round; dcnt = fixed elements
                                        // (dcnt > 0: touched this round)
  int64_t pad;              // unused (keeps the record one 64-B line)
  double rem, use;          // remaining, usage (maxmin.cpp:520-535, 603-658)
  double ratio;             // rem / use; +inf when out of the light table
  double bound;             // constraint bound
};
static_assert(sizeof(CstRec) == 64, "CstRec must be one 64-B line");

// Scale exponent of a non-negative magnitude bound m: 2^s * m < 2^61 (headroom 4x below int64).
__device__ __forceinline__ int dec_scale(double m) {
  if (!(m > 0) || !(m < __builtin_huge_val()))
    return 0;
  int s = 61 - __builtin_amdgcn_frexp_exp(m);  // m < 2^frexp_exp(m)
  return s < -1000 ? -1000 : (s > 1000 ? 1000 : s);
}
// One decrement as a fixed-point integer (the multiply by 2^s is exact; one rounding to integer).
__device__ __forceinline__ unsigned long long dec_q(double d, int s) {
  return (unsigned long long)__double2ll_rn(__builtin_amdgcn_ldexp(d, s));
}
__device__ __forceinline__ double dec_val(unsigned long long q, int s) {
  return __builtin_amdgcn_ldexp(double((long long)q), -s);
}
// Packed per-constraint word (cexp): bits 0-11 srem, 12-23 suse (signed: dec_scale stays within +-1000),
// bit 24 FATPIPE, bit 25 out of the light table.  A saturation pushing into constraint c reads this one word
// (scales, policy, liveness) instead of three arrays.
constexpr int32_t kCexpFat = 1 << 24;
constexpr int32_t kCexpDead = 1 << 25;
__host__ __device__ __forceinline__ int32_t cexp_pack(int srem, int suse, bool fat, bool dead) {
  return int32_t((uint32_t(srem) & 0xFFFu) | ((uint32_t(suse) & 0xFFFu) << 12)) | (fat ? kCexpFat : 0) |
         (dead ? kCexpDead : 0);
}
__device__ __forceinline__ int cexp_rem(int32_t e) { return int32_t(uint32_t(e) << 20) >> 20; }
__device__ __forceinline__ int cexp_use(int32_t e) { return int32_t(uint32_t(e) << 8) >> 20; }

// Relaxed agent-scope load: always a vector (global) load, never the scalar cache — for words other
// workgroups write inside a persistent launch (MI355X_MICROARCH.md, inter-workgroup visibility).
template <class T> __device__ __forceinline__ T ld_rlx(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> __device__ __forceinline__ void st_rlx(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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
  double* csc_u;             // [nnz] w / penalty of each CSC element (recomputed when penalties change)
  // [nnz] per CSC element, its variable's penalty and CSR row (begin | end << 32): a saturation reads them with
  // the element, coalesced, instead of gathering them per claimed variable after the claim (mm_elem_usage)
  double* csc_p;
  unsigned long long* csc_row;
  const double* pen;         // [nV]
  const double* vbound;      // [nV]
  const double* cbound;      // [nC]
  const uint8_t* cflags;     // [nC] bit0 FATPIPE, bit1 zero-weight enabled element
  // [nC] 1 = some variable has two elements on the constraint (expand() without expand_add; set at upload by
  // mm_dup_check): its saturation claims variables with atomicCAS.  Elsewhere a plain store claims — ready
  // constraints share no alive variable, so only a duplicate inside one constraint could claim twice.
  uint8_t* cdup;
  // per-variable state
  double* x;        // [nV] values (output)
  int32_t* fixr;    // [nV] fair bottleneck: last round the variable was listed (measurement only)
  int32_t* vstate;  // [nV] maxmin: 0 alive, r+1 = fixed or dropped in round r (claimed with atomicCAS)
  double* vtmp;     // [nV] fair bottleneck: mu
  uint8_t* vst;     // [nV] fair bottleneck: 1 listed / 0 not
  uint32_t* vstb;   // [nV/32 + 1] fair bottleneck: vst packed 32 per word for fbk_count (fb_pack_vst)
  // per-constraint state
  double* ratio;    // [nC] remaining/usage, +inf when out of the light table
  uint16_t* key;    // [nC] round-down 16-bit key of ratio, kDeadKey when out
  double* rem;      // [nC]
  double* use;      // [nC]
  CstRec* cst;      // [nC] maxmin: per-constraint record (one 64-B line, see CstRec)
  int32_t* cexp;    // [nC] maxmin: scale exponents of the decrements, FATPIPE and out flags (cexp_pack)
  // [nC] maxmin: alive elements whose variable votes for ANOTHER constraint (dense: mm_ready reads it
  // for every alive constraint each round); ready iff 0.  Vote moves add/subtract the moving
  // variable's multiplicity, fixed elements leave through the record's count in mm_update.
  int32_t* nvote;
  uint8_t* ctouch;  // [nC] maxmin, this round: 1 = received decrements, 2 = saturated (mm_update resets it)
  uint16_t* chg;    // [nC] last round (mod 2^16) in which ratio / liveness changed
  int32_t* ready;   // [nC + slack] ready constraints, one segment per mm_ready block
  int32_t* bready;  // [kMaxBlocks] ready count of each segment
  uint64_t* chgbits;  // [nC/64 + 2] bitmap: constraints changed in the last round (written by mm_update)
  int32_t* balive;  // [kMaxBlocks] constraints still alive after mm_update, per block
  int32_t* clist[2];  // [nC] alive-constraint lists (periodically compacted)
  // alive-row buffers: 0 = the original CSR (identity ids), 1/2 = compaction targets
  const int32_t* cvar[3];
  const uint32_t* crow[3];
  const int32_t* ccol[3];
  int32_t* rtgt[3];  // per row: constraint the variable votes for; kUnvoted / kRetired
  uint16_t* skey[3];  // per row: min key over the row's OTHER constraints at its last vote (0 if bounded)
  int32_t* bsum;    // compaction scratch: per-block rows / elems (2 x blocks)
  // fair bottleneck: CSC chunks (lmm_fb_kernels.hpp) and the per-constraint exchange buffers
  int32_t nch;               // number of chunks
  const int32_t* ch_cnst;    // [nch] constraint of each chunk
  const uint32_t* ch_beg;    // [nch] first CSC element of each chunk
  const int32_t* c_ch;       // [nC+1] first chunk of each constraint
  int32_t* pcnt;             // [nch] listed variables per chunk
  double* pacc;              // [nch] sum / min of w*mu per chunk
  uint8_t* erased;           // [nC] erased in the current round
  int32_t* xnb;              // [nC+1] listed count per constraint (+ any-listed flag); sharded: all-reduce SUM
  double* xmin;              // [nC] one context: min of w*mu per FATPIPE constraint
  double* fbd;               // [nnz] one context: w*mu of every shared constraint's element, CSC order
  int32_t* fb_long;          // [nC+1] one context: count, then the long shared constraints (fb_long_list)
  // one context, locality order of the increments' gathers (fb_perm): the variables sorted by their rows' first
  // and last constraint (a flow's source- and destination-side links), mu kept in that order too
  int32_t* vperm;            // [nV] position of each variable in the locality order
  int32_t* csc_vp;           // [nnz] csc_v through vperm
  double* mu_p;              // [nV] mu (vtmp) in the locality order
  uint64_t* flagbits;  // [nC/64 + 2] measurement only: targets of the rows the filter queued (kDiag)
  // frontier engine (lmm_frontier_kernels.hpp): votes registered at their target constraint
  const int2* csr_cs;        // [nnz] per CSR element: its constraint and its CSC position (one 8-B pair)
  double2* pvb;              // [nV] per variable: (bound, penalty) of this solve, one 16-B record
  uint32_t* key32;           // [nC] 32-bit key of the ratio (ratio_key32), kDead32 when out of the light table
  uint32_t* vslot;           // [nnz] per CSC element: floor of the vote registered there, kNoVoter if none
  uint32_t* minfl;           // [nC] lower bound of the floors registered at the constraint (kNoVoter: none)
  unsigned long long* fq_a;  // [nnz] re-vote queue, one segment per fr_update workgroup: variable | target << 32
  unsigned long long* fq_b;  // [nnz]   and the variable's CSR row (begin | end << 32)
  int32_t* fq_n;             // [nC / kFB + 1] queued variables per segment
  int32_t* rdq[2];   // round engine, short rows (LMMHIP_RDQ): constraints the vote made ready, by round parity
  int32_t* rqst;     // [nC] the round a constraint was last queued for (one entry per constraint and round)
  int32_t* useg;     // [blocks x kUSeg] the update's ready candidates for the next round, a segment per workgroup
  int32_t* ucnt;     // [blocks] their counts
  uint2* crec[3];    // round engine, short rows: per alive row {cvar, crow} in one 8-B record (vote_row)
  int32_t* ctl;     // control words
  // one-context FairBottleneck: pinned host words fbk_share writes itself (system scope) — [0] rounds started, [1] 1
  // once the solve is over — by which the host paces its rounds without a control-word copy kernel per round
  // (solve_fair_rounds).  Null elsewhere (the max-min engines, the sharded FairBottleneck phases)
  int32_t* hprog;
  int32_t* vstat;   // profiling only (else null): [round][block] re-evaluated rows / elements
  // round anatomy (diagnostic build LMM_ANAT=1 only, else null): per-wave stamps of the round engine's kernels in
  // the rounds anat_r[0..kAnatSlots) (lmm_anat below)
  unsigned long long* anat;
  int32_t anat_r[4];
};

// Alive-row variable ids carry the variable's "bounded" flag in the sign bit (set at every solve's init),
// so the re-vote of an unbounded variable skips its bound and penalty gathers.
__device__ __forceinline__ int rvar(int32_t cv) { return cv & 0x7FFFFFFF; }
__device__ __forceinline__ bool rbounded(int32_t cv) { return cv < 0; }

constexpr int kStatRounds = 4096;  // rounds covered by the profiling counters
constexpr int32_t kUnvoted = -1;   // row target: not evaluated yet
// A signalling NaN (quiet bit clear, distinctive payload): no fp64 arithmetic returns it, so it can mark "leave this
// slot alone" inside an array of values (rs_values_mark, lmmhip_res_values_sliced).
constexpr unsigned long long kValKeep = 0x7FF4C0FFEE5107E5ull;  // (= LMMHIP_VAL_KEEP, include/lmm/lmm_hip.h)
constexpr int32_t kRetired = -2;   // row target: variable fixed or dropped (skip until compaction)

__device__ __forceinline__ double dinf() { return __builtin_huge_val(); }

// 16-bit monotone key: round the ratio down to f32, keep the upper 16 bits (sign, exponent, 7 bits
// of mantissa).  Monotone non-decreasing, so key(a) < key(b) => a < b; equal keys need the exact
// fp64 comparison.
#ifndef LMM_KEY_MANT
#define LMM_KEY_MANT 7  // mantissa bits of the key (build knob, measurement)
#endif
__device__ __forceinline__ uint16_t ratio_key(double r) {
  float f = __double2float_rd(r);
  return uint16_t(__float_as_uint(f) >> (23 - LMM_KEY_MANT));
}

// 32-bit monotone key (frontier engine): the ratio rounded down to f32, its bits.  Ties between different
// ratios are 2^16 times rarer than with ratio_key, so a vote's floor is crossed only when its target's ratio
// really reaches another constraint's (within 2^-24).
constexpr uint32_t kDead32 = 0xFFFFFFFFu;  // > the bits of every non-negative f32, +inf included
__device__ __forceinline__ uint32_t ratio_key32(double r) { return __float_as_uint(__double2float_rd(r)); }

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
template <int W> __device__ __forceinline__ int grp_imin(int v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1)
    v = min(v, __shfl_xor(v, o, W));
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

// Append `pred` items to a global list with one atomic per wave (ballot + popcount).
__device__ __forceinline__ int wave_append(bool pred, int32_t* counter) {
  const unsigned long long m = __ballot(pred);
  if (!m)
    return -1;
  const int lane = threadIdx.x & (kWave - 1);
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader)
    base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader, kWave);
  return pred ? base + __popcll(m & ((1ull << lane) - 1)) : -1;
}

// Append `pred` items to a global list with ONE atomic per block (all kBlock threads must call).
__device__ __forceinline__ int block_append(bool pred, int32_t* counter) {
  __shared__ int wcnt[kBlock / kWave];
  __shared__ int bbase;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const unsigned long long m = __ballot(pred);
  if (lane == 0)
    wcnt[w] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int i = 0; i < kBlock / kWave; i++) {
      const int c = wcnt[i];
      wcnt[i] = tot;
      tot += c;
    }
    bbase = tot ? atomicAdd(counter, tot) : 0;
  }
  __syncthreads();
  const int pos = bbase + wcnt[w] + __popcll(m & ((1ull << lane) - 1));
  __syncthreads();
  return pred ? pos : -1;
}

inline int grid_for(int64_t n, int per_block) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1)
    g = 1;
  if (g > kMaxBlocks)
    g = kMaxBlocks;
  return int(g);
}

// ---- round anatomy (diagnostic build only: LMM_ANAT=1, scripts/anatomy.py) ----
// In the rounds named by Dev::anat_r, every wave of mm_vote_lane / mm_saturate_q / mm_update writes one record of
// kAnatFields words into anat[((slot * kAnatKernels + kernel) * kAnatWaves + wave) * kAnatFields]: its entry and exit on the
// 100-MHz wall clock (s_memrealtime, one clock for the whole chip), its workgroup, and the time it spent at each
// dependent level of its work (the clock read waits for the level's loaded values, so a level's time is from the
// previous stamp to the arrival of that level's data).  The stamps serialise what the real kernel overlaps: read
// the SHARES of a round, not the stamped build's length (cdna_hip_programming.md §7, in-kernel stamps).  In the
// product build (LMM_ANAT=0) none of this is compiled.
#ifndef LMM_ANAT
#define LMM_ANAT 0
#endif
constexpr int kAnatSlots = 4;
constexpr int kAnatKernels = 4;
constexpr int kAnatFields = 20;
constexpr int kAnatWaves = 8192;
// the round engine's vote / saturation / update; the frontier engine's fr_vote / fr_sat / fr_update / fr_sat_big
enum : int { ANAT_VOTE = 0, ANAT_SAT = 1, ANAT_UPD = 2, ANAT_SATB = 3 };
#if LMM_ANAT
__device__ __forceinline__ unsigned long long anat_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
// the clock read after `v` has arrived (a use of its register)
template <class T> __device__ __forceinline__ void anat_use(const T& v) {
  if constexpr (sizeof(T) == 8)
    asm volatile("" : : "v"(v) : "memory");
  else
    asm volatile("" : : "v"(uint32_t(v)) : "memory");
}
// per-wave accumulators of the dependent levels (registers; a field per level), and the running stamp
struct AnatAcc {
  unsigned lv[10];
  unsigned long long at;
};
#define ANAT_LVL(aa, i, dep)                      \
  do {                                            \
    anat_use(dep);                                \
    const unsigned long long t_ = anat_now();     \
    (aa).lv[i] += unsigned(t_ - (aa).at);         \
    (aa).at = t_;                                 \
  } while (0)
__device__ __forceinline__ unsigned anat_wmax(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v = max(v, (unsigned)__shfl_xor(int(v), o, kWave));
  return v;
}
__device__ __forceinline__ int anat_slot(const Dev& s, int round) {
  if (!s.anat)
    return -1;
  for (int k = 0; k < kAnatSlots; k++)
    if (s.anat_r[k] == round)
      return k;
  return -1;
}
__device__ __forceinline__ unsigned long long* anat_rec(const Dev& s, int slot, int kernel) {
  const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  if (slot < 0 || wave >= kAnatWaves)
    return nullptr;
  return s.anat + ((int64_t(slot) * kAnatKernels + kernel) * kAnatWaves + wave) * kAnatFields;
}
#endif

}  // namespace lmmdev
