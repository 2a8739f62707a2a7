// lmm_persist_kernels.hpp — System::lmm_solve as ONE persistent launch per solve (gfx950).
//
// The round loop of maxmin.cpp:560-680 (local-minimum progressive filling, lmm_maxmin_kernels.hpp) with
// every round's phases inside one cooperative launch, separated by XCD-hierarchical grid barriers, and
// the termination test (maxmin.cpp:680: the light table is empty) decided on the device — no host
// round-trips, no per-round launches.  One 1024-thread workgroup per CU (16 waves), so the vote phase
// can hold the changed-constraint bitmap (up to 2^20 constraints) in LDS.
//
//   init            mm_init_cnsts / mm_init_vars bodies (maxmin.cpp:509-555)
//   round r:  V     filter + re-vote of the rows whose target's key changed (vote_row)
//             |     grid barrier
//             S     ready test (nvote == 0) fused with saturation (sat_block: the ready constraints'
//             |     CSC chunks shared by the workgroup's waves), maxmin.cpp:578-606
//             |     grid barrier
//             U     constraint update (update_wave), maxmin.cpp:603-658; alive count
//             |     grid barrier; alive == 0 -> done (every block reads the same count)
//             [C]   every cmp_every rounds: compaction of the alive rows (one pass, one barrier)
//
// Results are bit-identical to the multi-launch engine (same phase bodies, integer / fixed-point
// atomics only): tests/test_gpu_engines.py.
#pragma once
#include "lmm_maxmin_kernels.hpp"

namespace lmmdev {

constexpr int kPB = 1024;            // threads per workgroup (one workgroup per CU)
constexpr int kPW = kPB / kWave;     // waves per workgroup
constexpr int kPBitWords = 16384;    // LDS bitmap: 2^20 constraints (128 KB)
constexpr int kPFilt = 4;            // rows per thread per filter step
constexpr long long kSpinTicks = 400000000;  // 4 s of the 100 MHz wall clock: a barrier wait gives up
constexpr unsigned kPBlkCap = 1024;          // barriers with per-workgroup timestamps (profiling)

// Grid-barrier words (zeroed by the host before every launch), each counter on its own 64-B line.
enum : int {
  BAR_XCNT = 0,     // [8 x 16] arrivals per XCC (monotonic: gen * blocks-on-the-XCC)
  BAR_TOP = 128,    // arrivals of the XCC leaders (monotonic: gen * XCCs)
  BAR_GEN = 144,    // chip generation (released by the last leader)
  BAR_XGEN = 160,   // [8 x 16] per-XCC generation (released by the XCC's leader)
  BAR_XSIZE = 288,  // [8 x 16] workgroups on each XCC (counted at launch)
  BAR_FLAT = 416,   // launch rendezvous
  BAR_ALLOC = 432,  // u64 (2 words, 8-B aligned): compaction allocator (rows << 32 | elements)
  BAR_PALIVE = 448,  // [2 parities x 16]: constraints alive after a round's update, 8 partial words each
  BAR_WORDS = 480
};

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v & 7u;
}

// Relaxed poll of one word until it reaches `target`; gives up (error word 1) after kSpinTicks.
__device__ __forceinline__ bool spin_geq(unsigned* w, unsigned target, int32_t* err) {
  const long long t0 = wall_clock64();
  while (ld_rlx(w) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > kSpinTicks) {
      st_rlx(err, 1);
      return false;
    }
  }
  return true;
}

struct PBar {
  unsigned* w;
  int32_t* err;
  unsigned xcc, xsize, nx;  // meaningful in thread 0 only
  long long* pt;            // profiling (else null): per barrier [last arrival, workgroup 0's exit] (wall clock)
  unsigned pt_cap;          // barriers covered
  int sysf;                 // 1: system-scope release / acquire (also writes back / invalidates the L2)
};

// Launch rendezvous with a short deadline ("co-residency"), at kernel start, before any store:
// a workgroup counts itself in BAR_FLAT with a compare-and-swap unless the rendezvous is closed, then waits until
// every workgroup of the grid has arrived.  One that has waited `ticks` (wall clock) closes the rendezvous instead
// — one compare-and-swap on the same word, so the count cannot complete behind it — and tells the host through
// the mapped word *hflag; every arrived workgroup then leaves, and a late one (held back by another kernel or
// process occupying CUs, possibly for seconds) finds it closed and returns at once.  None of them has written
// anything, so the host re-runs the solve with the multi-launch engine right away, on the free CUs.
constexpr unsigned kRdvClosed = 1u << 20;  // BAR_FLAT: closed flag above the arrival count

// (out of line: inlined into mm_persist, whose round phases sit at the 128-VGPR budget, it tipped it over)
__device__ __noinline__ int rdv_join(unsigned* w, unsigned xcc, unsigned grid, long long ticks, int32_t* hflag) {
  unsigned v = ld_rlx(&w[BAR_FLAT]);
  if (v & kRdvClosed)
    return 0;
  // the XCC count first (visible before the arrival: a workgroup that sees the full count reads it); a
  // workgroup that then finds the rendezvous closed leaves a count nobody reads
  __hip_atomic_fetch_add(&w[BAR_XSIZE + 16 * xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (;;) {
    const unsigned prev = atomicCAS(&w[BAR_FLAT], v, v + 1);
    if (prev == v)
      break;
    if (prev & kRdvClosed)
      return 0;
    v = prev;
  }
  const long long t0 = wall_clock64();
  for (;;) {
    v = ld_rlx(&w[BAR_FLAT]);
    if (v & kRdvClosed)
      return 0;
    if (v == grid)
      return 1;
    if (wall_clock64() - t0 > ticks && atomicCAS(&w[BAR_FLAT], v, v | kRdvClosed) == v) {
      if (hflag)
        __hip_atomic_store(hflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ bool bar_rdv(PBar& b, long long ticks, int32_t* hflag) {
  __shared__ int ok_sh;
  if (threadIdx.x == 0) {
    const int ok = rdv_join(b.w, xcc_id(), gridDim.x, ticks, hflag);
    if (ok) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      b.xcc = xcc_id();
      b.xsize = ld_rlx(&b.w[BAR_XSIZE + 16 * b.xcc]);
      b.nx = 0;
      for (int i = 0; i < 8; i++)
        b.nx += ld_rlx(&b.w[BAR_XSIZE + 16 * i]) != 0;
    }
    ok_sh = ok;
  }
  __syncthreads();
  return ok_sh;
}

// Grid barrier number `gen` (1, 2, ...): every wave drains its stores to L2; the last workgroup of
// each XCC writes that XCC's L2 back (agent release) and arrives at the chip counter; the last XCC
// leader releases the generation; every workgroup acquires (MI355X_MICROARCH.md, barrier-xcd and
// the valid producer / consumer forms).  Returns false when a wait timed out (the kernel then ends).
__device__ bool grid_sync(const PBar& b, unsigned gen) {
  __shared__ int ok_sh;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    if (b.pt && gen < b.pt_cap) {
      const long long now = wall_clock64();
      atomicMax(&b.pt[2 * gen], now);
      if (gen < kPBlkCap)  // per-workgroup arrival
        b.pt[2 * b.pt_cap + 2 * (size_t(gen) * gridDim.x + blockIdx.x)] = now;
    }
    const unsigned a =
        __hip_atomic_fetch_add(&b.w[BAR_XCNT + 16 * b.xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a == gen * b.xsize - 1) {  // XCC leader
      if (b.sysf)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      else
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&b.w[BAR_TOP], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == gen * b.nx - 1)
        st_rlx(&b.w[BAR_GEN], gen);
      else
        ok = spin_geq(&b.w[BAR_GEN], gen, b.err);
      if (ok)
        st_rlx(&b.w[BAR_XGEN + 16 * b.xcc], gen);
    } else {
      ok = spin_geq(&b.w[BAR_XGEN + 16 * b.xcc], gen, b.err);
    }
    if (b.sysf)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (b.pt && gen < b.pt_cap) {
      const long long now = wall_clock64();
      if (blockIdx.x == 0)
        b.pt[2 * gen + 1] = now;
      if (gen < kPBlkCap)  // per-workgroup exit
        b.pt[2 * b.pt_cap + 2 * (size_t(gen) * gridDim.x + blockIdx.x) + 1] = now;
    }
    ok_sh = ok;
  }
  __syncthreads();
  return ok_sh;
}

// Wave id interleaved over the workgroups (wave w of workgroup b -> w * grid + b): consecutive 64-item
// groups land on different CUs (and XCDs), so a small item count still spreads over the whole chip.
__device__ __forceinline__ int64_t pwave() { return int64_t(threadIdx.x / kWave) * gridDim.x + blockIdx.x; }

template <bool kBits> struct PVoteLds {
  uint64_t bits[kBits ? kPBitWords : 2];
  int q[kPW * kQW];  // per-wave queues of rows to re-vote (vote_waves)
  int st0, st1;
};
using PSatLds = SatLds<kPB, 4 * kPB>;
template <bool kBits> union PLds {
  PVoteLds<kBits> v;
  PSatLds sat;  // ready test + saturation
  int pre[kPW][kWave];  // compaction scratch
  int cnt;              // update: alive constraints of the workgroup
};

// V: the rows of buffer `buf`, one contiguous chunk (a multiple of 64) per workgroup, filtered and re-voted
// by vote_waves (every wave on its own share, no workgroup barrier after the bitmap load).
template <bool kBits, int R>
__device__ void p_vote(const Dev& s, int buf, int round, int64_t nrows, PVoteLds<kBits>& L, bool count) {
  if (threadIdx.x == 0)
    L.st0 = 0;
  if (kBits)
    load_bits<kPB>(s, L.bits);
  __syncthreads();
  const int64_t per = ((nrows + gridDim.x - 1) / gridDim.x + kWave - 1) / kWave * kWave;
  const int64_t lo = int64_t(blockIdx.x) * per;
  const int64_t hi = lo + per < nrows ? lo + per : nrows;
  int nq = 0;
  if (lo < hi)
    nq = vote_waves<kBits, R, kPFilt, 0>(s, buf, round, lo, hi, L.bits, L.q + (threadIdx.x / kWave) * kQW, &L.st0,
                                         &L.st1, s.key);
  if (count) {  // (profiling) one add per workgroup: a per-wave add to one word cost ~6 us per round on C4
    if ((threadIdx.x & (kWave - 1)) == 0 && nq)
      atomicAdd(&L.st0, nq);
    __syncthreads();
    if (threadIdx.x == 0 && L.st0)
      atomicAdd(&s.ctl[CTL_RESEVAL], L.st0);
  }
}

// S: ready test fused with saturation over every constraint (identity ids), sat_block (the ready
// constraints' CSC chunks shared by the workgroup's 16 waves).
__device__ void p_saturate(const Dev& s, int round, PSatLds& L) { sat_block<kPB, 4 * kPB>(s, round, nullptr, s.nC, L); }

// C: compaction of the alive rows of buffer `in` into `out`, one contiguous chunk of rows per workgroup:
// pass 1 counts the chunk's alive rows and elements, ONE 64-bit atomic per workgroup allocates both
// (rows << 32 | elements, so consecutive allocations stay consistent: row k's end = row k+1's start),
// pass 2 writes them in chunk order (workgroup scans).  Chunks land in allocation order: row order is
// free (every vote, claim and fixed-point sum is order-independent).
__device__ void p_compact(const Dev& s, int in, int out, int64_t nrows, unsigned long long* alloc, int* sh) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int32_t* ovar = const_cast<int32_t*>(s.cvar[out]);
  uint32_t* orow = const_cast<uint32_t*>(s.crow[out]);
  int32_t* ocol = const_cast<int32_t*>(s.ccol[out]);
  const int64_t per = ((nrows + gridDim.x - 1) / gridDim.x + kPB - 1) / kPB * kPB;
  const int64_t lo = int64_t(blockIdx.x) * per;
  const int64_t hi = lo + per < nrows ? lo + per : nrows;
  int nr = 0, ne = 0;  // pass 1
  for (int64_t row = lo + threadIdx.x; row < hi; row += kPB)
    if (s.vstate[rvar(s.cvar[in][row])] == 0) {
      nr++;
      ne += int(s.crow[in][row + 1] - s.crow[in][row]);
    }
  nr = grp_isum<kWave>(nr);
  ne = grp_isum<kWave>(ne);
  if (lane == 0) {
    sh[2 * w] = nr;
    sh[2 * w + 1] = ne;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tr = 0, te = 0;
    for (int i = 0; i < kPW; i++) {
      tr += unsigned(sh[2 * i]);
      te += unsigned(sh[2 * i + 1]);
    }
    const unsigned long long old = tr ? atomicAdd(alloc, (tr << 32) | te) : 0ull;
    sh[2 * kPW] = int(old >> 32);
    sh[2 * kPW + 1] = int(uint32_t(old));
    sh[2 * kPW + 2] = tr != 0;
  }
  __syncthreads();
  uint32_t rbase = uint32_t(sh[2 * kPW]), ebase = uint32_t(sh[2 * kPW + 1]);
  const bool allocated = sh[2 * kPW + 2] != 0;
  __syncthreads();
  for (int64_t b0 = lo; b0 < hi; b0 += kPB) {  // pass 2, workgroup-uniform
    const int64_t row = b0 + threadIdx.x;
    int32_t v = 0;  // (bounded flag kept)
    bool al = false;
    uint32_t b = 0, e = 0;
    if (row < hi) {
      v = s.cvar[in][row];
      al = s.vstate[rvar(v)] == 0;
      if (al) {
        b = s.crow[in][row];
        e = s.crow[in][row + 1];
      }
    }
    int xr = al, xe = int(e - b);
    int ir = xr, ie = xe;  // inclusive wave scans
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int tr = __shfl_up(ir, o, kWave), te = __shfl_up(ie, o, kWave);
      if (lane >= o) {
        ir += tr;
        ie += te;
      }
    }
    if (lane == kWave - 1) {
      sh[2 * w] = ir;
      sh[2 * w + 1] = ie;
    }
    __syncthreads();
    int orr = 0, oe = 0, tr = 0, te = 0;
    for (int i = 0; i < kPW; i++) {
      orr += i < w ? sh[2 * i] : 0;
      oe += i < w ? sh[2 * i + 1] : 0;
      tr += sh[2 * i];
      te += sh[2 * i + 1];
    }
    if (al) {
      const uint32_t o = rbase + uint32_t(orr + ir - xr);
      const uint32_t dst = ebase + uint32_t(oe + ie - xe);
      ovar[o] = v;
      s.rtgt[out][o] = s.rtgt[in][row];
      s.skey[out][o] = s.skey[in][row];
      orow[o] = dst;
      for (int j = 0; j < xe; j++)
        ocol[dst + j] = s.ccol[in][b + j];
    }
    rbase += uint32_t(tr);
    ebase += uint32_t(te);
    __syncthreads();
  }
  // the end of the workgroup's last row: the next allocation's start (or the total, for the last one)
  if (threadIdx.x == 0 && allocated)
    orow[rbase] = ebase;
}

template <bool kBits, int R>
__global__ void __launch_bounds__(kPB) mm_persist(Dev s, unsigned* barw, double prec, int max_rounds,
                                                  int cmp_every, long long* pt, unsigned pt_cap, int sysf,
                                                  long long rdv_ticks, int32_t* hflag) {
  __shared__ PLds<kBits> L;
  PBar b{barw, &s.ctl[CTL_ERR], 0, 0, 0, pt, pt_cap, sysf};
  if (pt && blockIdx.x == 0 && threadIdx.x == 0)
    pt[1] = wall_clock64();  // launch (barrier 0's exit slot)
  unsigned long long* alloc = reinterpret_cast<unsigned long long*>(barw + BAR_ALLOC);
  int32_t* palive = reinterpret_cast<int32_t*>(barw + BAR_PALIVE);
  const int lane = threadIdx.x & (kWave - 1);
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  // the launch rendezvous before any store: a workgroup that finds it closed (late: the host has fallen back to
  // the multi-launch engine, which is using the same buffers) or that closes it returns without having written
  if (!bar_rdv(b, rdv_ticks, hflag))
    return;
  unsigned gen = 0;
  init_cnsts_waves(s, prec, pwave(), int64_t(gridDim.x) * kPW);  // init (maxmin.cpp:509-555)
  init_vars_range(s, int64_t(blockIdx.x) * kPB + threadIdx.x, int64_t(gridDim.x) * kPB);
  if (!grid_sync(b, ++gen))
    return;
  int buf = 0;
  int64_t nrows = s.nV;
  for (int r = 0;; r++) {
    p_vote<kBits, R>(s, buf, r, nrows, L.v, pt != nullptr);
    if (!grid_sync(b, ++gen))
      return;
    if (lead) {  // words first used later in this round, last read before the previous barrier
      for (int i = 0; i < 8; i++)
        st_rlx(&palive[16 * ((r + 1) & 1) + i], 0);
      st_rlx(alloc, 0ull);
    }
    p_saturate(s, r, L.sat);
    if (!grid_sync(b, ++gen))
      return;
    if (threadIdx.x == 0)
      L.cnt = 0;
    __syncthreads();
    {
      int alive = 0;
      bool touch = false;
      constexpr int kU = 3;  // groups of 64 constraints per wave step, loads in flight together
      const int64_t stride = int64_t(gridDim.x) * kPB;
      for (int64_t base = pwave() * kWave; base < s.nC; base += kU * stride)  // wave-uniform
        alive += update_groups<kU>(s, base, stride, r, prec, &touch);
      alive = grp_isum<kWave>(alive);
      if (lane == 0 && alive)
        atomicAdd(&L.cnt, alive);
    }
    __syncthreads();
    // one add per workgroup, spread over 8 words (a single word takes ~88 atomics/us)
    if (threadIdx.x == 0 && L.cnt)
      atomicAdd(&palive[16 * (r & 1) + (blockIdx.x & 7)], L.cnt);
    if (!grid_sync(b, ++gen))
      return;
    int alive_all = 0;
    for (int i = 0; i < 8; i++)
      alive_all += ld_rlx(&palive[16 * (r & 1) + i]);
    if (alive_all == 0) {  // light table empty (maxmin.cpp:680)
      if (lead) {  // every round with a live constraint fixes a variable: rounds = r + 1
        s.ctl[CTL_ROUNDS] = r + 1;
        s.ctl[CTL_LASTR] = r;
      }
      return;
    }
    if (r + 1 >= max_rounds) {  // every round fixes a variable: a solver bug
      if (lead)
        st_rlx(&s.ctl[CTL_ERR], 2);
      return;
    }
    if (cmp_every > 0 && r % cmp_every == cmp_every - 1 && nrows > kPB) {
      const int out = buf == 1 ? 2 : 1;
      p_compact(s, buf, out, nrows, alloc, &L.pre[0][0]);
      if (!grid_sync(b, ++gen))
        return;
      nrows = int64_t(ld_rlx(alloc) >> 32);
      buf = out;
    }
  }
}

}  // namespace lmmdev
