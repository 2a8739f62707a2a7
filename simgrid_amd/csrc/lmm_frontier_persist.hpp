// lmm_frontier_persist.hpp — the frontier engine's rounds in ONE launch per solve (gfx950; included by lmm_hip.hip).
//
// The multi-launch frontier engine (lmm_frontier_kernels.hpp) spends three launches per round; on a system whose
// rounds are short (C4: 100 rounds of ~30 us) a kernel's fixed cost — a one-thread kernel takes ~4 us in the trace
// on this chip — is a large share of each.  Here the same phase bodies run inside one launch of G workgroups of
// kFB threads, each looping over the multi-launch grid's (virtual) workgroups, with the persistent engine's grid
// barriers between the phases (lmm_persist_kernels.hpp: XCD-hierarchical, agent release / acquire) and its launch
// rendezvous with a deadline (co-residency; the host falls back to the multi-launch frontier on a close):
//
//   round r:  [r >= 1]  fr_vote_blk    over ceil(nblk / spb) virtual workgroups   | barrier
//                       fr_sat_blk     over nblk                                  | barrier
//             [list]    fr_sat_big     over the grid's waves                      | barrier
//                       fr_update_blk  over nblk                                  | barrier
//             no constraint alive after the update -> done (every workgroup reads the same word)
//
// Round 0's vote (fr_vote_all, fr_minfl_all) and the init stay launches of their own, before this one.  The
// decisions, and so the values, are the multi-launch frontier engine's bit for bit (tests/test_gpu_engines.py).
#pragma once
#include "lmm_frontier_kernels.hpp"
#include "lmm_persist_kernels.hpp"

namespace lmmdev {

template <int R>
__global__ void __launch_bounds__(kFB) fr_persist(Dev s, unsigned* barw, double prec, int max_rounds, int spb,
                                                  int bigch, int bigw, int big, long long rdv_ticks,
                                                  int32_t* hflag) {
  __shared__ union {
    SatLds<kFB, kFB> sat;
    FrUpdLds upd;
    int wpre[kFB / kWave][kWave];
  } L;
  PBar b{barw, &s.ctl[CTL_ERR], 0, 0, 0, nullptr, 0, 0};
  if (!bar_rdv(b, rdv_ticks, hflag))  // before any store (the host may fall back to the multi-launch engine)
    return;
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  const int64_t nblk = (int64_t(s.nC) + kFB - 1) / kFB;
  const int64_t nvote = (nblk + spb - 1) / spb;
  unsigned gen = 0;
  for (int r = 0;; r++) {
    if (r > 0) {
      if (lead)
        st_rlx(&s.ctl[CTL_PALIVE0 + (r & 1)], 0);  // this round's update raises it (last read a barrier ago)
      for (int64_t vb = blockIdx.x; vb < nvote; vb += gridDim.x)  // workgroup-uniform
        fr_vote_blk<false, R, true>(s, r, spb, int(vb));
      if (!grid_sync(b, ++gen))
        return;
    }
    for (int64_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {
      fr_sat_blk<kFB, false>(s, r, bigch, int(vb), L.sat);
      __syncthreads();
    }
    if (!grid_sync(b, ++gen))
      return;
    if (big) {
      const int nb = ld_rlx(&s.ctl[CTL_NREADY]);
      if (nb > 0) {  // grid-uniform (read after the barrier)
        if (lead)
          s.ctl[CTL_LASTR] = r;
        const int64_t wave = (int64_t(blockIdx.x) * kFB + threadIdx.x) / kWave;
        fr_sat_big_waves<true>(s, r, bigw, nb, wave, int64_t(gridDim.x) * (kFB / kWave), L.wpre[threadIdx.x / kWave]);
        if (!grid_sync(b, ++gen))
          return;
      }
    }
    for (int64_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {  // (virtual workgroup 0 resets CTL_NREADY)
      fr_update_blk<true>(s, r, prec, int(vb), L.upd);
      __syncthreads();
    }
    if (!grid_sync(b, ++gen))
      return;
    if (ld_rlx(&s.ctl[CTL_PALIVE0 + (r & 1)]) == 0) {  // light table empty (maxmin.cpp:680)
      if (lead)
        st_rlx(&s.ctl[CTL_DONE], 1);
      return;
    }
    if (r + 1 >= max_rounds) {  // every round fixes a variable: a solver bug
      if (lead)
        st_rlx(&s.ctl[CTL_ERR], 2);
      return;
    }
  }
}

}  // namespace lmmdev
