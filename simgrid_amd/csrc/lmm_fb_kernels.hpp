// lmm_fb_kernels.hpp — FairBottleneck::bottleneck_solve on gfx950 (included by lmm_hip.hip).
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

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

}  // namespace lmmdev
