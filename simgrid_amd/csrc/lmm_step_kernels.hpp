// lmm_step_kernels.hpp — the model side of a simulation step on the device, over the
// values of the last solve: the action state (remains, max duration, latency) stays in HBM between
// steps, and only the few actions with an event go back to the host.
//   act_next_event  Model::next_occuring_event_full (Model.cpp:103-129): min over actions of
//                   remains / value (value > 0; 0 when remains <= 0) and of the max duration (>= 0);
//                   network / ptask models also take latency > 0 (network_interface.cpp:57-70,
//                   ptask_L07.cpp:69-82).
//   act_update      update_actions_state_full of CPU Cas01 (cpu_interface.cpp:37-51), network CM02
//                   (network_cm02.cpp:128-163) and ptask L07 (ptask_L07.cpp:84-118): latency, remains
//                   and max-duration updates with double_update (surf_interface.hpp:34-42) and the
//                   finish test.  Every action is independent: element-wise IEEE arithmetic in the
//                   reference's order (built with -ffp-contract=off), so results are bit-identical.
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

enum : int { MODEL_CPU = 0, MODEL_CM02 = 1, MODEL_L07 = 2 };
enum : uint8_t { EV_FINISHED = 1, EV_LATENCY_PAID = 2 };
enum : uint8_t { ACT_NO_CNST = 1, ACT_SUSPENDED = 2, ACT_NOT_STARTED = 4 };
// ActionHeap::Type (Action.hpp) of an action in the LAZY models' heap; UNSET = not in the heap.
enum : uint8_t { HEAP_UNSET = 0, HEAP_LATENCY = 1, HEAP_MAX_DURATION = 2, HEAP_NORMAL = 3 };
constexpr double kNoMaxDuration = -1.0;  // Action.hpp:17

struct ActDev {
  int64_t n;
  const int32_t* vidx;     // dense variable index of each action's variable, -1 = not solved (value 0)
  double* remains;
  double* max_duration;
  double* latency;
  double* penalty;         // the variable's current penalty (finish test)
  const double* share_pen; // CM02: sharing penalty restored once the latency is paid
  const uint8_t* flags;    // ACT_NO_CNST, ACT_SUSPENDED
  uint8_t* events;         // EV_* of the last update
  unsigned long long* umin;  // next-event reduction (bit pattern of a non-negative double)
  int32_t* nev;            // number of actions with an event in the last update
  // LAZY update (lmmhip_actions_lazy_*): Action::last_update_ / last_value_ / start_time_ and the
  // action's ActionHeap entry (date + type) — the heap itself is a min-reduction over `date`.
  double* last_update;
  double* last_value;
  const double* start_time;
  double* date;            // heap date (+inf when not in the heap)
  uint8_t* htype;          // HEAP_*
  int32_t* due;            // compacted due actions (lmmhip_actions_lazy_due)
  int32_t* ndue;
  int32_t* err;            // DIE_IMPOSSIBLE of next_occuring_event_lazy (Model.cpp:95-96)
};

__device__ __forceinline__ void double_update(double& v, double d, double prec) {
  v -= d;
  if (v < prec)
    v = 0.0;
}

__global__ void __launch_bounds__(kBlock) act_next_event(ActDev a, const double* x, int with_latency) {
  double m = dinf();
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t k = a.vidx[i];
    const double value = k >= 0 ? x[k] : 0.0;
    if (value > 0)
      m = fmin(m, a.remains[i] > 0 ? a.remains[i] / value : 0.0);
    const double md = a.max_duration[i];
    if (md >= 0)
      m = fmin(m, md);
    if (with_latency && a.latency[i] > 0)
      m = fmin(m, a.latency[i]);
  }
  m = wave_min(m) + 0.0;  // +0.0: no -0.0 in the unsigned ordering below
  if ((threadIdx.x & (kWave - 1)) == 0 && m != dinf())
    atomicMin(a.umin, (unsigned long long)__double_as_longlong(m));
}

__global__ void __launch_bounds__(kBlock) act_update(ActDev a, const double* x, int model, double delta,
                                                      double maxmin_prec, double surf_prec) {
  int nev = 0;
  const double rprec = maxmin_prec * surf_prec;  // Action::update_remains (Action.cpp:199-202)
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t k = a.vidx[i];
    const double value = k >= 0 ? x[k] : 0.0;
    const uint8_t fl = a.flags[i];
    double rem = a.remains[i], md = a.max_duration[i], lat = a.latency[i], pen = a.penalty[i];
    uint8_t ev = 0;
    if (model == MODEL_CM02) {  // network_cm02.cpp:136-148
      double deltap = delta;
      if (lat > 0) {
        if (lat > deltap) {
          double_update(lat, deltap, surf_prec);
          deltap = 0.0;
        } else {
          double_update(deltap, lat, surf_prec);
          lat = 0.0;
        }
        if (lat <= 0.0 && !(fl & ACT_SUSPENDED)) {
          pen = a.share_pen[i];
          ev |= EV_LATENCY_PAID;
        }
      }
      if (fl & ACT_NO_CNST)  // :150-155 no link used: complete at once
        double_update(rem, rem, rprec);
    } else if (model == MODEL_L07) {  // ptask_L07.cpp:89-100
      if (lat > 0) {
        if (lat > delta)
          double_update(lat, delta, surf_prec);
        else
          lat = 0.0;
        if (lat <= 0.0 && !(fl & ACT_SUSPENDED)) {
          pen = 1.0;  // + updateBound on the host
          ev |= EV_LATENCY_PAID;
        }
      }
    }
    double_update(rem, value * delta, rprec);
    if (md != kNoMaxDuration)  // Action::update_max_duration (Action.cpp:194-198)
      double_update(md, delta, surf_prec);
    if ((rem <= 0 && pen > 0) || (md != kNoMaxDuration && md <= 0))
      ev |= EV_FINISHED;
    a.remains[i] = rem;
    a.max_duration[i] = md;
    a.latency[i] = lat;
    a.penalty[i] = pen;
    a.events[i] = ev;
    nev += ev != 0;
  }
  nev = grp_isum<kWave>(nev);
  if ((threadIdx.x & (kWave - 1)) == 0 && nev)
    atomicAdd(a.nev, nev);
}

// ---- LAZY update (Model::next_occuring_event_lazy, Model.cpp:40-101) ----
// Order-preserving map of a double onto unsigned 64 bits (negative dates included).
__device__ __forceinline__ unsigned long long dorder(double d) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d + 0.0);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// One modified action (the Lazy modified_set_ after lmm_solve): skip non-started, suspended / bogus
// (penalty <= 0) and latency-hat actions (Model.cpp:51-56); update_remains_lazy (CpuAction,
// cpu_interface.cpp:141-157, or NetworkCm02Action, network_cm02.cpp:426-449, which also counts down the
// max duration and finishes the action); then the completion date and its heap entry (Model.cpp:60-93:
// the entry is (re)written even for an action that update_remains_lazy just finished, as in the
// reference).  The second update_remains_lazy hidden in Action::get_remains() (Action.cpp:184-192) runs
// at delta = 0 and changes nothing, so it is not repeated.
__global__ void __launch_bounds__(kBlock) act_lazy_update(ActDev a, const double* x, int model, double now,
                                                           double rprec, double sprec, int64_t nmod,
                                                           const int32_t* __restrict__ mod) {
  int nev = 0;
  for (int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x; j < nmod; j += int64_t(gridDim.x) * kBlock) {
    const int32_t i = mod[j];
    const uint8_t fl = a.flags[i];
    if (fl & ACT_NOT_STARTED)
      continue;
    const double pen = a.penalty[i];
    if (pen <= 0 || a.htype[i] == HEAP_LATENCY)
      continue;
    const int32_t k = a.vidx[i];
    const double value = k >= 0 ? x[k] : 0.0;
    double rem = a.remains[i], md = a.max_duration[i];
    const double delta = now - a.last_update[i];
    uint8_t ev = 0;
    if (rem > 0)
      double_update(rem, a.last_value[i] * delta, rprec);
    if (model != MODEL_CPU) {
      if (md != kNoMaxDuration)
        double_update(md, delta, sprec);
      if ((rem <= 0 && pen > 0) || (md != kNoMaxDuration && md <= 0))
        ev = EV_FINISHED;
    }
    a.last_update[i] = now;
    a.last_value[i] = value;
    double mn = -1;
    if (value > 0) {
      const double ttc = rem > 0 ? rem / value : 0.0;
      mn = now + ttc;
    }
    bool mdflag = false;
    const double st = a.start_time[i];
    if (md != kNoMaxDuration && (mn <= -1 || st + md < mn)) {
      mn = st + md;
      mdflag = true;
    }
    if (mn > -1) {
      a.date[i] = mn;
      a.htype[i] = mdflag ? HEAP_MAX_DURATION : HEAP_NORMAL;
    } else {
      atomicOr(a.err, 1);
    }
    a.remains[i] = rem;
    a.max_duration[i] = md;
    a.events[i] = ev;
    nev += ev != 0;
  }
  nev = grp_isum<kWave>(nev);
  if ((threadIdx.x & (kWave - 1)) == 0 && nev)
    atomicAdd(a.nev, nev);
}

// ActionHeap::top_date(): min over the heap entries (dorder-encoded).
__global__ void __launch_bounds__(kBlock) act_lazy_min(ActDev a) {
  unsigned long long m = ~0ull;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * kBlock)
    if (a.htype[i] != HEAP_UNSET) {
      const unsigned long long o = dorder(a.date[i]);
      m = o < m ? o : m;
    }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const unsigned long long t = __shfl_xor(m, off, kWave);
    m = t < m ? t : m;
  }
  if ((threadIdx.x & (kWave - 1)) == 0 && m != ~0ull)
    atomicMin(a.umin, m);
}

// update_actions_state_lazy (CpuModel, cpu_interface.cpp:25-35; NetworkCm02Model, network_cm02.cpp:
// 103-126): the heap pops every entry while double_equals(top_date, now, surf_precision).  Launched only
// when the top qualifies; then every entry d >= top satisfies d - now > -prec, so the popped prefix is
// exactly the entries with |d - now| < prec.  Latency hats (CM02) pay their latency (the host restores
// the penalty), the others finish; all leave the heap.
__global__ void __launch_bounds__(kBlock) act_lazy_due(ActDev a, int model, double now, double sprec) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * kBlock) {
    const uint8_t h = a.htype[i];
    if (h == HEAP_UNSET || !(fabs(a.date[i] - now) < sprec))
      continue;
    uint8_t ev = EV_FINISHED;
    if (model != MODEL_CPU && h == HEAP_LATENCY) {
      ev = EV_LATENCY_PAID;
      a.last_update[i] = now;
    }
    a.htype[i] = HEAP_UNSET;
    a.date[i] = dinf();
    a.events[i] = ev;
    a.due[atomicAdd(a.ndue, 1)] = int32_t(i);
  }
}

}  // namespace lmmdev
