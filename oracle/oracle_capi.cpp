// ORACLE — TEST INFRASTRUCTURE ONLY.  extern "C" surface of the CPU restatement, loaded with
// ctypes by tests/ and by bench.py's cpu_baseline leg.  Mirrors the product's System-level ABI
// (include/lmm/lmm_system.h) with an `oracle_` prefix so parity tests can drive both with the
// same call sequence.
#include <chrono>
#include <cstdint>
#include <cstring>

#include <memory>

#include "../include/lmm/lmm_system.h"
#include "../simgrid_amd/csrc/lmm_generators.hpp"
#include "lmm_oracle.hpp"

using namespace lmm_oracle;

namespace {
struct Builder {
  using Cnst = Constraint*;
  using Var = Variable*;
  System* s;
  Cnst constraint_new(double b) { return s->constraint_new(b); }
  void set_concurrency_limit(Cnst c, int l) { s->set_concurrency_limit(c, l); }
  void unshare(Cnst c) { c->policy = Policy::FATPIPE; }
  Var variable_new(double p, double b, int n) { return s->variable_new(nullptr, p, b, n); }
  void set_concurrency_share(Var v, int sh) { v->share = sh; }
  void expand(Cnst c, Var v, double w) { s->expand(c, v, w); }
  void expand_add(Cnst c, Var v, double w) { s->expand_add(c, v, w); }
};
inline System* S(void* p) { return static_cast<System*>(p); }
inline Constraint* C(void* p) { return static_cast<Constraint*>(p); }
inline Variable* V(void* p) { return static_cast<Variable*>(p); }
}  // namespace

extern "C" {

void oracle_set_precision(double p) { g_maxmin_precision = p; }
double oracle_get_precision() { return g_maxmin_precision; }
void oracle_set_default_concurrency_limit(int l) { g_concurrency_limit = l; }

void* oracle_system_new(int selective, int kind) {
  return kind == 1 ? static_cast<System*>(new FairBottleneck(selective != 0)) : new System(selective != 0);
}
void oracle_system_free(void* s) { delete S(s); }
void oracle_solve(void* s) { S(s)->solve(); }
long long oracle_last_rounds(void* s) { return S(s)->last_rounds; }
int oracle_is_modified(void* s) { return S(s)->modified; }

// Dependency depth of the next solves (System::depth_on; measurement only).  oracle_depth_stats: D, the saturation and
// bound-fix event counts, and the per-level histograms (saturations, bound fixes) into hist / bhist (cap entries);
// returns the number of levels (D + 1).
void oracle_set_depth(void* s, int on) { S(s)->depth_on = on != 0; }
int oracle_depth_stats(void* s, int* D, long long* sat_events, long long* bound_events, long long* hist,
                       long long* bhist, int cap) {
  System* y = S(s);
  *D = y->depth_D;
  *sat_events = y->depth_sat_events;
  *bound_events = y->depth_bound_events;
  const int n = int(y->depth_hist.size());
  for (int i = 0; i < n && i < cap; i++) {
    hist[i] = y->depth_hist[size_t(i)];
    bhist[i] = y->depth_bhist[size_t(i)];
  }
  return n;
}
// Per variable (the given handles): the level and sequential round of the event that fixed it, and the rank of the
// constraint whose saturation fixed it (0: a bound fix; -1 / -1 / 0: never fixed).
void oracle_variable_depth(void*, void** vs, long long n, int* lvl, long long* round, int* by) {
  for (long long i = 0; i < n; i++) {
    lvl[i] = V(vs[i])->fix_lvl;
    round[i] = V(vs[i])->fix_round;
    by[i] = V(vs[i])->fix_by;
  }
}
// Per constraint (the given handles): its saturation level and sequential round (-1: never saturated).
void oracle_constraint_depth(void*, void** cs, long long n, int* lvl, long long* round) {
  for (long long i = 0; i < n; i++) {
    lvl[i] = C(cs[i])->sat_lvl;
    round[i] = C(cs[i])->sat_round;
  }
}

// Times one solve() with steady_clock, excluding construction (maxmin_bench.cpp:81-83).
double oracle_timed_solve(void* s) {
  auto t0 = std::chrono::steady_clock::now();
  S(s)->solve();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

void* oracle_constraint_new(void* s, double bound) { return S(s)->constraint_new(bound); }
void oracle_constraint_unshare(void*, void* c) { C(c)->policy = Policy::FATPIPE; }
int oracle_constraint_is_shared(void*, void* c) { return C(c)->policy != Policy::FATPIPE; }
void oracle_constraint_set_concurrency_limit(void* s, void* c, int l) { S(s)->set_concurrency_limit(C(c), l); }
void oracle_constraint_concurrency(void*, void* c, int* cur, int* max, int* lim) {
  *cur = C(c)->conc_current;
  *max = C(c)->conc_maximum;
  *lim = C(c)->conc_limit;
}
void oracle_constraint_reset_concurrency_maximum(void*, void* c) { C(c)->conc_maximum = 0; }
double oracle_constraint_get_usage(void*, void* c) { return C(c)->get_usage(); }
int oracle_constraint_get_variable_amount(void*, void* c) { return C(c)->variable_amount(); }
double oracle_constraint_get_bound(void*, void* c) { return C(c)->bound; }
int oracle_constraint_rank(void*, void* c) { return C(c)->rank; }
int oracle_constraint_used(void* s, void* c) { return S(s)->constraint_used(C(c)); }
int oracle_constraint_init_state(void*, void* c, double* usage, double* remaining) {
  *usage = C(c)->init_usage;
  *remaining = C(c)->init_remaining;
  return C(c)->init_recorded;
}
// Elements of a constraint in System::print() order (maxmin.cpp:454-463): enabled then disabled.
int oracle_constraint_elements(void*, void* c, int* var_rank, double* w, double* val, int* enabled, int cap) {
  int n = 0;
  for (Element& e : C(c)->enabled) {
    if (n < cap) {
      var_rank[n] = e.var->rank;
      w[n] = e.weight;
      val[n] = e.var->value;
      enabled[n] = 1;
    }
    n++;
  }
  for (Element& e : C(c)->disabled) {
    if (n < cap) {
      var_rank[n] = e.var->rank;
      w[n] = e.weight;
      val[n] = e.var->value;
      enabled[n] = 0;
    }
    n++;
  }
  return n;
}

void* oracle_variable_new(void* s, double penalty, double bound, long n_cnst) {
  return S(s)->variable_new(nullptr, penalty, bound, (size_t)n_cnst);
}
void oracle_variable_free(void* s, void* v) { S(s)->variable_free(V(v)); }
void oracle_variable_free_all(void* s) { S(s)->variable_free_all(); }
void oracle_variable_set_concurrency_share(void*, void* v, int sh) { V(v)->share = sh; }
double oracle_variable_get_value(void*, void* v) { return V(v)->value; }
double oracle_variable_get_bound(void*, void* v) { return V(v)->bound; }
double oracle_variable_get_penalty(void*, void* v) { return V(v)->penalty; }
int oracle_variable_rank(void*, void* v) { return V(v)->rank; }
int oracle_variable_number_of_constraints(void*, void* v) { return (int)V(v)->elems.size(); }
void oracle_get_values(void*, void** vars, long long n, double* out) {
  for (long long i = 0; i < n; i++)
    out[i] = V(vars[i])->value;
}
// variable_set order (the MAX-MIN objective line of print(), maxmin.cpp:446-447)
int oracle_system_variables(void* s, void** out, int cap) {
  int n = 0;
  for (Variable& v : S(s)->variables) {
    if (n < cap)
      out[n] = &v;
    n++;
  }
  return n;
}
// active_constraint_set order (the constraint lines of print(), maxmin.cpp:454)
int oracle_system_active_constraints(void* s, void** out, int cap) {
  int n = 0;
  for (Constraint& c : S(s)->active_cnsts) {
    if (n < cap)
      out[n] = &c;
    n++;
  }
  return n;
}
int oracle_modified_actions(void* s, void** out, int cap) {
  auto& m = S(s)->modified_actions;
  int n = 0;
  for (Variable* v : m) {
    if (n < cap)
      out[n] = v;
    n++;
  }
  return n;
}
void oracle_clear_modified_actions(void* s) {
  for (Variable* v : S(s)->modified_actions)
    v->in_modified_set = false;
  S(s)->modified_actions.clear();
}

void oracle_expand(void* s, void* c, void* v, double w) { S(s)->expand(C(c), V(v), w); }
void oracle_expand_add(void* s, void* c, void* v, double w) { S(s)->expand_add(C(c), V(v), w); }
void oracle_update_variable_bound(void* s, void* v, double b) { S(s)->update_variable_bound(V(v), b); }
void oracle_update_variable_penalty(void* s, void* v, double p) { S(s)->update_variable_penalty(V(v), p); }
void oracle_update_constraint_bound(void* s, void* c, double b) { S(s)->update_constraint_bound(C(c), b); }

// maxmin_bench generator (class 0..3 = small/medium/big/huge), one run.
int oracle_gen_maxmin_bench(void* s, int klass, int run, void** cnst_out, void** var_out, int* check_start,
                            int* check_solve) {
  Builder b{S(s)};
  std::vector<Constraint*> cs;
  std::vector<Variable*> vs;
  lmm_gen::maxmin_bench(b, lmm_gen::kBenchClasses[klass], run, check_start, check_solve, &cs, &vs);
  if (cnst_out)
    std::memcpy(cnst_out, cs.data(), cs.size() * sizeof(void*));
  if (var_out)
    std::memcpy(var_out, vs.data(), vs.size() * sizeof(void*));
  return (int)vs.size();
}

// Scaled synthetic generator (SURVEY.md §8(d) C2 + stress variant).
long long oracle_gen_synthetic(void* s, long long nb_cnst, long long nb_var, int k, unsigned long long seed,
                               int max_share, int penalty_mix, int bounded_permille, int fatpipe_permille,
                               void** var_out) {
  Builder b{S(s)};
  lmm_gen::SynthParams p;
  p.nb_cnst = nb_cnst;
  p.nb_var = nb_var;
  p.elems_per_var = k;
  p.seed = seed;
  p.max_share = max_share;
  p.penalty_mix = penalty_mix;
  p.bounded_permille = bounded_permille;
  p.fatpipe_permille = fatpipe_permille;
  std::vector<Variable*> vs;
  lmm_gen::synthetic(b, p, nullptr, var_out ? &vs : nullptr);
  if (var_out)
    std::memcpy(var_out, vs.data(), vs.size() * sizeof(void*));
  return nb_var;
}

// Cluster platform + flows: the system oracle/platforms.py restates from the reference's zones
// and models, replayed as its API calls — constraint_new (+ unshare for FATPIPE) per constraint, then per flow
// variable_new(penalty, bound, number of constraints) and its elements in call order, expand_add where eadd is
// set, expand otherwise.  No generator logic here: it is independent of the product's lmm_platforms.hpp.
long long oracle_build_flows(void* s, long long nc, const double* cbound, const unsigned char* cfat, long long nv,
                             const double* vpen, const double* vbound, const int* vn, const long long* eptr,
                             const int* ecnst, const double* ew, const unsigned char* eadd, void** cnst_out,
                             void** var_out) {
  Builder b{S(s)};
  std::vector<Constraint*> cs(static_cast<size_t>(nc));
  for (long long i = 0; i < nc; i++) {
    cs[size_t(i)] = b.constraint_new(cbound[i]);
    if (cfat[i])
      b.unshare(cs[size_t(i)]);
    if (cnst_out)
      cnst_out[i] = cs[size_t(i)];
  }
  for (long long f = 0; f < nv; f++) {
    Variable* v = b.variable_new(vpen[f], vbound[f], vn[f]);
    for (long long e = eptr[f]; e < eptr[f + 1]; e++) {
      if (ecnst[e] < 0 || ecnst[e] >= nc)
        return -1;
      if (eadd[e])
        b.expand_add(cs[size_t(ecnst[e])], v, ew[e]);
      else
        b.expand(cs[size_t(ecnst[e])], v, ew[e]);
    }
    if (var_out)
      var_out[f] = v;
  }
  return nv;
}

}  // extern "C"
