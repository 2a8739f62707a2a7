// lmm_capi.cpp — extern "C" surface of include/lmm/lmm_system.h over simgrid_amd::lmm::System.
// No exception crosses the ABI: every C++ error becomes a negative return code + lmm_last_error().
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "../../include/lmm/lmm_hip.h"
#include "../../include/lmm/lmm_system.h"
#include "lmm_generators.hpp"
#include "lmm_platforms.hpp"
#include "lmm_system.hpp"

using simgrid_amd::lmm::Id;
using simgrid_amd::lmm::SolverKind;
using simgrid_amd::lmm::System;

struct lmm_sys {
  System sys;
  lmm_sys(bool sel, SolverKind k) : sys(sel, k) {}
};

namespace {
thread_local std::string g_err;

#define GUARD(body)                    \
  try {                                \
    body;                              \
    return 0;                          \
  } catch (const std::exception& ex) { \
    g_err = ex.what();                 \
    return -1;                         \
  }

bool cnst_ok(lmm_sys* s, int64_t c) { return s && c >= 0 && c < int64_t(1) << 31; }

struct Builder {
  using Cnst = Id;
  using Var = Id;
  System* s;
  void* var_id = nullptr;  // the opaque id (Action*) of the variables it creates
  Cnst constraint_new(double b) { return s->constraint_new(nullptr, b); }
  void set_concurrency_limit(Cnst c, int l) { s->set_concurrency_limit(c, l); }
  void unshare(Cnst c) { s->unshare(c); }
  Var variable_new(double p, double b, int n) { return s->variable_new(var_id, p, b, size_t(n)); }
  void set_concurrency_share(Var v, int sh) { s->set_concurrency_share(v, sh); }
  void expand(Cnst c, Var v, double w) { s->expand(c, v, w); }
  void expand_add(Cnst c, Var v, double w) { s->expand_add(c, v, w); }
};
}  // namespace

extern "C" {

void lmm_set_precision(double p) { simgrid_amd::lmm::maxmin_precision = p; }
double lmm_get_precision(void) { return simgrid_amd::lmm::maxmin_precision; }
void lmm_set_default_concurrency_limit(int l) { simgrid_amd::lmm::concurrency_limit = l; }
const char* lmm_last_error(void) { return g_err.c_str(); }
int lmm_device_count(void) { return lmmhip_device_count(); }

lmm_sys* lmm_system_new(int selective, int kind) {
  try {
    return new lmm_sys(selective != 0, kind == 1 ? SolverKind::FAIR_BOTTLENECK : SolverKind::MAXMIN);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}
void lmm_system_free(lmm_sys* s) { delete s; }

// --cfg-style configuration (sg_config.cpp:232-466 registers the reference's flags; "maxmin/solver"
// and "maxmin/resident" are this build's own): "key:value", one per call.
int lmm_config_set(const char* kv) {
  try {
    const std::string s(kv ? kv : "");
    const size_t colon = s.find(':');
    if (colon == std::string::npos)
      throw std::invalid_argument("lmm_config_set: expected key:value, got '" + s + "'");
    const std::string key = s.substr(0, colon), val = s.substr(colon + 1);
    if (key == "maxmin/precision") {
      simgrid_amd::lmm::maxmin_precision = std::stod(val);
    } else if (key == "maxmin/concurrency-limit") {
      simgrid_amd::lmm::concurrency_limit = std::stoi(val);
    } else if (key == "maxmin/solver") {
      // hip = hip-auto: the device engine chosen by size; hip-persistent / hip-rounds force one
      if (val == "hip" || val == "hip-auto")
        simgrid_amd::lmm::solver_engine = LMMHIP_ENGINE_AUTO;
      else if (val == "hip-persistent")
        simgrid_amd::lmm::solver_engine = LMMHIP_ENGINE_PERSISTENT;
      else if (val == "hip-rounds")
        simgrid_amd::lmm::solver_engine = LMMHIP_ENGINE_ROUNDS;
      else
        throw std::invalid_argument("maxmin/solver: hip, hip-auto, hip-persistent or hip-rounds (this build has no "
                                    "CPU solver), got '" + val + "'");
    } else if (key == "maxmin/resident") {
      if (val == "yes" || val == "1" || val == "on")
        simgrid_amd::lmm::resident_default = true;
      else if (val == "no" || val == "0" || val == "off")
        simgrid_amd::lmm::resident_default = false;
      else
        throw std::invalid_argument("maxmin/resident: yes or no, got '" + val + "'");
    } else {
      throw std::invalid_argument("lmm_config_set: unknown key '" + key + "'");
    }
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int lmm_config_get(const char* key, char* buf, int cap) {
  const std::string k(key ? key : "");
  std::string v;
  if (k == "maxmin/precision") {
    char tmp[32];  // %.17g: the value round-trips through lmm_config_set
    std::snprintf(tmp, sizeof tmp, "%.17g", simgrid_amd::lmm::maxmin_precision);
    v = tmp;
  } else if (k == "maxmin/concurrency-limit")
    v = std::to_string(simgrid_amd::lmm::concurrency_limit);
  else if (k == "maxmin/solver")
    v = simgrid_amd::lmm::solver_engine == LMMHIP_ENGINE_PERSISTENT ? "hip-persistent"
        : simgrid_amd::lmm::solver_engine == LMMHIP_ENGINE_ROUNDS   ? "hip-rounds"
                                                                    : "hip-auto";
  else if (k == "maxmin/resident")
    v = simgrid_amd::lmm::resident_default ? "yes" : "no";
  else {
    g_err = "lmm_config_get: unknown key '" + k + "'";
    return -1;
  }
  if (buf && cap > 0) {
    std::strncpy(buf, v.c_str(), size_t(cap) - 1);
    buf[cap - 1] = 0;
  }
  return int(v.size());
}

int64_t lmm_constraint_new_id(lmm_sys* s, void* id, double bound) {
  try {
    return s->sys.constraint_new(id, bound);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_variable_new_id(lmm_sys* s, void* id, double penalty, double bound, int64_t n_cnst) {
  try {
    return s->sys.variable_new(id, penalty, bound, size_t(n_cnst));
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

void* lmm_constraint_get_id(lmm_sys* s, int64_t c) { return s->sys.cnst(Id(c)).id; }
void* lmm_variable_get_id(lmm_sys* s, int64_t v) { return s->sys.var(Id(v)).id; }

int lmm_modified_action_ids(lmm_sys* s, void** out, int cap) {
  auto& v = s->sys.modified_actions();
  for (int i = 0; i < int(v.size()) && i < cap; i++)
    out[i] = s->sys.var(Id(v[i])).id;
  return int(v.size());
}

int64_t lmm_constraint_new(lmm_sys* s, double bound) {
  try {
    return s->sys.constraint_new(nullptr, bound);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}
int lmm_constraint_unshare(lmm_sys* s, int64_t c) { GUARD(s->sys.unshare(Id(c))) }
int lmm_constraint_is_shared(lmm_sys* s, int64_t c) {
  return s->sys.cnst(Id(c)).policy != simgrid_amd::lmm::SharingPolicy::FATPIPE;
}
int lmm_constraint_set_concurrency_limit(lmm_sys* s, int64_t c, int l) {
  GUARD(s->sys.set_concurrency_limit(Id(c), l))
}
int lmm_constraint_concurrency(lmm_sys* s, int64_t c, int* cur, int* max, int* lim) {
  if (!cnst_ok(s, c))
    return -1;
  const auto& k = s->sys.cnst(Id(c));
  *cur = k.conc_current;
  *max = k.conc_maximum;
  *lim = k.conc_limit;
  return 0;
}
int lmm_constraint_reset_concurrency_maximum(lmm_sys* s, int64_t c) { GUARD(s->sys.reset_concurrency_maximum(Id(c))) }
double lmm_constraint_get_usage(lmm_sys* s, int64_t c) { return s->sys.get_usage(Id(c)); }
int lmm_constraint_get_variable_amount(lmm_sys* s, int64_t c) { return s->sys.get_variable_amount(Id(c)); }
double lmm_constraint_get_bound(lmm_sys* s, int64_t c) { return s->sys.cnst(Id(c)).bound; }
int lmm_constraint_rank(lmm_sys* s, int64_t c) { return s->sys.cnst(Id(c)).rank; }
int lmm_constraint_used(lmm_sys* s, int64_t c) { return s->sys.constraint_used(Id(c)); }
int lmm_constraint_elements(lmm_sys* s, int64_t c, int* var_rank, double* w, double* val, int* enabled, int cap) {
  auto els = s->sys.constraint_elements(Id(c));
  int n = 0;
  for (Id e : els) {
    if (n < cap) {
      const auto& x = s->sys.elem(e);
      var_rank[n] = s->sys.var(x.var).rank;
      w[n] = x.weight;
      val[n] = s->sys.get_value(x.var);
      enabled[n] = x.where == 1;
    }
    n++;
  }
  return n;
}

int64_t lmm_variable_new(lmm_sys* s, double penalty, double bound, int64_t n_cnst) {
  try {
    return s->sys.variable_new(nullptr, penalty, bound, size_t(n_cnst));
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}
int lmm_variable_free(lmm_sys* s, int64_t v) { GUARD(s->sys.variable_free(Id(v))) }
int lmm_variable_free_all(lmm_sys* s) { GUARD(s->sys.variable_free_all()) }
int lmm_variable_set_concurrency_share(lmm_sys* s, int64_t v, int sh) { GUARD(s->sys.set_concurrency_share(Id(v), sh)) }
double lmm_variable_get_value(lmm_sys* s, int64_t v) { return s->sys.get_value(Id(v)); }
double lmm_variable_get_bound(lmm_sys* s, int64_t v) { return s->sys.get_bound(Id(v)); }
double lmm_variable_get_penalty(lmm_sys* s, int64_t v) { return s->sys.get_penalty(Id(v)); }
int lmm_variable_rank(lmm_sys* s, int64_t v) { return s->sys.var(Id(v)).rank; }
int lmm_variable_number_of_constraints(lmm_sys* s, int64_t v) { return s->sys.number_of_constraints(Id(v)); }
int lmm_get_values(lmm_sys* s, const int64_t* vars, int64_t n, double* out) {
  for (int64_t i = 0; i < n; i++)
    out[i] = s->sys.get_value(Id(vars[i]));
  return 0;
}
int lmm_system_variables(lmm_sys* s, int64_t* out, int cap) {
  auto v = s->sys.variables_in_order();
  for (int i = 0; i < int(v.size()) && i < cap; i++)
    out[i] = v[i];
  return int(v.size());
}
int lmm_system_active_constraints(lmm_sys* s, int64_t* out, int cap) {
  auto v = s->sys.active_constraints_in_order();
  for (int i = 0; i < int(v.size()) && i < cap; i++)
    out[i] = v[i];
  return int(v.size());
}
int lmm_modified_actions(lmm_sys* s, int64_t* out, int cap) {
  auto& v = s->sys.modified_actions();
  for (int i = 0; i < int(v.size()) && i < cap; i++)
    out[i] = v[i];
  return int(v.size());
}
int lmm_clear_modified_actions(lmm_sys* s) { GUARD(s->sys.clear_modified_actions()) }

int lmm_expand(lmm_sys* s, int64_t c, int64_t v, double w) { GUARD(s->sys.expand(Id(c), Id(v), w)) }
int lmm_expand_add(lmm_sys* s, int64_t c, int64_t v, double w) { GUARD(s->sys.expand_add(Id(c), Id(v), w)) }
int lmm_update_variable_bound(lmm_sys* s, int64_t v, double b) { GUARD(s->sys.update_variable_bound(Id(v), b)) }
int lmm_update_variable_penalty(lmm_sys* s, int64_t v, double p) { GUARD(s->sys.update_variable_penalty(Id(v), p)) }
int lmm_update_constraint_bound(lmm_sys* s, int64_t c, double b) { GUARD(s->sys.update_constraint_bound(Id(c), b)) }

int lmm_solve(lmm_sys* s) { GUARD(s->sys.solve()) }
int lmm_lmm_solve(lmm_sys* s) { GUARD(s->sys.lmm_solve()) }
int lmm_is_modified(lmm_sys* s) { return s->sys.modified(); }
int lmm_prepare(lmm_sys* s) { GUARD(s->sys.prepare()) }
int lmm_device_solve(lmm_sys* s) { GUARD(s->sys.device_solve()) }
int lmm_fetch(lmm_sys* s) { GUARD(s->sys.fetch()) }
int lmm_set_resident(lmm_sys* s, int on) { GUARD(s->sys.set_resident(on != 0)) }
int lmm_is_resident(lmm_sys* s) { return s->sys.resident() ? 1 : 0; }
int lmm_pending_deltas(lmm_sys* s, int64_t* out3) { GUARD(s->sys.pending_deltas(out3)) }
int64_t lmm_last_delta_records(lmm_sys* s) { return s->sys.last_stats().delta_records; }
int lmm_table_sizes(lmm_sys* s, int64_t* out3) {
  out3[0] = int64_t(s->sys.n_elem_slots());
  out3[1] = int64_t(s->sys.n_var_slots());
  out3[2] = int64_t(s->sys.n_cnst_slots());
  return 0;
}
int lmm_resident_drain(lmm_sys* s, int64_t* sizes6, int64_t* e_id, int32_t* e_cnst, double* e_weight,
                       uint8_t* e_flags, int32_t* v_id, int64_t* v_ebase, int32_t* v_nelem, double* v_penalty,
                       double* v_bound, int32_t* c_id, double* c_bound, uint8_t* c_flags) {
  int64_t pend[3];
  s->sys.pending_deltas(pend);
  const int64_t want[3] = {pend[0] < 0 ? int64_t(s->sys.n_elem_slots()) : pend[0],
                           pend[1] < 0 ? int64_t(s->sys.n_var_slots()) : pend[1],
                           pend[2] < 0 ? int64_t(s->sys.n_cnst_slots()) : pend[2]};
  if (!s->sys.resident() || want[0] > sizes6[0] || want[1] > sizes6[1] || want[2] > sizes6[2]) {
    g_err = "lmm_resident_drain: not resident, or buffers smaller than lmm_pending_deltas";
    return 1;
  }
  simgrid_amd::lmm::System::ResPacked p;
  try {
    s->sys.drain_deltas(p);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
  std::copy(p.e_id.begin(), p.e_id.end(), e_id);
  std::copy(p.e_cnst.begin(), p.e_cnst.end(), e_cnst);
  std::copy(p.e_w.begin(), p.e_w.end(), e_weight);
  std::copy(p.e_fl.begin(), p.e_fl.end(), e_flags);
  std::copy(p.v_id.begin(), p.v_id.end(), v_id);
  std::copy(p.v_eb.begin(), p.v_eb.end(), v_ebase);
  std::copy(p.v_n.begin(), p.v_n.end(), v_nelem);
  std::copy(p.v_p.begin(), p.v_p.end(), v_penalty);
  std::copy(p.v_b.begin(), p.v_b.end(), v_bound);
  std::copy(p.c_id.begin(), p.c_id.end(), c_id);
  std::copy(p.c_b.begin(), p.c_b.end(), c_bound);
  std::copy(p.c_fl.begin(), p.c_fl.end(), c_flags);
  sizes6[0] = int64_t(p.e_id.size());
  sizes6[1] = int64_t(p.v_id.size());
  sizes6[2] = int64_t(p.c_id.size());
  sizes6[3] = p.n_elem_total;
  sizes6[4] = p.n_var_total;
  sizes6[5] = p.n_cnst_total;
  return 0;
}
int lmm_last_stats(lmm_sys* s, int64_t* counts4, double* ms4) {
  const auto& st = s->sys.last_stats();
  counts4[0] = st.rounds;
  counts4[1] = st.n_var;
  counts4[2] = st.n_cnst;
  counts4[3] = st.nnz;
  ms4[0] = st.device_ms;
  ms4[1] = st.flatten_ms;
  ms4[2] = st.upload_ms;
  ms4[3] = st.fetch_ms;
  return 0;
}
struct lmmhip_ctx* lmm_system_device_ctx(lmm_sys* s) {
  try {
    return s->sys.ctx();
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}
int lmm_flat_export(lmm_sys* s, int64_t* counts3, int64_t* var_ptr, int32_t* cnst_idx, double* weight, double* penalty,
                    double* vbound, double* cbound, uint8_t* cflags, int64_t* var_ids) {
  try {
    System::Flat f;
    s->sys.flatten_into(f);
    const size_t nv = f.dense_vars.size(), nc = f.cbound.size(), nnz = f.cnst_idx.size();
    counts3[0] = int64_t(nv);
    counts3[1] = int64_t(nc);
    counts3[2] = int64_t(nnz);
    if (var_ptr)
      std::memcpy(var_ptr, f.var_ptr.data(), (nv + 1) * sizeof(int64_t));
    if (cnst_idx)
      std::memcpy(cnst_idx, f.cnst_idx.data(), nnz * sizeof(int32_t));
    if (weight)
      std::memcpy(weight, f.weight.data(), nnz * sizeof(double));
    if (penalty)
      std::memcpy(penalty, f.penalty.data(), nv * sizeof(double));
    if (vbound)
      std::memcpy(vbound, f.vbound.data(), nv * sizeof(double));
    if (cbound)
      std::memcpy(cbound, f.cbound.data(), nc * sizeof(double));
    if (cflags)
      std::memcpy(cflags, f.cflags.data(), nc);
    for (size_t i = 0; var_ids && i < nv; i++)
      var_ids[i] = f.dense_vars[i];
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int lmm_flat_export_order(lmm_sys* s, int64_t nnz, int64_t* csc_order) {
  try {
    System::Flat f;
    s->sys.flatten_into(f);
    if (int64_t(f.cnst_idx.size()) != nnz || (nnz > 0 && !csc_order)) {
      g_err = "lmm_flat_export_order: nnz differs from the flattened system's";
      return -1;
    }
    if (int64_t(f.csc_order.size()) == nnz) {
      std::copy(f.csc_order.begin(), f.csc_order.end(), csc_order);
      return 0;
    }
    std::vector<int64_t> cur(f.cbound.size() + 1, 0);  // ascending CSR order per constraint
    for (int32_t k : f.cnst_idx)
      cur[size_t(k) + 1]++;
    for (size_t k = 0; k < f.cbound.size(); k++)
      cur[k + 1] += cur[k];
    for (int64_t j = 0; j < nnz; j++)
      csc_order[cur[size_t(f.cnst_idx[size_t(j)])]++] = j;
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int lmm_solve_batch(lmm_sys** systems, int n) {
  try {
    std::vector<System*> v(size_t(n > 0 ? n : 0));
    for (int i = 0; i < n; i++)
      v[size_t(i)] = &systems[i]->sys;
    simgrid_amd::lmm::solve_batch(v.data(), n);
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int lmm_check_certificate(lmm_sys* s, double prec, double* max_excess, int64_t* n_infeasible,
                          int64_t* n_unbottlenecked) {
  GUARD(s->sys.check_certificate(prec, max_excess, n_infeasible, n_unbottlenecked))
}

int lmm_gen_maxmin_bench(lmm_sys* s, int klass, int run, int64_t* cnst_out, int64_t* var_out, int* check_start,
                         int* check_solve) {
  if (klass < 0 || klass > 3)
    return -1;
  try {
    Builder b{&s->sys};
    std::vector<Id> cs, vs;
    lmm_gen::maxmin_bench(b, lmm_gen::kBenchClasses[klass], run, check_start, check_solve, &cs, &vs);
    for (size_t i = 0; cnst_out && i < cs.size(); i++)
      cnst_out[i] = cs[i];
    for (size_t i = 0; var_out && i < vs.size(); i++)
      var_out[i] = vs[i];
    return int(vs.size());
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_gen_synthetic(lmm_sys* s, int64_t nb_cnst, int64_t nb_var, int k, uint64_t seed, int max_share,
                          int penalty_mix, int bounded_permille, int fatpipe_permille, int64_t* var_out) {
  try {
    Builder b{&s->sys};
    lmm_gen::SynthParams p;
    p.nb_cnst = nb_cnst;
    p.nb_var = nb_var;
    p.elems_per_var = k;
    p.seed = seed;
    p.max_share = max_share;
    p.penalty_mix = penalty_mix;
    p.bounded_permille = bounded_permille;
    p.fatpipe_permille = fatpipe_permille;
    std::vector<Id> vs;
    lmm_gen::synthetic(b, p, nullptr, var_out ? &vs : nullptr);
    for (size_t i = 0; var_out && i < vs.size(); i++)
      var_out[i] = vs[i];
    return nb_var;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int lmm_platform_size(const lmm_platform_params* p, int64_t* n_links, int64_t* n_hosts) {
  try {
    std::unique_ptr<lmm_plat::Platform> plat(lmm_plat::make_platform(lmm_plat::params_from(*p)));
    if (n_links)
      *n_links = int64_t(plat->links.size());
    if (n_hosts)
      *n_hosts = plat->n_hosts;
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_platform_dragonfly_coords(const lmm_platform_params* p, int32_t* coords_out, int64_t cap) {
  try {
    if (!p || p->topology != 1)
      throw std::invalid_argument("lmm_platform_dragonfly_coords: not a dragonfly platform");
    const lmm_plat::Dragonfly df(lmm_plat::params_from(*p));
    const int64_t n = df.n_hosts;
    for (int64_t h = 0; coords_out && h < n && 4 * (h + 1) <= cap; h++) {
      int c[4];
      df.coords(int(h), c);
      for (int k = 0; k < 4; k++)
        coords_out[4 * h + k] = c[k];
    }
    return n;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_gen_platform_flows(lmm_sys* s, const lmm_platform_params* p, int64_t* cnst_out, int64_t* var_out) {
  try {
    const lmm_plat::Params prm = lmm_plat::params_from(*p);
    std::unique_ptr<lmm_plat::Platform> plat(lmm_plat::make_platform(prm));
    Builder b{&s->sys};
    std::vector<Id> cs, vs;
    lmm_plat::flows(b, *plat, prm, &cs, var_out ? &vs : nullptr);
    for (size_t i = 0; cnst_out && i < cs.size(); i++)
      cnst_out[i] = cs[i];
    for (size_t i = 0; var_out && i < vs.size(); i++)
      var_out[i] = vs[i];
    return prm.n_flows;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_link_new(lmm_sys* s, int model, double bw, int fatpipe) {
  try {
    if (!s)
      throw std::invalid_argument("null system");
    Builder b{&s->sys};
    return lmm_plat::link_constraint(b, model, bw, fatpipe != 0);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_wifi_link_new(lmm_sys* s, int model) {
  try {
    if (!s)
      throw std::invalid_argument("null system");
    Builder b{&s->sys};
    return lmm_plat::wifi_link_constraint(b, model);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_communicate_ex(lmm_sys* s, void* id, int model, int64_t n_route, const int64_t* route_cnst,
                           const double* route_bw, const double* route_lat, const double* route_rates, int64_t n_back,
                           const int64_t* back_cnst, int crosstraffic, double rate, double tcp_gamma, int paid,
                           lmm_comm_info* out) {
  try {
    if (!s || n_route < 0 || n_back < 0 || (n_route && (!route_cnst || !route_bw || !route_lat)) ||
        (n_back && !back_cnst))
      throw std::invalid_argument("lmm_communicate: bad arguments");
    Builder b{&s->sys, id};
    std::vector<lmm_plat::Link> links;
    std::vector<Id> cn;
    std::vector<int> route, back;
    double lat = 0.0;  // route_to accumulates the route's latencies in route order
    for (int64_t i = 0; i < n_route; i++) {
      if (!cnst_ok(s, route_cnst[i]))
        throw std::invalid_argument("lmm_communicate: bad route constraint");
      lmm_plat::Link k{route_bw[i], route_lat[i], false};
      if (route_rates && (route_rates[2 * i] != 0.0 || route_rates[2 * i + 1] != 0.0)) {
        for (int e = 0; e < 2; e++)  // a station's rate on the access point, or -1 (not associated)
          if (!(route_rates[2 * i + e] > 0.0 || route_rates[2 * i + e] == -1.0))
            throw std::invalid_argument("lmm_communicate: a WIFI rate must be > 0 or -1 (not associated)");
        k.wifi = true;  // a WIFI access point: its own bandwidth (1 / bandwidth factor) and latency (0)
        k.lat = 0.0;
        k.src_rate = route_rates[2 * i];
        k.dst_rate = route_rates[2 * i + 1];
      }
      links.push_back(k);
      cn.push_back(Id(route_cnst[i]));
      route.push_back(int(i));
      lat += k.lat;
    }
    for (int64_t i = 0; i < n_back; i++) {
      if (!cnst_ok(s, back_cnst[i]))
        throw std::invalid_argument("lmm_communicate: bad back-route constraint");
      cn.push_back(Id(back_cnst[i]));
      back.push_back(int(n_route + i));
    }
    lmm_plat::Comm a;
    const Id v = lmm_plat::communicate(b, model, links, cn, route, back, lat, rate, tcp_gamma, paid != 0,
                                       crosstraffic != 0, &a);
    if (out) {
      out->latency = a.latency;
      out->lat_current = a.lat_current;
      out->sharing_penalty = a.sharing_penalty;
      out->bound = a.bound;
    }
    return v;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t lmm_communicate(lmm_sys* s, void* id, int model, int64_t n_route, const int64_t* route_cnst, const double* route_bw,
                        const double* route_lat, int64_t n_back, const int64_t* back_cnst, double rate,
                        double tcp_gamma, int paid, lmm_comm_info* out) {
  return lmm_communicate_ex(s, id, model, n_route, route_cnst, route_bw, route_lat, nullptr, n_back, back_cnst,
                            n_back > 0, rate, tcp_gamma, paid, out);
}

}  // extern "C"
