// lmm_system.cpp — host bookkeeping of the MI355X LMM solver (see lmm_system.hpp).
//
// Mutation semantics follow the reference line by line where they decide *which* variables are
// enabled (concurrency staging) — those are integer decisions and must be exact:
//   expand / expand_add           maxmin.cpp:234-323
//   enable_var / disable_var      maxmin.cpp:749-795
//   on_disabled_var               maxmin.cpp:804-843
//   update_variable_penalty       maxmin.cpp:846-881
//   var_free                      maxmin.cpp:106-138
//   selective-update closure      maxmin.cpp:898-937 (iterative here: no recursion depth limit)
// The solve itself runs on the GPU (lmm_hip.hip); this file only flattens and scatters.
#include "lmm_system.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <limits>
#include <stdexcept>

#include "../../include/lmm/lmm_hip.h"

namespace simgrid_amd {
namespace lmm {

double maxmin_precision = 1e-5;
int concurrency_limit = -1;
int solver_engine = LMMHIP_ENGINE_AUTO;
bool resident_default = true;

[[noreturn]] void fatal(const std::string& msg) { throw std::runtime_error("lmm: " + msg); }

static inline void check(bool cond, const char* msg) {
  if (!cond)
    fatal(msg);
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int CnstRec::slack() const {
  return conc_limit < 0 ? std::numeric_limits<int>::max() : conc_limit - conc_current;
}

// Max-min systems start in resident mode by default (HBM mirror + delta log + device flatten, §9 of
// DESIGN.md): the host never walks the whole system per solve.  FairBottleneck systems keep the host
// flatten, which hands the device each constraint's elements in the reference's list order
// (flatten_fair): the bit-identical element-by-element remaining update needs it.
System::System(bool selective_update, SolverKind kind)
    : selective_(selective_update), kind_(kind), resident_(resident_default && kind == SolverKind::MAXMIN),
      engine_(solver_engine) {}

System::~System() {
  if (ctx_)
    lmmhip_ctx_destroy(ctx_);
}

lmmhip_ctx* System::ctx() {
  if (!ctx_) {
    int rc = lmmhip_ctx_create(-1, &ctx_);
    if (rc)
      fatal(std::string("cannot create HIP context: ") + lmmhip_last_error());
    if ((rc = lmmhip_ctx_set_engine(ctx_, engine_)))
      fatal(std::string("cannot select the max-min engine: ") + lmmhip_last_error());
  }
  return ctx_;
}

// ------------------------------------------------------------------------------------------
// index-linked lists
// ------------------------------------------------------------------------------------------
void System::en_push_front(Id c, Id e) {
  CnstRec& k = cnsts_[c];
  ElemRec& x = elems_[e];
  x.prev = kNone;
  x.next = k.en_head;
  if (k.en_head != kNone)
    elems_[k.en_head].prev = e;
  else
    k.en_tail = e;
  k.en_head = e;
  x.where = 1;
  k.n_en++;
  touch_e(e);
}

void System::dis_push_back(Id c, Id e) {
  CnstRec& k = cnsts_[c];
  ElemRec& x = elems_[e];
  x.next = kNone;
  x.prev = k.dis_tail;
  if (k.dis_tail != kNone)
    elems_[k.dis_tail].next = e;
  else
    k.dis_head = e;
  k.dis_tail = e;
  x.where = 2;
  k.n_dis++;
  touch_e(e);
}

void System::elem_unlink(Id e) {
  ElemRec& x = elems_[e];
  if (!x.where)
    return;
  CnstRec& k = cnsts_[x.cnst];
  Id& head = x.where == 1 ? k.en_head : k.dis_head;
  Id& tail = x.where == 1 ? k.en_tail : k.dis_tail;
  if (x.prev != kNone)
    elems_[x.prev].next = x.next;
  else
    head = x.next;
  if (x.next != kNone)
    elems_[x.next].prev = x.prev;
  else
    tail = x.prev;
  (x.where == 1 ? k.n_en : k.n_dis)--;
  x.prev = x.next = kNone;
  x.where = 0;
  touch_e(e);
}

void System::vset_push_front(Id v) {
  VarRec& r = vars_[v];
  r.prev = kNone;
  r.next = vset_head_;
  if (vset_head_ != kNone)
    vars_[vset_head_].prev = v;
  else
    vset_tail_ = v;
  vset_head_ = v;
}
void System::vset_push_back(Id v) {
  VarRec& r = vars_[v];
  r.next = kNone;
  r.prev = vset_tail_;
  if (vset_tail_ != kNone)
    vars_[vset_tail_].next = v;
  else
    vset_head_ = v;
  vset_tail_ = v;
}
void System::vset_erase(Id v) {
  VarRec& r = vars_[v];
  if (r.prev != kNone)
    vars_[r.prev].next = r.next;
  else
    vset_head_ = r.next;
  if (r.next != kNone)
    vars_[r.next].prev = r.prev;
  else
    vset_tail_ = r.prev;
  r.prev = r.next = kNone;
}

void System::make_cnst_active(Id c) {
  CnstRec& k = cnsts_[c];
  if (k.in_active)
    return;
  k.in_active = true;
  k.act_next = kNone;
  k.act_prev = act_tail_;
  if (act_tail_ != kNone)
    cnsts_[act_tail_].act_next = c;
  else
    act_head_ = c;
  act_tail_ = c;
  flat_valid_ = false;
  act_cache_ok_ = false;
}

void System::make_cnst_inactive(Id c) {
  CnstRec& k = cnsts_[c];
  if (k.in_active) {
    if (k.act_prev != kNone)
      cnsts_[k.act_prev].act_next = k.act_next;
    else
      act_head_ = k.act_next;
    if (k.act_next != kNone)
      cnsts_[k.act_next].act_prev = k.act_prev;
    else
      act_tail_ = k.act_prev;
    k.act_prev = k.act_next = kNone;
    k.in_active = false;
    flat_valid_ = false;
    act_cache_ok_ = false;
  }
  if (k.in_modified)
    mod_erase(c);
}

void System::mod_push_back(Id c) {
  CnstRec& k = cnsts_[c];
  k.in_modified = true;
  k.mod_next = kNone;
  k.mod_prev = mod_tail_;
  if (mod_tail_ != kNone)
    cnsts_[mod_tail_].mod_next = c;
  else
    mod_head_ = c;
  mod_tail_ = c;
}
void System::mod_erase(Id c) {
  CnstRec& k = cnsts_[c];
  if (k.mod_prev != kNone)
    cnsts_[k.mod_prev].mod_next = k.mod_next;
  else
    mod_head_ = k.mod_next;
  if (k.mod_next != kNone)
    cnsts_[k.mod_next].mod_prev = k.mod_prev;
  else
    mod_tail_ = k.mod_prev;
  k.mod_prev = k.mod_next = kNone;
  k.in_modified = false;
}

// ------------------------------------------------------------------------------------------
// concurrency (maxmin.cpp:42-58, 730-743)
// ------------------------------------------------------------------------------------------
void System::inc_conc(Id e) {
  CnstRec& k = cnsts_[elems_[e].cnst];
  k.conc_current += elems_[e].concurrency();
  if (k.conc_current > k.conc_maximum)
    k.conc_maximum = k.conc_current;
  check(k.conc_limit < 0 || k.conc_current <= k.conc_limit, "Concurrency limit overflow!");
}
void System::dec_conc(Id e) {
  CnstRec& k = cnsts_[elems_[e].cnst];
  check(k.conc_current >= elems_[e].concurrency(), "concurrency underflow");
  k.conc_current -= elems_[e].concurrency();
}
int System::min_slack(Id v) const {
  int best = std::numeric_limits<int>::max();
  const VarRec& r = vars_[v];
  for (int i = 0; i < r.n_elems; i++) {
    int s = cnsts_[elems_[r.ebase + i].cnst].slack();
    if (s < best) {
      if (s == 0)
        return 0;
      best = s;
    }
  }
  return best;
}

void System::set_concurrency_limit(Id c, int limit) {
  check(limit < 0 || cnsts_[c].conc_maximum <= limit,
        "New concurrency limit should be larger than observed concurrency maximum");
  cnsts_[c].conc_limit = limit;
}

// ------------------------------------------------------------------------------------------
// creation / destruction
// ------------------------------------------------------------------------------------------
Id System::constraint_new(void* id, double bound) {
  check(cnsts_.size() < size_t(std::numeric_limits<Id>::max()), "too many constraints");
  CnstRec k;
  k.bound = bound;
  k.id = id;
  k.rank = next_cnst_rank_++;
  k.conc_limit = concurrency_limit;
  cnsts_.push_back(k);
  flat_valid_ = false;
  touch_c(Id(cnsts_.size() - 1));
  return Id(cnsts_.size() - 1);
}

Id System::variable_new(void* id, double penalty, double bound, size_t n_cnst) {
  Id v;
  if (!free_var_ids_.empty()) {
    v = free_var_ids_.back();
    free_var_ids_.pop_back();
  } else {
    check(vars_.size() < size_t(std::numeric_limits<Id>::max()), "too many variables");
    vars_.emplace_back();
    values_.push_back(0.0);
    v = Id(vars_.size() - 1);
  }
  VarRec& r = vars_[v];
  r = VarRec();
  values_[v] = 0.0;
  r.id = id;
  r.rank = next_var_rank_++;
  r.penalty = penalty;
  r.bound = bound;
  r.visited = visited_counter_ - 1;
  r.live = true;
  r.cap = int32_t(n_cnst);
  if (n_cnst < free_slabs_.size() && !free_slabs_[n_cnst].empty()) {
    r.ebase = free_slabs_[n_cnst].back();
    free_slabs_[n_cnst].pop_back();
  } else {
    r.ebase = int64_t(elems_.size());
    check(elems_.size() + n_cnst < size_t(std::numeric_limits<Id>::max()), "too many elements");
    elems_.resize(elems_.size() + n_cnst);
  }
  if (penalty > 0)
    vset_push_front(v);
  else
    vset_push_back(v);
  n_live_vars_++;
  flat_valid_ = false;
  touch_v(v);
  return v;
}

// maxmin.cpp:106-138
void System::var_free(Id v) {
  modified_ = true;
  flat_valid_ = false;
  VarRec& r = vars_[v];
  // The reference can re-enable a staged variable from inside its own free (two elements on one
  // constraint) and then double-erases it (undefined behaviour); a freed variable is never
  // re-enabled here (same definition as the oracle).
  r.staged = 0.0;
  if (r.n_elems)
    update_modified_set(elems_[r.ebase].cnst);
  for (int i = 0; i < r.n_elems; i++) {
    Id e = Id(r.ebase + i);
    Id c = elems_[e].cnst;
    if (vars_[v].penalty > 0)
      dec_conc(e);
    elem_unlink(e);
    if (cnsts_[c].n_en + cnsts_[c].n_dis == 0)
      make_cnst_inactive(c);
    else
      on_disabled_var(c);
  }
  VarRec& rr = vars_[v];
  for (int i = 0; i < rr.cap; i++)
    elems_[rr.ebase + i] = ElemRec();
  if (size_t(rr.cap) < 64) {
    if (free_slabs_.size() <= size_t(rr.cap))
      free_slabs_.resize(rr.cap + 1);
    free_slabs_[rr.cap].push_back(rr.ebase);
  }
  rr.n_elems = 0;
  rr.live = false;
  touch_v(v);
  free_var_ids_.push_back(v);
  n_live_vars_--;
}

void System::variable_free(Id v) {
  check(v >= 0 && size_t(v) < vars_.size() && vars_[v].live, "variable_free on a dead variable");
  vset_erase(v);
  var_free(v);
}

void System::variable_free_all() {
  while (vset_head_ != kNone)
    variable_free(vset_head_);
}

// ------------------------------------------------------------------------------------------
// expand / expand_add (maxmin.cpp:234-323)
// ------------------------------------------------------------------------------------------
void System::expand(Id c, Id v, double w) {
  modified_ = true;
  flat_valid_ = false;
  VarRec* r = &vars_[v];
  int current_share = 0;
  if (r->share > 1)
    for (int i = 0; i < r->n_elems; i++) {
      const ElemRec& e = elems_[r->ebase + i];
      if (e.cnst == c && e.where == 1)
        current_share += e.concurrency();
    }
  if (r->penalty > 0 && r->share - current_share > cnsts_[c].slack()) {
    double pen = r->penalty;
    disable_var(v);
    r = &vars_[v];
    for (int i = 0; i < r->n_elems; i++)
      on_disabled_var(elems_[r->ebase + i].cnst);
    w = 0;
    r = &vars_[v];
    r->staged = pen;
  }
  check(r->n_elems < r->cap, "Too much constraints");
  Id e = Id(r->ebase + r->n_elems);
  r->n_elems++;
  ElemRec& x = elems_[e];
  x.weight = w;
  x.cnst = c;
  x.var = v;
  touch_e(e);
  touch_v(v);
  if (r->penalty != 0) {
    en_push_front(c, e);
    inc_conc(e);
  } else {
    dis_push_back(c, e);
  }
  if (!selective_) {
    make_cnst_active(c);
  } else if (w > 0 || vars_[v].penalty > 0) {
    make_cnst_active(c);
    update_modified_set(c);
    if (vars_[v].n_elems > 1)
      update_modified_set(elems_[vars_[v].ebase].cnst);
  }
}

void System::expand_add(Id c, Id v, double w) {
  modified_ = true;
  flat_valid_ = false;
  VarRec& r = vars_[v];
  Id found = kNone;
  for (int i = 0; i < r.n_elems; i++)  // "first matching element" rule, maxmin.cpp:293-296
    if (elems_[r.ebase + i].cnst == c) {
      found = Id(r.ebase + i);
      break;
    }
  if (found == kNone) {
    expand(c, v, w);
    return;
  }
  if (vars_[v].penalty != 0)
    dec_conc(found);
  if (cnsts_[c].policy != SharingPolicy::FATPIPE)
    elems_[found].weight += w;
  else
    elems_[found].weight = std::max(elems_[found].weight, w);
  touch_e(found);
  if (vars_[v].penalty != 0) {
    if (cnsts_[c].slack() < elems_[found].concurrency()) {
      double pen = vars_[v].penalty;
      disable_var(v);
      for (int i = 0; i < vars_[v].n_elems; i++)
        on_disabled_var(elems_[vars_[v].ebase + i].cnst);
      vars_[v].staged = pen;
    }
    inc_conc(found);
  }
  update_modified_set(c);
}

// ------------------------------------------------------------------------------------------
// staging (maxmin.cpp:749-881)
// ------------------------------------------------------------------------------------------
void System::enable_var(Id v) {
  VarRec& r = vars_[v];
  r.penalty = r.staged;
  r.staged = 0;
  touch_v(v);
  vset_erase(v);
  vset_push_front(v);
  for (int i = 0; i < r.n_elems; i++) {
    Id e = Id(r.ebase + i);
    elem_unlink(e);
    en_push_front(elems_[e].cnst, e);
    inc_conc(e);
  }
  if (r.n_elems)
    update_modified_set(elems_[r.ebase].cnst);
  flat_valid_ = false;
}

void System::disable_var(Id v) {
  VarRec& r = vars_[v];
  check(r.staged == 0, "Staged penalty should have been cleared");
  vset_erase(v);
  vset_push_back(v);
  if (r.n_elems)
    update_modified_set(elems_[r.ebase].cnst);
  for (int i = 0; i < r.n_elems; i++) {
    Id e = Id(r.ebase + i);
    elem_unlink(e);
    dis_push_back(elems_[e].cnst, e);
    dec_conc(e);
  }
  r.penalty = 0.0;
  r.staged = 0.0;
  values_[v] = 0.0;
  touch_v(v);
  flat_valid_ = false;
}

void System::on_disabled_var(Id c) {
  if (cnsts_[c].conc_limit < 0)
    return;
  int budget = cnsts_[c].n_dis;
  if (!budget)
    return;
  Id e = cnsts_[c].dis_head;
  while (budget-- && e != kNone) {
    Id nxt = elems_[e].where == 2 ? elems_[e].next : kNone;
    Id v = elems_[e].var;
    if (vars_[v].staged > 0 && can_enable(v))
      enable_var(v);
    check(cnsts_[c].conc_current <= cnsts_[c].conc_limit, "Concurrency overflow!");
    if (cnsts_[c].conc_current == cnsts_[c].conc_limit)
      break;
    e = nxt;
  }
}

void System::update_variable_bound(Id v, double bound) {
  modified_ = true;
  flat_valid_ = false;
  vars_[v].bound = bound;
  touch_v(v);
  if (vars_[v].n_elems)
    update_modified_set(elems_[vars_[v].ebase].cnst);
}

void System::update_variable_penalty(Id v, double penalty) {
  check(penalty >= 0, "Variable penalty should not be negative!");
  VarRec& r = vars_[v];
  if (penalty == r.penalty)
    return;
  bool enabling = penalty > 0 && r.penalty <= 0;
  bool disabling = penalty <= 0 && r.penalty > 0;
  modified_ = true;
  flat_valid_ = false;
  if (enabling) {
    r.staged = penalty;
    if (min_slack(v) < r.share)
      return;  // staged instead of enabled
    enable_var(v);
  } else if (disabling) {
    disable_var(v);
  } else {
    r.penalty = penalty;
    touch_v(v);
  }
}

void System::update_constraint_bound(Id c, double bound) {
  modified_ = true;
  flat_valid_ = false;
  update_modified_set(c);
  cnsts_[c].bound = bound;
  touch_c(c);
}

// ------------------------------------------------------------------------------------------
// selective update closure (maxmin.cpp:898-937)
// ------------------------------------------------------------------------------------------
void System::update_modified_set(Id c) {
  if (selective_ && !cnsts_[c].in_modified) {
    mod_push_back(c);
    update_modified_set_rec(c);
  }
}

void System::update_modified_set_rec(Id c0) {
  // Same closure as the recursive reference (every constraint reachable through enabled elements
  // of unvisited variables), with an explicit stack.
  std::vector<Id> stack{c0};
  while (!stack.empty()) {
    Id c = stack.back();
    stack.pop_back();
    for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next) {
      Id v = elems_[e].var;
      VarRec& r = vars_[v];
      if (r.visited == visited_counter_)
        continue;
      for (int i = 0; i < r.n_elems; i++) {
        Id c2 = elems_[r.ebase + i].cnst;
        if (c2 != c && !cnsts_[c2].in_modified) {
          mod_push_back(c2);
          stack.push_back(c2);
        }
      }
      r.visited = visited_counter_;
    }
  }
}

void System::remove_all_modified_set() {
  if (++visited_counter_ == 1)
    for (Id v = vset_head_; v != kNone; v = vars_[v].next)
      vars_[v].visited = 0;
  while (mod_head_ != kNone)
    mod_erase(mod_head_);
}

void System::clear_modified_actions() {
  for (Id v : modified_actions_)
    if (size_t(v) < vars_.size())
      vars_[v].in_modified_set = false;
  modified_actions_.clear();
}

// ------------------------------------------------------------------------------------------
// read API
// ------------------------------------------------------------------------------------------
Id System::get_constraint(Id v, int i) const {
  return i < vars_[v].n_elems ? elems_[vars_[v].ebase + i].cnst : kNone;
}
double System::get_constraint_weight(Id v, int i) const {
  return i < vars_[v].n_elems ? elems_[vars_[v].ebase + i].weight : 0.0;
}
double System::get_usage(Id c) const {
  double r = 0.0;
  const bool fat = cnsts_[c].policy == SharingPolicy::FATPIPE;
  for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next) {
    const ElemRec& x = elems_[e];
    if (x.weight <= 0)
      continue;
    double u = x.weight * values_[x.var];
    r = fat ? std::max(r, u) : r + u;
  }
  return r;
}
int System::get_variable_amount(Id c) const {
  int n = 0;
  for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next)
    n += elems_[e].weight > 0;
  return n;
}
std::vector<Id> System::constraint_elements(Id c) const {
  std::vector<Id> out;
  for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next)
    out.push_back(e);
  for (Id e = cnsts_[c].dis_head; e != kNone; e = elems_[e].next)
    out.push_back(e);
  return out;
}
std::vector<Id> System::variables_in_order() const {
  std::vector<Id> out;
  for (Id v = vset_head_; v != kNone; v = vars_[v].next)
    out.push_back(v);
  return out;
}
std::vector<Id> System::active_constraints_in_order() const {
  std::vector<Id> out;
  for (Id c = act_head_; c != kNone; c = cnsts_[c].act_next)
    out.push_back(c);
  return out;
}

void System::check_certificate(double prec, double* max_excess, int64_t* n_infeasible,
                               int64_t* n_unbottlenecked) const {
  // usage / max level per constraint over enabled elements with w > 0
  std::vector<double> usage(cnsts_.size(), 0.0), top(cnsts_.size(), 0.0);
  for (size_t c = 0; c < cnsts_.size(); c++) {
    const bool fat = cnsts_[c].policy == SharingPolicy::FATPIPE;
    for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next) {
      const ElemRec& x = elems_[e];
      if (x.weight <= 0)
        continue;
      const VarRec& r = vars_[x.var];
      const double u = x.weight * values_[x.var];
      usage[c] = fat ? std::max(usage[c], u) : usage[c] + u;
      top[c] = std::max(top[c], values_[x.var] * r.penalty);
    }
  }
  double worst = -1e300;
  int64_t infeasible = 0, unb = 0;
  std::vector<uint8_t> sat(cnsts_.size(), 0);
  for (size_t c = 0; c < cnsts_.size(); c++) {
    const double b = cnsts_[c].bound;
    if (!(b > b * prec))  // ignored by lmm_solve (maxmin.cpp:524)
      continue;
    const double ex = (usage[c] - b) / b;
    worst = std::max(worst, ex);
    if (usage[c] - b > b * prec)
      infeasible++;
    sat[c] = !(b - usage[c] > b * prec);
  }
  for (Id v = 0; v < Id(vars_.size()); v++) {
    const VarRec& r = vars_[v];
    const double rv = values_[v];
    if (!r.live || !(r.penalty > 0) || !(rv > 0))
      continue;
    if (r.bound > 0 && std::fabs(rv - r.bound) <= std::max(prec, 1e-9 * r.bound))
      continue;  // at its bound
    const double lvl = rv * r.penalty;
    bool ok = false;
    for (int i = 0; i < r.n_elems && !ok; i++) {
      const ElemRec& x = elems_[r.ebase + i];
      ok = x.weight > 0 && sat[x.cnst] && lvl >= top[x.cnst] * (1 - 1e-9);
    }
    unb += !ok;
  }
  *max_excess = worst;
  *n_infeasible = infeasible;
  *n_unbottlenecked = unb;
}

// ------------------------------------------------------------------------------------------
// flattening
// ------------------------------------------------------------------------------------------
std::vector<Id> System::solve_constraint_list() const {
  std::vector<Id> list;
  if (kind_ == SolverKind::MAXMIN && selective_) {
    for (Id c = mod_head_; c != kNone; c = cnsts_[c].mod_next)
      list.push_back(c);
  } else {
    for (Id c = act_head_; c != kNone; c = cnsts_[c].act_next)
      list.push_back(c);
  }
  return list;
}

// Active part of lmm_solve's init (maxmin.cpp:509-540).  Members: variables with an enabled element
// of w > 0 on a listed constraint with bound > bound*prec (the "part" test, :523-525).  Values of every
// variable seen through an enabled element of a listed constraint are reset to 0 (:509-514).
// Constraints: every listed constraint on which a member has an enabled element of w > 0, whether it
// passes the part test or not -- the device init applies that test itself (init_cnsts_waves: such a
// constraint starts dead, as it never enters cnst_light_tab, :545-554), so a bound that crosses it
// leaves the flattened structure as it is and the resident refresh path still applies.
void System::flatten_maxmin(Flat& f, const std::vector<Id>& list) {
  const double prec = maxmin_precision;
  const int32_t coff = int32_t(f.cbound.size());
  std::vector<int32_t> dense_c(cnsts_.size(), -1);
  std::vector<uint8_t> vmark(vars_.size(), 0);
  int32_t nc = 0;
  for (Id c : list) {
    const CnstRec& k = cnsts_[c];
    const bool part = k.bound > k.bound * prec;
    for (Id e = k.en_head; e != kNone; e = elems_[e].next) {
      const ElemRec& x = elems_[e];
      values_[x.var] = 0.0;
      if (part && x.weight > 0) {
        vmark[x.var] = 1;
        if (selective_ && !vars_[x.var].in_modified_set) {  // maxmin.cpp:536-538
          vars_[x.var].in_modified_set = true;
          modified_actions_.push_back(x.var);
        }
      }
    }
  }
  for (Id c : list) {
    const CnstRec& k = cnsts_[c];
    bool any = false;
    for (Id e = k.en_head; e != kNone && !any; e = elems_[e].next)
      any = elems_[e].weight > 0 && vmark[elems_[e].var];
    if (any) {
      dense_c[c] = coff + nc++;
      f.cbound.push_back(k.bound);
      f.cflags.push_back(k.policy == SharingPolicy::FATPIPE ? 1 : 0);
    }
  }
  for (Id v = 0; v < Id(vars_.size()); v++) {
    if (!vmark[v])
      continue;
    const VarRec& r = vars_[v];
    for (int i = 0; i < r.n_elems; i++) {
      const ElemRec& x = elems_[r.ebase + i];
      const int32_t dc = dense_c[x.cnst];
      if (dc >= 0 && x.weight > 0) {
        f.cnst_idx.push_back(dc);
        f.weight.push_back(x.weight);
      }
    }
    f.var_ptr.push_back(int64_t(f.cnst_idx.size()));
    f.penalty.push_back(r.penalty);
    f.vbound.push_back(r.bound);
    f.dense_vars.push_back(v);
  }
}

// fair_bottleneck.cpp:29-50: every variable is reset; enabled variables with a non-zero weight are
// listed, enabled ones without get 1.0; all active constraints are listed.
void System::flatten_fair(Flat& f) {
  const int32_t coff = int32_t(f.cbound.size());
  std::vector<int32_t> dense_c(cnsts_.size(), -1);
  for (Id v = vset_head_; v != kNone; v = vars_[v].next) {
    VarRec& r = vars_[v];
    values_[v] = 0.0;
    if (r.penalty > 0.0) {
      bool any_nz = false, any_pos = false;
      for (int i = 0; i < r.n_elems; i++) {
        any_nz |= elems_[r.ebase + i].weight != 0.0;
        any_pos |= elems_[r.ebase + i].weight > 0.0;
      }
      if (!any_nz)
        values_[v] = 1.0;
      else
        check(any_pos, "FairBottleneck: negative consumption weights are not supported");
    }
  }
  int32_t nc = 0;
  for (Id c = act_head_; c != kNone; c = cnsts_[c].act_next) {
    const CnstRec& k = cnsts_[c];
    bool any = false, zero_w = false;
    for (Id e = k.en_head; e != kNone; e = elems_[e].next) {
      any |= elems_[e].weight > 0;
      zero_w |= elems_[e].weight == 0.0;
    }
    if (any) {
      dense_c[c] = coff + nc++;
      f.cbound.push_back(k.bound);
      f.cflags.push_back(uint8_t((k.policy == SharingPolicy::FATPIPE ? 1 : 0) | (zero_w ? 2 : 0)));
    }
  }
  // CSR index of every flattened element (-1 = not flattened), for the CSC order below
  const bool ordered = f.csc_order.size() == f.cnst_idx.size();
  std::vector<int32_t> csr_of(ordered ? elems_.size() : 0, -1);
  for (Id v = 0; v < Id(vars_.size()); v++) {
    const VarRec& r = vars_[v];
    if (!r.live || !(r.penalty > 0))
      continue;
    bool listed = false;
    for (int i = 0; i < r.n_elems; i++)
      listed |= elems_[r.ebase + i].weight > 0 && dense_c[elems_[r.ebase + i].cnst] >= 0;
    if (!listed)
      continue;
    for (int i = 0; i < r.n_elems; i++) {
      const ElemRec& x = elems_[r.ebase + i];
      if (x.weight > 0 && dense_c[x.cnst] >= 0) {
        if (ordered)
          csr_of[size_t(r.ebase + i)] = int32_t(f.cnst_idx.size());
        f.cnst_idx.push_back(dense_c[x.cnst]);
        f.weight.push_back(x.weight);
      }
    }
    f.var_ptr.push_back(int64_t(f.cnst_idx.size()));
    f.penalty.push_back(r.penalty);
    f.vbound.push_back(r.bound);
    f.dense_vars.push_back(v);
  }
  // each listed constraint's flattened elements in its enabled-list order (dense constraint order)
  if (ordered)
    for (Id c = act_head_; c != kNone; c = cnsts_[c].act_next)
      if (dense_c[c] >= 0)
        for (Id e = cnsts_[c].en_head; e != kNone; e = elems_[e].next)
          if (csr_of[size_t(e)] >= 0)
            f.csc_order.push_back(csr_of[size_t(e)]);
}

void System::flatten_into(Flat& f) {
  if (kind_ == SolverKind::FAIR_BOTTLENECK)
    flatten_fair(f);
  else
    flatten_maxmin(f, solve_constraint_list());
}

void System::scatter_values(const double* x) {
  for (size_t i = 0; i < flat_.dense_vars.size(); i++)
    values_[flat_.dense_vars[i]] = x[i];
}

void System::finish_solve() {
  if (kind_ == SolverKind::FAIR_BOTTLENECK) {
    modified_ = true;  // fair_bottleneck.cpp:148
  } else {
    modified_ = false;
    if (selective_)
      remove_all_modified_set();
  }
}

// ------------------------------------------------------------------------------------------
// solve
// ------------------------------------------------------------------------------------------
void System::prepare() {
  if (resident_) {
    prepare_resident();
    return;
  }
  res_prepared_ = false;
  auto t0 = std::chrono::steady_clock::now();
  flat_ = Flat();
  flatten_into(flat_);
  stats_.flatten_ms = ms_since(t0);
  const int64_t nV = int64_t(flat_.dense_vars.size());
  const int64_t nC = int64_t(flat_.cbound.size());
  const int64_t nnz = int64_t(flat_.cnst_idx.size());
  auto t1 = std::chrono::steady_clock::now();
  const bool ordered = int64_t(flat_.csc_order.size()) == nnz && nnz > 0;
  int rc = lmmhip_upload2(ctx(), nV, nC, nnz, flat_.var_ptr.data(), flat_.cnst_idx.data(), flat_.weight.data(),
                          flat_.penalty.data(), flat_.vbound.data(), flat_.cbound.data(), flat_.cflags.data(),
                          ordered ? flat_.csc_order.data() : nullptr);
  if (rc)
    fatal(std::string("upload failed: ") + lmmhip_last_error());
  stats_.upload_ms = ms_since(t1);
  stats_.n_var = nV;
  stats_.n_cnst = nC;
  stats_.nnz = nnz;
  flat_valid_ = true;
}

void System::device_solve() {
  int kind = kind_ == SolverKind::FAIR_BOTTLENECK ? LMMHIP_KIND_FAIR_BOTTLENECK : LMMHIP_KIND_MAXMIN;
  int rc = lmmhip_solve(ctx(), kind, maxmin_precision);
  if (rc)
    fatal(std::string("device solve failed: ") + lmmhip_last_error());
  lmmhip_stats st{};
  lmmhip_get_stats(ctx(), &st);
  stats_.rounds = st.rounds;
  stats_.device_ms = st.device_ms;
}

void System::fetch() {
  if (res_prepared_) {
    fetch_resident();
    return;
  }
  auto t0 = std::chrono::steady_clock::now();
  xbuf_.resize(flat_.dense_vars.size());
  int rc = lmmhip_get_values(ctx(), xbuf_.data());
  if (rc)
    fatal(std::string("fetch failed: ") + lmmhip_last_error());
  scatter_values(xbuf_.data());
  stats_.fetch_ms = ms_since(t0);
  finish_solve();
}

// ------------------------------------------------------------------------------------------
// resident mode: delta log + device flatten (lmm_resident_kernels.hpp)
// ------------------------------------------------------------------------------------------
static void log_id(std::vector<uint8_t>& flag, std::vector<Id>& ids, Id i, size_t table) {
  if (flag.size() < table)
    flag.resize(std::max(table, flag.size() * 2), 0);
  if (!flag[size_t(i)]) {
    flag[size_t(i)] = 1;
    ids.push_back(i);
  }
}

void System::touch_e(Id e) {
  if (resident_ && !res_full_)
    log_id(res_de_, res_le_, e, elems_.size());
}
void System::touch_v(Id v) {
  if (resident_ && !res_full_)
    log_id(res_dv_, res_lv_, v, vars_.size());
}
void System::touch_c(Id c) {
  if (resident_ && !res_full_)
    log_id(res_dc_, res_lc_, c, cnsts_.size());
}

void System::set_resident(bool on) {
  resident_ = on;
  res_full_ = true;
  res_prepared_ = false;
  res_de_.clear();
  res_dv_.clear();
  res_dc_.clear();
  res_le_.clear();
  res_lv_.clear();
  res_lc_.clear();
}

void System::pending_deltas(int64_t out3[3]) const {
  out3[0] = res_full_ ? -1 : int64_t(res_le_.size());
  out3[1] = res_full_ ? -1 : int64_t(res_lv_.size());
  out3[2] = res_full_ ? -1 : int64_t(res_lc_.size());
}

// Pack the delta log (or, after set_resident(true), every record) and clear it.
void System::drain_deltas(ResPacked& p) {
  if (res_full_) {
    res_le_.resize(elems_.size());
    for (size_t i = 0; i < elems_.size(); i++)
      res_le_[i] = Id(i);
    res_lv_.resize(vars_.size());
    for (size_t i = 0; i < vars_.size(); i++)
      res_lv_[i] = Id(i);
    res_lc_.resize(cnsts_.size());
    for (size_t i = 0; i < cnsts_.size(); i++)
      res_lc_[i] = Id(i);
  }
  const size_t ne = res_le_.size(), nv = res_lv_.size(), nc = res_lc_.size();
  p.n_elem_total = int64_t(elems_.size());
  p.n_var_total = int64_t(vars_.size());
  p.n_cnst_total = int64_t(cnsts_.size());
  p.e_id.resize(ne);
  p.e_cnst.resize(ne);
  p.e_w.resize(ne);
  p.e_fl.resize(ne);
  p.v_id = res_lv_;
  p.v_eb.resize(nv);
  p.v_n.resize(nv);
  p.v_p.resize(nv);
  p.v_b.resize(nv);
  p.c_id = res_lc_;
  p.c_b.resize(nc);
  p.c_fl.resize(nc);
  for (size_t i = 0; i < ne; i++) {
    const ElemRec& x = elems_[res_le_[i]];
    p.e_id[i] = res_le_[i];
    p.e_cnst[i] = x.cnst;
    p.e_w[i] = x.weight;
    p.e_fl[i] = x.where == 1 ? 1 : 0;
  }
  for (size_t i = 0; i < nv; i++) {
    const VarRec& r = vars_[res_lv_[i]];
    p.v_eb[i] = r.ebase;
    p.v_n[i] = r.live ? r.n_elems : -1;
    p.v_p[i] = r.penalty;
    p.v_b[i] = r.bound;
  }
  for (size_t i = 0; i < nc; i++) {
    const CnstRec& k = cnsts_[res_lc_[i]];
    p.c_b[i] = k.bound;
    p.c_fl[i] = k.policy == SharingPolicy::FATPIPE ? 1 : 0;
  }
  if (!res_full_) {
    for (Id e : res_le_)
      res_de_[size_t(e)] = 0;
    for (Id v : res_lv_)
      res_dv_[size_t(v)] = 0;
    for (Id c : res_lc_)
      res_dc_[size_t(c)] = 0;
  }
  res_le_.clear();
  res_lv_.clear();
  res_lc_.clear();
  res_full_ = false;
}

// Ship the delta log to the device mirror.
void System::res_sync() {
  ResPacked p;
  drain_deltas(p);
  int rc = lmmhip_res_apply(ctx(), p.n_elem_total, p.n_var_total, p.n_cnst_total, int64_t(p.e_id.size()),
                            p.e_id.data(), p.e_cnst.data(), p.e_w.data(), p.e_fl.data(), int64_t(p.v_id.size()),
                            p.v_id.data(), p.v_eb.data(), p.v_n.data(), p.v_p.data(), p.v_b.data(),
                            int64_t(p.c_id.size()), p.c_id.data(), p.c_b.data(), p.c_fl.data());
  if (rc)
    fatal(std::string("resident delta upload failed: ") + lmmhip_last_error());
  stats_.delta_records = int64_t(p.e_id.size() + p.v_id.size() + p.c_id.size());
}

void System::prepare_resident() {
  auto t0 = std::chrono::steady_clock::now();
  res_sync();
  // The active set rarely changes between simulation steps: its list (a pointer chase over the
  // constraint records, ~0.1 s at 1e6 constraints) is cached until make_cnst_(in)active.
  std::vector<Id> mod_list;
  if (selective_ && kind_ == SolverKind::MAXMIN)
    mod_list = solve_constraint_list();
  else if (!act_cache_ok_) {
    act_cache_ = solve_constraint_list();
    act_cache_ok_ = true;
  }
  const std::vector<Id>& list = selective_ && kind_ == SolverKind::MAXMIN ? mod_list : act_cache_;
  const bool fair = kind_ == SolverKind::FAIR_BOTTLENECK;
  if (selective_ && !fair) {  // Lazy side effect, maxmin.cpp:536-538 (the walk the reference does at init)
    const double prec = maxmin_precision;
    for (Id c : list) {
      const CnstRec& k = cnsts_[c];
      if (!(k.bound > k.bound * prec))
        continue;
      for (Id e = k.en_head; e != kNone; e = elems_[e].next) {
        const ElemRec& x = elems_[e];
        if (x.weight > 0 && !vars_[x.var].in_modified_set) {
          vars_[x.var].in_modified_set = true;
          modified_actions_.push_back(x.var);
        }
      }
    }
  }
  stats_.flatten_ms = ms_since(t0);
  auto t1 = std::chrono::steady_clock::now();
  int64_t cnt[3] = {0, 0, 0};
  int rc = fair ? lmmhip_res_flatten_fair(ctx(), int64_t(list.size()), list.data(), cnt)
                : lmmhip_res_flatten(ctx(), int64_t(list.size()), list.data(), maxmin_precision, cnt);
  if (rc)
    fatal(std::string("resident flatten failed: ") + lmmhip_last_error());
  stats_.upload_ms = ms_since(t1);
  stats_.n_var = cnt[0];
  stats_.n_cnst = cnt[1];
  stats_.nnz = cnt[2];
  flat_ = Flat();
  flat_valid_ = false;
  res_prepared_ = true;
}

void System::fetch_resident() {
  auto t0 = std::chrono::steady_clock::now();
  const size_t n = vars_.size();
  double* out = values_.data();
  // Large systems: the values arrive in slices (lmmhip_res_values_sliced: one array, LMMHIP_VAL_KEEP marks the
  // slots to leave alone) and host threads scatter each slice as soon as it has landed, while the next ones are
  // still crossing PCIe (C2: 1e7 slots, 80 MB).  Small ones: one copy, one thread.
  const size_t nt = n >= (size_t(1) << 20) ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
  const char* sl = std::getenv("LMM_FETCH_SLICES");  // measurement knob: slices per fetch (1: one copy, then scatter)
  const int ns = sl && *sl ? std::max(1, std::min(256, std::atoi(sl))) : nt > 1 ? int(4 * nt) : 1;
  const double* vals = nullptr;
  if (lmmhip_res_values_sliced(ctx(), int64_t(n), ns, &vals))
    fatal(std::string("resident fetch failed: ") + lmmhip_last_error());
  const size_t per = (n + size_t(ns) - 1) / size_t(ns);
  const uint64_t* bits = reinterpret_cast<const uint64_t*>(vals);
  std::atomic<int> err{0};
  auto work = [&](size_t t) {
    for (size_t i = t; i < size_t(ns); i += nt) {
      if (lmmhip_res_values_wait(ctx(), int(i))) {
        err = 1;
        return;
      }
      const size_t lo = std::min(n, i * per), hi = std::min(n, lo + per);
      for (size_t v = lo; v < hi; v++)
        if (bits[v] != LMMHIP_VAL_KEEP)
          out[v] = vals[v];
    }
  };
  if (nt <= 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (size_t t = 1; t < nt; t++)
      pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool)
      th.join();
  }
  if (err)
    fatal(std::string("resident fetch failed: ") + lmmhip_last_error());
  res_prepared_ = false;
  stats_.fetch_ms = ms_since(t0);
  finish_solve();
}

void System::lmm_solve() {
  if (!modified_)
    return;
  SolverKind saved = kind_;
  kind_ = SolverKind::MAXMIN;  // lmm_solve() is the max-min solver even on a FairBottleneck
  try {
    prepare();
    device_solve();
    fetch();
  } catch (...) {
    kind_ = saved;
    throw;
  }
  kind_ = saved;
}

void System::solve() {
  if (kind_ == SolverKind::MAXMIN) {
    lmm_solve();
    return;
  }
  if (!modified_)  // fair_bottleneck.cpp:25
    return;
  prepare();
  device_solve();
  fetch();
}

// ------------------------------------------------------------------------------------------
// batched solve: disjoint union of independent systems in one device solve
// ------------------------------------------------------------------------------------------
void solve_batch(System** systems, int n) {
  if (n <= 0)
    return;
  const SolverKind kind = systems[0]->kind();
  System::Flat f;
  std::vector<size_t> var_begin(size_t(n) + 1, 0);
  std::vector<int64_t> voff(size_t(n) + 1, 0), coff(size_t(n) + 1, 0);  // block-diagonal layout
  for (int i = 0; i < n; i++) {
    check(systems[i]->kind() == kind, "solve_batch: mixed solver kinds");
    size_t before = f.dense_vars.size();
    systems[i]->flatten_into(f);
    var_begin[i] = before;
    var_begin[i + 1] = f.dense_vars.size();
    voff[size_t(i) + 1] = int64_t(f.dense_vars.size());
    coff[size_t(i) + 1] = int64_t(f.cbound.size());
  }
  System* s0 = systems[0];
  const bool ordered = f.csc_order.size() == f.cnst_idx.size() && !f.cnst_idx.empty();
  int rc = lmmhip_upload2(s0->ctx(), int64_t(f.dense_vars.size()), int64_t(f.cbound.size()),
                          int64_t(f.cnst_idx.size()), f.var_ptr.data(), f.cnst_idx.data(), f.weight.data(),
                          f.penalty.data(), f.vbound.data(), f.cbound.data(), f.cflags.data(),
                          ordered ? f.csc_order.data() : nullptr);
  if (rc)
    fatal(std::string("batch upload failed: ") + lmmhip_last_error());
  if (kind == SolverKind::MAXMIN && (rc = lmmhip_set_batch(s0->ctx(), n, voff.data(), coff.data())))
    fatal(std::string("batch declaration failed: ") + lmmhip_last_error());
  rc = lmmhip_solve(s0->ctx(), kind == SolverKind::FAIR_BOTTLENECK ? 1 : 0, maxmin_precision);
  if (rc)
    fatal(std::string("batch solve failed: ") + lmmhip_last_error());
  std::vector<double> x(f.dense_vars.size());
  rc = lmmhip_get_values(s0->ctx(), x.data());
  if (rc)
    fatal(std::string("batch fetch failed: ") + lmmhip_last_error());
  for (int i = 0; i < n; i++) {
    System* s = systems[i];
    // values of the dense block of system i
    for (size_t j = var_begin[i]; j < var_begin[i + 1]; j++)
      s->set_value(f.dense_vars[j], x[j]);
    s->finish_solve();
  }
}

}  // namespace lmm
}  // namespace simgrid_amd
