// ORACLE — TEST INFRASTRUCTURE ONLY (see lmm_oracle.hpp header for the reference map).
#include "lmm_oracle.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>

namespace lmm_oracle {

double g_maxmin_precision = 1e-5;  // maxmin.cpp:12
int g_concurrency_limit = -1;      // maxmin.cpp:14

[[noreturn]] static void die(const char* what) {
  std::fprintf(stderr, "lmm_oracle: assertion failed: %s\n", what);
  std::abort();
}
#define ORACLE_ASSERT(c, msg) \
  do {                        \
    if (!(c))                 \
      die(msg);               \
  } while (0)

// surf_interface.hpp:34-54
static inline void dbl_update(double* x, double v, double prec) {
  *x -= v;
  if (*x < prec)
    *x = 0.0;
}
static inline bool dbl_positive(double v, double prec) { return v > prec; }
static inline bool dbl_equals(double a, double b, double prec) { return std::fabs(a - b) < prec; }

// ---- Element concurrency (maxmin.cpp:42-58) ----
void Element::dec_concurrency() {
  ORACLE_ASSERT(cnst->conc_current >= concurrency(), "concurrency underflow");
  cnst->conc_current -= concurrency();
}
void Element::inc_concurrency() {
  cnst->conc_current += concurrency();
  cnst->conc_maximum = std::max(cnst->conc_maximum, cnst->conc_current);
  ORACLE_ASSERT(cnst->conc_limit < 0 || cnst->conc_current <= cnst->conc_limit, "Concurrency limit overflow!");
}

int Constraint::slack() const {
  return conc_limit < 0 ? std::numeric_limits<int>::max() : conc_limit - conc_current;
}

// maxmin.cpp:948-961
double Constraint::get_usage() {
  double r = 0.0;
  for (Element& e : enabled) {
    if (e.weight <= 0)
      continue;
    double c = e.weight * e.var->value;
    r = (policy == Policy::FATPIPE) ? std::max(r, c) : r + c;
  }
  return r;
}
int Constraint::variable_amount() {
  int n = 0;
  for (Element& e : enabled)
    n += e.weight > 0;
  return n;
}

int Variable::min_slack() const {
  int best = std::numeric_limits<int>::max();
  for (const Element& e : elems) {
    int s = e.cnst->slack();
    if (s < best) {
      if (s == 0)
        return 0;
      best = s;
    }
  }
  return best;
}

// ---- System lifetime ----
System::System(bool sel) : selective(sel) {}

System::~System() {
  while (!variables.empty()) {
    Variable& v = variables.front();
    variables.pop_front();
    var_free(&v);
  }
  while (!all_cnsts.empty()) {
    Constraint& c = all_cnsts.front();
    all_cnsts.pop_front();
    make_cnst_inactive(&c);
    delete &c;
  }
}

Constraint* System::constraint_new(double bound) {
  auto* c = new Constraint;
  c->bound = bound;
  c->rank = next_cnst_rank++;
  c->conc_limit = g_concurrency_limit;
  all_cnsts.push_back(*c);
  return c;
}

Variable* System::variable_new(void* user, double penalty, double bound, size_t n_cnst) {
  auto* v = new Variable;
  v->user = user;
  v->rank = next_var_rank++;
  v->elems.reserve(n_cnst);
  v->penalty = penalty;
  v->bound = bound;
  v->visited = visited_counter - 1;
  if (penalty > 0)
    variables.push_front(*v);
  else
    variables.push_back(*v);
  return v;
}

void System::set_concurrency_limit(Constraint* c, int limit) {
  ORACLE_ASSERT(limit < 0 || c->conc_maximum <= limit, "new concurrency limit below observed maximum");
  c->conc_limit = limit;
}

// maxmin.cpp:106-138
void System::var_free(Variable* v) {
  modified = true;
  // A staged variable with two elements on one constraint could be re-enabled by its own
  // on_disabled_var() below and then erased from variable_set a second time: undefined behaviour
  // in the reference (crash).  Defined here as "a variable being freed is never re-enabled".
  v->staged_penalty = 0.0;
  if (!v->elems.empty())
    update_modified_set(v->elems[0].cnst);
  for (Element& e : v->elems) {
    Constraint* c = e.cnst;
    if (v->penalty > 0)
      e.dec_concurrency();
    if (e.enabled_link.linked())
      c->enabled.erase(e);
    if (e.disabled_link.linked())
      c->disabled.erase(e);
    if (e.active_link.linked())
      c->active.erase(e);
    if (c->enabled.size() + c->disabled.size() == 0)
      make_cnst_inactive(c);
    else
      on_disabled_var(c);
  }
  v->elems.clear();
  delete v;
}

void System::variable_free(Variable* v) {
  if (v->all_link.linked())
    variables.erase(*v);
  if (v->saturated_link.linked())
    saturated_vars.erase(*v);
  var_free(v);
}

void System::variable_free_all() {
  while (!variables.empty())
    variable_free(&variables.front());
}

// maxmin.cpp:234-285
void System::expand(Constraint* c, Variable* v, double w) {
  modified = true;
  int current_share = 0;
  if (v->share > 1)
    for (Element& e : v->elems)
      if (e.cnst == c && e.enabled_link.linked())
        current_share += e.concurrency();

  if (v->penalty > 0 && v->share - current_share > c->slack()) {
    double pen = v->penalty;
    disable_var(v);
    for (Element& e : v->elems)
      on_disabled_var(e.cnst);
    w = 0;
    v->staged_penalty = pen;
  }
  ORACLE_ASSERT(v->elems.size() < v->elems.capacity(), "Too much constraints");
  v->elems.emplace_back();
  Element& e = v->elems.back();
  e.weight = w;
  e.cnst = c;
  e.var = v;
  if (v->penalty != 0) {
    c->enabled.push_front(e);
    e.inc_concurrency();
  } else {
    c->disabled.push_back(e);
  }
  if (!selective) {
    make_cnst_active(c);
  } else if (e.weight > 0 || v->penalty > 0) {
    make_cnst_active(c);
    update_modified_set(c);
    if (v->elems.size() > 1)
      update_modified_set(v->elems[0].cnst);
  }
}

// maxmin.cpp:287-323
void System::expand_add(Constraint* c, Variable* v, double w) {
  modified = true;
  auto it = std::find_if(v->elems.begin(), v->elems.end(), [c](const Element& e) { return e.cnst == c; });
  if (it == v->elems.end()) {
    expand(c, v, w);
    return;
  }
  Element& e = *it;
  if (v->penalty != 0)
    e.dec_concurrency();
  if (c->policy != Policy::FATPIPE)
    e.weight += w;
  else
    e.weight = std::max(e.weight, w);
  if (v->penalty != 0) {
    if (c->slack() < e.concurrency()) {
      double pen = v->penalty;
      disable_var(v);
      for (Element& e2 : v->elems)
        on_disabled_var(e2.cnst);
      v->staged_penalty = pen;
    }
    e.inc_concurrency();
  }
  update_modified_set(c);
}

// maxmin.cpp:749-772
void System::enable_var(Variable* v) {
  v->penalty = v->staged_penalty;
  v->staged_penalty = 0;
  variables.erase(*v);
  variables.push_front(*v);
  for (Element& e : v->elems) {
    e.cnst->disabled.erase(e);
    e.cnst->enabled.push_front(e);
    e.inc_concurrency();
  }
  if (!v->elems.empty())
    update_modified_set(v->elems[0].cnst);
}

// maxmin.cpp:774-795
void System::disable_var(Variable* v) {
  ORACLE_ASSERT(v->staged_penalty == 0, "Staged penalty should have been cleared");
  variables.erase(*v);
  variables.push_back(*v);
  if (!v->elems.empty())
    update_modified_set(v->elems[0].cnst);
  for (Element& e : v->elems) {
    e.cnst->enabled.erase(e);
    e.cnst->disabled.push_back(e);
    if (e.active_link.linked())
      e.cnst->active.erase(e);
    e.dec_concurrency();
  }
  v->penalty = 0.0;
  v->staged_penalty = 0.0;
  v->value = 0.0;
}

// maxmin.cpp:804-843
void System::on_disabled_var(Constraint* c) {
  if (c->conc_limit < 0)
    return;
  int budget = (int)c->disabled.size();
  if (budget == 0)
    return;
  Element* e = c->disabled.first();
  while (budget-- && e) {
    Element* nxt = e->disabled_link.linked() ? c->disabled.after(*e) : nullptr;
    if (e->var->staged_penalty > 0 && e->var->can_enable())
      enable_var(e->var);
    ORACLE_ASSERT(c->conc_current <= c->conc_limit, "Concurrency overflow!");
    if (c->conc_current == c->conc_limit)
      break;
    e = nxt;
  }
}

// maxmin.cpp:703-710
void System::update_variable_bound(Variable* v, double b) {
  modified = true;
  v->bound = b;
  if (!v->elems.empty())
    update_modified_set(v->elems[0].cnst);
}

// maxmin.cpp:846-881
void System::update_variable_penalty(Variable* v, double p) {
  ORACLE_ASSERT(p >= 0, "Variable penalty should not be negative!");
  if (p == v->penalty)
    return;
  bool enabling = p > 0 && v->penalty <= 0;
  bool disabling = p <= 0 && v->penalty > 0;
  modified = true;
  if (enabling) {
    v->staged_penalty = p;
    if (v->min_slack() < v->share)
      return;  // staged
    enable_var(v);
  } else if (disabling) {
    disable_var(v);
  } else {
    v->penalty = p;
  }
}

// maxmin.cpp:883-888
void System::update_constraint_bound(Constraint* c, double b) {
  modified = true;
  update_modified_set(c);
  c->bound = b;
}

// maxmin.cpp:898-937
void System::update_modified_set_rec(Constraint* c) {
  for (Element& e : c->enabled) {
    Variable* v = e.var;
    for (Element& e2 : v->elems) {
      if (v->visited == visited_counter)
        break;
      if (e2.cnst != c && !e2.cnst->modified_link.linked()) {
        modified_cnsts.push_back(*e2.cnst);
        update_modified_set_rec(e2.cnst);
      }
    }
    v->visited = visited_counter;
  }
}
void System::update_modified_set(Constraint* c) {
  if (selective && !c->modified_link.linked()) {
    modified_cnsts.push_back(*c);
    update_modified_set_rec(c);
  }
}
void System::remove_all_modified_set() {
  if (++visited_counter == 1)
    for (Variable& v : variables)
      v.visited = 0;
  modified_cnsts.clear();
}

// maxmin.cpp:487-500
void System::lmm_solve() {
  if (!modified)
    return;
  if (selective)
    solve_list(modified_cnsts);
  else
    solve_list(active_cnsts);
}

// maxmin.cpp:397-409
static inline void sat_cnst_update(double ratio, int idx, std::vector<int>& sat, double* min_usage) {
  ORACLE_ASSERT(ratio > 0, "Impossible");
  if (*min_usage < 0 || *min_usage > ratio) {
    *min_usage = ratio;
    sat.assign(1, idx);
  } else if (*min_usage == ratio) {
    sat.push_back(idx);
  }
}

// maxmin.cpp:411-424
static inline void sat_var_update(Light* tab, const std::vector<int>& sat, System* s) {
  for (int i : sat)
    for (Element& e : tab[i].cnst->active) {
      ORACLE_ASSERT(e.var->penalty > 0, "inactive element in active set");
      if (e.weight > 0 && !e.var->saturated_link.linked())
        s->saturated_vars.push_back(*e.var);
    }
}

static inline void drop_light(Constraint* c, Light* tab, int& n) {
  if (!c->light)
    return;
  int idx = int(c->light - tab);
  tab[idx] = tab[n - 1];
  tab[idx].cnst->light = &tab[idx];
  n--;
  c->light = nullptr;
}

// maxmin.cpp:502-693
template <class List> void System::solve_list(List& list) {
  const double prec = g_maxmin_precision;
  double min_usage = -1, min_bound = -1;
  last_rounds = 0;

  for (Constraint& c : list)
    for (Element& e : c.enabled) {
      ORACLE_ASSERT(e.var->penalty > 0, "disabled var in enabled set");
      e.var->value = 0.0;
    }

  std::vector<Light> tab_storage(list.size() + 1);
  Light* tab = tab_storage.data();
  int n_light = 0;
  std::vector<int> sat;

  for (Constraint& c : list) {
    c.remaining = c.bound;
    c.init_recorded = false;
    if (!dbl_positive(c.remaining, c.bound * prec))
      continue;
    c.usage = 0;
    for (Element& e : c.enabled) {
      if (e.weight <= 0)
        continue;
      double u = e.weight / e.var->penalty;
      if (c.policy != Policy::FATPIPE)
        c.usage += u;
      else if (c.usage < u)
        c.usage = u;
      if (e.active_link.linked())  // defensive: the reference pushes unconditionally
        c.active.erase(e);
      c.active.push_front(e);
      if (selective && !e.var->in_modified_set) {
        e.var->in_modified_set = true;
        modified_actions.push_back(e.var);
      }
    }
    c.init_usage = c.usage;
    c.init_remaining = c.remaining;
    c.init_recorded = true;
    if (c.usage > 0) {
      tab[n_light].cnst = &c;
      c.light = &tab[n_light];
      tab[n_light].remaining_over_usage = c.remaining / c.usage;
      sat_cnst_update(tab[n_light].remaining_over_usage, n_light, sat, &min_usage);
      ORACLE_ASSERT(!c.active.empty(), "constraint without active element");
      n_light++;
    }
  }
  sat_var_update(tab, sat, this);

  if (depth_on) {
    depth_D = 0;
    depth_sat_events = depth_bound_events = 0;
    depth_hist.clear();
    depth_bhist.clear();
    for (Constraint& c : list) {
      c.dep_lvl = 0;
      c.sat_lvl = -1;
      c.sat_round = -1;
      for (Element& e : c.enabled) {
        e.var->fix_lvl = -1;
        e.var->fix_round = -1;
        e.var->fix_by = 0;
      }
    }
  }
  std::vector<std::pair<Variable*, int>> depth_fixed;  // (variable, level) fixed this round (depth_on)
  std::vector<Constraint*> depth_sat;                  // this round's minimal-ratio constraints
  do {
    last_rounds++;
    if (depth_on) {  // this round's saturating constraints (used only if no bound fix preempts them)
      depth_fixed.clear();
      depth_sat.clear();
      for (int i : sat) {
        tab[i].cnst->sat_round = last_rounds;
        depth_sat.push_back(tab[i].cnst);
      }
    }
    for (Variable& v : saturated_vars) {
      ORACLE_ASSERT(v.penalty > 0, "DIE_IMPOSSIBLE");
      if (v.bound > 0 && v.bound * v.penalty < min_usage) {
        if (min_bound < 0)
          min_bound = v.bound * v.penalty;
        else
          min_bound = std::min(min_bound, v.bound * v.penalty);
      }
    }
    while (!saturated_vars.empty()) {
      Variable& v = saturated_vars.front();
      if (min_bound < 0) {
        v.value = min_usage / v.penalty;
      } else if (dbl_equals(min_bound, v.bound * v.penalty, prec)) {
        v.value = v.bound;
      } else {
        saturated_vars.pop_front();
        continue;
      }
      if (depth_on) {  // the event's level, from the constraints' dependencies of earlier rounds only
        int lvl = 0, by = 0;
        for (Element& e : v.elems) {
          Constraint* c = e.cnst;
          if (min_bound >= 0) {  // a bound fix: its own node, after every constraint of the variable
            lvl = std::max(lvl, c->dep_lvl + 1);
          } else if (c->sat_round == last_rounds && c->dep_lvl + 1 > lvl) {  // this round's saturation of c (ties:
            lvl = c->dep_lvl + 1;                                           // the deepest)
            by = c->rank;
          }
        }
        v.fix_lvl = lvl;
        v.fix_round = last_rounds;
        v.fix_by = by;
        depth_fixed.emplace_back(&v, lvl);
      }
      for (Element& e : v.elems) {
        Constraint* c = e.cnst;
        if (c->policy != Policy::FATPIPE) {
          dbl_update(&c->remaining, e.weight * v.value, c->bound * prec);
          dbl_update(&c->usage, e.weight / v.penalty, prec);
          if (!dbl_positive(c->usage, prec) || !dbl_positive(c->remaining, c->bound * prec)) {
            drop_light(c, tab, n_light);
          } else if (c->light) {
            c->light->remaining_over_usage = c->remaining / c->usage;
          }
          if (e.active_link.linked())
            c->active.erase(e);
        } else {
          c->usage = 0.0;
          if (e.active_link.linked())
            c->active.erase(e);
          for (Element& e2 : c->enabled) {
            if (e2.var->value > 0)
              continue;
            if (e2.weight > 0)
              c->usage = std::max(c->usage, e2.weight / e2.var->penalty);
          }
          if (!dbl_positive(c->usage, prec) || !dbl_positive(c->remaining, c->bound * prec)) {
            drop_light(c, tab, n_light);
          } else if (c->light) {
            c->light->remaining_over_usage = c->remaining / c->usage;
            ORACLE_ASSERT(!c->active.empty(), "max constraint kept without active element");
          }
        }
      }
      saturated_vars.pop_front();
    }

    if (depth_on) {
      const bool bound_round = min_bound >= 0;
      for (auto& [v, lvl] : depth_fixed) {
        if (int(depth_hist.size()) <= lvl) {
          depth_hist.resize(size_t(lvl) + 1, 0);
          depth_bhist.resize(size_t(lvl) + 1, 0);
        }
        if (bound_round)
          depth_bhist[size_t(lvl)]++;
        depth_bound_events += bound_round;
        depth_D = std::max(depth_D, lvl);
      }
      if (!bound_round)
        for (Constraint* c : depth_sat) {
          c->sat_lvl = c->dep_lvl + 1;
          depth_sat_events++;
          if (int(depth_hist.size()) <= c->sat_lvl) {
            depth_hist.resize(size_t(c->sat_lvl) + 1, 0);
            depth_bhist.resize(size_t(c->sat_lvl) + 1, 0);
          }
          depth_hist[size_t(c->sat_lvl)]++;
          depth_D = std::max(depth_D, c->sat_lvl);
        }
      else
        for (Constraint* c : depth_sat)
          c->sat_round = -1;  // preempted by the bound fixes: it saturates in a later round
      for (auto& [v, lvl] : depth_fixed)  // then this round's fixes reach the constraints they touch
        for (Element& e : v->elems)
          e.cnst->dep_lvl = std::max(e.cnst->dep_lvl, lvl);
    }
    min_usage = -1;
    min_bound = -1;
    sat.clear();
    for (int pos = 0; pos < n_light; pos++) {
      ORACLE_ASSERT(!tab[pos].cnst->active.empty(), "Cannot saturate more a constraint that has no active element");
      sat_cnst_update(tab[pos].remaining_over_usage, pos, sat, &min_usage);
    }
    sat_var_update(tab, sat, this);
  } while (n_light > 0);

  modified = false;
  if (selective)
    remove_all_modified_set();
  for (Constraint& c : list)  // the light table dies here; never leave dangling pointers behind
    c.light = nullptr;
}

// fair_bottleneck.cpp:23-153
void FairBottleneck::solve() {
  if (!modified)
    return;
  const double prec = g_maxmin_precision;
  last_rounds = 0;
  for (Variable& v : variables) {
    v.value = 0.0;
    bool any_w = std::any_of(v.elems.begin(), v.elems.end(), [](const Element& e) { return e.weight != 0.0; });
    if (v.penalty > 0.0 && any_w)
      saturated_vars.push_back(v);
    else if (v.penalty > 0.0)
      v.value = 1.0;
  }
  for (Constraint& c : active_cnsts)
    saturated_cnsts.push_back(c);
  for (Constraint& c : saturated_cnsts) {
    c.remaining = c.bound;
    c.usage = 0.0;
  }

  auto& vlist = saturated_vars;
  auto& clist = saturated_cnsts;
  do {
    last_rounds++;
    for (Constraint* c = clist.first(); c;) {
      Constraint* nxt = clist.after(*c);
      int nb = 0;
      c->usage = 0.0;
      for (Element& e : c->enabled)
        if (e.weight > 0 && e.var->saturated_link.linked())
          nb++;
      if (nb > 0 && c->policy == Policy::FATPIPE)
        nb = 1;
      if (nb == 0) {
        c->remaining = 0.0;
        c->usage = 0.0;
        clist.erase(*c);
      } else {
        c->usage = c->remaining / nb;
      }
      c = nxt;
    }

    for (Variable* v = vlist.first(); v;) {
      Variable* nxt = vlist.after(*v);
      double inc = DBL_MAX;
      for (const Element& e : v->elems)
        if (e.weight > 0)
          inc = std::min(inc, e.cnst->usage / e.weight);
      if (v->bound > 0)
        inc = std::min(inc, v->bound - v->value);
      v->mu = inc;
      v->value += v->mu;
      if (v->value == v->bound)
        vlist.erase(*v);
      v = nxt;
    }

    for (Constraint* c = clist.first(); c;) {
      Constraint* nxt = clist.after(*c);
      if (c->policy != Policy::FATPIPE) {
        for (Element& e : c->enabled)
          dbl_update(&c->remaining, e.weight * e.var->mu, prec);
      } else {
        for (Element& e : c->enabled)
          c->usage = std::min(c->usage, e.weight * e.var->mu);
        dbl_update(&c->remaining, c->usage, prec);
      }
      if (c->remaining <= 0.0) {
        clist.erase(*c);
        for (Element& e : c->enabled) {
          if (e.var->penalty <= 0)
            break;
          if (e.weight > 0 && e.var->saturated_link.linked())
            vlist.erase(*e.var);
        }
      }
      c = nxt;
    }
  } while (!vlist.empty());

  clist.clear();
  modified = true;
}

}  // namespace lmm_oracle
