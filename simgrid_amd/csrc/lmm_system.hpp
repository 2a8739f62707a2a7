// lmm_system.hpp — host side of the MI355X LMM solver: a drop-in for SimGrid's lmm::System
// (src/kernel/lmm/maxmin.hpp:380-557).
//
// Same API surface and mutation semantics as the reference (constraint_new / variable_new /
// expand / expand_add / update_* / concurrency staging / selective update), but the bookkeeping is
// laid out for flattening, not for pointer chasing: constraints, variables and elements live in
// flat arrays addressed by 32-bit ids, a variable's elements are one contiguous slab (the
// reference's `cnsts_` vector reserved to number_of_constraints, maxmin.cpp:717), and the
// per-constraint enabled / disabled element sets are index-linked lists that keep the reference's
// push_front / push_back orders (they decide which staged variable on_disabled_var re-enables).
//
// solve() flattens the active part of the system into CSR (see include/lmm/lmm_hip.h), ships it
// to HBM and runs the HIP solver; there is no CPU fallback.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

struct lmmhip_ctx;

namespace simgrid_amd {
namespace lmm {

extern double maxmin_precision;  // sg_maxmin_precision, maxmin.cpp:12
extern int concurrency_limit;    // sg_concurrency_limit, maxmin.cpp:14
// solver selection (lmm_config_set "maxmin/solver", "maxmin/resident"): the engine of every new device
// context (LMMHIP_ENGINE_*) and whether new max-min systems start in resident mode
extern int solver_engine;
extern bool resident_default;

enum class SharingPolicy : int { FATPIPE = 0, SHARED = 1 };  // s4u::Link::SharingPolicy subset
enum class SolverKind : int { MAXMIN = 0, FAIR_BOTTLENECK = 1 };

using Id = int32_t;
constexpr Id kNone = -1;

struct ElemRec {
  Id cnst = kNone;
  Id var = kNone;
  double weight = 0.0;  // consumption_weight
  Id prev = kNone, next = kNone;  // link in the owning constraint's enabled OR disabled list
  uint8_t where = 0;              // 0 = unlinked, 1 = enabled list, 2 = disabled list
  int concurrency() const { return weight >= 1 ? 1 : 0; }  // maxmin.cpp:30-40
};

struct CnstRec {
  double bound = 0.0;
  int conc_current = 0, conc_maximum = 0, conc_limit = -1;
  SharingPolicy policy = SharingPolicy::SHARED;
  int rank = 0;
  void* id = nullptr;  // borrowed Resource*
  Id en_head = kNone, en_tail = kNone, dis_head = kNone, dis_tail = kNone;
  int32_t n_en = 0, n_dis = 0;
  Id act_prev = kNone, act_next = kNone;  // active_constraint_set
  Id mod_prev = kNone, mod_next = kNone;  // modified_constraint_set
  bool in_active = false, in_modified = false;
  int slack() const;
};

struct VarRec {
  double penalty = 0.0, staged = 0.0, bound = -1.0;  // value: System::values_ (a column of its own)
  int share = 1;
  int rank = 0;
  unsigned visited = 0;
  void* id = nullptr;  // borrowed Action*
  int64_t ebase = 0;   // element slab
  int32_t n_elems = 0, cap = 0;
  Id prev = kNone, next = kNone;  // variable_set
  bool live = false;
  bool in_modified_set = false;
};

struct SolveStats {
  int64_t rounds = 0, n_var = 0, n_cnst = 0, nnz = 0;
  double device_ms = 0.0, flatten_ms = 0.0, upload_ms = 0.0, fetch_ms = 0.0;
  int64_t delta_records = 0;  // resident mode: element + variable + constraint records shipped
};

class System {
public:
  explicit System(bool selective_update, SolverKind kind = SolverKind::MAXMIN);
  virtual ~System();
  System(const System&) = delete;
  System& operator=(const System&) = delete;

  Id constraint_new(void* id, double bound);
  Id variable_new(void* id, double penalty, double bound = -1.0, size_t number_of_constraints = 1);
  void variable_free(Id v);
  void variable_free_all();
  void expand(Id c, Id v, double w);
  void expand_add(Id c, Id v, double w);
  void update_variable_bound(Id v, double bound);
  void update_variable_penalty(Id v, double penalty);
  void update_constraint_bound(Id c, double bound);
  void unshare(Id c) {
    cnsts_[c].policy = SharingPolicy::FATPIPE;
    touch_c(c);
  }
  void set_concurrency_limit(Id c, int limit);
  void set_concurrency_share(Id v, int share) { vars_[v].share = share; }
  bool constraint_used(Id c) const { return cnsts_[c].in_active; }

  // System::lmm_solve (maxmin.cpp:487) — Lazy models call this one directly (Model.cpp:43), so
  // the device dispatch lives here, not only in the virtual solve().
  void lmm_solve();
  virtual void solve();  // maxmin.hpp:450 / FairBottleneck::solve (maxmin.hpp:550)

  // Split solve for measurement: flatten + upload (construction), device solve (inputs resident in
  // HBM), fetch (D2H + scatter).  solve() == prepare() ; device_solve() ; fetch().
  void prepare();
  void device_solve();
  void fetch();

  // read API (maxmin.hpp:296-331, :188-247)
  double get_value(Id v) const { return values_[v]; }
  double get_bound(Id v) const { return vars_[v].bound; }
  double get_penalty(Id v) const { return vars_[v].penalty; }
  int number_of_constraints(Id v) const { return vars_[v].n_elems; }
  Id get_constraint(Id v, int i) const;
  double get_constraint_weight(Id v, int i) const;
  double get_usage(Id c) const;  // maxmin.cpp:948-961
  int get_variable_amount(Id c) const;
  const CnstRec& cnst(Id c) const { return cnsts_[c]; }
  const VarRec& var(Id v) const { return vars_[v]; }
  void reset_concurrency_maximum(Id c) { cnsts_[c].conc_maximum = 0; }
  void set_value(Id v, double x) { values_[v] = x; }
  // elements of c in print order (enabled list, then disabled list), as element ids
  std::vector<Id> constraint_elements(Id c) const;
  const ElemRec& elem(Id e) const { return elems_[e]; }
  std::vector<Id> variables_in_order() const;
  std::vector<Id> active_constraints_in_order() const;

  // Max-min certificate of the current values (the checks System::print() asserts, maxmin.cpp:470-480,
  // plus the bottleneck property): returns the worst constraint excess (usage - bound)/bound, the
  // number of infeasible constraints, and the number of enabled variables with x > 0 that are below
  // their bound and have no saturated constraint on which their level x*penalty is maximal.
  void check_certificate(double prec, double* max_excess, int64_t* n_infeasible, int64_t* n_unbottlenecked) const;

  bool modified() const { return modified_; }
  bool selective() const { return selective_; }
  SolverKind kind() const { return kind_; }
  const SolveStats& last_stats() const { return stats_; }
  // Lazy-mode side effect of lmm_solve (maxmin.cpp:536-538): actions of newly active elements.
  std::vector<Id>& modified_actions() { return modified_actions_; }
  void clear_modified_actions();
  int64_t live_variables() const { return n_live_vars_; }
  size_t n_elem_slots() const { return elems_.size(); }
  size_t n_var_slots() const { return vars_.size(); }
  size_t n_cnst_slots() const { return cnsts_.size(); }

  // ---- flattening (also used by the batched multi-system path) ----
  struct Flat {
    std::vector<int64_t> var_ptr{0};
    std::vector<int32_t> cnst_idx;
    std::vector<double> weight, penalty, vbound, cbound;
    std::vector<uint8_t> cflags;
    std::vector<Id> dense_vars;  // dense index -> variable id
    // FairBottleneck: CSR element index of every CSC position, constraint-major, each constraint's
    // elements in the order of its enabled_element_set_ (the order bottleneck_solve subtracts them in,
    // fair_bottleneck.cpp:111-116); empty = the device's default order (lmmhip_upload2)
    std::vector<int64_t> csc_order;
  };
  // Append this system's active part to `f` (constraint indices offset by f.cbound.size()).
  void flatten_into(Flat& f);
  // Scatter device values (dense order of this system's block) back into variables.
  void scatter_values(const double* x);
  void finish_solve();

  lmmhip_ctx* ctx();

  // ---- resident mode ----
  // The element / variable / constraint records are mirrored in HBM (lmmhip_res_apply); every
  // mutation logs the records it touched, the log is shipped at the next max-min solve, and the
  // solver's CSR/CSC is rebuilt on the device (lmmhip_res_flatten) instead of flatten_maxmin + a full
  // upload.  Same results bit for bit (tests/test_gpu_resident.py), for lmm_solve and for
  // FairBottleneck::solve (flatten_fair's rules).  Turning it on ships the whole system at the next solve.
  void set_resident(bool on);
  bool resident() const { return resident_; }
  // Pending delta-log sizes (elements, variables, constraints; -1 each = full re-ship pending).
  void pending_deltas(int64_t out3[3]) const;
  // The delta log packed as lmmhip_res_apply takes it (res_sync ships it); draining clears the log.
  struct ResPacked {
    int64_t n_elem_total = 0, n_var_total = 0, n_cnst_total = 0;
    std::vector<int64_t> e_id, v_eb;
    std::vector<int32_t> e_cnst, v_id, v_n, c_id;
    std::vector<double> e_w, v_p, v_b, c_b;
    std::vector<uint8_t> e_fl, c_fl;
  };
  void drain_deltas(ResPacked& p);

private:
  void touch_e(Id e);
  void touch_v(Id v);
  void touch_c(Id c);
  void res_sync();
  void prepare_resident();
  void fetch_resident();
  // list helpers
  void en_push_front(Id c, Id e);
  void dis_push_back(Id c, Id e);
  void elem_unlink(Id e);
  void vset_push_front(Id v);
  void vset_push_back(Id v);
  void vset_erase(Id v);
  void make_cnst_active(Id c);
  void make_cnst_inactive(Id c);
  void mod_push_back(Id c);
  void mod_erase(Id c);

  void inc_conc(Id e);
  void dec_conc(Id e);
  int min_slack(Id v) const;
  bool can_enable(Id v) const { return vars_[v].staged > 0 && min_slack(v) >= vars_[v].share; }
  void enable_var(Id v);
  void disable_var(Id v);
  void on_disabled_var(Id c);
  void var_free(Id v);
  void update_modified_set(Id c);
  void update_modified_set_rec(Id c);
  void remove_all_modified_set();

  std::vector<Id> solve_constraint_list() const;
  void flatten_maxmin(Flat& f, const std::vector<Id>& list);
  void flatten_fair(Flat& f);

  bool selective_;
  SolverKind kind_;
  bool modified_ = false;
  unsigned visited_counter_ = 1;
  int next_var_rank_ = 1, next_cnst_rank_ = 1;

  std::vector<CnstRec> cnsts_;
  std::vector<VarRec> vars_;
  std::vector<double> values_;  // Variable::value_, kept as a column: the solve writes it as a stream
  std::vector<Id> free_var_ids_;
  std::vector<ElemRec> elems_;
  std::vector<std::vector<int64_t>> free_slabs_;  // by capacity (small caps only)
  Id vset_head_ = kNone, vset_tail_ = kNone;
  Id act_head_ = kNone, act_tail_ = kNone;
  Id mod_head_ = kNone, mod_tail_ = kNone;
  int64_t n_live_vars_ = 0;
  std::vector<Id> modified_actions_;

  // resident mode: delta log (dirty flags + lists of ids)
  bool resident_ = false, res_full_ = true, res_prepared_ = false;
  int engine_;  // maxmin/solver at construction (applied when the device context is created)
  std::vector<Id> act_cache_;  // active_constraint_set in list order (resident non-selective solves)
  bool act_cache_ok_ = false;
  std::vector<uint8_t> res_de_, res_dv_, res_dc_;
  std::vector<Id> res_le_, res_lv_, res_lc_;

  // device state
  lmmhip_ctx* ctx_ = nullptr;
  Flat flat_;
  bool flat_valid_ = false;
  std::vector<double> xbuf_;
  SolveStats stats_;
};

// Solve several independent systems as ONE device launch sequence (disjoint union: components
// never interact, so every system gets exactly its own solution).  All systems must share a kind.
void solve_batch(System** systems, int n);

[[noreturn]] void fatal(const std::string& msg);

}  // namespace lmm
}  // namespace simgrid_amd
