/* lmm_system.h — System-level C ABI of the MI355X LMM solver (liblmm_amd.so).
 *
 * One function per method of the reference's lmm::System / Constraint / Variable
 * (src/kernel/lmm/maxmin.hpp:179-557), so a SimGrid build (or a ctypes / cffi binding) can use the
 * GPU solver as a drop-in through the same call sequence the models already make:
 *   network_cm02.cpp:215-270, cpu_cas01.cpp:206-215, ptask_L07.cpp:181-201, maxmin_bench.cpp:45-83.
 * Handles: lmm_sys* is opaque; constraints and variables are int64 ids (>= 0) owned by the system.
 * Errors: functions returning int give 0 on success and a negative code on failure with the message
 * in lmm_last_error(); API misuse the reference would xbt_assert on (e.g. "Too much constraints")
 * is reported the same way instead of aborting the process.
 */
#ifndef LMM_SYSTEM_H
#define LMM_SYSTEM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lmm_sys lmm_sys;

/* globals — maxmin.cpp:12-14 (--cfg=maxmin/precision, --cfg=maxmin/concurrency-limit) */
void lmm_set_precision(double precision);
double lmm_get_precision(void);
void lmm_set_default_concurrency_limit(int limit);

/* --cfg-style configuration, "key:value" (sg_config.cpp:45 parses --cfg=key:value the same way):
 *   maxmin/precision:<double>         sg_maxmin_precision (sg_config.cpp:261)
 *   maxmin/concurrency-limit:<int>    sg_concurrency_limit (sg_config.cpp:264)
 *   maxmin/solver:hip|hip-auto|hip-persistent|hip-rounds
 *                                     the solver-selection flag the reference lacks: the
 *                                     device engine of the systems created afterwards (lmmhip_ctx_set_engine);
 *                                     this library has no CPU solver, so there is no "cpu" value
 *   maxmin/resident:yes|no            new max-min systems start in resident mode (default yes)
 * Returns 0, or -1 for an unknown key / bad value (message in lmm_last_error()).  lmm_config_get copies
 * the current value into buf (cap bytes) and returns its length. */
int lmm_config_set(const char* key_value);
int lmm_config_get(const char* key, char* buf, int cap);

/* make_new_maxmin_system (maxmin.cpp:25) / make_new_fair_bottleneck_system (fair_bottleneck.cpp:18) */
lmm_sys* lmm_system_new(int selective_update, int kind /* 0 maxmin, 1 fair bottleneck */);
void lmm_system_free(lmm_sys* s);

int64_t lmm_constraint_new(lmm_sys* s, double bound);                                  /* maxmin.hpp:395 */
/* The same with the opaque id the reference takes (Constraint::id_ = the Resource*, maxmin.hpp:395) */
int64_t lmm_constraint_new_id(lmm_sys* s, void* id, double bound);
void* lmm_constraint_get_id(lmm_sys* s, int64_t c);                                    /* :244 get_id */
int lmm_constraint_unshare(lmm_sys* s, int64_t c);                                     /* :185 */
int lmm_constraint_is_shared(lmm_sys* s, int64_t c);                                   /* :188 */
int lmm_constraint_set_concurrency_limit(lmm_sys* s, int64_t c, int limit);            /* :195 */
int lmm_constraint_concurrency(lmm_sys* s, int64_t c, int* current, int* maximum, int* limit);
int lmm_constraint_reset_concurrency_maximum(lmm_sys* s, int64_t c);                   /* :210 */
double lmm_constraint_get_usage(lmm_sys* s, int64_t c);                                /* :191 */
int lmm_constraint_get_variable_amount(lmm_sys* s, int64_t c);                         /* :192 */
double lmm_constraint_get_bound(lmm_sys* s, int64_t c);
int lmm_constraint_rank(lmm_sys* s, int64_t c);
int lmm_constraint_used(lmm_sys* s, int64_t c);                                        /* :441 */
/* elements in System::print() order (enabled then disabled); returns the count, fills up to cap */
int lmm_constraint_elements(lmm_sys* s, int64_t c, int* var_rank, double* weight, double* value, int* enabled,
                            int cap);

int64_t lmm_variable_new(lmm_sys* s, double penalty, double bound, int64_t n_cnst);   /* :404 */
/* The same with the opaque id the reference takes (Variable::id_ = the Action*, maxmin.hpp:404) */
int64_t lmm_variable_new_id(lmm_sys* s, void* id, double penalty, double bound, int64_t n_cnst);
void* lmm_variable_get_id(lmm_sys* s, int64_t v);                                      /* :330 get_id */
int lmm_variable_free(lmm_sys* s, int64_t v);                                         /* :411 */
int lmm_variable_free_all(lmm_sys* s);                                                /* :414 */
int lmm_variable_set_concurrency_share(lmm_sys* s, int64_t v, int share);             /* :305 */
double lmm_variable_get_value(lmm_sys* s, int64_t v);                                 /* :296 */
double lmm_variable_get_bound(lmm_sys* s, int64_t v);                                 /* :299 */
double lmm_variable_get_penalty(lmm_sys* s, int64_t v);                               /* :331 */
int lmm_variable_rank(lmm_sys* s, int64_t v);
int lmm_variable_number_of_constraints(lmm_sys* s, int64_t v);                        /* :325 */
int lmm_get_values(lmm_sys* s, const int64_t* vars, int64_t n, double* out);
int lmm_system_variables(lmm_sys* s, int64_t* out, int cap);          /* variable_set order      */
int lmm_system_active_constraints(lmm_sys* s, int64_t* out, int cap); /* active_constraint_set   */
int lmm_modified_actions(lmm_sys* s, int64_t* out, int cap);          /* Action::ModifiedSet     */
/* the same set as the variables' ids (the Action* the reference pushes, maxmin.cpp:536-538) */
int lmm_modified_action_ids(lmm_sys* s, void** out, int cap);
int lmm_clear_modified_actions(lmm_sys* s);

int lmm_expand(lmm_sys* s, int64_t c, int64_t v, double w);                            /* :422 */
int lmm_expand_add(lmm_sys* s, int64_t c, int64_t v, double w);                        /* :430 */
int lmm_update_variable_bound(lmm_sys* s, int64_t v, double bound);                    /* :433 */
int lmm_update_variable_penalty(lmm_sys* s, int64_t v, double penalty);                /* :436 */
int lmm_update_constraint_bound(lmm_sys* s, int64_t c, double bound);                  /* :439 */

int lmm_solve(lmm_sys* s);     /* virtual System::solve (maxmin.hpp:450 / :550)  */
int lmm_lmm_solve(lmm_sys* s); /* System::lmm_solve (maxmin.hpp:447)             */
int lmm_is_modified(lmm_sys* s);
/* split solve: flatten+upload / device-only solve (inputs resident in HBM) / D2H + scatter */
int lmm_prepare(lmm_sys* s);
int lmm_device_solve(lmm_sys* s);
int lmm_fetch(lmm_sys* s);
/* stats of the last solve: rounds, n_var, n_cnst, nnz (int64[4]); device/flatten/upload/fetch ms */
int lmm_last_stats(lmm_sys* s, int64_t* counts4, double* ms4);
/* Resident mode (lmmhip_res_*): the system lives in HBM, mutations since the
 * last solve (maxmin.cpp:205-323, 703-888) are shipped as a delta log and the max-min system is
 * flattened on the device.  Replaces the host flatten of lmm_prepare for max-min solves. */
int lmm_set_resident(lmm_sys* s, int on);
int lmm_is_resident(lmm_sys* s);
/* pending delta-log sizes {elements, variables, constraints}; -1 each = whole system pending */
int lmm_pending_deltas(lmm_sys* s, int64_t* out3);
/* records (elements + variables + constraints) shipped by the last resident solve */
int64_t lmm_last_delta_records(lmm_sys* s);
/* host table sizes {element slots, variable slots, constraint slots} (ids are < these) */
int lmm_table_sizes(lmm_sys* s, int64_t* out3);
/* Test/inspection hook: drain the pending delta log into caller buffers instead of shipping it (the
 * records lmmhip_res_apply would receive).  sizes6 in: capacities {elements, variables, constraints}
 * (>= lmm_pending_deltas, table sizes when -1); out: {ne, nv, nc, n_elem_total, n_var_total,
 * n_cnst_total}. */
int lmm_resident_drain(lmm_sys* s, int64_t* sizes6, int64_t* e_id, int32_t* e_cnst, double* e_weight,
                       uint8_t* e_flags, int32_t* v_id, int64_t* v_ebase, int32_t* v_nelem, double* v_penalty,
                       double* v_bound, int32_t* c_id, double* c_bound, uint8_t* c_flags);
/* The device context a system solves on (created on the current HIP device on first use);
 * gives access to the lmmhip_* measurement calls (profiling, per-round work profile). */
struct lmmhip_ctx* lmm_system_device_ctx(lmm_sys* s);
/* The device input of this system's next solve (System::flatten_into: the host half of solve(), which
 * resets the solved variables' values as solve() does).  Call with null arrays to get the sizes
 * (counts3 = n_var, n_cnst, nnz), then with arrays of those sizes; var_ids maps dense index -> variable
 * id.  Used by simgrid_amd/multi.py to split a system into connected components across GPUs. */
int lmm_flat_export(lmm_sys* s, int64_t* counts3, int64_t* var_ptr, int32_t* cnst_idx, double* weight, double* penalty,
                    double* vbound, double* cbound, uint8_t* cflags, int64_t* var_ids);
/* The order of each constraint's elements in that flattened system (as lmmhip_upload2's csc_order: the
 * CSR indices of constraint 0's elements, then constraint 1's, ...): the reference's enabled_element_set_
 * order for a FairBottleneck system (the order its per-element chain subtracts in, fair_bottleneck.cpp:
 * 111-116), ascending CSR order for a max-min one.  nnz must equal lmm_flat_export's count. */
int lmm_flat_export_order(lmm_sys* s, int64_t nnz, int64_t* csc_order);
/* Solve n independent systems as one device launch sequence (disjoint union). */
int lmm_solve_batch(lmm_sys** systems, int n);

/* Max-min certificate of the current values (validation utility, CPU): worst relative constraint
 * excess, number of infeasible constraints (the assertion of System::print(), maxmin.cpp:470), and
 * number of enabled variables with x > 0 below their bound that have no saturated constraint on
 * which their level x*penalty is maximal.  Size-independent parity property for large systems. */
int lmm_check_certificate(lmm_sys* s, double precision, double* max_excess, int64_t* n_infeasible,
                          int64_t* n_unbottlenecked);

/* generators (input construction through the API above): maxmin_bench class 0..3, run index */
int lmm_gen_maxmin_bench(lmm_sys* s, int klass, int run, int64_t* cnst_out, int64_t* var_out, int* check_start,
                         int* check_solve);
int64_t lmm_gen_synthetic(lmm_sys* s, int64_t nb_cnst, int64_t nb_var, int k, uint64_t seed, int max_share,
                          int penalty_mix, int bounded_permille, int fatpipe_permille, int64_t* var_out);

/* Cluster platforms: the links of one FAT_TREE / DRAGONFLY <cluster>
 * (FatTreeZone.cpp, DragonflyZone.cpp) and n_flows random host-to-host flows turned into variables
 * the way NetworkCm02Model::communicate (network_cm02.cpp:165-279, CM02 / LV08) or L07Action
 * (ptask_L07.cpp:143-208) does, in the state after each flow's latency is paid.  See
 * simgrid_amd/csrc/lmm_platforms.hpp for what is restated. */
typedef struct lmm_platform_params {
  int topology;                /* 0 FAT_TREE, 1 DRAGONFLY */
  const char* topo_parameters; /* e.g. "2;4,4;1,2;1,2" (fat tree), "3,4;4,3;5,1;2" (dragonfly) */
  double bw, lat;              /* cluster link bandwidth (B/s), latency (s) */
  int policy;                  /* 0 SHARED, 1 SPLITDUPLEX, 2 FATPIPE */
  double loopback_bw, loopback_lat, limiter_bw;
  double speed;                /* host speed (flop/s): L07 CPU constraints */
  int model;                   /* 0 CM02, 1 LV08, 2 L07 */
  int crosstraffic;            /* CM02 / LV08: the back route at weight 0.05 */
  int64_t n_flows;
  uint64_t seed;
  double size_min, size_max;   /* L07 flow sizes (bytes) */
  double tcp_gamma;            /* network/TCP-gamma */
} lmm_platform_params;
int lmm_platform_size(const lmm_platform_params* p, int64_t* n_links, int64_t* n_hosts);
/* DRAGONFLY only: DragonflyZone::rankId_to_coords (DragonflyZone.cpp:26-35) of every host — coords_out[4 h .. 4 h + 3]
 * = (group, chassis, blade, node) of host h, up to cap ints; returns the host count, or -1 (not a dragonfly, bad
 * topo_parameters: the errors of DragonflyZone::parse_specific_arguments). */
int64_t lmm_platform_dragonfly_coords(const lmm_platform_params* p, int32_t* coords_out, int64_t cap);
/* constraints: one per link (creation order), then for L07 one CPU per host; returns n_flows or -1 */
int64_t lmm_gen_platform_flows(lmm_sys* s, const lmm_platform_params* p, int64_t* cnst_out, int64_t* var_out);

/* One link and one communication over explicit links, through the same flow construction the platform
 * flows above use (lmm_platforms.hpp: link_constraint, communicate).
 * lmm_link_new replaces NetworkCm02Link's constraint (network_cm02.cpp:282-295): bound = bandwidth factor
 * (model 0 CM02: 1, 1 LV08: 0.97) * bw, FATPIPE unshared; returns the constraint id or -1.
 * lmm_communicate replaces the LMM part of NetworkCm02Model::communicate (network_cm02.cpp:165-274), the
 * variable carrying the opaque `id` (the reference passes the action, network_cm02.cpp:221-229): the route
 * (constraints, link bandwidths and latencies, in route order) at weight 1.0 and the back route (crosstraffic)
 * at 0.05; penalty 0 while the latency is unpaid (paid = 0) or the sharing penalty (paid = 1; 1.0 without
 * latency); bound from rate (< 0: none) and TCP-gamma.  Returns the variable id or -1; *out gets the action's
 * latency_ (after the latency factor 13.01 / 1), lat_current_, sharing_penalty_ and the bound. */
typedef struct lmm_comm_info {
  double latency, lat_current, sharing_penalty, bound;
} lmm_comm_info;
int64_t lmm_link_new(lmm_sys* s, int model, double bw, int fatpipe);
int64_t lmm_communicate(lmm_sys* s, void* id, int model, int64_t n_route, const int64_t* route_cnst, const double* route_bw,
                        const double* route_lat, int64_t n_back, const int64_t* back_cnst, double rate,
                        double tcp_gamma, int paid, lmm_comm_info* out);
/* WIFI access points (NetworkWifiLink, network_cm02.cpp:383-420).  lmm_wifi_link_new: the access point's
 * constraint, a shared link of bandwidth 1 / bandwidth factor (bound bf * (1 / bf)).  lmm_communicate_ex is
 * lmm_communicate with `crosstraffic` (the network/crosstraffic configuration: nonzero = on, whether or not the
 * back route holds links; lmm_communicate passes n_back > 0) and route_rates (NULL: no WIFI link on the route): 2
 * doubles per route link, the source and
 * destination stations' rates on that access point (NetworkWifiLink::get_host_rate, -1 = not associated), or
 * (0, 0) for an ordinary link.  A WIFI link weighs 1 / source rate (1 / destination rate when the source is not
 * associated, network_cm02.cpp:239-260), and its own bandwidth (1 / bf) and latency (0) are used, whatever
 * route_bw / route_lat hold for it.  Errors (-1, lmm_last_error) as the reference's assertions: crosstraffic on
 * with a WIFI link on the route (network_cm02.cpp:242), or neither station associated; and a rate that is neither
 * > 0 nor -1. */
int64_t lmm_wifi_link_new(lmm_sys* s, int model);
int64_t lmm_communicate_ex(lmm_sys* s, void* id, int model, int64_t n_route, const int64_t* route_cnst,
                           const double* route_bw, const double* route_lat, const double* route_rates, int64_t n_back,
                           const int64_t* back_cnst, int crosstraffic, double rate, double tcp_gamma, int paid,
                           lmm_comm_info* out);

int lmm_device_count(void);
const char* lmm_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LMM_SYSTEM_H */
