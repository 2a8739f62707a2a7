/* lmm_hip.h — device-side C ABI of the MI355X (gfx950) LMM solver.
 *
 * This is the boundary a SimGrid maintainer binds from src/kernel/lmm: the reference's
 * System::lmm_solve() (src/kernel/lmm/maxmin.cpp:487-500, called directly by Lazy models at
 * src/kernel/resource/Model.cpp:43 and through the virtual System::solve(), maxmin.hpp:450, by
 * Full models at Model.cpp:105) and FairBottleneck::solve() (maxmin.hpp:550 ->
 * fair_bottleneck.cpp:23) flatten their constraint x variable incidence into CSR and hand it
 * here.  Plain pointers and sizes only; no C++ or torch types cross this boundary.
 *
 * Conventions
 *   - every function returns 0 on success, a negative LMMHIP_E* code on failure; the
 *     thread-local message is available from lmmhip_last_error();
 *   - host pointers are borrowed for the duration of the call; device memory is owned by the
 *     context; one context per host thread (it owns one HIP stream);
 *   - the flattened system holds only the *active* elements (the ones lmm_solve's init loop,
 *     maxmin.cpp:520-540, would make active): enabled variable (penalty > 0), consumption
 *     weight > 0, constraint bound > bound * precision.  For FAIR_BOTTLENECK: enabled
 *     variables with weight > 0 on active constraints (fair_bottleneck.cpp:29-50).
 */
#ifndef LMM_HIP_H
#define LMM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LMMHIP_OK 0
#define LMMHIP_E_NODEVICE (-1)   /* no HIP device visible: the product has no CPU fallback */
#define LMMHIP_E_HIP (-2)        /* a HIP runtime call failed                                */
#define LMMHIP_E_ARG (-3)        /* invalid argument / shape                                 */
#define LMMHIP_E_STATE (-4)      /* call out of order (e.g. solve before upload)             */
#define LMMHIP_E_NOCONVERGE (-5) /* round guard tripped (solver bug; never expected)         */

#define LMMHIP_KIND_MAXMIN 0         /* System::lmm_solve           maxmin.cpp:502-693       */
#define LMMHIP_KIND_FAIR_BOTTLENECK 1 /* FairBottleneck::bottleneck_solve fair_bottleneck.cpp:23 */

typedef struct lmmhip_ctx lmmhip_ctx;

typedef struct lmmhip_stats {
  int64_t rounds;          /* device rounds of the last solve                               */
  int64_t n_var, n_cnst, nnz;
  double device_ms;        /* HIP-event time of the last solve (solve kernels only)         */
  double kernel_ms[8];     /* per-phase accumulated time, when profiling is enabled         */
  int64_t kernel_launches[8];
} lmmhip_stats;

/* Create a context on HIP device `device` (-1 = current device). */
int lmmhip_ctx_create(int device, lmmhip_ctx** out);
int lmmhip_ctx_destroy(lmmhip_ctx* ctx);

/* Upload a flattened system (replaces any previous one).
 *   n_var / n_cnst / nnz : sizes (nnz < 2^31)
 *   var_ptr[n_var+1]     : CSR row offsets (variable-major), int64
 *   cnst_idx[nnz]        : constraint index of each element, int32 in [0, n_cnst)
 *   weight[nnz]          : consumption weight of each element (> 0), fp64
 *   penalty[n_var]       : sharing penalty (> 0), fp64
 *   var_bound[n_var]     : variable bound (<= 0: unbounded), fp64
 *   cnst_bound[n_cnst]   : constraint bound, fp64
 *   cnst_flags[n_cnst]   : bit0 = FATPIPE (s4u::Link::SharingPolicy::FATPIPE),
 *                          bit1 = has an enabled zero-weight element (FairBottleneck FATPIPE quirk,
 *                                 fair_bottleneck.cpp:118-123)
 * The CSC (constraint-major) mirror is built by the library. */
int lmmhip_upload(lmmhip_ctx* ctx, int64_t n_var, int64_t n_cnst, int64_t nnz, const int64_t* var_ptr,
                  const int32_t* cnst_idx, const double* weight, const double* penalty, const double* var_bound,
                  const double* cnst_bound, const uint8_t* cnst_flags);

/* lmmhip_upload with the order of each constraint's elements given: csc_order[p] (p = 0..nnz-1,
 * constraint-major) is the CSR index of the p-th element of constraint k's segment, k ascending; NULL =
 * ascending CSR order.  FairBottleneck subtracts a constraint's increments one at a time in this order
 * (fair_bottleneck.cpp:111-116), so passing each constraint's enabled_element_set_ order makes a
 * one-context FAIR_BOTTLENECK solve bit-identical to the reference. */
int lmmhip_upload2(lmmhip_ctx* ctx, int64_t n_var, int64_t n_cnst, int64_t nnz, const int64_t* var_ptr,
                   const int32_t* cnst_idx, const double* weight, const double* penalty, const double* var_bound,
                   const double* cnst_bound, const uint8_t* cnst_flags, const int64_t* csc_order);

/* Update per-variable penalty/bound or per-constraint bound in place (no structural change). */
int lmmhip_update_vars(lmmhip_ctx* ctx, const double* penalty, const double* var_bound);
int lmmhip_update_cnsts(lmmhip_ctx* ctx, const double* cnst_bound);

/* ---- Resident System mirror + device-side delta log ----
 * Replaces the per-solve host flatten + full upload (System::lmm_solve's init walk, maxmin.cpp:509-555,
 * preceded by the mutations of maxmin.cpp:205-323 / 703-888) with: the host System's element /
 * variable / constraint records mirrored in HBM, only the records a mutation touched shipped per
 * solve, and the solver's CSR/CSC rebuilt on the device with System::flatten_maxmin's rules.
 *
 * lmmhip_res_apply: one delta batch.  *_total = sizes of the host tables (the mirror grows to them,
 *   keeping its contents).  Element e: constraint id (-1 = unused), weight, flags bit0 = in its
 *   constraint's enabled list.  Variable v: slab base (first element id), elements in use (-1 = dead),
 *   penalty, bound.  Constraint c: bound, flags bit0 = FATPIPE.  Host arrays are borrowed.
 * lmmhip_res_flatten: build the max-min system of the listed constraints (list order = dense order:
 *   the active set, or the modified set in selective mode) from the mirror; then lmmhip_solve(MAXMIN)
 *   as after lmmhip_upload.  counts3 (optional) = {n_var, n_cnst, nnz} of the built system.
 * lmmhip_res_values: after the solve, per variable slot (n = n_var_total of the mirror): values[v]
 *   and reset[v] = 1 iff lmm_solve assigns v (its solved value, or 0 for a variable seen through an
 *   enabled element of a listed constraint that is not part of the system, maxmin.cpp:509-514). */
int lmmhip_res_apply(lmmhip_ctx* ctx, int64_t n_elem_total, int64_t n_var_total, int64_t n_cnst_total, int64_t ne,
                     const int64_t* e_id, const int32_t* e_cnst, const double* e_weight, const uint8_t* e_flags,
                     int64_t nv, const int32_t* v_id, const int64_t* v_ebase, const int32_t* v_nelem,
                     const double* v_penalty, const double* v_bound, int64_t nc, const int32_t* c_id,
                     const double* c_bound, const uint8_t* c_flags);
int lmmhip_res_flatten(lmmhip_ctx* ctx, int64_t n_list, const int32_t* cnst_list, double precision, int64_t* counts3);
/* FairBottleneck flavour (System::flatten_fair, fair_bottleneck.cpp:29-50): every active constraint with
 * an enabled element of weight > 0 (cflags bit1 = one of weight 0), every live variable with penalty > 0
 * and such an element; values of the other live variables reset to 0, or 1.0 when penalised with no
 * non-zero weight; CSC chunks built on the device.  Then lmmhip_solve(FAIR_BOTTLENECK). */
int lmmhip_res_flatten_fair(lmmhip_ctx* ctx, int64_t n_list, const int32_t* cnst_list, int64_t* counts3);
int lmmhip_res_values(lmmhip_ctx* ctx, int64_t n, double* values, uint8_t* reset);
/* Same, into context-owned pinned host buffers (valid until the next call / lmmhip_ctx_destroy): the
 * D2H runs at full PCIe rate and the caller scatters from them without another copy. */
int lmmhip_res_values_pinned(lmmhip_ctx* ctx, int64_t n, const double** values, const uint8_t** reset);
/* Same values, fetched in `nslices` slices the caller can scatter while the next ones are still in flight
 * (System::fetch_resident): ONE array in context-owned pinned memory, where a slot the solve leaves alone holds
 * the bit pattern LMMHIP_VAL_KEEP (a signalling NaN no arithmetic produces) instead of a separate reset flag.
 * Returns once everything is queued; lmmhip_res_values_wait(ctx, i) blocks until slice i (slots
 * [i * ceil(n / nslices), ...)) has landed.  Valid until the next fetch / lmmhip_ctx_destroy. */
#define LMMHIP_VAL_KEEP 0x7FF4C0FFEE5107E5ull
int lmmhip_res_values_sliced(lmmhip_ctx* ctx, int64_t n, int nslices, const double** values);
int lmmhip_res_values_wait(lmmhip_ctx* ctx, int slice);
/* Number of lmmhip_res_flatten calls served by the refresh path (same constraint list and precision,
 * no element record / slab change since the last flatten, and no constraint bound crossing the part
 * test (maxmin.cpp:523-525) in a way that changes the member set: only the dense penalties and bounds
 * are rewritten).  Replaces nothing in the reference (its lmm_solve re-reads the lists every time). */
int lmmhip_res_refreshes(lmmhip_ctx* ctx, int64_t* n);
/* Of those, the calls that also had part-test crossings since the last flatten (judged on the device by
 * rs_cross_check: the flattened system lists every listed constraint a member lies on, whatever its
 * bound, so a crossing that leaves the member set as it is keeps the structure). */
int lmmhip_res_cross_refreshes(lmmhip_ctx* ctx, int64_t* n);
/* Inspection: download the flattened system the next lmmhip_solve runs on (from lmmhip_upload or
 * lmmhip_res_flatten).  counts3 = {n_var, n_cnst, nnz}; null arrays are skipped (sizes first). */
int lmmhip_flat_download(lmmhip_ctx* ctx, int64_t* counts3, uint32_t* var_ptr, int32_t* csr_c, double* csr_w,
                         uint32_t* cnst_ptr, int32_t* csc_v, double* csc_w, double* penalty, double* var_bound,
                         double* cnst_bound, uint8_t* cnst_flags);

/* Declare the uploaded system a disjoint union of nsys independent systems (a parameter sweep, SURVEY.md
 * §8(a) C3): system i owns the dense variables [var_off[i], var_off[i+1]) and constraints
 * [cnst_off[i], cnst_off[i+1]) (offsets cover the system; checked on the device: no element may link two
 * systems).  A MAXMIN lmmhip_solve then runs one workgroup per system with the system in LDS
 * (lmm_batch_kernels.hpp) when the largest one fits (< 65535 variables / constraints / elements,
 * <= 64 KB of LDS), else the global engines.  nsys = 0 clears; every upload clears. */
int lmmhip_set_batch(lmmhip_ctx* ctx, int64_t nsys, const int64_t* var_off, const int64_t* cnst_off);

/* Solve on the device; values stay resident in HBM until lmmhip_get_values(). */
int lmmhip_solve(lmmhip_ctx* ctx, int kind, double precision);

/* Copy the solved values (n_var doubles, CSR variable order) to host memory. */
int lmmhip_get_values(lmmhip_ctx* ctx, double* values_out);
/* Per variable of the last max-min solve (dense order, as lmmhip_get_values): 1 + the device round that fixed or
 * dropped it (0: never; measurement — the dependency-depth comparison of scripts/depth.py). */
int lmmhip_get_var_rounds(lmmhip_ctx* ctx, int32_t* rounds_out);
/* Saturated set of the last solve, one byte per constraint of the solved system (dense order):
 *   MAXMIN: sat(c) = NOT double_positive(bound - U_c, bound * precision), U_c = Constraint::get_usage()
 *           (maxmin.cpp:948-961) from the solved values — the saturated_constraint_set the reference
 *           leaves behind (maxmin.cpp:397-409), recomputed the way SURVEY.md A.6 compares it;
 *   FAIR_BOTTLENECK: c was erased (remaining <= 0, fair_bottleneck.cpp:129-140). */
int lmmhip_get_saturated(lmmhip_ctx* ctx, uint8_t* saturated_out);
/* Variables the last flatten put in the system — the Lazy models' modified_set_ side effect of the
 * solve (every variable of an active element of a listed constraint, maxmin.cpp:536-538) — in the
 * caller's id space: dense CSR indices after lmmhip_upload, host variable slots after
 * lmmhip_res_flatten (ascending).  *n = count; ids == NULL = size query; cap must be >= *n. */
int lmmhip_get_touched_vars(lmmhip_ctx* ctx, int32_t* ids, int64_t cap, int64_t* n);
/* Connected components of the uploaded (or resident-flattened) system's variable-constraint graph — the
 * closure System::update_modified_set walks from one constraint (maxmin.cpp:898-922), for every component at
 * once (components spread over GPUs).  Lock-free union-find on the device; component ids
 * are compact, 0..*ncomp-1, in the order of each component's smallest node (variables first, then
 * constraints, dense order): var_label[n_var], cnst_label[n_cnst] (a constraint without an element is a
 * component of its own).  Deterministic whatever the scheduling. */
int lmmhip_components(lmmhip_ctx* ctx, int32_t* var_label, int32_t* cnst_label, int64_t* ncomp);
/* Device pointer of the values (for device-resident consumers, e.g. model update kernels). */
int lmmhip_values_device_ptr(lmmhip_ctx* ctx, const double** dptr);

int lmmhip_get_stats(lmmhip_ctx* ctx, lmmhip_stats* out);
/* 1 = bracket every launch with HIP events (no host synchronisation) and accumulate per-phase
 * times into lmmhip_stats.kernel_ms; per-launch records via lmmhip_launch_profile(). */
int lmmhip_set_profiling(lmmhip_ctx* ctx, int on);
/* Per-launch records of the last profiled solve: phase slot (0/1 init, 2/3/4 round phases),
 * round index (-1 = init), duration in ms.  Returns the number of records (fills up to cap). */
int lmmhip_launch_profile(lmmhip_ctx* ctx, int* slot, int* round, float* ms, int cap);
/* Work profile of the last solve: alive variables / their elements at the start of each round
 * (from the per-variable exit round).  Returns the number of rounds. */
int lmmhip_round_profile(lmmhip_ctx* ctx, int64_t* alive_vars, int64_t* alive_elems, int cap);
/* Per round of the last profiled maxmin solve: variables re-evaluated by the vote phase and their
 * elements.  Returns the number of rounds. */
int lmmhip_vote_profile(lmmhip_ctx* ctx, int64_t* reeval_vars, int64_t* reeval_elems, int cap);
/* Vote diagnostics of the last profiled maxmin solve run with LMMHIP_VOTE_DIAG set, 8 per round: rows whose
 * target's key changed, sensitive rows (skey 0), rows queued for a re-vote, constraints flagged changed,
 * distinct targets of the queued rows, the sum of those targets' CSC degrees, queued sensitive rows, 0. */
int lmmhip_vote_diag_profile(lmmhip_ctx* ctx, int64_t* out8, int cap);

/* Launch on `hip_stream` (a hipStream_t, e.g. a torch.cuda.Stream's cuda_stream) instead of the
 * context's own stream.  Lets a caller order its collectives and the solver's kernels on one stream
 * without host synchronisation.  Every handle means that stream: 0 is the legacy null stream (torch's
 * default stream), ordered with the caller's work on it.  lmmhip_ctx_use_own_stream returns to the
 * context's own non-blocking stream (the state after lmmhip_ctx_create). */
int lmmhip_ctx_set_stream(lmmhip_ctx* ctx, void* hip_stream);
int lmmhip_ctx_use_own_stream(lmmhip_ctx* ctx);

/* Max-min engine (the round loop of maxmin.cpp:560-680):
 *   LMMHIP_ENGINE_PERSISTENT — ONE cooperative launch per solve: the rounds' phases separated by grid
 *     barriers, termination decided on the device, no host round-trip;
 *   LMMHIP_ENGINE_ROUNDS — one launch per phase per round, the host polling termination every few
 *     rounds (also the engine of the profiling mode, which times every phase launch);
 *   LMMHIP_ENGINE_AUTO (default) — persistent up to 2^14 variables, frontier (below) up to 2^18, rounds
 *     above.
 * All give bit-identical results.  The environment variable LMMHIP_ENGINE=rounds|persistent|frontier overrides
 * the context's engine ("auto" or any other value leaves it).  In profiling mode (lmmhip_set_profiling) every
 * phase launch is timed, so a persistent choice runs the ROUNDS engine instead; FRONTIER is kept. */
#define LMMHIP_ENGINE_PERSISTENT 0
#define LMMHIP_ENGINE_ROUNDS 1
#define LMMHIP_ENGINE_AUTO 2
/*   LMMHIP_ENGINE_FRONTIER — one launch per phase per round like ROUNDS, but each round only touches what
 *     changed: votes are registered at their target constraint, so the update pass queues exactly the votes
 *     a touched constraint may have invalidated (no pass over the alive rows; lmm_frontier_kernels.hpp). */
#define LMMHIP_ENGINE_FRONTIER 3
int lmmhip_ctx_set_engine(lmmhip_ctx* ctx, int engine);
/* Persistent solves of this context that were re-run by the multi-launch engine because the persistent grid
 * could not become co-resident: its launch rendezvous closed after LMMHIP_PERSIST_RDV_MS (default 20 ms) with
 * part of the grid held back (another kernel, library or process occupying CUs), or a later grid-barrier wait
 * timed out.  After a closed rendezvous a context on its own stream moves to a new stream, so the re-run starts
 * at once on the free CUs; the next LMMHIP_PERSIST_COOLDOWN (64) solves of the context use the multi-launch
 * engine directly.  Persistent launches of one process are serialised per device, so two Systems never starve
 * each other. */
int lmmhip_engine_fallbacks(lmmhip_ctx* ctx, int64_t* n);
/* Round anatomy (diagnostic builds only: make EXTRA_HIPFLAGS=-DLMM_ANAT=1; scripts/anatomy.py): in the solves run
 * with LMMHIP_ANAT_ROUNDS="r0,r1,..." (at most 4 rounds) every wave of the round engine's vote, saturation and update
 * launches of those rounds writes a record of 20 words — entry and exit on the 100-MHz wall clock, its workgroup,
 * and the clock ticks it spent at each dependent level of its work (lmm_dev.hpp, lmm_anat).  *n = the words of the
 * record array ([slot 0..3][kernel vote / saturation / update / big-constraint saturation][wave 0..8191][20]); out
 * (cap words) gets them,
 * rounds4 the recorded rounds.  LMMHIP_E_STATE in the product build. */
int lmmhip_anatomy(lmmhip_ctx* ctx, unsigned long long* out, int64_t cap, int64_t* n, int32_t* rounds4);
/* Measurement of the persistent engine: on = record, for every grid barrier of the next solves, the
 * wall-clock time (100 MHz) of the last workgroup's arrival and of workgroup 0's exit.  With t != NULL,
 * copies the last solve's records: t[2i] = last arrival at barrier i, t[2i+1] = exit (barrier 0 = the
 * launch); *n = barriers recorded (fills up to cap / 2). */
int lmmhip_persist_profile(lmmhip_ctx* ctx, int on, int64_t* t, int64_t cap, int64_t* n);
/* Per-workgroup records of the same profiled solve, for the first *nbar barriers: t[2 (g * nblk + b)] =
 * arrival of workgroup b at barrier g, t[... + 1] = its exit. */
int lmmhip_persist_profile_blocks(lmmhip_ctx* ctx, int64_t* t, int64_t cap, int64_t* nbar, int64_t* nblk);

/* FairBottleneck sharded over ranks (simgrid_amd/multi.py FbShardPlan), bit-identical to
 * the one-context solve and to the reference.  Each shard (one context) holds
 *   - a block of the variables: lmmhip_upload2 of their rows with EVERY constraint (global constraint ids);
 *   - a block of OWNED constraints (lmmhip_fb_shard_owner): each one's full element list in the reference's
 *     enabled_element_set_ order (fair_bottleneck.cpp:111-116), as (position of the element's variable in the
 *     gathered mu vector, weight); cpos[k] = position of constraint k's remaining in the gathered remaining
 *     vector; n_mu / n_rem = lengths of those two vectors.
 * A round (fair_bottleneck.cpp:59-145) is four phases; between them the caller exchanges, on the context's
 * stream:
 *   step(0) -> xnb[0..n_cnst) listed variables of this shard per constraint, xnb[n_cnst] = some variable of
 *              this shard still listed;                                     all-reduce SUM xnb
 *   step(1) -> shares, this shard's mu into xmu[mu_off .. mu_off + n_var);  all-gather xmu
 *   step(2) -> the owned constraints' remaining (the reference's per-element double_update chain over the
 *              gathered mu) into xrem[cpos[k]];                             all-gather xrem
 *   step(3) -> remaining of every listed constraint from xrem, erasure, delisting of this shard's variables
 * xnb (int32[n_cnst+1]), xmu (double[n_mu]), xrem (double[n_rem]) are device buffers owned by the caller.
 * The solve is over when poll() reports done (the same round on every shard: decided from xnb). */
int lmmhip_fb_shard_owner(lmmhip_ctx* ctx, int64_t n_own, const int32_t* own_cnst, const int64_t* optr,
                          const int32_t* ovar, const double* oweight, const int32_t* cpos, int64_t n_mu,
                          int64_t n_rem);
int lmmhip_fb_shard_begin(lmmhip_ctx* ctx, double precision, int32_t* xnb, double* xmu, int64_t mu_off,
                          double* xrem);
int lmmhip_fb_shard_step(lmmhip_ctx* ctx, int phase);
/* After phase 1 of a round (multi-process delta exchange of mu): the (position in xmu, mu) pairs of this
 * shard's variables listed at the round's start — the only mu values that moved (every variable in round 0).
 * pos / mu / count are DEVICE buffers on the context's stream (pos and mu hold up to n_var entries; *count must
 * be zeroed before; it receives the number of pairs).  The other ranks scatter the pairs into their xmu. */
int lmmhip_fb_shard_pack_mu(lmmhip_ctx* ctx, int32_t* pos, double* mu, int32_t* count);
int lmmhip_fb_shard_poll(lmmhip_ctx* ctx, int* done, int64_t* rounds); /* synchronises the stream */
/* Work of the last FairBottleneck solve (one context, or this shard's part), summed over its rounds — the
 * per-round sweeps of fair_bottleneck.cpp:59-144 that SURVEY.md §8(d) prices at 36 B per element + 32 B per
 * variable + 32 B per constraint: out3 = {elements of the listed constraints (this context's CSC), listed
 * variables, listed constraints}. */
int lmmhip_fb_work(lmmhip_ctx* ctx, int64_t* out3);

/* Model-side step glue on the device, over the values of the context's last solve:
 * the actions' remains / max duration / latency stay in HBM between steps.
 *   var_index[i]        dense index (CSR order of lmmhip_upload) of action i's variable, -1 = not solved
 *   penalty[i]          the variable's current penalty (finish test: remains <= 0 && penalty > 0)
 *   sharing_penalty[i]  CM02: the penalty restored when the latency is paid (network_cm02.cpp:145)
 *   flags[i]            bit0 = the variable has no constraint, bit1 = suspended
 * lmmhip_next_event_full: Model::next_occuring_event_full (Model.cpp:103-129), with_latency adds the
 *   network / ptask latency term (network_interface.cpp:57-70, ptask_L07.cpp:69-82); -1 = no event.
 * lmmhip_update_actions_full: update_actions_state_full of model LMMHIP_MODEL_CPU (cpu_interface.cpp:37-51),
 *   _CM02 (network_cm02.cpp:128-163) or _L07 (ptask_L07.cpp:84-118); events[i] gets
 *   LMMHIP_EV_FINISHED / LMMHIP_EV_LATENCY_PAID (the host then finishes the action / updates the
 *   variable's penalty, and for L07 its bound); *n_events = actions with an event. */
#define LMMHIP_MODEL_CPU 0
#define LMMHIP_MODEL_CM02 1
#define LMMHIP_MODEL_L07 2
#define LMMHIP_EV_FINISHED 1
#define LMMHIP_EV_LATENCY_PAID 2
int lmmhip_actions_upload(lmmhip_ctx* ctx, int64_t n, const int32_t* var_index, const double* remains,
                          const double* max_duration, const double* latency, const double* penalty,
                          const double* sharing_penalty, const uint8_t* flags);
int lmmhip_next_event_full(lmmhip_ctx* ctx, int with_latency, double* out);
int lmmhip_update_actions_full(lmmhip_ctx* ctx, int model, double delta, double maxmin_precision,
                               double surf_precision, int64_t* n_events);
int lmmhip_actions_download(lmmhip_ctx* ctx, double* remains, double* max_duration, double* latency, double* penalty,
                            uint8_t* events);

/* LAZY update models (the default for CPU and network, sg_config.cpp:252): the
 * ActionHeap (Action.cpp:209-241) becomes per-action (date, type) arrays in HBM whose top is a grid
 * min-reduction — no heap maintenance on the host.
 * lmmhip_actions_lazy_upload (after lmmhip_actions_upload): Action::last_update_ / last_value_ /
 *   start_time_, and each action's heap entry (date, heap_type LMMHIP_HEAP_*; UNSET = not in the heap,
 *   e.g. NetworkCm02Model::communicate's latency event, network_cm02.cpp:215-225, is LATENCY).
 *   flags bit2 (LMMHIP_ACT_NOT_STARTED) = not in the started set.
 * lmmhip_actions_lazy_update: the loop of Model::next_occuring_event_lazy (Model.cpp:46-94) over the
 *   modified actions of the last lmm_solve (action indices, each once): update_remains_lazy of the
 *   CPU (cpu_interface.cpp:141-157) or CM02 (network_cm02.cpp:426-449) action, completion date, heap
 *   update; *n_finished = actions update_remains_lazy finished (events[i] = LMMHIP_EV_FINISHED).
 * lmmhip_next_event_lazy: heap top date - now, or -1 when the heap is empty (Model.cpp:97-100).
 * lmmhip_actions_lazy_due: update_actions_state_lazy (cpu_interface.cpp:25-35, network_cm02.cpp:103-126):
 *   pops every entry while double_equals(top_date, now, surf_precision); returns the popped actions in
 *   ascending index order with their event (CM02 latency hat: LMMHIP_EV_LATENCY_PAID, the host restores
 *   the penalty; otherwise LMMHIP_EV_FINISHED).  The reference pops by (date, Action*): same set.
 * lmmhip_actions_lazy_download: inspection of the lazy state. */
#define LMMHIP_HEAP_UNSET 0
#define LMMHIP_HEAP_LATENCY 1
#define LMMHIP_HEAP_MAX_DURATION 2
#define LMMHIP_HEAP_NORMAL 3
#define LMMHIP_ACT_NOT_STARTED 4
int lmmhip_actions_lazy_upload(lmmhip_ctx* ctx, const double* last_update, const double* last_value,
                               const double* start_time, const double* date, const uint8_t* heap_type);
int lmmhip_actions_lazy_update(lmmhip_ctx* ctx, int model, double now, double maxmin_precision, double surf_precision,
                               int64_t n_modified, const int32_t* modified, int64_t* n_finished);
int lmmhip_next_event_lazy(lmmhip_ctx* ctx, double now, double* out);
int lmmhip_actions_lazy_due(lmmhip_ctx* ctx, int model, double now, double surf_precision, int32_t* ids,
                            uint8_t* events, int64_t cap, int64_t* n_due);
int lmmhip_actions_lazy_download(lmmhip_ctx* ctx, double* last_update, double* last_value, double* date,
                                 uint8_t* heap_type);

/* Number of visible HIP devices (0 when none; never initialises a context). */
int lmmhip_device_count(void);

const char* lmmhip_last_error(void);

/* Build provenance: the first 16 hex digits of a SHA-256 over the sources this library was compiled from
 * (simgrid_amd/csrc, include/lmm; simgrid_amd/build_id.py defines the hash, csrc/Makefile compiles it in).
 * smoke() compares it with the hash of the tree it runs from. */
const char* lmmhip_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* LMM_HIP_H */
