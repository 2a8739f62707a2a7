// lmm_hip.hip — device context + C ABI of include/lmm/lmm_hip.h for the MI355X (gfx950) LMM solver.
//
// Kernels: lmm_maxmin_kernels.hpp (System::lmm_solve, maxmin.cpp:487-693) and lmm_fb_kernels.hpp
// (FairBottleneck::bottleneck_solve, fair_bottleneck.cpp:23-153); layout in lmm_dev.hpp.
// All arithmetic is fp64; device code is compiled with -ffp-contract=off so every a*b+c rounds like the
// reference (the FairBottleneck `value == bound` test is exact).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <chrono>
#include <cstring>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lmm/lmm_hip.h"
#include "lmm_dev.hpp"
#include "lmm_fb_kernels.hpp"
#include "lmm_step_kernels.hpp"
#include "lmm_maxmin_kernels.hpp"
#include "lmm_persist_kernels.hpp"
#include "lmm_frontier_kernels.hpp"
#include "lmm_batch_kernels.hpp"
#include "lmm_resident_kernels.hpp"
#include "lmm_cc_kernels.hpp"
#include "lmm_scan.hpp"

using namespace lmmdev;

constexpr unsigned kPersistProfCap = 1 << 16;  // barriers covered by lmmhip_persist_profile
constexpr int64_t kAutoPersistVars = 1 << 18;   // LMMHIP_ENGINE_AUTO: one of the single-GPU small-system engines up to
constexpr int64_t kAutoPersistMaxVars = 1 << 14;  // this many variables: persistent up to 2^14, frontier above

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess)                                                                               \
      return fail(LMMHIP_E_HIP, std::string(#expr " -> ") + hipGetErrorString(e_) + " @" + __FILE__ + \
                                    ":" + std::to_string(__LINE__));                                    \
  } while (0)

}  // namespace

// =============================================================================================
// context + C ABI
// =============================================================================================
// Device buffers of one flattened system: allocated by alloc_flat, filled by the host upload
// (lmmhip_upload) or on the device by the resident flatten (lmmhip_res_flatten).
struct FlatBufs {
  uint32_t *vp, *cp, *chb;
  int32_t *csr_c, *csc_v, *cvar0, *chc, *cch;
  double *csr_w, *csc_w, *pen, *vb, *cb;
  uint8_t* cf;
};

struct lmmhip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;      // the stream every launch and copy goes to
  hipStream_t own_stream = nullptr;  // the context's own stream (back to it: lmmhip_ctx_use_own_stream)
  Dev d{};
  std::vector<void*> allocs;  // owned device allocations
  int32_t* h_ctl = nullptr;   // pinned mirror of the control words (+ 2 slots: pipelined polls of solve_maxmin;
                              // + 1: the words the device writes itself, Dev::hprog)
  hipEvent_t ev_poll[2] = {nullptr, nullptr};  // completion of the pipelined control-word copies
  std::vector<hipEvent_t> ev_slice;  // lmmhip_res_values_sliced: completion of each slice's copy
  bool uploaded = false;
  bool profiling = false;
  int group = 8;  // lanes per row in mm_vote (power of two >= mean row length, <= 64)
  int n_cu = 256;  // compute units (grid of the one-block-per-CU kernels)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // per-launch event pairs (profiling mode): recorded without synchronising, resolved after the
  // solve, so the timed launch sequence is not serialised by the measurement.
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  std::vector<int> launch_slot, launch_round;
  std::vector<float> launch_ms;
  lmmhip_stats stats{};
  int last_kind = LMMHIP_KIND_MAXMIN;
  double last_prec = 1e-5;  // precision of the last solve (lmmhip_get_saturated)
  bool solved = false;      // a solve completed since the last upload / flatten
  int32_t* vstat = nullptr;  // profiling counters of mm_vote ([round][block] x 2)
  unsigned long long* anat = nullptr;  // round anatomy records (LMM_ANAT builds, LMMHIP_ANAT_ROUNDS)
  // maxmin engine (lmmhip_ctx_set_engine): one persistent launch per solve (default) or the
  // multi-launch round chain; grid-barrier words of the persistent launch
  int engine = LMMHIP_ENGINE_AUTO;
  int sat_waves = 1;  // waves per ready constraint in mm_saturate (mean 64-element CSC chunks, 1/2/4)
  bool vote_diag = std::getenv("LMMHIP_VOTE_DIAG") != nullptr;  // profiling: diagnostic vote launches
  bool vote_bits = true;  // short-row vote: changed-constraint bitmap in LDS (LMMHIP_VOTE_BITS=0: the stamps' path)
  int64_t vote_bits_rows = 0;  // ... only while the alive rows (host view) are at least this many
  unsigned* pbar = nullptr;
  bool persist_prof = false;    // record barrier timestamps in the persistent launch
  long long* ptime = nullptr;   // [2 * kPersistProfCap] last arrival / exit per barrier
  int persist_grid = 0;  // workgroups of the persistent launch (one per CU, checked at first use)
  int64_t persist_fallbacks = 0;  // persistent solves re-run by the multi-launch engine (barrier timeout)
  // co-residency fallback (lmm_persist_kernels.hpp bar_rdv): mapped host word the closed-and-drained launch
  // rendezvous raises, the streams left behind holding such a launch (its late workgroups still to run), and the
  // solves left before the persistent engine is tried again on this context
  int32_t* h_rdv = nullptr;
  int32_t* d_rdv = nullptr;
  std::vector<hipStream_t> retired_streams;
  int64_t persist_cool = 0;
  bool ev1_done = false;  // the solve recorded ev1 itself (right behind its last kernel)
  // block-diagonal batch (lmmhip_set_batch): system offsets on the device, largest system
  int64_t bt_n = 0;
  int64_t* bt_voff = nullptr;
  int64_t* bt_coff = nullptr;
  int32_t* bt_rounds = nullptr;  // [grid] rounds of each workgroup's systems
  int bt_max_nv = 0, bt_max_nc = 0, bt_max_nnz = 0;
  int64_t bt_cap = 0;
  // fair bottleneck round state (lmmhip_solve and the sharded lmmhip_fb_shard_* protocol)
  int64_t fb_round = 0;
  // rounds the previous solve of this context had to queue before its termination test could fire (round engine:
  // LASTR + 1, mm_done at the end of the chunk; frontier: ROUNDS + 1, the vote after the last update): a hint for
  // where to end a chunk and wait for it (round_hint_chunk); 0 = none
  int64_t hint_rounds_mm = 0, hint_rounds_fr = 0;
  uint32_t fb_longmin = 0;  // solve_fair: shared constraints with >= this many elements use fbk_acc's increments
  int fb_nlb = 128;          // solve_fair: fbk_update_seq workgroups for the long chains
  double fb_prec = 0;
  bool fb_shard = false;
  FbOwner fbo{};                   // sharded solve: the owned constraints (lmmhip_fb_shard_owner)
  bool fbo_ready = false;
  int64_t fbo_nmu = 0;  // length of the gathered mu vector the owned elements index
  std::vector<void*> fbo_allocs;
  ActDev act{};                        // model-side action state (lmm_step_kernels.hpp)
  std::vector<void*> act_allocs;
  int32_t* xnb_own = nullptr;  // the context's own exchange buffers (unsharded solves)
  double* xmin_own = nullptr;
  int64_t fbd_cap = 0;  // elements of d.fbd (allocated by the first one-context FairBottleneck solve)
  // resident System mirror (lmmhip_res_*, lmm_resident_kernels.hpp): outlives uploads, freed with the
  // context.  Mirror arrays keep their contents when they grow; scratch buffers do not.
  struct Scr {
    void* p = nullptr;
    size_t bytes = 0;
  };
  ResDev res{};
  int64_t res_capE = 0, res_capV = 0, res_capC = 0;
  int64_t res_nE = 0, res_nV = 0, res_nC = 0;  // host table sizes of the last delta batch
  bool res_flat = false;                        // the uploaded system came from lmmhip_res_flatten
  FlatBufs fb_last{};
  int tune_upd = 0, tune_sat = 0;
  double* pin_vals = nullptr;  // pinned host staging of lmmhip_res_values_pinned
  uint8_t* pin_rst = nullptr;  // (lmmhip_res_values_pinned only: the sliced fetch marks kept slots in the values)
  int64_t pin_cap = 0, pin_rst_cap = 0;  // capacities of pin_vals / pin_rst (elements)
  int64_t fcap[4] = {0, 0, 0, 0};               // capacities of the flat-system buffers (nV, nC, nnz, nch)
  int64_t res_flat_nv = 0;                      // variable slots covered by that flatten
  // refresh path of lmmhip_res_flatten: the last flatten's list and precision, host-side structural
  // flag (element records shipped since), device flags of rs_apply_v / rs_apply_c (kResStruct / kResPenalty)
  // res_dirty: [0] flags, [1] fair error, [2] "mixed" member (rs_mark), [3] part-test crossings since the
  // last flatten, [4 ..) their constraint ids (kResCrossCap, rs_apply_c)
  std::vector<int32_t> res_last_list;
  double res_last_prec = -1.0;
  bool res_struct_host = true;
  int32_t* res_dirty = nullptr;
  int64_t res_refreshes = 0, res_cross_refreshes = 0;
  // refresh path: the variables the delta batches touched since the last flatten (-1: too many), and whether rs_c2c
  // (CSR -> CSC position map, written by the device flatten's transpose) matches the uploaded structure
  Scr rs_vlist, rs_c2c;
  int64_t res_vl_n = 0;
  bool res_pen_dirty = false;  // lmmhip_update_vars wrote penalties behind the mirror's back: recompute csc_u / csc_p
  bool res_c2c_ok = false;
  int res_flat_kind = LMMHIP_KIND_MAXMIN;  // solver the last resident flatten built for
  Scr sat_out, tv_out;  // lmmhip_get_saturated / lmmhip_get_touched_vars staging
  Scr cc_par, cc_flag, cc_rank, cc_out;  // lmmhip_components
  Scr fb_longl;                                   // solve_fair: the long shared constraints (fb_long_list)
  Scr fbp_k0, fbp_k1, fbp_v0, fbp_v1, fbp_tmp, fbp_perm, fbp_cscvp, fbp_mu;  // solve_fair: locality order (fb_perm)
  bool fb_perm_ok = false;                        // the order matches the uploaded system
  // frontier engine (lmm_frontier_kernels.hpp): CSR -> CSC map of the uploaded structure, vote slots, floors,
  // re-vote queue; the map and the largest CSC degree are rebuilt after every structural change
  Scr fr_c2s, fr_slot, fr_minfl, fr_qa, fr_qb, fr_qn, fr_md, fr_pvb, fr_key;
  Scr mm_crec[3];  // solve_maxmin: packed row records (LMMHIP_CREC)
  Scr mm_rdq[2], mm_rqst, mm_useg, mm_ucnt;  // solve_maxmin: ready queue / update segments (LMMHIP_RDQ)
  bool fr_map_ok = false;
  int fr_maxdeg = 0;
  Scr rs_stage[12], rs_pos, rs_list, rs_lpart, rs_lany, rs_dcl, rs_cdeg, rs_cptr, rs_vrst, rs_vm, rs_dv, rs_rl,
      rs_ro, rs_rowid, rs_kidx, rs_skey, rs_sval, rs_vout, rs_tmp, rs_lzero, rs_nck, rs_cch, rs_rowpen, rs_posd, rs_cls, rs_lanyc,
      rs_outc;
};

// Persistent launches are serialised per device, process-wide (solve_maxmin_persist_once): the completion event
// of each device's last persistent launch, and the number of live contexts on the device (the event is destroyed
// with the last one, so a device reset between two sets of contexts never leaves a stale event behind).
namespace {
std::mutex g_persist_mu;
std::map<int, hipEvent_t> g_persist_last;  // device -> completion event of its last persistent launch
std::map<int, int> g_persist_users;        // device -> live contexts
}  // namespace

static void persist_ctx_ref(int device, int delta) {
  std::lock_guard<std::mutex> lk(g_persist_mu);
  int& n = g_persist_users[device];
  n += delta;
  if (n <= 0) {
    g_persist_users.erase(device);
    auto it = g_persist_last.find(device);
    if (it != g_persist_last.end()) {
      if (it->second)
        (void)hipEventDestroy(it->second);
      g_persist_last.erase(it);
    }
  }
}

static void free_owner(lmmhip_ctx* c) {
  for (void* p : c->fbo_allocs)
    (void)hipFree(p);
  c->fbo_allocs.clear();
  c->fbo = FbOwner{};
  c->fbo_ready = false;
}

static void free_all(lmmhip_ctx* c) {
  for (void* p : c->allocs)
    (void)hipFree(p);
  c->allocs.clear();
  free_owner(c);
  c->d = Dev{};
  c->uploaded = false;
  c->xnb_own = nullptr;
  c->xmin_own = nullptr;
  c->fbd_cap = 0;
  c->fb_shard = false;
  c->res_flat = false;
}

template <class T> static int dalloc(lmmhip_ctx* c, T** out, int64_t n) {
  void* p = nullptr;
  size_t bytes = size_t(n > 0 ? n : 1) * sizeof(T);
  HIPCHK(hipMalloc(&p, bytes));
  c->allocs.push_back(p);
  *out = static_cast<T*>(p);
  return 0;
}

extern "C" {

const char* lmmhip_last_error(void) { return g_err.c_str(); }

int lmmhip_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_err = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    return 0;
  }
  return n;
}

int lmmhip_ctx_create(int device, lmmhip_ctx** out) {
  if (!out)
    return fail(LMMHIP_E_ARG, "null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(LMMHIP_E_NODEVICE, "no HIP device visible (the MI355X path has no CPU fallback)");
  auto* c = new lmmhip_ctx;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess)
      device = 0;
  }
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess)
    e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  c->stream = c->own_stream;
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&c->h_ctl, 4 * CTL_WORDS * sizeof(int32_t), hipHostMallocDefault);
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&c->h_rdv, 64, hipHostMallocMapped);
  if (e == hipSuccess)
    e = hipHostGetDevicePointer((void**)&c->d_rdv, c->h_rdv, 0);
  if (e == hipSuccess)
    e = hipEventCreateWithFlags(&c->ev_poll[0], hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipEventCreateWithFlags(&c->ev_poll[1], hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipEventCreate(&c->ev0);
  if (e == hipSuccess)
    e = hipEventCreate(&c->ev1);
  if (e != hipSuccess) {
    delete c;
    return fail(LMMHIP_E_HIP, std::string("context creation: ") + hipGetErrorString(e));
  }
  persist_ctx_ref(device, +1);
  *out = c;
  return 0;
}

int lmmhip_ctx_destroy(lmmhip_ctx* c) {
  if (!c)
    return 0;
  (void)hipSetDevice(c->device);
  if (c->stream)
    (void)hipStreamSynchronize(c->stream);
  if (c->own_stream && c->own_stream != c->stream)
    (void)hipStreamSynchronize(c->own_stream);
  for (hipStream_t st : c->retired_streams) {  // a persistent launch whose rendezvous closed: its late workgroups
    (void)hipStreamSynchronize(st);           // still read the barrier words
    (void)hipStreamDestroy(st);
  }
  if (c->h_rdv)
    (void)hipHostFree(c->h_rdv);
  persist_ctx_ref(c->device, -1);
  free_all(c);
  for (void* p : {(void*)c->res.e_cnst, (void*)c->res.e_w, (void*)c->res.e_fl, (void*)c->res.v_ebase,
                  (void*)c->res.v_n, (void*)c->res.v_pen, (void*)c->res.v_bound, (void*)c->res.c_bound,
                  (void*)c->res.c_fl})
    if (p)
      (void)hipFree(p);
  for (lmmhip_ctx::Scr* b : {&c->sat_out, &c->tv_out, &c->fb_longl, &c->fbp_k0, &c->fbp_k1, &c->fbp_v0, &c->fbp_v1, &c->fbp_tmp, &c->fbp_perm, &c->fbp_cscvp, &c->fbp_mu, &c->fr_c2s, &c->fr_slot, &c->fr_minfl, &c->fr_qa, &c->fr_qb, &c->fr_qn, &c->fr_md, &c->fr_pvb, &c->fr_key, &c->mm_crec[0], &c->mm_crec[1], &c->mm_crec[2], &c->mm_rdq[0], &c->mm_rdq[1], &c->mm_rqst, &c->mm_useg, &c->mm_ucnt, &c->cc_par, &c->cc_flag, &c->cc_rank, &c->cc_out, &c->rs_pos, &c->rs_list, &c->rs_lpart, &c->rs_lany, &c->rs_dcl, &c->rs_cdeg,
                             &c->rs_cptr, &c->rs_vrst, &c->rs_vm, &c->rs_dv, &c->rs_rl, &c->rs_ro, &c->rs_rowid,
                             &c->rs_kidx, &c->rs_skey, &c->rs_sval, &c->rs_vout, &c->rs_tmp, &c->rs_lzero,
                             &c->rs_nck, &c->rs_cch, &c->rs_rowpen, &c->rs_posd, &c->rs_cls, &c->rs_lanyc, &c->rs_outc, &c->rs_vlist, &c->rs_c2c})
    if (b->p)
      (void)hipFree(b->p);
  for (lmmhip_ctx::Scr& b : c->rs_stage)
    if (b.p)
      (void)hipFree(b.p);
  for (void* p : c->act_allocs)
    (void)hipFree(p);
  if (c->res_dirty)
    (void)hipFree(c->res_dirty);
  if (c->pin_vals)
    (void)hipHostFree(c->pin_vals);
  if (c->pin_rst)
    (void)hipHostFree(c->pin_rst);
  if (c->h_ctl)
    (void)hipHostFree(c->h_ctl);
  for (hipEvent_t ev : c->ev_poll)
    if (ev)
      (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->ev_slice)
    (void)hipEventDestroy(ev);
  if (c->vstat)
    (void)hipFree(c->vstat);
  if (c->anat)
    (void)hipFree(c->anat);
  if (c->pbar)
    (void)hipFree(c->pbar);
  for (void* p : {(void*)c->bt_voff, (void*)c->bt_coff, (void*)c->bt_rounds})
    if (p)
      (void)hipFree(p);
  if (c->ptime)
    (void)hipFree(c->ptime);
  if (c->ev0)
    (void)hipEventDestroy(c->ev0);
  if (c->ev1)
    (void)hipEventDestroy(c->ev1);
  for (hipEvent_t ev : c->pool)
    (void)hipEventDestroy(ev);
  if (c->own_stream)
    (void)hipStreamDestroy(c->own_stream);
  delete c;
  return 0;
}

static int alloc_flat_exact(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, int64_t nch, FlatBufs* o) {
  free_all(c);
  Dev& d = c->d;
  d.nV = int32_t(nV);
  d.nC = int32_t(nC);
  d.nnz = nnz;
  uint32_t *vp, *cp, *crow1, *crow2;
  int32_t *csr_c, *csc_v, *cvar0, *cvar1, *cvar2, *ccol1, *ccol2;
  double *csr_w, *csc_w, *pen, *vb, *cb;
  uint8_t* cf;
  const int64_t nblk = (nV + kCompactRows - 1) / kCompactRows + 1;
  int rc = 0;
  rc |= dalloc(c, &vp, nV + 1);
  rc |= dalloc(c, &csr_c, nnz);
  rc |= dalloc(c, &csr_w, nnz);
  rc |= dalloc(c, &cp, nC + 1);
  rc |= dalloc(c, &csc_v, nnz);
  rc |= dalloc(c, &csc_w, nnz);
  rc |= dalloc(c, &d.csc_u, nnz);
  rc |= dalloc(c, &d.csc_p, nnz);
  rc |= dalloc(c, &d.csc_row, nnz);
  rc |= dalloc(c, &pen, nV);
  rc |= dalloc(c, &vb, nV);
  rc |= dalloc(c, &cb, nC);
  rc |= dalloc(c, &cf, nC);
  rc |= dalloc(c, &d.x, nV);
  rc |= dalloc(c, &d.fixr, nV);
  rc |= dalloc(c, &d.vtmp, nV);
  rc |= dalloc(c, &d.vst, int64_t(nV) + 32);  // (+32: read 32 flags at a time by fb_pack_vst)
  rc |= dalloc(c, &d.vstb, (int64_t(nV) + 31) / 32 + 1);
  rc |= dalloc(c, &d.ratio, nC);
  rc |= dalloc(c, &d.key, nC);
  rc |= dalloc(c, &d.rem, nC);
  rc |= dalloc(c, &d.use, nC);
  rc |= dalloc(c, &d.cst, nC);
  rc |= dalloc(c, &d.cexp, nC);
  rc |= dalloc(c, &d.nvote, nC);
  rc |= dalloc(c, &cvar0, nV);
  rc |= dalloc(c, &cvar1, nV);
  rc |= dalloc(c, &cvar2, nV);
  rc |= dalloc(c, &crow1, nV + 1);
  rc |= dalloc(c, &crow2, nV + 1);
  rc |= dalloc(c, &ccol1, nnz);
  rc |= dalloc(c, &ccol2, nnz);
  rc |= dalloc(c, &d.vstate, nV);
  for (int b = 0; b < 3; b++) {
    rc |= dalloc(c, &d.rtgt[b], nV);
    rc |= dalloc(c, &d.skey[b], nV);
  }
  rc |= dalloc(c, &d.chg, nC);
  rc |= dalloc(c, &d.chgbits, (nC + 127) / 128 * 2 + 2);
  rc |= dalloc(c, &d.flagbits, (nC + 127) / 128 * 2 + 2);
  rc |= dalloc(c, &d.ready, nC + kMaxBlocks);
  rc |= dalloc(c, &d.bready, kMaxBlocks);
  rc |= dalloc(c, &d.ctouch, nC);
  rc |= dalloc(c, &d.cdup, nC);
  rc |= dalloc(c, &d.balive, kMaxBlocks);
  rc |= dalloc(c, &d.clist[0], nC);
  rc |= dalloc(c, &d.clist[1], nC);
  rc |= dalloc(c, &d.bsum, 2 * nblk);
  rc |= dalloc(c, &d.ctl, CTL_ALLOC);
  int32_t *chc, *cch;
  uint32_t* chb;
  rc |= dalloc(c, &chc, nch);
  rc |= dalloc(c, &chb, nch);
  rc |= dalloc(c, &cch, nC + 1);
  rc |= dalloc(c, &d.pcnt, nch);
  rc |= dalloc(c, &d.pacc, nch);
  rc |= dalloc(c, &d.erased, nC);
  rc |= dalloc(c, &c->xnb_own, nC + 1);
  rc |= dalloc(c, &c->xmin_own, nC);
  if (rc) {
    free_all(c);
    return LMMHIP_E_HIP;
  }
  d.nch = int32_t(nch);
  d.ch_cnst = chc;
  d.ch_beg = chb;
  d.c_ch = cch;
  d.xnb = c->xnb_own;
  d.xmin = c->xmin_own;
  d.var_ptr = vp;
  d.csr_c = csr_c;
  d.csr_w = csr_w;
  d.cnst_ptr = cp;
  d.csc_v = csc_v;
  d.csc_w = csc_w;
  d.pen = pen;
  d.vbound = vb;
  d.cbound = cb;
  d.cflags = cf;
  d.cvar[0] = cvar0;
  d.crow[0] = vp;
  d.ccol[0] = csr_c;
  d.cvar[1] = cvar1;
  d.crow[1] = crow1;
  d.ccol[1] = ccol1;
  d.cvar[2] = cvar2;
  d.crow[2] = crow2;
  d.ccol[2] = ccol2;
  *o = FlatBufs{vp, cp, chb, csr_c, csc_v, cvar0, chc, cch, csr_w, csc_w, pen, vb, cb, cf};
  return 0;
}

// Buffers for a system of this shape, reusing the current ones when they are large enough (a
// simulation re-solves systems of similar size every step: no hipMalloc / hipFree on that path);
// otherwise reallocated with 25 % headroom over the previous capacity.
static int alloc_flat(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, int64_t nch, FlatBufs* o) {
  const bool have = !c->allocs.empty();
  const bool fits = have && nV <= c->fcap[0] && nC <= c->fcap[1] && nnz <= c->fcap[2] && nch <= c->fcap[3];
  if (!fits) {
    int64_t a[4] = {nV, nC, nnz, nch};
    // headroom: a simulation's next system is usually a little larger (flows arriving, a link's bound
    // leaving 0); growing the flat buffers costs ~10 ms of frees and allocations at C2's size
    for (int i = 0; i < 4; i++)
      a[i] = have ? std::max(a[i], c->fcap[i] + c->fcap[i] / 4) : a[i] + a[i] / 16;
    if (a[2] > INT32_MAX)
      a[2] = std::max(nnz, int64_t(INT32_MAX));
    if (int rc = alloc_flat_exact(c, a[0], a[1], a[2], a[3], &c->fb_last))
      return rc;
    for (int i = 0; i < 4; i++)
      c->fcap[i] = a[i];
  } else {
    c->uploaded = false;
    c->res_flat = false;
    c->fb_shard = false;
    free_owner(c);  // owned constraints refer to the previous system
  }
  c->d.nV = int32_t(nV);
  c->d.nC = int32_t(nC);
  c->d.nnz = nnz;
  c->d.nch = int32_t(nch);
  *o = c->fb_last;
  return 0;
}

// Solver launch parameters from the system's shape + per-element usage; the system is then solvable.
static int finish_flat(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, bool elem_done = false) {
  Dev& d = c->d;
  c->fb_perm_ok = false;
  c->fr_map_ok = false;
  c->res_c2c_ok = false;  // (a resident flatten sets it again once finish_flat returns)
  const double mean = nV > 0 ? double(nnz) / double(nV) : 1.0;
  c->group = mean <= 4 ? 4 : mean <= 8 ? 8 : mean <= 16 ? 16 : mean <= 32 ? 32 : 64;
  const double cmean = nC > 0 ? double(nnz) / double(nC) : 1.0;  // mean constraint degree
  c->sat_waves = cmean <= 64 ? 1 : cmean <= 160 ? 2 : 4;
  if (nC > 0)  // constraints with a duplicate (variable, constraint) pair (structure only)
    HIPCHK(hipMemsetAsync(d.cdup, 0, size_t(nC), c->stream));
  if (nnz > 0) {  // per-element usage w / penalty, kept in step with pen (lmmhip_update_vars)
    if (!elem_done) {
      hipLaunchKernelGGL(mm_elem_usage, dim3(grid_for(nnz, kBlock)), dim3(kBlock), 0, c->stream, d, 1);
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(mm_dup_check, dim3(grid_for(nV, kBlock)), dim3(kBlock), 0, c->stream, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  c->uploaded = true;
  c->solved = false;
  c->bt_n = 0;  // a new system: no batch declared
  c->stats = lmmhip_stats{};
  c->stats.n_var = nV;
  c->stats.n_cnst = nC;
  c->stats.nnz = nnz;
  return 0;
}

int lmmhip_upload(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, const int64_t* var_ptr,
                  const int32_t* cnst_idx, const double* weight, const double* penalty, const double* var_bound,
                  const double* cnst_bound, const uint8_t* cnst_flags) {
  return lmmhip_upload2(c, nV, nC, nnz, var_ptr, cnst_idx, weight, penalty, var_bound, cnst_bound, cnst_flags,
                        nullptr);
}

int lmmhip_upload2(lmmhip_ctx* c, int64_t nV, int64_t nC, int64_t nnz, const int64_t* var_ptr,
                   const int32_t* cnst_idx, const double* weight, const double* penalty, const double* var_bound,
                   const double* cnst_bound, const uint8_t* cnst_flags, const int64_t* csc_order) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (nV < 0 || nC < 0 || nnz < 0 || nV >= (1 << 30) || nC >= (1 << 30) || nnz > INT32_MAX)
    return fail(LMMHIP_E_ARG, "sizes out of range");
  if (nV > 0 && (!var_ptr || !penalty || !var_bound))
    return fail(LMMHIP_E_ARG, "null variable arrays");
  if (nC > 0 && (!cnst_bound || !cnst_flags))
    return fail(LMMHIP_E_ARG, "null constraint arrays");
  if (nnz > 0 && (!cnst_idx || !weight))
    return fail(LMMHIP_E_ARG, "null element arrays");
  if (nV > 0 && (var_ptr[0] != 0 || var_ptr[nV] != nnz))
    return fail(LMMHIP_E_ARG, "var_ptr must start at 0 and end at nnz");
  // host-side validation + 32-bit offsets + CSC (constraint-major) mirror by a stable counting sort
  std::vector<uint32_t> vp32(static_cast<size_t>(nV) + 1, 0);
  for (int64_t v = 0; v < nV; v++) {
    if (var_ptr[v + 1] < var_ptr[v])
      return fail(LMMHIP_E_ARG, "var_ptr not monotone");
    vp32[size_t(v) + 1] = uint32_t(var_ptr[v + 1]);
  }
  std::vector<uint32_t> cptr(static_cast<size_t>(nC) + 1, 0);
  for (int64_t j = 0; j < nnz; j++) {
    int32_t k = cnst_idx[j];
    if (k < 0 || k >= nC)
      return fail(LMMHIP_E_ARG, "cnst_idx out of range");
    if (!(weight[j] > 0))
      return fail(LMMHIP_E_ARG, "element weights must be > 0 (only active elements are flattened)");
    cptr[size_t(k) + 1]++;
  }
  for (int64_t v = 0; v < nV; v++)
    if (!(penalty[v] > 0))
      return fail(LMMHIP_E_ARG, "penalties must be > 0 (only enabled variables are flattened)");
  for (int64_t k = 0; k < nC; k++)
    cptr[size_t(k) + 1] += cptr[size_t(k)];
  std::vector<int32_t> cv(static_cast<size_t>(nnz));
  std::vector<double> cw(static_cast<size_t>(nnz));
  if (!csc_order) {
    std::vector<uint32_t> cur(cptr.begin(), cptr.end() - 1);
    for (int64_t v = 0; v < nV; v++)
      for (int64_t j = var_ptr[v]; j < var_ptr[v + 1]; j++) {
        uint32_t pos = cur[size_t(cnst_idx[j])]++;
        cv[pos] = int32_t(v);
        cw[pos] = weight[j];
      }
  } else {  // the caller's order within each constraint: a permutation of its CSR elements
    std::vector<int32_t> row(static_cast<size_t>(nnz));
    for (int64_t v = 0; v < nV; v++)
      for (int64_t j = var_ptr[v]; j < var_ptr[v + 1]; j++)
        row[size_t(j)] = int32_t(v);
    std::vector<uint8_t> seen(static_cast<size_t>(nnz), 0);
    int64_t k = 0;
    for (int64_t pos = 0; pos < nnz; pos++) {
      while (k < nC && cptr[size_t(k) + 1] <= uint32_t(pos))
        k++;
      const int64_t j = csc_order[pos];
      if (j < 0 || j >= nnz || seen[size_t(j)] || cnst_idx[j] != k)
        return fail(LMMHIP_E_ARG, "csc_order is not a constraint-major permutation of the CSR elements");
      seen[size_t(j)] = 1;
      cv[size_t(pos)] = row[size_t(j)];
      cw[size_t(pos)] = weight[j];
    }
  }
  // fair bottleneck CSC chunks (lmm_fb_kernels.hpp)
  std::vector<int32_t> c_ch(static_cast<size_t>(nC) + 1, 0), ch_cnst;
  std::vector<uint32_t> ch_beg;
  for (int64_t k = 0; k < nC; k++) {
    c_ch[size_t(k)] = int32_t(ch_cnst.size());
    for (uint32_t b = cptr[size_t(k)]; b < cptr[size_t(k) + 1]; b += kFbChunk) {
      ch_cnst.push_back(int32_t(k));
      ch_beg.push_back(b);
    }
  }
  const int64_t nch = int64_t(ch_cnst.size());
  c_ch[size_t(nC)] = int32_t(nch);
  std::vector<int32_t> iota(static_cast<size_t>(nV));
  for (int64_t v = 0; v < nV; v++)
    iota[size_t(v)] = int32_t(v);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  FlatBufs fb;
  if (int rc = alloc_flat(c, nV, nC, nnz, nch, &fb))
    return rc;
  uint32_t *vp = fb.vp, *cp = fb.cp, *chb = fb.chb;
  int32_t *csr_c = fb.csr_c, *csc_v = fb.csc_v, *cvar0 = fb.cvar0, *chc = fb.chc, *cch = fb.cch;
  double *csr_w = fb.csr_w, *csc_w = fb.csc_w, *pen = fb.pen, *vb = fb.vb, *cb = fb.cb;
  uint8_t* cf = fb.cf;
  HIPCHK(hipMemcpyAsync(vp, vp32.data(), sizeof(uint32_t) * (nV + 1), hipMemcpyHostToDevice, c->stream));
  if (nnz > 0) {
    HIPCHK(hipMemcpyAsync(csr_c, cnst_idx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csr_w, weight, sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csc_v, cv.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(csc_w, cw.data(), sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipMemcpyAsync(cp, cptr.data(), sizeof(uint32_t) * (nC + 1), hipMemcpyHostToDevice, c->stream));
  if (nV > 0) {
    HIPCHK(hipMemcpyAsync(pen, penalty, sizeof(double) * nV, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(vb, var_bound, sizeof(double) * nV, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(cvar0, iota.data(), sizeof(int32_t) * nV, hipMemcpyHostToDevice, c->stream));
  }
  if (nC > 0) {
    HIPCHK(hipMemcpyAsync(cb, cnst_bound, sizeof(double) * nC, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(cf, cnst_flags, sizeof(uint8_t) * nC, hipMemcpyHostToDevice, c->stream));
  }
  if (nch > 0) {
    HIPCHK(hipMemcpyAsync(chc, ch_cnst.data(), sizeof(int32_t) * nch, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(chb, ch_beg.data(), sizeof(uint32_t) * nch, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipMemcpyAsync(cch, c_ch.data(), sizeof(int32_t) * (nC + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));  // host staging vectors die at return
  return finish_flat(c, nV, nC, nnz);
}

int lmmhip_update_vars(lmmhip_ctx* c, const double* penalty, const double* var_bound) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  HIPCHK(hipSetDevice(c->device));
  if (penalty && c->d.nV)
    HIPCHK(hipMemcpyAsync((void*)c->d.pen, penalty, sizeof(double) * c->d.nV, hipMemcpyHostToDevice, c->stream));
  if (penalty && c->d.nnz) {
    hipLaunchKernelGGL(mm_elem_usage, dim3(grid_for(c->d.nnz, kBlock)), dim3(kBlock), 0, c->stream, c->d, 0);
    HIPCHK(hipGetLastError());
  }
  if (var_bound && c->d.nV)
    HIPCHK(
        hipMemcpyAsync((void*)c->d.vbound, var_bound, sizeof(double) * c->d.nV, hipMemcpyHostToDevice, c->stream));
  // the dense penalties / bounds (and csc_u / csc_p) no longer match the resident records for variables the delta
  // list does not name: the next resident refresh must rewrite every member
  if (penalty || var_bound)
    c->res_vl_n = -1;
  if (penalty)
    c->res_pen_dirty = true;
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_update_cnsts(lmmhip_ctx* c, const double* cnst_bound) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  HIPCHK(hipSetDevice(c->device));
  if (cnst_bound && c->d.nC)
    HIPCHK(
        hipMemcpyAsync((void*)c->d.cbound, cnst_bound, sizeof(double) * c->d.nC, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// resident System mirror + delta log (lmm_resident_kernels.hpp)
// ---------------------------------------------------------------------------------------------
template <class T> static int scratch(lmmhip_ctx* c, lmmhip_ctx::Scr& b, int64_t n, T** out) {
  const size_t need = size_t(n > 0 ? n : 1) * sizeof(T);
  if (b.bytes < need) {
    HIPCHK(hipStreamSynchronize(c->stream));  // the old buffer may still be read by queued work
    if (b.p)
      HIPCHK(hipFree(b.p));
    const size_t bytes = b.bytes ? std::max(need, b.bytes + b.bytes / 2) : need + need / 16;  // (alloc_flat)
    b.p = nullptr;
    b.bytes = 0;
    HIPCHK(hipMalloc(&b.p, bytes));
    b.bytes = bytes;
  }
  *out = static_cast<T*>(b.p);
  return 0;
}

// Grow a mirror array to `cap` elements, keeping the first `used` ones.
template <class T> static int res_grow(lmmhip_ctx* c, T** p, int64_t used, int64_t cap) {
  T* q = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&q), size_t(cap > 0 ? cap : 1) * sizeof(T)));
  HIPCHK(hipMemsetAsync(q, 0, size_t(cap > 0 ? cap : 1) * sizeof(T), c->stream));
  if (*p && used > 0)
    HIPCHK(hipMemcpyAsync(q, *p, size_t(used) * sizeof(T), hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (*p)
    HIPCHK(hipFree(*p));
  *p = q;
  return 0;
}

// Integer knob from the environment (A/B switches, documented where read).
static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// Flags and crossing list of the delta batches (lmmhip_ctx::res_dirty), zeroed on first use.
// Chunk length under a round-count hint: a chunk that would cross the hinted end E is cut to end at it, and the
// caller waits for that chunk before queueing more (*stop), so a solve as long as the previous one runs no returning
// rounds after its last one; a longer one pays one host round trip there, a shorter one is caught by the usual polls.
// Consecutive solves of a simulation change little, so their round counts do too.  LMMHIP_ROUND_HINT=0: off.
static int round_hint_chunk(int64_t r, int chunk, int64_t hint, bool* stop) {
  *stop = false;
  if (hint > r && r + chunk >= hint) {
    *stop = true;
    return int(hint - r);
  }
  return chunk;
}

static int res_dirty_alloc(lmmhip_ctx* c) {
  if (c->res_dirty)
    return 0;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->res_dirty), (4 + kResCrossCap) * sizeof(int32_t)));
  HIPCHK(hipMemsetAsync(c->res_dirty, 0, 4 * sizeof(int32_t), c->stream));
  return 0;
}

template <class T> static int stage(lmmhip_ctx* c, int slot, const T* host, int64_t n, const T** out) {
  T* d = nullptr;
  if (int rc = scratch(c, c->rs_stage[slot], n, &d))
    return rc;
  if (n > 0)
    HIPCHK(hipMemcpyAsync(d, host, size_t(n) * sizeof(T), hipMemcpyHostToDevice, c->stream));
  *out = d;
  return 0;
}

static int dev_scan(lmmhip_ctx* c, const int64_t* in, int64_t* out, int64_t n) {
  size_t tb = 0;
  HIPCHK(scan_i64(nullptr, tb, in, out, n, c->stream));
  uint8_t* t = nullptr;
  if (int rc = scratch(c, c->rs_tmp, int64_t(tb), &t))
    return rc;
  HIPCHK(scan_i64(t, tb, in, out, n, c->stream));
  return 0;
}

static int64_t read_i64(lmmhip_ctx* c, const int64_t* dptr, int* rc) {
  int64_t h = 0;
  if (hipMemcpyAsync(&h, dptr, sizeof(h), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    *rc = fail(LMMHIP_E_HIP, "resident flatten: reading a count back failed");
  return h;
}

#define RS_LAUNCH(kern, n, ...)                                                                     \
  do {                                                                                              \
    hipLaunchKernelGGL(kern, dim3(grid_for((n) + 1, kBlock)), dim3(kBlock), 0, c->stream, __VA_ARGS__); \
    HIPCHK(hipGetLastError());                                                                      \
  } while (0)

extern "C" {

int lmmhip_res_apply(lmmhip_ctx* c, int64_t n_elem_total, int64_t n_var_total, int64_t n_cnst_total, int64_t ne,
                     const int64_t* e_id, const int32_t* e_cnst, const double* e_weight, const uint8_t* e_flags,
                     int64_t nv, const int32_t* v_id, const int64_t* v_ebase, const int32_t* v_nelem,
                     const double* v_penalty, const double* v_bound, int64_t nc, const int32_t* c_id,
                     const double* c_bound, const uint8_t* c_flags) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (n_elem_total < 0 || n_var_total < 0 || n_cnst_total < 0 || ne < 0 || nv < 0 || nc < 0 ||
      n_var_total >= (1 << 30) || n_cnst_total >= (1 << 30) || n_elem_total > INT32_MAX)
    return fail(LMMHIP_E_ARG, "resident sizes out of range");
  if ((ne && (!e_id || !e_cnst || !e_weight || !e_flags)) ||
      (nv && (!v_id || !v_ebase || !v_nelem || !v_penalty || !v_bound)) || (nc && (!c_id || !c_bound || !c_flags)))
    return fail(LMMHIP_E_ARG, "null delta arrays");
  // host-side validation: every record lands inside the tables, every slab inside the element table
  for (int64_t i = 0; i < ne; i++)
    if (e_id[i] < 0 || e_id[i] >= n_elem_total || e_cnst[i] < -1 || e_cnst[i] >= n_cnst_total)
      return fail(LMMHIP_E_ARG, "element delta out of range");
  for (int64_t i = 0; i < nv; i++)
    if (v_id[i] < 0 || v_id[i] >= n_var_total || v_nelem[i] < -1 || v_ebase[i] < 0 ||
        v_ebase[i] + std::max(v_nelem[i], 0) > n_elem_total)
      return fail(LMMHIP_E_ARG, "variable delta out of range");
  for (int64_t i = 0; i < nc; i++)
    if (c_id[i] < 0 || c_id[i] >= n_cnst_total)
      return fail(LMMHIP_E_ARG, "constraint delta out of range");
  HIPCHK(hipSetDevice(c->device));
  ResDev& r = c->res;
  if (n_elem_total > c->res_capE) {
    const int64_t cap = std::max(n_elem_total, c->res_capE + c->res_capE / 2);
    int rc = res_grow(c, &r.e_cnst, c->res_nE, cap) | res_grow(c, &r.e_w, c->res_nE, cap) |
             res_grow(c, &r.e_fl, c->res_nE, cap);
    if (rc)
      return rc;
    c->res_capE = cap;
  }
  if (n_var_total > c->res_capV) {
    const int64_t cap = std::max(n_var_total, c->res_capV + c->res_capV / 2);
    int rc = res_grow(c, &r.v_ebase, c->res_nV, cap) | res_grow(c, &r.v_n, c->res_nV, cap) |
             res_grow(c, &r.v_pen, c->res_nV, cap) | res_grow(c, &r.v_bound, c->res_nV, cap);
    if (rc)
      return rc;
    c->res_capV = cap;
  }
  if (n_cnst_total > c->res_capC) {
    const int64_t cap = std::max(n_cnst_total, c->res_capC + c->res_capC / 2);
    int rc = res_grow(c, &r.c_bound, c->res_nC, cap) | res_grow(c, &r.c_fl, c->res_nC, cap);
    if (rc)
      return rc;
    c->res_capC = cap;
  }
  if (int rc = res_dirty_alloc(c))
    return rc;
  if (ne || n_var_total > c->res_nV || n_cnst_total > c->res_nC)
    c->res_struct_host = true;
  c->res_nE = std::max(c->res_nE, n_elem_total);
  c->res_nV = std::max(c->res_nV, n_var_total);
  c->res_nC = std::max(c->res_nC, n_cnst_total);
  if (ne) {
    const int64_t* did;
    const int32_t* dcn;
    const double* dw;
    const uint8_t* dfl;
    int rc = stage(c, 0, e_id, ne, &did) | stage(c, 1, e_cnst, ne, &dcn) | stage(c, 2, e_weight, ne, &dw) |
             stage(c, 3, e_flags, ne, &dfl);
    if (rc)
      return rc;
    RS_LAUNCH(rs_apply_e, ne, ne, did, dcn, dw, dfl, r);
  }
  if (nv) {
    const int32_t* did;
    const int64_t* deb;
    const int32_t* dn;
    const double *dp, *db;
    int rc = stage(c, 4, v_id, nv, &did) | stage(c, 5, v_ebase, nv, &deb) | stage(c, 6, v_nelem, nv, &dn) |
             stage(c, 7, v_penalty, nv, &dp) | stage(c, 8, v_bound, nv, &db);
    if (rc)
      return rc;
    RS_LAUNCH(rs_apply_v, nv, nv, did, deb, dn, dp, db, r, c->res_dirty);
    // the touched variables, for the refresh path (up to 1/8 of the slots: beyond that a full pass is as cheap)
    if (c->res_vl_n >= 0 && c->res_vl_n + nv <= std::max<int64_t>(4096, n_var_total / 8)) {
      int32_t* vl = nullptr;
      if (c->rs_vlist.bytes < size_t(c->res_vl_n + nv) * sizeof(int32_t)) {  // grow, keeping the list
        lmmhip_ctx::Scr old = c->rs_vlist;
        c->rs_vlist = lmmhip_ctx::Scr{};
        if (int rc = scratch(c, c->rs_vlist, std::max<int64_t>(4096, 2 * (c->res_vl_n + nv)), &vl))
          return rc;
        if (old.p && c->res_vl_n > 0)
          HIPCHK(hipMemcpyAsync(vl, old.p, size_t(c->res_vl_n) * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (old.p)
          HIPCHK(hipFree(old.p));
      }
      vl = static_cast<int32_t*>(c->rs_vlist.p);
      HIPCHK(hipMemcpyAsync(vl + c->res_vl_n, did, size_t(nv) * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
      c->res_vl_n += nv;
    } else {
      c->res_vl_n = -1;  // too many: the refresh path rewrites every member
    }
  }
  if (nc) {
    const int32_t* did;
    const double* db;
    const uint8_t* dfl;
    int rc = stage(c, 9, c_id, nc, &did) | stage(c, 10, c_bound, nc, &db) | stage(c, 11, c_flags, nc, &dfl);
    if (rc)
      return rc;
    RS_LAUNCH(rs_apply_c, nc, nc, did, db, dfl, r, c->res_last_prec < 0 ? 1e-5 : c->res_last_prec, c->res_dirty,
              c->res_dirty + 3, c->res_dirty + 4);
  }
  HIPCHK(hipStreamSynchronize(c->stream));  // host delta arrays are borrowed for the call only
  return 0;
}

}  // extern "C"

static int res_flatten(lmmhip_ctx* c, bool fair, int64_t n_list, const int32_t* cnst_list, double precision,
                       int64_t* counts3) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (n_list < 0 || (n_list && !cnst_list))
    return fail(LMMHIP_E_ARG, "bad constraint list");
  for (int64_t i = 0; i < n_list; i++)
    if (cnst_list[i] < 0 || cnst_list[i] >= c->res_nC)
      return fail(LMMHIP_E_ARG, "listed constraint is not in the resident mirror");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const ResDev& r = c->res;
  const int64_t nl = n_list, nvs = c->res_nV;
  // Refresh path: same list, same precision, no element record and no slab change since the last
  // flatten, and no constraint-bound crossing of the part test that changes the member set (rs_cross_check)
  // -> the structure (CSR/CSC, dense maps, reset mask) stands; only penalties, variable bounds and
  // constraint bounds / policies are rewritten in dense order.
  if (!fair && c->res_flat && c->res_flat_kind == LMMHIP_KIND_MAXMIN && c->uploaded && !c->res_struct_host &&
      c->res_dirty && precision == c->res_last_prec &&
      nvs == c->res_flat_nv && size_t(nl) == c->res_last_list.size() &&
      (nl == 0 || std::memcmp(c->res_last_list.data(), cnst_list, size_t(nl) * sizeof(int32_t)) == 0)) {
    int32_t fl4[4] = {0, 0, 0, 0};  // flags, (fair error), mixed, crossings
    HIPCHK(hipMemcpyAsync(fl4, c->res_dirty, sizeof(fl4), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    int32_t flags = fl4[0];
    const int32_t nx = fl4[3];
    if (nx < 0 || (nx > 0 && (fl4[2] || nx > kResCrossCap || env_int("LMMHIP_RES_CROSS", 1) == 0)))
      flags |= kResStruct;
    if (!(flags & kResStruct)) {
      Dev& d = c->d;
      const int32_t* list = static_cast<const int32_t*>(c->rs_list.p);
      const int64_t* lany = static_cast<const int64_t*>(c->rs_lany.p);
      const int64_t* dcl = static_cast<const int64_t*>(c->rs_dcl.p);
      RS_LAUNCH(rs_cmeta, nl, nl, list, r, lany, dcl, nullptr, const_cast<double*>(d.cbound),
                const_cast<uint8_t*>(d.cflags));
      if (nx > 0) {  // part-test crossings: structural only if the member set changes
        const int grid = int(std::min<int64_t>(nx, 2048));
        hipLaunchKernelGGL(rs_cross_check, dim3(grid), dim3(kBlock), 0, c->stream, nx, c->res_dirty + 4, r,
                           precision, static_cast<const uint8_t*>(c->rs_cls.p),
                           static_cast<const uint8_t*>(c->rs_outc.p), static_cast<const int32_t*>(c->rs_posd.p),
                           d.cnst_ptr, d.csc_v, d.var_ptr, d.csr_c, d.cbound, c->res_dirty);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&flags, c->res_dirty, sizeof(flags), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
      }
    }
    if (!(flags & kResStruct)) {
      Dev& d = c->d;
      const int64_t* vm = static_cast<const int64_t*>(c->rs_vm.p);
      const int64_t* dv = static_cast<const int64_t*>(c->rs_dv.p);
      if (c->res_vl_n >= 0 && c->res_c2c_ok && env_int("LMMHIP_RES_VLIST", 1)) {  // the touched variables only
        const int64_t n = c->res_vl_n;
        if (n > 0)
          RS_LAUNCH(rs_refresh_vl, n, n, static_cast<const int32_t*>(c->rs_vlist.p), r, vm, dv,
                    const_cast<double*>(d.pen), const_cast<double*>(d.vbound), d.var_ptr,
                    static_cast<const int32_t*>(c->rs_c2c.p), d.csc_w, d.csc_u, d.csc_p, int(flags & kResPenalty));
      } else {
        RS_LAUNCH(rs_refresh_v, nvs, nvs, r, vm, dv, const_cast<double*>(d.pen), const_cast<double*>(d.vbound));
        if (((flags & kResPenalty) || c->res_pen_dirty) && d.nnz > 0)
          RS_LAUNCH(mm_elem_usage, d.nnz, d, 0);
      }
      c->res_vl_n = 0;
      c->res_pen_dirty = false;
      HIPCHK(hipMemsetAsync(c->res_dirty, 0, sizeof(int32_t), c->stream));
      HIPCHK(hipMemsetAsync(c->res_dirty + 3, 0, sizeof(int32_t), c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      c->res_refreshes++;
      c->res_cross_refreshes += nx > 0;
      if (counts3) {
        counts3[0] = d.nV;
        counts3[1] = d.nC;
        counts3[2] = d.nnz;
      }
      return 0;
    }
  }
  int32_t *pos, *list, *posd;
  uint8_t *lpart, *vrst, *lzero, *cls = nullptr, *lanyc = nullptr, *outc = nullptr;
  int64_t *lany, *dcl, *cdeg, *cptr, *vm, *dv, *rl, *ro;
  int rc = scratch(c, c->rs_pos, c->res_nC, &pos) | scratch(c, c->rs_list, nl, &list) |
           scratch(c, c->rs_lzero, nl, &lzero) |
           scratch(c, c->rs_lpart, nl, &lpart) | scratch(c, c->rs_lany, nl + 1, &lany) |
           scratch(c, c->rs_dcl, nl + 1, &dcl) | scratch(c, c->rs_cdeg, nl + 1, &cdeg) |
           scratch(c, c->rs_cptr, nl + 1, &cptr) | scratch(c, c->rs_vrst, nvs, &vrst) |
           scratch(c, c->rs_vm, nvs + 1, &vm) | scratch(c, c->rs_dv, nvs + 1, &dv) |
           scratch(c, c->rs_rl, nvs + 1, &rl) | scratch(c, c->rs_ro, nvs + 1, &ro) |
           scratch(c, c->rs_posd, std::max<int64_t>(c->res_nC, 1), &posd);
  if (!fair)
    rc |= scratch(c, c->rs_cls, c->res_nC, &cls) | scratch(c, c->rs_lanyc, c->res_nC, &lanyc) |
          scratch(c, c->rs_outc, c->res_nC, &outc);
  if (rc)
    return rc;
  if (nl)
    HIPCHK(hipMemcpyAsync(list, cnst_list, size_t(nl) * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  if (c->res_nC)
    HIPCHK(hipMemsetAsync(pos, 0xFF, size_t(c->res_nC) * sizeof(int32_t), c->stream));
  HIPCHK(hipMemsetAsync(cdeg, 0, size_t(nl + 1) * sizeof(int64_t), c->stream));
  if (int rc = res_dirty_alloc(c))
    return rc;
  if (!fair && c->res_nC) {
    HIPCHK(hipMemsetAsync(cls, 0, size_t(c->res_nC), c->stream));
    HIPCHK(hipMemsetAsync(lanyc, 0, size_t(c->res_nC), c->stream));
    HIPCHK(hipMemsetAsync(outc, 0, size_t(c->res_nC), c->stream));
  }
  RS_LAUNCH(rs_pos, nl, nl, list, r, precision, int(fair), pos, lpart, lany, lzero, cls);
  if (fair) {
    HIPCHK(hipMemsetAsync(c->res_dirty + 1, 0, sizeof(int32_t), c->stream));
    RS_LAUNCH(rs_mark_fair, nvs, nvs, r, pos, lany, lzero, vrst, vm, c->res_dirty + 1);
  } else {
    HIPCHK(hipMemsetAsync(c->res_dirty + 2, 0, sizeof(int32_t), c->stream));
    RS_LAUNCH(rs_mark, nvs, nvs, r, cls, lanyc, outc, vrst, vm, rl, c->res_dirty + 2);
    RS_LAUNCH(rs_lany_list, nl, nl, list, lanyc, lany);
  }
  if ((rc = dev_scan(c, lany, dcl, nl + 1)))
    return rc;
  // posd[c] = dense id of constraint c, or -1: one gather per element in rs_rowlen / rs_write instead of the
  // dependent pos -> lany -> dcl chain
  if (c->res_nC)
    HIPCHK(hipMemsetAsync(posd, 0xFF, size_t(c->res_nC) * sizeof(int32_t), c->stream));
  RS_LAUNCH(rs_posd, nl, nl, list, lany, dcl, posd);
  if (fair)
    RS_LAUNCH(rs_rowlen_fair, nvs, nvs, r, pos, lany, dcl, vm, rl, cdeg);
  else  // (max-min: rs_mark counted the rows unless a member has a disabled element; CSC offsets from the sort)
    RS_LAUNCH(rs_rowlen, nvs, nvs, r, posd, vm, rl, c->res_dirty + 2);
  if ((rc = dev_scan(c, vm, dv, nvs + 1)) || (rc = dev_scan(c, rl, ro, nvs + 1)) ||
      (fair && (rc = dev_scan(c, cdeg, cptr, nl + 1))))
    return rc;
  const int64_t nC = read_i64(c, dcl + nl, &rc);
  const int64_t nV = read_i64(c, dv + nvs, &rc);
  const int64_t nnz = read_i64(c, ro + nvs, &rc);
  if (rc)
    return rc;
  if (nnz > INT32_MAX)
    return fail(LMMHIP_E_ARG, "resident flatten: more than 2^31 active elements");
  int64_t nch = 0;
  int64_t *nck = nullptr, *cch = nullptr;
  if (fair) {  // chunk counts before the allocation (lmm_fb_kernels.hpp)
    int32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, c->res_dirty + 1, sizeof(err), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (err)
      return fail(LMMHIP_E_ARG, "FairBottleneck: negative consumption weights are not supported");
    if ((rc = scratch(c, c->rs_nck, nC + 1, &nck) | scratch(c, c->rs_cch, nC + 1, &cch)))
      return rc;
    RS_LAUNCH(rs_nchunks, nC, nC, cdeg, kFbChunk, nck);
    if ((rc = dev_scan(c, nck, cch, nC + 1)))
      return rc;
    nch = read_i64(c, cch + nC, &rc);
    if (rc)
      return rc;
  }
  FlatBufs fb;
  if ((rc = alloc_flat(c, nV, nC, nnz, nch, &fb)))
    return rc;
  c->res_flat = true;
  c->res_flat_kind = fair ? LMMHIP_KIND_FAIR_BOTTLENECK : LMMHIP_KIND_MAXMIN;
  c->res_flat_nv = nvs;
  int32_t *kidx, *skey, *sval;
  WRow* wrow;
  RowPen* rowpen;
  rc = scratch(c, c->rs_rowid, nnz, &wrow) | scratch(c, c->rs_kidx, nnz, &kidx) |
       scratch(c, c->rs_skey, nnz, &skey) | scratch(c, c->rs_sval, nnz, &sval) |
       scratch(c, c->rs_rowpen, std::max<int64_t>(nV, 1), &rowpen);
  if (rc)
    return rc;
  RS_LAUNCH(rs_cmeta, nl, nl, list, r, lany, dcl, fair ? lzero : nullptr, fb.cb, fb.cf);
  RS_LAUNCH(rs_write, nvs, nvs, r, posd, vm, dv, ro, fb.vp, fb.csr_c, fb.csr_w, fb.pen, fb.vb, fb.cvar0,
            wrow, kidx, rowpen);
  const uint32_t nnz32 = uint32_t(nnz);
  HIPCHK(hipMemcpyAsync(fb.vp + nV, &nnz32, sizeof(nnz32), hipMemcpyHostToDevice, c->stream));
  if (fair)
    RS_LAUNCH(rs_ptr32, nC, nC, cptr, fb.cp);
  else if (!nnz)
    HIPCHK(hipMemsetAsync(fb.cp, 0, size_t(nC + 1) * sizeof(uint32_t), c->stream));
  if (fair)
    RS_LAUNCH(rs_chunks, nC, nC, cptr, nck, cch, kFbChunk, fb.cch, fb.chc, fb.chb);
  else
    HIPCHK(hipMemsetAsync(fb.cch, 0, size_t(nC + 1) * sizeof(int32_t), c->stream));  // no FB chunks
  if (nnz) {
    int bits = 1;
    while (bits < 31 && (int64_t(1) << bits) < nC)
      bits++;
    size_t tb = 0;
    HIPCHK(sort_pairs_i32(nullptr, tb, fb.csr_c, skey, kidx, sval, nnz, bits, c->stream));
    uint8_t* t = nullptr;
    if ((rc = scratch(c, c->rs_tmp, int64_t(tb), &t)))
      return rc;
    HIPCHK(sort_pairs_i32(t, tb, fb.csr_c, skey, kidx, sval, nnz, bits, c->stream));
    int32_t* c2c = nullptr;
    if (!fair && (rc = scratch(c, c->rs_c2c, nnz, &c2c)))
      return rc;
    RS_LAUNCH(rs_csc, nnz, nnz, sval, wrow, rowpen, fb.csc_v, fb.csc_w, c->d.csc_u, c->d.csc_p,
              c->d.csc_row, c2c);
    if (!fair)
      RS_LAUNCH(rs_cptr_sorted, nnz, nnz, nC, skey, fb.cp);
  }
  HIPCHK(hipStreamSynchronize(c->stream));  // before the host's list buffer is released
  if ((rc = finish_flat(c, nV, nC, nnz, true)))  // (rs_csc wrote the per-element usage, penalty and row)
    return rc;
  c->res_last_list.assign(cnst_list, cnst_list + nl);
  c->res_last_prec = precision;
  c->res_struct_host = false;
  c->res_c2c_ok = !fair;
  c->res_vl_n = 0;
  c->res_pen_dirty = false;
  if (c->res_dirty) {
    HIPCHK(hipMemsetAsync(c->res_dirty, 0, sizeof(int32_t), c->stream));
    HIPCHK(hipMemsetAsync(c->res_dirty + 3, 0, sizeof(int32_t), c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  if (counts3) {
    counts3[0] = nV;
    counts3[1] = nC;
    counts3[2] = nnz;
  }
  return 0;
}

extern "C" {

int lmmhip_res_flatten(lmmhip_ctx* c, int64_t n_list, const int32_t* cnst_list, double precision, int64_t* counts3) {
  return res_flatten(c, false, n_list, cnst_list, precision, counts3);
}

int lmmhip_res_flatten_fair(lmmhip_ctx* c, int64_t n_list, const int32_t* cnst_list, int64_t* counts3) {
  return res_flatten(c, true, n_list, cnst_list, 0.0, counts3);
}

int lmmhip_res_refreshes(lmmhip_ctx* c, int64_t* n) {
  if (!c || !n)
    return fail(LMMHIP_E_ARG, "null argument");
  *n = c->res_refreshes;
  return 0;
}

int lmmhip_res_cross_refreshes(lmmhip_ctx* c, int64_t* n) {
  if (!c || !n)
    return fail(LMMHIP_E_ARG, "null argument");
  *n = c->res_cross_refreshes;
  return 0;
}

}  // extern "C"

// Pinned host staging of the value fetch, grown with 1/4 headroom (the headroom was computed after the
// capacity had been reset); the reset flags only for lmmhip_res_values_pinned.
static int pin_grow(lmmhip_ctx* c, int64_t n, bool with_rst) {
  if (n > c->pin_cap) {
    const int64_t cap = std::max(n, c->pin_cap + c->pin_cap / 4);
    if (c->pin_vals)
      HIPCHK(hipHostFree(c->pin_vals));
    c->pin_vals = nullptr;
    c->pin_cap = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->pin_vals), size_t(cap) * sizeof(double), hipHostMallocDefault));
    c->pin_cap = cap;
  }
  if (with_rst && n > c->pin_rst_cap) {
    const int64_t cap = std::max(n, c->pin_rst_cap + c->pin_rst_cap / 4);
    if (c->pin_rst)
      HIPCHK(hipHostFree(c->pin_rst));
    c->pin_rst = nullptr;
    c->pin_rst_cap = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->pin_rst), size_t(cap), hipHostMallocDefault));
    c->pin_rst_cap = cap;
  }
  return 0;
}

extern "C" {

int lmmhip_res_values_pinned(lmmhip_ctx* c, int64_t n, const double** values, const uint8_t** reset) {
  if (!c || !c->uploaded || !c->res_flat)
    return fail(LMMHIP_E_STATE, "no resident flatten to read values from");
  if (n != c->res_flat_nv || !values || !reset)
    return fail(LMMHIP_E_ARG, "values: n must be the variable slot count of the last resident flatten");
  HIPCHK(hipSetDevice(c->device));
  if (int rc = pin_grow(c, n, true))
    return rc;
  double* vout = nullptr;
  if (int rc = scratch(c, c->rs_vout, n, &vout))
    return rc;
  if (n) {  // (kernel stores straight into the mapped pinned buffers measured 1.0-1.4 ms slower in bench.py)
    const int64_t* vm = static_cast<const int64_t*>(c->rs_vm.p);
    const int64_t* dv = static_cast<const int64_t*>(c->rs_dv.p);
    RS_LAUNCH(rs_values, n, n, vm, dv, static_cast<const uint8_t*>(c->rs_vrst.p), c->d.x, vout,
              static_cast<uint8_t*>(nullptr));
    HIPCHK(hipMemcpyAsync(c->pin_vals, vout, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->pin_rst, c->rs_vrst.p, size_t(n), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  *values = c->pin_vals;
  *reset = c->pin_rst;
  return 0;
}

int lmmhip_res_values_sliced(lmmhip_ctx* c, int64_t n, int nslices, const double** values) {
  if (!c || !c->uploaded || !c->res_flat)
    return fail(LMMHIP_E_STATE, "no resident flatten to read values from");
  if (n != c->res_flat_nv || !values || nslices < 1 || nslices > 256)
    return fail(LMMHIP_E_ARG, "values: n must be the last resident flatten's slot count, 1 <= nslices <= 256");
  HIPCHK(hipSetDevice(c->device));
  if (int rc = pin_grow(c, n, false))
    return rc;
  while (int(c->ev_slice.size()) < nslices) {
    hipEvent_t ev;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->ev_slice.push_back(ev);
  }
  double* vout = nullptr;
  if (int rc = scratch(c, c->rs_vout, n, &vout))
    return rc;
  if (n) {
    const int64_t* vm = static_cast<const int64_t*>(c->rs_vm.p);
    const int64_t* dv = static_cast<const int64_t*>(c->rs_dv.p);
    RS_LAUNCH(rs_values_mark, n, n, vm, dv, static_cast<const uint8_t*>(c->rs_vrst.p), c->d.x,
              reinterpret_cast<unsigned long long*>(vout));
  }
  const int64_t per = (n + nslices - 1) / nslices;
  for (int i = 0; i < nslices; i++) {
    const int64_t lo = std::min(n, i * per), hi = std::min(n, lo + per);
    if (hi > lo)
      HIPCHK(hipMemcpyAsync(c->pin_vals + lo, vout + lo, size_t(hi - lo) * sizeof(double), hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHK(hipEventRecord(c->ev_slice[size_t(i)], c->stream));
  }
  *values = c->pin_vals;
  return 0;
}

int lmmhip_res_values_wait(lmmhip_ctx* c, int slice) {
  if (!c || slice < 0 || slice >= int(c->ev_slice.size()))
    return fail(LMMHIP_E_ARG, "no such slice");
  HIPCHK(hipEventSynchronize(c->ev_slice[size_t(slice)]));
  return 0;
}

int lmmhip_flat_download(lmmhip_ctx* c, int64_t* counts3, uint32_t* var_ptr, int32_t* csr_c, double* csr_w,
                         uint32_t* cnst_ptr, int32_t* csc_v, double* csc_w, double* penalty, double* var_bound,
                         double* cnst_bound, uint8_t* cnst_flags) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  if (!counts3)
    return fail(LMMHIP_E_ARG, "null counts");
  const Dev& d = c->d;
  counts3[0] = d.nV;
  counts3[1] = d.nC;
  counts3[2] = d.nnz;
  HIPCHK(hipSetDevice(c->device));
  auto get = [&](void* dst, const void* src, size_t bytes) -> int {
    if (dst && bytes)
      HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return 0;
  };
  int rc = get(var_ptr, d.var_ptr, sizeof(uint32_t) * (size_t(d.nV) + 1)) |
           get(csr_c, d.csr_c, sizeof(int32_t) * size_t(d.nnz)) | get(csr_w, d.csr_w, sizeof(double) * size_t(d.nnz)) |
           get(cnst_ptr, d.cnst_ptr, sizeof(uint32_t) * (size_t(d.nC) + 1)) |
           get(csc_v, d.csc_v, sizeof(int32_t) * size_t(d.nnz)) | get(csc_w, d.csc_w, sizeof(double) * size_t(d.nnz)) |
           get(penalty, d.pen, sizeof(double) * size_t(d.nV)) | get(var_bound, d.vbound, sizeof(double) * size_t(d.nV)) |
           get(cnst_bound, d.cbound, sizeof(double) * size_t(d.nC)) | get(cnst_flags, d.cflags, size_t(d.nC));
  if (rc)
    return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_res_values(lmmhip_ctx* c, int64_t n, double* values, uint8_t* reset) {
  if (!c || !c->uploaded || !c->res_flat)
    return fail(LMMHIP_E_STATE, "no resident flatten to read values from");
  if (n != c->res_flat_nv || (n && (!values || !reset)))
    return fail(LMMHIP_E_ARG, "values: n must be the variable slot count of the last resident flatten");
  HIPCHK(hipSetDevice(c->device));
  double* vout = nullptr;
  if (int rc = scratch(c, c->rs_vout, n, &vout))
    return rc;
  const int64_t* vm = static_cast<const int64_t*>(c->rs_vm.p);
  const int64_t* dv = static_cast<const int64_t*>(c->rs_dv.p);
  if (n) {
    RS_LAUNCH(rs_values, n, n, vm, dv, static_cast<const uint8_t*>(c->rs_vrst.p), c->d.x, vout,
              static_cast<uint8_t*>(nullptr));
    HIPCHK(hipMemcpyAsync(values, vout, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(reset, c->rs_vrst.p, size_t(n), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_set_profiling(lmmhip_ctx* c, int on) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  c->profiling = on != 0;
  return 0;
}

static int solve_maxmin(lmmhip_ctx* c, double prec);
static int solve_maxmin_persist(lmmhip_ctx* c, double prec);
static int solve_maxmin_frontier(lmmhip_ctx* c, double prec);
static int solve_fair(lmmhip_ctx* c, double prec);
static int engine_of(const lmmhip_ctx* c);
static bool batch_fits(const lmmhip_ctx* c);
static int solve_maxmin_batch(lmmhip_ctx* c, double prec);
static int resolve_profile(lmmhip_ctx* c);

int lmmhip_solve(lmmhip_ctx* c, int kind, double precision) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "solve before upload");
  if (kind != LMMHIP_KIND_MAXMIN && kind != LMMHIP_KIND_FAIR_BOTTLENECK)
    return fail(LMMHIP_E_ARG, "unknown solver kind");
  if (c->res_flat && kind != c->res_flat_kind)
    return fail(LMMHIP_E_STATE, "the resident flatten was built for the other solver kind");
  HIPCHK(hipSetDevice(c->device));
  for (int i = 0; i < 8; i++) {
    c->stats.kernel_ms[i] = 0;
    c->stats.kernel_launches[i] = 0;
  }
  c->pool_used = 0;
  c->launch_slot.clear();
  c->launch_round.clear();
  c->launch_ms.clear();
  HIPCHK(hipMemsetAsync(c->d.ctl, 0, CTL_ALLOC * sizeof(int32_t), c->stream));
  const size_t stat_bytes = sizeof(int32_t) * 2 * size_t(kStatRounds) * kMaxBlocks;
  if (c->profiling && !c->vstat)
    HIPCHK(hipMalloc(&c->vstat, stat_bytes));
  c->d.vstat = c->profiling ? c->vstat : nullptr;
  if (c->profiling)
    HIPCHK(hipMemsetAsync(c->vstat, 0, stat_bytes, c->stream));
  // round anatomy (diagnostic builds only): the round engine's waves stamp the rounds LMMHIP_ANAT_ROUNDS names
  c->d.anat = nullptr;
  for (int k = 0; k < kAnatSlots; k++)
    c->d.anat_r[k] = -1000;
  if (LMM_ANAT && std::getenv("LMMHIP_ANAT_ROUNDS")) {
    const size_t bytes = sizeof(unsigned long long) * size_t(kAnatSlots) * kAnatKernels * kAnatWaves * kAnatFields;
    if (!c->anat)
      HIPCHK(hipMalloc(&c->anat, bytes));
    HIPCHK(hipMemsetAsync(c->anat, 0, bytes, c->stream));
    const char* e = std::getenv("LMMHIP_ANAT_ROUNDS");
    for (int k = 0; k < kAnatSlots; k++) {
      char* end = nullptr;
      const long v = std::strtol(e, &end, 10);
      if (end == e)
        break;
      c->d.anat_r[k] = int(v);
      if (*end != ',')
        break;
      e = end + 1;
    }
    c->d.anat = c->anat;
  }
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  c->last_kind = kind;
  c->last_prec = precision;
  c->solved = false;
  c->ev1_done = false;
  int rc = kind == LMMHIP_KIND_FAIR_BOTTLENECK ? solve_fair(c, precision)
           : batch_fits(c)                             ? solve_maxmin_batch(c, precision)
           : engine_of(c) == LMMHIP_ENGINE_PERSISTENT ? solve_maxmin_persist(c, precision)
           : engine_of(c) == LMMHIP_ENGINE_FRONTIER   ? solve_maxmin_frontier(c, precision)
                                                     : solve_maxmin(c, precision);
  if (rc)
    return rc;
  if (!c->ev1_done)
    HIPCHK(hipEventRecord(c->ev1, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->stats.device_ms = ms;
  c->solved = true;
  c->stats.rounds = c->h_ctl[CTL_ROUNDS];
  if (kind == LMMHIP_KIND_MAXMIN && c->stats.rounds > 0)  // launched rounds include empty tail rounds
    c->stats.rounds = c->h_ctl[CTL_LASTR] + 1;
  if (c->profiling)
    return resolve_profile(c);
  return 0;
}

// Launch helper.  In profiling mode every launch is bracketed by two events from a pool (no host
// synchronisation); their elapsed times are resolved once the solve has finished.
static int prof_event(lmmhip_ctx* c, hipEvent_t* out) {
  if (c->pool_used == c->pool.size()) {
    hipEvent_t ev;
    HIPCHK(hipEventCreate(&ev));
    c->pool.push_back(ev);
  }
  *out = c->pool[c->pool_used++];
  return 0;
}

#define LAUNCH(slot, round, kern, grid, block, ...)                                 \
  do {                                                                              \
    hipEvent_t e0_ = nullptr, e1_ = nullptr;                                        \
    if (c->profiling) {                                                             \
      if (int rc_ = prof_event(c, &e0_))                                            \
        return rc_;                                                                 \
      HIPCHK(hipEventRecord(e0_, c->stream));                                       \
    }                                                                               \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, c->stream, __VA_ARGS__);  \
    HIPCHK(hipGetLastError());                                                      \
    if (c->profiling) {                                                             \
      if (int rc_ = prof_event(c, &e1_))                                            \
        return rc_;                                                                 \
      HIPCHK(hipEventRecord(e1_, c->stream));                                       \
      c->launch_slot.push_back(slot);                                               \
      c->launch_round.push_back(int(round));                                        \
    }                                                                               \
    c->stats.kernel_launches[slot] += 1;                                            \
  } while (0)

static int resolve_profile(lmmhip_ctx* c) {
  c->launch_ms.assign(c->launch_slot.size(), 0.f);
  for (size_t i = 0; i < c->launch_slot.size(); i++) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->pool[2 * i], c->pool[2 * i + 1]));
    c->launch_ms[i] = ms;
    c->stats.kernel_ms[c->launch_slot[i]] += ms;
  }
  return 0;
}

static int poll_ctl(lmmhip_ctx* c) {
  HIPCHK(hipMemcpyAsync(c->h_ctl, c->d.ctl, CTL_WORDS * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// The alive-row buffer in use is read by the vote on the device (ctl CTL_BUF); nrows (an upper bound of its
// rows, refreshed at every poll) only sizes the grid-stride variants' grids.
static int launch_vote(lmmhip_ctx* c, int64_t r, int64_t nrows) {
  const Dev& d = c->d;
  const int G = c->group;
  const int grid = grid_for(nrows, kBlock);  // one lane per row in the work-queue scan
  switch (G) {
  case 4:
  case 8:  // short rows: one lane per row (more gathers in flight per wave)
    // the LDS bitmap of changed constraints (one 1024-thread workgroup per CU); below LMMHIP_VOTE_BITS_ROWS alive rows
    // (host view, A/B knob; 0 = always) the change stamps gathered per row instead: no ~125-KB copy per CU
    if (int64_t(d.nC) <= int64_t(kBitWords) * 64 && c->vote_bits && nrows >= c->vote_bits_rows) {
      if (c->profiling && c->vote_diag) {  // measurement: bitmap load alone, filter alone (slot 7)
        LAUNCH(7, r + 1000000, (mm_vote_lane<kVBlock, true, 2>), c->n_cu, kVBlock, d, int(r));
        LAUNCH(7, r, (mm_vote_lane<kVBlock, true, 1>), c->n_cu, kVBlock, d, int(r));
        LAUNCH(7, r, mm_vote_diagcount, grid_for((int64_t(d.nC) + 63) / 64, kBlock), kBlock, d, int(r));
      }
      if (d.rdq[0])
        LAUNCH(2, r, (mm_vote_lane<kVBlock, true, 0, true, true>), c->n_cu, kVBlock, d, int(r));
      else if (d.crec[0])
        LAUNCH(2, r, (mm_vote_lane<kVBlock, true, 0, true>), c->n_cu, kVBlock, d, int(r));
      else
        LAUNCH(2, r, (mm_vote_lane<kVBlock, true>), c->n_cu, kVBlock, d, int(r));
    } else if (d.rdq[0]) {
      LAUNCH(2, r, (mm_vote_lane<kBlock, false, 0, true, true>), grid, kBlock, d, int(r));
    } else if (d.crec[0]) {
      LAUNCH(2, r, (mm_vote_lane<kBlock, false, 0, true>), grid, kBlock, d, int(r));
    } else {
      LAUNCH(2, r, (mm_vote_lane<kBlock, false>), grid, kBlock, d, int(r));
    }
    break;
  case 16:
    LAUNCH(2, r, mm_vote<16>, grid, kBlock, d, int(r));
    break;
  case 32:
    LAUNCH(2, r, mm_vote<32>, grid, kBlock, d, int(r));
    break;
  default:
    LAUNCH(2, r, mm_vote<64>, grid, kBlock, d, int(r));
    break;
  }
  return 0;
}

// Slots: 0 mm_init_cnsts, 1 mm_init_vars, 2 mm_vote, 3 mm_ready, 4 mm_saturate, 5 mm_update,
// 6 compaction.
static int solve_maxmin(lmmhip_ctx* c, double prec) {
  Dev& d = c->d;
  struct RowofOff {  // the other engines never see the row map / row records (their compactions do not
    Dev& d;          // maintain them)
    ~RowofOff() {
      d.crec[0] = d.crec[1] = d.crec[2] = nullptr;
      d.rdq[0] = d.rdq[1] = nullptr;
      d.rqst = d.useg = d.ucnt = nullptr;
    }
  } rowof_off{d};
  // packed row records for the re-votes (vote_row: the row's variable and CSR range from one 8-B record and
  // its successor instead of the cvar / crow arrays, one line per re-vote less): C2 25.94-26.00 vs 26.10-26.17
  // ms, stress 28.83 vs 29.13 (same box).  LMMHIP_CREC=0: off.
  d.crec[0] = d.crec[1] = d.crec[2] = nullptr;
  if ((c->group == 4 || c->group == 8) && env_int("LMMHIP_CREC", 1)) {
    for (int k = 0; k < 3; k++) {
      uint2* p = nullptr;
      if (int rc = scratch(c, c->mm_crec[k], int64_t(d.nV) + 1, &p))
        return rc;
      d.crec[k] = p;
    }
  }
  // ready constraints without the mm_ready pass: the update's workgroups (at most kMaxBlocks, each updating
  // at most kUSeg constraints) list them for the next round, the vote queues the ones it makes ready (C2
  // 25.07-25.22 vs 25.34-25.39 ms, stress 28.29 vs 28.46, same box; LMMHIP_RDQ=0: the mm_ready pass)
  d.rdq[0] = d.rdq[1] = nullptr;
  d.rqst = d.useg = d.ucnt = nullptr;
  // (<= kMaxBlocks) Update workgroups: 4 per CU, each with a longer segment, so that the saturation's prefix over
  // the segment counts is shorter — but enough of them to keep every segment within kUSeg (LMMHIP_UPDQ_BLOCKS).
  // Round 5, same box: C2 24.52-24.54 ms against 24.84-24.85 with one per 256 constraints (2,048 at C2), stress
  // 27.86-27.94 vs 28.14; with the saturation cap at 5 per CU below, 24.41-24.45 (stress 27.75-27.77)
  const int64_t gU_need = (int64_t(d.nC) + kUSeg - 1) / kUSeg;
  const int64_t gU_rdq = std::max<int64_t>(1, std::min<int64_t>(grid_for(d.nC, kBlock),
      std::max<int64_t>(gU_need, env_int("LMMHIP_UPDQ_BLOCKS", 4 * c->n_cu))));
  const int64_t per_blk = int64_t(kBlock) * ((int64_t(d.nC) + gU_rdq * kBlock - 1) / (gU_rdq * kBlock));
  if (d.crec[0] && env_int("LMMHIP_RDQ", 1) && per_blk <= kUSeg && env_int("LMMHIP_UPD_BLOCKS", c->tune_upd) == 0) {
    int32_t *q0 = nullptr, *q1 = nullptr, *st = nullptr, *sg = nullptr, *uc = nullptr;
    const int64_t n = std::max<int64_t>(d.nC, 1);
    if (int rc = scratch(c, c->mm_rdq[0], n, &q0) | scratch(c, c->mm_rdq[1], n, &q1) |
                 scratch(c, c->mm_rqst, n, &st) | scratch(c, c->mm_useg, gU_rdq * kUSeg, &sg) |
                 scratch(c, c->mm_ucnt, kMaxBlocks, &uc))
      return rc;
    HIPCHK(hipMemsetAsync(st, 0xFF, size_t(n) * sizeof(int32_t), c->stream));
    HIPCHK(hipMemsetAsync(uc, 0, size_t(kMaxBlocks) * sizeof(int32_t), c->stream));
    d.rdq[0] = q0;
    d.rdq[1] = q1;
    d.rqst = st;
    d.useg = sg;
    d.ucnt = uc;
  }
  c->vote_bits = env_int("LMMHIP_VOTE_BITS", 1) != 0;
  c->vote_bits_rows = env_int("LMMHIP_VOTE_BITS_ROWS", 0);
  const int gC4 = grid_for(d.nC, kBlock / kWave);
  const int gC = grid_for(d.nC, kBlock);
  LAUNCH(0, -1, mm_init_cnsts, gC4, kBlock, d, prec);
  LAUNCH(1, -1, mm_init_vars, grid_for(d.nV, kBlock), kBlock, d);
  LAUNCH(1, -1, mm_clist, std::min(gC, 2 * c->n_cu), kBlock, d, 1);
  HIPCHK(hipMemsetAsync(d.chgbits, 0, sizeof(uint64_t) * ((d.nC + 127) / 128 * 2 + 2), c->stream));
  // Launch-width caps (tuning knobs, environment; 0 = uncapped): fewer blocks cut the fixed per-round
  // cost of the grid-stride round kernels once the alive set is small.
  const int cap_upd = env_int("LMMHIP_UPD_BLOCKS", c->tune_upd);
  // the saturation's grid capped at 4 workgroups per CU (round 5, same box: C2 24.73-24.90 ms against 25.04-25.16
  // uncapped, i.e. up to kMaxBlocks = 2048; 768: 24.79-25.03, 1280: 24.76-24.81, 1536: 24.83-25.00, 512: 25.42-25.73;
  // stress 27.99-28.05 vs 28.29-28.36): every workgroup first rebuilds the prefix of the update's segment counts,
  // and half as many of them still give each ready constraint its waves
  // (with 4 update workgroups per CU: 5 per CU, 24.41-24.45 ms against 24.52-24.54 at 4 and 24.52-24.60 at 6 / 8)
  const int cap_sat = env_int("LMMHIP_SAT_BLOCKS", c->tune_sat > 0 ? c->tune_sat : 5 * c->n_cu);
  auto capped = [](int g, int cap) { return cap > 0 && g > cap ? cap : g; };
  const int gU = capped(gC, cap_upd);  // mm_update: thread per constraint, identity order
  const int gUq = int(gU_rdq);          // (ready-queue mode: at most kUSeg constraints per workgroup)
  // mm_saturate: waves per ready constraint and the grid's block cap (measurement knobs)
  const int sat_k = env_int("LMMHIP_SAT_WAVES", c->sat_waves);
  const int sat_max = env_int("LMMHIP_SAT_GRID_MAX", kMaxBlocks);
  auto sat_grid = [&](int64_t n) { return int(std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, sat_max))); };
  // Compaction cadence (knobs): alive rows are re-counted every cmp_every rounds and rewritten when
  // fewer than cmp_pct % of the scanned rows are alive; the alive-constraint list every cl_every rounds.
  // Both decide and switch buffers on the device (ctl CTL_BUF / CTL_CB): no host round trip.
  // (round 5, re-swept on the final code, same box: every 48 rounds 24.94-25.08 ms against 25.10-25.21 at 32, 25.49-25.56
  // at 16, 25.11-25.21 at 64, 25.30-25.34 at 96; stress 28.29-28.37 vs 28.42-28.44)
  const int cmp_every = env_int("LMMHIP_COMPACT_EVERY", 48);
  const int cmp_pct = env_int("LMMHIP_COMPACT_PCT", 75);
  const int cl_every = env_int("LMMHIP_CLIST_EVERY", 8);
  // Every round fixes at least one variable (progress), so nV + 2 rounds bound it.
  const int64_t max_rounds = int64_t(d.nV) + 2;
  // Host view of the sizes (upper bounds: rows and constraints only leave), refreshed at every poll; they
  // size grids only, the kernels read the exact counts from the control words.
  int64_t r = 0, last_compact = 0, last_clist = 0, nrows = d.nV, ncl = d.nC;
  // Termination polls are pipelined: the control words after chunk k are written into a pinned slot by a
  // one-wave kernel (mm_ctl_out) behind an event, chunk k+1 is queued, then the host waits for chunk k's
  // words — the GPU never idles on the host.  A chunk queued after the last round is a run of launches
  // that return at once (CTL_DONE).
  int chunk = 2, slot = 0;
  // rounds queued per poll: the host learns of termination one chunk late, so up to 2 x chunk_max no-op
  // rounds run after the last one (LMMHIP_CHUNK_MAX, A/B knob): C2 25.96-25.99 ms at 16, 26.01 at 8,
  // 26.15-26.20 at 4; round 5, with compactions every 48 rounds: 25.03-25.06 at 32 against 25.07-25.08 at 16
  const int64_t hint = env_int("LMMHIP_ROUND_HINT", 1) ? c->hint_rounds_mm : 0;  // (round_hint_chunk)
  // under a hint no returning rounds follow the last one, and 64-round chunks (fewer polls, a sparser list / compaction
  // cadence) measured 23.13-23.36 ms against 23.21-23.47 at 32 over five same-box pairs, stress 26.85 vs 26.88
  // (scripts/gpu_r06_v.sh, _w.sh)
  const int chunk_max = std::max(2, env_int("LMMHIP_CHUNK_MAX", hint > 0 ? 64 : 32));
  // Near the end of the solve, short chunks: the rounds queued after the last one are no-op launches of the full
  // grids (~32 of them after C2's last round with 32-round chunks, rocprofv3 trace of round 5), so once the alive rows
  // (host view: refreshed at each compaction) fall to LMMHIP_CHUNK_TAIL_PCT % of the variables (default 5), or below
  // LMMHIP_CHUNK_TAIL_ROWS / the alive-constraint list below LMMHIP_CHUNK_TAIL_CNST (A/B knobs), a chunk is at most
  // LMMHIP_CHUNK_TAIL rounds (default 4).  Round 5, same box, two passes (scripts/gpu_r05_ctail.sh,
  // profiles/r05_ab_c2_ctail.json): C2 23.90-23.95 ms at 5e5 rows (5 %) / 4 rounds against 24.10-24.12 without;
  // 1e6 / 8 and 2e6 / 8 23.92-23.94, 1e6 / 4 23.95-24.07; the constraint-list thresholds (2e4, 1e5) 24.06-24.11.
  const int64_t ctail_rows = env_int("LMMHIP_CHUNK_TAIL_ROWS",
                                     int(int64_t(d.nV) * std::max(0, env_int("LMMHIP_CHUNK_TAIL_PCT", 5)) / 100));
  const int64_t ctail_cnst = env_int("LMMHIP_CHUNK_TAIL_CNST", 0);
  const int ctail = std::max(1, env_int("LMMHIP_CHUNK_TAIL", 4));
  auto round_launches = [&](int64_t r) -> int {
    if (int rc = launch_vote(c, r, nrows))
      return rc;
    if (d.rdq[0]) {  // no mm_ready pass: the update's segments (gUq workgroups) and the vote's queue
      if (sat_k == 1)
        LAUNCH(4, r, mm_saturate_q<1>, capped(sat_grid(ncl), cap_sat), kBlock, d, int(r), gUq);
      else if (sat_k == 2)
        LAUNCH(4, r, mm_saturate_q<2>, capped(sat_grid(2 * ncl), cap_sat), kBlock, d, int(r), gUq);
      else
        LAUNCH(4, r, mm_saturate_q<4>, capped(sat_grid(4 * ncl), cap_sat), kBlock, d, int(r), gUq);
      LAUNCH(5, r, mm_update<true>, gUq, kBlock, d, int(r), prec);
      return 0;
    }
    const int gL = grid_for(ncl, kBlock);
    LAUNCH(3, r, mm_ready, gL, kBlock, d);
    if (sat_k == 1)
      LAUNCH(4, r, mm_saturate<1>, capped(sat_grid(ncl), cap_sat), kBlock, d, int(r), gL);
    else if (sat_k == 2)
      LAUNCH(4, r, mm_saturate<2>, capped(sat_grid(2 * ncl), cap_sat), kBlock, d, int(r), gL);
    else
      LAUNCH(4, r, mm_saturate<4>, capped(sat_grid(4 * ncl), cap_sat), kBlock, d, int(r), gL);
    LAUNCH(5, r, mm_update<false>, gU, kBlock, d, int(r), prec);
    return 0;
  };
  // the alive-constraint list and the alive-row compaction at the end of a chunk (their cadence is the chunks')
  auto chunk_end = [&](int64_t r) -> int {
    const int gL = grid_for(ncl, kBlock);
    bool cl = false, cm = false;
    if (r - last_clist >= cl_every && ncl > 4096) {  // alive-constraint list (order not preserved)
      LAUNCH(6, r, mm_clist, std::min(gL, 2 * c->n_cu), kBlock, d, 0);
      last_clist = r;
      cl = true;
    }
    if (r - last_compact >= cmp_every && nrows > 4096) {  // order-preserving compaction of the alive rows
      const int nblk = int((nrows + kCompactRows - 1) / kCompactRows);
      LAUNCH(6, r, cmp_count, nblk, kBlock, d);
      LAUNCH(6, r, cmp_scan, 1, 1024, d, nblk, cmp_pct);
      LAUNCH(6, r, cmp_write, nblk, kBlock, d);
      last_compact = r;
      cm = true;
    }
    if (cl || cm)
      LAUNCH(6, r, mm_flip, 1, 1, d, int(cl), int(cm));
    return 0;
  };
  bool pending = false;
  int32_t* hc[2] = {c->h_ctl + CTL_WORDS, c->h_ctl + 2 * CTL_WORDS};
  int32_t* hcd[2] = {nullptr, nullptr};  // the same slots as the device sees them (mm_ctl_out)
  for (int k = 0; k < 2; k++)
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hcd[k]), hc[k], 0));
  for (;;) {
    bool stop = false;
    const int n = round_hint_chunk(r, chunk, hint, &stop);
    for (int k = 0; k < n; k++, r++)
      if (int rc = round_launches(r))
        return rc;
    LAUNCH(6, r, mm_done, 1, kBlock, d, d.rdq[0] ? gUq : gU);
    if (int rc = chunk_end(r))
      return rc;
    LAUNCH(6, r, mm_ctl_out, 1, kWave, d, hcd[slot]);
    HIPCHK(hipEventRecord(c->ev_poll[slot], c->stream));
    if (pending) {  // the previous chunk's words (this chunk is queued behind them)
      HIPCHK(hipEventSynchronize(c->ev_poll[slot ^ 1]));
      const int32_t* h = hc[slot ^ 1];
      if (h[CTL_DONE])
        break;
      ncl = h[CTL_NCL0 + h[CTL_CB]];
      nrows = h[CTL_NROWS + h[CTL_BUF]];
    }
    pending = !stop;
    if (stop) {  // the hinted end: this chunk's words before anything more is queued
      HIPCHK(hipEventSynchronize(c->ev_poll[slot]));
      const int32_t* h = hc[slot];
      if (h[CTL_DONE])
        break;
      ncl = h[CTL_NCL0 + h[CTL_CB]];
      nrows = h[CTL_NROWS + h[CTL_BUF]];
    }
    slot ^= 1;
    if (r > max_rounds)
      return fail(LMMHIP_E_NOCONVERGE, "maxmin round guard tripped");
    if (chunk < chunk_max)
      chunk = std::min(2 * chunk, chunk_max);
    // (the short tail chunks stay under a hint too: dropping them measured 23.10 against 23.05-23.08 ms,
    // scripts/gpu_r06_t.sh)
    if ((nrows <= ctail_rows || ncl <= ctail_cnst) && chunk > ctail)
      chunk = ctail;
  }
  if (int rc = poll_ctl(c))  // (the queued tail has run: final words for the stats)
    return rc;
  c->hint_rounds_mm = int64_t(c->h_ctl[CTL_LASTR]) + 1;
  return 0;
}

// Frontier engine (lmm_frontier_kernels.hpp): three launches per round, work proportional to the touched
// constraints and the moving votes.  Slots: 2 fr_vote, 4 fr_sat (+ fr_sat_big), 5 fr_update, 6 the per-chunk
// control-word copy; 0 / 1 init.
static int solve_maxmin_frontier(lmmhip_ctx* c, double prec) {
  Dev d = c->d;  // (a copy: the frontier's buffers stay out of the context's Dev, which the other engines use)
  if (!c->vote_diag)  // per-round diagnostic counters only on request (LMMHIP_VOTE_DIAG): they cost atomics
    d.vstat = nullptr;
  const int64_t nnz = std::max<int64_t>(d.nnz, 1);
  const int nblk = int((int64_t(d.nC) + kFB - 1) / kFB);  // fr_update / fr_vote (/ fr_sat<256>) workgroups
  const int nblkS = int(std::max<int64_t>(1, (int64_t(d.nC) + kFS - 1) / kFS));  // fr_sat workgroups
  int2* cs = nullptr;
  int32_t* md = nullptr;
  int rc = scratch(c, c->fr_c2s, nnz, &cs);
  rc = rc ? rc : scratch(c, c->fr_pvb, std::max<int64_t>(d.nV, 1), &d.pvb);
  rc = rc ? rc : scratch(c, c->fr_slot, nnz, &d.vslot);
  rc = rc ? rc : scratch(c, c->fr_minfl, std::max<int64_t>(d.nC, 1), &d.minfl);
  rc = rc ? rc : scratch(c, c->fr_key, std::max<int64_t>(d.nC, 1), &d.key32);
  rc = rc ? rc : scratch(c, c->fr_qa, nnz, &d.fq_a);
  rc = rc ? rc : scratch(c, c->fr_qb, nnz, &d.fq_b);
  rc = rc ? rc : scratch(c, c->fr_qn, int64_t(nblk) + 1, &d.fq_n);
  rc = rc ? rc : scratch(c, c->fr_md, 1, &md);
  if (rc)
    return rc;
  d.csr_cs = cs;
  if (!c->fr_map_ok) {  // once per uploaded structure
    HIPCHK(hipMemsetAsync(md, 0, sizeof(int32_t), c->stream));
    if (d.nnz > 0) {
      hipLaunchKernelGGL(fr_c2s, dim3(grid_for(d.nC, kBlock / kWave)), dim3(kBlock), 0, c->stream, d, cs, md);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(&c->fr_maxdeg, md, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->fr_map_ok = true;
  }
  // constraints of more CSC chunks than this saturate in fr_sat_big, kFrBigWaves waves each over the whole grid
  // (LMMHIP_FR_BIGCH, A/B knob: fat-tree core links' chunk chains in C4)
  const int bigch = std::max(1, env_int("LMMHIP_FR_BIGCH", kFrBigCh));
  const bool big = c->fr_maxdeg > bigch * kWave;
  const int bigw = std::max(1, env_int("LMMHIP_FR_BIGW", kFrBigWaves));  // waves per big constraint (A/B knob)
  // (round 6, removed after their A/Bs: the re-vote reading the floors with the keys, LMMHIP_FR_MFEARLY, and the round
  // engine's chunk body in fr_sat, LMMHIP_FR_SATOLD — both slower on C2 and C4, scripts/gpu_fr_ab.sh)
  // re-votes keep 16 row elements in registers when the mean row is longer than 8 (LMMHIP_FR_R16=0: 8)
  const bool long_rows = c->group > 8 && env_int("LMMHIP_FR_R16", 1) != 0;
  // fr_vote: segments per workgroup, so that the grid still covers the chip twice (C2: 4, small systems: 1)
  const int spb = int(std::max<int64_t>(1, std::min<int64_t>(kFVS, int64_t(nblk) / (2 * int64_t(c->n_cu)))));
  // fr_sat workgroup: kFS threads (the round-4 choice on C2-size systems) unless that leaves the chip mostly
  // idle — C4 (25 workgroups of kFS): 3.37-3.40 ms with 256-thread workgroups against 3.49
  const int sat_b0 = int64_t(nblkS) >= 2 * int64_t(c->n_cu) ? kFS : 256;
  const int sat_b = env_int("LMMHIP_FR_SATB", sat_b0) == 256 ? 256 : kFS;
  // fr_update: every constraint's state loaded with its key (one dependent level less) on the small systems, where the
  // 256-thread saturation workgroups run (LMMHIP_FR_UPDSPEC, A/B knob)
  const int upd_spec = env_int("LMMHIP_FR_UPDSPEC", sat_b == 256 ? 1 : 0);
  const int gC4 = grid_for(d.nC, kBlock / kWave);
  LAUNCH(0, -1, mm_init_cnsts, gC4, kBlock, d, prec);
  LAUNCH(1, -1, fr_init_vars, grid_for(std::max<int64_t>(std::max<int64_t>(d.nV, d.nC), d.nnz / 4), kBlock), kBlock, d);
  const int64_t max_rounds = int64_t(d.nV) + 2;  // every round fixes a variable (progress)
  const int gbig = std::min(kMaxBlocks, 4 * c->n_cu);
  auto round_launches = [&](int64_t r) -> int {
    if (r == 0) {
      LAUNCH(2, r, fr_vote_all, grid_for(d.nV, kBlock), kBlock, d);
      LAUNCH(2, r, fr_minfl_all, grid_for(d.nC, kBlock / 16), kBlock, d);
    } else if (long_rows) {  // (LV08 routes: ~12 elements per row)
      LAUNCH(2, r, fr_vote<16>, (nblk + spb - 1) / spb, kFB, d, int(r), spb);
    } else {
      LAUNCH(2, r, fr_vote<8>, (nblk + spb - 1) / spb, kFB, d, int(r), spb);
    }
    if (sat_b == 256)
      LAUNCH(4, r, fr_sat<256>, nblk, 256, d, int(r), bigch);
    else
      LAUNCH(4, r, fr_sat<kFS>, nblkS, kFS, d, int(r), bigch);
    if (big)
      LAUNCH(4, r, fr_sat_big, gbig, kBlock, d, int(r), bigw);
    LAUNCH(5, r, fr_update, nblk, kFB, d, int(r), prec, upd_spec);
    return 0;
  };
  int64_t r = 0;
  // pipelined termination polls, as solve_maxmin: chunk k's control words land in a pinned slot behind an
  // event while chunk k + 1 is queued; rounds queued after the last one return at once (CTL_DONE).  (Round 6,
  // measured and not kept: fr_vote storing "done" into a pinned host word itself, so that a poll is the event
  // alone without mm_ctl_out — C4 3.083-3.091 ms against 3.060-3.069, scripts/gpu_r06_p.sh; and the launches paced
  // by a per-round progress word, 2-5 rounds queued ahead — 3.17-3.28 against 3.12, scripts/gpu_r06_o.sh.)
  int chunk = 2, slot = 0;
  // rounds queued per poll: the host learns of termination one chunk late, so up to 2 x chunk_max no-op
  // rounds run after the last one (LMMHIP_CHUNK_MAX, A/B knob): C4 3.48 ms at 8, 3.51-3.53 at 4, 3.55 at 16
  // (short rounds: the no-op tail is a larger share)
  const int chunk_max = std::max(2, env_int("LMMHIP_CHUNK_MAX", 8));
  bool pending = false;
  int32_t* hc[2] = {c->h_ctl + CTL_WORDS, c->h_ctl + 2 * CTL_WORDS};
  int32_t* hcd[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hcd[k]), hc[k], 0));
  const int64_t hint = env_int("LMMHIP_ROUND_HINT", 1) ? c->hint_rounds_fr : 0;
  // with a hint the returning rounds after the last one are gone, and what longer chunks cost is with them: fewer
  // polls (mm_ctl_out, 3.6 us of kernel each) up to the hinted end (LMMHIP_HINT_CHUNK_MAX, A/B knob)
  const int chunk_cap = hint > 0 ? std::max(chunk_max, env_int("LMMHIP_HINT_CHUNK_MAX", 32)) : chunk_max;
  // and the first chunk need not be short either (its point is an early poll for systems of few rounds)
  if (hint > 0)
    chunk = std::max(chunk, std::min(chunk_cap, env_int("LMMHIP_HINT_CHUNK0", chunk_cap)));
  for (;;) {
    bool stop = false;
    const int n = round_hint_chunk(r, chunk, hint, &stop);
    for (int k = 0; k < n; k++, r++)
      if (int rc = round_launches(r))
        return rc;
    LAUNCH(6, r, mm_ctl_out, 1, kWave, d, hcd[slot]);
    HIPCHK(hipEventRecord(c->ev_poll[slot], c->stream));
    if (pending) {
      HIPCHK(hipEventSynchronize(c->ev_poll[slot ^ 1]));
      if (hc[slot ^ 1][CTL_DONE])
        break;
    }
    pending = !stop;
    if (stop) {  // the hinted end: this chunk's words before anything more is queued
      HIPCHK(hipEventSynchronize(c->ev_poll[slot]));
      if (hc[slot][CTL_DONE])
        break;
    }
    slot ^= 1;
    if (r > max_rounds)
      return fail(LMMHIP_E_NOCONVERGE, "maxmin round guard tripped");
    if (chunk < chunk_cap)
      chunk = std::min(2 * chunk, chunk_cap);
  }
  if (int rc = poll_ctl(c))
    return rc;
  c->hint_rounds_fr = int64_t(c->h_ctl[CTL_ROUNDS]) + 1;
  return 0;
}

static int engine_of(const lmmhip_ctx* c) {
  // LMMHIP_ENGINE=rounds|persistent|frontier overrides the context's engine; "auto" (or any other value,
  // which is ignored) leaves the context's choice in place
  const char* e = std::getenv("LMMHIP_ENGINE");
  int eng = c->engine;
  if (e && std::strcmp(e, "rounds") == 0)
    eng = LMMHIP_ENGINE_ROUNDS;
  if (e && std::strcmp(e, "persistent") == 0)
    eng = LMMHIP_ENGINE_PERSISTENT;
  if (e && std::strcmp(e, "frontier") == 0)
    eng = LMMHIP_ENGINE_FRONTIER;
  // the profiling mode times every phase launch: a multi-launch engine
  if (c->profiling)
    return eng == LMMHIP_ENGINE_FRONTIER ? LMMHIP_ENGINE_FRONTIER : LMMHIP_ENGINE_ROUNDS;
  if (eng != LMMHIP_ENGINE_AUTO)
    return eng;
  // AUTO (measured): one launch per solve where the host round-trips and launches of the
  // round chain dominate (small systems: a tie at C4, 1e5 variables, and ahead below); the round chain
  // above, where the kernel boundaries (~1.5 us) are cheaper than grid barriers (~4 us) and per-launch
  // grids keep 32 waves per CU in flight instead of 16
  // round 4: the frontier engine between the two (C4, 1e5 LV08 flows: 3.54 ms against 4.34 persistent and
  // 4.48 rounds), the round engine above (C2: 25.8 against 28.2 frontier)
  if (int64_t(c->d.nV) <= kAutoPersistMaxVars)
    return LMMHIP_ENGINE_PERSISTENT;
  return int64_t(c->d.nV) <= kAutoPersistVars ? LMMHIP_ENGINE_FRONTIER : LMMHIP_ENGINE_ROUNDS;
}

// One persistent launch per solve (lmm_persist_kernels.hpp): one 1024-thread workgroup per CU, all
// resident (the occupancy query admits exactly one per CU); every barrier wait is bounded, so a fault in
// the protocol ends the launch with CTL_ERR instead of hanging the GPU.
// Persistent launches are serialised per device, process-wide: a persistent grid needs every CU for one
// workgroup at once (its barriers rely on co-residency), so two of them running side by side — two Systems
// on two streams, or two threads — could each hold part of the chip and wait on the other.  Each persistent
// launch waits (on its own stream, no host blocking) for the previous one's completion event
// (g_persist_last, above).

// A persistent solve that cannot run — its launch rendezvous closed because part of the grid could not become
// resident within LMMHIP_PERSIST_RDV_MS (another kernel or process holding CUs: bar_rdv), or, later, a
// grid-barrier wait timed out (CTL_ERR 1) — is not an error of the system: the solve is re-run by the
// multi-launch engine, whose results are bit-identical (tests/test_gpu_engines.py).  The next
// LMMHIP_PERSIST_COOLDOWN solves of the context then take the multi-launch engine directly (a
// fallback that did not stick made every later solve under sustained contention pay the wait again).
static int solve_maxmin_persist_once(lmmhip_ctx* c, double prec, bool* closed);

// Streams left behind by closed persistent launches (their late workgroups may still run): each one whose work has
// drained is destroyed; past kRetiredCap of them the oldest is waited for (under sustained contention
// the list grew by one stream per close without bound).
constexpr size_t kRetiredCap = 8;
static int reap_retired_streams(lmmhip_ctx* c) {
  auto& v = c->retired_streams;
  for (size_t i = 0; i < v.size();) {
    const hipError_t q = hipStreamQuery(v[i]);
    if (q == hipErrorNotReady) {
      i++;
      continue;
    }
    (void)hipStreamDestroy(v[i]);
    v.erase(v.begin() + long(i));
  }
  while (v.size() > kRetiredCap) {
    HIPCHK(hipStreamSynchronize(v.front()));
    (void)hipStreamDestroy(v.front());
    v.erase(v.begin());
  }
  return 0;
}

static int solve_maxmin_persist(lmmhip_ctx* c, double prec) {
  if (int rc = reap_retired_streams(c))
    return rc;
  if (c->persist_cool > 0) {
    c->persist_cool -= 1;
    return solve_maxmin(c, prec);
  }
  c->h_ctl[CTL_ERR] = 0;
  bool closed = false;
  const int rc = solve_maxmin_persist_once(c, prec, &closed);
  if (!closed && (rc != LMMHIP_E_HIP || c->h_ctl[CTL_ERR] != 1))
    return rc;
  c->persist_fallbacks += 1;
  c->persist_cool = env_int("LMMHIP_PERSIST_COOLDOWN", 64);
  HIPCHK(hipMemsetAsync(c->d.ctl, 0, CTL_ALLOC * sizeof(int32_t), c->stream));
  c->ev1_done = false;
  return solve_maxmin(c, prec);
}

static int solve_maxmin_persist_once(lmmhip_ctx* c, double prec, bool* closed) {
  Dev d = c->d;
  d.vstat = nullptr;
  const bool bits = int64_t(d.nC) <= int64_t(kPBitWords) * 64;
  // 8 row elements in registers in the re-vote, longer rows loop over the rest.  (A 10-register variant for
  // long mean rows — C4's LV08 routes, 11.7 elements, when C4 still ran here — sat at the 128-VGPR budget of a
  // 1024-thread workgroup and spilled once the launch rendezvous moved ahead of the init; C4 runs on the
  // frontier engine since round 4, and AUTO keeps this engine for systems of at most 2^14 variables.)
  const void* kern = bits ? reinterpret_cast<const void*>(&mm_persist<true, 8>)
                          : reinterpret_cast<const void*>(&mm_persist<false, 8>);
  if (!c->pbar)
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->pbar), BAR_WORDS * sizeof(unsigned)));
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kPB, 0));
  if (per_cu < 1)
    return fail(LMMHIP_E_HIP, "persistent maxmin kernel: not one workgroup per CU (occupancy query)");
  const int grid = c->n_cu;
  c->persist_grid = grid;
  const int max_rounds = int(std::min<int64_t>(int64_t(d.nV) + 2, INT32_MAX - 1));
  const int cmp_every = env_int("LMMHIP_COMPACT_EVERY", 16);
  unsigned* barw = c->pbar;
  long long* pt = nullptr;
  unsigned pt_cap = 0;
  if (c->persist_prof) {  // barrier timestamps (lmmhip_persist_profile)
    pt_cap = kPersistProfCap;
    const size_t bytes = sizeof(long long) * (2 * size_t(pt_cap) + 2 * size_t(kPBlkCap) * size_t(grid));
    if (!c->ptime)
      HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->ptime), bytes));
    HIPCHK(hipMemsetAsync(c->ptime, 0, bytes, c->stream));
    pt = c->ptime;
  }
  int sysf = env_int("LMMHIP_PERSIST_SYSFENCE", 0);
  // launch rendezvous deadline (bar_rdv): the grid's workgroups are dispatched within microseconds when the CUs
  // are free, so 20 ms of waiting means part of the chip is held by someone else
  long long rdv_ticks = 100000LL * env_int("LMMHIP_PERSIST_RDV_MS", 20);  // 100 MHz wall clock
  int32_t* hflag = c->d_rdv;
  void* args[] = {&d, &barw, &prec, const_cast<int*>(&max_rounds), const_cast<int*>(&cmp_every), &pt, &pt_cap, &sysf,
                  &rdv_ticks, &hflag};
  // A plain launch on the context's stream: the occupancy query above guarantees one workgroup per CU, so the
  // n_cu workgroups are co-resident once the stream's earlier work has drained and nothing else holds CUs; the
  // rendezvous deadline and the bounded barrier waits cover the case where something does.
  // hipLaunchCooperativeKernel (LMMHIP_PERSIST_COOP=1) runs the same kernel through the runtime's device-wide
  // cooperative queue, whose teardown at process exit crashed inside the HSA runtime under rocprofv3 (SIGSEGV
  // in libamdhip64's exit handler).
  {
    std::lock_guard<std::mutex> lk(g_persist_mu);
    hipEvent_t& last = g_persist_last[c->device];
    if (last && hipStreamWaitEvent(c->stream, last, 0) != hipSuccess) {  // (a stale event: make a new one)
      (void)hipGetLastError();
      (void)hipEventDestroy(last);
      last = nullptr;
    }
    if (!last)
      HIPCHK(hipEventCreateWithFlags(&last, hipEventDisableTiming));
    // the barrier words are reset behind the previous persistent launch (whose late workgroups, after a closed
    // rendezvous, still read them)
    HIPCHK(hipMemsetAsync(c->pbar, 0, BAR_WORDS * sizeof(unsigned), c->stream));
    HIPCHK(hipMemsetAsync(d.chgbits, 0, sizeof(uint64_t) * ((d.nC + 127) / 128 * 2 + 2), c->stream));
    __atomic_store_n(c->h_rdv, 0, __ATOMIC_RELEASE);
    if (env_int("LMMHIP_PERSIST_COOP", 0))
      HIPCHK(hipLaunchCooperativeKernel(kern, dim3(grid), dim3(kPB), args, 0, c->stream));
    else
      HIPCHK(hipLaunchKernel(kern, dim3(grid), dim3(kPB), args, 0, c->stream));
    HIPCHK(hipEventRecord(last, c->stream));
  }
  c->stats.kernel_launches[2] += 1;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  c->ev1_done = true;
  // wait for the launch, or for its rendezvous to close (the mapped word), whichever comes first
  for (;;) {
    const hipError_t q = hipEventQuery(c->ev1);
    if (q == hipSuccess)
      break;
    if (q != hipErrorNotReady)
      HIPCHK(q);
    if (__atomic_load_n(c->h_rdv, __ATOMIC_ACQUIRE)) {  // closed: no workgroup of it has written anything
      // The launch is left behind with its late workgroups (they return at once when they get CUs).  A context
      // on its own stream moves to a new one, so the fallback and everything after it run on the free CUs now;
      // a caller-provided stream keeps its order (the fallback then waits for the late workgroups).
      *closed = true;
      if (c->stream == c->own_stream) {
        hipStream_t ns = nullptr;
        HIPCHK(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
        c->retired_streams.push_back(c->own_stream);
        c->own_stream = c->stream = ns;
      }
      return fail(LMMHIP_E_HIP, "persistent maxmin kernel: the launch rendezvous closed (grid not co-resident)");
    }
    std::this_thread::yield();
  }
  if (int rc = poll_ctl(c))
    return rc;
  if (c->h_ctl[CTL_ERR] == 1)
    return fail(LMMHIP_E_HIP, "persistent maxmin kernel: a grid-barrier wait timed out");
  if (c->h_ctl[CTL_ERR] == 2)
    return fail(LMMHIP_E_NOCONVERGE, "maxmin round guard tripped");
  return 0;
}

// ---- block-diagonal batches: one workgroup per system, the system in LDS (lmm_batch_kernels.hpp) ----
constexpr size_t kBatchLdsMax = 64 * 1024;  // per workgroup; larger systems take the global engines

static bool batch_fits(const lmmhip_ctx* c) {
  if (c->bt_n <= 0 || c->profiling)
    return false;
  if (const char* e = std::getenv("LMMHIP_BATCH"); e && *e == '0')
    return false;
  return c->bt_max_nv < 65535 && c->bt_max_nc < 65535 && c->bt_max_nnz < 65535 &&
         batch_lds_bytes(c->bt_max_nv, c->bt_max_nc, c->bt_max_nnz) <= kBatchLdsMax;
}

static int solve_maxmin_batch(lmmhip_ctx* c, double prec) {
  const size_t lds = batch_lds_bytes(c->bt_max_nv, c->bt_max_nc, c->bt_max_nnz);
  int per_cu = 0;
  HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&mm_batch_lds),
                             hipFuncAttributeMaxDynamicSharedMemorySize, int(kBatchLdsMax)));
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&mm_batch_lds), kBB,
                                                      lds));
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(c->bt_n, int64_t(c->n_cu) * std::max(per_cu, 1)));
  if (grid > c->bt_cap) {
    if (c->bt_rounds)
      HIPCHK(hipFree(c->bt_rounds));
    c->bt_rounds = nullptr;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->bt_rounds), sizeof(int32_t) * size_t(grid)));
    c->bt_cap = grid;
  }
  Dev d = c->d;
  hipLaunchKernelGGL(mm_batch_lds, dim3(unsigned(grid)), dim3(kBB), lds, c->stream, d, c->bt_voff, c->bt_coff,
                     c->bt_n, prec, c->bt_max_nv, c->bt_max_nc, c->bt_max_nnz, c->bt_rounds);
  HIPCHK(hipGetLastError());
  c->stats.kernel_launches[2] += 1;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  c->ev1_done = true;
  hipLaunchKernelGGL(mm_batch_rounds, dim3(1), dim3(kBlock), 0, c->stream, c->bt_rounds, int(grid), d.ctl);
  HIPCHK(hipGetLastError());
  if (int rc = poll_ctl(c))
    return rc;
  if (c->h_ctl[CTL_ERR] == 2)
    return fail(LMMHIP_E_NOCONVERGE, "batch maxmin round guard tripped");
  return 0;
}

static int fb_begin(lmmhip_ctx* c, double prec) {
  Dev& d = c->d;
  c->fb_round = 0;
  c->fb_prec = prec;
  LAUNCH(0, -1, fb_init, grid_for(std::max(d.nV, d.nC), kBlock), kBlock, d);
  return 0;
}

// One phase of a fair-bottleneck round (lmm_fb_kernels.hpp); phase 2 ends the round.
static int fb_phase(lmmhip_ctx* c, int phase) {
  Dev& d = c->d;
  const int64_t r = c->fb_round;
  const int par = int(r & 1);
  const int gQ = grid_for(d.nch, kBlock / kWave);
  const int gC = grid_for(d.nC, kBlock);
  const int gV = grid_for(d.nV, kBlock);
  switch (phase) {
  case 0:  // round 0 lists every flattened variable (fair_bottleneck.cpp:29-41): counts without gathers
    if (r > 0)
      LAUNCH(2, r, fb_pack_vst, grid_for((int64_t(d.nV) + 31) / 32, kBlock), kBlock, d);
    LAUNCH(2, r, fbk_count, gQ, kBlock, d, int(r == 0));
    LAUNCH(2, r, fbk_nb, gC, kBlock, d, par);
    break;
  case 1:
    LAUNCH(3, r, fbk_share, gC, kBlock, d, par);
    LAUNCH(3, r, fb_var_inc, gV, kBlock, d, par, int(r));
    if (c->fb_shard) {  // shards: this shard's mu into the gathered vector, then the caller's all-gather
      LAUNCH(3, r, fbo_put_mu, gV, kBlock, d, c->fbo);
      break;
    }
    LAUNCH(4, r, fbk_acc, gQ, kBlock, d, int(r == 0), c->fb_longmin);
    LAUNCH(4, r, fbk_accc, gC, kBlock, d);
    break;
  case 2:
    if (c->fb_shard) {  // the owned constraints' chains from the gathered mu -> xrem (all-gathered)
      LAUNCH(4, r, fbo_acc, grid_for(c->fbo.nch, kBlock / kWave), kBlock, d, c->fbo);
      LAUNCH(5, r, fbo_chain, grid_for(c->fbo.nc, kBlock / kWave), kBlock, d, c->fbo, c->fb_prec);
      break;
    }
    // one context: element by element in the CSC order, bit-identical to the reference
    LAUNCH(5, r, fbk_update_seq, c->fb_nlb + grid_for(d.nC, kBlock / kWave), kBlock, d, c->fb_prec,
           c->fb_longmin, c->fb_nlb);
    LAUNCH(5, r, fbk_unlist, gQ, kBlock, d, int(r > 0));  // (vstb is packed in rounds > 0)
    c->fb_round++;
    break;
  case 3:
    if (!c->fb_shard)
      return fail(LMMHIP_E_ARG, "phase 3 exists only in a sharded solve");
    LAUNCH(5, r, fbo_apply, gC, kBlock, d, c->fbo);
    LAUNCH(5, r, fbk_unlist, gQ, kBlock, d, int(r > 0));  // (vstb is packed in rounds > 0)
    c->fb_round++;
    break;
  default:
    return fail(LMMHIP_E_ARG, "fair-bottleneck phase must be 0..2 (one context) or 0..3 (shard)");
  }
  return 0;
}

// The locality order of the one-context FairBottleneck's mu gathers (lmm_fb_kernels.hpp fbp_*): once per
// uploaded system, outside the solve.  LMMHIP_FB_PERM=0 gathers mu by variable id instead (measurement knob).
static int fb_perm(lmmhip_ctx* c) {
  Dev& d = c->d;
  if (!env_int("LMMHIP_FB_PERM", 1) || d.nV == 0) {
    d.mu_p = nullptr;
    return 0;
  }
  int32_t *v0, *v1;
  unsigned long long *k0, *k1;
  int rc = scratch(c, c->fbp_k0, d.nV, &k0);
  rc = rc ? rc : scratch(c, c->fbp_k1, d.nV, &k1);
  rc = rc ? rc : scratch(c, c->fbp_v0, d.nV, &v0);
  rc = rc ? rc : scratch(c, c->fbp_v1, d.nV, &v1);
  rc = rc ? rc : scratch(c, c->fbp_perm, d.nV, &d.vperm);
  rc = rc ? rc : scratch(c, c->fbp_cscvp, std::max<int64_t>(d.nnz, 1), &d.csc_vp);
  rc = rc ? rc : scratch(c, c->fbp_mu, d.nV, &d.mu_p);
  if (rc)
    return rc;
  if (!c->fb_perm_ok) {
    const unsigned long long span = (unsigned long long)d.nC * (unsigned long long)d.nC + 1;
    const int bits = std::min(64, 64 - __builtin_clzll(span));
    hipLaunchKernelGGL(fbp_keys, dim3(grid_for(d.nV, kBlock)), dim3(kBlock), 0, c->stream, d, k0, v0);
    HIPCHK(hipGetLastError());
    size_t tb = 0;
    HIPCHK(sort_pairs_u64_i32(nullptr, tb, k0, k1, v0, v1, d.nV, 64, c->stream));
    uint8_t* t = nullptr;
    if ((rc = scratch(c, c->fbp_tmp, int64_t(tb), &t)))
      return rc;
    // (keys of empty rows are all ones: sorted with the 64-bit width when the span needs it)
    HIPCHK(sort_pairs_u64_i32(t, tb, k0, k1, v0, v1, d.nV, bits < 64 ? 64 : bits, c->stream));
    hipLaunchKernelGGL(fbp_inv, dim3(grid_for(d.nV, kBlock)), dim3(kBlock), 0, c->stream, d, v1);
    HIPCHK(hipGetLastError());
    if (d.nnz > 0) {
      hipLaunchKernelGGL(fbp_csc, dim3(grid_for(d.nnz, kBlock)), dim3(kBlock), 0, c->stream, d);
      HIPCHK(hipGetLastError());
    }
    c->fb_perm_ok = true;
  }
  return 0;
}

static int solve_fair_rounds(lmmhip_ctx* c, double prec);

static int solve_fair(lmmhip_ctx* c, double prec) {
  c->fb_shard = false;
  // shared constraints of at least this many elements get their increments precomputed element-parallel
  // (fbk_acc) and streamed into their chains (fb_chain); shorter ones compute them inside the chain
  // (fb_chain_pull).  Pulling in round 0 and streaming fbk_acc's listed-variable rewrites afterwards measured
  // 3 % slower on C5 (9.68 vs 9.42 ms, same box): the increments' gathers move, they do not go away.
  c->fb_longmin = uint32_t(std::max(0, env_int("LMMHIP_FB_LONG", 16384)));
  if (c->fbd_cap < c->d.nnz) {  // increments in CSC order (fbk_acc -> fbk_update_seq)
    if (int rc = dalloc(c, &c->d.fbd, c->d.nnz))
      return rc;
    c->fbd_cap = c->d.nnz;
  }
  if (int rc = scratch(c, c->fb_longl, int64_t(c->d.nC) + 1, &c->d.fb_long))  // the long shared constraints
    return rc;
  HIPCHK(hipMemsetAsync(c->d.fb_long, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(fb_long_list, dim3(grid_for(c->d.nC, kBlock)), dim3(kBlock), 0, c->stream, c->d,
                     c->fb_longmin);
  HIPCHK(hipGetLastError());
  // the long chains by LMMHIP_FB_LONGWG workgroups
  c->fb_nlb = std::max(1, env_int("LMMHIP_FB_LONGWG", kLongBlocks));
  c->d.xnb = c->xnb_own;
  c->d.xmin = c->xmin_own;
  if (int rc = fb_perm(c))
    return rc;
  return solve_fair_rounds(c, prec);
}

static int solve_fair_rounds(lmmhip_ctx* c, double prec) {
  if (int rc = fb_begin(c, prec))
    return rc;
  // The reference's rounds are not bounded by the system size (FATPIPE remaining can shrink
  // geometrically: millions of rounds on 60-variable systems); give up past this budget.
  const int64_t max_rounds = 64 * (int64_t(c->d.nV) + int64_t(c->d.nC)) + 4096;
  // (LMMHIP_FB_PACE=0) One round queued ahead of the termination poll: after round r the control words go to a pinned
  // slot (mm_ctl_out), round r + 1 is queued, then the host waits for round r's words.  A FairBottleneck round is
  // long (C5: 0.2-3 ms), so the GPU never waits on the host and at most one empty round (its launches return
  // at once) runs after the last one; chunks of 4, 8, ... rounds left up to 7 empty rounds (63 launches,
  // ~0.2 ms on C5) plus a host round trip between chunks.
  // Pacing by progress words (default; LMMHIP_FB_PACE=0: the polls below): fbk_share stores the number of rounds
  // it has started into a pinned host word, or "done" beside it when nothing is listed (lmm_fb_kernels.hpp), and the
  // host queues round r + 1 once round r's fbk_share has started — the rest of round r (its chains: 0.1-1 ms on C5)
  // covers the queueing, no copy kernel or event per round, and no returning round after the one that finds the
  // solve over.  Round 6, C5: 7.94-7.96 ms against 7.99-8.00 with LMMHIP_FB_PACE=0 (one box, scripts/gpu_r06_o.sh),
  // 7.82-7.93 against 7.92-7.93 for the previous build (scripts/gpu_r06_p.sh).
  if (env_int("LMMHIP_FB_PACE", 1)) {
    volatile int32_t* hp = c->h_ctl + 3 * CTL_WORDS;
    hp[0] = 0;
    hp[1] = 0;
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d.hprog), c->h_ctl + 3 * CTL_WORDS, 0));
    struct HprogOff {  // (the context's Dev: the other engines and the sharded phases run without the words)
      Dev& d;
      ~HprogOff() { d.hprog = nullptr; }
    } hprog_off{c->d};
    // rounds shorter than the host's queueing of the next one (small systems: a round is its ~9 launches) would
    // leave the GPU idle under this pacing, so when the rounds come faster than every 150 us one round stays queued
    // ahead (lag 1), as with the polls below
    int lag = 0;
    auto t_last = std::chrono::steady_clock::now();
    for (;;) {
      for (int ph = 0; ph < 3; ph++)
        if (int rc = fb_phase(c, ph))
          return rc;
      const int32_t want = int32_t(c->fb_round) - lag;  // rounds started, counting the one just queued
      for (unsigned spin = 0;; spin++) {
        if (hp[1] || hp[0] >= want) {
          const auto t = std::chrono::steady_clock::now();
          lag = t - t_last < std::chrono::microseconds(150) ? 1 : 0;
          t_last = t;
          break;
        }
        if ((spin & 1023) == 1023) {  // everything queued has run (a guard: the words should have said so)
          const hipError_t q = hipStreamQuery(c->stream);
          if (q == hipSuccess)
            break;
          if (q != hipErrorNotReady)
            return fail(LMMHIP_E_HIP, std::string("fair-bottleneck pacing: ") + hipGetErrorString(q));
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
      if (hp[1])
        break;
      if (c->fb_round > max_rounds)
        return fail(LMMHIP_E_NOCONVERGE, "fair-bottleneck round guard tripped");
    }
    return poll_ctl(c);
  }
  int slot = 0;
  bool pending = false;
  int32_t* hc[2] = {c->h_ctl + CTL_WORDS, c->h_ctl + 2 * CTL_WORDS};
  int32_t* hcd[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hcd[k]), hc[k], 0));
  for (;;) {
    for (int ph = 0; ph < 3; ph++)
      if (int rc = fb_phase(c, ph))
        return rc;
    const Dev& d = c->d;
    LAUNCH(6, c->fb_round, mm_ctl_out, 1, kWave, d, hcd[slot]);
    HIPCHK(hipEventRecord(c->ev_poll[slot], c->stream));
    if (pending) {
      HIPCHK(hipEventSynchronize(c->ev_poll[slot ^ 1]));
      if (hc[slot ^ 1][CTL_DONE])
        break;
    }
    pending = true;
    slot ^= 1;
    if (c->fb_round > max_rounds)
      return fail(LMMHIP_E_NOCONVERGE, "fair-bottleneck round guard tripped");
  }
  return poll_ctl(c);  // (the queued round has run: final words for the stats)
}

int lmmhip_ctx_set_stream(lmmhip_ctx* c, void* stream) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->stream = static_cast<hipStream_t>(stream);  // 0 = the legacy null stream, like any other handle
  return 0;
}

int lmmhip_ctx_use_own_stream(lmmhip_ctx* c) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->stream = c->own_stream;
  return 0;
}

int lmmhip_set_batch(lmmhip_ctx* c, int64_t nsys, const int64_t* var_off, const int64_t* cnst_off) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  c->bt_n = 0;
  if (nsys == 0)
    return 0;
  if (nsys < 0 || !var_off || !cnst_off)
    return fail(LMMHIP_E_ARG, "bad batch arguments");
  const Dev& d = c->d;
  if (var_off[0] != 0 || var_off[nsys] != d.nV || cnst_off[0] != 0 || cnst_off[nsys] != d.nC)
    return fail(LMMHIP_E_ARG, "batch offsets must cover the uploaded system");
  for (int64_t i = 0; i < nsys; i++)
    if (var_off[i + 1] < var_off[i] || cnst_off[i + 1] < cnst_off[i])
      return fail(LMMHIP_E_ARG, "batch offsets not monotone");
  HIPCHK(hipSetDevice(c->device));
  std::vector<uint32_t> vp(size_t(d.nV) + 1);
  HIPCHK(hipMemcpyAsync(vp.data(), d.var_ptr, vp.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  int64_t mv = 0, mc = 0, me = 0;
  for (int64_t i = 0; i < nsys; i++) {
    mv = std::max(mv, var_off[i + 1] - var_off[i]);
    mc = std::max(mc, cnst_off[i + 1] - cnst_off[i]);
    me = std::max(me, int64_t(vp[size_t(var_off[i + 1])]) - int64_t(vp[size_t(var_off[i])]));
  }
  for (void* p : {(void*)c->bt_voff, (void*)c->bt_coff})
    if (p)
      HIPCHK(hipFree(p));
  c->bt_voff = c->bt_coff = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->bt_voff), sizeof(int64_t) * size_t(nsys + 1)));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->bt_coff), sizeof(int64_t) * size_t(nsys + 1)));
  HIPCHK(hipMemcpyAsync(c->bt_voff, var_off, sizeof(int64_t) * size_t(nsys + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bt_coff, cnst_off, sizeof(int64_t) * size_t(nsys + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(d.ctl + CTL_ERR, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(mm_batch_check, dim3(unsigned(std::min<int64_t>(nsys, 4096))), dim3(kBlock), 0, c->stream, d,
                     c->bt_voff, c->bt_coff, nsys, d.ctl + CTL_ERR);
  HIPCHK(hipGetLastError());
  int32_t bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, d.ctl + CTL_ERR, sizeof(bad), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (bad)
    return fail(LMMHIP_E_ARG, "batch: an element links two declared systems (not block-diagonal)");
  c->bt_n = nsys;
  c->bt_max_nv = int(mv);
  c->bt_max_nc = int(mc);
  c->bt_max_nnz = int(me);
  return 0;
}

int lmmhip_persist_profile(lmmhip_ctx* c, int on, int64_t* t, int64_t cap, int64_t* n) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  c->persist_prof = on != 0;
  if (n)
    *n = 0;
  if (!t || !c->ptime)
    return 0;
  HIPCHK(hipSetDevice(c->device));
  std::vector<long long> h(2 * size_t(kPersistProfCap));
  HIPCHK(hipMemcpyAsync(h.data(), c->ptime, h.size() * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  int64_t m = 0;
  while (m < int64_t(kPersistProfCap) && h[2 * size_t(m) + 1] != 0)
    m++;
  for (int64_t i = 0; i < m && 2 * i + 1 < cap; i++) {
    t[2 * i] = h[2 * size_t(i)];
    t[2 * i + 1] = h[2 * size_t(i) + 1];
  }
  if (n)
    *n = m;
  return 0;
}

int lmmhip_persist_profile_blocks(lmmhip_ctx* c, int64_t* t, int64_t cap, int64_t* nbar, int64_t* nblk) {
  if (!c || !c->ptime || !c->persist_grid)
    return fail(LMMHIP_E_STATE, "no profiled persistent solve");
  HIPCHK(hipSetDevice(c->device));
  const size_t n = 2 * size_t(kPBlkCap) * size_t(c->persist_grid);
  std::vector<long long> h(n);
  HIPCHK(hipMemcpyAsync(h.data(), c->ptime + 2 * size_t(kPersistProfCap), n * sizeof(long long),
                        hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < n && int64_t(i) < cap; i++)
    t[i] = h[i];
  *nbar = kPBlkCap;
  *nblk = c->persist_grid;
  return 0;
}

int lmmhip_anatomy(lmmhip_ctx* c, unsigned long long* out, int64_t cap, int64_t* n, int32_t* rounds4) {
  if (!c || !n)
    return fail(LMMHIP_E_ARG, "null argument");
  const int64_t words = int64_t(kAnatSlots) * kAnatKernels * kAnatWaves * kAnatFields;
  *n = 0;
  if (!LMM_ANAT)
    return fail(LMMHIP_E_STATE, "not an anatomy build (make EXTRA_HIPFLAGS=-DLMM_ANAT=1)");
  if (!c->anat || !c->solved)
    return fail(LMMHIP_E_STATE, "no solve recorded an anatomy (set LMMHIP_ANAT_ROUNDS)");
  *n = words;
  if (rounds4)
    for (int k = 0; k < kAnatSlots; k++)
      rounds4[k] = c->d.anat_r[k];
  if (out) {
    if (cap < words)
      return fail(LMMHIP_E_ARG, "anatomy: cap too small");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(out, c->anat, size_t(words) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  }
  return 0;
}

int lmmhip_engine_fallbacks(lmmhip_ctx* c, int64_t* n) {
  if (!c || !n)
    return fail(LMMHIP_E_ARG, "null argument");
  *n = c->persist_fallbacks;
  return 0;
}

int lmmhip_ctx_set_engine(lmmhip_ctx* c, int engine) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (engine != LMMHIP_ENGINE_PERSISTENT && engine != LMMHIP_ENGINE_ROUNDS && engine != LMMHIP_ENGINE_AUTO &&
      engine != LMMHIP_ENGINE_FRONTIER)
    return fail(LMMHIP_E_ARG, "unknown maxmin engine");
  c->engine = engine;
  return 0;
}

int lmmhip_fb_shard_owner(lmmhip_ctx* c, int64_t n_own, const int32_t* own_cnst, const int64_t* optr,
                          const int32_t* ovar, const double* oweight, const int32_t* cpos, int64_t n_mu,
                          int64_t n_rem) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  const Dev& d = c->d;
  if (n_own < 0 || n_own > d.nC || n_mu < 0 || n_rem < 0 || (n_own > 0 && (!own_cnst || !optr)) ||
      (d.nC > 0 && !cpos))
    return fail(LMMHIP_E_ARG, "bad owner arguments");
  const int64_t onnz = n_own > 0 ? optr[n_own] : 0;
  if (n_own > 0 && optr[0] != 0)
    return fail(LMMHIP_E_ARG, "optr must start at 0");
  if (onnz > INT32_MAX || (onnz > 0 && (!ovar || !oweight)))
    return fail(LMMHIP_E_ARG, "bad owned elements");
  std::vector<uint32_t> op(size_t(n_own) + 1, 0);
  std::vector<int32_t> och_o;
  std::vector<uint32_t> och_b;
  for (int64_t i = 0; i < n_own; i++) {
    if (own_cnst[i] < 0 || own_cnst[i] >= d.nC || optr[i + 1] < optr[i])
      return fail(LMMHIP_E_ARG, "owned constraint id / offsets out of range");
    op[size_t(i) + 1] = uint32_t(optr[i + 1]);
    for (int64_t b = optr[i]; b < optr[i + 1]; b += kFbChunk) {
      och_o.push_back(int32_t(i));
      och_b.push_back(uint32_t(b));
    }
  }
  for (int64_t j = 0; j < onnz; j++)
    if (ovar[j] < 0 || ovar[j] >= n_mu || !(oweight[j] > 0))
      return fail(LMMHIP_E_ARG, "owned element: variable position outside the gathered mu, or weight <= 0");
  for (int64_t k = 0; k < d.nC; k++)
    if (cpos[k] < 0 || cpos[k] >= n_rem)
      return fail(LMMHIP_E_ARG, "cpos outside the gathered remaining");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  free_owner(c);
  FbOwner& o = c->fbo;
  auto get = [&](auto** p, int64_t n, const void* src, size_t elt) -> int {
    void* q = nullptr;
    HIPCHK(hipMalloc(&q, size_t(n > 0 ? n : 1) * elt));
    c->fbo_allocs.push_back(q);
    if (src && n > 0)
      HIPCHK(hipMemcpyAsync(q, src, size_t(n) * elt, hipMemcpyHostToDevice, c->stream));
    *p = static_cast<std::remove_reference_t<decltype(**p)>*>(q);
    return 0;
  };
  int32_t *oc, *ov, *cho, *cp;
  uint32_t *opp, *chb;
  double* ow;
  int rc = 0;
  rc |= get(&oc, n_own, own_cnst, sizeof(int32_t));
  rc |= get(&opp, n_own + 1, op.data(), sizeof(uint32_t));
  rc |= get(&ov, onnz, ovar, sizeof(int32_t));
  rc |= get(&ow, onnz, oweight, sizeof(double));
  rc |= get(&cho, int64_t(och_o.size()), och_o.data(), sizeof(int32_t));
  rc |= get(&chb, int64_t(och_b.size()), och_b.data(), sizeof(uint32_t));
  rc |= get(&cp, d.nC, cpos, sizeof(int32_t));
  rc |= get(&o.fbd, onnz, nullptr, sizeof(double));
  if (rc) {
    free_owner(c);
    return rc;
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  o.nc = int32_t(n_own);
  o.nch = int32_t(och_o.size());
  o.oc = oc;
  o.optr = opp;
  o.ovar = ov;
  o.ow = ow;
  o.och_o = cho;
  o.och_b = chb;
  o.cpos = cp;
  c->fbo_ready = true;
  c->fbo_nmu = n_mu;
  return 0;
}

int lmmhip_fb_shard_begin(lmmhip_ctx* c, double precision, int32_t* xnb, double* xmu, int64_t mu_off, double* xrem) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  if (!c->fbo_ready)
    return fail(LMMHIP_E_STATE, "lmmhip_fb_shard_owner first");
  if (!xnb || !xmu || !xrem)
    return fail(LMMHIP_E_ARG, "null exchange buffer");
  if (mu_off < 0 || mu_off + c->d.nV > c->fbo_nmu)
    return fail(LMMHIP_E_ARG, "this shard's mu block lies outside the gathered mu");
  HIPCHK(hipSetDevice(c->device));
  c->pool_used = 0;
  c->launch_slot.clear();
  c->launch_round.clear();
  c->launch_ms.clear();
  HIPCHK(hipMemsetAsync(c->d.ctl, 0, CTL_ALLOC * sizeof(int32_t), c->stream));
  c->d.xnb = xnb;
  c->d.xmin = c->xmin_own;
  c->fbo.xmu = xmu;
  c->fbo.xrem = xrem;
  c->fbo.mu_off = mu_off;
  c->fb_shard = true;
  c->d.mu_p = nullptr;  // (the shard kernels gather mu by variable id; fb_perm is the one-context path's)
  c->last_kind = LMMHIP_KIND_FAIR_BOTTLENECK;
  return fb_begin(c, precision);
}

int lmmhip_fb_shard_step(lmmhip_ctx* c, int phase) {
  if (!c || !c->fb_shard)
    return fail(LMMHIP_E_STATE, "lmmhip_fb_shard_begin first");
  HIPCHK(hipSetDevice(c->device));
  return fb_phase(c, phase);
}

int lmmhip_fb_shard_pack_mu(lmmhip_ctx* c, int32_t* pos, double* mu, int32_t* count) {
  if (!c || !c->fb_shard)
    return fail(LMMHIP_E_STATE, "lmmhip_fb_shard_begin first");
  if (!pos || !mu || !count)
    return fail(LMMHIP_E_ARG, "null buffer");
  HIPCHK(hipSetDevice(c->device));
  Dev& d = c->d;
  LAUNCH(3, c->fb_round, fbo_pack_mu, grid_for(d.nV, kBlock), kBlock, d, c->fbo, int(c->fb_round == 0), pos, mu,
         count);
  return 0;
}

int lmmhip_fb_work(lmmhip_ctx* c, int64_t* out3) {
  if (!c || !out3)
    return fail(LMMHIP_E_ARG, "null argument");
  if (c->last_kind != LMMHIP_KIND_FAIR_BOTTLENECK)
    return fail(LMMHIP_E_STATE, "the last solve was not a FairBottleneck solve");
  HIPCHK(hipSetDevice(c->device));
  if (int rc = poll_ctl(c))
    return rc;
  uint64_t sl[3 * kFbwSlots];
  HIPCHK(hipMemcpy(sl, c->d.ctl + CTL_FBW_AT, sizeof sl, hipMemcpyDeviceToHost));
  for (int k = 0; k < 3; k++) {
    uint64_t v = 0;
    for (int i = 0; i < kFbwSlots; i++)
      v += sl[k * kFbwSlots + i];
    out3[k] = int64_t(v);
  }
  return 0;
}

int lmmhip_fb_shard_poll(lmmhip_ctx* c, int* done, int64_t* rounds) {
  if (!c || !c->fb_shard)
    return fail(LMMHIP_E_STATE, "lmmhip_fb_shard_begin first");
  HIPCHK(hipSetDevice(c->device));
  if (int rc = poll_ctl(c))
    return rc;
  if (done)
    *done = c->h_ctl[CTL_DONE];
  if (rounds)
    *rounds = c->h_ctl[CTL_ROUNDS];
  c->stats.rounds = c->h_ctl[CTL_ROUNDS];
  return 0;
}

// ---- model-side step glue (lmm_step_kernels.hpp) ----
extern "C++" template <class T> static int act_alloc(lmmhip_ctx* c, T** out, int64_t n, const T* src) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, size_t(n > 0 ? n : 1) * sizeof(T)));
  c->act_allocs.push_back(p);
  *out = static_cast<T*>(p);
  if (src && n > 0)
    HIPCHK(hipMemcpyAsync(p, src, size_t(n) * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return 0;
}

int lmmhip_actions_upload(lmmhip_ctx* c, int64_t n, const int32_t* var_index, const double* remains,
                          const double* max_duration, const double* latency, const double* penalty,
                          const double* sharing_penalty, const uint8_t* flags) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (n < 0 || (n > 0 && (!var_index || !remains || !max_duration || !latency || !penalty || !sharing_penalty ||
                          !flags)))
    return fail(LMMHIP_E_ARG, "null action arrays");
  const int64_t nV = c->uploaded ? c->d.nV : 0;
  for (int64_t i = 0; i < n; i++)
    if (var_index[i] < -1 || var_index[i] >= nV)
      return fail(LMMHIP_E_ARG, "action var_index out of range of the uploaded system");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (void* p : c->act_allocs)
    (void)hipFree(p);
  c->act_allocs.clear();
  ActDev& a = c->act;
  a = ActDev{};
  a.n = n;
  int32_t* vidx;
  double *sp;
  uint8_t* fl;
  int rc = 0;
  rc |= act_alloc(c, &vidx, n, var_index);
  rc |= act_alloc(c, &a.remains, n, remains);
  rc |= act_alloc(c, &a.max_duration, n, max_duration);
  rc |= act_alloc(c, &a.latency, n, latency);
  rc |= act_alloc(c, &a.penalty, n, penalty);
  rc |= act_alloc(c, &sp, n, sharing_penalty);
  rc |= act_alloc(c, &fl, n, flags);
  rc |= act_alloc<uint8_t>(c, &a.events, n, nullptr);
  rc |= act_alloc<unsigned long long>(c, &a.umin, 1, nullptr);
  rc |= act_alloc<int32_t>(c, &a.nev, 1, nullptr);
  if (rc)
    return rc;
  a.vidx = vidx;
  a.share_pen = sp;
  a.flags = fl;
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_next_event_full(lmmhip_ctx* c, int with_latency, double* out) {
  if (!c || !out)
    return fail(LMMHIP_E_ARG, "null argument");
  if (!c->act.umin)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_upload first");
  HIPCHK(hipSetDevice(c->device));
  unsigned long long h = ~0ull;
  HIPCHK(hipMemsetAsync(c->act.umin, 0xFF, sizeof(unsigned long long), c->stream));
  if (c->act.n > 0)
    LAUNCH(7, -1, act_next_event, grid_for(c->act.n, kBlock), kBlock, c->act, c->d.x, with_latency);
  HIPCHK(hipMemcpyAsync(&h, c->act.umin, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (h == ~0ull) {
    *out = -1.0;
  } else {
    double m;
    std::memcpy(&m, &h, sizeof(m));
    *out = m;
  }
  return 0;
}

int lmmhip_update_actions_full(lmmhip_ctx* c, int model, double delta, double maxmin_precision,
                               double surf_precision, int64_t* n_events) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (!c->act.nev)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_upload first");
  if (model != MODEL_CPU && model != MODEL_CM02 && model != MODEL_L07)
    return fail(LMMHIP_E_ARG, "unknown model");
  HIPCHK(hipSetDevice(c->device));
  int32_t h = 0;
  HIPCHK(hipMemsetAsync(c->act.nev, 0, sizeof(int32_t), c->stream));
  if (c->act.n > 0)
    LAUNCH(7, -1, act_update, grid_for(c->act.n, kBlock), kBlock, c->act, c->d.x, model, delta, maxmin_precision,
           surf_precision);
  HIPCHK(hipMemcpyAsync(&h, c->act.nev, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (n_events)
    *n_events = h;
  return 0;
}

int lmmhip_actions_download(lmmhip_ctx* c, double* remains, double* max_duration, double* latency, double* penalty,
                            uint8_t* events) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  HIPCHK(hipSetDevice(c->device));
  const size_t n = size_t(c->act.n);
  if (n) {
    if (remains)
      HIPCHK(hipMemcpyAsync(remains, c->act.remains, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (max_duration)
      HIPCHK(hipMemcpyAsync(max_duration, c->act.max_duration, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (latency)
      HIPCHK(hipMemcpyAsync(latency, c->act.latency, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (penalty)
      HIPCHK(hipMemcpyAsync(penalty, c->act.penalty, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (events)
      HIPCHK(hipMemcpyAsync(events, c->act.events, n, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_actions_lazy_upload(lmmhip_ctx* c, const double* last_update, const double* last_value,
                               const double* start_time, const double* date, const uint8_t* heap_type) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (!c->act.nev)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_upload first");
  const int64_t n = c->act.n;
  if (n > 0 && (!last_update || !last_value || !start_time || !date || !heap_type))
    return fail(LMMHIP_E_ARG, "null lazy action arrays");
  if (n >= (int64_t(1) << 30))
    return fail(LMMHIP_E_ARG, "too many actions for the lazy heap (< 2^30)");
  for (int64_t i = 0; i < n; i++)
    if (heap_type[i] > HEAP_NORMAL)
      return fail(LMMHIP_E_ARG, "unknown heap type");
  HIPCHK(hipSetDevice(c->device));
  ActDev& a = c->act;
  double* st;
  std::vector<double> d(date, date + n);
  for (int64_t i = 0; i < n; i++)
    if (heap_type[i] == HEAP_UNSET)
      d[size_t(i)] = __builtin_huge_val();
  int rc = act_alloc(c, &a.last_update, n, last_update) | act_alloc(c, &a.last_value, n, last_value) |
           act_alloc(c, &st, n, start_time) | act_alloc(c, &a.date, n, d.data()) |
           act_alloc(c, &a.htype, n, heap_type) | act_alloc<int32_t>(c, &a.due, n, nullptr) |
           act_alloc<int32_t>(c, &a.ndue, 1, nullptr) | act_alloc<int32_t>(c, &a.err, 1, nullptr);
  if (rc)
    return rc;
  a.start_time = st;
  HIPCHK(hipMemsetAsync(a.err, 0, sizeof(int32_t), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_actions_lazy_update(lmmhip_ctx* c, int model, double now, double maxmin_precision, double surf_precision,
                               int64_t n_modified, const int32_t* modified, int64_t* n_finished) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (!c->act.htype)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_lazy_upload first");
  if (model != MODEL_CPU && model != MODEL_CM02)
    return fail(LMMHIP_E_ARG, "lazy update: CPU or CM02 model");
  if (n_modified < 0 || (n_modified && !modified))
    return fail(LMMHIP_E_ARG, "bad modified-action list");
  {  // the modified set holds each action once (its hook): a duplicate would race on the action
    std::vector<uint8_t> seen(size_t(c->act.n), 0);
    for (int64_t j = 0; j < n_modified; j++) {
      if (modified[j] < 0 || modified[j] >= c->act.n)
        return fail(LMMHIP_E_ARG, "modified action out of range");
      if (seen[size_t(modified[j])]++)
        return fail(LMMHIP_E_ARG, "duplicate action in the modified list");
    }
  }
  HIPCHK(hipSetDevice(c->device));
  int32_t h[2] = {0, 0};
  HIPCHK(hipMemsetAsync(c->act.nev, 0, sizeof(int32_t), c->stream));
  if (n_modified) {
    int32_t* dmod = nullptr;
    if (int rc = scratch(c, c->rs_stage[0], n_modified, &dmod))
      return rc;
    HIPCHK(hipMemcpyAsync(dmod, modified, size_t(n_modified) * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    LAUNCH(7, -1, act_lazy_update, grid_for(n_modified, kBlock), kBlock, c->act, c->d.x, model, now,
           maxmin_precision * surf_precision, surf_precision, n_modified, dmod);
  }
  HIPCHK(hipMemcpyAsync(&h[0], c->act.nev, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(&h[1], c->act.err, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (h[1])
    return fail(LMMHIP_E_STATE, "next_occuring_event_lazy: an action got no date (DIE_IMPOSSIBLE, Model.cpp:96)");
  if (n_finished)
    *n_finished = h[0];
  return 0;
}

static int lazy_top(lmmhip_ctx* c, bool* any, double* top) {
  unsigned long long h = ~0ull;
  HIPCHK(hipMemsetAsync(c->act.umin, 0xFF, sizeof(unsigned long long), c->stream));
  if (c->act.n > 0)
    LAUNCH(7, -1, act_lazy_min, grid_for(c->act.n, kBlock), kBlock, c->act);
  HIPCHK(hipMemcpyAsync(&h, c->act.umin, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *any = h != ~0ull;
  if (*any) {
    const unsigned long long b = (h >> 63) ? (h & 0x7FFFFFFFFFFFFFFFull) : ~h;
    std::memcpy(top, &b, sizeof(*top));
  }
  return 0;
}

int lmmhip_next_event_lazy(lmmhip_ctx* c, double now, double* out) {
  if (!c || !out)
    return fail(LMMHIP_E_ARG, "null argument");
  if (!c->act.htype)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_lazy_upload first");
  HIPCHK(hipSetDevice(c->device));
  bool any = false;
  double top = 0;
  if (int rc = lazy_top(c, &any, &top))
    return rc;
  *out = any ? top - now : -1.0;  // Model.cpp:95-100
  return 0;
}

int lmmhip_actions_lazy_due(lmmhip_ctx* c, int model, double now, double surf_precision, int32_t* ids,
                            uint8_t* events, int64_t cap, int64_t* n_due) {
  if (!c || !n_due)
    return fail(LMMHIP_E_ARG, "null argument");
  if (!c->act.htype)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_lazy_upload first");
  if (model != MODEL_CPU && model != MODEL_CM02)
    return fail(LMMHIP_E_ARG, "lazy update: CPU or CM02 model");
  HIPCHK(hipSetDevice(c->device));
  *n_due = 0;
  bool any = false;
  double top = 0;
  if (int rc = lazy_top(c, &any, &top))
    return rc;
  if (!any || !(std::fabs(top - now) < surf_precision))  // the heap loop's first test
    return 0;
  int32_t h = 0;
  HIPCHK(hipMemsetAsync(c->act.ndue, 0, sizeof(int32_t), c->stream));
  LAUNCH(7, -1, act_lazy_due, grid_for(c->act.n, kBlock), kBlock, c->act, model, now, surf_precision);
  HIPCHK(hipMemcpyAsync(&h, c->act.ndue, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (h > cap || (h && (!ids || !events)))
    return fail(LMMHIP_E_ARG, "lazy due: output capacity too small (the heap entries are already popped)");
  if (h) {
    std::vector<int32_t> v(static_cast<size_t>(h));
    std::vector<uint8_t> e(static_cast<size_t>(c->act.n));
    HIPCHK(hipMemcpyAsync(v.data(), c->act.due, size_t(h) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(e.data(), c->act.events, size_t(c->act.n), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    std::sort(v.begin(), v.end());  // deterministic order (the reference pops by (date, Action*))
    for (int32_t k = 0; k < h; k++) {
      ids[k] = v[size_t(k)];
      events[k] = e[size_t(v[size_t(k)])];
    }
  }
  *n_due = h;
  return 0;
}

int lmmhip_actions_lazy_download(lmmhip_ctx* c, double* last_update, double* last_value, double* date,
                                 uint8_t* heap_type) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  if (!c->act.htype)
    return fail(LMMHIP_E_STATE, "lmmhip_actions_lazy_upload first");
  HIPCHK(hipSetDevice(c->device));
  const size_t n = size_t(c->act.n);
  if (n) {
    if (last_update)
      HIPCHK(hipMemcpyAsync(last_update, c->act.last_update, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (last_value)
      HIPCHK(hipMemcpyAsync(last_value, c->act.last_value, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (date)
      HIPCHK(hipMemcpyAsync(date, c->act.date, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (heap_type)
      HIPCHK(hipMemcpyAsync(heap_type, c->act.htype, n, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_launch_profile(lmmhip_ctx* c, int* slot, int* round, float* ms, int cap) {
  if (!c)
    return fail(LMMHIP_E_ARG, "null context");
  int n = int(c->launch_ms.size());
  for (int i = 0; i < n && i < cap; i++) {
    slot[i] = c->launch_slot[size_t(i)];
    round[i] = c->launch_round[size_t(i)];
    ms[i] = c->launch_ms[size_t(i)];
  }
  return n;
}

int lmmhip_round_profile(lmmhip_ctx* c, int64_t* alive_vars, int64_t* alive_elems, int cap) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  const int64_t nV = c->d.nV;
  std::vector<int32_t> fr(size_t(nV > 0 ? nV : 1));
  std::vector<uint32_t> vp(size_t(nV) + 1);
  HIPCHK(hipSetDevice(c->device));
  if (nV) {
    // maxmin: vstate = exit round + 1 (0 = never fixed); fair bottleneck: fixr = last listed round
    const int32_t* src = c->last_kind == LMMHIP_KIND_MAXMIN ? c->d.vstate : c->d.fixr;
    HIPCHK(hipMemcpyAsync(fr.data(), src, sizeof(int32_t) * nV, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(vp.data(), c->d.var_ptr, sizeof(uint32_t) * (nV + 1), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->last_kind == LMMHIP_KIND_MAXMIN)
    for (auto& f : fr)
      f -= 1;
  const int R = int(c->stats.rounds);
  // a variable is alive in rounds 0..fixr (inclusive); -1 = never processed
  std::vector<int64_t> dv(size_t(R) + 2, 0), de(size_t(R) + 2, 0);
  for (int64_t v = 0; v < nV; v++) {
    int f = fr[size_t(v)];
    if (f < 0)
      continue;
    if (f > R)
      f = R;
    dv[size_t(f)] += 1;
    de[size_t(f)] += vp[size_t(v) + 1] - vp[size_t(v)];
  }
  int64_t av = 0, ae = 0;
  for (int r = R; r >= 0; r--) {  // suffix sums
    av += dv[size_t(r)];
    ae += de[size_t(r)];
    if (r < cap) {
      alive_vars[r] = av;
      alive_elems[r] = ae;
    }
  }
  return R;
}

int lmmhip_vote_profile(lmmhip_ctx* c, int64_t* rows, int64_t* elems, int cap) {
  if (!c || !c->vstat)
    return fail(LMMHIP_E_STATE, "no profiled maxmin solve");
  const int R = int(std::min<int64_t>(c->stats.rounds, kStatRounds));
  std::vector<int32_t> h(size_t(2) * kStatRounds * kMaxBlocks);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpy(h.data(), c->vstat, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost));
  for (int r = 0; r < R && r < cap; r++) {
    int64_t a = 0, b = 0;
    for (int k = 0; k < kDiagSlot; k++) {
      a += h[2 * (size_t(r) * kMaxBlocks + k)];
      b += h[2 * (size_t(r) * kMaxBlocks + k) + 1];
    }
    rows[r] = a;
    elems[r] = b;
  }
  return R;
}

int lmmhip_vote_diag_profile(lmmhip_ctx* c, int64_t* out8, int cap) {
  if (!c || !c->vstat)
    return fail(LMMHIP_E_STATE, "no profiled maxmin solve");
  const int R = int(std::min<int64_t>(c->stats.rounds, kStatRounds));
  std::vector<int32_t> h(size_t(2) * kStatRounds * kMaxBlocks);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpy(h.data(), c->vstat, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost));
  for (int r = 0; r < R && r < cap; r++)
    for (int k = 0; k < 8; k++)
      out8[8 * r + k] = h[2 * (size_t(r) * kMaxBlocks + kDiagSlot) + k];
  return R;
}

int lmmhip_get_values(lmmhip_ctx* c, double* out) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  if (!out && c->d.nV)
    return fail(LMMHIP_E_ARG, "null output");
  HIPCHK(hipSetDevice(c->device));
  if (c->d.nV)
    HIPCHK(hipMemcpyAsync(out, c->d.x, sizeof(double) * c->d.nV, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_get_var_rounds(lmmhip_ctx* c, int32_t* out) {
  if (!c || !c->solved || c->last_kind != LMMHIP_KIND_MAXMIN)
    return fail(LMMHIP_E_STATE, "no max-min solve to read rounds from");
  if (!out && c->d.nV)
    return fail(LMMHIP_E_ARG, "null output");
  HIPCHK(hipSetDevice(c->device));
  if (c->d.nV)
    HIPCHK(hipMemcpyAsync(out, c->d.vstate, sizeof(int32_t) * c->d.nV, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_get_saturated(lmmhip_ctx* c, uint8_t* sat) {
  if (!c || !c->uploaded || !c->solved)
    return fail(LMMHIP_E_STATE, "no solved system");
  if (!sat && c->d.nC)
    return fail(LMMHIP_E_ARG, "null output");
  HIPCHK(hipSetDevice(c->device));
  if (c->d.nC) {
    uint8_t* o = nullptr;
    if (int rc = scratch(c, c->sat_out, c->d.nC, &o))
      return rc;
    hipLaunchKernelGGL(mm_saturated, dim3(grid_for(c->d.nC, kBlock / kWave)), dim3(kBlock), 0, c->stream, c->d,
                       c->last_prec, int(c->last_kind == LMMHIP_KIND_FAIR_BOTTLENECK), o);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(sat, o, size_t(c->d.nC), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_components(lmmhip_ctx* c, int32_t* var_label, int32_t* cnst_label, int64_t* ncomp) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  if (!ncomp || (c->d.nV && !var_label) || (c->d.nC && !cnst_label))
    return fail(LMMHIP_E_ARG, "null output");
  HIPCHK(hipSetDevice(c->device));
  const int64_t nv = c->d.nV, n = int64_t(c->d.nV) + int64_t(c->d.nC);
  *ncomp = 0;
  if (n == 0)
    return 0;
  if (n > INT32_MAX)  // union-find node ids are int32 (lmm_cc_kernels.hpp)
    return fail(LMMHIP_E_ARG, "components: variables + constraints exceed 2^31 - 1");
  int32_t *par = nullptr, *out = nullptr;
  int64_t *flag = nullptr, *rank = nullptr;
  if (int rc = scratch(c, c->cc_par, n, &par))
    return rc;
  if (int rc = scratch(c, c->cc_flag, n, &flag))
    return rc;
  if (int rc = scratch(c, c->cc_rank, n, &rank))
    return rc;
  if (int rc = scratch(c, c->cc_out, n, &out))
    return rc;
  hipLaunchKernelGGL(cc_init, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, c->stream, par, n);
  HIPCHK(hipGetLastError());
  if (nv > 0) {
    hipLaunchKernelGGL(cc_hook, dim3(grid_for(nv, kBlock)), dim3(kBlock), 0, c->stream, c->d, par);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(cc_root, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, c->stream, par, n, flag);
  HIPCHK(hipGetLastError());
  if (int rc = dev_scan(c, flag, rank, n))
    return rc;
  hipLaunchKernelGGL(cc_label, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, c->stream, par, rank, nv, n, out,
                     out + nv);
  HIPCHK(hipGetLastError());
  int rc = 0;
  const int64_t last = read_i64(c, rank + n - 1, &rc) + read_i64(c, flag + n - 1, &rc);
  if (rc)
    return rc;
  if (nv)
    HIPCHK(hipMemcpyAsync(var_label, out, size_t(nv) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  if (n > nv)
    HIPCHK(hipMemcpyAsync(cnst_label, out + nv, size_t(n - nv) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *ncomp = last;
  return 0;
}

int lmmhip_get_touched_vars(lmmhip_ctx* c, int32_t* ids, int64_t cap, int64_t* n) {
  if (!c || !c->uploaded || !n)
    return fail(LMMHIP_E_STATE, "no system uploaded / null count");
  const int64_t nv = c->d.nV;
  *n = nv;
  if (!ids)
    return 0;  // size query
  if (cap < nv)
    return fail(LMMHIP_E_ARG, "touched vars: output capacity below the system's variable count");
  HIPCHK(hipSetDevice(c->device));
  if (!c->res_flat) {  // lmmhip_upload: the caller's ids are the dense CSR indices
    for (int64_t v = 0; v < nv; v++)
      ids[v] = int32_t(v);
    return 0;
  }
  int32_t* o = nullptr;
  if (int rc = scratch(c, c->tv_out, nv, &o))
    return rc;
  const int64_t ns = c->res_flat_nv;
  if (ns) {
    hipLaunchKernelGGL(rs_touched, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, c->stream, ns,
                       static_cast<const int64_t*>(c->rs_vm.p), static_cast<const int64_t*>(c->rs_dv.p), o);
    HIPCHK(hipGetLastError());
  }
  if (nv)
    HIPCHK(hipMemcpyAsync(ids, o, size_t(nv) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int lmmhip_values_device_ptr(lmmhip_ctx* c, const double** dptr) {
  if (!c || !c->uploaded)
    return fail(LMMHIP_E_STATE, "no system uploaded");
  *dptr = c->d.x;
  return 0;
}

int lmmhip_get_stats(lmmhip_ctx* c, lmmhip_stats* out) {
  if (!c || !out)
    return fail(LMMHIP_E_ARG, "null argument");
  *out = c->stats;
  return 0;
}

}  // extern "C"
