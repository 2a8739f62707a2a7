"""Multi-GPU layer: one process per GPU, work split so that no collective sits on
the solve's data path.

* Independent systems (a parameter sweep, or the batched systems of config C3): contiguous blocks of
  systems per rank balanced by nnz (`balanced_blocks`); each rank solves its block as one device launch
  sequence (`lmm.solve_batch`).  Weak scaling, nothing exchanged during the solve.
* Connected components of one system: the closure System::update_modified_set walks
  (maxmin.cpp:898-922) splits a system into independent sub-systems.  `device_components` labels them on
  the device (lmmhip_components, union-find over the flattened system; `System.components()` labels a
  System's own device flatten), `pack_components` bin-packs them on the
  ranks by nnz, every rank solves its share (`solve_components`), and one all-reduce(SUM) of the disjoint
  per-rank value vectors assembles the result.  A random C2 system or a fat tree carrying random flows
  is one giant component: such a system is solved by replicas only.
* FairBottleneck sharded over ranks (config C5: one system, an exchange between the phases of each
  round, `FbShardPlan` + `fb_solve_sharded`, device side lmmhip_fb_shard_*): each shard holds an
  nnz-balanced block of the variables (with every constraint) and OWNS an nnz-balanced block of the
  constraints, i.e. their full element lists in the reference's enabled_element_set_ order.  Per round:
  all-reduce(SUM) of the per-constraint listed counts (integers, exact), all-gather of the variables'
  increments mu, the owners' per-element double_update chains (fair_bottleneck.cpp:107-127, operation for
  operation), all-gather of the owned remaining values.  Every shard takes the same erase decisions from
  the same values, and the result is bit-identical to the one-context solve and to the reference.
* The simulation step's only cross-rank dependency is the next event date,
  `Model::next_occuring_event` (Model.cpp:40-129): one all-reduce(MIN) of a scalar (`next_event_date`).

Launch as `torchrun --nproc-per-node N` with MASTER_ADDR=127.0.0.1; the same code runs on gloo (CPU
tests) and nccl (RCCL over xGMI).
"""
import ctypes as ct
import os
from collections import namedtuple

import numpy as np

from simgrid_amd import lmm

# csc_order: each constraint's elements as CSR indices, constraint-major (lmm_flat_export_order: the
# reference's enabled_element_set_ order for FairBottleneck, whose per-element chain depends on it)
Flat = namedtuple("Flat", "var_ptr cnst_idx weight penalty vbound cbound cflags var_ids csc_order",
                  defaults=(None,))


def dist_env():
    """(rank, world, local_rank) from the torchrun environment (1 process when unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


# ---- partitioning -----------------------------------------------------------------------------

def balanced_blocks(weights, parts):
    """Split items 0..n-1 into `parts` contiguous blocks minimising the heaviest block (binary search
    on the block capacity, greedy fill).  Returns the parts+1 block boundaries."""
    w = np.asarray(weights, dtype=np.int64)
    n = len(w)
    if parts <= 0:
        raise ValueError("parts must be positive")
    pre = np.concatenate([[0], np.cumsum(w)])

    def cut(cap):
        bounds, lo = [0], 0
        for _ in range(parts):
            hi = int(np.searchsorted(pre, pre[lo] + cap, side="right")) - 1
            hi = max(hi, min(lo + 1, n)) if lo < n else n
            bounds.append(hi)
            lo = hi
        return bounds if bounds[-1] == n else None

    lo, hi = int(w.max(initial=0)), int(pre[-1])
    while lo < hi:
        mid = (lo + hi) // 2
        if cut(mid) is None:
            lo = mid + 1
        else:
            hi = mid
    return cut(lo)


def pack_components(sizes, parts):
    """Longest-processing-time bin packing: component i -> rank, heaviest first onto the lightest rank."""
    sizes = np.asarray(sizes, dtype=np.int64)
    owner = np.empty(len(sizes), dtype=np.int64)
    load = np.zeros(parts, dtype=np.int64)
    for i in np.argsort(-sizes, kind="stable"):
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += sizes[i]
    return owner


# ---- flattened systems and their components --------------------------------------------------

def export_flat(s):
    """The device input of System `s`'s next solve (lmm_flat_export)."""
    L = lmm.lib()
    cnt = (ct.c_int64 * 3)()
    if L.lmm_flat_export(s.h, cnt, None, None, None, None, None, None, None, None) != 0:
        raise lmm.LmmError(L.lmm_last_error().decode())
    nv, nc, nnz = cnt[0], cnt[1], cnt[2]
    f = Flat(np.empty(nv + 1, np.int64), np.empty(nnz, np.int32), np.empty(nnz, np.float64),
             np.empty(nv, np.float64), np.empty(nv, np.float64), np.empty(nc, np.float64), np.empty(nc, np.uint8),
             np.empty(nv, np.int64))

    def p(a, t):
        return a.ctypes.data_as(ct.POINTER(t))

    if L.lmm_flat_export(s.h, cnt, p(f.var_ptr, ct.c_int64), p(f.cnst_idx, ct.c_int32), p(f.weight, ct.c_double),
                         p(f.penalty, ct.c_double), p(f.vbound, ct.c_double), p(f.cbound, ct.c_double),
                         p(f.cflags, ct.c_uint8), p(f.var_ids, ct.c_int64)) != 0:
        raise lmm.LmmError(L.lmm_last_error().decode())
    order = np.empty(nnz, np.int64)
    if L.lmm_flat_export_order(s.h, nnz, p(order, ct.c_int64)) != 0:
        raise lmm.LmmError(L.lmm_last_error().decode())
    return f._replace(csc_order=order)


def csc_order_of(f):
    """`f.csc_order`, or ascending CSR order per constraint when the flat carries none."""
    if f.csc_order is not None:
        return f.csc_order
    return np.argsort(f.cnst_idx, kind="stable").astype(np.int64)


def device_components(f, device=None):
    """Connected components of flat `f`'s variable-constraint graph on the device (lmmhip_components:
    lock-free union-find, maxmin.cpp:898-922's closure for every component at once): (label per variable,
    label per constraint, count), labels in the order of each component's smallest node (variables first)."""
    L = lmm.lib()
    if device is None:
        import torch

        device = torch.cuda.current_device()
    ctx = ct.c_void_p()
    if L.lmmhip_ctx_create(device, ct.byref(ctx)) != 0:
        raise lmm.LmmError(L.lmmhip_last_error().decode())
    try:
        def p(a, t):
            return a.ctypes.data_as(ct.POINTER(t))

        nv, nc, nnz = len(f.penalty), len(f.cbound), len(f.cnst_idx)
        if L.lmmhip_upload(ctx, nv, nc, nnz, p(f.var_ptr, ct.c_int64), p(f.cnst_idx, ct.c_int32),
                           p(f.weight, ct.c_double), p(f.penalty, ct.c_double), p(f.vbound, ct.c_double),
                           p(f.cbound, ct.c_double), p(f.cflags, ct.c_uint8)) != 0:
            raise lmm.LmmError(L.lmmhip_last_error().decode())
        return lmm.ctx_components(ctx, nv, nc)
    finally:
        L.lmmhip_ctx_destroy(ctx)


def components_host(f):
    """Connected components of the variable-constraint graph on the host (scipy): (label per variable,
    label per constraint, count).  Constraints without an element get labels of their own.  The checker of
    the device labelling and the labeler of the CPU-only tests; the product path is device_components."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    nv, nc = len(f.penalty), len(f.cbound)
    rows = np.repeat(np.arange(nv, dtype=np.int64), np.diff(f.var_ptr))
    g = coo_matrix((np.ones(len(rows), np.int8), (rows, nv + f.cnst_idx.astype(np.int64))),
                   shape=(nv + nc, nv + nc))
    n, lab = connected_components(g, directed=False)
    return lab[:nv], lab[nv:], n


def sub_flat(f, var_mask, cnst_mask):
    """The part of `f` on the selected variables / constraints (a union of whole components),
    re-indexed densely.  Returns (flat, dense indices of its variables in f)."""
    vsel = np.nonzero(var_mask)[0]
    cmap = np.full(len(f.cbound), -1, np.int64)
    csel = np.nonzero(cnst_mask)[0]
    cmap[csel] = np.arange(len(csel))
    lens = np.diff(f.var_ptr)[vsel]
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    eidx = np.arange(int(ptr[-1]), dtype=np.int64) + np.repeat(f.var_ptr[vsel] - ptr[:-1], lens)
    ci = cmap[f.cnst_idx[eidx]]
    if np.any(ci < 0):
        raise ValueError("selection is not a union of components")
    order = None
    if f.csc_order is not None:  # the kept elements in their old relative order (constraint ids stay monotone)
        new_of = np.full(len(f.cnst_idx), -1, np.int64)
        new_of[eidx] = np.arange(len(eidx), dtype=np.int64)
        order = new_of[f.csc_order]
        order = order[order >= 0]
    out = Flat(ptr, ci.astype(np.int32), f.weight[eidx],
               f.penalty[vsel], f.vbound[vsel], f.cbound[csel], f.cflags[csel], f.var_ids[vsel], order)
    return out, vsel


def device_solve_flat(f, kind, precision=None, device=None):
    """Solve a flattened system on the current HIP device with the lmmhip_* ABI: dense values."""
    L = lmm.lib()
    prec = lmm.get_precision() if precision is None else precision
    if device is None:
        import torch

        device = torch.cuda.current_device()
    ctx = ct.c_void_p()
    if L.lmmhip_ctx_create(device, ct.byref(ctx)) != 0:
        raise lmm.LmmError(L.lmmhip_last_error().decode())
    try:
        def p(a, t):
            return a.ctypes.data_as(ct.POINTER(t))

        nv, nc, nnz = len(f.penalty), len(f.cbound), len(f.cnst_idx)
        order = None if f.csc_order is None else p(np.ascontiguousarray(f.csc_order, np.int64), ct.c_int64)
        if L.lmmhip_upload2(ctx, nv, nc, nnz, p(f.var_ptr, ct.c_int64), p(f.cnst_idx, ct.c_int32),
                            p(f.weight, ct.c_double), p(f.penalty, ct.c_double), p(f.vbound, ct.c_double),
                            p(f.cbound, ct.c_double), p(f.cflags, ct.c_uint8), order) != 0 \
                or L.lmmhip_solve(ctx, kind, prec) != 0:
            raise lmm.LmmError(L.lmmhip_last_error().decode())
        x = np.empty(nv, np.float64)
        if L.lmmhip_get_values(ctx, p(x, ct.c_double)) != 0:
            raise lmm.LmmError(L.lmmhip_last_error().decode())
        return x
    finally:
        L.lmmhip_ctx_destroy(ctx)


class DeviceBatch:
    """Independent max-min systems (a parameter sweep) as ONE block-diagonal device
    system: their flattened systems concatenated, uploaded once (lmmhip_upload) and declared a batch
    (lmmhip_set_batch), so every solve() runs one workgroup per system with the system in LDS
    (lmm_batch_kernels.hpp).  Inputs stay resident in HBM across solves."""

    def __init__(self, systems, precision=None, device=None):
        import torch

        L = lmm.lib()
        self.L = L
        self.prec = lmm.get_precision() if precision is None else precision
        flats = [export_flat(s) for s in systems]
        nvs = np.array([len(f.penalty) for f in flats], np.int64)
        ncs = np.array([len(f.cbound) for f in flats], np.int64)
        self.var_off = np.concatenate([[0], np.cumsum(nvs)]).astype(np.int64)
        self.cnst_off = np.concatenate([[0], np.cumsum(ncs)]).astype(np.int64)
        nnzs = np.array([len(f.cnst_idx) for f in flats], np.int64)
        eoff = np.concatenate([[0], np.cumsum(nnzs)])
        var_ptr = np.concatenate([f.var_ptr[:-1] + eoff[i] for i, f in enumerate(flats)] + [[eoff[-1]]]).astype(np.int64)
        cnst_idx = np.concatenate([f.cnst_idx + self.cnst_off[i] for i, f in enumerate(flats)]).astype(np.int32)
        cat = lambda name, dt: np.ascontiguousarray(np.concatenate([getattr(f, name) for f in flats]), dtype=dt)
        self.arrays = (var_ptr, cnst_idx, cat("weight", np.float64), cat("penalty", np.float64),
                       cat("vbound", np.float64), cat("cbound", np.float64), cat("cflags", np.uint8))
        self.var_ids = [f.var_ids for f in flats]
        self.n_var, self.n_cnst, self.nnz = int(self.var_off[-1]), int(self.cnst_off[-1]), int(len(cnst_idx))
        self.ctx = ct.c_void_p()
        dev = torch.cuda.current_device() if device is None else device
        if L.lmmhip_ctx_create(dev, ct.byref(self.ctx)) != 0:
            raise lmm.LmmError(L.lmmhip_last_error().decode())

        def p(a, t):
            return a.ctypes.data_as(ct.POINTER(t))

        vp, ci, w, pen, vb, cb, cf = self.arrays
        self._check(L.lmmhip_upload(self.ctx, self.n_var, self.n_cnst, self.nnz, p(vp, ct.c_int64),
                                    p(ci, ct.c_int32), p(w, ct.c_double), p(pen, ct.c_double), p(vb, ct.c_double),
                                    p(cb, ct.c_double), p(cf, ct.c_uint8)))
        self._check(L.lmmhip_set_batch(self.ctx, len(flats), p(self.var_off, ct.c_int64),
                                       p(self.cnst_off, ct.c_int64)))

    def _check(self, rc):
        if rc != 0:
            raise lmm.LmmError(self.L.lmmhip_last_error().decode())

    def solve(self):
        self._check(self.L.lmmhip_solve(self.ctx, 0, self.prec))

    def stats(self):
        st = lmm.LmmhipStats()
        self._check(self.L.lmmhip_get_stats(self.ctx, ct.byref(st)))
        return dict(rounds=st.rounds, device_ms=st.device_ms, n_var=st.n_var, n_cnst=st.n_cnst, nnz=st.nnz)

    def values(self):
        """Dense values of every system (concatenated, the systems' dense orders)."""
        x = np.empty(self.n_var, np.float64)
        self._check(self.L.lmmhip_get_values(self.ctx, x.ctypes.data_as(ct.POINTER(ct.c_double))))
        return x

    def saturated(self):
        """The device's saturated set of the last solve (lmmhip_get_saturated: SURVEY.md A.6, maxmin.cpp:948-961),
        one flag per dense constraint of the concatenated systems."""
        out = np.empty(self.n_cnst, np.uint8)
        self._check(self.L.lmmhip_get_saturated(self.ctx, out.ctypes.data_as(ct.POINTER(ct.c_uint8))))
        return out.astype(bool)

    def flat(self):
        """The concatenated flattened system as a Flat (dense ids; var_ids / csc_order unset)."""
        vp, ci, w, pen, vb, cb, cf = self.arrays
        return Flat(vp, ci, w, pen, vb, cb, cf, None, None)

    def close(self):
        if self.ctx:
            self.L.lmmhip_ctx_destroy(self.ctx)
            self.ctx = None


# ---- collectives ------------------------------------------------------------------------------

class LocalExchange:
    """World of one process: the collectives are identities."""
    rank, world = 0, 1

    def sum(self, x):
        return x

    def min(self, x):
        return x

    def allreduce_(self, buf, op):
        pass

    def allgather_(self, buf, n):
        pass

    def gather_pairs_(self, buf, packs):
        pass  # every shard of the only rank wrote its chunk of buf itself


class DistExchange:
    """torch.distributed collectives on numpy data (gloo: CPU tensors, nccl/RCCL: device tensors)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.wire_bytes = 0  # bytes this rank contributed to the gathers (the FairBottleneck exchange's traffic)

    def _reduce(self, x, op):
        import torch

        t = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64)).to(self.device)
        self.dist.all_reduce(t, op=op, group=self.group)
        return t.cpu().numpy()

    def sum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM)

    def min(self, x):
        return self._reduce(x, self.dist.ReduceOp.MIN)

    def allreduce_(self, buf, op):
        """In place on a torch tensor (on this backend's device) or a numpy array; op "sum" / "min"."""
        import torch

        rop = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MIN
        if isinstance(buf, torch.Tensor):
            if buf.device.type == self.device.type:
                self.dist.all_reduce(buf, op=rop, group=self.group)
            else:  # e.g. device shards over gloo: reduce a copy on the backend's device
                t = buf.to(self.device)
                self.dist.all_reduce(t, op=rop, group=self.group)
                buf.copy_(t)
        else:
            t = torch.as_tensor(np.asarray(buf)).to(self.device)
            self.dist.all_reduce(t, op=rop, group=self.group)
            buf[...] = t.cpu().numpy()

    def allgather_(self, buf, n):
        """In place: rank r's chunk buf[r*n : (r+1)*n] to every rank (buf holds world * n items; a torch
        tensor on this backend's device or elsewhere, or a numpy array)."""
        import torch

        is_np = not isinstance(buf, torch.Tensor)
        t = torch.as_tensor(buf) if is_np else buf
        work = t if t.device.type == self.device.type else t.to(self.device)
        mine = work[self.rank * n:(self.rank + 1) * n].clone()
        self.wire_bytes += mine.numel() * mine.element_size()
        if self.device.type == "cuda":
            self.dist.all_gather_into_tensor(work, mine, group=self.group)
        else:
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            self.dist.all_gather(parts, mine, group=self.group)
            work.copy_(torch.cat(parts))
        if work is not t:
            t.copy_(work)


    def gather_pairs_(self, buf, packs):
        """Scatter every rank's (position, value) pairs into `buf` (the gathered mu of the FairBottleneck
        shards): packs = [(pos, val, count)] of this rank's shards (torch tensors or numpy arrays; count a
        1-element array / tensor).  Counts all-gathered first, then the pairs padded to the largest count:
        12 B per listed variable on the wire instead of 8 B per variable of the whole system."""
        import torch

        dev = self.device
        lp = len(packs)  # the same on every rank (FbShardPlan: len(shards) parts per rank)
        if lp == 0:
            return
        cnt = torch.cat([torch.as_tensor(c).to(dev, torch.int64).reshape(1) for _, _, c in packs])
        allc = torch.empty(self.world * lp, dtype=torch.int64, device=dev)
        self._gather(allc, cnt)
        allc = allc.cpu()  # the round's one host synchronisation: the padded length and this rank's counts
        k = int(allc.max())
        if k == 0:
            return
        mine = allc[self.rank * lp:(self.rank + 1) * lp].tolist()
        spos = torch.full((lp * k,), -1, dtype=torch.int32, device=dev)
        sval = torch.zeros(lp * k, dtype=torch.float64, device=dev)
        for i, (pos, val, _) in enumerate(packs):
            n = int(mine[i])
            if n:
                spos[i * k:i * k + n] = torch.as_tensor(pos[:n]).to(dev, torch.int32)
                sval[i * k:i * k + n] = torch.as_tensor(val[:n]).to(dev, torch.float64)
        rpos = torch.empty(self.world * lp * k, dtype=torch.int32, device=dev)
        rval = torch.empty(self.world * lp * k, dtype=torch.float64, device=dev)
        self._gather(rpos, spos)
        self._gather(rval, sval)
        ok = rpos >= 0
        idx, vals = rpos[ok].long(), rval[ok]
        if isinstance(buf, torch.Tensor):
            buf[idx.to(buf.device)] = vals.to(buf.device)
        else:
            buf[idx.cpu().numpy()] = vals.cpu().numpy()

    def _gather(self, out, mine):
        import torch

        self.wire_bytes += mine.numel() * mine.element_size()
        if self.device.type == "cuda":
            self.dist.all_gather_into_tensor(out, mine, group=self.group)
        else:
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            self.dist.all_gather(parts, mine, group=self.group)
            out.copy_(torch.cat(parts))


def next_event_date(local_min, exchange):
    """Model::next_occuring_event across ranks (Model.cpp:40-129): every rank's earliest date, -1 = none."""
    v = float(local_min) if local_min >= 0 else np.inf
    m = float(exchange.min(np.array([v]))[0])
    return -1.0 if m == np.inf else m


# ---- sharded solves ---------------------------------------------------------------------------

def solve_components(f, kind, exchange, solve_flat=None, labeler=None):
    """Solve flattened system `f` (identical on every rank) with its connected components spread over
    the ranks.  Returns the dense value vector (all ranks get all values).  `solve_flat(sub, kind)`
    defaults to the device solver, `labeler(f)` to the device labelling (device_components)."""
    solve_flat = solve_flat or device_solve_flat
    var_lab, cnst_lab, n = (labeler or device_components)(f)
    nnz = np.bincount(np.repeat(var_lab, np.diff(f.var_ptr)), minlength=n) + np.bincount(var_lab, minlength=n)
    owner = pack_components(nnz, exchange.world)
    mine = owner == exchange.rank
    x = np.zeros(len(f.penalty), np.float64)
    if np.any(mine[var_lab]):
        sub, idx = sub_flat(f, mine[var_lab], mine[cnst_lab])
        x[idx] = solve_flat(sub, kind)
    return exchange.sum(x)


def solve_batch_block(build, n_systems, weights, exchange, solve=None):
    """Independent systems 0..n-1 spread over ranks in nnz-balanced contiguous blocks; `build(i)`
    makes system i on this rank.  Returns {i: system} of this rank's block, solved."""
    bounds = balanced_blocks(weights, exchange.world)
    lo, hi = bounds[exchange.rank], bounds[exchange.rank + 1]
    mine = {i: build(i) for i in range(lo, hi)}
    if mine:
        (solve or lmm.solve_batch)(list(mine.values()))
    return mine


_FB_STREAMS = {}


def _fb_stream():
    """The process's FairBottleneck shard stream on the current device (created once)."""
    import torch

    dev = torch.cuda.current_device()
    if dev not in _FB_STREAMS:
        _FB_STREAMS[dev] = torch.cuda.Stream(dev)
    return _FB_STREAMS[dev]


class FbShardPlan:
    """How a FairBottleneck system (flat `f`, with its csc_order) splits over `parts` shards: shard p holds
    the variable block [vb[p], vb[p+1]) (nnz-balanced) and owns the constraint block [cb[p], cb[p+1])
    (balanced by element count: the owners' chains are per-element work).  The gathered vectors are padded
    per shard: variable v of shard p sits at p * Pv + (v - vb[p]) of the mu vector, constraint k of owner q
    at q * Pc + (k - cb[q]) of the remaining vector, so each shard's part is one contiguous chunk."""

    def __init__(self, f, parts):
        nv, nc = len(f.penalty), len(f.cbound)
        self.f, self.parts, self.nv, self.nc = f, parts, nv, nc
        self.vb = balanced_blocks(np.diff(f.var_ptr) + 1, parts)
        cdeg = np.bincount(f.cnst_idx, minlength=nc).astype(np.int64)
        self.cb = balanced_blocks(cdeg + 1, parts)
        self.Pv = max(1, max(hi - lo for lo, hi in zip(self.vb, self.vb[1:])))
        self.Pc = max(1, max(hi - lo for lo, hi in zip(self.cb, self.cb[1:])))
        self.mu_len, self.rem_len = parts * self.Pv, parts * self.Pc
        vpart = np.repeat(np.arange(parts), np.diff(self.vb))
        self.vpos = (vpart * self.Pv + np.arange(nv) - np.asarray(self.vb)[vpart]).astype(np.int64)
        cpart = np.repeat(np.arange(parts), np.diff(self.cb))
        self.cpos = (cpart * self.Pc + np.arange(nc) - np.asarray(self.cb)[cpart]).astype(np.int32)
        self.order = csc_order_of(f)
        self.cptr = np.concatenate([[0], np.cumsum(cdeg)]).astype(np.int64)
        self.rows = np.repeat(np.arange(nv, dtype=np.int64), np.diff(f.var_ptr))

    def variables(self, p):
        """(flat of shard p's variable rows with every constraint, dense indices of those variables)."""
        mask = np.zeros(self.nv, bool)
        mask[self.vb[p]:self.vb[p + 1]] = True
        return sub_flat(self.f, mask, np.ones(self.nc, bool))

    def owned(self, p):
        """Shard p's owned constraints: (global ids, element offsets, element variable positions in the
        gathered mu vector, weights), the elements in the reference's order."""
        lo, hi = self.cb[p], self.cb[p + 1]
        e = self.order[self.cptr[lo]:self.cptr[hi]]
        return (np.arange(lo, hi, dtype=np.int32), (self.cptr[lo:hi + 1] - self.cptr[lo]).astype(np.int64),
                self.vpos[self.rows[e]].astype(np.int32), np.ascontiguousarray(self.f.weight[e]))

    def mu_off(self, p):
        return p * self.Pv


class FbGather:
    """The gathered vectors shared by the shards of one process (each writes its own chunk): mu and
    remaining, torch device tensors (device shards) or numpy arrays."""

    def __init__(self, plan, device=True, stream=None):
        if device:
            import torch

            with torch.cuda.stream(stream or _fb_stream()):
                self.xmu = torch.zeros(plan.mu_len, dtype=torch.float64, device="cuda")
                self.xrem = torch.zeros(plan.rem_len, dtype=torch.float64, device="cuda")
        else:
            self.xmu = np.zeros(plan.mu_len)
            self.xrem = np.zeros(plan.rem_len)
        self.Pv, self.Pc = plan.Pv, plan.Pc


class DeviceFbShard:
    """Shard p of a FairBottleneck plan on the current HIP device: its variable block (lmmhip_upload2), its
    owned constraints (lmmhip_fb_shard_owner) and the four phases of lmmhip_fb_shard_step.  The exchange
    buffers are torch tensors on the device (RCCL reduces / gathers them in place, stream-ordered with the
    solver's kernels): the context launches on `stream`, by default the process's dedicated shard stream
    `_fb_stream()`, on which fb_solve_sharded also runs the exchanges."""

    def __init__(self, plan, p, gather, precision=None, stream=None):
        import torch

        L = lmm.lib()
        f, self.idx = plan.variables(p)
        self.L, self.n, self.gather = L, len(f.penalty), gather
        self.mu_off = plan.mu_off(p)
        self.ctx = ct.c_void_p()
        if L.lmmhip_ctx_create(torch.cuda.current_device(), ct.byref(self.ctx)) != 0:
            raise lmm.LmmError(L.lmmhip_last_error().decode())

        def ptr(a, t):
            return a.ctypes.data_as(ct.POINTER(t))

        nc = len(f.cbound)
        # One torch stream shared by every shard of the process: the context's kernels and the torch-side
        # reductions / gathers of the exchange buffers (fb_solve_sharded runs them on it) are then
        # stream-ordered.  Any torch stream works, torch's default stream (handle 0) included.
        self.stream = _fb_stream() if stream is None else stream
        self._check(L.lmmhip_ctx_set_stream(self.ctx, ct.c_void_p(self.stream.cuda_stream)))
        order = np.ascontiguousarray(f.csc_order, np.int64)
        self._check(L.lmmhip_upload2(self.ctx, self.n, nc, len(f.cnst_idx), ptr(f.var_ptr, ct.c_int64),
                                     ptr(f.cnst_idx, ct.c_int32), ptr(f.weight, ct.c_double), ptr(f.penalty, ct.c_double),
                                     ptr(f.vbound, ct.c_double), ptr(f.cbound, ct.c_double), ptr(f.cflags, ct.c_uint8),
                                     ptr(order, ct.c_int64)))
        oc, optr, ovar, ow = plan.owned(p)
        cpos = np.ascontiguousarray(plan.cpos, np.int32)
        self._check(L.lmmhip_fb_shard_owner(self.ctx, len(oc), ptr(oc, ct.c_int32), ptr(optr, ct.c_int64),
                                            ptr(ovar, ct.c_int32), ptr(ow, ct.c_double), ptr(cpos, ct.c_int32),
                                            plan.mu_len, plan.rem_len))
        with torch.cuda.stream(self.stream):
            self.xnb = torch.zeros(nc + 1, dtype=torch.int32, device="cuda")
        self.prec = lmm.get_precision() if precision is None else precision
        self.begin()

    def begin(self):
        """Start a solve (fair_bottleneck.cpp:29-50 initialisation); rounds follow with step()."""
        self._check(self.L.lmmhip_fb_shard_begin(self.ctx, self.prec, ct.c_void_p(self.xnb.data_ptr()),
                                                 ct.c_void_p(self.gather.xmu.data_ptr()), self.mu_off,
                                                 ct.c_void_p(self.gather.xrem.data_ptr())))

    def _check(self, rc):
        if rc != 0:
            raise lmm.LmmError(self.L.lmmhip_last_error().decode())

    def step(self, phase):
        self._check(self.L.lmmhip_fb_shard_step(self.ctx, phase))

    def pack_mu(self):
        """(pos, mu, count) device tensors: this shard's variables listed at the round's start and their new mu
        (lmmhip_fb_shard_pack_mu), for the delta exchange of mu."""
        import torch

        if not hasattr(self, "_dpos"):
            with torch.cuda.stream(self.stream):
                self._dpos = torch.empty(max(self.n, 1), dtype=torch.int32, device="cuda")
                self._dmu = torch.empty(max(self.n, 1), dtype=torch.float64, device="cuda")
                self._dcnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        with torch.cuda.stream(self.stream):
            self._dcnt.zero_()
        self._check(self.L.lmmhip_fb_shard_pack_mu(self.ctx, ct.c_void_p(self._dpos.data_ptr()),
                                                   ct.c_void_p(self._dmu.data_ptr()), ct.c_void_p(self._dcnt.data_ptr())))
        return self._dpos, self._dmu, self._dcnt

    def poll(self):
        done, rounds = ct.c_int(), ct.c_int64()
        self._check(self.L.lmmhip_fb_shard_poll(self.ctx, ct.byref(done), ct.byref(rounds)))
        return bool(done.value), rounds.value

    def fb_work(self):
        """This shard's part of the solve's work (lmmhip_fb_work): (elements, variables, constraints)."""
        w = (ct.c_int64 * 3)()
        self._check(self.L.lmmhip_fb_work(self.ctx, w))
        return w[0], w[1], w[2]

    def values(self):
        x = np.empty(self.n, np.float64)
        self._check(self.L.lmmhip_get_values(self.ctx, x.ctypes.data_as(ct.POINTER(ct.c_double))))
        return x

    def close(self):
        if self.ctx:
            self.L.lmmhip_ctx_destroy(self.ctx)
            self.ctx = None


def shard_variables(f, parts):
    """Contiguous nnz-balanced variable blocks of flat `f`, every constraint kept in each (the variable
    side of an FbShardPlan).  Returns [(flat, dense indices)]."""
    plan = FbShardPlan(f, parts)
    return [plan.variables(p) for p in range(parts)]


def fb_solve_sharded(shards, exchange, gather, poll_every=16):
    """Drive the four-phase FairBottleneck rounds of `shards`, this process's shards: parts
    rank * len(shards) .. (rank + 1) * len(shards) - 1 of the plan, sharing `gather` (FbGather).
    Between the phases: all-reduce(SUM) of the listed counts (over the local shards, then the ranks),
    all-gather of mu, all-gather of the owned remaining values.  Returns the round count.  All ranks stop
    in the same round: `done` comes from the reduced counts, and the stop decision is all-reduced."""
    stream = getattr(shards[0], "stream", None) if shards else None
    if stream is not None:  # device shards: the exchanges run on the shards' stream
        import torch

        with torch.cuda.stream(stream):
            return _fb_rounds(shards, exchange, gather, poll_every)
    return _fb_rounds(shards, exchange, gather, poll_every)


FB_DELTA = True  # multi-process FairBottleneck: ship only the listed variables' mu after round 0 (measurement knob)


def _fb_rounds(shards, exchange, gather, poll_every):
    lp = len(shards)
    # a multi-process exchange ships only the listed variables' mu after round 0 (all shards must pack); decided
    # once for all ranks (a rank shipping pairs while another ships the full vector would mismatch collectives)
    delta = FB_DELTA and isinstance(exchange, DistExchange) and all(hasattr(sh, "pack_mu") for sh in shards)
    if isinstance(exchange, DistExchange):
        delta = bool(exchange.min(np.array([float(delta)]))[0] == 1.0)
    max_rounds = 64 * (gather.xmu.shape[0] + gather.xrem.shape[0]) + 4096
    rounds = 0
    while True:
        for _ in range(poll_every):
            for sh in shards:
                sh.step(0)
            acc = shards[0].xnb
            for sh in shards[1:]:
                acc += sh.xnb
            exchange.allreduce_(acc, "sum")
            for sh in shards[1:]:
                sh.xnb[...] = acc
            for sh in shards:
                sh.step(1)
            if rounds == 0 or not delta:  # round 0: every mu is new
                exchange.allgather_(gather.xmu, lp * gather.Pv)
            else:  # later rounds: only the listed variables' mu moved (fair_bottleneck.cpp:89-105)
                exchange.gather_pairs_(gather.xmu, [sh.pack_mu() for sh in shards])
            for sh in shards:
                sh.step(2)
            exchange.allgather_(gather.xrem, lp * gather.Pc)
            for sh in shards:
                sh.step(3)
            rounds += 1
        states = [sh.poll() for sh in shards]
        done = float(all(d for d, _ in states))
        if exchange.min(np.array([done]))[0] == 1.0:
            return max(r for _, r in states)
        if rounds > max_rounds:
            raise lmm.LmmError("fair-bottleneck round guard tripped")
