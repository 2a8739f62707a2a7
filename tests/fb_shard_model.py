"""TEST INFRASTRUCTURE: a numpy model of one shard of the constraint-owner sharded FairBottleneck round
(the four-phase protocol of lmmhip_fb_shard_*, lmm_fb_kernels.hpp fbo_*), so that multi.fb_solve_sharded
and its exchanges (all-reduce of counts, all-gathers of mu and of the owned remaining values) run on gloo
without a GPU.  Restates fair_bottleneck.cpp:59-145 phase by phase; the owned constraints' remaining is the
reference's own per-element double_update chain (:110-116, surf_interface.hpp:34-44) in a Python loop, so
the values must equal the oracle's bit for bit."""
import numpy as np

DBL_MAX = np.finfo(np.float64).max


class NumpyFbShard:
    def __init__(self, plan, p, gather, precision):
        f, self.idx = plan.variables(p)
        self.prec = precision
        self.gather = gather
        nv, nc = len(f.penalty), len(f.cbound)
        self.nv, self.nc = nv, nc
        self.rows = np.repeat(np.arange(nv), np.diff(f.var_ptr))
        self.cols = f.cnst_idx.astype(np.int64)
        self.w = f.weight
        self.vbound = f.vbound
        self.fat = (f.cflags & 1) > 0
        self.zero_w = (f.cflags & 2) > 0
        self.x = np.zeros(nv)
        self.mu = np.zeros(nv)
        self.listed = np.ones(nv, bool)
        self.rem = f.cbound.astype(np.float64).copy()
        self.use = np.zeros(nc)
        self.inlist = np.ones(nc, bool)
        self.any = nv > 0
        self.done, self.rounds = False, 0
        self.xnb = np.zeros(nc + 1, np.int32)
        self.mu_off = plan.mu_off(p)
        self.cpos = plan.cpos
        oc, optr, ovar, ow = plan.owned(p)
        self.owned = [(int(c), ovar[optr[i]:optr[i + 1]], ow[optr[i]:optr[i + 1]]) for i, c in enumerate(oc)]

    def step(self, phase):
        if self.done:
            return
        nc, rows, cols = self.nc, self.rows, self.cols
        g = self.gather
        if phase == 0:  # :67-74 counts of this shard's listed variables
            live = self.listed[rows] & self.inlist[cols]
            self.xnb[:nc] = np.bincount(cols, weights=live, minlength=nc).astype(np.int32)
            self.xnb[nc] = int(self.any)
        elif phase == 1:
            if self.xnb[nc] == 0:  # :145 nothing listed anywhere
                self.done = True
                return
            self.rounds += 1
            nb = self.xnb[:nc].astype(np.float64)
            nb[(nb > 0) & self.fat] = 1.0
            erase = self.inlist & (nb == 0)  # :78-81
            self.rem[erase] = 0.0
            self.use[erase] = 0.0
            self.inlist[erase] = False
            keep = self.inlist
            self.use[keep] = self.rem[keep] / nb[keep]
            inc = np.full(self.nv, DBL_MAX)  # :89-105
            np.minimum.at(inc, rows, self.use[cols] / self.w)
            b = self.vbound > 0
            inc[b] = np.minimum(inc[b], self.vbound[b] - self.x[b])
            lst = self.listed.copy()
            self.lst_start = lst
            self.mu[lst] = inc[lst]
            self.x[lst] += inc[lst]
            drop = lst & (self.x == self.vbound)
            self.listed[drop] = False
            self.any = bool(np.any(lst & ~drop))
            g.xmu[self.mu_off:self.mu_off + self.nv] = self.mu  # delisted variables keep their last mu
        elif phase == 2:  # :107-127 on the owned constraints, from the gathered mu
            prec = self.prec
            for c, pos, w in self.owned:
                r = float(self.rem[c])
                if self.inlist[c]:
                    d = w * g.xmu[pos]
                    if self.fat[c]:  # :118-125
                        u = float(self.use[c])
                        if self.zero_w[c]:
                            u = min(u, 0.0)
                        u = min(u, float(d.min()))
                        r -= u
                        if r < prec:
                            r = 0.0
                    else:  # :111-116 one double_update per element, in the reference's order
                        for x in d.tolist():
                            r -= x
                            if r < prec:
                                r = 0.0
                g.xrem[self.cpos[c]] = r
        else:  # :129-140 every listed constraint takes its owner's remaining
            upd = self.inlist.copy()
            self.rem[upd] = g.xrem[self.cpos[upd]]
            erased = upd & (self.rem <= 0.0)
            self.inlist[erased] = False
            self.listed[rows[erased[cols]]] = False

    def pack_mu(self):
        """(positions in xmu, mu, [count]) of the variables listed at the round's start (lmmhip_fb_shard_pack_mu)."""
        lst = getattr(self, "lst_start", np.zeros(self.nv, bool)) if not self.done else np.zeros(self.nv, bool)
        v = np.flatnonzero(lst)
        return (self.mu_off + v).astype(np.int32), self.mu[v].copy(), np.array([len(v)])

    def poll(self):
        return self.done, self.rounds

    def values(self):
        return self.x
