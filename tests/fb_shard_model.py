"""TEST INFRASTRUCTURE: a numpy model of one rank's part of the variable-sharded FairBottleneck round
(the phase protocol of lmmhip_fb_shard_*, lmm_fb_kernels.hpp), so that multi.fb_solve_sharded and its
exchanges can run on gloo without a GPU.  Restates fair_bottleneck.cpp:59-145 phase by phase."""
import numpy as np

DBL_MAX = np.finfo(np.float64).max


class NumpyFbShard:
    def __init__(self, f, precision):
        self.prec = precision
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
        self.xsum = np.zeros(nc)
        self.xmin = np.zeros(nc)

    def buffers(self, phase):
        return [(self.xnb, "sum")] if phase == 0 else [(self.xsum, "sum"), (self.xmin, "min")]

    def step(self, phase):
        if self.done:
            return
        nc, rows, cols = self.nc, self.rows, self.cols
        if phase == 0:  # :67-74 counts of listed variables
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
            self.mu[lst] = inc[lst]
            self.x[lst] += inc[lst]
            drop = lst & (self.x == self.vbound)
            self.listed[drop] = False
            self.any = bool(np.any(lst & ~drop))
            d = self.w * self.mu[rows]  # :107-127, stale mu included
            self.xsum[:] = np.bincount(cols, weights=d, minlength=nc)
            self.xmin[:] = np.inf
            np.minimum.at(self.xmin, cols, d)
            self.xsum[~self.inlist | self.fat] = 0.0
            self.xmin[~self.inlist | ~self.fat] = np.inf
        else:  # :110-140
            upd = self.inlist.copy()
            fat = upd & self.fat
            u = self.use.copy()
            u[fat & self.zero_w] = np.minimum(u[fat & self.zero_w], 0.0)
            u[fat] = np.minimum(u[fat], self.xmin[fat])
            self.use[fat] = u[fat]
            self.rem[fat] -= u[fat]
            shared = upd & ~self.fat
            self.rem[shared] -= self.xsum[shared]
            self.rem[upd & (self.rem < self.prec)] = 0.0
            erased = upd & (self.rem <= 0.0)
            self.inlist[erased] = False
            self.listed[rows[erased[cols]]] = False

    def poll(self):
        return self.done, self.rounds

    def values(self):
        return self.x
