"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end of the CPU restatement (oracle/lmm_oracle.cpp).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product
(simgrid_amd/) never does.  The API mirrors lmm::System (maxmin.hpp:380-557) method for method.
"""
import ctypes as ct
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liblmm_oracle.so")
_lib = None

P = ct.c_void_p
D = ct.c_double
I = ct.c_int
LL = ct.c_longlong

FAT_TREE, DRAGONFLY = 0, 1
SHARED, SPLITDUPLEX, FATPIPE = 0, 1, 2
CM02, LV08, L07 = 0, 1, 2


def platform_params(topology=FAT_TREE, topo_parameters="", bw=1.25e8, lat=5e-5, policy=SPLITDUPLEX, loopback_bw=0.0,
                    loopback_lat=0.0, limiter_bw=0.0, speed=1e9, model=LV08, crosstraffic=True, n_flows=1000,
                    seed=1, size_min=1e6, size_max=1e9, tcp_gamma=4194304.0):
    """The parameters of a generated platform (the fields of lmm_platform_params, include/lmm/lmm_system.h),
    for oracle/platforms.py."""
    if policy not in (SHARED, SPLITDUPLEX, FATPIPE):
        raise ValueError(f"unknown sharing policy {policy}")
    if n_flows < 0:
        raise ValueError("negative flow count")
    return dict(topology=topology, topo_parameters=topo_parameters, bw=bw, lat=lat, policy=policy,
                loopback_bw=loopback_bw, loopback_lat=loopback_lat, limiter_bw=limiter_bw, speed=speed, model=model,
                crosstraffic=bool(crosstraffic), n_flows=int(n_flows), seed=int(seed), size_min=size_min,
                size_max=size_max, tcp_gamma=tcp_gamma)


def params_dict(p):
    return dict(p)


def platform_size(p):
    """(links, hosts) of platform p (oracle/platforms.py)."""
    from oracle import platforms as PL
    return PL.platform_size(p)


_SIGS = {
    "oracle_set_precision": (None, [D]),
    "oracle_get_precision": (D, []),
    "oracle_set_default_concurrency_limit": (None, [I]),
    "oracle_system_new": (P, [I, I]),
    "oracle_system_free": (None, [P]),
    "oracle_solve": (None, [P]),
    "oracle_timed_solve": (D, [P]),
    "oracle_last_rounds": (LL, [P]),
    "oracle_set_depth": (None, [P, I]),
    "oracle_depth_stats": (I, [P, ct.POINTER(I), ct.POINTER(LL), ct.POINTER(LL), ct.POINTER(LL), ct.POINTER(LL), I]),
    "oracle_constraint_depth": (None, [P, ct.POINTER(P), LL, ct.POINTER(I), ct.POINTER(LL)]),
    "oracle_variable_depth": (None, [P, ct.POINTER(P), LL, ct.POINTER(I), ct.POINTER(LL), ct.POINTER(I)]),
    "oracle_is_modified": (I, [P]),
    "oracle_constraint_new": (P, [P, D]),
    "oracle_constraint_unshare": (None, [P, P]),
    "oracle_constraint_is_shared": (I, [P, P]),
    "oracle_constraint_set_concurrency_limit": (None, [P, P, I]),
    "oracle_constraint_concurrency": (None, [P, P, ct.POINTER(I), ct.POINTER(I), ct.POINTER(I)]),
    "oracle_constraint_reset_concurrency_maximum": (None, [P, P]),
    "oracle_constraint_get_usage": (D, [P, P]),
    "oracle_constraint_get_variable_amount": (I, [P, P]),
    "oracle_constraint_get_bound": (D, [P, P]),
    "oracle_constraint_rank": (I, [P, P]),
    "oracle_constraint_used": (I, [P, P]),
    "oracle_constraint_init_state": (I, [P, P, ct.POINTER(D), ct.POINTER(D)]),
    "oracle_constraint_elements": (I, [P, P, ct.POINTER(I), ct.POINTER(D), ct.POINTER(D), ct.POINTER(I), I]),
    "oracle_variable_new": (P, [P, D, D, ct.c_long]),
    "oracle_variable_free": (None, [P, P]),
    "oracle_variable_free_all": (None, [P]),
    "oracle_variable_set_concurrency_share": (None, [P, P, I]),
    "oracle_variable_get_value": (D, [P, P]),
    "oracle_variable_get_bound": (D, [P, P]),
    "oracle_variable_get_penalty": (D, [P, P]),
    "oracle_variable_rank": (I, [P, P]),
    "oracle_variable_number_of_constraints": (I, [P, P]),
    "oracle_get_values": (None, [P, ct.POINTER(P), LL, ct.POINTER(D)]),
    "oracle_system_variables": (I, [P, ct.POINTER(P), I]),
    "oracle_system_active_constraints": (I, [P, ct.POINTER(P), I]),
    "oracle_modified_actions": (I, [P, ct.POINTER(P), I]),
    "oracle_clear_modified_actions": (None, [P]),
    "oracle_expand": (None, [P, P, P, D]),
    "oracle_expand_add": (None, [P, P, P, D]),
    "oracle_update_variable_bound": (None, [P, P, D]),
    "oracle_update_variable_penalty": (None, [P, P, D]),
    "oracle_update_constraint_bound": (None, [P, P, D]),
    "oracle_gen_maxmin_bench": (I, [P, I, I, ct.POINTER(P), ct.POINTER(P), ct.POINTER(I), ct.POINTER(I)]),
    "oracle_gen_synthetic": (LL, [P, LL, LL, I, ct.c_ulonglong, I, I, I, I, ct.POINTER(P)]),
    "oracle_build_flows": (LL, [P, LL, ct.POINTER(D), ct.POINTER(ct.c_ubyte), LL, ct.POINTER(D), ct.POINTER(D),
                                ct.POINTER(ct.c_int), ct.POINTER(LL), ct.POINTER(ct.c_int), ct.POINTER(D),
                                ct.POINTER(ct.c_ubyte), ct.POINTER(P), ct.POINTER(P)]),
}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ct.CDLL(_LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(_lib, name)
            f.restype = res
            f.argtypes = args
    return _lib


def set_precision(p):
    lib().oracle_set_precision(p)


def get_precision():
    return lib().oracle_get_precision()


class Constraint:
    __slots__ = ("sys", "h")

    def __init__(self, sys, h):
        self.sys, self.h = sys, h

    def unshare(self):
        lib().oracle_constraint_unshare(self.sys.h, self.h)

    def is_shared(self):
        return bool(lib().oracle_constraint_is_shared(self.sys.h, self.h))

    def set_concurrency_limit(self, l):
        lib().oracle_constraint_set_concurrency_limit(self.sys.h, self.h, l)

    def concurrency(self):
        a, b, c = I(), I(), I()
        lib().oracle_constraint_concurrency(self.sys.h, self.h, ct.byref(a), ct.byref(b), ct.byref(c))
        return a.value, b.value, c.value

    def get_concurrency_limit(self):
        return self.concurrency()[2]

    def get_concurrency_maximum(self):
        return self.concurrency()[1]

    def reset_concurrency_maximum(self):
        lib().oracle_constraint_reset_concurrency_maximum(self.sys.h, self.h)

    def get_usage(self):
        return lib().oracle_constraint_get_usage(self.sys.h, self.h)

    def get_variable_amount(self):
        return lib().oracle_constraint_get_variable_amount(self.sys.h, self.h)

    def get_bound(self):
        return lib().oracle_constraint_get_bound(self.sys.h, self.h)

    @property
    def rank(self):
        return lib().oracle_constraint_rank(self.sys.h, self.h)

    def init_state(self):
        u, r = D(), D()
        ok = lib().oracle_constraint_init_state(self.sys.h, self.h, ct.byref(u), ct.byref(r))
        return (u.value, r.value) if ok else None

    def elements(self):
        """[(var_rank, weight, value, enabled)] in System::print() order."""
        n = lib().oracle_constraint_elements(self.sys.h, self.h, None, None, None, None, 0)
        rk, w, x, en = (I * n)(), (D * n)(), (D * n)(), (I * n)()
        lib().oracle_constraint_elements(self.sys.h, self.h, rk, w, x, en, n)
        return [(rk[i], w[i], x[i], bool(en[i])) for i in range(n)]


class Variable:
    __slots__ = ("sys", "h")

    def __init__(self, sys, h):
        self.sys, self.h = sys, h

    def get_value(self):
        return lib().oracle_variable_get_value(self.sys.h, self.h)

    def get_bound(self):
        return lib().oracle_variable_get_bound(self.sys.h, self.h)

    def get_penalty(self):
        return lib().oracle_variable_get_penalty(self.sys.h, self.h)

    def set_concurrency_share(self, s):
        lib().oracle_variable_set_concurrency_share(self.sys.h, self.h, s)

    def get_number_of_constraint(self):
        return lib().oracle_variable_number_of_constraints(self.sys.h, self.h)

    @property
    def rank(self):
        return lib().oracle_variable_rank(self.sys.h, self.h)


class System:
    """lmm::System (maxmin.hpp:380) / FairBottleneck (maxmin.hpp:547) restated on the CPU."""

    MAXMIN, FAIR_BOTTLENECK = 0, 1

    def __init__(self, selective_update=False, kind=0):
        self.h = lib().oracle_system_new(int(selective_update), kind)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_system_free(self.h)
            self.h = None

    def constraint_new(self, id_, bound):
        return Constraint(self, lib().oracle_constraint_new(self.h, bound))

    def variable_new(self, id_, penalty, bound=-1.0, number_of_constraints=1):
        return Variable(self, lib().oracle_variable_new(self.h, penalty, bound, number_of_constraints))

    def variable_free(self, v):
        lib().oracle_variable_free(self.h, v.h)

    def variable_free_all(self):
        lib().oracle_variable_free_all(self.h)

    def expand(self, c, v, w):
        lib().oracle_expand(self.h, c.h, v.h, w)

    def expand_add(self, c, v, w):
        lib().oracle_expand_add(self.h, c.h, v.h, w)

    def update_variable_bound(self, v, b):
        lib().oracle_update_variable_bound(self.h, v.h, b)

    def update_variable_penalty(self, v, p):
        lib().oracle_update_variable_penalty(self.h, v.h, p)

    def update_constraint_bound(self, c, b):
        lib().oracle_update_constraint_bound(self.h, c.h, b)

    def constraint_used(self, c):
        return bool(lib().oracle_constraint_used(self.h, c.h))

    def solve(self):
        lib().oracle_solve(self.h)

    def timed_solve(self):
        return lib().oracle_timed_solve(self.h)

    def set_depth(self, on):
        """Record the dependency depth of the next solves (measurement only; lmm_oracle.hpp depth_on)."""
        lib().oracle_set_depth(self.h, int(bool(on)))

    def depth_stats(self):
        """(D, saturation events, bound-fix events, per-level saturation histogram, per-level bound-fix histogram)."""
        import numpy as np
        d, ns, nb = I(), LL(), LL()
        cap = 1 << 20
        h = np.zeros(cap, dtype=np.int64)
        bh = np.zeros(cap, dtype=np.int64)
        n = lib().oracle_depth_stats(self.h, ct.byref(d), ct.byref(ns), ct.byref(nb),
                                     h.ctypes.data_as(ct.POINTER(LL)), bh.ctypes.data_as(ct.POINTER(LL)), cap)
        return d.value, ns.value, nb.value, h[:n].copy(), bh[:n].copy()

    def variable_depth(self, vs):
        """Per variable handle: (level, sequential round, rank of the constraint that fixed it: 0 = bound fix)."""
        import numpy as np
        arr = vs if isinstance(vs, ct.Array) else (P * len(vs))(*[getattr(v, "h", v) for v in vs])
        lv = np.zeros(len(vs), dtype=np.int32)
        rd = np.zeros(len(vs), dtype=np.int64)
        by = np.zeros(len(vs), dtype=np.int32)
        lib().oracle_variable_depth(self.h, arr, len(vs), lv.ctypes.data_as(ct.POINTER(I)),
                                    rd.ctypes.data_as(ct.POINTER(LL)), by.ctypes.data_as(ct.POINTER(I)))
        return lv, rd, by

    def constraint_depth(self, cs):
        """Per constraint handle: (saturation level, sequential round), -1 if it never saturated."""
        import numpy as np
        arr = (P * len(cs))(*[c.h for c in cs])
        lv = np.zeros(len(cs), dtype=np.int32)
        rd = np.zeros(len(cs), dtype=np.int64)
        lib().oracle_constraint_depth(self.h, arr, len(cs), lv.ctypes.data_as(ct.POINTER(I)),
                                      rd.ctypes.data_as(ct.POINTER(LL)))
        return lv, rd

    @property
    def last_rounds(self):
        return lib().oracle_last_rounds(self.h)

    @property
    def modified(self):
        return bool(lib().oracle_is_modified(self.h))

    def variables(self):
        n = lib().oracle_system_variables(self.h, None, 0)
        arr = (P * n)()
        lib().oracle_system_variables(self.h, arr, n)
        return [Variable(self, arr[i]) for i in range(n)]

    def active_constraints(self):
        n = lib().oracle_system_active_constraints(self.h, None, 0)
        arr = (P * n)()
        lib().oracle_system_active_constraints(self.h, arr, n)
        return [Constraint(self, arr[i]) for i in range(n)]

    def modified_actions(self):
        n = lib().oracle_modified_actions(self.h, None, 0)
        arr = (P * n)()
        lib().oracle_modified_actions(self.h, arr, n)
        return [Variable(self, arr[i]) for i in range(n)]

    def clear_modified_actions(self):
        lib().oracle_clear_modified_actions(self.h)

    # ---- generators (input construction, same call sequence as the product) ----
    def gen_maxmin_bench(self, klass, run):
        C, V = {0: (10, 10), 1: (100, 100), 2: (2000, 2000), 3: (20000, 20000)}[klass]
        cs, vs = (P * C)(), (P * V)()
        a, b = I(), I()
        lib().oracle_gen_maxmin_bench(self.h, klass, run, cs, vs, ct.byref(a), ct.byref(b))
        return ([Constraint(self, cs[i]) for i in range(C)], [Variable(self, vs[i]) for i in range(V)],
                a.value, b.value)

    def gen_synthetic(self, nb_cnst, nb_var, k=8, seed=1, max_share=2, penalty_mix=0, bounded_permille=0,
                      fatpipe_permille=0, want_vars=True):
        vs = (P * nb_var)() if want_vars else None
        lib().oracle_gen_synthetic(self.h, nb_cnst, nb_var, k, seed, max_share, penalty_mix, bounded_permille,
                                   fatpipe_permille, vs)
        return vs

    def gen_platform_flows(self, p):
        """Links (+ L07 CPUs) and p.n_flows flows built by oracle/platforms.py, the oracle's own restatement of
        the reference's zones and flow models: (constraint list, variable handle array)."""
        import numpy as np

        from oracle import platforms as PL
        ops = PL.flow_ops(params_dict(p))
        nc, nv = len(ops["cbound"]), len(ops["vpen"])
        cs, vs = (P * nc)(), (P * nv)()

        def ptr(a, t):
            return np.ascontiguousarray(a).ctypes.data_as(ct.POINTER(t))
        keep = [np.ascontiguousarray(ops[k]) for k in ("cbound", "cfat", "vpen", "vbound", "vn", "eptr", "ecnst",
                                                        "ew", "eadd")]
        rc = lib().oracle_build_flows(self.h, nc, ptr(keep[0], D), ptr(keep[1], ct.c_ubyte), nv, ptr(keep[2], D),
                                      ptr(keep[3], D), ptr(keep[4], ct.c_int), ptr(keep[5], LL),
                                      ptr(keep[6], ct.c_int), ptr(keep[7], D), ptr(keep[8], ct.c_ubyte), cs, vs)
        if rc < 0:
            raise ValueError("bad flow element")
        return [Constraint(self, cs[i]) for i in range(nc)], vs

    def values_of(self, handles, n):
        import numpy as np
        out = np.empty(n, dtype=np.float64)
        lib().oracle_get_values(self.h, handles, n, out.ctypes.data_as(ct.POINTER(D)))
        return out
