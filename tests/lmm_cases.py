"""Shared system builders for the parity tests.

Every builder takes a module exposing the reference's System API (simgrid_amd.lmm for the HIP
product, oracle.pyoracle for the CPU restatement) and replays the same call sequence on it, so the
two systems are identical by construction.

Parity criteria (written here once):
  * values:        |x_gpu - x_ref| <= max(ABS_TOL, REL_TOL * |x_ref|)   (fp64, sg_maxmin_precision 1e-5)
  * tesh goldens:  |x - golden| <= GOLDEN_TOL  (goldens are printed with %f)
  * saturated set: sat(c) = not double_positive(bound - get_usage(c), bound * prec), identical sets.
"""
import random

ABS_TOL = 1e-9
REL_TOL = 1e-6
GOLDEN_TOL = 1.0e-6 + 5e-7  # %f rounding (5e-7) + slack


def close(a, b, abs_tol=ABS_TOL, rel_tol=REL_TOL):
    return abs(a - b) <= max(abs_tol, rel_tol * abs(b))


# ---------------------------------------------------------------------------------------------
# Known-answer tests of src/kernel/lmm/maxmin_test.cpp (the reference's Catch unit tests)
# ---------------------------------------------------------------------------------------------
def kat_shared_penalty(M):  # maxmin_test.cpp:17-42
    s = M.System(False)
    c = s.constraint_new(None, 3)
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 2)
    s.expand(c, r1, 1)
    s.expand(c, r2, 1)
    s.solve()
    return s, [(r1, 2.0), (r2, 1.0)]


def kat_shared_weight(M):  # :44-70
    s = M.System(False)
    c = s.constraint_new(None, 3)
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 1)
    s.expand(c, r1, 1)
    s.expand(c, r2, 2)
    s.solve()
    return s, [(r1, 1.0), (r2, 1.0)]


def kat_shared_weight_penalty(M):  # :72-100
    s = M.System(False)
    c = s.constraint_new(None, 20)
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 2)
    s.expand(c, r1, 1)
    s.expand(c, r2, 2)
    s.solve()
    return s, [(r1, 10.0), (r2, 5.0)]


def kat_shared_multi(M):  # :102-142
    s = M.System(False)
    c1 = s.constraint_new(None, 20)
    c2 = s.constraint_new(None, 60)
    r1 = s.variable_new(None, 1, -1, 2)
    r2 = s.variable_new(None, 2, -1, 1)
    r3 = s.variable_new(None, 1, -1, 1)
    s.expand(c1, r1, 1)
    s.expand(c1, r2, 2)
    s.expand(c2, r1, 2)
    s.expand(c2, r3, 1)
    s.solve()
    return s, [(r1, 10.0), (r2, 5.0), (r3, 40.0)]


def kat_fatpipe_penalty(M):  # :152-180
    s = M.System(False)
    c = s.constraint_new(None, 10)
    c.unshare()
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 2)
    s.expand(c, r1, 1)
    s.expand(c, r2, 1)
    s.solve()
    return s, [(r1, 10.0), (r2, 5.0)]


def kat_fatpipe_weight(M):  # :182-211
    s = M.System(False)
    c = s.constraint_new(None, 10)
    c.unshare()
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 1)
    s.expand(c, r1, 1)
    s.expand(c, r2, 2)
    s.solve()
    return s, [(r1, 5.0), (r2, 5.0)]


def kat_fatpipe_weight_penalty(M):  # :213-242
    s = M.System(False)
    c = s.constraint_new(None, 10)
    c.unshare()
    r1 = s.variable_new(None, 1)
    r2 = s.variable_new(None, 2)
    s.expand(c, r1, 1)
    s.expand(c, r2, 2)
    s.solve()
    return s, [(r1, 10.0), (r2, 5.0)]


def kat_fatpipe_multi(M):  # :244-286
    s = M.System(False)
    c1 = s.constraint_new(None, 10)
    c2 = s.constraint_new(None, 60)
    c1.unshare()
    c2.unshare()
    r1 = s.variable_new(None, 1, -1, 2)
    r2 = s.variable_new(None, 2, -1, 1)
    r3 = s.variable_new(None, 1, -1, 1)
    s.expand(c1, r1, 1)
    s.expand(c1, r2, 2)
    s.expand(c2, r1, 2)
    s.expand(c2, r3, 1)
    s.solve()
    return s, [(r1, 10.0), (r2, 5.0), (r3, 60.0)]


MAXMIN_TEST_KATS = [kat_shared_penalty, kat_shared_weight, kat_shared_weight_penalty, kat_shared_multi,
                    kat_fatpipe_penalty, kat_fatpipe_weight, kat_fatpipe_weight_penalty, kat_fatpipe_multi]


# ---------------------------------------------------------------------------------------------
# teshsuite/surf/lmm_usage/lmm_usage.cpp — values are not printed by the tesh (DEBUG level), so
# the expected answers below are derived analytically.
# ---------------------------------------------------------------------------------------------
def lmm_usage_test1(M):  # lmm_usage.cpp:28-68
    s = M.System(False)
    L1 = s.constraint_new(None, 1.0)
    L2 = s.constraint_new(None, 10.0)
    L3 = s.constraint_new(None, 1.0)
    R123 = s.variable_new(None, 1.0, -1.0, 3)
    R1 = s.variable_new(None, 1.0, -1.0, 1)
    R2 = s.variable_new(None, 1.0, -1.0, 1)
    R3 = s.variable_new(None, 1.0, -1.0, 1)
    for v in (R123, R1, R2, R3):
        s.update_variable_penalty(v, 1.0)
    s.expand(L1, R123, 1.0)
    s.expand(L2, R123, 1.0)
    s.expand(L3, R123, 1.0)
    s.expand(L1, R1, 1.0)
    s.expand(L2, R2, 1.0)
    s.expand(L3, R3, 1.0)
    s.solve()
    return s, [(R123, 0.5), (R1, 0.5), (R2, 9.5), (R3, 0.5)]


def lmm_usage_test2(M):  # :70-94
    s = M.System(False)
    CPU1 = s.constraint_new(None, 200.0)
    CPU2 = s.constraint_new(None, 100.0)
    T1 = s.variable_new(None, 1.0, -1.0, 1)
    T2 = s.variable_new(None, 1.0, -1.0, 1)
    s.update_variable_penalty(T1, 1.0)
    s.update_variable_penalty(T2, 1.0)
    s.expand(CPU1, T1, 1.0)
    s.expand(CPU2, T2, 1.0)
    s.solve()
    return s, [(T1, 200.0), (T2, 100.0)]


def lmm_usage_test3(M):  # :96-160 (11 flows on 10 links + 5 fictitious single-flow constraints)
    A = [[0.0] * 16 for _ in range(15)]
    for (i, js) in [(0, [1, 7]), (1, [1, 7, 8]), (2, [1, 8]), (3, [8]), (4, [0, 3, 9]), (5, [0, 3, 4, 9]),
                    (6, [0, 4, 9, 10]), (7, [2, 4, 6, 9, 10]), (8, [2, 10]), (9, [5, 6, 9]), (10, [11]), (11, [12]),
                    (12, [13]), (13, [14]), (14, [15])]:
        for j in js:
            A[i][j] = 1.0
    B = [10] * 10 + [1] * 5
    s = M.System(False)
    cs = [s.constraint_new(None, B[i]) for i in range(15)]
    vs = []
    for j in range(16):
        v = s.variable_new(None, 1.0, -1.0, 15)
        s.update_variable_penalty(v, 1.0)
        vs.append(v)
    for i in range(15):
        for j in range(16):
            if A[i][j]:
                s.expand(cs[i], vs[j], 1.0)
    s.solve()
    return s, vs


# ---------------------------------------------------------------------------------------------
# Random operation scripts (replayed identically on both implementations)
# ---------------------------------------------------------------------------------------------
def random_script(seed, n_cnst=30, n_var=60, max_el=6, fatpipe_p=0.1, bounded_p=0.2, penalty_mix=True,
                  conc_limits=False, zero_bound_p=0.05, dup_p=0.2, frees=0, penalty_updates=0, bound_updates=0,
                  zero_w_p=0.05):
    """A deterministic list of API operations covering penalties, bounds, FATPIPE, duplicate
    elements, zero-bound constraints, concurrency limits/staging, frees and updates."""
    rng = random.Random(seed)
    ops = []
    for c in range(n_cnst):
        b = 0.0 if rng.random() < zero_bound_p else round(rng.uniform(0.5, 20.0), 3)
        ops.append(("cnst", c, b))
        if rng.random() < fatpipe_p:
            ops.append(("unshare", c))
        if conc_limits and rng.random() < 0.5:
            ops.append(("limit", c, rng.randint(2, 6)))
    for v in range(n_var):
        p = rng.choice([1.0, 2.0, 0.5, 4.0]) if penalty_mix else 1.0
        if rng.random() < 0.05:
            p = 0.0
        b = round(rng.uniform(0.05, 3.0), 3) if rng.random() < bounded_p else -1.0
        k = rng.randint(1, max_el)
        ops.append(("var", v, p, b, k + 2))
        if rng.random() < dup_p:
            ops.append(("share", v, 2))
        cs = rng.sample(range(n_cnst), min(k, n_cnst))
        for c in cs:
            ops.append(("expand", c, v, round(rng.uniform(0.0, 2.0), 4) if rng.random() >= zero_w_p else 0.0))
            if rng.random() < 0.3:
                ops.append(("expand_add", c, v, round(rng.uniform(0.0, 1.0), 4)))
        if rng.random() < dup_p:
            ops.append(("expand", cs[0], v, round(rng.uniform(0.1, 1.0), 4)))
    alive = list(range(n_var))
    for _ in range(frees):
        v = alive.pop(rng.randrange(len(alive)))
        ops.append(("free", v))
    for _ in range(penalty_updates):
        ops.append(("penalty", rng.choice(alive), rng.choice([0.0, 1.0, 2.0, 3.0])))
    for _ in range(bound_updates):
        if rng.random() < 0.5:
            ops.append(("vbound", rng.choice(alive), round(rng.uniform(0.05, 3.0), 3)))
        else:
            ops.append(("cbound", rng.randrange(n_cnst), round(rng.uniform(0.5, 20.0), 3)))
    return ops


def replay(M, ops, selective=False, kind=0, sys_=None, cs=None, vs=None):
    s = sys_ if sys_ is not None else M.System(selective, kind)
    cs = {} if cs is None else cs
    vs = {} if vs is None else vs
    for op in ops:
        t = op[0]
        if t == "cnst":
            cs[op[1]] = s.constraint_new(None, op[2])
        elif t == "unshare":
            cs[op[1]].unshare()
        elif t == "limit":
            cs[op[1]].set_concurrency_limit(op[2])
        elif t == "var":
            vs[op[1]] = s.variable_new(None, op[2], op[3], op[4])
        elif t == "share":
            vs[op[1]].set_concurrency_share(op[2])
        elif t == "expand":
            s.expand(cs[op[1]], vs[op[2]], op[3])
        elif t == "expand_add":
            s.expand_add(cs[op[1]], vs[op[2]], op[3])
        elif t == "free":
            s.variable_free(vs.pop(op[1]))
        elif t == "penalty":
            if op[1] in vs:
                s.update_variable_penalty(vs[op[1]], op[2])
        elif t == "vbound":
            if op[1] in vs:
                s.update_variable_bound(vs[op[1]], op[2])
        elif t == "cbound":
            s.update_constraint_bound(cs[op[1]], op[2])
        else:
            raise ValueError(t)
    return s, cs, vs


def saturated(s, cs, prec):
    out = set()
    for k, c in cs.items():
        b = c.get_bound()
        if not (b - c.get_usage() > b * prec):
            out.add(k)
    return out


def compare_values(vs_a, vs_b, abs_tol=ABS_TOL, rel_tol=REL_TOL):
    """Returns (worst abs diff, list of mismatching keys)."""
    worst, bad = 0.0, []
    for k in vs_b:
        a, b = vs_a[k].get_value(), vs_b[k].get_value()
        worst = max(worst, abs(a - b))
        if not close(a, b, abs_tol, rel_tol):
            bad.append((k, a, b))
    return worst, bad
