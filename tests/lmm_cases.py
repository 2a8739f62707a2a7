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
# ---------------------------------------------------------------------------------------------
# FairBottleneck known answers pinned by the reference's own L07 (ptask) tesh outputs.  Each builds
# the system the L07 model builds for one parallel task (L07Action, ptask_L07.cpp:143-207: one
# variable of penalty 1 and bound -1; expand() on every host's CPU constraint with its flops, 0 when
# there is no computation; expand_add() of the bytes on every link of every (i, j) route; latencies
# already paid), on the platform of the test (CPU bound = speed, ptask_L07.cpp:239-241; link bound =
# bandwidth, :247-249; FATPIPE links unshared), solves it with FairBottleneck::bottleneck_solve, and
# returns [(variable, expected value, scale, printed value, tolerance)]: value * scale is what the
# tesh prints (%f -> +-5e-7 rounding, %g -> 6 significant digits).
# ---------------------------------------------------------------------------------------------
def _l07_task(M, s, host_cnsts, flops, routes):
    """One L07Action: routes = [(bytes, [link constraints])] per (i, j) with bytes > 0."""
    links = {id(c) for _, r in routes for c in r}
    v = s.variable_new(None, 1.0, -1.0, len(host_cnsts) + len(links))
    for c, f in zip(host_cnsts, flops if flops is not None else [0.0] * len(host_cnsts)):
        s.expand(c, v, f)
    for b, r in routes:
        for c in r:
            s.expand_add(c, v, b)
    return v


def fb_exec_ptask_comm(M):
    """examples/s4u/exec-ptask/s4u-exec-ptask.tesh:9-12 on examples/platforms/energy_platform.xml:
    3 x 1 Gflop on 100 Mf hosts, 10 MB between each pair over the 100 kBps 'bus' -> x = 1e5 / 3e7,
    'speed_used 3333333.333333' per host and 'bus bandwidth_used 100000.000000' (x * weight,
    instr_platform.cpp:254-260)."""
    s = M.System(False, M.System.FAIR_BOTTLENECK)
    hosts = [s.constraint_new(None, 100e6) for _ in range(3)]
    bus = s.constraint_new(None, 100e3)
    v = _l07_task(M, s, hosts, [1e9] * 3, [(1e7, [bus]) for i in range(3) for j in range(i + 1, 3)])
    s.solve()
    return s, [(v, 3333333.333333, 1e9, 5e-7), (v, 100000.0, 3e7, 5e-7)]


def fb_exec_ptask_comp(M):
    """s4u-exec-ptask.tesh:17-19: computation only, 3e8 / 6e8 / 1e9 flops on the three 100 Mf hosts ->
    x = 0.1, 'speed_used 30000000 / 60000000 / 100000000'."""
    s = M.System(False, M.System.FAIR_BOTTLENECK)
    hosts = [s.constraint_new(None, 100e6) for _ in range(3)]
    s.constraint_new(None, 100e3)  # the bus, unused
    v = _l07_task(M, s, hosts, [3e8, 6e8, 1e9], [])
    s.solve()
    return s, [(v, 30000000.0, 3e8, 5e-7), (v, 60000000.0, 6e8, 5e-7), (v, 100000000.0, 1e9, 5e-7)]


def _platform_4p_1switch(M, s):
    """teshsuite/simdag/platforms/platform_4p_1switch.xml: 4 hosts of 1 flop/s, link_k 1 Bps SHARED,
    'switch' 2 Bps FATPIPE, route i->j = link_i, switch, link_j (latency 0.5 + 1 + 0.5 = 2 s)."""
    cpus = [s.constraint_new(None, 1.0) for _ in range(4)]
    sw = s.constraint_new(None, 2.0)
    sw.unshare()
    links = [s.constraint_new(None, 1.0) for _ in range(4)]
    return cpus, links, sw


def _fb_mxn(M, amounts):
    s = M.System(False, M.System.FAIR_BOTTLENECK)
    cpus, links, sw = _platform_4p_1switch(M, s)
    routes = [(amounts[i][j], [links[i], sw, links[j]]) for i in range(4) for j in range(4) if amounts[i][j] > 0]
    v = _l07_task(M, s, cpus, None, routes)
    s.solve()
    return s, v


def fb_mxn_all2all(M):
    """teshsuite/simdag/comm-mxn-all2all.tesh: 1 B between every ordered pair; the task ends at 8 s =
    2 s latency + 6 s of transfer -> x = 1/6 (each link carries 6 B at 1 Bps; the FATPIPE switch takes
    the max, 1 B, maxmin.cpp:301-304)."""
    s, v = _fb_mxn(M, [[0, 1, 1, 1], [1, 0, 1, 1], [1, 1, 0, 1], [1, 1, 1, 0]])
    return s, [(v, 1.0 / 6.0, 1.0, 1e-12)]


def fb_mxn_scatter(M):
    """teshsuite/simdag/comm-mxn-scatter.tesh: 1 / 2 / 3 B from cpu0 to cpu1..3; ends at 8 s -> x = 1/6
    (link0 carries 6 B)."""
    s, v = _fb_mxn(M, [[0, 1, 2, 3], [0] * 4, [0] * 4, [0] * 4])
    return s, [(v, 1.0 / 6.0, 1.0, 1e-12)]


def fb_mxn_independent(M):
    """teshsuite/simdag/comm-mxn-independent.tesh: cpu0->cpu1 and cpu2->cpu3, 1 B each; ends at 3 s ->
    x = 1 (every link carries 1 B at 1 Bps, the switch max 1 B at 2 Bps)."""
    s, v = _fb_mxn(M, [[0, 1, 0, 0], [0] * 4, [0, 0, 0, 1], [0] * 4])
    return s, [(v, 1.0, 1.0, 1e-12)]


def fb_p2p_latency_bound(M):
    """teshsuite/simdag/comm-p2p-latency-bound.tesh on platform_2p_1bb.xml: three concurrent 1-B comms
    cpu0->cpu1 over link0 (2 Bps, 10000 s latency) plus the root task's zero-cost host elements; the
    simulation ends at 10001.5 -> each comm gets x = 2/3 (1.5 s for 1 B)."""
    s = M.System(False, M.System.FAIR_BOTTLENECK)
    cpus = [s.constraint_new(None, 1.0) for _ in range(2)]
    link = s.constraint_new(None, 2.0)
    vs = [_l07_task(M, s, cpus, [0.0, 0.0], [(1.0, [link])]) for _ in range(3)]
    s.solve()
    return s, [(v, 2.0 / 3.0, 1.0, 1e-12) for v in vs]


FB_TESH_KATS = [fb_exec_ptask_comm, fb_exec_ptask_comp, fb_mxn_all2all, fb_mxn_scatter, fb_mxn_independent,
                fb_p2p_latency_bound]


def check_fb_kat(expect):
    """[(variable, printed value, scale, tol)]: |x * scale - printed| <= tol (+ a 1e-12 relative slack)."""
    bad = []
    for v, want, scale, tol in expect:
        got = v.get_value() * scale
        if not abs(got - want) <= tol + 1e-12 * abs(want):
            bad.append((got, want))
    return bad


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
