"""Python mirror of the reference lmm::System API over the MI355X solver (liblmm_amd.so).

Same class and method names as src/kernel/lmm/maxmin.hpp (System, Constraint, Variable,
constraint_new / variable_new / expand / expand_add / update_* / solve / get_value ...), so tests
read like the reference's own maxmin_test.cpp.  Every call goes through the C ABI of
include/lmm/lmm_system.h; solving runs the HIP kernels (no CPU fallback: without a GPU, solve()
raises LmmError).
"""
import ctypes as ct
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "liblmm_amd.so")
# measurement only (A/B of two builds in one GPU call): LMM_AMD_LIB names another build of the same library
LIB_PATH = os.environ.get("LMM_AMD_LIB") or LIB_PATH

P, D, I, I64, U64 = ct.c_void_p, ct.c_double, ct.c_int, ct.c_int64, ct.c_uint64
PI, PD, PI64 = ct.POINTER(I), ct.POINTER(D), ct.POINTER(I64)

# cluster platforms (lmm_platform_params, include/lmm/lmm_system.h)
FAT_TREE, DRAGONFLY = 0, 1
SHARED, SPLITDUPLEX, FATPIPE = 0, 1, 2
CM02, LV08, L07 = 0, 1, 2


class PlatformParams(ct.Structure):
    _fields_ = [("topology", I), ("topo_parameters", ct.c_char_p), ("bw", D), ("lat", D), ("policy", I),
                ("loopback_bw", D), ("loopback_lat", D), ("limiter_bw", D), ("speed", D), ("model", I),
                ("crosstraffic", I), ("n_flows", I64), ("seed", U64), ("size_min", D), ("size_max", D),
                ("tcp_gamma", D)]


def platform_params(topology=FAT_TREE, topo_parameters="", bw=1.25e8, lat=5e-5, policy=SPLITDUPLEX, loopback_bw=0.0,
                    loopback_lat=0.0, limiter_bw=0.0, speed=1e9, model=LV08, crosstraffic=True, n_flows=1000,
                    seed=1, size_min=1e6, size_max=1e9, tcp_gamma=4194304.0):
    """A <cluster> (bw / lat / loopback / limiter as in examples/platforms/cluster_*.xml) and its flows."""
    return PlatformParams(topology, topo_parameters.encode(), bw, lat, policy, loopback_bw, loopback_lat, limiter_bw,
                          speed, model, int(crosstraffic), n_flows, seed, size_min, size_max, tcp_gamma)

class CommInfo(ct.Structure):
    """lmm_comm_info (include/lmm/lmm_system.h): a communication's action parameters."""
    _fields_ = [("latency", D), ("lat_current", D), ("sharing_penalty", D), ("bound", D)]


class LmmhipStats(ct.Structure):
    """lmmhip_stats (include/lmm/lmm_hip.h)."""
    _fields_ = [("rounds", I64), ("n_var", I64), ("n_cnst", I64), ("nnz", I64), ("device_ms", D),
                ("kernel_ms", D * 8), ("kernel_launches", I64 * 8)]


SIGNATURES = {
    # include/lmm/lmm_system.h
    "lmm_set_precision": (None, [D]),
    "lmm_get_precision": (D, []),
    "lmm_set_default_concurrency_limit": (None, [I]),
    "lmm_config_set": (I, [ct.c_char_p]),
    "lmm_config_get": (I, [ct.c_char_p, ct.c_char_p, I]),
    "lmm_constraint_new_id": (I64, [P, P, D]),
    "lmm_variable_new_id": (I64, [P, P, D, D, I64]),
    "lmm_constraint_get_id": (P, [P, I64]),
    "lmm_variable_get_id": (P, [P, I64]),
    "lmm_modified_action_ids": (I, [P, ct.POINTER(P), I]),
    "lmm_system_new": (P, [I, I]),
    "lmm_system_free": (None, [P]),
    "lmm_constraint_new": (I64, [P, D]),
    "lmm_constraint_unshare": (I, [P, I64]),
    "lmm_constraint_is_shared": (I, [P, I64]),
    "lmm_constraint_set_concurrency_limit": (I, [P, I64, I]),
    "lmm_constraint_concurrency": (I, [P, I64, PI, PI, PI]),
    "lmm_constraint_reset_concurrency_maximum": (I, [P, I64]),
    "lmm_constraint_get_usage": (D, [P, I64]),
    "lmm_constraint_get_variable_amount": (I, [P, I64]),
    "lmm_constraint_get_bound": (D, [P, I64]),
    "lmm_constraint_rank": (I, [P, I64]),
    "lmm_constraint_used": (I, [P, I64]),
    "lmm_constraint_elements": (I, [P, I64, PI, PD, PD, PI, I]),
    "lmm_variable_new": (I64, [P, D, D, I64]),
    "lmm_variable_free": (I, [P, I64]),
    "lmm_variable_free_all": (I, [P]),
    "lmm_variable_set_concurrency_share": (I, [P, I64, I]),
    "lmm_variable_get_value": (D, [P, I64]),
    "lmm_variable_get_bound": (D, [P, I64]),
    "lmm_variable_get_penalty": (D, [P, I64]),
    "lmm_variable_rank": (I, [P, I64]),
    "lmm_variable_number_of_constraints": (I, [P, I64]),
    "lmm_get_values": (I, [P, PI64, I64, PD]),
    "lmm_system_variables": (I, [P, PI64, I]),
    "lmm_system_active_constraints": (I, [P, PI64, I]),
    "lmm_modified_actions": (I, [P, PI64, I]),
    "lmm_clear_modified_actions": (I, [P]),
    "lmm_expand": (I, [P, I64, I64, D]),
    "lmm_expand_add": (I, [P, I64, I64, D]),
    "lmm_update_variable_bound": (I, [P, I64, D]),
    "lmm_update_variable_penalty": (I, [P, I64, D]),
    "lmm_update_constraint_bound": (I, [P, I64, D]),
    "lmm_solve": (I, [P]),
    "lmm_lmm_solve": (I, [P]),
    "lmm_is_modified": (I, [P]),
    "lmm_prepare": (I, [P]),
    "lmm_device_solve": (I, [P]),
    "lmm_fetch": (I, [P]),
    "lmm_last_stats": (I, [P, PI64, PD]),
    "lmm_set_resident": (I, [P, I]),
    "lmm_is_resident": (I, [P]),
    "lmm_pending_deltas": (I, [P, PI64]),
    "lmm_last_delta_records": (ct.c_int64, [P]),
    "lmm_table_sizes": (I, [P, PI64]),
    "lmm_resident_drain": (I, [P, PI64, PI64, ct.POINTER(ct.c_int32), PD, ct.POINTER(ct.c_uint8), ct.POINTER(ct.c_int32), PI64, ct.POINTER(ct.c_int32), PD, PD, ct.POINTER(ct.c_int32), PD, ct.POINTER(ct.c_uint8)]),
    "lmm_flat_export": (I, [P, PI64, PI64, ct.POINTER(ct.c_int32), PD, PD, PD, PD, ct.POINTER(ct.c_uint8), PI64]),
    "lmm_flat_export_order": (I, [P, I64, PI64]),
    "lmm_solve_batch": (I, [ct.POINTER(P), I]),
    "lmm_system_device_ctx": (P, [P]),
    "lmm_check_certificate": (I, [P, D, PD, PI64, PI64]),
    "lmm_gen_maxmin_bench": (I, [P, I, I, PI64, PI64, PI, PI]),
    "lmm_gen_synthetic": (I64, [P, I64, I64, I, U64, I, I, I, I, PI64]),
    "lmm_platform_size": (I, [ct.POINTER(PlatformParams), PI64, PI64]),
    "lmm_platform_dragonfly_coords": (I64, [ct.POINTER(PlatformParams), ct.POINTER(ct.c_int32), I64]),
    "lmm_gen_platform_flows": (I64, [P, ct.POINTER(PlatformParams), PI64, PI64]),
    "lmm_link_new": (I64, [P, I, D, I]),
    "lmm_communicate": (I64, [P, P, I, I64, PI64, PD, PD, I64, PI64, D, D, I, P]),
    "lmm_wifi_link_new": (I64, [P, I]),
    "lmm_communicate_ex": (I64, [P, P, I, I64, PI64, PD, PD, PD, I64, PI64, I, D, D, I, P]),
    "lmm_device_count": (I, []),
    "lmm_last_error": (ct.c_char_p, []),
    # include/lmm/lmm_hip.h
    "lmmhip_ctx_create": (I, [I, ct.POINTER(P)]),
    "lmmhip_ctx_destroy": (I, [P]),
    "lmmhip_upload": (I, [P, I64, I64, I64, PI64, ct.POINTER(ct.c_int32), PD, PD, PD, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_upload2": (I, [P, I64, I64, I64, PI64, ct.POINTER(ct.c_int32), PD, PD, PD, PD, ct.POINTER(ct.c_uint8),
                           PI64]),
    "lmmhip_update_vars": (I, [P, PD, PD]),
    "lmmhip_update_cnsts": (I, [P, PD]),
    "lmmhip_res_apply": (I, [P, I64, I64, I64, I64, PI64, ct.POINTER(ct.c_int32), PD, ct.POINTER(ct.c_uint8), I64, ct.POINTER(ct.c_int32), PI64, ct.POINTER(ct.c_int32), PD, PD, I64, ct.POINTER(ct.c_int32), PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_res_flatten": (I, [P, I64, ct.POINTER(ct.c_int32), D, PI64]),
    "lmmhip_res_values": (I, [P, I64, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_res_flatten_fair": (I, [P, I64, ct.POINTER(ct.c_int32), PI64]),
    "lmmhip_res_values_pinned": (I, [P, I64, ct.POINTER(P), ct.POINTER(P)]),
    "lmmhip_res_values_sliced": (I, [P, I64, I, ct.POINTER(P)]),
    "lmmhip_res_values_wait": (I, [P, I]),
    "lmmhip_res_refreshes": (I, [P, PI64]),
    "lmmhip_res_cross_refreshes": (I, [P, PI64]),
    "lmmhip_flat_download": (I, [P, PI64, P, P, P, P, P, P, P, P, P, P]),
    "lmmhip_solve": (I, [P, I, D]),
    "lmmhip_set_batch": (I, [P, I64, PI64, PI64]),
    "lmmhip_get_values": (I, [P, PD]),
    "lmmhip_get_var_rounds": (I, [P, ct.POINTER(ct.c_int32)]),
    "lmmhip_values_device_ptr": (I, [P, ct.POINTER(P)]),
    "lmmhip_get_saturated": (I, [P, ct.POINTER(ct.c_uint8)]),
    "lmmhip_get_touched_vars": (I, [P, ct.POINTER(ct.c_int32), I64, PI64]),
    "lmmhip_get_stats": (I, [P, P]),
    "lmmhip_set_profiling": (I, [P, I]),
    "lmmhip_launch_profile": (I, [P, PI, PI, ct.POINTER(ct.c_float), I]),
    "lmmhip_round_profile": (I, [P, PI64, PI64, I]),
    "lmmhip_vote_profile": (I, [P, PI64, PI64, I]),
    "lmmhip_vote_diag_profile": (I, [P, PI64, I]),
    "lmmhip_ctx_set_stream": (I, [P, P]),
    "lmmhip_ctx_use_own_stream": (I, [P]),
    "lmmhip_ctx_set_engine": (I, [P, I]),
    "lmmhip_engine_fallbacks": (I, [P, PI64]),
    "lmmhip_persist_profile": (I, [P, I, PI64, I64, PI64]),
    "lmmhip_persist_profile_blocks": (I, [P, PI64, I64, PI64, PI64]),
    "lmmhip_fb_shard_owner": (I, [P, I64, ct.POINTER(ct.c_int32), PI64, ct.POINTER(ct.c_int32), PD,
                                  ct.POINTER(ct.c_int32), I64, I64]),
    "lmmhip_fb_shard_begin": (I, [P, D, P, P, I64, P]),
    "lmmhip_fb_shard_step": (I, [P, I]),
    "lmmhip_fb_shard_pack_mu": (I, [P, P, P, P]),
    "lmmhip_fb_shard_poll": (I, [P, PI, PI64]),
    "lmmhip_fb_work": (I, [P, PI64]),
    "lmmhip_components": (I, [P, PI, PI, PI64]),
    "lmmhip_actions_upload": (I, [P, I64, ct.POINTER(ct.c_int32), PD, PD, PD, PD, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_next_event_full": (I, [P, I, PD]),
    "lmmhip_update_actions_full": (I, [P, I, D, D, D, PI64]),
    "lmmhip_actions_download": (I, [P, PD, PD, PD, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_actions_lazy_upload": (I, [P, PD, PD, PD, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_actions_lazy_update": (I, [P, I, D, D, D, I64, ct.POINTER(ct.c_int32), PI64]),
    "lmmhip_next_event_lazy": (I, [P, D, PD]),
    "lmmhip_actions_lazy_due": (I, [P, I, D, D, ct.POINTER(ct.c_int32), ct.POINTER(ct.c_uint8), I64, PI64]),
    "lmmhip_actions_lazy_download": (I, [P, PD, PD, PD, ct.POINTER(ct.c_uint8)]),
    "lmmhip_device_count": (I, []),
    "lmmhip_last_error": (ct.c_char_p, []),
    "lmmhip_build_id": (ct.c_char_p, []),
    "lmmhip_anatomy": (I, [P, ct.POINTER(ct.c_uint64), I64, PI64, ct.POINTER(ct.c_int32)]),
}

_lib = None


class LmmError(RuntimeError):
    pass


def _missing_symbol(name):
    def stub(*_a, **_k):
        raise LmmError(f"{name} not exported by the LMM_AMD_LIB build ({LIB_PATH})")
    return stub


def lib():
    """Load liblmm_amd.so (built by __graft_entry__.build() / `make -C simgrid_amd/csrc`)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 and loads it by path;
        # if ours (/opt/rocm) were loaded first, the two runtimes would race for the device and the
        # second one sees "no ROCm-capable device".  Loading torch first makes this library bind to
        # the already-loaded runtime (same soname).
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise LmmError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        l = ct.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name, None)
            if f is None and os.environ.get("LMM_AMD_LIB"):  # measurement A/B against an older build
                setattr(l, name, _missing_symbol(name))  # a call fails loudly instead of passing garbage
                continue
            if f is None:
                raise LmmError(f"{LIB_PATH} does not export {name}: rebuild it")
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _check(rc):
    if rc != 0:
        raise LmmError(lib().lmm_last_error().decode())
    return rc


def _check_hip(rc):
    if rc != 0:
        raise LmmError(lib().lmmhip_last_error().decode())
    return rc


def build_id():
    """The source hash compiled into the loaded library (lmmhip_build_id, simgrid_amd/build_id.py)."""
    return lib().lmmhip_build_id().decode()


def set_precision(p):
    lib().lmm_set_precision(p)


def get_precision():
    return lib().lmm_get_precision()


def config_set(key_value):
    """--cfg-style "key:value" (lmm_config_set): maxmin/precision, maxmin/concurrency-limit,
    maxmin/solver (hip, hip-auto, hip-persistent, hip-rounds), maxmin/resident (yes, no)."""
    _check(lib().lmm_config_set(key_value.encode()))


def config_get(key):
    buf = ct.create_string_buffer(64)
    if lib().lmm_config_get(key.encode(), buf, 64) < 0:
        raise LmmError(lib().lmm_last_error().decode())
    return buf.value.decode()


def device_count():
    return lib().lmm_device_count()


def platform_size(p):
    """(links, hosts) of the cluster `p` describes."""
    nl, nh = I64(), I64()
    _check(lib().lmm_platform_size(ct.byref(p), ct.byref(nl), ct.byref(nh)))
    return nl.value, nh.value


def dragonfly_coords(p):
    """(n_hosts x 4) array of DragonflyZone::rankId_to_coords (group, chassis, blade, node) of every host of the
    dragonfly `p` describes (lmm_platform_dragonfly_coords)."""
    n = lib().lmm_platform_dragonfly_coords(ct.byref(p), None, 0)
    if n < 0:
        raise LmmError(lib().lmm_last_error().decode())
    out = np.zeros(4 * n, np.int32)
    _check(0 if lib().lmm_platform_dragonfly_coords(ct.byref(p), out.ctypes.data_as(ct.POINTER(ct.c_int32)),
                                                    4 * n) == n else -1)
    return out.reshape(n, 4)


class Constraint:
    __slots__ = ("sys", "h")

    def __init__(self, sys, h):
        self.sys, self.h = sys, h

    def unshare(self):
        _check(lib().lmm_constraint_unshare(self.sys.h, self.h))

    def is_shared(self):
        return bool(lib().lmm_constraint_is_shared(self.sys.h, self.h))

    def set_concurrency_limit(self, l):
        _check(lib().lmm_constraint_set_concurrency_limit(self.sys.h, self.h, l))

    def concurrency(self):
        a, b, c = I(), I(), I()
        _check(lib().lmm_constraint_concurrency(self.sys.h, self.h, ct.byref(a), ct.byref(b), ct.byref(c)))
        return a.value, b.value, c.value

    def get_concurrency_limit(self):
        return self.concurrency()[2]

    def get_concurrency_maximum(self):
        return self.concurrency()[1]

    def reset_concurrency_maximum(self):
        _check(lib().lmm_constraint_reset_concurrency_maximum(self.sys.h, self.h))

    def get_usage(self):
        return lib().lmm_constraint_get_usage(self.sys.h, self.h)

    def get_variable_amount(self):
        return lib().lmm_constraint_get_variable_amount(self.sys.h, self.h)

    def get_bound(self):
        return lib().lmm_constraint_get_bound(self.sys.h, self.h)

    def get_id(self):
        return lib().lmm_constraint_get_id(self.sys.h, self.h)

    @property
    def rank(self):
        return lib().lmm_constraint_rank(self.sys.h, self.h)

    def elements(self):
        """[(var_rank, weight, value, enabled)] in System::print() order."""
        n = lib().lmm_constraint_elements(self.sys.h, self.h, None, None, None, None, 0)
        rk, w, x, en = (I * n)(), (D * n)(), (D * n)(), (I * n)()
        lib().lmm_constraint_elements(self.sys.h, self.h, rk, w, x, en, n)
        return [(rk[i], w[i], x[i], bool(en[i])) for i in range(n)]


class Variable:
    __slots__ = ("sys", "h")

    def __init__(self, sys, h):
        self.sys, self.h = sys, h

    def get_value(self):
        return lib().lmm_variable_get_value(self.sys.h, self.h)

    def get_bound(self):
        return lib().lmm_variable_get_bound(self.sys.h, self.h)

    def get_penalty(self):
        return lib().lmm_variable_get_penalty(self.sys.h, self.h)

    def get_id(self):
        return lib().lmm_variable_get_id(self.sys.h, self.h)

    def set_concurrency_share(self, s):
        _check(lib().lmm_variable_set_concurrency_share(self.sys.h, self.h, s))

    def get_number_of_constraint(self):
        return lib().lmm_variable_number_of_constraints(self.sys.h, self.h)

    @property
    def rank(self):
        return lib().lmm_variable_rank(self.sys.h, self.h)


class System:
    """lmm::System (maxmin.hpp:380) — FairBottleneck (maxmin.hpp:547) with kind=FAIR_BOTTLENECK."""

    MAXMIN, FAIR_BOTTLENECK = 0, 1

    def __init__(self, selective_update=False, kind=0):
        self.h = lib().lmm_system_new(int(selective_update), kind)
        if not self.h:
            raise LmmError(lib().lmm_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.lmm_system_free(self.h)
            self.h = None

    def constraint_new(self, id_, bound):
        h = lib().lmm_constraint_new_id(self.h, id_, bound) if isinstance(id_, int) else \
            lib().lmm_constraint_new(self.h, bound)
        if h < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return Constraint(self, h)

    def variable_new(self, id_, penalty, bound=-1.0, number_of_constraints=1):
        h = lib().lmm_variable_new_id(self.h, id_, penalty, bound, number_of_constraints) if isinstance(id_, int) \
            else lib().lmm_variable_new(self.h, penalty, bound, number_of_constraints)
        if h < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return Variable(self, h)

    def variable_free(self, v):
        _check(lib().lmm_variable_free(self.h, v.h))

    def variable_free_all(self):
        _check(lib().lmm_variable_free_all(self.h))

    def expand(self, c, v, w):
        _check(lib().lmm_expand(self.h, c.h, v.h, w))

    def expand_add(self, c, v, w):
        _check(lib().lmm_expand_add(self.h, c.h, v.h, w))

    def update_variable_bound(self, v, b):
        _check(lib().lmm_update_variable_bound(self.h, v.h, b))

    def update_variable_penalty(self, v, p):
        _check(lib().lmm_update_variable_penalty(self.h, v.h, p))

    def update_constraint_bound(self, c, b):
        _check(lib().lmm_update_constraint_bound(self.h, c.h, b))

    def constraint_used(self, c):
        return bool(lib().lmm_constraint_used(self.h, c.h))

    def solve(self):
        _check(lib().lmm_solve(self.h))

    def lmm_solve(self):
        _check(lib().lmm_lmm_solve(self.h))

    # split solve (bench): construction / device-resident solve / results
    def prepare(self):
        _check(lib().lmm_prepare(self.h))

    def device_solve(self):
        _check(lib().lmm_device_solve(self.h))

    def fetch(self):
        _check(lib().lmm_fetch(self.h))

    def last_stats(self):
        c, m = (I64 * 4)(), (D * 4)()
        lib().lmm_last_stats(self.h, c, m)
        return dict(rounds=c[0], n_var=c[1], n_cnst=c[2], nnz=c[3], device_ms=m[0], flatten_ms=m[1],
                    upload_ms=m[2], fetch_ms=m[3], delta_records=lib().lmm_last_delta_records(self.h))

    def components(self):
        """Connected components of the system the next solve() runs on (its device flatten, lmm_prepare):
        (label per dense variable, label per dense constraint, count) — see ctx_components."""
        self.prepare()
        st = self.last_stats()
        return ctx_components(self.device_ctx(), st["n_var"], st["n_cnst"])

    def fb_work(self):
        """The last FairBottleneck solve's work summed over its rounds (lmmhip_fb_work): (elements of the
        listed constraints, listed variables, listed constraints) — SURVEY.md §8(d)'s nnz_r, V_r, C_r."""
        w = (I64 * 3)()
        _check_hip(lib().lmmhip_fb_work(self.device_ctx(), w))
        return w[0], w[1], w[2]

    # resident mode (include/lmm/lmm_system.h, lmm_set_resident): HBM mirror + delta log + device flatten
    def set_resident(self, on=True):
        _check(lib().lmm_set_resident(self.h, int(bool(on))))

    def resident(self):
        return bool(lib().lmm_is_resident(self.h))

    def drain_deltas(self):
        """Drain the delta log without shipping it (test hook): dict of numpy arrays as lmmhip_res_apply
        would receive them."""
        ne, nv, nc = self.pending_deltas()
        sz = (I64 * 6)(ne, nv, nc, 0, 0, 0)
        if min(ne, nv, nc) < 0:  # whole system pending: every record
            _check(lib().lmm_table_sizes(self.h, sz))
        a = dict(e_id=np.zeros(sz[0], np.int64), e_cnst=np.zeros(sz[0], np.int32), e_w=np.zeros(sz[0]),
                 e_fl=np.zeros(sz[0], np.uint8), v_id=np.zeros(sz[1], np.int32), v_eb=np.zeros(sz[1], np.int64),
                 v_n=np.zeros(sz[1], np.int32), v_p=np.zeros(sz[1]), v_b=np.zeros(sz[1]),
                 c_id=np.zeros(sz[2], np.int32), c_b=np.zeros(sz[2]), c_fl=np.zeros(sz[2], np.uint8))
        ptr = lambda x: x.ctypes.data_as(ct.POINTER(np.ctypeslib.as_ctypes_type(x.dtype)))
        _check(lib().lmm_resident_drain(self.h, sz, *(ptr(a[k]) for k in (
            "e_id", "e_cnst", "e_w", "e_fl", "v_id", "v_eb", "v_n", "v_p", "v_b", "c_id", "c_b", "c_fl"))))
        n = dict(e=sz[0], v=sz[1], c=sz[2])
        out = {k: v[:n[k[0]]] for k, v in a.items()}
        out["totals"] = (sz[3], sz[4], sz[5])
        return out

    def device_flat(self):
        """The flattened system on the device (after prepare()): dict of numpy arrays."""
        ctx = self.device_ctx()
        n = (I64 * 3)()
        _check_hip(lib().lmmhip_flat_download(ctx, n, *([None] * 10)))
        nV, nC, nnz = n
        a = dict(var_ptr=np.zeros(nV + 1, np.uint32), csr_c=np.zeros(nnz, np.int32), csr_w=np.zeros(nnz),
                 cnst_ptr=np.zeros(nC + 1, np.uint32), csc_v=np.zeros(nnz, np.int32), csc_w=np.zeros(nnz),
                 pen=np.zeros(nV), vbound=np.zeros(nV), cbound=np.zeros(nC), cflags=np.zeros(nC, np.uint8))
        _check_hip(lib().lmmhip_flat_download(ctx, n, *(x.ctypes.data for x in a.values())))
        return a

    def pending_deltas(self):
        """(elements, variables, constraints) logged since the last solve; (-1, -1, -1) = whole system."""
        o = (I64 * 3)()
        _check(lib().lmm_pending_deltas(self.h, o))
        return tuple(o)

    def check_certificate(self, precision=None):
        """(max relative excess, #infeasible constraints, #variables without a bottleneck)."""
        ex, ni, nu = D(), I64(), I64()
        p = get_precision() if precision is None else precision
        _check(lib().lmm_check_certificate(self.h, p, ct.byref(ex), ct.byref(ni), ct.byref(nu)))
        return ex.value, ni.value, nu.value

    # ---- device-side measurement (lmmhip_* on this system's context) ----
    def device_ctx(self):
        c = lib().lmm_system_device_ctx(self.h)
        if not c:
            raise LmmError(lib().lmm_last_error().decode())
        return c

    ENGINE_PERSISTENT, ENGINE_ROUNDS, ENGINE_AUTO, ENGINE_FRONTIER = 0, 1, 2, 3

    def set_engine(self, engine):
        """Max-min engine of this system's device context (lmmhip_ctx_set_engine): ENGINE_PERSISTENT (one
        launch per solve), ENGINE_ROUNDS (one launch per phase per round), ENGINE_FRONTIER (one launch per
        phase per round, work proportional to what changed) or ENGINE_AUTO (default)."""
        _check_hip(lib().lmmhip_ctx_set_engine(self.device_ctx(), int(engine)))

    def engine_fallbacks(self):
        """Persistent solves of this system's context re-run by the multi-launch engine after a grid-barrier
        timeout (lmmhip_engine_fallbacks)."""
        n = ct.c_int64()
        _check_hip(lib().lmmhip_engine_fallbacks(self.device_ctx(), ct.byref(n)))
        return n.value

    def device_values(self):
        """Values of the last solve in the device's dense (CSR) order (lmmhip_get_values)."""
        n = self.last_stats()["n_var"]
        x = np.empty(n, np.float64)
        _check_hip(lib().lmmhip_get_values(self.device_ctx(), x.ctypes.data_as(PD)))
        return x

    def device_var_rounds(self):
        """1 + the device round that fixed each variable of the last max-min solve, dense order
        (lmmhip_get_var_rounds; 0 = never)."""
        n = self.last_stats()["n_var"]
        r = np.empty(n, np.int32)
        _check_hip(lib().lmmhip_get_var_rounds(self.device_ctx(), r.ctypes.data_as(ct.POINTER(ct.c_int32))))
        return r

    def device_saturated(self):
        """Saturated set of the last solve, dense constraint order (lmmhip_get_saturated)."""
        out = np.empty(self.last_stats()["n_cnst"], np.uint8)
        _check_hip(lib().lmmhip_get_saturated(self.device_ctx(), out.ctypes.data_as(ct.POINTER(ct.c_uint8))))
        return out.astype(bool)

    def device_touched_vars(self):
        """Variables of the solved system in the context's id space (lmmhip_get_touched_vars)."""
        n = I64()
        ctx = self.device_ctx()
        _check_hip(lib().lmmhip_get_touched_vars(ctx, None, 0, ct.byref(n)))
        out = np.empty(n.value, np.int32)
        _check_hip(lib().lmmhip_get_touched_vars(ctx, out.ctypes.data_as(ct.POINTER(ct.c_int32)), n.value,
                                                 ct.byref(n)))
        return out

    def persist_profile(self, on=True):
        """Barrier timestamps of the persistent engine (lmmhip_persist_profile): (last arrival, exit) per
        barrier of the last solve, in 10-ns ticks, as an (n, 2) array."""
        ctx = self.device_ctx()
        n = I64()
        cap = 1 << 17
        t = np.zeros(cap, np.int64)
        _check_hip(lib().lmmhip_persist_profile(ctx, int(on), t.ctypes.data_as(PI64), cap, ct.byref(n)))
        return t[:2 * n.value].reshape(-1, 2)

    def persist_profile_blocks(self):
        """Per-workgroup (arrival, exit) ticks of the profiled persistent solve: (barriers, workgroups, 2)."""
        ctx = self.device_ctx()
        cap = 2 * 1024 * 1024
        t = np.zeros(cap, np.int64)
        nb, nw = I64(), I64()
        _check_hip(lib().lmmhip_persist_profile_blocks(ctx, t.ctypes.data_as(PI64), cap, ct.byref(nb), ct.byref(nw)))
        return t[:2 * nb.value * nw.value].reshape(nb.value, nw.value, 2)

    def set_profiling(self, on):
        if lib().lmmhip_set_profiling(self.device_ctx(), int(on)) != 0:
            raise LmmError(lib().lmmhip_last_error().decode())

    def launch_profile(self):
        """(slot, round, ms) arrays of every launch of the last profiled solve."""
        c = self.device_ctx()
        n = lib().lmmhip_launch_profile(c, None, None, None, 0)
        if n < 0:
            raise LmmError(lib().lmmhip_last_error().decode())
        slot, rnd = np.empty(n, np.int32), np.empty(n, np.int32)
        ms = np.empty(n, np.float32)
        lib().lmmhip_launch_profile(c, slot.ctypes.data_as(PI), rnd.ctypes.data_as(PI),
                                    ms.ctypes.data_as(ct.POINTER(ct.c_float)), n)
        return slot, rnd, ms

    def round_profile(self):
        """Alive variables / elements at the start of every round of the last solve."""
        c = self.device_ctx()
        cap = 1 << 20
        av, ae = np.zeros(cap, np.int64), np.zeros(cap, np.int64)
        r = lib().lmmhip_round_profile(c, av.ctypes.data_as(PI64), ae.ctypes.data_as(PI64), cap)
        if r < 0:
            raise LmmError(lib().lmmhip_last_error().decode())
        return av[:r], ae[:r]

    def vote_profile(self):
        """Re-evaluated variables / elements per round of the last profiled maxmin solve."""
        c = self.device_ctx()
        cap = 1 << 16
        rv, re_ = np.zeros(cap, np.int64), np.zeros(cap, np.int64)
        r = lib().lmmhip_vote_profile(c, rv.ctypes.data_as(PI64), re_.ctypes.data_as(PI64), cap)
        if r < 0:
            raise LmmError(lib().lmmhip_last_error().decode())
        return rv[:r], re_[:r]

    def vote_diag_profile(self):
        """LMMHIP_VOTE_DIAG runs: per round (target-changed rows, sensitive rows, queued rows, changed constraints,
        distinct targets of the queued rows, sum of their CSC degrees, queued sensitive rows, 0)."""
        c = self.device_ctx()
        cap = 1 << 14
        out = np.zeros(8 * cap, np.int64)
        r = lib().lmmhip_vote_diag_profile(c, out.ctypes.data_as(PI64), cap)
        if r < 0:
            raise LmmError(lib().lmmhip_last_error().decode())
        return out[:8 * r].reshape(r, 8)

    @property
    def modified(self):
        return bool(lib().lmm_is_modified(self.h))

    def variables(self):
        n = lib().lmm_system_variables(self.h, None, 0)
        arr = (I64 * n)()
        lib().lmm_system_variables(self.h, arr, n)
        return [Variable(self, arr[i]) for i in range(n)]

    def active_constraints(self):
        n = lib().lmm_system_active_constraints(self.h, None, 0)
        arr = (I64 * n)()
        lib().lmm_system_active_constraints(self.h, arr, n)
        return [Constraint(self, arr[i]) for i in range(n)]

    def modified_action_ids(self):
        """The opaque ids (Action*) of the modified set, in modified_actions() order."""
        n = lib().lmm_modified_action_ids(self.h, None, 0)
        arr = (P * n)()
        lib().lmm_modified_action_ids(self.h, arr, n)
        return [arr[i] for i in range(n)]

    def modified_actions(self):
        n = lib().lmm_modified_actions(self.h, None, 0)
        arr = (I64 * n)()
        lib().lmm_modified_actions(self.h, arr, n)
        return [Variable(self, arr[i]) for i in range(n)]

    def clear_modified_actions(self):
        _check(lib().lmm_clear_modified_actions(self.h))

    # ---- generators ----
    def gen_maxmin_bench(self, klass, run):
        C, V = {0: (10, 10), 1: (100, 100), 2: (2000, 2000), 3: (20000, 20000)}[klass]
        cs, vs = (I64 * C)(), (I64 * V)()
        a, b = I(), I()
        if lib().lmm_gen_maxmin_bench(self.h, klass, run, cs, vs, ct.byref(a), ct.byref(b)) < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return ([Constraint(self, cs[i]) for i in range(C)], [Variable(self, vs[i]) for i in range(V)],
                a.value, b.value)

    def gen_synthetic(self, nb_cnst, nb_var, k=8, seed=1, max_share=2, penalty_mix=0, bounded_permille=0,
                      fatpipe_permille=0, want_vars=True):
        vs = np.empty(nb_var, dtype=np.int64) if want_vars else None
        r = lib().lmm_gen_synthetic(self.h, nb_cnst, nb_var, k, seed, max_share, penalty_mix, bounded_permille,
                                    fatpipe_permille, vs.ctypes.data_as(PI64) if want_vars else None)
        if r < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return vs

    def gen_platform_flows(self, p, want_vars=True):
        """Links (+ L07 CPUs) and p.n_flows flows of a cluster platform: (constraint ids, variable ids)."""
        nl, nh = platform_size(p)
        cs = np.empty(nl + (nh if p.model == L07 else 0), dtype=np.int64)
        vs = np.empty(p.n_flows, dtype=np.int64) if want_vars else None
        r = lib().lmm_gen_platform_flows(self.h, ct.byref(p), cs.ctypes.data_as(PI64),
                                         vs.ctypes.data_as(PI64) if want_vars else None)
        if r < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return cs, vs

    def link_new(self, model, bw, fatpipe=False):
        """A link's constraint (lmm_link_new: NetworkCm02Link, bound = bandwidth factor * bw)."""
        h = lib().lmm_link_new(self.h, model, bw, int(fatpipe))
        if h < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return Constraint(self, h)

    def wifi_link_new(self, model):
        """A WIFI access point's constraint (lmm_wifi_link_new: NetworkWifiLink, bandwidth 1 / bandwidth factor)."""
        h = lib().lmm_wifi_link_new(self.h, model)
        if h < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return Constraint(self, h)

    def communicate(self, model, route, back=(), rate=-1.0, tcp_gamma=4194304.0, paid=False, id_=None,
                    crosstraffic=None):
        """NetworkCm02Model::communicate's LMM part (lmm_communicate): route = [(Constraint, bw, lat)] in route
        order — a WIFI access point as (Constraint, bw, lat, (src_rate, dst_rate)), the stations' rates on it
        (-1: not associated; lmm_communicate_ex) —, back = the back route's Constraints (crosstraffic), id_ = the
        variable's opaque id (an int: the action; modified_action_ids() reports it), crosstraffic = the
        network/crosstraffic configuration (None: on iff `back` has links).  Returns (Variable,
        dict(latency, lat_current, sharing_penalty, bound))."""
        xt = bool(len(back)) if crosstraffic is None else bool(crosstraffic)
        n = len(route)
        rc = np.array([r[0].h for r in route], dtype=np.int64)
        rb = np.array([r[1] for r in route], dtype=np.float64)
        rl = np.array([r[2] for r in route], dtype=np.float64)
        bc = np.array([c.h for c in back], dtype=np.int64)
        info = CommInfo()
        if any(len(r) > 3 for r in route) or xt != bool(len(back)):
            rr = np.array([r[3] if len(r) > 3 else (0.0, 0.0) for r in route], dtype=np.float64).reshape(-1)
            h = lib().lmm_communicate_ex(self.h, id_, model, n, rc.ctypes.data_as(PI64), rb.ctypes.data_as(PD),
                                         rl.ctypes.data_as(PD), rr.ctypes.data_as(PD), len(bc),
                                         bc.ctypes.data_as(PI64), int(xt), rate, tcp_gamma, int(paid), ct.byref(info))
        else:
            h = lib().lmm_communicate(self.h, id_, model, n, rc.ctypes.data_as(PI64), rb.ctypes.data_as(PD),
                                      rl.ctypes.data_as(PD), len(bc), bc.ctypes.data_as(PI64), rate, tcp_gamma,
                                      int(paid), ct.byref(info))
        if h < 0:
            raise LmmError(lib().lmm_last_error().decode())
        return Variable(self, h), {k: getattr(info, k) for k, _ in CommInfo._fields_}

    def values_of(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        out = np.empty(len(ids), dtype=np.float64)
        lib().lmm_get_values(self.h, ids.ctypes.data_as(PI64), len(ids), out.ctypes.data_as(PD))
        return out


def ctx_components(ctx, nv, nc):
    """lmmhip_components on a device context holding an uploaded / flattened system of nv variables and nc
    constraints: (var labels, cnst labels, count), compact ids in the order of each component's smallest
    node (variables first, then constraints)."""
    vl, cl, n = np.empty(nv, np.int32), np.empty(nc, np.int32), I64()
    _check_hip(lib().lmmhip_components(ctx, vl.ctypes.data_as(PI), cl.ctypes.data_as(PI), ct.byref(n)))
    return vl, cl, n.value


def solve_batch(systems):
    """Solve independent systems as one device launch sequence (disjoint union)."""
    arr = (P * len(systems))(*[s.h for s in systems])
    _check(lib().lmm_solve_batch(arr, len(systems)))


def make_new_maxmin_system(selective_update=False):
    return System(selective_update, System.MAXMIN)


def make_new_fair_bottleneck_system(selective_update=False):
    return System(selective_update, System.FAIR_BOTTLENECK)
