#!/usr/bin/env python
"""LMM solve throughput on MI355X (BASELINE.json metric: "LMM solve throughput (vars/s) at
1/2/4/8 GPUs; % of HBM peak").

Workload (BASELINE.json configs[1]): a maxmin_bench-style synthetic system of
10^6 constraints x 10^7 variables x 8 elements/variable, built through the lmm::System API and
solved with System::lmm_solve semantics on one MI355X.  One step = one full solve of that system
with its inputs already resident in HBM (flatten + upload happen before the timed region, like
maxmin_bench.cpp:81-83 times only solve()).  With --gpus N every rank solves its own independent
system (seed = rank + 1): a parameter sweep, weak scaling, no data-path collective.

Prints ONE JSON line on rank 0 (contract in the task statement), with a `roofline` object for the
dominant kernel (HIP events on the solver's own stream, per-launch algorithmic bytes from the
per-round work profile) and a `cpu_baseline` object (the oracle, single-threaded, on a bounded
1/10-scale sample of the same generator).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
SLOT_NAMES = {0: "mm_init_cnsts", 1: "mm_init_vars", 2: "mm_vote", 3: "mm_ready", 4: "mm_saturate",
              5: "mm_update", 6: "compaction", 7: "vote_diag"}


def traffic_json(workload):
    """The newest rocprofv3 PMC summary of this workload (scripts/parse_rocprof.py: FETCH_SIZE and
    WRITE_SIZE passes of `bench.py --workload <w>`, counter bytes per solve over the solve's kernels)."""
    for k in (9, 8, 7, 6, 5, 4, 3):
        p = os.path.join(ROOT, "profiles", f"r0{k}_traffic_{workload}.json")
        if os.path.exists(p):
            return p
    return None


def solve_traffic(workload):
    """(HBM bytes per solve from the PMC counters with the gfx950 streaming-read correction — 2 x FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md HBM —, the raw FETCH + WRITE, the summary's path) or Nones."""
    p = traffic_json(workload)
    if p is None:
        return None, None, None
    with open(p) as f:
        t = json.load(f)
    return int(t["solve_counter_bytes_fetch_x2"]), int(t["solve_counter_bytes_raw"]), os.path.relpath(p, ROOT)


def kernel_class(e):
    """The dominant request class of one kernel's counters: read, write or atomic."""
    rd = e.get("TCC_EA0_RDREQ_sum_per_launch", 0.0)
    wr = e.get("TCC_EA0_WRREQ_sum_per_launch", 0.0)
    at = e.get("TCC_EA0_ATOMIC_sum_per_launch", 0.0)
    return max((("read", rd), ("write", wr - at), ("atomic", at)), key=lambda kv: kv[1])[0]


def class_frac(e, rates):
    """A kernel's request rate over the calibrated rate of its dominant class (None without calibration)."""
    r = rates.get({"read": "gather<double>", "write": "scatter_u8", "atomic": "atomics_f64"}[kernel_class(e)])
    return round(e["requests_per_s"] / r, 3) if r and e.get("requests_per_s") else None


def request_roofline(workload, ms):
    """The request-rate roofline: memory-side requests per solve (rocprofv3 TCC_EA0_RDREQ_sum +
    TCC_EA0_WRREQ_sum over the solve's kernels, scripts/profile.sh PARTS=req, scripts/parse_rocprof.py) over the
    solve's time, against the best rate the calibration kernels (scripts/ubench_gather.hip: random 8-B gathers,
    random fp64 atomics, random byte stores on 8-80 MB tables) reached under the same counters on this chip."""
    for k in (9, 8, 7, 6, 5):
        p = os.path.join(ROOT, "profiles", f"r0{k}_requests_{workload}.json")
        if os.path.exists(p):
            break
    else:
        return None
    with open(p) as f:
        t = json.load(f)
    per = float(t["solve_requests"])
    ach = per / (ms * 1e-3)
    rates = {k: float(v["requests_per_s"]) for k, v in (t.get("calibration") or {}).items()
             if v.get("requests_per_s")}
    # the request-rate roofline: each class of the solve's requests at the rate the calibration kernel of that
    # class reached on this chip — reads as random 8-B gathers, plain writes as random byte stores, atomics as
    # random fp64 atomics — one after the other (the floor if the classes do not overlap) and side by side (if
    # they overlap perfectly)
    rd, wr, at = float(t["solve_rdreq"]), float(t["solve_wrreq"]), float(t["solve_atomic"])
    cls = {"read": (rd, rates.get("gather<double>")), "write": (wr - at, rates.get("scatter_u8")),
           "atomic": (at, rates.get("atomics_f64"))}
    floor = None
    if all(r for _, r in cls.values()):
        parts = {k: n / r * 1e3 for k, (n, r) in cls.items()}
        floor = {"serial_ms": round(sum(parts.values()), 3), "overlap_ms": round(max(parts.values()), 3),
                 "class_ms": {k: round(v, 3) for k, v in parts.items()},
                 "class_rates_per_s": {k: round(r, 1) for k, (_, r) in cls.items()},
                 "frac_serial": round(sum(parts.values()) / ms, 4), "frac_overlap": round(max(parts.values()) / ms, 4)}
    best = max(rates, key=rates.get) if rates else None
    upload = ("rs_", "rocprim", "__amd", "mm_elem_usage", "mm_dup_check", "fr_c2s", "fbp_")  # not the solve's kernels
    top = sorted(((k, e) for k, e in t["kernels"].items() if e.get("requests_per_s") and not k.startswith(upload)),
                 key=lambda kv: -(kv[1]["TCC_EA0_RDREQ_sum"] + kv[1]["TCC_EA0_WRREQ_sum"]))[:4]
    return {"unit": "requests/s", "per_solve": round(per), "rdreq_per_solve": round(float(t["solve_rdreq"])),
            "wrreq_per_solve": round(float(t["solve_wrreq"])), "atomic_per_solve": round(float(t["solve_atomic"])),
            "achieved": round(ach, 1),
            "ceiling": round(per / (floor["serial_ms"] * 1e-3), 1) if floor else None,
            "frac": floor["frac_serial"] if floor else None, "floor": floor,
            "ceiling_note": "the solve's reads / plain writes / atomics at the calibrated random-gather / random-store /"
                            " random-atomic rates, one class after the other (frac = that floor / the solve time;"
                            " floor.frac_overlap: all classes side by side)",
            "calibration_rates": {k: round(v, 1) for k, v in rates.items()},
            "per_kernel": {k: {"requests_per_launch": round(e["TCC_EA0_RDREQ_sum_per_launch"] +
                                                            e["TCC_EA0_WRREQ_sum_per_launch"]),
                               "requests_per_s": round(e["requests_per_s"], 1), "avg_us": round(e["avg_ns"] / 1e3, 2),
                               # (VERDICT r05 Next #5) the kernel's rate against the ceiling of its dominant class:
                               # reads at the calibrated random-gather rate, writes / atomics at theirs
                               "class": kernel_class(e),
                               "class_frac": class_frac(e, rates)}
                           for k, e in top},
            "source": os.path.relpath(p, ROOT)}


def roofline_obj(alg_bytes, ms, workload, note, gpus=1):
    """Solve-level roofline: the algorithmic bytes of one solve (all `gpus` ranks' parts)
    over the solve's time, against `gpus` x the HBM peak.  The PMC traffic summaries are single-GPU runs:
    reported at N = 1 only."""
    ach = alg_bytes / (ms * 1e-3) / 1e9
    peak = HBM_PEAK_GBS * gpus
    traffic, raw, src = solve_traffic(workload) if gpus == 1 else (None, None, None)
    out = {"bound": "hbm", "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
           "frac": round(ach / peak, 5), "traffic": traffic, "traffic_raw": raw, "traffic_source": src,
           "traffic_unit": "bytes per solve (rocprofv3 PMC, 2 x FETCH_SIZE + WRITE_SIZE over the solve kernels)",
           "alg_bytes": int(alg_bytes), "kernel": "whole solve", "alg_model": note}
    if raw:
        # the HBM rate the counters saw over the solve's time (VERDICT r05 Weak #4): where it is below `achieved` the
        # algorithmic bytes include work served on chip (LDS, L2) — the solve is not HBM-bound, `frac` overstates it
        cfrac = raw / (ms * 1e-3) / 1e9 / peak
        out["counter_frac"] = round(cfrac, 5)
        out["counter_frac_note"] = ("raw FETCH + WRITE counter bytes per solve over the solve time / HBM peak"
                                    + ("; below frac: part of the algorithmic traffic never reaches HBM (LDS / L2"
                                       " resident), so the kernels are bound by on-chip latency, not by HBM"
                                       if raw < alg_bytes else ""))
    return out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_info():
    """CPU model and core counts of the box the CPU baseline ran on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity}


def mean_sd(xs):
    import numpy as np

    a = np.asarray(xs, dtype=np.float64)
    return float(a.mean()), float(a.std(ddof=1)) if len(a) > 1 else 0.0


def kernel_bytes(slot, nV, nC, av, ae, fv, fe, rv, re_):
    """Algorithmic bytes one launch must move: `av`/`ae` alive variables / elements at
    the start of the round, `fv`/`fe` variables / elements fixed in it, `rv`/`re_` variables /
    elements re-evaluated by the vote phase."""
    if slot == 2:  # mm_vote: per alive row rtgt 4 + skey 2 + chg[t] 2;
        #            per re-evaluated row cvar 4 + vstate 4 + crow 8 + vbound 8 + pen 8 + rtgt/skey 6;
        #            per re-evaluated element ccol 4 + key 2
        return av * 8 + rv * 38 + re_ * 6
    if slot == 3:  # mm_ready: list entry 4 + key 2 + nvote 4 per alive constraint
        return nC * 10
    if slot == 4:  # mm_saturate: per fixed var csc idx 4 + vstate 4 + pen 8 + x 8 + row ptr 8;
        #            per fixed element csr idx 4 + w 8 + key 2 + cflags 1 + touch 1 + atomics dcnt 4, drem 8, duse 8
        return fv * 32 + fe * 36
    if slot == 5:  # mm_update: key 2 + touch flag 1 per constraint; per touched constraint ~56 B of state
        return nC * 3 + min(fe, nC) * 56
    if slot == 0:  # mm_init_cnsts: CSC idx 4 + w 8 + pen gather 8 per element; bound 8 + state writes 48 per constraint
        return 20 * ae + 56 * nC
    if slot == 1:
        return nV * 25
    return 0


def main():
    if os.environ.get("LMM_SEGV_TRACE") == "1":  # diagnostics: native backtrace of a crash (scripts/segv_trace.c)
        import ctypes

        ctypes.CDLL(os.path.join(ROOT, "scripts", "libsegv_trace.so"))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cnst", type=int, default=1_000_000)
    ap.add_argument("--vars", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-div", type=int, default=10, help="CPU baseline sample = 1/div of the workload")
    ap.add_argument("--profile-json", default=None, help="write the per-launch profile here")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2 = the BASELINE metric's config (default); c3/c4/c5 = the other SURVEY.md §8(d) configs")
    ap.add_argument("--flows", type=int, default=None, help="c4/c5: number of flows (default 1e5 / 1e7)")
    ap.add_argument("--c3-weak", action="store_true",
                    help="c3: 4096 systems per rank (weak scaling; default: 4096 in total, strong scaling)")
    ap.add_argument("--variant", default="plain", choices=["plain", "stress"],
                    help="c2: stress = 5%% FATPIPE constraints, 10%% bounded variables, penalties {1,2,4}")
    ap.add_argument("--dropin-steps", type=int, default=3,
                    help="c2: System::solve() steps through the public API after the timed region (0 = skip)")
    ap.add_argument("--cpu-reps", type=int, default=3, help="CPU baseline repetitions (mean and sd reported)")
    ap.add_argument("--cpu-worker", nargs=3, metavar=("WORKLOAD", "LO", "HI"), default=None,
                    help=argparse.SUPPRESS)  # child process of the N-process CPU baseline
    args = ap.parse_args()
    if args.cpu_worker:
        return cpu_worker(*args.cpu_worker)
    if args.workload != "c2":
        return run_config(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    from simgrid_amd import lmm

    assert torch.cuda.is_available(), "bench.py needs an MI355X"
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- construction (not timed) ----
    t = time.time()
    s = lmm.System(False)
    gen_kw = STRESS_KW if args.variant == "stress" else {}
    vs = s.gen_synthetic(args.cnst, args.vars, args.k, seed=rank + 1, want_vars=args.dropin_steps > 0, **gen_kw)
    t_gen = time.time() - t
    t = time.time()
    s.prepare()  # flatten + upload: inputs resident in HBM from here on
    st = s.last_stats()
    log(f"[rank {rank}] built {args.cnst}x{args.vars}x{args.k} in {t_gen:.1f}s, flatten {st['flatten_ms']:.0f} ms,"
        f" upload {st['upload_ms']:.0f} ms: nV={st['n_var']} nC={st['n_cnst']} nnz={st['nnz']}")

    for _ in range(args.warmup):
        s.device_solve()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.device_solve()
    barrier()
    elapsed = time.perf_counter() - t0
    st = s.last_stats()
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    n_vars_total = args.vars * world * args.steps
    value = n_vars_total / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # ---- profiled solve: per-launch HIP events on the solver's stream + per-round work ----
    s.set_profiling(True)
    s.device_solve()
    s.set_profiling(False)
    slot, rnd, ms = s.launch_profile()
    av, ae = s.round_profile()
    rv, re_ = s.vote_profile()
    nV, nC, nnz, rounds = st["n_var"], st["n_cnst"], st["nnz"], st["rounds"]
    per_kernel = {}
    for k in sorted(set(slot.tolist())):
        sel = slot == k
        byts = 0
        for r in rnd[sel]:
            if 0 <= r < len(av):
                nxt_v = int(av[r + 1]) if r + 1 < len(av) else 0
                nxt_e = int(ae[r + 1]) if r + 1 < len(ae) else 0
                rr = (int(rv[r]), int(re_[r])) if r < len(rv) else (0, 0)
                byts += kernel_bytes(int(k), nV, nC, int(av[r]), int(ae[r]), int(av[r]) - nxt_v,
                                     int(ae[r]) - nxt_e, *rr)
            elif r < 0:
                byts += kernel_bytes(int(k), nV, nC, nV, nnz, 0, 0, 0, 0)
        per_kernel[SLOT_NAMES[int(k)]] = dict(launches=int(sel.sum()), total_ms=float(ms[sel].sum()),
                                              avg_us=float(1000 * ms[sel].mean()), alg_bytes=int(byts))
    dom = max(per_kernel, key=lambda n: per_kernel[n]["total_ms"])
    d = per_kernel[dom]
    kach = d["alg_bytes"] / (d["total_ms"] * 1e-3) / 1e9
    solve_alg = 56 * nnz + 24 * nV + 32 * nC
    roofline = roofline_obj(solve_alg * world, ms_per_step, "c2" if args.variant == "plain" else "c2_stress",
                            "SURVEY.md §8(d) lmm_solve: 56 nnz + 24 V + 32 C bytes per solve (x ranks)", gpus=world)
    if world == 1 and args.variant == "plain":
        roofline["requests"] = request_roofline("c2", ms_per_step)
    # secondary: the dominant kernel's own per-launch byte model (kernel_bytes) over its HIP-event time
    roofline["dominant_kernel"] = {"name": dom, "avg_us": round(d["avg_us"], 2), "launches": d["launches"],
                                   "alg_bytes_per_launch": int(d["alg_bytes"] / max(1, d["launches"])),
                                   "achieved_gbs": round(kach, 1), "kernel_frac": round(kach / HBM_PEAK_GBS, 4)}
    if args.profile_json and rank == 0:
        extra = {}
        if os.environ.get("LMMHIP_VOTE_DIAG"):
            extra["vote_diag"] = s.vote_diag_profile().tolist()
        with open(args.profile_json, "w") as f:
            json.dump(dict(per_kernel=per_kernel, rounds=rounds, alive_vars=av.tolist(), alive_elems=ae.tolist(), **extra,
                           reeval_vars=rv.tolist(), reeval_elems=re_.tolist(),
                           device_ms=st["device_ms"], launch_slot=slot.tolist(), launch_round=rnd.tolist(),
                           launch_ms=ms.tolist()), f)

    # ---- drop-in step: System::solve() through the public API after simulation-side mutations ----
    # Each step first changes 1e4 variable penalties and 1e3 constraint bounds through the API (untimed: the
    # simulation's own work), then times solve() = delta-log ship + device flatten or refresh + device solve
    # + value scatter into the host System (resident mode, the default).
    dropin = None
    if args.dropin_steps > 0:
        rng = np.random.default_rng(9 + rank)
        rows = []
        for _ in range(args.dropin_steps):
            for i in rng.choice(args.vars, 10_000, replace=False):
                s.update_variable_penalty(lmm.Variable(s, int(vs[i])), float(rng.choice([0.5, 1.0, 2.0])))
            for c in rng.choice(args.cnst, 1_000, replace=False):
                s.update_constraint_bound(lmm.Constraint(s, int(c)), float(rng.uniform(0.5, 10.0)))
            t1 = time.perf_counter()
            s.solve()
            wall = (time.perf_counter() - t1) * 1e3
            st2 = s.last_stats()
            rows.append((wall, st2["flatten_ms"], st2["upload_ms"], st2["device_ms"], st2["fetch_ms"]))
        med = np.median(np.array(rows), axis=0)
        dropin = {"solve_step_ms": round(float(med[0]), 2), "host_ms": round(float(med[1]), 2),
                  "ship_and_device_flatten_ms": round(float(med[2]), 2), "device_solve_ms": round(float(med[3]), 2),
                  "value_scatter_ms": round(float(med[4]), 2), "steps": args.dropin_steps,
                  "vars_per_s": round(args.vars / (float(med[0]) * 1e-3), 1),
                  "mutations_per_step": "1e4 penalty + 1e3 constraint-bound updates (untimed)",
                  "path": "System::solve(), resident mode (default): median over the steps"}

    # ---- CPU baseline: the oracle (single-threaded restatement), bounded sample, rank 0, N=1 ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import pyoracle as O

        div = args.cpu_sample_div
        times, cpu_rounds = [], 0
        for _ in range(max(1, args.cpu_reps)):  # a fresh system per repetition (solve() runs once per change)
            o = O.System(False)
            o.gen_synthetic(args.cnst // div, args.vars // div, args.k, seed=1, want_vars=False, **gen_kw)
            times.append(o.timed_solve())
            cpu_rounds = o.last_rounds
            del o
        m, sd = mean_sd(times)
        parity = c2_sample_parity(args, div, gen_kw)
        full = c2_full_size_baseline(args, value) if args.variant == "plain" else None
        cpu = {"value": round((args.vars // div) / m, 1), "unit": "vars/s", "cores": 1, "kind": "port",
               "sample": f"same generator at 1/{div} scale ({args.cnst // div} cnst x {args.vars // div} vars x {args.k}),"
                         f" solve() timed with steady_clock, {len(times)} reps: {m:.3f} +- {sd:.3f} s,"
                         f" {cpu_rounds} sequential rounds",
               "reps": len(times), "solve_s_mean": round(m, 4), "solve_s_sd": round(sd, 4),
               "gpu_vs_oracle": parity, **host_info()}
        cpu["gpu_vs_sample_ratio"] = round(value / cpu["value"], 1)
        if full:
            cpu["full_size"] = full

    if rank == 0:
        out = {
            "metric": "LMM solve throughput (vars/s)", "value": round(value, 1), "unit": "vars/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (maxmin_bench-style generator, splitmix64 seed = rank+1)",
            "config": {"workload": "C2: 1e6 constraints x 1e7 variables x 8 elements/var, one lmm_solve per step"
                                   + (" (stress variant: 5% FATPIPE, 10% bounded, penalties {1,2,4})"
                                      if args.variant == "stress" else ""),
                       "nb_cnst": args.cnst, "nb_var": args.vars, "elems_per_var": args.k, "variant": args.variant,
                       "active_vars": nV, "active_cnsts": nC, "nnz": nnz, "device_rounds": rounds,
                       "device_solve_ms": round(ms_per_step, 3), "dropin_step": dropin,
                       "parallelism": f"replicas x{world} (independent systems per rank)"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    del s  # free the device context while the HIP runtime is up (not in interpreter teardown)
    if dist is not None:
        dist.destroy_process_group()


def c2_full_size_baseline(args, gpu_value):
    """The reference algorithm's throughput AT the metric's configuration, from the committed full-size fixture
    (tests/golden/c2_full_sample.npz: the oracle's one solve of the full C2 system, 449,160 sequential rounds of
    the O(rounds x constraints) light-table rescan, maxmin.cpp:663-680) — measured once in the build container,
    not on this box's host (tests/golden/c2_full_sample_meta.json); the timed 1/10 sample above is the
    GPU box's own CPU leg."""
    import numpy as np

    if (args.cnst, args.vars, args.k) != (1_000_000, 10_000_000, 8):
        return None
    path = os.path.join(ROOT, "tests", "golden", "c2_full_sample.npz")
    meta = os.path.join(ROOT, "tests", "golden", "c2_full_sample_meta.json")
    if not os.path.exists(path):
        return None
    fx = np.load(path)
    secs = float(fx["oracle_seconds"])
    host = None
    if os.path.exists(meta):
        with open(meta) as f:
            host = json.load(f).get("oracle_host")
    v = args.vars / secs
    return {"value": round(v, 1), "unit": "vars/s", "cores": 1, "kind": "port", "solve_s": round(secs, 1),
            "sequential_rounds": int(fx["oracle_rounds"]), "host": host,
            "source": "tests/golden/c2_full_sample.npz (one oracle solve of the full C2 system, seed 1)",
            "gpu_vs_full_size_ratio": round(gpu_value / v, 1)}


def c2_sample_parity(args, div, gen_kw):
    """The CPU-baseline sample (the C2 generator at 1/div scale) solved on the GPU through System::solve()
    and by the oracle: the largest value difference and the variables outside the parity tolerance
    (tests/lmm_cases.py: max(1e-9, 1e-6 |x_oracle|)) — parity at the size the baseline is timed on."""
    import numpy as np

    from oracle import pyoracle as O
    from simgrid_amd import lmm

    nc, nv = args.cnst // div, args.vars // div
    o = O.System(False)
    ov = o.gen_synthetic(nc, nv, args.k, seed=1, **gen_kw)
    o.solve()
    y = o.values_of(ov, nv)
    del o, ov
    p = lmm.System(False)
    pv = p.gen_synthetic(nc, nv, args.k, seed=1, **gen_kw)
    p.solve()
    x = p.values_of(pv)
    del p
    diff = np.abs(x - y)
    tol = np.maximum(1e-9, 1e-6 * np.abs(y))
    return {"sample": f"{nc} x {nv} x {args.k}", "max_abs_diff_vs_oracle": float(diff.max()),
            "max_rel_diff_vs_oracle": float((diff / np.maximum(np.abs(y), 1e-300)).max()),
            "vars_outside_tolerance": int(np.count_nonzero(diff > tol)), "tolerance": "max(1e-9, 1e-6 |x|)"}


C4_PLATFORM = dict(topology=0, topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e8)  # FAT_TREE
C5_PLATFORM = dict(topology=1, topo_parameters="8,4;16,3;8,2;4", loopback_bw=1e9, limiter_bw=2e8)  # DRAGONFLY


STRESS_KW = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50)  # C2 stress variant (generator knobs)
C3_SYSTEMS = 4096


def c3_cpu_slice(lo, hi):
    """Σ solve() seconds and sequential rounds of medium systems lo..hi-1 on the oracle (one core)."""
    from oracle import pyoracle as O

    tcpu, rounds = 0.0, 0
    for i in range(lo, hi):
        o = O.System(False)
        o.gen_maxmin_bench(1, i)
        tcpu += o.timed_solve()
        rounds += o.last_rounds
    return tcpu, rounds


def cpu_worker(workload, lo, hi):
    """Child process of the N-process CPU baseline: prints its slice's Σ solve() seconds."""
    assert workload == "c3"
    tcpu, rounds = c3_cpu_slice(int(lo), int(hi))
    print(json.dumps({"solve_s": tcpu, "rounds": rounds}), flush=True)


def c3_cpu_processes(nproc):
    """the 4096 systems split over `nproc` processes (one per host core), each solving its
    contiguous slice; throughput = Σ variables / the slowest process's Σ solve() time.  Processes are
    children started with subprocess (nothing forks or execs the GPU-initialised parent)."""
    import subprocess

    cuts = [C3_SYSTEMS * k // nproc for k in range(nproc + 1)]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", "c3", str(cuts[k]),
                               str(cuts[k + 1])], stdout=subprocess.PIPE, text=True) for k in range(nproc)]
    t0 = time.perf_counter()
    res = []
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"CPU baseline worker failed (rc {p.returncode})")
        res.append(json.loads(out.strip().splitlines()[-1]))
    wall = time.perf_counter() - t0
    slowest = max(r["solve_s"] for r in res)
    return {"value": round(100 * C3_SYSTEMS / slowest, 1), "unit": "vars/s", "cores": nproc,
            "slowest_process_solve_s": round(slowest, 4), "wall_s_incl_generation": round(wall, 2)}


def config_cpu_baseline(workload, flows, reps=3):
    """The oracle (single-threaded restatement of maxmin.cpp / fair_bottleneck.cpp) on a bounded sample of
    the same workload, rank 0, N=1, `reps` repetitions (mean and sd): C3 solves its 4096 medium systems
    one lmm_solve each (the reference solves independent systems one by one), plus the N-process leg of
    BASELINE.md §2; C4 the same 1e5-flow fat-tree system; C5 the same dragonfly generator at 1e6 flows (1/10
    of the GPU workload)."""
    from oracle import pyoracle as O

    reps = max(1, reps)
    if workload == "c3":
        times = []
        for _ in range(reps):
            tcpu, rounds = c3_cpu_slice(0, C3_SYSTEMS)
            times.append(tcpu)
        m, sd = mean_sd(times)
        hi = host_info()
        nproc = max(1, min(16, hi["affinity_cpus"] or 1))  # the box's CPU share is 16 cores per GPU
        return {"value": round(100 * C3_SYSTEMS / m, 1), "unit": "vars/s", "cores": 1, "kind": "port",
                "sample": f"the same 4096 medium systems, one solve() each timed with steady_clock, {reps} reps:"
                          f" {m:.4f} +- {sd:.4f} s in total, {rounds} sequential rounds",
                "reps": reps, "solve_s_mean": round(m, 5), "solve_s_sd": round(sd, 5),
                "n_process": c3_cpu_processes(nproc), **hi}
    times = []
    for _ in range(reps):  # a fresh system per repetition (solve() runs once per change)
        if workload == "c4":
            n = flows or 100_000
            o = O.System(False)
            o.gen_platform_flows(O.platform_params(model=O.LV08, n_flows=n, seed=1, **C4_PLATFORM))
        else:
            n = min(flows or 10_000_000, 1_000_000)
            o = O.System(False, O.System.FAIR_BOTTLENECK)
            o.gen_platform_flows(O.platform_params(model=O.L07, n_flows=n, seed=1, **C5_PLATFORM))
        times.append(o.timed_solve())
        rounds = o.last_rounds
        del o
    m, sd = mean_sd(times)
    return {"value": round(n / m, 1), "unit": "vars/s", "cores": 1, "kind": "port",
            "sample": f"same generator, {n} flows, solve() timed with steady_clock, {reps} reps: {m:.3f} +- {sd:.3f} s,"
                      f" {rounds} sequential rounds",
            "reps": reps, "solve_s_mean": round(m, 4), "solve_s_sd": round(sd, 4), **host_info()}


def run_config(args):
    """The other SURVEY.md §8(d) configs, each with its multi-GPU scheme (§8(e)):
    c3  4096 independent maxmin_bench "medium" systems (one disjoint-union system per rank, systems
        split over the ranks in nnz-balanced blocks): strong scaling, no data-path collective;
    c4  LV08 flows on a 4096-host fat tree (SMPI-style cluster, crosstraffic on), maxmin: one giant
        component, so replicas (weak scaling);
    c5  L07 flows on a 4096-host dragonfly, FairBottleneck; at N > 1 sharded over the ranks (variables and
        owned constraints, multi.FbShardPlan: per round one all-reduce of counts and two all-gathers,
        bit-identical to the one-context solve), strong scaling.
    One step = one full solve with the inputs resident in HBM."""
    import numpy as np
    import torch

    from simgrid_amd import lmm
    from simgrid_amd import multi as M

    rank, world, local_rank = M.dist_env()
    assert torch.cuda.is_available(), "bench.py needs an MI355X"
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    ex = M.DistExchange() if dist is not None else M.LocalExchange()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    t = time.time()
    shards = None
    batch = None
    if args.workload == "c3":
        # strong scaling: the 4096 seeds split over the ranks; weak (--c3-weak): 4096 per rank, rank r taking
        # seeds 4096 r .. 4096 (r + 1) - 1 of the same generator (SURVEY.md §8(e) reports both)
        n_sys = 4096 * world if args.c3_weak else 4096
        bounds = [r * 4096 for r in range(world + 1)] if args.c3_weak else M.balanced_blocks(np.ones(n_sys), world)
        systems = []
        for i in range(bounds[rank], bounds[rank + 1]):
            systems.append(lmm.System(False))
            systems[-1].gen_maxmin_bench(1, i)
        batch = M.DeviceBatch(systems)  # block-diagonal upload: one workgroup per system, system in LDS
        del systems
        work_vars, scaling = 100 * n_sys, "weak" if args.c3_weak else "strong"
        desc = dict(workload=f"C3: {n_sys} independent maxmin_bench medium systems (100 cnst x 100 vars), "
                             "one block-diagonal batch per rank (lmmhip_set_batch: one workgroup per system, "
                             "the system in LDS)", systems=n_sys,
                    parallelism=f"systems in nnz-balanced blocks x{world}")
    elif args.workload == "c4":
        flows = args.flows or 100_000
        s = lmm.System(False)
        s.gen_platform_flows(lmm.platform_params(model=lmm.LV08, n_flows=flows, seed=rank + 1, **C4_PLATFORM),
                             want_vars=False)
        work_vars, scaling = flows * world, "weak"
        desc = dict(workload=f"C4: {flows} LV08 flows on fat tree {C4_PLATFORM['topo_parameters']} (4096 hosts)",
                    flows=flows, parallelism=f"replicas x{world} (one component per system)")
    else:
        flows = args.flows or 10_000_000
        s = lmm.System(False, lmm.System.FAIR_BOTTLENECK)
        s.gen_platform_flows(lmm.platform_params(model=lmm.L07, n_flows=flows, seed=1, **C5_PLATFORM),
                             want_vars=False)
        work_vars, scaling = flows, "strong"
        desc = dict(workload=f"C5: {flows} L07 flows on dragonfly {C5_PLATFORM['topo_parameters']} (4096 hosts), "
                             "FairBottleneck", flows=flows)
        if world > 1:  # variables and owned constraints sharded over the ranks (multi.FbShardPlan)
            f = M.export_flat(s)
            del s
            plan = M.FbShardPlan(f, world)
            gather = M.FbGather(plan)
            shards = [M.DeviceFbShard(plan, rank, gather)]
            sub_n = (shards[0].n, len(f.cbound), int(np.diff(f.var_ptr)[plan.vb[rank]:plan.vb[rank + 1]].sum()))
            del f, plan
            desc["parallelism"] = (f"variables + owned constraints sharded x{world}: per round 1 all-reduce"
                                   " (counts) + 2 all-gathers (mu, remaining)")
        else:  # one GPU: the drop-in FairBottleneck::solve path (element order of the reference, bit-identical)
            desc["parallelism"] = "one context (System::solve, fbk_update_seq)"
    if batch is not None:
        nV, nC, nnz = batch.n_var, batch.n_cnst, batch.nnz
    elif shards is None:
        s.prepare()
        st = s.last_stats()
        nV, nC, nnz = st["n_var"], st["n_cnst"], st["nnz"]
    else:
        nV, nC, nnz = sub_n
    log(f"[rank {rank}] {args.workload}: built in {time.time() - t:.1f}s: nV={nV} nC={nC} nnz={nnz}")

    def step():
        if batch is not None:
            batch.solve()
            return batch.stats()["rounds"]
        if shards is None:
            s.device_solve()
            return s.last_stats()["rounds"]
        for sh in shards:
            sh.begin()
        return M.fb_solve_sharded(shards, ex, gather)

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rounds = step()
    barrier()
    elapsed = time.perf_counter() - t0
    tot = np.array([nV, nnz, nC], dtype=np.float64)  # summed over ranks below
    if args.workload == "c5":  # the reference's per-round sweeps, counted on the device over the last solve
        w = shards[0].fb_work() if shards is not None else s.fb_work()
        # elements and variables are split over the ranks; every rank lists every constraint: count rank 0's
        work = np.array([w[0], w[1], w[2] if rank == 0 else 0], dtype=np.float64)
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tot = ex.sum(tot)
        if args.workload == "c5":
            work = ex.sum(work)
    ms_per_step = 1000.0 * elapsed / args.steps
    # algorithmic bytes of one solve: maxmin 56 B/element + 24 B/variable + 32 B/constraint;
    # fair bottleneck sum over the rounds of 36 B/element + 32 B/variable + 32 B/constraint of the listed ones
    if args.workload == "c5":
        alg = 36 * work[0] + 32 * work[1] + 32 * work[2]
        note = ("SURVEY.md §8(d) bottleneck_solve: sum over rounds of 36 nnz_r + 32 V_r + 32 C_r bytes, nnz_r / V_r /"
                " C_r = elements of the listed constraints / listed variables / listed constraints (lmmhip_fb_work)")
        desc["fb_work"] = dict(elements=int(work[0]), variables=int(work[1]), constraints=int(work[2]))
    else:
        alg = 56 * tot[1] + 24 * tot[0] + 32 * tot[2]
        note = "SURVEY.md §8(d) lmm_solve: 56 nnz + 24 V + 32 C bytes per solve"
    if args.profile_json and rank == 0 and shards is None and batch is None:  # per-launch HIP events of one extra solve
        s.set_profiling(True)
        s.device_solve()
        s.set_profiling(False)
        slot, rnd, ms = s.launch_profile()
        per_kernel = {SLOT_NAMES[int(k)]: dict(launches=int((slot == k).sum()), total_ms=float(ms[slot == k].sum()),
                                               avg_us=float(1000 * ms[slot == k].mean()))
                      for k in sorted(set(slot.tolist()))}
        with open(args.profile_json, "w") as f:
            json.dump(dict(per_kernel=per_kernel, rounds=s.last_stats()["rounds"],
                           device_ms=s.last_stats()["device_ms"], launch_slot=slot.tolist(),
                           launch_round=rnd.tolist(), launch_ms=ms.tolist()), f)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = config_cpu_baseline(args.workload, args.flows, args.cpu_reps)
    roof = roofline_obj(alg, ms_per_step, args.workload, note, gpus=world)
    if world == 1 and args.workload in ("c4", "c5"):  # the request-rate roofline of the solve (VERDICT r05 Next #5)
        rq = request_roofline(args.workload, ms_per_step)
        if rq:
            roof["requests"] = rq
    if rank == 0:
        desc.update(active_vars=int(tot[0]), nnz=int(tot[1]), device_rounds=int(rounds))
        print(json.dumps({
            "metric": "LMM solve throughput (vars/s)", "value": round(work_vars * args.steps / elapsed, 1),
            "unit": "vars/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (generators of simgrid_amd/csrc/lmm_generators.hpp / lmm_platforms.hpp)",
            "config": desc,
            "roofline": roof, "cpu_baseline": cpu}), flush=True)
    if shards is not None:
        for sh in shards:
            sh.close()
    if batch is not None:
        batch.close()
    s = None  # free the device context while the HIP runtime is up (not in interpreter teardown)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
