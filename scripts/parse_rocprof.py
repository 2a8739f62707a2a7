#!/usr/bin/env python
"""Summarise scripts/profile.sh output (gpurun_out/rp_*) into profiles/<tag>_*.

  profiles/<tag>_kernel_stats[_<w>].csv  rocprofv3 --kernel-trace --stats summaries (per-kernel average duration)
  profiles/<tag>_traffic_<w>.json        per workload (c2 c3 c4 c5): FETCH_SIZE / WRITE_SIZE of every kernel, and
                                         the counter bytes of ONE SOLVE (the solve's kernels summed, divided by the
                                         number of solves in the run) — bench.py's roofline.traffic
  profiles/<tag>_calibration.json        the counters on known byte counts (scripts/ubench_gather.hip)

gfx950 counter notes (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read — confirmed by the calibration pass (320 MB int32 stream -> 160 MB) — while random
1-8 B gathers report about one 64-B request per L2 miss; WRITE_SIZE is exact for streaming stores.  The
traffic bench.py reports is the guide's correction, 2 x FETCH + WRITE; the raw FETCH + WRITE is kept beside
it (the truth lies between the two for kernels that mix streams and gathers).
usage: python scripts/parse_rocprof.py <tag>
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
# one launch per solve of each workload's engine: the number of solves in a counter run
SOLVE_MARK = {"c2": "mm_init_vars", "c2_stress": "mm_init_vars", "c3": "mm_batch_lds", "c4": "fr_init_vars",
              "c5": "fb_init"}
# kernels of the upload / device flatten (before the timed region), not of a solve
NOT_SOLVE = ("rs_", "rocprim", "__amd_rocclr_copyBuffer", "mm_elem_usage", "mm_dup_check", "mm_batch_check",
             "fr_c2s")


def load(path):
    d = collections.defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"]][0] += float(r["Counter_Value"]) * 1024.0  # KB -> B
            d[r["Kernel_Name"]][1] += 1
    return d


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("lmmdev::", "")
    return n.split("<")[0]


def solve_kernel(k):
    return not k.startswith(NOT_SOLVE)


def workload_traffic(w):
    fp = os.path.join(OUT, f"rp_FETCH_SIZE_{w}", "run_counter_collection.csv")
    wp = os.path.join(OUT, f"rp_WRITE_SIZE_{w}", "run_counter_collection.csv")
    if not (os.path.exists(fp) and os.path.exists(wp)):
        return None
    fetch, write = load(fp), load(wp)
    kernels = {}
    for name in set(fetch) | set(write):
        k = short(name)
        e = kernels.setdefault(k, dict(fetch_bytes=0.0, write_bytes=0.0, launches=0))
        e["fetch_bytes"] += fetch.get(name, [0.0, 0])[0]
        e["write_bytes"] += write.get(name, [0.0, 0])[0]
        e["launches"] += max(fetch.get(name, [0, 0])[1], write.get(name, [0, 0])[1])
    solves = kernels.get(SOLVE_MARK[w], {}).get("launches", 0)
    if solves == 0:
        raise SystemExit(f"{w}: no {SOLVE_MARK[w]} launch in the counter run")
    for e in kernels.values():
        n = max(e["launches"], 1)
        e["fetch_bytes_per_launch"] = e["fetch_bytes"] / n
        e["write_bytes_per_launch"] = e["write_bytes"] / n
    f_s = sum(e["fetch_bytes"] for k, e in kernels.items() if solve_kernel(k)) / solves
    w_s = sum(e["write_bytes"] for k, e in kernels.items() if solve_kernel(k)) / solves
    return dict(workload=w, solves=solves, solve_marker=SOLVE_MARK[w],
                solve_kernels=sorted(k for k in kernels if solve_kernel(k)),
                solve_fetch_bytes=int(f_s), solve_write_bytes=int(w_s),
                solve_counter_bytes_raw=int(f_s + w_s), solve_counter_bytes_fetch_x2=int(2 * f_s + w_s),
                kernels=kernels)


REQ_CTRS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_ATOMIC_sum")


def load_count(path):
    """Per kernel (full name): [summed counter value, dispatches] of a one-counter rocprofv3 pass (a count, no
    unit scaling)."""
    d = collections.defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"]][0] += float(r["Counter_Value"])
            d[r["Kernel_Name"]][1] += 1
    return d


def trace_avg_ns(path, key=None):
    """kernel name (short(), or `key`) -> (average duration ns, calls) from a --kernel-trace --stats summary;
    instances that map to one name are merged, weighted by their calls."""
    key = key or short
    acc = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = key(r["Name"])
            ns, n = acc.get(k, (0.0, 0))
            acc[k] = (ns + float(r["TotalDurationNs"]), n + int(r["Calls"]))
    return {k: (ns / max(n, 1), n) for k, (ns, n) in acc.items()}


def cal_key(name):
    """Calibration kernels keep their template argument (gather<double> vs gather<float>)."""
    n = name.split("(")[0].replace("void ", "").strip()
    return n


def workload_requests(w, tag):
    """Memory-side requests (L2 -> fabric: TCC_EA0_RDREQ / WRREQ, and the atomic part of WRREQ) per kernel launch
    and per solve of workload w, with the kernels' average durations from the same tag's kernel trace."""
    paths = {c: os.path.join(OUT, f"rp_{c}_{w}", "run_counter_collection.csv") for c in REQ_CTRS}
    if not all(os.path.exists(p) for p in paths.values()):
        return None
    ctr = {c: load_count(p) for c, p in paths.items()}
    kernels = {}
    for c, d in ctr.items():
        for name, (v, n) in d.items():
            e = kernels.setdefault(short(name), {"launches": 0})
            e[c] = e.get(c, 0.0) + v
            e["launches"] = max(e["launches"], n)
    solves = kernels.get(SOLVE_MARK[w], {}).get("launches", 0)
    if solves == 0:
        raise SystemExit(f"{w}: no {SOLVE_MARK[w]} launch in the request-counter run")
    tr = os.path.join(ROOT, "profiles", f"{tag}_kernel_stats{'' if w == 'c2' else '_' + w}.csv")
    dur = trace_avg_ns(tr) if os.path.exists(tr) else {}
    tot = {c: 0.0 for c in REQ_CTRS}
    for k, e in kernels.items():
        n = max(e["launches"], 1)
        for c in REQ_CTRS:
            e[c + "_per_launch"] = e.get(c, 0.0) / n
            if solve_kernel(k):
                tot[c] += e.get(c, 0.0) / solves
        if k in dur:
            e["avg_ns"] = dur[k][0]
            req = e.get("TCC_EA0_RDREQ_sum", 0.0) / n + e.get("TCC_EA0_WRREQ_sum", 0.0) / n
            e["requests_per_s"] = req / (dur[k][0] * 1e-9) if dur[k][0] > 0 else None
    return dict(workload=w, solves=solves, solve_marker=SOLVE_MARK[w], kernel_trace=os.path.relpath(tr, ROOT),
                solve_rdreq=tot["TCC_EA0_RDREQ_sum"], solve_wrreq=tot["TCC_EA0_WRREQ_sum"],
                solve_atomic=tot["TCC_EA0_ATOMIC_sum"],
                solve_requests=tot["TCC_EA0_RDREQ_sum"] + tot["TCC_EA0_WRREQ_sum"], kernels=kernels)


def calibration_requests():
    """Request ceilings of the calibration kernels (scripts/ubench_gather.hip): requests per second of each kernel
    (counter pass / its average duration in the kernel trace of the same program)."""
    paths = {c: os.path.join(OUT, f"rp_cal_{c}", "run_counter_collection.csv") for c in REQ_CTRS}
    tr = os.path.join(OUT, "rp_trace_cal", "run_kernel_stats.csv")
    if not all(os.path.exists(p) for p in paths.values()) or not os.path.exists(tr):
        return None
    dur = trace_avg_ns(tr, cal_key)
    out = {}
    for c, p in paths.items():
        for name, (v, n) in load_count(p).items():
            e = out.setdefault(cal_key(name), {"dispatches": n})
            e[c + "_per_dispatch"] = v / max(n, 1)
    for k, e in out.items():
        d = dur.get(k)
        if d:
            e["avg_ns"] = d[0]
            e["requests_per_s"] = (e.get("TCC_EA0_RDREQ_sum_per_dispatch", 0) + e.get("TCC_EA0_WRREQ_sum_per_dispatch", 0)) \
                / (d[0] * 1e-9)
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "latest"
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for sub, suffix in (("rp_trace", ""), ("rp_trace_c3", "_c3"), ("rp_trace_c4", "_c4"), ("rp_trace_c5", "_c5")):
        p = os.path.join(OUT, sub, "run_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_kernel_stats{suffix}.csv"))
    for w in SOLVE_MARK:
        t = workload_traffic(w)
        if t is None:
            continue
        with open(os.path.join(prof, f"{tag}_traffic_{w}.json"), "w") as f:
            json.dump(t, f, indent=1)
        print(f"{w}: {t['solves']} solves, counter bytes per solve {t['solve_counter_bytes_raw'] / 1e9:.3f} GB raw,"
              f" {t['solve_counter_bytes_fetch_x2'] / 1e9:.3f} GB with FETCH x2")
        for k, e in sorted(t["kernels"].items(), key=lambda kv: -(kv[1]["fetch_bytes"] + kv[1]["write_bytes"]))[:8]:
            print(f"   {k:24s} launches {e['launches']:5d}  fetch/launch {e['fetch_bytes_per_launch'] / 1e6:9.2f} MB"
                  f"  write/launch {e['write_bytes_per_launch'] / 1e6:9.2f} MB")
    for w in ("c2", "c4", "c5"):
        t = workload_requests(w, tag)
        if t is None:
            continue
        cal = calibration_requests()
        t["calibration"] = cal
        with open(os.path.join(prof, f"{tag}_requests_{w}.json"), "w") as f:
            json.dump(t, f, indent=1)
        print(f"{w}: requests per solve {t['solve_requests']:.4g} (rd {t['solve_rdreq']:.4g}, wr {t['solve_wrreq']:.4g}, "
              f"atomic {t['solve_atomic']:.4g})")
    cf = os.path.join(OUT, "rp_cal_FETCH_SIZE", "run_counter_collection.csv")
    cw = os.path.join(OUT, "rp_cal_WRITE_SIZE", "run_counter_collection.csv")
    if os.path.exists(cf) and os.path.exists(cw):
        cal_f, cal_w = load(cf), load(cw)
        cal = {short(n): dict(fetch_bytes=v[0] / v[1], write_bytes=cal_w.get(n, [0, 1])[0] / max(cal_w.get(n, [0, 1])[1], 1))
               for n, v in cal_f.items()}
        with open(os.path.join(prof, f"{tag}_calibration.json"), "w") as f:
            json.dump(dict(calibration=cal, note="stream_idx reads 320e6 B (int32 x 8e7); gather<T> gathers 8e7 "
                                                 "elements at random from 1e6 / 4e6 / 1e7-entry tables; atomics/"
                                                 "scatter touch 8e7 random elements"), f, indent=1)


if __name__ == "__main__":
    main()
