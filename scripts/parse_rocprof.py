#!/usr/bin/env python
"""Summarise scripts/profile.sh output (gpurun_out/rp_*) into profiles/<tag>_*.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (per-kernel average duration)
  profiles/<tag>_traffic.json       per-kernel FETCH_SIZE / WRITE_SIZE per launch (bytes), the
                                    calibration pass on known byte counts, and the HBM bytes per launch
                                    bench.py reports as roofline.traffic

gfx950 counter notes (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read — confirmed by the calibration pass (320 MB int32 stream -> 160 MB) — while
random 1-8 B gathers report about one 64-B request per L2 miss.  The round kernels mix both, so the
traffic reported is FETCH + WRITE as counted (no correction), with the calibration kept alongside.
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


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "latest"
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(OUT, "rp_trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = load(os.path.join(OUT, "rp_FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(OUT, "rp_WRITE_SIZE", "run_counter_collection.csv"))
    cal_f = load(os.path.join(OUT, "rp_cal_FETCH_SIZE", "run_counter_collection.csv"))
    cal_w = load(os.path.join(OUT, "rp_cal_WRITE_SIZE", "run_counter_collection.csv"))
    kernels = {}
    for name in set(fetch) | set(write):
        f, nf = fetch.get(name, [0.0, 1])
        w, nw = write.get(name, [0.0, 1])
        k = short(name)
        e = kernels.setdefault(k, dict(fetch_bytes_per_launch=0.0, write_bytes_per_launch=0.0, launches=0))
        e["fetch_bytes_per_launch"] += f / max(nf, 1)
        e["write_bytes_per_launch"] += w / max(nw, 1)
        e["launches"] = max(nf, nw)
    for e in kernels.values():
        e["hbm_bytes_per_launch"] = int(e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"])
    cal = {short(n): dict(fetch_bytes=v[0] / v[1], write_bytes=cal_w.get(n, [0, 1])[0] / max(cal_w.get(n, [0, 1])[1], 1))
           for n, v in cal_f.items()}
    # counter bytes against the algorithmic bytes of bench.py's per-kernel model (gpurun_out/prof_c2.json, the
    # per-launch profile of the same workload): raw FETCH + WRITE, and with FETCH doubled (the gfx950 correction
    # for wide streaming reads, MI355X_MICROARCH.md HBM; random gathers are counted per 64-B request, so the
    # truth lies between the two for kernels that mix both)
    ratios = {}
    pj = os.path.join(OUT, "prof_c2.json")
    if os.path.exists(pj):
        with open(pj) as f:
            pk = json.load(f)["per_kernel"]
        for bench_name, rp_name in (("mm_vote", "mm_vote_lane"), ("mm_ready", "mm_ready"),
                                    ("mm_saturate", "mm_saturate"), ("mm_update", "mm_update"),
                                    ("mm_init_cnsts", "mm_init_cnsts")):
            if bench_name not in pk or rp_name not in kernels:
                continue
            alg = pk[bench_name]["alg_bytes"] / max(pk[bench_name]["launches"], 1)
            e = kernels[rp_name]
            raw = e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"]
            cor = 2 * e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"]
            ratios[rp_name] = dict(alg_bytes_per_launch=int(alg), counter_bytes_per_launch=int(raw),
                                   counter_bytes_fetch_x2=int(cor), ratio_raw=round(raw / alg, 2) if alg else None,
                                   ratio_fetch_x2=round(cor / alg, 2) if alg else None,
                                   avg_us=round(pk[bench_name]["avg_us"], 2))
    out = dict(kernels=kernels, counter_vs_algorithmic=ratios, calibration=cal,
               calibration_note="stream_idx reads 320e6 B (int32 x 8e7); gather<T> gathers 8e7 elements "
                                "at random from 1e6 / 4e6 / 1e7-entry tables; atomics/scatter touch 8e7 random elements")
    with open(os.path.join(prof, f"{tag}_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        print(f"{k:24s} launches {e['launches']:5d}  fetch/launch {e['fetch_bytes_per_launch']/1e6:9.2f} MB"
              f"  write/launch {e['write_bytes_per_launch']/1e6:9.2f} MB")
    for k, r in ratios.items():
        print(f"{k:24s} alg {r['alg_bytes_per_launch']/1e6:8.2f} MB  counters {r['ratio_raw']}x (fetch x2: "
              f"{r['ratio_fetch_x2']}x)  {r['avg_us']} us")


if __name__ == "__main__":
    main()
