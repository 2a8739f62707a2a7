"""Collect the round-6 same-box A/B bench lines (gpurun_out/ab*_*.out, one bench.py JSON line each) into
profiles/r06_ab.json: per GPU pass (B, C, D, E: one box each) the variant's ms per solve and the launch-average of
its dominant kernel, with what each variant was (scripts/gpu_r06_[b-e].sh)."""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {
    "ab_": ("B", "scripts/gpu_r06_b.sh", {
        "base": "round-6 pruned build before the levers", "rdq": "+ wave-level vote ready queue",
        "pipe": "+ saturation tasks pipelined (LMM_SATQ_PIPE)", "new": "+ per-XCD update candidate lists",
        "sb6": "saturation grid 6 workgroups per CU", "vbr": "vote bitmap off in the tail (LMMHIP_VOTE_BITS_ROWS)"}),
    "abc_": ("C", "scripts/gpu_r06_c.sh", {
        "base": "round-5 code (abl/base)", "pipe": "+ pipelined saturation + wave-level vote queue",
        "new": "+ workgroup-level vote queue (RdqLds) = product"}),
    "abd_": ("D", "scripts/gpu_r06_d.sh", {
        "b0": "mm_saturate_q (product)", "b2": "batched saturation M = 2", "b4": "batched saturation M = 4",
        "w64": "frontier saturation 64-element chunks (product)", "w32": "32-element chunks", "w16": "16-element chunks"}),
    "abe_": ("E", "scripts/gpu_r06_e.sh", {
        "q": "mm_saturate_q (product)", "b64": "batched saturation M = 4", "b32": "batched, 32-element chunks"}),
    "abg_": ("G", "scripts/gpu_r06_g.sh", {
        "prev": "build before the two levers (abl/prev)", "new": "tied ratios loaded together + deferred frontier pushes",
        "nodf": "tied ratios loaded together, LMMHIP_FR_DEFER=0"}),
    "abh_": ("H", "scripts/gpu_r06_h.sh", {
        "prev": "before the tie loads (abl/prev)", "tie": "tie loads, no deferral (abl/tie, LMMHIP_FR_DEFER=0)",
        "nous": "+ one-level ready test with LDS-stashed state + floor read before the slot store, LMMHIP_FR_UPDSPEC=0",
        "new": "+ fr_update state loads with the keys (LMMHIP_FR_UPDSPEC=1, the default)"}),
    "abi_": ("I", "scripts/gpu_r06_i.sh", {
        "ag0": "LMMHIP_FR_AGG=0 (pushes straight to the constraint records)",
        "ag1": "pushes aggregated per constraint in LDS (default)",
        "tie": "FairBottleneck before the load reorder (abl/tie)", "new": "FB chain / increment loads before stores"}),
    "abj_": ("J", "scripts/gpu_r06_j.sh", {
        "u8": "frontier saturation 8 claimed-row elements per lane per pass (LMMHIP_FR_SATU16=0)",
        "u16": "16 per lane per pass on the small systems (default)"}),
    "abl_": ("L", "scripts/gpu_r06_l.sh", {
        "h": "final build before the speculative queue-entry load (abl/h)",
        "new": "fr_vote's first queue entry loaded with the count"}),
    "abm_": ("M", "scripts/gpu_r06_m.sh", {
        "base": "product build", "wt": "round kernels' state stores written through (LMM_WT=1, abl/wt)"}),
    "abn_": ("N", "scripts/gpu_r06_n.sh", {
        "n0": "build before (abl/n0)", "new0": "no single-address atomic drains (init count, FB counters, LASTR)",
        "new": "+ the vote's ready segments (LMMHIP_VOTE_SEG=1, default)"}),
}


def main(out=os.path.join(ROOT, "profiles", "r06_ab.json")):
    res = {}
    for pre, (name, script, what) in PASSES.items():
        rows = {}
        for p in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", pre + "*.out"))):
            m = re.match(re.escape(pre) + r"(c2s|c2|c3|c4|c5)_([a-z0-9]+?)(?:_(\d))?\.out$", os.path.basename(p))
            if not m:
                continue
            try:
                d = json.loads(open(p).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                continue
            wl, var = m.group(1), m.group(2)
            dk = d.get("roofline", {}).get("dominant_kernel") or {}
            rows.setdefault(wl, {}).setdefault(var, {"what": what.get(var, var), "ms_per_step": []})
            rows[wl][var]["ms_per_step"].append(d["ms_per_step"])
            if dk:
                rows[wl][var].setdefault("dominant_kernel_avg_us", []).append(dk.get("avg_us"))
        if rows:
            res[name] = {"script": script, "workloads": rows}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: {w: {v: x["ms_per_step"] for v, x in r.items()} for w, r in p["workloads"].items()}
                      for k, p in res.items()}))


if __name__ == "__main__":
    main(*sys.argv[1:])
