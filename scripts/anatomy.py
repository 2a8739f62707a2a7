#!/usr/bin/env python3
"""Round anatomy of the max-min round engine (VERDICT r05 Next #1b): where one round's time goes, level by level.

Runs one C2 solve (or --cnst/--vars for a smaller system) on the DIAGNOSTIC build of the solver
(`make -C simgrid_amd/csrc OUT=../_anat EXTRA_HIPFLAGS=-DLMM_ANAT=1`, loaded through LMM_AMD_LIB), in which every wave
of the vote, saturation and update launches of the chosen rounds writes its entry / exit on the chip's 100-MHz wall
clock and the ticks it spent waiting at each dependent level of its work (lmm_dev.hpp "round anatomy").  The stamps
serialise what the product kernels overlap, so the stamped round is longer than the real one: the JSON reports the
stamped anatomy as SHARES and, beside it, the product build's own per-launch HIP-event times of the same rounds
(--product-profile: a `bench.py --profile-json` file of the product build on the same system).

Accounting (100 % by construction): a round runs from its vote's first wave entry to the next round's vote's first
wave entry.  Each launch's span = [dispatch / fill: the entry of the wave that exits last, minus the launch's first
entry] + [that critical wave's own segments, stamped] ; between launches = the boundary gap (last exit -> next
first entry).  The critical wave's segments are its dependent levels; what the stamps do not name is "other".

usage: LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --rounds 70,71,200,201 --out f.json
"""
import argparse
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS, KERN, WAVES, FIELDS = 4, 4, 8192, 20
TICK_US = 0.01  # s_memrealtime: 100 MHz

VOTE_LEVELS = ["row record (rtgt, crec)", "variable state (vstate, bound)", "row elements (ccol)",
               "keys of the row's constraints", "exact ratios (key ties / bounded)", "vote move (nvote atomics)"]
SAT_LEVELS = ["candidate id (update segment / vote queue)", "CSC elements (csc_v, csc_p, csc_row)",
              "variable states + claims + x stores", "claimed rows' elements (csr_c, csr_w)",
              "their constraints' words (cexp)", "decrement pushes (atomics) issued", "candidate state (key, nvote, "
              "ratio, CSC range)"]
UPD_LEVELS = ["keys + touch flags", "touched constraints' records", "arithmetic + stores + bitmap ballot"]
# frontier engine (C4): fr_vote / fr_sat / fr_sat_big / fr_update records (lmm_frontier_kernels.hpp)
FRV_LEVELS = ["queue entry (fq_a, fq_b)", "row (csr_cs) + bound / penalty", "keys + registered floors",
              "rest of the row + exact ratios", "vote stores + atomics issued"]
FRS_LEVELS = ["ready test + workgroup collection (LDS)", "(unused)", "CSC elements + variable states",
              "claimed rows' elements (csr_c, csr_w)", "their constraints' words (cexp)", "decrement pushes issued",
              "claims + values stored"]
FRU_LEVELS = ["keys + touch flags", "touched records + floors", "arithmetic + scan prefix + barrier",
              "slots (vslot)", "queued voters (csc_v, csc_row)", "stores + barriers"]


def frontier_view(rec, kind):
    """A frontier kernel's waves: span, entry / exit spread, the critical wave's levels (kind: fr_vote / fr_sat /
    fr_satb / fr_upd)."""
    live = rec[rec[:, 0] > 0]
    if len(live) == 0:
        return None
    t_in, t_out = live[:, 0].astype(np.int64), live[:, 1].astype(np.int64)
    first, last = int(t_in.min()), int(t_out.max())
    crit = live[int(np.argmax(t_out))]
    c_in, c_out = int(crit[0]), int(crit[1])
    v = {"waves": int(len(live)), "first_entry": first, "last_exit": last, "span_us": us(last - first),
         "entry_spread_us": {"p50": us(np.median(t_in) - first), "max": us(t_in.max() - first)},
         "wave_time_us": {"p50": us(np.median(t_out - t_in)), "max": us((t_out - t_in).max())}}
    seg = {"dispatch/fill (critical wave's entry - first entry)": us(c_in - first)}
    if kind == "fr_vote":
        names, cols = ["queue counts (fq_n, segment offsets)"] + FRV_LEVELS, list(range(3, 9))
        v["counts"] = {"queued_rows": int(live[::4, 10].sum()), "max_revotes_per_lane": int(live[:, 9].max())}
    elif kind in ("fr_sat", "fr_satb"):
        names, cols = FRS_LEVELS, list(range(3, 10))
        v["counts"] = {"chunks": int(live[:, 11].sum()), "fixed_vars": int(live[:, 12].sum()),
                       "pushes": int(live[:, 13].sum()), "critical_wave_chunks": int(crit[11])}
        if kind == "fr_satb":
            v["counts"]["big_constraints"] = int(live[0, 10])
    else:
        names, cols = FRU_LEVELS, list(range(3, 9))
        v["counts"] = {"scanned_slots": int(live[:, 9].sum())}
    named = 0
    for n, c in zip(names, cols):
        if n != "(unused)":
            seg[n] = us(crit[c])
            named += int(crit[c])
    seg["other"] = us(c_out - c_in - named)
    v["critical_wave"] = {"workgroup": int(crit[2]), "time_us": us(c_out - c_in), "segments_us": seg}
    v["wave_us_summed_over_waves"] = {n: us(live[:, c].sum()) for n, c in zip(names, cols) if n != "(unused)"}
    return v


def frontier_round_view(recs, rounds, k):
    r = rounds[k]
    order = [("fr_vote", 0), ("fr_sat", 1), ("fr_satb", 3), ("fr_upd", 2)]
    kv = {name: frontier_view(recs[k, i], name) for name, i in order}
    if kv["fr_vote"] is None or kv["fr_sat"] is None or kv["fr_upd"] is None:
        return None
    seq = [n for n, _ in order if kv[n] is not None]
    out = {"round": r, "kernels": kv}
    gaps = {}
    for a, b in zip(seq, seq[1:]):
        gaps[f"{a} -> {b}"] = us(kv[b]["first_entry"] - kv[a]["last_exit"])
    nxt = [j for j in range(SLOTS) if rounds[j] == r + 1]
    end = kv["fr_upd"]["last_exit"]
    if nxt and recs[nxt[0], 0][:, 0].max() > 0:
        nv = recs[nxt[0], 0]
        nfirst = int(nv[nv[:, 0] > 0][:, 0].min())
        gaps["fr_update -> next fr_vote"] = us(nfirst - end)
        end = nfirst
    span = end - kv["fr_vote"]["first_entry"]
    acc = {}
    for n in seq:
        for sg, x in kv[n]["critical_wave"]["segments_us"].items():
            acc[f"{n}: {sg}"] = x
    for g, x in gaps.items():
        acc[f"boundary {g}"] = x
    out["round_span_us_stamped"] = us(span)
    out["boundary_gaps_us"] = gaps
    out["accounting_us"] = acc
    out["accounted_share"] = round(sum(acc.values()) / max(1e-9, us(span)), 4)
    out["other_share"] = round(sum(x for sg, x in acc.items() if "other" in sg) / max(1e-9, us(span)), 4)
    out["shares"] = {sg: round(x / max(1e-9, us(span)), 4) for sg, x in acc.items()}
    return out


def load_records(s, L):
    n = ct.c_int64()
    r4 = (ct.c_int32 * 4)()
    L._check_hip(L.lib().lmmhip_anatomy(s.device_ctx(), None, 0, ct.byref(n), r4))
    buf = np.zeros(n.value, dtype=np.uint64)
    L._check_hip(L.lib().lmmhip_anatomy(s.device_ctx(), buf.ctypes.data_as(ct.POINTER(ct.c_uint64)), n.value,
                                        ct.byref(n), r4))
    return buf.reshape(SLOTS, KERN, WAVES, FIELDS), list(r4)


def us(t):
    return round(float(t) * TICK_US, 3)


def kernel_view(rec, kind):
    live = rec[rec[:, 0] > 0]
    if len(live) == 0:
        return None
    t_in, t_out = live[:, 0].astype(np.int64), live[:, 1].astype(np.int64)
    first, last = int(t_in.min()), int(t_out.max())
    crit = live[int(np.argmax(t_out))]
    v = {"waves": int(len(live)), "first_entry": first, "last_exit": last, "span_us": us(last - first),
         "entry_spread_us": {"p50": us(np.median(t_in) - first), "p90": us(np.percentile(t_in, 90) - first),
                             "max": us(t_in.max() - first)},
         "wave_time_us": {"p50": us(np.median(t_out - t_in)), "p90": us(np.percentile(t_out - t_in, 90)),
                          "max": us((t_out - t_in).max())},
         "exit_spread_us": {"p50": us(np.median(t_out) - first), "p90": us(np.percentile(t_out, 90) - first)}}
    c_in, c_out = int(crit[0]), int(crit[1])
    seg = {"dispatch/fill (critical wave's entry - first entry)": us(c_in - first)}
    if kind == "vote":
        seg["LDS bitmap copy + barrier"] = us(int(crit[3]) - c_in)
        seg["filter: row target / floor stream"] = us(crit[5])
        seg["filter: bitmap test + target key gathers"] = us(crit[6])
        lv = [us(x) for x in crit[9:15]]
        for name, x in zip(VOTE_LEVELS, lv):
            seg[f"re-vote: {name}"] = x
        named = int(crit[3]) - c_in + int(crit[5]) + int(crit[6]) + int(sum(crit[9:15]))
        seg["other (queueing, batch tails, record)"] = us(c_out - c_in - named)
        v["counts_critical_wave"] = {"filter_steps": int(crit[4]), "revote_batches": int(crit[7]),
                                     "rows_requeued": int(crit[15]), "rows": int(crit[16])}
        v["counts_all_waves"] = {"rows": int(live[:, 16].sum()), "revoted_rows": int(live[:, 15].sum()),
                                 "filter_steps": int(live[:, 4].sum()), "revote_batches": int(live[:, 7].sum())}
        tot = {"LDS bitmap copy + barrier": us(np.sum(live[:, 3].astype(np.int64) - t_in)),
               "filter: row target / floor stream": us(live[:, 5].sum()),
               "filter: bitmap test + target key gathers": us(live[:, 6].sum()),
               "re-vote batches (wave time)": us(live[:, 8].sum())}
        for i, name in enumerate(VOTE_LEVELS):
            tot[f"re-vote: {name} (slowest lane)"] = us(live[:, 9 + i].sum())
        v["wave_us_summed_over_waves"] = tot
    elif kind == "sat":
        seg["segment-count prefix (ucnt load + scan)"] = us(int(crit[3]) - c_in)
        for i, name in enumerate(SAT_LEVELS):
            seg[name] = us(crit[4 + i])
        named = int(crit[3]) - c_in + int(sum(crit[4:11]))
        seg["other (scan, batch loop, record)"] = us(c_out - c_in - named)
        v["counts_critical_wave"] = {"candidates": int(crit[11]), "chunks": int(crit[12]), "fixed_vars": int(crit[13]),
                                     "pushes": int(crit[14])}
        v["counts_all_waves"] = {"candidates": int(live[:, 11].sum()), "chunks": int(live[:, 12].sum()),
                                 "fixed_vars": int(live[:, 13].sum()), "pushes": int(live[:, 14].sum()),
                                 "waves_with_chunks": int((live[:, 12] > 0).sum())}
        v["wave_us_summed_over_waves"] = {name: us(live[:, 4 + i].sum()) for i, name in enumerate(SAT_LEVELS)}
        v["wave_us_summed_over_waves"]["segment-count prefix"] = us(np.sum(live[:, 3].astype(np.int64) - t_in))
    else:
        for i, name in enumerate(UPD_LEVELS):
            seg[name] = us(crit[4 + i])
        seg["workgroup tail (alive count, candidate segment write)"] = us(c_out - int(crit[3]))
        named = int(sum(crit[4:7])) + c_out - int(crit[3])
        seg["other"] = us(c_out - c_in - named)
        v["counts_critical_wave"] = {"steps": int(crit[7]), "touched": int(crit[8])}
        v["counts_all_waves"] = {"steps": int(live[:, 7].sum()), "touched": int(live[:, 8].sum())}
        v["wave_us_summed_over_waves"] = {name: us(live[:, 4 + i].sum()) for i, name in enumerate(UPD_LEVELS)}
    v["critical_wave"] = {"workgroup": int(crit[2]), "entry_us": us(c_in - first), "time_us": us(c_out - c_in),
                          "segments_us": seg}
    return v


def round_view(recs, rounds, k):
    r = rounds[k]
    kv = {name: kernel_view(recs[k, i], name) for i, name in enumerate(("vote", "sat", "upd"))}
    if any(x is None for x in kv.values()):
        return None
    out = {"round": r, "kernels": kv}
    gaps = {"vote -> saturation": us(kv["sat"]["first_entry"] - kv["vote"]["last_exit"]),
            "saturation -> update": us(kv["upd"]["first_entry"] - kv["sat"]["last_exit"])}
    nxt = [j for j in range(SLOTS) if rounds[j] == r + 1]
    end = kv["upd"]["last_exit"]
    if nxt and recs[nxt[0], 0][:, 0].max() > 0:
        nv = recs[nxt[0], 0]
        nfirst = int(nv[nv[:, 0] > 0][:, 0].min())
        gaps["update -> next vote"] = us(nfirst - kv["upd"]["last_exit"])
        end = nfirst
    span = end - kv["vote"]["first_entry"]
    out["round_span_us_stamped"] = us(span)
    out["boundary_gaps_us"] = gaps
    # the accounting: every microsecond of the span, by launch and segment
    acc = {}
    for name in ("vote", "sat", "upd"):
        for seg, x in kv[name]["critical_wave"]["segments_us"].items():
            acc[f"{name}: {seg}"] = x
    for g, x in gaps.items():
        acc[f"boundary {g}"] = x
    total = sum(acc.values())
    out["accounting_us"] = acc
    out["accounted_share"] = round(total / max(1e-9, us(span)), 4)
    out["other_share"] = round(sum(x for s, x in acc.items() if "other" in s) / max(1e-9, us(span)), 4)
    out["shares"] = {s: round(x / max(1e-9, us(span)), 4) for s, x in acc.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cnst", type=int, default=1_000_000)
    ap.add_argument("--vars", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--rounds", default="70,71,200,201")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--product-profile", default=None, help="bench.py --profile-json of the product build")
    ap.add_argument("--out", required=True)
    ap.add_argument("--raw", default=None, help="also save the raw per-wave records here (.npz)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4"], help="c4: the frontier engine on C4")
    args = ap.parse_args()
    assert os.environ.get("LMM_AMD_LIB"), "load the diagnostic build: LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so"
    import torch

    from simgrid_amd import lmm as L

    assert torch.cuda.is_available()
    s = L.System(False)
    t = time.time()
    if args.workload == "c4":
        s.gen_platform_flows(L.platform_params(model=L.LV08, n_flows=100_000, seed=1, topology=L.FAT_TREE,
                                               topo_parameters="3;16,16,16;1,16,16;1,1,1", loopback_bw=1e8),
                             want_vars=False)
        sysname = "C4: 1e5 LV08 flows on fat tree 3;16,16,16;1,16,16;1,1,1 (seed 1), frontier engine"
    else:
        s.gen_synthetic(args.cnst, args.vars, args.k, seed=1, want_vars=False)
        sysname = f"{args.cnst} x {args.vars} x {args.k} (C2 generator, seed 1)"
    s.prepare()
    print(f"built {sysname} in {time.time() - t:.1f}s", flush=True)
    for _ in range(args.warmup):
        s.device_solve()
    os.environ["LMMHIP_ANAT_ROUNDS"] = args.rounds
    s.device_solve()
    st = s.last_stats()
    recs, rounds = load_records(s, L)
    if args.raw:
        np.savez_compressed(args.raw, recs=recs, rounds=np.array(rounds))
    del os.environ["LMMHIP_ANAT_ROUNDS"]
    s.device_solve()
    plain_ms = s.last_stats()["device_ms"]
    out = {"system": sysname, "rounds_total": st["rounds"],
           "stamped_solve_ms": st["device_ms"], "same_build_unstamped_solve_ms": plain_ms,
           "clock": "s_memrealtime, 100 MHz (10 ns ticks), one clock for the chip", "recorded_rounds": rounds,
           "rounds": []}
    for k in range(SLOTS):
        if rounds[k] < 0:
            continue
        rv = (frontier_round_view if args.workload == "c4" else round_view)(recs, rounds, k)
        if rv is not None and any(rounds[j] == rounds[k] + 1 for j in range(SLOTS)):
            out["rounds"].append(rv)
    if args.product_profile and os.path.exists(args.product_profile):
        pp = json.load(open(args.product_profile))
        names = {2: "vote", 4: "saturation", 5: "update"}  # (frontier: slot 4 = fr_sat + fr_sat_big)
        slot, rnd, ms = np.array(pp["launch_slot"]), np.array(pp["launch_round"]), np.array(pp["launch_ms"])
        for rv in out["rounds"]:
            r = rv["round"]
            sel = {names[k]: round(float(1000 * ms[(slot == k) & (rnd == r)].sum()), 2) for k in names}
            rv["product_build_hip_event_us"] = sel
            if "alive_vars" in pp:
                rv["product_alive_rows"] = int(pp["alive_vars"][r]) if r < len(pp["alive_vars"]) else None
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    for rv in out["rounds"]:
        print(f"round {rv['round']}: stamped span {rv['round_span_us_stamped']} us, accounted "
              f"{100 * rv['accounted_share']:.1f} % (other {100 * rv['other_share']:.1f} %)")
        for sname, x in sorted(rv["shares"].items(), key=lambda kv: -kv[1])[:12]:
            print(f"   {100 * x:5.1f} %  {sname}")
    del s


if __name__ == "__main__":
    main()
