"""Summary line of one A/B variant (scripts/gpu_ab.sh): timed C2 / C4 solves, C2 per-kernel averages from the
per-launch profile, C4 persistent-engine phase sums."""
import json
import sys

tag, i = sys.argv[1], sys.argv[2]
out = [tag]
for w in ("c2", "c3", "c4", "c5"):
    try:
        d = json.load(open(f"gpurun_out/ab_{i}_{w}.json"))
    except OSError:
        continue
    out.append(f"{w} {d['ms_per_step']} ms ({d['config'].get('device_rounds')} rounds)")
try:
    p = json.load(open(f"gpurun_out/ab_{i}_c2prof.json"))
    out.append("c2 per launch us: " + " ".join(f"{k}={v['avg_us']:.1f}" for k, v in p["per_kernel"].items()
                                               if k not in ("mm_init_vars",)))
except (OSError, KeyError):
    pass
try:
    q = json.load(open(f"gpurun_out/persist_c4.json"))
    ph = q["phase_us"]
    v = s = u = 0.0
    k, r = 0, 0
    while k + 2 < len(ph) and r < q["rounds"]:
        v, s, u, k = v + ph[k], s + ph[k + 1], u + ph[k + 2], k + 3
        if r % 16 == 15 and r < q["rounds"] - 1:
            k += 1
        r += 1
    n = max(r, 1)
    out.append(f"c4 persistent per round us: vote={v / n:.1f} sat={s / n:.1f} upd={u / n:.1f} "
               f"barrier={sum(q['barrier_us']) / n:.1f}")
except (OSError, KeyError):
    pass
print(" | ".join(out), flush=True)
