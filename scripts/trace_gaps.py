"""Per-solve kernel timeline of a rocprofv3 --kernel-trace run (gpurun_out/<dir>): busy time per kernel, idle gaps
between consecutive kernels (launch / drain overhead), per-round totals of the last max-min solve.
usage: python scripts/trace_gaps.py gpurun_out/rp_gap [solve-start-kernel]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "mm_init_cnsts"
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
starts = [i for i, r in enumerate(rows) if mark in r[2]]
a = starts[-1]
b = len(rows)
seg = rows[a:b]
# stop at the first kernel that is not part of a solve after the last mm_ctl_out burst
busy = collections.Counter()
cnt = collections.Counter()
gap_after = collections.Counter()
for i, (s, e, n) in enumerate(seg):
    short = n.replace("void lmmdev::", "").replace("lmmdev::", "")
    busy[short] += e - s
    cnt[short] += 1
    if i + 1 < len(seg):
        gap_after[short] += max(0, seg[i + 1][0] - e)
span = seg[-1][1] - seg[0][0]
print(f"solve span {span/1e3:.1f} us, kernels {len(seg)}, busy {sum(busy.values())/1e3:.1f} us, "
      f"gaps {sum(gap_after.values())/1e3:.1f} us")
for k, v in busy.most_common():
    print(f"  {k[:60]:60s} n={cnt[k]:4d} busy {v/1e3:9.1f} us avg {v/cnt[k]/1e3:7.2f} us  gap-after avg "
          f"{gap_after[k]/cnt[k]/1e3:6.2f} us")
