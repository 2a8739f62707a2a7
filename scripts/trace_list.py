"""Launch-by-launch listing of the last solve in a rocprofv3 --kernel-trace run: kernel, duration, gap before.
usage: python scripts/trace_list.py gpurun_out/<dir> <solve-start-kernel> [max-lines]"""
import csv
import glob
import sys

f = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))[0]
mark = sys.argv[2]
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 400
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lmmdev::", "")))
rows.sort()
a = [i for i, r in enumerate(rows) if mark in r[2]][-2]  # the second-to-last solve (the last may be profiled)
t0 = rows[a][0]
prev = rows[a][0]
for s, e, n in rows[a:a + cap]:
    if n.startswith(mark) and s != rows[a][0]:
        break
    print(f"{(s - t0) / 1e3:9.1f} +{(s - prev) / 1e3:6.1f} {n[:40]:40s} {(e - s) / 1e3:8.1f} us")
    prev = e
