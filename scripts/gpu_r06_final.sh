#!/bin/bash
# Round-6 evidence in three calls (each under gpurun's 20-minute limit), on the final build:
#   scripts/gpu_r06_final.sh 1   every -m gpu test, smoke() (build id == tree id), the default bench line (C2)
#   scripts/gpu_r06_final.sh 2   the C2 stress / C3 / C4 / C5 bench lines, kernel traces, calibration, C2 FETCH/WRITE
#   scripts/gpu_r06_final.sh 3   FETCH/WRITE of C3 / C4 / C5, request counts (RDREQ / WRREQ / ATOMIC) of C2 / C4 / C5
# then python scripts/parse_rocprof.py r06 summarises gpurun_out/rp_* into profiles/r06_*.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
case $1 in
  1) scripts/gpu_full.sh || exit $?;;
  2) scripts/gpu_configs.sh || exit $?
     PARTS="trace c3 c4 c5 cal pmc" PMC_WORKLOADS="c2" scripts/profile.sh || exit $?;;
  3) PARTS="pmc req" PMC_WORKLOADS="c3 c4 c5" REQ_WORKLOADS="c2 c4 c5" scripts/profile.sh || exit $?;;
  *) echo "usage: $0 1|2|3"; exit 2;;
esac
echo done
