#!/bin/bash
# Round-5 rocprofv3 evidence in two calls (each under gpurun's 20-minute limit):
#   scripts/gpu_r05_evidence.sh 1   kernel traces (C2, C3, C4, C5), calibration, FETCH/WRITE passes of C2 and C2 stress
#   scripts/gpu_r05_evidence.sh 2   FETCH/WRITE passes of C3, C4, C5
# then python scripts/parse_rocprof.py r05 summarises gpurun_out/rp_* into profiles/r05_*.
cd "$GRAFT_REPO_ROOT" || exit 1
case $1 in
  1) PARTS="trace c3 c4 c5 pmc cal" PMC_WORKLOADS="c2 c2_stress" scripts/profile.sh || exit $?;;
  2) PARTS="pmc" PMC_WORKLOADS="c3 c4 c5" scripts/profile.sh || exit $?;;
  *) echo "usage: $0 1|2"; exit 2;;
esac
echo done
