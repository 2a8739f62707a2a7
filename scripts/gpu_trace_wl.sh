#!/bin/bash
# rocprofv3 kernel trace of a short bench run of one workload: usage WL=c5 scripts/gpu_trace_wl.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rp_$WL -o run \
  -- python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rp_$WL.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/rp_$WL.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/rp_$WL.log; exit $rc; }
exit 0
