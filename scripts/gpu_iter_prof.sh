#!/bin/bash
# gpu_iter.sh + one rocprofv3 kernel-trace pass of the C2 bench (per-kernel durations without the
# per-launch HIP events).  Stops at the first failure.
bash scripts/gpu_iter.sh "$@" || exit $?
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_iter -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rp_iter.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/rp_iter.log; exit $rc
