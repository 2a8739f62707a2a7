#!/bin/bash
# rocprofv3 kernel trace of a short C2 run (timeline: busy time and inter-kernel gaps, scripts/trace_gaps.py).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rp_gap -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 ${BENCH_ARGS} > gpurun_out/rp_gap.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/rp_gap.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/rp_gap.log; exit $rc; }
python3 scripts/trace_gaps.py gpurun_out/rp_gap
