#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun).  Counter passes are separate from
# the kernel-trace pass, as MI355X_MICROARCH.md prescribes (FETCH_SIZE and WRITE_SIZE do not fit in
# one pass).  Output: gpurun_out/rp_*/ (CSV).  usage: scripts/profile.sh [bench args...]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 $*"
PARTS=${PARTS:-"trace c3 c5 pmc c4"}  # subset to run (e.g. PARTS="c4 pmc")
has() { case " $PARTS " in *" $1 "*) return 0;; *) return 1;; esac; }
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if has trace; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace -o run \
    -- python3 $BENCH > gpurun_out/rp_trace.log 2>&1
  rc=$?; echo "trace rc=$rc" >> gpurun_out/rp_trace.log; if fatal $rc; then exit $rc; fi
fi
for w in c3 c5; do  # the batch kernel (C3: one dispatch per solve) and the FairBottleneck kernels (C5)
  has $w || continue
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace_$w -o run \
    -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rp_trace_$w.log 2>&1
  rc=$?; echo "trace $w rc=$rc" >> gpurun_out/rp_trace_$w.log; if fatal $rc; then exit $rc; fi
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  has pmc || continue
  timeout -k 10 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_$ctr -o run \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --dropin-steps 0 "$@" > gpurun_out/rp_$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc" >> gpurun_out/rp_$ctr.log; if fatal $rc; then exit $rc; fi
  # calibration on known byte counts (scripts/ubench_gather.hip: 320 MB int32 stream, gathers)
  timeout -k 10 200 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_cal_$ctr -o run \
    -- ./scripts/ubench_gather > gpurun_out/rp_cal_$ctr.log 2>&1
  rc=$?; echo "cal $ctr rc=$rc" >> gpurun_out/rp_cal_$ctr.log; if fatal $rc; then exit $rc; fi
done
# the persistent engine (C4) last: rocprofv3 has crashed in its exit handler after writing this trace
# (SIGSEGV in the tool's teardown, outputs complete), and nothing may run after a crash in one call
if has c4; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace_c4 -o run \
    -- python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rp_trace_c4.log 2>&1
  rc=$?; echo "trace c4 rc=$rc" >> gpurun_out/rp_trace_c4.log
fi
exit 0
