#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun).  Counter passes are separate from
# the kernel-trace passes, one counter per pass, as MI355X_MICROARCH.md prescribes (FETCH_SIZE and
# WRITE_SIZE do not fit in one pass).  Output: gpurun_out/rp_*/ (CSV), summarised into profiles/ by
# scripts/parse_rocprof.py.  usage: PARTS="trace c3 c4 c5 pmc req cal" scripts/profile.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PARTS=${PARTS:-"trace c3 c4 c5 pmc cal"}
PMC_WORKLOADS=${PMC_WORKLOADS:-"c2 c3 c4 c5"}
has() { case " $PARTS " in *" $1 "*) return 0;; *) return 1;; esac; }
# every step: its own time limit, its rc logged, and the script ends at the first failure of any kind
run() {  # run <log> <limit s> <command...>
  local log=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$log"
  if [ $rc -ne 0 ]; then echo "step failed (rc=$rc): $log"; tail -5 "$log"; exit $rc; fi
}
wl_args() {  # bench arguments of one short run of a workload
  case $1 in
    c2) echo "--steps $2 --warmup 1 --no-cpu-baseline --dropin-steps 0";;
    c2_stress) echo "--variant stress --steps $2 --warmup 1 --no-cpu-baseline --dropin-steps 0";;
    *) echo "--workload $1 --steps $2 --warmup 1 --no-cpu-baseline";;
  esac
}
if has trace; then  # C2 (the BASELINE metric's config)
  run gpurun_out/rp_trace.log 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace -o run \
    -- python3 bench.py $(wl_args c2 3)
fi
for w in c3 c4 c5; do
  has $w || continue
  run gpurun_out/rp_trace_$w.log 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace_$w \
    -o run -- python3 bench.py $(wl_args $w 10)
done
if has pmc; then
  for w in $PMC_WORKLOADS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      run gpurun_out/rp_${ctr}_$w.log 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_${ctr}_$w -o run \
        -- python3 bench.py $(wl_args $w 2)
    done
  done
fi
REQ_WORKLOADS=${REQ_WORKLOADS:-"c2"}
if has req; then  # request counts (the request-rate roofline): one counter per pass, per workload
  run gpurun_out/rp_trace_cal.log 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_trace_cal \
    -o run -- ./scripts/ubench_gather
  for ctr in TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum; do
    for w in $REQ_WORKLOADS; do
      run gpurun_out/rp_${ctr}_$w.log 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_${ctr}_$w -o run \
        -- python3 bench.py $(wl_args $w 2)
    done
    run gpurun_out/rp_cal_$ctr.log 200 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_cal_$ctr -o run \
      -- ./scripts/ubench_gather
  done
fi
if has cal; then  # calibration on known byte counts (scripts/ubench_gather.hip: 320 MB int32 stream, gathers)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run gpurun_out/rp_cal_$ctr.log 200 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/rp_cal_$ctr -o run \
      -- ./scripts/ubench_gather
  done
fi
exit 0
