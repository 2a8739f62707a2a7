#!/bin/bash
# Bench lines for the SURVEY.md §8(d) configs other than C2 (one GPU), plus the C2 stress variant (5% FATPIPE,
# 10% bounded, penalties {1,2,4}); each step under its own limit.
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --variant stress --steps 5 --warmup 1 --dropin-steps 0 --cpu-reps 3 \
  > gpurun_out/bench_c2_stress.json 2> gpurun_out/bench_c2_stress.log
rc=$?; echo "stress rc=$rc" >> gpurun_out/bench_c2_stress.log
if [ $rc -ne 0 ]; then echo "STOP stress rc=$rc"; tail -20 gpurun_out/bench_c2_stress.log; exit $rc; fi
cat gpurun_out/bench_c2_stress.json
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.log
  rc=$?; echo "$w rc=$rc" >> gpurun_out/bench_$w.log
  if [ $rc -ne 0 ]; then echo "STOP $w rc=$rc"; tail -20 gpurun_out/bench_$w.log; exit $rc; fi
  cat gpurun_out/bench_$w.json
done
