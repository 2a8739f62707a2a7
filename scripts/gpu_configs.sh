#!/bin/bash
# Bench lines for the SURVEY.md §8(d) configs other than C2 (one GPU), each step under its own limit.
mkdir -p gpurun_out
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 5 --warmup 1 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.log
  rc=$?; echo "$w rc=$rc" >> gpurun_out/bench_$w.log
  if [ $rc -ne 0 ]; then echo "STOP $w rc=$rc"; tail -20 gpurun_out/bench_$w.log; exit $rc; fi
  cat gpurun_out/bench_$w.json
done
