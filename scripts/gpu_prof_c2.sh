#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/prof_c2.json > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || { echo "bench failed"; exit 1; }
