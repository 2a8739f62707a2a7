#!/bin/bash
# Round 6: the bench lines again, now that profiles/r06_traffic_* and r06_requests_{c2,c4,c5}.json exist (the C4 / C5
# lines carry roofline.requests with each kernel's fraction of its request-class ceiling).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || { tail -20 gpurun_out/bench_default.log; exit 1; }
cat gpurun_out/bench_default.json
scripts/gpu_configs.sh || exit $?
