#!/bin/bash
# C5 iteration: the bit-identical FairBottleneck tests, then C5 lines with the renumbered solve and without.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "c5" -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_c5.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 40 gpurun_out/pytest_c5.log; exit $rc; fi
for rn in 1 0; do
  LMMHIP_FB_RENUM=$rn timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/c5_renum$rn.json 2> gpurun_out/c5_renum$rn.log; rc=$?
  if [ $rc -ne 0 ]; then echo "STOP renum=$rn rc=$rc"; tail -n 20 gpurun_out/c5_renum$rn.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/c5_renum$rn.json').read().strip().splitlines()[-1]); print('c5 renum=$rn', d['ms_per_step'], d['value'])"
done
echo done
