#!/bin/bash
# Frontier-engine iteration: bit-identity tests vs the round engine, then C2 lines (frontier / default) and a
# per-launch profile of the frontier engine.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_engines.py} -k "${TK:-frontier}" -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_fr.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_fr.log
if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; tail -n 40 gpurun_out/pytest_fr.log; exit $rc; fi
for w in ${WL:-c2 c4}; do
  engs="frontier rounds"; [ "$w" = c4 ] && engs="frontier persistent"
  for eng in $engs; do
    LMMHIP_ENGINE=$eng timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
      > gpurun_out/fr_${eng}_$w.json 2> gpurun_out/fr_${eng}_$w.log; rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $eng $w rc=$rc"; tail -n 20 gpurun_out/fr_${eng}_$w.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/fr_${eng}_$w.json').read().strip().splitlines()[-1]); print('$eng $w', d['ms_per_step'], d['value'])"
  done
done
env ${DIAGENV:-X=1} LMMHIP_ENGINE=frontier timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --profile-json gpurun_out/fr_c2prof.json > /dev/null 2> gpurun_out/fr_c2prof.log; rc=$?
if [ $rc -ne 0 ]; then echo "STOP c2prof rc=$rc"; tail -n 20 gpurun_out/fr_c2prof.log; exit $rc; fi
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    LMMHIP_ENGINE=frontier timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/fr_pmc_$ctr -o run \
      -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > gpurun_out/fr_pmc_$ctr.log 2>&1; rc=$?
    if [ $rc -ne 0 ]; then echo "STOP pmc $ctr rc=$rc"; tail -n 20 gpurun_out/fr_pmc_$ctr.log; exit $rc; fi
  done
fi
echo done
