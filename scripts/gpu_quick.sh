#!/bin/bash
# Short GPU session: micro-benchmark + selected tests + smoke.  Stops on GPU fault/abort/timeout.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 ./scripts/ubench_gather > gpurun_out/ubench.txt 2>&1; rc=$?
if fatal $rc; then echo "STOP ubench rc=$rc"; exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -k "${1:-fair}" > gpurun_out/pytest_quick.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
if fatal $rc; then echo "STOP pytest rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.log
exit 0
