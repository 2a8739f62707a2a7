#!/bin/bash
# Round evidence (through gpurun): every -m gpu test, smoke(), the default bench line (C2), then the other
# configs' lines (scripts/gpu_configs.sh).  Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
scripts/gpu_full.sh || exit $?
scripts/gpu_configs.sh || exit $?
