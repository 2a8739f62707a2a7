#!/bin/bash
# Round 5: C2 kernel trace + the request-count passes (request-rate roofline) -> gpurun_out/rp_*
cd "$GRAFT_REPO_ROOT" || exit 1
PARTS="trace req" scripts/profile.sh || exit $?
echo done
