#!/bin/bash
# Round-2 records on the GPU box: rocprofv3 kernel trace + stats and FETCH/WRITE
# passes of the default bench (tools/profile.sh), bench lines of the other
# single-GPU configs (tools/configs.sh), single-game latency (tools/latency.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile.sh || exit $?
bash tools/configs.sh || exit $?
timeout -k 10 600 python tools/latency.py > gpurun_out/latency.log 2>&1; rc=$?; echo "== latency rc=$rc"; cat gpurun_out/latency.log | grep '^{'
exit $rc
