#!/bin/bash
# one-off GPU call: smoke(), then the round artifacts (tests, bench, rocprof stats, FETCH/WRITE
# PMC) of the current code under TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG:-r03l}.log 2>&1 || { tail -20 gpurun_out/smoke_${TAG:-r03l}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG:-r03l}.log
TAG=${TAG:-r03l} bash scripts/gpu_round_artifacts.sh || exit 1
