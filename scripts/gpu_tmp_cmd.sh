#!/bin/bash
# one-off GPU call: round artifacts (tests, bench, rocprof stats, FETCH/WRITE PMC) of the
# current code under TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03h} bash scripts/gpu_round_artifacts.sh || exit 1
