#!/bin/bash
# Focused GPU check: the given pytest -k expression (default: the consensus tests) with -s, one
# process, every step under its own time limit.  Usage: K='consensus' bash scripts/gpu_focus.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${K:-consensus}
TAG=${TAG:-focus}
timeout -k 10 600 python -u -m pytest tests -x -v -s -m gpu -k "$K" -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
grep -E "PASS|FAIL|survivors|binned" gpurun_out/pytest_${TAG}.log | tail -40
