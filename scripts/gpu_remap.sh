#!/bin/bash
# section 8f remaps: their parity tests and a rocprofv3 kernel-trace of the remap bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== remap tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_remap.py -v -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_remap.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert|certified" gpurun_out/pytest_remap.log | tail -40; tail -3 gpurun_out/pytest_remap.log; exit $rc
