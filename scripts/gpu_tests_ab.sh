#!/bin/bash
# GPU parity tests of the in-tree library, then an A/B bench of library variants
# (bash scripts/gpu_tests_ab.sh base devlibs/x ...; see scripts/dev/ab_bench.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "== a/b" && bash scripts/dev/ab_bench.sh "$@"
