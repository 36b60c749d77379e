#!/bin/bash
# GPU suite, then the sampler / find tests with the split replay forced on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${TAG:-s}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_${TAG:-s}.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_${TAG:-s}.log
ERP_SAMPLER_SPLIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sampler or sample or full or find or fixture" > gpurun_out/pytest_split_${TAG:-s}.log 2>&1 || { tail -30 gpurun_out/pytest_split_${TAG:-s}.log; exit 1; }
tail -1 gpurun_out/pytest_split_${TAG:-s}.log
