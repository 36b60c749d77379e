#!/bin/bash
# round 5: the lite estimates (no hypothesis-record round trip) -- GPU suite + bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
TAG=${TAG:-r05b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -15 | tee gpurun_out/pytest_gpu_$TAG.log &&
timeout -k 10 300 python -u bench.py --profile-tag $TAG > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
python scripts/bench_summary.py gpurun_out/bench_$TAG.json 2>&1 | tail -30
