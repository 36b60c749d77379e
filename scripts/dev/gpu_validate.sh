#!/bin/bash
# round 5: the no-packed-FP32 build -- overlap bisection probe, overlapped vs serial records,
# the GPU suite, the bench (one call; every step under its own limit, chained with &&)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
TAG=${TAG:-r05a}
env SAMPLER=0 REPS=10 MASKS=8,31 GUARD=0 PAIRS=1 PK=0 timeout -k 10 300 python -u scripts/dev/lds_guard_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/validate_pairs_$TAG.log &&
timeout -k 10 300 python -u scripts/dev/determinism_streams.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/validate_streams_$TAG.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -15 | tee gpurun_out/pytest_gpu_$TAG.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
python scripts/bench_summary.py gpurun_out/bench_$TAG.json 2>&1 | tail -30
