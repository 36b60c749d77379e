#!/bin/bash
# round 5: GPU suite on the release library and on the launch-checking debug build, then the
# round-4-scale determinism measurement (40 overlapped 768-pair steps = 30 720 records)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
TAG=${TAG:-r05c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -8 | tee gpurun_out/pytest_gpu_$TAG.log &&
ERP_LIB_PATH=scripts/dev/libs/dbglaunch/liberp_match.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -8 | tee gpurun_out/pytest_gpu_dbglaunch_$TAG.log &&
WANT= REPEAT=40 timeout -k 10 600 python -u scripts/dev/determinism_rvec.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/determinism_rvec_$TAG.log
