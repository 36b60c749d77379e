#!/bin/bash
# round 5: which VALU instruction classes return wrong results beside MFMA waves
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python -u scripts/dev/pk_synth.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pk_probe3.log
