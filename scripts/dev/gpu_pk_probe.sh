#!/bin/bash
# round 5 bisection, third call: the packed-f32 pruning test beside each stage group
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
: > gpurun_out/pk_probe.log
env SAMPLER=0 REPS=20 MASKS=1,4,8,16,31 GUARD=0 PAIRS=0 PK=1 timeout -k 10 300 python -u scripts/dev/lds_guard_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/pk_probe.log
