#!/bin/bash
# The N > 1 bench path rehearsed on ONE leased GPU (VERDICT r05 "next" 5): N ranks started by
# bench.py's own launcher (torch.distributed.run as a child), every rank on device 0, gloo
# collectives on host copies (RCCL refuses two ranks on one GPU).  Path readiness, not scaling.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r06b}; N=${N:-2}
echo "== bench --gpus $N on one device" && timeout -k 10 600 python bench.py --gpus $N --dist-backend gloo \
  --ranks-on-device 0 --steps 3 --warmup 1 --hard-steps 0 --worst-steps 0 \
  > gpurun_out/bench_ranks${N}_${TAG}.json 2> gpurun_out/bench_ranks${N}_${TAG}.err \
  || { tail -30 gpurun_out/bench_ranks${N}_${TAG}.err; exit 1; }
tail -c 1500 gpurun_out/bench_ranks${N}_${TAG}.json
