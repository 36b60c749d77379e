#!/bin/bash
# smoke() and the bench through the torch.distributed launcher (world size 1 on the box's GPU:
# the RCCL init / barrier / max-over-ranks path the driver's N-GPU runs take)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== launcher" && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_launcher.json 2> gpurun_out/bench_launcher.err || { tail -20 gpurun_out/bench_launcher.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_launcher.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['config']['parallelism'], d['roofline']['traffic'])"
