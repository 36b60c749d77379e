set -o pipefail
timeout -k 10 200 python scripts/dev/determinism.py 64 2 twin || exit 1
TAG=r03dot KNOB=ERP_DOT_BOUNDS VALUES="1 0" TEST_K="consensus or find or manual or shard or fullsize or batch" bash scripts/gpu_ab_prof.sh
