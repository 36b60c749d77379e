set -o pipefail
for v in 1; do echo "ERP_LIP2=$v"; ERP_LIP2=$v timeout -k 10 200 python scripts/dev/determinism.py 64 3 twin || exit 1; done
timeout -k 10 200 python scripts/dev/determinism.py 128 2 || exit 1
TAG=r03lipd KNOB=ERP_LIP2 VALUES="1 0" TEST_K="consensus or find or manual or shard" bash scripts/gpu_ab.sh
