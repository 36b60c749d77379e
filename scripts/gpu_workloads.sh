#!/bin/bash
# The non-headline workloads at the current tree, each as a bench line and a rocprofv3
# kernel-trace --stats pass of the same command (VERDICT r05 "next" 4):
#   dense  -- configs[3], one 16384 x 16384 match on both matcher methods
#   manual -- configs[4], one 100k-iteration find() on the manual-pickup regime
#   e2e    -- do_all + find from 5376 x 2688 images
#   remap  -- the band remap + rectification of 5376 x 2688 images
# Every GPU step has its own time limit; the first failure ends the call.
# Then, in the container: python scripts/kstats_copy.py --tag $TAG (-> profiles/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06a}
WL=${WORKLOADS:-"dense manual e2e remap"}
for w in $WL; do
  case $w in
    dense)  A="--workload dense --steps 5 --warmup 2" ;;
    manual) A="--workload manual --steps 5 --warmup 2" ;;
    e2e)    A="--workload e2e --steps 8 --warmup 2" ;;
    remap)  A="--workload remap --steps 5 --warmup 2" ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
  echo "== bench $w" && timeout -k 10 300 python bench.py $A > gpurun_out/bench_${w}_${TAG}.json \
    2> gpurun_out/bench_${w}_${TAG}.err || { tail -20 gpurun_out/bench_${w}_${TAG}.err; exit 1; }
  tail -c 300 gpurun_out/bench_${w}_${TAG}.json
  echo "== rocprof $w" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${w}_${TAG} \
    -o run --output-format csv -- python3 bench.py $A > gpurun_out/prof_${w}_${TAG}.log 2>&1 \
    || { tail -20 gpurun_out/prof_${w}_${TAG}.log; exit 1; }
done
find gpurun_out -path "*_${TAG}*" -name "*kernel_stats.csv"
echo done
