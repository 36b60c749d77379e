#!/bin/bash
# Round artifacts on one MI355X, every step under its own time limit and chained so that the
# first failure ends the call:
#   1. the GPU parity tests (SKIP_TESTS=1 skips them: the bench / profile passes alone), with the
#      real-pair gaps against the reference's recovered (R, T) written to real_gaps_<TAG>.json;
#   2. the default bench (with the CPU baseline and the oracle parity check);
#   3. EXTRA_BENCH=1: the worst-case batch as the timed batch (--main-batch worst: its stage
#      times and its own oracle parity), configs[2]'s shape (--kpts 2048 --pairs 1024), the
#      single-pair latency probe, and with PHILOX=1 the counter-based sampler line;
#   4. a rocprofv3 kernel-trace --stats run and two PMC passes (FETCH_SIZE, WRITE_SIZE; separate
#      passes, kernel trace only) of the bench workload with --steps 0 --warmup 2: bench.py then
#      runs only its serial profile pass (the default step's sub-batches one after the other), so
#      rocprof sees exactly the launches whose durations bench.py measures with HIP events.
# Then, in the container:
#   python scripts/pmc_summarize.py --tag $TAG --stats gpurun_out/prof_$TAG \
#     --fetch gpurun_out/pmc_fetch_$TAG --write gpurun_out/pmc_write_$TAG      (-> profiles/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r04a}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== gpu tests" && ERP_REAL_GAPS_OUT=gpurun_out/real_gaps_${TAG}.json \
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_${TAG}.log
fi
echo "== bench (default, with cpu baseline)" && timeout -k 10 600 python bench.py --profile-tag ${TAG} \
  > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
tail -c 400 gpurun_out/bench_${TAG}.json
if [ "${EXTRA_BENCH:-0}" = "1" ]; then
  if [ "${PHILOX:-0}" = "1" ]; then  # (the counter-based sampler: an option, not measured every round)
    echo "== bench --sampler philox" && timeout -k 10 600 python bench.py --sampler philox --profile-tag ${TAG} \
      --hard-steps 0 --worst-steps 0 > gpurun_out/bench_philox_${TAG}.json 2> gpurun_out/bench_philox_${TAG}.err \
      || { tail -20 gpurun_out/bench_philox_${TAG}.err; exit 1; }
    tail -c 300 gpurun_out/bench_philox_${TAG}.json
  fi
  # the worst-case batch as the timed batch, with its own oracle check (a bounded CPU sample of
  # the first pair of every sub-batch, then the second, ...) and timed-vs-serial comparison
  echo "== bench --main-batch worst" && timeout -k 10 600 python bench.py --main-batch worst --steps 3 \
    --hard-steps 0 --worst-steps 0 --cpu-seconds 8 --profile-tag ${TAG} > gpurun_out/bench_worst_${TAG}.json \
    2> gpurun_out/bench_worst_${TAG}.err || { tail -20 gpurun_out/bench_worst_${TAG}.err; exit 1; }
  tail -c 300 gpurun_out/bench_worst_${TAG}.json
  echo "== bench configs[2] shape (2048 x 2048 keypoints, 1024 pairs per step)" && timeout -k 10 600 \
    python bench.py --kpts 2048 --pairs 1024 --hard-steps 0 --worst-steps 0 --profile-tag ${TAG} \
    > gpurun_out/bench_configs2_${TAG}.json 2> gpurun_out/bench_configs2_${TAG}.err \
    || { tail -20 gpurun_out/bench_configs2_${TAG}.err; exit 1; }
  tail -c 300 gpurun_out/bench_configs2_${TAG}.json
  echo "== single-pair latency (host) + kernel trace" && timeout -k 10 300 python scripts/latency_probe.py --runs 20 \
    > gpurun_out/latency_host_${TAG}.json 2> gpurun_out/latency_${TAG}.err || { tail -20 gpurun_out/latency_${TAG}.err; exit 1; }
  cat gpurun_out/latency_host_${TAG}.json
  timeout -k 10 300 python scripts/latency_probe.py --runs 20 --graph > gpurun_out/latency_host_graph_${TAG}.json \
    2>> gpurun_out/latency_${TAG}.err || { tail -20 gpurun_out/latency_${TAG}.err; exit 1; }
  cat gpurun_out/latency_host_graph_${TAG}.json
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lat_${TAG} -o run --output-format csv -- \
    python3 scripts/latency_probe.py --runs 20 > gpurun_out/lat_${TAG}.log 2>&1 || { tail -20 gpurun_out/lat_${TAG}.log; exit 1; }
fi
if [ "${SKIP_PROFILE:-0}" != "1" ]; then
  echo "== rocprofv3 kernel-trace stats" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} \
    -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 --profile-tag ${TAG} \
    > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
  echo "== pmc FETCH_SIZE" && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run \
    --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 --profile-tag ${TAG} \
    > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
  echo "== pmc WRITE_SIZE" && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run \
    --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 2 --profile-tag ${TAG} \
    > gpurun_out/pmc_write_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
  find gpurun_out/prof_${TAG} gpurun_out/pmc_fetch_${TAG} gpurun_out/pmc_write_${TAG} -name "*.csv"
fi
echo done
