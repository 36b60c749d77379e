set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "consensus or find or manual or shard or fullsize or batch" > gpurun_out/pytest_rows.log 2>&1 || { tail -30 gpurun_out/pytest_rows.log; exit 1; }
tail -2 gpurun_out/pytest_rows.log
timeout -k 10 200 python scripts/dev/determinism.py 64 2 twin || exit 1
timeout -k 10 400 python bench.py --main-batch worst --steps 2 --warmup 1 --no-cpu-baseline --hard-steps 0 --worst-steps 0 > gpurun_out/bench_worst.json 2> gpurun_out/bench_worst.err || { tail gpurun_out/bench_worst.err; exit 1; }
python scripts/bench_summary.py gpurun_out/bench_worst.json
timeout -k 10 400 python bench.py --no-cpu-baseline --hard-steps 0 --worst-steps 0 --steps 10 > gpurun_out/bench_main.json 2> gpurun_out/bench_main.err || { tail gpurun_out/bench_main.err; exit 1; }
python scripts/bench_summary.py gpurun_out/bench_main.json
