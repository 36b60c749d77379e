set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/dev/sampler_sol.py > gpurun_out/sol_r06b.json 2> gpurun_out/sol_r06b.err || { tail -20 gpurun_out/sol_r06b.err; exit 1; }
cat gpurun_out/sol_r06b.json
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_sol_r06b -o run --output-format csv -- python3 scripts/dev/sampler_sol.py --reps 1 > gpurun_out/pmc_sol_r06b.log 2>&1 || { tail -20 gpurun_out/pmc_sol_r06b.log; exit 1; }
echo done
