set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SMEM"
for F in 1 0; do
  ERP_FUSE_SAMPLER=$F ERP_FUSED_DIAG=1 timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_sq_f$F -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --hard-steps 0 --pairs 64 --streams 1 > gpurun_out/pmc_sq_f$F.log 2>&1 || { tail -5 gpurun_out/pmc_sq_f$F.log; exit 1; }
done
C2="SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"
for F in 1 0; do
  ERP_FUSE_SAMPLER=$F ERP_FUSED_DIAG=1 timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/pmc_sq2_f$F -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --hard-steps 0 --pairs 64 --streams 1 > gpurun_out/pmc_sq2_f$F.log 2>&1 || { tail -5 gpurun_out/pmc_sq2_f$F.log; exit 1; }
done
find gpurun_out/pmc_sq*_f* -name "*counter_collection.csv"
