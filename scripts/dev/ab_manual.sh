# A/B of library variants on the configs[4] manual workload: bash scripts/dev/ab_manual.sh base devlibs/x ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L="$PWD/$v/liberp_match.so"; fi
  t=$(basename "$v")
  ERP_LIB_PATH=$L timeout -k 10 200 python bench.py --workload manual > gpurun_out/abm_$t.json 2> gpurun_out/abm_$t.err || { tail -5 gpurun_out/abm_$t.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/abm_$t.json'));st=d['stages_ms_rank0']
print('$t', round(d['ms_per_step'],3), {k:round(v,3) for k,v in st.items() if v > 0.05}, {k:v['same_winner'] for k,v in d['row_shard_emulation'].items()})"
done
