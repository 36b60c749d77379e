# A/B of an environment knob on the in-tree library: bash scripts/dev/ab_env.sh "" "ERP_NO_ZOOM=1" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --cpu-seconds 2 --steps 10 --warmup 2 --hard-steps 3 > gpurun_out/abe.json 2> gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/abe.json'));st=d['stages_ms_serial_step']
print('[$v]', round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in st.items() if k.startswith('consensus') or k.startswith('knn2')}, 'binned_hard', d['hard_data'].get('binned_rows_mean'), d['check']['parity']['all_equal'], 'hard', round(d['hard_data']['value']))"
done
