set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in base lip8 lip32 base; do
  if [ $v = base ]; then L=""; else L="$PWD/devlibs/$v/liberp_match.so"; fi
  ERP_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --hard-steps 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));st=d['stages_ms_serial_step']
print('$v', round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in st.items() if k.startswith('consensus')}, d['check']['parity']['all_equal'] if d['check'].get('parity') else None)"
done
