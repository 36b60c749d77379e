# A/B of library variants on one MI355X: bash scripts/dev/ab_bench.sh base devlibs/x ...
# ("base" = the in-tree library); bench with parity check, per-stage times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L="$PWD/$v/liberp_match.so"; fi
  t=$(basename "$v")
  ERP_LIB_PATH=$L timeout -k 10 200 python bench.py --cpu-seconds 2 --steps 10 --warmup 2 --hard-steps 0 > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || { tail -5 gpurun_out/ab_$t.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_$t.json'));st=d['stages_ms_serial_step']
print('$t', round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in st.items() if v > 0.3}, d['check']['parity']['all_equal'])"
done
