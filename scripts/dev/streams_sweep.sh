# pairs-per-step / stream-count sweep: bash scripts/dev/streams_sweep.sh "384 3" "768 6" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "$@"; do set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --hard-steps 0 --pairs $1 --streams $2 > gpurun_out/st.json 2> gpurun_out/st.err || { tail -3 gpurun_out/st.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/st.json'));print('$1 $2', round(d['value']), round(d['ms_per_step'],2))"
done
