# determinism_rvec.py under several knob combinations (CONFIGS: ';'-separated env assignments)
cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra CFGS <<< "${CONFIGS:-ERP_LIPG=1}"
for c in "${CFGS[@]}"; do
  echo "== $c"
  env $c WANT="${WANT:-}" timeout -k 10 300 python -u scripts/dev/determinism_rvec.py > gpurun_out/det_rvec.log 2>&1 || { tail -20 gpurun_out/det_rvec.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/det_rvec.log
done
