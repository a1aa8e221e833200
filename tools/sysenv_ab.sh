# native closed loop (bench --mode system) under values of one environment knob, alternating:
# bash tools/sysenv_ab.sh VAR V1 V2 ...   (a value '-' runs with VAR unset)
mkdir -p gpurun_out/sysenv
var=$1; shift
vals=("$@")
for i in 1 2; do
  for v in "${vals[@]}"; do
    if [ "$v" = "-" ]; then kv=(); else kv=("$var=$v"); fi
    env -u $var "${kv[@]}" timeout -k 10 400 python bench.py --mode system --no-cpu-baseline > gpurun_out/sysenv/${var}_${v}_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/sysenv/${var}_${v}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$var=$v'", d["value"], d["ate_rmse_m"], d["phase_ms_per_frame"], d["local_mapping_ms_per_keyframe"]["total"], d["synchronous_local_mapping"]["frames_per_s"])' | tee -a gpurun_out/sysenv/summary.txt
  done
done
