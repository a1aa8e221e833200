# native closed loop (bench --mode system) on two library builds, alternating: bash tools/sys_ab.sh LIB_A LIB_B
mkdir -p gpurun_out/sysab
for i in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    ORBMI_LIB=$L timeout -k 10 400 python bench.py --mode system --no-cpu-baseline > gpurun_out/sysab/${n}_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/sysab/${n}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n'", d["value"], d["ate_rmse_m"], d["phase_ms_per_frame"], d["synchronous_local_mapping"]["frames_per_s"])' | tee -a gpurun_out/sysab/summary.txt
  done
done
