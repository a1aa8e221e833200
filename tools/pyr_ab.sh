# config 5 (bench --mode batch): the one-launch pyramid (k_pyr_chain) vs a launch per level
# (ORBMI_PYR=levels), and band counts: bash tools/pyr_ab.sh [BANDS ...].  Kept for the record of
# profiles/r05/pyr_chain_ab.txt: k_pyr_chain measured no faster and was removed, so today every
# variant runs the per-level launches.
mkdir -p gpurun_out/pyrab
for i in 1 2 3; do
  for v in levels chain "$@"; do
    case $v in
      levels) kv="ORBMI_PYR=levels";;
      chain) kv="ORBMI_PYR=chain";;
      *) kv="ORBMI_PYR_BANDS=$v";;
    esac
    env $kv timeout -k 10 200 python bench.py --mode batch --steps 50 --warmup 4 --no-cpu-baseline > gpurun_out/pyrab/${v}_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/pyrab/${v}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$kv'", d["value"], d.get("stage_ms_per_step"))' | tee -a gpurun_out/pyrab/summary.txt
  done
done
