# A/B of stereo extraction (--mode extract) and config 5 (--mode batch) under environment settings:
# bash tools/exab.sh "VAR=VAL ..." ...   ("X=1" = the defaults); results in gpurun_out/exab/exab.txt
set -o pipefail
mkdir -p gpurun_out/exab
for i in 1 2; do
for v in "$@"; do
  for m in extract batch; do
    env $v timeout -k 10 200 python bench.py --mode $m --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/exab/run.log 2>&1 || exit 1
    echo "$m $v: $(tail -1 gpurun_out/exab/run.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("stage_ms_per_launch"))')" | tee -a gpurun_out/exab/exab.txt
  done
done; done
