# LocalBA (config 3) under ORBMI_BA_SLACK settings (trial steps enqueued beyond the iterations): bash tools/slack_ab.sh
set -o pipefail
mkdir -p gpurun_out/slack
for i in 1 2; do for v in "X=1" "ORBMI_BA_SLACK=0" "ORBMI_BA_SLACK=3"; do
  env $v timeout -k 10 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/slack/run.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/slack/run.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["iterations"])')" | tee -a gpurun_out/slack/slack.txt
done; done
