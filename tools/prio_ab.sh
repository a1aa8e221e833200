mkdir -p gpurun_out/prio
for r in 1 2; do
for cfg in "none" "ORBMI_PRIO_MATCHER=high" "ORBMI_PRIO_MATCHER=high ORBMI_PRIO_EXTRACTOR=high" "ORBMI_PRIO_BA=low ORBMI_PRIO_VOCAB=low"; do
  tag=$(echo $cfg | tr ' =' '__')
  if [ "$cfg" = none ]; then timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/prio/$tag.$r.log 2>&1 || exit 2
  else env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/prio/$tag.$r.log 2>&1 || exit 2; fi
  python -c "import json;d=json.loads(open('gpurun_out/prio/$tag.$r.log').read().strip().splitlines()[-1]);print('$tag',d['value'],d['roofline']['avg_launch_us'],d['track_only_ms_per_frame_back_to_back'],d['local_ba'])"
done; done
