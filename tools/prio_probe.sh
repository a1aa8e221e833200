#!/bin/bash
# Headline bench under stream-priority settings (ORBMI_PRIO_<ROLE>); one line per setting.
OUT=gpurun_out/${1:-prio}
mkdir -p $OUT
for cfg in "" "ORBMI_PRIO_BA=high" "ORBMI_PRIO_VOCAB=high" "ORBMI_PRIO_BA=high ORBMI_PRIO_VOCAB=high" "ORBMI_PRIO_EXTRACTOR=low"; do
    name=$(echo "base $cfg" | tr ' =' '__')
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/$name.log 2>&1
    rc=$?
    echo -n "[$cfg] rc=$rc "
    tail -1 $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['local_ba'].get('ms_per_keyframe_idle_gpu (ComputeBoW + LocalBA)'))" 2>/dev/null || echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
