set -e
mkdir -p gpurun_out/sp
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --frame-events > gpurun_out/sp/A$i.log 2>&1
ORBMI_TRACK_UNFUSED=1 timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --frame-events > gpurun_out/sp/B$i.log 2>&1
ORBMI_TRACK_UNFUSED=1 ORBMI_LIB=tools/ab/liborbmi_head.so timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --frame-events > gpurun_out/sp/C$i.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sp/pA -o a -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/sp/pA.log 2>&1
ORBMI_TRACK_UNFUSED=1 ORBMI_LIB=tools/ab/liborbmi_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sp/pC -o c -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/sp/pC.log 2>&1
