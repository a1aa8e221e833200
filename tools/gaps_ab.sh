# kernel traces of the default bench on two library builds, then the tracking stream's kernel
# durations and gaps (tools/stream_gaps.py): bash tools/gaps_ab.sh LIB_A LIB_B
set -e
mkdir -p gpurun_out/gaps
for L in "$@"; do
  n=$(basename $L .so)
  ORBMI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/gaps/$n -o t -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/gaps/$n.log 2>&1
  python3 tools/stream_gaps.py gpurun_out/gaps/$n > gpurun_out/gaps/$n.txt
  cat gpurun_out/gaps/$n.txt
done
