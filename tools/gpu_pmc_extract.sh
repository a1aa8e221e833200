#!/bin/bash
# SQ counters of the extractor kernels on the extraction bench (two passes of 8 SQ counters).
# Usage (via gpurun): bash tools/gpu_pmc_extract.sh TAG [bench args...] -> gpurun_out/TAG/
TAG=${1:-pmcx}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${@:-"--mode extract --steps 20 --warmup 4 --no-cpu-baseline"}
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P1=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS
P2=SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,SQ_LDS_IDX_ACTIVE
timeout -s KILL 120 rocprofv3 --pmc $(echo $P1 | tr , ' ') --kernel-trace -f csv -d $OUT/p1 -o p1 -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
echo "p1 exit $?"
timeout -s KILL 120 rocprofv3 --pmc $(echo $P2 | tr , ' ') --kernel-trace -f csv -d $OUT/p2 -o p2 -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
echo "p2 exit $?"
python tools/pmc_sq.py $OUT > $OUT/sq.txt
cat $OUT/sq.txt | head -120
