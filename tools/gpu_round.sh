#!/bin/bash
# One GPU session of round evidence (via gpurun): bash tools/gpu_round.sh TAG -> gpurun_out/TAG/
# The parity suite, rocprofv3 kernel stats and HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the
# default bench, then the bench line of every mode; summaries under gpurun_out/TAG/profiles/
# (copy them into profiles/TAG/).  Steps: tools/gpu.sh.
exec bash tools/gpu.sh ${1:-round} tests smoke prof pmc bench bench_lba bench_batch bench_extract bench_system
