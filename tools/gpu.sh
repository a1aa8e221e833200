#!/bin/bash
# The one GPU runner (via gpurun): bash tools/gpu.sh TAG STEP [STEP ...]
# Each step runs under its own time limit; the script stops at the first step that crashes or
# times out (exit status other than 0/1) and starts nothing more on the GPU.  Output goes to
# gpurun_out/TAG/ (summaries worth keeping under gpurun_out/TAG/profiles/, which gpurun merges
# back: copy them into profiles/TAG/ here).
#
# Steps:
#   tests            pytest -m gpu (whole suite)
#   tests=EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            bench.py (default track mode, with the CPU baseline)
#   bench_quick      bench.py --steps 60 --warmup 8 --no-cpu-baseline
#   bench_MODE       bench.py --mode MODE (lba, batch, extract, system)
#   gloo2            bench.py --gpus 2 --dist-backend gloo (config 4 rehearsal on one device)
#   prof             rocprofv3 --kernel-trace --stats of the default bench
#   prof_MODE        the same for --mode MODE
#   proflib=LIB      the default bench's kernel stats on another library build
#   hiptrace         kernel + HIP API trace of a short default bench
#   sqpmc[_MODE]     two SQ counter passes (waves, issue, LDS, VMEM) -> per-kernel means
#   poselat[=LIB]    tools/pose_latency.py (PoseOptimization latency), optionally on another build
#   greedy[=LIB]     tools/greedy_probe.py (k_greedy rounds and phase cycles), optionally on another build
#   ktrace[_MODE]    rocprofv3 --kernel-trace of a short bench run + tools/trace_gaps.py
#   pmc              FETCH_SIZE and WRITE_SIZE passes of the default bench -> traffic.json
#   pmc_MODE         the same for --mode MODE
#   native[_async]   tools/native_probe.py (sync / concurrent LocalMapping)
#   nativeprof[_async] its rocprofv3 kernel stats
#   lmprobe          tools/lm_chain_probe.py (per-call split of the LocalMapping chain)
#   solvetrace[=VAR=1]  per-step split of the reduced-system solve (tools/ubench/solve_trace)
#   mfma_pmc         MFMA counters of tools/ubench/mfma_schur (build it first)
#   ab=A,B           bench A/B of two library builds (ORBMI_LIB paths), 3 alternations
#   abbatch=A,B      the same in --mode batch (config 5)
#   envab=VAR=VALUE  the default bench without / with an environment knob, 3 alternations
#   descab           config 5: four keypoints per wave in k_describe vs one (ORBMI_DESC=wave)
#   fastab           config 5: bit-sliced k_fast2 vs the per-lane k_fast (ORBMI_FAST=v1)
#   blurab           config 5: GaussianBlur on a side stream / in the octree launch / after it
TAG=${1:-run}
shift
OUT=gpurun_out/$TAG
P=$OUT/profiles
mkdir -p $OUT $P
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name exit $rc" | tee -a $OUT/status.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -40 $OUT/$name.log; exit $rc; fi
    return 0
}
modeargs() {  # MODE -> bench args
    case $1 in
        track) echo "";;
        lba) echo "--mode lba --steps 50 --warmup 10";;
        batch) echo "--mode batch --steps 50 --warmup 4";;
        extract) echo "--mode extract";;
        extractq) echo "--mode extract --steps 20 --warmup 4";;
        system) echo "--mode system";;
    esac
}
python -c "import torch; print(torch.cuda.get_device_name(0))" > $OUT/device.txt 2>&1
for step in "$@"; do
    case $step in
        tests)
            run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread
            tail -4 $OUT/pytest_gpu.log; cp $OUT/pytest_gpu.log $P/;;
        libtests=*)
            # libtests=LIB:EXPR -- pytest -m gpu -k EXPR on another library build (A/B variants)
            v=${step#libtests=}; l=${v%%:*}; e=${v#*:}; n=$(basename $l .so)
            ORBMI_LIB=$l run libtests_$n 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "$e"
            tail -5 $OUT/libtests_$n.log;;
        tests=*)
            run pytest_sel 600 python -u -m pytest tests -m gpu -v -rf -s --timeout 300 --timeout-method thread -k "${step#tests=}"
            tail -30 $OUT/pytest_sel.log;;
        smoke)
            run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; cat $OUT/smoke.log;;
        bench)
            run bench 500 python bench.py; tail -1 $OUT/bench.log | tee $P/bench.json;;
        frame_events)
            # which chain ends the headline's timed region (tracking_done_ms / mapping_done_ms)
            run frame_events 500 python bench.py --frame-events --steps 200 --warmup 10 --no-cpu-baseline
            tail -1 $OUT/frame_events.log | tee $P/bench_frame_events.json;;
        bench_quick)
            run bench_quick 300 python bench.py --steps 60 --warmup 8 --no-cpu-baseline; tail -1 $OUT/bench_quick.log;;
        bench_*)
            m=${step#bench_}
            run bench_$m 500 python bench.py $(modeargs $m); tail -1 $OUT/bench_$m.log | tee $P/bench_$m.json;;
        gloo2)
            run gloo2 500 python bench.py --gpus 2 --dist-backend gloo --steps 40 --warmup 8 --no-cpu-baseline
            tail -1 $OUT/gloo2.log | tee $P/bench_config4_gloo2.json;;
        hiptrace)
            # kernel trace + HIP API trace of a short default bench (host enqueue vs GPU timeline)
            run hiptrace 300 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/hiptrace -o ht -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline
            find $OUT/hiptrace -name "*.csv" | head;;
        proflib=*)
            # kernel stats of the default bench on another library build (A/B of a kernel variant)
            l=${step#proflib=}; n=$(basename $l .so)
            ORBMI_LIB=$l run prof_$n 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$n -o stats -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline
            find $OUT/prof_$n -name "*kernel_stats.csv" -exec cp {} $P/kernel_stats_$n.csv \;
            cut -d, -f1-5 $P/kernel_stats_$n.csv | head -12;;
        prof|prof_*)
            m=${step#prof}; m=${m#_}; m=${m:-track}
            run prof_$m 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$m -o stats -- python3 bench.py $(modeargs $m) --steps 100 --warmup 10 --no-cpu-baseline
            find $OUT/prof_$m -name "*kernel_stats.csv" -exec cp {} $P/kernel_stats_$m.csv \;
            cp $OUT/prof_$m.log $P/prof_stats_$m.log
            cut -d, -f1-5 $P/kernel_stats_$m.csv | head -25;;
        ktrace|ktrace_*)
            # kernel trace (start / end per dispatch) and the idle gaps between dependent launches
            m=${step#ktrace}; m=${m#_}; m=${m:-track}
            run ktrace_$m 500 rocprofv3 --kernel-trace -f csv -d $OUT/ktrace_$m -o kt -- python3 bench.py $(modeargs $m) --steps 20 --warmup 4 --no-cpu-baseline
            f=$(find $OUT/ktrace_$m -name "*kernel_trace.csv" | head -1)
            python tools/trace_gaps.py $f > $P/trace_gaps_$m.txt; cp $f $P/kernel_trace_$m.csv; cat $P/trace_gaps_$m.txt;;
        pmc|pmc_*)
            m=${step#pmc}; m=${m#_}; m=${m:-track}
            run pmc_fetch_$m 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc_fetch_$m -o fetch -- python3 bench.py $(modeargs $m) --steps 20 --warmup 4 --no-cpu-baseline
            run pmc_write_$m 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_write_$m -o write -- python3 bench.py $(modeargs $m) --steps 20 --warmup 4 --no-cpu-baseline
            cfg=$(python bench.py $(modeargs $m) --print-traffic-config)
            python tools/pmc_traffic.py $OUT/pmc_fetch_$m $OUT/pmc_write_$m $P/traffic_$m.json "$cfg" && head -40 $P/traffic_$m.json;;
        native|native_async)
            a=${step#native}; a=${a#_}
            run native_probe$a 300 python tools/native_probe.py 200 $a; cat $OUT/native_probe$a.log;;
        nativeprof|nativeprof_async)
            a=${step#nativeprof}; a=${a#_}
            run native_prof$a 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/native_prof$a -o np -- python3 tools/native_probe.py 200 $a
            find $OUT/native_prof$a -name "*kernel_stats.csv" -exec cp {} $P/native${a}_kernel_stats.csv \;
            cut -d, -f1-5 $P/native${a}_kernel_stats.csv | head -30;;
        concur)
            # tools/concur_breakdown.py: the concurrent native loop's outcomes per regime, 3 runs each
            run concur 300 python tools/concur_breakdown.py 3; grep -v "^{" $OUT/concur.log | tee $P/concur_breakdown.txt; tail -1 $OUT/concur.log > $P/concur_breakdown.json;;
        lmprobe)
            run lmprobe 300 python tools/lm_chain_probe.py 20; tail -14 $OUT/lmprobe.log;;
        solvetrace|solvetrace=*)
            # per-step cycle split of the reduced-system solve (tools/ubench/solve_trace, built beforehand)
            v=${step#solvetrace}; v=${v#=}
            run solvetrace$v 60 env $v ./tools/ubench/solve_trace 20; cat $OUT/solvetrace$v.log;;
        solvebin=*)
            # a solve_trace build variant: solvebin=NAME runs tools/ubench/solve_trace_NAME
            b=${step#solvebin=}
            run solvebin_$b 60 ./tools/ubench/solve_trace_$b 20; cat $OUT/solvebin_$b.log;;
        solvepmc|solvepmc=*)
            # SQ counters of the reduced-system solve (tools/ubench/solve_trace), one pass
            v=${step#solvepmc}; v=${v#=}
            run solvepmc$v 90 env $v timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace -f csv -d $OUT/solvepmc$v -o sp -- ./tools/ubench/solve_trace 20
            f=$(find $OUT/solvepmc$v -name "*counter_collection.csv" | head -1); cp $f $P/solve_pmc$v.csv
            python3 -c "import csv,collections,sys; d=collections.defaultdict(list); [d[(r['Kernel_Name'][:40],r['Counter_Name'])].append(float(r['Counter_Value'])) for r in csv.DictReader(open(sys.argv[1]))]; [print(k, sum(v)/len(v)) for k,v in sorted(d.items())]" $f;;
        sqpmc|sqpmc_*)
            # two passes of 8 SQ counters over a short bench run -> per-kernel means (tools/pmc_sq.py)
            m=${step#sqpmc}; m=${m#_}; m=${m:-track}
            P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
            P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE"
            run sqpmc1_$m 150 timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -f csv -d $OUT/sqpmc_$m/p1 -o p1 -- python3 bench.py $(modeargs $m) --steps 20 --warmup 4 --no-cpu-baseline
            run sqpmc2_$m 150 timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -f csv -d $OUT/sqpmc_$m/p2 -o p2 -- python3 bench.py $(modeargs $m) --steps 20 --warmup 4 --no-cpu-baseline
            python tools/pmc_sq.py $OUT/sqpmc_$m > $P/sq_counters_$m.txt; head -60 $P/sq_counters_$m.txt;;
        poselat|poselat=*)
            # PoseOptimization latency probe (tools/pose_latency.py); poselat=LIB runs it on another build
            l=${step#poselat}; l=${l#=}
            if [ -n "$l" ]; then n=$(basename $l .so); ORBMI_LIB=$l run poselat_$n 120 python tools/pose_latency.py; cat $OUT/poselat_$n.log
            else run poselat 120 python tools/pose_latency.py; cat $OUT/poselat.log; fi;;
        greedy|greedy=*)
            # k_greedy statistics and phase cycles (tools/greedy_probe.py); greedy=LIB on another build
            l=${step#greedy}; l=${l#=}
            if [ -n "$l" ]; then n=$(basename $l .so); ORBMI_LIB=$l run greedy_$n 120 python tools/greedy_probe.py 64; cat $OUT/greedy_$n.log
            else run greedy 120 python tools/greedy_probe.py 64; cat $OUT/greedy.log; fi;;
        mfma_pmc)
            # MFMA A/B of the Schur products: MFMA issue / busy counters of each variant's kernel
            run mfma_pmc 90 timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -f csv -d $OUT/mfma_pmc -o mfma -- ./tools/ubench/mfma_schur
            find $OUT/mfma_pmc -name "*counter_collection.csv" -exec cp {} $P/mfma_schur_pmc.csv \;
            cp $OUT/mfma_pmc.log $P/mfma_schur_pmc.log; tail -12 $OUT/mfma_pmc.log;;
        envab=*)
            # default bench with / without an environment knob (VAR=VALUE), 3 alternations
            kv=${step#envab=}
            for i in 1 2 3; do
                run envab_A$i 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
                run envab_B$i 300 env $kv python bench.py --steps 100 --warmup 10 --no-cpu-baseline
                echo "default $(tail -1 $OUT/envab_A$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d.get("pcie_inclusive", {}).get("value"), d["phase_ms_per_frame"])')  $kv $(tail -1 $OUT/envab_B$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d.get("pcie_inclusive", {}).get("value"), d["phase_ms_per_frame"])')" | tee -a $OUT/envab.txt
            done;;
        envbatch=*)
            # config 5 (batch mode): default against an environment knob (VAR=VALUE), 3 alternations
            kv=${step#envbatch=}
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d.get("stage_ms_per_launch"))'; }
            for i in 1 2 3; do
                run envb_A$i 300 python bench.py --mode batch --steps 50 --warmup 4 --no-cpu-baseline
                run envb_B$i 300 env $kv python bench.py --mode batch --steps 50 --warmup 4 --no-cpu-baseline
                echo "default $(v envb_A$i) | $kv $(v envb_B$i)" | tee -a $OUT/envbatch.txt
            done;;
        abbatch=*)
            # config-5 (batch mode) A/B of two library builds, 3 alternations, stage times kept
            pair=${step#abbatch=}; A=${pair%,*}; B=${pair#*,}
            for i in 1 2 3; do
                ORBMI_LIB=$A run abb_A$i 300 python bench.py --mode batch --steps 50 --warmup 4 --no-cpu-baseline
                ORBMI_LIB=$B run abb_B$i 300 python bench.py --mode batch --steps 50 --warmup 4 --no-cpu-baseline
                echo "A $(tail -1 $OUT/abb_A$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d.get("stage_ms_per_launch") or d.get("stage_ms_per_step"))')  B $(tail -1 $OUT/abb_B$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d.get("stage_ms_per_launch") or d.get("stage_ms_per_step"))')" | tee -a $OUT/abbatch.txt
            done;;
        ab=*)
            pair=${step#ab=}; A=${pair%,*}; B=${pair#*,}
            for i in 1 2 3; do
                ORBMI_LIB=$A run ab_A$i 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
                ORBMI_LIB=$B run ab_B$i 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
                echo "A $(tail -1 $OUT/ab_A$i.log | python -c 'import json,sys; print(json.load(sys.stdin)["value"])')  B $(tail -1 $OUT/ab_B$i.log | python -c 'import json,sys; print(json.load(sys.stdin)["value"])')" | tee -a $OUT/ab.txt
            done;;
        absys=*)
            # native loop (bench --mode system) A/B/... over library builds (absys=LIB1,LIB2,...), 3 rounds:
            # frames/s, ATE, per-frame phases and the LocalMapping job split per keyframe
            libs=${step#absys=}
            for i in 1 2 3; do
                for l in ${libs//,/ }; do
                    n=$(basename $l .so)
                    ORBMI_LIB=$l run absys_${n}_$i 300 python bench.py --mode system --no-cpu-baseline
                    echo "$n $(tail -1 $OUT/absys_${n}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ate_rmse_m"], d["phase_ms_per_frame"]["total"], d["local_mapping_ms_per_keyframe"], d["synchronous_local_mapping"]["frames_per_s"])')" | tee -a $OUT/absys.txt
                done
            done;;
        ablba=*)
            # LocalBA (config 3) A/B/... over library builds: ablba=LIB1,LIB2,... alternating, 3 rounds
            libs=${step#ablba=}
            for i in 1 2 3; do
                for l in ${libs//,/ }; do
                    n=$(basename $l .so)
                    ORBMI_LIB=$l run ablba_${n}_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                    echo "$n $(tail -1 $OUT/ablba_${n}_$i.log | python -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')" | tee -a $OUT/ablba.txt
                done
            done;;
        mfmatrace|mfmatrace=*)
            # per-panel split of the MFMA reduced-system solve (tools/ubench/mfma_solve_trace, built
            # beforehand) and the VALU pivot-wave solve on the same system
            np_=${step#mfmatrace}; np_=${np_#=}; np_=${np_:-20}
            run mfmatrace$np_ 60 ./tools/ubench/mfma_solve_trace $np_; cat $OUT/mfmatrace$np_.log
            PIPE=1 run mfmatrace_pipe$np_ 60 ./tools/ubench/mfma_solve_trace $np_; cat $OUT/mfmatrace_pipe$np_.log
            cat $OUT/mfmatrace$np_.log $OUT/mfmatrace_pipe$np_.log > $P/mfma_solve_trace_np$np_.txt;;
        ubench=*)
            # a microbenchmark binary under tools/ubench (built beforehand)
            b=${step#ubench=}
            run ubench_$b 60 ./tools/ubench/$b; cat $OUT/ubench_$b.log; cp $OUT/ubench_$b.log $P/;;
        fetchcal)
            # FETCH_SIZE / WRITE_SIZE per load / store width (tools/ubench/fetch_calib, built beforehand)
            run fetchcal_f 90 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetchcal_f -o f -- ./tools/ubench/fetch_calib
            run fetchcal_w 90 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/fetchcal_w -o w -- ./tools/ubench/fetch_calib
            python3 tools/fetch_calib_report.py $OUT/fetchcal_f $OUT/fetchcal_w | tee $P/fetch_calibration.txt;;
        lbasolve)
            # config 3: the MFMA solve fused with the Schur complement, the MFMA solve alone, the
            # VALU pivot-wave solve
            ms() { tail -1 $OUT/$1.log | python -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])'; }
            for i in 1 2 3; do
                ORBMI_BA_SOLVE=mfma ORBMI_BA_FUSE=1 run lbasolve_fused_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                ORBMI_BA_SOLVE=mfma run lbasolve_mfma_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                ORBMI_BA_SOLVE=pipe run lbasolve_pipe_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                echo "fused $(ms lbasolve_fused_$i)  mfma $(ms lbasolve_mfma_$i)  pipe $(ms lbasolve_pipe_$i)" | tee -a $OUT/lbasolve.txt
            done; cp $OUT/lbasolve.txt $P/;;
        mfmapmc|mfmapmc_*)
            # MFMA issue / busy counters per kernel over a short bench run (one pass)
            m=${step#mfmapmc}; m=${m#_}; m=${m:-lba}
            run mfmapmc_$m 150 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -f csv -d $OUT/mfmapmc_$m -o mp -- python3 bench.py $(modeargs $m) --steps 10 --warmup 2 --no-cpu-baseline
            f=$(find $OUT/mfmapmc_$m -name "*counter_collection.csv" | head -1); cp $f $P/mfma_pmc_$m.csv
            python3 -c "import csv,collections,sys; d=collections.defaultdict(list); [d[(r['Kernel_Name'][:48],r['Counter_Name'])].append(float(r['Counter_Value'])) for r in csv.DictReader(open(sys.argv[1]))]; [print(k, len(v), sum(v)/len(v)) for k,v in sorted(d.items()) if 'ba_' in k[0]]" $f | tee $P/mfma_pmc_$m.txt;;
        concur)
            # the concurrent-LocalMapping test three times on the device-resident tracking path and
            # three times on the staged one (ORBMI_SLAM_STAGED=1), ATE lines collected
            for i in 1 2 3; do
                run concur_dev_$i 200 python -u -m pytest -x -q -s -m gpu --timeout 150 --timeout-method thread tests/test_native_slam_gpu.py -k test_native_concurrent_local_mapping
                ORBMI_SLAM_STAGED=1 run concur_staged_$i 200 python -u -m pytest -x -q -s -m gpu --timeout 150 --timeout-method thread tests/test_native_slam_gpu.py -k test_native_concurrent_local_mapping
                echo "dev: $(grep -o 'ATE [0-9.]* m (synchronous [0-9.]* m)' $OUT/concur_dev_$i.log)  staged: $(grep -o 'ATE [0-9.]* m (synchronous [0-9.]* m)' $OUT/concur_staged_$i.log)" | tee -a $OUT/concur.txt
            done;;
        concurbd)
            # tools/concur_breakdown.py: the concurrent LocalMapping's accuracy per regime (back to
            # back, back to back without InterruptBA, paced), 3 runs each
            run concurbd 600 python -u tools/concur_breakdown.py 3; grep -v "^{" $OUT/concurbd.log | tee $P/concur_breakdown.txt
            tail -1 $OUT/concurbd.log > $P/concur_breakdown.json;;
        concurprobe|concurprobe=*)
            # concurprobe=MS: frames paced MS apart (stereo_kitti.cc's timestamp wait)
            ms=${step#concurprobe}; ms=${ms#=}; ms=${ms:-0}
            run concurprobe$ms 300 python -u tools/concur_probe.py 2 $ms; grep -v "^   frame" $OUT/concurprobe$ms.log;;
        prio)
            # native loop (bench --mode system): the default stream priorities (Tracking high,
            # LocalMapping low) against all streams at the device default, 3 alternations
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["phase_ms_per_frame"]["local_search"], d["phase_ms_per_frame"]["frame_ctor"], d["ate_rmse_m"])'; }
            for i in 1 2 3; do
                run prio_hl_$i 300 python bench.py --mode system --no-cpu-baseline
                ORBMI_PRIO_LM=default ORBMI_PRIO_MATCHER=default ORBMI_PRIO_POSE=default ORBMI_PRIO_EXTRACTOR=default run prio_flat_$i 300 python bench.py --mode system --no-cpu-baseline
                echo "tracking high / LM low: $(v prio_hl_$i) | all default: $(v prio_flat_$i)" | tee -a $OUT/prio.txt
            done;;
        schurxcd)
            # LocalBA (config 3): Schur blocks grouped by row onto one XCD (default) vs row-major,
            # 3 alternations, plus FETCH_SIZE of each layout
            ms() { tail -1 $OUT/$1.log | python -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])'; }
            for i in 1 2 3; do
                run sx_xcd_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                ORBMI_BA_SCHUR_ROWMAJOR=1 run sx_row_$i 200 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline
                echo "xcd rows $(ms sx_xcd_$i)  row-major $(ms sx_row_$i)" | tee -a $OUT/schurxcd.txt
            done
            run sx_fetch_xcd 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/sx_fetch_xcd -o f -- python3 bench.py --mode lba --steps 10 --warmup 2 --no-cpu-baseline
            ORBMI_BA_SCHUR_ROWMAJOR=1 run sx_fetch_row 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/sx_fetch_row -o f -- python3 bench.py --mode lba --steps 10 --warmup 2 --no-cpu-baseline
            for v in xcd row; do
                f=$(find $OUT/sx_fetch_$v -name "*counter_collection.csv" | head -1)
                python3 -c "import csv,collections,sys; d=collections.defaultdict(list); [d[r['Kernel_Name'][:40]].append(float(r['Counter_Value'])) for r in csv.DictReader(open(sys.argv[1])) if r['Counter_Name']=='FETCH_SIZE']; [print(sys.argv[2], k, len(v), round(2*sum(v)/len(v)/1024,3), 'MB (2 x FETCH_SIZE)') for k,v in sorted(d.items()) if 'ba_' in k]" $f $v | tee -a $OUT/schurxcd.txt
            done
            cp $OUT/schurxcd.txt $P/;;
        descab)
            # config 5 batch: the four-keypoints-per-wave describe (default) vs one keypoint per
            # wave (ORBMI_DESC=wave), 2 alternations
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["stage_ms_per_launch"])'; }
            for i in 1 2; do
                run descab_4_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                ORBMI_DESC=wave run descab_w_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                echo "4/wave: $(v descab_4_$i) | 1/wave: $(v descab_w_$i)" | tee -a $OUT/descab.txt
            done; cp $OUT/descab.txt $P/;;
        octtrace)
            # k_octree phase trace of every level (tools/octree_trace, built in-tree on the CPU) on a
            # config-5 frame (synthetic EuRoC-shaped 752x480, 5000 features)
            python -c "import numpy as np; from orb_slam2_with_comment_amd import synth; np.ascontiguousarray(synth.mono(synth.EUROC, 0, seed_base=5000), np.uint8).tofile('$OUT/euroc0.u8')"
            run octtrace 120 ./tools/octree_trace $OUT/euroc0.u8 480 752 5000; cp $OUT/octtrace.log $P/octree_trace_levels.txt
            grep -E "== level|total" $OUT/octtrace.log;;
        octab)
            # the octree phase trace of every level on a KITTI-shaped left image (2000 features), this
            # tree's kernel against tools/octree_trace_old (another build of the trace tool)
            python -c "import numpy as np; from orb_slam2_with_comment_amd import synth; np.ascontiguousarray(synth.stereo_pair(synth.KITTI, 0)[0], np.uint8).tofile('$OUT/kitti0.u8')"
            run octab_new 120 ./tools/octree_trace $OUT/kitti0.u8 376 1241 2000 && run octab_old 120 ./tools/octree_trace_old $OUT/kitti0.u8 376 1241 2000
            for v in new old; do echo "== $v"; grep -E "== level|total" $OUT/octab_$v.log; done | tee $P/octree_ab_kitti.txt;;
        fastab)
            # config 5 batch: k_fast2 with the one-pass arc strength (default) vs its separate
            # segment-test and score stages (ORBMI_FAST=split), 3 alternations
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["stage_ms_per_launch"]["fast"])'; }
            for i in 1 2 3; do
                run fastab_s_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                ORBMI_FAST=split run fastab_p_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                echo "one pass: $(v fastab_s_$i) | split: $(v fastab_p_$i)" | tee -a $OUT/fastab.txt
            done; cp $OUT/fastab.txt $P/;;
        fastseg)
            # config 5 batch: k_fast2's arc-test split (ORBMI_FAST_SEG=0 scalar, 1 per lane, 2 mixed)
            # and the per-lane k_fast (ORBMI_FAST=v1), 2 alternations
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["stage_ms_per_launch"]["fast"])'; }
            for i in 1 2; do
                for sg in 0 1 2; do
                    ORBMI_FAST_SEG=$sg run fastseg_${sg}_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                    echo "seg $sg: $(v fastseg_${sg}_$i)" | tee -a $OUT/fastseg.txt
                done
                ORBMI_FAST=v1 run fastseg_v1_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                echo "v1: $(v fastseg_v1_$i)" | tee -a $OUT/fastseg.txt
            done; cp $OUT/fastseg.txt $P/;;
        blurab)
            # config 5 batch: GaussianBlur on a side stream (default) / inside the octree launch / after it
            v() { tail -1 $OUT/$1.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])'; }
            for i in 1 2; do
                for m in side fused serial; do
                    ORBMI_BLUR=$m run blurab_${m}_$i 300 python bench.py --mode batch --steps 20 --warmup 4 --no-cpu-baseline
                    echo "$m: $(v blurab_${m}_$i)" | tee -a $OUT/blurab.txt
                done
            done; cp $OUT/blurab.txt $P/;;
        profenv=*)
            # rocprofv3 kernel stats of --mode lba under an environment setting: profenv=VAR=VALUE
            kv=${step#profenv=}; tag=$(echo $kv | tr '=' '_')
            env $kv timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/profenv_$tag -o stats -- python3 bench.py --mode lba --steps 20 --warmup 4 --no-cpu-baseline > $OUT/profenv_$tag.log 2>&1
            echo "profenv_$tag exit $?" | tee -a $OUT/status.txt
            f=$(find $OUT/profenv_$tag -name "*kernel_stats.csv" | head -1); echo "== $kv"; cut -d, -f1-4 $f | grep "k_ba_s\|k_ba_u";;
        *) echo "unknown step $step"; exit 2;;
    esac
done
