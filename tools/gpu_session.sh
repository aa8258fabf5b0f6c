#!/bin/bash
# One GPU session, assembled from steps (the reusable A/B driver; replaces round 4's one-off tools/r04_*.sh).
#   STEPS   comma list, run in order (default: suite,ab_c3,latency):
#     suite      the full -m gpu suite on the working tree's library
#     parity     the parity subset only (parity, random parity, rotation, drain, rare channels)
#     ab_c3      C3 (K = 32) with each prebuilt library of LIBS, interleaved twice (tools/ab_libs.sh)
#     stall      two PMC passes per library of LIBS: the SQ wave-cycle split, LDS / branch / fetch counters
#                (STALL_ARGS: bench.py arguments, e.g. "--workload c2"; default the C3 line)
#     rcp        the time step's reciprocal against RN32(1 / b) for every f32 b the stepper divides by (ecdna-evo_amd/bin/rcp_check, tools/rcp_check.hip)
#     latency    C2, C4 rank-0 shard, C5 rank-0 shard with each library (tools/ab_latency.sh)
#     pmc        one SQ-counter pass (VALU / SALU / LDS per wave-event of one C3 step) per library
#     c3s        the C3 fixed-total shards (G = 1, 2, 4, 8; all ranks) with the working tree (tools/c3_strong.py)
#     c3s_knobs  launch knobs on the C3 fixed-total rank-0 shards (G = 2, 4, 8)
#     c4s        the eight C4 8-GPU shards one after another (tools/c4_shards.sh)
#     c4split    the C4 shard split by initial copy number onto two concurrent instances (tools/c4_split.py)
#     prof_bins, prof_rows   tools/gpu_profile.sh ${TAG}_<store> <store>: bench, rocprofv3 kernel trace, PMC passes
#     bench_ref  the C3 line under the reference's own draws (--store rows --draws reference)
#     bench_c3, bench_rows   the metric's line (defaults) and the row store's C3 line
#     smoke      __graft_entry__.smoke()
#     bench_c2, bench_c4, bench_c5   the other workloads' bench lines
#     cyc        loop-section cycle counters (tools/cycle_stats.py) of the configs in CYC (default c3s8,c2,c3) with the
#                -DECDNA_CYCLE_STATS library LIBS names (EXTRA=-DECDNA_CYCLE_STATS bash tools/ab_build.sh WORKTREE <name>)
#     inject     the indexing guard under fault injection (tools/inject_check.py) with the library LIBS names
#                (EXTRA=-DECDNA_INJECT_EMPTY_NPLUS bash tools/ab_build.sh WORKTREE <name>)
#     ab_ref     the reference-draws C3 line with each library of LIBS, interleaved twice (tools/ab_ref.sh)
#     cyc_ref    section cycle counters of the reference-draws stepper (tools/cycle_stats_ref.py c3) with the
#                -DECDNA_CYCLE_STATS library LIBS names
#     c5curve    the C5 rank-0 shards of 8, 4 and 2 GPUs and the whole run (G = 1) at K = 64, one after another
#                (tools/probe_configs.py c5): the same-K strong-scaling curve
#     pmc_ref    SQ counters (two passes) of one C3 step under the reference's own draws (ssa_stepper_refdraws)
#   LIBS    prebuilt libraries ecdna-evo_amd/lib_ab/<name>/ (tools/ab_build.sh <ref|WORKTREE> <name>)
#   TAG     prefix of the outputs under gpurun_out/
# Usage: STEPS=parity,ab_c3 LIBS="base new" TAG=r05x bash tools/gpu_session.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=${STEPS:-suite,ab_c3,latency}
LIBS=${LIBS:-}
TAG=${TAG:-sess}
L=$PWD/ecdna-evo_amd/lib_ab
for step in ${STEPS//,/ }; do
  echo "== $step"
  # (only the A/B steps load prebuilt libraries, which may be of an earlier ABI with the same Params layout; every
  # other step runs the working tree's library under the ABI check)
  case $step in ab_c3|latency|pmc|cyc|inject|ab_ref|cyc_ref) export ECDNA_SSA_ABI_ANY=1 ;; *) unset ECDNA_SSA_ABI_ANY ;; esac
  case $step in
    suite)
      timeout -k 10 700 python3 -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_gpu_suite.txt 2>&1 || { echo SUITE FAILED; tail -40 gpurun_out/${TAG}_gpu_suite.txt; exit 1; }
      tail -1 gpurun_out/${TAG}_gpu_suite.txt ;;
    parity)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py \
        tests/test_gpu_rotation.py tests/test_gpu_drain.py tests/test_gpu_rare_channels.py -q -x --timeout 300 \
        --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/${TAG}_parity.txt; exit 1; }
      tail -1 gpurun_out/${TAG}_parity.txt ;;
    ab_c3)
      bash tools/ab_libs.sh $LIBS 2>&1 | grep "^{" | tee gpurun_out/${TAG}_ab_c3.txt ;;
    latency)
      bash tools/ab_latency.sh $LIBS 2>&1 | tail -$((6 * $(echo $LIBS | wc -w))) | tee gpurun_out/${TAG}_ab_latency.txt ;;
    pmc)
      for n in $LIBS; do
        ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
          SQ_WAVES SQ_BUSY_CYCLES -T --output-format csv -d gpurun_out/${TAG}_pmc_$n -o pmc -- python3 bench.py --steps 1 \
          --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_pmc_$n.log 2>&1
        python3 tools/ab_pmc_summary.py gpurun_out/${TAG}_pmc_$n gpurun_out/${TAG}_pmc_$n.log "$n" | tee -a gpurun_out/${TAG}_pmc.txt
      done ;;
    rcp)
      rc=0; timeout -k 10 120 ecdna-evo_amd/bin/rcp_check > gpurun_out/${TAG}_rcp_check.json || rc=$?
      cat gpurun_out/${TAG}_rcp_check.json; [ $rc -le 1 ] || exit 1 ;;  # (1: mismatches found, reported)
    stall)  # the SQ wave-cycle split (waiting on waitcnt / issue-stalled / issuing) and the LDS, branch and fetch counters
      for n in $LIBS; do
        k=0
        for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
                    "SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAVES" \
                    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_WAVES"; do
          k=$((k + 1))
          ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -s KILL 300 rocprofv3 --pmc $pass -T --output-format csv \
            -d gpurun_out/${TAG}_stall_${n}_$k -o pmc -- python3 bench.py ${STALL_ARGS:-} --steps 1 --warmup 0 --no-cpu-baseline \
            > gpurun_out/${TAG}_stall_${n}_$k.log 2>&1
          python3 tools/ab_pmc_summary.py gpurun_out/${TAG}_stall_${n}_$k gpurun_out/${TAG}_stall_${n}_$k.log "$n" all \
            | tee -a gpurun_out/${TAG}_stall.txt
        done
      done ;;
    c3s)
      timeout -k 10 300 python3 -u tools/c3_strong.py > gpurun_out/${TAG}_c3_strong.jsonl 2> gpurun_out/${TAG}_c3_strong.err
      grep makespan gpurun_out/${TAG}_c3_strong.jsonl ;;
    c3s_knobs)
      O=gpurun_out/${TAG}_c3_strong_knobs.txt; : > $O
      knob() {  # label, env...
        local label=$1; shift
        env "$@" C3S_RANKS=0 C3S_REPS=3 timeout -k 10 200 python3 tools/c3_strong.py 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if 'best_ms' in d: i=d['instance']; print('$label', 'G=%d' % d['gpus'], d['best_ms'], d['stepper_ms'], 'sched', i['schedule'], 'rot', i['rotation'], 'drain', i['drain_control'], 'bpc', i['blocks_per_cu'], 'K', i['bin_kmax'])
" >> $O
      }
      knob auto C3S_GPUS=2,4,8
      knob rot1 C3S_GPUS=2,4 ECDNA_SSA_ROTATE=1
      knob rot1min1 C3S_GPUS=2,4 ECDNA_SSA_ROTATE=1 ECDNA_SSA_ROT_PARK_MIN=1
      knob sched0 C3S_GPUS=2,4,8 ECDNA_SSA_SCHED=0
      knob k64 C3S_GPUS=2,4,8 PROBE_KMAX=64
      knob admit8 C3S_GPUS=2 ECDNA_SSA_ADMIT_X8=8
      cat $O ;;
    c4s)
      bash tools/c4_shards.sh | tee gpurun_out/${TAG}_c4_shards.txt ;;
    c4split)
      timeout -k 10 600 python3 -u tools/c4_split.py > gpurun_out/${TAG}_c4_split.jsonl 2> gpurun_out/${TAG}_c4_split.err
      cut -c1-200 gpurun_out/${TAG}_c4_split.jsonl ;;
    cyc)
      for n in $LIBS; do
        C=${CYC:-c3s8,c2,c3}
        for cfg in ${C//,/ }; do
          ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -k 10 300 python3 tools/cycle_stats.py $cfg | tee -a gpurun_out/${TAG}_cyc.jsonl
        done
      done ;;
    ab_ref)
      bash tools/ab_ref.sh $LIBS | tee gpurun_out/${TAG}_ab_ref.txt ;;
    cyc_ref)
      for n in $LIBS; do
        ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -k 10 300 python3 tools/cycle_stats_ref.py c3 | tee -a gpurun_out/${TAG}_cyc_ref.jsonl
        ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -k 10 300 python3 tools/cycle_stats_ref.py c2 | tee -a gpurun_out/${TAG}_cyc_ref.jsonl
      done ;;
    c5curve)
      for G in 8 4 2 1; do
        PROBE_FLAGS=0x20 PROBE_KMAX=64 PROBE_GPUS=$G timeout -k 10 200 python3 tools/probe_configs.py c5 2>/dev/null | \
          python3 -c "import json,sys; d=json.loads(sys.stdin.read()); i=d['instance']; print('c5 G=$G rank0', round(d['stepper_ms'],1), 'ms', 'replicates', d['replicates'], 'events', d['events'], 'K', i['bin_kmax'], 'paired', i['paired'], 'schedule', i['schedule'], 'errors', d['errors'])" | tee -a gpurun_out/${TAG}_c5curve.txt
      done ;;
    inject)
      for n in $LIBS; do
        ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so timeout -k 10 120 python3 tools/inject_check.py | tee -a gpurun_out/${TAG}_inject.jsonl
      done ;;
    pmc_ref)
      O=gpurun_out/${TAG}_pmc_ref; mkdir -p $O
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
        SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES -T --output-format csv -d $O/p1 -o pmc -- python3 bench.py --store rows \
        --draws reference --steps 1 --warmup 0 --no-cpu-baseline > $O/p1.log 2>&1
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -T --output-format csv -d $O/p2 -o pmc -- python3 bench.py --store rows \
        --draws reference --steps 1 --warmup 0 --no-cpu-baseline > $O/p2.log 2>&1
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/p3 -o pmc -- python3 bench.py --store rows \
        --draws reference --steps 1 --warmup 0 --no-cpu-baseline > $O/p3.log 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/p4 -o pmc -- python3 bench.py --store rows \
        --draws reference --steps 1 --warmup 0 --no-cpu-baseline > $O/p4.log 2>&1
      echo "pmc_ref done" ;;
    prof_bins|prof_rows)
      bash tools/gpu_profile.sh ${TAG}_${step#prof_} ${step#prof_} ;;
    bench_ref)
      timeout -k 10 600 python3 bench.py --store rows --draws reference > gpurun_out/${TAG}_bench_ref_c3.json \
        2> gpurun_out/${TAG}_bench_ref_c3.err
      cut -c1-300 gpurun_out/${TAG}_bench_ref_c3.json ;;
    bench_c3)
      timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err
      cut -c1-300 gpurun_out/${TAG}_bench_c3.json ;;
    bench_rows)
      timeout -k 10 600 python3 bench.py --store rows > gpurun_out/${TAG}_bench_rows_c3.json 2> gpurun_out/${TAG}_bench_rows_c3.err
      cut -c1-300 gpurun_out/${TAG}_bench_rows_c3.json ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
      tail -3 gpurun_out/${TAG}_smoke.txt ;;
    bench_c2|bench_c4|bench_c5)
      timeout -k 10 900 python3 bench.py --workload ${step#bench_} --steps 2 --warmup 1 > gpurun_out/${TAG}_${step}.json \
        2> gpurun_out/${TAG}_${step}.err
      cut -c1-300 gpurun_out/${TAG}_${step}.json ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
