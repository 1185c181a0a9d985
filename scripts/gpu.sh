#!/bin/bash
# One parameterised GPU job runner (replaces the per-experiment gpu_job_*.sh files of rounds 1-3; git history keeps
# them). Every step runs under its own time limit and the steps of one call are chained with &&: a failing, aborted
# or timed-out step ends the call.
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps (outputs under gpurun_out/TAG/):
#   smoke                 __graft_entry__.smoke()
#   tests[=PATHS]         pytest -m gpu (one process, 120 s per test)
#   bench                 headline bench.py at the driver's setting (20 steps) x3 + 400 steps
#   configs[=NAMES]       scripts/bench_configs.py (default breakout_ppo,mujoco_ppo_dp8)
#   trace=NAME            rocprofv3 kernel trace + per-update summary; NAME in pong | breakout | mujoco
#   pmc=NAME              rocprofv3 PMC passes (SQ counters; FETCH_SIZE) + roofline table; NAME in pong | breakout | mujoco
#   cmd=FILE              bash FILE (a one-off experiment kept in the tree)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
PONG="python3 bench.py --steps 40 --warmup 5"
BR="python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1"
MJ="python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 2 --warmup 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"

prog() {   # NAME -> program, trace marker, kernels per update, updates summarised
  case $1 in
    pong) echo "pong_fused_step 5 30 $PONG" ;;
    breakout) echo "pong_fused_env_step 128 1 $BR" ;;
    mujoco) echo "mlp_rollout 1 1 $MJ" ;;
    *) echo "unknown program $1" >&2; return 1 ;;
  esac
}

step() {
  local s=$1 arg=
  [[ $s == *=* ]] && { arg=${s#*=}; s=${s%%=*}; }
  case $s in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        && tail -1 $O/smoke.log || { tail -5 $O/smoke.log; return 1; } ;;
    tests)
      python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || return 3
      timeout -k 10 1000 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
        > $O/tests.log 2>&1
      local rc=$?
      grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error" $O/tests.log | head -20
      return $rc ;;
    bench)
      for i in 1 2 3; do
        timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err \
          || { tail -5 $O/bench_$i.err; return 1; }
        echo "bench20 $i: $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d['ms_per_step'])")"
      done
      timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench_400.json 2> $O/bench_400.err \
        || { tail -5 $O/bench_400.err; return 1; }
      echo "bench400: $(python3 -c "import json;d=json.load(open('$O/bench_400.json'));print(d['value'], d['ms_per_step'])")" ;;
    configs)
      timeout -k 10 400 python -u scripts/bench_configs.py --configs ${arg:-breakout_ppo,mujoco_ppo_dp8} --updates 5 \
        --warmup 2 >> $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; return 1; }
      cat $O/configs.jsonl ;;
    trace)
      local p; p=($(prog $arg)) || return 1
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$arg -o run -- "${p[@]:3}" \
        > $O/tr_$arg.log 2>&1 || { tail -5 $O/tr_$arg.log; return 1; }
      python3 scripts/trace_summary.py $(find $O/tr_$arg -name "*kernel_trace.csv") --updates ${p[2]} \
        --marker ${p[0]} --per-update ${p[1]} > $O/${arg}_trace_summary.txt && head -40 $O/${arg}_trace_summary.txt
      find $O/tr_$arg -name "*.csv" -size +6M -delete ;;
    pmc)
      local p; p=($(prog $arg)) || return 1
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $SQ -d $O/pmc_${arg}_sq -o run -- \
        "${p[@]:3}" > $O/pmc_${arg}_sq.log 2>&1 || { tail -5 $O/pmc_${arg}_sq.log; return 1; }
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
        -d $O/pmc_${arg}_fetch -o run -- "${p[@]:3}" > $O/pmc_${arg}_fetch.log 2>&1 \
        || { tail -5 $O/pmc_${arg}_fetch.log; return 1; }
      # WRITE_SIZE takes 2 of the 4 TCC counters of a pass, the L2 hit / miss sums the other two
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum \
        -d $O/pmc_${arg}_write -o run -- "${p[@]:3}" > $O/pmc_${arg}_write.log 2>&1 \
        || { tail -5 $O/pmc_${arg}_write.log; return 1; }
      python3 scripts/pmc_table.py --last 4 $(find $O/pmc_${arg}_sq $O/pmc_${arg}_fetch $O/pmc_${arg}_write \
        -name "*counter_collection.csv") \
        > $O/${arg}_pmc.txt && head -40 $O/${arg}_pmc.txt
      find $O -name "*.csv" -size +8M -delete ;;
    cmd)
      timeout -k 10 900 bash $arg > $O/cmd.log 2>&1; local rc=$?; tail -40 $O/cmd.log; return $rc ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  step "$s" || { echo "step $s failed ($?)"; exit 1; }
done
