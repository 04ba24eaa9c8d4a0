#!/bin/bash
# One GPU call made of named steps, each under its own time limit; the call
# stops at the first failing step (no retries, nothing more on the GPU after
# a crash, an abort or a time limit).  Replaces the per-round one-off scripts.
#
#   gpurun -- bash tools/gpu_steps.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/.  Steps (arguments after ':'; spaces
# inside an argument list are written as ','):
#   tests                       the whole -m gpu suite
#   tests:FILE,FILE             those test files only
#   bench:TAG:ARGS              bench.py ARGS > OUT/bench_TAG.json
#   trace:TAG:ARGS              rocprofv3 --kernel-trace --stats of bench.py ARGS
#   runner                      tools/runner_time.py, eager and graph replay
#   runnertrace                 rocprofv3 kernel trace of one robot's run (graph replay)
#   stamps:TAG:LIB:ENV          tools/phase_stamps.py with HMPC_LIB=LIB and ENV
#                               (NAME=VALUE pairs)
#   ricstamps:TAG:LIB:ARGS      tools/ric_stamps.py ARGS with HMPC_LIB=LIB
#   ab:TAG:ARGS:LIB,LIB         tools/ab.py interleaved A/B (3 rounds)
#   profile:TAG                 tools/profile.sh TAG (all configurations)
#   waits:TAG:CFG:ARGS          tools/wait_pmc.sh (latency decomposition)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
stop() { case $1 in 124|134|137|139) echo "GPU step died ($1): stopping"; exit 1;; esac; }
sp() { echo "${1//,/ }"; }
for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  cd $R
  case $kind in
    tests)
      files=${a1:+$(sp $a1)}
      timeout -k 10 900 python -u -m pytest ${files:-tests -m gpu} -x -q --timeout 120 --timeout-method thread \
        > $OUT/tests.log 2>&1; rc=$?
      tail -2 $OUT/tests.log; stop $rc; [ $rc -eq 0 ] || exit 1 ;;
    bench)
      timeout -k 10 400 python bench.py $(sp $a2) > $OUT/bench_$a1.json 2> $OUT/bench_$a1.err; rc=$?
      stop $rc; [ $rc -eq 0 ] || { echo "bench $a1 failed"; tail -5 $OUT/bench_$a1.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,3), 'M/s', d['ms_per_step'], 'ms', (d.get('parity_sample') or {}).get('max_abs_du_vs_port'))" \
        $OUT/bench_$a1.json $a1 ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$a1 -o run -- \
        python3 $R/bench.py $(sp $a2) --cpu-seconds 0 > $OUT/trace_$a1.log 2>&1); rc=$?
      stop $rc; [ $rc -eq 0 ] || { echo "trace $a1 failed"; exit 1; }
      find $OUT/trace_$a1 -name "*kernel_stats.csv" -exec cut -d, -f1-5 {} \; | head -12 ;;
    runner)
      timeout -k 10 300 python tools/runner_time.py > $OUT/runner_eager.json 2>&1 || { echo "runner eager failed"; exit 1; }
      timeout -k 10 300 python tools/runner_time.py graph > $OUT/runner_graph.json 2>&1 || { echo "runner graph failed"; exit 1; }
      tail -c 400 $OUT/runner_graph.json; echo ;;
    runnertrace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/runnertrace -o run -- \
        python3 $R/tools/runner_time.py graph ${RUNNER_B:-1} > $OUT/runnertrace.log 2>&1); rc=$?
      stop $rc; [ $rc -eq 0 ] || { echo "runnertrace failed"; exit 1; }
      find $OUT/runnertrace -name "*kernel_stats.csv" -exec cut -d, -f1-5 {} \; | head -14 ;;
    stamps)
      envs=$(sp $a3)
      env HMPC_LIB=hopper-mpc-inertial_amd/$a2 $envs timeout -k 10 180 python tools/phase_stamps.py \
        > $OUT/stamps_$a1.json 2> $OUT/stamps_$a1.err || { echo "stamps $a1 failed"; exit 1; } ;;
    ricstamps)
      HMPC_LIB=hopper-mpc-inertial_amd/$a2 timeout -k 10 200 python tools/ric_stamps.py $(sp $a3) \
        > $OUT/ricstamps_$a1.json 2> $OUT/ricstamps_$a1.err || { echo "ricstamps $a1 failed"; tail -3 $OUT/ricstamps_$a1.err; exit 1; }
      cat $OUT/ricstamps_$a1.json ;;
    ab)
      timeout -k 10 1000 python tools/ab.py --tag $a1 --rounds ${ROUNDS:-3} --args "$(sp $a2)" $(sp $a3) \
        > $OUT/ab_$a1.log 2>&1; rc=$?
      stop $rc; [ $rc -eq 0 ] || { echo "ab $a1 failed"; tail -5 $OUT/ab_$a1.log; exit 1; }
      tail -4 $OUT/ab_$a1.log ;;
    profile)
      bash tools/profile.sh $a1 || exit 1 ;;
    waits)
      bash tools/wait_pmc.sh $a1 $a2 $(sp $a3) || exit 1 ;;
    *)
      echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "steps done"
