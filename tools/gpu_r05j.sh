# round 5: what the Riccati bucket pass spends its 9.6 us on (probe builds:
# bk1 = no C reads, bk2 = 1024-thread blocks), then the Runner's latency with
# the bucket pass skipped at B <= resident workgroups
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r05j
mkdir -p $O
for lib in libhmpc.so libhmpc_ab_bk1.so libhmpc_ab_bk2.so; do
  (cd /tmp && HMPC_LIB=$R/hopper-mpc-inertial_amd/$lib TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/$lib -o run -- \
    python3 $R/bench.py --N 60 --straight --batch 4096 --steps 20 --cpu-seconds 0 > $R/$O/$lib.log 2>&1) || { echo "$lib trace failed"; exit 1; }
  echo "$lib $(grep -h buckets $O/$lib/run_kernel_stats.csv | cut -d, -f2-4)"
done
timeout -k 10 300 python tools/runner_time.py graph > $O/runner_graph.json 2> $O/runner.err || { echo "runner failed"; exit 1; }
tail -30 $O/runner_graph.json
