# round 5: GPU suite (buckets kernel rewrite), the buckets kernel's time at
# N = 60 B = 4096, and phase stamps of configs[1] (2f straight B = 4096)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/n60 -o run -- \
  python3 $R/bench.py --N 60 --straight --batch 4096 --steps 10 --cpu-seconds 0 > $R/$O/n60.log 2>&1) || { echo "n60 trace failed"; exit 1; }
grep -h buckets $O/n60/*/run_kernel_stats.csv $O/n60/run_kernel_stats.csv 2>/dev/null | cut -d, -f1-4
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so VARIANT=2f STRAIGHT=1 B=4096 timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_2f_B4096.json 2> $O/stamps_2f.err || { echo "stamps failed"; exit 1; }
echo "stamps ok"
