# round 5 probe: the cost of the dense split's early-exit workgroups
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r05v
mkdir -p $O
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/trace -o run -- python3 $R/tools/empty_dispatch.py > $R/$O/empty.log 2>&1) || { echo "probe failed"; tail -5 $O/empty.log; exit 1; }
grep "all-swing" $O/empty.log
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05v/trace/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1000, 2), 'us')
PY
