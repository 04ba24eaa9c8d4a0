# round 5 final evidence: the profile suite (every configuration), configs[1]
# stamps (slowest instance), the Runner at 1 / 256 / 4096 robots (eager, graph)
set -o pipefail
bash tools/profile.sh r05 || exit 1
O=gpurun_out/r05q
mkdir -p $O
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so VARIANT=2f STRAIGHT=1 B=4096 timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_2f_B4096.json 2> $O/s2.err || { echo "stamps failed"; exit 1; }
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_3f_B65536.json 2> $O/s1.err || { echo "stamps failed"; exit 1; }
timeout -k 10 300 python tools/runner_time.py > $O/runner_eager.json 2> $O/re.err || { echo "runner failed"; exit 1; }
timeout -k 10 300 python tools/runner_time.py graph > $O/runner_graph.json 2> $O/rg.err || { echo "runner graph failed"; exit 1; }
echo final ok
