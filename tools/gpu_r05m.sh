# round 5: phase stamps after the sweep rewrite (configs[2] and configs[1])
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
L=hopper-mpc-inertial_amd/libhmpc_stamps.so
HMPC_LIB=$L timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_3f_B65536.json 2> $O/s1.err || { echo "stamps 3f failed"; exit 1; }
HMPC_LIB=$L VARIANT=2f STRAIGHT=1 B=4096 timeout -k 10 180 python tools/phase_stamps.py > $O/stamps_2f_B4096.json 2> $O/s2.err || { echo "stamps 2f failed"; exit 1; }
echo stamps ok
