# Riccati phase stamps (N=20, N=60) and the bench's RCCL path at world size 1
set -o pipefail
mkdir -p gpurun_out/rs
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python tools/ric_stamps.py 3f 20 65536 1 > gpurun_out/rs/n20.json 2> gpurun_out/rs/n20.err || { echo STAMPS20 FAILED; tail gpurun_out/rs/n20.err; exit 1; }
HMPC_LIB=hopper-mpc-inertial_amd/libhmpc_stamps.so timeout -k 10 200 python tools/ric_stamps.py 3f 60 4096 > gpurun_out/rs/n60.json 2> gpurun_out/rs/n60.err || { echo STAMPS60 FAILED; tail gpurun_out/rs/n60.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/rs/dist1.json 2> gpurun_out/rs/dist1.err || { echo DIST FAILED; tail -20 gpurun_out/rs/dist1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/rs/dist1.json')); print(d['value'], d['dist'])"
