# round 5: the profile suite (all configurations), then the wait decomposition of
# configs[3] (N = 20) and of configs[2] for comparison
set -o pipefail
bash tools/profile.sh r05 || exit 1
bash tools/wait_pmc.sh r05w n20 --N 20 --straight --mu-sweep --global-batch 262144 || exit 1
bash tools/wait_pmc.sh r05w n10 --N 10 || exit 1
