set -o pipefail
echo "== concurrent"; timeout -k 10 300 python -u tools/feas_diag.py 2>&1 | grep -v amdgpu.ids | grep "rep\|b "
echo "== nosplit"; HMPC_SPLIT=0 timeout -k 10 300 python -u tools/feas_diag.py 2>&1 | grep -v amdgpu.ids | grep "rep\|b "
