set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_policy.log 2>&1; echo "pytest rc=$?"
tail -3 $O/pytest_policy.log
PROBE_STAMPS=1 timeout -k 10 120 python tools/probe_policy.py > $O/policy_stamps.log 2>&1 &&
PROBE_N=4096 timeout -k 10 120 python tools/probe_policy.py > $O/probe_policy.log 2>&1
echo "rc=$?"; cat $O/policy_stamps.log $O/probe_policy.log | grep -v amdgpu.ids
