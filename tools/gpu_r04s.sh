set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_architect_update.py tests/test_gpu_policy.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python -u tools/probe_arch_update.py > $O/probe_arch.log 2>&1; echo "probe rc=$?"
PROBE_STAMPS=1 timeout -k 10 120 python tools/probe_policy.py > $O/policy_stamps.log 2>&1 &&
PROBE_N=4096 timeout -k 10 120 python tools/probe_policy.py > $O/probe_policy.log 2>&1 &&
timeout -k 10 300 python tools/probe_train.py > $O/probe_train.log 2>&1
echo "rc=$?"
