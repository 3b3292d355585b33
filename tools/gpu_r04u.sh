set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-r04u}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_architect_update.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/pytest_arch.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed|vs eager" $O/pytest_arch.log
timeout -k 10 300 python -u tools/probe_arch_update.py > $O/probe_arch.log 2>&1; echo "probe rc=$?"
head -2 $O/probe_arch.log; grep -A31 "wg0 step" $O/probe_arch.log
