set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_architect_update.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/pytest_arch.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python -u tools/probe_arch_update.py > $O/probe_arch.log 2>&1; echo "probe rc=$?"
PROBE_STAMPS=1 timeout -k 10 120 python tools/probe_policy.py > $O/policy_stamps_default.log 2>&1 &&
HEIST_LIB=$PWD/tools/forensic/_ref/libheist_hip_policy_noslp.so PROBE_STAMPS=1 timeout -k 10 120 python tools/probe_policy.py > $O/policy_stamps_noslp.log 2>&1 &&
PROBE_N=4096 timeout -k 10 120 python tools/probe_policy.py > $O/probe_policy_default.log 2>&1 &&
HEIST_LIB=$PWD/tools/forensic/_ref/libheist_hip_policy_noslp.so PROBE_N=4096 timeout -k 10 120 python tools/probe_policy.py > $O/probe_policy_noslp.log 2>&1 &&
PROBE_N=4096 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d $O/pmc1 -o pmc1 --output-format csv -- python tools/probe_policy.py > $O/pmc1.log 2>&1
echo "rc=$?"
