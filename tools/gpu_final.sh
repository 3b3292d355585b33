set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-final}; mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-final} PROBE=tools/probe_arch_update.py bash tools/gpu_check.sh || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary > $O/prof_bench.log 2>&1
echo "rocprof rc=$?"
find $O/prof -name "*kernel_stats.csv" | head -3
