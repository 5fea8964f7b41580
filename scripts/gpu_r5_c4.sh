# Round 5: GPU tests, then the config-4 corpus line (1,000,000 documents on one GPU, 8 batches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${V:-v1}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests_$V.log 2>&1
rc=$?
echo tests rc=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u bench.py --workload config4 ${C4ARGS:-} > gpurun_out/r5_bench_config4_1M_$V.json 2> gpurun_out/r5_bench_config4_1M_$V.err && echo c4-ok
