# Round-5 start: GPU tests, the default bench line and one WRITE_SIZE / FETCH_SIZE pass of the clean
# AP k_replay launch at HEAD (baseline for this round's A/B runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_gpu_tests_base.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r5_bench_base.json 2> gpurun_out/r5_bench_base.err && echo bench-ok && \
DOCS=8192 TAG=_r5base bash scripts/gpu_pmc_all.sh > gpurun_out/r5_pmc_base.log 2>&1 && echo pmc-ok
