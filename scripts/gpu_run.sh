# GPU tests (round RN, default r06), then the lines named in RUNS (ap = bench.py default; c5 = config 5 at 8,192
# documents; c3 = config 3 at 65,536; c4 = config 4 corpus), each under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${V:-v1}
RN=${RN:-r06}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${RN}_gpu_tests_$V.log 2>&1
  rc=$?; echo tests rc=$rc; tail -2 gpurun_out/${RN}_gpu_tests_$V.log
  [ $rc -le 1 ] || exit $rc
fi
for r in ${RUNS:-ap}; do
  case $r in
    ap) timeout -k 10 600 python -u bench.py > gpurun_out/${RN}_bench_$V.json 2> gpurun_out/${RN}_bench_$V.err || exit 1;;
    c5) timeout -k 10 600 python -u scripts/bench_config5.py --docs 8192 > gpurun_out/${RN}_bench_config5_8192_$V.json 2> gpurun_out/${RN}_bench_config5_8192_$V.err || exit 1;;
    c3) timeout -k 10 600 python -u scripts/bench_config3.py > gpurun_out/${RN}_bench_config3_65536_$V.json 2> gpurun_out/${RN}_bench_config3_65536_$V.err || exit 1;;
    c3ns) timeout -k 10 600 python -u scripts/bench_config3.py --docs 32768 --no-share > gpurun_out/${RN}_bench_config3_32768_noshare_$V.json 2> gpurun_out/${RN}_bench_config3_32768_noshare_$V.err || exit 1;;
    c4) timeout -k 10 900 python -u bench.py --workload config4 > gpurun_out/${RN}_bench_config4_1M_$V.json 2> gpurun_out/${RN}_bench_config4_1M_$V.err || exit 1;;
  esac
  echo $r-ok
done
