set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 300 python -u bench.py --docs 256 --steps 2 --warmup 1 --cpu-docs 16 > gpurun_out/bench_256.json 2> gpurun_out/bench_256.err && echo bench256-ok && cat gpurun_out/bench_256.json && \
timeout -k 10 600 python -u bench.py --docs 4096 --steps 3 --warmup 1 --cpu-docs 64 > gpurun_out/bench_4096.json 2> gpurun_out/bench_4096.err && echo bench4096-ok && cat gpurun_out/bench_4096.json
echo "exit $?"
tail -5 gpurun_out/bench_256.err gpurun_out/bench_4096.err 2>/dev/null
