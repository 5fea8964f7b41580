# One GPU call: parity tests, the default bench line (with CPU baseline), a kernel-trace profile
# of the bench, and two PMC passes (FETCH_SIZE, WRITE_SIZE) of one clean k_replay launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${DOCS:-4096}
TAG=${TAG:-r01}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench-ok && cat gpurun_out/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o ktrace --output-format csv -- python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/ktrace.log 2>&1 && echo ktrace-ok && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc_fetch.log 2>&1 && echo fetch-ok && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc_write.log 2>&1 && echo write-ok && \
python scripts/traffic_from_pmc.py $D gpurun_out/traffic_k_replay.json
echo "exit $?"
