# The secondary measurement lines: config 3 (65,536 documents), config 4 (125,000 documents per
# GPU) and device interning (125,000 documents x 16 names).  JSON lines under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-}
timeout -k 10 500 python -u scripts/bench_config3.py > gpurun_out/config3$TAG.json 2> gpurun_out/config3$TAG.err && echo c3-ok && cat gpurun_out/config3$TAG.json && \
timeout -k 10 600 python -u scripts/bench_config4.py > gpurun_out/config4$TAG.json 2> gpurun_out/config4$TAG.err && echo c4-ok && cat gpurun_out/config4$TAG.json && \
timeout -k 10 300 python -u scripts/bench_intern.py > gpurun_out/intern$TAG.json 2> gpurun_out/intern$TAG.err && echo intern-ok && cat gpurun_out/intern$TAG.json
