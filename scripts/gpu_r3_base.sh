# Round-3 baseline at HEAD: GPU tests, smoke, bench line, kernel trace, then the secondary lines
# (config 5, config 4, kevin at the reference size), each step under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v1}
bash scripts/gpu_final.sh && \
timeout -k 10 400 python -u scripts/bench_config5.py > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err && echo c5-ok && \
timeout -k 10 400 python -u scripts/bench_config4.py > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err && echo c4-ok && \
timeout -k 10 300 python -u scripts/bench_kevin.py > gpurun_out/kevin_$TAG.json 2> gpurun_out/kevin_$TAG.err && echo kevin-ok
[ $? -eq 0 ] && \
timeout -k 10 300 python -u scripts/bench_intern.py --replicated --docs 8192 > gpurun_out/intern_repl_$TAG.json 2>&1 && echo intern-ok && \
DOCS=8192 bash scripts/gpu_pmc_mat.sh
