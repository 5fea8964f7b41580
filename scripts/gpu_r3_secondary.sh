# Round-3 secondary lines at the current library (bench JSON schema) + the AP PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3f}
timeout -k 10 500 python -u scripts/bench_config5.py --docs 4096 > gpurun_out/c5_4096_$TAG.json 2> gpurun_out/c5_4096_$TAG.err && echo c5-ok && \
timeout -k 10 500 python -u scripts/bench_config4.py > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err && echo c4-ok && \
timeout -k 10 500 python -u scripts/bench_config3.py > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err && echo c3-ok && \
timeout -k 10 300 python -u scripts/bench_kevin.py > gpurun_out/kevin_$TAG.json 2> gpurun_out/kevin_$TAG.err && echo kevin-ok && \
TAG=_$TAG DOCS=8192 bash scripts/gpu_pmc_all.sh
