# Secondary lines: config 5 (1,024 docs, full per-document size) and config 4 (125,000 docs/GPU),
# each in the bench JSON schema; then SQ passes of one clean config-5 launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v1}
timeout -k 10 600 python -u scripts/bench_config5.py ${C5ARGS:-} > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err && echo c5-ok && \
python -c "import json; d=json.load(open('gpurun_out/c5_$TAG.json')); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d['parity_ok'], (d['cpu_baseline'] or {}).get('value'))" && \
timeout -k 10 600 python -u scripts/bench_config4.py ${C4ARGS:-} > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err && echo c4-ok && \
python -c "import json; d=json.load(open('gpurun_out/c4_$TAG.json')); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d['parity_ok'], d['cpu_baseline']['value'])"
