# Why the config-5 bench (8 histories, per-document wires) is slower than one replicated history
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for X in 1 8; do
  timeout -k 10 300 python -u scripts/bench_config5.py --docs 1024 --distinct $X --no-cpu > gpurun_out/c5dbg_$X.json 2> gpurun_out/c5dbg_$X.err && \
  python -c "import json; d=json.load(open('gpurun_out/c5dbg_$X.json')); print('distinct', $X, d['value']/1e6, 'M ops/s', d['kernels_ms'])" || exit 1
done
timeout -k 10 200 python scripts/prof_replay.py --docs 1024 --config5 --clean | tail -1
