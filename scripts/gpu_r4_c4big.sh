# config 4 at 125,000 documents per GPU (1 M / 8): the bench line of scripts/bench_config4.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/bench_config4.py --docs ${DOCS:-125000} > gpurun_out/c4big.json 2> gpurun_out/c4big.err || { tail -5 gpurun_out/c4big.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4big.json')); print('c4', d['config'].get('docs_per_gpu'), round(d['value']/1e9, 3), 'G ops/s', d['kernels_ms'], d['parity_ok'])"
