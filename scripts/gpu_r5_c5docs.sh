# Round 5: config 5 at more documents per GPU (more resident waves per SIMD for the latency-bound
# general path), one bench_config5.py run per size, CRDT_DEBUG_MEM layout lines in the .err files.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for D in ${DOCS:-5120 6144}; do
  CRDT_DEBUG_MEM=1 timeout -k 10 420 python -u scripts/bench_config5.py --docs $D --no-cpu > gpurun_out/c5docs_$D.json 2> gpurun_out/c5docs_$D.err || { tail -5 gpurun_out/c5docs_$D.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5docs_$D.json'));print($D, d['value']/1e6, d['roofline']['kernel_ms'], d['config']['hbm_bytes_per_doc']/1e6, d['config']['device_peak_bytes']/1e9, d['parity_ok'])"
done
