# config 5 at 4,096 documents (the verdict's target size): base vs new library, k_replay ms.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in ${LIBS:-libcrdt_gpu_base.so libcrdt_gpu.so}; do
  N=$(basename $L .so)
  CRDT_GPU_LIB=text-crdt-rust_amd/build/$L timeout -k 10 300 python -u scripts/bench_config5.py --docs ${DOCS:-4096} --no-cpu > gpurun_out/c5big_$N.json 2> gpurun_out/c5big_$N.err || { tail -3 gpurun_out/c5big_$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5big_$N.json')); print('c5-${DOCS:-4096} $N', round(d['value']/1e6, 2), 'M ops/s', d['kernels_ms'], d['parity_ok'])" || exit 1
done
