# Round 3: config 5 across libraries (before the block -> group map, with it, with the
# lane-parallel frontier), AP A/B of the last two, then the config-5 bench line at 1,024 and
# 4,096 documents with the current library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v6}
B=text-crdt-rust_amd/build
for L in $B/libcrdt_gpu_premap.so $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so; do
  echo -n "c5-1024 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 200 python scripts/prof_replay.py --docs 1024 --config5 --clean | tail -1 || exit 1
done
for L in $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
for D in 1024 4096; do
  timeout -k 10 400 python -u scripts/bench_config5.py --docs $D > gpurun_out/c5_${D}_$TAG.json 2> gpurun_out/c5_${D}_$TAG.err && \
  python -c "import json; d=json.load(open('gpurun_out/c5_${D}_$TAG.json')); print('c5', $D, d['value']/1e6, 'M ops/s', d['kernels_ms'], d['parity_ok'])" || exit 1
done
