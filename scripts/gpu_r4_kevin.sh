# kevin (benches/yjs.rs:51-62): one document and the 512-document batch (round 3's fit OOM case),
# plus the per-path profile of the compact local loop (-DCRDT_PROF build, 4 documents).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r4}
timeout -k 10 400 python -u scripts/bench_kevin.py --docs ${DOCS:-512} --reps 2 > gpurun_out/kevin_$TAG.json 2> gpurun_out/kevin_$TAG.err || { tail -5 gpurun_out/kevin_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/kevin_$TAG.json')); print('kevin single', d['single_doc']['k_replay_ms'], 'ms; batch', d['batch']['docs'], d['batch']['k_replay_ms'], 'ms', d['batch']['ops_per_s']/1e9, 'G ops/s', d['parity_ok'])" || exit 1
if [ -f text-crdt-rust_amd/build/libcrdt_gpu_prof.so ]; then
  KEVIN_OPS=5000000 CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 300 python scripts/prof_paths.py 4 kevin || exit 1
fi
