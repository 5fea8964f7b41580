# Config 5 staging experiment: one shared record stream (replicated) vs per-document copies of
# 1 or 8 distinct histories (bench_config5.py), 1,024 documents, k_replay ms.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for D in 1 8; do
  timeout -k 10 300 python -u scripts/bench_config5.py --docs 1024 --distinct $D --no-cpu > gpurun_out/c5x_d$D.json 2> gpurun_out/c5x_d$D.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c5x_d$D.json')); print('c5 distinct $D', d['kernels_ms'], d['parity_ok'])" || exit 1
done
echo -n "c5 replicated (prof_replay) "
timeout -k 10 300 python scripts/prof_replay.py --docs 1024 --config5 --clean | tail -1 || exit 1
