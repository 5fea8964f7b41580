# SQ + HBM PMC passes of the publish kernels (k_publish, k_pub_index) over 8,192 AP documents.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
DOCS=8192 TAG=pub R="--kernel-include-regex k_publish" bash scripts/gpu_pmc_all.sh && \
SQ_KERNEL=k_publish SQ_WORKLOAD="k_publish, automerge-paper remote, 8192 docs" python scripts/sq_summary.py gpurun_out/sq_pub.json 8192 259778 pub && cat gpurun_out/sq_pub.json && \
python scripts/traffic_from_pmc.py 8192 gpurun_out/traffic_pub.json k_publish pub "k_publish, automerge-paper remote, 8192 docs" && cat gpurun_out/traffic_pub.json
