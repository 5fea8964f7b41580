# PMC passes (FETCH_SIZE, WRITE_SIZE) of one k_materialize launch over 8,192 AP documents, each
# reading its own content copy (the bench's materialize leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${DOCS:-8192}
W="automerge-paper remote, per-document content copies, one launch"
timeout -s KILL 180 rocprofv3 --kernel-include-regex k_materialize --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_mat -o pmc --output-format csv -- python scripts/prof_materialize.py --docs $D > gpurun_out/pmc_fetch_mat.log 2>&1 && echo fetch-ok && \
timeout -s KILL 180 rocprofv3 --kernel-include-regex k_materialize --pmc WRITE_SIZE -d gpurun_out/pmc_write_mat -o pmc --output-format csv -- python scripts/prof_materialize.py --docs $D > gpurun_out/pmc_write_mat.log 2>&1 && echo write-ok && \
python scripts/traffic_from_pmc.py $D gpurun_out/traffic_k_materialize.json k_materialize _mat "$W"
