# PMC passes (FETCH_SIZE, WRITE_SIZE) of one k_materialize launch over 4096 AP documents.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_mat -o pmc --output-format csv -- python scripts/prof_materialize.py --docs 4096 > gpurun_out/pmc_fetch_mat.log 2>&1 && echo fetch-ok && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_mat -o pmc --output-format csv -- python scripts/prof_materialize.py --docs 4096 > gpurun_out/pmc_write_mat.log 2>&1 && echo write-ok && \
python scripts/traffic_from_pmc.py 4096 gpurun_out/traffic_k_materialize.json k_materialize _mat
