# PC sampling (host trap) of one clean k_replay launch, config 2 at 2048 documents.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs -o pcs --output-format csv -- python scripts/prof_replay.py --docs 2048 --clean > gpurun_out/pcs.log 2>&1
echo rc $?
ls -la gpurun_out/pcs gpurun_out/pcs/* 2>/dev/null | head; tail -5 gpurun_out/pcs.log
