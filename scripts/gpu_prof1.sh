set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python bench.py --docs 512 --steps 2 --warmup 1 --no-cpu --queries 1024 > gpurun_out/prof_kt.log 2>&1; echo "kt exit $?"
ls -R gpurun_out/prof_kt | head -20
