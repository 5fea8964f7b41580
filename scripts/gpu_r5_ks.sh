# Round 5: rocprofv3 kernel trace + stats of the default bench command (config 2), the bench line
# it printed, and the stats summary copied to gpurun_out/profiles/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${V:-v1}
mkdir -p gpurun_out/profiles
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$V -o ks --output-format csv -- python -u bench.py > gpurun_out/r5_bench_ks_$V.json 2> gpurun_out/r5_bench_ks_$V.err || exit 1
f=$(ls gpurun_out/ks_$V/*/ks_kernel_stats.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find gpurun_out/ks_$V -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/profiles/r05_kernel_stats_$V.csv && cp gpurun_out/r5_bench_ks_$V.json gpurun_out/profiles/r05_bench_ks_$V.json
echo ks-ok
