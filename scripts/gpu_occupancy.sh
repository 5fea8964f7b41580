set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for D in 2048 8192 12288 16384; do
timeout -k 10 200 python bench.py --no-cpu --no-text --steps 3 --warmup 1 --docs $D > gpurun_out/occ_$D.json 2> gpurun_out/occ_$D.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/occ_$D.json')); print($D, d['ms_per_step'], d['value']/1e9, d['roofline']['kernel_ms'])"
done
