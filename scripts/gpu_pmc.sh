# PMC passes (round RN, default r06) of ONE clean k_replay launch per workload (the last dispatch of each pass;
# scripts/gpu_pmc_all.sh: three SQ passes, then FETCH_SIZE and WRITE_SIZE each in its own run),
# summarised with the workload's own label (scripts/sq_summary.py, traffic_from_pmc.py).  The
# summaries are also copied to gpurun_out/profiles/ (only gpurun_out/ comes back from the box).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out profiles
WL=${WL:-"ap c3 c4 c5"}
V=${V:-v1}
RN=${RN:-r06}
for w in $WL; do
  case $w in
    ap) D=8192; OPS=259778; P="python scripts/prof_replay.py --docs $D --clean"; T=""; LBL="automerge-paper remote, one clean launch";;
    c3) D=65536; OPS=$(python -c "
import sys; sys.path.insert(0, 'text-crdt-rust_amd'); sys.path.insert(0, '.')
from bench import splitmix64; from crdt_amd.traces import load_trace
n = [load_trace(x).n_patches for x in ('automerge-paper', 'rustcode', 'sveltecomponent')]
print(round(sum(n[splitmix64(d) % 3] for d in range($D)) / $D))"); P="python scripts/prof_replay.py --docs $D --config3 --clean"; T="_config3"; LBL="config 3: mixed local corpus, shared record streams, one clean launch";;
    c3ns) D=32768; OPS=$(python -c "
import sys; sys.path.insert(0, 'text-crdt-rust_amd'); sys.path.insert(0, '.')
from bench import splitmix64; from crdt_amd.traces import load_trace
n = [load_trace(x).n_patches for x in ('automerge-paper', 'rustcode', 'sveltecomponent')]
print(round(sum(n[splitmix64(d) % 3] for d in range($D)) / $D))"); P="python scripts/prof_replay.py --docs $D --config3 --no-share --clean"; T="_config3_noshare"; LBL="config 3: mixed local corpus, per-document record streams, one clean launch";;
    c4) D=125000; OPS=20000; P="python scripts/prof_replay.py --docs $D --random 20000 --clean"; T="_config4"; LBL="config 4: generated random edits (20,000 ops/doc), one clean launch";;
    c5d) D=8192; OPS=65537; P="python scripts/bench_config5.py --docs 8192 --steps 1 --no-cpu --check-docs 2"; T="_config5d"; LBL="config 5: per-document concurrent histories (1 M-char base, 16 agents), one clean launch";;
    c5) D=8192; OPS=65537; P="python scripts/prof_replay.py --docs $D --config5 --clean"; T="_config5"; LBL="config 5: concurrent histories (1 M-char base, 16 agents), one clean launch";;
  esac
  PT=150; [ $w = c5d ] && PT=400  # (c5d: generation + staging of 8,192 histories in every pass)
  TAG=_$w P="$P" PT=$PT bash scripts/gpu_pmc_all.sh > gpurun_out/pmc_$w.log 2>&1 || { cat gpurun_out/pmc_$w.log; exit 1; }
  python scripts/traffic_from_pmc.py $D profiles/traffic_k_replay$T.json k_replay _$w "$LBL" || exit 1
  python scripts/sq_summary.py profiles/${RN}_sq_k_replay_${w}_${D}_${V}.json $D $OPS _$w "$LBL" > /dev/null || exit 1
  cp profiles/traffic_k_replay$T.json profiles/${RN}_traffic_k_replay_${w}_${D}_${V}.json
  mkdir -p gpurun_out/profiles && cp profiles/traffic_k_replay$T.json profiles/${RN}_*_k_replay_${w}_${D}_${V}.json gpurun_out/profiles/
  echo $w-ok
done
