# Round 4 PMC passes of ONE clean k_replay launch per workload (scripts/gpu_pmc_all.sh's passes:
# three SQ passes, then FETCH_SIZE and WRITE_SIZE each in its own run): config 2 (8,192 AP
# documents), config 4 (16,384 documents x 20,000 generated ops), config 5 (1,024 documents).
# Summaries: scripts/sq_summary.py / traffic_from_pmc.py -> profiles/r04_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-"ap c4 c5"}
for w in $WL; do
  case $w in
    ap) P="python scripts/prof_replay.py --docs 8192 --clean";;
    c4) P="python scripts/prof_replay.py --docs 16384 --random 20000 --clean";;
    c5) P="python scripts/prof_replay.py --docs 1024 --config5 --clean";;
  esac
  TAG=_$w P="$P" bash scripts/gpu_pmc_all.sh || exit 1
done
