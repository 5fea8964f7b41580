# Round-end evidence at the final source, in stages that each fit one gpurun call (STAGE=...):
#   pmc1  PMC passes (3 SQ + FETCH_SIZE + WRITE_SIZE) of one clean k_replay launch: automerge-paper
#         remote at 8,192 documents, config 4 at 125,000 (one corpus batch), config 3 at 65,536
#   pmc2  the same for config 5 with per-document histories at 8,192 documents
#   main  all GPU tests, smoke(), the default bench line (config 2 + stated size + materialize +
#         the 1 M-document corpus leg) and rocprofv3 --kernel-trace --stats of the same command
#   lines the secondary lines: config 3, config 5 (per-document histories), kevin, single document
# The PMC stages run first: the bench lines read the traffic files they write (profiles/traffic_*,
# copied back from gpurun_out/profiles/ before the next stage).  RN names the round's files.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out profiles
RN=${RN:-r06}
case ${STAGE:-main} in
  pmc1) WL="ap c4 c3" V=final RN=$RN bash scripts/gpu_pmc.sh;;
  pmc2) WL="c5d" V=final RN=$RN bash scripts/gpu_pmc.sh;;
  main)
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${RN}_gpu_tests_final.log 2>&1 && echo tests-ok && \
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${RN}_smoke_final.log 2>&1 && echo smoke-ok && \
    timeout -k 10 500 python -u bench.py > gpurun_out/${RN}_bench_final.json 2> gpurun_out/${RN}_bench_final.err && echo bench-ok && \
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o ktrace --output-format csv -- python bench.py > gpurun_out/${RN}_bench_ks_final.json 2> gpurun_out/ktrace.log && echo ktrace-ok
    ;;
  lines)
    timeout -k 10 400 python -u scripts/bench_config3.py --docs 65536 > gpurun_out/${RN}_bench_config3_65536_final.json 2> gpurun_out/c3.err && echo c3-ok && \
    timeout -k 10 400 python -u scripts/bench_config5.py --docs 8192 > gpurun_out/${RN}_bench_config5_8192_distinct_final.json 2> gpurun_out/c5.err && echo c5-ok && \
    timeout -k 10 300 python -u scripts/bench_kevin.py --docs 512 > gpurun_out/${RN}_bench_kevin_512_final.json 2> gpurun_out/kevin.err && echo kevin-ok && \
    timeout -k 10 300 python -u scripts/bench_single.py > gpurun_out/${RN}_bench_single_final.jsonl 2> gpurun_out/single.err && echo single-ok
    ;;
esac
