# Device-only compile of the engine (same codegen flags as crdt_amd.build) and the register /
# spill metadata of k_replay<32>: a quick register-budget check while editing replay_core.h.
# usage: bash scripts/dev_regs.sh [-DNAME ...]
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/text-crdt-rust_amd/csrc
O=${DEV_O:-/tmp/dev_regs_$$.o}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-strict-aliasing -mllvm -phi-elim-split-all-critical-edges=1 \
  -mllvm -structurizecfg-skip-uniform-regions=1 -I$ROOT/include -I$CS --cuda-device-only --no-gpu-bundle-output -c "$@" \
  $CS/engine.hip -o $O 2>/dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $O | awk '/\.name:/{n=$2} /vgpr_count|vgpr_spill|sgpr_spill|sgpr_count|private_segment_fixed/{if (n ~ /k_replayILi32/) print n, $0}' | sort -u
rm -f $O
