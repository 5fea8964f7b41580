# CPU-only estimate of k_replay's dynamic instruction profile on one AP remote document:
# the gfx950 code object built with -g (ISA + DWARF) x gcov line counts of the CPU emulation of
# the same replay_core.h (scripts/isa_dynamic.py).  No GPU needed; ranks the hot code.
# usage: bash scripts/isa_profile.sh [TOP] [WIRE_TRACE]
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${ISA_OUT:-/tmp/isa}
TOP=${1:-60}
TRACE=${2:-automerge-paper}
mkdir -p $OUT
CS=$ROOT/text-crdt-rust_amd/csrc
[ -n "$SKIP_DEV" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -g -std=c++17 -fno-strict-aliasing -mllvm -phi-elim-split-all-critical-edges=1 \
  -mllvm -structurizecfg-skip-uniform-regions=1 -I$ROOT/include -I$CS --cuda-device-only --no-gpu-bundle-output -c \
  $CS/engine.hip -o $OUT/dev.o
LB=/opt/rocm/lib/llvm/bin
[ -n "$SKIP_DEV" ] || $LB/llvm-objdump -d --no-show-raw-insn $OUT/dev.o > $OUT/dis.txt
[ -n "$SKIP_DEV" ] || $LB/llvm-dwarfdump --debug-info $OUT/dev.o > $OUT/dwarf.txt
[ -n "$SKIP_DEV" ] || $LB/llvm-dwarfdump --debug-line $OUT/dev.o > $OUT/lines.txt
rm -rf $OUT/cov && mkdir -p $OUT/cov
( cd $OUT/cov && g++ -O0 --coverage -g -std=c++17 -fPIC -w -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$CS -I$ROOT/tests/emu \
    -c -o emu.o $ROOT/tests/emu/emu.cpp && g++ --coverage -shared -o libemu_cov.so emu.o )
OPS=$(cd $ROOT/tests && CRDT_EMU_LIB=$OUT/cov/libemu_cov.so python -c "
import sys; sys.path.insert(0, '$ROOT/text-crdt-rust_amd')
from emu_lib import EmuDoc
from crdt_amd.traces import load_remote_wire, load_trace
e = EmuDoc(32)
if '$TRACE' == 'config4':  # generated ops (bench_config4.py's shape, one document)
    assert e.run_random(e.agent('gen'), 20000, 0xC0FFEE, 64) == 0
    print(20000)
elif '$TRACE' == 'kevin':  # 200k single-char prepends (benches/yjs.rs:51-62 shape)
    import numpy as np
    n = 200000
    c = np.ones(n, np.uint32); pt = np.zeros((n, 3), np.uint32); pt[:, 2] = 1
    assert e.run_local(e.agent('seph'), c, pt, 64) == 0
    print(n)
elif '$TRACE' == 'config5':  # one config-5 history (SURVEY 8(d) shape)
    sys.path.insert(0, '$ROOT/tests')
    from fuzz_gen import config5_wire
    sys.path.insert(0, '$ROOT')
    from bench import wire_ops
    w = config5_wire(7, base_len=1 << 20, n_agents=16, rounds=64, ops=64)
    assert e.run_wire(w, 64) == 0
    print(wire_ops(w)[0])
elif '$TRACE'.endswith('.rtx.gz'):  # a wire file (e.g. data/micro/*.rtx.gz): ops = its RemoteOps
    import gzip, os
    sys.path.insert(0, '$ROOT')
    from bench import wire_ops
    w = gzip.open(os.path.join('$ROOT', '$TRACE'), 'rb').read()
    assert e.run_wire(w, 64) == 0
    print(wire_ops(w)[0])
else:
    assert e.run_wire(load_remote_wire('$TRACE'), 64) == 0
    t = load_trace('$TRACE')
    print(int(t.patches.shape[0]) if t.patches.ndim > 1 else len(t.patches) // 3)
")
( cd $OUT/cov && gcov -o . $ROOT/tests/emu/emu.cpp > /dev/null 2>&1 || true )
python $ROOT/scripts/isa_dynamic.py $OUT/dev.o $OUT/dis.txt $OUT/dwarf.txt $OUT/lines.txt $OUT/cov $OPS $TOP
