#!/usr/bin/env python3
"""Generate the remote-txn form of each trace (fixture for BASELINE config 2).

Each local txn of the trace (agent "jeremy", as benches/yjs.rs:12) is replayed through the oracle's
restated apply_local_txn and re-expressed as the reference's RemoteTxn (external_txn.rs:25-30):
Ins{origin_left, origin_right} from the inserted span, Del{id, len} per deleted run, parents =
frontier.  Output: data/traces/<name>.rtx.gz (wire batch, see oracle/wire.hpp).  The script also
checks that remote replay reproduces the local replay exactly (raw entry layout + digest), the
reference's own remote_txns equivalence test (doc.rs:620-676) applied to a whole trace.
"""
import gzip
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc, trace_to_wire  # noqa: E402
from crdt_amd.traces import DATA_DIR, TRACE_NAMES, load_trace  # noqa: E402

if __name__ == "__main__":
    for name in TRACE_NAMES:
        t = load_trace(name)
        w = trace_to_wire(t.counts, t.patches, "jeremy")
        loc = OracleDoc()
        loc.apply_trace(loc.agent("jeremy"), t.counts, t.patches)
        rem = OracleDoc()
        assert rem.apply_remote_wire(w) == 0
        el, er = loc.export(), rem.export()
        assert all(np.array_equal(el[k], er[k]) for k in ("raw", "leaf_sizes", "cwo", "deletes", "txns", "frontier"))
        assert loc.digest() == rem.digest()
        with gzip.open(os.path.join(DATA_DIR, name + ".rtx.gz"), "wb", compresslevel=9) as f:
            f.write(w)
        print(name, len(w), "bytes, digest", hex(rem.digest()))
