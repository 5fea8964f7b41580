#!/usr/bin/env python3
"""Golden query answers from the oracle (restatement of the reference; test infrastructure):
pos -> (agent, seq) for every visible position of automerge-paper replayed as remote txns at the
release layout (cursor_at_content_pos + client_with_order.get, README.md:22-25).  The trace has one
author (agent 0), so the fixture is the seq per position, stored as little-endian i32 deltas,
gzipped: tests/golden/ap_remote_pos_seq.delta.gz.  bench.py checks every timed pos -> loc answer
against it (the bench's documents hold this state, with the author renamed per document)."""
import gzip
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc  # noqa: E402
from crdt_amd.traces import load_remote_wire  # noqa: E402

o = OracleDoc(32, 16)
assert o.apply_remote_wire(load_remote_wire("automerge-paper")) == 0
pos = np.arange(len(o), dtype=np.uint32)
agent, seq = o.pos_to_loc(pos)
assert (agent == 0).all()
d = np.diff(seq.astype(np.int64), prepend=0).astype(np.int32)
with gzip.open(os.path.join(HERE, "ap_remote_pos_seq.delta.gz"), "wb", compresslevel=9) as f:
    f.write(d.tobytes())
print(len(o), "positions")
