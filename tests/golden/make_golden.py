#!/usr/bin/env python3
"""Golden vectors from the oracle (restatement of the reference), committed as tests/golden/oracle_golden.json.

Pins: per-trace final length (== endContent length, the reference's own bench assertion
benches/yjs.rs:46), table sizes and the canonical-state digest for release (32/16) and debug (4/8)
tree shapes, for local replay and for remote replay of the converted trace.  `text_digest` is the
text digest (k_materialize / crdt_oracle.hpp text_digest) of the materialised text, asserted here to
be the trace's endContent (FNV-1a of the reference's fixture).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc  # noqa: E402
from crdt_amd.traces import TRACE_NAMES, content_by_order, fnv1a64, load_remote_wire, load_trace, utf32_to_str  # noqa: E402

out = {}
for name in TRACE_NAMES:
    t = load_trace(name)
    for L, N in ((32, 16), (4, 8)):
        d = OracleDoc(L, N)
        assert d.apply_trace(d.agent("jeremy"), t.counts, t.patches) == 0
        r = OracleDoc(L, N)
        assert r.apply_remote_wire(load_remote_wire(name)) == 0
        txt, tdg = d.text(content_by_order(t))
        assert fnv1a64(utf32_to_str(txt).encode()) == t.end_fnv
        assert r.text(content_by_order(t))[1] == tdg
        out[f"{name}/L{L}"] = dict(len=len(d), end_len=t.end_len, digest=hex(d.digest()),
                                   remote_digest=hex(r.digest()), sizes=d.sizes(), text_digest=hex(tdg))
json.dump(out, open(os.path.join(HERE, "oracle_golden.json"), "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1)[:2000])
