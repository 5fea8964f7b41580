#!/usr/bin/env python3
"""Per-path micro workloads for k_replay instruction accounting (diagnostic fixtures).

Each workload is a base document (P: `BASE` chars typed at the end, one typing run) followed by
`N` ops of one shape, so SQ instruction counts of (P + X) - (P) divided by N give the replay cost
per op of that shape (scripts/micro_paths.py).  Local traces are made here with numpy; their
remote form comes from the oracle's restated apply_local_txn (as tests/golden/make_remote.py), so
the generated wires are test fixtures.  Output: data/micro/<name>.rtx.gz.
"""
import gzip
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc, trace_to_wire  # noqa: E402

OUT = os.path.normpath(os.path.join(HERE, "..", "..", "data", "micro"))
BASE = 50000
N = 20000


def workload(kind: str, seed: int = 1):
    rng = np.random.default_rng(seed)
    pats = [(i, 0, 1) for i in range(BASE)]  # P: one typing run
    length = BASE
    if kind == "typing":
        pats += [(length + i, 0, 1) for i in range(N)]
    elif kind in ("jump10", "jump1"):
        run = 10 if kind == "jump10" else 1
        for _ in range(N // run):
            p = int(rng.integers(1, length))
            pats += [(p + i, 0, 1) for i in range(run)]
            length += run
    elif kind in ("bs10", "del1", "bs200"):
        run = {"bs10": 10, "del1": 1, "bs200": 200}[kind]
        for _ in range(N // run):
            p = int(rng.integers(run, length))
            pats += [(p - i, 1, 0) for i in range(run)]  # backspace: each deletes the char before
            length -= run
    elif kind == "fd200":  # forward delete runs: each deletes the char at the same position
        run = 200
        for _ in range(N // run):
            p = int(rng.integers(0, length - run))
            pats += [(p, 1, 0) for i in range(run)]
            length -= run
    elif kind != "base":
        raise ValueError(kind)
    patches = np.array(pats, np.uint32)
    counts = np.ones(patches.shape[0], np.uint32)
    return counts, patches


KINDS = ("base", "typing", "jump10", "jump1", "bs10", "del1", "bs200", "fd200")

if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    for k in (sys.argv[1:] or KINDS):
        c, p = workload(k)
        w = trace_to_wire(c, p, "jeremy")
        loc = OracleDoc()
        assert loc.apply_trace(loc.agent("jeremy"), c, p) == 0
        rem = OracleDoc()
        assert rem.apply_remote_wire(w) == 0 and rem.digest() == loc.digest()
        with gzip.open(os.path.join(OUT, k + ".rtx.gz"), "wb", compresslevel=9) as f:
            f.write(w)
        print(k, p.shape[0], "ops", len(w), "wire bytes, digest", hex(rem.digest()))
