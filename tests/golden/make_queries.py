#!/usr/bin/env python3
"""Golden query answers from the oracle (restatement of the reference; test infrastructure), the
README's two lookups (README.md:22-25) on the release layout (leaf 32 / node 16):

* pos -> (agent, seq): cursor_at_content_pos + get_item + client_with_order.get
  (root.rs:54-88, cursor.rs:233-239, simple_rle.rs:98-103);
* (agent, seq) -> (pos, deleted): seq_to_order + get_cursor_before + Cursor::count_pos
  (doc.rs:26-29, 109-119, cursor.rs:147-190); a deleted item reports the position of the next
  visible one; an unknown (agent, seq) answers (0xFFFFFFFF, 2).

Files (tests/golden/):
* ap_remote_pos_seq.delta.gz -- automerge-paper replayed as remote txns: the seq of every visible
  position (one author, agent 0), little-endian i32 deltas.  bench.py checks every timed
  pos -> loc answer against it.
* ap_remote_seq_pos.delta.gz -- the same document: (pos, deleted) of every seq the author ever
  used (inserted and deleted items, and the seqs its deletes consumed), as i32 position deltas
  followed by one u8 deleted flag per seq.  bench.py checks every timed loc -> pos answer against
  it; tests/test_gpu_parity.py every seq.
* queries_{rustcode,sveltecomponent}.npz -- 4,096 seeded random positions with their
  (agent, seq), and 4,096 seeded random seqs (all of the author's seqs, visible or not) with their
  (pos, deleted), of the remote replay of each trace.
Run from the repo root: python tests/golden/make_queries.py"""
import gzip
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc  # noqa: E402
from crdt_amd.traces import load_remote_wire  # noqa: E402


def write_gz(name, data: bytes):
    with open(os.path.join(HERE, name), "wb") as raw, gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
        f.write(data)  # (mtime 0: the file is a function of its content)


def replay(trace):
    o = OracleDoc(32, 16)
    assert o.apply_remote_wire(load_remote_wire(trace)) == 0
    return o


def main():
    o = replay("automerge-paper")
    pos = np.arange(len(o), dtype=np.uint32)
    agent, seq = o.pos_to_loc(pos)
    assert (agent == 0).all()
    d = np.diff(seq.astype(np.int64), prepend=0).astype(np.int32)
    write_gz("ap_remote_pos_seq.delta.gz", d.tobytes())
    n_seq = o.sizes()["next_order"]  # one author: its seqs are 0 .. next_order - 1
    seqs = np.arange(n_seq, dtype=np.uint32)
    p, dl = o.loc_to_pos(np.zeros(n_seq, np.uint16), seqs)
    dp = np.diff(p.astype(np.int64), prepend=0).astype(np.int32)
    write_gz("ap_remote_seq_pos.delta.gz", dp.tobytes() + dl.astype(np.uint8).tobytes())
    print("automerge-paper:", len(o), "positions,", n_seq, "seqs", "deleted", int((dl == 1).sum()), "unknown", int((dl == 2).sum()))
    for tr, seed in (("rustcode", 11), ("sveltecomponent", 12)):
        o = replay(tr)
        rng = np.random.default_rng(seed)
        qp = rng.integers(0, len(o), 4096).astype(np.uint32)
        qa, qs = o.pos_to_loc(qp)
        n_seq = o.sizes()["next_order"]
        ls = rng.integers(0, n_seq, 4096).astype(np.uint32)
        la = np.zeros(4096, np.uint16)
        lp, ld = o.loc_to_pos(la, ls)
        np.savez_compressed(os.path.join(HERE, f"queries_{tr}.npz"), pos=qp, pos_agent=qa, pos_seq=qs,
                            loc_agent=la, loc_seq=ls, loc_pos=lp, loc_deleted=ld)
        print(tr, len(o), "positions", n_seq, "seqs; sampled deleted", int((ld == 1).sum()), "unknown", int((ld == 2).sum()))


if __name__ == "__main__":
    main()
