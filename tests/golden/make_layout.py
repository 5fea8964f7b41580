#!/usr/bin/env python3
"""Layout sensitivity of the reference's results: every history replayed by the
oracle (the reference restated; test infrastructure) at the release layout (leaf 32 / node 16),
the debug layout (4 / 8) and one unbounded leaf, with integrate's Q2 triggers counted (the
tie-break reads the agent of the entry's first order, doc.rs:207).  Writes
tests/golden/layout_q2.json: per history and layout the status, q2_triggers and digest, and
against the release layout whether the items' document order and deleted flags agree (same_order)
and how many stored origins differ (ol_diff / orr_diff: YjsSpan::prepend keeps the entry's
origin_left, span.rs:61-64, and prepends only happen inside one leaf, mutations.rs:84-109).
tests/test_layout.py re-derives the fast cases.  Run from the repo root (a few minutes: the
unbounded leaf shifts linearly)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "text-crdt-rust_amd"))
from oracle_lib import OracleDoc, LEAF_UNBOUNDED, compare_layouts  # noqa: E402
from crdt_amd.traces import load_remote_wire  # noqa: E402
from fuzz_gen import config5_wire  # noqa: E402

LAYOUTS = {"L32": (32, 16), "L4": (4, 8), "Linf": (LEAF_UNBOUNDED, 16)}


def histories(full: bool):
    for tr in ("sveltecomponent", "rustcode", "automerge-paper"):
        yield f"{tr}/remote", lambda tr=tr: load_remote_wire(tr)
    for seed in range(4):
        yield f"config5/seed{seed}/rounds8", lambda seed=seed: config5_wire(seed, base_len=1 << 20, n_agents=16, rounds=8, ops=64)
    if full:
        for seed in range(2):
            yield f"config5/seed{seed}/rounds64", lambda seed=seed: config5_wire(seed, base_len=1 << 20, n_agents=16, rounds=64, ops=64)


def run(wire):
    out, ex = {}, {}
    for k, (L, N) in LAYOUTS.items():
        o = OracleDoc(L, N)
        st = o.apply_remote_wire(wire)
        out[k] = {"status": st, "q2_triggers": o.stats()["q2_triggers"], "digest": f"{o.digest():016x}", "len": len(o)}
        ex[k] = o.export()
    for k in ("L4", "Linf"):
        out[k].update(compare_layouts(ex["L32"], ex[k]))
    return out


def main():
    res = {}
    for name, mk in histories(full="--quick" not in sys.argv):
        res[name] = run(mk())
        print(name, json.dumps(res[name]), flush=True)
    with open(os.path.join(HERE, "layout_q2.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
