#!/usr/bin/env python3
"""Convert the reference's editing traces into this repo's compact binary trace format.

Test/bench input infrastructure (run once, in the build container, where /root/reference exists).
Input : /root/reference/benchmark_data/{automerge-paper,rustcode,sveltecomponent}.json.gz
        schema = src/testdata/src/lib.rs:10-27 ({startContent, endContent, txns:[{time, patches:[[pos, del, ins]]}]})
Output: data/traces/<name>.trc.gz   (committed; the GPU box never sees /root/reference)

Positions / lengths count Unicode scalar values, as the reference does (`chars().count()`,
src/list/doc.rs:383). All three traces start empty.

Binary layout (little endian), gzip-compressed:
  b"CRDTTRC1"
  u32 n_txns, u32 n_patches, u32 start_len, u32 end_len (chars), u32 end_bytes (utf-8 bytes)
  u64 end_fnv1a64 (FNV-1a over endContent utf-8 bytes)
  u32 patches_per_txn[n_txns]
  u32 patch[n_patches][3]  = (pos, del_len, ins_len_chars)
  u32 text_bytes ; u8 inserted_text_utf8[text_bytes]   (all inserted strings concatenated)
"""
import gzip
import json
import os
import struct
import sys

import numpy as np

REF = "/root/reference/benchmark_data"
NAMES = ["automerge-paper", "rustcode", "sveltecomponent"]


def fnv1a64(b: bytes) -> int:
    h = 0xCBF29CE484222325
    for x in b:
        h ^= x
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def convert(name: str, out_dir: str) -> dict:
    d = json.load(gzip.open(os.path.join(REF, name + ".json.gz")))
    txns = d["txns"]
    counts = np.array([len(t["patches"]) for t in txns], dtype=np.uint32)
    patches = np.zeros((int(counts.sum()), 3), dtype=np.uint32)
    text = []
    k = 0
    for t in txns:
        for pos, dl, ins in t["patches"]:
            patches[k] = (pos, dl, len(ins))
            text.append(ins)
            k += 1
    text_b = "".join(text).encode("utf-8")
    end = d["endContent"]
    end_b = end.encode("utf-8")
    hdr = b"CRDTTRC1" + struct.pack("<5IQ", len(txns), len(patches), len(d["startContent"]),
                                    len(end), len(end_b), fnv1a64(end_b))
    blob = hdr + counts.tobytes() + patches.tobytes() + struct.pack("<I", len(text_b)) + text_b
    path = os.path.join(out_dir, name + ".trc.gz")
    with gzip.open(path, "wb", compresslevel=9) as f:
        f.write(blob)
    return dict(name=name, txns=len(txns), patches=len(patches), end_len=len(end),
                end_bytes=len(end_b), end_fnv=fnv1a64(end_b))


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "..", "data", "traces")
    os.makedirs(out, exist_ok=True)
    for n in NAMES:
        print(convert(n, out))
