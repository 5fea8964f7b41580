"""Static instruction census of one kernel, attributed to source lines / functions.

Compile the device code with line info (`hipcc --offload-arch=gfx950 -O3 -g --cuda-device-only -S`),
then: python scripts/isa_lines.py krg.s _ZN4crdt8k_replayILi32EEEvNS_5PoolsEjjjPKj [--by func|line]
Each instruction is charged to the innermost `.loc` before it; counts are split into scalar (s_*),
vector (v_*), memory (global_/buffer_/ds_/flat_) and readlane/writelane.  Functions are found by
the `CRDT_HD ... name(` definitions of the csrc headers (the enclosing definition of the line)."""
import collections
import os
import re
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "text-crdt-rust_amd", "csrc")


def func_table(path):
    out = []
    pat = re.compile(r"^\s*(?:template\s*<[^>]*>\s*)?(?:CRDT_HD|__device__|static|inline|CRDT_INLINE)[^(;]*?\b(\w+)\s*\(")
    with open(path) as f:
        for i, line in enumerate(f, 1):
            m = pat.match(line)
            if m and m.group(1) not in ("if", "for", "while", "return"):
                out.append((i, m.group(1)))
    return out


def main():
    src, sym = sys.argv[1], sys.argv[2]
    by = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--by" else "func"
    files = {}
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    cur = None
    cnt = collections.defaultdict(lambda: collections.Counter())
    for l in lines[:start]:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(3)
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or re.match(r"^_Z\w+:", l) or l.strip().startswith(".Lfunc_end"):
            break
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(3)
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        m = re.match(r"\s+([sv]_\w+|global_\w+|buffer_\w+|ds_\w+|flat_\w+|scratch_\w+)", l)
        if not m:
            continue
        op = m.group(1)
        if op.startswith("s_nop") or op.startswith("s_waitcnt"):
            kind = "wait"
        elif op.startswith("v_readlane") or op.startswith("v_writelane") or op.startswith("v_readfirstlane"):
            kind = "lane"
        elif op.startswith("s_"):
            kind = "salu" if not re.match(r"s_(cbranch|branch|setpc|swappc)", op) else "branch"
        elif op.startswith("v_"):
            kind = "valu"
        else:
            kind = "mem"
        cnt[cur][kind] += 1
    tables = {}
    agg = collections.defaultdict(collections.Counter)
    for (fn, ln), c in cnt.items():
        if by == "line":
            key = f"{fn}:{ln}"
        else:
            if fn not in tables:
                p = os.path.join(CSRC, fn)
                tables[fn] = func_table(p) if os.path.exists(p) else []
            name = "?"
            for i, nm in tables[fn]:
                if i <= ln:
                    name = nm
                else:
                    break
            key = f"{fn}:{name}"
        agg[key].update(c)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1].values()))
    tot = collections.Counter()
    for _, c in rows:
        tot.update(c)
    print(f"{'where':60s} {'all':>6s} {'salu':>6s} {'valu':>6s} {'lane':>6s} {'br':>5s} {'mem':>5s} {'wait':>5s}")
    for k, c in rows[:int(os.environ.get("TOP", "60"))]:
        print(f"{k[:60]:60s} {sum(c.values()):6d} {c['salu']:6d} {c['valu']:6d} {c['lane']:6d} {c['branch']:5d} {c['mem']:5d} {c['wait']:5d}")
    print(f"{'TOTAL':60s} {sum(tot.values()):6d} {tot['salu']:6d} {tot['valu']:6d} {tot['lane']:6d} {tot['branch']:5d} {tot['mem']:5d} {tot['wait']:5d}")


if __name__ == "__main__":
    main()
