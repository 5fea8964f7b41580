"""VGPR liveness census of one kernel in a `hipcc -S -g` dump: where the register pressure peaks
and which values are live there (each live register is tagged with the source line of a def that
reaches it).  Approximate (operand roles by mnemonic; partial writes counted as uses too), but
enough to find the code region that sets a kernel's VGPR count.

usage: python scripts/isa_liveness.py dump.s KERNEL_SYMBOL [TOP]"""
import collections
import re
import sys


def regs_of(tok):
    out = []
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", tok):
        if m.group(3):
            out.append(int(m.group(3)))
        else:
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


STORE = re.compile(r"^(global_store|buffer_store|ds_write|ds_bpermute_b32_dummy|flat_store|scratch_store|global_atomic\w*(?<!_rtn)$)")


def parse(path, sym):
    lines = open(path).read().split("\n")
    files, loc = {}, None
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    for l in lines[:start]:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(3)
    insts = []  # (label or None, mnemonic, defs, uses, loc, text)
    for l in lines[start + 1:]:
        if re.match(r"^_Z\w+:", l) or l.strip().startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            insts.append((m.group(1), None, [], [], loc, l))
            continue
        m = re.match(r"\s+([a-z_0-9]+)\s*(.*)", l)
        if not m or m.group(1).startswith(".") or not re.match(r"[svgdbf]", m.group(1)):
            continue
        mn, ops = m.group(1), m.group(2).split(";")[0]
        parts = [p.strip() for p in re.split(r",(?![^\[]*\])", ops) if p.strip()]
        defs, uses = [], []
        if mn.startswith("v_") and not mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_cmpx")) and parts:
            defs = regs_of(parts[0])
            uses = [r for p in parts[1:] for r in regs_of(p)]
            if mn.startswith(("v_writelane", "v_cndmask", "v_mov_b32_dpp")) or "dpp" in ops:
                uses += defs  # partial writes keep the old value live
        elif mn.startswith(("global_load", "buffer_load", "ds_read", "ds_bpermute", "ds_permute", "flat_load", "scratch_load", "ds_swizzle")) and parts:
            defs = regs_of(parts[0])
            uses = [r for p in parts[1:] for r in regs_of(p)]
        else:
            uses = [r for p in parts for r in regs_of(p)]
        insts.append((None, mn, defs, uses, loc, l.strip()))
    return insts


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    insts = parse(path, sym)
    # basic blocks
    leaders = [0] + [i for i, x in enumerate(insts) if x[0]] + [len(insts)]
    leaders = sorted(set(leaders))
    blocks = [(a, b) for a, b in zip(leaders, leaders[1:]) if a < b]
    label_block = {insts[a][0]: k for k, (a, b) in enumerate(blocks) if insts[a][0]}
    succ = collections.defaultdict(list)
    for k, (a, b) in enumerate(blocks):
        last = insts[b - 1]
        mn = last[1] or ""
        tgt = re.search(r"(\.LBB\w+)", last[5]) if mn.startswith(("s_branch", "s_cbranch")) else None
        if tgt and tgt.group(1) in label_block:
            succ[k].append(label_block[tgt.group(1)])
        if not mn.startswith(("s_branch", "s_endpgm", "s_setpc")) and k + 1 < len(blocks):
            succ[k].append(k + 1)
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks) - 1, -1, -1):
            a, b = blocks[k]
            live = set()
            for s in succ[k]:
                live |= live_in[s]
            for i in range(b - 1, a - 1, -1):
                _, mn, defs, uses, _, _ = insts[i]
                live -= set(defs)
                live |= set(uses)
            if live != live_in[k]:
                live_in[k] = live
                changed = True
    # per-instruction live counts
    last_def_loc = {}
    for x in insts:
        for r in x[2]:
            last_def_loc.setdefault(r, collections.Counter())[x[4]] += 1
    peaks = []
    for k, (a, b) in enumerate(blocks):
        live = set()
        for s in succ[k]:
            live |= live_in[s]
        for i in range(b - 1, a - 1, -1):
            _, mn, defs, uses, loc, txt = insts[i]
            peaks.append((len(live | set(defs)), i, loc, txt, sorted(live | set(defs))))
            live -= set(defs)
            live |= set(uses)
    peaks.sort(key=lambda t: -t[0])
    hist = collections.Counter(p[0] // 8 * 8 for p in peaks)
    print("live-VGPR histogram (instructions per band):", sorted(hist.items()))
    seen = set()
    shown = 0
    for n, i, loc, txt, regs in peaks:
        if loc in seen:
            continue
        seen.add(loc)
        print(f"\n{n} live at #{i} {loc}: {txt[:80]}")
        if shown < 2:
            for r in regs:
                c = last_def_loc.get(r, collections.Counter())
                print(f"   v{r}: defs at {[f'{f}:{ln}' for (f, ln), _ in c.most_common(3)]}")
        shown += 1
        if shown >= top:
            break


if __name__ == "__main__":
    main()
