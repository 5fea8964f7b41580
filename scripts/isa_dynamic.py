"""Estimated dynamic instruction profile of k_replay, by source line and function.

Combines (1) the gfx950 device ELF of the engine built with -g (instruction addresses, DWARF line
table, inlined-subroutine tree) with (2) gcov line counts of the CPU emulation (tests/emu) of the
same replay_core.h on the same input.  Every inlined instance of a Replayer function gets the share
of that function's executions its call site accounts for (recursively from run()), and each
instruction executes gcov(its line) x that share times.  Instructions of WaveGPU helpers (no gcov:
the emulator has its own backend) count once per call of their instance.  Approximate (a line with
several calls, loops inside helpers), but it ranks the hot code.

usage: python scripts/isa_dynamic.py ELF DIS DWARF LINES GCOV_DIR OPS [TOP]
  ELF: device code object (clang-offload-bundler --unbundle of `hipcc -g --cuda-device-only -c`)
  DIS: llvm-objdump -d --no-show-raw-insn; DWARF: llvm-dwarfdump --debug-info; LINES: --debug-line
  GCOV_DIR: *.gcov of an -O0 --coverage emulator run; OPS: ops replayed in that run"""
import collections
import os
import re
import sys

SYM = os.environ.get("ISA_SYM", "_ZN4crdt8k_replayILi32ELj1EEEvNS_5PoolsEjjjPKj")  # (k_replay<32, SHAPE_REMOTE>)
FILTER = int(os.environ.get("FILTER_CALL_LINE", "0"))
FN = os.environ.get("FILTER_FN", "")
DUMP = open(os.environ["DUMP_ADDR"], "w") if os.environ.get("DUMP_ADDR") else None  # per-instruction counts  # print this function's instructions (address, count/op)
LANE_CALLERS = os.environ.get("LANE_CALLERS")  # also rank context lane reads/writes by the line that asked for them
HELPER = re.compile(r"(E1gEj$|E1pEjj$|E3incEjj$|2xgEj$|2xsEjj$|6rdlaneE|6wrlaneE)")
MNS = tuple(x for x in os.environ.get("FILTER_MN", "").split(",") if x)  # only these mnemonic prefixes  # only code inlined from a call at this line


def load_dis(path):
    out, on = [], False
    for l in open(path):
        if l.startswith("0000"):
            on = SYM in l
            continue
        if not on:
            continue
        m = re.match(r"\s+([a-z_0-9]+)\b.*//\s*([0-9A-F]+):(?:.*<\w+\+0x([0-9a-f]+)>)?", l)
        if m:
            out.append((int(m.group(2), 16), m.group(1), int(m.group(3), 16) if m.group(3) else None))
    return out


def load_lines(path):
    files, rows, cur = {}, [], None
    for l in open(path):
        m = re.match(r"file_names\[\s*(\d+)\]:", l)
        if m:
            cur = int(m.group(1))
            continue
        m = re.match(r'\s+name: "([^"]+)"', l)
        if m and cur is not None:
            files[cur] = m.group(1)
            cur = None
            continue
        m = re.match(r"0x([0-9a-f]+)\s+(\d+)\s+\d+\s+(\d+)", l)
        if m:
            rows.append((int(m.group(1), 16), int(m.group(2)), int(m.group(3))))
    rows.sort()
    return files, rows


class Die:
    __slots__ = ("tag", "name", "ranges", "call_file", "call_line", "kids", "parent")

    def __init__(self, tag):
        self.tag, self.name, self.ranges, self.call_file, self.call_line = tag, None, [], None, None
        self.kids, self.parent = [], None


def load_dwarf(path):
    root = Die("root")
    stack = [(-1, root)]
    cur = None
    in_ranges = False
    for l in open(path):
        m = re.match(r"0x[0-9a-f]+:(\s+)(DW_TAG_\w+|NULL)", l)
        if m:
            depth = len(m.group(1))
            in_ranges = False
            if m.group(2) == "NULL":
                cur = None
                continue
            d = Die(m.group(2))
            while stack and stack[-1][0] >= depth:
                stack.pop()
            d.parent = stack[-1][1]
            d.parent.kids.append(d)
            stack.append((depth, d))
            cur = d
            continue
        if cur is None:
            continue
        m = re.search(r'DW_AT_(?:abstract_origin|linkage_name)\s+\((?:0x[0-9a-f]+ )?"([^"]+)"\)', l)
        if m and cur.name is None:
            cur.name = m.group(1)
        m = re.search(r"DW_AT_low_pc\s+\(0x([0-9a-f]+)\)", l)
        if m:
            cur.ranges.append([int(m.group(1), 16), None])
        m = re.search(r"DW_AT_high_pc\s+\(0x([0-9a-f]+)\)", l)
        if m and cur.ranges:
            cur.ranges[-1][1] = int(m.group(1), 16)
        if "DW_AT_ranges" in l:
            in_ranges = True
        if in_ranges:
            for a, b in re.findall(r"\[0x([0-9a-f]+), 0x([0-9a-f]+)\)", l):
                cur.ranges.append([int(a, 16), int(b, 16)])
        m = re.search(r'DW_AT_call_file\s+\("([^"]+)"\)', l)
        if m:
            cur.call_file = os.path.basename(m.group(1))
        m = re.search(r"DW_AT_call_line\s+\((\d+)\)", l)
        if m:
            cur.call_line = int(m.group(1))
    return root


def contains(d, a):
    return any(lo <= a < (hi if hi is not None else lo + 4) for lo, hi in d.ranges)


def load_gcov(d):
    out = {}
    for fn in ("replay_core.h", "crdt_types.h"):
        p = os.path.join(d, fn + ".gcov")
        c = {}
        for l in open(p):
            m = re.match(r"\s*([0-9]+|#####|=====)\*?:\s*(\d+):", l)
            if m:
                v = int(m.group(1)) if m.group(1)[0].isdigit() else 0
                c[int(m.group(2))] = max(c.get(int(m.group(2)), 0), v)
        out[fn] = c
    return out


def main():
    elf, dis, dwarf, lines, gdir, ops = sys.argv[1:7]
    ops = float(ops)
    top = int(sys.argv[7]) if len(sys.argv) > 7 else 50
    insts = load_dis(dis)
    files, rows = load_lines(lines)
    root = load_dwarf(dwarf)
    gc = load_gcov(gdir)
    kern = None
    stack = [root]
    while stack:
        d = stack.pop()
        if d.tag == "DW_TAG_subprogram" and d.name == SYM and d.ranges:
            kern = d
            break
        stack.extend(d.kids)
    assert kern, "kernel DIE not found"
    # instances of every inlined function, with their parent instance
    inst = []  # (die, parent_index)

    def walk(d, parent):
        for k in d.kids:
            if k.tag == "DW_TAG_inlined_subroutine":
                inst.append((k, parent))
                walk(k, len(inst) - 1)
            else:
                walk(k, parent)
    walk(kern, -1)
    # entries: gcov of the call line (replay_core / crdt_types call sites) x parent's share
    by_func = collections.defaultdict(list)
    for i, (d, p) in enumerate(inst):
        by_func[d.name].append(i)
    entries = [0.0] * len(inst)
    ratio = [1.0] * len(inst)
    order = sorted(range(len(inst)), key=lambda i: 0)  # parents precede children in walk order
    for i in order:
        d, p = inst[i]
        pr = ratio[p] if p >= 0 else 1.0
        g = gc.get(d.call_file, {}).get(d.call_line)
        if g is None:  # call site in the kernel body or a helper: once per parent entry
            g = entries[p] if p >= 0 else 1.0
            entries[i] = g
        else:
            entries[i] = g * pr
        ratio[i] = None  # filled below after all siblings of the same function are known
        # ratio of this instance among all instances of its function, computed lazily
        tot = sum(entries[j] for j in by_func[d.name] if j <= i) or 1.0
        ratio[i] = 1.0  # provisional
    for name, idx in by_func.items():
        tot = sum(entries[j] for j in idx) or 1.0
        for j in idx:
            ratio[j] = entries[j] / tot
    # second pass now that ratios exist (children entries depend on parent ratios)
    for _ in range(3):
        for i, (d, p) in enumerate(inst):
            g = gc.get(d.call_file, {}).get(d.call_line)
            pr = ratio[p] if p >= 0 else 1.0
            entries[i] = (g * pr) if g is not None else (entries[p] if p >= 0 else 1.0)
        for name, idx in by_func.items():
            tot = sum(entries[j] for j in idx) or 1.0
            for j in idx:
                ratio[j] = entries[j] / tot
    # per instruction
    import bisect
    addrs = [r[0] for r in rows]

    def line_of(a):
        k = bisect.bisect_right(addrs, a) - 1
        if k < 0:
            return ("?", 0)
        r = rows[k]
        return (os.path.basename(files.get(r[2], "?")), r[1])

    def chain(a):
        out, d = [], kern
        while True:
            nxt = None
            for k in d.kids:
                if k.tag in ("DW_TAG_inlined_subroutine", "DW_TAG_lexical_block") and contains(k, a):
                    nxt = k
                    break
            if nxt is None:
                return out
            if nxt.tag == "DW_TAG_inlined_subroutine":
                out.append(nxt)
            d = nxt
    die_index = {id(d): i for i, (d, p) in enumerate(inst)}
    # basic blocks (split at branch targets and after branches): one count per block, the median
    # of the gcov-derived estimates of its instructions (helper-only blocks: their entry estimate)
    start = insts[0][0] - 0  # function start address = first instruction
    targets = {start + t for _, _, t in insts if t is not None}
    blocks, cur = [], []
    for x in insts:
        if x[0] in targets and cur:
            blocks.append(cur)
            cur = []
        cur.append(x)
        if x[1].startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    kinds = collections.Counter()
    by_mn = collections.Counter()
    by_line = collections.defaultdict(collections.Counter)
    by_fn = collections.defaultdict(collections.Counter)
    prev_cnt = 0.0
    by_caller = collections.Counter()
    for blk in blocks:
        good, helper = [], []
        info = []
        for a, mn, _ in blk:
            fl, ln = line_of(a)
            ch = chain(a)
            info.append((fl, ln, ch))
            if fl in gc and ln in gc[fl] and ln > 0:
                rc = [d for d in ch if d.name and (("Replayer" in d.name) if fl == "replay_core.h" else True)]
                r = ratio[die_index[id(rc[-1])]] if rc else 1.0
                good.append(gc[fl][ln] * r)
            elif ch:
                helper.append(entries[die_index[id(ch[-1])]])
        if good:
            good.sort()
            cnt = good[len(good) // 2]
        elif helper and any(l > 0 for _, l, _ in info):
            cnt = min(helper)
        else:  # compiler-made block (copies at a merge): as the block before it
            cnt = prev_cnt
        prev_cnt = cnt
        for (a, mn, _), (fl, ln, ch) in zip(blk, info):
            if mn.startswith(("s_nop", "s_waitcnt")):
                continue
            if FILTER and not any(d.call_line == FILTER for d in ch):
                continue
            if MNS and not mn.startswith(MNS):
                continue
            kind = ("branch" if mn.startswith(("s_cbranch", "s_branch")) else "scratch" if mn.startswith("scratch_")
                    else "salu" if mn.startswith("s_")
                    else "lane" if mn.startswith(("v_readlane", "v_writelane", "v_readfirstlane"))
                    else "valu" if mn.startswith("v_") else "mem")
            fn = ch[-1].name if ch else SYM
            if DUMP is not None:
                DUMP.write(f"{a:#x} {cnt / float(sys.argv[6]):.6f} {mn} {fl}:{ln}\n")
            if FN and FN in fn:
                print(f"  {a:#x} {cnt / float(sys.argv[6]):6.3f} {mn:24s} {fl}:{ln}")
            kinds[kind] += cnt
            by_mn[mn] += cnt
            by_line[(fl, ln)][kind] += cnt
            by_fn[fn][kind] += cnt
            if LANE_CALLERS and kind == "lane":
                k = len(ch) - 1
                while k >= 0 and ch[k].name and HELPER.search(ch[k].name):
                    k -= 1
                site = (ch[k + 1].call_file, ch[k + 1].call_line) if k + 1 < len(ch) else (fl, ln)
                by_caller[site] += cnt
    tot = sum(kinds.values())
    print(f"estimated per op: total {tot / ops:.1f}  " + "  ".join(f"{k} {v / ops:.1f}" for k, v in kinds.items()))
    print("\nby mnemonic, per op:")
    for mn, c in by_mn.most_common(top):
        print(f"  {c / ops:7.2f}  {mn}")
    print("\nby function (innermost inlined instance), per op:")
    for fn, c in sorted(by_fn.items(), key=lambda kv: -sum(kv[1].values()))[:top]:
        print(f"  {sum(c.values()) / ops:7.2f}  salu {c['salu'] / ops:6.2f}  valu {c['valu'] / ops:6.2f}  lane {c['lane'] / ops:5.2f}  br {c['branch'] / ops:5.2f}  {fn[:90]}")
    if LANE_CALLERS:
        print("\ncontext lane reads/writes by requesting line, per op:")
        for (fl, ln), c in by_caller.most_common(top):
            print(f"  {c / ops:7.2f}  {fl}:{ln}")
    print("\nby source line, per op:")
    for (fl, ln), c in sorted(by_line.items(), key=lambda kv: -sum(kv[1].values()))[:top]:
        print(f"  {sum(c.values()) / ops:7.2f}  salu {c['salu'] / ops:6.2f}  valu {c['valu'] / ops:6.2f}  lane {c['lane'] / ops:5.2f}  br {c['branch'] / ops:5.2f}  {fl}:{ln}")


if __name__ == "__main__":
    main()
