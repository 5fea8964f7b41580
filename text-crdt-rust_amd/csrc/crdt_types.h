// Shared device/host types for the MI355X list-CRDT engine.
//
// Reference mapping (josephg/text-crdt-rust):
//   Span        == YjsSpan                         src/list/span.rs:5-119
//   CwoRun      == KVPair<CRDTSpan> (client_with_order)   src/list/mod.rs:63, range_tree/entry.rs:43-129
//   ARun        == KVPair<OrderSpan> (ClientData::item_orders)  mod.rs:42, order.rs:6-104
//   DelRun      == KVPair<DeleteEntry>             list/delete.rs:6-40
//   DDRun       == KVPair<DoubleDelete>            list/double_delete.rs:11-38
//   TxnRec      == TxnSpan (+ parents in a pool)   list/txn.rs:9-60
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace crdt {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef int32_t i32;
typedef uint64_t u64;
typedef int64_t i64;

#define CRDT_HD __host__ __device__ __forceinline__
// Event counters of the CPU emulation's statistics build (tests/emu stats: path counts for the
// design notes); nothing in the product builds.
#ifndef CRDT_MEM_EPOCH  // (emulator statistics build: one op's memory lines end here)
#define CRDT_MEM_EPOCH() ((void)0)
#endif
#ifndef CRDT_STAT
#define CRDT_STAT(k, v) ((void)0)
#endif
// Preconditions the replay relies on without testing them, checked by the CPU emulation (tests/emu
// defines CRDT_EMU_CHECKS: the emulator parity tests abort on a violation); nothing on the GPU.
#ifdef CRDT_EMU_CHECKS
#define CRDT_EXPECT(c) do { if (!(c)) { fprintf(stderr, "replay precondition failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); abort(); } } while (0)
#else
#define CRDT_EXPECT(c) ((void)0)
#endif

constexpr u32 ROOT_ORDER = 0xFFFFFFFFu;   // list/mod.rs:30
constexpr u32 ROOT_AGENT = 0xFFFFu;       // "ROOT" -> AgentId::MAX (doc.rs:68)
constexpr u32 UNKNOWN_AGENT = 0xFFFEu;    // a name that is not (yet) interned for this document
constexpr u32 INVALID = 0xFFFFFFFFu;
constexpr u32 VS_BAD = 0x80000000u;       // the cached leaf's visible start is unknown (no position is in range)

constexpr u32 GROUP = 64;                 // directory slots per block (one wavefront)
// Root level of the directory: one group (block id, slot count, visible count) per directory
// block, held in LDS while a wave replays its document.  Its size per wave is chosen per launch
// (a multiple of 64 groups, 12 B each): a single one-wave workgroup may declare all 160 KiB of a
// CU's LDS, so a document can have up to ROOT_CAP_MAX blocks = at least 32*(ROOT_CAP_MAX-1)
// leaves (every block but the first holds >= 32 slots) = 13.9M entries at the release layout.
constexpr u32 ROOT_CAP_MIN = 256;
// (the two-level root's top entries: 12 B each + two words + the agent ranks + the prefetch row +
// the double-delete top level within 160 KiB, floor((163840 - 8 - 4 * (RANK_LDS + PF_LDS + DDT_LDS))
// / 12 / 64) * 64; static_assert below)
constexpr u32 ROOT_CAP_MAX = 13568;
// The flat LDS root also keeps a block -> group map (4 B per group: 16 B per group in all), so its
// largest class is floor((163840 - 4 * (RANK_LDS + PF_LDS + DDT_LDS)) / 16 / 64) * 64 groups; documents past it use
// the two-level root.
constexpr u32 ROOT_CAP_LDS = 10176;
// Agent ranks (the integrate tie-break's name order, doc.rs:207) of documents with at most
// RANK_LDS agents sit in LDS next to the root while a wave replays (integrate's scan reads one per
// scanned entry); documents with more read them from HBM.
constexpr u32 RANK_LDS = 64;
// A wave's LDS slice (kernels.h wave_with_root): a 512 B leaf row integrate's scan prefetches the
// successor leaf into (LDS-DMA), the root (flat: blk / cnt / vis / block -> group map, 4 u32 per
// group; two-level: 3 u32 per top entry + 2 words) and the agent ranks; 16 B aligned.
constexpr u32 PF_LDS = 128;
// The double-delete directory's top level (replay_core.h dd_upper): word j = the first key of
// block 64 j, for documents with at most 64 * DDT_LDS blocks (others search the directory in HBM).
// (32 words: the smallest root class's 4-wave workgroup stays within 1/8 of the CU's LDS, so
// 8 waves per SIMD stay resident)
#ifndef CRDT_DDT_LDS
#define CRDT_DDT_LDS 32  // (the emulator's test build shrinks it to cross the threshold: tests/emu Makefile ddt)
#endif
constexpr u32 DDT_LDS = CRDT_DDT_LDS;
CRDT_HD constexpr u32 wave_lds_words(u32 rcap, bool hr) {
  return (PF_LDS + (hr ? 3u * rcap + 2u : 4u * rcap) + RANK_LDS + DDT_LDS + 3u) & ~3u;
}
static_assert(8u * 4u * 4u * wave_lds_words(ROOT_CAP_MIN, false) <= 163840u, "smallest root class: 8 waves per SIMD fit the LDS");
static_assert(4u * wave_lds_words(ROOT_CAP_MAX, true) <= 163840u, "two-level root: one wave's LDS fits 160 KiB");
static_assert(4u * wave_lds_words(ROOT_CAP_LDS, false) <= 163840u, "flat root: one wave's LDS fits 160 KiB");
// Past it the root has two levels (wave_gpu.h HR): LDS top entries of rows that hold 32..64 groups
// each in HBM, up to ROOT_CAP_MAX - 64 top entries (LDS: 12 B each + two words) -- over 434k
// groups, 13.9M leaves, 445M entries at the release layout.
constexpr u32 HROOT_ROW = 192;            // u32 per HBM root row: blk[64], cnt[64], vis[64]
constexpr u32 FRONTIER_CAP0 = 4;          // initial frontier capacity (grows on demand)

// Status codes (identical to include/crdt_gpu.h and the oracle)
enum : i32 {
  ST_OK = 0,
  ST_POS_OOB = -1,
  ST_SEQ = -2,
  ST_UNKNOWN_AGENT = -3,
  ST_UNKNOWN_ID = -4,
  ST_NONTERMINATING = -5,
  ST_CAPACITY = -6,
  ST_EMPTY_TXN = -7,
  ST_FRONTIER = -8,
  ST_BAD_INPUT = -9,
  ST_INTERNAL = -10,
  ST_NEED_CAPACITY = -11,  // resumable: the txn at rec_pos was not started; grow (cap_need) and relaunch
};

struct Span {  // YjsSpan, 16 B
  u32 order, ol, orr;
  i32 len;
};

CRDT_HD u32 slen(const Span& s) { return (u32)(s.len < 0 ? -s.len : s.len); }
CRDT_HD u32 clen(const Span& s) { return s.len > 0 ? (u32)s.len : 0u; }
CRDT_HD i32 sgn(i32 x) { return (x > 0) - (x < 0); }
CRDT_HD u32 origin_left_at_offset(const Span& s, u32 at) { return at == 0 ? s.ol : s.order + at - 1; }
CRDT_HD Span truncate(Span& s, u32 at) {  // span.rs:33-45
  i32 at_s = (i32)at * sgn(s.len);
  Span o{s.order + at, s.order + at - 1, s.orr, s.len - at_s};
  s.len = at_s;
  return o;
}
CRDT_HD Span truncate_keeping_right(Span& s, u32 at) {  // span.rs:68-85
  i32 at_s = (i32)at * sgn(s.len);
  Span o{s.order, s.ol, s.orr, at_s};
  s.order += at;
  s.ol = s.order - 1;
  s.len -= at_s;
  return o;
}
// An opaque copy of a wave-uniform integer: the compiler cannot see it is a 0/1 compare result,
// so it stays a u32 in an SGPR (one s_cmp to branch on) instead of a 64-bit lane mask that every
// later use re-combines with exec.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ u32 opq(u32 x) {
  x = __builtin_amdgcn_readfirstlane(x);  // (free for a value already in an SGPR)
  asm("" : "+s"(x));
  return x;
}
#else
inline u32 opq(u32 x) { return x; }
#endif
CRDT_HD bool can_append(const Span& a, const Span& b) {  // span.rs:47-53
  return ((a.len > 0) == (b.len > 0)) && b.order == a.order + slen(a) && b.ol == b.order - 1 && b.orr == a.orr;
}
// ... branch-free, for per-lane operands (bitwise: && on lane values compiles to exec-masked branches)
CRDT_HD bool can_append_b(const Span& a, const Span& b) {
  return ((a.len > 0) == (b.len > 0)) & (b.order == a.order + slen(a)) & (b.ol == b.order - 1) & (b.orr == a.orr);
}
// The same test as early exits, for wave-uniform operands (the replay's scalar code): a branch per
// condition instead of lane-mask booleans.  (can_append stays branch-free for lane-parallel use.)
CRDT_HD bool can_append_u(const Span& a, const Span& b) {
  // (a.len > 0) == (b.len > 0) as integer sign bits ((u32)-len >> 31 = len > 0 for |len| < 2^31):
  // one compare and branch instead of two booleans combined as lane masks
  if (((u32)(-a.len) >> 31) != ((u32)(-b.len) >> 31)) return false;
  if (b.order != a.order + slen(a)) return false;
  if (b.ol != b.order - 1) return false;
  return b.orr == a.orr;
}

struct CwoRun { u32 key, agent, seq, len; };   // client_with_order
struct ARun { u32 key, order, len, pad; };     // item_orders of one agent (seq -> order)
struct DelRun { u32 key, order, len; };        // deletes
struct DDRun { u32 key, len, excess; };        // double_deletes
// The double-delete RLE is kept in 64-entry blocks (physical block p = entries [64p, 64p+64))
// ordered by a block directory, so an insertion shifts one block, not the table's tail.
constexpr u32 DD_BLK = 64;
struct DDBlk { u32 phys, first, cnt, pad; };   // physical block, first key, entries
struct TxnRec { u32 order, len, shadow, poff, pn, pad[3]; };  // txns (32 B)
// Per-document agent table.  tkey / torder / tlen: a copy of the agent's last item_orders run
// (valid when run_cnt > 0), written whenever it stops being the replay's current author, so
// switching authors is one 32 B load instead of the record and then its last run.
struct AgentRec { u32 run_base, run_cnt, run_cap, rank, tkey, torder, tlen, pad; };
struct GroupRec { u32 blk, cnt, vis, pad; };   // persisted root level of the directory

// ---------------------------------------------------------------------------------------------
// Op record stream (16 B records, per document, in causal order)
// ---------------------------------------------------------------------------------------------
enum : u32 { REC_LTXN = 1, REC_LOP = 2, REC_RTXN = 3, REC_RINS = 4, REC_RDEL = 5, REC_RPARENT = 6, REC_GEN = 7,
             REC_RC = 8, REC_LC = 9, REC_PROBE = 10 };
struct Rec { u32 w0, w1, w2, w3; };
// LTXN    w0 = kind<<28 | n_ops         w1 = agent                  w2 = sum(del) w3 = txn_len
// LOP     w0 = kind<<28                 w1 = pos                    w2 = del   w3 = ins
// RTXN    w0 = kind<<28 | zero_op<<27 | has_del<<26 | n_ops (26b)
//                                       w1 = agent | n_parents<<16  w2 = seq   w3 = txn_len
// RINS    w0 = kind<<28 | len (28b)     w1 = ol_agent | or_agent<<16  w2 = ol_seq  w3 = or_seq
// RDEL    w0 = kind<<28 | len (28b)     w1 = agent                  w2 = seq
// RPARENT w0 = kind<<28                 w1 = agent                  w2 = seq
// GEN     w0 = kind<<28                 w1 = agent                  w2 = n_ops w3 = seed
// (remote ops follow their RTXN, then the txn's RPARENT records; a GEN record expands on the
//  device into n_ops local txns of one LocalOp each, see gen_op)
// Compact one-record txns (the common shape of real traces: 16 B per op instead of 48 / 32):
// RC      w0 = kind<<28 | del<<27 | len<<16 (11 b, 1..2047) | author
//                                       w1 = seq   w2 = ins: origin_left seq, del: target seq
//                                                  w3 = ins: origin_right seq
//         one RemoteOp; its origins / target are the author's items (a seq of 0xFFFFFFFF names
//         ROOT); the one parent is (author, seq - 1)
// LC      w0 = kind<<28 | agent (16 b)  w1 = pos   w2 = del   w3 = ins   (one LocalOp)
// PROBE   w0 = kind<<28                 w1 = pos   w2 = agent w3 = seq
//         answers pos -> (agent, seq) and (agent, seq) -> (pos, deleted) on the state reached so far
//         (config 1's per-op check); the answer goes to probe_out[record index]
CRDT_HD u32 rec_kind(const Rec& r) { return r.w0 >> 28; }
// Stream shapes (Replayer::run<SH>): which record kinds a document's staged stream holds.  The
// host classifies every stream at staging and launches each shape in its own k_replay instance.
enum : u32 { SHAPE_ALL = 0, SHAPE_REMOTE = 1, SHAPE_GEN = 2, SHAPE_LOCAL = 3, N_SHAPES = 4 };
CRDT_HD constexpr u32 shape_kinds(u32 sh) {
  return sh == SHAPE_REMOTE ? (1u << REC_RTXN | 1u << REC_RINS | 1u << REC_RDEL | 1u << REC_RPARENT | 1u << REC_RC)
       : sh == SHAPE_GEN ? (1u << REC_GEN)
       : sh == SHAPE_LOCAL ? (1u << REC_LTXN | 1u << REC_LOP | 1u << REC_LC | 1u << REC_PROBE)
       : 0xFFFFFFFFu;
}
// the narrowest shape holding a stream whose record kinds are the bits of `kinds`
inline u32 shape_of_kinds(u32 kinds) {
  if ((kinds & ~shape_kinds(SHAPE_REMOTE)) == 0u) return SHAPE_REMOTE;
  if ((kinds & ~shape_kinds(SHAPE_GEN)) == 0u) return SHAPE_GEN;
  if ((kinds & ~shape_kinds(SHAPE_LOCAL)) == 0u) return SHAPE_LOCAL;
  return SHAPE_ALL;
}
// RTXN header: has_del (a delete op follows: the double-delete reserve applies, fits()) and n_ops
constexpr u32 RTXN_DEL_BIT = 26, RTXN_NOPS_MASK = 0x03FFFFFFu;
constexpr u32 RC_HDR_MASK = 0xF800FFFFu;  // kind | del | author (not len)
CRDT_HD u32 rc_len(const Rec& r) { return (r.w0 >> 16) & 0x7FFu; }
// the general records a compact txn stands for (header, op, parent)
CRDT_HD void expand_rc(const Rec r, Rec& h, Rec& o, Rec& pr) {  // (r by value: h may alias it)
  u32 a = r.w0 & 0xFFFFu, len = rc_len(r);
  h = Rec{(REC_RTXN << 28) | (((r.w0 >> 27) & 1u) << RTXN_DEL_BIT) | 1u, a | (1u << 16), r.w1, len};
  if ((r.w0 >> 27) & 1u) {
    o = Rec{(REC_RDEL << 28) | len, a, r.w2, 0u};
  } else {
    u32 la = r.w2 == 0xFFFFFFFFu ? ROOT_AGENT : a, ra = r.w3 == 0xFFFFFFFFu ? ROOT_AGENT : a;
    o = Rec{(REC_RINS << 28) | len, la | (ra << 16), r.w2, r.w3};
  }
  pr = Rec{REC_RPARENT << 28, a, r.w1 - 1u, 0u};
}
CRDT_HD void expand_lc(const Rec r, Rec& h, Rec& o) {
  h = Rec{(REC_LTXN << 28) | 1u, r.w0 & 0xFFFFu, r.w2, r.w2 + r.w3};
  o = Rec{REC_LOP << 28, r.w1, r.w2, r.w3};
}

CRDT_HD u64 mix64(u64 z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// On-device edit generator (BASELINE config 4).  Semantics of the reference's
// make_random_change (doc.rs:544-569): insert with probability 0.55 while len < 100, else 0.45
// (always when empty); insert 1 char at U[0, len]; delete U[1, min(10, len - pos)] chars at
// U[0, len - 1].  The reference's SmallRng stream is Rust-only, so draws come from a counter-based
// hash of (seed, op#) with fixed-point thresholds: integer-exact on the device and in the oracle.
// Returns the LOP record of op `i` for a document of visible length `len`.
// The draws of op i: r = mix64(seed << 32 | i) (hi, lo halves) and r2 = low half of mix64(r).
// They do not depend on the document, so the replay computes 64 ops' draws lane-parallel.
struct GenDraw { u32 hi, lo, r2; };
CRDT_HD GenDraw gen_draw(u32 seed, u32 i) {
  u64 r = mix64(((u64)seed << 32) | i);
  return GenDraw{(u32)(r >> 32), (u32)r, (u32)mix64(r)};
}
// The LocalOp of a draw for a document of visible length len.
CRDT_HD Rec gen_op_of(u32 hi, u32 lo, u32 r2, u32 len) {
  u32 thr = len < 100u ? 0x8CCCCCCDu : 0x73333333u;  // 0.55 / 0.45 of 2^32
  if (len == 0u || hi < thr) return Rec{REC_LOP << 28, (u32)(((u64)lo * (len + 1u)) >> 32), 0u, 1u};
  u32 p = (u32)(((u64)lo * len) >> 32);
  u32 mx = len - p < 10u ? len - p : 10u;
  return Rec{REC_LOP << 28, p, 1u + (u32)(((u64)r2 * mx) >> 32), 0u};
}
CRDT_HD Rec gen_op(u32 seed, u32 i, u32 len) {
  GenDraw d = gen_draw(seed, i);
  return gen_op_of(d.hi, d.lo, d.r2, len);
}

// ---------------------------------------------------------------------------------------------
// Per-document segments (host-assigned, read-only during replay) and mutable header
// ---------------------------------------------------------------------------------------------
// DOC_TRACK_MAP: the document keeps its order -> leaf map (the SplitList replacement), which only
// remote ops read (find_order); documents that only ever apply local ops skip it entirely.
// DOC_TRACK_AGENT: the document also keeps an order -> agent map (u16 per order, same slots as the
// order -> leaf map): documents with several agents, whose integrate ties read the agent of an
// entry's first order (doc.rs:207) -- one load instead of a client_with_order search.
enum : u32 { DOC_TRACK_MAP = 1u, DOC_TRACK_AGENT = 2u };

struct DocSeg {
  u64 leaf_base;   // first leaf (pool index) of this doc; entries at leaf_base*L
  u64 blk_base;    // first directory block; slots at blk_base*64
  u64 map_base;    // order -> leaf table (u32 per order)
  u64 cwo_base, arun_base, del_base, dd_base, txn_base, par_base, fr_base, agent_base, grp_base;
  // dd_base / dd_cap count double-delete BLOCKS: directory at ddb[dd_base], entries at dd[dd_base*64]
  u64 rec_base;    // first record of this call's stream
  u32 leaf_cap, blk_cap, map_cap, cwo_cap;
  u32 arun_cap, del_cap, dd_cap, txn_cap;
  u32 par_cap, agent_cap, rec_n, flags;
  u32 fr_cap, grp_cap;  // frontier heads; root groups (= blk_cap)
  // published index (k_publish): canonical spans + vpos + rank -> span at canon_base (canon_cap
  // spans); the span-start bitmap and its per-word prefix at pub_base (2 x pub_words(ord_cap)
  // words); text (k_materialize) at ord_base (ord_cap code points); ord_cap > every order
  u64 canon_base, pub_base, ord_base;
  u32 canon_cap, ord_cap;
  u64 hrow_base;   // two-level root documents: first row (192 u32 each) of the HBM root rows
};
CRDT_HD u32 pub_words(u32 ord_cap) { return ord_cap / 32u + 1u; }

struct DocState {
  i32 status;
  u32 rec_pos;     // records of the current stream already applied (resume point)
  u32 n_leaves, n_blocks;
  u32 ng, next_order, len, n_cwo;
  u32 n_del, n_dd, n_txn, n_par;
  u32 n_fr, n_agents, n_items, cap_need;
  u32 n_entries, gen_done;  // gen_done: ops of the current GEN record applied
  u32 n_ddb;                // double-delete blocks in use
  u32 prof0, prof1, prof2, prof3;  // diagnostic cycle counters (-DCRDT_PROF builds only)
};

// Per-leaf cache of the agents of the leaf's entries (read by DOC_TRACK_AGENT documents): word 0 = 1 when
// the row is current, words [lag_words/2, +L/2) = the agent of entry j's first order (u16, two
// per word).  integrate's scan reads one row per leaf instead of one order -> agent map line per
// entry; a commit of the leaf (or its creation) clears word 0, the scan rewrites a stale row.
constexpr u32 lag_words(int L) { return L >= 16 ? (u32)L : 16u; }
// The row's scan summary (written with it, current with it): word LAG_EPOCH = the agent count its
// ranks are of (| LAG_MIXED when the entries' origin_left differ or the leaf is empty), LAG_OL =
// the entries' common origin_left, LAG_RANK = their highest agent rank, [LAG_OMIN, LAG_OMAX] = the
// range of their first orders.  integrate's scan passes a leaf with a summary of X / rank below
// its own / orr outside the range unread (replay_core.h skip_leaves).
enum : u32 { LAG_EPOCH = 1, LAG_OL = 4, LAG_RANK = 5, LAG_OMIN = 6, LAG_OMAX = 7 };
constexpr u32 LAG_MIXED = 0x80000000u;
static_assert(LAG_OMAX < lag_words(4) / 2, "summary words before the agent words");
struct Pools {
  Span* leaves;        // [leaf][L]
  u32* dir_leaf;       // [blk*64 + i]
  u32* dir_vis;
  u32* slot_of_leaf;   // [2 * (leaf_base + leaf)] = blk<<6 | i, [+1] = successor leaf (END_LEAF: last)
  u32* leaf_of;        // [map_base + order]
  u16* agent_of;       // [map_base + order] (DOC_TRACK_AGENT documents)
  u32* leaf_agents;    // [(leaf_base + leaf) * lag_words(L)]: integrate's scan cache, see lag_words
  CwoRun* cwo;
  ARun* arun;
  DelRun* dels;
  DDRun* dd;
  DDBlk* ddb;
  uint4* probe;        // [rec_base + record]: answers of PROBE records (nullptr: none staged)
  TxnRec* txns;
  u32* parents;
  u32* frontier;       // [fr_base .. + fr_cap]
  AgentRec* agents;
  GroupRec* groups;    // [grp_base .. + grp_cap]
  u32* hrows;          // [hrow_base * 192 ..]: two-level root rows (kernels launched with an HBM root)
  u32* gsob;           // [blk_base + block]: row << 6 | slot of each block's group (same)
  const Rec* recs;
  const DocSeg* seg;
  DocState* st;
};

}  // namespace crdt
