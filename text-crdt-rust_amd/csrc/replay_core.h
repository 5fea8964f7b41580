// Wave-per-document replay of list-CRDT transactions (local + remote) on the MI355X.
//
// This is the B-tree replacement.  The reference keeps a 16-ary B-tree of YjsSpan runs with
// 32-entry leaves (src/range_tree/*) plus an order->leaf SplitList (src/split_list).  Here a
// document is:
//   * leaves of L entries (L = 32 release / 4 debug) in HBM, with *exactly* the reference's
//     leaf-level mutation rules (insert_internal / split_at / mutate_entry), so the entry layout
//     -- which leaks into results through YjsSpan::prepend (span.rs:61-64 keeps origin_left) and
//     the integrate tie-break (doc.rs:207) -- is bit-identical to the reference's;
//   * a two-level wave directory instead of internal nodes: 64-slot blocks (leaf id + visible
//     count) in HBM and a root level of up to 256 groups in LDS, so every descent is two
//     wave-wide scans and every leaf insertion one 64-lane shift;
//   * a write-back leaf cache in VGPRs (lane i = entry i) that also remembers its directory slot
//     and visible count, so runs of edits in one leaf touch neither HBM loads nor the directory;
//     lookups that only need a position in another leaf (integrate's origin compare, the item
//     after the end of a leaf) peek at that leaf without evicting the cached one;
//   * an order->leaf table (u32 per order) replacing the SplitList, written only when a run
//     changes leaf (the reference's notify() semantics);
//   * write-back tails of every RLE table (client_with_order, the author's item_orders,
//     deletes, txns, frontier[0]) kept on chip (a coalescing append costs no store; the tail is
//     written when a new run starts and at the end), the cached leaf's successor and its first
//     order, and a 64-record prefetch of the op stream: the common op issues no dependent HBM
//     load at all and one store (its order -> leaf entry).  On CDNA4 stores count in vmcnt, so
//     every store avoided also shortens the next dependent load's wait.
//
// Code shape (what makes this fast on CDNA4):
//   * one op interpreter loop per document in which every heavy routine -- integrate's scan,
//     mutate_entry, insert_internal, split_at -- has exactly ONE inlined instance;
//   * every piece of per-document state that lives across ops (table pointers, capacities,
//     DocState, cache bookkeeping, RLE tails) sits in two "context" VGPRs, one field per lane,
//     read with v_readlane and written with v_writelane at compile-time lane numbers.  Only
//     op-transient values are SGPRs, so control-flow merges in the interpreter do not shuffle
//     ~90 scalar registers around (which is what the compiler does with SSA state this size).
// Control flow is wave-uniform; every lane-parallel step goes through the backend W:
//   W = WaveGPU (wave_gpu.h, the product) or WaveCPU (tests/emu, a test-only emulation used to
//   debug this file against the oracle without a GPU).
#pragma once
#include "crdt_types.h"

namespace crdt {

struct Cursor {
  u32 leaf, idx, off;
};
constexpr u32 END_LEAF = 0xFFFFFFFEu;  // memoised "no successor leaf"

// Context slots: lane numbers of the three context VGPRs (f / 64 = the register).  x0 holds what
// the replay never writes (table pointers, capacities), so writes to the others do not make the
// compiler re-read it (a v_writelane defines a new value of its whole register); x1 DocState and
// the per-call flags; x2 the leaf cache bookkeeping and the RLE tails.
enum : u32 {
  // x0: table pointers, 2 slots each, and capacities (read-only while a document replays)
  P_LV = 0, P_DL = 2, P_DV = 4, P_SOL = 6, P_LOF = 8, P_CWO = 10, P_ARUN = 12, P_DELS = 14,
  P_DD = 16, P_TXNS = 18, P_PAR = 20, P_FR = 22, P_AGENTS = 24, P_GROUPS = 26, P_RECS = 28, P_STP = 30,
  P_DDB = 32,             // (2 slots) double-delete block directory
  P_PROBE = P_DDB + 2,    // (2 slots) probe answers
  K_LEAF = P_PROBE + 2, K_MAP, K_CWO, K_TXN, K_DEL, K_DD, K_PAR, K_RECN,
  K_FR,                   // frontier capacity
  P_OAG,                  // (2 slots) order -> agent map
  K_AGMAP = P_OAG + 2,    // 1: the document keeps the order -> agent map (DOC_TRACK_AGENT)
  P_LAG,                  // (2 slots) leaf agent rows (crdt_types.h lag_words)
  // x1: DocState, field for field (struct order), then the per-call flags
  S_BASE = 64,
  S_STATUS = 64, S_REC_POS, S_N_LEAVES, S_N_BLOCKS, S_NG, S_NEXT_ORDER, S_LEN, S_N_CWO, S_N_DEL,
  S_N_DD, S_N_TXN, S_N_PAR, S_N_FR, S_N_AGENTS, S_N_ITEMS, S_CAP_NEED, S_N_ENTRIES, S_GEN_DONE, S_N_DDB,
  S_PROF0, S_PROF1, S_PROF2, S_PROF3,  // -DCRDT_PROF: cycles in typing / general / delete / insert paths
  // 1: the txn-level invariants fast_txn_ok checks hold (set by a fast commit, cleared by apply_txn)
  F_FAST,
  // a one-insert txn the fast path resolved but could not place (no free leaf for its split):
  // flag, the item (4) and the cursor after its origin_left (3), handed to apply_txn.  Context
  // lanes, not registers: this is the rare path, and registers live around the replay loop are
  // what the 8-waves/SIMD budget spills.
  F_PRE, PRE_ITEM, PRE_C = PRE_ITEM + 4,
  F_GEN = PRE_C + 3,  // the record being replayed is a GEN record (generated ops)
  T_RB_BASE,
  // While F_FAST is set, the client_with_order / txns tail lengths and frontier[0] are kept as of
  // next_order == F_BASE: fast commits only advance next_order (and the author's item_orders
  // tail, which the fast path reads); materialize_tails() brings them up to date.
  F_BASE,
  // Frontier heads 1..n_fr-1 while n_fr <= FR_LANES + 1 (head 0 is T_FR0): slot FR_S0 + k - 1 holds
  // head k.  A concurrent history's frontier (one head per active agent) is then advanced in the
  // context register, with no dependent HBM load per remote txn; the HBM array is written back
  // with the tails (flush_tails) and holds larger frontiers.
  FR_S0 = 104,
  // x2: leaf cache bookkeeping
  C_LEAF = 128, C_N, C_VIS, C_NOW, C_BLK, C_I, C_VSTART, C_DIRTY, C_VS_OK /* (unused) */,
  C_SUCC, C_SUCC_ORD,  // successor leaf of the cached one (INVALID: not known) + its first order (INVALID: not known)
  // RLE tails
  T_CWO_KEY, T_CWO_AGENT, T_CWO_SEQ, T_CWO_LEN,
  T_DEL_KEY, T_DEL_ORDER, T_DEL_LEN,
  T_TX_ORDER, T_TX_LEN, T_TX_SHADOW,
  T_FR0,
  T_AG_ID, T_AG_BASE, T_AG_CNT, T_AG_CAP,
  T_AGL_KEY, T_AGL_ORDER, T_AGL_LEN,
  // the last non-author agent seq_to_order looked up: its item_orders runs (base, count).  Valid
  // while that agent authors nothing (use_agent drops it when it becomes the author).
  T_OA_ID, T_OA_BASE, T_OA_CNT,
  // the author's item_orders run before its tail (a txn that starts a run retires the tail to
  // it): a remote txn's parent is usually its author's previous item, which is there.  Valid
  // while the author stays (use_agent clears it; T_AGP_LEN = 0: none)
  T_AGP_KEY, T_AGP_ORDER, T_AGP_LEN,
  // ... and that non-author agent's last run (its record's copy; T_OA_LEN = 0: none)
  T_OA_KEY, T_OA_ORDER, T_OA_LEN,
  N_SLOTS
};
static_assert(P_LAG + 1 < 64, "read-only slots live in the first context register");
static_assert(S_PROF3 - S_BASE + 1 == sizeof(DocState) / 4, "DocState slot mirror");
static_assert(F_BASE < FR_S0, "DocState and the flags live in the second context register, below the frontier heads");
constexpr u32 FR_LANES = 128u - FR_S0;  // frontier heads kept in context lanes
static_assert(N_SLOTS <= 192, "three context registers");

template <class W, int L>
struct Replayer {
  W w;  // owned by value: its lane registers stay SSA values, never a scratch object
  // record format of the txn fast_txn is working on: compact one-record txns (RC / LC) or the
  // general header + ops (+ parents) form
  u32 cpt = 0;
  CRDT_HD u32 per_txn(u32 remote) const { return cpt ? 1u : (remote ? 3u : 2u); }
  // the op record of the one-op txn at window slot b
  CRDT_HD Rec op_at(u32 b, u32 remote) const {
    Rec r = w.rec_get(cpt ? b : b + 1u);
    if (!cpt) return r;
    Rec h, o, pr;
    if (remote) expand_rc(r, h, o, pr);
    else expand_lc(r, h, o);
    return o;
  }
#ifdef CRDT_PROF
  u32 prof_cat = 0;  // diagnostic: which fast path ran (0 typing, 2 delete, 3 insert)
  u32 prof_mode = 0; // document d % 4: 0 cycles, 1 calls, 2 txns per path, 3 detail (below)
  u32 prof_gen = 0;  // generated ops (config 4): detail = gen / fast path / cursor / leaf switch
  u32 prof_cur = 0, prof_sw = 0;  // cycles in cursor_at_content_pos and in its leaf switches
  u64 prof_t2 = 0;    // (compact local loop detail)
  u32 prof_split = 0;  // cycles in split_at (-DCRDT_PROF_LOOP: detail of fast_deletes' leaf-split loop)
  // -DCRDT_PROF_TXN: apply_txn's cycles by part (txn bookkeeping / integrate's scan / deletes /
  // op fetch + origins + insert_internal), added to the DocState counters of d % 4 == 3 documents
  u32 pt_scan = 0, pt_del = 0, pt_ins = 0;
#endif
#ifdef CRDT_EMU_STATS
  u32 st_prev_leaf = INVALID;  // (statistics build: the leaf cached before the current one)
#endif

  // ------------------------------------------------------------------ context access
  CRDT_HD u32 g(u32 f) const { return w.xg(f); }
  CRDT_HD void p(u32 f, u32 v) { w.xs(f, v); }
  CRDT_HD void inc(u32 f, u32 d = 1) { w.xs(f, w.xg(f) + d); }
  // (W::gptr tells the compiler the address is global memory: global_load/store, not flat)
  template <class T> CRDT_HD T* ptr(u32 f) const { return w.template gptr<T>(((u64)w.xg(f + 1) << 32) | w.xg(f)); }
  CRDT_HD void pset(u32 f, const void* q) {
    u64 v = (u64)q;
    w.xs(f, (u32)v);
    w.xs(f + 1, (u32)(v >> 32));
  }
  CRDT_HD Span* lv() const { return ptr<Span>(P_LV); }
  CRDT_HD u32* dl() const { return ptr<u32>(P_DL); }
  CRDT_HD u32* dv() const { return ptr<u32>(P_DV); }
  CRDT_HD u32* sol() const { return ptr<u32>(P_SOL); }
  CRDT_HD u32* lof() const { return ptr<u32>(P_LOF); }
  CRDT_HD u16* oag() const { return ptr<u16>(P_OAG); }
  CRDT_HD u32* lagp(u32 leaf) const { return w.template at<lag_words(L)>(ptr<u32>(P_LAG), leaf); }
  // a leaf's agent row is no longer current (its entries change, or it is new).  (Every document
  // has the rows; only documents that read them store: a lane predicate, where a branch on
  // K_AGMAP at every commit cost the register budget.)
  CRDT_HD void lag_stale(u32 leaf) {
    if (g(K_AGMAP)) w.st(lagp(leaf), 0u);  // (a uniform branch: local-only documents skip the address too)
  }
  CRDT_HD CwoRun* cwo() const { return ptr<CwoRun>(P_CWO); }
  CRDT_HD ARun* arun() const { return ptr<ARun>(P_ARUN); }
  CRDT_HD DelRun* dels() const { return ptr<DelRun>(P_DELS); }
  CRDT_HD DDRun* dd() const { return ptr<DDRun>(P_DD); }
  CRDT_HD DDBlk* ddb() const { return ptr<DDBlk>(P_DDB); }
  CRDT_HD TxnRec* txns() const { return ptr<TxnRec>(P_TXNS); }
  CRDT_HD u32* par() const { return ptr<u32>(P_PAR); }
  CRDT_HD u32* fr() const { return ptr<u32>(P_FR); }
  CRDT_HD AgentRec* agents() const { return ptr<AgentRec>(P_AGENTS); }
  CRDT_HD GroupRec* groups() const { return ptr<GroupRec>(P_GROUPS); }
  CRDT_HD const Rec* recs() const { return ptr<const Rec>(P_RECS); }
  CRDT_HD DocState* stp() const { return ptr<DocState>(P_STP); }
  CRDT_HD i32 status() const { return (i32)g(S_STATUS); }
  CRDT_HD u32 rec_n() const { return g(K_RECN); }

  CRDT_HD Replayer(const Pools& P, u32 d, const W& w0 = W()) : w(w0) {
#ifdef CRDT_PROF
    prof_mode = d & 3u;
#endif
    DocSeg sg = w.ld_seg(P.seg + d);
    w.bind_root(P, sg);  // (the two-level root's HBM rows, for documents past the LDS root)
    pset(P_LV, P.leaves + sg.leaf_base * (u64)L);
    pset(P_DL, P.dir_leaf + sg.blk_base * (u64)GROUP);
    pset(P_DV, P.dir_vis + sg.blk_base * (u64)GROUP);
    pset(P_SOL, P.slot_of_leaf + 2u * sg.leaf_base);  // {slot, successor} per leaf
    pset(P_LOF, P.leaf_of + sg.map_base);
    pset(P_OAG, P.agent_of + sg.map_base);
    pset(P_LAG, P.leaf_agents + sg.leaf_base * (u64)lag_words(L));
    pset(P_CWO, P.cwo + sg.cwo_base);
    pset(P_ARUN, P.arun + sg.arun_base);
    pset(P_DELS, P.dels + sg.del_base);
    pset(P_DD, P.dd + sg.dd_base * (u64)DD_BLK);
    pset(P_DDB, P.ddb + sg.dd_base);
    pset(P_PROBE, P.probe ? P.probe + sg.rec_base : nullptr);
    pset(P_TXNS, P.txns + sg.txn_base);
    pset(P_PAR, P.parents + sg.par_base);
    pset(P_FR, P.frontier + sg.fr_base);
    pset(P_AGENTS, P.agents + sg.agent_base);
    pset(P_GROUPS, P.groups + sg.grp_base);
    pset(P_RECS, P.recs + sg.rec_base);
    pset(P_STP, P.st + d);
    p(K_LEAF, sg.leaf_cap);
    p(K_MAP, (sg.flags & DOC_TRACK_MAP) ? sg.map_cap : INVALID);  // INVALID: no order -> leaf map
    p(K_CWO, sg.cwo_cap);
    p(K_TXN, sg.txn_cap);
    p(K_DEL, sg.del_cap);
    p(K_DD, sg.dd_cap);
    p(K_PAR, sg.par_cap);
    p(K_RECN, sg.rec_n);
    p(K_FR, sg.fr_cap);
    p(K_AGMAP, (sg.flags & DOC_TRACK_AGENT) ? 1u : 0u);
    w.x_load_state(P.st + d, S_BASE);
    p(C_LEAF, INVALID);
    p(C_N, 0);
    p(C_VIS, 0);
    p(C_NOW, 0);
    p(C_BLK, 0);
    p(C_I, 0);
    p(C_VSTART, VS_BAD);
    p(C_DIRTY, 0);
    p(C_SUCC, INVALID);
    p(C_SUCC_ORD, 0);
    p(T_CWO_KEY, 0); p(T_CWO_AGENT, 0); p(T_CWO_SEQ, 0); p(T_CWO_LEN, 0);
    p(T_DEL_KEY, INVALID); p(T_DEL_ORDER, 0); p(T_DEL_LEN, 0);  // (no run: no key continues it)
    p(T_TX_ORDER, 0); p(T_TX_LEN, 0); p(T_TX_SHADOW, 0);
    p(T_FR0, ROOT_ORDER);
    p(T_AG_ID, INVALID); p(T_AG_BASE, 0); p(T_AG_CNT, 0); p(T_AG_CAP, 0);
    p(T_AGL_KEY, 0); p(T_AGL_ORDER, 0); p(T_AGL_LEN, 0); p(T_AGP_LEN, 0);
    p(T_OA_ID, INVALID); p(T_OA_BASE, 0); p(T_OA_CNT, 0);
    p(T_RB_BASE, 0x80000000u);  // pos - rb_base >= 64 for every valid pos
    p(F_FAST, 0);
    p(F_PRE, 0);
    p(F_GEN, 0);
  }

  CRDT_HD Span* leafp(u32 leaf) const { return w.template at<L>(lv(), leaf); }
  CRDT_HD u32* dleaf(u32 blk) const { return w.template at<GROUP>(dl(), blk); }
  CRDT_HD u32* dvis(u32 blk) const { return w.template at<GROUP>(dv(), blk); }

  // ------------------------------------------------------------------ init / begin / finish
  // New empty document: ListCRDT::new (doc.rs:51-64): one empty root leaf, frontier [ROOT].
  CRDT_HD void init_empty() {
    p(S_STATUS, (u32)ST_OK);
    p(S_REC_POS, 0);
    p(S_N_LEAVES, 1);
    p(S_N_BLOCKS, 1);
    p(S_NG, 1);
    p(S_NEXT_ORDER, 0);
    p(S_LEN, 0);
    p(S_N_CWO, 0); p(S_N_DEL, 0); p(S_N_DD, 0); p(S_N_TXN, 0); p(S_N_PAR, 0);
    p(S_N_FR, 1);
    p(S_N_ITEMS, 0);  // (not maintained: no reader)
    p(S_CAP_NEED, 0);
    p(S_N_ENTRIES, 0);
    p(S_GEN_DONE, 0);
    p(S_N_DDB, 0);
    w.zero_leaf(leafp(0), L);
    lag_stale(0u);
    w.st(dl(), 0u);
    w.st(dv(), 0u);
    w.st(sol(), 0u);
    w.st(sol() + 1, END_LEAF);
    w.st(fr(), ROOT_ORDER);
    w.root_init(0u, 1u, 0u);
  }
  CRDT_HD void begin() {
    w.root_load(groups(), g(S_NG));
    w.rank_load(agents(), g(S_N_AGENTS));
    u32 n = g(S_N_CWO);
    if (n) {
      CwoRun r = w.ld_cwo(w.at(cwo(), n - 1));
      p(T_CWO_KEY, r.key); p(T_CWO_AGENT, r.agent); p(T_CWO_SEQ, r.seq); p(T_CWO_LEN, r.len);
    }
    n = g(S_N_DEL);
    if (n) {
      DelRun r = w.ld_del(w.at(dels(), n - 1));
      p(T_DEL_KEY, r.key); p(T_DEL_ORDER, r.order); p(T_DEL_LEN, r.len);
    }
    n = g(S_N_TXN);
    if (n) {
      TxnRec t = w.ld_txn(w.at(txns(), n - 1));
      p(T_TX_ORDER, t.order); p(T_TX_LEN, t.len); p(T_TX_SHADOW, t.shadow);
    }
    p(T_FR0, w.ld(fr()));
    n = g(S_N_FR);
    if (n <= FR_LANES + 1u) w.fr_lanes_load(fr(), n);
    n = g(S_N_DDB);
    if (n <= 64u * DDT_LDS) w.ddt_rebuild(ddb(), 0u, n);
  }
  // write-back tails -> HBM (the tables' last entries; frontier[0])
  // the tails a run of fast commits left behind next_order (F_BASE)
  CRDT_HD void materialize_tails() {
    if (!g(F_FAST)) return;
    u32 no = g(S_NEXT_ORDER), d = no - g(F_BASE);
    if (d == 0u) return;
    inc(T_CWO_LEN, d);
    inc(T_TX_LEN, d);
    p(T_FR0, no - 1u);
    p(F_BASE, no);
  }
  CRDT_HD void flush_tails() {
    materialize_tails();
    agent_fill_tail();
    u32 n = g(S_N_CWO);
    if (n) w.st(&w.at(cwo(), n - 1)->len, g(T_CWO_LEN));
    n = g(S_N_DEL);
    if (n) w.st(&w.at(dels(), n - 1)->len, g(T_DEL_LEN));
    n = g(S_N_TXN);
    if (n) w.st(&w.at(txns(), n - 1)->len, g(T_TX_LEN));
    flush_agent();
    w.st(fr(), g(T_FR0));
    n = g(S_N_FR);
    if (n <= FR_LANES + 1u) w.fr_lanes_store(fr(), n);
  }
  CRDT_HD void flush_agent() {
    u32 a = g(T_AG_ID), cnt = g(T_AG_CNT);
    if (a != INVALID && cnt) {
      u32 ln = g(T_AGL_LEN);
      w.st(&w.at(arun(), g(T_AG_BASE) + cnt - 1)->len, ln);
      w.st_agent_tail(w.at(agents(), a), g(T_AGL_KEY), g(T_AGL_ORDER), ln);  // (AgentRec tail copy)
    }
  }
  CRDT_HD void finish() {
    commit();
    flush_tails();
    w.root_store(groups(), g(S_NG));
    w.x_store_state(stp(), S_BASE);
  }

  // ------------------------------------------------------------------ records
  // The op stream is read through a 64-record window [T_RB_BASE, +64) in VGPR lanes plus the
  // following 64 records, loaded ahead asynchronously: moving the window forward by d <= 64
  // slides it over the block ahead with lane shuffles and only issues the next block's load, so
  // the replay almost never waits for a record load.
  CRDT_HD void rec_window(u32 base) {
    u32 d = base - g(T_RB_BASE);
    u32 nn = rec_n() - base;
    u32 ahead = nn > 64u ? nn - 64u : 0u;
    if (d <= 64u) w.rec_slide(d, recs() + base + 64u, ahead < 64u ? ahead : 64u);
    else w.rec_load2(recs() + base, nn < 64u ? nn : 64u, ahead < 64u ? ahead : 64u);
    p(T_RB_BASE, base);
  }
  // The record at pos, moving the window so that it holds [pos, pos + 3) (a whole general-form
  // one-op txn).  The ONLY place the window moves: its registers then have one definition in the
  // replay loop, so the compiler keeps them in place instead of copying them at every merge.
  CRDT_HD Rec rec(u32 pos) {
    u32 base = g(T_RB_BASE);
    u32 d = pos - base;
    if (d > 61u) rec_window(d <= 64u ? pos : (d < 125u ? base + 64u : pos));
    return w.rec_get(pos - g(T_RB_BASE));
  }
  // The record at pos without moving the window (general path: from HBM when outside it).
  CRDT_HD Rec rec_at(u32 pos) const {
    u32 d = pos - g(T_RB_BASE);
    return d < 64u ? w.rec_get(d) : w.ld_rec(w.at(recs(), pos));
  }

  // ------------------------------------------------------------------ directory
  CRDT_HD void slot_of(u32 leaf, u32& blk, u32& i) const {
    if (leaf == g(C_LEAF)) { blk = g(C_BLK); i = g(C_I); return; }
    u32 v = w.ld(w.template at<2>(sol(), leaf));
    blk = v >> 6;
    i = v & 63u;
  }
  CRDT_HD u32 pos_key(u32 leaf) const {  // total order of leaves in the document
    u32 blk, i;
    slot_of(leaf, blk, i);
    return (w.root_find_blk(g(S_NG), blk) << 6) | i;
  }
  // The first leaf of the document is always leaf 0: init_empty creates it in slot 0 of block 0,
  // and leaves are only ever linked in after an existing one (split_at; blk_split moves the upper
  // half of a block to a block after it), never before it or removed -- as the reference's
  // leftmost leaf stays leftmost (root.rs:133-150).  (No directory lookup: an LDS read and a
  // dependent load per insert at position 0 before.)
  CRDT_HD u32 leaf_at_start() const {
    CRDT_EXPECT(w.ld(dleaf(w.root_blk(0))) == 0u);
    return 0u;
  }
  CRDT_HD u32 leaf_at_end() const {
    u32 gg = g(S_NG) - 1;
    return w.ld(dleaf(w.root_blk(gg)) + w.root_cnt(gg) - 1);
  }
  // Record the cached leaf's new visible count in the directory.
  CRDT_HD void dir_set_cached_vis(u32 v) {
    u32 old = g(C_VIS);
    if (v == old) return;
    u32 blk = g(C_BLK);
    w.st(dvis(blk) + g(C_I), v);
    w.root_add_vis_blk(g(S_NG), blk, v - old);
    inc(S_LEN, v - old);
    p(C_VIS, v);
  }
  // First leaf whose visible range contains `pos` (root.rs:54-88 descent, ContentIndex).
  CRDT_HD bool find_by_pos(u32 pos, u32& leaf, u32& vstart, u32& blk, u32& i) const {
    u32 gg, base;
    if (!w.root_find_pos(g(S_NG), pos, gg, base)) return false;
    blk = w.root_blk(gg);
    u32 before;
    if (!w.blk_find_pos(dvis(blk), dleaf(blk), w.root_cnt(gg), pos - base, i, before, leaf)) return false;
    vstart = base + before;
    return true;
  }

  // ------------------------------------------------------------------ leaf cache
  CRDT_HD void commit() {
    u32 lf = g(C_LEAF);
    if (lf == INVALID) return;
    if (!g(C_DIRTY)) return;
    w.cache_store(leafp(lf));
    lag_stale(lf);
    dir_set_cached_vis(g(C_NOW));
    p(C_DIRTY, 0);
  }
  // Cache `leaf`; `slot` = its directory slot (blk << 6 | i), possibly a load still in flight:
  // the leaf's entries are requested before the slot is first used, so both arrive together.
  // `succ`: its successor leaf if the caller has it (INVALID: not known yet).
  CRDT_HD void load_cache(u32 leaf, u32 slot, u32 succ = INVALID) {
#ifdef CRDT_EMU_STATS  // leaf switches; 71: back to the leaf cached before the current one; 72: the current one was dirty
    CRDT_STAT(70, 1); CRDT_STAT(71, leaf == st_prev_leaf); CRDT_STAT(72, g(C_DIRTY) != 0u);
    st_prev_leaf = g(C_LEAF);
#endif
    commit();
    p(C_N, w.cache_load(leafp(leaf)));
    u32 sl = w.uni_(slot);
    p(C_LEAF, leaf);
    p(C_BLK, sl >> 6);
    p(C_I, sl & 63u);
    p(C_DIRTY, 0);
    u32 v = w.cache_vis_from(0u);
    p(C_NOW, v);
    p(C_VIS, v);
    p(C_VSTART, VS_BAD);
    p(C_SUCC, w.uni_(succ));
    p(C_SUCC_ORD, INVALID);
  }
  // Successor of the cached leaf (INVALID at the end of the document): each leaf's slot entry
  // links its successor (the leaf list split_at maintains, as the reference's leaves are linked
  // in document order), so a leaf walk needs no directory lookup.
  CRDT_HD u32 cached_succ_leaf() {
    u32 sc = g(C_SUCC);
    if (sc == INVALID) {
      sc = w.ld(w.template at<2>(sol(), g(C_LEAF)) + 1);
      p(C_SUCC, sc);
    }
    return sc == END_LEAF ? INVALID : sc;
  }
  // ... and its first order (loaded once per cached leaf)
  CRDT_HD u32 cached_succ(u32& first_order) {
    u32 nl = cached_succ_leaf();
    if (nl == INVALID) { first_order = 0u; return INVALID; }
    u32 fo = g(C_SUCC_ORD);
    if (fo == INVALID) {
      fo = w.ld(&leafp(nl)->order);
      p(C_SUCC_ORD, fo);
    }
    first_order = fo;
    return nl;
  }
  CRDT_HD void ensure(u32 leaf) {
    if (leaf == g(C_LEAF)) return;
    // slot, successor and entries: one round trip (commits the cached leaf first)
    u32 slot, succ;
    w.ld_raw2(w.template at<2>(sol(), leaf), slot, succ);  // (one 8-byte load)
    load_cache(leaf, slot, succ);
  }
  // The successor of the cached leaf requested ahead: its entries (W::leaf_prefetch, into LDS) and
  // its slot entry {slot, successor}, in flight while the cached leaf is scanned; INVALID: none.
  CRDT_HD u32 prefetch_succ(u32& slot, u32& succ) {
    u32 nl = cached_succ_leaf();
    if (nl == INVALID) return INVALID;
    w.leaf_prefetch(leafp(nl));
    w.ld_raw2(w.template at<2>(sol(), nl), slot, succ);
    return nl;
  }
  // ... made the cached leaf (load_cache with the entries already in registers)
  CRDT_HD void switch_to_prefetched(u32 leaf, u32 slot, u32 succ) {
    commit();
    p(C_N, w.cache_from_prefetch());
    u32 sl = w.uni_(slot);
    p(C_LEAF, leaf);
    p(C_BLK, sl >> 6);
    p(C_I, sl & 63u);
    p(C_DIRTY, 0);
    u32 v = w.cache_vis_from(0u);
    p(C_NOW, v);
    p(C_VIS, v);
    p(C_VSTART, VS_BAD);
    p(C_SUCC, w.uni_(succ));
    p(C_SUCC_ORD, INVALID);
  }
  // set entry idx of the cached leaf (tracks the cached visible count exactly)
  CRDT_HD void set(u32 idx, const Span& e) {
    p(C_NOW, g(C_NOW) - clen_i(w.cget_len(idx)) + clen(e));
    w.cset(idx, e);
    p(C_DIRTY, 1u);
  }
  CRDT_HD u32 olc_stat(u32 order, const Cursor& left) {  // (statistics build only: 1 cached leaf, 2 left's leaf, 0 another, 3 ROOT)
    if (order == ROOT_ORDER) return 3;
    if (g(C_LEAF) != INVALID && w.cfind_order(g(C_N), order) >= 0) return 1;
    u32 lf = w.ld(w.at(lof(), order));
    return lf == left.leaf ? 2 : 0;
  }
  CRDT_HD static u32 clen_i(i32 len) { return len > 0 ? (u32)len : 0u; }
  CRDT_HD static u32 slen_i(i32 len) { return (u32)(len < 0 ? -len : len); }
  CRDT_HD u32 cur_len() const { return g(S_LEN) + g(C_NOW) - g(C_VIS); }

  // ------------------------------------------------------------------ order -> leaf map
  // ListCRDT::notify (doc.rs:143-153): all orders of `e` now live in `leaf`.  `home` is the
  // leaf the run already lives in (INVALID for freshly inserted orders): no write if unchanged.
  CRDT_HD void notify(const Span& e, u32 leaf, u32 home) {
    if (home == leaf) return;
    map_fill(e.order, slen(e), leaf);
  }
  // Writes of the order -> leaf map, for documents that keep it (K_MAP != INVALID; the capacity
  // checks against K_MAP then never trigger for the others).
  CRDT_HD u32 tracked() const { return g(K_MAP) != INVALID; }
  CRDT_HD void map_fill(u32 order, u32 n, u32 v) {
    if (tracked()) w.fill(w.at(lof(), order), n, v);
  }

  // ------------------------------------------------------------------ cursor ops
  // cursor.rs:127-145 (next_entry) / cursor.rs:26-103 (traverse).  Moves the cache along.
  CRDT_HD bool next_entry(Cursor& c) {
    ensure(c.leaf);
    if (c.idx + 1 < g(C_N)) { c.idx++; c.off = 0; return true; }
    u32 nl = cached_succ_leaf();
    if (nl == INVALID) return false;
    c.leaf = nl;
    c.idx = 0;
    c.off = 0;
    ensure(nl);
    return true;
  }
  // cursor.rs:210-231
  CRDT_HD bool roll(Cursor& c) {
    ensure(c.leaf);
    if (c.off == slen_i(w.cget_len(c.idx))) {
      c.off = 0;
      c.idx++;
      if (c.idx >= g(C_N)) return next_entry(c);
    }
    return true;
  }
  // cursor.rs:233-239 get_item: the item at a copy of the cursor rolled forward.  Rolling past
  // the end of the leaf only peeks at the next leaf's first entry (no cache change).
  CRDT_HD bool get_item(const Cursor& c, u32& out) {
    ensure(c.leaf);
    u32 idx = c.idx, off = c.off;
    if (off == slen_i(w.cget_len(idx))) {
      off = 0;
      idx++;
      if (idx >= g(C_N)) {
        u32 fo;
        if (cached_succ(fo) == INVALID) return false;
        out = fo;
        return true;
      }
    }
    out = w.cget_order(idx) + off;
    return true;
  }
  // cursor.rs:274-304
  CRDT_HD int cmp(const Cursor& a, const Cursor& b) const {
    if (a.leaf == b.leaf) {
      if (a.idx == b.idx) return (a.off > b.off) - (a.off < b.off);
      return (a.idx > b.idx) - (a.idx < b.idx);
    }
    u32 ka = pos_key(a.leaf), kb = pos_key(b.leaf);
    return (ka > kb) - (ka < kb);
  }
  CRDT_HD Cursor cursor_at_start() const { return Cursor{leaf_at_start(), 0, 0}; }  // root.rs:133-150
  // integrate's scan (doc.rs:183-221) past whole leaves: the leaves after the cached one, in
  // document order (directory block rows, 64 leaves per step), whose summary (crdt_types.h LAG_*)
  // shows every entry passing the scan with no event -- origin_left X (a tie), agent rank below
  // the new item's (scanning = false, go on), not orr -- are passed unread, as the sequential scan
  // would pass them entry by entry.  Returns the first leaf that must be read (INVALID: none; the
  // scan then runs off the end of the document, ST_NONTERMINATING as before).
  CRDT_HD u32 skip_leaves(u32 X, u32 orr, u32 agent) {
    u32 na = g(S_N_AGENTS), ng = g(S_NG);
    u32 my_rank = w.rank_of(agents(), na, agent);
    u32 blk = g(C_BLK), a = g(C_I) + 1u;
    u32 gg = w.root_find_blk(ng, blk);
    while (true) {
      u32 cnt = w.root_cnt(gg), leaf;
      u32 j = w.skip_scan(dleaf(blk), a, cnt, ptr<u32>(P_LAG), X, orr, my_rank, na, lv(), agents(), leaf);
      if (j < cnt) return leaf;
      if (++gg >= ng) return INVALID;
      blk = w.root_blk(gg);
      a = 0u;
    }
  }
  // root.rs:54-88 + 401-411, leaf.rs:61-84 (stick_end = false)
  CRDT_HD bool cursor_at_content_pos(u32 pos, Cursor& c) {
#ifdef CRDT_PROF
    u64 pc0 = w.clock();
#endif
    u32 vs = g(C_VSTART);
    // (pos in [vs, vs + now) is one unsigned compare; an unknown start is VS_BAD, which no
    // position passes, and there is no cached leaf only while it is VS_BAD)
    if (!(pos - vs < g(C_NOW))) {
#ifdef CRDT_PROF
      u64 ps0 = w.clock();
#endif
      commit();
      u32 lf, blk, i;
      if (!find_by_pos(pos, lf, vs, blk, i)) return false;
      if (lf != g(C_LEAF)) load_cache(lf, (blk << 6) | i, w.ld_raw(w.template at<2>(sol(), lf) + 1));  // (successor: in flight with the entries)
      p(C_VSTART, vs);
#ifdef CRDT_PROF
      prof_sw += (u32)(w.clock() - ps0);
#endif
    }
    u32 idx, off;
    if (!w.cfind_content(g(C_N), pos - vs, idx, off)) return false;
    c = Cursor{g(C_LEAF), idx, off};
#ifdef CRDT_PROF
    prof_cur += (u32)(w.clock() - pc0);
#endif
    return true;
  }
  // doc.rs:101-136 (marker_at + cursor_before_item, leaf.rs:41-57).  `load`: move the cache to
  // the item's leaf (the caller mutates there); otherwise only peek (the caller compares).
  CRDT_HD bool find_order(u32 order, bool load, Cursor& c) {
    if (order == ROOT_ORDER) {  // root.rs:90-123 cursor_at_end
      u32 lf = leaf_at_end();
      ensure(lf);
      u32 n = g(C_N);
      if (n == 0) return false;
      c = Cursor{lf, n - 1, slen_i(w.cget_len(n - 1))};
      return true;
    }
    if (order >= g(S_NEXT_ORDER)) return false;
    u32 cl = g(C_LEAF);
    i32 idx = cl != INVALID ? w.cfind_order(g(C_N), order) : -1;  // cached leaf first: no load
    if (idx >= 0) {
      c = Cursor{cl, (u32)idx, order - w.cget_order((u32)idx)};
      return true;
    }
    if (!tracked()) return false;  // (only remote ops look orders up: the host tracks their documents)
    u32 lf = w.ld(w.at(lof(), order));
    // (the fast paths leave the entries of delete orders unwritten: any value may be read there,
    // so a leaf id is trusted only if it exists, and then only if the order is found in it)
    if (lf >= g(S_N_LEAVES)) return false;
    if (lf == cl) return false;
    if (load) {
      ensure(lf);
      idx = w.cfind_order(g(C_N), order);
      if (idx < 0) return false;
      c = Cursor{lf, (u32)idx, order - w.cget_order((u32)idx)};
      return true;
    }
    u32 start;
    idx = w.peek_find_order(leafp(lf), order, start);
    if (idx < 0) return false;
    c = Cursor{lf, (u32)idx, order - start};
    return true;
  }
  // doc.rs:121-136 get_cursor_after
  CRDT_HD bool cursor_after(u32 order, bool load, Cursor& c) {
    if (order == ROOT_ORDER) {
      c = cursor_at_start();
      if (load) ensure(c.leaf);
      return true;
    }
    if (!find_order(order, load, c)) return false;
    c.off += 1;
    return true;
  }

  // ------------------------------------------------------------------ leaf mutation
  // mutations.rs:623-669 split_at: [idx, n) of the cached leaf moves to a new leaf (after
  // `padding` empty slots), which is linked right after the cached leaf.  Returns its id.
  // extra_vis: visible items the caller puts into the new leaf's padding slots in HBM itself
  // (counted in its directory slot, its group and the document length here)
  CRDT_HD u32 split_at(u32 idx, u32 padding, u32 extra_vis = 0u) {
#ifdef CRDT_PROF
    u64 psa = w.clock();
#endif
    u32 blk = g(C_BLK), i = g(C_I);
    // the cached leaf's directory block rows (blk_insert_at shifts them), requested first: their
    // latency overlaps the successor, leaf and order-map writes below
    u32 rl = w.row_ld(dleaf(blk)), rv = w.row_ld(dvis(blk));
    u32 nl = g(S_N_LEAVES);
    p(S_N_LEAVES, nl + 1);
    CRDT_STAT(0, 1); CRDT_STAT(1, g(C_N) - idx); CRDT_STAT(16 + (idx & 15u), 1);
    // the leaf list: nl goes right after the cached leaf
    u32 osucc = cached_succ_leaf();
    w.st(w.template at<2>(sol(), nl) + 1, osucc == INVALID ? END_LEAF : osucc);
    w.st(w.template at<2>(sol(), g(C_LEAF)) + 1, nl);
    u32 n = g(C_N);
    u32 stolen = w.cache_vis_from(idx);
    u32 first_moved = w.cget_order(idx);
    w.cache_write_moved(leafp(nl), idx, n, padding);
    lag_stale(nl);
    if (tracked()) w.fill_runs(lof(), idx, n, nl);  // notify every moved entry
    w.cache_clear(idx, n);
    p(C_NOW, g(C_NOW) - stolen);
    p(C_N, idx);
    p(C_DIRTY, 1u);
    dir_link(rl, rv, blk, i, nl, stolen, extra_vis);
    p(C_SUCC, nl);
    p(C_SUCC_ORD, padding ? INVALID : first_moved);  // (padding: the caller writes nl's first entries)
#ifdef CRDT_PROF
    prof_split += (u32)(w.clock() - psa);
#endif
    return nl;
  }
  // Link leaf nl right after the cached leaf (slot i of block blk, whose directory rows rl / rv
  // were requested by the caller): a directory block insert; the block splits when full.  The
  // cached leaf's slot loses `stolen` visible items (moved to nl); the group's visible total
  // changes only by extra_vis (items the caller placed in nl itself).
  CRDT_HD void dir_link(u32 rl, u32 rv, u32 blk, u32 i, u32 nl, u32 stolen, u32 extra_vis) {
    u32 ng = g(S_NG);
    u32 gg = w.root_find_blk(ng, blk);
    u32 cnt = w.root_cnt(gg);
    if (cnt == GROUP) {  // split the block: [32, 64) -> new block in group gg+1
      u32 nb = g(S_N_BLOCKS);
      p(S_N_BLOCKS, nb + 1);
      u32 mv = w.blk_split_r(rl, rv, dleaf(blk), dvis(blk), dleaf(nb), dvis(nb), sol(), nb);
      w.root_set(gg, blk, 32u, w.root_vis(gg) - mv);
      w.root_insert(ng, gg + 1, nb, 32u, mv);
      p(S_NG, ng + 1);
      if (i >= 32) {
        w.rows_upper(rl, rv, dleaf(nb), dvis(nb));
        blk = nb; i -= 32; gg = gg + 1; p(C_BLK, nb); p(C_I, i);
      }
      cnt = 32;
    }
    u32 cv = g(C_VIS) - stolen;
    w.blk_insert_at(rl, rv, dleaf(blk), dvis(blk), cnt, i, cv, nl, stolen + extra_vis, sol(), blk);
    w.root_set_cnt(gg, cnt + 1u);
    if (extra_vis) {
      w.root_add_vis(gg, extra_vis);
      inc(S_LEN, extra_vis);
    }
    p(C_VIS, cv);
  }
  // A backspace run inside visible entry E (idx) of the cached leaf, right after a leaf split, in
  // closed form over whole leaves.  In a full leaf every delete_general splits at idx + 1; from
  // then on the run repeats one cycle -- fill the leaf after E (delete_run_closed: pieces of two
  // deleted items each), then split it again -- so each cycle is a new leaf of known entries linked
  // right after the cached leaf, and E shrinks by the cycle's deletes:
  //  * follow split (idx + 1 >= L/2: the pieces of the splitting delete go to the new leaf; the
  //    cached leaf is [0, idx]): cycle of 2r + 1 deletes, r = L - idx - 1; for first target t the
  //    new leaf is [{t-2r, t-2r-1, -1}, {t-2r+1, t-2r+1, -2}, ..., {t-1, t-1, -2}];
  //  * otherwise (the split leaves [0, idx] + D = {t+1, t, -1} in the cached leaf): the cycle's
  //    first delete prepends onto D (span.rs:61-64 keeps D's origin_left), 2r more fill the leaf
  //    (r = L - idx - 2), and the splitting delete stays in the cached leaf as the next D: cycle of
  //    2r + 2 deletes, new leaf [{t-2r, t-2r, -2}, {t-2r+2, t-2r+2, -2}, ..., {t, t, -2}].
  // (mutations.rs:520-570 mutate_entry + :17-179 insert_internal + :623-669 split_at, op by op,
  // give the same leaves; the CPU emulation runs both.)  All entries share E's origin_right.
  // t: the run's next target (E's last item), rem: deletes left.  Returns the deletes applied (0:
  // not this state).
  CRDT_HD u32 back_cycles(u32 idx, u32 t, u32 rem) {
    u32 n = g(C_N);
    Span E = w.cget(idx);
    u32 follow = idx + 1u == n ? 1u : 0u;
    if (!follow) {  // [.., E, D] with D the run's last deleted item
      if (idx + 2u != n) return 0;
      Span D = w.cget(idx + 1u);
      if (D.order != t + 1u || D.ol != t || D.len != -1 || D.orr != E.orr) return 0;
    }
    if (E.len <= 0 || E.order + (u32)E.len - 1u != t) return 0;
    // (follow is the split's own rule: a split at idx + 1 >= L/2 moves the pieces with the new leaf)
    if (follow != (idx + 1u >= (u32)L / 2u ? 1u : 0u)) return 0;
    u32 r = (u32)L - n, per = 2u * r + 1u + (follow ^ 1u);
    u32 cyc = rem / per, c2 = ((u32)E.len - 1u) / per, c3 = g(K_LEAF) - g(S_N_LEAVES);
    cyc = cyc < c2 ? cyc : c2;
    cyc = c3 < 2u ? 0u : (cyc < c3 - 2u ? cyc : c3 - 2u);
    if (cyc == 0u) return 0;
    u32 orr = E.orr;
    for (u32 q = 0; q < cyc; q++) {
      u32 blk = g(C_BLK), i = g(C_I);
      u32 rl = w.row_ld(dleaf(blk)), rv = w.row_ld(dvis(blk));  // (dir_link's rows, requested first)
      u32 nl = g(S_N_LEAVES);
      p(S_N_LEAVES, nl + 1);
      u32 osucc = cached_succ_leaf();
      w.st(w.template at<2>(sol(), nl) + 1, osucc == INVALID ? END_LEAF : osucc);
      w.st(w.template at<2>(sol(), g(C_LEAF)) + 1, nl);
      u32 base = t - 2u * r;  // the new leaf's first order (its items are [base, base + per - ...])
      w.leaf_write_lanes(leafp(nl), r + 1u, [&](u32 lane) {
        u32 o = follow ? base + 2u * lane - 1u : base + 2u * lane;
        u32 first = follow & (lane == 0u ? 1u : 0u);
        return Span{first ? base : o, first ? base - 1u : o, orr, first ? -1 : -2};
      });
      lag_stale(nl);
      map_fill(base, follow ? 2u * r + 1u : 2u * r + 2u, nl);  // notify (doc.rs:143-153)
      dir_link(rl, rv, blk, i, nl, 0u, 0u);
      p(C_SUCC, nl);
      p(C_SUCC_ORD, base);
      inc(S_N_ENTRIES, r + 1u);
      t -= per;
    }
    u32 done = cyc * per;
    E.len -= (i32)done;
    w.cset(idx, E);
    if (!follow) w.cset(idx + 1u, Span{t + 1u, t, orr, -1});
    p(C_NOW, g(C_NOW) - done);
    p(C_DIRTY, 1u);
    return done;
  }
  // mutations.rs:17-179 insert_internal.  Items a0..a(n-1) (n <= 3) stay in named registers;
  // home: the leaf the items already live in (INVALID for fresh orders), for notify().
  CRDT_HD bool insert_items(Span a0, Span a1, Span a2, u32 n, Cursor& c, u32 home) {
    if (n == 0) return true;
    ensure(c.leaf);
    if (c.off == 0 && c.idx > 0) {
      c.idx -= 1;
      c.off = slen_i(w.cget_len(c.idx));
    }
    Span cur = w.cget(c.idx);
    bool has_rem = false;
    Span rem{0, 0, 0, 0};
    if (!(c.off == slen(cur) || c.off == 0)) {
      rem = truncate(cur, c.off);
      set(c.idx, cur);
      has_rem = true;
    }
    if (c.off != 0) {
      bool any = false;
      while (n > 0 && can_append_u(cur, a0)) {  // append to the entry at the cursor
        notify(a0, c.leaf, home);
        cur.len += a0.len;
        c.off = slen(cur);
        a0 = a1;
        a1 = a2;
        n--;
        any = true;
      }
      if (any) set(c.idx, cur);
      if (n == 0 && !has_rem) return true;
      c.off = 0;
      c.idx += 1;
      if (!has_rem && c.idx < g(C_N)) {  // prepend the tail of the items onto the next entry
        Span nx = w.cget(c.idx);
        bool pre = false;
        while (true) {
          Span last = n == 1 ? a0 : (n == 2 ? a1 : a2);
          if (!can_append_u(last, nx)) break;
          notify(last, c.leaf, home);
          nx.order = last.order;  // YjsSpan::prepend (span.rs:61-64): origin_left is NOT updated
          nx.len += last.len;
          pre = true;
          n--;
          if (n == 0) break;
        }
        if (pre) set(c.idx, nx);
        if (n == 0) return true;
      }
    }
    u32 space = n + (has_rem ? 1u : 0u);
    if (space > (u32)L / 2) return false;  // mutations.rs:121 assert
    inc(S_N_ENTRIES, space);
    bool rem_moved = false;
    u32 cn = g(C_N);
    if (cn + space > (u32)L) {
      CRDT_STAT(8, 1);
      bool follow = c.idx >= (u32)L / 2;
      u32 moved = cn - c.idx;
      u32 succ = g(C_SUCC), succ_ord = g(C_SUCC_ORD);  // the old leaf's successor follows nl
#ifdef CRDT_PROF
      u64 ts = w.clock();
#endif
      u32 nl = split_at(c.idx, follow ? space : 0u);
#ifdef CRDT_PROF
      (void)ts;
#endif
      if (follow) {  // the cursor follows the new leaf; its first `space` slots are padding
        u32 nblk = g(C_BLK), ni = g(C_I) + 1u;  // nl sits right after the old leaf
        commit();
        // nl becomes the cached leaf straight from registers (split_at just wrote it to HBM)
        w.cache_from_moved();
        u32 v = w.cache_vis_from(0u);
        p(C_LEAF, nl); p(C_BLK, nblk); p(C_I, ni);
        p(C_NOW, v); p(C_VIS, v); p(C_DIRTY, 0); p(C_VSTART, VS_BAD);
        p(C_SUCC, succ); p(C_SUCC_ORD, succ_ord);
        p(C_N, space + moved);
        c.leaf = nl;
        c.idx = 0;
        rem_moved = true;
      } else {
        p(C_N, g(C_N) + space);  // split_at left idx entries
      }
    } else {
      w.cache_shift_right(c.idx, cn, space);
      p(C_N, cn + space);
    }
    notify(a0, c.leaf, home);
    set(c.idx, a0);
    if (n > 1) { notify(a1, c.leaf, home); set(c.idx + 1, a1); }
    if (n > 2) { notify(a2, c.leaf, home); set(c.idx + 2, a2); }
    Span last = n == 1 ? a0 : (n == 2 ? a1 : a2);
    c.idx += n - 1;
    c.off = slen(last);
    if (has_rem) {
      if (rem_moved) notify(rem, c.leaf, INVALID);
      set(c.idx + 1, rem);
    }
    return true;
  }

  // ------------------------------------------------------------------ RLE side tables
  CRDT_HD void use_agent(u32 a) {  // agent cache (author of the current txn)
    if (a == g(T_AG_ID)) return;
    if (a == g(T_OA_ID)) p(T_OA_ID, INVALID);  // (its run count changes from now on)
    flush_agent();
    p(T_AG_ID, a);
    p(T_AGP_LEN, 0);
    AgentRec r = w.ld_agent(w.at(agents(), a));  // (with the copy of its last run: no second load)
    p(T_AG_BASE, r.run_base);
    p(T_AG_CNT, r.run_cnt);
    p(T_AG_CAP, r.run_cap);
    if (r.run_cnt) {
      p(T_AGL_KEY, r.tkey); p(T_AGL_ORDER, r.torder); p(T_AGL_LEN, r.tlen);
    } else {
      p(T_AGL_LEN, 0);  // no runs: the tail test in seq_to_order fails on its own
    }
  }
  CRDT_HD u32 agent_next_seq(u32 agent) {  // doc.rs:20-24
    use_agent(agent);
    return g(T_AG_CNT) ? g(T_AGL_KEY) + g(T_AGL_LEN) : 0u;
  }
  CRDT_HD bool seq_to_order(u32 agent, u32 seq, u32& order) {  // doc.rs:26-29
    u32 base, cnt;
    if (agent == g(T_AG_ID)) {
      u32 key = g(T_AGL_KEY);
      if (seq - key < g(T_AGL_LEN)) {  // (T_AGL_LEN = 0 while the agent has no runs)
        order = g(T_AGL_ORDER) + (seq - key);
        return true;
      }
      u32 pk = g(T_AGP_KEY);
      if (seq - pk < g(T_AGP_LEN)) {  // the run before the tail
        order = g(T_AGP_ORDER) + (seq - pk);
        return true;
      }
      base = g(T_AG_BASE);
      cnt = g(T_AG_CNT);
    } else if (agent == g(T_OA_ID)) {
      u32 ok_ = g(T_OA_KEY);
      if (seq - ok_ < g(T_OA_LEN)) {
        order = g(T_OA_ORDER) + (seq - ok_);
        return true;
      }
      base = g(T_OA_BASE);
      cnt = g(T_OA_CNT);
    } else {
      AgentRec A = w.ld_agent(w.at(agents(), agent));
      base = A.run_base;
      cnt = A.run_cnt;
      p(T_OA_ID, agent); p(T_OA_BASE, base); p(T_OA_CNT, cnt);
      // its last run, copied in its record (current: only its own txns change it, and use_agent
      // writes the copy back when it stops being the author)
      u32 tl = cnt != 0u ? A.tlen : 0u;
      p(T_OA_KEY, A.tkey); p(T_OA_ORDER, A.torder); p(T_OA_LEN, tl);
      if (seq - A.tkey < tl) {
        order = A.torder + (seq - A.tkey);
        return true;
      }
    }
    ARun r;
    if (w.search_run_recent(arun() + base, cnt, seq, r) < 0) return false;  // (recent runs first)
    order = r.order + (seq - r.key);
    return true;
  }
  CRDT_HD bool order_to_loc(u32 order, u32& agent, u32& seq) const {  // client_with_order.get() (simple_rle.rs:98-103)
    u32 n = g(S_N_CWO), key = g(T_CWO_KEY);
    if (order - key < g(T_CWO_LEN)) {  // (T_CWO_LEN = 0 while the table is empty)
      agent = g(T_CWO_AGENT);
      seq = g(T_CWO_SEQ) + (order - key);
      return true;
    }
    CwoRun r;
    if (w.search_run(cwo(), n, order, r) < 0) return false;
    agent = r.agent;
    seq = r.seq + (order - r.key);
    return true;
  }
  CRDT_HD bool order_to_agent(u32 order, u32& agent) const {  // client_with_order.get()
    u32 n = g(S_N_CWO), key = g(T_CWO_KEY);
    if (order - key < g(T_CWO_LEN)) { agent = g(T_CWO_AGENT); return true; }
    if (g(K_AGMAP)) {  // the order -> agent map (every assigned order has its author there)
      if (order >= g(S_NEXT_ORDER)) return false;
      agent = w.ld16(w.at(oag(), order));
      return true;
    }
    CwoRun r;
    if (w.search_run(cwo(), n, order, r) < 0) return false;
    agent = r.agent;
    return true;
  }
  // The order -> agent map, if kept, is written when a client_with_order run is retired (a new
  // run starts) and at the end of a launch: order_to_agent answers the current tail run from the
  // context lanes, so the fast paths, which only extend the tail, write nothing.
  CRDT_HD void agent_fill_tail() {
    if (g(K_AGMAP)) {
      if (g(S_N_CWO)) w.fill16(w.at(oag(), g(T_CWO_KEY)), g(T_CWO_LEN), g(T_CWO_AGENT));
    }
  }
  // doc.rs:155-165 assign_order_to_client
  CRDT_HD void assign_order_to_client(u32 agent, u32 seq, u32 order, u32 len) {
    u32 n = g(S_N_CWO);
    u32 ck = g(T_CWO_KEY), cl = g(T_CWO_LEN);
    if (n > 0 && order == ck + cl && agent == g(T_CWO_AGENT) && seq == g(T_CWO_SEQ) + cl) {
      p(T_CWO_LEN, cl + len);
    } else {
      if (n) w.st(&w.at(cwo(), n - 1)->len, cl);  // retire the old tail
      agent_fill_tail();
      p(T_CWO_KEY, order); p(T_CWO_AGENT, agent); p(T_CWO_SEQ, seq); p(T_CWO_LEN, len);
      w.st_cwo(w.at(cwo(), n), CwoRun{order, agent, seq, len});
      p(S_N_CWO, n + 1);
    }
    use_agent(agent);
    u32 an = g(T_AG_CNT), base = g(T_AG_BASE);
    u32 lk = g(T_AGL_KEY), ll = g(T_AGL_LEN);
    if (an > 0 && seq == lk + ll && order == g(T_AGL_ORDER) + ll) {
      p(T_AGL_LEN, ll + len);
    } else {
      if (an) {
        w.st(&w.at(arun(), base + an - 1)->len, ll);
        p(T_AGP_KEY, lk); p(T_AGP_ORDER, g(T_AGL_ORDER)); p(T_AGP_LEN, ll);
      }
      p(T_AGL_KEY, seq); p(T_AGL_ORDER, order); p(T_AGL_LEN, len);
      w.st_arun(w.at(arun(), base + an), ARun{seq, order, len, 0});
      p(T_AG_CNT, an + 1);
      w.st(&w.at(agents(), agent)->run_cnt, an + 1);
    }
  }
  CRDT_HD void append_delete(u32 key, u32 target, u32 len) {  // Rle<KVPair<DeleteEntry>>::append
    u32 n = g(S_N_DEL);
    u32 dk = g(T_DEL_KEY), dlen = g(T_DEL_LEN);
    if (key == dk + dlen) {  // (with no run yet dk + dlen is INVALID, which no key equals)
      if (g(T_DEL_ORDER) + dlen == target) {
        p(T_DEL_LEN, dlen + len);
        return;
      }
    }
    if (n) w.st(&w.at(dels(), n - 1)->len, dlen);
    p(T_DEL_KEY, key); p(T_DEL_ORDER, target); p(T_DEL_LEN, len);
    w.st_del(w.at(dels(), n), DelRun{key, target, len});
    p(S_N_DEL, n + 1);
  }
  // ---- double_deletes: an RLE of DDRun in 64-entry blocks (crdt_types.h DDBlk).  A position is
  // (logical block, index); (n_ddb, 0) is the end.
  struct DDPos { u32 lb, i; };
  CRDT_HD u32 dd_nb() const { return g(S_N_DDB); }
  CRDT_HD u32 dd_cnt(u32 lb) const { return w.ld(&ddb()[lb].cnt); }
  CRDT_HD DDRun* dd_ptr(DDPos q) const { return dd() + (u64)w.ld(&ddb()[q.lb].phys) * DD_BLK + q.i; }
  CRDT_HD DDRun dd_get(DDPos q) const { return w.ld_dd(dd_ptr(q)); }
  CRDT_HD DDPos dd_next(DDPos q) const { return q.i + 1u < dd_cnt(q.lb) ? DDPos{q.lb, q.i + 1u} : DDPos{q.lb + 1u, 0u}; }
  CRDT_HD DDPos dd_prev(DDPos q) const {  // q is not the first position
    if (q.i) return DDPos{q.lb, q.i - 1u};
    return DDPos{q.lb - 1u, dd_cnt(q.lb - 1u) - 1u};
  }
  // the position after the last entry with key <= x (entries are sorted by key)
  CRDT_HD DDPos dd_upper(u32 x) const {
    u32 nb = dd_nb();
    i32 lb = nb == 0u ? -1 : nb <= 64u * DDT_LDS ? w.dd_search_top(ddb(), nb, x) : w.search_first(ddb(), nb, x);
    if (lb < 0) return DDPos{0u, 0u};
    DDBlk B = w.ld_ddblk(ddb() + lb);
    u32 k = w.dd_count_le(dd() + (u64)B.phys * DD_BLK, B.cnt, x);  // >= 1: first <= x
    return k < B.cnt ? DDPos{(u32)lb, k} : DDPos{(u32)lb + 1u, 0u};
  }
  // Insert r before position q (Vec::insert); q becomes r's position.  A full block splits
  // first: its upper 32 entries move to a new physical block linked right after it.
  CRDT_HD bool dd_insert(DDPos& q, DDRun r) {
    u32 nb = dd_nb();
    if (nb == 0) {
      if (g(K_DD) == 0) return false;
      w.st_dd(dd(), r);
      w.st_ddblk(ddb(), DDBlk{0u, r.key, 1u, 0u});
      w.ddt_set(0u, r.key);
      p(S_N_DDB, 1u);
      inc(S_N_DD);
      q = DDPos{0u, 0u};
      return true;
    }
    if (q.lb >= nb) q = DDPos{nb - 1u, dd_cnt(nb - 1u)};  // the end: append to the last block
    DDBlk B = w.ld_ddblk(ddb() + q.lb);
    u32 bp = B.phys, bc = B.cnt;  // (two scalars, not the block record: no 4-register tuple to keep)
    if (bc == DD_BLK) {
      if (nb >= g(K_DD)) return false;
      u32 np = nb;  // physical blocks are allocated in order
      u32 first2 = w.dd_split(dd() + (u64)bp * DD_BLK, dd() + (u64)np * DD_BLK);
      w.ddb_insert(ddb(), nb, q.lb + 1u, DDBlk{np, first2, DD_BLK / 2u, 0u});
      if (nb + 1u <= 64u * DDT_LDS) w.ddt_rebuild(ddb(), (q.lb + 64u) >> 6, nb + 1u);  // (blocks 64 j >= q.lb + 1 moved)
      w.st(&ddb()[q.lb].cnt, DD_BLK / 2u);
      p(S_N_DDB, nb + 1u);
      if (q.i > DD_BLK / 2u) { q.lb += 1u; q.i -= DD_BLK / 2u; bp = np; }
      bc = DD_BLK / 2u;
    }
    w.dd_block_insert(dd() + (u64)bp * DD_BLK, bc, q.i, r);
    w.st(&ddb()[q.lb].cnt, bc + 1u);
    if (q.i == 0u) {
      w.st(&ddb()[q.lb].first, r.key);
      if (((q.lb & 63u) == 0u) & ((q.lb >> 6) < DDT_LDS)) w.ddt_set(q.lb >> 6, r.key);
    }
    inc(S_N_DD);
    return true;
  }
  // double_delete.rs:41-107 increment_delete_range (on the blocked RLE; same steps as the
  // reference's flat Vec: `idx` is a block position, Vec::insert is dd_insert)
  CRDT_HD bool increment_delete_range(u32 base, u32 len) {
    DDRun next{base, len, 1};
    // the entry containing base (Rle::search), else the first entry with key > base
    DDPos idx = dd_upper(base);
    if (idx.lb | idx.i) {
      DDPos q = dd_prev(idx);
      DDRun e = dd_get(q);
      if (base - e.key < e.len) idx = q;
    }
    while (true) {
      bool end = idx.lb >= dd_nb();
      DDRun cur = end ? DDRun{0, 0, 0} : dd_get(idx);
      if (end || cur.key > base) {  // quirk Q9 (double_delete.rs:52)
        DDRun here = next;
        bool done_here;
        if (!end && next.key + next.len > cur.key) {
          u32 at = cur.key - here.key;
          next = DDRun{here.key + at, here.len - at, here.excess};
          here.len = at;
          done_here = false;
        } else done_here = true;
        bool app = false;
        if (idx.lb | idx.i) {
          DDPos q = dd_prev(idx);
          DDRun qq = dd_get(q);
          if (here.key == qq.key + qq.len && here.excess == qq.excess) { w.st(&dd_ptr(q)->len, qq.len + here.len); app = true; }
        }
        if (!app) {
          if (!dd_insert(idx, here)) return false;
          idx = dd_next(idx);
        }
        if (done_here) break;
      }
      DDRun e = dd_get(idx);
      if (e.key < next.key) {
        u32 at = next.key - e.key;
        DDRun rm{e.key + at, e.len - at, e.excess};
        w.st(&dd_ptr(idx)->len, at);
        idx = dd_next(idx);
        if (!dd_insert(idx, rm)) return false;
      }
      DDRun e2 = dd_get(idx);
      if (e2.len <= next.len) {
        w.st(&dd_ptr(idx)->excess, e2.excess + 1);
        next.key += e2.len;
        next.len -= e2.len;
        if (next.len == 0) break;
        idx = dd_next(idx);
      } else {
        DDRun rm{e2.key + next.len, e2.len - next.len, e2.excess};
        w.st_dd(dd_ptr(idx), DDRun{e2.key, next.len, e2.excess + 1});
        DDPos after = dd_next(idx);
        if (!dd_insert(after, rm)) return false;
        break;
      }
    }
    return true;
  }
  CRDT_HD bool par_contains(const u32* pp, u32 np, u32 p0, u32 x) const {
    if (np == 0) return false;
    if (p0 == x) return true;
    for (u32 j = 1; j < np; j++) if (w.ld(pp + j) == x) return true;
    return false;
  }
  // doc.rs:350-374 insert_txn (+ advance_branch_by :34-48).  Remote parents: np of them, the
  // first in p0; when np > 1 all of them are already in the pool at [n_par, n_par + np).  A
  // single parent is written to the pool only if the txn does not coalesce (a merged txn keeps
  // no parents).  frontier[0] lives in T_FR0 (write-back); frontier[1..] in HBM.
  CRDT_HD i32 insert_txn(bool remote, u32 first, u32 len, u32 np, u32 p0) {
    u32 npar = g(S_N_PAR);
    u32* pp = par() + npar;
    u32* f = fr();
    u32 last = first + len - 1;
    u32 nfr = g(S_N_FR);
    u32 f0 = g(T_FR0);
    if (remote) {
      if (nfr == 1) {
        if (f0 == first) return ST_FRONTIER;
        if (par_contains(pp, np, p0, f0)) p(T_FR0, last);
        else { p(FR_S0, last); p(S_N_FR, 2); }  // (head 1 in its context lane)
      } else if (nfr <= 64u && np <= 64u) {
        // lane-parallel (one head / one parent per lane): heads that name `first` make the txn a
        // duplicate; heads among the parents go, the rest stay in order, `last` joins.  Heads in
        // context lanes (FR_S0) while they fit, else in HBM; a frontier that crosses the bound
        // moves with the result
        u32 nf0, r;
        bool lanes = nfr <= FR_LANES + 1u;
        if (lanes) r = w.frontier_advance_x(nfr, f0, pp, np, p0, first, last, g(K_FR), nf0, f);
        else r = w.frontier_advance(f, nfr, f0, pp, np, p0, first, last, g(K_FR), nf0);
        if (r == 0u) return ST_FRONTIER;
        if (r == INVALID) return ST_CAPACITY;  // (fits() reserved room for nfr + 1 heads)
        if (!lanes && r <= FR_LANES + 1u) w.fr_lanes_load(f, r);
        p(S_N_FR, r);
        p(T_FR0, nf0);
      } else {
        if (nfr <= FR_LANES + 1u) w.fr_lanes_store(f, nfr);  // (this form reads and writes the heads in HBM)
        for (u32 k = 0; k < nfr; k++) if ((k == 0 ? f0 : w.ld(f + k)) == first) return ST_FRONTIER;
        u32 m = 0, nf0 = f0;
        for (u32 k = 0; k < nfr; k++) {
          u32 o = k == 0 ? f0 : w.ld(f + k);
          if (!par_contains(pp, np, p0, o)) {
            if (m == 0) nf0 = o;
            else w.st(f + m, o);
            m++;
          }
        }
        if (m + 1 > g(K_FR)) return ST_CAPACITY;  // (fits() reserved room for nfr + 1 heads)
        if (m == 0) nf0 = last;
        else w.st(f + m, last);
        if (m + 1u <= FR_LANES + 1u) w.fr_lanes_load(f, m + 1u);
        p(S_N_FR, m + 1);
        p(T_FR0, nf0);
      }
    } else {
      np = nfr;
      p0 = f0;
      if (np <= FR_LANES + 1u) w.fr_lanes_store(pp, np);  // (the heads become the txn's parents)
      else for (u32 k = 1; k < np; k++) w.st(pp + k, w.ld(f + k));
      p(T_FR0, last);
      p(S_N_FR, 1);
    }
    u32 ntx = g(S_N_TXN);
    u32 txo = g(T_TX_ORDER), txl = g(T_TX_LEN), txs = g(T_TX_SHADOW);
    u32 shadow = first;
    while (shadow >= 1 && par_contains(pp, np, p0, shadow - 1)) {
      u32 x = shadow - 1;
      if (ntx && x >= txo && x - txo < txl) { shadow = txs; continue; }
      i32 k = w.search_txn(txns(), ntx, x);
      if (k < 0) return ST_UNKNOWN_ID;
      shadow = w.ld(&w.at(txns(), (u32)k)->shadow);
    }
    if (ntx > 0 && np == 1 && p0 == txo + txl - 1 && shadow == txs) {
      p(T_TX_LEN, txl + len);  // write-back: the merged length reaches HBM with the tail
      return ST_OK;            // parents of a merged txn are not kept
    }
    if (np) w.st(pp, p0);
    if (ntx) w.st(&w.at(txns(), ntx - 1)->len, txl);  // retire the old tail
    p(T_TX_ORDER, first);
    p(T_TX_LEN, len);
    p(T_TX_SHADOW, shadow);
    w.st_txn(w.at(txns(), ntx), TxnRec{first, len, shadow, npar, np, {0, 0, 0}});
    p(S_N_TXN, ntx + 1);
    p(S_N_PAR, npar + np);
    return ST_OK;
  }

  CRDT_HD i32 id_to_order(u32 agent, u32 seq, u32& order) {  // doc.rs:236-240
    if (agent == ROOT_AGENT) { order = ROOT_ORDER; return ST_OK; }
    if (agent >= g(S_N_AGENTS)) return ST_UNKNOWN_AGENT;
    if (!seq_to_order(agent, seq, order)) return ST_UNKNOWN_ID;
    return ST_OK;
  }

  // ------------------------------------------------------------------ txn application
  // Capacity needed by a txn (checked before any mutation, so a capacity stop is resumable at
  // this txn).  Every block but the first holds >= 32 slots, so blk_cap = leaf_cap/32 + 2 bounds
  // the blocks and the root groups as well (the host sizes the LDS root to blk_cap groups).
  // On failure S_CAP_NEED records which table (bit) must grow.
  CRDT_HD bool fits(bool remote, u32 agent, u32 n_ops, u32 n_dels, u32 txn_len, u32 n_parents) {
    // room = cap - count (count <= cap always holds), compared in 32 bits
    u32 need = 0;
    if (g(K_LEAF) - g(S_N_LEAVES) < 2ull * n_ops) need |= 1u;
    if (g(K_CWO) == g(S_N_CWO) || g(K_TXN) == g(S_N_TXN)) need |= 2u;
    if (g(K_DEL) - g(S_N_DEL) < n_dels) need |= 4u;
    if (g(K_PAR) - g(S_N_PAR) < (remote ? n_parents : g(S_N_FR))) need |= 8u;
    if (g(K_MAP) - g(S_NEXT_ORDER) < txn_len) need |= 16u;
    if (remote && g(K_FR) <= g(S_N_FR)) need |= 128u;  // a remote txn leaves <= nfr + 1 heads
    // double deletes (remote only): one txn adds at most 3 entries per existing entry it overlaps
    // (entries are disjoint runs of >= 1 item, so it overlaps <= min(entries, txn_len) of them)
    // plus 2 per increment_delete_range call (<= one per deleted item); every block but the
    // first holds >= 32 entries, so E entries need <= E/32 + 1 blocks
    u32 ndd = g(S_N_DD);
    if (remote && n_dels) {
      u64 ov = ndd < txn_len ? ndd : txn_len;
      if ((ndd + 3ull * ov + 2ull * txn_len + 2ull) / 32ull + 2ull > (u64)g(K_DD)) need |= 64u;
    }
    use_agent(agent);
    if (g(T_AG_CAP) == g(T_AG_CNT)) need |= 32u;
    p(S_CAP_NEED, need);
    return need == 0;
  }

  // Op interpreter modes
  enum : u32 { M_FETCH = 0, M_LDEL = 1, M_RDEL = 2, M_LINS = 3, M_INS = 4 };

  // One txn: doc.rs:376-469 apply_local_txn (remote = false) or doc.rs:242-348
  // apply_remote_txn (remote = true).  Header at record `pos`; ops (then parents) follow.
  // gen: the txn comes from a GEN record; its single LocalOp is `gop` (no op record to read).
  // inl: the txn's single op (and for a remote txn its single parent) are gop / gpar, not records
  // after the header (a compact record, or a generated op)
  CRDT_HD i32 apply_txn(const Rec& h, u32 pos, bool remote, u32 inl, const Rec& gop, const Rec& gpar) {
    CRDT_STAT(47, 1); CRDT_MEM_EPOCH();
#ifdef CRDT_PROF
    u64 prof_t0 = w.clock();
#endif
    materialize_tails();
    p(F_FAST, 0u);  // the general path changes the tails fast_txn_ok relies on
    u32 nops, agent, np = 0, seq, txn_len;
    if (!remote) {
      nops = h.w0 & 0x0FFFFFFFu;
      agent = h.w1;
      txn_len = h.w3;
      if (agent >= g(S_N_AGENTS)) return ST_UNKNOWN_AGENT;
      if (txn_len == 0) return ST_EMPTY_TXN;
      if (!fits(false, agent, nops, h.w2, txn_len, 0)) return ST_NEED_CAPACITY;
      seq = agent_next_seq(agent);
    } else {
      nops = h.w0 & RTXN_NOPS_MASK;
      agent = h.w1 & 0xFFFFu;
      np = h.w1 >> 16;
      seq = h.w2;
      txn_len = h.w3;
      if (agent >= g(S_N_AGENTS)) return ST_UNKNOWN_AGENT;
      if (agent_next_seq(agent) != seq) return ST_SEQ;
      if ((h.w0 >> 27) & 1u) return ST_BAD_INPUT;
      if (txn_len == 0) return ST_EMPTY_TXN;
      // (delete-log and double-delete room only for a txn with a delete op: RTXN has_del)
      if (!fits(true, agent, nops, ((h.w0 >> RTXN_DEL_BIT) & 1u) ? nops : 0u, txn_len, np)) return ST_NEED_CAPACITY;
    }
    u32 first = g(S_NEXT_ORDER);
    u32 next = first;
    assign_order_to_client(agent, seq, first, txn_len);
    p(S_NEXT_ORDER, first + txn_len);
#ifdef CRDT_PROF_TXN2
    u64 prof_ta = w.clock();
#endif

    u32 k = 0;
    u32 mode = M_FETCH;
    u32 remaining = 0, target = 0, lpos = 0, lins = 0;
    Span item{0, 0, 0, 0};
    Cursor c{0, 0, 0};
    if (g(F_PRE)) {  // a fast-path attempt already resolved this one-insert txn (origins, cursor)
      item = Span{g(PRE_ITEM), g(PRE_ITEM + 1), g(PRE_ITEM + 2), (i32)g(PRE_ITEM + 3)};
      c = Cursor{g(PRE_C), g(PRE_C + 1), g(PRE_C + 2)};
      next = first + (u32)item.len;
      k = 1;
      mode = M_INS;
    }
    while (true) {
      // ---------------------------------------------------------------- next op
      if (mode == M_FETCH) {
        if (k == nops) break;
        Rec op = inl ? gop : rec_at(pos + 1 + k);
        k++;
        if (!remote) {  // LocalOp: delete (visible range) first, then insert (doc.rs:386-465)
          lpos = op.w1;
          u32 del = op.w2;
          lins = op.w3;
          if (del > 0) {
            if ((u64)lpos + del > cur_len()) return ST_POS_OOB;
            if (!cursor_at_content_pos(lpos, c)) return ST_POS_OOB;
            map_fill(next, del, INVALID);  // delete orders name no item
            roll(c);                             // mutations.rs:539
            remaining = del;
            mode = M_LDEL;
          } else if (lins > 0) {
            mode = M_LINS;
          } else {
            continue;
          }
        } else {
          u32 kind = rec_kind(op);
          u32 len = op.w0 & 0x0FFFFFFFu;
          if (kind == REC_RINS) {
            u32 ol, orr;
            i32 st = id_to_order(op.w1 & 0xFFFFu, op.w2, ol);
            if (st != ST_OK) return st;
            st = id_to_order(op.w1 >> 16, op.w3, orr);
            if (st != ST_OK) return st;
            item = Span{next, ol, orr, (i32)len};
            next += len;
            if (!cursor_after(ol, true, c)) return ST_UNKNOWN_ID;  // doc.rs:176-178
            mode = M_INS;
          } else if (kind == REC_RDEL) {
            i32 st = id_to_order(op.w1 & 0xFFFFu, op.w2, target);
            if (st != ST_OK) return st;
            append_delete(next, target, len);  // doc.rs:305-308
            map_fill(next, len, INVALID);
            next += len;
            remaining = len;
            mode = M_RDEL;
          } else {
            return ST_BAD_INPUT;
          }
        }
      }
      // ---------------------------------------------------------------- local insert origins
      if (mode == M_LINS) {  // doc.rs:436-463
        u32 ol;
        if (lpos == 0) {
          ol = ROOT_ORDER;
          c = cursor_at_start();
        } else {
          if (lpos > cur_len()) return ST_POS_OOB;
          if (!cursor_at_content_pos(lpos - 1, c)) return ST_POS_OOB;
          if (!get_item(c, ol)) return ST_POS_OOB;
          if (!roll(c)) return ST_POS_OOB;  // Cursor::next (cursor.rs:242-248)
          c.off++;
        }
        u32 orr;
        if (!get_item(c, orr)) orr = ROOT_ORDER;
        item = Span{next, ol, orr, (i32)lins};
        next += lins;
        mode = M_INS;
      }
      // ---------------------------------------------------------------- produce one mutation
      Span a0{0, 0, 0, 0}, a1{0, 0, 0, 0}, a2{0, 0, 0, 0};
      u32 n = 0;
      u32 home = INVALID;
#ifdef CRDT_PROF_TXN
      u64 pq0 = w.clock();
      u32 pq_ins = mode == M_INS;
#endif
      if (mode == M_INS) {
        // integrate (doc.rs:167-234): scan entries from the insertion point
        Cursor left = c, scan_start = c;
        bool scanning = false;
        u32 first_step = 1;
        u32 tk_ = g(T_CWO_KEY), tl_ = g(T_CWO_LEN), ta_ = g(T_CWO_AGENT);  // (fixed while integrate scans)
        while (true) {
          // From the second step on the cursor sits at the start of an entry of the cached leaf
          // (next_entry), so the entry's item is its first order and its origin_left is the
          // entry's ol: the leaf's entries from the cursor on are evaluated lane-parallel
          // (W::scan_batch: one gather of their first orders' agents and ranks).  An entry whose
          // origin_left is integrate's own (cmp == 0 by identity: cursor_after of one item) and
          // that does not break changes only (scanning, scan_start), and the last such entry
          // before the first event decides them; the first event -- origin_right reached, a
          // tie that breaks, or an origin_left elsewhere (a real cursor compare) -- is then
          // evaluated by the sequential step below.  Documents without the order -> agent map
          // take every step sequentially.
          if (!first_step) {
            if (g(K_AGMAP)) {
              u32 nn = g(C_N), last, last_scan;
              u32 na = g(S_N_AGENTS);
              CRDT_STAT(45, 1); CRDT_STAT(46, nn - c.idx);
              // (the successor leaf is requested before this leaf is evaluated: a scan that runs
              // through it finds it in LDS)
              // the agents of the leaf's entries: its agent row when current (a leaf with
              // uncommitted changes has none), else gathered from the order -> agent map and
              // written as its row
              u32 clean = g(C_DIRTY) ^ 1u;
              u32 lw = 0u;
              if (clean) lw = w.lag_ld(lagp(c.leaf));
              u32 rt = w.rank_row(na);
              u32 pslot, psucc;
              u32 pl = prefetch_succ(pslot, psucc);
              u32 ag;
              CRDT_STAT(55, clean); CRDT_STAT(56, clean && w.lag_valid(lw));
              if (clean && w.lag_valid(lw)) {
                ag = w.lag_agents(lw, nn, oag(), tk_, tl_, ta_);
              } else {
                ag = w.scan_gather(nn, oag());
                if (clean) w.lag_store(lagp(c.leaf), ag, nn, tk_, tl_, ta_, rt, na, agents());
              }
              u32 f = w.scan_batch(ag, rt, agent, c.idx, nn, item.ol, item.orr, agents(), na,
                                   tk_, tl_, ta_, last, last_scan);
              if (last != INVALID) {
                scanning = last_scan != 0u;
                if (last_scan) scan_start = Cursor{c.leaf, last, 0u};
              }
              if (f >= nn) {  // no event in this leaf: on to the next one (next_entry, cursor.rs:127-145)
                if (pl == INVALID) return ST_NONTERMINATING;
                // ... past every following leaf whose summary shows it passes with no event
                u32 jl = skip_leaves(item.ol, item.orr, agent);
                CRDT_STAT(66, 1); CRDT_STAT(67, jl != pl);
                if (jl == pl) {
                  switch_to_prefetched(pl, pslot, psucc);
                } else {
                  if (jl == INVALID) return ST_NONTERMINATING;
                  scanning = false;  // (every skipped entry ranks below the new item)
                  w.prefetch_drain();
                  ensure(jl);
                }
                c = Cursor{jl, 0u, 0u};
                continue;
              }
              c.idx = f;
            }
          }
          first_step = 0;
          u32 other_order;
          if (!get_item(c, other_order)) break;
          if (other_order == item.orr) break;
          Span oe = w.cget(c.idx);  // get_item ensured c.leaf
          u32 oo = origin_left_at_offset(oe, c.off);
          CRDT_STAT(40, 1); CRDT_STAT(41 + olc_stat(oo, left), 1);
          // the other item's origin_left is the new item's own (a concurrent sibling): the same
          // cursor (cursor_after of one order, found above), so cmp is 0 without looking it up --
          // no order -> leaf lookup and no peek at left's leaf once the scan has left it
          int r = 0;
          if (oo != item.ol) {
            Cursor olc;
            if (!cursor_after(oo, false, olc)) return ST_UNKNOWN_ID;
            r = cmp(olc, left);
          }
          if (r < 0) break;
          if (r == 0) {
            u32 oa;
            if (!order_to_agent(oe.order, oa)) return ST_UNKNOWN_ID;
            u32 my_rank = w.rank_of(agents(), g(S_N_AGENTS), agent);
            u32 other_rank = w.rank_of(agents(), g(S_N_AGENTS), oa);
            if (my_rank > other_rank) scanning = false;
            else if (item.orr == oe.orr) break;
            else { scanning = true; scan_start = c; }
          }
          if (!next_entry(c)) return ST_NONTERMINATING;  // cursor unchanged -> loops forever
        }
        if (scanning) c = scan_start;
        a0 = item;
        n = 1;
        mode = M_FETCH;
      } else {
        if (mode == M_LDEL) {  // mutations.rs:541-556 local_deactivate
          ensure(c.leaf);
          while (w.cget_len(c.idx) <= 0) {
            if (!next_entry(c)) return ST_POS_OOB;
          }
        } else {  // doc.rs:311-327 + mutations.rs:579-615 remote_deactivate
          if (target == ROOT_ORDER) return ST_NONTERMINATING;
          if (!find_order(target, true, c)) return ST_UNKNOWN_ID;
          roll(c);
          i32 el = w.cget_len(c.idx);
          if (el <= 0) {  // already deleted: count the double delete, mutate nothing
            u32 avail = (u32)(-el) - c.off;
            u32 here = remaining < avail ? remaining : avail;
            if (here == 0) return ST_NONTERMINATING;
            if (!increment_delete_range(target, here)) return ST_CAPACITY;
            remaining -= here;
            target += here;
            if (remaining == 0) mode = M_FETCH;
            continue;
          }
        }
        // mutate_entry (mutations.rs:227-277) + replace_entry (:185-200)
        Span e = w.cget(c.idx);
        u32 elen = slen(e);
        if (!(c.off < elen)) return ST_INTERNAL;
        bool ha = c.off > 0, hc = false;
        Span pa{0, 0, 0, 0}, pc{0, 0, 0, 0};
        if (ha) { elen -= c.off; pa = truncate_keeping_right(e, c.off); }
        u32 r = elen;
        if (remaining < elen) { pc = truncate(e, remaining); hc = true; r = remaining; }
        if (mode == M_LDEL) {  // extend_delete + deletes.append (doc.rs:414-426)
          append_delete(next, e.order, (u32)e.len);
          next += (u32)e.len;
        }
        e.len = -e.len;
        Span first_part = ha ? pa : e;
        set(c.idx, first_part);
        c.off = slen(first_part);
        if (ha) { a0 = e; a1 = pc; n = hc ? 2u : 1u; }
        else if (hc) { a0 = pc; n = 1; }
        home = c.leaf;
        remaining -= r;
        if (mode == M_RDEL) target += r;
        if (remaining == 0) mode = (mode == M_LDEL && lins > 0) ? M_LINS : M_FETCH;
      }
      // ---------------------------------------------------------------- the one insert site
#ifdef CRDT_PROF_TXN
      u64 pq1 = w.clock();
      if (pq_ins) pt_scan += (u32)(pq1 - pq0);
      else pt_del += (u32)(pq1 - pq0);
#endif
      if (!insert_items(a0, a1, a2, n, c, home)) return ST_INTERNAL;
#ifdef CRDT_PROF_TXN
      pt_ins += (u32)(w.clock() - pq1);
#endif
    }
    if (!remote && next != first + txn_len) return ST_BAD_INPUT;
#ifdef CRDT_PROF_TXN2
    u64 prof_tb = w.clock();
#endif
    u32 p0 = 0;
    if (remote) {
      u32* pp = par() + g(S_N_PAR);
      for (u32 j = 0; j < np; j++) {
        Rec pr = inl ? gpar : rec_at(pos + 1 + nops + j);
        if (rec_kind(pr) != REC_RPARENT) return ST_BAD_INPUT;
        u32 o;
        i32 st = id_to_order(pr.w1 & 0xFFFFu, pr.w2, o);
        if (st != ST_OK) return st;
        if (j == 0) p0 = o;
        else w.st(pp + j, o);  // pp[0] is written by insert_txn (only if the txn is kept)
      }
    }
#ifdef CRDT_PROF
    u64 prof_t1 = w.clock();
    i32 rst = insert_txn(remote, first, txn_len, np, p0);
    (void)prof_t0; (void)prof_t1;
#ifdef CRDT_PROF_TXN2
    if (prof_mode == 3u) {  // prologue (agent switch, fits, assign_order_to_client) / ops / parents / insert_txn
      u64 prof_td = w.clock();
      inc(S_PROF0, (u32)(prof_ta - prof_t0)); inc(S_PROF1, (u32)(prof_tb - prof_ta));
      inc(S_PROF2, (u32)(prof_t1 - prof_tb)); inc(S_PROF3, (u32)(prof_td - prof_t1));
    }
#endif
#ifdef CRDT_PROF_TXN
    if (prof_mode == 3u) {
      u32 tot = (u32)(w.clock() - prof_t0);
      inc(S_PROF0, tot - pt_scan - pt_del - pt_ins); inc(S_PROF1, pt_scan); inc(S_PROF2, pt_del); inc(S_PROF3, pt_ins);
    }
    pt_scan = pt_del = pt_ins = 0;
#endif
    return rst;
#else
    return insert_txn(remote, first, txn_len, np, p0);
#endif
  }

  // ------------------------------------------------------------------ fast paths
  // Real edit traces are dominated by two single-op txn shapes: typing (an insert right after
  // the agent's previous item) and a delete inside one visible entry.  For those, apply_txn's
  // effects reduce to a few context updates, so they are recognised up front -- every condition
  // apply_txn would evaluate is checked against the same state before anything changes -- and
  // applied directly; everything else takes the general interpreter.  A typing run is validated
  // for the rest of the 64-record prefetch block at once, lane-parallel (W::typing_scan), and
  // applied as one append.
  //
  // Txn level (doc.rs:155-165 assign_order_to_client, doc.rs:350-374 insert_txn): the txn
  // continues its agent's last item_orders run and the last client_with_order run, its single
  // parent is the previous order, the frontier is that one order, so the txn coalesces into the
  // last TxnSpan (TxnSpan::can_append, txn.rs:44-48: shadow unchanged, parents not kept).
  //
  // A fast commit (fast_txn_commit) extends every one of these tails by the txn, so after it all
  // conditions that do not name the next txn's author and seq still hold (F_FAST); only
  // apply_txn changes them otherwise.  Then the check is: same author, next seq.
  //
  // Conditions are written as early exits throughout the fast paths: each is one s_cmp and one
  // branch, where an `a & b & ...` chain of uniform compares becomes 64-bit lane masks (s_cmp,
  // s_cselect_b64, s_and_b64 per term) on the scalar unit this kernel is bound by.
  // (local: seq is the author's next seq by definition (doc.rs:393-398), so that check is skipped)
  CRDT_HD u32 fast_txn_ok(u32 agent, u32 seq, u32 first, u32 local = 0u) const {
    if (agent != g(T_AG_ID)) return 0;
    u32 ll = g(T_AGL_LEN);
    if (!local) {
      if (seq != g(T_AGL_KEY) + ll) return 0;
    }
    if (g(F_FAST)) return 1;
    if (g(T_AG_CNT) == 0u) return 0;
    if (g(T_AGL_ORDER) + ll != first) return 0;
    if (g(S_N_CWO) == 0u) return 0;
    if (g(T_CWO_AGENT) != agent) return 0;
    u32 cl = g(T_CWO_LEN);
    if (g(T_CWO_SEQ) + cl != seq) return 0;
    if (g(T_CWO_KEY) + cl != first) return 0;
    if (g(S_N_FR) != 1u) return 0;
    if (g(T_FR0) != first - 1u) return 0;
    if (g(S_N_TXN) == 0u) return 0;
    return g(T_TX_ORDER) + g(T_TX_LEN) == first;
  }
  // (S_CAP_NEED is read by the host only after a capacity stop, which fits() records afresh)
  CRDT_HD void fast_txn_commit(u32 first, u32 len) {
    if (!g(F_FAST)) {  // the first fast commit after the general path: the lazy tails start here
      p(F_BASE, first);
      p(F_FAST, 1u);
    }
    p(S_NEXT_ORDER, first + len);
    inc(T_AGL_LEN, len);
  }
  // the first order after entry idx of the cached leaf (get_item at the entry's end, cursor.rs:233-239)
  CRDT_HD u32 next_item_after(u32 idx, u32& order) {
    if (idx + 1u < g(C_N)) { order = w.cget_order(idx + 1u); return 1u; }
    u32 fo;
    u32 has = cached_succ(fo) != INVALID;
    order = fo;
    return has;
  }
  // Typing: origin_left = the previous txn's last item = the last item of entry idx,
  // origin_right = the item after that entry (or none).  integrate stops at once (doc.rs:184-190)
  // and insert_internal appends to the entry (mutations.rs:57-80, YjsSpan::can_append); every
  // later txn of the run is the same case.  Returns records consumed (0: not applicable).
  // The run of typing txns starting with the one at b0 (validated by the caller): W::typing_scan
  // over the window, continued past it by sliding the window to the run's last txn.  ow1: the op
  // word (origin_left agent | origin_right agent << 16) every later txn must carry.  Returns the
  // run's txns (>= 1) and, in `total`, their total length.  nv == 0: a generated op (no window).
  CRDT_HD u32 typing_run(u32 b0, u32 nv, u32 remote, u32 agent, u32 ow1, const Rec& o, u32& total) {
    u32 nt = 1u;
    total = remote ? (o.w0 & 0x0FFFFFFFu) : o.w3;
    if (!nv) return nt;
    nt = w.typing_scan(b0, nv, remote, cpt, agent, ow1, o.w3, total);
    u32 per = per_txn(remote), rn = rec_n();
    u32 pos0 = g(T_RB_BASE) + b0;
    u32 end = g(T_RB_BASE) + nv;  // records scanned so far: [pos0, end)
    while (true) {  // the run reaches the end: scan on
      if (pos0 + (nt + 1u) * per <= end) break;
      if (end >= rn) break;
      u32 last = pos0 + (nt - 1u) * per;
      u32 n = rn - last < 64u ? rn - last : 64u;
      u32 t2, l0;
      u32 n2 = w.typing_scan_at(w.at(recs(), last), n, remote, cpt, agent, ow1, o.w3, t2, l0);
      end = last + n;
      if (n2 <= 1u) break;
      total += t2 - l0;
      nt += n2 - 1u;
    }
    return nt;
  }
  CRDT_HD u32 fast_typing(u32 b0, u32 nv, u32 remote, u32 idx, u32 orr, u32 agent, const Rec& o, u32 first) {
    Span e = w.cget(idx);
    if (e.len <= 0) return 0;
    if (e.order + (u32)e.len != first) return 0;
    if (e.orr != orr) return 0;
    u32 total;
    u32 nt = typing_run(b0, nv, remote, agent, o.w1, o, total);
    if (g(K_MAP) - first < total) return 0;     // capacity: the general path stops exactly
    map_fill(first, total, g(C_LEAF));   // notify (doc.rs:143-153)
    e.len += (i32)total;
    w.cset(idx, e);  // (e is visible: the count grows by total)
    p(C_NOW, g(C_NOW) + total);
    p(C_DIRTY, 1u);
    fast_txn_commit(first, total);
    return nt * per_txn(remote);
  }
  // Delete `l` items at offset `off` of visible entry idx of the cached leaf: mutate_entry
  // (mutations.rs:227-277) and insert_internal's prepend / shift (mutations.rs:84-146) without a
  // leaf split.  Returns 0, having changed nothing, when the leaf has no room.
  CRDT_HD u32 leaf_delete(u32 idx, u32 off, u32 l) {
    Span e = w.cget(idx);
    u32 n = g(C_N);
    u32 target = e.order + off;
    u32 ha = off > 0u, hc = off + l < (u32)e.len;
    Span pa{e.order, e.ol, e.orr, (i32)off};
    Span dd{target, ha ? target - 1u : e.ol, e.orr, -(i32)l};
    Span pc{target + l, target + l - 1u, e.orr, e.len - (i32)(off + l)};
    Span x0 = ha ? dd : pc;  // pieces after the cursor entry: [x0, pc][:m]
    u32 m = ha + hc;
    u32 pre = 0;
    Span nx{0, 0, 0, 0};
    if (m != 0u) {
      if (idx + 1u < n) {
        nx = w.cget(idx + 1u);
        Span last = m == 2u ? pc : x0;
        if (can_append_u(last, nx)) {
          nx.order = last.order;  // YjsSpan::prepend keeps origin_left (span.rs:61-64)
          nx.len += last.len;
          pre = 1;
          m -= 1u;
        }
      }
    }
    if (n + m > (u32)L) return 0;
    // entry writes straight to the cache; the visible count drops by exactly the l deleted items
    w.cset(idx, ha ? pa : dd);
    if (pre) w.cset(idx + 1u, nx);
    if (m) {
      w.cache_shift_right(idx + 1u, n, m);
      p(C_N, n + m);
      w.cset(idx + 1u, x0);
      if (m == 2u) w.cset(idx + 2u, pc);
      inc(S_N_ENTRIES, m);
    }
    p(C_NOW, g(C_NOW) - l);
    p(C_DIRTY, 1u);
    return 1;
  }
  // A run of k >= 2 one-item deletes in closed form (the per-op rules of leaf_delete, solved once):
  //  * backspacing from the last item of entry E (idx): every delete splits E's last item off and
  //    either prepends it onto the entry after E or inserts it there.  A fresh single deleted item
  //    {t, t-1} accepts the next one (YjsSpan::can_append), after which its origin_left equals
  //    its order (span.rs:61-64) and it accepts no more: new entries alternate insert / prepend,
  //    starting with a prepend onto the next entry N0 iff can_append_u(first deleted item, N0);
  //  * forward deleting from item `off` of E (the remainder never prepends onto the next
  //    entry): E becomes [E[..off]] [k single deleted items] [the rest of E].
  // Returns k' <= k deletes applied (0: not this shape / no room; nothing changed).
  CRDT_HD u32 delete_run_closed(u32 idx, u32 off, u32 t1, u32 k, u32 back) {
    Span E = w.cget(idx);
    u32 n = g(C_N);
    u32 orr = E.orr;
    u32 has_nx = idx + 1u < n;
    Span N0 = w.cget(idx + 1u);
    u32 room = (u32)L - n;  // new entries the leaf can take
    u32 delta;
    if (back) {
      // Backspacing from inside E (not its last item): the run's first delete splits E after its
      // target, so E[off+1..] becomes the entry after E; it is visible and the deleted items are
      // not, so nothing prepends onto it (p0 = 0) and the run is the end-of-entry case on
      // E[..off+1] with one entry more (mutate_entry, mutations.rs:227-277, gives the same leaf).
      u32 mid = off + 1u != (u32)E.len ? 1u : 0u;
      u32 p0 = 0u;
      if (mid) {
        if (room == 0u) return 0;
        room -= 1u;
      } else if (has_nx) {
        p0 = can_append_u(Span{t1, t1 - 1u, orr, -1}, N0) ? 1u : 0u;
      }
      u32 kmax = 2u * room + p0;
      k = k < off ? k : off;  // E keeps its first item (deleting it is a different shape)
      k = k < kmax ? k : kmax;
      if (k < 2u) return 0;
      if (mid) {
        Span pc = truncate(E, off + 1u);  // (E's visible items stay in E + pc)
        w.cache_shift_right(idx + 1u, n, 1u);
        w.cset(idx + 1u, pc);
        n += 1u;
        inc(S_N_ENTRIES, 1u);
      }
      delta = p0 ? k / 2u : (k + 1u) / 2u;  // new entries F_1..F_delta, newest first after E
      w.cache_shift_right(idx + 1u, n, delta);
      w.cset_lanes(idx + 1u, idx + 1u + delta, [&](u32 lane) {
        u32 q = delta - (lane - idx - 1u);           // F_q
        u32 jc = p0 ? 2u * q : 2u * q - 1u;          // the op (1-based) that created it
        u32 tc = t1 - (jc - 1u);
        u32 two = jc + 1u <= k ? 1u : 0u;  // {tc-1, tc-1, orr, -2} or {tc, tc-1, orr, -1}: arithmetic, no selects
        return Span{tc - two, tc - 1u, orr, (i32)~two};
      });
      if (p0) w.cset(idx + 1u + delta, Span{t1, N0.ol, N0.orr, N0.len - 1});
      E.len = (i32)(off + 1u - k);
      w.cset(idx, E);
    } else {
      u32 ha = off > 0u;
      if (has_nx && can_append_u(Span{t1 + 1u, t1, orr, E.len - (i32)off - 1}, N0)) return 0;
      u32 kmax = room > ha ? room - ha : 0u;  // adds ha + k entries with a remainder (one fewer without)
      k = k < kmax ? k : kmax;
      if (k < 2u) return 0;
      u32 rest = (u32)E.len - off - k;
      u32 cnt = ha + k + (rest != 0u);
      delta = cnt - 1u;
      w.cache_shift_right(idx + 1u, n, delta);
      w.cset_lanes(idx, idx + cnt, [&](u32 lane) {
        u32 p = lane - idx;
        u32 j = p - ha;  // deleted item j (0-based), or the remainder when j == k
        if (ha && p == 0u) return Span{E.order, E.ol, orr, (i32)off};
        if (j < k) return Span{t1 + j, (j == 0u && !ha) ? E.ol : t1 + j - 1u, orr, -1};
        return Span{t1 + k, t1 + k - 1u, orr, (i32)rest};
      });
    }
    p(C_N, n + delta);
    inc(S_N_ENTRIES, delta);
    p(C_NOW, g(C_NOW) - k);
    p(C_DIRTY, 1u);
    return k;
  }
  // Delete txns: the one at b0 (l items at `off` of entry idx) and, when it deletes one item, the
  // run of one-item delete txns that follows it in the prefetch block -- backspacing (each
  // deletes the item before the previous one) or forward deleting (the item after) -- validated
  // lane-parallel (W::delete_scan).  Each delete is applied to the leaf exactly as apply_txn
  // would (leaf_delete); the RLE tables, the order map and the txn log are updated once for the
  // run.  Returns records consumed (0: nothing applied).
  CRDT_HD u32 fast_deletes(u32 b0, u32 nv, u32 remote, u32 agent, u32 idx, u32 off, u32 l, u32 first, const Rec& o) {
#ifdef CRDT_PROF
    u64 pt0 = w.clock();  // detail (prof_mode 3): cycles of run detection / first segment / leaf-split loop / tail
#endif
    u32 per = per_txn(remote);
    u32 t1 = w.cget_order(idx) + off;
    u32 split_first = 0;
    if (g(C_N) + 2u > (u32)L) {  // near-full leaf: does the first delete fit (leaf_delete's rule)?
      Span e = w.cget(idx);
      u32 n = g(C_N), ha = off > 0u, hc = off + l < (u32)e.len, m = ha + hc;
      if (m && idx + 1u < n) {
        Span last = hc ? Span{t1 + l, t1 + l - 1u, e.orr, e.len - (i32)(off + l)}
                       : Span{t1, ha ? t1 - 1u : e.ol, e.orr, -(i32)l};
        m -= can_append_u(last, w.cget(idx + 1u));
      }
      if (n + m > (u32)L) split_first = 1;  // the leaf must split for it
    }
    u32 k = 1, back = 0;
    u32 key = g(T_AGL_KEY);
    // a run of one-item deletes follows?  The shape checks fold into one integer (one branch, so
    // the two results have one merge), the next txn's target / pos read unconditionally (a window
    // lane; ignored unless the checks pass)
    u32 delta;
    u32 has_next = b0 + 2u * per <= nv ? 1u : 0u;
    u32 bn = has_next ? b0 + per : b0;  // (a valid window slot either way)
    if (cpt) {  // compact records: the next txn's target seq (RC w2) / pos (LC w1) read directly
      Rec r2 = w.rec_get(bn);
      delta = remote ? r2.w2 - o.w2 : r2.w1 - o.w1;
    } else {
      Rec o2 = op_at(bn, remote);
      delta = remote ? o2.w2 - o.w2 : o2.w1 - o.w1;
    }
    u32 bk = delta == 0xFFFFFFFFu ? 1u : 0u;
    u32 bad = (l ^ 1u) | (has_next ^ 1u) | ((delta != (remote ? 1u : 0u) ? 1u : 0u) & (bk ^ 1u));
    if (remote) bad |= ((o.w1 & 0xFFFFu) ^ agent) | (o.w2 - key >= g(T_AGL_LEN) ? 1u : 0u);
    if (opq(bad) == 0u) {
      back = opq(bk);
      {
        u32 room = back ? off + 1u : (u32)w.cget_len(idx) - off;  // targets stay in this entry
        if (remote) {  // ... and in the author's last item_orders run (contiguous orders)
          u32 r2 = back ? o.w2 - key + 1u : key + g(T_AGL_LEN) - o.w2;
          room = room < r2 ? room : r2;
        }
        k = w.delete_scan(b0, nv, remote, cpt, agent, delta);
        // the run may go on past the window: slide the window to its last txn and scan on
        u32 rn = rec_n();
        u32 pos0 = g(T_RB_BASE) + b0;
        u32 end = g(T_RB_BASE) + nv;
        while (true) {
          if (k >= room) break;
          if (pos0 + (k + 1u) * per <= end) break;
          if (end >= rn) break;
          u32 last = pos0 + (k - 1u) * per;
          u32 n = rn - last < 64u ? rn - last : 64u;
          u32 n2 = w.delete_scan_at(w.at(recs(), last), n, remote, cpt, agent, delta);
          end = last + n;
          if (n2 <= 1u) break;
          k += n2 - 1u;
        }
#ifdef CRDT_PROF

#endif
        k = k < room ? k : room;
      }
    }
#ifdef CRDT_PROF

#endif
    if (g(K_MAP) - first < k * l) return 0;
    // delete-log room: a backspace run logs one run per item, a forward run coalesces into one
    // (was k for both: after crdt_fit the log's room is the stream's own count, so every forward
    // run of a fitted document took the general path)
    if (g(K_DEL) - g(S_N_DEL) < (back ? k : 1u)) return 0;
#ifdef CRDT_PROF
    u64 pt1 = w.clock();
#endif
    u32 done = split_first ? 0u : delete_segment(idx, off, t1, k, back, l);
#ifdef CRDT_PROF
    u64 pt2 = w.clock();
#endif
    // The leaf ran out of room (or the run reached a shape the segment does not take): the next
    // delete goes the general way -- mutate_entry + insert_internal, splitting the leaf -- and the
    // rest of the run continues from wherever its next target now lives.
    CRDT_STAT(9, 1); CRDT_STAT(12, k); CRDT_STAT(13, split_first);
#ifdef CRDT_PROF_LOOP
    u32 lp_gen = 0, lp_split = 0, lp_find = 0, lp_seg = 0;
#endif
    while (done < k) {
#ifdef CRDT_PROF_LOOP
      u64 q0 = w.clock();
#endif
      CRDT_STAT(10, 1);
      if (g(K_LEAF) - g(S_N_LEAVES) < 2u) break;
      Cursor c{g(C_LEAF), idx, off};
      if (done != 0u) {
        if (!find_order(back ? t1 - done : t1 + done, true, c)) break;
      }
      i32 el = w.cget_len(c.idx);
      if (el <= 0) break;
      if (c.off + l > (u32)el) break;
      if (back & (el == 1)) {  // a one-item entry: mutate_entry deactivates it in place (mutations.rs:265-273)
        w.cset_len(c.idx, -1);
        p(C_NOW, g(C_NOW) - 1u);
        p(C_DIRTY, 1u);
        done++;
        continue;
      }
      CRDT_STAT(back ? 48 : 49, 1); CRDT_STAT(52, c.off == 0u);
#ifdef CRDT_PROF_LOOP
      u64 q1 = w.clock();
      prof_split = 0;
#endif
      delete_general(c.idx, c.off, l, back);
#ifdef CRDT_PROF_LOOP
      u64 q2 = w.clock();
      lp_gen += (u32)(q2 - q1) - prof_split;
      lp_split += prof_split;
      lp_find += (u32)(q1 - q0);
#endif
      done++;
      if (done == k) break;
      u32 t2 = back ? t1 - done : t1 + done;
      // (backspacing from inside an entry: the item before the deleted one ends the entry's first
      // part, which stays at its index of the cached leaf -- no lookup)
      if (back & (c.off != 0u)) c.off -= 1u;
      else if (!find_order(t2, true, c)) break;
      el = w.cget_len(c.idx);
      if (el <= 0) break;
      if (c.off + l > (u32)el) break;
#ifdef CRDT_PROF_LOOP
      u64 q3 = w.clock();
      lp_find += (u32)(q3 - q2);
#endif
      // the split left the run in its repeating state: whole cycles in closed form
      if (back & (c.leaf == g(C_LEAF)) & (l == 1u)) {
        u32 dc = back_cycles(c.idx, t2, k - done);
        CRDT_STAT(57, dc != 0u); CRDT_STAT(58, dc);
        if (dc) {
          done += dc;
          if (done == k) break;
          t2 -= dc;
          c.off -= dc;
        }
      }
      u32 dseg = delete_segment(c.idx, c.off, t2, k - done, back, l);
#ifdef CRDT_PROF_LOOP
      lp_seg += (u32)(w.clock() - q3);
#endif
      CRDT_STAT(53, dseg); CRDT_STAT(54, dseg == 0u);
      done += dseg;
    }
#ifdef CRDT_PROF
    u64 pt3 = w.clock();
#endif
    if (done == 0u) return 0;
    if (back) {  // doc.rs:305-308 / 420-423: backspaced targets never coalesce: one run each
      append_delete(first, t1, 1u);
      if (done > 1u) {
        u32 n = g(S_N_DEL);
        w.st(&w.at(dels(), n - 1u)->len, g(T_DEL_LEN));  // retire the tail
        w.st_del_run(w.at(dels(), n), done - 1u, first + 1u, t1 - 1u);
        p(S_N_DEL, n + done - 1u);
        p(T_DEL_KEY, first + done - 1u);
        p(T_DEL_ORDER, t1 - (done - 1u));
        p(T_DEL_LEN, 1u);
      }
    } else {
      append_delete(first, t1, done * l);  // forward deletes coalesce into one run (Rle::append)
    }
    fast_txn_commit(first, done * l);  // (delete orders name no item: no order -> leaf entries)
#ifdef CRDT_PROF
    if (prof_mode == 3u && !prof_gen) {
#ifdef CRDT_PROF_LOOP
      (void)pt0; (void)pt1; (void)pt2; (void)pt3;
      inc(S_PROF0, lp_gen); inc(S_PROF1, lp_split); inc(S_PROF2, lp_find); inc(S_PROF3, lp_seg);
#else
      inc(S_PROF0, (u32)(pt1 - pt0)); inc(S_PROF1, (u32)(pt2 - pt1));
      inc(S_PROF2, (u32)(pt3 - pt2)); inc(S_PROF3, (u32)(w.clock() - pt3));
#endif
    }
#endif
    return done * per;
  }
  // Up to k one-item deletes of a run (the first at `off` of entry idx, target t), in closed form
  // or op by op, while the leaf has room.  Returns the deletes applied.
  CRDT_HD u32 delete_segment(u32 idx, u32 off, u32 t, u32 k, u32 back, u32 l) {
    u32 done = k >= 2u ? delete_run_closed(idx, off, t, k, back) : 0u;
    CRDT_STAT(11, done); CRDT_STAT(14, 1);
    if (done == 0u) {  // op by op
      for (u32 j = 0; j < k; j++) {
        u32 ij = back ? idx : (j == 0u ? idx : idx + (off > 0u) + j);  // forward: the remainder moves right
        u32 oj = back ? off - j : (j == 0u ? off : 0u);
        u32 tj = back ? t - j : t + j;
        if (w.cget_order(ij) + oj != tj) break;
        if (w.cget_len(ij) <= (i32)oj) break;
        if (!leaf_delete(ij, oj, l)) break;
        done++;
      }
    }
    return done;
  }
  // One delete of l items at offset `off` of visible entry idx, exactly as apply_txn does it:
  // mutate_entry (mutations.rs:227-277: the entry's first part stays at idx, the deleted piece and
  // the visible remainder go after it) and insert_internal (mutations.rs:17-179), splitting the
  // leaf when the pieces do not fit (split_at, :623-669).  insert_internal's steps specialised to
  // these pieces: the first part never absorbs the next piece (one is visible, the other deleted),
  // at most the last piece prepends onto the entry after idx (YjsSpan::prepend keeps origin_left),
  // and the rest (m <= 2 entries) is inserted at idx + 1.  The caller checked that a leaf is free.
  // back: a backspace run goes on at the item before t, in the first part at idx: a split that
  // would move the cache to the new leaf writes the pieces there in HBM and keeps the old leaf.
  CRDT_HD void delete_general(u32 idx, u32 off, u32 l, u32 back) {
    CRDT_STAT(7, 1);
    Span e = w.cget(idx);
    u32 n = g(C_N);
    u32 t = e.order + off;
    u32 ha = off > 0u ? 1u : 0u, hc = off + l < (u32)e.len ? 1u : 0u;
    Span pa{e.order, e.ol, e.orr, (i32)off};
    Span dd{t, ha ? t - 1u : e.ol, e.orr, -(i32)l};
    Span pc{t + l, t + l - 1u, e.orr, e.len - (i32)(off + l)};
    Span x0 = ha ? dd : pc;  // pieces after the first part: [x0, pc][:m]
    u32 m = ha + hc;
    u32 pre = 0, pre_vis = 0;
    Span nx{0, 0, 0, 0};
    if (m != 0u) {
      if (idx + 1u < n) {
        nx = w.cget(idx + 1u);
        Span last = m == 2u ? pc : x0;
        if (can_append_u(last, nx)) {
          nx.order = last.order;
          nx.len += last.len;
          pre = 1;
          pre_vis = last.len > 0 ? (u32)last.len : 0u;
          m -= 1u;
        }
      }
    }
    w.cset(idx, ha ? pa : dd);
    if (pre) w.cset(idx + 1u, nx);
    // the cache now holds everything but the m unplaced pieces: e's l deleted items and the
    // visible pieces still to place are off its count
    u32 unplaced_vis = (hc && !pre) ? (u32)pc.len : 0u;
    p(C_NOW, g(C_NOW) - l - unplaced_vis);
    p(C_DIRTY, 1u);
    (void)pre_vis;
    CRDT_STAT(50, m == 0u);
    if (m == 0u) return;
    inc(S_N_ENTRIES, m);
    u32 ci = idx + 1u;
    u32 home = g(C_LEAF);
    u32 leaf = home;
    u32 at = ci;
    if (n + m > (u32)L) {
      u32 follow = ci >= (u32)L / 2u ? 1u : 0u;
      u32 moved = n - ci;
      u32 succ = g(C_SUCC), succ_ord = g(C_SUCC_ORD);  // the old leaf's successor follows nl
      CRDT_STAT(follow & back ? 4 : follow ? 5 : 6, 1);
      if (follow & back) {  // the pieces lead the new leaf in HBM; the old leaf stays cached
        u32 nl = split_at(ci, m, unplaced_vis);
        Span* q = leafp(nl);
        w.st_span(q, x0);
        notify(x0, nl, home);
        if (m == 2u) {
          w.st_span(q + 1, pc);
          notify(pc, nl, home);
        }
        return;
      }
      u32 nl = split_at(ci, follow ? m : 0u);
      if (follow) {  // the pieces lead the new leaf, which becomes the cached one (insert_items)
        u32 nblk = g(C_BLK), ni = g(C_I) + 1u;
        commit();
        w.cache_from_moved();
        u32 v = w.cache_vis_from(0u);
        p(C_LEAF, nl); p(C_BLK, nblk); p(C_I, ni);
        p(C_NOW, v); p(C_VIS, v); p(C_DIRTY, 1u); p(C_VSTART, VS_BAD);
        p(C_SUCC, succ); p(C_SUCC_ORD, succ_ord);
        p(C_N, m + moved);
        leaf = nl;
        at = 0u;
      } else {
        p(C_N, ci + m);
      }
    } else {
      CRDT_STAT(51, 1);
      w.cache_shift_right(ci, n, m);
      p(C_N, n + m);
    }
    notify(x0, leaf, home);
    w.cset(at, x0);
    if (m == 2u) {
      notify(pc, leaf, home);
      w.cset(at + 1u, pc);
    }
    p(C_NOW, g(C_NOW) + unplaced_vis);
  }
  // Insert one item run right after the cursor (idx, off), 0 < off <= |entry|, when integrate
  // stops at once and the run cannot be appended: insert_internal (mutations.rs:17-179) splits
  // the entry at the cursor (remainder after the item) and makes room, without a leaf split.
  // Returns 0, having changed nothing, when the leaf or the order map has no room.
  CRDT_HD u32 leaf_insert(u32 idx, u32 off, const Span& item) {
    Span e = w.cget(idx);
    u32 n = g(C_N);
    u32 len = (u32)item.len;
    u32 has_rem = off < slen(e);
    u32 space = 1u + has_rem;  // (fits: the caller sent n + space > L to the split path)
    CRDT_EXPECT(n + space <= (u32)L);
    if (g(K_MAP) - item.order < len) return 0;
    // entry writes straight to the cache (truncating e keeps its visible items in e + rem); the
    // visible count grows by exactly the item's len
    if (has_rem) {
      Span rem = truncate(e, off);
      w.cset(idx, e);
      w.cache_shift_right(idx + 1u, n, 2u);
      w.cset(idx + 2u, rem);
    } else {
      w.cache_shift_right(idx + 1u, n, 1u);
    }
    p(C_N, n + space);
    inc(S_N_ENTRIES, space);
    map_fill(item.order, len, g(C_LEAF));  // notify (doc.rs:143-153)
    w.cset(idx + 1u, item);
    p(C_NOW, g(C_NOW) + len);
    p(C_DIRTY, 1u);
    return 1;
  }
  // The item as entry 0 of the cached first leaf (cursor at the start of the document, offset 0 at
  // index 0: insert_internal neither rolls back nor splits, mutations.rs:34-52) without a leaf split
  // -- and with it the rest of a front run: k local txns that each insert len chars at position 0
  // (the reference's `kevin` benchmark shape, benches/yjs.rs:51-62).  Prepend j (0-based) gets
  // orders first + j*len, origin_left ROOT and origin_right = the item at position 0 before it
  // (the item's for j = 0, else prepend j-1's first item; doc.rs:443-453); integrate stops at once
  // and insert_internal puts it at index 0, never prepending it onto entry 0 (orders only grow).
  // So the prepends that fit the leaf are one shift plus one lane-parallel write, newest at lane
  // 0.  The prepend that finds the leaf full is what insert_internal does with an item at index
  // 0 of a full leaf: split_at(0) moves every entry to a new leaf linked right after it
  // (mutations.rs:96-121, the cursor does not follow), and the item is entry 0 of the emptied
  // leaf -- which the next prepends fill again.  So a front run goes on through the splits.
  // Each chunk is committed as it is placed (fast_txn_commit: the first one's order is
  // S_NEXT_ORDER).  orr0: the first prepend's origin_right.  Returns the txns placed (0: no room,
  // nothing changed).
  // A front run's prepends that fit the cached leaf, committed (fast_txn_commit; the first one's
  // order is S_NEXT_ORDER).  Returns the txns placed (0: no room, nothing changed).
  CRDT_HD u32 leaf_insert_front(u32 orr0, u32 len, u32 rem) {
    u32 n = g(C_N);
    u32 m = (u32)L - n;
    m = m < rem ? m : rem;
    if (m == 0u) return 0u;
    u32 first = g(S_NEXT_ORDER);
    if (g(K_MAP) - first < m * len) return 0u;
    w.cache_shift_right(0u, n, m);
    p(C_N, n + m);
    inc(S_N_ENTRIES, m);
    map_fill(first, m * len, g(C_LEAF));  // notify (doc.rs:143-153)
    u32 top = m - 1u;
    w.cset_lanes(0u, m, [&](u32 lane) {
      u32 j = top - lane;
      u32 o = first + j * len;
      return Span{o, ROOT_ORDER, j == 0u ? orr0 : o - len, (i32)len};
    });
    p(C_NOW, g(C_NOW) + m * len);
    p(C_DIRTY, 1u);
    fast_txn_commit(first, m * len);
    return m;
  }
  // A local delete of l visible items that starts at offset `off` of visible entry idx of the
  // cached leaf and runs past that entry (rem: the visible position of its first item within the
  // leaf).  local_deactivate (mutations.rs:520-570) visits the entries in order, skipping deleted
  // ones, and mutate_entry (:227-277) deactivates each visible one:
  //  * entry idx: in place from offset 0, else [E[..off]] then the deleted rest d0, which
  //    insert_internal (:17-179) prepends onto the entry after idx when that one is a deleted run
  //    d0 can append to (a visible entry cannot take it), else inserts at idx + 1;
  //  * every visible entry up to the last one: in place (the delete continues past it);
  //  * the last entry kl: in place when the delete ends at its end, else [its deleted head] then
  //    the visible rest c, prepended onto the entry after kl or inserted there.
  // The deletes log gets one append per deactivated piece, in document order (doc.rs:414-426).
  // Conditions are evaluated on the leaf as the reference's order of steps sees it: the entry
  // after idx is untouched when d0 goes in, the entry after kl when c goes in.  Returns 0, having
  // changed nothing, when the delete leaves the leaf or the leaf has no room (the general path
  // then splits it).
  CRDT_HD u32 leaf_delete_span(u32 idx, u32 off, u32 l, u32 rem, u32 first) {
    // (few scalars live at a time, entries re-read from the cache where they are written: this
    // path shares the replay's register budget with the hot loops)
    u32 n = g(C_N);
    u32 kl, ol;
    if (!w.cfind_content(n, rem + l - 1u, kl, ol)) return 0;
    if (kl >= n) return 0;
    if (g(K_DEL) - g(S_N_DEL) < (l < (u32)L ? l : (u32)L)) return 0;  // (one delete run per deactivated piece at most: <= L pieces)
    if (g(K_MAP) - first < l) return 0;
    u32 rl = ol + 1u;  // items deleted from entry kl
    // the pieces insert_internal places, and whether each prepends onto the entry after it
    u32 c_add = 0u, c_pre = 0u;
    {
      Span Z = w.cget(kl);
      if (rl < (u32)Z.len) {
        c_add = 1u;
        if (kl + 1u < n) c_pre = can_append_u(Span{Z.order + rl, Z.order + rl - 1u, Z.orr, Z.len - (i32)rl}, w.cget(kl + 1u)) ? 1u : 0u;
      }
    }
    u32 d_add = 0u, d_pre = 0u;
    if (off) {
      Span E = w.cget(idx);
      d_add = 1u;
      d_pre = can_append_u(Span{E.order + off, E.order + off - 1u, E.orr, (i32)off - E.len}, w.cget(idx + 1u)) ? 1u : 0u;  // (idx < kl < n)
    }
    u32 add = (d_add & (d_pre ^ 1u)) + (c_add & (c_pre ^ 1u));
    if (n + add > (u32)L) return 0;
    // deletes log: the deactivated pieces in document order (entries idx .. kl as they are now)
    u32 key = first;
    for (u64 m = w.vis_lanes(idx, kl + 1u); m; m &= m - 1ull) {
      u32 j = W::first_lane(m);
      u32 s0 = j == idx ? off : 0u;
      u32 ln = (j == kl ? rl : (u32)w.cget_len(j)) - s0;
      append_delete(key, w.cget_order(j) + s0, ln);
      key += ln;
    }
    // the leaf, from the right end (so that earlier indices stay put)
    {
      Span Z = w.cget(kl);
      Span cc{Z.order + rl, Z.order + rl - 1u, Z.orr, Z.len - (i32)rl};
      Z.len = -(i32)rl;
      w.cset(kl, Z);
      if (c_add) {
        if (c_pre) {
          Span nx = w.cget(kl + 1u);
          nx.order = cc.order;  // YjsSpan::prepend keeps origin_left (span.rs:61-64)
          nx.len += cc.len;
          w.cset(kl + 1u, nx);
        } else {
          w.cache_shift_right(kl + 1u, n, 1u);
          w.cset(kl + 1u, cc);
          n += 1u;
        }
      }
    }
    w.negate_visible(idx + 1u, kl);  // the entries strictly between idx and kl
    {
      Span E = w.cget(idx);
      if (d_add) {
        Span d0{E.order + off, E.order + off - 1u, E.orr, (i32)off - E.len};
        E.len = (i32)off;
        w.cset(idx, E);
        if (d_pre) {
          Span n1 = w.cget(idx + 1u);
          n1.order = d0.order;
          n1.len += d0.len;
          w.cset(idx + 1u, n1);
        } else {
          w.cache_shift_right(idx + 1u, n, 1u);
          w.cset(idx + 1u, d0);
          n += 1u;
        }
      } else {
        E.len = -E.len;
        w.cset(idx, E);
      }
    }
    p(C_N, n);
    inc(S_N_ENTRIES, add);
    p(C_NOW, g(C_NOW) - l);
    p(C_DIRTY, 1u);
    fast_txn_commit(first, l);
    return 1;
  }
  // A local delete of l visible items at pos that leaf_delete_span could not place in the cached
  // leaf (it runs past the leaf's end, or the leaf has no room): local_deactivate's pieces one at a
  // time (mutations.rs:520-570).  Each step finds the first visible item still at pos (the deleted
  // ones are no longer visible there), deactivates its entry in place when the piece is the whole
  // entry (mutate_entry, mutations.rs:265-273), else splits it the way mutate_entry +
  // insert_internal do (delete_general: the deleted piece and the visible rest placed after the
  // head, prepended onto the next entry of the same leaf when it can take them, the leaf split when
  // they do not fit), and logs the piece (doc.rs:414-426, document order).  Only the first and the
  // last piece split an entry, so at most two leaf splits: with the general path's room for one op
  // (two free leaves) and delete-log room for l runs nothing can stop it part-way.  Returns 0,
  // having changed nothing, when that room is not there or the range is past the document's end
  // (the general path then reports it).
  CRDT_HD u32 local_delete_pieces(u32 pos, u32 l, u32 first) {
    if ((u64)pos + l > cur_len()) return 0;
    if (g(K_LEAF) - g(S_N_LEAVES) < 2u) return 0;
    if (g(K_DEL) - g(S_N_DEL) < l) return 0;
    if (g(K_MAP) - first < l) return 0;
    u32 key = first, rem = l;
    while (rem) {
      Cursor c;
      bool ok = cursor_at_content_pos(pos, c);
      CRDT_EXPECT(ok && c.idx < g(C_N) && w.cget_len(c.idx) > 0);
      i32 sl = ok ? w.cget_len(c.idx) : 0;
      if (sl <= (i32)c.off) {  // (cannot happen: pos + rem <= len holds at every step; never loop on it)
        p(S_STATUS, (u32)ST_INTERNAL);
        return 1;
      }
      u32 el = (u32)sl;
      u32 piece = el - c.off < rem ? el - c.off : rem;
      u32 t = w.cget_order(c.idx) + c.off;
      if ((c.off == 0u) & (piece == el)) {
        w.cset_len(c.idx, -(i32)el);
        p(C_NOW, g(C_NOW) - el);
        p(C_DIRTY, 1u);
      } else {
        delete_general(c.idx, c.off, piece, 0u);
      }
      append_delete(key, t, piece);
      key += piece;
      rem -= piece;
    }
    fast_txn_commit(first, l);
    return 1;
  }
  // Returns the records consumed by a fast-path txn at `pos`, or 0 (use apply_txn).
  // gen: a txn expanded from a GEN record (header gh, op go; no record window, no runs).
  // kind: the record kind at `pos` (RTXN / LTXN / RC / LC; LTXN for a generated op).
  CRDT_HD u32 fast_txn(u32 pos, u32 kind, u32 gen, const Rec& gh, const Rec& go) {
    CRDT_MEM_EPOCH();
    // set membership by bitmask: no lane-mask booleans
    cpt = ((1u << REC_RC | 1u << REC_LC) >> kind) & 1u;
    u32 remote = ((1u << REC_RTXN | 1u << REC_RC) >> kind) & 1u;
    u32 per = per_txn(remote);
    u32 rn = rec_n();
    if (!gen) {  // (the GEN loop is entered with a cached leaf, which the fast paths never drop)
      if (g(C_LEAF) == INVALID) return 0;
    }
    u32 b0 = 0, nv = 0;
    Rec h = gh, o = go, pr{0, 0, 0, 0};
    if (!gen) {
      // run() read the record at pos through the window (gh): a compact txn is that one record
      b0 = pos - g(T_RB_BASE);
      if (cpt) {
        if (!remote) expand_lc(h, h, o);  // (RC is decoded directly below)
      } else {
        if (rn - pos < per) return 0;  // (rec() left the whole txn inside the window: b0 <= 61)
        h = w.rec_get(b0);
        o = w.rec_get(b0 + 1u);
        if (remote) pr = w.rec_get(b0 + 2u);
      }
      nv = rn - g(T_RB_BASE);
      nv = nv < 64u ? nv : 64u;
    }
    // compact records and generated ops are one-op txns by construction (expand_rc / expand_lc
    // / gen_op): only the general form needs its header checked
    u32 gen_form = !(cpt | gen);
    u32 first = g(S_NEXT_ORDER);
    u32 agent, l, ins, ol = 0, orr = ROOT_ORDER;
    Cursor c;
    if (remote && cpt) {
      // RC: the compact record's fields directly (expand_rc's header, op and parent, without its
      // origin-agent selects): author, seq, len, del; origins / target are the author's own items
      // (a seq of 0xFFFFFFFF names ROOT) and the one parent is (author, seq - 1), so once
      // fast_txn_ok has matched the author with the cached agent, every lookup is a tail check
      Rec r = gh;
      agent = r.w0 & 0xFFFFu;
      u32 seq = r.w1;
      l = rc_len(r);
      u32 del = (r.w0 >> 27) & 1u;
      ins = del ^ 1u;
      u32 ra = r.w3 == 0xFFFFFFFFu ? ROOT_AGENT : agent;
      // the op record as expand_rc's insert form; the delete paths read only its author (low half
      // of w1) and target seq (w2), which the two forms share, so no per-field select
      o = Rec{(REC_RINS << 28) | l, agent | (ra << 16), r.w2, r.w3};
      if (l == 0u) return 0;
      if (!fast_txn_ok(agent, seq, first)) return 0;
      if (r.w2 == 0xFFFFFFFFu) return 0;                   // origin_left / target ROOT
      if (!seq_to_order(agent, r.w2, ol)) return 0;        // (agent == T_AG_ID: a valid agent)
      if (ins) {
        if (r.w3 != 0xFFFFFFFFu) {
          if (!seq_to_order(agent, r.w3, orr)) return 0;
        }
      }
      if (!find_order(ol, true, c)) return 0;  // doc.rs:101-136 (loads the item's leaf)
      c.off += ins;                             // get_cursor_after
    } else if (remote) {
      agent = h.w1 & 0xFFFFu;
      u32 seq = h.w2;
      l = o.w0 & 0x0FFFFFFFu;
      u32 k = rec_kind(o);
      ins = k == REC_RINS;
      if (gen_form) {
        u32 ok = ((h.w0 & ~(1u << RTXN_DEL_BIT)) == ((REC_RTXN << 28) | 1u)) & ((h.w1 >> 16) == 1u) & (h.w3 == l) & (l - 1u < 0xFFFFu) &
                 (pr.w0 == (REC_RPARENT << 28)) & (pr.w1 == agent) & (pr.w2 == seq - 1u) & (ins | (k == REC_RDEL));
        if (!ok) return 0;
      } else if (l == 0u) {
        return 0;
      }
      if (!fast_txn_ok(agent, seq, first)) return 0;
      if (id_to_order(o.w1 & 0xFFFFu, o.w2, ol) != ST_OK) return 0;  // origin_left / target
      if (ol == ROOT_ORDER) return 0;
      if (ins) {
        if (id_to_order(o.w1 >> 16, o.w3, orr) != ST_OK) return 0;
      }
      if (!find_order(ol, true, c)) return 0;  // doc.rs:101-136 (loads the item's leaf)
      c.off += ins;                             // get_cursor_after
    } else {
      agent = h.w1;
      u32 lp = o.w1, del = o.w2;
      ins = o.w3 != 0u;
#ifdef CRDT_PROF
      prof_cat = ins ? 3u : 2u;
#endif
      l = del + o.w3;
      if (!gen) {  // (a generated op is one insert of 1 char or one delete of 1..10: well-formed by construction)
        if ((del != 0u) == ins) return 0;
        if (l - 1u >= 0xFFFFu) return 0;
      }
      if (gen_form) {
        u32 ok = (h.w0 == ((REC_LTXN << 28) | 1u)) & (o.w0 == (REC_LOP << 28)) & (h.w2 == del) & (h.w3 == l);
        if (!ok) return 0;
      }
      if (!gen) {  // (the GEN loop checks it once on entry: its fast commits keep it true)
        if (!fast_txn_ok(agent, g(T_AGL_KEY) + g(T_AGL_LEN), first, 1u)) return 0;
      }
      if (ins && lp == 0u) {
        // doc.rs:443-444: origin_left ROOT, the cursor at the start of the document (root.rs:133-
        // 150); integrate stops at once (origin_right is the item there) and insert_internal puts
        // the item before entry 0 (offset 0 at index 0: nothing to append to)
        c = cursor_at_start();
        ensure(c.leaf);
        p(C_VSTART, 0u);  // (the first leaf starts at visible position 0)
        ol = ROOT_ORDER;
      } else {
        if (!cursor_at_content_pos(ins ? lp - 1u : lp, c)) return 0;  // root.rs:54-88 (loads the leaf)
        ol = w.cget_order(c.idx) + c.off;  // doc.rs:446-449: the item at pos - 1, then Cursor::next
        c.off += ins;
        if (!ins) {
          // a delete that runs past its first entry (local_deactivate over several entries of
          // the cached leaf): the multi-entry form, when it stays in the leaf
          i32 el = w.cget_len(c.idx);
          if (el > 0 && c.off + l > (u32)el) {
            if (leaf_delete_span(c.idx, c.off, l, lp - g(C_VSTART), first)) return per;
            return local_delete_pieces(lp, l, first) ? per : 0u;  // (past the leaf, or no room in it)
          }
        }
      }
    }
    u32 idx = c.idx;
    if (ins) {
      u32 el = slen_i(w.cget_len(idx)), nxo, has;
      if (c.off < el) { nxo = w.cget_order(idx) + c.off; has = 1; }
      else has = next_item_after(idx, nxo);
      if (remote) {
        if (has) {
          if (nxo != orr) return 0;  // integrate would scan (doc.rs:183-221)
        }
      } else {
        orr = has ? nxo : ROOT_ORDER;  // doc.rs:453; integrate then stops at once
      }
      Span item{first, ol, orr, (i32)l};
      Span e = w.cget(idx);
#ifdef CRDT_PROF
      prof_cat = ((c.off == el) & can_append_u(e, item)) ? 0u : 3u;
#endif
      if (c.off == el) {
        if (can_append_u(e, item)) return fast_typing(b0, nv, remote, idx, orr, agent, o, first);
      }
      // a local insert at position 0 (offset 0 only there) may start a front run
      u32 front = remote ? 0u : (c.off == 0u ? 1u : 0u);
      // no room for the item (+ the entry's remainder): a leaf split, the general path's job
      if (g(C_N) + 1u + (c.off < el) > (u32)L) {
        // integrate stops at once here (checked above), so apply_txn would only insert_internal
        // the item, splitting the leaf (mutations.rs:17-179): do that here when a leaf is free
        if ((g(K_LEAF) - g(S_N_LEAVES) >= 2u) && (g(K_MAP) - first >= l)) {
#ifdef CRDT_PROF
          prof_cat = 1u;
#endif
          insert_items(item, Span{0, 0, 0, 0}, Span{0, 0, 0, 0}, 1u, c, INVALID);
          fast_txn_commit(first, l);
          // a prepend that split a full leaf at index 0 (insert_internal: split_at(0) moves every
          // entry to a new leaf linked right after it, the cursor does not follow, mutations.rs:
          // 96-121) is entry 0 of the emptied leaf: the front run it starts refills it
          if (front & cpt) {
            u32 kf = w.front_scan(b0, nv, agent, l);
            if (kf > 1u) return (1u + leaf_insert_front(first, l, kf - 1u)) * per;
          }
          return per;
        }
        p(F_PRE, 1u);
        p(PRE_ITEM, item.order); p(PRE_ITEM + 1, item.ol); p(PRE_ITEM + 2, item.orr); p(PRE_ITEM + 3, (u32)item.len);
        p(PRE_C, c.leaf); p(PRE_C + 1, c.idx); p(PRE_C + 2, c.off);
        return 0;
      }
      // the typing that follows the inserted item appends to it: one entry for the whole run
      u32 total;
      u32 nt = typing_run(b0, nv, remote, agent, (agent & 0xFFFFu) | (o.w1 & 0xFFFF0000u), o, total);
      item.len = (i32)total;
      u32 kf = (front & cpt) && nt == 1u ? w.front_scan(b0, nv, agent, l) : 1u;
      if (front) {  // (a front run commits itself; with kf > 1, nt == 1)
        u32 r = leaf_insert_front(item.orr, total, kf);
        return r ? (nt + r - 1u) * per : 0u;
      }
      if (!leaf_insert(idx, c.off, item)) return 0;
      fast_txn_commit(first, total);
      return nt * per;
    }
    i32 el = w.cget_len(idx);
    if (el <= 0) return 0;                // already deleted
    if (remote) {  // (a local delete that spans entries went to leaf_delete_span above)
      if (c.off + l > (u32)el) return 0;  // spans entries
    }
#ifdef CRDT_PROF
    prof_cat = 2u;
#endif
    if (gen) {  // a generated op starts no run (no window): one leaf_delete when the leaf has room
      u32 t1 = w.cget_order(idx) + c.off;
      if (g(K_MAP) - first >= l) {
        if (g(K_DEL) != g(S_N_DEL)) {
          if (leaf_delete(idx, c.off, l)) {
            append_delete(first, t1, l);  // doc.rs:414-426
            fast_txn_commit(first, l);
            return per;
          }
        }
      }
    }
    return fast_deletes(b0, nv, remote, agent, idx, c.off, l, first, o);
  }

  // PROBE record (config 1: check every position <-> CRDT location lookup as the replay goes): the
  // README's two queries on the live state.  pos -> (agent, seq): the item at visible position
  // q.w1 (root.rs:54-88 cursor_at_content_pos, cursor.rs:233-239 get_item, client_with_order.get);
  // (agent, seq) -> (position, deleted): Cursor::count_pos (cursor.rs:147-190) of the item's cursor
  // = visible items in the leaves before it (root level + directory block prefix) + in its leaf
  // before it; deleted items report the position of the next visible one.  Unknown answers are
  // (0xFFFF, 0xFFFFFFFF) and (0xFFFFFFFF, 2), as the published-index queries answer.
  CRDT_HD void probe(const Rec& q, u32 pos) {
    materialize_tails();  // (order_to_loc reads the client_with_order tail)
    u32 a = 0xFFFFu, s = INVALID, ps = INVALID, dl = 2u;
    Cursor c;
    u32 o;
    if (q.w1 < cur_len() && cursor_at_content_pos(q.w1, c) && get_item(c, o)) {
      u32 a2, s2;
      if (order_to_loc(o, a2, s2)) { a = a2; s = s2; }
    }
    if (q.w2 < g(S_N_AGENTS) && seq_to_order(q.w2, q.w3, o) && find_order(o, false, c)) {
      commit();  // the directory's counts include the cached leaf's edits
      u32 blk, i;
      slot_of(c.leaf, blk, i);
      u32 v = w.root_vis_before(w.root_find_blk(g(S_NG), blk)) + w.blk_vis_before(dvis(blk), i);
      i32 el;
      if (c.leaf == g(C_LEAF)) {
        v += w.cache_vis_before(c.idx);
        el = w.cget_len(c.idx);
      } else {
        v += w.peek_vis_before(leafp(c.leaf), c.idx, el);
      }
      ps = v + (el > 0 ? c.off : 0u);
      dl = el < 0 ? 1u : 0u;
    }
    uint4* out = ptr<uint4>(P_PROBE);
    if (out) w.st_probe(out + pos, a, s, ps, dl);
  }

  // Replay this document's record stream from its rec_pos.  A GEN record stays current until
  // all its ops are applied (progress in S_GEN_DONE, so a capacity stop resumes mid-record).
  // SH (crdt_types.h SHAPE_*): the record kinds the stream may hold, known to the host at staging.
  // A stream of remote records only (SHAPE_REMOTE: the remote-batch configs) or of GEN records
  // only (SHAPE_GEN: config 4) replays in an instance without the other kinds' loops and without
  // the other side of the general interpreter (apply_txn's `remote` is then a constant), so the
  // hot loop's registers are allocated around less code.  A record of a kind the shape excludes
  // stops the document (ST_BAD_INPUT; the host never launches such a stream in that instance).
  template <u32 SH = SHAPE_ALL>
  CRDT_HD void run() {
    constexpr bool any_remote = SH == SHAPE_ALL || SH == SHAPE_REMOTE;
    constexpr bool any_lc = SH == SHAPE_ALL || SH == SHAPE_LOCAL, any_gen = SH == SHAPE_ALL || SH == SHAPE_GEN;
    u32 pos = g(S_REC_POS);
    u32 rn = rec_n();
    while (pos < rn) {
      w.x_pin();
      Rec h = rec(pos);
      u32 kind = rec_kind(h);
      if constexpr (SH != SHAPE_ALL) {
        if (!((shape_kinds(SH) >> kind) & 1u)) { p(S_STATUS, (u32)ST_BAD_INPUT); pos += 1; break; }
      }
      u32 tried = 0;  // the fast path already declined this record
      if (any_remote && kind == REC_RC) {
        // the remote-batch hot loop: compact remote txns through one fast-path instance, in a loop
        // of their own (its registers do not meet the other record kinds' paths at every txn)
        u32 fast;
        while (true) {
#ifdef CRDT_PROF
          u64 t0 = w.clock();
          fast = fast_txn(pos, REC_RC, 0u, h, Rec{0, 0, 0, 0});
          u32 dt = prof_mode == 0u ? (u32)(w.clock() - t0) : prof_mode == 1u ? 1u : fast;
          if (prof_mode != 3u && fast) {
            if (prof_cat == 0u) inc(S_PROF0, dt);
            else if (prof_cat == 2u) inc(S_PROF2, dt);
            else inc(S_PROF3, dt);
          }
#else
          fast = fast_txn(pos, REC_RC, 0u, h, Rec{0, 0, 0, 0});
#endif
          if (!fast) break;
          pos += fast;
          if (pos >= rn) break;
          w.x_pin();
          h = rec(pos);
          kind = rec_kind(h);
          if (kind != REC_RC) break;
        }
        if (pos >= rn) break;
        tried = kind == REC_RC ? 1u : 0u;
      } else if (any_lc && kind == REC_LC) {
        // the same for compact local txns (local-trace corpora: configs 1 and 3)
        while (true) {
#ifdef CRDT_PROF
          u64 t0 = w.clock();
          prof_split = 0u;
          u32 fast = fast_txn(pos, REC_LC, 0u, h, Rec{0, 0, 0, 0});
          u64 t1 = w.clock();
          u32 dt = prof_mode == 0u ? (u32)(t1 - t0) : prof_mode == 1u ? 1u : fast;
          if (prof_mode != 3u && fast) {  // (1: an insert that splits the leaf)
            if (prof_cat == 0u) inc(S_PROF0, dt);
            else if (prof_cat == 1u) inc(S_PROF1, dt);
            else if (prof_cat == 2u) inc(S_PROF2, dt);
            else inc(S_PROF3, dt);
          }
          if (prof_mode == 3u && fast) {  // detail: split_at / the rest of a splitting insert / other fast txns / the loop
            if (prof_cat == 1u) { inc(S_PROF0, prof_split); inc(S_PROF1, (u32)(t1 - t0) - prof_split); }
            else inc(S_PROF2, (u32)(t1 - t0));
            prof_t2 = t1;
          }
#else
          u32 fast = fast_txn(pos, REC_LC, 0u, h, Rec{0, 0, 0, 0});
#endif
          if (!fast) break;
          pos += fast;
          if (pos >= rn) break;
          w.x_pin();
          h = rec(pos);
          kind = rec_kind(h);
#ifdef CRDT_PROF
          if (prof_mode == 3u) inc(S_PROF3, (u32)(w.clock() - prof_t2));
#endif
          if (kind != REC_LC) break;
        }
        if (pos >= rn) break;
        tried = kind == REC_LC ? 1u : 0u;
      } else if (any_gen && kind == REC_GEN) {
        // generated ops (config 4) in a loop of their own: gen_op and one fast-path instance per
        // op, no trip through the record window and the kind dispatch
        // The draws of 64 ops at a time are computed lane-parallel into the record window's
        // registers (the window is reloaded at the next record: T_RB_BASE invalid).
        u32 done = g(S_GEN_DONE), n_gen = h.w2;
        p(T_RB_BASE, 0x80000000u);
        u32 base = done;
        w.gen_draws(h.w3, base);
        // The general path goes first while there is no cached leaf yet, or while the fast-commit
        // conditions (fast_txn_ok) do not hold; once they do, every fast commit keeps them (the
        // author stays cached and its tails extend), so the generated ops skip the check
        if (g(C_LEAF) == INVALID || !fast_txn_ok(h.w1, g(T_AGL_KEY) + g(T_AGL_LEN), g(S_NEXT_ORDER), 1u)) n_gen = done;
        while (done < n_gen) {
          if (done - base >= 64u) {
            base = done;
            w.gen_draws(h.w3, base);
          }
#ifdef CRDT_PROF
          u64 pg0 = w.clock();
#endif
          Rec d = w.rec_get(done - base);
          Rec go = gen_op_of(d.w0, d.w1, d.w2, cur_len());
          Rec gh{(REC_LTXN << 28) | 1u, h.w1, go.w2, go.w2 + go.w3};
#ifdef CRDT_PROF
          u64 pg1 = w.clock();
          prof_gen = 1u; prof_cur = 0u; prof_sw = 0u;
          u32 okg = fast_txn(pos, REC_LTXN, 1u, gh, go);
          prof_gen = 0u;
          if (prof_mode == 3u && okg) {
            u32 ft = (u32)(w.clock() - pg1);
            inc(S_PROF0, (u32)(pg1 - pg0)); inc(S_PROF1, ft - prof_cur);
            inc(S_PROF2, prof_cur - prof_sw); inc(S_PROF3, prof_sw);
          } else if (okg) {  // modes 0-2: cycles / calls / txns of the fast path by kind (typing, delete, insert)
            u32 dt = prof_mode == 0u ? (u32)(w.clock() - pg1) : 1u;
            if (prof_cat == 0u) inc(S_PROF0, dt);
            else if (prof_cat == 2u) inc(S_PROF2, dt);
            else inc(S_PROF3, dt);
          }
          if (!okg) break;
#else
          if (!fast_txn(pos, REC_LTXN, 1u, gh, go)) break;
#endif
          // (the loop skips fast_txn_ok: every fast commit keeps it true and keeps a cached leaf)
          CRDT_EXPECT(g(F_FAST) == 1u && g(C_LEAF) != INVALID);
          done++;
        }
        p(S_GEN_DONE, done);
        tried = 1u;  // (the general path takes op `done`, or the record ends below)
      }
      u32 gen = any_gen ? opq(kind == REC_GEN ? 1u : 0u) : 0u;
      Rec gop{0, 0, 0, 0}, gpar{0, 0, 0, 0};
      u32 inl = 0;
      if (gen) {  // (F_GEN carries the flag past the txn: no register lives across the loop body)
        u32 done = g(S_GEN_DONE);
        if (done >= h.w2) { p(S_GEN_DONE, 0); p(F_GEN, 0); pos += 1; continue; }
        p(F_GEN, 1);
        gop = gen_op(h.w3, done, cur_len());
        h = Rec{(REC_LTXN << 28) | 1u, h.w1, gop.w2, gop.w2 + gop.w3};
        kind = REC_LTXN;
        inl = 1;
      }
      i32 st;
      u32 consumed;
      if (((1u << REC_LTXN | 1u << REC_RTXN | 1u << REC_RC | 1u << REC_LC) >> kind) & 1u) {
#ifdef CRDT_PROF
        u64 t0 = w.clock();
#endif
        // compact remote txns (the remote-batch hot path) get their own instance of the fast paths,
        // with record kind, format and stride known at compile time
        // (also the compact local form and generated ops: the other batch shapes)
        // (a general remote txn by another author than the cached one, or with several frontier
        // heads, fails fast_txn_ok at once: skip the attempt's record decoding)
        if (kind == REC_RTXN) tried |= (((h.w1 & 0xFFFFu) != g(T_AG_ID)) | (g(S_N_FR) != 1u)) ? 1u : 0u;
        if constexpr (SH == SHAPE_GEN) tried = 1u;  // (only synthesized generated ops get here: tried in the GEN loop)
        u32 fast = tried ? 0u : fast_txn(pos, kind, 0u, h, gop);  // (a GEN record was tried above)
#ifdef CRDT_PROF
        u64 t1 = w.clock();
        u32 dt = prof_mode == 0u ? (u32)(t1 - t0) : prof_mode == 1u ? 1u : (fast ? fast / per_txn(kind == REC_RTXN || kind == REC_RC) : 0u);
        if (prof_mode == 3u) {  // detail: apply_txn parts (below)
        } else if (!fast) inc(S_PROF1, prof_mode == 0u ? dt : 0u);
        else if (prof_cat == 0u) inc(S_PROF0, dt);
        else if (prof_cat == 2u) inc(S_PROF2, dt);
        else inc(S_PROF3, dt);
#endif
        if (fast) {
          if (g(F_GEN)) inc(S_GEN_DONE);
          else pos += fast;
          continue;
        }
        bool remote = SH == SHAPE_REMOTE ? true : (SH == SHAPE_GEN || SH == SHAPE_LOCAL) ? false
                                                : (((1u << REC_RTXN | 1u << REC_RC) >> kind) & 1u);
        if (any_remote && kind == REC_RC) { expand_rc(h, h, gop, gpar); inl = 1; }
        if (any_lc && kind == REC_LC) { expand_lc(h, h, gop); inl = 1; }
        u32 nops = remote ? (h.w0 & RTXN_NOPS_MASK) : (h.w0 & 0x0FFFFFFFu);
        consumed = inl ? 1u : 1 + nops + (remote ? (h.w1 >> 16) : 0u);
        st = (pos + consumed <= rn) ? apply_txn(h, pos, remote, inl, gop, gpar) : ST_BAD_INPUT;
        p(F_PRE, 0u);
#ifdef CRDT_PROF
        if (prof_mode != 3u) inc(S_PROF1, prof_mode == 0u ? (u32)(w.clock() - t1) : 1u);
#endif
      } else if (any_lc && kind == REC_PROBE) {
        probe(h, pos);
        st = ST_OK;
        consumed = 1;
      } else {
        st = ST_BAD_INPUT;
        consumed = 1;
      }
      if (st == ST_NEED_CAPACITY) { p(S_STATUS, (u32)st); break; }  // resumable at `pos` after growth
      if (st != ST_OK) { p(S_STATUS, (u32)st); pos += consumed; break; }
      if (g(F_GEN)) { inc(S_GEN_DONE); continue; }
      pos += consumed;
    }
    p(S_REC_POS, pos);
  }
};

}  // namespace crdt
