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
//     count) in HBM and a root level of up to 256 groups held in VGPRs (lane = group), so every
//     descent is two wave-wide scans and every leaf insertion one 64-lane shift;
//   * a write-back leaf cache in VGPRs (lane i = entry i) that also remembers its directory slot
//     and visible count, so runs of edits in one leaf touch neither HBM loads nor the directory;
//     lookups that only need a position in another leaf (integrate's origin compare, the item
//     after the end of a leaf) peek at that leaf without evicting the cached one;
//   * an order->leaf table (u32 per order) replacing the SplitList, written only when a run
//     changes leaf (the reference's notify() semantics);
//   * register-resident tails of every RLE table (client_with_order, the author's item_orders,
//     deletes, txns, frontier) and a 64-record prefetch of the op stream, so the common op issues
//     no dependent HBM load at all (stores are fire-and-forget).
//
// Code shape (what makes this fast on CDNA4): one op interpreter loop per document in which
// every heavy routine -- integrate's scan, mutate_entry, insert_internal, split_at -- has exactly
// ONE inlined instance, so the hot loop stays small in the instruction cache and short in
// register live ranges.  Control flow is wave-uniform; every lane-parallel step goes through the
// backend W:
//   W = WaveGPU (wave_gpu.h, the product) or WaveCPU (tests/emu, a test-only emulation used to
//   debug this file against the oracle without a GPU).
#pragma once
#include "crdt_types.h"

namespace crdt {

struct Cursor {
  u32 leaf, idx, off;
};

template <class W, int L>
struct Replayer {
  W w;  // owned by value: its lane registers must stay SSA values, never a scratch object
  // ---- this document's tables (Pools + DocSeg bases, resolved once)
  Span* lv;
  u32* dl;
  u32* dv;
  u32* sol;
  u32* lof;
  CwoRun* cwo;
  ARun* arun;
  DelRun* dels;
  DDRun* dd;
  TxnRec* txns;
  u32* par;
  u32* fr;
  AgentRec* agents;
  GroupRec* groups;
  const Rec* recs;
  DocState* stp;
  u32 cap_leaf, cap_map, cap_cwo, cap_txn, cap_del, cap_dd, cap_par, rec_n;
  DocState s;

  // ---- leaf cache bookkeeping (the entries themselves live in W)
  u32 c_leaf = INVALID;
  u32 c_n = 0;
  u32 c_vis = 0;      // visible count of c_leaf as recorded in the directory
  u32 c_now = 0;      // visible count of the cached entries right now
  u32 c_blk = 0, c_i = 0;  // directory slot of c_leaf
  u32 c_vstart = 0;   // visible items before c_leaf (valid if c_vs_ok)
  bool c_dirty = false;
  bool c_vs_ok = false;

  // ---- register-resident RLE tails (written through to HBM on every change)
  CwoRun cwo_last{0, 0, 0, 0};
  DelRun del_last{0, 0, 0};
  u32 tx_order = 0, tx_len = 0, tx_shadow = 0;  // last txns entry
  u32 fr0 = ROOT_ORDER;
  u32 ag_id = INVALID;  // agent cache (the txn author): its AgentRec and last item_orders run
  u32 ag_base = 0, ag_cnt = 0, ag_cap = 0;
  ARun ag_last{0, 0, 0, 0};

  // ---- record prefetch
  u32 rb_base = 0x80000000u;  // pos - rb_base >= 64 for every valid pos

  CRDT_HD Replayer(const Pools& P, u32 d, const W& w0 = W()) : w(w0) {
    DocSeg g = w.ld_seg(P.seg + d);
    lv = P.leaves + g.leaf_base * (u64)L;
    dl = P.dir_leaf + g.blk_base * (u64)GROUP;
    dv = P.dir_vis + g.blk_base * (u64)GROUP;
    sol = P.slot_of_leaf + g.leaf_base;
    lof = P.leaf_of + g.map_base;
    cwo = P.cwo + g.cwo_base;
    arun = P.arun + g.arun_base;
    dels = P.dels + g.del_base;
    dd = P.dd + g.dd_base;
    txns = P.txns + g.txn_base;
    par = P.parents + g.par_base;
    fr = P.frontier + g.fr_base;
    agents = P.agents + g.agent_base;
    groups = P.groups + g.grp_base;
    recs = P.recs + g.rec_base;
    stp = P.st + d;
    cap_leaf = g.leaf_cap;
    cap_map = g.map_cap;
    cap_cwo = g.cwo_cap;
    cap_txn = g.txn_cap;
    cap_del = g.del_cap;
    cap_dd = g.dd_cap;
    cap_par = g.par_cap;
    rec_n = g.rec_n;
    s = w.ld_state(stp);
  }

  CRDT_HD Span* leafp(u32 leaf) const { return lv + (u64)leaf * L; }
  CRDT_HD u32* dleaf(u32 blk) const { return dl + (u64)blk * GROUP; }
  CRDT_HD u32* dvis(u32 blk) const { return dv + (u64)blk * GROUP; }

  // ------------------------------------------------------------------ init / begin / finish
  // New empty document: ListCRDT::new (doc.rs:51-64): one empty root leaf, frontier [ROOT].
  CRDT_HD void init_empty() {
    s.status = ST_OK;
    s.rec_pos = 0;
    s.n_leaves = 1;
    s.n_blocks = 1;
    s.ng = 1;
    s.next_order = 0;
    s.len = 0;
    s.n_cwo = s.n_del = s.n_dd = s.n_txn = s.n_par = 0;
    s.n_fr = 1;
    s.n_items = 0;
    s.cap_need = 0;
    s.n_entries = 0;
    w.zero_leaf(leafp(0), L);
    w.st(dl, 0u);
    w.st(dv, 0u);
    w.st(sol, 0u);
    w.st(fr, ROOT_ORDER);
    w.root_init(0u, 1u, 0u);
  }
  CRDT_HD void begin() {
    w.root_load(groups, s.ng);
    if (s.n_cwo) cwo_last = w.ld_cwo(cwo + s.n_cwo - 1);
    if (s.n_del) del_last = w.ld_del(dels + s.n_del - 1);
    if (s.n_txn) {
      TxnRec t = w.ld_txn(txns + s.n_txn - 1);
      tx_order = t.order;
      tx_len = t.len;
      tx_shadow = t.shadow;
    }
    fr0 = w.ld(fr);
  }
  CRDT_HD void finish() {
    commit();
    w.root_store(groups, s.ng);
    w.st_state(stp, s);
  }

  // ------------------------------------------------------------------ records
  CRDT_HD Rec rec(u32 pos) {
    if (pos - rb_base >= 64u) {
      rb_base = pos;
      u32 n = rec_n - pos;
      w.rec_block_load(recs + pos, n < 64u ? n : 64u);
    }
    return w.rec_get(pos - rb_base);
  }

  // ------------------------------------------------------------------ directory
  CRDT_HD void slot_of(u32 leaf, u32& blk, u32& i) const {
    if (leaf == c_leaf) { blk = c_blk; i = c_i; return; }
    u32 v = w.ld(sol + leaf);
    blk = v >> 6;
    i = v & 63u;
  }
  CRDT_HD u32 pos_key(u32 leaf) const {  // total order of leaves in the document
    u32 blk, i;
    slot_of(leaf, blk, i);
    return (w.root_find_blk(s.ng, blk) << 6) | i;
  }
  CRDT_HD u32 leaf_at_start() const { return w.ld(dleaf(w.root_blk(0))); }
  CRDT_HD u32 leaf_at_end() const {
    u32 g = s.ng - 1;
    return w.ld(dleaf(w.root_blk(g)) + w.root_cnt(g) - 1);
  }
  CRDT_HD u32 next_leaf(u32 leaf) const {
    u32 blk, i;
    slot_of(leaf, blk, i);
    u32 g = w.root_find_blk(s.ng, blk);
    if (i + 1 < w.root_cnt(g)) return w.ld(dleaf(blk) + i + 1);
    if (g + 1 < s.ng) return w.ld(dleaf(w.root_blk(g + 1)));
    return INVALID;
  }
  // Record the cached leaf's new visible count in the directory.
  CRDT_HD void dir_set_cached_vis(u32 v) {
    if (v == c_vis) return;
    w.st(dvis(c_blk) + c_i, v);
    w.root_add_vis(w.root_find_blk(s.ng, c_blk), v - c_vis);
    s.len += v - c_vis;
    c_vis = v;
  }
  // First leaf whose visible range contains `pos` (root.rs:54-88 descent, ContentIndex).
  CRDT_HD bool find_by_pos(u32 pos, u32& leaf, u32& vstart, u32& blk, u32& i) const {
    u32 g, base;
    if (!w.root_find_pos(s.ng, pos, g, base)) return false;
    blk = w.root_blk(g);
    u32 before;
    if (!w.blk_find_pos(dvis(blk), dleaf(blk), w.root_cnt(g), pos - base, i, before, leaf)) return false;
    vstart = base + before;
    return true;
  }

  // ------------------------------------------------------------------ leaf cache
  CRDT_HD void commit() {
    if (c_leaf == INVALID || !c_dirty) return;
    w.cache_store(leafp(c_leaf));
    dir_set_cached_vis(c_now);
    c_dirty = false;
  }
  CRDT_HD void load_cache(u32 leaf, u32 blk, u32 i) {
    commit();
    c_n = w.cache_load(leafp(leaf));
    c_leaf = leaf;
    c_blk = blk;
    c_i = i;
    c_dirty = false;
    c_now = c_vis = w.cache_vis_from(0u);
    c_vs_ok = false;
  }
  CRDT_HD void ensure(u32 leaf) {
    if (leaf == c_leaf) return;
    u32 v = w.ld(sol + leaf);
    load_cache(leaf, v >> 6, v & 63u);
  }
  // set entry idx of the cached leaf (tracks the cached visible count exactly)
  CRDT_HD void set(u32 idx, const Span& e) {
    c_now = c_now - clen_i(w.cget_len(idx)) + clen(e);
    w.cset(idx, e);
    c_dirty = true;
  }
  CRDT_HD static u32 clen_i(i32 len) { return len > 0 ? (u32)len : 0u; }
  CRDT_HD static u32 slen_i(i32 len) { return (u32)(len < 0 ? -len : len); }
  CRDT_HD u32 cur_len() const { return s.len + c_now - c_vis; }

  // ------------------------------------------------------------------ order -> leaf map
  // ListCRDT::notify (doc.rs:143-153): all orders of `e` now live in `leaf`.  `home` is the
  // leaf the run already lives in (INVALID for freshly inserted orders): no write if unchanged.
  CRDT_HD void notify(const Span& e, u32 leaf, u32 home) {
    if (home == leaf) return;
    w.fill(lof + e.order, slen(e), leaf);
  }

  // ------------------------------------------------------------------ cursor ops
  // cursor.rs:127-145 (next_entry) / cursor.rs:26-103 (traverse).  Moves the cache along.
  CRDT_HD bool next_entry(Cursor& c) {
    ensure(c.leaf);
    if (c.idx + 1 < c_n) { c.idx++; c.off = 0; return true; }
    u32 nl = next_leaf(c.leaf);
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
      if (c.idx >= c_n) return next_entry(c);
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
      if (idx >= c_n) {
        u32 nl = next_leaf(c.leaf);
        if (nl == INVALID) return false;
        out = w.ld(&leafp(nl)->order);
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
  // root.rs:54-88 + 401-411, leaf.rs:61-84 (stick_end = false)
  CRDT_HD bool cursor_at_content_pos(u32 pos, Cursor& c) {
    if (!(c_leaf != INVALID && c_vs_ok && pos >= c_vstart && pos < c_vstart + c_now)) {
      commit();
      u32 lf, vs, blk, i;
      if (!find_by_pos(pos, lf, vs, blk, i)) return false;
      if (lf != c_leaf) load_cache(lf, blk, i);
      c_vstart = vs;
      c_vs_ok = true;
    }
    u32 idx, off;
    if (!w.cfind_content(c_n, pos - c_vstart, idx, off)) return false;
    c = Cursor{c_leaf, idx, off};
    return true;
  }
  // doc.rs:101-136 (marker_at + cursor_before_item, leaf.rs:41-57).  `load`: move the cache to
  // the item's leaf (the caller mutates there); otherwise only peek (the caller compares).
  CRDT_HD bool find_order(u32 order, bool load, Cursor& c) {
    if (order == ROOT_ORDER) {  // root.rs:90-123 cursor_at_end
      u32 lf = leaf_at_end();
      ensure(lf);
      if (c_n == 0) return false;
      c = Cursor{lf, c_n - 1, slen_i(w.cget_len(c_n - 1))};
      return true;
    }
    if (order >= s.next_order) return false;
    i32 idx = c_leaf != INVALID ? w.cfind_order(c_n, order) : -1;  // cached leaf first: no load
    if (idx >= 0) {
      c = Cursor{c_leaf, (u32)idx, order - w.cget_order((u32)idx)};
      return true;
    }
    u32 lf = w.ld(lof + order);
    if (lf == INVALID || lf == c_leaf) return false;
    if (load) {
      ensure(lf);
      idx = w.cfind_order(c_n, order);
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
  CRDT_HD u32 split_at(u32 idx, u32 padding) {
    u32 nl = s.n_leaves++;
    u32 stolen = w.cache_vis_from(idx);
    w.cache_write_moved(leafp(nl), idx, c_n, padding);
    for (u64 m = w.lanes_in(idx, c_n); m; m &= m - 1) {  // notify every moved entry
      Span e = w.cget(w.first_lane(m));
      w.fill(lof + e.order, slen(e), nl);
    }
    w.cache_clear(idx, c_n);
    c_now -= stolen;
    c_n = idx;
    c_dirty = true;
    // link nl right after the cached leaf (directory block insert; the block splits when full)
    u32 blk = c_blk, i = c_i;
    u32 g = w.root_find_blk(s.ng, blk);
    u32 cnt = w.root_cnt(g);
    if (cnt == GROUP) {  // split the block: [32, 64) -> new block in group g+1
      u32 nb = s.n_blocks++;
      u32 mv = w.blk_split(dleaf(blk), dvis(blk), dleaf(nb), dvis(nb), sol, nb);
      w.root_set(g, blk, 32u, w.root_vis(g) - mv);
      w.root_insert(s.ng, g + 1, nb, 32u, mv);
      s.ng++;
      if (i >= 32) { blk = nb; i -= 32; g = g + 1; c_blk = nb; c_i = i; }
      cnt = 32;
    }
    w.blk_insert(dleaf(blk), dvis(blk), cnt, i + 1, nl, stolen, sol, blk);
    // the cached leaf's directory count loses `stolen` (moved to nl); group total unchanged
    w.root_set(g, blk, cnt + 1, w.root_vis(g));
    w.st(dvis(c_blk) + c_i, c_vis - stolen);
    c_vis -= stolen;
    return nl;
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
      while (n > 0 && can_append(cur, a0)) {  // append to the entry at the cursor
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
      if (!has_rem && c.idx < c_n) {  // prepend the tail of the items onto the next entry
        Span nx = w.cget(c.idx);
        bool pre = false;
        while (true) {
          Span last = n == 1 ? a0 : (n == 2 ? a1 : a2);
          if (!can_append(last, nx)) break;
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
    s.n_entries += space;
    bool rem_moved = false;
    if (c_n + space > (u32)L) {
      bool follow = c.idx >= (u32)L / 2;
      u32 moved = c_n - c.idx;
      u32 nl = split_at(c.idx, follow ? space : 0u);
      if (follow) {  // the cursor follows the new leaf; its first `space` slots are padding
        commit();
        ensure(nl);
        c_n = space + moved;
        c.leaf = nl;
        c.idx = 0;
        rem_moved = true;
      } else {
        c_n += space;
      }
    } else {
      w.cache_shift_right(c.idx, c_n, space);
      c_n += space;
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
    if (a == ag_id) return;
    ag_id = a;
    AgentRec r = w.ld_agent(agents + a);
    ag_base = r.run_base;
    ag_cnt = r.run_cnt;
    ag_cap = r.run_cap;
    if (ag_cnt) ag_last = w.ld_arun(arun + ag_base + ag_cnt - 1);
  }
  CRDT_HD u32 agent_next_seq(u32 agent) {  // doc.rs:20-24
    use_agent(agent);
    return ag_cnt ? ag_last.key + ag_last.len : 0u;
  }
  CRDT_HD bool seq_to_order(u32 agent, u32 seq, u32& order) const {  // doc.rs:26-29
    u32 base, cnt;
    if (agent == ag_id) {
      if (ag_cnt && seq >= ag_last.key && seq - ag_last.key < ag_last.len) {
        order = ag_last.order + (seq - ag_last.key);
        return true;
      }
      base = ag_base;
      cnt = ag_cnt;
    } else {
      AgentRec A = w.ld_agent(agents + agent);
      base = A.run_base;
      cnt = A.run_cnt;
    }
    i32 k = w.search_arun(arun + base, cnt, seq);
    if (k < 0) return false;
    ARun r = w.ld_arun(arun + base + k);
    order = r.order + (seq - r.key);
    return true;
  }
  CRDT_HD bool order_to_agent(u32 order, u32& agent) const {  // client_with_order.get()
    if (s.n_cwo && order >= cwo_last.key && order - cwo_last.key < cwo_last.len) { agent = cwo_last.agent; return true; }
    i32 k = w.search_cwo(cwo, s.n_cwo, order);
    if (k < 0) return false;
    agent = w.ld_cwo(cwo + k).agent;
    return true;
  }
  // doc.rs:155-165 assign_order_to_client
  CRDT_HD void assign_order_to_client(u32 agent, u32 seq, u32 order, u32 len) {
    if (s.n_cwo > 0 && order == cwo_last.key + cwo_last.len && agent == cwo_last.agent && seq == cwo_last.seq + cwo_last.len) {
      cwo_last.len += len;
      w.st(&cwo[s.n_cwo - 1].len, cwo_last.len);
    } else {
      cwo_last = CwoRun{order, agent, seq, len};
      w.st_cwo(cwo + s.n_cwo, cwo_last);
      s.n_cwo++;
    }
    use_agent(agent);
    if (ag_cnt > 0 && seq == ag_last.key + ag_last.len && order == ag_last.order + ag_last.len) {
      ag_last.len += len;
      w.st(&arun[ag_base + ag_cnt - 1].len, ag_last.len);
    } else {
      ag_last = ARun{seq, order, len, 0};
      w.st_arun(arun + ag_base + ag_cnt, ag_last);
      ag_cnt++;
      w.st(&agents[agent].run_cnt, ag_cnt);
    }
  }
  CRDT_HD void append_delete(u32 key, u32 target, u32 len) {  // Rle<KVPair<DeleteEntry>>::append
    if (s.n_del > 0 && key == del_last.key + del_last.len && del_last.order + del_last.len == target) {
      del_last.len += len;
      w.st(&dels[s.n_del - 1].len, del_last.len);
      return;
    }
    del_last = DelRun{key, target, len};
    w.st_del(dels + s.n_del, del_last);
    s.n_del++;
  }
  // double_delete.rs:41-107 increment_delete_range (rare path; scalar)
  CRDT_HD bool dd_insert_at(u32 idx, DDRun r) {
    if (s.n_dd + 1 > cap_dd) return false;
    for (u32 k = s.n_dd; k > idx; k--) w.st_dd(dd + k, w.ld_dd(dd + k - 1));
    w.st_dd(dd + idx, r);
    s.n_dd++;
    return true;
  }
  CRDT_HD bool increment_delete_range(u32 base, u32 len) {
    DDRun* b = dd;
    DDRun next{base, len, 1};
    i32 k = w.search_dd(b, s.n_dd, base);
    u32 idx;
    if (k >= 0) idx = (u32)k;
    else {  // insertion point: first entry with key > base
      idx = 0;
      while (idx < s.n_dd && w.ld_dd(b + idx).key <= base) idx++;
    }
    while (true) {
      if (idx == s.n_dd || w.ld_dd(b + idx).key > next.key) {
        DDRun here = next;
        bool done_here;
        if (idx < s.n_dd && next.key + next.len > w.ld_dd(b + idx).key) {
          u32 at = w.ld_dd(b + idx).key - here.key;
          next = DDRun{here.key + at, here.len - at, here.excess};
          here.len = at;
          done_here = false;
        } else done_here = true;
        bool app = false;
        if (idx >= 1) {
          DDRun p = w.ld_dd(b + idx - 1);
          if (here.key == p.key + p.len && here.excess == p.excess) { w.st(&b[idx - 1].len, p.len + here.len); app = true; }
        }
        if (!app) { if (!dd_insert_at(idx, here)) return false; idx++; }
        if (done_here) break;
      }
      DDRun e = w.ld_dd(b + idx);
      if (e.key < next.key) {
        u32 at = next.key - e.key;
        DDRun rm{e.key + at, e.len - at, e.excess};
        w.st(&b[idx].len, at);
        idx++;
        if (!dd_insert_at(idx, rm)) return false;
      }
      DDRun e2 = w.ld_dd(b + idx);
      if (e2.len <= next.len) {
        w.st(&b[idx].excess, e2.excess + 1);
        next.key += e2.len;
        next.len -= e2.len;
        if (next.len == 0) break;
        idx++;
      } else {
        DDRun rm{e2.key + next.len, e2.len - next.len, e2.excess};
        w.st_dd(b + idx, DDRun{e2.key, next.len, e2.excess + 1});
        if (!dd_insert_at(idx + 1, rm)) return false;
        break;
      }
    }
    return true;
  }
  CRDT_HD bool par_contains(const u32* p, u32 np, u32 p0, u32 x) const {
    if (np == 0) return false;
    if (p0 == x) return true;
    for (u32 j = 1; j < np; j++) if (w.ld(p + j) == x) return true;
    return false;
  }
  // doc.rs:350-374 insert_txn (+ advance_branch_by :34-48).  Remote parents are already in the
  // pool at [n_par, n_par + np), the first one also in p0.
  CRDT_HD i32 insert_txn(bool remote, u32 first, u32 len, u32 np, u32 p0) {
    u32* pp = par + s.n_par;
    u32 last = first + len - 1;
    if (remote) {
      if (s.n_fr == 1) {
        if (fr0 == first) return ST_FRONTIER;
        if (par_contains(pp, np, p0, fr0)) { fr0 = last; w.st(fr, last); }
        else { w.st(fr + 1, last); s.n_fr = 2; }
      } else {
        for (u32 k = 0; k < s.n_fr; k++) if (w.ld(fr + k) == first) return ST_FRONTIER;
        u32 m = 0;
        for (u32 k = 0; k < s.n_fr; k++) {
          u32 o = w.ld(fr + k);
          if (!par_contains(pp, np, p0, o)) { w.st(fr + m, o); m++; }
        }
        if (m + 1 > FRONTIER_CAP) return ST_CAPACITY;
        w.st(fr + m, last);
        s.n_fr = m + 1;
        fr0 = w.ld(fr);
      }
    } else {
      np = s.n_fr;
      p0 = fr0;
      w.st(pp, fr0);
      for (u32 k = 1; k < np; k++) w.st(pp + k, w.ld(fr + k));
      w.st(fr, last);
      fr0 = last;
      s.n_fr = 1;
    }
    u32 shadow = first;
    while (shadow >= 1 && par_contains(pp, np, p0, shadow - 1)) {
      u32 x = shadow - 1;
      if (s.n_txn && x >= tx_order && x - tx_order < tx_len) { shadow = tx_shadow; continue; }
      i32 k = w.search_txn(txns, s.n_txn, x);
      if (k < 0) return ST_UNKNOWN_ID;
      shadow = w.ld(&txns[k].shadow);
    }
    if (s.n_txn > 0 && np == 1 && p0 == tx_order + tx_len - 1 && shadow == tx_shadow) {
      tx_len += len;
      w.st(&txns[s.n_txn - 1].len, tx_len);
      return ST_OK;  // parents of a merged txn are not kept
    }
    tx_order = first;
    tx_len = len;
    tx_shadow = shadow;
    w.st_txn(txns + s.n_txn, TxnRec{first, len, shadow, s.n_par, np, {0, 0, 0}});
    s.n_txn++;
    s.n_par += np;
    return ST_OK;
  }

  CRDT_HD i32 id_to_order(u32 agent, u32 seq, u32& order) const {  // doc.rs:236-240
    if (agent == ROOT_AGENT) { order = ROOT_ORDER; return ST_OK; }
    if (agent >= s.n_agents) return ST_UNKNOWN_AGENT;
    if (!seq_to_order(agent, seq, order)) return ST_UNKNOWN_ID;
    return ST_OK;
  }

  // ------------------------------------------------------------------ txn application
  // Capacity needed by a txn (checked before any mutation, so a capacity stop is resumable at
  // this txn).  Every block but the first holds >= 32 slots, so blk_cap = leaf_cap/32 + 2 and
  // leaf_cap <= 32*(MAX_GROUPS-1) (host-enforced) bound blocks and root groups as well.
  // On failure s.cap_need records which table (bit) must grow.
  CRDT_HD bool fits(bool remote, u32 agent, u32 n_ops, u32 n_dels, u32 txn_len, u32 n_parents) {
    u32 need = 0;
    if ((u64)s.n_leaves + 2ull * n_ops > cap_leaf) need |= 1u;
    if (s.n_cwo + 1 > cap_cwo || s.n_txn + 1 > cap_txn) need |= 2u;
    if ((u64)s.n_del + n_dels > cap_del) need |= 4u;
    if ((u64)s.n_par + (remote ? n_parents : s.n_fr) > cap_par) need |= 8u;
    if ((u64)s.next_order + txn_len > cap_map) need |= 16u;
    use_agent(agent);
    if (ag_cnt + 1 > ag_cap) need |= 32u;
    s.cap_need = need;
    return need == 0;
  }

  // Op interpreter modes
  enum : u32 { M_FETCH = 0, M_LDEL = 1, M_RDEL = 2, M_LINS = 3, M_INS = 4 };

  // One txn: doc.rs:376-469 apply_local_txn (remote = false) or doc.rs:242-348
  // apply_remote_txn (remote = true).  Header at record `pos`; ops (then parents) follow.
  CRDT_HD i32 apply_txn(const Rec& h, u32 pos, bool remote) {
    u32 nops, agent, np = 0, seq, txn_len;
    if (!remote) {
      nops = h.w0 & 0x0FFFFFFFu;
      agent = h.w1;
      txn_len = h.w3;
      if (agent >= s.n_agents) return ST_UNKNOWN_AGENT;
      if (txn_len == 0) return ST_EMPTY_TXN;
      if (!fits(false, agent, nops, h.w2, txn_len, 0)) return ST_NEED_CAPACITY;
      seq = agent_next_seq(agent);
    } else {
      nops = h.w0 & 0x07FFFFFFu;
      agent = h.w1 & 0xFFFFu;
      np = h.w1 >> 16;
      seq = h.w2;
      txn_len = h.w3;
      if (agent >= s.n_agents) return ST_UNKNOWN_AGENT;
      if (agent_next_seq(agent) != seq) return ST_SEQ;
      if ((h.w0 >> 27) & 1u) return ST_BAD_INPUT;
      if (txn_len == 0) return ST_EMPTY_TXN;
      if (!fits(true, agent, nops, nops, txn_len, np)) return ST_NEED_CAPACITY;
    }
    u32 first = s.next_order;
    u32 next = first;
    assign_order_to_client(agent, seq, first, txn_len);
    s.next_order = first + txn_len;

    u32 k = 0;
    u32 mode = M_FETCH;
    u32 remaining = 0, target = 0, lpos = 0, lins = 0;
    Span item{0, 0, 0, 0};
    Cursor c{0, 0, 0};
    while (true) {
      // ---------------------------------------------------------------- next op
      if (mode == M_FETCH) {
        if (k == nops) break;
        Rec op = rec(pos + 1 + k);
        k++;
        if (!remote) {  // LocalOp: delete (visible range) first, then insert (doc.rs:386-465)
          lpos = op.w1;
          u32 del = op.w2;
          lins = op.w3;
          if (del > 0) {
            if ((u64)lpos + del > cur_len()) return ST_POS_OOB;
            if (!cursor_at_content_pos(lpos, c)) return ST_POS_OOB;
            w.fill(lof + next, del, INVALID);  // delete orders name no item
            roll(c);                           // mutations.rs:539
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
            w.fill(lof + next, len, INVALID);
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
      if (mode == M_INS) {
        // integrate (doc.rs:167-234): scan entries from the insertion point
        Cursor left = c, scan_start = c;
        bool scanning = false;
        while (true) {
          u32 other_order;
          if (!get_item(c, other_order)) break;
          if (other_order == item.orr) break;
          Span oe = w.cget(c.idx);  // get_item ensured c.leaf
          Cursor olc;
          if (!cursor_after(origin_left_at_offset(oe, c.off), false, olc)) return ST_UNKNOWN_ID;
          int r = cmp(olc, left);
          if (r < 0) break;
          if (r == 0) {
            u32 oa;
            if (!order_to_agent(oe.order, oa)) return ST_UNKNOWN_ID;
            u32 my_rank = w.ld(&agents[agent].rank);
            u32 other_rank = w.ld(&agents[oa].rank);
            if (my_rank > other_rank) scanning = false;
            else if (item.orr == oe.orr) break;
            else { scanning = true; scan_start = c; }
          }
          if (!next_entry(c)) return ST_NONTERMINATING;  // cursor unchanged -> loops forever
        }
        if (scanning) c = scan_start;
        a0 = item;
        n = 1;
        s.n_items += (u32)item.len;
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
      if (!insert_items(a0, a1, a2, n, c, home)) return ST_INTERNAL;
    }
    if (!remote && next != first + txn_len) return ST_BAD_INPUT;
    u32 p0 = 0;
    if (remote) {
      u32* pp = par + s.n_par;
      for (u32 j = 0; j < np; j++) {
        Rec pr = rec(pos + 1 + nops + j);
        if (rec_kind(pr) != REC_RPARENT) return ST_BAD_INPUT;
        u32 o;
        i32 st = id_to_order(pr.w1 & 0xFFFFu, pr.w2, o);
        if (st != ST_OK) return st;
        w.st(pp + j, o);
        if (j == 0) p0 = o;
      }
    }
    return insert_txn(remote, first, txn_len, np, p0);
  }

  // Replay this document's record stream from s.rec_pos.
  CRDT_HD void run() {
    u32 pos = s.rec_pos;
    while (s.status == ST_OK && pos < rec_n) {
      Rec h = rec(pos);
      u32 kind = rec_kind(h);
      i32 st;
      u32 consumed;
      if (kind == REC_LTXN || kind == REC_RTXN) {
        bool remote = kind == REC_RTXN;
        u32 nops = remote ? (h.w0 & 0x07FFFFFFu) : (h.w0 & 0x0FFFFFFFu);
        consumed = 1 + nops + (remote ? (h.w1 >> 16) : 0u);
        st = (pos + consumed <= rec_n) ? apply_txn(h, pos, remote) : ST_BAD_INPUT;
      } else {
        st = ST_BAD_INPUT;
        consumed = 1;
      }
      if (st == ST_NEED_CAPACITY) { s.status = st; break; }  // resumable at `pos` after growth
      if (st != ST_OK) { s.status = st; pos += consumed; break; }
      pos += consumed;
    }
    s.rec_pos = pos;
  }
};

}  // namespace crdt
