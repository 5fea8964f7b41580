// Wave-per-document replay of list-CRDT transactions (local + remote) on the MI355X.
//
// This is the B-tree replacement.  The reference keeps a 16-ary B-tree of YjsSpan runs with
// 32-entry leaves (src/range_tree/*) plus an order->leaf SplitList (src/split_list).  Here a
// document is:
//   * leaves of L entries (L = 32 release / 4 debug) in HBM, with *exactly* the reference's
//     leaf-level mutation rules (insert_internal / split_at / mutate_entry), so the entry layout
//     -- which leaks into results through YjsSpan::prepend and the integrate tie-break -- is
//     bit-identical to the reference's;
//   * a two-level wave directory instead of internal nodes: 64-slot blocks (leaf id + visible
//     count) in HBM and a root level of up to 256 groups held in VGPRs (lane = group), so every
//     descent is two wave-wide scans and every leaf insertion one 64-lane shift;
//   * a write-back leaf cache in VGPRs (lane i = entry i) that also remembers its directory slot
//     and visible count, so runs of edits in one leaf touch neither HBM loads nor the directory;
//   * an order->leaf table (u32 per order) replacing the SplitList, written only when a run
//     changes leaf (the reference's notify() semantics) and never read when the target item is
//     in the cached leaf;
//   * register-resident tails of every RLE table (client_with_order, the author's item_orders,
//     deletes, txns, frontier) and a 64-record prefetch of the op stream, so the common op issues
//     no dependent HBM load at all (stores are fire-and-forget).
//
// Control flow is wave-uniform; every lane-parallel step goes through the backend W:
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
  W& w;
  const Pools& P;
  u32 d;
  DocSeg seg;
  DocState s;
  bool track;

  // ---- leaf cache bookkeeping (the entries themselves live in W)
  u32 c_leaf = INVALID;
  u32 c_n = 0;
  bool c_dirty = false;
  u32 c_vis = 0;      // visible count of c_leaf as recorded in the directory
  u32 c_now = 0;      // visible count of the cached entries right now
  u32 c_blk = 0, c_i = 0;  // directory slot of c_leaf
  bool c_vs_ok = false;
  u32 c_vstart = 0;   // visible items before c_leaf (valid if c_vs_ok)

  // ---- register-resident RLE tails (written through to HBM on every change)
  CwoRun cwo_last{0, 0, 0, 0};
  DelRun del_last{0, 0, 0};
  TxnRec txn_last{0, 0, 0, 0, 0, {0, 0, 0}};
  u32 txn_last_p0 = 0;
  u32 fr0 = ROOT_ORDER;
  u32 ag_id = INVALID;  // agent cache (the txn author)
  AgentRec ag{0, 0, 0, 0};
  ARun ag_last{0, 0, 0, 0};

  // ---- record prefetch
  u32 rb_base = 0x80000000u;  // pos - rb_base >= 64 for every valid pos

  CRDT_HD Replayer(W& w_, const Pools& p, u32 doc) : w(w_), P(p), d(doc) {
    seg = w.ld_seg(P.seg + d);
    s = w.ld_state(P.st + d);
    track = (seg.flags & DOC_TRACK_MAP) != 0;
  }

  // ------------------------------------------------------------------ memory helpers
  CRDT_HD Span* leafptr(u32 leaf) const { return P.leaves + (seg.leaf_base + leaf) * (u64)L; }
  CRDT_HD u32* dleaf(u32 blk) const { return P.dir_leaf + (seg.blk_base + blk) * (u64)GROUP; }
  CRDT_HD u32* dvis(u32 blk) const { return P.dir_vis + (seg.blk_base + blk) * (u64)GROUP; }
  CRDT_HD u32* sol() const { return P.slot_of_leaf + seg.leaf_base; }
  CRDT_HD AgentRec* agp(u32 a) const { return P.agents + seg.agent_base + a; }
  CRDT_HD ARun* arunp(const AgentRec& A) const { return P.arun + seg.arun_base + A.run_base; }

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
    w.zero_leaf(leafptr(0), L);
    w.st(dleaf(0), 0u);
    w.st(dvis(0), 0u);
    w.st(sol(), 0u);
    w.st(P.frontier + seg.fr_base, ROOT_ORDER);
    w.root_init(0u, 1u, 0u);
  }
  CRDT_HD void begin() {
    w.root_load(P.groups + seg.grp_base, s.ng);
    if (s.n_cwo) cwo_last = w.ld_cwo(P.cwo + seg.cwo_base + s.n_cwo - 1);
    if (s.n_del) del_last = w.ld_del(P.dels + seg.del_base + s.n_del - 1);
    if (s.n_txn) {
      txn_last = w.ld_txn(P.txns + seg.txn_base + s.n_txn - 1);
      if (txn_last.pn) txn_last_p0 = w.ld(P.parents + seg.par_base + txn_last.poff);
    }
    fr0 = w.ld(P.frontier + seg.fr_base);
  }
  CRDT_HD void finish() {
    commit();
    w.root_store(P.groups + seg.grp_base, s.ng);
    w.st_state(P.st + d, s);
  }

  // ------------------------------------------------------------------ records
  CRDT_HD Rec rec(u32 pos) {
    if (pos - rb_base >= 64u) {
      rb_base = pos;
      u32 n = seg.rec_n - pos;
      w.rec_block_load(P.recs + seg.rec_base + pos, n < 64u ? n : 64u);
    }
    return w.rec_get(pos - rb_base);
  }

  // ------------------------------------------------------------------ directory
  CRDT_HD void slot_of(u32 leaf, u32& blk, u32& i) const {
    if (leaf == c_leaf) { blk = c_blk; i = c_i; return; }
    u32 v = w.ld(sol() + leaf);
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
  // Insert leaf `nl` (visible count v) right after the cached leaf in document order.
  CRDT_HD void dir_insert_after_cached(u32 nl, u32 v) {
    u32 blk = c_blk, i = c_i;
    u32 g = w.root_find_blk(s.ng, blk);
    u32 cnt = w.root_cnt(g);
    if (cnt == GROUP) {  // split the block: [32, 64) -> new block in group g+1
      u32 nb = s.n_blocks++;
      u32 mv = w.blk_split(dleaf(blk), dvis(blk), dleaf(nb), dvis(nb), sol(), nb);
      w.root_set(g, blk, 32u, w.root_vis(g) - mv);
      w.root_insert(s.ng, g + 1, nb, 32u, mv);
      s.ng++;
      if (i >= 32) { blk = nb; i -= 32; g = g + 1; c_blk = nb; c_i = i; }
      cnt = 32;
    }
    w.blk_insert(dleaf(blk), dvis(blk), cnt, i + 1, nl, v, sol(), blk);
    w.root_set(g, blk, cnt + 1, w.root_vis(g) + v);
    s.len += v;
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
    w.cache_store(leafptr(c_leaf), c_n);
    dir_set_cached_vis(c_now);
    c_dirty = false;
  }
  CRDT_HD void load_cache(u32 leaf, u32 blk, u32 i) {
    commit();
    c_n = w.cache_load(leafptr(leaf));
    c_leaf = leaf;
    c_blk = blk;
    c_i = i;
    c_dirty = false;
    c_now = c_vis = w.cache_vis(0, (u32)L);
    c_vs_ok = false;
  }
  CRDT_HD void ensure(u32 leaf) {
    if (leaf == c_leaf) return;
    u32 v = w.ld(sol() + leaf);
    load_cache(leaf, v >> 6, v & 63u);
  }
  CRDT_HD Span get(u32 leaf, u32 idx) {
    ensure(leaf);
    return w.cget(idx);
  }
  // set entry idx of the cached leaf (tracks the cached visible count exactly)
  CRDT_HD void set(u32 idx, const Span& e) {
    c_now = c_now - clen(w.cget(idx)) + clen(e);
    w.cset(idx, e);
    c_dirty = true;
  }
  CRDT_HD u32 cur_len() const { return s.len + c_now - c_vis; }

  // ------------------------------------------------------------------ order -> leaf map
  // ListCRDT::notify (doc.rs:143-153): all orders of `e` now live in `leaf`.  `home` is the
  // leaf the run already lives in (INVALID for freshly inserted orders): no write if unchanged.
  CRDT_HD void notify(const Span& e, u32 leaf, u32 home) {
    if (!track || home == leaf) return;
    w.fill(P.leaf_of + seg.map_base + e.order, slen(e), leaf);
  }

  // ------------------------------------------------------------------ cursor ops
  // cursor.rs:127-145 (next_entry) / cursor.rs:26-103 (traverse)
  CRDT_HD bool next_entry(Cursor& c) {
    ensure(c.leaf);
    if (c.idx + 1 < c_n) { c.idx++; c.off = 0; return true; }
    u32 nl = next_leaf(c.leaf);
    if (nl == INVALID) return false;
    c.leaf = nl;
    c.idx = 0;
    c.off = 0;
    return true;
  }
  // cursor.rs:210-231
  CRDT_HD bool roll(Cursor& c) {
    ensure(c.leaf);
    u32 seq_len = slen(w.cget(c.idx));
    if (c.off == seq_len) {
      c.off = 0;
      c.idx++;
      if (c.idx >= c_n) return next_entry(c);
    }
    return true;
  }
  // cursor.rs:233-239
  CRDT_HD bool get_item(const Cursor& c0, u32& out) {
    Cursor c = c0;
    if (!roll(c)) return false;
    out = get(c.leaf, c.idx).order + c.off;
    return true;
  }
  // cursor.rs:242-248
  CRDT_HD bool next_item(Cursor& c) {
    if (!roll(c)) return false;
    c.off++;
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
  CRDT_HD bool cursor_at_end(Cursor& c) {                                           // root.rs:90-123
    u32 lf = leaf_at_end();
    ensure(lf);
    if (c_n == 0) return false;
    c = Cursor{lf, c_n - 1, slen(w.cget(c_n - 1))};
    return true;
  }
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
  // doc.rs:101-136 (marker_at + cursor_before_item, leaf.rs:41-57)
  CRDT_HD bool get_cursor_before(u32 order, Cursor& c) {
    if (order == ROOT_ORDER) return cursor_at_end(c);
    if (!track || order >= s.next_order) return false;
    i32 idx = c_leaf != INVALID ? w.cfind_order(c_n, order) : -1;  // cached leaf first: no load
    if (idx < 0) {
      u32 lf = w.ld(P.leaf_of + seg.map_base + order);
      if (lf == INVALID || lf == c_leaf) return false;
      ensure(lf);
      idx = w.cfind_order(c_n, order);
      if (idx < 0) return false;
    }
    c = Cursor{c_leaf, (u32)idx, order - w.cget((u32)idx).order};
    return true;
  }
  CRDT_HD bool get_cursor_after(u32 order, Cursor& c) {
    if (order == ROOT_ORDER) { c = cursor_at_start(); return true; }
    if (!get_cursor_before(order, c)) return false;
    c.off += 1;
    return true;
  }

  // ------------------------------------------------------------------ leaf mutation
  // mutations.rs:623-669 split_at: [idx, n) of the cached leaf moves to a new leaf (after
  // `padding` empty slots), which is linked right after the cached leaf.  Returns its id.
  CRDT_HD u32 split_at(u32 idx, u32 padding) {
    u32 nl = s.n_leaves++;
    u32 stolen = w.cache_vis(idx, c_n);
    w.cache_write_moved(leafptr(nl), idx, c_n, padding);
    if (track)
      for (u32 j = idx; j < c_n; j++) notify(w.cget(j), nl, INVALID);
    w.cache_clear(idx, c_n);
    c_now -= stolen;
    c_n = idx;
    c_dirty = true;
    dir_insert_after_cached(nl, stolen);
    // the cached leaf's directory count loses `stolen` (dir_insert_after added it for nl)
    w.st(dvis(c_blk) + c_i, c_vis - stolen);
    w.root_add_vis(w.root_find_blk(s.ng, c_blk), 0u - stolen);
    s.len -= stolen;
    c_vis -= stolen;
    return nl;
  }
  // mutations.rs:17-179 insert_internal.  items: up to three named values (stay in registers);
  // home: leaf the items already live in (INVALID for fresh orders), for notify().
  CRDT_HD static Span pick(const Span& a, const Span& b, const Span& c, u32 k) { return k == 0 ? a : (k == 1 ? b : c); }
  CRDT_HD bool insert_internal(Span i0, Span i1, Span i2, u32 nitems, Cursor& c, u32 home) {
    if (nitems == 0) return true;
    u32 ib = 0;  // items[ib .. ib+nitems)
    ensure(c.leaf);
    if (c.off == 0 && c.idx > 0) {
      c.idx -= 1;
      c.off = slen(w.cget(c.idx));
    }
    u32 seq_len = slen(w.cget(c.idx));
    bool has_rem = false;
    Span rem{0, 0, 0, 0};
    if (!(c.off == seq_len || c.off == 0)) {
      Span cur = w.cget(c.idx);
      rem = truncate(cur, c.off);
      set(c.idx, cur);
      has_rem = true;
    }
    if (c.off != 0) {
      Span cur = w.cget(c.idx);
      u32 it = 0;
      while (it < nitems) {
        Span nx = pick(i0, i1, i2, ib + it);
        if (!can_append(cur, nx)) break;
        notify(nx, c.leaf, home);
        cur.len += nx.len;
        c.off = slen(cur);
        it++;
      }
      if (it > 0) set(c.idx, cur);
      if (it == nitems && !has_rem) return true;
      ib += it;
      nitems -= it;
      c.off = 0;
      c.idx += 1;
      if (!has_rem && c.idx < c_n) {
        u32 end = nitems - 1;
        Span nx2 = w.cget(c.idx);
        bool any = false;
        while (true) {
          Span it2 = pick(i0, i1, i2, ib + end);
          if (!can_append(it2, nx2)) break;
          notify(it2, c.leaf, home);
          nx2.order = it2.order;  // prepend (span.rs:61-64): origin_left is NOT updated
          nx2.len += it2.len;
          any = true;
          if (end == 0) { set(c.idx, nx2); return true; }
          end--;
        }
        if (any) set(c.idx, nx2);
        nitems = end + 1;
      }
    }
    u32 space = nitems + (has_rem ? 1u : 0u);
    if (space > (u32)L / 2) return false;  // mutations.rs:121 assert
    s.n_entries += space;
    bool rem_moved = false;
    if (c_n + space > (u32)L) {
      if (c.idx < (u32)L / 2) {
        split_at(c.idx, 0);
        c_n += space;
      } else {
        u32 moved = c_n - c.idx;
        u32 nl = split_at(c.idx, space);
        commit();
        ensure(nl);  // cursor follows the new leaf; its first `space` slots are padding
        c_n = space + moved;
        c.leaf = nl;
        c.idx = 0;
        rem_moved = true;
      }
    } else {
      w.cache_shift_right(c.idx, c_n, space);
      c_n += space;
    }
    for (u32 k = 0; k < nitems; k++) {
      Span x = pick(i0, i1, i2, ib + k);
      notify(x, c.leaf, home);
      set(c.idx + k, x);
    }
    Span last = pick(i0, i1, i2, ib + nitems - 1);
    c.idx += nitems - 1;
    c.off = slen(last);
    if (has_rem) {
      if (rem_moved) notify(rem, c.leaf, INVALID);
      set(c.idx + 1, rem);
    }
    return true;
  }
  // mutations.rs:185-200 (items = i0 then up to two more)
  CRDT_HD bool replace_entry(Cursor& c, Span i0, Span i1, Span i2, u32 n) {
    u32 home = c.leaf;
    set(c.idx, i0);
    c.off = slen(i0);
    return insert_internal(i1, i2, i2, n - 1, c, home);
  }
  // mutations.rs:227-277.  del_next != nullptr: local delete, stream the deactivated run into
  // the delete log (extend_delete + Rle::append compose to the same list).
  CRDT_HD bool mutate_entry(Cursor& c, u32 replace_max, u32* del_next, u32& replaced) {
    ensure(c.leaf);
    Span entry = w.cget(c.idx);
    u32 elen = slen(entry);
    if (!(c.off < elen)) return false;
    bool ha = false, hc = false;
    Span a{0, 0, 0, 0}, cc{0, 0, 0, 0};
    if (c.off > 0) { elen -= c.off; a = truncate_keeping_right(entry, c.off); ha = true; }
    if (replace_max < elen) { cc = truncate(entry, replace_max); hc = true; replaced = replace_max; }
    else replaced = elen;
    if (del_next) {
      append_delete(*del_next, entry.order, (u32)entry.len);
      *del_next += (u32)entry.len;
    }
    entry.len = -entry.len;
    if (ha && hc) return replace_entry(c, a, entry, cc, 3);
    if (ha) return replace_entry(c, a, entry, entry, 2);
    if (hc) return replace_entry(c, entry, cc, cc, 2);
    set(c.idx, entry);
    c.off = replaced;
    return true;
  }
  // mutations.rs:520-570
  CRDT_HD i32 local_deactivate(Cursor c, u32 del_len, u32& del_next) {
    roll(c);
    u32 remaining = del_len;
    while (remaining > 0) {
      while (get(c.leaf, c.idx).len <= 0)
        if (!next_entry(c)) return ST_POS_OOB;
      u32 r;
      if (!mutate_entry(c, remaining, &del_next, r)) return ST_INTERNAL;
      remaining -= r;
    }
    return ST_OK;
  }
  // mutations.rs:579-615
  CRDT_HD i64 remote_deactivate(Cursor c, u32 max_len, bool& ok) {
    roll(c);
    Span e = get(c.leaf, c.idx);
    ok = true;
    if (e.len > 0) {
      u32 r;
      ok = mutate_entry(c, max_len, nullptr, r);
      return (i64)r;
    }
    u32 avail = slen(e) - c.off;
    return -(i64)(max_len < avail ? max_len : avail);
  }

  // ------------------------------------------------------------------ RLE side tables
  CRDT_HD void use_agent(u32 a) {  // agent cache (author of the current txn)
    if (a == ag_id) return;
    ag_id = a;
    ag = w.ld_agent(agp(a));
    if (ag.run_cnt) ag_last = w.ld_arun(arunp(ag) + ag.run_cnt - 1);
  }
  CRDT_HD u32 agent_next_seq(u32 agent) {  // doc.rs:20-24
    use_agent(agent);
    return ag.run_cnt ? ag_last.key + ag_last.len : 0u;
  }
  CRDT_HD bool seq_to_order(u32 agent, u32 seq, u32& order) const {  // doc.rs:26-29
    if (agent == ag_id) {
      if (ag.run_cnt && seq >= ag_last.key && seq - ag_last.key < ag_last.len) {
        order = ag_last.order + (seq - ag_last.key);
        return true;
      }
      i32 k = w.search_arun(arunp(ag), ag.run_cnt, seq);
      if (k < 0) return false;
      ARun r = w.ld_arun(arunp(ag) + k);
      order = r.order + (seq - r.key);
      return true;
    }
    AgentRec A = w.ld_agent(agp(agent));
    i32 k = w.search_arun(arunp(A), A.run_cnt, seq);
    if (k < 0) return false;
    ARun r = w.ld_arun(arunp(A) + k);
    order = r.order + (seq - r.key);
    return true;
  }
  CRDT_HD bool order_to_agent(u32 order, u32& agent) const {  // client_with_order.get()
    if (s.n_cwo && order >= cwo_last.key && order - cwo_last.key < cwo_last.len) { agent = cwo_last.agent; return true; }
    const CwoRun* base = P.cwo + seg.cwo_base;
    i32 k = w.search_cwo(base, s.n_cwo, order);
    if (k < 0) return false;
    agent = w.ld_cwo(base + k).agent;
    return true;
  }
  // doc.rs:155-165 assign_order_to_client
  CRDT_HD void assign_order_to_client(u32 agent, u32 seq, u32 order, u32 len) {
    CwoRun* cb = P.cwo + seg.cwo_base;
    if (s.n_cwo > 0 && order == cwo_last.key + cwo_last.len && agent == cwo_last.agent && seq == cwo_last.seq + cwo_last.len) {
      cwo_last.len += len;
      w.st(&cb[s.n_cwo - 1].len, cwo_last.len);
    } else {
      cwo_last = CwoRun{order, agent, seq, len};
      w.st_cwo(cb + s.n_cwo, cwo_last);
      s.n_cwo++;
    }
    use_agent(agent);
    ARun* rb = arunp(ag);
    if (ag.run_cnt > 0 && seq == ag_last.key + ag_last.len && order == ag_last.order + ag_last.len) {
      ag_last.len += len;
      w.st(&rb[ag.run_cnt - 1].len, ag_last.len);
    } else {
      ag_last = ARun{seq, order, len, 0};
      w.st_arun(rb + ag.run_cnt, ag_last);
      ag.run_cnt++;
      w.st(&agp(agent)->run_cnt, ag.run_cnt);
    }
    if (track) w.fill(P.leaf_of + seg.map_base + order, len, INVALID);
  }
  CRDT_HD void append_delete(u32 key, u32 target, u32 len) {  // Rle<KVPair<DeleteEntry>>::append
    DelRun* b = P.dels + seg.del_base;
    if (s.n_del > 0 && key == del_last.key + del_last.len && del_last.order + del_last.len == target) {
      del_last.len += len;
      w.st(&b[s.n_del - 1].len, del_last.len);
      return;
    }
    del_last = DelRun{key, target, len};
    w.st_del(b + s.n_del, del_last);
    s.n_del++;
  }
  // double_delete.rs:41-107 increment_delete_range (rare path; scalar)
  CRDT_HD bool dd_insert_at(u32 idx, DDRun r) {
    if (s.n_dd + 1 > seg.dd_cap) return false;
    DDRun* b = P.dd + seg.dd_base;
    for (u32 k = s.n_dd; k > idx; k--) w.st_dd(b + k, w.ld_dd(b + k - 1));
    w.st_dd(b + idx, r);
    s.n_dd++;
    return true;
  }
  CRDT_HD bool increment_delete_range(u32 base, u32 len) {
    DDRun* b = P.dd + seg.dd_base;
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
  CRDT_HD bool par_contains(const u32* par, u32 np, u32 p0, u32 x) const {
    if (np == 0) return false;
    if (p0 == x) return true;
    for (u32 j = 1; j < np; j++) if (w.ld(par + j) == x) return true;
    return false;
  }
  // doc.rs:350-374 insert_txn (+ advance_branch_by :34-48).  Remote parents are already in the
  // pool at [n_par, n_par + np), the first one also in p0.
  CRDT_HD i32 insert_txn(bool remote, u32 first, u32 len, u32 np, u32 p0) {
    u32* fr = P.frontier + seg.fr_base;
    u32* par = P.parents + seg.par_base + s.n_par;
    u32 last = first + len - 1;
    if (remote) {
      if (s.n_fr == 1) {
        if (fr0 == first) return ST_FRONTIER;
        if (par_contains(par, np, p0, fr0)) { fr0 = last; w.st(fr, last); }
        else { w.st(fr + 1, last); s.n_fr = 2; }
      } else {
        for (u32 k = 0; k < s.n_fr; k++) if (w.ld(fr + k) == first) return ST_FRONTIER;
        u32 m = 0;
        for (u32 k = 0; k < s.n_fr; k++) {
          u32 o = w.ld(fr + k);
          if (!par_contains(par, np, p0, o)) { w.st(fr + m, o); m++; }
        }
        if (m + 1 > FRONTIER_CAP) return ST_CAPACITY;
        w.st(fr + m, last);
        s.n_fr = m + 1;
        fr0 = w.ld(fr);
      }
    } else {
      np = s.n_fr;
      p0 = fr0;
      w.st(par, fr0);
      for (u32 k = 1; k < np; k++) w.st(par + k, w.ld(fr + k));
      w.st(fr, last);
      fr0 = last;
      s.n_fr = 1;
    }
    u32 shadow = first;
    TxnRec* tb = P.txns + seg.txn_base;
    while (shadow >= 1 && par_contains(par, np, p0, shadow - 1)) {
      u32 x = shadow - 1;
      if (s.n_txn && x >= txn_last.order && x - txn_last.order < txn_last.len) { shadow = txn_last.shadow; continue; }
      i32 k = w.search_txn(tb, s.n_txn, x);
      if (k < 0) return ST_UNKNOWN_ID;
      shadow = w.ld(&tb[k].shadow);
    }
    if (s.n_txn > 0 && np == 1 && p0 == txn_last.order + txn_last.len - 1 && shadow == txn_last.shadow) {
      txn_last.len += len;
      w.st(&tb[s.n_txn - 1].len, txn_last.len);
      return ST_OK;  // parents of a merged txn are not kept
    }
    txn_last = TxnRec{first, len, shadow, s.n_par, np, {0, 0, 0}};
    txn_last_p0 = p0;
    w.st_txn(tb + s.n_txn, txn_last);
    s.n_txn++;
    s.n_par += np;
    return ST_OK;
  }

  // ------------------------------------------------------------------ integrate (doc.rs:167-234)
  CRDT_HD i32 integrate(u32 agent, const Span& item, const Cursor* hint) {
    Cursor cursor;
    if (hint) cursor = *hint;
    else if (!get_cursor_after(item.ol, cursor)) return ST_UNKNOWN_ID;
    Cursor left = cursor, scan_start = cursor;
    bool scanning = false;
    u32 my_rank = 0;
    bool have_rank = false;
    while (true) {
      u32 other_order;
      if (!get_item(cursor, other_order)) break;
      if (other_order == item.orr) break;
      Span other_entry = get(cursor.leaf, cursor.idx);
      u32 other_left_order = origin_left_at_offset(other_entry, cursor.off);
      Cursor olc;
      if (!get_cursor_after(other_left_order, olc)) return ST_UNKNOWN_ID;
      int c = cmp(olc, left);
      if (c < 0) break;
      if (c == 0) {
        u32 oa;
        if (!order_to_agent(other_entry.order, oa)) return ST_UNKNOWN_ID;
        if (!have_rank) { my_rank = w.ld_agent(agp(agent)).rank; have_rank = true; }
        u32 other_rank = w.ld_agent(agp(oa)).rank;
        if (my_rank > other_rank) scanning = false;
        else if (item.orr == other_entry.orr) break;
        else { scanning = true; scan_start = cursor; }
      }
      if (!next_entry(cursor)) return ST_NONTERMINATING;  // cursor unchanged -> loops forever
    }
    if (scanning) cursor = scan_start;
    // RangeTree::insert (mutations.rs:202-224)
    if (!insert_internal(item, item, item, 1, cursor, INVALID)) return ST_INTERNAL;
    s.n_items += (u32)item.len;
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
    if ((u64)s.n_leaves + 2ull * n_ops > seg.leaf_cap) need |= 1u;
    if (s.n_cwo + 1 > seg.cwo_cap || s.n_txn + 1 > seg.txn_cap) need |= 2u;
    if ((u64)s.n_del + n_dels > seg.del_cap) need |= 4u;
    if ((u64)s.n_par + (remote ? n_parents : s.n_fr) > seg.par_cap) need |= 8u;
    if (track && (u64)s.next_order + txn_len > seg.map_cap) need |= 16u;
    use_agent(agent);
    if (ag.run_cnt + 1 > ag.run_cap) need |= 32u;
    s.cap_need = need;
    return need == 0;
  }

  // doc.rs:376-469 apply_local_txn.  Header at record `pos`; ops follow.
  CRDT_HD i32 apply_local_txn(const Rec& hdr, u32 pos) {
    u32 nops = hdr.w0 & 0x0FFFFFFFu;
    u32 agent = hdr.w1;
    u32 span = hdr.w3;
    if (agent >= s.n_agents) return ST_UNKNOWN_AGENT;
    if (span == 0) return ST_EMPTY_TXN;
    if (!fits(false, agent, nops, hdr.w2, span, 0)) return ST_NEED_CAPACITY;
    u32 first = s.next_order;
    u32 next = first;
    assign_order_to_client(agent, agent_next_seq(agent), first, span);
    s.next_order = first + span;
    for (u32 k = 0; k < nops; k++) {
      Rec op = rec(pos + 1 + k);
      u32 p = op.w1, del = op.w2, ins = op.w3;
      if (del > 0) {
        if ((u64)p + del > cur_len()) return ST_POS_OOB;
        Cursor c;
        if (!cursor_at_content_pos(p, c)) return ST_POS_OOB;
        u32 before = next;
        i32 st = local_deactivate(c, del, next);
        if (st != ST_OK) return st;
        if (next - before != del) return ST_POS_OOB;
      }
      if (ins > 0) {
        u32 order = next;
        next += ins;
        u32 ol;
        Cursor c;
        if (p == 0) { ol = ROOT_ORDER; c = cursor_at_start(); }
        else {
          if (p > cur_len()) return ST_POS_OOB;
          if (!cursor_at_content_pos(p - 1, c)) return ST_POS_OOB;
          if (!get_item(c, ol)) return ST_POS_OOB;
          if (!next_item(c)) return ST_POS_OOB;
        }
        u32 orr;
        if (!get_item(c, orr)) orr = ROOT_ORDER;
        Span item{order, ol, orr, (i32)ins};
        i32 st = integrate(agent, item, &c);
        if (st != ST_OK) return st;
      }
    }
    if (next != first + span) return ST_BAD_INPUT;
    return insert_txn(false, first, span, 0, 0);
  }

  // doc.rs:242-348 apply_remote_txn.  Header at record `pos`; ops then parents follow.
  CRDT_HD i32 apply_remote_txn(const Rec& hdr, u32 pos) {
    u32 nops = hdr.w0 & 0x07FFFFFFu;
    bool zero_op = (hdr.w0 >> 27) & 1u;
    u32 agent = hdr.w1 & 0xFFFFu;
    u32 np = hdr.w1 >> 16;
    u32 seq = hdr.w2;
    u32 txn_len = hdr.w3;
    if (agent >= s.n_agents) return ST_UNKNOWN_AGENT;
    if (agent_next_seq(agent) != seq) return ST_SEQ;
    if (zero_op) return ST_BAD_INPUT;
    if (txn_len == 0) return ST_EMPTY_TXN;
    if (!fits(true, agent, nops, nops, txn_len, np)) return ST_NEED_CAPACITY;
    u32 first = s.next_order;
    u32 next = first;
    assign_order_to_client(agent, seq, first, txn_len);
    s.next_order = first + txn_len;
    for (u32 k = 0; k < nops; k++) {
      Rec op = rec(pos + 1 + k);
      u32 kind = rec_kind(op);
      u32 len = op.w0 & 0x0FFFFFFFu;
      if (kind == REC_RINS) {
        u32 order = next;
        next += len;
        u32 ol, orr;
        i32 st = id_to_order(op.w1 & 0xFFFFu, op.w2, ol);
        if (st != ST_OK) return st;
        st = id_to_order(op.w1 >> 16, op.w3, orr);
        if (st != ST_OK) return st;
        Span item{order, ol, orr, (i32)len};
        st = integrate(agent, item, nullptr);
        if (st != ST_OK) return st;
      } else if (kind == REC_RDEL) {
        u32 order = next;
        next += len;
        u32 target;
        i32 st = id_to_order(op.w1 & 0xFFFFu, op.w2, target);
        if (st != ST_OK) return st;
        append_delete(order, target, len);
        u32 remaining = len;
        while (remaining > 0) {
          if (target == ROOT_ORDER) return ST_NONTERMINATING;
          Cursor c;
          if (!get_cursor_before(target, c)) return ST_UNKNOWN_ID;
          bool ok;
          i64 amt = remote_deactivate(c, remaining, ok);
          if (!ok) return ST_INTERNAL;
          u32 here = (u32)(amt < 0 ? -amt : amt);
          if (here == 0) return ST_NONTERMINATING;
          if (amt < 0 && !increment_delete_range(target, here)) return ST_CAPACITY;
          remaining -= here;
          target += here;
        }
      } else {
        return ST_BAD_INPUT;
      }
    }
    u32* par = P.parents + seg.par_base + s.n_par;
    u32 p0 = 0;
    for (u32 k = 0; k < np; k++) {
      Rec pr = rec(pos + 1 + nops + k);
      if (rec_kind(pr) != REC_RPARENT) return ST_BAD_INPUT;
      u32 o;
      i32 st = id_to_order(pr.w1 & 0xFFFFu, pr.w2, o);
      if (st != ST_OK) return st;
      w.st(par + k, o);
      if (k == 0) p0 = o;
    }
    return insert_txn(true, first, txn_len, np, p0);
  }

  // Replay this document's record stream from s.rec_pos.
  CRDT_HD void run() {
    u32 pos = s.rec_pos;
    while (s.status == ST_OK && pos < seg.rec_n) {
      Rec h = rec(pos);
      u32 kind = rec_kind(h);
      i32 st;
      u32 consumed;
      if (kind == REC_LTXN) {
        u32 nops = h.w0 & 0x0FFFFFFFu;
        consumed = 1 + nops;
        st = (pos + consumed <= seg.rec_n) ? apply_local_txn(h, pos) : ST_BAD_INPUT;
      } else if (kind == REC_RTXN) {
        u32 nops = h.w0 & 0x07FFFFFFu;
        consumed = 1 + nops + (h.w1 >> 16);
        st = (pos + consumed <= seg.rec_n) ? apply_remote_txn(h, pos) : ST_BAD_INPUT;
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
