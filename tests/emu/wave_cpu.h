// TEST INFRASTRUCTURE: a sequential CPU emulation of the WaveGPU backend, so replay_core.h's
// control logic can be run (and debugged under ASan/gdb) against the oracle without a GPU.
// Each method is the plain-loop meaning of the matching lane-parallel WaveGPU method.
// Never linked into the product library.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crdt_types.h"

// (statistics build of the emulator: counts of context / cache-lane accesses, the GPU's
// v_readlane / v_writelane traffic)
#ifndef WCPU_COUNT
#define WCPU_COUNT(kind, f) ((void)0)
#endif
// (statistics build: the bytes each method reads / writes in device memory, as the WaveGPU method
// accesses them -- a lane-parallel load touches every lane's element)
#ifndef WCPU_MEM
#define WCPU_MEM(p, n, wr) ((void)0)
#endif

namespace crdt {

template <int L>
struct WaveCPU {
  Span c[64];
  std::vector<u32> gb, gc, gv;  // the root, flat (the GPU's two-level root has the same semantics)
  void root_room(u32 n) { if (gb.size() < n) { gb.resize(n, 0); gc.resize(n, 0); gv.resize(n, 0); } }

  WaveCPU() { std::memset(c, 0, sizeof(c)); }

  // context registers (plain array: slot f)
  u32 x[192] = {};
  u32 xg(u32 f) const { WCPU_COUNT(0, f); return x[f]; }
  template <class T> static T* gptr(u64 v) { return (T*)v; }
  void xs(u32 f, u32 v) { WCPU_COUNT(1, f); x[f] = v; }
  void x_pin() {}
  void bind_root(const Pools&, const DocSeg&) {}
  void x_load_state(const DocState* p, u32 base) { std::memcpy(x + base, p, sizeof(DocState)); }
  void x_store_state(DocState* p, u32 base) const { std::memcpy(p, x + base, sizeof(DocState)); }

  static u64 clock() { return 0; }
  u32 ld(const u32* p) const { WCPU_MEM(p, 4, 0); return *p; }
  u32 ld_raw(const u32* p) const { WCPU_MEM(p, 4, 0); return *p; }
  void ld_raw2(const u32* p, u32& a, u32& b) const { WCPU_MEM(p, 8, 0); a = p[0]; b = p[1]; }
  static u32 uni_(u32 x) { return x; }
  void st(u32* p, u32 v) const { WCPU_MEM(p, 4, 1); *p = v; }
  void st(i32* p, i32 v) const { WCPU_MEM(p, 4, 1); *p = v; }
  void st_lanes(u32* p, u32 v, u32 n) const { if (n) { WCPU_MEM(p, 4, 1); *p = v; } }
  template <class T> T ldT(const T* p) const { WCPU_MEM(p, sizeof(T), 0); return *p; }
  template <class T> void stT(T* p, const T& v) const { WCPU_MEM(p, sizeof(T), 1); *p = v; }
  AgentRec ld_agent(const AgentRec* p) const { WCPU_MEM(p, sizeof(AgentRec), 0); return *p; }
  void st_agent_tail(AgentRec* p, u32 key, u32 order, u32 len) const { WCPU_MEM(&p->tkey, 12, 1); p->tkey = key; p->torder = order; p->tlen = len; }
  ARun ld_arun(const ARun* p) const { WCPU_MEM(p, sizeof(ARun), 0); return *p; }
  void st_arun(ARun* p, const ARun& v) const { WCPU_MEM(p, sizeof(ARun), 1); *p = v; }
  CwoRun ld_cwo(const CwoRun* p) const { WCPU_MEM(p, sizeof(CwoRun), 0); return *p; }
  void st_cwo(CwoRun* p, const CwoRun& v) const { WCPU_MEM(p, sizeof(CwoRun), 1); *p = v; }
  DelRun ld_del(const DelRun* p) const { WCPU_MEM(p, sizeof(DelRun), 0); return *p; }
  void st_del(DelRun* p, const DelRun& v) const { WCPU_MEM(p, sizeof(DelRun), 1); *p = v; }
  DDRun ld_dd(const DDRun* p) const { WCPU_MEM(p, sizeof(DDRun), 0); return *p; }
  void st_dd(DDRun* p, const DDRun& v) const { WCPU_MEM(p, sizeof(DDRun), 1); *p = v; }
  TxnRec ld_txn(const TxnRec* p) const { WCPU_MEM(p, sizeof(TxnRec), 0); return *p; }
  void st_txn(TxnRec* p, const TxnRec& v) const { WCPU_MEM(p, sizeof(TxnRec), 1); *p = v; }
  Rec ld_rec(const Rec* p) const { WCPU_MEM(p, sizeof(Rec), 0); return *p; }
  template <u32 M = 1, class T> static T* at(T* base, u32 idx) { return base + (u64)idx * M; }
  void st_state(DocState* p, const DocState& s) const { *p = s; }
  DocState ld_state(const DocState* p) const { return *p; }
  DocSeg ld_seg(const DocSeg* p) const { return *p; }
  void fill(u32* p, u32 n, u32 v) const { WCPU_MEM(p, 4ull * n, 1); for (u32 k = 0; k < n; k++) p[k] = v; }
  void fill16(u16* p, u32 n, u32 v) const { WCPU_MEM(p, 2ull * n, 1); for (u32 k = 0; k < n; k++) p[k] = (u16)v; }
  u32 ld16(const u16* p) const { WCPU_MEM(p, 2, 0); return *p; }
  void zero_leaf(Span* p, u32 n) const { WCPU_MEM(p, sizeof(Span) * n, 1); std::memset(p, 0, sizeof(Span) * n); }

  template <class T> static u32 rkey(const T& r) { return ((const u32*)&r)[0]; }
  static u32 rlen(const ARun& r) { return r.len; }
  static u32 rlen(const CwoRun& r) { return r.len; }
  static u32 rlen(const DDRun& r) { return r.len; }
  static u32 rlen(const TxnRec& r) { return r.len; }
  // the elements the GPU's 64-ary search samples (wave_gpu.h search / search_first), key(i) of element i
  template <class T, class K> void search_touch(const T* b, u32 n, u32 x, K key) const {
    u32 lo = 0, hi = n;
    while (hi - lo > 64) {
      u32 step = (hi - lo + 63) / 64, best = INVALID;
      for (u32 l = 0; l < 64; l++) {
        u32 idx = lo + l * step;
        if (idx >= hi) break;
        WCPU_MEM(b + idx, sizeof(T), 0);
        if (key(idx) <= x) best = l;
      }
      if (best == INVALID) return;
      lo = lo + best * step;
      hi = lo + step < hi ? lo + step : hi;
    }
    WCPU_MEM(b + lo, sizeof(T) * (hi - lo), 0);
  }
  template <class T> i32 search(const T* b, u32 n, u32 x) const {  // simple_rle.rs:18-25
    search_touch(b, n, x, [&](u32 i) { return rkey(b[i]); });
    u32 lo = 0, hi = n;
    while (lo < hi) {
      u32 mid = (lo + hi) / 2;
      u32 k = rkey(b[mid]);
      if (x < k) hi = mid;
      else if (x >= k + rlen(b[mid])) lo = mid + 1;
      else return (i32)mid;
    }
    return -1;
  }
  i32 search_arun(const ARun* b, u32 n, u32 x) const { return search(b, n, x); }
  template <class T> i32 search_run(const T* b, u32 n, u32 x, T& out) const {
    i32 k = search(b, n, x);
    if (k >= 0) out = b[k];
    return k;
  }
  template <class T> i32 search_run_recent(const T* b, u32 n, u32 x, T& out) const {
    if (n <= 64u) return search_run(b, n, x, out);
    WCPU_MEM(b + n - 64u, sizeof(T) * 64u, 0);
    if (rkey(b[n - 64u]) > x) return search_run(b, n - 64u, x, out);
    u32 k = n - 64u;
    while (k + 1u < n && rkey(b[k + 1u]) <= x) k++;
    if (x - rkey(b[k]) >= rlen(b[k])) return -1;
    out = b[k];
    return (i32)k;
  }
  i32 search_cwo(const CwoRun* b, u32 n, u32 x) const { return search(b, n, x); }
  DDBlk ld_ddblk(const DDBlk* p) const { return *p; }
  void st_ddblk(DDBlk* p, const DDBlk& v) const { *p = v; }
  i32 search_first(const DDBlk* b, u32 n, u32 x) const {
    search_touch(b, n, x, [&](u32 i) { return b[i].first; });
    i32 r = -1;
    for (u32 i = 0; i < n; i++) if (b[i].first <= x) r = (i32)i;
    return r;
  }
  // the directory's top level (WaveGPU: in LDS): word j = the first key of block 64 j; every
  // search checks it against the directory (a stale word aborts)
  u32 dt[DDT_LDS] = {};
  i32 dd_search_top(const DDBlk* b, u32 nb, u32 x) const {
    u32 nt = (nb + 63u) >> 6;
    for (u32 j = 0; j < nt; j++)
      if (dt[j] != b[64u * j].first) {
        std::fprintf(stderr, "wave_cpu: stale double-delete top level (word %u: %u, block %u)\n", j, dt[j], b[64u * j].first);
        std::abort();
      }
    i32 g = -1;
    for (u32 j = 0; j < nt; j++) if (dt[j] <= x) g = (i32)j;
    if (g < 0) return -1;
    u32 base = (u32)g * 64u, cnt = nb - base < 64u ? nb - base : 64u;
    WCPU_MEM(b + base, sizeof(DDBlk) * cnt, 0);
    i32 r = -1;
    for (u32 i = 0; i < cnt; i++) if (b[base + i].first <= x) r = (i32)(base + i);
    return r;
  }
  void ddt_set(u32 j, u32 key) { dt[j] = key; }
  void ddt_rebuild(const DDBlk* b, u32 j0, u32 nb) {
    u32 nt = (nb + 63u) >> 6;
    for (u32 j = j0; j < nt; j++) { WCPU_MEM(b + 64u * j, sizeof(DDBlk), 0); dt[j] = b[64u * j].first; }
  }
  u32 dd_count_le(const DDRun* blk, u32 cnt, u32 x) const { WCPU_MEM(blk, sizeof(DDRun) * cnt, 0); u32 k = 0; for (u32 i = 0; i < cnt; i++) k += blk[i].key <= x; return k; }
  u32 dd_split(const DDRun* src, DDRun* dst) const { WCPU_MEM(src + 32, sizeof(DDRun) * 32, 0); WCPU_MEM(dst, sizeof(DDRun) * 32, 1); for (u32 i = 32; i < 64; i++) dst[i - 32] = src[i]; return dst[0].key; }
  void dd_block_insert(DDRun* blk, u32 cnt, u32 i, const DDRun& r) const {
    WCPU_MEM(blk, sizeof(DDRun) * cnt, 0); WCPU_MEM(blk + i, sizeof(DDRun) * (cnt + 1 - i), 1);
    for (u32 k = cnt; k > i; k--) blk[k] = blk[k - 1];
    blk[i] = r;
  }
  void ddb_insert(DDBlk* b, u32 n, u32 at, const DDBlk& v) const {
    WCPU_MEM(b + at, sizeof(DDBlk) * (n - at), 0); WCPU_MEM(b + at, sizeof(DDBlk) * (n + 1 - at), 1);
    for (u32 k = n; k > at; k--) b[k] = b[k - 1];
    b[at] = v;
  }
  i32 search_txn(const TxnRec* b, u32 n, u32 x) const { return search(b, n, x); }

  // leaf cache
  u32 cache_load(const Span* p) {
    WCPU_MEM(p, sizeof(Span) * L, 0);
    u32 n = 0;
    for (u32 i = 0; i < 64; i++) c[i] = i < (u32)L ? p[i] : Span{0, 0, 0, 0};
    for (u32 i = 0; i < (u32)L; i++) n += c[i].len != 0;
    return n;
  }
  void cache_store(Span* p) const { WCPU_MEM(p, sizeof(Span) * L, 1); for (u32 i = 0; i < (u32)L; i++) p[i] = c[i]; }
  Span cget(u32 i) const { WCPU_COUNT(2, 0); return c[i & 63]; }
  u32 cget_order(u32 i) const { WCPU_COUNT(3, 0); return c[i & 63].order; }
  i32 cget_len(u32 i) const { WCPU_COUNT(3, 1); return c[i & 63].len; }
  void cset(u32 i, const Span& s) { WCPU_COUNT(4, 0); c[i & 63] = s; }
  void cset_len(u32 i, i32 len) { c[i & 63].len = len; }
  template <class F> void cset_lanes(u32 a, u32 b, F f) { for (u32 l = a; l < b && l < 64; l++) c[l] = f(l); }
  template <class F> void leaf_write_lanes(Span* dst, u32 n, F f) const {
    WCPU_MEM(dst, sizeof(Span) * L, 1);
    for (u32 l = 0; l < (u32)L; l++) dst[l] = l < n ? f(l) : Span{0, 0, 0, 0};
  }
  u32 cache_vis_from(u32 a) const { u32 t = 0; for (u32 i = a; i < 64; i++) t += clen(c[i]); return t; }
  void rank_load(const AgentRec*, u32) const {}
  u32 rank_of(const AgentRec* agents, u32, u32 a) const { return agents[a].rank; }
  mutable const u16* oag = nullptr;  // (scan_gather's map, read by scan_batch)
  u32 scan_gather(u32 nn, const u16* m) const { for (u32 j = 0; j < nn && j < 64; j++) WCPU_MEM(m + c[j].order, 2, 0); oag = m; return 0u; }
  // agent rows: word 0 (valid) is what the replay sees; a current row must hold exactly the map's
  // agents of the cached leaf's entries (checked here: a stale row taken as current aborts)
  mutable const u32* lag_p = nullptr;
  u32 lag_ld(const u32* p) const { WCPU_MEM(p, 4 * lag_words(L), 0); lag_p = p; return p[0]; }
  u32 lag_valid(u32 lw) const { return lw == 1u; }
  u32 lag_agents(u32, u32 n, const u16* m, u32 tkey, u32 tlen, u32 tagent) const {
    oag = m;
    for (u32 j = 0; j < n; j++) {
      u32 o = c[j].order, want = o - tkey < tlen ? tagent : m[o];
      u32 v = lag_p[lag_words(L) / 2 + j / 2];
      u32 got = (j & 1) ? v >> 16 : v & 0xFFFFu;
      if (got != want) {
        std::fprintf(stderr, "wave_cpu: stale leaf agent row (entry %u: %u, map %u)\n", j, got, want);
        std::abort();
      }
    }
    return 0u;
  }
  void lag_store(u32* p, u32, u32 n, u32 tkey, u32 tlen, u32 tagent, u32, u32 n_agents, const AgentRec* agents) const {
    WCPU_MEM(p, 4 * lag_words(L), 1);
    for (u32 j = 0; j < (u32)L / 2; j++) p[lag_words(L) / 2 + j] = 0;
    u32 mr = 0, omin = 0xFFFFFFFFu, omax = 0, mixed = n == 0 ? LAG_MIXED : 0u;
    for (u32 j = 0; j < n; j++) {
      u32 o = c[j].order, a = (o - tkey < tlen ? tagent : oag[o]) & 0xFFFFu;
      p[lag_words(L) / 2 + j / 2] |= (j & 1) ? a << 16 : a;
      mr = std::max(mr, agents[a].rank);
      omin = std::min(omin, o);
      omax = std::max(omax, o);
      if (c[j].ol != c[0].ol) mixed = LAG_MIXED;
    }
    p[LAG_EPOCH] = n_agents | mixed;
    p[LAG_OL] = c[0].ol;
    p[LAG_RANK] = mr;
    p[LAG_OMIN] = omin;
    p[LAG_OMAX] = omax;
    p[0] = 1u;
  }
  // skip_leaves' block step; every leaf it passes is checked against its entries (the scan must
  // pass each with no event: origin_left X, rank below my_rank, first order not orr)
  u32 skip_scan(const u32* row, u32 a, u32 cnt, const u32* lag, u32 X, u32 orr, u32 my_rank, u32 n_agents,
                const Span* leaves, const AgentRec* agents, u32& leaf) const {
    WCPU_MEM(row, 4 * 64, 0);
    for (u32 j = a; j < cnt; j++) {
      const u32* q = lag + (size_t)row[j] * lag_words(L);
      WCPU_MEM(q, 4 * (LAG_OMAX + 1), 0);
      bool skip = q[0] == 1u && q[1] == n_agents && q[LAG_OL] == X && q[LAG_RANK] < my_rank &&
                  orr - q[LAG_OMIN] > q[LAG_OMAX] - q[LAG_OMIN];
      if (!skip) { leaf = row[j]; return j; }
      const Span* e = leaves + (size_t)row[j] * L;
      for (u32 k = 0; k < (u32)L; k++) {
        if (e[k].len == 0) continue;
        u32 ag = q[lag_words(L) / 2 + k / 2];
        ag = (k & 1) ? ag >> 16 : ag & 0xFFFFu;
        if (e[k].ol != X || e[k].order == orr || agents[ag].rank >= my_rank) {
          std::fprintf(stderr, "wave_cpu: leaf %u skipped by a stale summary (entry %u)\n", row[j], k);
          std::abort();
        }
      }
    }
    return cnt;
  }
  void prefetch_drain() const {}
  u32 rank_row(u32) const { return 0u; }
  u32 scan_batch(u32, u32, u32 me, u32 a, u32 n, u32 X, u32 orr, const AgentRec* agents, u32 n_agents, u32 tkey,
                 u32 tlen, u32 tagent, u32& last, u32& last_scan) const {
    u32 my_rank = agents[me].rank;
    auto agent_of = [&](u32 o) -> u32 { return o - tkey < tlen ? tagent : oag[o]; };
    u32 f = n;
    for (u32 j = a; j < n; j++) {
      u32 rk = agents[agent_of(c[j].order)].rank;
      bool lt = my_rank > rk;
      if (c[j].order == orr || c[j].ol != X || (!lt && c[j].orr == orr)) { f = j; break; }
    }
    last = f > a ? f - 1u : INVALID;
    last_scan = 0;
    if (f > a) last_scan = my_rank > agents[agent_of(c[f - 1].order)].rank ? 0u : 1u;
    return f;
  }
  u64 vis_lanes(u32 a, u32 b) const { u64 m = 0; for (u32 i = a; i < b && i < 64; i++) if (c[i].len > 0) m |= 1ull << i; return m; }
  void negate_visible(u32 a, u32 b) { for (u32 i = a; i < b && i < 64; i++) if (c[i].len > 0) c[i].len = -c[i].len; }
  u64 lanes_in(u32 a, u32 b) const { u64 m = 0; for (u32 i = a; i < b && i < 64; i++) m |= 1ull << i; return m; }
  static u32 first_lane(u64 m) { return (u32)__builtin_ctzll(m); }
  i32 peek_find_order(const Span* p, u32 order, u32& start) const {
    WCPU_MEM(p, sizeof(Span) * L, 0);
    for (u32 i = 0; i < (u32)L; i++)
      if (p[i].len != 0 && order >= p[i].order && order - p[i].order < slen(p[i])) { start = p[i].order; return (i32)i; }
    return -1;
  }
  bool cfind_content(u32 n, u32 rem, u32& idx, u32& off) const {
    for (u32 i = 0; i < n; i++) {
      u32 e = clen(c[i]);
      if (rem < e) { idx = i; off = rem; return true; }
      rem -= e;
    }
    if (rem == 0) { idx = n; off = 0; return true; }
    return false;
  }
  i32 cfind_order(u32 n, u32 order) const {
    // WaveGPU::cfind_order relies on it: the cached leaf's lanes from n on are empty
    for (u32 i = n; i < 64; i++) if (c[i].len != 0) __builtin_trap();
    for (u32 i = 0; i < n; i++) if (order >= c[i].order && order - c[i].order < slen(c[i])) return (i32)i;
    return -1;
  }
  Span mv[64];
  void cache_write_moved(Span* dst, u32 idx, u32 n, u32 padding) {
    WCPU_MEM(dst, sizeof(Span) * L, 1);
    for (u32 j = 0; j < 64; j++) {
      u32 src = j + idx - padding;
      mv[j] = (j < (u32)L && j >= padding && src < n) ? c[src] : Span{0, 0, 0, 0};
      if (j < (u32)L) dst[j] = mv[j];
    }
  }
  void cache_from_moved() { for (u32 j = 0; j < 64; j++) c[j] = mv[j]; }
  Span pfr[64];
  void leaf_prefetch(const Span* p) { WCPU_MEM(p, sizeof(Span) * L, 0); for (u32 j = 0; j < 64; j++) pfr[j] = j < (u32)L ? p[j] : Span{0, 0, 0, 0}; }
  u32 cache_from_prefetch() { u32 n = 0; for (u32 j = 0; j < 64; j++) { c[j] = pfr[j]; n += c[j].len != 0; } return n; }
  void fill_runs(u32* base, u32 a, u32 b, u32 v) const {
    for (u32 i = a; i < b; i++) { WCPU_MEM(base + c[i].order, 4ull * slen(c[i]), 1); for (u32 t = 0; t < slen(c[i]); t++) base[c[i].order + t] = v; }
  }
  void cache_clear(u32 a, u32 b) { for (u32 i = a; i < b; i++) c[i] = Span{0, 0, 0, 0}; }
  void cache_shift_right(u32 idx, u32 n, u32 k) {
    for (i32 i = (i32)n - 1; i >= (i32)idx; i--) c[i + k] = c[i];
    for (u32 i = idx; i < idx + k; i++) c[i] = Span{0, 0, 0, 0};
  }
  Rec rb[64], qb[64];
  void rec_load2(const Rec* p, u32 n, u32 n_ahead) {
    WCPU_MEM(p, sizeof(Rec) * n, 0); WCPU_MEM(p + 64, sizeof(Rec) * n_ahead, 0);
    for (u32 i = 0; i < n; i++) rb[i] = p[i];
    for (u32 i = 0; i < n_ahead; i++) qb[i] = p[64 + i];
  }
  void rec_slide(u32 d, const Rec* p_ahead, u32 n_ahead) {
    WCPU_MEM(p_ahead, sizeof(Rec) * n_ahead, 0);
    Rec t[128];
    for (u32 i = 0; i < 64; i++) { t[i] = rb[i]; t[64 + i] = qb[i]; }
    for (u32 i = 0; i < 64; i++) rb[i] = t[(i + d) & 127];
    for (u32 i = 0; i < n_ahead; i++) qb[i] = p_ahead[i];
  }
  Rec rec_get(u32 k) const { return rb[k]; }
  void gen_draws(u32 seed, u32 base) {
    for (u32 i = 0; i < 64; i++) { GenDraw d = gen_draw(seed, base + i); rb[i] = Rec{d.hi, d.lo, d.r2, 0u}; }
  }
  // the GPU backend's scans over 64 records at p (no window move); len0 = the first txn's length
  u32 typing_scan_at(const Rec* p, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1, u32 ow3, u32& total, u32& len0) const {
    WCPU_MEM(p, sizeof(Rec) * nv, 0);
    Rec t[64];
    for (u32 i = 0; i < nv; i++) t[i] = p[i];
    len0 = (compact & remote) ? rc_len(t[0]) : t[0].w3;
    return typing_scan_b(t, 0u, nv, remote, compact, agent, ow1, ow3, total);
  }
  u32 delete_scan_at(const Rec* p, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) const {
    WCPU_MEM(p, sizeof(Rec) * nv, 0);
    Rec t[64];
    for (u32 i = 0; i < nv; i++) t[i] = p[i];
    return delete_scan_b(t, 0u, nv, remote, compact, agent, delta);
  }
  u32 typing_scan(u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1, u32 ow3, u32& total) const {
    return typing_scan_b(rb, b0, nv, remote, compact, agent, ow1, ow3, total);
  }
  u32 delete_scan(u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) const {
    return delete_scan_b(rb, b0, nv, remote, compact, agent, delta);
  }
  u32 frontier_advance(u32* f, u32 nfr, u32 f0, const u32* pp, u32 np, u32 p0, u32 first, u32 last, u32 cap,
                       u32& nf0) const {
    WCPU_MEM(f, 4ull * nfr + 4, 0); WCPU_MEM(pp, 4ull * np, 0); WCPU_MEM(f, 4ull * nfr + 4, 1);
    std::vector<u32> h(nfr);
    for (u32 k = 0; k < nfr; k++) h[k] = k == 0 ? f0 : f[k];
    for (u32 k = 0; k < nfr; k++) if (h[k] == first) return 0u;
    auto has = [&](u32 x) {
      if (np == 0) return false;
      if (p0 == x) return true;
      for (u32 j = 1; j < np; j++) if (pp[j] == x) return true;
      return false;
    };
    std::vector<u32> kept;
    for (u32 k = 0; k < nfr; k++) if (!has(h[k])) kept.push_back(h[k]);
    u32 m = (u32)kept.size();
    if (m + 1u > cap) return INVALID;
    nf0 = m ? kept[0] : last;
    for (u32 k = 1; k < m; k++) f[k] = kept[k];
    if (m) f[m] = last;
    return m + 1u;
  }
  void fr_lanes_load(const u32* f, u32 n) {
    WCPU_MEM(f, 4ull * n, 0);
    for (u32 k = 1; k < n; k++) x[FR_S0 + k - 1u] = f[k];
  }
  void fr_lanes_store(u32* f, u32 n) const {
    WCPU_MEM(f, 4ull * n, 1);
    for (u32 k = 1; k < n; k++) f[k] = x[FR_S0 + k - 1u];
  }
  u32 frontier_advance_x(u32 nfr, u32 f0, const u32* pp, u32 np, u32 p0, u32 first, u32 last, u32 cap, u32& nf0,
                         u32* f) {
    WCPU_MEM(pp, 4ull * np, 0);
    std::vector<u32> h(nfr);
    for (u32 k = 0; k < nfr; k++) h[k] = k == 0 ? f0 : x[FR_S0 + k - 1u];
    for (u32 k = 0; k < nfr; k++) if (h[k] == first) return 0u;
    auto has = [&](u32 v) {
      if (np == 0) return false;
      if (p0 == v) return true;
      for (u32 j = 1; j < np; j++) if (pp[j] == v) return true;
      return false;
    };
    std::vector<u32> kept;
    for (u32 k = 0; k < nfr; k++) if (!has(h[k])) kept.push_back(h[k]);
    u32 m = (u32)kept.size();
    if (m + 1u > cap) return INVALID;
    nf0 = m ? kept[0] : last;
    if (m <= FR_LANES) {
      for (u32 k = 1; k < m; k++) x[FR_S0 + k - 1u] = kept[k];
      if (m) x[FR_S0 + m - 1u] = last;
    } else {
      WCPU_MEM(f, 4ull * (m + 1u), 1);
      for (u32 k = 1; k < m; k++) f[k] = kept[k];
      f[m] = last;
    }
    return m + 1u;
  }
  u32 front_scan(u32 b0, u32 nv, u32 agent, u32 len) const {
    u32 n = 1;
    for (u32 j = b0 + 1; j < nv; j++) {
      const Rec& r = rb[j];
      if (!(r.w0 == ((REC_LC << 28) | agent) && r.w1 == 0u && r.w2 == 0u && r.w3 == len)) break;
      n++;
    }
    return n;
  }
  static u32 typing_scan_b(const Rec* rb, u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1, u32 ow3, u32& total) {
    if (compact) {
      u32 n = 1;
      total = remote ? rc_len(rb[b0]) : rb[b0].w3;
      for (u32 j = b0 + 1; j < nv; j++) {
        const Rec &r = rb[j], &p = rb[j - 1];
        bool ok;
        u32 hl;
        if (remote) {
          hl = rc_len(r);
          u32 ra = r.w3 == 0xFFFFFFFFu ? 0xFFFFu : agent;
          ok = (r.w0 & RC_HDR_MASK) == ((REC_RC << 28) | agent) && hl != 0 && r.w1 == p.w1 + rc_len(p) &&
               r.w2 == r.w1 - 1u && r.w3 == ow3 && (agent | (ra << 16)) == ow1;
        } else {
          hl = r.w3;
          ok = r.w0 == ((REC_LC << 28) | agent) && r.w2 == 0u && r.w3 - 1u < 0xFFFFu && r.w1 == p.w1 + p.w3;
        }
        if (!ok) break;
        n++;
        total += hl;
      }
      return n;
    }
    u32 per = remote ? 3u : 2u;
    u32 n = 1;
    total = rb[b0].w3;
    for (u32 j = b0 + per; j + per <= nv; j += per) {
      const Rec &h = rb[j], &o = rb[j + 1], &ph = rb[j - per], &po = rb[j - per + 1];
      bool ok;
      if (remote) {
        const Rec& pr = rb[j + 2];
        ok = h.w0 == ((REC_RTXN << 28) | 1u) && h.w1 == (agent | (1u << 16)) && h.w2 == ph.w2 + ph.w3 &&
             h.w3 - 1u < 0xFFFFu && (o.w0 >> 28) == REC_RINS && (o.w0 & 0x0FFFFFFFu) == h.w3 && o.w1 == ow1 &&
             o.w3 == ow3 && o.w2 == h.w2 - 1u && pr.w0 == (REC_RPARENT << 28) && pr.w1 == agent && pr.w2 == h.w2 - 1u;
      } else {
        ok = h.w0 == ((REC_LTXN << 28) | 1u) && h.w1 == agent && h.w2 == 0u && h.w3 - 1u < 0xFFFFu &&
             o.w0 == (REC_LOP << 28) && o.w2 == 0u && o.w3 == h.w3 && o.w1 == po.w1 + po.w3;
      }
      (void)ph;
      if (!ok) break;
      n++;
      total += h.w3;
    }
    return n;
  }

  static u32 delete_scan_b(const Rec* rb, u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) {
    if (compact) {
      u32 n = 1;
      for (u32 j = b0 + 1; j < nv; j++) {
        const Rec &r = rb[j], &p = rb[j - 1];
        bool ok = remote ? (r.w0 == ((REC_RC << 28) | (1u << 27) | (1u << 16) | agent) && r.w1 == p.w1 + 1u && r.w2 == p.w2 + delta)
                         : (r.w0 == ((REC_LC << 28) | agent) && r.w2 == 1u && r.w3 == 0u && r.w1 == p.w1 + delta);
        if (!ok) break;
        n++;
      }
      return n;
    }
    u32 per = remote ? 3u : 2u;
    u32 n = 1;
    for (u32 j = b0 + per; j + per <= nv; j += per) {
      const Rec &h = rb[j], &o = rb[j + 1], &ph = rb[j - per], &po = rb[j - per + 1];
      bool ok;
      if (remote) {
        const Rec& pr = rb[j + 2];
        ok = h.w0 == ((REC_RTXN << 28) | (1u << RTXN_DEL_BIT) | 1u) && h.w1 == (agent | (1u << 16)) && h.w2 == ph.w2 + 1u && h.w3 == 1u &&
             o.w0 == ((REC_RDEL << 28) | 1u) && o.w1 == agent && o.w2 == po.w2 + delta &&
             pr.w0 == (REC_RPARENT << 28) && pr.w1 == agent && pr.w2 == h.w2 - 1u;
      } else {
        ok = h.w0 == ((REC_LTXN << 28) | 1u) && h.w1 == agent && h.w2 == 1u && h.w3 == 1u &&
             o.w0 == (REC_LOP << 28) && o.w2 == 1u && o.w3 == 0u && o.w1 == po.w1 + delta;
      }
      if (!ok) break;
      n++;
    }
    return n;
  }
  void st_del_run(DelRun* p, u32 cnt, u32 key0, u32 t0) const {
    WCPU_MEM(p, sizeof(DelRun) * cnt, 1);
    for (u32 j = 0; j < cnt; j++) p[j] = DelRun{key0 + j, t0 - j, 1u};
  }

  // directory root
  void root_init(u32 blk, u32 cnt, u32 vis) {
    gb.assign(64, 0); gc.assign(64, 0); gv.assign(64, 0);
    gb[0] = blk; gc[0] = cnt; gv[0] = vis;
  }
  void root_load(const GroupRec* g, u32 ng) {
    root_room(ng + 1);
    for (u32 i = 0; i < ng; i++) { gb[i] = g[i].blk; gc[i] = g[i].cnt; gv[i] = g[i].vis; }
  }
  void root_store(GroupRec* g, u32 ng) const { for (u32 i = 0; i < ng; i++) g[i] = GroupRec{gb[i], gc[i], gv[i], 0}; }
  u32 root_blk(u32 g) const { return gb[g]; }
  u32 root_cnt(u32 g) const { return gc[g]; }
  u32 root_vis(u32 g) const { return gv[g]; }
  u32 root_find_blk(u32 ng, u32 blk) const { for (u32 i = 0; i < ng; i++) if (gb[i] == blk) return i; return INVALID; }
  void root_add_vis(u32 g, u32 d) { gv[g] += d; }
  void root_add_vis_blk(u32 ng, u32 blk, u32 d) { root_add_vis(root_find_blk(ng, blk), d); }
  void root_set(u32 g, u32 blk, u32 cnt, u32 vis) { gb[g] = blk; gc[g] = cnt; gv[g] = vis; }
  void root_set_cnt(u32 g, u32 cnt) { gc[g] = cnt; }
  void root_insert(u32 ng, u32 g, u32 blk, u32 cnt, u32 vis) {
    root_room(ng + 2);
    for (u32 i = ng; i > g; i--) { gb[i] = gb[i - 1]; gc[i] = gc[i - 1]; gv[i] = gv[i - 1]; }
    root_set(g, blk, cnt, vis);
  }
  bool root_find_pos(u32 ng, u32 pos, u32& g, u32& base) const {
    u32 acc = 0;
    for (u32 i = 0; i < ng; i++) {
      if (pos < acc + gv[i]) { g = i; base = acc; return true; }
      acc += gv[i];
    }
    return false;
  }
  u32 root_vis_before(u32 g) const { u32 t = 0; for (u32 i = 0; i < g; i++) t += gv[i]; return t; }
  u32 blk_vis_before(const u32* dv, u32 i) const { WCPU_MEM(dv, 4 * 64, 0); u32 t = 0; for (u32 k = 0; k < i; k++) t += dv[k]; return t; }
  u32 cache_vis_before(u32 idx) const { u32 t = 0; for (u32 i = 0; i < idx; i++) t += clen(c[i]); return t; }
  u32 peek_vis_before(const Span* p, u32 idx, i32& len_idx) const {
    WCPU_MEM(p, sizeof(Span) * L, 0);
    u32 t = 0;
    for (u32 i = 0; i < idx; i++) t += clen(p[i]);
    len_idx = p[idx].len;
    return t;
  }
  void st_span(Span* p, const Span& s) const { WCPU_MEM(p, sizeof(Span), 1); *p = s; }
  void st_probe(uint4* p, u32 a, u32 s, u32 ps, u32 dl) const { *p = make_uint4(a, s, ps, dl); }
  bool blk_find_pos(const u32* dv, const u32* dl, u32 cnt, u32 rem, u32& i, u32& before, u32& leaf) const {
    WCPU_MEM(dv, 4 * 64, 0); WCPU_MEM(dl, 4 * 64, 0);
    u32 acc = 0;
    for (u32 k = 0; k < cnt; k++) {
      if (rem < acc + dv[k]) { i = k; before = acc; leaf = dl[k]; return true; }
      acc += dv[k];
    }
    return false;
  }
  // (the GPU's row_ld returns a row one slot per lane; here a digest of the row, which blk_insert
  // checks against the row's current contents: the early-requested rows must still be current)
  static u32 row_digest(const u32* p) { u32 h = 2166136261u; for (u32 k = 0; k < 64; k++) h = (h ^ p[k]) * 16777619u; return h; }
  u32 row_ld(const u32* p) const { WCPU_MEM(p, 4 * 64, 0); return row_digest(p); }
  static void row_check(u32 ol, u32 ov, const u32* dl, const u32* dv) {
    if (ol != row_digest(dl) || ov != row_digest(dv)) {
      std::fprintf(stderr, "wave_cpu: directory row changed between row_ld and its use\n");
      std::abort();
    }
  }
  void blk_insert_at(u32 ol, u32 ov, u32* dl, u32* dv, u32 cnt, u32 i, u32 vis_i, u32 leaf, u32 vis, u32* sol, u32 blk) const {
    row_check(ol, ov, dl, dv);
    WCPU_MEM(dl, 4 * 64, 1); WCPU_MEM(dv, 4 * 64, 1);
    for (u32 k = i + 1; k <= cnt; k++) WCPU_MEM(sol + 2 * (k == i + 1 ? leaf : dl[k - 1]), 4, 1);
    dv[i] = vis_i;
    for (u32 k = cnt; k > i + 1; k--) { dl[k] = dl[k - 1]; dv[k] = dv[k - 1]; }
    dl[i + 1] = leaf;
    dv[i + 1] = vis;
    for (u32 k = i + 1; k <= cnt; k++) sol[2 * dl[k]] = (blk << 6) | k;  // ({slot, successor} entries)
  }
  u32 blk_split_r(u32 rl, u32 rv, const u32* dl, const u32* dv, u32* ndl, u32* ndv, u32* sol, u32 nb) const {
    row_check(rl, rv, dl, dv);
    WCPU_MEM(ndl, 4 * 32, 1); WCPU_MEM(ndv, 4 * 32, 1);
    for (u32 k = 32; k < 64; k++) WCPU_MEM(sol + 2 * dl[k], 4, 1);
    u32 t = 0;
    for (u32 k = 32; k < 64; k++) {
      ndl[k - 32] = dl[k];
      ndv[k - 32] = dv[k];
      sol[2 * dl[k]] = (nb << 6) | (k - 32);
      t += dv[k];
    }
    return t;
  }
  // (the GPU shifts the rows it holds; here the new block's rows as blk_split_r wrote them)
  void rows_upper(u32& rl, u32& rv, const u32* ndl, const u32* ndv) const { rl = row_digest(ndl); rv = row_digest(ndv); }
};

}  // namespace crdt
