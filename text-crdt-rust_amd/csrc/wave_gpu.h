// WaveGPU: the CDNA4 (gfx950, wave64) backend of replay_core.h.
//
// One wavefront owns one document.  Lane-parallel state held in VGPRs:
//   * the leaf cache: lane i < L holds entry i of the cached leaf (4 VGPRs: order, ol, orr, len);
//   * the directory root in LDS: group g = (block id, slot count, visible count), a per-launch
//     number of groups per wave (crdt_types.h ROOT_CAP_*).
// Cross-lane steps use DPP row_shr / row_bcast scans (GFX9 form) and ds_bpermute shuffles;
// uniform values are pulled to SGPRs with readfirstlane / readlane.
#pragma once
#include "crdt_types.h"

namespace crdt {

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }
// The lane id, re-derived at every use inside the replay loop (volatile: never hoisted).  A hoisted
// lane id lets the compiler hoist every lane-derived constant (l | 32, l - 1, l * 16 ...) out of
// the replay loop, where each then holds a VGPR for the whole kernel and the 8-waves/SIMD register
// budget spills them to scratch.  Two VALU per use instead.
__device__ __forceinline__ u32 lane_here() {
  u32 l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u32 rdlane(u32 x, u32 l) { return __builtin_amdgcn_readlane(x, l); }
// llvm.amdgcn.writelane (clang has no builtin for it): lane l of old := v (v, l uniform)
__device__ int crdt_writelane_i32(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ u32 wrlane(u32 old, u32 v, u32 l) { return (u32)crdt_writelane_i32((int)v, (int)l, (int)old); }
// (the builtin takes the i1 predicate directly: no v_cndmask + v_cmp round trip as __ballot has)
__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ u32 shfl(u32 v, u32 src) { return __builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v); }

// Inclusive wave64 prefix sum (LLVM AMDGPUAtomicOptimizer GFX9 sequence).
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ u32 wave_sum(u32 v) { return rdlane(wave_incl_scan(v), 63); }
// OR over the wave (the same DPP sequence with |)
__device__ __forceinline__ u32 wave_or(u32 v) {
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);
  return rdlane(v, 63);
}

template <int L>
struct WaveGPU {
  // The lane id, computed once; lane() hands out a copy at every use (volatile: never hoisted).  A
  // hoisted lane id lets the compiler hoist every lane-derived constant (l | 32, l - 1, l * 16 ...)
  // out of the replay loop, where each then holds a VGPR for the whole kernel and the
  // 8-waves/SIMD register budget spills them.  One v_mov per use (two v_mbcnt re-deriving it).
  u32 lid_ = lane_id();
  __device__ __forceinline__ u32 lane() const {
    u32 l;
    asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"(lid_));
    return l;
  }
  // ---------------------------------------------------------------- context registers
  // Per-document scalar state, one field per lane (replay_core.h slot enum), accessed at
  // compile-time lane numbers: v_readlane / v_writelane, no memory, no SGPR pressure.
  u32 x0 = 0, x1 = 0, x2 = 0;
  __device__ __forceinline__ u32 xg(u32 f) const {
    return f < 64 ? rdlane(x0, f) : f < 128 ? rdlane(x1, f - 64) : rdlane(x2, f - 128);
  }
  __device__ __forceinline__ void xs(u32 f, u32 v) {  // v_writelane (no lane mask to keep live)
    u32 sv = uni(v);  // folds away for values the compiler already knows are uniform
    if (f < 64) x0 = wrlane(x0, sv, f);
    else if (f < 128) x1 = wrlane(x1, sv, f - 64);
    else x2 = wrlane(x2, sv, f - 128);
  }
  // x0 (read-only in the replay) redefined opaquely once per replayed record: its reads are shared
  // within a record's code but not hoisted out of the replay loop into long-lived SGPRs
  __device__ __forceinline__ void x_pin() { asm volatile("" : "+v"(x0)); }
  // Element idx (x M) of a table, the byte offset computed in a VGPR: the compiler then addresses
  // it as table base (SGPR pair) + 32-bit VGPR offset -- one or two VALU ops -- instead of the
  // 64-bit SALU shift / add / add-with-carry chain a uniform index compiles to.  The replay is
  // bound by scalar issue, so address arithmetic belongs on the vector side.  (A document's
  // tables are < 4 GiB each: offsets fit 32 bits.)
  __device__ __forceinline__ static u32 vo(u32 x) {
    u32 r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
  }
  template <u32 M = 1, class T> __device__ __forceinline__ static T* at(T* base, u32 idx) {
    return (T*)((char*)base + (u64)(vo(idx) * (u32)(M * sizeof(T))));
  }
  // A pointer rebuilt from context lanes is a plain integer to the compiler; casting through
  // address space 1 lets it emit global_load/store (vmcnt only) instead of flat ops, which
  // also count in lgkmcnt and so would make every LDS wait drain all pending stores.
  template <class T> __device__ __forceinline__ static T* gptr(u64 v) {
    typedef __attribute__((address_space(1))) T GT;
    return (T*)(GT*)v;
  }
  // DocState <-> the first lanes of x1 (slot base 64): one lane-parallel load / store
  __device__ __forceinline__ void x_load_state(const DocState* p, u32 base) {
    (void)base;
    u32 l = lane();
    const u32* q = (const u32*)p;
    bool mine = l < (u32)(sizeof(DocState) / 4);
    u32 v = q[mine ? l : 0u];  // clamped address: unconditional load, no exec branch
    x1 = mine ? v : x1;
  }
  __device__ __forceinline__ void x_store_state(DocState* p, u32 base) const {
    (void)base;
    u32 l = lane();
    u32* q = (u32*)p;
    if (l < (u32)(sizeof(DocState) / 4)) q[l] = x1;
  }

  __device__ __forceinline__ static u64 clock() { return __builtin_amdgcn_s_memtime(); }

  // ---------------------------------------------------------------- leaf cache
  u32 eo = 0, el = 0, er = 0;
  i32 en = 0;
  // ---------------------------------------------------------------- root level (LDS)
  // This wave's slice of the kernel's LDS: blk[rcap], cnt[rcap], vis[rcap] (structure of
  // arrays: lane-parallel sweeps are bank-conflict free).  Kept out of VGPRs so that no register
  // is ever indexed by a run-time group number.
  typedef __attribute__((address_space(3))) u32 lds_u32;  // ds_read/ds_write, never flat
  lds_u32* rt = nullptr;
  u32 rcap = 0;

  // ---- scalar memory helpers (every lane touches the same address: uniform results, and a
  //      store is then visible to every lane's later loads by per-thread program order)
  __device__ __forceinline__ u32 ld(const u32* p) const { return uni(*(const u32*)p); }
  // a load whose wait is deferred to the first uni_() of its value (overlaps later loads)
  __device__ __forceinline__ u32 ld_raw(const u32* p) const { return *(const u32*)p; }
  __device__ __forceinline__ static u32 uni_(u32 x) { return uni(x); }
  __device__ __forceinline__ void st(u32* p, u32 v) const { *(u32*)p = v; }
  __device__ __forceinline__ void st(i32* p, i32 v) const { *(i32*)p = v; }
  template <class T> __device__ __forceinline__ T ldT(const T* p) const {
    T t;
    const u32* s = (const u32*)p;
    u32* o = (u32*)&t;
#pragma unroll
    for (u32 k = 0; k < sizeof(T) / 4; k++) o[k] = uni(s[k]);
    return t;
  }
  template <class T> __device__ __forceinline__ void stT(T* p, const T& v) const {
    u32* s = (u32*)p;
    const u32* o = (const u32*)&v;
#pragma unroll
    for (u32 k = 0; k < sizeof(T) / 4; k++) s[k] = o[k];
  }
  __device__ __forceinline__ AgentRec ld_agent(const AgentRec* p) const { return ldT(p); }
  __device__ __forceinline__ ARun ld_arun(const ARun* p) const { return ldT(p); }
  __device__ __forceinline__ void st_arun(ARun* p, const ARun& v) const { stT(p, v); }
  __device__ __forceinline__ CwoRun ld_cwo(const CwoRun* p) const { return ldT(p); }
  __device__ __forceinline__ void st_cwo(CwoRun* p, const CwoRun& v) const { stT(p, v); }
  __device__ __forceinline__ DelRun ld_del(const DelRun* p) const { return ldT(p); }
  __device__ __forceinline__ void st_del(DelRun* p, const DelRun& v) const { stT(p, v); }
  __device__ __forceinline__ DDRun ld_dd(const DDRun* p) const { return ldT(p); }
  __device__ __forceinline__ void st_dd(DDRun* p, const DDRun& v) const { stT(p, v); }
  __device__ __forceinline__ TxnRec ld_txn(const TxnRec* p) const { return ldT(p); }
  __device__ __forceinline__ void st_txn(TxnRec* p, const TxnRec& v) const { stT(p, v); }
  __device__ __forceinline__ Rec ld_rec(const Rec* p) const {
    uint4 v = *(const uint4*)p;
    return Rec{uni(v.x), uni(v.y), uni(v.z), uni(v.w)};
  }
  __device__ __forceinline__ void st_state(DocState* p, const DocState& s) const { stT(p, s); }
  __device__ __forceinline__ DocState ld_state(const DocState* p) const { return ldT(p); }
  __device__ __forceinline__ DocSeg ld_seg(const DocSeg* p) const { return ldT(p); }

  // lane-parallel fill of n u32
  __device__ __forceinline__ void fill(u32* p, u32 n, u32 v) const {
    if (n == 1) { *p = v; return; }  // the common single-item case: one coalesced store
    u32 l = lane();
    if (n <= 64u) {  // one store, lanes >= n repeating item n - 1 (same value): no exec mask
      u32 m = n - 1u;
      p[l < m ? l : m] = v;
      return;
    }
    for (u32 k = l; k < n; k += 64) p[k] = v;
  }
  __device__ __forceinline__ void zero_leaf(Span* p, u32 n) const {
    u32 l = lane();
    if (l < n) *(uint4*)(p + l) = make_uint4(0, 0, 0, 0);
  }

  // 64-ary search over sorted runs: index k with key(k) <= needle < key(k)+len(k), or -1.
  template <class T>
  __device__ __forceinline__ i32 search(const T* base, u32 n, u32 needle) const {
    if (n == 0) return -1;
    u32 lo = 0, hi = n;  // answer (last key <= needle) in [lo, hi)
    u32 l = lane();
    while (hi - lo > 64) {
      u32 step = (hi - lo + 63) / 64;
      u32 idx = lo + l * step;
      u32 key = *(const u32*)&base[idx < hi ? idx : hi - 1];  // key is the first field
      bool ok = idx < hi && key <= needle;
      u64 m = ballot(ok);
      if (m == 0) return -1;
      u32 t = 63 - __builtin_clzll(m);
      lo = lo + t * step;
      u32 nh = lo + step;
      hi = nh < hi ? nh : hi;
    }
    u32 idx = lo + l;
    u32 key0 = *(const u32*)&base[idx < hi ? idx : hi - 1];
    bool ok = idx < hi && key0 <= needle;
    u64 m = ballot(ok);
    if (m == 0) return -1;
    u32 k = lo + (63 - __builtin_clzll(m));
    T r = ldT(base + k);
    u32 key = ((const u32*)&r)[0];
    u32 len = rlen(r);
    return (needle < key + len) ? (i32)k : -1;
  }
  __device__ __forceinline__ static u32 rlen(const ARun& r) { return r.len; }
  __device__ __forceinline__ static u32 rlen(const CwoRun& r) { return r.len; }
  __device__ __forceinline__ static u32 rlen(const DDRun& r) { return r.len; }
  __device__ __forceinline__ static u32 rlen(const TxnRec& r) { return r.len; }
  __device__ __forceinline__ i32 search_arun(const ARun* b, u32 n, u32 x) const { return search(b, n, x); }
  __device__ __forceinline__ i32 search_cwo(const CwoRun* b, u32 n, u32 x) const { return search(b, n, x); }
  // ---- double-delete blocks (replay_core.h dd_*)
  __device__ __forceinline__ DDBlk ld_ddblk(const DDBlk* p) const { return ldT(p); }
  __device__ __forceinline__ void st_ddblk(DDBlk* p, const DDBlk& v) const { stT(p, v); }
  // last block with first key <= x, or -1 (64-ary search, as `search`)
  __device__ __forceinline__ i32 search_first(const DDBlk* b, u32 n, u32 x) const {
    u32 lo = 0, hi = n;
    u32 l = lane();
    while (hi - lo > 64) {
      u32 step = (hi - lo + 63) / 64;
      u32 idx = lo + l * step;
      u32 key = b[idx < hi ? idx : hi - 1].first;
      u64 m = ballot(idx < hi && key <= x);
      if (m == 0) return -1;
      lo = lo + (63 - __builtin_clzll(m)) * step;
      u32 nh = lo + step;
      hi = nh < hi ? nh : hi;
    }
    u32 idx = lo + l;
    u32 key = b[idx < hi ? idx : hi - 1].first;
    u64 m = ballot(idx < hi && key <= x);
    return m ? (i32)(lo + (63 - __builtin_clzll(m))) : -1;
  }
  // entries of one block (cnt >= 1) with key <= x
  __device__ __forceinline__ u32 dd_count_le(const DDRun* blk, u32 cnt, u32 x) const {
    u32 l = lane();
    u32 key = blk[l < cnt ? l : 0u].key;
    return (u32)__popcll(ballot(l < cnt && key <= x));
  }
  // entries [32, 64) of a full block move to [0, 32) of dst; returns dst's first key
  __device__ __forceinline__ u32 dd_split(const DDRun* src, DDRun* dst) const {
    u32 l = lane();
    const u32* s = (const u32*)(src + (l | 32u));
    u32 a = s[0], b = s[1], c = s[2];
    if (l >= 32u) {
      u32* d = (u32*)(dst + (l - 32u));
      d[0] = a; d[1] = b; d[2] = c;
    }
    return rdlane(a, 32);
  }
  // Vec::insert at i of a block with cnt < 64 entries: [i, cnt) move up one, r goes to i
  __device__ __forceinline__ void dd_block_insert(DDRun* blk, u32 cnt, u32 i, const DDRun& r) const {
    u32 l = lane();
    const u32* s = (const u32*)(blk + (l ? l - 1u : 0u));
    u32 a = s[0], b = s[1], c = s[2];
    bool me = l == i;
    if (l >= i && l <= cnt) {
      u32* d = (u32*)(blk + l);
      d[0] = me ? r.key : a; d[1] = me ? r.len : b; d[2] = me ? r.excess : c;
    }
  }
  // directory insert at `at` of n blocks: [at, n) move up one (64-block chunks, top down: each
  // chunk's loads complete before its stores, and no later chunk reads what it stores)
  __device__ __forceinline__ void ddb_insert(DDBlk* b, u32 n, u32 at, const DDBlk& v) const {
    u32 l = lane();
    for (i32 r = (i32)(n & ~63u); r >= (i32)(at & ~63u); r -= 64) {
      u32 i = (u32)r + l;
      uint4 x = *(const uint4*)(b + (i > 0u && i <= n ? i - 1u : 0u));
      if (i > at && i <= n) *(uint4*)(b + i) = x;
    }
    stT(b + at, v);
  }
  __device__ __forceinline__ i32 search_txn(const TxnRec* b, u32 n, u32 x) const { return search(b, n, x); }

  // ---------------------------------------------------------------- leaf cache
  __device__ __forceinline__ u32 cache_load(const Span* p) {
    u32 l = lane();
    bool in = l < (u32)L;
    uint4 v = *(const uint4*)(p + (l & (u32)(L - 1)));  // lanes >= L re-read a valid entry
    eo = in ? v.x : 0u; el = in ? v.y : 0u; er = in ? v.z : 0u; en = in ? (i32)v.w : 0;
    return __popcll(ballot(en != 0));
  }
  __device__ __forceinline__ void cache_store(Span* p) const {
    u32 l = lane();
    if (l < (u32)L) *(uint4*)(p + l) = make_uint4(eo, el, er, (u32)en);
  }
  __device__ __forceinline__ Span cget(u32 i) const {
    return Span{rdlane(eo, i), rdlane(el, i), rdlane(er, i), (i32)rdlane((u32)en, i)};
  }
  __device__ __forceinline__ u32 cget_order(u32 i) const { return rdlane(eo, i); }
  __device__ __forceinline__ i32 cget_len(u32 i) const { return (i32)rdlane((u32)en, i); }
  // entry i := s (i and s uniform): one v_writelane per field (the compiler sets M0 for a run-time
  // lane select), instead of a lane-compare mask, an SGPR -> VGPR copy and a v_cndmask per field
  __device__ __forceinline__ void cset(u32 i, const Span& s) {
    eo = wrlane(eo, s.order, i);
    el = wrlane(el, s.ol, i);
    er = wrlane(er, s.orr, i);
    en = (i32)wrlane((u32)en, (u32)s.len, i);
  }
  // entries [a, b) := f(lane), lane-parallel (f computes each lane's entry in VALU)
  template <class F> __device__ __forceinline__ void cset_lanes(u32 a, u32 b, F f) {
    u32 l = lane();
    Span s = f(l);
    bool in = l >= a && l < b;
    eo = in ? s.order : eo;
    el = in ? s.ol : el;
    er = in ? s.orr : er;
    en = in ? s.len : en;
  }
  // the visible entries among lanes [a, b), as a lane mask
  __device__ __forceinline__ u64 vis_lanes(u32 a, u32 b) const { u32 l = lane(); return ballot(l >= a && l < b && en > 0); }
  // deactivate (negate) the visible entries among lanes [a, b)
  __device__ __forceinline__ void negate_visible(u32 a, u32 b) {
    u32 l = lane();
    en = (l >= a && l < b && en > 0) ? -en : en;
  }
  // lanes [a, b) as a mask, and the lowest lane of a mask (wave-uniform)
  __device__ __forceinline__ u64 lanes_in(u32 a, u32 b) const { u32 l = lane(); return ballot(l >= a && l < b); }
  __device__ __forceinline__ static u32 first_lane(u64 m) { return (u32)__builtin_ctzll(m); }
  // leaf.rs:41-57 find on a leaf that is NOT the cached one (peek: no cache change)
  __device__ __forceinline__ i32 peek_find_order(const Span* p, u32 order, u32& start) const {
    u32 l = lane();
    uint4 v = *(const uint4*)(p + (l & (u32)(L - 1)));
    u32 o = v.x;
    i32 n = (i32)v.w;
    u32 sl = (u32)(n < 0 ? -n : n);
    // one unsigned compare: order < o wraps to >= 2^31 > sl (orders < 2^31); empty entries have
    // sl = 0; lanes >= L repeat lanes l & (L - 1), so the lowest match is < L
    u64 m = ballot(order - o < sl);
    if (!m) return -1;
    u32 k = (u32)__builtin_ctzll(m);
    start = rdlane(o, k);
    return (i32)k;
  }
  __device__ __forceinline__ u32 clen_l() const { return en > 0 ? (u32)en : 0u; }
  __device__ __forceinline__ u32 cache_vis_from(u32 a) const {  // visible items in lanes >= a
    return wave_sum(lane() >= a ? clen_l() : 0u);
  }
  // leaf.rs:61-84 find_offset (stick_end = false) over clen
  __device__ __forceinline__ bool cfind_content(u32 n, u32 rem, u32& idx, u32& off) const {
    u32 l = lane();
    // lanes >= n are empty (clen 0: every cache update keeps the tail clear), so they add nothing
    // and their prefix is the total: counted only when rem >= total, i.e. when k >= n anyway
    (void)l;
    u32 x = clen_l();
    u32 incl = wave_incl_scan(x);
    u32 k = __popcll(ballot(incl <= rem));
    if (k < n) {
      idx = k;
      off = rem - (rdlane(incl, k) - rdlane(x, k));
      return true;
    }
    u32 total = rdlane(incl, 63);
    if (rem == total) { idx = n; off = 0; return true; }
    return false;
  }
  // leaf.rs:41-57 find
  __device__ __forceinline__ i32 cfind_order(u32 n, u32 order) const {
    u32 l = lane();
    u32 sl = (u32)(en < 0 ? -en : en);
    // one unsigned compare (order < eo wraps past sl; lanes >= n are empty: sl = 0)
    (void)l; (void)n;
    u64 m = ballot(order - eo < sl);
    return m ? (i32)(__builtin_ctzll(m)) : -1;
  }
  // the split-off entries [idx, n) of the cached leaf, after `padding` empty slots: written to
  // the new leaf and kept in registers (cache_from_moved) for a cursor that follows them
  u32 mo = 0, ml = 0, mr = 0, mn = 0;
  __device__ __forceinline__ void cache_write_moved(Span* dst, u32 idx, u32 n, u32 padding) {
    u32 l = lane();
    u32 src = l + idx - padding;  // valid only when l >= padding
    u32 o = shfl(eo, src), a = shfl(el, src), b = shfl(er, src), c = shfl((u32)en, src);
    bool take = l >= padding && src < n && l < (u32)L;
    mo = take ? o : 0u; ml = take ? a : 0u; mr = take ? b : 0u; mn = take ? c : 0u;
    if (l < (u32)L) *(uint4*)(dst + l) = make_uint4(mo, ml, mr, mn);
  }
  __device__ __forceinline__ void cache_from_moved() { eo = mo; el = ml; er = mr; en = (i32)mn; }
  // lof[order + t] = v for every item of the entries in lanes [a, b): 64 items per step, each
  // lane finding its entry by a 6-step search over the entries' length prefix
  __device__ __forceinline__ void fill_runs(u32* base, u32 a, u32 b, u32 v) const {
    u32 l = lane();
    u32 ln = l >= a && l < b ? (u32)(en < 0 ? -en : en) : 0u;
    u32 Pi = wave_incl_scan(ln);
    u32 T = rdlane(Pi, 63);
    for (u32 t = 0; t < T; t += 64) {
      u32 j = t + l;
      u32 m = 0;
      for (u32 step = 32; step; step >>= 1)
        if (shfl(Pi, m + step - 1u) <= j) m += step;
      u32 pm = shfl(Pi, m), lm = shfl(ln, m), om = shfl(eo, m);
      if (j < T) base[om + (j - (pm - lm))] = v;
    }
  }
  __device__ __forceinline__ void cache_clear(u32 a, u32 b) {
    u32 l = lane();
    bool z = l >= a && l < b;
    eo = z ? 0u : eo;
    el = z ? 0u : el;
    er = z ? 0u : er;
    en = z ? 0 : en;
  }
  // entries [idx, n) move to [idx+k, n+k); the vacated slots [idx, idx+k) become empty.  Lanes
  // >= idx take lane l - k, the gap's lanes take lane 63 (always empty: L <= 32), and lanes
  // >= n + k take an empty lane >= n: no lane-range masks to combine.
  __device__ __forceinline__ void cache_shift_right(u32 idx, u32 n, u32 k) {
    static_assert(L <= 32, "lane 63 of the cache is always empty");
    u32 l = lane();
    (void)n;
    u32 src = l >= idx + k ? l - k : 63u;
    u32 o = shfl(eo, src), a = shfl(el, src), b = shfl(er, src), c = shfl((u32)en, src);
    bool up = l >= idx;
    eo = up ? o : eo;
    el = up ? a : el;
    er = up ? b : er;
    en = up ? (i32)c : en;
  }

  // ---------------------------------------------------------------- record window (64 + 64 ahead)
  u32 rx = 0, ry = 0, rz = 0, rw = 0;  // window: lane k = record base + k
  u32 qx = 0, qy = 0, qz = 0, qw = 0;  // next 64 records, loaded ahead
  __device__ __forceinline__ uint4 rec_lane_load(const Rec* p, u32 n) const {  // n >= 1
    u32 l = lane();
    u32 m = n - 1u;
    return *(const uint4*)(p + (l < m ? l : m));
  }
  __device__ __forceinline__ void rec_load2(const Rec* p, u32 n, u32 n_ahead) {
    uint4 v = rec_lane_load(p, n);
    rx = v.x; ry = v.y; rz = v.z; rw = v.w;
    if (n_ahead) {
      uint4 q = rec_lane_load(p + 64, n_ahead);
      qx = q.x; qy = q.y; qz = q.z; qw = q.w;
    }
  }
  // window += d (d <= 64): lanes take records from the window or the block ahead; then load the
  // block after the new window (n_ahead records at p_ahead) ahead
  __device__ __forceinline__ void rec_slide(u32 d, const Rec* p_ahead, u32 n_ahead) {
    if (d >= 64u) {
      rx = qx; ry = qy; rz = qz; rw = qw;
      d -= 64u;
    }
    if (d) {
      u32 l = lane();
      u32 src = (l + d) & 63u;
      bool own = l + d < 64u;
      u32 ax = shfl(rx, src), ay = shfl(ry, src), az = shfl(rz, src), aw = shfl(rw, src);
      u32 bx = shfl(qx, src), by = shfl(qy, src), bz = shfl(qz, src), bw = shfl(qw, src);
      rx = own ? ax : bx; ry = own ? ay : by; rz = own ? az : bz; rw = own ? aw : bw;
    }
    if (n_ahead) {
      uint4 q = rec_lane_load(p_ahead, n_ahead);
      qx = q.x; qy = q.y; qz = q.z; qw = q.w;
    }
  }
  __device__ __forceinline__ Rec rec_get(u32 k) const {
    return Rec{rdlane(rx, k), rdlane(ry, k), rdlane(rz, k), rdlane(rw, k)};
  }
  // The generator draws of ops [base, base + 64) into the window registers (lane k: hi, lo, r2 of
  // op base + k), computed lane-parallel on the vector unit; read back with rec_get.  (A GEN record
  // uses no record window: the replay invalidates the window while it runs one.)
  __device__ __forceinline__ void gen_draws(u32 seed, u32 base) {
    GenDraw d = gen_draw(seed, base + lane());
    rx = d.hi; ry = d.lo; rz = d.r2;
  }
  // Typing-run scan (replay_core.h fast_typing): lane k checks record k of the prefetch block
  // against "txn continues the typing txn before it" -- remote: RTXN{1 op, 1 parent}, RINS with
  // origin_left = (agent, seq-1) and the same origin_right, RPARENT (agent, seq-1), seq = previous
  // seq + previous length; local: LTXN{1 op}, LOP insert at the previous pos + previous length.
  // The txn at b0 was checked by the caller.  Returns the run length in txns (>= 1) and the
  // total inserted length.  nv = valid records in the block.
  // compact: one record per txn (crdt_types.h RC / LC), lane k checks record k against record k-1.
  __device__ __forceinline__ u32 typing_scan_r(u32 X, u32 Y, u32 Z, u32 Q, u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1, u32 ow3,
                                             u32& total) const {
    u32 l = lane();
    if (compact) {
      u32 p0 = shfl(X, l - 1u), p1 = shfl(Y, l - 1u), p3 = shfl(Q, l - 1u);
      bool ok;
      u32 hl;
      if (remote) {
        hl = (X >> 16) & 0x7FFu;
        // origin_right's agent (ROOT or the author) follows from Q == ow3: a uniform check
        u32 ra = ow3 == 0xFFFFFFFFu ? 0xFFFFu : agent;
        u32 ubad = (agent | (ra << 16)) != ow1 ? 1u : 0u;
        // the equality terms folded into one word (one compare instead of a mask AND per term)
        u32 d = ((X & RC_HDR_MASK) ^ ((REC_RC << 28) | agent)) | (Y ^ (p1 + ((p0 >> 16) & 0x7FFu))) |
                (Z ^ (Y - 1u)) | (Q ^ ow3) | ubad;
        ok = d == 0u && hl != 0u;
      } else {
        hl = Q;
        ok = X == ((REC_LC << 28) | agent) && Z == 0u && Q - 1u < 0xFFFFu && Y == p1 + p3;
      }
      // lanes above b0 by a scalar mask (b0 < 64), the window end folded into the lane test, the
      // run range as one unsigned compare: no lane-mask ANDs on the scalar unit
      u64 stop = ballot(!ok || l >= nv) & (~1ull << b0);
      u32 f = stop ? (u32)__builtin_ctzll(stop) : 64u;
      total = wave_sum(l - b0 < f - b0 ? hl : 0u);
      return f - b0;
    }
    u32 rel = l - b0;  // wraps below b0: those lanes are masked
    u32 per = remote ? 3u : 2u;
    u32 t = remote ? (rel * 43u) >> 7 : rel >> 1;  // rel / 3 exactly for rel < 64
    u32 r = rel - t * per;
    bool ok;
    if (remote) {
      u32 src = r == 0u ? l - 3u : (r == 1u ? l - 1u : l - 2u);  // previous header / own header
      u32 hs = shfl(Z, src), hl = shfl(Q, src);
      bool okh = X == ((REC_RTXN << 28) | 1u) && Y == (agent | (1u << 16)) && Z == hs + hl && Q - 1u < 0xFFFFu;
      bool oko = (X >> 28) == REC_RINS && (X & 0x0FFFFFFFu) == hl && Y == ow1 && Q == ow3 && Z == hs - 1u;
      bool okp = X == (REC_RPARENT << 28) && Y == agent && Z == hs - 1u;
      ok = r == 0u ? okh : (r == 1u ? oko : okp);
    } else {
      u32 hl = shfl(Q, l - 1u), ps = shfl(Y, l - 2u), pl = shfl(Q, l - 2u);
      bool okh = X == ((REC_LTXN << 28) | 1u) && Y == agent && Z == 0u && Q - 1u < 0xFFFFu;
      bool oko = X == (REC_LOP << 28) && Z == 0u && Q == hl && Y == ps + pl;
      ok = r == 0u ? okh : oko;
    }
    u64 stop = ballot(l >= b0 + per && (!ok || l >= nv));
    u32 f = stop ? (u32)__builtin_ctzll(stop) : 64u;
    u32 n = remote ? ((f - b0) * 43u) >> 7 : (f - b0) >> 1;
    total = wave_sum(l >= b0 && r == 0u && t < n ? Q : 0u);
    return n;
  }

  // Delete-run scan (replay_core.h fast_deletes): lane k checks record k against "one-item delete
  // txn continuing the previous one" -- remote: RTXN{1 op, 1 parent} of length 1, seq = previous
  // seq + 1, RDEL of 1 item of `agent` at the previous target seq + delta, RPARENT (agent, seq-1);
  // local: LTXN{1 op} deleting 1 item at the previous pos + delta.  Returns the run length in
  // txns (>= 1; the txn at b0 was checked by the caller).
  __device__ __forceinline__ u32 delete_scan_r(u32 X, u32 Y, u32 Z, u32 Q, u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) const {
    u32 l = lane();
    if (compact) {  // one record per txn: lane k against record k-1
      u32 p1 = shfl(Y, l - 1u), p2 = shfl(Z, l - 1u);
      // the equality terms folded into one word (one compare instead of a mask AND per term)
      u32 d = remote ? ((X ^ ((REC_RC << 28) | (1u << 27) | (1u << 16) | agent)) | (Y ^ (p1 + 1u)) | (Z ^ (p2 + delta)))
                     : ((X ^ ((REC_LC << 28) | agent)) | (Z ^ 1u) | Q | (Y ^ (p1 + delta)));
      bool ok = d == 0u;
      u64 stop = ballot(!ok || l >= nv) & (~1ull << b0);
      u32 f = stop ? (u32)__builtin_ctzll(stop) : 64u;
      return f - b0;
    }
    u32 rel = l - b0;
    u32 per = remote ? 3u : 2u;
    u32 t = remote ? (rel * 43u) >> 7 : rel >> 1;
    u32 r = rel - t * per;
    bool ok;
    if (remote) {
      u32 ps = shfl(Z, r == 2u ? l - 2u : l - 3u);  // previous header / previous op / own header
      bool okh = X == ((REC_RTXN << 28) | 1u) && Y == (agent | (1u << 16)) && Z == ps + 1u && Q == 1u;
      bool oko = X == ((REC_RDEL << 28) | 1u) && Y == agent && Z == ps + delta;
      bool okp = X == (REC_RPARENT << 28) && Y == agent && Z == ps - 1u;
      ok = r == 0u ? okh : (r == 1u ? oko : okp);
    } else {
      u32 pp = shfl(Y, l - 2u);  // previous op's pos
      bool okh = X == ((REC_LTXN << 28) | 1u) && Y == agent && Z == 1u && Q == 1u;
      bool oko = X == (REC_LOP << 28) && Z == 1u && Q == 0u && Y == pp + delta;
      ok = r == 0u ? okh : oko;
    }
    u64 stop = ballot(l >= b0 + per && (!ok || l >= nv));
    u32 f = stop ? (u32)__builtin_ctzll(stop) : 64u;
    return remote ? ((f - b0) * 43u) >> 7 : (f - b0) >> 1;
  }
  // The scans over the record window, and over the 64 records at p (loaded here, waited for; the
  // window does not move: only Replayer::rec moves it).  len0: the length of the txn at p.
  __device__ __forceinline__ u32 typing_scan(u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1, u32 ow3,
                                             u32& total) const {
    return typing_scan_r(rx, ry, rz, rw, b0, nv, remote, compact, agent, ow1, ow3, total);
  }
  __device__ __forceinline__ u32 typing_scan_at(const Rec* p, u32 nv, u32 remote, u32 compact, u32 agent, u32 ow1,
                                                u32 ow3, u32& total, u32& len0) const {
    uint4 v = rec_lane_load(p, nv);
    len0 = (compact & remote) ? (rdlane(v.x, 0) >> 16) & 0x7FFu : rdlane(v.w, 0);
    return typing_scan_r(v.x, v.y, v.z, v.w, 0u, nv, remote, compact, agent, ow1, ow3, total);
  }
  __device__ __forceinline__ u32 delete_scan(u32 b0, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) const {
    return delete_scan_r(rx, ry, rz, rw, b0, nv, remote, compact, agent, delta);
  }
  __device__ __forceinline__ u32 delete_scan_at(const Rec* p, u32 nv, u32 remote, u32 compact, u32 agent, u32 delta) const {
    uint4 v = rec_lane_load(p, nv);
    return delete_scan_r(v.x, v.y, v.z, v.w, 0u, nv, remote, compact, agent, delta);
  }
  // runs {key0 + j, t0 - j, 1} for j < cnt (backspaced deletes), lane-parallel
  __device__ __forceinline__ void st_del_run(DelRun* p, u32 cnt, u32 key0, u32 t0) const {
    for (u32 j = lane(); j < cnt; j += 64) {
      u32* q = (u32*)(p + j);
      q[0] = key0 + j;
      q[1] = t0 - j;
      q[2] = 1u;
    }
  }

  // ---------------------------------------------------------------- directory root (LDS)
  // Group g of the root: rblk()[g], rcnt()[g], rvis()[g]; rcap groups per array (a multiple of
  // 64, chosen per launch).  Sweeps go 64 groups at a time, one group per lane.
  __device__ __forceinline__ lds_u32* rblk() const { return rt; }
  __device__ __forceinline__ lds_u32* rcnt() const { return rt + rcap; }
  __device__ __forceinline__ lds_u32* rvis() const { return rt + 2 * rcap; }
  // Groups [ng, rcap) hold block id INVALID (no block has that id), so root_find_blk needs no
  // bounds test; the root only grows while a wave runs (root_insert writes at most up to ng).
  __device__ __forceinline__ void root_clear_from(u32 ng) {
    for (u32 i = lane(); i < rcap; i += 64)
      if (i >= ng) rblk()[i] = INVALID;
  }
  __device__ __forceinline__ void root_init(u32 blk, u32 cnt, u32 vis) {
    root_clear_from(1u);
    rblk()[0] = blk;  // every lane stores the same value: no branch
    rcnt()[0] = cnt;
    rvis()[0] = vis;
  }
  __device__ __forceinline__ void root_load(const GroupRec* g, u32 ng) {
    root_clear_from(ng);
    for (u32 i = lane(); i < ng; i += 64) {
      uint4 x = *(const uint4*)(g + i);
      rblk()[i] = x.x;
      rcnt()[i] = x.y;
      rvis()[i] = x.z;
    }
  }
  __device__ __forceinline__ void root_store(GroupRec* g, u32 ng) const {
    for (u32 i = lane(); i < ng; i += 64) *(uint4*)(g + i) = make_uint4(rblk()[i], rcnt()[i], rvis()[i], 0);
  }
  __device__ __forceinline__ u32 root_blk(u32 g) const { return uni(rblk()[g]); }
  __device__ __forceinline__ u32 root_cnt(u32 g) const { return uni(rcnt()[g]); }
  __device__ __forceinline__ u32 root_vis(u32 g) const { return uni(rvis()[g]); }
  __device__ __forceinline__ u32 root_find_blk(u32 ng, u32 blk) const {
    u32 l = lane();
    for (u32 r = 0; r < ng; r += 64) {
      u32 i = r + l;
      u32 b = rblk()[i];  // i < rcap (a multiple of 64): always inside this wave's LDS slice
      u64 m = ballot(b == blk);  // (groups >= ng hold INVALID: root_clear_from)
      if (m) return r + (u32)__builtin_ctzll(m);
    }
    return INVALID;
  }
  __device__ __forceinline__ void root_add_vis(u32 g, u32 delta) {
    u32 v = uni(rvis()[g]) + delta;
    rvis()[g] = v;
  }
  __device__ __forceinline__ void root_set(u32 g, u32 blk, u32 cnt, u32 vis) {
    rblk()[g] = blk;
    rcnt()[g] = cnt;
    rvis()[g] = vis;
  }
  // insert a group at index g, shifting [g, ng) up by one: 64-group chunks from the top down, each
  // read completely before it is written (a chunk's lane 0 reads the top of the chunk below,
  // which is written only afterwards)
  __device__ __forceinline__ void root_insert(u32 ng, u32 g, u32 blk, u32 cnt, u32 vis) {
    u32 l = lane();
    for (i32 r = (i32)(ng & ~63u); r >= (i32)(g & ~63u); r -= 64) {
      u32 i = (u32)r + l;
      u32 jj = i > 0u ? i - 1u : 0u;
      u32 b = rblk()[jj], c = rcnt()[jj], v = rvis()[jj];
      __builtin_amdgcn_wave_barrier();
      if (i > g && i <= ng) { rblk()[i] = b; rcnt()[i] = c; rvis()[i] = v; }
      __builtin_amdgcn_wave_barrier();
    }
    root_set(g, blk, cnt, vis);
  }
  // first group whose cumulative visible count exceeds pos
  __device__ __forceinline__ bool root_find_pos(u32 ng, u32 pos, u32& g, u32& base) const {
    u32 l = lane();
    u32 carry = 0;
    for (u32 r = 0; r < ng; r += 64) {
      u32 i = r + l;
      bool valid = i < ng;
      u32 xv = rvis()[i];
      u32 x = valid ? xv : 0u;
      u32 incl = wave_incl_scan(x) + carry;
      u32 nvalid = ng - r < 64 ? ng - r : 64;
      u32 k = __popcll(ballot(incl <= pos));  // (invalid lanes add 0: counted only if k >= nvalid)
      if (k < nvalid) {
        g = r + k;
        base = rdlane(incl, k) - rdlane(x, k);
        return true;
      }
      carry = rdlane(incl, 63);
    }
    return false;
  }

  // visible items in the groups before g (probe: Cursor::count_pos)
  __device__ __forceinline__ u32 root_vis_before(u32 g) const {
    u32 l = lane(), t = 0;
    for (u32 r = 0; r < g; r += 64) t += wave_sum(r + l < g ? (u32)rvis()[r + l] : 0u);
    return t;
  }

  // ---------------------------------------------------------------- directory blocks (HBM)
  // visible items in the slots before i of a block row
  __device__ __forceinline__ u32 blk_vis_before(const u32* dv, u32 i) const {
    u32 l = lane();
    u32 x = dv[l];  // 64-slot rows: always in bounds
    return wave_sum(l < i ? x : 0u);
  }
  // visible items before entry idx of the cached leaf / of another leaf (+ that entry's length)
  __device__ __forceinline__ u32 cache_vis_before(u32 idx) const { return wave_sum(lane() < idx ? clen_l() : 0u); }
  __device__ __forceinline__ u32 peek_vis_before(const Span* p, u32 idx, i32& len_idx) const {
    u32 l = lane();
    i32 n = (i32)p[l & (u32)(L - 1)].len;
    len_idx = (i32)rdlane((u32)n, idx);
    return wave_sum(l < idx && l < (u32)L && n > 0 ? (u32)n : 0u);
  }
  __device__ __forceinline__ void st_span(Span* p, const Span& s) const {  // every lane stores the same entry
    *(uint4*)p = make_uint4(s.order, s.ol, s.orr, (u32)s.len);
  }
  __device__ __forceinline__ void st_probe(uint4* p, u32 a, u32 s, u32 ps, u32 dl) const {
    *p = make_uint4(a, s, ps, dl);  // every lane stores the same values
  }
  // slot of a block whose cumulative visible count first exceeds rem (+ its leaf id; both block
  // rows are loaded together so the descent costs one HBM round trip)
  __device__ __forceinline__ bool blk_find_pos(const u32* dv, const u32* dl, u32 cnt, u32 rem, u32& i, u32& before, u32& leaf) const {
    u32 l = lane();
    u32 xv = dv[l], lf = dl[l];  // block rows are 64 slots wide: always in bounds
    u32 x = l < cnt ? xv : 0u;
    u32 incl = wave_incl_scan(x);
    u32 k = __popcll(ballot(incl <= rem));  // (lanes >= cnt add 0: counted only if k >= cnt)
    if (k >= cnt) return false;
    i = k;
    before = rdlane(incl, k) - rdlane(x, k);
    leaf = rdlane(lf, k);
    return true;
  }
  __device__ __forceinline__ void blk_insert(u32* dl, u32* dv, u32 cnt, u32 i, u32 leaf, u32 vis, u32* sol, u32 blk) const {
    u32 l = lane();
    u32 ol = *(u32*)(dl + l);
    u32 ov = *(u32*)(dv + l);
    u32 sl = shfl(ol, l - 1), sv = shfl(ov, l - 1);
    u32 nlf = l < i ? ol : (l == i ? leaf : sl);
    u32 nvs = l < i ? ov : (l == i ? vis : sv);
    if (l >= i && l <= cnt) {
      *(u32*)(dl + l) = nlf;
      *(u32*)(dv + l) = nvs;
      *(u32*)(sol + nlf) = (blk << 6) | l;
    }
  }
  __device__ __forceinline__ u32 blk_split(const u32* dl, const u32* dv, u32* ndl, u32* ndv, u32* sol, u32 nb) const {
    u32 l = lane();
    u32 lf = 0, v = 0;
    if (l >= 32) {
      lf = *(const u32*)(dl + l);
      v = *(const u32*)(dv + l);
      *(u32*)(ndl + l - 32) = lf;
      *(u32*)(ndv + l - 32) = v;
      *(u32*)(sol + lf) = (nb << 6) | (l - 32);
    }
    return wave_sum(v);
  }
};

}  // namespace crdt
