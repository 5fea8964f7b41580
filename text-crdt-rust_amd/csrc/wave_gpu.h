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

// Unsigned max / min over the wave (the DPP sequence of wave_or; lanes without a source take the
// identity)
__device__ __forceinline__ u32 wave_umax(u32 v) {
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ u32 wave_umin(u32 v) { return ~wave_umax(~v); }
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

// HR (HBM root): the root level for documents past the LDS root's capacity (ROOT_CAP_MAX
// groups): LDS holds a top level of rows (row id, groups, visible count) and the groups live in
// 64-slot rows in HBM (block id, slot count, visible count), with gsob[block] = row << 6 | slot.
// The replay sees the same flat group indices either way (root_* below).
template <int L, bool HR = false>
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
  lds_u32* rk = nullptr;  // agent ranks (documents with <= RANK_LDS agents)
  lds_u32* pf = nullptr;  // integrate's scan: the successor leaf, requested ahead (LDS-DMA)
  u32 rcap = 0;
  u32* hrow = nullptr;  // HR: this document's rows (192 u32 each: blk[64], cnt[64], vis[64])
  u32* gsob = nullptr;  // HR: block -> row << 6 | slot
  __device__ __forceinline__ void bind_root(const Pools& P, const DocSeg& sg) {
    if constexpr (HR) {
      hrow = P.hrows + sg.hrow_base * (u64)HROOT_ROW;
      gsob = P.gsob + sg.blk_base;
    } else {
      (void)P; (void)sg;
    }
  }

  // ---- scalar memory helpers (every lane touches the same address: uniform results, and a
  //      store is then visible to every lane's later loads by per-thread program order)
  __device__ __forceinline__ u32 ld(const u32* p) const { return uni(*(const u32*)p); }
  // a load whose wait is deferred to the first uni_() of its value (overlaps later loads)
  __device__ __forceinline__ u32 ld_raw(const u32* p) const { return *(const u32*)p; }
  __device__ __forceinline__ void ld_raw2(const u32* p, u32& a, u32& b) const {  // p 8-byte aligned
    uint2 v = *(const uint2*)p;
    a = v.x;
    b = v.y;
  }
  __device__ __forceinline__ static u32 uni_(u32 x) { return uni(x); }
  __device__ __forceinline__ void st(u32* p, u32 v) const { *(u32*)p = v; }
  __device__ __forceinline__ void st(i32* p, i32 v) const { *(i32*)p = v; }
  // the store by lanes [0, n) (n in {0, 1}: a predicated store of one word)
  __device__ __forceinline__ void st_lanes(u32* p, u32 v, u32 n) const { if (lane() < n) *(u32*)p = v; }
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
  __device__ __forceinline__ void st_agent_tail(AgentRec* p, u32 key, u32 order, u32 len) const {
    *(uint4*)&p->tkey = make_uint4(key, order, len, 0u);  // (every lane stores the same values)
  }
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
  // lane-parallel fill of n u16 (the order -> agent map)
  __device__ __forceinline__ void fill16(u16* p, u32 n, u32 v) const {
    u32 l = lane();
    if (n == 0u) return;
    if (n <= 64u) {  // one store, lanes >= n repeating item n - 1
      u32 m = n - 1u;
      p[l < m ? l : m] = (u16)v;
      return;
    }
    for (u32 k = l; k < n; k += 64) p[k] = (u16)v;
  }
  __device__ __forceinline__ u32 ld16(const u16* p) const { return uni((u32)*p); }
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
  // As search, and the run itself: the last level loads each lane's whole 16 B run, so the caller
  // needs no second (dependent) load for the run it found.
  template <class T>
  __device__ __forceinline__ i32 search_run(const T* base, u32 n, u32 needle, T& out) const {
    static_assert(sizeof(T) == 16, "16 B runs");
    if (n == 0) return -1;
    u32 lo = 0, hi = n;
    u32 l = lane();
    while (hi - lo > 64) {
      u32 step = (hi - lo + 63) / 64;
      u32 idx = lo + l * step;
      u32 key = *(const u32*)&base[idx < hi ? idx : hi - 1];
      u64 m = ballot(idx < hi && key <= needle);
      if (m == 0) return -1;
      u32 t = 63 - __builtin_clzll(m);
      lo = lo + t * step;
      u32 nh = lo + step;
      hi = nh < hi ? nh : hi;
    }
    u32 idx = lo + l;
    uint4 v = *(const uint4*)&base[idx < hi ? idx : hi - 1];
    u64 m = ballot(idx < hi && v.x <= needle);
    if (m == 0) return -1;
    u32 t = 63 - __builtin_clzll(m);
    u32 f[4] = {rdlane(v.x, t), rdlane(v.y, t), rdlane(v.z, t), rdlane(v.w, t)};
    __builtin_memcpy(&out, f, 16);
    return needle < f[0] + rlen(out) ? (i32)(lo + t) : -1;
  }
  // As search_run, the last 64 runs first (one coalesced 1 KB load, no top level): a recent key --
  // a round-start frontier head of a concurrent history, a few dozen runs back -- is answered there
  template <class T>
  __device__ __forceinline__ i32 search_run_recent(const T* base, u32 n, u32 needle, T& out) const {
    if (n <= 64u) return search_run(base, n, needle, out);
    u32 lo = n - 64u;
    uint4 v = *(const uint4*)&base[lo + lane()];
    u64 m = ballot(v.x <= needle);  // (keys ascend: a prefix of the lanes)
    if (!(m & 1ull)) return search_run(base, lo, needle, out);
    u32 t = 63 - __builtin_clzll(m);
    u32 f[4] = {rdlane(v.x, t), rdlane(v.y, t), rdlane(v.z, t), rdlane(v.w, t)};
    __builtin_memcpy(&out, f, 16);
    return needle < f[0] + rlen(out) ? (i32)(lo + t) : -1;
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
  // The directory's top level in LDS (crdt_types.h DDT_LDS; after the agent ranks): word j = the
  // first key of block 64 j.  Last block with first key <= x, or -1, for nb <= 64 * DDT_LDS blocks:
  // the top level picks the 64-block group (one LDS read), one read of the group's 64 records
  // picks the block -- instead of the strided 64-ary search, whose first step reads 64 records
  // 16 B wide in 64 different lines
  __device__ __forceinline__ i32 dd_search_top(const DDBlk* b, u32 nb, u32 x) const {
    u32 l = lane();
    u32 nt = (nb + 63u) >> 6;
    u32 key = l < nt ? (u32)rk[RANK_LDS + l] : 0u;
    u64 m = ballot(l < nt && key <= x);
    if (m == 0) return -1;
    u32 base = (63u - (u32)__builtin_clzll(m)) << 6;
    u32 cnt = nb - base < 64u ? nb - base : 64u;
    u32 k2 = b[base + (l < cnt ? l : 0u)].first;
    u64 m2 = ballot(l < cnt && k2 <= x);  // (bit 0: the group's first key is the top level's)
    return (i32)(base + (63u - (u32)__builtin_clzll(m2)));
  }
  __device__ __forceinline__ void ddt_set(u32 j, u32 key) const {
    if (lane() == 0u) rk[RANK_LDS + j] = key;
  }
  // top-level words [j0, ceil(nb / 64)) from the directory (after a block insert shifted it)
  __device__ __forceinline__ void ddt_rebuild(const DDBlk* b, u32 j0, u32 nb) const {
    u32 l = lane();
    u32 nt = (nb + 63u) >> 6;
    if (l >= j0 && l < nt) rk[RANK_LDS + l] = b[(u64)l << 6].first;
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
  __device__ __forceinline__ void cset_len(u32 i, i32 len) { en = (i32)wrlane((u32)en, (u32)len, i); }
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
  // integrate's scan (replay_core.h apply_txn M_INS) over entries [a, n) of the cached leaf, each
  // at its start: entry j's item is eo_j, its origin_left el_j.  Lane j: stop = its item is the
  // new item's origin_right; eq = its origin_left is the new item's (X); then the name tie-break
  // with the rank of the agent of its first order (order -> agent map, agents table):
  // my_rank > rank: scanning = false and go on; else break if its origin_right is the new item's,
  // else scanning from it.  Returns the first lane with an event (a break, or an origin_left
  // other than X: a cursor compare) or n; `last` = the last lane before it (INVALID if none),
  // `last_scan` = whether it left scanning on.
  // the document's agent ranks into LDS (replay start; n agents, fixed during a launch)
  __device__ __forceinline__ void rank_load(const AgentRec* agents, u32 n) const {
    u32 l = lane();
    if (l < n && l < RANK_LDS) rk[l] = agents[l].rank;
    __builtin_amdgcn_wave_barrier();
  }
  // agent a's rank (uniform a)
  __device__ __forceinline__ u32 rank_of(const AgentRec* agents, u32 n, u32 a) const {
    return n <= RANK_LDS ? uni(rk[a]) : ld(&at(agents, a)->rank);
  }
  // the agents of the cached leaf's entries [0, n) from the order -> agent map (lanes >= n read
  // entry 0's)
  __device__ __forceinline__ u32 scan_gather(u32 n, const u16* oag) const {
    u32 l = lane();
    u32 o = l < n ? (u32)eo : rdlane(eo, 0);
    return *(const u16*)((const char*)oag + (u64)(o * 2u));
  }
  // A leaf's agent row (crdt_types.h lag_words): one word per lane ...
  __device__ __forceinline__ u32 lag_ld(const u32* p) const {
    u32 l = lane();
    return l < lag_words(L) ? *(const u32*)(p + l) : 0u;
  }
  __device__ __forceinline__ u32 lag_valid(u32 lw) const { return rdlane(lw, 0) == 1u; }
  // ... entry l's agent from it ...
  __device__ __forceinline__ u32 lag_agents(u32 lw, u32 n, const u16* oag, u32 tkey, u32 tlen, u32 tagent) const {
    (void)n; (void)oag; (void)tkey; (void)tlen; (void)tagent;
    u32 l = lane();
    u32 v = shfl(lw, lag_words(L) / 2u + (l >> 1));
    return (l & 1u) ? v >> 16 : v & 0xFFFFu;
  }
  // ... and written from the gathered agents (the client_with_order tail run's orders are not in
  // the map yet: their agent is the tail's), with word 0 = 1, and the leaf's scan summary
  // (crdt_types.h LAG_*): the agent count the ranks are of, the entries' common origin_left (or
  // "mixed"), their highest agent rank and the range of their first orders
  __device__ __forceinline__ void lag_store(u32* p, u32 ag, u32 n, u32 tkey, u32 tlen, u32 tagent, u32 rt, u32 n_agents,
                                            const AgentRec* agents) const {
    u32 l = lane();
    bool in = l < n;
    u32 o = in ? (u32)eo : rdlane(eo, 0);
    ag = o - tkey < tlen ? tagent : ag;
    u32 lo = shfl(ag, 2u * (l - lag_words(L) / 2u)), hi = shfl(ag, 2u * (l - lag_words(L) / 2u) + 1u);
    u32 v = l == 0u ? 1u : ((hi << 16) | (lo & 0xFFFFu));
    u32 rk = n_agents <= RANK_LDS ? (u32)__builtin_amdgcn_ds_bpermute((int)(ag * 4u), (int)rt)
                                  : *(const u32*)((const char*)agents + (u64)(ag * (u32)sizeof(AgentRec) + 12u));
    u32 mr = wave_umax(in ? rk : 0u);
    u32 omin = wave_umin(in ? o : 0xFFFFFFFFu), omax = wave_umax(in ? o : 0u);
    u32 el0 = rdlane(el, 0);
    u32 mixed = (n == 0u || ballot(in && el != el0) != 0ull) ? LAG_MIXED : 0u;
    v = l == LAG_EPOCH ? (n_agents | mixed) : l == LAG_OL ? el0 : l == LAG_RANK ? mr : l == LAG_OMIN ? omin : l == LAG_OMAX ? omax : v;
    if (l <= LAG_OMAX || (l >= lag_words(L) / 2u && l < lag_words(L) / 2u + (u32)L / 2u)) *(u32*)(p + l) = v;
  }
  // integrate's scan over whole leaves (replay_core.h skip_leaves): of the leaves in slots [a, cnt)
  // of a directory leaf row, the first whose summary does not show that every entry passes the
  // scan with no event -- a current row (of this launch's agent count) whose entries all have
  // origin_left X, rank below my_rank and a first order other than orr.  Returns its slot (cnt:
  // none) and its leaf id.
  __device__ __forceinline__ u32 skip_scan(const u32* row, u32 a, u32 cnt, const u32* lag, u32 X, u32 orr, u32 my_rank,
                                           u32 n_agents, const Span* leaves, const AgentRec* agents, u32& leaf) const {
    (void)leaves; (void)agents;  // (the CPU emulation checks every skipped leaf against them)
    u32 l = lane();
    bool in = l >= a && l < cnt;
    u32 lf = row[l];  // 64-slot row: always in bounds
    // (32-bit byte offsets from the uniform base: saddr loads, one offset VGPR)
    u32 off = (in ? lf : 0u) * (lag_words(L) * 4u);
    uint2 h = *(const uint2*)((const char*)lag + (u64)off);                 // current flag, epoch
    uint4 sm = *(const uint4*)((const char*)lag + (u64)(off + LAG_OL * 4u));  // origin_left, max rank, first-order range
    bool skip = h.x == 1u && h.y == n_agents && sm.x == X && sm.y < my_rank && orr - sm.z > sm.w - sm.z;
    u64 stop = ballot(in && !skip);
    if (!stop) return cnt;
    u32 j = (u32)__builtin_ctzll(stop);
    leaf = rdlane(lf, j);
    return j;
  }
  // the LDS rank table as one row (lane a: agent a's rank), read before an LDS-DMA is requested:
  // an LDS read issued after one waits for every outstanding load, the DMA's included
  __device__ __forceinline__ u32 rank_row(u32 n_agents) const { return n_agents <= RANK_LDS ? (u32)rk[lane()] : 0u; }
  __device__ __forceinline__ u32 scan_batch(u32 ag, u32 rt, u32 me, u32 a, u32 n, u32 X, u32 orr,
                                            const AgentRec* agents, u32 n_agents, u32 tkey, u32 tlen, u32 tagent, u32& last,
                                            u32& last_scan) const {
    // (the replay's register budget is spent: per-lane values are transient, the per-lane tests
    // become lane masks at once, and the rest is scalar mask arithmetic)
    u32 l = lane();
    u32 o = (l >= a && l < n) ? (u32)eo : rdlane(eo, a);
    ag = o - tkey < tlen ? tagent : ag;  // the client_with_order tail run is not in the map yet
    bool small = n_agents <= RANK_LDS;  // AgentRec::rank from the rank row when it fits (bpermute: no LDS read)
    u32 my_rank = small ? rdlane(rt, me) : ld(&at(agents, me)->rank);
    u32 rk = small ? (u32)__builtin_amdgcn_ds_bpermute((int)(ag * 4u), (int)rt)
                   : *(const u32*)((const char*)agents + (u64)(ag * (u32)sizeof(AgentRec) + 12u));
    u64 lt = ballot(my_rank > rk);
    u64 ev = ballot(eo == orr) | ballot(el != X) | (~lt & ballot(er == orr));
    u64 in = (n >= 64u ? ~0ull : ((1ull << n) - 1ull)) & (~0ull << a);
    ev &= in;
    u32 f = ev ? (u32)__builtin_ctzll(ev) : n;
    last = f > a ? f - 1u : INVALID;
    last_scan = f > a ? (u32)((~lt >> (f - 1u)) & 1ull) : 0u;
    return f;
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
  // a new leaf's entries [0, n) := f(lane), the rest empty: computed lane-parallel, one store
  template <class F> __device__ __forceinline__ void leaf_write_lanes(Span* dst, u32 n, F f) const {
    u32 l = lane();
    Span e = f(l);
    bool in = l < n;
    if (l < (u32)L) *(uint4*)(dst + l) = in ? make_uint4(e.order, e.ol, e.orr, (u32)e.len) : make_uint4(0, 0, 0, 0);
  }
  // A leaf requested ahead into this wave's LDS row by LDS-DMA (global_load_lds_dwordx4: lane l's
  // entry to row + 16 l, no VGPR holds it in flight), made the cached leaf once integrate's scan
  // reaches it (returns its entry count).
  __device__ __forceinline__ void leaf_prefetch(const Span* p) const {
    typedef __attribute__((address_space(1))) u32 g_u32;
    u32 l = lane();
    if (l < (u32)L) __builtin_amdgcn_global_load_lds((g_u32*)(p + l), pf, 16, 0, 0);
  }
  // a requested successor the scan does not take (skip_leaves): its LDS-DMA completes first
  __device__ __forceinline__ void prefetch_drain() const { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
  __device__ __forceinline__ u32 cache_from_prefetch() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA counts in vmcnt; it is not a VGPR the compiler tracks)
    u32 l = lane();
    bool in = l < (u32)L;
    const lds_u32* q = pf + 4u * (l & (u32)(L - 1));
    u32 a = q[0], b = q[1], c = q[2], d = q[3];
    eo = in ? a : 0u; el = in ? b : 0u; er = in ? c : 0u; en = in ? (i32)d : 0;
    return __popcll(ballot(en != 0));
  }
  // lof[order + t] = v for every item of the entries in lanes [a, b): 64 items per step, each
  // lane finding its entry by a binary search over the entries' length prefix (entries sit in
  // lanes < L: log2(L) steps, on bpermute byte addresses), then the item's order from one more
  // bpermute of (entry order - entry start)
  __device__ __forceinline__ void fill_runs(u32* base, u32 a, u32 b, u32 v) const {
    u32 l = lane();
    u32 ln = l >= a && l < b ? (u32)(en < 0 ? -en : en) : 0u;
    u32 Pi = wave_incl_scan(ln);
    u32 T = rdlane(Pi, 63);
    u32 vb = eo - (Pi - ln);  // item j (of all the entries' items) of this lane's entry: order vb + j
    for (u32 t = 0; t < T; t += 64) {
      u32 j = t + l;
      u32 m4 = 0;  // 4 x the entry's lane (a bpermute byte address)
      for (u32 step = (u32)L / 2u; step; step >>= 1) {
        u32 x = (u32)__builtin_amdgcn_ds_bpermute((int)(m4 + 4u * (step - 1u)), (int)Pi);
        m4 = x <= j ? m4 + 4u * step : m4;
      }
      u32 o = (u32)__builtin_amdgcn_ds_bpermute((int)m4, (int)vb) + j;
      if (j < T) *(u32*)((char*)base + (u64)(o * 4u)) = v;
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
      bool okh = X == ((REC_RTXN << 28) | (1u << RTXN_DEL_BIT) | 1u) && Y == (agent | (1u << 16)) && Z == ps + 1u && Q == 1u;
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
  // Front-run scan (replay_core.h leaf_insert_front): lane k checks compact local record k against "one
  // LocalOp inserting `len` chars at position 0 by `agent`" (the txn at b0 was checked by the
  // caller).  Returns the run length in txns (>= 1).
  __device__ __forceinline__ u32 front_scan(u32 b0, u32 nv, u32 agent, u32 len) const {
    u32 l = lane();
    u32 d = (rx ^ ((REC_LC << 28) | agent)) | ry | rz | (rw ^ len);
    u64 stop = ballot(d != 0u || l >= nv) & (~1ull << b0);
    u32 f = stop ? (u32)__builtin_ctzll(stop) : 64u;
    return f - b0;
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
  // advance_branch_by for a remote txn (doc.rs:34-48), one frontier head and one parent per lane
  // (nfr, np <= 64): head 0 is f0 (the write-back tail), heads 1.. live at f[1..].  Returns 0 if a
  // head is `first` (the txn is known), INVALID if the new frontier would pass cap, else the new
  // head count: the heads not among the parents (p0, then pp[1..np)) in order, then
  // `last`; the first of them in nf0, the others at f[1..].
  __device__ __forceinline__ u32 frontier_advance(u32* f, u32 nfr, u32 f0, const u32* pp, u32 np, u32 p0, u32 first,
                                                  u32 last, u32 cap, u32& nf0) const {
    u32 l = lane();
    bool in = l < nfr;
    u32 fv = f[in ? l : 0u];
    fv = l == 0u ? f0 : fv;
    if (ballot(in && fv == first)) return 0u;
    u32 pv = np > 1u ? pp[l < np ? l : 0u] : 0u;  // (parent 0 is p0: pp[0] is not written yet)
    pv = l == 0u ? p0 : pv;
    bool hit = false;
    for (u32 j = 0; j < np; j++) hit |= fv == rdlane(pv, j);
    u64 keep = ballot(in && !hit);
    u32 m = (u32)__popcll(keep);
    if (m + 1u > cap) return INVALID;
    nf0 = m ? rdlane(fv, (u32)__builtin_ctzll(keep)) : last;
    u32 at = (u32)__popcll(keep & ((1ull << l) - 1ull));  // this head's place in the new frontier
    if (((keep >> l) & 1ull) && at >= 1u) f[at] = fv;
    if (m) f[m] = last;  // (every lane stores the same value)
    return m + 1u;
  }
  // ---- frontier heads 1..n-1 in context lanes (replay_core.h FR_S0: x1 lane FR_S0 - 64 + k - 1
  // holds head k, n <= FR_LANES + 1), moved in from / out to the HBM array f[1..n)
  static constexpr u32 FR_L0 = FR_S0 - 64u;
  __device__ __forceinline__ void fr_lanes_load(const u32* f, u32 n) {
    u32 l = lane();
    bool mine = (l >= FR_L0) & (l < FR_L0 + n - 1u);
    u32 v = f[mine ? l - FR_L0 + 1u : 0u];  // (clamped address: unconditional load)
    x1 = mine ? v : x1;
  }
  __device__ __forceinline__ void fr_lanes_store(u32* f, u32 n) const {
    u32 l = lane();
    if ((l >= FR_L0) & (l < FR_L0 + n - 1u)) f[l - FR_L0 + 1u] = x1;
  }
  // frontier_advance with heads 1.. read from the context lanes; the new heads go back to the
  // lanes (a push: kept head of rank a >= 1 to lane FR_L0 + a - 1, `last` after them) while they
  // fit, else to f[1..] in HBM
  __device__ __forceinline__ u32 frontier_advance_x(u32 nfr, u32 f0, const u32* pp, u32 np, u32 p0, u32 first,
                                                    u32 last, u32 cap, u32& nf0, u32* f) {
    u32 l = lane();
    bool in = l < nfr;
    u32 fv = shfl(x1, l + FR_L0 - 1u);  // (lane l >= 1: head l; lane 0's is replaced)
    fv = l == 0u ? f0 : fv;
    if (ballot(in && fv == first)) return 0u;
    u32 pv = np > 1u ? pp[l < np ? l : 0u] : 0u;  // (parent 0 is p0: pp[0] is not written yet)
    pv = l == 0u ? p0 : pv;
    bool hit = false;
    for (u32 j = 0; j < np; j++) hit |= fv == rdlane(pv, j);
    u64 keep = ballot(in && !hit);
    u32 m = (u32)__popcll(keep);
    if (m + 1u > cap) return INVALID;
    nf0 = m ? rdlane(fv, (u32)__builtin_ctzll(keep)) : last;
    u32 at = (u32)__popcll(keep & ((1ull << l) - 1ull));
    bool mv = ((keep >> l) & 1ull) && at >= 1u;
    if (m <= FR_LANES) {
      u32 moved = (u32)__builtin_amdgcn_ds_permute((int)((mv ? FR_L0 + at - 1u : 0u) << 2), (int)fv);
      if (m) x1 = ((l >= FR_L0) & (l < FR_L0 + m - 1u)) ? moved : l == FR_L0 + m - 1u ? last : x1;
    } else {
      if (mv) f[at] = fv;
      f[m] = last;
    }
    return m + 1u;
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

  // ---------------------------------------------------------------- directory root
  // Flat LDS root (!HR): group g of the root: rblk()[g], rcnt()[g], rvis()[g]; rcap groups per
  // array (a multiple of 64, chosen per launch).  Sweeps go 64 groups at a time, one per lane.
  // Two-level root (HR): top entry t in LDS: trow()[t], tcnt()[t], tvis()[t] (rcap entries), the
  // top count and the row count in two more LDS words; rows in HBM.  Flat group g is slot j of the
  // row of top entry t, where t is the first entry whose cumulative group count exceeds g.
  __device__ __forceinline__ lds_u32* rblk() const { return rt; }
  __device__ __forceinline__ lds_u32* rcnt() const { return rt + rcap; }
  __device__ __forceinline__ lds_u32* rvis() const { return rt + 2 * rcap; }
  __device__ __forceinline__ lds_u32* gob() const { return rt + 3 * rcap; }  // block -> group (!HR)
  __device__ __forceinline__ lds_u32* trow() const { return rt; }
  __device__ __forceinline__ lds_u32* tcnt() const { return rt + rcap; }
  __device__ __forceinline__ lds_u32* tvis() const { return rt + 2 * rcap; }
  __device__ __forceinline__ u32 ntop() const { return uni(rt[3 * rcap]); }
  __device__ __forceinline__ void set_ntop(u32 v) const { rt[3 * rcap] = v; }
  __device__ __forceinline__ u32 nrows() const { return uni(rt[3 * rcap + 1]); }
  __device__ __forceinline__ void set_nrows(u32 v) const { rt[3 * rcap + 1] = v; }
  __device__ __forceinline__ u32* hb(u32 row) const { return hrow + (u64)row * 192u; }
  __device__ __forceinline__ u32* hc(u32 row) const { return hrow + (u64)row * 192u + 64u; }
  __device__ __forceinline__ u32* hv(u32 row) const { return hrow + (u64)row * 192u + 128u; }
  // HR: top entry t of flat group g (g < the group count) and its slot j; INVALID past the end.
  // cbefore / vbefore: groups / visible items in the top entries before t.
  __device__ __forceinline__ u32 hr_locate(u32 g, u32& j, u32& cbefore, u32& vbefore) const {
    u32 l = lane(), cc = 0, cv = 0, nt = ntop();
    for (u32 r = 0; r < nt; r += 64) {
      u32 i = r + l;
      bool valid = i < nt;
      u32 c = valid ? (u32)tcnt()[i] : 0u, v = valid ? (u32)tvis()[i] : 0u;
      u32 ic = wave_incl_scan(c) + cc, iv = wave_incl_scan(v) + cv;
      u32 k = __popcll(ballot(ic <= g));  // (invalid lanes add 0: counted only if k >= nvalid)
      u32 nvalid = nt - r < 64u ? nt - r : 64u;
      if (k < nvalid) {
        cbefore = rdlane(ic, k) - rdlane(c, k);
        vbefore = rdlane(iv, k) - rdlane(v, k);
        j = g - cbefore;
        return r + k;
      }
      cc = rdlane(ic, 63);
      cv = rdlane(iv, 63);
    }
    return INVALID;
  }
  // HR: top entry of a row, with the groups / visible items before it
  __device__ __forceinline__ u32 hr_top_of_row(u32 row, u32& cbefore, u32& vbefore) const {
    u32 l = lane(), cc = 0, cv = 0, nt = ntop();
    for (u32 r = 0; r < nt; r += 64) {
      u32 i = r + l;
      bool valid = i < nt;
      u32 tr = valid ? (u32)trow()[i] : INVALID;
      u32 c = valid ? (u32)tcnt()[i] : 0u, v = valid ? (u32)tvis()[i] : 0u;
      u32 ic = wave_incl_scan(c) + cc, iv = wave_incl_scan(v) + cv;
      u64 m = ballot(tr == row);
      if (m) {
        u32 k = (u32)__builtin_ctzll(m);
        cbefore = rdlane(ic, k) - rdlane(c, k);
        vbefore = rdlane(iv, k) - rdlane(v, k);
        return r + k;
      }
      cc = rdlane(ic, 63);
      cv = rdlane(iv, 63);
    }
    return INVALID;
  }
  // HR: insert top entry (row, cnt, vis) at t, shifting [t, ntop) up (as root_insert below)
  __device__ __forceinline__ void hr_top_insert(u32 t, u32 row, u32 cnt, u32 vis) {
    u32 l = lane(), nt = ntop();
    for (i32 r = (i32)(nt & ~63u); r >= (i32)(t & ~63u); r -= 64) {
      u32 i = (u32)r + l;
      u32 jj = i > 0u ? i - 1u : 0u;
      u32 b = trow()[jj], c = tcnt()[jj], v = tvis()[jj];
      __builtin_amdgcn_wave_barrier();
      if (i > t && i <= nt) { trow()[i] = b; tcnt()[i] = c; tvis()[i] = v; }
      __builtin_amdgcn_wave_barrier();
    }
    trow()[t] = row;
    tcnt()[t] = cnt;
    tvis()[t] = vis;
    __builtin_amdgcn_wave_barrier();
    set_ntop(nt + 1u);
    __builtin_amdgcn_wave_barrier();
  }

  // Groups [ng, rcap) hold block id INVALID (no block has that id), so root_find_blk needs no
  // bounds test; the root only grows while a wave runs (root_insert writes at most up to ng).
  __device__ __forceinline__ void root_clear_from(u32 ng) {
    if constexpr (HR) {
      (void)ng;
    } else {
      for (u32 i = lane(); i < rcap; i += 64)
        if (i >= ng) rblk()[i] = INVALID;
    }
  }
  __device__ __forceinline__ void root_init(u32 blk, u32 cnt, u32 vis) {
    if constexpr (HR) {
      trow()[0] = 0u;
      tcnt()[0] = 1u;
      tvis()[0] = vis;
      set_ntop(1u);
      set_nrows(1u);
      *hb(0) = blk;
      *hc(0) = cnt;
      *hv(0) = vis;
      gsob[blk] = 0u;
      __builtin_amdgcn_wave_barrier();
    } else {
      root_clear_from(1u);
      rblk()[0] = blk;  // every lane stores the same value: no branch
      rcnt()[0] = cnt;
      rvis()[0] = vis;
      gob()[blk] = 0u;
    }
  }
  __device__ __forceinline__ void root_load(const GroupRec* g, u32 ng) {
    if constexpr (HR) {
      // rows of 32 groups (half full: room to insert before a row splits)
      u32 nr = (ng + 31u) / 32u;
      for (u32 i = lane(); i < ng; i += 64) {
        uint4 x = *(const uint4*)(g + i);
        u32 r = i >> 5, s = i & 31u;
        hb(r)[s] = x.x;
        hc(r)[s] = x.y;
        hv(r)[s] = x.z;
        gsob[x.x] = (r << 6) | s;
      }
      for (u32 t = lane(); t < nr; t += 64) {
        u32 c = ng - 32u * t < 32u ? ng - 32u * t : 32u, v = 0;
        for (u32 k = 0; k < c; k++) v += g[32u * t + k].vis;
        trow()[t] = t;
        tcnt()[t] = c;
        tvis()[t] = v;
      }
      __builtin_amdgcn_wave_barrier();
      set_ntop(nr);
      set_nrows(nr);
      __builtin_amdgcn_wave_barrier();
    } else {
      root_clear_from(ng);
      for (u32 i = lane(); i < ng; i += 64) {
        uint4 x = *(const uint4*)(g + i);
        rblk()[i] = x.x;
        rcnt()[i] = x.y;
        rvis()[i] = x.z;
        gob()[x.x] = i;
      }
    }
  }
  __device__ __forceinline__ void root_store(GroupRec* g, u32 ng) const {
    if constexpr (HR) {
      (void)ng;
      u32 nt = ntop(), base = 0, l = lane();
      for (u32 t = 0; t < nt; t++) {
        u32 row = uni(trow()[t]), c = uni(tcnt()[t]);
        if (l < c) *(uint4*)(g + base + l) = make_uint4(hb(row)[l], hc(row)[l], hv(row)[l], 0);
        base += c;
      }
    } else {
      for (u32 i = lane(); i < ng; i += 64) *(uint4*)(g + i) = make_uint4(rblk()[i], rcnt()[i], rvis()[i], 0);
    }
  }
  __device__ __forceinline__ u32 root_blk(u32 g) const {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      return ld(hb(uni(trow()[t])) + j);
    } else {
      return uni(rblk()[g]);
    }
  }
  __device__ __forceinline__ u32 root_cnt(u32 g) const {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      return ld(hc(uni(trow()[t])) + j);
    } else {
      return uni(rcnt()[g]);
    }
  }
  __device__ __forceinline__ u32 root_vis(u32 g) const {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      return ld(hv(uni(trow()[t])) + j);
    } else {
      return uni(rvis()[g]);
    }
  }
  __device__ __forceinline__ u32 root_find_blk(u32 ng, u32 blk) const {
    if constexpr (HR) {
      (void)ng;
      u32 s = ld(gsob + blk), cb, vb;
      u32 t = hr_top_of_row(s >> 6, cb, vb);
      return t == INVALID ? INVALID : cb + (s & 63u);
    } else {
      (void)ng;
      return uni(gob()[blk]);  // (one LDS read; every block id < ng is a group's)
    }
  }
  // the visible count of block blk's group += delta
  __device__ __forceinline__ void root_add_vis_blk(u32 ng, u32 blk, u32 delta) {
    if constexpr (HR) {
      (void)ng;
      u32 s = ld(gsob + blk), cb, vb;
      u32 row = s >> 6;
      u32 t = hr_top_of_row(row, cb, vb);
      u32* p = hv(row) + (s & 63u);
      *p = ld(p) + delta;
      tvis()[t] = uni(tvis()[t]) + delta;
    } else {
      root_add_vis(root_find_blk(ng, blk), delta);
    }
  }
  __device__ __forceinline__ void root_add_vis(u32 g, u32 delta) {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      u32* p = hv(uni(trow()[t])) + j;
      *p = ld(p) + delta;
      tvis()[t] = uni(tvis()[t]) + delta;
    } else {
      u32 v = uni(rvis()[g]) + delta;
      rvis()[g] = v;
    }
  }
  __device__ __forceinline__ void root_set(u32 g, u32 blk, u32 cnt, u32 vis) {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      u32 row = uni(trow()[t]);
      u32 old = ld(hv(row) + j);
      hb(row)[j] = blk;
      hc(row)[j] = cnt;
      hv(row)[j] = vis;
      gsob[blk] = (row << 6) | j;
      tvis()[t] = uni(tvis()[t]) + vis - old;
    } else {
      rblk()[g] = blk;
      rcnt()[g] = cnt;
      rvis()[g] = vis;
      gob()[blk] = g;
    }
  }
  // the slot count of group g := cnt (its block, visible count and block -> group entry unchanged)
  __device__ __forceinline__ void root_set_cnt(u32 g, u32 cnt) {
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 t = hr_locate(g, j, cb, vb);
      hc(uni(trow()[t]))[j] = cnt;
    } else {
      rcnt()[g] = cnt;
    }
  }
  // insert a group at index g, shifting [g, ng) up by one: 64-group chunks from the top down, each
  // read completely before it is written (a chunk's lane 0 reads the top of the chunk below,
  // which is written only afterwards).  HR: a 64-lane shift inside the group's row; a full row
  // splits first (its upper 32 groups move to a new row linked after it in the top level).
  __device__ __forceinline__ void root_insert(u32 ng, u32 g, u32 blk, u32 cnt, u32 vis) {
    if constexpr (HR) {
      u32 l = lane(), j, cb, vb, t;
      if (g < ng) {
        t = hr_locate(g, j, cb, vb);
      } else {  // append after the last group
        t = ntop() - 1u;
        j = uni(tcnt()[t]);
      }
      u32 row = uni(trow()[t]), c = uni(tcnt()[t]);
      if (c == 64u) {  // split the row: [32, 64) -> a new row after it
        u32 nr = nrows();
        set_nrows(nr + 1u);
        u32 b = hb(row)[l], cn = hc(row)[l], v = hv(row)[l];
        u32 mv = wave_sum(l >= 32u ? v : 0u);
        if (l >= 32u) {
          hb(nr)[l - 32u] = b;
          hc(nr)[l - 32u] = cn;
          hv(nr)[l - 32u] = v;
          gsob[b] = (nr << 6) | (l - 32u);
        }
        tcnt()[t] = 32u;
        tvis()[t] = uni(tvis()[t]) - mv;
        __builtin_amdgcn_wave_barrier();
        hr_top_insert(t + 1u, nr, 32u, mv);
        if (j > 32u) { t += 1u; row = nr; j -= 32u; }
        c = 32u;
      }
      // slots [j, c) of the row move up one; the new group goes to slot j
      u32 ob = hb(row)[l], oc = hc(row)[l], ov = hv(row)[l];
      u32 sb = shfl(ob, l - 1u), sc = shfl(oc, l - 1u), sv = shfl(ov, l - 1u);
      if (l > j && l <= c) {
        hb(row)[l] = sb;
        hc(row)[l] = sc;
        hv(row)[l] = sv;
        gsob[sb] = (row << 6) | l;
      }
      if (l == j) {
        hb(row)[l] = blk;
        hc(row)[l] = cnt;
        hv(row)[l] = vis;
        gsob[blk] = (row << 6) | l;
      }
      tcnt()[t] = c + 1u;
      tvis()[t] = uni(tvis()[t]) + vis;
      __builtin_amdgcn_wave_barrier();
    } else {
      u32 l = lane();
      for (i32 r = (i32)(ng & ~63u); r >= (i32)(g & ~63u); r -= 64) {
        u32 i = (u32)r + l;
        u32 jj = i > 0u ? i - 1u : 0u;
        u32 b = rblk()[jj], c = rcnt()[jj], v = rvis()[jj];
        __builtin_amdgcn_wave_barrier();
        if (i > g && i <= ng) { rblk()[i] = b; rcnt()[i] = c; rvis()[i] = v; gob()[b] = i; }
        __builtin_amdgcn_wave_barrier();
      }
      root_set(g, blk, cnt, vis);
    }
  }
  // first group whose cumulative visible count exceeds pos
  __device__ __forceinline__ bool root_find_pos(u32 ng, u32 pos, u32& g, u32& base) const {
    u32 l = lane();
    if constexpr (HR) {
      (void)ng;
      u32 cc = 0, cv = 0, nt = ntop();
      for (u32 r = 0; r < nt; r += 64) {
        u32 i = r + l;
        bool valid = i < nt;
        u32 c = valid ? (u32)tcnt()[i] : 0u, v = valid ? (u32)tvis()[i] : 0u;
        u32 ic = wave_incl_scan(c) + cc, iv = wave_incl_scan(v) + cv;
        u32 k = __popcll(ballot(iv <= pos));
        u32 nvalid = nt - r < 64u ? nt - r : 64u;
        if (k < nvalid) {
          u32 t = r + k, cb = rdlane(ic, k) - rdlane(c, k), vb = rdlane(iv, k) - rdlane(v, k);
          u32 row = uni(trow()[t]), n = uni(tcnt()[t]);
          u32 x = l < n ? hv(row)[l] : 0u;
          u32 incl = wave_incl_scan(x) + vb;
          u32 s = __popcll(ballot(incl <= pos));  // < n: the top entry's groups hold pos
          g = cb + s;
          base = rdlane(incl, s) - rdlane(x, s);
          return true;
        }
        cc = rdlane(ic, 63);
        cv = rdlane(iv, 63);
      }
      return false;
    } else {
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
  }

  // visible items in the groups before g (probe: Cursor::count_pos)
  __device__ __forceinline__ u32 root_vis_before(u32 g) const {
    u32 l = lane(), t = 0;
    if constexpr (HR) {
      u32 j, cb, vb;
      u32 te = hr_locate(g, j, cb, vb);
      u32 row = uni(trow()[te]);
      return vb + wave_sum(l < j ? (u32)hv(row)[l] : 0u);
    } else {
      for (u32 r = 0; r < g; r += 64) t += wave_sum(r + l < g ? (u32)rvis()[r + l] : 0u);
      return t;
    }
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
  // a 64-slot directory row, one slot per lane (requested first by split_at: see blk_insert_at)
  __device__ __forceinline__ u32 row_ld(const u32* p) const { return *(const u32*)(p + lane()); }
  // A leaf inserted after slot i of a block whose rows ol / ov (row_ld) hold cnt slots: slot i's
  // visible count becomes vis_i, (leaf, vis) goes to slot i + 1 and slots [i + 1, cnt) move up one.
  // One store per row and one slot-table store per moved leaf (lanes [i, cnt]).
  __device__ __forceinline__ void blk_insert_at(u32 ol, u32 ov, u32* dl, u32* dv, u32 cnt, u32 i, u32 vis_i, u32 leaf, u32 vis,
                                                u32* sol, u32 blk) const {
    u32 l = lane();
    u32 sl = shfl(ol, l - 1), sv = shfl(ov, l - 1);
    u32 j = i + 1u;
    u32 nlf = l <= i ? ol : (l == j ? leaf : sl);
    u32 nvs = l < i ? ov : (l == i ? vis_i : (l == j ? vis : sv));
    if (l >= i && l <= cnt) {
      *(u32*)(dl + l) = nlf;
      *(u32*)(dv + l) = nvs;
      *(u32*)(sol + 2u * nlf) = (blk << 6) | l;  // (slot entries are {slot, successor})
    }
  }
  // slots [32, 64) of a full block (rows rl / rv, row_ld) move to [0, 32) of block nb; returns
  // their visible total
  __device__ __forceinline__ u32 blk_split_r(u32 rl, u32 rv, const u32* dl, const u32* dv, u32* ndl, u32* ndv, u32* sol,
                                             u32 nb) const {
    (void)dl; (void)dv;
    u32 l = lane();
    if (l >= 32) {
      *(u32*)(ndl + l - 32) = rl;
      *(u32*)(ndv + l - 32) = rv;
      *(u32*)(sol + 2u * rl) = (nb << 6) | (l - 32);
    }
    return wave_sum(l >= 32 ? rv : 0u);
  }
  // the rows of the new block after blk_split_r (lanes >= 32 wrap: past its 32 slots)
  __device__ __forceinline__ void rows_upper(u32& rl, u32& rv, const u32* ndl, const u32* ndv) const {
    (void)ndl; (void)ndv;
    u32 s = lane() + 32u;
    rl = shfl(rl, s);
    rv = shfl(rv, s);
  }
};

}  // namespace crdt
