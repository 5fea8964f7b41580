// Device kernels of the engine.
//   k_init      ListCRDT::new() per document (wave per document)
//   k_replay    apply the staged record stream (wave per document, replay_core.h)
//   k_relayout_pool  move every document's part of one pool into its re-sized pool (block per document)
//   k_publish   flat index build: canonical spans (can_append compaction of the leaf entries in
//               document order), visible-prefix vpos, order->span scatter, digest
//   k_pub_index the order->span index of k_publish's documents, built in LDS (block per document)
//   k_pos_to_loc / k_loc_to_pos   batched lookups on the published index (thread per query)
//   k_materialize  document text from the published index + content streams (block per document)
#pragma once
#include "replay_core.h"
#include "wave_gpu.h"

namespace crdt {

struct PubOut {
  Span* canon;    // [canon_base + k]
  u32* vpos;      // [canon_base + k]  visible items before canonical span k
  u32* sorted;    // [canon_base + r]  the canonical spans by first order (rank -> span)
  u32* corder;    // [canon_base + k]  first order of canonical span k (k_pub_index's input: 4 B
                  //                   per span instead of re-reading the 16 B spans)
  u32* pub;       // [pub_base + w]    bit (o & 31) of word o >> 5: a canonical span starts at order o;
                  // [pub_base + pub_words + w]  set bits in words [0, w)
  u32* canon_n;   // [doc]
  u32* len;       // [doc]
  u64* digest;    // [doc]
};

// Order -> canonical span through the published index: r = span starts at or below `order`;
// the span is sorted[r - 1] if it contains the order (delete orders lie in no span).  Returns
// the span index or INVALID.
#ifdef PUB_PLAIN_LOADS
__device__ __forceinline__ u32 ld_l2(const u32* p) { return *p; }
#else
__device__ __forceinline__ u32 ld_l2(const u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
#endif
__device__ __forceinline__ u32 span_of_order(const PubOut& O, const DocSeg& seg, u32 cn, u32 order) {
  u32 nw = pub_words(seg.ord_cap);
  const u32* bits = O.pub + seg.pub_base;
  u32 wd = order >> 5;
  if (wd >= nw) return INVALID;
  u32 r = bits[nw + wd] + (u32)__popc(bits[wd] & (0xFFFFFFFFu >> (31u - (order & 31u))));
  if (r == 0u || r > cn) return INVALID;
  u32 k = O.sorted[seg.canon_base + r - 1u];
  if (k >= cn) return INVALID;
  Span sp = O.canon[seg.canon_base + k];
  return order - sp.order < slen(sp) ? k : INVALID;
}

#define WAVES_PER_BLOCK 4

// Dynamic LDS of the wave-per-document kernels: each wave's slice (crdt_types.h wave_lds_words):
// the scan's prefetch row, the directory root (flat: 4 x rcap u32; two-level: 3 x rcap + 2) and
// the document's agent ranks (RANK_LDS u32; launch shape: engine.hip launch_shape).
extern __shared__ u32 s_dyn[];
template <int L, bool HR = false>
__device__ __forceinline__ WaveGPU<L, HR> wave_with_root(u32 rcap) {
  WaveGPU<L, HR> w;
  // the LDS address space survives into the member: root accesses are ds_* (lgkmcnt only);
  // a generic pointer would make them flat ops, whose waits also drain every pending store
  w.rcap = rcap;
  u32 root = HR ? 3u * rcap + 2u : 4u * rcap;
  w.pf = (typename WaveGPU<L, HR>::lds_u32*)(s_dyn + uni(threadIdx.x >> 6) * wave_lds_words(rcap, HR));
  w.rt = w.pf + PF_LDS;
  w.rk = w.rt + root;
  return w;
}
// Document of the calling wave: wave k of the launch takes list[k] (or k without a list).
__device__ __forceinline__ u32 wave_doc(u32 wpb, const u32* list, u32 n, u32& d) {
  u32 k = uni(blockIdx.x * wpb + (threadIdx.x >> 6));
  if (k >= n) return 0;
  d = list ? uni(list[k]) : k;
  return 1;
}

template <int L>
__global__ __launch_bounds__(256) void k_init(Pools P, u32 n, u32 wpb, u32 rcap) {
  u32 d;
  if (!wave_doc(wpb, nullptr, n, d)) return;
  Replayer<WaveGPU<L>, L> r(P, d, wave_with_root<L>(rcap));
  r.init_empty();
  AgentRec* ag = r.agents();
  for (u32 a = lane_id(); a < r.g(S_N_AGENTS); a += 64) ag[a].run_cnt = 0;
  r.finish();
}

// n: waves of this launch (documents in `list`, or the first n documents)
// Register budget: 8 waves per SIMD (<= 64 VGPRs, <= 80 SGPRs).  Each document is one dependent
// chain, so resident waves are what hides its latencies: 8 waves/SIMD replays 8,192 automerge-paper
// documents in 185 ms where the compiler's own choice (84 VGPRs: 5 waves/SIMD) takes 199 ms and
// 97 VGPRs (4 waves/SIMD) took 216 ms (scripts/gpu_ab.sh).  What the budget costs is a few spills
// in cold paths.
template <int L, bool HR, u32 SH = SHAPE_ALL>
__device__ __forceinline__ void replay_doc(Pools P, u32 n, u32 wpb, u32 rcap, const u32* list) {
  u32 d;
  if (!wave_doc(wpb, list, n, d)) return;
  Replayer<WaveGPU<L, HR>, L> r(P, d, wave_with_root<L, HR>(rcap));
  WaveGPU<L, HR>& w = r.w;
  if (r.status() == ST_NEED_CAPACITY) r.p(S_STATUS, (u32)ST_OK);  // resume after growth
  if (r.status() != ST_OK || r.g(S_REC_POS) >= r.rec_n()) {
    w.st((u32*)&P.st[d].status, (u32)r.status());
    return;
  }
  r.begin();
  r.template run<SH>();
  r.finish();
}
#ifndef CRDT_REPLAY_WAVES
#define CRDT_REPLAY_WAVES 8  // waves per SIMD the replay's register budget is held to (diagnostic builds vary it)
#endif
// SH: the stream shape of every document of the launch (crdt_types.h SHAPE_*; the host launches
// each shape's documents in their own instance: SHAPE_ALL is the general one)
#ifndef CRDT_REPLAY_WAVES_GEN
#define CRDT_REPLAY_WAVES_GEN CRDT_REPLAY_WAVES  // (the generated-op instance's budget; diagnostic builds vary it)
#endif
template <int L, u32 SH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SH == SHAPE_GEN ? CRDT_REPLAY_WAVES_GEN : CRDT_REPLAY_WAVES))) void k_replay(Pools P, u32 n, u32 wpb, u32 rcap, const u32* list) {
  replay_doc<L, false, SH>(P, n, wpb, rcap, list);
}
// Documents past the LDS root replay with the two-level root (wave_gpu.h HR).  They are few and
// long, so this instance is held to 4 waves per SIMD (<= 128 VGPRs: no scratch for its extra
// root state) instead of the batch kernel's 8.
template <int L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_replay_hr(Pools P, u32 n, u32 wpb, u32 rcap, const u32* list) {
  replay_doc<L, true>(P, n, wpb, rcap, list);
}

// crdt_reseed_random_async: every document whose staged stream is one GEN record (crdt_stage_random)
// gets the generator seed of document id_base + d, (u32)mix64(seed ^ (id_base + d)) -- the seed
// crdt_stage_random gives document d for id_base 0 -- so one engine replays the batches of a
// larger corpus (BASELINE config 4: 1 M documents) without restaging.  Other documents are untouched.
__global__ void k_reseed_gen(Pools P, u32 n, u64 seed, u64 id_base) {
  u32 d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  DocSeg sg = P.seg[d];
  if (sg.rec_n != 1u) return;
  Rec* r = const_cast<Rec*>(P.recs + sg.rec_base);  // (the staged record pool: read-only to the replay)
  if (rec_kind(*r) != REC_GEN) return;
  r->w3 = (u32)mix64(seed ^ (id_base + d));
}

// Reset the per-call record cursor of every document (new stream staged).
__global__ void k_reset_recpos(DocState* st, u32 n, u32 n_agents_dummy) {
  u32 d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < n) st[d].rec_pos = 0;
}

// Host-side agent counts into every document's state (before k_init / a replay).
__global__ void k_set_n_agents(DocState* st, const u32* na, u32 n) {
  u32 d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < n) st[d].n_agents = na[d];
}

template <class T>
__device__ __forceinline__ void bcopy(T* dst, const T* src, u64 n) {
  for (u64 k = threadIdx.x; k < n; k += blockDim.x) dst[k] = src[k];
}

// Move one pool of document state into re-sized pools (growth / re-staging / fit; engine.hip layout: the pools move one at a time, each freed
// before the next is allocated, so a relayout needs the old pools + the largest new one, not both
// sets).  Block per document.  src / dst differ only in the pool being moved (and, for
// RL_ARUN, in the agent tables: src.agents the old one, dst.agents the new one with its run
// bases); RL_AGENTS moves the agents' run counts and last-run copies into the new table.
enum : u32 { RL_LEAVES, RL_SOL, RL_DIR_LEAF, RL_DIR_VIS, RL_LEAF_OF, RL_AGENT_OF, RL_CWO, RL_DELS, RL_DD, RL_DDB,
             RL_TXNS, RL_PARENTS, RL_FRONTIER, RL_GROUPS, RL_ARUN, RL_AGENTS, RL_N };
template <int L>
__global__ __launch_bounds__(256) void k_relayout_pool(Pools src, Pools dst, const DocSeg* old_seg, const u32* new_n_agents, u32 n,
                                                       u32 which) {
  u32 d = blockIdx.x;
  if (d >= n) return;
  DocState s = dst.st[d];
  DocSeg o = old_seg[d];
  DocSeg w = dst.seg[d];
  switch (which) {
    case RL_LEAVES: bcopy(dst.leaves + w.leaf_base * L, src.leaves + o.leaf_base * L, (u64)s.n_leaves * L); break;
    case RL_SOL: bcopy(dst.slot_of_leaf + 2 * w.leaf_base, src.slot_of_leaf + 2 * o.leaf_base, 2ull * s.n_leaves); break;
    case RL_DIR_LEAF: bcopy(dst.dir_leaf + w.blk_base * GROUP, src.dir_leaf + o.blk_base * GROUP, (u64)s.n_blocks * GROUP); break;
    case RL_DIR_VIS: bcopy(dst.dir_vis + w.blk_base * GROUP, src.dir_vis + o.blk_base * GROUP, (u64)s.n_blocks * GROUP); break;
    case RL_LEAF_OF:
      if (w.flags & o.flags & DOC_TRACK_MAP) bcopy(dst.leaf_of + w.map_base, src.leaf_of + o.map_base, s.next_order);
      break;
    case RL_AGENT_OF:
      if (w.flags & o.flags & DOC_TRACK_AGENT) bcopy(dst.agent_of + w.map_base, src.agent_of + o.map_base, s.next_order);
      break;
    case RL_CWO: bcopy(dst.cwo + w.cwo_base, src.cwo + o.cwo_base, s.n_cwo); break;
    case RL_DELS: bcopy(dst.dels + w.del_base, src.dels + o.del_base, s.n_del); break;
    case RL_DD: bcopy(dst.dd + w.dd_base * DD_BLK, src.dd + o.dd_base * DD_BLK, (u64)s.n_ddb * DD_BLK); break;
    case RL_DDB: bcopy(dst.ddb + w.dd_base, src.ddb + o.dd_base, s.n_ddb); break;
    case RL_TXNS: bcopy(dst.txns + w.txn_base, src.txns + o.txn_base, s.n_txn); break;
    case RL_PARENTS: bcopy(dst.parents + w.par_base, src.parents + o.par_base, s.n_par); break;
    case RL_FRONTIER: bcopy(dst.frontier + w.fr_base, src.frontier + o.fr_base, s.n_fr); break;
    case RL_GROUPS: bcopy(dst.groups + w.grp_base, src.groups + o.grp_base, s.ng); break;
    case RL_ARUN:
      for (u32 a = 0; a < s.n_agents; a++) {
        AgentRec ao = src.agents[o.agent_base + a];
        AgentRec an = dst.agents[w.agent_base + a];
        bcopy(dst.arun + w.arun_base + an.run_base, src.arun + o.arun_base + ao.run_base, ao.run_cnt);
      }
      break;
    case RL_AGENTS:
      for (u32 a = threadIdx.x; a < s.n_agents; a += blockDim.x) {
        AgentRec ao = src.agents[o.agent_base + a];  // (run base / cap: the new layout's)
        AgentRec* q = dst.agents + w.agent_base + a;
        q->run_cnt = ao.run_cnt;
        q->tkey = ao.tkey;
        q->torder = ao.torder;
        q->tlen = ao.tlen;
      }
      __syncthreads();
      if (threadIdx.x == 0) dst.st[d].n_agents = new_n_agents[d];
      break;
  }
}

// Order -> leaf map of documents that start keeping it (their first remote stream after local
// ones): INVALID everywhere, then every entry's orders -> its leaf, in directory order.  Block per
// listed document; the barrier orders the two sweeps' stores.
template <int L>
__global__ __launch_bounds__(256) void k_build_map(Pools P, const u32* docs, u32 n) {
  if (blockIdx.x >= n) return;
  u32 d = docs[blockIdx.x];
  DocState s = P.st[d];
  DocSeg sg = P.seg[d];
  u32* lof = P.leaf_of + sg.map_base;
  for (u64 o = threadIdx.x; o < s.next_order; o += blockDim.x) lof[o] = INVALID;
  __syncthreads();
  const GroupRec* gr = P.groups + sg.grp_base;
  const Span* lv = P.leaves + sg.leaf_base * L;
  for (u32 g = 0; g < s.ng; g++) {
    GroupRec G = gr[g];
    for (u32 i = 0; i < G.cnt; i++) {
      u32 leaf = P.dir_leaf[(sg.blk_base + G.blk) * GROUP + i];
      for (u32 e = 0; e < (u32)L; e++) {
        Span sp = lv[(u64)leaf * L + e];
        for (u32 t = threadIdx.x; t < slen(sp); t += blockDim.x) lof[sp.order + t] = leaf;
      }
    }
  }
}

// Order -> agent map of documents that start keeping it (a second agent appears in a tracked
// document that already holds state): every client_with_order run's orders -> its agent.
__global__ __launch_bounds__(256) void k_build_agent_map(Pools P, const u32* docs, u32 n) {
  if (blockIdx.x >= n) return;
  u32 d = docs[blockIdx.x];
  DocState s = P.st[d];
  DocSeg sg = P.seg[d];
  u16* oag = P.agent_of + sg.map_base;
  const CwoRun* cw = P.cwo + sg.cwo_base;
  for (u32 k = 0; k < s.n_cwo; k++) {
    CwoRun r = cw[k];  // (the last run's length is current: the replay's tails were flushed)
    for (u32 t = threadIdx.x; t < r.len; t += blockDim.x) oag[r.key + t] = (u16)r.agent;
  }
}

// ---------------------------------------------------------------------------------------------
// digest helpers (identical to oracle/crdt_oracle.hpp)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ u64 elem_hash(u32 section, u64 idx, u64 a, u64 b) {
  u64 k = mix64(((u64)section << 56) ^ idx);
  return mix64(mix64(k ^ a) ^ b);
}
__device__ __forceinline__ u64 wave_sum64(u64 v) {
  for (u32 off = 32; off >= 1; off >>= 1) {
    u32 lo = (u32)v, hi = (u32)(v >> 32);
    u32 src = lane_id() ^ off;
    u32 olo = shfl(lo, src), ohi = shfl(hi, src);
    v += ((u64)ohi << 32) | olo;
  }
  return v;
}

// ---------------------------------------------------------------------------------------------
// k_publish: the flat index of every document (canonical spans in document order, visible prefix,
// order -> span index, digest).  One wave per document (k_publish), or for long documents one
// workgroup of PUB_BIG_WAVES waves (k_publish_big): the leaf sequence is cut into one range per
// wave, each wave compacts its range, the spans that cross range boundaries are resolved once,
// and the index sweeps are split over the waves.
// ---------------------------------------------------------------------------------------------
#ifndef PUB_DEPTH
#define PUB_DEPTH 1  // compaction steps whose leaf loads are in flight at once (compact_range)
#endif
#define PUB_BIG_WAVES 16
#define PUB_BIG_MIN 2048u        // leaves from which a document may publish with a workgroup ...
#define PUB_BIG_FEW_DOCS 1024u   // ... when the batch has at most this many documents
#define PUB_BIG_MAX 16384u       // leaves from which it always does

// A published document whose digest k_digest has not computed yet (publish writes it; k_digest
// replaces it)
constexpr u64 DIGEST_PENDING = 1ull;
// Digest term of canonical span k (section 1; oracle/crdt_oracle.hpp digest()).
__device__ __forceinline__ u64 span_hash(u32 k, const Span& sp) {
  return elem_hash(1, k, ((u64)sp.order << 32) | sp.ol, ((u64)sp.orr << 32) | (u32)sp.len);
}

// What one wave's leaf range contributes (k_publish_big boundary resolution).
struct RangeSum {
  u32 spans;      // canonical spans starting in the range (its first entry counts as a start)
  u32 vis;        // visible items
  u32 single;     // the whole range is one span
  i32 lead_len;   // signed length of the range's first span inside the range
  Span first, last;  // first and last raw entries
};

// Canonical compaction of leaves [a, b) (directory order) by one wave, lane i = entry i of a leaf:
// an entry starts a new span unless YjsSpan::can_append(previous entry, entry) (span.rs:47-53;
// merging is transitive, so the previous raw entry stands for the open span); span lengths are
// segmented sums of a prefix scan; the span still open at a leaf's end carries over (uniform
// registers).  WRITE: spans go to canon/vpos from index `out` with visible offsets from `vis`;
// skip_first: the range's first span continues the previous range's (not written); extra: the
// signed length the range's last span continues by in later ranges.  !WRITE: fill `sum`.
// Every written span's first order also goes to corder.
template <int L, bool WRITE>
__device__ __forceinline__ void compact_range(const Pools& P, const DocSeg& seg, u32 ng, u32 a, u32 b, Span* canon,
                                              u32* vpos, u32* corder, u32 ccap, u32& out, u32& vis, u32 skip_first,
                                              i32 extra, RangeSum& sum) {
  const u32 l = lane_id();
  const Span* leaves = P.leaves + seg.leaf_base * L;
  const GroupRec* groups = P.groups + seg.grp_base;  // the root level, read in order from HBM
  const u32 vis0 = vis;
  u32 have = 0, skip = skip_first, nsp = 0, first_done = 0;
  Span open{0, 0, 0, 0};
  u32 open_vpos = 0;
  // the group holding leaf a: prefix of the groups' slot counts
  u32 g = 0, base = 0;
  if (a) {
    for (u32 r = 0; r < ng; r += 64) {
      u32 c = r + l < ng ? groups[r + l].cnt : 0u;
      u32 incl = wave_incl_scan(c);
      u32 k = (u32)__popcll(ballot(r + l < ng && incl + base <= a));
      if (k < 64u && r + k < ng) { g = r + k; base += k ? rdlane(incl, k - 1u) : 0u; break; }
      base += rdlane(incl, 63);
    }
  }
  for (u32 idx = a; g < ng && idx < b; g++) {
    u32 blk = uni(groups[g].blk), cnt = uni(groups[g].cnt);
    u32 i0 = idx - base;        // first slot of this group in the range
    base += cnt;
    if (i0 >= cnt) continue;
    u32 iend = b - (base - cnt) < cnt ? b - (base - cnt) : cnt;  // slot bound in this group
    u32 mydl = P.dir_leaf[(seg.blk_base + blk) * GROUP + l];  // 64-slot row: always in bounds
    // 64/L leaves per step: lane l holds entry l%L of leaf i + l/L; the valid entries (packed at
    // the front of each leaf) are then compacted to lanes [0, nn) with one ds_permute, so the
    // scan below sees one contiguous run of entries in document order.  Software pipeline: the
    // next step's loads are in flight while this step is scanned and its spans stored (vmcnt
    // counts stores too, so an unpipelined load would wait behind them).
    constexpr u32 PER = 64u / (u32)L;
    u32 sub = l / (u32)L;
    // (lane-parallel conditions below are bitwise, not short-circuit: && on per-lane values
    // compiles to exec-masked branches; the load is unconditional from a valid leaf, then masked)
    // (the masking happens when the step uses the entries, so a prefetched load is not waited for)
    auto ld = [&](u32 i) -> uint4 {
      u32 li = i + sub;
      u32 leaf = shfl(mydl, li < iend ? li : 0u);
      return *(const uint4*)(leaves + (u64)leaf * L + (l & (u32)(L - 1)));
    };
    // PUB_DEPTH steps of loads in flight (Little's law: one wave's 1 KiB per step is too little to
    // cover HBM latency at 8 waves per SIMD)
    uint4 vn = ld(i0);
#if PUB_DEPTH >= 2
    uint4 vn2 = i0 + PER < iend ? ld(i0 + PER) : uint4{0, 0, 0, 0};
#endif
#if PUB_DEPTH >= 3
    uint4 vn3 = i0 + 2u * PER < iend ? ld(i0 + 2u * PER) : uint4{0, 0, 0, 0};
#endif
    for (u32 i = i0; i < iend; i += PER) {
      uint4 v = vn;
      {  // lanes of leaves past the group's range: empty
        bool in = i + sub < iend;
        v = uint4{in ? v.x : 0u, in ? v.y : 0u, in ? v.z : 0u, in ? v.w : 0u};
      }
#if PUB_DEPTH >= 3
      vn = vn2;
      vn2 = vn3;
      if (i + 3u * PER < iend) vn3 = ld(i + 3u * PER);
#elif PUB_DEPTH >= 2
      vn = vn2;
      if (i + 2u * PER < iend) vn2 = ld(i + 2u * PER);
#else
      if (i + PER < iend) vn = ld(i + PER);
#endif
      u64 VM = ballot(v.w != 0u);
      u32 nn = (u32)__popcll(VM);
      if (PER > 1) {
        u64 below = (1ull << l) - 1ull;
        u32 c1 = (u32)__popcll(VM & below);  // (valid entries below this lane; the empty ones are l - c1)
        u32 dst = v.w != 0u ? c1 : nn + l - c1;
        int ad = (int)(dst << 2);
        v.x = (u32)__builtin_amdgcn_ds_permute(ad, (int)v.x);
        v.y = (u32)__builtin_amdgcn_ds_permute(ad, (int)v.y);
        v.z = (u32)__builtin_amdgcn_ds_permute(ad, (int)v.z);
        v.w = (u32)__builtin_amdgcn_ds_permute(ad, (int)v.w);
      }
      if (nn == 0u) continue;
      bool valid = l < nn;
      Span e{v.x, v.y, v.z, (i32)v.w};
      u32 px = shfl(v.x, l - 1u), py = shfl(v.y, l - 1u), pz = shfl(v.z, l - 1u), pw = shfl(v.w, l - 1u);
      Span prev = l == 0u ? sum.last : Span{px, py, pz, (i32)pw};
      bool app = valid & ((l != 0u) | (have != 0u)) & can_append_b(prev, e);
      bool start = valid & !app;
      u64 M = ballot(start);
      u32 len_u = valid ? v.w : 0u;
      u32 Pl = wave_incl_scan(len_u);  // signed lengths, two's complement sums
      u32 cl = valid && (i32)v.w > 0 ? v.w : 0u;
      u32 V = wave_incl_scan(cl);
      u32 leaf_vis = rdlane(V, 63);
      u64 above = M & ~((2ull << l) - 1ull);
      u32 nxt = above ? (u32)__builtin_ctzll(above) : nn;
      u32 p_end = shfl(Pl, nxt - 1u);
      i32 glen = (i32)(p_end - (Pl - len_u));  // span starting at this lane: lanes [l, nxt)
      u32 fs = M ? (u32)__builtin_ctzll(M) : nn;
      if (have && fs) open.len += (i32)rdlane(Pl, fs - 1u);
      if (!first_done) {
        if (!have) sum.first = Span{rdlane(v.x, 0), rdlane(v.y, 0), rdlane(v.z, 0), (i32)rdlane(v.w, 0)};
      }
      if (M) {
        if (have) {  // the open span closes
          if (!first_done) { sum.lead_len = open.len; first_done = 1; }
          if (WRITE) {
            if (skip) skip = 0;
            else {
              if (l == 0u && out < ccap) {
                canon[out] = open; vpos[out] = open_vpos; corder[out] = open.order;
              }
              out++;
            }
          }
        }
        u32 ls = 63u - (u32)__builtin_clzll(M);
        u32 rank = (u32)__popcll(M & ((1ull << l) - 1ull));
        u32 firsts = (u32)__popcll(M) - 1u;  // spans that also close in this step
        if (!first_done && firsts) { sum.lead_len = (i32)rdlane((u32)glen, fs); first_done = 1; }
        if (WRITE) {
          u32 sk = skip && firsts ? 1u : 0u;  // the skipped first span is the step's first start
          if (start && l != ls && rank >= sk && out + rank - sk < ccap) {
            Span sp{v.x, v.y, v.z, glen};
            canon[out + rank - sk] = sp;
            vpos[out + rank - sk] = vis + V - cl;
            corder[out + rank - sk] = v.x;
          }
          out += firsts - sk;
          if (sk) skip = 0;
        }
        nsp += (u32)__popcll(M);
        open = Span{rdlane(v.x, ls), rdlane(v.y, ls), rdlane(v.z, ls), (i32)rdlane((u32)glen, ls)};
        open_vpos = vis + rdlane(V - cl, ls);
        have = 1;
      }
      sum.last = Span{rdlane(v.x, nn - 1u), rdlane(v.y, nn - 1u), rdlane(v.z, nn - 1u), (i32)rdlane(v.w, nn - 1u)};
      vis += leaf_vis;
    }
    idx = base;
  }
  if (have) {
    if (!first_done) { sum.lead_len = open.len; sum.single = 1; }
    else sum.single = 0;
    if (WRITE && !skip) {
      open.len += extra;
      if (l == 0 && out < ccap) {
        canon[out] = open; vpos[out] = open_vpos; corder[out] = open.order;
      }
      out++;
    }
  }
  sum.spans = nsp;
  sum.vis = vis - vis0;
}

// Order -> canonical span index (replaces a 4 B/order table): a bitmap over the
// orders with a bit at every canonical span's first order, the exclusive count of set bits before
// every word, and the spans listed by first order.  Three sweeps: set the bits (atomic OR: spans
// are in document order, not order order), prefix-count the words, scatter every span to its
// rank.  Per document 2 bits per order + 4 B per span are written instead of 4 B per item order.
// Reads go through L2 (ld_l2): other lanes wrote them.  Wave `wv` of `nwv` takes every nwv-th
// chunk; the word prefix is one contiguous word range per wave plus a cross-wave carry (lds_c:
// nwv u32 of LDS, k_publish_big only).
template <int NWV>
__device__ __forceinline__ void publish_index(const PubOut& O, const DocSeg& seg, const DocState& s, const Span* canon,
                                              u32 out, u32 wv, u32* lds_c) {
  const u32 l = lane_id();
#ifdef PUB_NO_INDEX
  const u32 nw = pub_words(seg.ord_cap), used = 0u;
#else
  const u32 nw = pub_words(seg.ord_cap), used = s.next_order / 32u + 1u;
#endif
  u32* bits = O.pub + seg.pub_base;
  u32* pre = bits + nw;
  u32* sorted = O.sorted + seg.canon_base;
  for (u32 i = wv * 64u + l; i < used; i += 64u * NWV) bits[i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (NWV > 1) __syncthreads();
  for (u32 k0 = wv * 64u; k0 < out; k0 += 64u * NWV) {
    u32 k = k0 + l;
    Span sp = k < out ? canon[k] : Span{0, 0, 0, 0};
#ifndef PUB_NO_INDEX
    // nearby spans share bitmap words: OR each distinct word's bits across the wave first, then
    // one atomic per word (same-address atomics serialise at L2)
    u32 wd = sp.order >> 5, bit = 1u << (sp.order & 31u);
    for (u64 todo = ballot(k < out); todo;) {
      u32 wl = rdlane(wd, (u32)__builtin_ctzll(todo));
      u64 m = ballot(k < out && wd == wl);
      u32 word = wave_or((m >> l) & 1u ? bit : 0u);
      if (l == (u32)__builtin_ctzll(m)) atomicOr(bits + wl, word);
      todo &= ~m;
    }
#endif
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  // word prefix: this wave's contiguous word range [wa, wb), 4 steps per iteration (their loads
  // in flight together)
  const u32 per_wave = ((used + NWV - 1u) / NWV + 63u) & ~63u;
  const u32 wa = wv * per_wave < used ? wv * per_wave : used, wb = wa + per_wave < used ? wa + per_wave : used;
  u32 carry = 0;
  if (NWV > 1) {
    __syncthreads();  // every wave's atomics are done
    u32 t = 0;
    for (u32 i = wa + l; i < wb; i += 64) t += (u32)__popc(ld_l2(bits + i));
    t = wave_sum(t);
    if (l == 0) lds_c[wv] = t;
    __syncthreads();
    u32 c = l < wv ? lds_c[l] : 0u;
    carry = wave_sum(c);
  }
  for (u32 i0 = wa; i0 < wb; i0 += 256) {
    u32 x[4];
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 i = i0 + 64 * u + l;
      x[u] = i < wb ? (u32)__popc(ld_l2(bits + i)) : 0u;
    }
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 i = i0 + 64 * u + l;
      u32 incl = wave_incl_scan(x[u]);
      if (i < wb) pre[i] = carry + incl - x[u];
      carry += rdlane(incl, 63);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (NWV > 1) __syncthreads();
#ifndef PUB_NO_INDEX
  for (u32 k0 = wv * 256u; k0 < out; k0 += 256u * NWV) {
    u32 o[4], r[4];
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 k = k0 + 64 * u + l;
      o[u] = k < out ? canon[k].order : 0u;
    }
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 wd = o[u] >> 5;
      r[u] = ld_l2(pre + wd) + (u32)__popc(ld_l2(bits + wd) & ((1u << (o[u] & 31u)) - 1u));
    }
#pragma unroll
    for (u32 u = 0; u < 4; u++) {
      u32 k = k0 + 64 * u + l;
      if (k < out) sorted[r[u]] = k;
    }
  }
#endif
}

// The digest's other sections (client_with_order, deletes, double deletes, txns + parents,
// frontier) by one wave, and the counts.  Identical to oracle/crdt_oracle.hpp digest().
template <int L>
__device__ __forceinline__ u64 digest_tables(const Pools& P, const DocSeg& seg, const DocState& s, WaveGPU<L>& w) {
  const u32 l = lane_id();
  u64 h = 0;
  const CwoRun* cwo = P.cwo + seg.cwo_base;
  for (u32 k = l; k < s.n_cwo; k += 64) {
    CwoRun r = cwo[k];
    h += elem_hash(2, k, ((u64)r.key << 32) | r.agent, ((u64)r.seq << 32) | r.len);
  }
  const DelRun* dels = P.dels + seg.del_base;
  for (u32 k = l; k < s.n_del; k += 64) {
    DelRun r = dels[k];
    h += elem_hash(3, k, ((u64)r.key << 32) | r.order, r.len);
  }
  const DDRun* dd = P.dd + seg.dd_base * DD_BLK;  // blocks in directory order = the flat RLE
  const DDBlk* ddb = P.ddb + seg.dd_base;
  for (u32 lb = 0, k0 = 0; lb < s.n_ddb; lb++) {
    DDBlk B = w.ldT(ddb + lb);
    if (l < B.cnt) {
      DDRun r = dd[(u64)B.phys * DD_BLK + l];
      h += elem_hash(4, k0 + l, ((u64)r.key << 32) | r.len, r.excess);
    }
    k0 += B.cnt;
  }
  const TxnRec* tx = P.txns + seg.txn_base;
  const u32* par = P.parents + seg.par_base;
  for (u32 k = l; k < s.n_txn; k += 64) {
    TxnRec t = tx[k];
    h += elem_hash(5, k, ((u64)t.order << 32) | t.len, ((u64)t.shadow << 32) | t.pn);
    for (u32 j = 0; j < t.pn; j++) h += elem_hash(6, t.poff + j, par[t.poff + j], k);
  }
  const u32* fr = P.frontier + seg.fr_base;
  for (u32 k = l; k < s.n_fr; k += 64) h += elem_hash(7, k, fr[k], 0);
  return h;
}
__device__ __forceinline__ u64 digest_counts(const DocState& s, u32 out) {
  u64 counts = elem_hash(8, 0, ((u64)s.len << 32) | out, ((u64)s.n_cwo << 32) | s.n_del);
  return counts ^ elem_hash(9, 0, ((u64)s.n_dd << 32) | s.n_txn, ((u64)s.n_fr << 32) | s.n_par);
}

// xw: documents whose bitmap has at most xw words get their order -> span index from k_pub_index
// (launched next); the others build it here.
// (8 waves per SIMD need <= 80 SGPRs: unconstrained, the compiler took 102, i.e. 6 waves per SIMD and
// 8,192 documents in 1.33 rounds)
template <int L>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_publish(Pools P, PubOut O, u32 n, const u32* list, u32 xw) {
  u32 d;
  if (!wave_doc(WAVES_PER_BLOCK, list, n, d)) return;
  WaveGPU<L> w;
  DocState s = w.ldT(P.st + d);
  DocSeg seg = w.ld_seg(P.seg + d);
  u32 l = lane_id();
  if ((s.status != ST_OK && s.status != ST_NEED_CAPACITY) || s.next_order >= seg.ord_cap) {
    if (l == 0) { O.canon_n[d] = 0; O.len[d] = s.len; O.digest[d] = 0; }
    return;
  }
  Span* canon = O.canon + seg.canon_base;
  u32* vpos = O.vpos + seg.canon_base;
  u32 out = 0, vis = 0;
  RangeSum sum{};
  compact_range<L, true>(P, seg, s.ng, 0u, s.n_leaves, canon, vpos, O.corder + seg.canon_base, seg.canon_cap,
                         out, vis, 0u, 0, sum);
  if (out > seg.canon_cap) {  // canonical spans beyond the planned capacity: report, never write past it
    if (l == 0) { O.canon_n[d] = 0; O.len[d] = s.len; O.digest[d] = 0; }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (pub_words(seg.ord_cap) > xw) publish_index<1>(O, seg, s, canon, out, 0u, nullptr);
  if (l == 0) {
    O.canon_n[d] = out;
    O.len[d] = s.len;
    O.digest[d] = DIGEST_PENDING;  // (k_digest computes it on request)
  }
}

// Long documents: one workgroup of PUB_BIG_WAVES waves per listed document.
template <int L>
__global__ __launch_bounds__(64 * PUB_BIG_WAVES) void k_publish_big(Pools P, PubOut O, const u32* list) {
  constexpr u32 NWV = PUB_BIG_WAVES;
  __shared__ RangeSum s_sum[NWV];
  __shared__ u32 s_base[NWV], s_vbase[NWV], s_skip[NWV], s_c[NWV], s_total;
  __shared__ i32 s_extra[NWV];
  const u32 d = list[blockIdx.x];
  const u32 l = lane_id(), wv = uni(threadIdx.x >> 6);
  WaveGPU<L> w;
  DocState s = w.ldT(P.st + d);
  DocSeg seg = w.ld_seg(P.seg + d);
  if ((s.status != ST_OK && s.status != ST_NEED_CAPACITY) || s.next_order >= seg.ord_cap) {
    if (threadIdx.x == 0) { O.canon_n[d] = 0; O.len[d] = s.len; O.digest[d] = 0; }
    return;
  }
  Span* canon = O.canon + seg.canon_base;
  u32* vpos = O.vpos + seg.canon_base;
  // this wave's leaves (every range holds leaves: the host sends only documents with many)
  const u32 a = (u32)((u64)s.n_leaves * wv / NWV), b = (u32)((u64)s.n_leaves * (wv + 1u) / NWV);
  u32 out = 0, vis = 0;
  RangeSum sum{};
  u32* corder = O.corder + seg.canon_base;
  compact_range<L, false>(P, seg, s.ng, a, b, canon, vpos, corder, seg.canon_cap, out, vis, 0u, 0, sum);
  if (l == 0) s_sum[wv] = sum;
  __syncthreads();
  if (wv == 0) {  // boundary resolution, lane = range
    RangeSum me = s_sum[l < NWV ? l : 0u];
    Span prv = s_sum[l > 0u && l <= NWV ? l - 1u : 0u].last;
    u32 merge = l > 0u && l < NWV && can_append(prv, me.first);
    u32 cnt = l < NWV ? me.spans - merge : 0u;
    u32 ci = wave_incl_scan(cnt), vi = wave_incl_scan(l < NWV ? me.vis : 0u);
    if (l < NWV) { s_base[l] = ci - cnt; s_vbase[l] = vi - me.vis; s_skip[l] = merge; }
    if (l == 0) s_total = rdlane(ci, NWV - 1u);
    // extra_r = merge_{r+1} ? lead_{r+1} + (single_{r+1} ? extra_{r+1} : 0) : 0, from the last range back
    i32 extra = 0;
    for (i32 r = (i32)NWV - 1; r >= 0; r--) {
      u32 mr = rdlane(merge, (u32)r + 1u < NWV ? (u32)r + 1u : 0u) & ((u32)r + 1u < NWV);
      i32 nx = (i32)rdlane((u32)me.lead_len, (u32)r + 1u < NWV ? (u32)r + 1u : 0u);
      u32 sg = rdlane(me.single, (u32)r + 1u < NWV ? (u32)r + 1u : 0u);
      extra = mr ? nx + (sg ? extra : 0) : 0;
      if (l == 0) s_extra[r] = extra;
    }
  }
  __syncthreads();
  out = s_base[wv];
  vis = s_vbase[wv];
  RangeSum sum2{};
  compact_range<L, true>(P, seg, s.ng, a, b, canon, vpos, corder, seg.canon_cap, out, vis, s_skip[wv], s_extra[wv],
                         sum2);
  const u32 total = s_total;
  if (total > seg.canon_cap) {
    if (threadIdx.x == 0) { O.canon_n[d] = 0; O.len[d] = s.len; O.digest[d] = 0; }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  publish_index<NWV>(O, seg, s, canon, total, wv, s_c);
  if (threadIdx.x == 0) {
    O.canon_n[d] = total;
    O.len[d] = s.len;
    O.digest[d] = DIGEST_PENDING;  // (k_digest computes it on request)
  }
}

// k_digest: the 64-bit state digest of every published document (oracle/crdt_oracle.hpp digest():
// canonical spans, then the RLE tables and the counts), one wave per document, run on request
// (crdt_digest, crdt_digest_dev_async) after a publish -- the digest is the parity checker's
// summary of a state, not part of the flat index the queries read, so publish does not compute
// it.  Documents publish refused (not OK, or past their planned index capacity) keep digest 0.
template <int L>
__global__ __launch_bounds__(256) void k_digest(Pools P, PubOut O, u32 n) {
  u32 d;
  if (!wave_doc(WAVES_PER_BLOCK, nullptr, n, d)) return;
  if (O.digest[d] != DIGEST_PENDING) return;
  WaveGPU<L> w;
  DocState s = w.ldT(P.st + d);
  DocSeg seg = w.ld_seg(P.seg + d);
  const u32 l = lane_id();
  const u32 out = O.canon_n[d];
  const Span* canon = O.canon + seg.canon_base;
  u64 h = 0;
  for (u32 k = l; k < out; k += 64) h += span_hash(k, canon[k]);
  h += digest_tables<L>(P, seg, s, w);
  h = wave_sum64(h);
  if (l == 0) O.digest[d] = mix64(h ^ digest_counts(s, out));
}

// ---------------------------------------------------------------------------------------------
// k_pub_index: the order -> span index (publish_index's three sweeps) of the documents k_publish
// left it to, one PUBX_THREADS block per document, with the bitmap in LDS: the bits are set with
// LDS atomics (ds_or) instead of one global atomic per distinct word, and the word prefix and the
// scatter's ranks read LDS instead of L2.  Global traffic per document: the span first orders
// (corder, 4 B per span) twice, the bitmap and its word prefix written once, the rank -> span
// table scattered once.  LDS: xw bitmap words + an exclusive prefix per 8-word group.
// ---------------------------------------------------------------------------------------------
#define PUBX_THREADS 256
#define PUBX_MAX_WORDS 16384u  // bitmaps up to 524,288 orders (72 KiB of LDS: two blocks per CU)
CRDT_HD u32 pubx_lds_bytes(u32 xw) { return (xw + xw / 8u + 1u) * 4u; }

__global__ __launch_bounds__(PUBX_THREADS) void k_pub_index(Pools P, PubOut O, const u32* list, u32 xw) {
  extern __shared__ u32 xl[];
  __shared__ u32 s_w[PUBX_THREADS / 64];
  u32* lb = xl;       // [xw] bitmap
  u32* lg = xl + xw;  // [xw / 8 + 1] set bits in the 8-word groups before each group
  const u32 d = list ? list[blockIdx.x] : blockIdx.x;
  const u32 t = threadIdx.x;
  const DocState* sp = P.st + d;
  const DocSeg seg = P.seg[d];
  const i32 status = sp->status;
  const u32 next_order = sp->next_order;
  if ((status != ST_OK && status != ST_NEED_CAPACITY) || next_order >= seg.ord_cap) return;
  const u32 nw = pub_words(seg.ord_cap);
  if (nw > xw) return;  // k_publish built this one
  const u32 out = O.canon_n[d];  // 0 when k_publish refused the document
  const u32 used = next_order / 32u + 1u;  // <= nw
  const u32* co = O.corder + seg.canon_base;
  u32* bits = O.pub + seg.pub_base;
  u32* pre = bits + nw;
  u32* sorted = O.sorted + seg.canon_base;
  for (u32 i = t; i < used; i += PUBX_THREADS) lb[i] = 0u;
  __syncthreads();
  // (corder sweeps 8 loads per thread at a time: one dependent HBM wait per 8 spans, not per span)
  for (u32 k0 = t; k0 < out; k0 += 8u * PUBX_THREADS) {
    u32 ov[8];
#pragma unroll
    for (u32 u = 0; u < 8u; u++) {
      u32 k = k0 + u * PUBX_THREADS;
      ov[u] = k < out ? co[k] : INVALID;
    }
#pragma unroll
    for (u32 u = 0; u < 8u; u++)
      if (ov[u] != INVALID) atomicOr(lb + (ov[u] >> 5), 1u << (ov[u] & 31u));
  }
  __syncthreads();
  // group prefix: thread t owns groups [g0, g1)
  const u32 ngr = (used + 7u) / 8u, per = (ngr + PUBX_THREADS - 1u) / PUBX_THREADS;
  const u32 g0 = t * per < ngr ? t * per : ngr, g1 = g0 + per < ngr ? g0 + per : ngr;
  u32 c = 0;
  for (u32 i = g0 * 8u; i < g1 * 8u && i < used; i++) c += (u32)__popc(lb[i]);
  const u32 incl = wave_incl_scan(c);
  if ((t & 63u) == 63u) s_w[t >> 6] = incl;
  __syncthreads();
  u32 run = incl - c;
  for (u32 wv = 0; wv < (t >> 6); wv++) run += s_w[wv];
  for (u32 g = g0; g < g1; g++) {
    lg[g] = run;
    for (u32 i = g * 8u; i < g * 8u + 8u && i < used; i++) run += (u32)__popc(lb[i]);
  }
  __syncthreads();
  // the bitmap and its word prefix, written once (coalesced)
  for (u32 i = t; i < used; i += PUBX_THREADS) {
    u32 r = lg[i >> 3];
    for (u32 j = i & ~7u; j < i; j++) r += (u32)__popc(lb[j]);
    bits[i] = lb[i];
    pre[i] = r;
  }
  // rank -> span
  for (u32 k0 = t; k0 < out; k0 += 8u * PUBX_THREADS) {
    u32 ov[8];
#pragma unroll
    for (u32 u = 0; u < 8u; u++) {
      u32 k = k0 + u * PUBX_THREADS;
      ov[u] = k < out ? co[k] : INVALID;
    }
#pragma unroll
    for (u32 u = 0; u < 8u; u++) {
      u32 o = ov[u];
      if (o == INVALID) continue;
      u32 wd = o >> 5;
      u32 r = lg[wd >> 3];
      for (u32 j = wd & ~7u; j < wd; j++) r += (u32)__popc(lb[j]);
      r += (u32)__popc(lb[wd] & ((1u << (o & 31u)) - 1u));
      sorted[r] = k0 + u * PUBX_THREADS;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Text materialisation.  The reference keeps a rope in step with the tree when
// USE_INNER_ROPE is on: insert the content at cursor.count_pos() (doc.rs:230-233), remove the
// deleted visible range (doc.rs:430-432; the remote delete arm is todo!() at doc.rs:329-333).
// The rope therefore always equals "content of the visible items in document order", which is
// what this kernel writes from the published index: for canonical span k with len > 0,
// text[vpos[k] + i] = content[order_k + i].  Content is an order-indexed UTF-32 table (entries at
// delete orders are never read).
// ---------------------------------------------------------------------------------------------
#define NO_CONTENT 0xFFFFFFFFFFFFFFFFull

struct TextIO {
  const u32* content;  // order-indexed code points: document d reads content[cbase[d] + order]
  const u64* cbase;    // [doc] (NO_CONTENT: no content staged)
  const u64* clen;     // [doc] entries available from cbase
  u32* text;           // [ord_base + pos]
  u32* tlen;           // [doc] visible chars written, INVALID if not materialised
  u64* tdigest;        // [doc] text digest (0 if not materialised)
};

// text digest, identical in oracle/crdt_oracle.hpp (text_digest): a 32-bit murmur3 finaliser per
// (position, code point), summed in 64 bits, mixed once at the end (full-rate-friendly: two 32-bit
// multiplies per char instead of a 64-bit splitmix)
__device__ __forceinline__ u32 text_hash(u32 pos, u32 cp) {
  u32 h = (pos * 0x9E3779B1u) ^ cp;
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

// One block (MAT_WAVES waves) per document; wave w takes chunks w, w+MAT_WAVES, ... of 64
// canonical spans (each chunk's output starts at vpos[k0], so chunks are independent).  Within a
// chunk a prefix scan of the visible lengths gives each output position j; lane l owns positions
// t+l and finds its span through LDS start flags (below), so stores are fully coalesced
// (contiguous positions) and loads are contiguous within a span.  U positions per lane are in
// flight per step.
#define MAT_WAVES 4
template <int L>
__global__ __launch_bounds__(64 * MAT_WAVES) void k_materialize(Pools P, PubOut O, TextIO T, u32 n) {
  u32 d = blockIdx.x;
  if (d >= n) return;
  u32 l = lane_id();
  u32 wv = uni(threadIdx.x >> 6);
  __shared__ u64 s_h[MAT_WAVES];
  i32 stt = P.st[d].status;
  u32 next_order = P.st[d].next_order;
  u64 cb = T.cbase[d], cl = T.clen[d];
  if ((stt != ST_OK && stt != ST_NEED_CAPACITY) || cb == NO_CONTENT || cl < (u64)next_order) {
    if (threadIdx.x == 0) { T.tlen[d] = INVALID; T.tdigest[d] = 0; }
    return;
  }
  DocSeg seg = P.seg[d];
  const Span* cn = O.canon + seg.canon_base;
  const u32* vp = O.vpos + seg.canon_base;
  u32 ns = O.canon_n[d];
  const u32* src = T.content + cb;
  u32* dst = T.text + seg.ord_base;
  constexpr u32 U = 4;
  // span of output position j: spans with visible items flag their first position in a 64-slot
  // LDS row per window (tag = step number, no clearing) together with base = order - start;
  // position j takes the highest flag at or below it, else the last span starting at or before
  // the window (a uniform readlane).  Two LDS writes, one ballot and one LDS read per window
  // instead of a 6-step bpermute search.
  __shared__ u32 s_tag[MAT_WAVES][U][64], s_base[MAT_WAVES][U][64];
#pragma unroll
  for (u32 u = 0; u < U; u++) s_tag[wv][u][l] = ~0u;
  u32 tag = 0;
  u64 h = 0;
  for (u32 k0 = wv * 64; k0 < ns; k0 += 64 * MAT_WAVES) {
    u32 k = k0 + l;
    Span sp = k < ns ? cn[k] : Span{0, 0, 0, 0};
    u32 ln = sp.len > 0 ? (u32)sp.len : 0u;
    u32 base = uni(vp[k0]);
    u32 Pi = wave_incl_scan(ln);
    u32 Tn = rdlane(Pi, 63);
    u32 st = Pi - ln;            // first output position of span k within the chunk
    u32 ob = sp.order - st;      // content index of position j in span k = ob + j
    for (u32 t = 0; t < Tn; t += 64 * U) {
      ++tag;
#pragma unroll
      for (u32 u = 0; u < U; u++) {
        u32 tu = t + u * 64;
        if (ln > 0 && st >= tu && st - tu < 64u) {
          s_tag[wv][u][st - tu] = tag;
          s_base[wv][u][st - tu] = ob;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      u32 cp[U], jj[U];
#pragma unroll
      for (u32 u = 0; u < U; u++) {
        u32 tu = t + u * 64;
        u32 j = tu + l;
        u64 hm = ballot(s_tag[wv][u][l] == tag) & ((2ull << l) - 1ull);
        u64 B0 = ballot(ln > 0 && st <= tu);
        u32 lt = B0 ? 63u - (u32)__builtin_clzll(B0) : 0u;
        u32 b = hm ? s_base[wv][u][63u - (u32)__builtin_clzll(hm)] : rdlane(ob, lt);
        jj[u] = j;
        cp[u] = j < Tn ? src[b + j] : 0u;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
      for (u32 u = 0; u < U; u++) {
        if (jj[u] < Tn) {
          dst[base + jj[u]] = cp[u];
          h += text_hash(base + jj[u], cp[u]);
        }
      }
    }
  }
  h = wave_sum64(h);
  if (l == 0) s_h[wv] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 hs = 0;
    for (u32 w = 0; w < MAT_WAVES; w++) hs += s_h[w];
    u32 len = O.len[d];
    T.tlen[d] = len;
    T.tdigest[d] = mix64(hs ^ ((u64)len << 32 | 0x54ull));
  }
}

template <class T>
__device__ __forceinline__ i32 find_run(const T* b, u32 n, u32 x) {  // simple_rle.rs:18-25 search
  u32 lo = 0, hi = n;
  while (lo < hi) {
    u32 mid = (lo + hi) >> 1;
    u32 k = ((const u32*)&b[mid])[0];
    u32 ln = WaveGPU<32>::rlen(b[mid]);
    if (x < k) hi = mid;
    else if (x >= k + ln) lo = mid + 1;
    else return (i32)mid;
  }
  return -1;
}

template <int L>
__global__ void k_pos_to_loc(Pools P, PubOut O, u32 n_docs, u64 nq, const u32* doc, const u32* pos, u16* agent, u32* seq) {
  for (u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (u64)gridDim.x * blockDim.x) {
    u32 d = doc[q], p = pos[q];
    u16 a = 0xFFFF;
    u32 sq = INVALID;
    if (d < n_docs) {
      i32 stt = P.st[d].status;
      if ((stt == ST_OK || stt == ST_NEED_CAPACITY) && p < O.len[d]) {
        DocSeg seg = P.seg[d];
        const u32* vp = O.vpos + seg.canon_base;
        const Span* cn = O.canon + seg.canon_base;
        u32 lo = 0, hi = O.canon_n[d];
        while (lo < hi) {
          u32 mid = (lo + hi) >> 1;
          if (vp[mid] <= p) lo = mid + 1; else hi = mid;
        }
        u32 k = lo - 1;
        u32 order = cn[k].order + (p - vp[k]);
        const CwoRun* cw = P.cwo + seg.cwo_base;
        i32 r = find_run(cw, P.st[d].n_cwo, order);
        if (r >= 0) { a = (u16)cw[r].agent; sq = cw[r].seq + (order - cw[r].key); }
      }
    }
    agent[q] = a;
    seq[q] = sq;
  }
}

// pos -> loc for a query batch whose queries come in runs per document (the usual shape: a
// document's cursors, or a batch sorted by document): block b answers queries
// [b * QBLK_Q, (b + 1) * QBLK_Q).  When they all name one document whose visible prefix vpos fits
// QBLK_MAX entries, the block stages vpos in LDS with coalesced loads (each entry read from HBM
// once per block instead of ~log2(spans) dependent gathers per query) and every query's binary
// search runs in LDS; any other chunk answers thread by thread from HBM, as k_pos_to_loc.
#define QBLK_Q 4096u
#define QBLK_T 1024u    // threads per block (16 waves: one block per CU holds the LDS)
#define QBLK_MAX 36864u  // 144 KiB of LDS
#define QBLK_CWO 512u    // client_with_order runs staged with it (8 KiB)
#define QBLK_LDS (QBLK_MAX * 4u + QBLK_CWO * 16u)
template <int L>
__global__ __launch_bounds__(QBLK_T) void k_pos_to_loc_blk(Pools P, PubOut O, u32 n_docs, u64 nq, const u32* doc, const u32* pos,
                                                        u16* agent, u32* seq) {
  extern __shared__ u32 s_vp[];
  __shared__ u32 s_mixed;
  const u32 t = threadIdx.x;
  const u64 q0 = (u64)blockIdx.x * QBLK_Q;
  const u64 q1 = q0 + QBLK_Q < nq ? q0 + QBLK_Q : nq;
  const u32 d0 = doc[q0];
  if (t == 0) s_mixed = 0;
  __syncthreads();
  u32 mixed = 0;
#pragma unroll
  for (u32 j = 0; j < QBLK_Q / QBLK_T; j++) {  // (unrolled: the loads are in flight together)
    u64 q = q0 + (u64)j * QBLK_T + t;
    mixed |= (q < q1 && doc[q] != d0) ? 1u : 0u;
  }
  if (mixed) s_mixed = 1;  // (any writer stores the same value)
  __syncthreads();
  bool staged = false;
  u32 cn = 0, dlen = 0, ncwo = 0;
  DocSeg seg{};
  if (!s_mixed && d0 < n_docs) {
    i32 stt = P.st[d0].status;
    cn = O.canon_n[d0];
    if ((stt == ST_OK || stt == ST_NEED_CAPACITY) && cn <= QBLK_MAX) {
      seg = P.seg[d0];
      dlen = O.len[d0];
      ncwo = P.st[d0].n_cwo;
      const u32* vp = O.vpos + seg.canon_base;
      for (u32 i0 = 0; i0 < cn; i0 += QBLK_T * 16u) {  // 16 loads per thread in flight per step
        u32 v[16];
#pragma unroll
        for (u32 u = 0; u < 16u; u++) {
          u32 i = i0 + u * QBLK_T + t;
          v[u] = i < cn ? vp[i] : 0u;
        }
#pragma unroll
        for (u32 u = 0; u < 16u; u++) {
          u32 i = i0 + u * QBLK_T + t;
          if (i < cn) s_vp[i] = v[u];
        }
      }
      staged = true;
    }
  }
  __syncthreads();
  if (!staged) {  // mixed chunk, long document or a failed one: per-thread search in HBM
    for (u64 q = q0 + t; q < q1; q += QBLK_T) {
      u32 d = doc[q], p = pos[q];
      u16 a = 0xFFFF;
      u32 sq = INVALID;
      if (d < n_docs) {
        i32 stt = P.st[d].status;
        if ((stt == ST_OK || stt == ST_NEED_CAPACITY) && p < O.len[d]) {
          DocSeg sg = P.seg[d];
          const u32* vp = O.vpos + sg.canon_base;
          u32 lo = 0, hi = O.canon_n[d];
          while (lo < hi) {
            u32 mid = (lo + hi) >> 1;
            if (vp[mid] <= p) lo = mid + 1; else hi = mid;
          }
          u32 k = lo - 1;
          u32 order = O.canon[sg.canon_base + k].order + (p - vp[k]);
          const CwoRun* cw = P.cwo + sg.cwo_base;
          i32 r = find_run(cw, P.st[d].n_cwo, order);
          if (r >= 0) { a = (u16)cw[r].agent; sq = cw[r].seq + (order - cw[r].key); }
        }
      }
      agent[q] = a;
      seq[q] = sq;
    }
    return;
  }
  // 16 queries per thread in three sweeps, so that each sweep's independent loads are in flight
  // together: binary searches in LDS, then the spans' first orders (corder, 4 B per span), then
  // client_with_order runs (staged in LDS too when the table is short)
  const u32* co = O.corder + seg.canon_base;
  const CwoRun* cw = P.cwo + seg.cwo_base;
  CwoRun* s_cw = (CwoRun*)(s_vp + QBLK_MAX);
  const bool cw_lds = ncwo <= QBLK_CWO;
  if (cw_lds) {
    for (u32 i = t; i < ncwo; i += QBLK_T) s_cw[i] = cw[i];
  }
  __syncthreads();
  constexpr u32 QPT = QBLK_Q / QBLK_T;
  u32 kk[QPT], pp[QPT];
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u64 q = q0 + (u64)j * QBLK_T + t;
    pp[j] = q < q1 ? pos[q] : INVALID;
    kk[j] = 0u;
  }
  // the 16 searches in lockstep (the halving sequence depends only on cn), so each step's 16 LDS
  // reads are in flight together: kk = the last span whose vpos <= p
  for (u32 n = cn; n > 1u;) {
    u32 half = n >> 1;
#pragma unroll
    for (u32 j = 0; j < QPT; j++) kk[j] = s_vp[kk[j] + half] <= pp[j] ? kk[j] + half : kk[j];
    n -= half;
  }
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u32 p = pp[j];
    if (p < dlen) pp[j] = p - s_vp[kk[j]];  // (vpos[0] = 0 <= p: kk is a span)
    else kk[j] = INVALID;
  }
#pragma unroll
  for (u32 j = 0; j < QPT; j++) pp[j] = kk[j] != INVALID ? co[kk[j]] + pp[j] : INVALID;  // orders
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u64 q = q0 + (u64)j * QBLK_T + t;
    if (q >= q1) break;
    u16 a = 0xFFFF;
    u32 sq = INVALID;
    if (kk[j] != INVALID) {
      u32 order = pp[j];
      i32 r = cw_lds ? find_run(s_cw, ncwo, order) : find_run(cw, ncwo, order);
      if (r >= 0) {
        CwoRun c = cw_lds ? s_cw[r] : cw[r];
        a = (u16)c.agent;
        sq = c.seq + (order - c.key);
      }
    }
    agent[q] = a;
    seq[q] = sq;
  }
}

// loc -> pos in the same 4,096-query chunks: a one-document chunk stages the used words of its
// span-start bitmap and their prefix counts in LDS (coalesced), so order -> span rank is two LDS
// reads; the agent's item_orders run, the rank -> span entry and the span itself are gathered in
// sweeps with every thread's queries in flight together.  Other chunks: as k_loc_to_pos.
#define QBLK_W 16384u  // bitmap words staged (+ as many prefix words: 128 KiB)
template <int L>
__global__ __launch_bounds__(QBLK_T) void k_loc_to_pos_blk(Pools P, PubOut O, u32 n_docs, u64 nq, const u32* doc, const u16* agent,
                                                         const u32* seq, u32* pos, u8* deleted) {
  extern __shared__ u32 s_bw[];  // [0, used) bitmap words, [QBLK_W, QBLK_W + used) prefixes
  __shared__ u32 s_mixed;
  const u32 t = threadIdx.x;
  const u64 q0 = (u64)blockIdx.x * QBLK_Q;
  const u64 q1 = q0 + QBLK_Q < nq ? q0 + QBLK_Q : nq;
  const u32 d0 = doc[q0];
  if (t == 0) s_mixed = 0;
  __syncthreads();
  u32 mixed = 0;
#pragma unroll
  for (u32 j = 0; j < QBLK_Q / QBLK_T; j++) {
    u64 q = q0 + (u64)j * QBLK_T + t;
    mixed |= (q < q1 && doc[q] != d0) ? 1u : 0u;
  }
  if (mixed) s_mixed = 1;
  __syncthreads();
  bool staged = false;
  DocState st{};
  DocSeg seg{};
  u32 used = 0, cn = 0;
  if (!s_mixed && d0 < n_docs) {
    st = P.st[d0];
    used = st.next_order / 32u + 1u;
    if ((st.status == ST_OK || st.status == ST_NEED_CAPACITY) && used <= QBLK_W) {
      seg = P.seg[d0];
      cn = O.canon_n[d0];
      u32 nw = pub_words(seg.ord_cap);
      const u32* bits = O.pub + seg.pub_base;
      for (u32 i = t; i < used; i += QBLK_T) {
        u32 b = i < nw ? bits[i] : 0u, c = i < nw ? bits[nw + i] : 0u;
        s_bw[i] = b;
        s_bw[QBLK_W + i] = c;
      }
      staged = true;
    }
  }
  __syncthreads();
  if (!staged) {
    for (u64 q = q0 + t; q < q1; q += QBLK_T) {
      u32 d = doc[q];
      u32 ps = INVALID;
      u8 dl = 2;
      if (d < n_docs) {
        DocState s = P.st[d];
        if ((s.status == ST_OK || s.status == ST_NEED_CAPACITY) && agent[q] < s.n_agents) {
          DocSeg sg = P.seg[d];
          AgentRec A = P.agents[sg.agent_base + agent[q]];
          const ARun* ar = P.arun + sg.arun_base + A.run_base;
          i32 r = find_run(ar, A.run_cnt, seq[q]);
          if (r >= 0) {
            u32 order = ar[r].order + (seq[q] - ar[r].key);
            u32 k = span_of_order(O, sg, O.canon_n[d], order);
            if (k != INVALID) {
              Span sp = O.canon[sg.canon_base + k];
              ps = O.vpos[sg.canon_base + k] + (sp.len > 0 ? order - sp.order : 0u);
              dl = sp.len < 0 ? 1 : 0;
            }
          }
        }
      }
      pos[q] = ps;
      deleted[q] = dl;
    }
    return;
  }
  constexpr u32 QPT = QBLK_Q / QBLK_T;
  u32 od[QPT], kk[QPT];
  // sweep 1: (agent, seq) -> order (the agent's item_orders runs)
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u64 q = q0 + (u64)j * QBLK_T + t;
    od[j] = INVALID;
    if (q < q1) {
      u32 a = agent[q], sq = seq[q];
      if (a < st.n_agents) {
        AgentRec A = P.agents[seg.agent_base + a];
        const ARun* ar = P.arun + seg.arun_base + A.run_base;
        i32 r = find_run(ar, A.run_cnt, sq);
        if (r >= 0) od[j] = ar[r].order + (sq - ar[r].key);
      }
    }
  }
  // sweep 2: order -> span rank in LDS, rank -> span index (gathered together)
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u32 o = od[j], wd = o >> 5;
    u32 r = wd < used ? s_bw[QBLK_W + wd] + (u32)__popc(s_bw[wd] & (0xFFFFFFFFu >> (31u - (o & 31u)))) : 0u;
    kk[j] = (o != INVALID && r != 0u && r <= cn) ? O.sorted[seg.canon_base + r - 1u] : INVALID;
  }
  // sweep 3: the span and its visible prefix
#pragma unroll
  for (u32 j = 0; j < QPT; j++) {
    u64 q = q0 + (u64)j * QBLK_T + t;
    if (q >= q1) break;
    u32 ps = INVALID;
    u8 dl = 2;
    u32 k = kk[j];
    if (k < cn) {
      Span sp = O.canon[seg.canon_base + k];
      u32 o = od[j];
      if (o - sp.order < slen(sp)) {
        ps = O.vpos[seg.canon_base + k] + (sp.len > 0 ? o - sp.order : 0u);
        dl = sp.len < 0 ? 1 : 0;
      }
    }
    pos[q] = ps;
    deleted[q] = dl;
  }
}

template <int L>
__global__ void k_loc_to_pos(Pools P, PubOut O, u32 n_docs, u64 nq, const u32* doc, const u16* agent, const u32* seq, u32* pos, u8* deleted) {
  for (u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (u64)gridDim.x * blockDim.x) {
    u32 d = doc[q];
    u32 ps = INVALID;
    u8 dl = 2;
    if (d < n_docs) {
      DocState s = P.st[d];
      if ((s.status == ST_OK || s.status == ST_NEED_CAPACITY) && agent[q] < s.n_agents) {
        DocSeg seg = P.seg[d];
        AgentRec A = P.agents[seg.agent_base + agent[q]];
        const ARun* ar = P.arun + seg.arun_base + A.run_base;
        i32 r = find_run(ar, A.run_cnt, seq[q]);
        if (r >= 0) {
          u32 order = ar[r].order + (seq[q] - ar[r].key);
          u32 k = span_of_order(O, seg, O.canon_n[d], order);
          if (k != INVALID) {
            Span sp = O.canon[seg.canon_base + k];
            ps = O.vpos[seg.canon_base + k] + (sp.len > 0 ? order - sp.order : 0u);
            dl = sp.len < 0 ? 1 : 0;
          }
        }
      }
    }
    pos[q] = ps;
    deleted[q] = dl;
  }
}

// pos -> loc for sorted query batches by merge path (BASELINE north_star's sorted batches): a
// chunk of QBLK_Q queries that name one document, positions ascending, is merged against the
// document's visible prefix vpos[0..cn) (ascending, vpos[0] = 0) tile by tile.  vpos streams
// through LDS in QM_TILE-entry tiles (coalesced, the next tile's loads in flight while the current
// one is searched); the queries of a tile are the contiguous run of the sorted chunk below the
// next tile's first entry, and each searches only its tile (Cursor at content pos, root.rs:54-88).
// vpos is read once per chunk and the LDS footprint is small (24 KiB), so several chunks run per
// CU -- unlike k_pos_to_loc_blk, which stages the whole prefix (up to 144 KiB) first.  Pass 1
// writes each query's order into seq[], pass 2 maps orders to (agent, seq) through
// client_with_order.  A mixed or unsorted chunk is answered per thread.
#define QM_T 256u
#define QM_TILE 2048u
template <int L>
__global__ __launch_bounds__(QM_T) void k_pos_to_loc_merge(Pools P, PubOut O, u32 n_docs, u64 nq, const u32* doc, const u32* pos,
                                                          u16* agent, u32* seq) {
  __shared__ u32 s_q[QBLK_Q];
  __shared__ u32 s_a[QM_TILE];
  __shared__ u32 s_bad;
  const u32 t = threadIdx.x;
  const u64 q0 = (u64)blockIdx.x * QBLK_Q;
  const u64 q1 = q0 + QBLK_Q < nq ? q0 + QBLK_Q : nq;
  const u32 nb = (u32)(q1 - q0);
  const u32 d0 = doc[q0];
  if (t == 0) s_bad = 0;
  for (u32 j = t; j < nb; j += QM_T) s_q[j] = pos[q0 + j];
  __syncthreads();
  u32 bad = 0;
  for (u32 j = t; j < nb; j += QM_T) {  // one document, positions ascending
    bad |= doc[q0 + j] != d0 ? 1u : 0u;
    if (j) bad |= s_q[j - 1] > s_q[j] ? 1u : 0u;
  }
  if (bad) s_bad = 1;  // (any writer stores the same value)
  __syncthreads();
  i32 stt = d0 < n_docs ? P.st[d0].status : ST_BAD_INPUT;
  if (s_bad || d0 >= n_docs || !(stt == ST_OK || stt == ST_NEED_CAPACITY)) {
    for (u64 q = q0 + t; q < q1; q += QM_T) {
      u32 d = doc[q], p = pos[q];
      u16 a = 0xFFFF;
      u32 sq = INVALID;
      if (d < n_docs) {
        i32 s2 = P.st[d].status;
        if ((s2 == ST_OK || s2 == ST_NEED_CAPACITY) && p < O.len[d]) {
          DocSeg sg = P.seg[d];
          const u32* vp = O.vpos + sg.canon_base;
          u32 lo = 0, hi = O.canon_n[d];
          while (lo < hi) {
            u32 mid = (lo + hi) >> 1;
            if (vp[mid] <= p) lo = mid + 1; else hi = mid;
          }
          u32 k = lo - 1;
          u32 order = O.corder[sg.canon_base + k] + (p - vp[k]);
          const CwoRun* cw = P.cwo + sg.cwo_base;
          i32 r = find_run(cw, P.st[d].n_cwo, order);
          if (r >= 0) { a = (u16)cw[r].agent; sq = cw[r].seq + (order - cw[r].key); }
        }
      }
      agent[q] = a;
      seq[q] = sq;
    }
    return;
  }
  const DocSeg sg = P.seg[d0];
  const u32 cn = O.canon_n[d0], dlen = O.len[d0];
  const u32* A = O.vpos + sg.canon_base;
  const u32* co = O.corder + sg.canon_base;
  constexpr u32 PT = QM_TILE / QM_T;  // tile entries per thread
  u32 nx[PT];
#pragma unroll
  for (u32 u = 0; u < PT; u++) nx[u] = u * QM_T + t < cn ? A[u * QM_T + t] : 0u;
  u32 qa = 0;  // queries [0, qa) answered
  for (u32 ts = 0; ts < cn && qa < nb; ts += QM_TILE) {
    const u32 tn = cn - ts < QM_TILE ? cn - ts : QM_TILE;
#pragma unroll
    for (u32 u = 0; u < PT; u++) s_a[u * QM_T + t] = nx[u];
    const u32 te = ts + QM_TILE;
    const u32 bound = te < cn ? A[te] : INVALID;  // the next tile's first entry (queries below it are here)
#pragma unroll
    for (u32 u = 0; u < PT; u++) nx[u] = te + u * QM_T + t < cn ? A[te + u * QM_T + t] : 0u;  // next tile, in flight
    __syncthreads();
    // this tile's queries: [qa, qb), qb = the first query >= bound (every thread alike)
    u32 lo = qa, hi = nb;
    while (lo < hi) {
      u32 mid = (lo + hi) >> 1;
      if (s_q[mid] < bound) lo = mid + 1; else hi = mid;
    }
    const u32 qb = bound == INVALID ? nb : lo;
    for (u32 j = qa + t; j < qb; j += QM_T) {
      u32 p = s_q[j];
      u32 l2 = 0, h2 = tn;  // the last tile entry <= p (s_a[0] <= p: earlier queries are answered)
      while (l2 < h2) {
        u32 mid = (l2 + h2) >> 1;
        if (s_a[mid] <= p) l2 = mid + 1; else h2 = mid;
      }
      u32 k = l2 - 1u;
      seq[q0 + j] = p < dlen ? co[ts + k] + (p - s_a[k]) : INVALID;
    }
    qa = qb;
    __syncthreads();
  }
  // pass 2: order -> (agent, seq), client_with_order.get (simple_rle.rs:98-103)
  const CwoRun* cw = P.cwo + sg.cwo_base;
  const u32 ncwo = P.st[d0].n_cwo;
  for (u64 q = q0 + t; q < q1; q += QM_T) {
    u32 order = (u32)(q - q0) < qa ? seq[q] : INVALID;  // (an empty document answers nothing)
    u16 a = 0xFFFF;
    u32 sq = INVALID;
    if (order != INVALID) {
      i32 r = find_run(cw, ncwo, order);
      if (r >= 0) { a = (u16)cw[r].agent; sq = cw[r].seq + (order - cw[r].key); }
    }
    agent[q] = a;
    seq[q] = sq;
  }
}

// ---------------------------------------------------------------------------------------------
// Agent-name interning on the device (ListCRDT::get_or_create_agent_id, doc.rs:66-89; SURVEY
// §8f row 3).  One wave per group (a document's name references in call order): ids in order of
// first appearance ("ROOT" -> ROOT_AGENT, never stored), and every distinct name's rank in
// byte-lexicographic order (Rust `str` Ord, the integrate tie-break's order, doc.rs:207).
// Group g owns refs [roff[g], roff[g+1]); ref r names bytes [noff[r], noff[r+1]).  A wave hashes
// 64 refs at once (FNV-1a), looks them up in an LDS open-addressing table, and admits the new
// names of the chunk one distinct name per step in lane order (the first appearance leads).
// ---------------------------------------------------------------------------------------------
constexpr u32 INTERN_MAX = 1024, INTERN_HT = 2 * INTERN_MAX;
struct InternIO {
  const u64* roff;
  const u32* noff;
  const unsigned char* bytes;
  u16* id;      // per ref
  u32* rank;    // per ref (INVALID for ROOT)
  u32* n_out;   // per group: distinct names
  i32* status;  // per group: 0, or -1 when a group has more than INTERN_MAX distinct names
};
__device__ __forceinline__ bool intern_eq(const unsigned char* b, u32 a0, u32 a1, u32 c0, u32 c1) {
  if (a1 - a0 != c1 - c0) return false;
  for (u32 i = 0; i < a1 - a0; i++)
    if (b[a0 + i] != b[c0 + i]) return false;
  return true;
}
__device__ __forceinline__ bool intern_less(const unsigned char* b, u32 a0, u32 a1, u32 c0, u32 c1) {
  u32 la = a1 - a0, lc = c1 - c0, m = la < lc ? la : lc;
  for (u32 i = 0; i < m; i++) {
    unsigned char x = b[a0 + i], y = b[c0 + i];
    if (x != y) return x < y;
  }
  return la < lc;
}
// One group's names -> ids by first appearance (one wave: the admission is sequential in ref
// order, which is what makes the ids the reference's).  ht / hh: open-addressing table of
// ht_slots (a power of two) slots, 0 = empty else id + 1, with the slot name's FNV-1a hash; rep:
// a ref naming each id.  Returns the distinct names (k); st = -1 past max_names.
__device__ __forceinline__ u32 intern_admit(const InternIO& io, u32 g, u32* ht, u32* hh, u32* rep, u32 ht_slots,
                                            u32 max_names, i32& st) {
  u32 l = threadIdx.x & 63u;
  const unsigned char* B = io.bytes;
  u64 r0 = io.roff[g], r1 = io.roff[g + 1];
  u32 k = 0;
  st = 0;
  for (u64 c = r0; c < r1 && st == 0; c += 64) {
    u64 r = c + l;
    bool v = r < r1;
    u32 a = v ? io.noff[r] : 0u, b = v ? io.noff[r + 1] : 0u;
    u32 h = 2166136261u;
    for (u32 i = a; i < b; i++) h = (h ^ B[i]) * 16777619u;
    bool root = v && b - a == 4u && B[a] == 'R' && B[a + 1] == 'O' && B[a + 2] == 'O' && B[a + 3] == 'T';
    u32 id = INVALID;
    if (v && !root) {  // lookup
      for (u32 s = h & (ht_slots - 1u);; s = (s + 1u) & (ht_slots - 1u)) {
        u32 e = ht[s];
        if (e == 0u) break;
        if (hh[s] == h && intern_eq(B, a, b, io.noff[rep[e - 1u]], io.noff[rep[e - 1u] + 1u])) { id = e - 1u; break; }
      }
    }
    u64 need = __builtin_amdgcn_ballot_w64(v && !root && id == INVALID);
    while (need) {  // admit the chunk's new names, first appearance first
      u32 ld = (u32)__builtin_ctzll(need);
      u32 lh = __builtin_amdgcn_readlane(h, ld), la = __builtin_amdgcn_readlane(a, ld), lb = __builtin_amdgcn_readlane(b, ld);
      if (k >= max_names) { st = -1; break; }
      bool mine = (need >> l) & 1ull;
      bool same = mine && h == lh && intern_eq(B, a, b, la, lb);
      if (same) id = k;
      if (l == ld) {
        u32 s = h & (ht_slots - 1u);
        while (ht[s] != 0u) s = (s + 1u) & (ht_slots - 1u);
        ht[s] = k + 1u;
        hh[s] = h;
        rep[k] = (u32)r;
      }
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      k++;
      need &= ~__builtin_amdgcn_ballot_w64(same);
    }
    if (v) io.id[r] = (u16)(root ? ROOT_AGENT : id);
  }
  return k;
}
__global__ __launch_bounds__(64) void k_intern(InternIO io, u32 n_groups) {
  __shared__ u32 ht[INTERN_HT];      // 0 = empty, else id + 1
  __shared__ u32 hh[INTERN_HT];      // hash of the slot's name
  __shared__ u32 rep[INTERN_MAX];    // a ref naming each id (its first appearance)
  __shared__ u32 rk[INTERN_MAX];     // rank of each id
  u32 g = blockIdx.x, l = threadIdx.x;
  if (g >= n_groups) return;
  for (u32 i = l; i < INTERN_HT; i += 64) ht[i] = 0u;
  __builtin_amdgcn_wave_barrier();
  const unsigned char* B = io.bytes;
  u64 r0 = io.roff[g], r1 = io.roff[g + 1];
  i32 st;
  u32 k = intern_admit(io, g, ht, hh, rep, INTERN_HT, INTERN_MAX, st);
  __builtin_amdgcn_wave_barrier();
  // ranks: names smaller than each distinct name (lane per name)
  for (u32 i = l; i < k; i += 64) {
    u32 ra = rep[i], a = io.noff[ra], b = io.noff[ra + 1], cnt = 0;
    for (u32 j = 0; j < k; j++) {
      u32 rj = rep[j];
      cnt += intern_less(B, io.noff[rj], io.noff[rj + 1], a, b) ? 1u : 0u;
    }
    rk[i] = cnt;
  }
  __builtin_amdgcn_wave_barrier();
  for (u64 r = r0 + l; r < r1; r += 64) {
    u32 id = io.id[r];
    io.rank[r] = (id == ROOT_AGENT || id >= k) ? INVALID : rk[id];
  }
  if (l == 0) {
    io.n_out[g] = k;
    io.status[g] = st;
  }
}

// Groups past INTERN_MAX distinct names (a document with more agents than the LDS table holds;
// the reference allows 65,535, AgentId = u16): the same admission with the table in HBM scratch,
// and ranks from a block-wide bitonic sort of the names (byte-lexicographic) instead of k^2
// counting.  Block (256 threads) per listed group; scratch per block: INTERN_BIG_HT slots x 2 +
// INTERN_BIG_MAX x 3 u32.
constexpr u32 INTERN_BIG_MAX = 65534, INTERN_BIG_HT = 1u << 17, INTERN_BIG_SORT = 1u << 16;
constexpr u64 INTERN_BIG_SCRATCH = 2ull * INTERN_BIG_HT + 3ull * INTERN_BIG_SORT;  // u32 per group
__global__ __launch_bounds__(256) void k_intern_big(InternIO io, const u32* groups, u32 n, u32* scratch) {
  if (blockIdx.x >= n) return;
  u32 g = groups[blockIdx.x], t = threadIdx.x;
  u32* ht = scratch + (u64)blockIdx.x * INTERN_BIG_SCRATCH;
  u32* hh = ht + INTERN_BIG_HT;
  u32* rep = hh + INTERN_BIG_HT;
  u32* rk = rep + INTERN_BIG_SORT;
  u32* srt = rk + INTERN_BIG_SORT;
  for (u32 i = t; i < INTERN_BIG_HT; i += 256) ht[i] = 0u;
  __syncthreads();
  __shared__ u32 sk;
  __shared__ i32 sst;
  if (t < 64) {
    i32 st;
    u32 k = intern_admit(io, g, ht, hh, rep, INTERN_BIG_HT, INTERN_BIG_MAX, st);
    if (t == 0) { sk = k; sst = st; }
  }
  __syncthreads();
  u32 k = sk;
  const unsigned char* B = io.bytes;
  u32 P = 1;
  while (P < k) P <<= 1;
  for (u32 i = t; i < P; i += 256) srt[i] = i < k ? i : INVALID;
  __syncthreads();
  auto less = [&](u32 x, u32 y) -> bool {  // INVALID (padding) sorts last
    if (y == INVALID) return x != INVALID;
    if (x == INVALID) return false;
    u32 rx = rep[x], ry = rep[y];
    return intern_less(B, io.noff[rx], io.noff[rx + 1], io.noff[ry], io.noff[ry + 1]);
  };
  for (u32 size = 2; size <= P; size <<= 1) {
    for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
      for (u32 i = t; i < P / 2; i += 256) {
        u32 lo = 2 * i - (i & (stride - 1)), hi = lo + stride;  // pair (lo, hi) of this step
        bool up = (lo & size) == 0;
        u32 x = srt[lo], y = srt[hi];
        if (less(y, x) == up) { srt[lo] = y; srt[hi] = x; }
      }
      __syncthreads();
    }
  }
  for (u32 i = t; i < k; i += 256) rk[srt[i]] = i;
  __syncthreads();
  u64 r0 = io.roff[g], r1 = io.roff[g + 1];
  for (u64 r = r0 + t; r < r1; r += 256) {
    u32 id = io.id[r];
    io.rank[r] = (id == ROOT_AGENT || id >= k) ? INVALID : rk[id];
  }
  if (t == 0) {
    io.n_out[g] = k;
    io.status[g] = sst;
  }
}

}  // namespace crdt
