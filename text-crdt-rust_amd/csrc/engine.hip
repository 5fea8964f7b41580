// MI355X list-CRDT engine: host side (pool allocation, staging, growth) + the C ABI of
// include/crdt_gpu.h.  All compute runs in the HIP kernels of kernels.h; there is no CPU
// fallback: without a usable gfx950 device every entry point returns CRDT_E_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "crdt_gpu.h"
#include "host_plan.h"
#include "kernels.h"

using namespace crdt;

namespace {

thread_local std::string g_last_error;

#define HIPCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      g_last_error = std::string(#x) + ": " + hipGetErrorString(e_);                    \
      return CRDT_E_DEVICE;                                                             \
    }                                                                                   \
  } while (0)

// Device allocations of the engines of this process, with their current and peak total (the
// relayout's peak footprint: crdt_device_bytes).
std::mutex g_mem_mu;
std::unordered_map<void*, u64> g_mem_size;
u64 g_mem_cur = 0, g_mem_peak = 0;
long long g_fail_alloc_after = -1;  // crdt_test_fail_alloc_after: the allocations left before one fails
template <class T>
hipError_t dalloc(T*& p, u64 n) {
  p = nullptr;
  if (n == 0) n = 1;
  {
    std::lock_guard<std::mutex> g(g_mem_mu);
    if (g_fail_alloc_after == 0) return hipErrorOutOfMemory;
    if (g_fail_alloc_after > 0) g_fail_alloc_after--;
  }
  hipError_t e = hipMalloc((void**)&p, sizeof(T) * n);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> g(g_mem_mu);
    g_mem_size[(void*)p] = sizeof(T) * n;
    g_mem_cur += sizeof(T) * n;
    g_mem_peak = std::max(g_mem_peak, g_mem_cur);
  }
  return e;
}
// bytes of a live dalloc allocation (0 for anything else)
u64 dsize(const void* p) {
  std::lock_guard<std::mutex> g(g_mem_mu);
  auto it = g_mem_size.find(const_cast<void*>(p));
  return it == g_mem_size.end() ? 0 : it->second;
}
template <class T>
void dfree(T*& p) {
  if (p) {
    (void)hipFree((void*)p);
    std::lock_guard<std::mutex> g(g_mem_mu);
    auto it = g_mem_size.find((void*)p);
    if (it != g_mem_size.end()) { g_mem_cur -= it->second; g_mem_size.erase(it); }
  }
  p = nullptr;
}

// Relocatable per-document pools (sized by the per-document capacities).
struct PoolSet {
  Span* leaves = nullptr;
  u32* sol = nullptr;
  u32* dir_leaf = nullptr;
  u32* dir_vis = nullptr;
  u32* leaf_of = nullptr;
  u16* agent_of = nullptr;  // (allocated for every map slot when some document keeps it)
  u32* lag = nullptr;       // leaf agent rows (crdt_types.h lag_words; every leaf slot)
  u32* hrows = nullptr;     // two-level root rows (documents past the LDS root)
  u32* gsob = nullptr;      // their blocks' row slots (every block slot when some document needs it)
  CwoRun* cwo = nullptr;
  ARun* arun = nullptr;
  DelRun* dels = nullptr;
  DDRun* dd = nullptr;
  DDBlk* ddb = nullptr;
  TxnRec* txns = nullptr;
  u32* parents = nullptr;
  u32* frontier = nullptr;
  GroupRec* groups = nullptr;
  AgentRec* agents = nullptr;
  u64 bytes = 0;
  void free_all() {
    dfree(leaves); dfree(sol); dfree(dir_leaf); dfree(dir_vis); dfree(leaf_of); dfree(agent_of); dfree(lag); dfree(hrows); dfree(gsob); dfree(cwo); dfree(arun);
    dfree(dels); dfree(dd); dfree(ddb); dfree(txns); dfree(parents); dfree(frontier); dfree(groups); dfree(agents);
    bytes = 0;
  }
};

struct DocHost {
  AgentTable agents;
  StreamNeeds cum;          // needs of every stream applied since the last reset (capacity plan)
  StreamNeeds staged;       // needs of the stream staged now (a reset replays it: cum = staged)
  Caps caps{};              // current capacities (grow; crdt_fit shrinks them to the replay's use)
  Caps fit_max{};           // crdt_fit_note: per-field maximum of the fitted capacities noted so far
  bool fit_noted = false;
  bool tracked = false;     // keeps the order -> leaf map (once a remote stream was staged)
  bool agent_map = false;   // keeps the order -> agent map (tracked, and more than one agent)
  u32 shape = SHAPE_ALL;    // record kinds of the staged stream (crdt_types.h SHAPE_*): its k_replay instance
  std::vector<u32> agent_cap;
};

// field-wise maximum of two capacity plans (crdt_fit_note)
inline void caps_max(Caps& a, const Caps& b) {
  static_assert(sizeof(Caps) % 4 == 0, "Caps is u32 fields");
  u32* x = (u32*)&a;
  const u32* y = (const u32*)&b;
  for (size_t k = 0; k < sizeof(Caps) / 4; k++) x[k] = std::max(x[k], y[k]);
}

inline void add_needs(StreamNeeds& c, const StreamNeeds& n) {
  c.n_txn += n.n_txn; c.n_ltxn += n.n_ltxn; c.n_rtxn += n.n_rtxn; c.n_ops += n.n_ops; c.orders += n.orders;
  c.local_del += n.local_del; c.remote_del_ops += n.remote_del_ops; c.remote_parents += n.remote_parents;
  if (c.txns_per_agent.size() < n.txns_per_agent.size()) c.txns_per_agent.resize(n.txns_per_agent.size(), 0);
  for (size_t a = 0; a < n.txns_per_agent.size(); a++) c.txns_per_agent[a] += n.txns_per_agent[a];
  c.txn_max(n.max_ops, n.max_del, n.max_len, n.max_parents);
  c.max_rdel_len = std::max(c.max_rdel_len, n.max_rdel_len);
  c.probes += n.probes;
  c.local_del_ops += n.local_del_ops;
}

// Launch shape of a wave-per-document kernel whose waves hold an LDS root of `rcap` groups:
// up to 4 waves per workgroup within the 160 KiB a workgroup may declare.
// (flat root: blk / cnt / vis + the block -> group map, 16 B per group; hr: the two-level root:
// rcap top entries of 12 B + two words per wave; both + RANK_LDS agent ranks)
struct LaunchShape { u32 wpb, rcap; size_t lds; };
inline LaunchShape launch_shape(u32 rcap, bool hr = false) {
  u32 per_wave = 4u * wave_lds_words(rcap, hr);  // (+ the agent ranks and the scan's prefetch row)
  u32 wpb = std::max<u32>(1u, std::min<u32>(WAVES_PER_BLOCK, 163840u / per_wave));
  return LaunchShape{wpb, rcap, (size_t)wpb * per_wave};
}
// LDS root classes: a launch serves documents whose root fits its class.
constexpr u32 ROOT_CLASSES[4] = {ROOT_CAP_MIN, 1024, 4096, ROOT_CAP_LDS};
inline u32 root_class(u32 grp_cap) {
  for (u32 c : ROOT_CLASSES) if (grp_cap <= c) return c;
  return 0;  // past the LDS root: the two-level root (hroot_top)
}
// Documents whose root groups exceed the LDS root replay with the two-level root (wave_gpu.h HR):
// rows of 32..64 groups in HBM (<= grp_cap/32 + 2 of them) under an LDS top level of that many
// entries.  CRDT_FORCE_HBM_ROOT=1 puts every document there (tests of the two-level root).
// (read at every layout: tests switch it per engine)
thread_local bool g_force_hroot = false;
inline bool uses_hroot(u32 grp_cap) { return g_force_hroot || root_class(grp_cap) == 0; }
inline u32 hroot_rows(u32 grp_cap) { return grp_cap / 32u + 2u; }
inline u32 hroot_top(u32 grp_cap) {  // LDS top entries per wave (a multiple of 64)
  return (hroot_rows(grp_cap) + 63u) & ~63u;
}

}  // namespace

// Pools field `which` (kernels.h RL_*) := ptr; RL_ARUN also sets the agent table the move reads
// the run bases from (src: the old table, dst: the new one).
inline void set_pool_ptr(Pools& p, u32 which, void* ptr, AgentRec* agents) {
  switch (which) {
    case RL_LEAVES: p.leaves = (Span*)ptr; break;
    case RL_SOL: p.slot_of_leaf = (u32*)ptr; break;
    case RL_DIR_LEAF: p.dir_leaf = (u32*)ptr; break;
    case RL_DIR_VIS: p.dir_vis = (u32*)ptr; break;
    case RL_LEAF_OF: p.leaf_of = (u32*)ptr; break;
    case RL_AGENT_OF: p.agent_of = (u16*)ptr; break;
    case RL_CWO: p.cwo = (CwoRun*)ptr; break;
    case RL_DELS: p.dels = (DelRun*)ptr; break;
    case RL_DD: p.dd = (DDRun*)ptr; break;
    case RL_DDB: p.ddb = (DDBlk*)ptr; break;
    case RL_TXNS: p.txns = (TxnRec*)ptr; break;
    case RL_PARENTS: p.parents = (u32*)ptr; break;
    case RL_FRONTIER: p.frontier = (u32*)ptr; break;
    case RL_GROUPS: p.groups = (GroupRec*)ptr; break;
    case RL_ARUN: p.arun = (ARun*)ptr; p.agents = agents; break;
    default: break;
  }
}

struct crdt_engine {
  u32 L = 32;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  u64 n_docs = 0;
  std::vector<DocHost> docs;
  std::vector<DocSeg> seg_h;
  std::vector<DocState> st_h;
  // fixed per-document buffers
  DocState* st = nullptr;
  DocSeg* segs = nullptr;
  u32* canon_n = nullptr;
  u32* len = nullptr;
  u64* digest = nullptr;
  u32* n_agents_d = nullptr;
  std::vector<u32> n_agents_pushed;  // host copy of what n_agents_d holds
  // replay launches: one per LDS root class present; `doc_list` holds the classes' documents
  struct RootClass { u32 rcap; u64 off, n; bool hr; u32 shape; };
  std::vector<RootClass> classes;
  u32* doc_list = nullptr;
  PoolSet pools;
  Rec* recs = nullptr;
  u64 rec_cap = 0;
  uint4* probe = nullptr;  // PROBE answers, one slot per staged record (when probes are staged)
  u64 probe_cap = 0;
  bool has_probes = false;
  bool share_streams = false;  // documents staged with the same host stream read one device copy
  bool intern_on_device = false;  // crdt_stage_remote_replicated interns through k_intern
  int query_kernel = -1;  // crdt_set_query_kernel (-1: not set; CRDT_QUERY_PER_THREAD selects 1)
  bool published = false;
  bool digested = false;   // k_digest ran on the current published index
  // A relayout (growth, crdt_fit) that failed after it began moving pools leaves some pools at
  // their new bases and the rest at the old ones: the engine is then unusable, and every call but
  // release / crdt_docs_alloc returns CRDT_E_NOMEM (no half-moved engine is replayed).
  bool poisoned = false;
  int qmode() const {
    if (query_kernel >= 0) return query_kernel;
    static const bool per_thread = getenv("CRDT_QUERY_PER_THREAD") != nullptr;  // (A/B switch)
    return per_thread ? CRDT_QUERY_PER_THREAD : CRDT_QUERY_LDS;
  }
  double last_replay_ms = 0, last_publish_ms = 0, last_materialize_ms = 0;
  // text materialisation: order-indexed content streams, per-document stream offsets, output text
  u32* content = nullptr;
  u64 content_cap = 0;
  std::vector<u64> cbase_h, clen_h;
  u64* cbase = nullptr;
  u64* clen = nullptr;
  u32* text = nullptr;
  u64 text_cap = 0;
  u64 ord_total = 0;  // text buffer entries (sum of ord_cap)
  // published index (k_publish output, no state: re-sized without copying, see size_pub)
  Span* canon = nullptr;
  u32* vpos = nullptr;
  u32* sorted = nullptr;
  u32* corder = nullptr;  // first order of every canonical span (k_pub_index input)
  u32* pub = nullptr;
  u64 canon_alloc = 0, pub_alloc = 0;
  bool pub_sized = false;   // the index pools fit the device state (else publish sizes them first)
  bool pub_fitted = false;  // crdt_fit sized them for the staged stream (replays need no check)
  // publish launches: documents with >= PUB_BIG_MIN leaves get a workgroup each (k_publish_big)
  std::vector<u32> pub_small, pub_big;
  u32* pub_list = nullptr;  // [small docs..., big docs...] when there are big ones
  // the small documents' order -> span index is built in LDS (k_pub_index) when their bitmap has
  // at most PUBX_MAX_WORDS words; pubx_words = the largest such bitmap (the launch's LDS size)
  u32 pubx_words = 0;
  u32* tlen = nullptr;
  u64* tdigest = nullptr;
  bool materialized = false;
  // query scratch
  void* qbuf = nullptr;
  u64 qbuf_bytes = 0;

  Pools pools_view(const PoolSet& ps) const {
    Pools p{};
    p.leaves = ps.leaves;
    p.dir_leaf = ps.dir_leaf;
    p.dir_vis = ps.dir_vis;
    p.slot_of_leaf = ps.sol;
    p.leaf_of = ps.leaf_of;
    p.agent_of = ps.agent_of;
    p.leaf_agents = ps.lag;
    p.hrows = ps.hrows;
    p.gsob = ps.gsob;
    p.cwo = ps.cwo;
    p.arun = ps.arun;
    p.dels = ps.dels;
    p.dd = ps.dd;
    p.ddb = ps.ddb;
    p.txns = ps.txns;
    p.parents = ps.parents;
    p.frontier = ps.frontier;
    p.agents = ps.agents;
    p.groups = ps.groups;
    p.recs = recs;
    p.probe = has_probes ? probe : nullptr;
    p.seg = segs;
    p.st = st;
    return p;
  }
  PubOut pub_view() const {
    PubOut o{};
    o.canon = canon;
    o.vpos = vpos;
    o.sorted = sorted;
    o.corder = corder;
    o.pub = pub;
    o.canon_n = canon_n;
    o.len = len;
    o.digest = digest;
    return o;
  }

  void release() {
    pools.free_all();
    dfree(canon); dfree(vpos); dfree(sorted); dfree(corder); dfree(pub); dfree(pub_list);
    pub_small.clear();
    pub_big.clear();
    canon_alloc = pub_alloc = 0;
    pub_sized = pub_fitted = false;
    dfree(st); dfree(segs); dfree(canon_n); dfree(len); dfree(digest); dfree(n_agents_d); dfree(doc_list);
    n_agents_pushed.clear();
    classes.clear();
    dfree(recs);
    rec_cap = 0;
    dfree(probe);
    probe_cap = 0;
    has_probes = false;
    dfree(content); dfree(cbase); dfree(clen); dfree(text); dfree(tlen); dfree(tdigest);
    content_cap = 0;
    text_cap = 0;
    materialized = false;
    if (qbuf) (void)hipFree(qbuf);
    qbuf = nullptr;
    qbuf_bytes = 0;
  }

  int set_device() {
    HIPCHK(hipSetDevice(device));
    return 0;
  }

  int alloc_docs(u64 n) {
    int r = set_device();
    if (r) return r;
    HIPCHK(hipStreamSynchronize(stream));
    release();
    poisoned = false;
    n_docs = n;
    docs.assign(n, DocHost{});
    seg_h.assign(n, DocSeg{});
    st_h.assign(n, DocState{});
    HIPCHK(dalloc(st, n));
    HIPCHK(dalloc(segs, n));
    HIPCHK(dalloc(canon_n, n));
    HIPCHK(dalloc(len, n));
    HIPCHK(dalloc(digest, n));
    HIPCHK(dalloc(n_agents_d, n));
    HIPCHK(dalloc(cbase, n));
    HIPCHK(dalloc(clen, n));
    HIPCHK(dalloc(tlen, n));
    HIPCHK(dalloc(tdigest, n));
    cbase_h.assign(n, NO_CONTENT);
    clen_h.assign(n, 0);
    HIPCHK(hipMemsetAsync(cbase, 0xFF, sizeof(u64) * std::max<u64>(n, 1), stream));
    HIPCHK(hipMemsetAsync(clen, 0, sizeof(u64) * std::max<u64>(n, 1), stream));
    HIPCHK(hipMemsetAsync(st, 0, sizeof(DocState) * std::max<u64>(n, 1), stream));
    // size every document for an empty stream and initialise it
    for (u64 d = 0; d < n; d++) docs[d].caps = plan_caps(StreamNeeds{}, 0, true, 48);
    r = layout(false);
    if (r) return r;
    return init_all();
  }

  // Assign per-document bases from docs[].caps into a fresh PoolSet; if `move`, relocate the
  // existing state into it (k_relayout_pool, one pool at a time), else just install it.
  int layout(bool move) {
    int r = 0;
    g_force_hroot = getenv("CRDT_FORCE_HBM_ROOT") != nullptr && getenv("CRDT_FORCE_HBM_ROOT")[0] == '1';
    PoolSet np;
    u64 nl = 0, nb = 0, nm = 0, nc = 0, na = 0, ndl = 0, ndd = 0, nt = 0, npar = 0, nag = 0, nfr = 0;
    std::vector<DocSeg> nseg(n_docs);
    std::vector<AgentRec> agent_tab;
    std::vector<u32> n_agents(n_docs);
    bool any_agent_map = false, any_hroot = false;
    u64 nhr = 0;
    for (u64 d = 0; d < n_docs; d++) {
      DocHost& h = docs[d];
      const Caps& c = h.caps;
      DocSeg s{};
      s.leaf_base = nl; s.leaf_cap = c.leaf; nl += c.leaf;
      s.blk_base = nb; s.blk_cap = c.blk; nb += c.blk;
      s.map_base = nm; s.map_cap = c.map; nm += c.map;
      s.cwo_base = nc; s.cwo_cap = c.cwo; nc += c.cwo;
      s.del_base = ndl; s.del_cap = c.del; ndl += c.del;
      s.dd_base = ndd; s.dd_cap = c.dd; ndd += c.dd;
      s.txn_base = nt; s.txn_cap = c.txn; nt += c.txn;
      s.par_base = npar; s.par_cap = c.par; npar += c.par;
      s.fr_base = nfr; s.fr_cap = c.fr; nfr += c.fr;
      s.canon_base = seg_h[d].canon_base; s.canon_cap = seg_h[d].canon_cap;  // (size_pub's)
      s.pub_base = seg_h[d].pub_base; s.ord_base = seg_h[d].ord_base; s.ord_cap = seg_h[d].ord_cap;
      s.grp_base = s.blk_base; s.grp_cap = c.blk;  // one root group per directory block
      s.hrow_base = nhr;
      if (uses_hroot(c.blk)) { nhr += hroot_rows(c.blk); any_hroot = true; }
      s.agent_base = nag;
      u32 ag = (u32)h.agents.names.size();
      s.agent_cap = ag;
      n_agents[d] = ag;
      s.arun_base = na;
      std::vector<u32> rk = h.agents.ranks();
      u32 rb = 0;
      h.agent_cap.resize(ag, 0);
      for (u32 a = 0; a < ag; a++) {
        u32 t = a < h.cum.txns_per_agent.size() ? h.cum.txns_per_agent[a] : 0;
        u32 need = std::min<u32>(t + 1, 64 + t / 64);
        if (h.agent_cap[a] < need) h.agent_cap[a] = need;
        agent_tab.push_back(AgentRec{rb, 0, h.agent_cap[a], rk[a], 0, 0, 0, 0});
        rb += h.agent_cap[a];
      }
      s.arun_cap = rb;
      na += rb;
      nag += ag;
      s.flags = (h.tracked ? DOC_TRACK_MAP : 0u) | (h.agent_map ? DOC_TRACK_AGENT : 0u);
      any_agent_map |= h.agent_map;
      s.rec_base = seg_h[d].rec_base;
      s.rec_n = seg_h[d].rec_n;
      nseg[d] = s;
    }
    // sizes of the new pools (element counts; 0 -> one element)
    // leaf agent rows only when some document keeps the order -> agent map: the others never read
    // or store a row (lag_stale is a lane-predicated store on K_AGMAP), so the pool is one element
    const u64 n_lag = any_agent_map ? nl * lag_words(L) : 1;
    const u64 n_agent_of = any_agent_map ? nm : 1, n_hrows = any_hroot ? nhr * HROOT_ROW : 1, n_gsob = any_hroot ? nb : 1;
    np.bytes = nl * L * 16 + nl * 8 + nb * GROUP * 8 + nm * 4 + (any_agent_map ? nm * 2 : 0) + n_lag * 4 +
               (any_hroot ? nhr * HROOT_ROW * 4 + nb * 4 : 0) + nc * 16 + na * 16 + ndl * 12 +
               ndd * (DD_BLK * 12 + 16) + nt * 32 + npar * 4 + nag * (u64)sizeof(AgentRec) + nfr * 4 + nb * 16;
    if (getenv("CRDT_DEBUG_MEM"))
      fprintf(stderr, "layout: leaves %llu blocks %llu map %llu cwo %llu arun %llu del %llu ddblk %llu txn %llu par %llu agents %llu fr %llu -> %.1f MB\n",
              (unsigned long long)nl, (unsigned long long)nb, (unsigned long long)nm, (unsigned long long)nc,
              (unsigned long long)na, (unsigned long long)ndl, (unsigned long long)ndd, (unsigned long long)nt,
              (unsigned long long)npar, (unsigned long long)nag, (unsigned long long)nfr, np.bytes / 1e6);
    DocSeg* old_segs = nullptr;
    struct Cleanup {
      PoolSet& np;
      DocSeg*& os;
      ~Cleanup() { dfree(np.agents); dfree(os); }
    } cleanup{np, old_segs};
    // The two allocations come before any engine state changes: an out-of-memory error here
    // leaves the engine intact (the caller may free memory and retry).
    HIPCHK(dalloc(np.agents, nag));  // (the new agent table first: the run move reads its bases)
    if (move) HIPCHK(dalloc(old_segs, n_docs));
    // From here on the engine's state changes pool by pool: until the last pool has moved, a
    // failure leaves it poisoned (and frees what this call allocated).
    poisoned = true;
    if (!agent_tab.empty())
      HIPCHK(hipMemcpyAsync(np.agents, agent_tab.data(), agent_tab.size() * sizeof(AgentRec), hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(n_agents_d, n_agents.data(), n_docs * 4, hipMemcpyHostToDevice, stream));
    if (move) HIPCHK(hipMemcpyAsync(old_segs, segs, n_docs * sizeof(DocSeg), hipMemcpyDeviceToDevice, stream));
    HIPCHK(hipMemcpyAsync(segs, nseg.data(), n_docs * sizeof(DocSeg), hipMemcpyHostToDevice, stream));
    // Pool by pool: allocate the new one, move every document's part (k_relayout_pool), free the
    // old one.  The peak is the old pools + the largest new pool (2x both sets before).  A pool
    // whose every document keeps its capacity (so its base: bases are prefix sums) and whose
    // element count is unchanged stays where it is -- growth of one table, or crdt_fit of a
    // config-5 corpus whose order maps are already exact, then moves no order map (the largest
    // pools) and the peak is lower by that much.
    auto same_caps = [&](u32 DocSeg::*cap) {
      if (!move) return false;
      for (u64 d = 0; d < n_docs; d++)
        if (nseg[d].*cap != seg_h[d].*cap) return false;
      return true;
    };
    const bool s_leaf = same_caps(&DocSeg::leaf_cap), s_blk = same_caps(&DocSeg::blk_cap), s_map = same_caps(&DocSeg::map_cap),
               s_cwo = same_caps(&DocSeg::cwo_cap), s_del = same_caps(&DocSeg::del_cap), s_dd = same_caps(&DocSeg::dd_cap),
               s_txn = same_caps(&DocSeg::txn_cap), s_par = same_caps(&DocSeg::par_cap), s_fr = same_caps(&DocSeg::fr_cap);
    auto step = [&](auto& old_p, auto& new_p, u64 count, u32 which, bool same = false) -> int {
      if (move && same && old_p && dsize(old_p) == sizeof(*old_p) * std::max<u64>(count, 1)) {
        new_p = nullptr;  // (stays: same bases, same size)
        return 0;
      }
      HIPCHK(dalloc(new_p, count));
      if (move && which < RL_N) {
        Pools src = pools_view(pools), dst = pools_view(pools);
        set_pool_ptr(src, which, (void*)old_p, pools.agents);
        set_pool_ptr(dst, which, (void*)new_p, np.agents);
        if (L == 32) hipLaunchKernelGGL(k_relayout_pool<32>, dim3((u32)n_docs), dim3(256), 0, stream, src, dst, old_segs, n_agents_d, (u32)n_docs, which);
        else hipLaunchKernelGGL(k_relayout_pool<4>, dim3((u32)n_docs), dim3(256), 0, stream, src, dst, old_segs, n_agents_d, (u32)n_docs, which);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(stream));
      }
      dfree(old_p);
      old_p = new_p;
      return 0;
    };
    r = 0;
    if (!r) r = step(pools.leaves, np.leaves, nl * L, RL_LEAVES, s_leaf);
    if (!r) r = step(pools.sol, np.sol, 2 * nl, RL_SOL, s_leaf);  // {directory slot, successor leaf} per leaf
    if (!r) r = step(pools.dir_leaf, np.dir_leaf, nb * GROUP, RL_DIR_LEAF, s_blk);
    if (!r) r = step(pools.dir_vis, np.dir_vis, nb * GROUP, RL_DIR_VIS, s_blk);
    if (!r) r = step(pools.leaf_of, np.leaf_of, nm, RL_LEAF_OF, s_map);
    if (!r) r = step(pools.agent_of, np.agent_of, n_agent_of, RL_AGENT_OF, s_map);
    if (!r) r = step(pools.lag, np.lag, n_lag, RL_N, s_leaf);  // (not moved: every row starts stale)
    if (!r) HIPCHK(hipMemsetAsync(pools.lag, 0, n_lag * 4, stream));
    if (!r) r = step(pools.hrows, np.hrows, n_hrows, RL_N);  // (rebuilt from the groups at every launch)
    if (!r) r = step(pools.gsob, np.gsob, n_gsob, RL_N);
    if (!r) r = step(pools.cwo, np.cwo, nc, RL_CWO, s_cwo);
    if (!r) r = step(pools.dels, np.dels, ndl, RL_DELS, s_del);
    if (!r) r = step(pools.dd, np.dd, ndd * DD_BLK, RL_DD, s_dd);
    if (!r) r = step(pools.ddb, np.ddb, ndd, RL_DDB, s_dd);
    if (!r) r = step(pools.txns, np.txns, nt, RL_TXNS, s_txn);
    if (!r) r = step(pools.parents, np.parents, npar, RL_PARENTS, s_par);
    if (!r) r = step(pools.frontier, np.frontier, nfr, RL_FRONTIER, s_fr);
    if (!r) r = step(pools.groups, np.groups, nb, RL_GROUPS, s_blk);
    if (!r) r = step(pools.arun, np.arun, na, RL_ARUN);
    if (r) return r;
    if (move) {  // the agents' run counts and last-run copies into the new table
      Pools src = pools_view(pools), dst = pools_view(pools);
      dst.agents = np.agents;
      if (L == 32) hipLaunchKernelGGL(k_relayout_pool<32>, dim3((u32)n_docs), dim3(256), 0, stream, src, dst, old_segs, n_agents_d, (u32)n_docs, (u32)RL_AGENTS);
      else hipLaunchKernelGGL(k_relayout_pool<4>, dim3((u32)n_docs), dim3(256), 0, stream, src, dst, old_segs, n_agents_d, (u32)n_docs, (u32)RL_AGENTS);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(stream));
    dfree(pools.agents);
    pools.agents = np.agents;
    np.agents = nullptr;
    pools.bytes = np.bytes;
    seg_h = nseg;
    poisoned = false;
    r = plan_classes();
    if (r) return r;
    pub_sized = false;
    published = false;
    materialized = false;
    return 0;
  }

  // Size the published-index pools for the documents' current state: canonical spans <= the
  // state's leaf entries (or crdt_fit's exact count), orders < ord_cap.  Outputs only, so the
  // pools are freed before the new ones are allocated (no copy, no double footprint).
  int size_pub() {
    int r = pull_states();
    if (r) return r;
    u64 ncan = 0, npub = 0, nord = 0;
    for (u64 d = 0; d < n_docs; d++) {
      DocSeg& s = seg_h[d];
      Caps& c = docs[d].caps;
      if (st_h[d].next_order >= c.ord) c.ord = st_h[d].next_order + 1;
      s.canon_cap = std::max<u32>(c.canon ? c.canon : st_h[d].n_entries, 1u);
      s.canon_base = ncan; ncan += s.canon_cap;
      s.ord_cap = std::max<u32>(c.ord, 1u);
      s.ord_base = nord; nord += s.ord_cap;
      s.pub_base = npub; npub += 2ull * pub_words(s.ord_cap);
    }
    if (ncan > canon_alloc || ncan < canon_alloc / 2) {
      dfree(canon); dfree(vpos); dfree(sorted); dfree(corder);
      canon_alloc = 0;
      HIPCHK(dalloc(canon, ncan));
      HIPCHK(dalloc(vpos, ncan));
      HIPCHK(dalloc(sorted, ncan));
      HIPCHK(dalloc(corder, ncan));
      canon_alloc = ncan;
    }
    if (npub > pub_alloc || npub < pub_alloc / 2) {
      dfree(pub);
      pub_alloc = 0;
      HIPCHK(dalloc(pub, npub));
      pub_alloc = npub;
    }
    ord_total = nord;
    HIPCHK(hipMemcpyAsync(segs, seg_h.data(), n_docs * sizeof(DocSeg), hipMemcpyHostToDevice, stream));
    // long documents publish with a workgroup each: always from PUB_BIG_MAX leaves, and from
    // PUB_BIG_MIN when the batch is too small to fill the GPU with one wave per document (for
    // thousands of mid-sized documents one wave each moves more per second)
    pub_small.clear();
    pub_big.clear();
    pubx_words = 0;
    for (u64 d = 0; d < n_docs; d++) {
      u32 nl = st_h[d].n_leaves;
      bool big = nl >= PUB_BIG_MAX || (nl >= PUB_BIG_MIN && n_docs <= PUB_BIG_FEW_DOCS);
      (big ? pub_big : pub_small).push_back((u32)d);
      u32 nw = pub_words(seg_h[d].ord_cap);
      if (!big && nw <= PUBX_MAX_WORDS) pubx_words = std::max(pubx_words, nw);
    }
    dfree(pub_list);
    if (!pub_big.empty()) {
      std::vector<u32> all(pub_small);
      all.insert(all.end(), pub_big.begin(), pub_big.end());
      HIPCHK(dalloc(pub_list, all.size()));
      HIPCHK(hipMemcpyAsync(pub_list, all.data(), all.size() * 4, hipMemcpyHostToDevice, stream));
    }
    HIPCHK(hipStreamSynchronize(stream));
    pub_sized = true;
    return 0;
  }

  // Replay launch classes (LDS root sizes) from the documents' root capacities; the documents
  // of every class go to the device list when more than one class is present.
  int plan_classes() {
    // classes 0-3: the LDS root sizes; class 4: the two-level root (top size: the largest needed);
    // the LDS-root classes split further by stream shape (one k_replay instance per shape), bucket
    // k * N_SHAPES + shape; the two-level root has one instance (SHAPE_ALL), bucket 4 * N_SHAPES
    std::vector<std::vector<u32>> by(4 * N_SHAPES + 1);
    u32 hr_top = 64;
    // documents with nothing to replay go with the shape of the first one that has a stream (no
    // launch of their own: they return at once in any instance)
    u32 sh0 = SHAPE_ALL;
    for (u64 d = 0; d < n_docs; d++)
      if (seg_h[d].rec_n) { sh0 = docs[d].shape; break; }
    for (u64 d = 0; d < n_docs; d++) {
      u32 gc = seg_h[d].grp_cap;
      if (uses_hroot(gc)) {
        by[4 * N_SHAPES].push_back((u32)d);
        hr_top = std::max(hr_top, hroot_top(gc));
        continue;
      }
      u32 c = root_class(gc);
      u32 k = 0;
      while (ROOT_CLASSES[k] != c) k++;
      by[k * N_SHAPES + (seg_h[d].rec_n ? docs[d].shape : sh0)].push_back((u32)d);
    }
    if (hr_top > ROOT_CAP_MAX) {
      g_last_error = "a document's root exceeds the two-level root's top level";
      return CRDT_E_NOMEM;
    }
    auto rc = [&](u32 b) { return b < 4 * N_SHAPES ? ROOT_CLASSES[b / N_SHAPES] : hr_top; };
    auto cls = [&](u32 b, u64 off, u64 n) {
      return RootClass{rc(b), off, n, b == 4 * N_SHAPES, b < 4 * N_SHAPES ? b % N_SHAPES : (u32)SHAPE_ALL};
    };
    // Within a class the longest staged streams launch first (LPT order): a workgroup's waves hold
    // their slots until its last one ends, so workgroups of similar documents, longest first, leave
    // the short ones to fill the end of the launch (mixed corpora: config 3).  Equal streams keep
    // the document order (stable sort).
    // Documents of equal length that replay one shared record stream (the same history) go next
    // to each other: a workgroup of equal histories ends together (config 5's 8 histories differ in
    // cost at equal op counts).  Unshared streams sit at increasing offsets: document order.
    auto work = [&](u32 d) { return docs[d].staged.n_ops + docs[d].staged.n_txn; };
    bool identity = true;
    for (auto& v : by) {
      std::stable_sort(v.begin(), v.end(), [&](u32 a, u32 b) {
        u64 wa = work(a), wb = work(b);
        return wa != wb ? wa > wb : seg_h[a].rec_base < seg_h[b].rec_base;
      });
      for (size_t i = 1; i < v.size(); i++) identity &= v[i] == v[i - 1] + 1u;
    }
    classes.clear();
    dfree(doc_list);
    u32 present = 0;
    for (auto& v : by) present += !v.empty();
    if (present <= 1 && identity) {
      for (u32 k = 0; k < by.size(); k++)
        if (!by[k].empty()) classes.push_back(cls(k, INVALID, by[k].size()));
      return 0;
    }
    std::vector<u32> all;
    for (u32 k = 0; k < by.size(); k++) {
      if (by[k].empty()) continue;
      classes.push_back(cls(k, all.size(), by[k].size()));
      all.insert(all.end(), by[k].begin(), by[k].end());
    }
    HIPCHK(dalloc(doc_list, all.size()));
    HIPCHK(hipMemcpyAsync(doc_list, all.data(), all.size() * 4, hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return 0;
  }

  // Every document to ListCRDT::new().  Agents interned since the last layout get their table
  // slots first (a relayout; the old state is discarded anyway).
  int init_all() {
    bool relayout = false;
    for (u64 d = 0; d < n_docs; d++)
      if (docs[d].agents.names.size() != seg_h[d].agent_cap) relayout = true;
    if (relayout) {
      int r = layout(false);
      if (r) return r;
    }
    // host-side agent counts into the state before k_init (k_init keeps n_agents)
    int r = push_agent_counts();
    if (r) return r;
    LaunchShape sh = launch_shape(64);
    u32 blocks = (u32)((n_docs + sh.wpb - 1) / sh.wpb);
    if (n_docs) {
      if (L == 32) hipLaunchKernelGGL(k_init<32>, dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pools_view(pools), (u32)n_docs, sh.wpb, sh.rcap);
      else hipLaunchKernelGGL(k_init<4>, dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pools_view(pools), (u32)n_docs, sh.wpb, sh.rcap);
      HIPCHK(hipGetLastError());
    }
    published = false;
    materialized = false;
    return 0;
  }

  // st[d].n_agents := the host's interned count for every document (clamped to the document's
  // agent table, which layout() sized).  Uploaded only when it changed; the host copy outlives
  // the asynchronous copy (the stream is synchronised right after it).
  int push_agent_counts() {
    std::vector<u32> na(n_docs);
    for (u64 d = 0; d < n_docs; d++) na[d] = std::min<u32>((u32)docs[d].agents.names.size(), seg_h[d].agent_cap);
    if (na != n_agents_pushed) {
      n_agents_pushed = na;
      HIPCHK(hipMemcpyAsync(n_agents_d, n_agents_pushed.data(), n_docs * 4, hipMemcpyHostToDevice, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
    if (n_docs) {  // one launch for every document (not one 4-byte copy per document)
      hipLaunchKernelGGL(k_set_n_agents, dim3((u32)((n_docs + 255) / 256)), dim3(256), 0, stream, st, (const u32*)n_agents_d, (u32)n_docs);
      HIPCHK(hipGetLastError());
    }
    return 0;
  }

  // Stage per-document record streams (host-encoded) and grow capacities if needed.
  int stage(const std::vector<u64>& doc_ids, std::vector<const std::vector<Rec>*>& streams, std::vector<StreamNeeds>& needs) {
    int r = set_device();
    if (r) return r;
    HIPCHK(hipStreamSynchronize(stream));
    // a stage replaces every document's staged stream (documents not named get none)
    {
      std::vector<char> seen(n_docs, 0);
      for (u64 d : doc_ids) {
        if (seen[d]) return CRDT_E_ARG;  // a document named twice in one call
        seen[d] = 1;
      }
      for (u64 d = 0; d < n_docs; d++)
        if (!seen[d]) docs[d].staged = StreamNeeds{};
    }
    // documents that receive their first remote stream start keeping the order -> leaf map (only
    // remote ops read it); one that already holds state gets it rebuilt from its leaves
    std::vector<u32> rebuild;
    bool pulled = false;
    bool grow = false;
    for (size_t i = 0; i < doc_ids.size(); i++) {
      DocHost& h = docs[doc_ids[i]];
      if (h.tracked || (needs[i].n_rtxn == 0 && needs[i].probes == 0)) continue;
      h.tracked = true;
      grow = true;
      if (!pulled) {
        r = pull_states();
        if (r) return r;
        pulled = true;
      }
      if (st_h[doc_ids[i]].next_order) rebuild.push_back((u32)doc_ids[i]);
    }
    // tracked documents with several agents keep the order -> agent map too (integrate's name
    // tie-breaks); one that already holds state gets it rebuilt from client_with_order
    std::vector<u32> rebuild_ag;
    for (size_t i = 0; i < doc_ids.size(); i++) {
      DocHost& h = docs[doc_ids[i]];
      if (h.agent_map || !h.tracked || h.agents.names.size() < 2) continue;
      h.agent_map = true;
      grow = true;
      if (!pulled) {
        r = pull_states();
        if (r) return r;
        pulled = true;
      }
      if (st_h[doc_ids[i]].next_order) rebuild_ag.push_back((u32)doc_ids[i]);
    }
    // stream shapes: the record kinds of each distinct host stream (k_replay instance per shape;
    // CRDT_NO_SHAPES=1 in the environment keeps every stream on the general instance, for A/B)
    {
      static const bool no_shapes = getenv("CRDT_NO_SHAPES") && getenv("CRDT_NO_SHAPES")[0] == '1';
      std::unordered_map<const std::vector<Rec>*, u32> kinds_of;
      for (u64 d = 0; d < n_docs; d++) docs[d].shape = SHAPE_ALL;
      for (size_t i = 0; i < doc_ids.size(); i++) {
        auto f = kinds_of.find(streams[i]);
        if (f == kinds_of.end()) {
          u32 k = 0;
          for (const Rec& x : *streams[i]) k |= 1u << rec_kind(x);
          f = kinds_of.emplace(streams[i], k).first;
        }
        docs[doc_ids[i]].shape = no_shapes ? (u32)SHAPE_ALL : shape_of_kinds(f->second);
      }
    }
    // cumulative needs -> capacities
    for (size_t i = 0; i < doc_ids.size(); i++) {
      DocHost& h = docs[doc_ids[i]];
      StreamNeeds& c = h.cum;
      add_needs(c, needs[i]);
      h.staged = needs[i];
      pub_fitted = false;
      Caps nc = plan_caps(c, (u32)h.agents.names.size(), h.tracked, 48);
      Caps& oc = h.caps;
      auto up = [&](u32& o, u32 v) { if (v > o) { o = v; grow = true; } };
      up(oc.ord, nc.ord);
      if (oc.canon) { oc.canon = 0; grow = true; }  // a fitted canonical-span capacity: back to the bound
      up(oc.leaf, nc.leaf); up(oc.blk, nc.blk); up(oc.map, nc.map); up(oc.cwo, nc.cwo); up(oc.arun, nc.arun);
      up(oc.del, nc.del); up(oc.dd, nc.dd); up(oc.txn, nc.txn); up(oc.par, nc.par); up(oc.agent, nc.agent);
      up(oc.fr, nc.fr);
      for (size_t a = 0; a < h.agents.names.size(); a++) {
        u32 t = a < c.txns_per_agent.size() ? c.txns_per_agent[a] : 0;
        u32 need = std::min<u32>(t + 1, 64 + t / 64);
        if (a >= h.agent_cap.size() || h.agent_cap[a] < need) grow = true;
      }
      if (h.agents.names.size() != h.agent_cap.size()) grow = true;
    }
    // records: one buffer for this call
    u64 total = 0, n_probes = 0;
    for (auto& n : needs) n_probes += n.probes;
    bool share = share_streams && n_probes == 0;  // (probe answers are per record slot)
    {
      std::unordered_map<const std::vector<Rec>*, char> seen;
      for (auto* s : streams)
        if (!share || seen.emplace(s, 1).second) total += s->size();
    }
    if (total > rec_cap) {  // (the new buffer first: a failed allocation leaves the old one in place)
      Rec* nr = nullptr;
      u64 cap = std::max<u64>(total, 1024);
      HIPCHK(dalloc(nr, cap));
      dfree(recs);
      recs = nr;
      rec_cap = cap;
    }
    has_probes = n_probes > 0;
    if (has_probes && probe_cap < total) {
      uint4* np_ = nullptr;
      HIPCHK(dalloc(np_, total));
      dfree(probe);
      probe = np_;
      probe_cap = total;
    }
    if (has_probes) {
      // every probe slot starts as the "unknown" answer: probes after a document's stop point
      // never run, and must not report a previous call's (or uninitialised) answers
      std::vector<uint4> unk(total, make_uint4(0xFFFFu, INVALID, INVALID, 2u));
      HIPCHK(hipMemcpyAsync(probe, unk.data(), total * sizeof(uint4), hipMemcpyHostToDevice, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
    for (auto& sg : seg_h) { sg.rec_base = 0; sg.rec_n = 0; }
    // Consecutive distinct streams go up in one host->device copy; a replicated stream (same
    // host vector as the previous document) is a device-to-device copy of that upload.
    u64 off = 0;
    const std::vector<Rec>* prev = nullptr;
    u64 prev_off = 0;
    std::unordered_map<const std::vector<Rec>*, u64> uploaded;  // shared stream -> first device copy
    std::vector<Rec> hb;
    u64 hb_off = 0;
    auto flush = [&]() -> int {
      if (hb.empty()) return 0;
      HIPCHK(hipMemcpyAsync(recs + hb_off, hb.data(), hb.size() * sizeof(Rec), hipMemcpyHostToDevice, stream));
      HIPCHK(hipStreamSynchronize(stream));
      hb.clear();
      return 0;
    };
    for (size_t i = 0; i < doc_ids.size(); i++) {
      DocSeg& sg = seg_h[doc_ids[i]];
      const std::vector<Rec>& sv = *streams[i];
      sg.rec_base = off;
      sg.rec_n = (u32)sv.size();
      auto up = uploaded.find(&sv);
      if (share && up != uploaded.end()) {  // read-only input: reference the first copy
        sg.rec_base = up->second;
        continue;
      }
      if (!sv.empty()) {
        if (&sv == prev || up != uploaded.end()) {
          r = flush();
          if (r) return r;
          u64 src = &sv == prev ? prev_off : up->second;
          HIPCHK(hipMemcpyAsync(recs + off, recs + src, sv.size() * sizeof(Rec), hipMemcpyDeviceToDevice, stream));
        } else if (sv.size() > (1u << 20)) {  // large stream: straight from the caller's vector
          r = flush();
          if (r) return r;
          HIPCHK(hipMemcpyAsync(recs + off, sv.data(), sv.size() * sizeof(Rec), hipMemcpyHostToDevice, stream));
          HIPCHK(hipStreamSynchronize(stream));
        } else {
          if (hb.empty()) hb_off = off;
          hb.insert(hb.end(), sv.begin(), sv.end());
        }
      }
      if (up == uploaded.end()) uploaded.emplace(&sv, off);
      prev = &sv;
      prev_off = off;
      off += sv.size();
    }
    r = flush();
    if (r) return r;
    HIPCHK(hipStreamSynchronize(stream));
    if (grow) {
      r = layout(true);
      if (r) return r;
      if (!rebuild.empty()) {
        u32* dl = nullptr;
        HIPCHK(dalloc(dl, rebuild.size()));
        HIPCHK(hipMemcpyAsync(dl, rebuild.data(), rebuild.size() * 4, hipMemcpyHostToDevice, stream));
        if (L == 32) hipLaunchKernelGGL(k_build_map<32>, dim3((u32)rebuild.size()), dim3(256), 0, stream, pools_view(pools), (const u32*)dl, (u32)rebuild.size());
        else hipLaunchKernelGGL(k_build_map<4>, dim3((u32)rebuild.size()), dim3(256), 0, stream, pools_view(pools), (const u32*)dl, (u32)rebuild.size());
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(stream));
        dfree(dl);
      }
      if (!rebuild_ag.empty()) {
        u32* dl = nullptr;
        HIPCHK(dalloc(dl, rebuild_ag.size()));
        HIPCHK(hipMemcpyAsync(dl, rebuild_ag.data(), rebuild_ag.size() * 4, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(k_build_agent_map, dim3((u32)rebuild_ag.size()), dim3(256), 0, stream, pools_view(pools), (const u32*)dl, (u32)rebuild_ag.size());
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(stream));
        dfree(dl);
      }
    } else {
      HIPCHK(hipMemcpyAsync(segs, seg_h.data(), n_docs * sizeof(DocSeg), hipMemcpyHostToDevice, stream));
      r = push_agent_counts();
      if (r) return r;
      r = plan_classes();  // (launch order: the new streams' lengths)
      if (r) return r;
    }
    if (n_docs) {
      hipLaunchKernelGGL(k_reset_recpos, dim3((u32)((n_docs + 255) / 256)), dim3(256), 0, stream, st, (u32)n_docs, 0u);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(stream));
    published = false;
    materialized = false;
    return 0;
  }

  int launch_replay() {
    if (!n_docs) return 0;
    Pools pv = pools_view(pools);
    for (const RootClass& c : classes) {  // one launch per root class (usually one)
      LaunchShape sh = launch_shape(c.rcap, c.hr);
      u32 blocks = (u32)((c.n + sh.wpb - 1) / sh.wpb);
      const u32* list = c.off == INVALID ? nullptr : doc_list + c.off;
      if (c.hr) {
        if (L == 32) hipLaunchKernelGGL(k_replay_hr<32>, dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
        else hipLaunchKernelGGL(k_replay_hr<4>, dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
      } else {  // (one instance per stream shape)
        if (L == 32) {
          if (c.shape == SHAPE_REMOTE) hipLaunchKernelGGL((k_replay<32, SHAPE_REMOTE>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else if (c.shape == SHAPE_GEN) hipLaunchKernelGGL((k_replay<32, SHAPE_GEN>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else if (c.shape == SHAPE_LOCAL) hipLaunchKernelGGL((k_replay<32, SHAPE_LOCAL>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else hipLaunchKernelGGL((k_replay<32, SHAPE_ALL>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
        } else {
          if (c.shape == SHAPE_REMOTE) hipLaunchKernelGGL((k_replay<4, SHAPE_REMOTE>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else if (c.shape == SHAPE_GEN) hipLaunchKernelGGL((k_replay<4, SHAPE_GEN>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else if (c.shape == SHAPE_LOCAL) hipLaunchKernelGGL((k_replay<4, SHAPE_LOCAL>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
          else hipLaunchKernelGGL((k_replay<4, SHAPE_ALL>), dim3(blocks), dim3(64 * sh.wpb), sh.lds, stream, pv, (u32)c.n, sh.wpb, sh.rcap, list);
        }
      }
      HIPCHK(hipGetLastError());
    }
    if (!pub_fitted) pub_sized = false;  // the state grows: size the index again before publishing
    published = false;
    materialized = false;
    return 0;
  }

  int pull_states() {
    HIPCHK(hipMemcpyAsync(st_h.data(), st, n_docs * sizeof(DocState), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return 0;
  }

  // Replay with growth: on ST_NEED_CAPACITY grow the flagged tables and resume.
  int run(int32_t* status_out) {
    int r = set_device();
    if (r) return r;
    for (int iter = 0; iter < 40; iter++) {
      HIPCHK(hipEventRecord(ev[0], stream));
      r = launch_replay();
      if (r) return r;
      HIPCHK(hipEventRecord(ev[1], stream));
      r = pull_states();
      if (r) return r;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
      last_replay_ms = ms;
      bool any = false;
      for (u64 d = 0; d < n_docs; d++) {
        if (st_h[d].status != ST_NEED_CAPACITY) continue;
        any = true;
        Caps& c = docs[d].caps;
        u32 need = st_h[d].cap_need;
        if (need & 1u) {
          if (c.leaf >= MAX_LEAVES) { need &= ~1u; }
          c.leaf = std::min<u32>(c.leaf * 2, MAX_LEAVES);
          c.blk = blk_cap_for(c.leaf);
        }
        if (need & 128u) c.fr = c.fr * 2;
        if (need & 2u) { c.cwo = c.cwo * 2 + 1; c.txn = c.txn * 2 + 1; }
        if (need & 4u) c.del = c.del * 2 + 16;
        if (need & 8u) c.par = c.par * 2 + 16;
        if (need & 16u) c.map = c.map * 2 + 16;
        if (need & 64u) c.dd = c.dd * 2 + 2;
        if (need & 32u) for (auto& x : docs[d].agent_cap) x = x * 2 + 1;
        if (need == 0) {  // cannot grow: make it a hard capacity error
          st_h[d].status = ST_CAPACITY;
          HIPCHK(hipMemcpyAsync(&st[d].status, &st_h[d].status, 4, hipMemcpyHostToDevice, stream));
        }
      }
      HIPCHK(hipStreamSynchronize(stream));
      if (!any) break;
      r = layout(true);
      if (r) return r;
    }
    // the published index (and the text) for this state: sized now, while the stream is idle
    r = size_pub();
    if (r) return r;
    if (status_out)
      for (u64 d = 0; d < n_docs; d++) status_out[d] = st_h[d].status == ST_NEED_CAPACITY ? ST_CAPACITY : st_h[d].status;
    return 0;
  }

  // Shrink every document's capacities to what its staged stream used, keeping the room the
  // replay reserves ahead of one txn (fits()): called after a full replay + publish of the staged
  // streams, so that replaying them again (reset + run) needs exactly this much.
  // mode 0: fit (capacities = what the staged streams used); 1: note those capacities into each
  // document's running maximum (no relayout); 2: capacities = the noted maxima (and forget them)
  int fit(int mode = 0) {
    int r = ensure_published();
    if (r) return r;
    r = pull_states();
    if (r) return r;
    std::vector<u32> cn(n_docs);
    HIPCHK(hipMemcpy(cn.data(), canon_n, n_docs * 4, hipMemcpyDeviceToHost));
    for (u64 d = 0; d < n_docs; d++) {
      const DocState& s = st_h[d];
      DocHost& h = docs[d];
      if (s.status != ST_OK) {
        // (its state says nothing about its needs; mode 2 still applies and forgets what earlier
        // notes gathered, so no stale maximum carries into the next note cycle)
        if (mode == 2 && h.fit_noted) {
          caps_max(h.caps, h.fit_max);
          h.fit_noted = false;
        }
        continue;
      }
      const StreamNeeds& m = h.cum;
      Caps fc = h.caps;
      Caps& c = mode == 0 ? h.caps : fc;
      c.leaf = std::max<u32>(s.n_leaves + 2 * m.max_ops + 2, 2);
      c.blk = blk_cap_for(c.leaf);
      c.cwo = s.n_cwo + 1;
      c.txn = s.n_txn + 1;
      c.del = s.n_del + m.max_del + 1;
      c.par = s.n_par + std::max<u32>(m.max_parents, s.n_fr) + 64;
      // (every txn checks map room for its own orders, next_order + txn_len <= map_cap, and orders
      // only grow: the final next_order bounds every check of a replay from reset)
      if (h.tracked) c.map = (u32)std::min<u64>((u64)s.next_order + 1, 0xFFFFFFFFull);
      c.ord = s.next_order + 1;
      c.canon = std::max<u32>(cn[d], 1);
      c.fr = std::max<u32>(s.n_fr + 1, FRONTIER_CAP0);
      // double-delete blocks: fits()' reserve before the stream's last remote delete txn (the
      // entry count only grows, so the final count bounds every earlier reserve)
      if (c.dd) {
        u64 ov = std::min<u64>(s.n_dd, m.max_rdel_len);
        c.dd = std::max<u32>(4u, (u32)std::min<u64>(((u64)s.n_dd + 3 * ov + 2ull * m.max_rdel_len + 2) / 32 + 3, 0x7FFFFFFFull));
      }
      if (mode == 0) continue;
      if (!h.fit_noted) { h.fit_max = fc; h.fit_noted = true; }
      else caps_max(h.fit_max, fc);
      if (mode == 2) {
        h.caps = h.fit_max;
        h.fit_noted = false;
      }
    }
    if (mode == 1) return 0;
    r = layout(true);
    if (r) return r;
    r = size_pub();
    if (r) return r;
    pub_fitted = true;  // replays of the staged streams publish exactly this much
    return 0;
  }

  int publish() {
    int r = set_device();
    if (r) return r;
    u32 blocks = (u32)((n_docs + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    if (!n_docs) return 0;
    if (!pub_sized) {  // (waits for the replay in flight: the index is sized from its state)
      r = size_pub();
      if (r) return r;
    }
    HIPCHK(hipEventRecord(ev[2], stream));
    Pools pv = pools_view(pools);
    PubOut ov = pub_view();
    u32 ns = pub_list ? (u32)pub_small.size() : (u32)n_docs;
    blocks = (ns + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (ns) {
      // documents whose bitmap fits pubx_words get their index from k_pub_index (k_publish skips it)
      u32 xw = pubx_words;
      if (L == 32) hipLaunchKernelGGL(k_publish<32>, dim3(blocks), dim3(256), 0, stream, pv, ov, ns, (const u32*)pub_list, xw);
      else hipLaunchKernelGGL(k_publish<4>, dim3(blocks), dim3(256), 0, stream, pv, ov, ns, (const u32*)pub_list, xw);
      HIPCHK(hipGetLastError());
      if (xw) {
        hipLaunchKernelGGL(k_pub_index, dim3(ns), dim3(PUBX_THREADS), pubx_lds_bytes(xw), stream, pv, ov,
                           (const u32*)pub_list, xw);
        HIPCHK(hipGetLastError());
      }
    }
    if (pub_list && !pub_big.empty()) {
      const u32* bl = pub_list + pub_small.size();
      if (L == 32) hipLaunchKernelGGL(k_publish_big<32>, dim3((u32)pub_big.size()), dim3(64 * PUB_BIG_WAVES), 0, stream, pv, ov, bl);
      else hipLaunchKernelGGL(k_publish_big<4>, dim3((u32)pub_big.size()), dim3(64 * PUB_BIG_WAVES), 0, stream, pv, ov, bl);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev[3], stream));
    published = true;
    digested = false;
    materialized = false;
    return 0;
  }
  // The per-document digests of the published state (k_digest, on request: the parity checker's
  // summary, not part of the index publish builds for the queries)
  int digest_now() {
    if (!published) {
      int r = publish();
      if (r) return r;
    }
    if (digested || !n_docs) return 0;
    u32 blocks = (u32)((n_docs + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    if (L == 32) hipLaunchKernelGGL(k_digest<32>, dim3(blocks), dim3(256), 0, stream, pools_view(pools), pub_view(), (u32)n_docs);
    else hipLaunchKernelGGL(k_digest<4>, dim3(blocks), dim3(256), 0, stream, pools_view(pools), pub_view(), (u32)n_docs);
    HIPCHK(hipGetLastError());
    digested = true;
    return 0;
  }
  int ensure_published() {
    if (published) return 0;
    int r = publish();
    if (r) return r;
    HIPCHK(hipStreamSynchronize(stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev[2], ev[3]);
    last_publish_ms = ms;
    return 0;
  }
  TextIO text_view() const {
    TextIO t{};
    t.content = content;
    t.cbase = cbase;
    t.clen = clen;
    t.text = text;
    t.tlen = tlen;
    t.tdigest = tdigest;
    return t;
  }
  // Content streams (order-indexed UTF-32); document docs[i] reads stream stream_of_doc[i].
  // Replaces all previously set content; documents not named have none.
  int set_content(u64 n, const uint32_t* docs, const uint32_t* stream_of_doc, u32 n_streams, const uint64_t* stream_off,
                  const uint32_t* data) {
    int r = set_device();
    if (r) return r;
    for (u32 k = 0; k < n_streams; k++)
      if (stream_off[k + 1] < stream_off[k]) return CRDT_E_ARG;
    for (u64 i = 0; i < n; i++)
      if (docs[i] >= n_docs || stream_of_doc[i] >= n_streams) return CRDT_E_ARG;
    u64 total = stream_off[n_streams];
    HIPCHK(hipStreamSynchronize(stream));
    if (total == 0) {  // no content: release the table
      dfree(content);
      content_cap = 0;
    }
    if (total > content_cap) {
      dfree(content);
      HIPCHK(dalloc(content, total));
      content_cap = std::max<u64>(total, 1);
    }
    if (total) HIPCHK(hipMemcpyAsync(content, data, total * 4, hipMemcpyHostToDevice, stream));
    std::fill(cbase_h.begin(), cbase_h.end(), NO_CONTENT);
    std::fill(clen_h.begin(), clen_h.end(), 0);
    for (u64 i = 0; i < n; i++) {
      u32 k = stream_of_doc[i];
      cbase_h[docs[i]] = stream_off[k];
      clen_h[docs[i]] = stream_off[k + 1] - stream_off[k];
    }
    HIPCHK(hipMemcpyAsync(cbase, cbase_h.data(), n_docs * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(clen, clen_h.data(), n_docs * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
    materialized = false;
    return 0;
  }
  // Every listed document gets its own device copy of one content stream (a corpus whose documents
  // do not share a cache-resident table).
  int set_content_copies(u64 n, const uint32_t* docs, const uint32_t* data, u64 len) {
    int r = set_device();
    if (r) return r;
    for (u64 i = 0; i < n; i++)
      if (docs[i] >= n_docs) return CRDT_E_ARG;
    u64 total = n * len;
    HIPCHK(hipStreamSynchronize(stream));
    if (total > content_cap || total == 0) {
      dfree(content);
      content_cap = 0;
      if (total) {
        HIPCHK(dalloc(content, total));
        content_cap = total;
      }
    }
    if (total) {
      HIPCHK(hipMemcpyAsync(content, data, len * 4, hipMemcpyHostToDevice, stream));
      for (u64 i = 1; i < n; i++)
        HIPCHK(hipMemcpyAsync(content + i * len, content, len * 4, hipMemcpyDeviceToDevice, stream));
    }
    std::fill(cbase_h.begin(), cbase_h.end(), NO_CONTENT);
    std::fill(clen_h.begin(), clen_h.end(), 0);
    for (u64 i = 0; i < n; i++) {
      cbase_h[docs[i]] = i * len;
      clen_h[docs[i]] = len;
    }
    HIPCHK(hipMemcpyAsync(cbase, cbase_h.data(), n_docs * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(clen, clen_h.data(), n_docs * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
    materialized = false;
    return 0;
  }
  int materialize() {
    int r = set_device();
    if (r) return r;
    if (!n_docs) return 0;
    if (!published) {
      r = publish();
      if (r) return r;
    }
    if (text_cap < ord_total) {
      HIPCHK(hipStreamSynchronize(stream));
      dfree(text);
      HIPCHK(dalloc(text, ord_total));
      text_cap = std::max<u64>(ord_total, 1);
    }
    HIPCHK(hipEventRecord(ev[4], stream));
    if (L == 32) hipLaunchKernelGGL(k_materialize<32>, dim3((u32)n_docs), dim3(64 * MAT_WAVES), 0, stream, pools_view(pools), pub_view(), text_view(), (u32)n_docs);
    else hipLaunchKernelGGL(k_materialize<4>, dim3((u32)n_docs), dim3(64 * MAT_WAVES), 0, stream, pools_view(pools), pub_view(), text_view(), (u32)n_docs);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev[5], stream));
    materialized = true;
    return 0;
  }
  int ensure_materialized() {
    if (!materialized) {
      int r = materialize();
      if (r) return r;
    }
    HIPCHK(hipStreamSynchronize(stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev[4], ev[5]);
    last_materialize_ms = ms;
    return 0;
  }
  int scratch(u64 bytes) {
    if (bytes <= qbuf_bytes) return 0;
    if (qbuf) (void)hipFree(qbuf);
    qbuf = nullptr;
    HIPCHK(hipMalloc(&qbuf, bytes));
    qbuf_bytes = bytes;
    return 0;
  }
};

static bool valid(const crdt_engine* e) { return e && e->n_docs > 0; }
static bool poisoned(const crdt_engine* e) {
  if (!e || !e->poisoned) return false;
  g_last_error = "engine poisoned: a relayout failed part-way (out of device memory); destroy it or crdt_docs_alloc again";
  return true;
}
// The documents a stage call names: in range and none twice (checked before any interning, so a
// rejected call leaves every agent table -- and so the agent ids of later calls -- unchanged)
static bool ids_ok(const crdt_engine* e, uint64_t n, const uint32_t* docs) {
  std::vector<char> seen(e->n_docs, 0);
  for (uint64_t i = 0; i < n; i++) {
    if (docs[i] >= e->n_docs || seen[docs[i]]) return false;
    seen[docs[i]] = 1;
  }
  return true;
}

extern "C" {

int crdt_engine_create(const crdt_cfg* cfg, crdt_engine** out) {
  if (!cfg || !out || (cfg->leaf_cap != 32 && cfg->leaf_cap != 4)) return CRDT_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= cfg->device || cfg->device < 0) return CRDT_E_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return CRDT_E_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CRDT_E_DEVICE;
  std::unique_ptr<crdt_engine> e(new crdt_engine());
  e->L = cfg->leaf_cap;
  e->device = cfg->device;
  if (hipSetDevice(e->device) != hipSuccess) return CRDT_E_DEVICE;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return CRDT_E_DEVICE;
  // the replay's LDS root may take a workgroup's whole 160 KiB (one wave per workgroup)
  (void)hipFuncSetAttribute((const void*)k_replay<32, SHAPE_ALL>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<4, SHAPE_ALL>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<32, SHAPE_REMOTE>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<4, SHAPE_REMOTE>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<32, SHAPE_GEN>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<32, SHAPE_LOCAL>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<4, SHAPE_GEN>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay<4, SHAPE_LOCAL>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay_hr<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_replay_hr<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)k_pos_to_loc_blk<32>, hipFuncAttributeMaxDynamicSharedMemorySize, QBLK_LDS);
  (void)hipFuncSetAttribute((const void*)k_pos_to_loc_blk<4>, hipFuncAttributeMaxDynamicSharedMemorySize, QBLK_LDS);
  (void)hipFuncSetAttribute((const void*)k_loc_to_pos_blk<32>, hipFuncAttributeMaxDynamicSharedMemorySize, QBLK_W * 8u);
  (void)hipFuncSetAttribute((const void*)k_loc_to_pos_blk<4>, hipFuncAttributeMaxDynamicSharedMemorySize, QBLK_W * 8u);
  (void)hipFuncSetAttribute((const void*)k_pub_index, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)pubx_lds_bytes(PUBX_MAX_WORDS));
  for (auto& x : e->ev)
    if (hipEventCreate(&x) != hipSuccess) return CRDT_E_DEVICE;
  *out = e.release();
  return 0;
}

void crdt_engine_destroy(crdt_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  e->release();
  for (auto& x : e->ev)
    if (x) (void)hipEventDestroy(x);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

int crdt_docs_alloc(crdt_engine* e, uint64_t n) {
  if (!e || n == 0 || n > 0xFFFFFFFFull) return CRDT_E_ARG;
  return e->alloc_docs(n);
}
uint64_t crdt_num_docs(const crdt_engine* e) { return e ? e->n_docs : 0; }

int crdt_test_fail_alloc_after(long long k) {
  std::lock_guard<std::mutex> g(g_mem_mu);
  g_fail_alloc_after = k < 0 ? -1 : k;
  return 0;
}

int crdt_agent_intern(crdt_engine* e, uint64_t n, const uint32_t* doc, const char* const* names, uint16_t* out) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n && (!doc || !names || !out))) return CRDT_E_ARG;
  for (uint64_t i = 0; i < n; i++) {
    if (doc[i] >= e->n_docs) return CRDT_E_ARG;
    out[i] = (uint16_t)e->docs[doc[i]].agents.get_or_create(names[i]);
  }
  return 0;
}

// Device interning (kernels.h k_intern): the same results as crdt_agent_intern on the same call.
// Each document named in the call forms one group: its existing names (in id order, so the
// first-appearance numbering reproduces their ids) followed by this call's names for it.
int crdt_agent_intern_dev(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint64_t* name_off,
                          const char* bytes, uint16_t* out, uint32_t* rank_out) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n && (!doc || !name_off || !bytes || !out))) return CRDT_E_ARG;
  if (!n) return 0;
  int rs = e->set_device();  // (scratch and the launch belong on the engine's device)
  if (rs) return rs;
  std::unordered_map<u32, u32> gmap;
  std::vector<u32> gdoc;
  std::vector<std::vector<u64>> grefs;  // per group: call refs (indices into the call)
  for (u64 i = 0; i < n; i++) {
    if (doc[i] >= e->n_docs || name_off[i + 1] < name_off[i]) return CRDT_E_ARG;
    auto it = gmap.find(doc[i]);
    u32 g;
    if (it == gmap.end()) { g = (u32)gdoc.size(); gmap[doc[i]] = g; gdoc.push_back(doc[i]); grefs.emplace_back(); }
    else g = it->second;
    grefs[g].push_back(i);
  }
  // blob: per group the existing names, then the call's names
  std::vector<unsigned char> blob;
  std::vector<u32> noff{0};
  std::vector<u64> roff{0};
  std::vector<u64> call_ref(n);  // call index -> ref index
  for (u32 g = 0; g < gdoc.size(); g++) {
    const AgentTable& t = e->docs[gdoc[g]].agents;
    for (const std::string& nm : t.names) {
      blob.insert(blob.end(), nm.begin(), nm.end());
      noff.push_back((u32)blob.size());
    }
    for (u64 i : grefs[g]) {
      call_ref[i] = noff.size() - 1;
      blob.insert(blob.end(), bytes + name_off[i], bytes + name_off[i + 1]);
      if (blob.size() >= 0xFFFFFFFFull) return CRDT_E_ARG;
      noff.push_back((u32)blob.size());
    }
    roff.push_back(noff.size() - 1);
  }
  u64 nr = noff.size() - 1, ng = gdoc.size();
  u64 sz = blob.size() + 16 + noff.size() * 4 + roff.size() * 8 + nr * (2 + 4) + ng * 8 + 256;
  int r = e->scratch(sz);
  if (r) return r;
  char* q = (char*)e->qbuf;
  auto carve = [&](u64 bytes_) { char* p = q; q += (bytes_ + 15) & ~15ull; return p; };
  u64* d_roff = (u64*)carve(roff.size() * 8);
  u32* d_noff = (u32*)carve(noff.size() * 4);
  u32* d_rank = (u32*)carve(nr * 4);
  u32* d_n = (u32*)carve(ng * 4);
  i32* d_st = (i32*)carve(ng * 4);
  u16* d_id = (u16*)carve(nr * 2);
  unsigned char* d_b = (unsigned char*)carve(blob.size() + 1);
  HIPCHK(hipMemcpyAsync(d_roff, roff.data(), roff.size() * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(d_noff, noff.data(), noff.size() * 4, hipMemcpyHostToDevice, e->stream));
  if (!blob.empty()) HIPCHK(hipMemcpyAsync(d_b, blob.data(), blob.size(), hipMemcpyHostToDevice, e->stream));
  InternIO io{d_roff, d_noff, d_b, d_id, d_rank, d_n, d_st};
  hipLaunchKernelGGL(k_intern, dim3((u32)ng), dim3(64), 0, e->stream, io, (u32)ng);
  HIPCHK(hipGetLastError());
  std::vector<u16> id(nr);
  std::vector<u32> rank(nr), gn(ng);
  std::vector<i32> gst(ng);
  HIPCHK(hipMemcpyAsync(id.data(), d_id, nr * 2, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(rank.data(), d_rank, nr * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(gn.data(), d_n, ng * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(gst.data(), d_st, ng * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  // documents past the LDS table's INTERN_MAX names: again with the table in HBM (k_intern_big)
  std::vector<u32> big;
  for (u32 g = 0; g < ng; g++)
    if (gst[g] != 0) big.push_back(g);
  if (!big.empty()) {
    u32* d_big = nullptr;
    u32* d_scr = nullptr;
    HIPCHK(dalloc(d_big, big.size()));
    HIPCHK(dalloc(d_scr, big.size() * INTERN_BIG_SCRATCH));
    HIPCHK(hipMemcpyAsync(d_big, big.data(), big.size() * 4, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_intern_big, dim3((u32)big.size()), dim3(256), 0, e->stream, io, (const u32*)d_big, (u32)big.size(), d_scr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(id.data(), d_id, nr * 2, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(rank.data(), d_rank, nr * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(gn.data(), d_n, ng * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(gst.data(), d_st, ng * 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    dfree(d_big);
    dfree(d_scr);
  }
  for (u32 g = 0; g < ng; g++) {
    if (gst[g] != 0) {
      g_last_error = "crdt_agent_intern_dev: more than 65,534 distinct names in one document (AgentId is u16)";
      return CRDT_E_ARG;
    }
  }
  // mirror the new names into the host tables (capacity planning, host lookups), in id order
  for (u32 g = 0; g < ng; g++) {
    AgentTable& t = e->docs[gdoc[g]].agents;
    u32 old = (u32)t.names.size();
    for (u64 ref = roff[g]; ref < roff[g] + old; ref++)
      if (id[ref] != ref - roff[g]) { g_last_error = "crdt_agent_intern_dev: existing id mismatch"; return CRDT_E_DEVICE; }
    for (u64 ref = roff[g] + old; ref < roff[g + 1]; ref++) {
      if (id[ref] == (u16)t.names.size()) {
        std::string nm((const char*)blob.data() + noff[ref], noff[ref + 1] - noff[ref]);
        t.ids[nm] = id[ref];
        t.names.push_back(nm);
      }
    }
    if (t.names.size() != gn[g]) { g_last_error = "crdt_agent_intern_dev: name count mismatch"; return CRDT_E_DEVICE; }
  }
  for (u64 i = 0; i < n; i++) {
    out[i] = id[call_ref[i]];
    if (rank_out) rank_out[i] = rank[call_ref[i]];
  }
  return 0;
}

// probes (optional): one per txn, encoded after it; probe_rec gets each probe's record index
static int stage_local_impl(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                            const crdt_local_txn* txns, const crdt_local_op* ops,
                            const crdt_probe* probes = nullptr, std::vector<std::vector<u32>>* probe_rec = nullptr) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !docs || !txn_off || (!txns && txn_off[n_docs]) ) return CRDT_E_ARG;
  if (!ids_ok(e, n_docs, docs)) return CRDT_E_ARG;
  if (probe_rec) probe_rec->assign(n_docs, {});
  std::vector<u64> ids(n_docs);
  std::vector<std::vector<Rec>> streams(n_docs);
  std::vector<StreamNeeds> needs(n_docs);
  std::vector<const std::vector<Rec>*> sp(n_docs);
  for (uint64_t i = 0; i < n_docs; i++) sp[i] = &streams[i];
  // op offsets: ops are concatenated in txn order over all docs
  u64 op = 0;
  for (u64 t = 0; t < txn_off[0]; t++) op += txns[t].n_ops;
  for (uint64_t i = 0; i < n_docs; i++) {
    if (docs[i] >= e->n_docs) return CRDT_E_ARG;
    ids[i] = docs[i];
    for (u64 t = txn_off[i]; t < txn_off[i + 1]; t++) {
      encode_local_txn(streams[i], needs[i], txns[t].agent, (const u32*)(ops + op), txns[t].n_ops);
      op += txns[t].n_ops;
      if (probes) {
        (*probe_rec)[i].push_back((u32)streams[i].size());
        encode_probe(streams[i], needs[i], probes[t].pos, probes[t].agent, probes[t].seq);
      }
    }
  }
  return e->stage(ids, sp, needs);
}

int crdt_apply_local_probed(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                            const crdt_local_txn* txns, const crdt_local_op* ops, const crdt_probe* probes,
                            crdt_probe_answer* answers, int32_t* doc_status) {
  if (!probes || !answers) return CRDT_E_ARG;
  std::vector<std::vector<u32>> where;
  int r = stage_local_impl(e, n_docs, docs, txn_off, txns, ops, probes, &where);
  if (r) return r;
  std::vector<int32_t> all(e->n_docs);
  r = e->run(all.data());
  if (r) return r;
  std::vector<uint4> buf(e->probe_cap);
  HIPCHK(hipMemcpy(buf.data(), e->probe, buf.size() * sizeof(uint4), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < n_docs; i++) {
    if (doc_status) doc_status[i] = all[docs[i]];
    u64 base = e->seg_h[docs[i]].rec_base;
    for (u64 t = txn_off[i], k = 0; t < txn_off[i + 1]; t++, k++) {
      const uint4& x = buf[base + where[i][k]];
      answers[t] = crdt_probe_answer{x.x, x.y, x.z, x.w};
    }
  }
  return 0;
}

int crdt_stage_local(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                     const crdt_local_txn* txns, const crdt_local_op* ops) {
  return stage_local_impl(e, n_docs, docs, txn_off, txns, ops);
}

int crdt_stage_local_shared(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* stream_of_doc,
                            uint32_t n_streams, const uint64_t* stream_txn_off, const crdt_local_txn* txns,
                            const crdt_local_op* ops) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !docs || !stream_of_doc || !stream_txn_off || !n_streams) return CRDT_E_ARG;
  if (!ids_ok(e, n_docs, docs)) return CRDT_E_ARG;
  std::vector<std::vector<Rec>> enc(n_streams);
  std::vector<StreamNeeds> snd(n_streams);
  u64 op = 0;
  for (u64 t = 0; t < stream_txn_off[0]; t++) op += txns[t].n_ops;
  for (u32 k = 0; k < n_streams; k++)
    for (u64 t = stream_txn_off[k]; t < stream_txn_off[k + 1]; t++) {
      encode_local_txn(enc[k], snd[k], txns[t].agent, (const u32*)(ops + op), txns[t].n_ops);
      op += txns[t].n_ops;
    }
  std::vector<u64> ids(n_docs);
  std::vector<StreamNeeds> needs(n_docs);
  std::vector<const std::vector<Rec>*> sp(n_docs);
  for (uint64_t i = 0; i < n_docs; i++) {
    if (docs[i] >= e->n_docs || stream_of_doc[i] >= n_streams) return CRDT_E_ARG;
    ids[i] = docs[i];
    sp[i] = &enc[stream_of_doc[i]];
    needs[i] = snd[stream_of_doc[i]];
  }
  return e->stage(ids, sp, needs);
}

int crdt_stage_remote_wire(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint8_t* const* wire,
                           const uint64_t* wire_len) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !docs || !wire || !wire_len) return CRDT_E_ARG;
  if (!ids_ok(e, n_docs, docs)) return CRDT_E_ARG;
  std::vector<u64> ids(n_docs);
  std::vector<std::vector<Rec>> streams(n_docs);
  std::vector<StreamNeeds> needs(n_docs);
  std::vector<const std::vector<Rec>*> sp(n_docs);
  // documents handed the same wire buffer whose encoding comes out identical (same name -> agent
  // ids) stage one host stream: stage() then copies it on the device (or, with shared streams,
  // references one device copy)
  std::map<std::pair<const uint8_t*, uint64_t>, uint64_t> first_of;
  for (uint64_t i = 0; i < n_docs; i++) {
    if (docs[i] >= e->n_docs) return CRDT_E_ARG;
    ids[i] = docs[i];
    WireView wv;
    if (!wv.parse(wire[i], wire_len[i])) return CRDT_E_WIRE;
    encode_remote(streams[i], needs[i], e->docs[docs[i]].agents, wv);
    sp[i] = &streams[i];
    auto f = first_of.emplace(std::make_pair(wire[i], wire_len[i]), i);
    if (!f.second) {
      const std::vector<Rec>& a = streams[f.first->second];
      if (a.size() == streams[i].size() && std::memcmp(a.data(), streams[i].data(), a.size() * sizeof(Rec)) == 0) {
        sp[i] = &a;
        std::vector<Rec>().swap(streams[i]);
      }
    }
  }
  return e->stage(ids, sp, needs);
}

int crdt_stage_remote_replicated(crdt_engine* e, const uint8_t* wire, uint64_t wire_len, uint32_t rename_idx,
                                 const char* const* names) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !wire) return CRDT_E_ARG;
  WireView wv;
  if (!wv.parse(wire, wire_len)) return CRDT_E_WIRE;
  // Every document gets its own interned names; documents whose name->agent-id mapping equals
  // the first document's share one host-encoded stream (device copies are still per document).
  std::vector<u64> ids(e->n_docs);
  std::vector<std::vector<Rec>> uniq;
  std::vector<const std::vector<Rec>*> sp(e->n_docs);
  std::vector<StreamNeeds> needs(e->n_docs);
  uniq.reserve(e->n_docs);
  std::vector<u32> first_map;
  // Authors in order of first appearance: interning that list (get_or_create is idempotent per
  // name) leaves an AgentTable identical to interning every txn's author in txn order, at a cost
  // of #names instead of #txns per document.
  std::vector<u32> authors;
  {
    std::vector<char> seen(wv.names.size(), 0);
    for (const auto& t : wv.txns)
      if (!seen[t.agent_name]) seen[t.agent_name] = 1, authors.push_back(t.agent_name);
  }
  if (e->intern_on_device) {
    // Every document's authors, in order of first appearance, interned by k_intern in one call
    // (one wave per document); the host tables are mirrored by crdt_agent_intern_dev, so the
    // mapping check below finds every fresh document already interned.
    std::vector<u32> ddoc;
    std::vector<u64> off{0};
    std::string blob;
    ddoc.reserve(e->n_docs * authors.size());
    for (u64 d = 0; d < e->n_docs; d++) {
      for (u32 a : authors) {
        const std::string& nm = (names && a == rename_idx) ? std::string(names[d]) : wv.names[a];
        blob += nm;
        ddoc.push_back((u32)d);
        off.push_back(blob.size());
      }
    }
    std::vector<uint16_t> out(ddoc.size());
    int r = crdt_agent_intern_dev(e, ddoc.size(), ddoc.data(), off.data(), blob.data(), out.data(), nullptr);
    if (r) return r;
  }
  for (u64 d = 0; d < e->n_docs; d++) {
    ids[d] = d;
    std::vector<std::string> nm = wv.names;  // only the names differ per document
    if (names && rename_idx < nm.size()) nm[rename_idx] = names[d];
    AgentTable& at = e->docs[d].agents;
    std::vector<Rec> tmp;
    bool fresh = at.names.empty();
    if (d > 0 && e->intern_on_device && !uniq.empty()) {
      // (interned above: only the mapping decides whether document 0's stream fits)
      std::vector<u32> m;
      for (const auto& n : nm) m.push_back(at.lookup(n));
      if (m == first_map) {
        sp[d] = &uniq[0];
        needs[d] = needs[0];
        continue;
      }
    } else if (d > 0 && fresh && !uniq.empty()) {
      // intern in txn order (authors create, others look up) exactly as encode_remote does
      AgentTable probe = at;
      for (u32 a : authors) probe.get_or_create(nm[a]);
      std::vector<u32> m;
      for (const auto& n : nm) m.push_back(probe.lookup(n));
      if (m == first_map) {
        at = probe;
        sp[d] = &uniq[0];
        needs[d] = needs[0];
        continue;
      }
    }
    WireView w2 = wv;
    w2.names = std::move(nm);
    uniq.emplace_back();
    encode_remote(uniq.back(), needs[d], at, w2);
    sp[d] = &uniq.back();
    if (d == 0) for (const auto& n : w2.names) first_map.push_back(at.lookup(n));
  }
  return e->stage(ids, sp, needs);
}

int crdt_stage_random(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const char* agent, uint32_t n_ops,
                      uint64_t seed) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !docs || !agent || n_ops == 0 || std::strcmp(agent, "ROOT") == 0) return CRDT_E_ARG;
  if (!ids_ok(e, n_docs, docs)) return CRDT_E_ARG;
  std::vector<u64> ids(n_docs);
  std::vector<std::vector<Rec>> streams(n_docs);
  std::vector<StreamNeeds> needs(n_docs);
  std::vector<const std::vector<Rec>*> sp(n_docs);
  for (uint64_t i = 0; i < n_docs; i++) {
    if (docs[i] >= e->n_docs) return CRDT_E_ARG;
    ids[i] = docs[i];
    u32 a = e->docs[docs[i]].agents.get_or_create(agent);
    encode_gen(streams[i], needs[i], a, n_ops, (u32)mix64(seed ^ docs[i]));
    sp[i] = &streams[i];
  }
  return e->stage(ids, sp, needs);
}

int crdt_reset_async(crdt_engine* e) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  // capacities planned from now on cover the histories since this reset: the staged streams
  for (auto& h : e->docs) h.cum = h.staged;
  hipLaunchKernelGGL(k_reset_recpos, dim3((u32)((e->n_docs + 255) / 256)), dim3(256), 0, e->stream, e->st, (u32)e->n_docs, 0u);
  return e->init_all();
}

int crdt_run(crdt_engine* e, int32_t* doc_status) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  return e->run(doc_status);
}

int crdt_run_async(crdt_engine* e) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  return e->launch_replay();
}

int crdt_publish_async(crdt_engine* e) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  return e->publish();
}

int crdt_sync(crdt_engine* e) {
  if (!e) return CRDT_E_ARG;
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

int crdt_apply_local(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                     const crdt_local_txn* txns, const crdt_local_op* ops, int32_t* doc_status) {
  int r = stage_local_impl(e, n_docs, docs, txn_off, txns, ops);
  if (r) return r;
  std::vector<int32_t> all(e->n_docs);
  r = e->run(all.data());
  if (r) return r;
  if (doc_status)
    for (uint64_t i = 0; i < n_docs; i++) doc_status[i] = all[docs[i]];
  return 0;
}

int crdt_apply_remote_wire(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint8_t* const* wire,
                           const uint64_t* wire_len, int32_t* doc_status) {
  int r = crdt_stage_remote_wire(e, n_docs, docs, wire, wire_len);
  if (r) return r;
  std::vector<int32_t> all(e->n_docs);
  r = e->run(all.data());
  if (r) return r;
  if (doc_status)
    for (uint64_t i = 0; i < n_docs; i++) doc_status[i] = all[docs[i]];
  return 0;
}

int crdt_set_share_streams(crdt_engine* e, int on) {
  if (!e) return CRDT_E_ARG;
  e->share_streams = on != 0;
  return 0;
}

int crdt_set_query_kernel(crdt_engine* e, int mode) {
  if (!e || mode < CRDT_QUERY_LDS || mode > CRDT_QUERY_MERGE) return CRDT_E_ARG;
  e->query_kernel = mode;
  return 0;
}

int crdt_set_device_intern(crdt_engine* e, int on) {
  if (!e) return CRDT_E_ARG;
  e->intern_on_device = on != 0;
  return 0;
}

int crdt_fit(crdt_engine* e) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  return e->fit();
}

int crdt_fit_note(crdt_engine* e, int apply) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  return e->fit(apply ? 2 : 1);
}

int crdt_reseed_random_async(crdt_engine* e, uint64_t seed, uint64_t id_base) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  if (!e->n_docs) return 0;
  hipLaunchKernelGGL(k_reseed_gen, dim3((u32)((e->n_docs + 255) / 256)), dim3(256), 0, e->stream, e->pools_view(e->pools),
                     (u32)e->n_docs, (u64)seed, (u64)id_base);
  HIPCHK(hipGetLastError());
  e->published = false;
  e->materialized = false;
  return 0;
}

int crdt_digest_dev_async(crdt_engine* e, uint64_t* dev_out) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !dev_out) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  r = e->digest_now();  // (the current state's: never the previous replay's)
  if (r) return r;
  HIPCHK(hipMemcpyAsync(dev_out, e->digest, e->n_docs * 8, hipMemcpyDeviceToDevice, e->stream));
  return 0;
}

int crdt_pos_to_loc_dev_async(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint32_t* pos, uint16_t* agent, uint32_t* seq) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  if (!e->published) {
    int r = e->publish();
    if (r) return r;
  }
  if (!n) return 0;
  int mode = e->qmode();
  if (mode == CRDT_QUERY_MERGE) {  // sorted batches: merge path against vpos, chunk by chunk
    u64 blocks = (n + QBLK_Q - 1) / QBLK_Q;
    if (blocks > 0x7FFFFFFFull) return CRDT_E_ARG;
    if (e->L == 32) hipLaunchKernelGGL(k_pos_to_loc_merge<32>, dim3((u32)blocks), dim3(QM_T), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
    else hipLaunchKernelGGL(k_pos_to_loc_merge<4>, dim3((u32)blocks), dim3(QM_T), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
  } else if (mode == CRDT_QUERY_PER_THREAD) {
    u32 blocks = (u32)std::min<u64>((n + 255) / 256, 8192);
    if (e->L == 32) hipLaunchKernelGGL(k_pos_to_loc<32>, dim3(blocks), dim3(256), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
    else hipLaunchKernelGGL(k_pos_to_loc<4>, dim3(blocks), dim3(256), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
  } else {  // chunks of QBLK_Q queries; a one-document chunk searches its vpos staged in LDS
    u64 blocks = (n + QBLK_Q - 1) / QBLK_Q;
    if (blocks > 0x7FFFFFFFull) return CRDT_E_ARG;
    if (e->L == 32) hipLaunchKernelGGL(k_pos_to_loc_blk<32>, dim3((u32)blocks), dim3(QBLK_T), QBLK_LDS, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
    else hipLaunchKernelGGL(k_pos_to_loc_blk<4>, dim3((u32)blocks), dim3(QBLK_T), QBLK_LDS, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, pos, agent, seq);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int crdt_loc_to_pos_dev_async(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint16_t* agent, const uint32_t* seq, uint32_t* pos, uint8_t* deleted) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  if (!e->published) {
    int r = e->publish();
    if (r) return r;
  }
  if (!n) return 0;
  u32 blocks = (u32)std::min<u64>((n + 255) / 256, 8192);
  // (merge mode: sorted (agent, seq) batches keep item_orders / bitmap / rank reads in cache, so
  // the thread-per-query kernel needs no staging)
  int mode = e->qmode();
  if (mode == CRDT_QUERY_PER_THREAD || mode == CRDT_QUERY_MERGE) {
    if (e->L == 32) hipLaunchKernelGGL(k_loc_to_pos<32>, dim3(blocks), dim3(256), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, agent, seq, pos, deleted);
    else hipLaunchKernelGGL(k_loc_to_pos<4>, dim3(blocks), dim3(256), 0, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, agent, seq, pos, deleted);
  } else {  // chunks of QBLK_Q queries; a one-document chunk ranks orders in its LDS-staged bitmap
    u64 nb = (n + QBLK_Q - 1) / QBLK_Q;
    if (nb > 0x7FFFFFFFull) return CRDT_E_ARG;
    if (e->L == 32) hipLaunchKernelGGL(k_loc_to_pos_blk<32>, dim3((u32)nb), dim3(QBLK_T), QBLK_W * 8u, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, agent, seq, pos, deleted);
    else hipLaunchKernelGGL(k_loc_to_pos_blk<4>, dim3((u32)nb), dim3(QBLK_T), QBLK_W * 8u, e->stream, e->pools_view(e->pools), e->pub_view(), (u32)e->n_docs, n, doc, agent, seq, pos, deleted);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int crdt_pos_to_loc(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint32_t* pos, uint16_t* agent, uint32_t* seq) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n && (!doc || !pos || !agent || !seq))) return CRDT_E_ARG;
  if (!n) return 0;
  int r = e->ensure_published();
  if (r) return r;
  u64 bytes = n * (4 + 4 + 2 + 4) + 64;
  r = e->scratch(bytes);
  if (r) return r;
  char* b = (char*)e->qbuf;
  u32* d_doc = (u32*)b;
  u32* d_pos = d_doc + n;
  u32* d_seq = d_pos + n;
  u16* d_ag = (u16*)(d_seq + n);
  HIPCHK(hipMemcpyAsync(d_doc, doc, n * 4, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(d_pos, pos, n * 4, hipMemcpyHostToDevice, e->stream));
  r = crdt_pos_to_loc_dev_async(e, n, d_doc, d_pos, d_ag, d_seq);
  if (r) return r;
  HIPCHK(hipMemcpyAsync(agent, d_ag, n * 2, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(seq, d_seq, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

int crdt_loc_to_pos(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint16_t* agent, const uint32_t* seq, uint32_t* pos, uint8_t* deleted) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n && (!doc || !agent || !seq || !pos || !deleted))) return CRDT_E_ARG;
  if (!n) return 0;
  int r = e->ensure_published();
  if (r) return r;
  u64 bytes = n * (4 + 4 + 4 + 2 + 1) + 64;
  r = e->scratch(bytes);
  if (r) return r;
  char* b = (char*)e->qbuf;
  u32* d_doc = (u32*)b;
  u32* d_seq = d_doc + n;
  u32* d_pos = d_seq + n;
  u16* d_ag = (u16*)(d_pos + n);
  u8* d_del = (u8*)(d_ag + n);
  HIPCHK(hipMemcpyAsync(d_doc, doc, n * 4, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(d_seq, seq, n * 4, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(d_ag, agent, n * 2, hipMemcpyHostToDevice, e->stream));
  r = crdt_loc_to_pos_dev_async(e, n, d_doc, d_ag, d_seq, d_pos, d_del);
  if (r) return r;
  HIPCHK(hipMemcpyAsync(pos, d_pos, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(deleted, d_del, n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

int crdt_doc_len(crdt_engine* e, uint64_t n, const uint32_t* doc, uint32_t* len) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n && (!doc || !len))) return CRDT_E_ARG;
  int r = e->pull_states();
  if (r) return r;
  for (uint64_t i = 0; i < n; i++) {
    if (doc[i] >= e->n_docs) return CRDT_E_ARG;
    len[i] = e->st_h[doc[i]].len;
  }
  return 0;
}

int crdt_doc_status(crdt_engine* e, int32_t* status) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !status) return CRDT_E_ARG;
  int r = e->pull_states();
  if (r) return r;
  for (u64 d = 0; d < e->n_docs; d++) status[d] = e->st_h[d].status == ST_NEED_CAPACITY ? ST_CAPACITY : e->st_h[d].status;
  return 0;
}

int crdt_digest(crdt_engine* e, uint64_t* per_doc) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !per_doc) return CRDT_E_ARG;
  int r = e->ensure_published();
  if (r) return r;
  r = e->digest_now();
  if (r) return r;
  HIPCHK(hipMemcpyAsync(per_doc, e->digest, e->n_docs * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

int crdt_canon_counts(crdt_engine* e, uint32_t* per_doc) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !per_doc) return CRDT_E_ARG;
  int r = e->ensure_published();
  if (r) return r;
  HIPCHK(hipMemcpyAsync(per_doc, e->canon_n, e->n_docs * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

// Export: walk the document's directory on the host from device copies.
int crdt_export_sizes(crdt_engine* e, uint32_t doc, uint64_t* s) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || doc >= e->n_docs || !s) return CRDT_E_ARG;
  int r = e->ensure_published();
  if (r) return r;
  r = e->pull_states();
  if (r) return r;
  const DocState& st = e->st_h[doc];
  u32 cn = 0;
  HIPCHK(hipMemcpy(&cn, e->canon_n + doc, 4, hipMemcpyDeviceToHost));
  s[0] = st.n_entries; s[1] = st.n_leaves; s[2] = cn; s[3] = st.n_cwo; s[4] = st.n_del; s[5] = st.n_dd;
  s[6] = st.n_txn; s[7] = st.n_par; s[8] = st.n_fr; s[9] = st.n_agents; s[10] = st.next_order; s[11] = st.len;
  return 0;
}

int crdt_export(crdt_engine* e, uint32_t doc, uint32_t* raw4, uint32_t* leaf_sizes, uint32_t* canon4, uint32_t* cwo4,
                uint32_t* del3, uint32_t* dd3, uint32_t* txn5, uint32_t* parents, uint32_t* frontier) {
  uint64_t s[12];
  int r = crdt_export_sizes(e, doc, s);
  if (r) return r;
  const DocState& st = e->st_h[doc];
  const DocSeg& sg = e->seg_h[doc];
  u32 L = e->L;
  if (raw4 || leaf_sizes) {
    std::vector<GroupRec> groups(st.ng);
    HIPCHK(hipMemcpy(groups.data(), e->pools.groups + sg.grp_base, st.ng * sizeof(GroupRec), hipMemcpyDeviceToHost));
    std::vector<u32> dl((size_t)st.n_blocks * GROUP);
    HIPCHK(hipMemcpy(dl.data(), e->pools.dir_leaf + sg.blk_base * GROUP, dl.size() * 4, hipMemcpyDeviceToHost));
    std::vector<Span> lv((size_t)st.n_leaves * L);
    HIPCHK(hipMemcpy(lv.data(), e->pools.leaves + sg.leaf_base * L, lv.size() * sizeof(Span), hipMemcpyDeviceToHost));
    u64 k = 0, li = 0;
    for (u32 g = 0; g < st.ng; g++)
      for (u32 i = 0; i < groups[g].cnt; i++) {
        u32 leaf = dl[(size_t)groups[g].blk * GROUP + i];
        u32 n = 0;
        for (u32 j = 0; j < L; j++) {
          const Span& sp = lv[(size_t)leaf * L + j];
          if (sp.len == 0) continue;
          if (raw4) std::memcpy(raw4 + 4 * k, &sp, 16);
          k++;
          n++;
        }
        if (leaf_sizes) leaf_sizes[li] = n;
        li++;
      }
  }
  if (canon4 && s[2]) HIPCHK(hipMemcpy(canon4, e->canon + sg.canon_base, s[2] * 16, hipMemcpyDeviceToHost));
  if (cwo4 && st.n_cwo) HIPCHK(hipMemcpy(cwo4, e->pools.cwo + sg.cwo_base, st.n_cwo * 16, hipMemcpyDeviceToHost));
  if (del3 && st.n_del) HIPCHK(hipMemcpy(del3, e->pools.dels + sg.del_base, st.n_del * 12, hipMemcpyDeviceToHost));
  if (dd3 && st.n_dd) {  // flatten the blocks in directory order
    std::vector<DDBlk> dir(st.n_ddb);
    std::vector<DDRun> ent((size_t)st.n_ddb * DD_BLK);
    HIPCHK(hipMemcpy(dir.data(), e->pools.ddb + sg.dd_base, dir.size() * sizeof(DDBlk), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ent.data(), e->pools.dd + sg.dd_base * DD_BLK, ent.size() * sizeof(DDRun), hipMemcpyDeviceToHost));
    u64 k = 0;
    for (const DDBlk& B : dir)
      for (u32 i = 0; i < B.cnt && k < st.n_dd; i++, k++) std::memcpy(dd3 + 3 * k, &ent[(size_t)B.phys * DD_BLK + i], 12);
  }
  if (txn5 && st.n_txn) {
    std::vector<TxnRec> t(st.n_txn);
    HIPCHK(hipMemcpy(t.data(), e->pools.txns + sg.txn_base, st.n_txn * sizeof(TxnRec), hipMemcpyDeviceToHost));
    for (u32 i = 0; i < st.n_txn; i++) {
      txn5[5 * i] = t[i].order; txn5[5 * i + 1] = t[i].len; txn5[5 * i + 2] = t[i].shadow;
      txn5[5 * i + 3] = t[i].poff; txn5[5 * i + 4] = t[i].pn;
    }
  }
  if (parents && st.n_par) HIPCHK(hipMemcpy(parents, e->pools.parents + sg.par_base, st.n_par * 4, hipMemcpyDeviceToHost));
  if (frontier && st.n_fr) HIPCHK(hipMemcpy(frontier, e->pools.frontier + sg.fr_base, st.n_fr * 4, hipMemcpyDeviceToHost));
  return 0;
}

int crdt_debug_state(crdt_engine* e, uint32_t doc, uint32_t* out23) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || doc >= e->n_docs || !out23) return CRDT_E_ARG;
  int r = e->set_device();
  if (r) return r;
  HIPCHK(hipMemcpyAsync(out23, e->st + doc, sizeof(DocState), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return 0;
}

int crdt_device_bytes(uint64_t* current, uint64_t* peak, int reset_peak) {
  std::lock_guard<std::mutex> g(g_mem_mu);
  if (current) *current = g_mem_cur;
  if (peak) *peak = g_mem_peak;
  if (reset_peak) g_mem_peak = g_mem_cur;
  return 0;
}

uint64_t crdt_mem_bytes(const crdt_engine* e) {
  if (!e) return 0;
  return e->pools.bytes + e->rec_cap * sizeof(Rec) + e->content_cap * 4 + e->text_cap * 4 + e->canon_alloc * 28 +
         e->pub_alloc * 4 + e->probe_cap * 16 +
         e->n_docs * (sizeof(DocState) + sizeof(DocSeg) + 4 + 4 + 8);
}

int crdt_last_timings(crdt_engine* e, double* replay_ms, double* publish_ms) {
  if (!e) return CRDT_E_ARG;
  if (replay_ms) *replay_ms = e->last_replay_ms;
  if (publish_ms) *publish_ms = e->last_publish_ms;
  return 0;
}

void* crdt_stream(crdt_engine* e) { return e ? (void*)e->stream : nullptr; }

int crdt_set_content(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* stream_of_doc,
                     uint32_t n_streams, const uint64_t* stream_off, const uint32_t* content) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n_docs && (!docs || !stream_of_doc)) || !stream_off || (stream_off[n_streams] && !content))
    return CRDT_E_ARG;
  return e->set_content(n_docs, docs, stream_of_doc, n_streams, stream_off, content);
}

int crdt_set_content_copies(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* content,
                            uint64_t len) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || (n_docs && !docs) || (len && !content)) return CRDT_E_ARG;
  return e->set_content_copies(n_docs, docs, content, len);
}

int crdt_materialize_async(crdt_engine* e) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e)) return CRDT_E_ARG;
  return e->materialize();
}

int crdt_text(crdt_engine* e, uint32_t doc, uint32_t* out, uint64_t cap, uint64_t* n_out) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || doc >= e->n_docs || !n_out) return CRDT_E_ARG;
  int r = e->ensure_materialized();
  if (r) return r;
  u32 n = 0;
  HIPCHK(hipMemcpy(&n, e->tlen + doc, 4, hipMemcpyDeviceToHost));
  if (n == INVALID) return CRDT_E_ARG;  // no (or too short) content for this document
  *n_out = n;
  if (!out) return 0;
  if (cap < n) return CRDT_E_ARG;
  if (n) HIPCHK(hipMemcpy(out, e->text + e->seg_h[doc].ord_base, (u64)n * 4, hipMemcpyDeviceToHost));
  return 0;
}

int crdt_text_digest(crdt_engine* e, uint64_t* per_doc) {
  if (poisoned(e)) return CRDT_E_NOMEM;
  if (!valid(e) || !per_doc) return CRDT_E_ARG;
  int r = e->ensure_materialized();
  if (r) return r;
  HIPCHK(hipMemcpy(per_doc, e->tdigest, e->n_docs * 8, hipMemcpyDeviceToHost));
  return 0;
}

int crdt_last_materialize_ms(crdt_engine* e, double* ms) {
  if (!e || !ms) return CRDT_E_ARG;
  *ms = e->last_materialize_ms;
  return 0;
}

const char* crdt_last_error(void) { return g_last_error.c_str(); }

#ifndef CRDT_SRC_HASH
#define CRDT_SRC_HASH "unknown"
#endif
const char* crdt_build_id(void) { return CRDT_SRC_HASH; }

}  // extern "C"

// Shared with the host-only sources (trace_ingest.cpp) so every entry point reports through
// crdt_last_error().
namespace crdt {
void set_last_error(const std::string& s) { g_last_error = s; }
}  // namespace crdt
