// TEST INFRASTRUCTURE: runs replay_core.h on the CPU (WaveCPU backend) for single documents,
// using the same host planning code as the engine, and exports the resulting state in the
// oracle's export format so tests can diff the GPU algorithm against the oracle without a GPU.
#define CRDT_EMU_CHECKS 1  // replay preconditions checked (crdt_types.h CRDT_EXPECT)
#ifdef CRDT_EMU_STATS  // statistics build (make stats): event counters of replay_core.h's CRDT_STAT sites
static unsigned long long g_stat[128];
#define CRDT_STAT(k, v) (g_stat[(k)] += (unsigned long long)(v))
static unsigned long long g_field[2][192];  // context reads / writes per slot
#define WCPU_COUNT(kind, f) (g_stat[124 + (kind > 3 ? 3 : kind)]++, (kind) < 2 ? (void)g_field[(kind)][(f) % 192]++ : (void)0)  // (context reads / writes / cache reads / other)
// memory lines (128 B) each op touches, by pool: WaveCPU reports the bytes its WaveGPU twin reads /
// writes (WCPU_MEM); an epoch (one fast_txn / apply_txn call, CRDT_MEM_EPOCH) counts every line it
// touched once, as a read line and / or a written line
void emu_mem_touch(const void* p, unsigned long long n, int wr);
void emu_mem_epoch();
static const void* g_mem_doc = nullptr;  // (the EmuDoc being replayed)
#define WCPU_MEM(p, n, wr) emu_mem_touch((const void*)(p), (unsigned long long)(n), (wr))
#define CRDT_MEM_EPOCH() emu_mem_epoch()
#endif
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "host_plan.h"
#include "replay_core.h"
#include "wave_cpu.h"

using namespace crdt;

namespace {

struct EmuDoc {
  u32 L;
  AgentTable agents;
  std::vector<Span> leaves;
  std::vector<u32> dir_leaf, dir_vis, sol, leaf_of, parents, frontier;
  std::vector<u16> agent_of;
  std::vector<u32> leaf_agents;
  std::vector<CwoRun> cwo;
  std::vector<ARun> arun;
  std::vector<DelRun> dels;
  std::vector<DDRun> dd;
  std::vector<DDBlk> ddb;
  std::vector<TxnRec> txns;
  std::vector<AgentRec> agent_tab;
  std::vector<GroupRec> groups;
  std::vector<Rec> recs;
  std::vector<uint4> probe;
  DocSeg seg{};
  DocState st{};
  bool inited = false;

  Pools pools() {
    Pools p{};
    p.leaves = leaves.data();
    p.dir_leaf = dir_leaf.data();
    p.dir_vis = dir_vis.data();
    p.slot_of_leaf = sol.data();
    p.leaf_of = leaf_of.data();
    p.agent_of = agent_of.data();
    p.leaf_agents = leaf_agents.data();
    p.cwo = cwo.data();
    p.arun = arun.data();
    p.dels = dels.data();
    p.dd = dd.data();
    p.ddb = ddb.data();
    p.txns = txns.data();
    p.parents = parents.data();
    p.frontier = frontier.data();
    p.agents = agent_tab.data();
    p.groups = groups.data();
    p.recs = recs.data();
    p.probe = probe.empty() ? nullptr : probe.data();
    p.seg = &seg;
    p.st = &st;
    return p;
  }

  // (Re)allocate for a stream; a fresh document only (emulator scope).
  void prepare(const StreamNeeds& nd, bool track, u32 leaf_div) {
    Caps c = plan_caps(nd, (u32)agents.names.size(), track, leaf_div);
    leaves.assign((size_t)c.leaf * L, Span{0, 0, 0, 0});
    sol.assign(2 * (size_t)c.leaf, 0);  // {slot, successor} per leaf
    dir_leaf.assign((size_t)c.blk * GROUP, 0);
    dir_vis.assign((size_t)c.blk * GROUP, 0);
    leaf_of.assign(std::max<u32>(c.map, 1), 0xDEADBEEFu);
    agent_of.assign(std::max<u32>(c.map, 1), 0xBEEFu);
    leaf_agents.assign((size_t)c.leaf * lag_words(L), 0xDEADBEEFu);  // (garbage but word 0: rows are stale until written)
    for (size_t k = 0; k < leaf_agents.size(); k += lag_words(L)) leaf_agents[k] = 0;
    cwo.assign(c.cwo, CwoRun{});
    arun.assign(c.arun, ARun{});
    dels.assign(c.del, DelRun{});
    dd.assign((size_t)std::max<u32>(c.dd, 1) * DD_BLK, DDRun{});
    ddb.assign(std::max<u32>(c.dd, 1), DDBlk{});
    txns.assign(c.txn, TxnRec{});
    parents.assign(c.par, 0);
    frontier.assign(c.fr, 0);
    groups.assign(c.blk, GroupRec{});
    agent_tab.assign(std::max<u32>(c.agent, 1), AgentRec{});
    std::vector<u32> rk = agents.ranks();
    u32 base = 0;
    for (u32 a = 0; a < agents.names.size(); a++) {
      u32 cap = (a < nd.txns_per_agent.size() ? nd.txns_per_agent[a] : 0) + 1;
      agent_tab[a] = AgentRec{base, 0, cap, rk[a], 0, 0, 0, 0};
      base += cap;
    }
    seg = DocSeg{};
    seg.leaf_cap = c.leaf; seg.blk_cap = c.blk; seg.map_cap = c.map; seg.cwo_cap = c.cwo;
    seg.arun_cap = c.arun; seg.del_cap = c.del; seg.dd_cap = c.dd; seg.txn_cap = c.txn;
    seg.par_cap = c.par; seg.agent_cap = c.agent; seg.rec_n = (u32)recs.size();
    seg.fr_cap = c.fr; seg.grp_cap = c.blk;
    seg.flags = track ? DOC_TRACK_MAP : 0;
    if (track && agents.names.size() > 1) seg.flags |= DOC_TRACK_AGENT;  // (as the engine's stage())
    st = DocState{};
    st.n_agents = (u32)agents.names.size();
  }

  u32 grow_events = 0, grow_mask = 0;

  // Grow the tables named by cap_need (the engine does the same on the device pools).
  void grow(u32 need) {
    grow_events++;
    grow_mask |= need;
    leaf_agents.assign((size_t)seg.leaf_cap * 2 * lag_words(L), 0u);  // (the engine's relayout: every row stale)
    if (need & 1u) {
      u32 nl = seg.leaf_cap * 2 > MAX_LEAVES ? MAX_LEAVES : seg.leaf_cap * 2;
      leaves.resize((size_t)nl * L, Span{0, 0, 0, 0});
      sol.resize(2 * (size_t)nl, 0);
      seg.leaf_cap = nl;
      seg.blk_cap = blk_cap_for(nl);
      seg.grp_cap = seg.blk_cap;
      dir_leaf.resize((size_t)seg.blk_cap * GROUP, 0);
      dir_vis.resize((size_t)seg.blk_cap * GROUP, 0);
      groups.resize(seg.grp_cap, GroupRec{});
    }
    if (need & 128u) { seg.fr_cap *= 2; frontier.resize(seg.fr_cap, 0); }
    if (need & 2u) { seg.cwo_cap *= 2; seg.txn_cap *= 2; cwo.resize(seg.cwo_cap); txns.resize(seg.txn_cap); }
    if (need & 4u) { seg.del_cap = seg.del_cap * 2 + 16; dels.resize(seg.del_cap); }
    if (need & 8u) { seg.par_cap = seg.par_cap * 2 + 16; parents.resize(seg.par_cap); }
    if (need & 16u) { seg.map_cap = seg.map_cap * 2 + 16; leaf_of.resize(seg.map_cap, 0xDEADBEEFu); agent_of.resize(seg.map_cap, 0xBEEFu); }
    if (need & 64u) { seg.dd_cap = seg.dd_cap * 2 + 2; dd.resize((size_t)seg.dd_cap * DD_BLK); ddb.resize(seg.dd_cap); }
    if (need & 32u) {  // re-space every agent's run list with doubled capacity
      std::vector<ARun> na;
      for (u32 a = 0; a < st.n_agents; a++) {
        AgentRec& A = agent_tab[a];
        u32 base = (u32)na.size();
        for (u32 k = 0; k < A.run_cnt; k++) na.push_back(arun[A.run_base + k]);
        na.resize(base + A.run_cap * 2 + 1);
        A.run_base = base;
        A.run_cap = A.run_cap * 2 + 1;
      }
      arun = na;
    }
  }

  template <int LL> int run_impl() {
#ifdef CRDT_EMU_STATS
    g_mem_doc = this;
#endif
    bool first = true;
    while (true) {
      Pools p = pools();
      Replayer<WaveCPU<LL>, LL> r(p, 0);
      if (first) { r.init_empty(); r.p(S_N_AGENTS, (u32)agents.names.size()); first = false; }
      else { r.p(S_STATUS, (u32)ST_OK); r.begin(); }
      // the stream's shape picks the run<> instance, as the engine picks a k_replay instance
      u32 kinds = 0;
      for (const Rec& x : recs) kinds |= 1u << rec_kind(x);
      u32 sh = shape_of_kinds(kinds);
      if (sh == SHAPE_REMOTE) r.template run<SHAPE_REMOTE>();
      else if (sh == SHAPE_GEN) r.template run<SHAPE_GEN>();
      else if (sh == SHAPE_LOCAL) r.template run<SHAPE_LOCAL>();
      else r.template run<SHAPE_ALL>();
      r.finish();
      if (st.status != ST_NEED_CAPACITY) break;
      if (st.cap_need == 0 || ((st.cap_need & 1u) && seg.leaf_cap >= MAX_LEAVES) || grow_events > 64) {
        st.status = ST_CAPACITY;  // cannot grow further
        break;
      }
      grow(st.cap_need);
    }
    return st.status;
  }
  int run() { return L == 32 ? run_impl<32>() : run_impl<4>(); }

  // walk the directory in document order
  void raw(std::vector<Span>& out, std::vector<u32>& leaf_sizes) const {
    out.clear();
    leaf_sizes.clear();
    for (u32 g = 0; g < st.ng; g++) {
      const GroupRec& G = groups[g];
      for (u32 i = 0; i < G.cnt; i++) {
        u32 lf = dir_leaf[(size_t)G.blk * GROUP + i];
        u32 n = 0;
        for (u32 k = 0; k < L; k++) if (leaves[(size_t)lf * L + k].len != 0) { out.push_back(leaves[(size_t)lf * L + k]); n++; }
        leaf_sizes.push_back(n);
      }
    }
  }
};

}  // namespace

#ifdef CRDT_EMU_STATS
#include <unordered_map>
enum { MC_LEAVES, MC_DIR, MC_SOL, MC_LEAF_OF, MC_AGENT_OF, MC_LAG, MC_CWO, MC_ARUN, MC_DELS, MC_DD, MC_DDB, MC_TXNS,
       MC_PARENTS, MC_FRONTIER, MC_AGENTS, MC_GROUPS, MC_RECS, MC_OTHER, MC_N };
static std::unordered_map<unsigned long long, unsigned> g_mem_lines;
static unsigned long long g_mem_rd[MC_N], g_mem_wr[MC_N], g_mem_epochs;
template <class V> static bool in_vec(const V& v, const void* p) {
  const char* a = (const char*)v.data();
  return (const char*)p >= a && (const char*)p < a + v.size() * sizeof(v[0]);
}
static int mem_cat(const void* p) {
  const EmuDoc* d = (const EmuDoc*)g_mem_doc;
  if (!d) return MC_OTHER;
  if (in_vec(d->leaves, p)) return MC_LEAVES;
  if (in_vec(d->dir_leaf, p) || in_vec(d->dir_vis, p)) return MC_DIR;
  if (in_vec(d->sol, p)) return MC_SOL;
  if (in_vec(d->leaf_of, p)) return MC_LEAF_OF;
  if (in_vec(d->agent_of, p)) return MC_AGENT_OF;
  if (in_vec(d->leaf_agents, p)) return MC_LAG;
  if (in_vec(d->cwo, p)) return MC_CWO;
  if (in_vec(d->arun, p)) return MC_ARUN;
  if (in_vec(d->dels, p)) return MC_DELS;
  if (in_vec(d->dd, p)) return MC_DD;
  if (in_vec(d->ddb, p)) return MC_DDB;
  if (in_vec(d->txns, p)) return MC_TXNS;
  if (in_vec(d->parents, p)) return MC_PARENTS;
  if (in_vec(d->frontier, p)) return MC_FRONTIER;
  if (in_vec(d->agent_tab, p)) return MC_AGENTS;
  if (in_vec(d->groups, p)) return MC_GROUPS;
  if (in_vec(d->recs, p)) return MC_RECS;
  return MC_OTHER;
}
void emu_mem_touch(const void* p, unsigned long long n, int wr) {
  if (!n) return;
  unsigned long long a = (unsigned long long)p;
  unsigned c = (unsigned)mem_cat(p);
  for (unsigned long long ln = a >> 7; ln <= (a + n - 1) >> 7; ln++) {
    unsigned& f = g_mem_lines[ln];
    f |= (wr ? 2u : 1u) | ((c + 1u) << 2);
  }
}
void emu_mem_epoch() {
  for (auto& kv : g_mem_lines) {
    unsigned c = (kv.second >> 2) - 1u;
    if (c >= MC_N) c = MC_OTHER;
    if (kv.second & 1u) g_mem_rd[c]++;
    if (kv.second & 2u) g_mem_wr[c]++;
  }
  g_mem_lines.clear();
  g_mem_epochs++;
}
#endif

extern "C" {

#ifdef CRDT_EMU_STATS
// lines read / written per pool (MC_* order) summed over every epoch so far; returns the epochs
unsigned long long emu_mem_stats(unsigned long long* rd, unsigned long long* wr, int reset) {
  emu_mem_epoch();
  for (int k = 0; k < MC_N; k++) { rd[k] = g_mem_rd[k]; wr[k] = g_mem_wr[k]; if (reset) g_mem_rd[k] = g_mem_wr[k] = 0; }
  unsigned long long e = g_mem_epochs;
  if (reset) g_mem_epochs = 0;
  return e;
}
#endif

void* emu_new(uint32_t leaf_cap) {
  if (leaf_cap != 4 && leaf_cap != 32) return nullptr;
  EmuDoc* d = new EmuDoc();
  d->L = leaf_cap;
  return d;
}
void emu_free(void* h) { delete (EmuDoc*)h; }
#ifdef CRDT_EMU_STATS
void emu_field_stats(uint64_t* out, int reset) {  // [2][192]: context reads, then writes, per slot
  for (int k = 0; k < 2 * 192; k++) { out[k] = g_field[k / 192][k % 192]; if (reset) g_field[k / 192][k % 192] = 0; }
}
void emu_stats(uint64_t* out, int reset) {
  for (int k = 0; k < 128; k++) { out[k] = g_stat[k]; if (reset) g_stat[k] = 0; }
}
#endif
int emu_agent(void* h, const char* name) { return (int)((EmuDoc*)h)->agents.get_or_create(name); }

// Apply a local trace (as one stream) to a fresh emulated document.
int emu_run_local(void* h, uint16_t agent, uint32_t ntxn, const uint32_t* counts, const uint32_t* patches3, uint32_t leaf_div) {
  EmuDoc* d = (EmuDoc*)h;
  StreamNeeds nd;
  d->recs.clear();
  const uint32_t* p = patches3;
  for (uint32_t t = 0; t < ntxn; t++) { encode_local_txn(d->recs, nd, agent, p, counts[t]); p += 3 * counts[t]; }
  d->prepare(nd, false, leaf_div);  // local streams never read the order -> leaf map (untracked)
  return d->run();
}

// local trace with a PROBE record after every txn; answers4 gets (agent, seq, pos, deleted)
int emu_run_local_probed(void* h, uint16_t agent, uint32_t ntxn, const uint32_t* counts, const uint32_t* patches3,
                         const uint32_t* probes3, uint32_t* answers4, uint32_t leaf_div) {
  EmuDoc* d = (EmuDoc*)h;
  StreamNeeds nd;
  d->recs.clear();
  std::vector<size_t> at;
  const uint32_t* p = patches3;
  for (uint32_t t = 0; t < ntxn; t++) {
    encode_local_txn(d->recs, nd, agent, p, counts[t]);
    p += 3 * counts[t];
    at.push_back(d->recs.size());
    encode_probe(d->recs, nd, probes3[3 * t], probes3[3 * t + 1], probes3[3 * t + 2]);
  }
  d->probe.assign(d->recs.size(), make_uint4(~0u, ~0u, ~0u, ~0u));
  d->prepare(nd, true, leaf_div);
  int st = d->run();
  for (uint32_t t = 0; t < ntxn; t++) {
    const uint4& x = d->probe[at[t]];
    answers4[4 * t] = x.x; answers4[4 * t + 1] = x.y; answers4[4 * t + 2] = x.z; answers4[4 * t + 3] = x.w;
  }
  d->probe.clear();
  return st;
}

int emu_run_random(void* h, uint16_t agent, uint32_t n_ops, uint32_t seed, uint32_t leaf_div) {
  EmuDoc* d = (EmuDoc*)h;
  StreamNeeds nd;
  d->recs.clear();
  encode_gen(d->recs, nd, agent, n_ops, seed);
  d->prepare(nd, false, leaf_div);
  return d->run();
}

int emu_run_wire(void* h, const uint8_t* wire, size_t len, uint32_t leaf_div) {
  EmuDoc* d = (EmuDoc*)h;
  WireView wv;
  if (!wv.parse(wire, len)) return ST_BAD_INPUT;
  StreamNeeds nd;
  d->recs.clear();
  encode_remote(d->recs, nd, d->agents, wv);
  d->prepare(nd, true, leaf_div);
  return d->run();
}

// A remote wire, then local txns by agent `name` (interned after the wire's agents, as a document
// that merged the wire and then edited locally names it), in one stream of the general shape.
int emu_run_wire_local(void* h, const uint8_t* wire, size_t len, const char* name, uint32_t ntxn, const uint32_t* counts,
                       const uint32_t* patches3, uint32_t leaf_div) {
  EmuDoc* d = (EmuDoc*)h;
  WireView wv;
  if (!wv.parse(wire, len)) return ST_BAD_INPUT;
  StreamNeeds nd;
  d->recs.clear();
  encode_remote(d->recs, nd, d->agents, wv);
  u16 agent = (u16)d->agents.get_or_create(name);
  const uint32_t* p = patches3;
  for (uint32_t t = 0; t < ntxn; t++) { encode_local_txn(d->recs, nd, agent, p, counts[t]); p += 3 * counts[t]; }
  d->prepare(nd, true, leaf_div);
  return d->run();
}

// sizes: [n_raw, n_leaves, n_cwo, n_del, n_dd, n_txn, n_parents, n_frontier, n_agents, next_order, len, rec_pos]
void emu_sizes(void* h, uint64_t* s) {
  EmuDoc* d = (EmuDoc*)h;
  std::vector<Span> raw;
  std::vector<u32> ls;
  d->raw(raw, ls);
  s[0] = raw.size(); s[1] = ls.size(); s[2] = d->st.n_cwo; s[3] = d->st.n_del; s[4] = d->st.n_dd;
  s[5] = d->st.n_txn; s[6] = d->st.n_par; s[7] = d->st.n_fr; s[8] = d->st.n_agents; s[9] = d->st.next_order;
  s[10] = d->st.len; s[11] = d->st.rec_pos; s[12] = d->grow_events; s[13] = d->grow_mask;
}

void emu_export(void* h, uint32_t* raw4, uint32_t* leaf_sizes, uint32_t* cwo4, uint32_t* del3, uint32_t* dd3,
                uint32_t* txn5, uint32_t* parents, uint32_t* frontier) {
  EmuDoc* d = (EmuDoc*)h;
  std::vector<Span> raw;
  std::vector<u32> ls;
  d->raw(raw, ls);
  std::memcpy(raw4, raw.data(), raw.size() * 16);
  std::memcpy(leaf_sizes, ls.data(), ls.size() * 4);
  std::memcpy(cwo4, d->cwo.data(), d->st.n_cwo * 16);
  std::memcpy(del3, d->dels.data(), d->st.n_del * 12);
  for (u32 lb = 0, k = 0; lb < d->st.n_ddb; lb++)
    for (u32 i = 0; i < d->ddb[lb].cnt; i++, k++) std::memcpy(dd3 + 3 * k, &d->dd[(size_t)d->ddb[lb].phys * DD_BLK + i], 12);
  for (u32 i = 0; i < d->st.n_txn; i++) {
    const TxnRec& t = d->txns[i];
    txn5[5 * i] = t.order; txn5[5 * i + 1] = t.len; txn5[5 * i + 2] = t.shadow; txn5[5 * i + 3] = t.poff; txn5[5 * i + 4] = t.pn;
  }
  std::memcpy(parents, d->parents.data(), d->st.n_par * 4);
  std::memcpy(frontier, d->frontier.data(), d->st.n_fr * 4);
}

// Structural invariants of the wave directory (the analogue of RangeTree::check, root.rs:165-253).
// Returns 0 if consistent, else a code and writes a message.
int emu_check(void* h, char* msg, int cap) {
  EmuDoc* d = (EmuDoc*)h;
  u64 total = 0;
  for (u32 g = 0; g < d->st.ng; g++) {
    const GroupRec& G = d->groups[g];
    u64 gsum = 0;
    for (u32 i = 0; i < G.cnt; i++) {
      u32 lf = d->dir_leaf[(size_t)G.blk * GROUP + i];
      u32 dv = d->dir_vis[(size_t)G.blk * GROUP + i];
      u32 v = 0;
      for (u32 k = 0; k < d->L; k++) v += clen(d->leaves[(size_t)lf * d->L + k]);
      if (v != dv) { snprintf(msg, cap, "group %u slot %u leaf %u: dir_vis %u content %u", g, i, lf, dv, v); return 1; }
      if (d->sol[2 * lf] != ((G.blk << 6) | i)) { snprintf(msg, cap, "slot_of_leaf[%u]=%x expected blk %u i %u", lf, d->sol[2 * lf], G.blk, i); return 2; }
      gsum += dv;
    }
    if (gsum != G.vis) { snprintf(msg, cap, "group %u vis %u sum %llu", g, G.vis, (unsigned long long)gsum); return 3; }
    total += gsum;
  }
  if (total != d->st.len) { snprintf(msg, cap, "len %u total %llu", d->st.len, (unsigned long long)total); return 4; }
  // the leaf list (slot entries' successor links) follows the directory order
  u32 prev = INVALID;
  for (u32 g = 0; g < d->st.ng; g++) {
    const GroupRec& G = d->groups[g];
    for (u32 i = 0; i < G.cnt; i++) {
      u32 lf = d->dir_leaf[(size_t)G.blk * GROUP + i];
      if (prev != INVALID && d->sol[2 * prev + 1] != lf) {
        snprintf(msg, cap, "leaf %u: successor link %u, directory successor %u", prev, d->sol[2 * prev + 1], lf);
        return 5;
      }
      prev = lf;
    }
  }
  if (prev != INVALID && d->sol[2 * prev + 1] != END_LEAF) { snprintf(msg, cap, "last leaf %u links %u", prev, d->sol[2 * prev + 1]); return 6; }
  return 0;
}

}  // extern "C"
