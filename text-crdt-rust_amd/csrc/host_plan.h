// Host-side planning for the replay kernel: agent interning (ListCRDT::get_or_create_agent_id,
// doc.rs:66-89), encoding of local txns / remote wire batches into the device record stream,
// and per-document capacity planning.  Used by the engine (engine.cpp) and by the test-only CPU
// emulation harness (tests/emu).
#pragma once
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "crdt_types.h"

namespace crdt {

// Remote wire batch (see include/crdt_gpu.h):  'RTX1', name table, txns.
struct WireTxnView {
  u32 agent_name, seq, n_parents, n_ops;
  const u32* parents;  // pairs
  const u32* ops;      // 6 words each
};
struct WireView {
  std::vector<std::string> names;
  std::vector<WireTxnView> txns;
  bool parse(const uint8_t* p, size_t len) {
    size_t off = 0;
    auto rd = [&](u32& v) -> bool {
      if (off + 4 > len) return false;
      std::memcpy(&v, p + off, 4);
      off += 4;
      return true;
    };
    u32 magic, nn;
    if (!rd(magic) || magic != 0x31585452u || !rd(nn)) return false;
    names.resize(nn);
    for (u32 i = 0; i < nn; i++) {
      u32 bl;
      if (!rd(bl) || off + bl > len) return false;
      names[i].assign((const char*)p + off, bl);
      off += (bl + 3) & ~3u;
    }
    u32 nt;
    if (!rd(nt)) return false;
    if (off % 4) return false;
    txns.resize(nt);
    for (u32 t = 0; t < nt; t++) {
      WireTxnView& x = txns[t];
      if (!rd(x.agent_name) || !rd(x.seq) || !rd(x.n_parents) || !rd(x.n_ops)) return false;
      if (x.agent_name >= nn) return false;
      if (off + 8ull * x.n_parents + 24ull * x.n_ops > len) return false;
      x.parents = (const u32*)(p + off);
      off += 8ull * x.n_parents;
      x.ops = (const u32*)(p + off);
      off += 24ull * x.n_ops;
      for (u32 k = 0; k < x.n_parents; k++) if (x.parents[2 * k] >= nn) return false;
      for (u32 k = 0; k < x.n_ops; k++) {
        const u32* o = x.ops + 6 * k;
        if (o[0] > 1 || o[1] >= nn || (o[0] == 0 && o[3] >= nn)) return false;
      }
    }
    return true;
  }
};

// Per-document host metadata: agent names (creation order) and name ranks.
struct AgentTable {
  std::vector<std::string> names;
  std::unordered_map<std::string, u32> ids;
  // ListCRDT::get_or_create_agent_id
  u32 get_or_create(const std::string& n) {
    if (n == "ROOT") return ROOT_AGENT;
    auto it = ids.find(n);
    if (it != ids.end()) return it->second;
    u32 id = (u32)names.size();
    names.push_back(n);
    ids[n] = id;
    return id;
  }
  // ListCRDT::get_agent_id (lookup only; unknown -> UNKNOWN_AGENT)
  u32 lookup(const std::string& n) const {
    if (n == "ROOT") return ROOT_AGENT;
    auto it = ids.find(n);
    return it == ids.end() ? UNKNOWN_AGENT : it->second;
  }
  // rank[a] = position of names[a] in byte-lexicographic order (Rust str Ord)
  std::vector<u32> ranks() const {
    std::vector<u32> idx(names.size());
    for (u32 i = 0; i < idx.size(); i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](u32 a, u32 b) { return names[a] < names[b]; });
    std::vector<u32> r(names.size());
    for (u32 i = 0; i < idx.size(); i++) r[idx[i]] = i;
    return r;
  }
};

// Statistics of a record stream, for capacity planning.
struct StreamNeeds {
  u64 n_txn = 0, n_ltxn = 0, n_rtxn = 0, n_ops = 0, orders = 0, local_del = 0, remote_del_ops = 0, remote_parents = 0;
  // largest single txn (the replay checks room for one txn before applying it)
  u32 max_ops = 0, max_del = 0, max_len = 0, max_parents = 0;
  u64 probes = 0;  // PROBE records (their documents keep the order -> leaf map)
  u64 local_del_ops = 0;  // LocalOps that delete
  u32 max_rdel_len = 0;   // longest remote txn with a delete op (the double-delete reserve, fits())
  std::vector<u32> txns_per_agent;
  void txn_max(u32 ops, u64 del, u64 len, u32 parents) {
    max_ops = std::max(max_ops, ops);
    max_del = (u32)std::min<u64>(std::max<u64>(max_del, del), 0xFFFFFFFFull);
    max_len = (u32)std::min<u64>(std::max<u64>(max_len, len), 0xFFFFFFFFull);
    max_parents = std::max(max_parents, parents);
  }
  void agent_txn(u32 a) {
    if (a >= 0xFFFE) return;
    if (txns_per_agent.size() <= a) txns_per_agent.resize(a + 1, 0);
    txns_per_agent[a]++;
  }
};

// Encode one local txn (LocalOp list, common.rs:45-50) for `agent`.
// One compact local record: one LocalOp of one txn (LC: pos, del, ins).
inline void encode_lc(std::vector<Rec>& out, StreamNeeds& nd, u32 agent, u32 pos, u32 del, u32 ins) {
  out.push_back(Rec{(REC_LC << 28) | agent, pos, del, ins});
  nd.txn_max(1, del, (u64)del + ins, 0);
  nd.local_del += del;
  nd.local_del_ops += del != 0;
  nd.n_txn++;
  nd.n_ltxn++;
  nd.n_ops++;
  nd.orders += (u64)del + ins;
  nd.agent_txn(agent);
}
// A local txn whose LocalOps each delete or insert, not both, is what the replay's fast paths take
// (fast_txn: one op, a delete or an insert); a replace op (delete then insert at the same pos) and
// a txn of several ops go to the general interpreter -- 7 % of rustcode's and sveltecomponent's
// txns, at ~8x the cost of a fast one.  Such a txn is encoded as one compact record per part,
// each part a txn of its own, in order: [pos, pos + del) deleted, then the insert at pos, then the
// next op.  The state is the same: apply_local_txn applies a txn's ops in order, deletes before
// the insert (doc.rs:386-465), with consecutive orders and seqs; a local txn's parents are the
// frontier, which is the previous part's last order, so insert_txn merges every part into the
// previous part's txn run (doc.rs:350-374: one parent = the run's last order, same shadow), and
// client_with_order / item_orders / deletes extend their runs exactly as one txn's ops do.
// Ops that neither delete nor insert are skipped (apply_local_txn skips them); a txn of only such
// ops keeps its general form (its empty-txn status).
inline void encode_local_txn(std::vector<Rec>& out, StreamNeeds& nd, u32 agent, const u32* ops3, u32 nops) {
  u64 span = 0, dels = 0;
  for (u32 k = 0; k < nops; k++) { span += (u64)ops3[3 * k + 1] + ops3[3 * k + 2]; dels += ops3[3 * k + 1]; }
  u32 span32 = span > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)span;
  u32 dels32 = dels > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)dels;
  if (agent <= 0xFFFFu && span != 0 && span <= 0xFFFFFFFFull &&
      (nops > 1 || (ops3[1] != 0 && ops3[2] != 0))) {  // parts, one compact record each
    for (u32 k = 0; k < nops; k++) {
      u32 pos = ops3[3 * k], del = ops3[3 * k + 1], ins = ops3[3 * k + 2];
      if (del) encode_lc(out, nd, agent, pos, del, 0);
      if (ins) encode_lc(out, nd, agent, pos, 0, ins);
    }
    return;
  }
  nd.txn_max(nops, dels, span, 0);
  if (nops == 1 && agent <= 0xFFFFu && span <= 0xFFFFFFFFull) {  // one LocalOp: one compact record
    out.push_back(Rec{(REC_LC << 28) | agent, ops3[0], ops3[1], ops3[2]});
    nd.local_del += ops3[1];
    nd.local_del_ops += ops3[1] != 0;
  } else {
    out.push_back(Rec{(REC_LTXN << 28) | (nops & 0x0FFFFFFFu), agent, dels32, span32});
    for (u32 k = 0; k < nops; k++) {
      out.push_back(Rec{REC_LOP << 28, ops3[3 * k], ops3[3 * k + 1], ops3[3 * k + 2]});
      nd.local_del += ops3[3 * k + 1];
      nd.local_del_ops += ops3[3 * k + 1] != 0;
    }
  }
  nd.n_txn++;
  nd.n_ltxn++;
  nd.n_ops += nops;
  nd.orders += span;
  nd.agent_txn(agent);
}

// Encode a remote wire batch for one document, interning authors in txn order exactly as
// apply_remote_txn does (doc.rs:243 get_or_create for the author; doc.rs:237 lookup for ids).
inline void encode_remote(std::vector<Rec>& out, StreamNeeds& nd, AgentTable& at, const WireView& wv) {
  std::vector<u32> cache(wv.names.size(), 0xFFFFFFFFu);
  for (const WireTxnView& t : wv.txns) {
    size_t before = at.names.size();
    u32 author = at.get_or_create(wv.names[t.agent_name]);
    if (at.names.size() != before)  // a new agent exists from now on: forget negative lookups
      for (u32 i = 0; i < cache.size(); i++) if (cache[i] == UNKNOWN_AGENT) cache[i] = 0xFFFFFFFFu;
    auto res = [&](u32 ni) -> u32 {
      if (cache[ni] == 0xFFFFFFFFu) cache[ni] = at.lookup(wv.names[ni]);
      return cache[ni];
    };
    u64 tl = 0;
    bool zero = false;
    for (u32 k = 0; k < t.n_ops; k++) {
      u32 len = t.ops[6 * k + 5];
      if (len == 0 || len > 0x0FFFFFFFu) zero = true;
      tl += len;
    }
    u32 tl32 = tl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)tl;
    nd.txn_max(t.n_ops, t.n_ops, tl, t.n_parents);
    u32 has_del = 0;
    for (u32 k = 0; k < t.n_ops; k++)
      if (t.ops[6 * k] != 0) { has_del = 1; nd.max_rdel_len = std::max<u32>(nd.max_rdel_len, tl32); break; }
    // the common shape -- one op on the author's own items (or ROOT), the author's previous txn
    // as the only parent -- is one compact record (crdt_types.h RC)
    if (t.n_ops == 1 && t.n_parents == 1 && author < 0xFFFEu && t.seq >= 1 && res(t.parents[0]) == author &&
        t.parents[1] == t.seq - 1) {
      const u32* o = t.ops;
      u32 len = o[5];
      auto org = [&](u32 ni, u32 seq, u32& enc) -> bool {  // author's item or ROOT
        u32 a = res(ni);
        if (a == ROOT_AGENT) { enc = 0xFFFFFFFFu; return true; }
        enc = seq;
        return a == author && seq != 0xFFFFFFFFu;
      };
      u32 e2 = 0, e3 = 0;
      bool ok = len >= 1 && len <= 0x7FFu;
      if (ok && o[0] == 0) ok = org(o[1], o[2], e2) && org(o[3], o[4], e3);
      else if (ok) ok = res(o[1]) == author && o[2] != 0xFFFFFFFFu && (e2 = o[2], true);
      if (ok) {
        out.push_back(Rec{(REC_RC << 28) | ((o[0] ? 1u : 0u) << 27) | (len << 16) | author, t.seq, e2, e3});
        if (o[0]) nd.remote_del_ops++;
        nd.n_txn++;
        nd.n_rtxn++;
        nd.n_ops += 1;
        nd.orders += tl;
        nd.remote_parents += 1;
        nd.agent_txn(author);
        continue;
      }
    }
    if (t.n_ops > RTXN_NOPS_MASK) zero = true;  // (no stream holds such a txn: rejected as malformed)
    out.push_back(Rec{(REC_RTXN << 28) | ((zero ? 1u : 0u) << 27) | (has_del << RTXN_DEL_BIT) | (t.n_ops & RTXN_NOPS_MASK),
                      (author & 0xFFFFu) | ((t.n_parents & 0xFFFFu) << 16), t.seq, tl32});
    for (u32 k = 0; k < t.n_ops; k++) {
      const u32* o = t.ops + 6 * k;
      u32 len = o[5] & 0x0FFFFFFFu;
      if (o[0] == 0) {
        out.push_back(Rec{(REC_RINS << 28) | len, (res(o[1]) & 0xFFFFu) | ((res(o[3]) & 0xFFFFu) << 16), o[2], o[4]});
      } else {
        out.push_back(Rec{(REC_RDEL << 28) | len, res(o[1]) & 0xFFFFu, o[2], 0});
        nd.remote_del_ops++;
      }
    }
    for (u32 k = 0; k < t.n_parents; k++)
      out.push_back(Rec{REC_RPARENT << 28, res(t.parents[2 * k]) & 0xFFFFu, t.parents[2 * k + 1], 0});
    nd.n_txn++;
    nd.n_rtxn++;
    nd.n_ops += t.n_ops;
    nd.orders += tl;
    nd.remote_parents += t.n_parents;
    nd.agent_txn(author);
  }
}

// A PROBE record: after the txns before it, answer pos_to_loc(pos) and loc_to_pos(agent, seq).
inline void encode_probe(std::vector<Rec>& out, StreamNeeds& nd, u32 pos, u32 agent, u32 seq) {
  out.push_back(Rec{REC_PROBE << 28, pos, agent, seq});
  nd.probes++;
}

// One GEN record: `n_ops` local txns of one generated LocalOp each (gen_op, on the device).
// Orders and delete runs are estimates (about 2.8 orders per op for make_random_change's
// distribution); a table that fills stops the document resumably and grows.
inline void encode_gen(std::vector<Rec>& out, StreamNeeds& nd, u32 agent, u32 n_ops, u32 seed) {
  out.push_back(Rec{REC_GEN << 28, agent, n_ops, seed});
  nd.txn_max(1, 10, 10, 0);  // make_random_change deletes <= 10 chars
  nd.n_txn += n_ops;
  nd.n_ltxn += n_ops;
  nd.n_ops += n_ops;
  nd.orders += 3ull * n_ops;
  nd.local_del += n_ops;
  nd.local_del_ops += n_ops;
  if (agent < 0xFFFE) {
    if (nd.txns_per_agent.size() <= agent) nd.txns_per_agent.resize(agent + 1, 0);
    nd.txns_per_agent[agent] += n_ops;
  }
}

// Capacities for a fresh document that will apply `nd` (heuristic leaf capacity; everything
// else is an upper bound).  Growth for leaves/blocks is handled by the caller on ST_CAPACITY.
// Leaves are bounded only by the two-level root's LDS top level: blk_cap = leaf_cap/32 + 2 groups
// in rows of >= 32, under <= ROOT_CAP_MAX top entries (engine.hip hroot_top).
constexpr u32 MAX_LEAVES = 32u * 32u * (ROOT_CAP_MAX - 64u);

struct Caps {
  u32 leaf, blk, map, cwo, arun, del, dd, txn, par, agent, fr;
  u32 ord;        // > every order the document will hold (published index, text)
  u32 canon = 0;  // canonical spans (0: bounded by the leaf capacity, leaf * L)
};
inline u32 blk_cap_for(u32 leaf_cap) { return leaf_cap / 32 + 2; }
// LDS root groups per wave for a document with `blk_cap` directory blocks (a multiple of 64)
inline u32 root_cap_for(u32 blk_cap) {
  u32 r = (blk_cap + 63u) & ~63u;
  return r < ROOT_CAP_MIN ? ROOT_CAP_MIN : r;
}
inline Caps plan_caps(const StreamNeeds& nd, u32 n_agents, bool track, u32 leaf_div = 48) {
  Caps c;
  u64 leaves = 64 + nd.n_ops / leaf_div;
  c.leaf = (u32)std::min<u64>(leaves, 1 + 2 * nd.n_ops + 1);
  if (c.leaf < 64) c.leaf = 64;
  if (c.leaf > MAX_LEAVES) c.leaf = MAX_LEAVES;
  c.blk = blk_cap_for(c.leaf);
  c.fr = FRONTIER_CAP0;
  c.map = track ? (u32)std::min<u64>(nd.orders + 1, 0xFFFFFFFFull) : 0;
  c.ord = (u32)std::min<u64>(nd.orders + 1, 0xFFFFFFFFull);
  // RLE tables usually coalesce far below one run per txn; start small and grow on demand
  // (ST_NEED_CAPACITY is resumable), exact bounds otherwise.
  c.cwo = (u32)std::min<u64>(nd.n_txn + 1, 256 + nd.n_txn / 64);
  c.txn = c.cwo;
  u64 arun = 0;
  for (u32 a = 0; a < n_agents; a++) arun += (a < nd.txns_per_agent.size() ? nd.txns_per_agent[a] : 0) + 1;
  c.arun = (u32)arun;
  // delete runs: at most one per deleted item, usually one or two per delete op (a table that
  // fills stops its document resumably and grows)
  c.del = (u32)std::min<u64>(std::min<u64>(nd.local_del + nd.remote_del_ops, 2 * (nd.local_del_ops + nd.remote_del_ops) + 64) + 1,
                             0xFFFFFFFFull);
  // double-delete blocks: grown on demand (rare but for config 5).  fits() reserves
  // (4 * entries + 2 * txn_len + 2) / 32 + 2 blocks before a remote delete txn, so the first
  // capacity covers the stream's longest txn on an empty table: no relaunch just for its reserve.
  c.dd = nd.remote_del_ops ? std::max<u32>(4u, (u32)std::min<u64>((2ull * nd.max_rdel_len + 2) / 32 + 3, 0x7FFFFFFFull)) : 0u;
  c.par = (u32)std::min<u64>(nd.remote_parents + nd.n_txn + 64 + 1, 1024 + (nd.remote_parents + nd.n_txn) / 64);
  c.agent = n_agents;
  return c;
}

}  // namespace crdt
