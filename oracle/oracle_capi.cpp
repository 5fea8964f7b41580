// ORACLE — TEST INFRASTRUCTURE ONLY (see crdt_oracle.hpp header).
// C ABI over the restatement, for tests/ (ctypes), fixture generation and bench.py's cpu_baseline leg.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>

#include "crdt_oracle.hpp"
#include "wire.hpp"

using namespace orc;

namespace {

// Records a local txn in the reference's remote form (RemoteTxn, external_txn.rs:5-30) so that
// local traces can be re-delivered through apply_remote_txn.
struct Recorder {
  wire::Writer* w;
};

RemoteId loc_id(const Doc& d, u32 order) {
  if (order == ROOT_ORDER) return RemoteId{"ROOT", 0xFFFFFFFFu};  // doc.rs:613-618 root_id()
  u16 a = 0; u32 s = 0;
  d.order_to_loc(order, a, s);
  return RemoteId{d.clients[a].name, s};
}

// Apply one local txn and emit its remote equivalent.  Deleted runs are split at
// client_with_order run boundaries so every emitted Del names contiguous (agent, seq) ranges.
int apply_local_recording(Doc& d, u16 agent, const LocalOp* ops, u32 nops, RemoteTxn& out) {
  out = RemoteTxn{};
  out.id = RemoteId{d.clients[agent].name, d.next_seq(agent)};
  for (u32 o : d.frontier) out.parents.push_back(loc_id(d, o));
  // Replay op by op through single-op txns would change the txn structure, so instead we apply
  // the whole txn and reconstruct ops from the state deltas recorded during the apply.
  size_t del_before = d.deletes.size();
  u32 del_last_len = del_before ? d.deletes.back().len : 0;
  // Inserted items are recovered from the tree by order after the apply.
  u32 first = d.next_order();
  int st = d.apply_local_txn(agent, ops, nops);
  if (st != OK) return st;
  // Walk ops again in order, consuming orders exactly as apply_local_txn assigned them.
  u32 next = first;
  // Deletes appended by this txn (DelRun keys in [first, next_order)), in key order.
  std::vector<DelRun> dl;
  for (size_t i = (del_before ? del_before - 1 : 0); i < d.deletes.size(); i++) {
    DelRun r = d.deletes[i];
    if (i + 1 == del_before) {  // last pre-existing run may have been extended by this txn
      if (r.len == del_last_len) continue;
      u32 skip = del_last_len;
      r.key += skip; r.order += skip; r.len -= skip;
    }
    if (r.key + r.len <= first) continue;
    dl.push_back(r);
  }
  size_t di = 0;
  u32 dl_off = 0;  // offset consumed inside dl[di]
  for (u32 i = 0; i < nops; i++) {
    u32 need = ops[i].del;
    while (need > 0) {
      DelRun r = dl[di];
      u32 avail = r.len - dl_off;
      u32 take = std::min(avail, need);
      u32 tgt = r.order + dl_off;
      // split at cwo run boundaries
      u32 left = take;
      while (left > 0) {
        i64 s = rle_search(d.cwo, tgt, [](const CwoRun& c) { return c.key; }, [](const CwoRun& c) { return c.len; });
        const CwoRun& c = d.cwo[s];
        u32 in_run = std::min(left, c.key + c.len - tgt);
        RemoteOp op{true, loc_id(d, tgt), RemoteId{}, in_run};
        out.ops.push_back(op);
        tgt += in_run; left -= in_run;
      }
      need -= take;
      next += take;
      dl_off += take;
      if (dl_off == r.len) { di++; dl_off = 0; }
    }
    if (ops[i].ins > 0) {
      // find the inserted span by order: origin_left = its ol, origin_right = its orr
      Cursor c;
      if (!d.get_cursor_before(next, c)) return ERR_UNKNOWN_ID;
      Span e = c.node->data[c.idx];
      u32 ol = origin_left_at_offset(e, c.off);
      RemoteOp op{false, loc_id(d, ol), loc_id(d, e.orr), ops[i].ins};
      out.ops.push_back(op);
      next += ops[i].ins;
    }
  }
  return OK;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

void* orc_doc_new(uint32_t leaf_cap, uint32_t node_cap, int track_index) {
  // leaf_cap 0: the unbounded leaf (L_UNBOUNDED, crdt_oracle.hpp)
  if (leaf_cap == 0) return new Doc(L_UNBOUNDED, 16, track_index != 0, false);
  if (leaf_cap < 4 || leaf_cap > 32 || node_cap < 8 || node_cap > 16) return nullptr;
  return new Doc(leaf_cap, node_cap, track_index != 0, track_index == 2);  // 2: the SplitList index
}
void orc_doc_free(void* h) { delete (Doc*)h; }
int orc_status(void* h) { return ((Doc*)h)->status; }
uint32_t orc_len(void* h) { return ((Doc*)h)->len(); }
uint64_t orc_digest(void* h) { return digest(*(Doc*)h); }
int orc_agent(void* h, const char* name) { return ((Doc*)h)->get_or_create_agent_id(name); }

int orc_apply_local(void* h, uint16_t agent, uint32_t nops, const uint32_t* ops3) {
  return ((Doc*)h)->apply_local_txn(agent, (const LocalOp*)ops3, nops);
}

// Apply a whole trace (txn patch counts + (pos, del, ins) patches) as local txns of `agent`.
int orc_apply_local_trace(void* h, uint16_t agent, uint32_t ntxn, const uint32_t* counts, const uint32_t* patches3) {
  Doc* d = (Doc*)h;
  const LocalOp* p = (const LocalOp*)patches3;
  for (uint32_t t = 0; t < ntxn; t++) {
    int st = d->apply_local_txn(agent, p, counts[t]);
    if (st != OK) return st;
    p += counts[t];
  }
  return OK;
}

// Config 1's per-op check: after txn t, answer pos_to_loc(probes[3t]) and
// loc_to_pos(probes[3t+1], probes[3t+2]) into answers[4t .. 4t+4) = (agent, seq, pos, deleted).
// After a failing txn every later answer is 0xFFFFFFFF (the document stopped).
void orc_pos_to_loc(void* h, uint32_t n, const uint32_t* pos, uint16_t* agent, uint32_t* seq);
void orc_loc_to_pos(void* h, uint32_t n, const uint16_t* agent, const uint32_t* seq, uint32_t* pos, uint8_t* deleted);
int orc_probe_trace(void* h, uint16_t agent, uint32_t ntxn, const uint32_t* counts, const uint32_t* patches3,
                    const uint32_t* probes3, uint32_t* answers4) {
  Doc* d = (Doc*)h;
  const LocalOp* p = (const LocalOp*)patches3;
  int st = OK;
  for (uint32_t t = 0; t < ntxn; t++) {
    uint32_t* a = answers4 + 4 * (size_t)t;
    if (st == OK) st = d->apply_local_txn(agent, p, counts[t]);
    p += counts[t];
    if (st != OK) { a[0] = a[1] = a[2] = a[3] = 0xFFFFFFFFu; continue; }
    uint16_t ag; uint32_t sq, ps; uint8_t dl;
    orc_pos_to_loc(h, 1, probes3 + 3 * (size_t)t, &ag, &sq);
    uint16_t qa = (uint16_t)probes3[3 * (size_t)t + 1];
    orc_loc_to_pos(h, 1, &qa, probes3 + 3 * (size_t)t + 2, &ps, &dl);
    a[0] = ag; a[1] = sq; a[2] = ps; a[3] = dl;
  }
  return st;
}

// n_ops generated local edits by `agent` (config 4), one LocalOp per txn.
int orc_apply_random(void* h, uint16_t agent, uint32_t n_ops, uint32_t seed) {
  Doc* d = (Doc*)h;
  for (uint32_t i = 0; i < n_ops; i++) {
    LocalOp op = random_change(seed, i, d->len());
    int st = d->apply_local_txn(agent, &op, 1);
    if (st != OK) return st;
  }
  return OK;
}

int orc_apply_remote_wire(void* h, const uint8_t* buf, size_t len) {
  Doc* d = (Doc*)h;
  wire::Batch b;
  if (!wire::parse(buf, len, b)) return ERR_BAD_INPUT;
  for (const auto& t : b.txns) {
    RemoteTxn rt = b.to_remote(t);
    int st = d->apply_remote_txn(rt);
    if (st != OK) return st;
  }
  return d->status;
}

// Replay a local trace and emit the equivalent remote wire batch.  out==nullptr -> returns size.
int64_t orc_local_trace_to_wire(void* h, uint16_t agent, uint32_t ntxn, const uint32_t* counts,
                                const uint32_t* patches3, uint8_t* out, int64_t cap) {
  Doc* d = (Doc*)h;
  const LocalOp* p = (const LocalOp*)patches3;
  wire::Writer w;
  for (uint32_t t = 0; t < ntxn; t++) {
    RemoteTxn rt;
    int st = apply_local_recording(*d, agent, p, counts[t], rt);
    if (st != OK) return st;
    w.add(rt);
    p += counts[t];
  }
  std::vector<uint8_t> bytes = w.finish();
  if (out) {
    if ((int64_t)bytes.size() > cap) return -1000;
    std::memcpy(out, bytes.data(), bytes.size());
  }
  return (int64_t)bytes.size();
}

// sizes: [n_raw, n_leaves, n_canon, n_cwo, n_del, n_dd, n_txn, n_parents, n_frontier, n_agents, next_order, len]
void orc_sizes(void* h, uint64_t* s) {
  Doc* d = (Doc*)h;
  std::vector<Span> raw, canon;
  std::vector<u32> ls;
  d->raw_entries(raw, ls);
  d->canonical(canon);
  u64 np = 0;
  for (auto& t : d->txns) np += t.parents.size();
  s[0] = raw.size(); s[1] = ls.size(); s[2] = canon.size(); s[3] = d->cwo.size(); s[4] = d->deletes.size();
  s[5] = d->double_deletes.size(); s[6] = d->txns.size(); s[7] = np; s[8] = d->frontier.size();
  s[9] = d->clients.size(); s[10] = d->next_order(); s[11] = d->len();
}

void orc_export(void* h, uint32_t* raw4, uint32_t* leaf_sizes, uint32_t* canon4, uint32_t* cwo4, uint32_t* del3,
                uint32_t* dd3, uint32_t* txn5, uint32_t* parents, uint32_t* frontier) {
  Doc* d = (Doc*)h;
  std::vector<Span> raw, canon;
  std::vector<u32> ls;
  d->raw_entries(raw, ls);
  d->canonical(canon);
  if (raw4) std::memcpy(raw4, raw.data(), raw.size() * 16);
  if (leaf_sizes) std::memcpy(leaf_sizes, ls.data(), ls.size() * 4);
  if (canon4) std::memcpy(canon4, canon.data(), canon.size() * 16);
  if (cwo4) std::memcpy(cwo4, d->cwo.data(), d->cwo.size() * 16);
  if (del3) std::memcpy(del3, d->deletes.data(), d->deletes.size() * 12);
  if (dd3) std::memcpy(dd3, d->double_deletes.data(), d->double_deletes.size() * 12);
  u32 po = 0;
  for (size_t i = 0; i < d->txns.size(); i++) {
    const TxnRec& t = d->txns[i];
    if (txn5) { txn5[5 * i] = t.order; txn5[5 * i + 1] = t.len; txn5[5 * i + 2] = t.shadow; txn5[5 * i + 3] = po; txn5[5 * i + 4] = (u32)t.parents.size(); }
    for (u32 p : t.parents) { if (parents) parents[po] = p; po++; }
  }
  if (frontier) std::memcpy(frontier, d->frontier.data(), d->frontier.size() * 4);
}

// §3.3: pos -> (agent, seq).  Invalid positions -> agent 0xFFFF, seq 0xFFFFFFFF.
void orc_pos_to_loc(void* h, uint32_t n, const uint32_t* pos, uint16_t* agent, uint32_t* seq) {
  Doc* d = (Doc*)h;
  for (uint32_t i = 0; i < n; i++) {
    agent[i] = 0xFFFF; seq[i] = 0xFFFFFFFFu;
    Cursor c;
    if (pos[i] >= d->len() || !d->tree.cursor_at_content_pos(pos[i], c)) continue;
    u32 o;
    if (!d->tree.get_item(c, o)) continue;
    u16 a; u32 s;
    if (d->order_to_loc(o, a, s)) { agent[i] = a; seq[i] = s; }
  }
}

// §3.4: (agent, seq) -> (pos, deleted) via Cursor::count_pos (cursor.rs:147-190).
// Unknown locations -> pos 0xFFFFFFFF, deleted 2.
void orc_loc_to_pos(void* h, uint32_t n, const uint16_t* agent, const uint32_t* seq, uint32_t* pos, uint8_t* deleted) {
  Doc* d = (Doc*)h;
  for (uint32_t i = 0; i < n; i++) {
    pos[i] = 0xFFFFFFFFu; deleted[i] = 2;
    if (agent[i] >= d->clients.size()) continue;
    u32 o;
    if (!d->seq_to_order(agent[i], seq[i], o)) continue;
    Cursor c;
    if (!d->get_cursor_before(o, c)) continue;
    u32 p = 0;
    for (u32 k = 0; k < c.idx; k++) p += clen(c.node->data[k]);
    p += std::min(clen(c.node->data[c.idx]), c.off);
    NodeBase* child = c.node;
    Internal* par = c.node->parent;
    while (par) {
      int ci = Tree::find_child(par, child);
      for (int k = 0; k < ci; k++) p += par->cnt[k];
      child = par;
      par = par->parent;
    }
    pos[i] = p;
    deleted[i] = c.node->data[c.idx].len < 0 ? 1 : 0;
  }
}

// Text (UTF-32) of the document from an order-indexed content table; returns its length, -1 if
// the table is too short, -2 if out is too small.  out may be NULL (length only).
int64_t orc_text(void* h, const uint32_t* content, uint64_t clen, uint32_t* out, uint64_t cap, uint64_t* digest_out) {
  std::vector<u32> t;
  if (!text_of(*(Doc*)h, content, clen, t)) return -1;
  if (digest_out) *digest_out = text_digest(t);
  if (out) {
    if (cap < t.size()) return -2;
    std::memcpy(out, t.data(), t.size() * 4);
  }
  return (int64_t)t.size();
}

// stats: [q2_triggers, integrate_iters, n_leaves]
void orc_stats(void* h, uint64_t* s) {
  Doc* d = (Doc*)h;
  s[0] = d->stats.q2_triggers;
  s[1] = d->stats.integrate_iters;
  s[2] = d->tree.leaves.size();
}

// Double-delete RLE driver for the reference's inc_delete_range unit test.
void* orc_dd_new() { return new std::vector<DDRun>(); }
void orc_dd_free(void* h) { delete (std::vector<DDRun>*)h; }
void orc_dd_increment(void* h, uint32_t base, uint32_t len) { increment_delete_range(*(std::vector<DDRun>*)h, base, len); }
uint32_t orc_dd_get(void* h, uint32_t* out3, uint32_t cap) {
  auto& v = *(std::vector<DDRun>*)h;
  for (size_t i = 0; i < v.size() && i < cap; i++) { out3[3 * i] = v[i].key; out3[3 * i + 1] = v[i].len; out3[3 * i + 2] = v[i].excess; }
  return (uint32_t)v.size();
}

// ---------------------------------------------------------------------------------------------
// CPU baseline (bench.py cpu_baseline leg): the restated reference B-tree path (leaf 32 /
// node 16, order index maintained), one document per task from an atomic work queue
// (rayon-equivalent), `threads` host threads.  Returns seconds of the timed region.
// ---------------------------------------------------------------------------------------------
double orc_cpu_baseline_local(uint32_t ndocs, uint32_t threads, uint32_t ntxn, const uint32_t* counts,
                              const uint32_t* patches3, uint64_t* checksum, int split_index) {
  std::atomic<uint32_t> next{0};
  std::atomic<uint64_t> sum{0};
  auto worker = [&]() {
    uint64_t local = 0;
    while (true) {
      uint32_t i = next.fetch_add(1);
      if (i >= ndocs) break;
      Doc d(32, 16, true, split_index != 0);
      u16 a = d.get_or_create_agent_id("jeremy");
      const LocalOp* p = (const LocalOp*)patches3;
      for (uint32_t t = 0; t < ntxn; t++) { d.apply_local_txn(a, p, counts[t]); p += counts[t]; }
      local += d.len() + (uint64_t)d.status;
    }
    sum += local;
  };
  double t0 = now_s();
  std::vector<std::thread> ts;
  for (uint32_t k = 0; k < threads; k++) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  double t1 = now_s();
  if (checksum) *checksum = sum.load();
  return t1 - t0;
}

// Config 4 on host cores: document i replays n_ops generated local txns (random_change, seed
// seeds[i]) on `threads` threads, one document per task (split_index: SplitList order index).
double orc_cpu_baseline_random(uint32_t ndocs, uint32_t threads, uint32_t n_ops, const uint32_t* seeds,
                               uint64_t* checksum, int split_index) {
  std::atomic<uint32_t> next{0};
  std::atomic<uint64_t> sum{0};
  auto worker = [&]() {
    uint64_t local = 0;
    while (true) {
      uint32_t i = next.fetch_add(1);
      if (i >= ndocs) break;
      Doc d(32, 16, true, split_index != 0);
      u16 a = d.get_or_create_agent_id("gen");
      for (uint32_t k = 0; k < n_ops; k++) {
        LocalOp op = random_change(seeds[i], k, d.len());
        if (d.apply_local_txn(a, &op, 1) != OK) break;
      }
      local += d.len() + (uint64_t)d.status;
    }
    sum += local;
  };
  double t0 = now_s();
  std::vector<std::thread> ts;
  for (uint32_t k = 0; k < threads; k++) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  double t1 = now_s();
  if (checksum) *checksum = sum.load();
  return t1 - t0;
}

// Remote replay of a wire batch for `ndocs` documents (the reference takes &RemoteTxn, so each
// worker materialises the RemoteTxn list once, before the timed region, with document i's name at
// index `rename_idx` replaced by names[i] for the first document it owns; names never change the
// amount of work of a single-agent trace).  Timed region: from a start barrier to the last join.
double orc_cpu_baseline_remote(uint32_t ndocs, uint32_t threads, const uint8_t* buf, size_t len,
                               uint32_t rename_idx, const char* const* names, uint64_t* checksum, int split_index) {
  wire::Batch b;
  if (!wire::parse(buf, len, b)) return -1.0;
  std::atomic<uint32_t> next{0}, ready{0};
  std::atomic<bool> go{false};
  std::atomic<uint64_t> sum{0};
  auto worker = [&](uint32_t tid) {
    wire::Batch bi = b;
    if (rename_idx < bi.names.size() && names) bi.names[rename_idx] = names[tid % ndocs];
    std::vector<RemoteTxn> txns;
    txns.reserve(bi.txns.size());
    for (const auto& t : bi.txns) txns.push_back(bi.to_remote(t));
    ready++;
    while (!go.load()) std::this_thread::yield();
    uint64_t local = 0;
    while (true) {
      uint32_t i = next.fetch_add(1);
      if (i >= ndocs) break;
      Doc d(32, 16, true, split_index != 0);
      for (const auto& t : txns) d.apply_remote_txn(t);
      local += d.len() + (uint64_t)d.status;
    }
    sum += local;
  };
  std::vector<std::thread> ts;
  for (uint32_t k = 0; k < threads; k++) ts.emplace_back(worker, k);
  while (ready.load() < threads) std::this_thread::yield();
  double t0 = now_s();
  go = true;
  for (auto& t : ts) t.join();
  double t1 = now_s();
  if (checksum) *checksum = sum.load();
  return t1 - t0;
}

}  // extern "C"
