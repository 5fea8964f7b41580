// INPUT SYNTHESIS (test / bench infrastructure, never the product): BASELINE config 5 histories
// (concurrent, deletion-heavy remote merges) as RTX1 wire batches, generated in C++
// so that every document of a batch can have its own history (scripts/bench_config5.py
// --distinct = docs).  The same shape as tests/fuzz_gen.py config5_wire -- agent "base" inserts
// base_len chars in one txn (contiguous orders); then `rounds` rounds in which each of `n_agents`
// agents makes `ops` single-op txns against the round-start snapshot: with probability del_frac a
// delete of 1..64 base items (contiguous targets; overlapping deletes are the double
// deletes), else an insert of 1..8 chars at one of `hot` shared hotspots (origin_left base item h,
// origin_right base item h + 1: concurrent inserts tie in integrate's Equal branch, doc.rs:198-
// 216).  A txn's parents are the round-start frontier (the agent's first txn of the round) or the
// agent's previous txn; delivery within a round is a seeded interleaving that keeps each agent's
// order, so every history is causally ordered (apply_remote_txn's in-order seq assert,
// doc.rs:245-247) and the delivery order differs per seed.  The random stream is splitmix64 of
// (seed, draw index), not Python's Mersenne Twister, so the histories differ from config5_wire's
// at equal seeds; parity is checked per history by the oracle's replay, as for config5_wire.
// Wire layout: oracle/wire.hpp (include/crdt_gpu.h "Remote wire batch").
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>
#include <atomic>

namespace {
typedef uint32_t u32;
typedef uint64_t u64;

struct Rng {
  u64 s;
  u64 next() {
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  u32 below(u32 n) { return (u32)(((next() >> 32) * (u64)n) >> 32); }  // uniform in [0, n)
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Txn { u32 agent, seq; u32 kind, s, len; };  // one op per txn: kind 0 insert at hotspot s, 1 delete [s, s+len)

std::vector<uint8_t> history(u64 seed, u32 base_len, u32 n_agents, u32 rounds, u32 ops, u32 hot, double del_frac) {
  Rng rng{seed * 0xD1B54A32D192ED03ull + 0x5851F42D4C957F2Dull};
  // name table: "base" (0), "ROOT" (1), then the agents (2 + i), as build_wire's first-use order
  // would give for histories where every agent appears in round 0
  std::vector<std::string> names = {"base", "ROOT"};
  for (u32 i = 0; i < n_agents; i++) {
    char b[32];
    snprintf(b, sizeof b, "a%02u_%05x", i, (u32)(rng.next() & 0xFFFFFu));
    names.push_back(b);
  }
  hot = std::min<u32>(hot, base_len - 1);
  std::vector<u32> spots;
  {  // `hot` distinct hotspots in [0, base_len - 1): partial Fisher-Yates over a sparse swap map
    std::vector<std::pair<u32, u32>> sw;
    auto get = [&](u32 i) { for (auto& p : sw) if (p.first == i) return p.second; return i; };
    auto put = [&](u32 i, u32 v) { for (auto& p : sw) if (p.first == i) { p.second = v; return; } sw.push_back({i, v}); };
    u32 n = base_len - 1;
    for (u32 k = 0; k < hot; k++) {
      u32 j = k + rng.below(n - k);
      u32 a = get(k), b = get(j);
      put(k, b); put(j, a);
      spots.push_back(b);
    }
    std::sort(spots.begin(), spots.end());
  }
  const u32 ROOT_SEQ = 0xFFFFFFFFu;
  std::vector<u32> body;
  body.reserve((size_t)rounds * n_agents * ops * 13 + 16);
  u32 n_txns = 1;
  // txn 0: base inserts base_len chars, parents [ROOT]
  u32 t0[] = {0, 0, 1, 1, 1, ROOT_SEQ, 0, 1, ROOT_SEQ, 1, ROOT_SEQ, base_len};
  body.insert(body.end(), t0, t0 + 12);
  std::vector<u32> seq(n_agents, 0);
  // round-start frontier: (name index, seq) pairs
  std::vector<std::pair<u32, u32>> frontier = {{0u, base_len - 1u}};
  std::vector<std::vector<Txn>> per(n_agents);
  std::vector<u32> live, head(n_agents);
  for (u32 r = 0; r < rounds; r++) {
    for (u32 a = 0; a < n_agents; a++) {
      per[a].clear();
      for (u32 k = 0; k < ops; k++) {
        Txn t;
        t.agent = a;
        t.seq = seq[a];
        if (rng.unit() < del_frac) {
          u32 mx = std::min<u32>(64u, base_len);
          t.kind = 1;
          t.len = 1 + rng.below(mx);
          t.s = rng.below(base_len - t.len + 1);
        } else {
          t.kind = 0;
          t.s = spots[rng.below((u32)spots.size())];
          t.len = 1 + rng.below(8);
        }
        seq[a] += t.len;
        per[a].push_back(t);
      }
    }
    live.clear();
    for (u32 a = 0; a < n_agents; a++) { if (ops) live.push_back(a); head[a] = 0; }
    while (!live.empty()) {  // a seeded interleaving that keeps each agent's order
      u32 li = rng.below((u32)live.size());
      u32 a = live[li];
      const Txn& t = per[a][head[a]];
      body.push_back(2 + a);
      body.push_back(t.seq);
      if (head[a] == 0) {  // the agent's first txn of the round: the round-start frontier
        body.push_back((u32)frontier.size());
        body.push_back(1);
        for (auto& f : frontier) { body.push_back(f.first); body.push_back(f.second); }
      } else {  // its previous txn's last item
        body.push_back(1);
        body.push_back(1);
        body.push_back(2 + a);
        body.push_back(t.seq - 1);
      }
      if (t.kind == 1) {
        u32 op[] = {1, 0, t.s, 0, 0, t.len};
        body.insert(body.end(), op, op + 6);
      } else {
        u32 op[] = {0, 0, t.s, 0, t.s + 1, t.len};
        body.insert(body.end(), op, op + 6);
      }
      n_txns++;
      if (++head[a] == ops) { live[li] = live.back(); live.pop_back(); }
    }
    frontier.clear();
    for (u32 a = 0; a < n_agents; a++) frontier.push_back({2 + a, seq[a] - 1});
  }
  std::vector<uint8_t> out;
  auto put32 = [&](u32 v) { uint8_t b[4]; memcpy(b, &v, 4); out.insert(out.end(), b, b + 4); };
  put32(0x31585452u);
  put32((u32)names.size());
  for (auto& n : names) {
    put32((u32)n.size());
    out.insert(out.end(), n.begin(), n.end());
    out.resize((out.size() + 3) & ~(size_t)3, 0);
  }
  put32(n_txns);
  size_t o = out.size();
  out.resize(o + body.size() * 4);
  memcpy(out.data() + o, body.data(), body.size() * 4);
  return out;
}
}  // namespace

extern "C" {
// n histories (seeds[i]) generated on `threads` threads; out[i] / out_len[i]: malloc'ed wire bytes
// (free with c5_free).  Returns 0, or -1 on bad parameters.
int c5_gen_batch(uint64_t n, const uint64_t* seeds, uint32_t base_len, uint32_t n_agents, uint32_t rounds,
                 uint32_t ops, uint32_t hot, double del_frac, int threads, uint8_t** out, uint64_t* out_len) {
  if (base_len < 2 || n_agents == 0 || n_agents > 60000 || hot == 0) return -1;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    for (uint64_t i; (i = next++) < n;) {
      std::vector<uint8_t> w = history(seeds[i], base_len, n_agents, rounds, ops, hot, del_frac);
      out[i] = (uint8_t*)malloc(w.size());
      memcpy(out[i], w.data(), w.size());
      out_len[i] = w.size();
    }
  };
  int t = threads < 1 ? 1 : threads;
  std::vector<std::thread> th;
  for (int k = 1; k < t; k++) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  return 0;
}
void c5_free(uint8_t* p) { free(p); }
}
