/*
 * crdt_gpu.h — C ABI of the MI355X list-CRDT engine (drop-in boundary for the hot path of
 * josephg/text-crdt-rust: position <-> CRDT-location remapping and batch merge of list-CRDT
 * edits, across many documents at once).
 *
 * The reference exposes this path only as a Rust crate API (src/lib.rs:3-14); there is no FFI.
 * Each entry point below names the reference function it replaces; a Rust binding would wrap
 * these in `ListCRDT`-shaped methods (see INTEGRATION.md for the cgo-free Rust `extern "C"`
 * block and a ctypes stub).
 *
 * Conventions
 *   - Caller-owned host buffers; the engine owns device memory.  Calls are synchronous at return
 *     unless named *_async (then crdt_sync()).  One engine per host thread per device.
 *   - Positions and lengths count Unicode scalar values (chars().count(), doc.rs:383).
 *   - Agent 0xFFFF = ROOT (doc.rs:68).  Order 0xFFFFFFFF = ROOT_ORDER (list/mod.rs:30).
 *   - A failing op poisons only its document (doc_status < 0); later ops of that document are
 *     skipped.  This mirrors "the reference panics": the document is dead, the rest live on.
 *   - Return value of every function: 0 = ok, < 0 = API error (CRDT_E_*).
 *   - A stage / apply call names each document at most once (its docs[] has no duplicates);
 *     a call that names a document twice returns CRDT_E_ARG and changes nothing.  Every stage
 *     call replaces the staged streams of all documents (documents not named get none).
 */
#ifndef CRDT_GPU_H
#define CRDT_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-document status codes (identical in the oracle and the kernels) ---------------- */
#define CRDT_OK 0
#define CRDT_ERR_POS_OOB -1          /* local op outside the document (root.rs:71,79; mutations.rs:573) */
#define CRDT_ERR_SEQ -2              /* remote txn seq != next seq of its agent (doc.rs:247) */
#define CRDT_ERR_UNKNOWN_AGENT -3    /* agent name/id not known to the document (doc.rs:92,237) */
#define CRDT_ERR_UNKNOWN_ID -4       /* (agent, seq) does not name an inserted item (doc.rs:27, root.rs:288) */
#define CRDT_ERR_NONTERMINATING -5   /* the reference's integrate / remote-delete loop never exits here */
#define CRDT_ERR_CAPACITY -6         /* a per-document structural limit was exceeded */
#define CRDT_ERR_EMPTY_TXN -7        /* zero-length txn (reference underflows first_order+0-1, doc.rs:351) */
#define CRDT_ERR_FRONTIER -8         /* advance_branch_by assertion (doc.rs:43) */
#define CRDT_ERR_BAD_INPUT -9        /* malformed record / zero-length remote op */
#define CRDT_ERR_INTERNAL -10

/* ---- API errors ---------------------------------------------------------------------------- */
#define CRDT_E_ARG -100
#define CRDT_E_DEVICE -101   /* no usable MI355X / HIP error */
#define CRDT_E_NOMEM -102
#define CRDT_E_WIRE -103     /* malformed remote wire batch */

typedef struct crdt_engine crdt_engine;

typedef struct {
  uint32_t leaf_cap;   /* 32 = reference release layout (range_tree/mod.rs:38), 4 = debug layout */
  int32_t device;      /* HIP device ordinal */
} crdt_cfg;

/* LocalOp (src/common.rs:45-50) with the inserted string replaced by its char count. */
typedef struct {
  uint32_t pos;
  uint32_t del_len;
  uint32_t ins_len;
} crdt_local_op;

/* One apply_local_txn(agent, &ops[..n_ops]) call (doc.rs:376). */
typedef struct {
  uint32_t agent;
  uint32_t n_ops;
} crdt_local_txn;

/* ListCRDT::new() x n — (re)creates n_docs empty documents (doc.rs:51-64). */
int crdt_engine_create(const crdt_cfg* cfg, crdt_engine** out);
void crdt_engine_destroy(crdt_engine* e);
int crdt_docs_alloc(crdt_engine* e, uint64_t n_docs);
uint64_t crdt_num_docs(const crdt_engine* e);

/* ListCRDT::get_or_create_agent_id (doc.rs:66-80), n independent (doc, name) requests. */
int crdt_agent_intern(crdt_engine* e, uint64_t n, const uint32_t* doc, const char* const* names,
                      uint16_t* agent_out);
/* The same interning done by a device kernel (one wave per document): name i is
 * the bytes [name_off[i], name_off[i+1]) of `bytes` (any bytes, not NUL-terminated).  Ids are
 * identical to crdt_agent_intern on the same call.  rank_out (optional): each name's rank among
 * the document's names in byte-lexicographic order (Rust str Ord; the order the integrate
 * tie-break compares, doc.rs:207), INVALID for "ROOT".  Up to 65,534 names per document (AgentId is
 * u16, doc.rs:66-80; CRDT_E_ARG beyond): documents with at most 1,024 names intern in an LDS table,
 * larger ones again with the table in HBM and ranks from a sort. */
int crdt_agent_intern_dev(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint64_t* name_off,
                          const char* bytes, uint16_t* agent_out, uint32_t* rank_out);

/* ListCRDT::apply_local_txn (doc.rs:376-469) for many documents.  Document docs[i] applies txns
 * txns[txn_off[i] .. txn_off[i+1]) in order; ops are concatenated in txn order. */
int crdt_apply_local(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                     const crdt_local_txn* txns, const crdt_local_op* ops, int32_t* doc_status);

/* ListCRDT::apply_remote_txn (doc.rs:242-348) for many documents: wire[i] (wire_len[i] bytes) is
 * a remote wire batch applied to docs[i].
 *
 * Remote wire batch (serialises RemoteTxn, src/list/external_txn.rs:5-30; little endian u32s):
 *   'RTX1' (0x31585452) | n_names | n_names x {byte_len, utf-8 bytes, zero pad to 4}
 *   | n_txns | n_txns x { agent_name, seq, n_parents, n_ops,
 *                         n_parents x {name, seq},
 *                         n_ops x {kind (0 Ins, 1 Del), a_name, a_seq, b_name, b_seq, len} }
 *   Ins: a = origin_left, b = origin_right, len = chars inserted.  Del: a = target, len.
 *   The name "ROOT" denotes the root id (doc.rs:68). */
int crdt_apply_remote_wire(crdt_engine* e, uint64_t n_docs, const uint32_t* docs,
                           const uint8_t* const* wire, const uint64_t* wire_len, int32_t* doc_status);

/* Staged form (inputs resident in HBM, then replay without host transfers): */
int crdt_stage_local(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                     const crdt_local_txn* txns, const crdt_local_op* ops);
int crdt_stage_remote_wire(crdt_engine* e, uint64_t n_docs, const uint32_t* docs,
                           const uint8_t* const* wire, const uint64_t* wire_len);
/* Shared local streams: stream k = txns[stream_txn_off[k] .. stream_txn_off[k+1]) (ops concatenated
 * in txn order); document docs[i] replays stream stream_of_doc[i].  Each stream is encoded and
 * uploaded once (device copies per document), e.g. a corpus of documents drawn from few traces. */
int crdt_stage_local_shared(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* stream_of_doc,
                            uint32_t n_streams, const uint64_t* stream_txn_off, const crdt_local_txn* txns,
                            const crdt_local_op* ops);
/* One wire batch replicated to docs [0, n_docs) of a fresh engine; name index `rename_idx` of the
 * batch's name table is replaced per document by names[d] (randomised client ids). */
int crdt_stage_remote_replicated(crdt_engine* e, const uint8_t* wire, uint64_t wire_len,
                                 uint32_t rename_idx, const char* const* names);
/* On-device edit generator (BASELINE config 4): each document docs[i] gets n_ops local txns by
 * `agent`, one LocalOp each, drawn on the GPU inside the replay wave with the semantics of the
 * reference's make_random_change (doc.rs:544-569; insert 1 char w.p. 0.55 below 100 chars else
 * 0.45, delete 1..10 chars).  Per-document seed = low 32 bits of splitmix64(seed ^ doc).  Only
 * one GEN record per document is staged, so 10^6 documents need no host-side op stream. */
int crdt_stage_random(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const char* agent, uint32_t n_ops,
                      uint64_t seed);
/* Reset every document to ListCRDT::new() state, keeping interned agents and staged records. */
int crdt_reset_async(crdt_engine* e);
/* Replay the staged records of every document (+ capacity growth/resume as needed). */
int crdt_run(crdt_engine* e, int32_t* doc_status /* n_docs, may be NULL */);
int crdt_run_async(crdt_engine* e);   /* single launch; no growth handling */
/* Rebuild the flat per-document index: canonical span array (stream compaction of the leaf
 * entries with YjsSpan::can_append), visible-prefix scan, order->span scatter, digests. */
int crdt_publish_async(crdt_engine* e);
int crdt_sync(crdt_engine* e);

/* ---- queries (the reference's README operations, README.md:22-25) ------------------------- */
/* Doc location -> CRDT location (§3.3: cursor_at_content_pos + client_with_order.get).
 * Invalid positions give agent 0xFFFF, seq 0xFFFFFFFF. */
int crdt_pos_to_loc(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint32_t* pos,
                    uint16_t* agent, uint32_t* seq);
/* CRDT location -> doc location (§3.4: seq_to_order + Cursor::count_pos).  deleted: 0/1, 2 = unknown id. */
int crdt_loc_to_pos(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint16_t* agent,
                    const uint32_t* seq, uint32_t* pos, uint8_t* deleted);
/* Device-pointer forms for batched query benchmarking (inputs/outputs already in HBM). */
int crdt_pos_to_loc_dev_async(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint32_t* pos,
                              uint16_t* agent, uint32_t* seq);
int crdt_loc_to_pos_dev_async(crdt_engine* e, uint64_t n, const uint32_t* doc, const uint16_t* agent,
                              const uint32_t* seq, uint32_t* pos, uint8_t* deleted);

/* ---- text materialisation (the reference's USE_INNER_ROPE rope) ----------
 * The reference's rope (doc.rs:14-17, 59, 98 of list/mod.rs) receives the inserted string at
 * cursor.count_pos() on every integrate (doc.rs:230-233) and loses the deleted visible range on
 * every local delete (doc.rs:430-432); its remote-delete arm is todo!() (doc.rs:329-333), and
 * ListCRDT::to_string returns it (doc.rs:498-505).  Here the rope is computed from the published
 * index instead: the visible items in document order, each replaced by its code point.
 *
 * Content is an order-indexed UTF-32 table per document: content[order] is the code point of the
 * item with that order (orders are assigned as in assign_order_to_client, doc.rs:155-165: within a
 * txn, op by op, a LocalOp's deleted orders first, then its inserted chars).  Entries at delete
 * orders are never read.  Streams are shared: document docs[i] reads stream stream_of_doc[i] =
 * content[stream_off[k] .. stream_off[k+1]).  A call replaces all content set before. */
int crdt_set_content(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* stream_of_doc,
                     uint32_t n_streams, const uint64_t* stream_off, const uint32_t* content);
/* Write every document's text on the device (publishes first if needed; stream-ordered). */
// As crdt_set_content, with one stream that every listed document gets its own device copy of
// (docs[i] reads copy i); replaces all previously set content.
int crdt_set_content_copies(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint32_t* content,
                            uint64_t len);
int crdt_materialize_async(crdt_engine* e);
/* ListCRDT::to_string (doc.rs:498-505) as UTF-32: *n_out = visible chars; out may be NULL (size
 * query), else cap >= *n_out.  CRDT_E_ARG if the document has no content or its stream is shorter
 * than the document's orders, or if it is poisoned. */
int crdt_text(crdt_engine* e, uint32_t doc, uint32_t* out, uint64_t cap, uint64_t* n_out);
/* Per-document 64-bit digest of the text (same as the oracle's text_digest; 0 = not materialised). */
int crdt_text_digest(crdt_engine* e, uint64_t* per_doc /* n_docs */);
int crdt_last_materialize_ms(crdt_engine* e, double* ms);

/* ListCRDT::len (doc.rs:484-486) */
int crdt_doc_len(crdt_engine* e, uint64_t n, const uint32_t* doc, uint32_t* len);
int crdt_doc_status(crdt_engine* e, int32_t* status /* n_docs */);
/* 64-bit digest of each document's canonical state (DESIGN.md "Digest"; same as the oracle). */
int crdt_digest(crdt_engine* e, uint64_t* per_doc /* n_docs */);
/* Canonical spans of each document's published index (YjsSpan::can_append runs; sizes[2] of
 * crdt_export_sizes for every document at once: the roofline's per-document span counts). */
int crdt_canon_counts(crdt_engine* e, uint32_t* per_doc /* n_docs */);

/* Export one document (parity / debugging).  sizes[12] = {raw entries, leaves, canonical spans,
 * cwo runs, delete runs, double-delete runs, txns, parents, frontier, agents, next_order, len}.
 * Any output pointer may be NULL.  raw/canon: 4 u32 per span (order, origin_left, origin_right,
 * len as i32); cwo: (order, agent, seq, len); deletes/dd: 3 u32; txns: (order, len, shadow,
 * parents_off, n_parents). */
int crdt_export_sizes(crdt_engine* e, uint32_t doc, uint64_t* sizes);
int crdt_export(crdt_engine* e, uint32_t doc, uint32_t* raw4, uint32_t* leaf_sizes, uint32_t* canon4,
                uint32_t* cwo4, uint32_t* del3, uint32_t* dd3, uint32_t* txn5, uint32_t* parents,
                uint32_t* frontier);

// Shrink every document's per-table capacities to what its staged stream used (call after a
// crdt_run + publish of it; a later reset + crdt_run_async replays it in exactly that room).
// Capacities grow again on the next stage.  (Host-side planning; no reference counterpart.)
int crdt_fit(crdt_engine* e);
// crdt_fit over several corpora replayed one after another on the same documents (BASELINE config
// 4's batches): apply = 0 notes the capacities crdt_fit would set into each document's running
// maximum (no relayout); apply = 1 sets every document's capacities to its noted maximum (one
// relayout) and forgets the maxima.  (Host-side planning; no reference counterpart.)
int crdt_fit_note(crdt_engine* e, int apply);
// Config 4 corpus batches: every document whose staged stream is one generated-edit record
// (crdt_stage_random) gets the seed crdt_stage_random would give document id_base + d
// ((u32)splitmix64(seed ^ (id_base + d)); the generator follows make_random_change,
// /root/reference/src/list/doc.rs:544-569).  Device-side, async on the engine stream; the next
// reset + crdt_run_async replays the new documents.
int crdt_reseed_random_async(crdt_engine* e, uint64_t seed, uint64_t id_base);
// crdt_digest into a device buffer (n_docs u64), async on the engine stream after the publish
// that computes the digests (crdt_publish_async).
int crdt_digest_dev_async(crdt_engine* e, uint64_t* dev_out);
// on != 0: documents staged in one call from the same host stream (crdt_stage_local_shared,
// crdt_stage_remote_replicated) read one device copy of it instead of a copy each (records
// are read-only input).  Off by default.
int crdt_set_share_streams(crdt_engine* e, int on);
// on != 0: crdt_stage_remote_replicated interns every document's authors on the device
// (crdt_agent_intern_dev, one wave per document) instead of on the host.  Same ids either way
// (get_or_create_agent_id, doc.rs:66-80).  Off by default.
int crdt_set_device_intern(crdt_engine* e, int on);
/* Kernel family behind crdt_pos_to_loc_dev_async / crdt_loc_to_pos_dev_async (same answers):
 *   CRDT_QUERY_LDS (default): 4,096-query chunks of one document stage its index in LDS and
 *     search in lockstep;
 *   CRDT_QUERY_PER_THREAD: one thread per query, binary searches in HBM;
 *   CRDT_QUERY_MERGE: for batches sorted per document (pos ascending; loc->pos by (agent, seq)):
 *     pos->loc merges each chunk against the document's visible prefix (merge path), loc->pos
 *     searches per thread; unsorted or mixed chunks are answered per thread. */
enum { CRDT_QUERY_LDS = 0, CRDT_QUERY_PER_THREAD = 1, CRDT_QUERY_MERGE = 2 };
int crdt_set_query_kernel(crdt_engine* e, int mode);
// Device bytes the engine holds (per-document pools, staged records, content, text).
uint64_t crdt_mem_bytes(const crdt_engine* e);
// Device bytes the engines of this process hold through their own allocations now, and the most
// they held at once since the last reset (a relayout -- growth, crdt_fit -- moves the pools one
// at a time: its peak is the old pools + the largest new one).  Diagnostic; never fails.
int crdt_device_bytes(uint64_t* current, uint64_t* peak, int reset_peak);
// Test hook: after k more device allocations by any engine of this process, the next one fails as
// out of memory (k < 0: never).  A relayout that fails part-way poisons its engine: every later
// call but crdt_engine_destroy / crdt_docs_alloc returns CRDT_E_NOMEM.
int crdt_test_fail_alloc_after(long long k);
// Config 1's per-op check: after txn t (of every listed document), ask pos_to_loc(probes[t].pos)
// and loc_to_pos(probes[t].agent, probes[t].seq) on the state reached so far (the README's two
// mappings, cursor.rs:147-190 count_pos; answers as crdt_pos_to_loc / crdt_loc_to_pos).
// Otherwise as crdt_apply_local.  The probed documents keep the order -> leaf map.
typedef struct { uint32_t pos, agent, seq; } crdt_probe;
typedef struct { uint32_t agent, seq, pos, deleted; } crdt_probe_answer;
int crdt_apply_local_probed(crdt_engine* e, uint64_t n_docs, const uint32_t* docs, const uint64_t* txn_off,
                            const crdt_local_txn* txns, const crdt_local_op* ops, const crdt_probe* probes,
                            crdt_probe_answer* answers, int32_t* doc_status);
/* Raw per-document replay state (23 u32: status, resume point, table sizes, ...; debugging). */
int crdt_debug_state(crdt_engine* e, uint32_t doc, uint32_t* out23);
/* Device time of the last replay / publish launches in ms (HIP events on the engine stream). */
int crdt_last_timings(crdt_engine* e, double* replay_ms, double* publish_ms);
/* Engine stream (hipStream_t) for callers that time or order their own work. */
void* crdt_stream(crdt_engine* e);
/* Text of the last HIP error seen by this thread (empty if none). */
const char* crdt_last_error(void);
/* The source hash this library was built from (crdt_amd.build(): sha256 over the sources and the
 * build line, also stored beside the library), so a run can prove which sources it executed. */
const char* crdt_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_GPU_H */
