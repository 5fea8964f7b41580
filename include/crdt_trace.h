/*
 * crdt_trace.h — native trace ingestion: the reference's editing-trace files
 * decoded straight into the arrays the engine's staging calls take (crdt_apply_local /
 * crdt_stage_local / crdt_stage_local_shared / crdt_set_content), with no Python JSON pass.
 *
 * Replaces crdt-testdata's `load_testing_data` (src/testdata/src/lib.rs:29-48): gzip (flate2)
 * -> serde_json into `TestData { startContent, endContent, txns: [TestTxn { time, patches:
 * [TestPatch(pos, del_span, ins_content)] }] }` (lib.rs:10-27).  The decoder streams: the gzip
 * member is inflated 1 MiB at a time and parsed in one pass, so memory is the output arrays only.
 *
 * Output form (what benches/yjs.rs:11-29 apply_edits reads from each patch):
 *   counts[n_txns]        patches per txn
 *   patches[n_patches][3] (pos, del_span, ins_len) — ins_len = ins_content.chars().count()
 *                         (doc.rs:383), i.e. Unicode scalar values
 *   text                  every ins_content, UTF-8, concatenated in patch order
 *   start / end           startContent / endContent, UTF-8
 * Unknown keys (e.g. `time`) are skipped as serde does.  JSON string escapes are decoded
 * (\uXXXX surrogate pairs -> one scalar); a lone surrogate, bad UTF-8, a negative or non-integer
 * pos/del, or a patch that is not [int, int, string] is CRDT_E_TRACE, as serde_json would
 * reject it.  Return values follow crdt_gpu.h: 0 = ok, < 0 = error (text: crdt_last_error()).
 * Host-only: no call here touches the GPU.
 */
#ifndef CRDT_TRACE_H
#define CRDT_TRACE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_E_TRACE -104   /* malformed trace file / JSON */
#define CRDT_E_IO -105      /* cannot open / read / inflate the file */

typedef struct crdt_trace crdt_trace;

/* Decode a trace file: gzip'd JSON (.json.gz, as in benchmark_data/) or plain JSON. */
int crdt_trace_load(const char* path, crdt_trace** out);
/* Decode JSON text already in memory (not gzip'd). */
int crdt_trace_parse(const char* json, uint64_t len, crdt_trace** out);
/* sizes[7] = {n_txns, n_patches, text_bytes, start_len, start_bytes, end_len, end_bytes}
 * (_len = Unicode scalar values, _bytes = UTF-8 bytes). */
int crdt_trace_sizes(const crdt_trace* t, uint64_t* sizes7);
/* Copy out; any pointer may be NULL.  Sizes as crdt_trace_sizes reports them. */
int crdt_trace_copy(const crdt_trace* t, uint32_t* counts, uint32_t* patches3, char* text, char* start,
                    char* end);
void crdt_trace_free(crdt_trace* t);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_TRACE_H */
