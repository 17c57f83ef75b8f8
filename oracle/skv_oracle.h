/*
 * skv_oracle.h — CPU restatement of skyvault's compaction path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline. The product path
 * (libskv.so, include/skv.h) never links, loads or calls it.
 *
 * Parity pinning: the restatement is checked against the known-answer tests held by the
 * reference's own unit tests (runs.rs:775-1000, k_way.rs:42-226, cache_service.rs:349-391),
 * transcribed as fixtures under tests/golden/, and against an independent pure-Python
 * restatement (tests/pyref.py) on generated inputs. The Rust reference itself cannot be
 * built here (no cargo/rustc in the image), so it is never run.
 */
#ifndef SKV_ORACLE_H
#define SKV_ORACLE_H

#include "skv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A WriteOperation (runs.rs:38-43): Put(key, value) or Delete(key). */
typedef struct {
    uint32_t is_put;
    uint32_t key_len;
    const uint8_t* key;
    uint64_t val_len;
    const uint8_t* val;
} skvo_op;

/* Decoded ops of one run; ops point into `arena` (owned by the list). */
typedef struct {
    skvo_op* ops;
    uint64_t n_ops;
    uint8_t* arena;
} skvo_op_list;

/* runs::read_run_stream (runs.rs:517-628): every op yielded before the first error, then the
 * error (return code) with its Display text in errbuf. */
int skvo_decode_run(const uint8_t* run, uint64_t len, skvo_op_list** out, char* errbuf, size_t errlen);
void skvo_op_list_free(skvo_op_list* l);

/* runs::build_runs (runs.rs:166-282) over an already-merged op sequence. */
int skvo_build_runs(const skvo_op* ops, uint64_t n_ops, uint64_t max_run_size, skv_result** out,
                    char* errbuf, size_t errlen);

/* k_way::merge (k_way.rs:113-179) of already-decoded op sequences: the emitted sequence. */
int skvo_merge_ops(const skvo_op* const* ops, const uint64_t* n_ops, const int64_t* seq_nos,
                   uint32_t n_streams, skvo_op_list** out, char* errbuf, size_t errlen);

/* The full job composition: decode every member run (read_run_stream), flatten members per
 * stream, k_way::merge, optional Delete filter, build_runs or WAL table split. Same inputs,
 * outputs and status codes as skv_compact(). */
int skvo_compact(const skv_stream* streams, uint32_t n_streams, uint64_t max_run_size,
                 uint32_t flags, skv_result** out, char* errbuf, size_t errlen);

/* cache_service.rs:97-151 ScanFromRun over fetched runs: read_run_iter decode (runs.rs:400-510),
 * key > start filter, k_way::merge at SeqNo i64::MAX - index, read until the max_results-th Put.
 * The response items come back as one v1 run (0 runs when empty). Same contract as skv_scan_runs. */
int skvo_scan_runs(const uint8_t* const* runs, const uint64_t* lens, uint32_t n_runs, const uint8_t* start_key,
                   uint64_t start_len, uint64_t max_results, skv_result** out, char* errbuf, size_t errlen);

void skvo_result_free(skv_result* r);

/* Streaming build_runs for full-size checks (test infrastructure): feed the merged op sequence
 * as consecutive v1 runs; the greedy split and order check carry across feeds. skvo_sb_drain
 * moves the output bytes produced so far out (skvo_sb_pending of them); skvo_sb_finish ends
 * the stream (runs.rs:270-280) and returns the undrained tail bytes and every run descriptor
 * (absolute offsets; result->in_bytes = bytes drained before the tail). */
typedef struct skvo_sb skvo_sb;
skvo_sb* skvo_sb_new(uint64_t max_run_size);
int skvo_sb_feed_run(skvo_sb* s, const uint8_t* run, uint64_t len, char* errbuf, size_t errlen);
uint64_t skvo_sb_pending(const skvo_sb* s);
void skvo_sb_drain(skvo_sb* s, uint8_t* dst);
int skvo_sb_finish(skvo_sb* s, skv_result** out);
void skvo_sb_free(skvo_sb* s);

#ifdef __cplusplus
}
#endif
#endif
