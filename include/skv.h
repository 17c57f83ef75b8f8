/*
 * skv.h — C ABI of the MI355X compaction path for skyvault v1 runs.
 *
 * This is the drop-in boundary for skyvault's byte-heavy compaction core:
 *
 *     runs::read_run_stream   (src/runs.rs:517-628)     decode every input run
 *  -> k_way::merge            (src/k_way.rs:113-179)    newest seq_no wins per key
 *  -> [Delete filter]         (src/jobs/table_tree_compaction.rs:139-145)
 *  -> [WAL table split]       (src/jobs/wal_compaction.rs:66-174)
 *  -> runs::build_runs        (src/runs.rs:166-282)     greedy split into <= max-byte runs
 *
 * One skv_compact() call replaces that whole composition as it appears in the three
 * compaction jobs (table_buffer_compaction.rs:48-121, table_tree_compaction.rs:81-167,
 * wal_compaction.rs:34-174). The jobs keep doing everything around it (forest
 * snapshot, get_run/put_run, metadata commit), so the Rust side binds this header through
 * a thin `extern "C"` block called from `tokio::task::spawn_blocking`.
 *
 * Conventions
 *  - Blocking calls. One skv_ctx per GPU; calls on one ctx are serialised by the caller,
 *    different ctxs (GPUs) may run concurrently from different threads.
 *  - Inputs are borrowed for the duration of the call and never modified.
 *  - All-or-nothing: on error no result is produced. (The reference streams finished
 *    output runs to S3 before a later error surfaces; those orphans are invisible to the
 *    forest, so "job failed" is the only observable outcome and is what we model.)
 *  - The result owns its memory; free it with skv_result_free().
 *  - Error messages are the reference's Display text of RunError / JobError.
 */
#ifndef SKV_H
#define SKV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKV_ABI_VERSION 9  /* 2: skv_timings gained sorted, fp_rerun; 3: host_parts; 4: skv_scan_runs;
                              5: skv_timings.span_parse (was reserved); 6: skv_timings.wal_stage;
                              7: skv_ctx_host_info; 8: skv_compact_split; 9: skv_host_plan,
                              skv_split_deal, skv_test_option */

typedef struct skv_ctx skv_ctx;

/*
 * One input stream of k_way::merge: a (SeqNo, stream) pair (k_way.rs:113). The stream is
 * the flattened concatenation of its member runs, each decoded separately by
 * read_run_stream — exactly how the jobs build their inputs (table_buffer_compaction.rs
 * :67-100 concatenates all L0 runs into one stream at SeqNo 0; table_tree_compaction.rs
 * :105-135 does the same for the overlapping next-level runs). A stream with n_runs == 0
 * yields nothing (k_way.rs:138); a member run of 0 bytes yields RunError::EmptyInput.
 * seq_no values must be pairwise distinct (k_way.rs:121 keys streams by SeqNo).
 */
typedef struct {
    const uint8_t* const* runs; /* member runs, in order (host or device pointers, see below) */
    const uint64_t* run_lens;   /* byte length of each member run */
    uint32_t n_runs;
    int64_t seq_no;
} skv_stream;

/*
 * One output run, as yielded by build_runs (runs.rs:221-228, :271-280) together with
 * its Stats::StatsV1 (runs.rs:102-109). len == StatsV1.size_bytes (the version byte is
 * counted, runs.rs:241-244). min_key / max_key point into the result bytes.
 */
typedef struct {
    uint64_t off;          /* byte offset of the run within skv_result.bytes */
    uint64_t len;          /* run size in bytes == StatsV1.size_bytes */
    uint64_t put_count;    /* StatsV1.put_count */
    uint64_t delete_count; /* StatsV1.delete_count */
    uint64_t min_key_off;  /* StatsV1.min_key = bytes[min_key_off .. +min_key_len] */
    uint64_t min_key_len;
    uint64_t max_key_off;  /* StatsV1.max_key = bytes[max_key_off .. +max_key_len] */
    uint64_t max_key_len;
    int64_t table_id;      /* SKV_SPLIT_BY_TABLE: owning table (wal_compaction.rs:75-79); else 0 */
    uint64_t reserved;
} skv_run_desc;

typedef struct {
    uint8_t* bytes;      /* concatenated output runs (host memory, or device memory for skv_compact_dev) */
    uint64_t n_bytes;
    skv_run_desc* runs;  /* host memory, n_runs entries, in emission order */
    uint64_t n_runs;
    /* diagnostics */
    uint64_t in_bytes;       /* total input run bytes (the metric's I) */
    uint64_t in_records;     /* records decoded from the inputs */
    uint64_t out_records;    /* records written to the output runs */
    uint64_t dropped_tables; /* SKV_SPLIT_BY_TABLE: tables whose build the reference discards
                                (wal_compaction.rs:103, :168 swallow a failed table task) */
} skv_result;

/* Status codes. The first five mirror the reference's error variants. */
enum {
    SKV_OK = 0,
    SKV_E_EMPTY_INPUT = 1,         /* RunError::EmptyInput          (runs.rs:93, :537-540) */
    SKV_E_UNSUPPORTED_VERSION = 2, /* RunError::UnsupportedVersion  (runs.rs:91, :553-556) */
    SKV_E_IO = 3,                  /* RunError::Io, UnexpectedEof   (runs.rs:85, :570-576, :598-604) */
    SKV_E_FORMAT = 4,              /* RunError::Format(..)          (runs.rs:87; :194, :581, :588, :609, :622) */
    SKV_E_INVALID_INPUT = 5,       /* JobError::InvalidInput, WAL key (jobs/mod.rs:26; wal_compaction.rs:71-79) */
    SKV_E_INVALID_ARG = 6,         /* API misuse: NULL pointers, duplicate seq_no, bad device */
    SKV_E_DEVICE = 7,              /* HIP runtime failure or device capacity exceeded */
    SKV_E_UNSUPPORTED = 8,         /* input shape outside what this build supports (message says which) */
    SKV_E_INTERNAL = 9             /* JobError::Internal (jobs/mod.rs:29-30): a WAL table channel send that
                                      cannot succeed (wal_compaction.rs:157-161) */
};

/* skv_compact flags */
enum {
    SKV_DROP_TOMBSTONES = 1, /* drop Delete ops after the merge: compaction into Level::max()
                                (table_tree_compaction.rs:139-145, metadata.rs:117-126) */
    SKV_SPLIT_BY_TABLE = 2   /* WAL compaction: split merged ops by "{table_id}." key prefix, strip
                                it, one build_runs per table with the reference's exactly-one-run
                                rule and error swallowing (wal_compaction.rs:66-174) */
};

/* Per-phase device timings of the last call (HIP events on the ctx stream), when enabled. */
typedef struct {
    double total_ms;    /* first kernel -> last kernel of the compaction */
    double parse_ms;    /* record-boundary discovery + key extraction */
    double check_ms;    /* in-stream order / error triggers */
    double merge_ms;    /* splitters + tile merge + dedup/filter + prefix sums */
    double chain_ms;    /* greedy max-size split (run boundaries + stats) */
    double gather_ms;   /* byte gather of surviving records into output runs */
    uint64_t gather_read_bytes;  /* algorithmic bytes read by the gather (surviving input records) */
    uint64_t gather_write_bytes; /* algorithmic bytes written by the gather (== output bytes) */
    uint64_t host_syncs;
    double host_total_ms;  /* wall time inside the skv_compact* call */
    double host_sync_ms;   /* of which: waiting in stream synchronisations */
    /* which device path produced the result (SKV_PATH_*) and its dominant kernel: HIP-event
       time of that one launch and its algorithmic bytes */
    uint32_t path;
    uint32_t fused_reject;   /* SKV_PATH_FUSED attempted but poisoned: reason bits, else 0 */
    double hot_ms;
    uint64_t hot_read_bytes;
    uint64_t hot_write_bytes;
    uint32_t sorted;         /* 1: merge fan-in above 1536 streams took the record sort (one list) */
    uint32_t fp_rerun;       /* 1: the merge's key-fingerprint shortcut misordered a tile and the
                                call was rerun with exact key compares (a 64-bit collision) */
    uint32_t host_parts;     /* skv_compact: key-range parts whose H2D, kernels and D2H overlapped
                                (0: the serial copy -> compact -> copy) */
    uint32_t span_parse;     /* always 0 since ABI 7 (the opt-in one-pass span parse was removed; the
                                field keeps the struct layout) */
    uint32_t wal_stage;      /* SKV_SPLIT_BY_TABLE: 1 the one-pass stage (every table kept), 2 the exact
                                stage (the one-pass stage declined or does not apply), 0 no WAL stage */
    uint32_t reserved2;
} skv_timings;

/* skv_timings.path */
enum {
    SKV_PATH_GENERAL = 1, /* chunk-walk parse, record arrays, merge, chain, gather */
    SKV_PATH_FIXED = 2,   /* fixed-stride verifying parse, record arrays, merge, chain, gather */
    SKV_PATH_FUSED = 3    /* one record size and key length <= 16: fused verify/merge/copy tiles */
};

int skv_abi_version(void);
int skv_device_count(int* out);

/* device >= 0: HIP device ordinal. There is no CPU mode: the CPU restatement under oracle/
 * is test infrastructure and is not reachable through this ABI. */
int skv_ctx_create(int device, skv_ctx** out);
void skv_ctx_destroy(skv_ctx* ctx);
const char* skv_last_error(const skv_ctx* ctx); /* reference Display text of the last error */
int skv_ctx_set_profiling(skv_ctx* ctx, int enable);
int skv_ctx_get_timings(const skv_ctx* ctx, skv_timings* out);
/* The host side of a ctx's device: the NUMA node its GPU hangs off (-1: unknown) and the host
 * threads of that device's worker pool (the 10^6-entry table passes of a call run on it). Each
 * device has its own pool, bound to the CPUs of that node, and a ctx's pinned staging and output
 * buffers are allocated on that node. */
int skv_ctx_host_info(const skv_ctx* ctx, int* numa_node, int* host_threads);

/*
 * The placement plans behind the multi-GPU entry points, as pure functions (no HIP device needed:
 * schedulers that place jobs across the GPUs of a node, and CPU tests, call them directly).
 *
 * skv_host_plan: the host side the library gives the GPU whose PCI bus id is `pci_bus_id`
 * ("0000:c1:00.0"), read from `sysfs_root` ("/sys" on a live system; NULL = "/sys") on a machine of
 * `n_devices` GPUs and `hw_threads` CPUs: its NUMA node (-1: unknown), the size of its host pool
 * (the caller + pool_threads - 1 workers, SKV_HOST_THREADS capped at hw_threads / n_devices) and the
 * node's CPUs the pool is bound to (at most max_cpus written). Returns the node's CPU count, or -1
 * when the node is unknown. skv_ctx_host_info reports the same plan for a live ctx.
 *
 * skv_split_deal: how skv_compact_split deals its n_parts key-range parts over n_ctx ctxs whose
 * devices are ctx_device[g]: ctx_of_part[p] = p % n_ctx (the ctx, hence the GPU, that merges part
 * p); h2d_after[p] = the latest earlier part dealt to ANOTHER ctx of the same device, whose H2D copy
 * must land first (ctxs sharing one PCIe link take their inputs in part order), or -1.
 * (orchestrator_service.rs:119-170 places independent jobs; this places one job's parts.)
 */
int skv_host_plan(const char* sysfs_root, const char* pci_bus_id, int n_devices, int hw_threads, int* numa_node,
                  int* pool_threads, int* cpus, int max_cpus);
int skv_split_deal(const int* ctx_device, uint32_t n_ctx, uint64_t n_parts, uint32_t* ctx_of_part,
                   int64_t* h2d_after);

/*
 * Test hooks, for the parity suite only: they force the rare paths a call would otherwise take only
 * on rare data (the general path where the fused one applies, the record sort at small fan-in, a
 * fingerprint collision and its exact rerun, small parse chunks, the exact WAL stage, kernel ingest,
 * an injected failure after a pipeline part, split modes, sort search variants, a small grid's worth
 * of fused tile slots). Names: SKV_FUSED, SKV_SORT, SKV_FP_TEST, SKV_FP_GATHER, SKV_CHUNK_BYTES,
 * SKV_WAL_FUSED, SKV_INGEST, SKV_TEST_FAIL_PART, SKV_PAR_COPY_MIN, SKV_HI_STEP, SKV_SPLIT,
 * SKV_SPLIT_DEBUG, SKV_SPLIT_SEG, SKV_SPLIT_NC, SKV_SORT_TWO_PASS, SKV_SB_NT, SKV_SB_GMAX,
 * SKV_FX_TAIL_SLOTS. value NULL clears one hook, name NULL clears every hook; an unknown name is
 * SKV_E_INVALID_ARG. Process-wide. The library reads none of them from the environment; the only
 * environment variables it reads are the host-pipeline thresholds (SKV_HOST_PIPE, SKV_HOST_PIPE_MIN,
 * SKV_HOST_PARTS, SKV_SPLIT_PARTS), the host pool size (SKV_HOST_THREADS) and two profiling
 * switches (SKV_HOST_TRACE, SKV_SORT_PROF_PRINT).
 */
int skv_test_option(const char* name, const char* value);

/*
 * Host-memory entry point: the shape skyvault's jobs have (Bytes in from get_run,
 * Bytes out to put_run). Inputs are staged to HBM, compacted on the GPU, and the output
 * runs come back in pinned host memory.
 */
int skv_compact(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams,
                uint64_t max_run_size, uint32_t flags, skv_result** out);

/*
 * Device-resident entry point: every runs[i] is a device pointer on the ctx's GPU, and the
 * returned result->bytes is a device pointer owned by the ctx (valid until the next call
 * on the ctx or skv_result_free). Descriptors are host memory.
 */
int skv_compact_dev(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams,
                    uint64_t max_run_size, uint32_t flags, skv_result** out);

/*
 * One compaction split across several GPUs by key range: skv_compact's inputs,
 * semantics, errors and result (pinned host memory, owned by ctxs[0]'s pool), with the work of one
 * call spread over n_ctx distinct ctxs -- normally one per GPU. The call's key-range parts (equal
 * keys never straddle a cut) are staged, merged and deduplicated on the ctxs in parallel;
 * build_runs' greedy split (runs.rs:211-238) is carried across the parts: arithmetically from the
 * parts' survivor counts for one record size with keys of at most 16 bytes, else by each part's
 * split continuing the open run the previous part left; a WAL flush (SKV_SPLIT_BY_TABLE) is cut at
 * table prefixes, so its parts carry nothing. Calls of more than 2^16 member runs, a WAL flush that
 * needs the exact WAL stage, and any call a part finds a data error in run as skv_compact on
 * ctxs[0], which reports the reference's outcome. Errors are reported on ctxs[0]. The ctxs must
 * not be used by other threads during the call. n_ctx == 1 is skv_compact.
 */
int skv_compact_split(skv_ctx* const* ctxs, uint32_t n_ctx, const skv_stream* streams, uint32_t n_streams,
                      uint64_t max_run_size, uint32_t flags, skv_result** out);

/*
 * Writer-side batch encode (replaces writer_service.rs:148-162 process_batch's BTreeMap + build_runs):
 * ops_run holds the batch's WriteOperations in request order, serialized as one v1 run (unsorted,
 * duplicates allowed). The result is build_runs(max_run_size) over the ops sorted by key with
 * the LAST op of each key kept, exactly as the BTreeMap collection does. Decode errors of ops_run
 * are reported like skv_compact's. skv_encode_batch_dev takes a device pointer.
 */
int skv_encode_batch(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size,
                     skv_result** out);
int skv_encode_batch_dev(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size,
                         skv_result** out);

/*
 * Batched point lookups in one run: runs::search_run (runs.rs:285-398) for n_keys keys at once,
 * the cache service's per-key scan (cache_service.rs:52-151). keys = the keys' bytes
 * concatenated, key i = keys[key_offs[i] .. key_offs[i+1]). out[i] gets the key's outcome; a
 * value is at run + val_off. Where search_run would panic for a key, out[i].kind =
 * SKV_LOOKUP_PANIC and the call returns SKV_E_FORMAT with the panic text of the lowest such key
 * ("Invalid marker byte: 7", "Incomplete key data", "Empty run data", ...); the other keys'
 * outcomes are still filled in. run and keys are host memory.
 */
typedef struct {
    uint32_t kind;     /* SKV_LOOKUP_* */
    uint32_t panic;    /* SKV_LOOKUP_PANIC: which check (SKV_PANIC_*) | offending byte << 8 */
    uint64_t val_off;  /* SKV_LOOKUP_FOUND: value bytes at run + val_off, val_len of them */
    uint64_t val_len;
} skv_lookup;
enum { SKV_LOOKUP_NOT_FOUND = 0, SKV_LOOKUP_FOUND = 1, SKV_LOOKUP_TOMBSTONE = 2, SKV_LOOKUP_PANIC = 3 };
enum {
    SKV_PANIC_EMPTY = 1,           /* "Empty run data" */
    SKV_PANIC_VERSION = 2,         /* "Unsupported version: {v}" */
    SKV_PANIC_MARKER = 3,          /* "Invalid marker byte: {m}" */
    SKV_PANIC_KEYLEN = 4,          /* "Incomplete key length data" */
    SKV_PANIC_KEY = 5,             /* "Incomplete key data" */
    SKV_PANIC_VALLEN = 6,          /* "Incomplete value length data" */
    SKV_PANIC_VAL = 7,             /* "Incomplete value data" */
    SKV_PANIC_VALLEN_FOUND = 8,    /* "Incomplete value length data for found key" */
    SKV_PANIC_VAL_FOUND = 9        /* "Incomplete value data for found key" */
};
int skv_search_run(skv_ctx* ctx, const uint8_t* run, uint64_t len, const uint8_t* keys, const uint64_t* key_offs,
                   uint32_t n_keys, skv_lookup* out);

/*
 * A run parsed once for many lookup batches: the cache service keeps a run for many GetFromRun /
 * Prefetch calls (cache_service.rs:52-94), so its boundary index is built once. create stages the
 * run (host memory) into HBM owned by the index and parses it; search is skv_search_run's
 * contract (same outcomes, same panic texts) without re-staging or re-parsing. An index is used
 * with ctxs of the device it was created on; free it with skv_run_index_free.
 */
typedef struct skv_run_index skv_run_index;
int skv_run_index_create(skv_ctx* ctx, const uint8_t* run, uint64_t len, skv_run_index** out);
int skv_run_index_search(skv_ctx* ctx, const skv_run_index* index, const uint8_t* keys, const uint64_t* key_offs,
                         uint32_t n_keys, skv_lookup* out);
void skv_run_index_free(skv_run_index* index);

/*
 * The cache service's ScanFromRun (cache_service.rs:97-151) over runs it has fetched: run i is
 * decoded by runs::read_run_iter (runs.rs:400-510) at SeqNo i64::MAX - i (:113-115), filtered to
 * keys strictly above exclusive_start_key (:125-129), merged by k_way::merge (:134), and read until
 * the max_results-th Put (:140-148; Deletes are returned but not counted). The response items come
 * back as ONE v1 run in response order (an item is a record: Put key + value, or Delete key) with
 * its StatsV1 in runs[0]; no item -> n_runs == 0. max_results outside 1..=10000 -> SKV_E_INVALID_ARG
 * with the reference's text ("max_results must be between 1 and 10000", Status::invalid_argument).
 * A merge error the reader reaches -> its RunError code and Display text, with read_run_iter's
 * texts ("Data format error: Incomplete key length data" / "... value length data" where
 * read_run_stream reports an Io error); the service wraps it as "Merge stream error: {e}" (:141).
 * Unsorted runs are merged in the reference's heap pop order. skv_scan_runs takes host runs and
 * returns the run in pinned host memory; skv_scan_runs_dev takes device pointers and returns a
 * device pointer owned by the ctx (as skv_compact_dev).
 */
int skv_scan_runs(skv_ctx* ctx, const uint8_t* const* runs, const uint64_t* run_lens, uint32_t n_runs,
                  const uint8_t* exclusive_start_key, uint64_t start_len, uint64_t max_results, skv_result** out);
int skv_scan_runs_dev(skv_ctx* ctx, const uint8_t* const* runs, const uint64_t* run_lens, uint32_t n_runs,
                      const uint8_t* exclusive_start_key, uint64_t start_len, uint64_t max_results, skv_result** out);

void skv_result_free(skv_result* r);

#ifdef __cplusplus
}
#endif

#endif /* SKV_H */
