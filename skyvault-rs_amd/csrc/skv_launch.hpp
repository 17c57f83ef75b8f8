// skv_launch.hpp — host-side launch wrappers of skv_kernels.hip (declarations shared by both TUs)
#pragma once
#include "skv_dev.hpp"

// a test hook's value (include/skv.h skv_test_option; skv_ctx.hip), or null
const char* test_opt(const char* name);

namespace skv {
// Raise a kernel's dynamic-LDS limit to the CU's 160 KiB, once per (device, kernel), under a lock:
// the limit is a ceiling, so one value serves every launch size and concurrent ctxs never lower it
// between another thread's set and launch (skv_ctx.hip).
void lds_limit(const void* kernel);
void launch_run_header(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint32_t* hdr_err, RunFmt* fmt,
                       bool slices = false);
void launch_spec(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                 const RunFmt* fmt, uint32_t* run_broken, uint64_t* ch_start, uint64_t* ch_end, uint32_t* ch_cnt,
                 uint32_t* ch_err, bool utf8, uint64_t chunk, uint16_t* slots, uint32_t cap, StgRec* stg,
                 uint32_t scap, uint8_t* ch_stg);
void launch_validate(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                     const uint64_t* ch_start, const uint64_t* ch_end, const uint32_t* ch_err,
                     unsigned long long* bad_bits, uint32_t* run_first_bad);
void launch_fixup(hipStream_t, const RunInfo* runs, uint32_t n_runs, const uint32_t* hdr_err,
                  const uint32_t* run_first_bad, const unsigned long long* bad_bits, uint64_t* ch_start,
                  uint64_t* ch_end, uint32_t* ch_cnt, uint32_t* ch_err, bool utf8, uint64_t chunk, uint16_t* slots,
                  uint32_t cap, uint8_t* ch_stg);
void launch_err_chunk(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                      const uint32_t* ch_err, uint32_t* run_err_chunk);
void launch_mask(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                 const uint32_t* run_err_chunk, const uint32_t* ch_cnt, uint64_t* cnt64);
void launch_run_summary(hipStream_t, const RunInfo* runs, uint32_t n_runs, const uint32_t* hdr_err,
                        const uint32_t* run_err_chunk, const uint32_t* ch_err, const uint64_t* ch_rec_base,
                        RunSummary* out, uint64_t* run_recb);
void launch_emit(hipStream_t, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const RunFmt* fmt,
                 const uint32_t* run_broken, const uint64_t* ch_start, const uint64_t* ch_rec_base,
                 const uint64_t* run_recb, uint64_t R, uint64_t* rec_addr, uint64_t* rec_hi, uint64_t* rec_lo,
                 uint32_t* rec_klen, uint32_t* rec_meta, uint32_t* flags, uint64_t* rec_fp, uint32_t* utf8_bad,
                 const uint16_t* slots, uint32_t cap, uint64_t chunk, const uint64_t* ch_end,
                 const uint64_t* stream_base, unsigned long long* first_dec, const StgRec* stg, uint32_t scap,
                 const uint8_t* ch_stg, uint64_t R_all, uint32_t* blk_chunk);  // blk_chunk: R_all / 64 + 1 + n_chunks
void launch_parse_fixed(hipStream_t, const RunInfo* runs, uint32_t n_runs, const RunFmt* fmt, uint32_t* run_broken,
                        const uint64_t* run_recb, uint64_t R, uint64_t* rec_addr, uint64_t* rec_hi, uint64_t* rec_lo,
                        uint32_t* rec_klen, uint32_t* rec_meta, uint32_t* flags, const uint64_t* stream_base,
                        unsigned long long* first_dec, uint64_t* rec_fp, uint32_t* wave_run,
                        SElem* E = nullptr);
void launch_order_check(hipStream_t, uint64_t R, const uint64_t* stream_base, uint32_t k, const uint64_t* rec_addr,
                        const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen,
                        unsigned long long* first_dec, uint32_t* any_dec);
void launch_sample(hipStream_t, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                   const uint32_t* klen, const uint64_t* off_src, const uint64_t* off_dst, uint32_t k, uint64_t S,
                   uint64_t n_dst, uint64_t* dhi, uint64_t* dlo, uint64_t* dc);
void launch_bounds(hipStream_t, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                   const uint32_t* klen, const uint64_t* off, uint32_t k, const uint64_t* shi, const uint64_t* slo,
                   const uint64_t* sc, uint64_t m, uint64_t T, const uint64_t* rec_addr, uint64_t* bounds,
                   const uint32_t* poison, const L1Cnt* C = nullptr);
// level-1 sample counts per (splitter t, list j) for the level-0 bounds (sc: sorted level-1 samples)
void launch_l1_cnt(hipStream_t, const uint64_t* sc, uint64_t N1, const uint64_t* off0, const uint64_t* l1off,
                   uint32_t k, uint64_t S, uint64_t m, uint64_t T, uint32_t* posof, uint32_t* cnt);
void launch_tile_n(hipStream_t, const uint64_t* bounds, uint32_t k, uint64_t T, uint64_t* tile_n);
void launch_key_fp(hipStream_t, uint64_t R, const uint64_t* rec_addr, const uint32_t* rec_klen, uint64_t* fp);
size_t tile_lds_bytes(uint32_t k);
hipError_t launch_tile(hipStream_t, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                       const uint32_t* klen, const uint64_t* bounds, uint32_t k, uint64_t T, const uint64_t* tile_base,
                       const uint32_t* rec_meta, const uint64_t* rec_addr, uint32_t drop, TileOut O,
                       const uint32_t* poison, uint64_t grid = 0);
void launch_chain(hipStream_t, const uint64_t* Kp, const uint64_t* P, uint64_t max_size, const uint32_t* tile_max,
                  uint64_t n_tiles, uint64_t* run_b, uint64_t* n_runs, uint32_t* tbl, uint64_t max_K,
                  uint64_t max_bytes, const SplitBufs* sp = nullptr);
uint64_t chain_table_entries(uint64_t max_bytes);
// A part of a compaction split over several GPUs (skv_compact_split) that continues the previous
// part's open run of c bytes: out[0] = e1, the records [0, e1) that still join that run, out[1] = K - e1
void launch_carry_first(hipStream_t, const uint64_t* Kp, const uint64_t* P, uint64_t max_size, uint64_t c,
                        uint64_t* out);
// the split of records [e1, K) (written at run_b + 1, relative to e1) turned into the part's split:
// run 0 = the continuation [0, e1), the others shifted by e1
void launch_carry_fix(hipStream_t, uint64_t* run_b, uint64_t* n_runs_out, const uint64_t* P, uint64_t e1, uint64_t K);
// the open run the part leaves to the next one: its bytes (version byte included)
void launch_carry_out(hipStream_t, const uint64_t* run_b, const uint64_t* n_runs_out, const uint64_t* P,
                      uint64_t c, uint32_t cont, uint64_t* out);
void launch_run_stats(hipStream_t, const uint64_t* n_runs, const uint64_t* run_b, const uint64_t* P,
                      const uint64_t* Dp, const uint32_t* m_rec, const uint32_t* rec_klen, DevRunDesc* descs,
                      uint64_t* seg_r0, uint64_t max_runs);
void launch_gather(hipStream_t, const uint64_t* Kp, const uint64_t* n_runs, const uint64_t* run_b, const uint64_t* P,
                   const uint64_t* m_src, const uint64_t* seg_r0, uint8_t* out, uint64_t max_K,
                   const uint64_t* m_dup = nullptr, uint32_t* fp_bad = nullptr);
// skv_wal.hip — SKV_SPLIT_BY_TABLE (wal_compaction.rs:66-174)
constexpr uint32_t WAL_FUSED_RPT = 2;                 // merged records per k_wal_fused thread
constexpr uint32_t WAL_FUSED_G = 256 * WAL_FUSED_RPT;  // merged records per k_wal_fused workgroup
// k_wal_fused's mode word: bits 0-1 diagnostics (2: no output bytes); WAL_STRICT_CANON: a key whose
// prefix is not the canonical "{id}." fails the stage (key-range parts of a pipelined host call)
constexpr uint32_t WAL_STRICT_CANON = 4;
struct WalTStart {  // a table start of k_wal_fused (unordered list; the host sorts by b)
    uint64_t b, W, Dp;  // first merged record, output offset of the table's version byte, deletes before b
    int64_t tid;
    uint32_t nk, prev_nk;  // stripped key length of it and of the record before it
    uint64_t prev_ws;      // stripped size of the record before it
};
void launch_wal_fused(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint64_t* m_src, const uint64_t* P,
                      const uint64_t* Dp, uint8_t* out, uint64_t* tstate, uint32_t* ticket, uint32_t* fail,
                      WalTStart* tlist, uint32_t* tcount, uint32_t tcap, uint64_t* tail, uint32_t diag = 0,
                      const SElem* S = nullptr, const uint32_t* m_rec = nullptr);
void launch_wal_keys(hipStream_t, const uint64_t* Kp, uint64_t max_K, const uint64_t* m_src, const uint64_t* P,
                     int64_t* tid, uint32_t* strip, uint32_t* wnk, uint64_t* wsize, uint8_t* canon,
                     unsigned long long* first_err);
void launch_wal_flags(hipStream_t, const uint64_t* Kp, uint64_t max_K, const int64_t* tid, const uint32_t* strip,
                      const uint8_t* canon, const uint64_t* m_src, const uint32_t* wnk, uint64_t* is_new,
                      uint32_t* bad, bool exact);
void launch_wal_index(hipStream_t, const uint64_t* Kp, uint64_t max_K, const uint64_t* is_new, const uint64_t* new_ex,
                      const uint32_t* bad, uint32_t* tix, uint64_t* tstart, uint32_t* tbad,
                      unsigned long long* tfirst);
void launch_wal_tables(hipStream_t, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart, const uint64_t* Pw,
                       const uint32_t* tbad, uint64_t max_size, uint64_t* run_len, uint64_t* keep);
void launch_wal_desc(hipStream_t, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart, const uint64_t* Pw,
                     const uint64_t* Dp, const uint64_t* keep, const uint64_t* keep_ex, const uint64_t* run_off,
                     const int64_t* tid, const uint32_t* wnk, DevRunDesc* descs);
void launch_wal_gather(hipStream_t, const uint64_t* Kp, uint64_t max_K, const uint32_t* tix, const uint64_t* tstart,
                       const uint64_t* keep, const uint64_t* run_off, const uint64_t* Pw, const uint32_t* strip,
                       const uint64_t* m_src, const uint32_t* wnk, const uint8_t* canon, uint8_t* out);
// skv_heap.hip — k_way::merge's heap pop order for unsorted streams (heap-order mode)
void launch_heap_keys(hipStream_t, uint64_t R, const uint64_t* base, uint32_t k, const uint64_t* hi,
                      const uint64_t* lo, const uint32_t* klen, const uint64_t* addr, uint32_t* eff, uint64_t* blk_agg,
                      uint32_t* carry, uint64_t* ehi, uint64_t* elo, uint32_t* eklen, uint64_t* eaddr);
uint64_t heap_key_blocks(uint64_t R);
void launch_heap_sorted(hipStream_t, uint64_t R, const SElem* S, const uint64_t* hi, const uint64_t* lo,
                        const uint32_t* klen, const uint64_t* addr, uint64_t* shi, uint64_t* slo, uint32_t* sklen,
                        uint64_t* saddr, uint32_t* inv);
void launch_merged_order(hipStream_t, const uint64_t* Kp, uint64_t max_K, const uint32_t* m_rec, const uint64_t* hi,
                         const uint64_t* lo, const uint32_t* klen, const uint64_t* addr, unsigned long long* first_bad);
void launch_wal_sendfail(hipStream_t, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart,
                         const unsigned long long* tfirst, unsigned long long* first_fail);
// skv_stride.hip — fused stride path
void launch_fx_sample(hipStream_t, const FxArgs& A, const uint64_t* off_dst, uint64_t Sstep, uint64_t n_dst,
                      uint64_t* dhi, uint64_t* dlo, uint64_t* dc, const FxUpLevels& up);
void launch_fx_l1cnt(hipStream_t, const FxArgs& A, const uint64_t* sc, uint64_t N1, uint32_t* posof, uint32_t* cnt);
void launch_fx_bounds(hipStream_t, const FxArgs& A, const uint64_t* shi, const uint64_t* slo, uint64_t m,
                      const uint64_t* l1hi, const uint64_t* l1lo, const uint64_t* l1off, uint64_t Sstep);
size_t fx_tile_lds_bytes(uint32_t k);
hipError_t launch_fx_tile(hipStream_t, const FxArgs& A);
uint64_t fx_tile_slots(uint32_t k);
void launch_fx_desc(hipStream_t, const FxArgs& A, DevRunDesc* descs, uint64_t* n_runs_out, uint64_t max_runs);
// *dst = *src with a system-scope store: dst is host-mapped pinned memory the host polls
// the pairs k_tile<true> took as equal keys by fingerprint: any that differ set *fp_bad
void launch_fp_verify(hipStream_t, const unsigned long long* vlo, const unsigned long long* vcount,
                      const uint64_t* vpairs, uint64_t cap, uint32_t* fp_bad, unsigned max_blocks = 8192);
void launch_fx_publish(hipStream_t, const uint64_t* src, uint64_t* dst);
// n bytes src -> dst by a kernel (src may be host-mapped pinned memory): small table uploads that
// must not queue behind bulk DMA on a copy engine (pipelined host calls)
void launch_copy_bytes(hipStream_t, uint8_t* dst, const uint8_t* src, uint64_t n);
// skv_sort.hip — record sort (fan-in above TILE_TARGET / 2)
void launch_sort_load(hipStream_t, uint64_t R, const uint64_t* hi, const uint64_t* lo, const uint64_t* addr,
                      const uint32_t* klen, SElem* E, bool last_wins);
// The merged arrays of a record-sorted call taken straight from the sort (no level-0 merge tiles):
// survivor g = the first record of the g-th distinct key. size / del are the survivors' record sizes
// and Delete bits (scanned into m_P / m_Dp afterwards); mm = (min, max) survivor size. All null: the
// merge stage runs its tiles over the sorted list instead.
struct SortMerged {
    uint32_t* m_rec = nullptr;
    uint64_t* m_src = nullptr;
    uint64_t* size = nullptr;
    uint64_t* del = nullptr;
    uint32_t* mm = nullptr;  // (min, max) surviving record size per k_sort_store block (sort_store_blocks(R) pairs)
    bool arrays = true;      // also the sorted record arrays (hi / lo / addr / klen / cmp_klen / meta)
};
// the record arrays from the sort's elements in record order (the fixed-stride parse wrote the elements)
void launch_sort_unload(hipStream_t, uint64_t R, const SElem* E, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                        uint32_t* klen);
uint64_t sort_store_blocks(uint64_t R);
constexpr uint32_t SORT_MM_OUT = 256;
void sort_prof_read(unsigned long long* out16);  // SKV_SORT_PROF builds: the record sort's phase ticks  // pairs after launch_sort_mm_reduce
void launch_sort_mm_reduce(hipStream_t, const uint32_t* in, uint64_t n, uint32_t* out);
void launch_sort_store(hipStream_t, uint64_t R, const SElem* E, const uint32_t* meta_in, uint32_t const_meta,
                       const uint64_t* newkey, const uint64_t* newkey_ex, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                       uint32_t* klen, uint32_t* cmp_klen, uint32_t* meta, bool last_wins, SortMerged M = SortMerged{});
void launch_sort_sample(hipStream_t, const SElem* E, uint64_t n, uint64_t Ns, SElem* S);
void launch_sort_prefix(hipStream_t, const SElem* Ss, uint64_t ov, uint64_t Tb, uint32_t* L);
void launch_sort_bucket(hipStream_t, const SElem* E, uint64_t n, const SElem* Ss, uint64_t ov, uint64_t nsp,
                        void* split_buf, uint64_t* cnt, uint64_t* bs, bool diag = false);
size_t sort_split_bytes(uint64_t nsp);
void launch_sort_scatter(hipStream_t, const SElem* E, uint64_t n, const uint64_t* bs, const uint64_t* start,
                         const uint32_t* Lb, SElem* out);
void launch_sort_tile(hipStream_t, SElem* in, const uint64_t* start, const uint32_t* L, uint64_t Tb, SElem* out,
                      uint64_t* newkey, bool pre,
                      const void* split_buf = nullptr, uint64_t two_pass_top = 0);
// two-pass bucketing at depth 0 (skv_sort.hip): top (the group size) when it applies, else 0
uint64_t sort_two_pass_top(uint64_t nsp);
uint64_t sort_two_pass_groups(uint64_t nsp);  // super-buckets
void launch_sort_pass_a(hipStream_t, const SElem* E, uint64_t n, const SElem* Ss, uint64_t ov, uint64_t nsp,
                        void* split_buf, uint64_t* scnt, uint64_t* as);
const uint32_t* sort_super_prefix(const void* split_buf, uint64_t nsp);  // per super-bucket common prefix
void launch_sort_pass_b(hipStream_t, const SElem* T, uint64_t n, const uint64_t* sstart, uint64_t nsp,
                        const void* split_buf, uint64_t* cnt, uint64_t* bs);
// skv_search.hip — batched run lookups
void launch_search_bsearch(hipStream_t, const uint8_t* run, uint64_t len, uint64_t R, const uint64_t* rec_addr,
                           const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen,
                           const uint32_t* rec_meta, const uint8_t* qbytes, const uint64_t* qoff, uint32_t n_q,
                           SrResult* out);
void launch_search_scan(hipStream_t, const uint8_t* run, uint64_t len, const uint8_t* qbytes, const uint64_t* qoff,
                        uint32_t n_q, SrResult* out);
uint64_t scan_tmp_words(uint64_t n);
void launch_scan(hipStream_t, const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* tmp);
// skv_stride.hip: a pipelined host call's slices, pinned host -> HBM by the GPU (src == dst mod 16)
struct IngestSlice {
    uint64_t src, dst, len;
};
void launch_ingest(hipStream_t, const IngestSlice* slices, uint32_t n, uint32_t blocks_per_slice);
void launch_ingest_slices(hipStream_t, const IngestSlice* slices, uint64_t n, uint32_t grid);
// per-run record counts of fixed-stride runs ((len - 1) / S) and run-table flags, for calls whose
// run tables stay on the device (skv_compact.hip, wide fixed-stride calls)
enum : uint32_t { RT_NOT_FIXED = 0, RT_NOT_UNIFORM = 1, RT_ANY_FIXED = 2, RT_BODYLESS = 3 };
void launch_run_tables(hipStream_t, const RunInfo* runs, const RunFmt* fmt, uint32_t n_runs, uint64_t* cnt,
                       uint32_t* flags);
// the run table on the device for one-run streams in monotone seq_no order (chunk_base: n + 1 entries)
void launch_run_info(hipStream_t, const uint64_t* ptr, const uint64_t* len, uint32_t n, bool reversed, uint64_t chunk,
                     uint64_t* nch, uint64_t* chunk_base, uint64_t* scan_tmp, RunInfo* runs);
// skv_scan.hip: ScanFromRun after the merge
void launch_scan_filter(hipStream_t, uint64_t R, uint32_t k, const uint64_t* stream_base, const uint64_t* a_addr,
                        const uint64_t* a_hi, const uint64_t* a_lo, const uint32_t* a_klen, const uint32_t* a_meta,
                        const uint8_t* start, uint32_t slen, uint64_t* keep, uint64_t* keepx, uint64_t* scan_tmp,
                        uint64_t* b_addr, uint64_t* b_hi, uint64_t* b_lo, uint32_t* b_klen, uint32_t* b_meta,
                        uint64_t* new_base);
void launch_scan_mark(hipStream_t, const uint64_t* d_K, uint64_t R, const uint32_t* m_rec, const uint64_t* rec_addr,
                      const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen, const uint32_t* rec_meta,
                      const uint8_t* start, uint32_t slen, uint64_t* keep, uint64_t* put, uint64_t* size);
void launch_scan_cut(hipStream_t, const uint64_t* d_K, const uint64_t* putx, const uint64_t* keepx,
                     const uint64_t* offx, uint64_t max_results, uint64_t* info);
void launch_scan_gather(hipStream_t, uint64_t R, const uint64_t* info, const uint64_t* keep, const uint64_t* offx,
                        const uint64_t* size, const uint64_t* m_src, uint8_t* out);
void launch_scan_dn(hipStream_t, const uint64_t* in, const uint64_t* dn, uint64_t max_n, uint64_t* out, uint64_t* tmp);

}  // namespace skv
