// skv_scan_host.hip — ScanFromRun (cache_service.rs:97-151) on the device: skv_scan_runs[_dev].
//
// The scan is the compaction's parse + merge in a job mode (Job::scan): one stream per run at
// SeqNo i64::MAX - index (:113-115), heap-order mode whenever a run is unsorted or undecodable
// (the reference's merge pops such runs in heap order, and a run's decode error surfaces right
// after the pop of its last record that passed the filter). scan_stage then filters the merged
// survivors to key > start (:125-129), cuts after the max_results-th Put (:140-148) and writes the
// response items as one v1 run. Errors are read_run_iter's (runs.rs:400-510): the same checks in
// the same order as read_run_stream, but a length field cut short is a Format error with its own
// text ("Incomplete key length data" :428-430, "Incomplete value length data" :457-459).
#include "skv_host.hpp"

using namespace skv;

// read_run_iter's Display text for a device decode error word. A DERR_IO is a length field cut
// short: the key length when the record's marker leaves fewer than 4 bytes (err_off = the failing
// record's first byte), else the value length.
int scan_err_to_api(uint32_t derr, uint64_t err_off, uint64_t run_len, std::string& msg) {
    if ((derr & 0xFF) == DERR_IO) {
        msg = err_off + 1 + 4 > run_len ? "Data format error: Incomplete key length data"
                                        : "Data format error: Incomplete value length data";
        return SKV_E_FORMAT;
    }
    return derr_to_api(derr, msg);
}

int scan_stage(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint32_t* m_rec,
               const uint64_t* m_src, const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
               const uint32_t* rec_klen, const uint32_t* rec_meta, const uint8_t* d_start, const uint32_t* fp_bad,
               const HeapRes* heap, const std::vector<ScanEvent>& events, skv_result** out) {
    hipStream_t st = ctx->stream;
    uint64_t* keep = dbuf<uint64_t>(ctx, "sc_keep", R + 1);
    uint64_t* put = dbuf<uint64_t>(ctx, "sc_put", R + 1);
    uint64_t* size = dbuf<uint64_t>(ctx, "sc_size", R + 1);
    uint64_t* keepx = dbuf<uint64_t>(ctx, "sc_keepx", R + 1);
    uint64_t* putx = dbuf<uint64_t>(ctx, "sc_putx", R + 1);
    uint64_t* offx = dbuf<uint64_t>(ctx, "sc_offx", R + 1);
    uint64_t* info = dbuf<uint64_t>(ctx, "sc_info", 8);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, "sc_scan_tmp", scan_tmp_words(R + 1) + 64);
    const uint32_t slen = (uint32_t)job.scan_start.size();
    // K survivors (<= R); the scans run over R entries, those past K zeroed
    HIPCHK(hipMemsetAsync(keep, 0, (R + 1) * 8, st));
    HIPCHK(hipMemsetAsync(put, 0, (R + 1) * 8, st));
    HIPCHK(hipMemsetAsync(size, 0, (R + 1) * 8, st));
    launch_scan_mark(st, d_K, R, m_rec, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_start, slen, keep, put, size);
    launch_scan(st, keep, R, keepx, scan_tmp);
    launch_scan(st, put, R, putx, scan_tmp);
    launch_scan(st, size, R, offx, scan_tmp);
    launch_scan_cut(st, d_K, putx, keepx, offx, job.scan_max, info);
    mark(ctx, PH_CHAIN);
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", job.in_bytes + 16);
    launch_scan_gather(st, R, info, keep, offx, size, m_src, d_out);
    HIPCHK(hipGetLastError());
    mark(ctx, PH_GATHER);
    uint64_t h[8];
    {
        uint64_t* hp = (uint64_t*)pinned(ctx, 128);
        d2h(ctx, hp, info, 48);
        d2h(ctx, hp + 6, d_K, 8);
        d2h(ctx, hp + 7, fp_bad, 4);
        sync(ctx);
        memcpy(h, hp, 64);
    }
    if ((uint32_t)h[7]) return RC_RETRY_EXACT;
    const uint64_t gend = h[0], items = h[1], rec_bytes = h[2], puts = h[3], g_first = h[4], g_last = h[5], K = h[6];
    // A run's decode error surfaces after the pop of its last record above the start key, unless
    // the reader has stopped by then: it stops right after the item holding the max-th Put, so the
    // error is seen iff fewer than max Puts were emitted up to that pop. The first error in pop
    // order is the only candidate (a later one is reached later still).
    if (!events.empty()) {
        if (!heap) throw DevError("internal: scan errors without heap-order positions");
        auto g_pop = [&](uint64_t g) { return read_dev(heap->pop_pos + read_dev(m_rec + g)); };
        const ScanEvent* first = nullptr;
        uint64_t first_pos = ~0ull;
        for (const ScanEvent& e : events) {
            const uint64_t p = heap->pos_of_original(e.after_rec);
            if (p < first_pos) {
                first_pos = p;
                first = &e;
            }
        }
        // Puts emitted up to and including pop position first_pos: survivors are in pop order
        uint64_t lo = 0, hi = K, n_le = 0;  // n_le = survivors popped at or before first_pos
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (g_pop(mid) <= first_pos) lo = mid + 1;
            else hi = mid;
        }
        n_le = lo;
        const uint64_t puts_through = n_le ? read_dev(putx + n_le) : 0;
        if (puts_through < job.scan_max) throw ApiError{first->code, first->msg};
    }
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(sizeof(skv_run_desc));
    res->bytes = d_out;
    res->in_bytes = job.in_bytes;
    res->in_records = R;
    res->out_records = items;
    if (items) {
        skv_run_desc& d = res->runs[0];
        memset(&d, 0, sizeof d);
        d.off = 0;
        d.len = 1 + rec_bytes;
        d.put_count = puts;
        d.delete_count = items - puts;
        d.min_key_off = 1 + 5;  // the first item sits right after the version byte
        d.min_key_len = read_dev(rec_klen + read_dev(m_rec + g_first));
        d.max_key_off = 1 + read_dev(offx + g_last) + 5;
        d.max_key_len = read_dev(rec_klen + read_dev(m_rec + g_last));
        res->n_runs = 1;
        res->n_bytes = 1 + rec_bytes;
    }
    (void)gend;
    if (ctx->profiling) {
        HIPCHK(hipEventSynchronize(ctx->ev[PH_GATHER]));
        float ms[PH_N] = {};
        for (int p = PH_PARSE; p < PH_N; ++p) HIPCHK(hipEventElapsedTime(&ms[p], ctx->ev[p - 1], ctx->ev[p]));
        float tot = 0;
        HIPCHK(hipEventElapsedTime(&tot, ctx->ev[PH_START], ctx->ev[PH_GATHER]));
        skv_timings& t = ctx->timings;
        t.total_ms = tot;
        t.parse_ms = ms[PH_PARSE];
        t.check_ms = ms[PH_CHECK];
        t.merge_ms = ms[PH_MERGE];
        t.chain_ms = ms[PH_CHAIN];
        t.gather_ms = ms[PH_GATHER];
        t.hot_ms = ms[PH_MERGE];
    }
    ctx->timings.path = SKV_PATH_GENERAL;
    ctx->timings.host_syncs = ctx->syncs;
    *out = res;
    return SKV_OK;
}

// the scan's job: run i as stream i at SeqNo i64::MAX - i
static int scan_job(skv_ctx* ctx, const uint8_t* const* runs, const uint64_t* run_lens, uint32_t n_runs,
                    const uint8_t* start_key, uint64_t start_len, uint64_t max_results, Job& job) {
    if (max_results < 1 || max_results > 10000)  // cache_service.rs:101-104 (Status::invalid_argument)
        return set_err(ctx, SKV_E_INVALID_ARG, "max_results must be between 1 and 10000");
    if (n_runs && (!runs || !run_lens)) return set_err(ctx, SKV_E_INVALID_ARG, "runs/run_lens is NULL");
    if (start_len && !start_key) return set_err(ctx, SKV_E_INVALID_ARG, "start key is NULL");
    if (start_len >= (1ull << 31)) return set_err(ctx, SKV_E_INVALID_ARG, "start key of 2 GiB or more");
    std::vector<skv_stream> st(n_runs);
    for (uint32_t i = 0; i < n_runs; ++i) st[i] = skv_stream{&runs[i], &run_lens[i], 1u, INT64_MAX - (int64_t)i};
    const int rc = build_job(ctx, st.data(), n_runs, 1ull << 62, 0, job);
    job.scan = true;
    job.scan_start.assign((const char*)start_key, start_len);
    job.scan_max = max_results;
    return rc;
}

extern "C" {

int skv_scan_runs(skv_ctx* ctx, const uint8_t* const* runs, const uint64_t* run_lens, uint32_t n_runs,
                  const uint8_t* start_key, uint64_t start_len, uint64_t max_results, skv_result** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;
    const int rc = scan_job(ctx, runs, run_lens, n_runs, start_key, start_len, max_results, job);
    if (rc) return rc;
    return compact_host_job(ctx, job, out, t_entry);
}

int skv_scan_runs_dev(skv_ctx* ctx, const uint8_t* const* runs, const uint64_t* run_lens, uint32_t n_runs,
                      const uint8_t* start_key, uint64_t start_len, uint64_t max_results, skv_result** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;
    const int rc = scan_job(ctx, runs, run_lens, n_runs, start_key, start_len, max_results, job);
    if (rc) return rc;
    return run_guarded(ctx, job, out, t_entry);
}

}  // extern "C"
