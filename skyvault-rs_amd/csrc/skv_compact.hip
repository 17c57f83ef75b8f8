// skv_compact.hip — compact_device: the general / fixed-stride / record-sort path of one compaction
// (parse -> merge -> [filter | WAL split] -> split -> gather), the fp-shortcut rerun, the WAL stage
// and the writer batch entry points. skv_compact_dev is the device-resident C entry.
#include "skv_host.hpp"

using namespace skv;

// the whole call again with exact key compares in the merge rounds
int rerun_exact(skv_ctx* ctx, const Job& job, skv_result** out) {
    ctx->exact_keys = true;
    int rc;
    try {
        rc = compact_device(ctx, job, out, false);
    } catch (...) {
        ctx->exact_keys = false;
        throw;
    }
    ctx->exact_keys = false;
    ctx->timings.fp_rerun = 1;
    return rc;
}

// the WAL stage's result (both paths): descriptors already on the host
static int wal_result(skv_ctx* ctx, const Job& job, uint64_t R, uint8_t* d_out, skv_run_desc* runs, uint64_t n_tables,
                      uint64_t n_kept, uint64_t n_bytes, skv_result** out) {
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = runs;
    uint64_t out_records = 0;
    for (uint64_t i = 0; i < n_kept; ++i) out_records += res->runs[i].put_count + res->runs[i].delete_count;
    res->n_runs = n_kept;
    res->bytes = d_out;
    res->n_bytes = n_bytes;
    res->in_bytes = job.in_bytes;
    res->in_records = R;
    res->out_records = out_records;
    res->dropped_tables = n_tables - n_kept;
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
        t.gather_read_bytes = n_bytes - n_kept;
        t.gather_write_bytes = n_bytes;
        t.hot_ms = ms[PH_GATHER];
    }
    ctx->timings.path = SKV_PATH_GENERAL;  // WAL stage: the dominant launch is k_wal_gather / k_wal_fused
    ctx->timings.hot_read_bytes = n_bytes - n_kept;
    ctx->timings.hot_write_bytes = n_bytes;
    ctx->timings.host_syncs = ctx->syncs;
    *out = res;
    return SKV_OK;
}

// The one-pass WAL stage (k_wal_fused, skv_wal.hip) for sorted inputs: every table kept, checked
// after the fact. RC_DECLINED when that does not hold (a bad key, an order error, a table over max,
// more than WF_TCAP tables): the exact stage below then runs and gives the reference's outcome.
constexpr int RC_DECLINED = -1000;
constexpr uint32_t WF_TCAP = 1u << 16, WF_GUESS = 1024;
static int wal_fused(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint64_t* m_src,
                     const uint64_t* m_P, const uint64_t* m_Dp, const uint32_t* fp_bad, skv_result** out,
                     const SElem* S, const uint32_t* m_rec) {
    hipStream_t st = ctx->stream;
    // a part of a pipelined host call writes into the call's shared output buffer
    uint8_t* d_out = job.dev_out ? job.dev_out : dbuf<uint8_t>(ctx, "out", job.in_bytes + R + 16);
    const uint64_t nwg = (R + WAL_FUSED_G - 1) / WAL_FUSED_G;
    uint64_t* tstate = dbuf<uint64_t>(ctx, "wf_state", nwg + 1);
    uint32_t* words = dbuf<uint32_t>(ctx, "wf_words", 4);  // ticket, fail bits, table count
    uint64_t* tail = dbuf<uint64_t>(ctx, "wf_tail", 8);
    WalTStart* tl = dbuf<WalTStart>(ctx, "wf_tlist", WF_TCAP);
    HIPCHK(hipMemsetAsync(tstate, 0, (nwg + 1) * 8, st));
    HIPCHK(hipMemsetAsync(words, 0, 16, st));
    HIPCHK(hipMemsetAsync(tail, 0, 64, st));
    mark(ctx, PH_CHAIN);
    // in a key-range part every key must carry the canonical "{id}." prefix: the cuts are canonical
    // prefixes, so only then does no table straddle two parts (WAL_STRICT_CANON)
    launch_wal_fused(st, d_K, R, m_src, m_P, m_Dp, d_out, tstate, words, words + 1, tl, words + 2, WF_TCAP, tail,
                     job.part ? WAL_STRICT_CANON : 0u, S, m_rec);
    HIPCHK(hipGetLastError());
    mark(ctx, PH_GATHER);
    uint8_t* hp = (uint8_t*)pinned(ctx, 128 + WF_GUESS * sizeof(WalTStart));
    d2h(ctx, hp, d_K, 8);
    d2h(ctx, hp + 8, fp_bad, 4);
    d2h(ctx, hp + 16, words, 16);
    d2h(ctx, hp + 32, tail, 64);
    d2h(ctx, hp + 128, tl, WF_GUESS * sizeof(WalTStart));
    sync(ctx);
    htrace("wal fused read");
    uint64_t K, tw[8];
    uint32_t fpb, w[4];
    memcpy(&K, hp, 8);
    memcpy(&fpb, hp + 8, 4);
    memcpy(w, hp + 16, 16);
    memcpy(tw, hp + 32, 64);
    if (fpb) return RC_RETRY_EXACT;
    const uint32_t nt = w[2];
    if (w[1] || nt > WF_TCAP) return RC_DECLINED;
    std::vector<WalTStart> E(nt);
    memcpy(E.data(), hp + 128, (size_t)std::min(nt, WF_GUESS) * sizeof(WalTStart));
    if (nt > WF_GUESS)
        HIPCHK(hipMemcpy(E.data() + WF_GUESS, tl + WF_GUESS, (nt - WF_GUESS) * sizeof(WalTStart), hipMemcpyDeviceToHost));
    std::sort(E.begin(), E.end(), [](const WalTStart& a, const WalTStart& b) { return a.b < b.b; });
    // tw: output bytes of the call, stripped size and key length of the last record, -, deletes
    const uint64_t n_bytes = tw[0], ws_last = tw[1], nk_last = tw[2], Dp_all = tw[4];
    skv_run_desc* runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, nt) * sizeof(skv_run_desc));
    for (uint32_t t = 0; t < nt; ++t) {  // k_wal_desc's fields, and the one-run rule (:126-137)
        const bool last = t + 1 == nt;
        const uint64_t b = E[t].b, e = last ? K : E[t + 1].b;
        const uint64_t off = E[t].W, end = last ? n_bytes : E[t + 1].W;  // [version byte, records]
        const uint64_t Dpe = last ? Dp_all : E[t + 1].Dp;
        if (!(e - b == 1 || end - off <= job.max_run_size)) {
            free(runs);
            return RC_DECLINED;
        }
        skv_run_desc& d = runs[t];
        d.off = off;
        d.len = end - off;
        d.delete_count = Dpe - E[t].Dp;
        d.put_count = (e - b) - d.delete_count;
        d.min_key_off = off + 1 + 5;
        d.min_key_len = E[t].nk;
        // the last record's piece: its stripped size back from the table's end (+ the version byte
        // when it is the table's only record)
        const uint64_t lws = (last ? ws_last : E[t + 1].prev_ws) + (e - b == 1 ? 1 : 0);
        d.max_key_off = end - lws + (e - b == 1 ? 1 : 0) + 5;
        d.max_key_len = last ? nk_last : E[t + 1].prev_nk;
        d.table_id = E[t].tid;
        d.reserved = 0;
    }
    return wal_result(ctx, job, R, d_out, runs, nt, nt, n_bytes, out);
}

// SKV_SPLIT_BY_TABLE after the merge: table split, prefix strip, one run per kept table
// (skv_wal.hip): the one-pass stage when it applies, else the exact one (one extra host sync reads
// the surviving record count first).
int wal_stage(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint32_t* m_rec,
                     const uint64_t* m_src, const uint64_t* m_P, const uint64_t* m_Dp, const uint64_t* rec_addr,
                     const uint32_t* rec_klen, const uint32_t* fp_bad, const HeapRes* heap, skv_result** out,
                     const SElem* sorted) {
    hipStream_t st = ctx->stream;
    const char* fe = test_opt("SKV_WAL_FUSED");
    if (!heap && !(fe && fe[0] == '0') && R > 0) {
        // sorted: the record sort's output, its elements' true key prefixes by sorted position (m_rec)
        const int rc = wal_fused(ctx, job, R, d_K, m_src, m_P, m_Dp, fp_bad, out, sorted, m_rec);
        if (rc != RC_DECLINED) {
            ctx->timings.wal_stage = 1;
            return rc;
        }
    }
    // A part of a pipelined host call takes only the one-pass outcome (every table kept, whole inside
    // the part): a dropped table, a bad key or a non-canonical prefix ends the attempt, and the serial
    // path gives the reference's outcome for the whole call.
    if (job.part) throw ApiError{SKV_E_FORMAT, "part: the WAL stage needs the exact path"};
    ctx->timings.wal_stage = 2;
    uint64_t K = 0;
    {
        uint64_t* hp = (uint64_t*)pinned(ctx, 64);
        d2h(ctx, hp, d_K, 8);
        d2h(ctx, hp + 1, fp_bad, 4);
        sync(ctx);
        K = hp[0];
        if ((uint32_t)hp[1]) return RC_RETRY_EXACT;
    }
    htrace("wal K read");
    (void)R;
    int64_t* tid = dbuf<int64_t>(ctx, "w_tid", K + 1);
    uint32_t* strip = dbuf<uint32_t>(ctx, "w_strip", K + 1);
    uint8_t* canon = dbuf<uint8_t>(ctx, "w_canon", K + 1);
    uint32_t* wnk = dbuf<uint32_t>(ctx, "w_nk", K + 1);
    uint64_t* wsize = dbuf<uint64_t>(ctx, "w_size", K + 1);
    uint64_t* is_new = dbuf<uint64_t>(ctx, "w_new", K + 1);
    uint64_t* new_ex = dbuf<uint64_t>(ctx, "w_new_ex", K + 1);
    uint32_t* bad = dbuf<uint32_t>(ctx, "w_bad", K + 1);
    uint32_t* tix = dbuf<uint32_t>(ctx, "w_tix", K + 1);
    uint64_t* tstart = dbuf<uint64_t>(ctx, "w_tstart", K + 2);
    uint32_t* tbad = dbuf<uint32_t>(ctx, "w_tbad", K + 1);
    uint64_t* Pw = dbuf<uint64_t>(ctx, "w_P", K + 1);
    uint64_t* run_len = dbuf<uint64_t>(ctx, "w_run_len", K + 1);
    uint64_t* keep = dbuf<uint64_t>(ctx, "w_keep", K + 1);
    uint64_t* run_off = dbuf<uint64_t>(ctx, "w_run_off", K + 1);
    uint64_t* keep_ex = dbuf<uint64_t>(ctx, "w_keep_ex", K + 1);
    unsigned long long* first_err = dbuf<unsigned long long>(ctx, "w_first_err", 2);  // bad key, failed send
    unsigned long long* tfirst = dbuf<unsigned long long>(ctx, "w_tfirst", K + 1);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, "w_scan_tmp", scan_tmp_words(K + 1) + 64);
    DevRunDesc* d_desc = dbuf<DevRunDesc>(ctx, "descs", K + 1);
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", job.in_bytes + K + 16);  // in_bytes: the run lengths' sum
    HIPCHK(hipMemsetAsync(first_err, 0xFF, 16, st));
    HIPCHK(hipMemsetAsync(tfirst, 0xFF, (K + 1) * 8, st));
    HIPCHK(hipMemsetAsync(tbad, 0, (K + 1) * 4, st));
    // run_len / keep: k_wal_tables writes the first NT (the table count, on the device) and the
    // scans below read no further
    launch_wal_keys(st, d_K, K, m_src, m_P, tid, strip, wnk, wsize, canon, first_err);
    launch_wal_flags(st, d_K, K, tid, strip, canon, m_src, wnk, is_new, bad, heap != nullptr);
    launch_scan(st, is_new, K, new_ex, scan_tmp);  // new_ex[K] = number of tables
    launch_wal_index(st, d_K, K, is_new, new_ex, bad, tix, tstart, tbad, tfirst);
    launch_wal_sendfail(st, new_ex + K, K, tstart, tfirst, first_err + 1);
    launch_scan(st, wsize, K, Pw, scan_tmp);       // stripped record offsets
    const uint64_t* d_NT = new_ex + K;
    launch_wal_tables(st, d_NT, K, tstart, Pw, tbad, job.max_run_size, run_len, keep);
    launch_scan_dn(st, run_len, d_NT, K, run_off, scan_tmp);  // output offset per table, total at [K]
    launch_scan_dn(st, keep, d_NT, K, keep_ex, scan_tmp);     // run index per kept table, count at [K]
    launch_wal_desc(st, d_NT, K, tstart, Pw, m_Dp, keep, keep_ex, run_off, tid, wnk, d_desc);
    mark(ctx, PH_CHAIN);
    launch_wal_gather(st, d_K, K, tix, tstart, keep, run_off, Pw, strip, m_src, wnk, canon, d_out);
    HIPCHK(hipGetLastError());
    mark(ctx, PH_GATHER);
    uint64_t h[5];
    {
        uint64_t* hp = (uint64_t*)pinned(ctx, 64);
        d2h(ctx, hp, first_err, 8);
        d2h(ctx, hp + 1, d_NT, 8);
        d2h(ctx, hp + 2, keep_ex + K, 8);
        d2h(ctx, hp + 3, run_off + K, 8);
        d2h(ctx, hp + 4, first_err + 1, 8);
        sync(ctx);
        memcpy(h, hp, 40);
    }
    htrace("wal outcome read");
    // The job's first failure in merged order: a bad key (:67-79 `?`), a send to a table whose task
    // has failed (:157-161), or (heap-order mode) a stream's decode error (:66-67 `result?`).
    // Sorted inputs without decode errors: survivor indices are the merged order.
    std::vector<JobEvent> ev;
    auto pos_of_survivor = [&](uint64_t j) -> uint64_t {
        return heap ? read_dev(heap->pop_pos + read_dev(m_rec + j)) : j;
    };
    if (h[0] != ~0ull)
        ev.push_back({pos_of_survivor(h[0]), 0, SKV_E_INVALID_INPUT,
                      wal_key_error(fetch_key_at(ctx, read_dev(m_src + h[0])))});
    if (h[4] != ~0ull)
        ev.push_back({pos_of_survivor(h[4]), 1, SKV_E_INTERNAL, "Internal error: Failed to send operation to table channel"});
    if (heap)
        for (const HeapRes::Dec& d : heap->dec) {
            std::string msg;
            const int code = derr_to_api(d.err, msg);
            ev.push_back({heap->pos_of_original(d.rec), 2, code, msg});
        }
    throw_first(ev);
    const uint64_t n_tables = h[1], n_kept = h[2], n_bytes = h[3];
    skv_run_desc* runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, n_kept) * sizeof(skv_run_desc));
    if (n_kept) HIPCHK(hipMemcpy(runs, d_desc, n_kept * sizeof(DevRunDesc), hipMemcpyDeviceToHost));
    return wal_result(ctx, job, R, d_out, runs, n_tables, n_kept, n_bytes, out);
}

// Sorts n SElems by (key, record index) (skv_sort.hip); E and T are n-element buffers, the
// result is in the returned one of the two. Samples recurse with their own buffers (depth).
SElem* sort_elems(skv_ctx* ctx, SElem* E, SElem* T, uint64_t n, int depth, uint64_t* newkey) {
    hipStream_t st = ctx->stream;
    char nm[64];
    if (n <= (uint64_t)SORT_CAP) {  // one bucket
        snprintf(nm, sizeof nm, "sort_one%d", depth);
        uint64_t* start = dbuf<uint64_t>(ctx, nm, 2);
        const uint64_t h[2] = {0, n};
        h2d_up(ctx, start, h, 16);
        launch_sort_tile(st, E, start, nullptr, 1, T, newkey, false);
        return T;
    }
    const uint64_t Ns = (n + SORT_EVERY - 1) / SORT_EVERY;
    snprintf(nm, sizeof nm, "sort_s%d", depth);
    SElem* S = dbuf<SElem>(ctx, nm, Ns);
    snprintf(nm, sizeof nm, "sort_sT%d", depth);
    SElem* S2 = dbuf<SElem>(ctx, nm, Ns);
    launch_sort_sample(st, E, n, Ns, S);
    const SElem* Ss = sort_elems(ctx, S, S2, Ns, depth + 1);
    const uint64_t Tb = (Ns + SORT_OV - 1) / SORT_OV;  // buckets; Tb - 1 splitters
    snprintf(nm, sizeof nm, "sort_L%d", depth);
    uint32_t* L = dbuf<uint32_t>(ctx, nm, Tb);
    snprintf(nm, sizeof nm, "sort_cnt%d", depth);
    uint64_t* cnt = dbuf<uint64_t>(ctx, nm, Tb + 1);
    snprintf(nm, sizeof nm, "sort_bs%d", depth);
    uint64_t* bs = dbuf<uint64_t>(ctx, nm, n);
    snprintf(nm, sizeof nm, "sort_start%d", depth);
    uint64_t* start = dbuf<uint64_t>(ctx, nm, Tb + 1);
    snprintf(nm, sizeof nm, "sort_scan%d", depth);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, nm, scan_tmp_words(Tb) + 64);
    launch_sort_prefix(st, Ss, SORT_OV, Tb, L);
    HIPCHK(hipMemsetAsync(cnt, 0, (Tb + 1) * 8, st));
    snprintf(nm, sizeof nm, "sort_split%d", depth);
    uint8_t* split_buf = dbuf<uint8_t>(ctx, nm, sort_split_bytes(Tb - 1));
    // depth 0 (the records themselves): the scatter stores each element's window from its bucket's
    // common prefix on, so the bucket sort reads no record bytes (and restores the true prefixes on
    // output from the bucket's splitter). Sample levels keep their keys.
    const bool pre = depth == 0;
    const uint64_t top2 = pre ? sort_two_pass_top(Tb - 1) : 0;
    if (top2) {  // two-pass bucketing (skv_sort.hip): super-buckets, then buckets, both searched in LDS
        const uint64_t G = sort_two_pass_groups(Tb - 1);
        uint64_t* scnt = dbuf<uint64_t>(ctx, "sort_scnt", G + 1);
        uint64_t* sstart = dbuf<uint64_t>(ctx, "sort_sstart", G + 1);
        uint64_t* sscan = dbuf<uint64_t>(ctx, "sort_sscan", scan_tmp_words(G) + 64);
        HIPCHK(hipMemsetAsync(scnt, 0, (G + 1) * 8, st));
        launch_sort_pass_a(st, E, n, Ss, SORT_OV, Tb - 1, split_buf, scnt, bs);
        launch_scan(st, scnt, G, sstart, sscan);
        launch_sort_scatter(st, E, n, bs, sstart, sort_super_prefix(split_buf, Tb - 1), T);
        launch_sort_pass_b(st, T, n, sstart, Tb - 1, split_buf, cnt, bs);
        launch_scan(st, cnt, Tb, start, scan_tmp);
        launch_sort_scatter(st, T, n, bs, start, nullptr, E);
        launch_sort_tile(st, E, start, L, Tb, T, newkey, true, split_buf, top2);
        return T;
    }
    launch_sort_bucket(st, E, n, Ss, SORT_OV, Tb - 1, split_buf, cnt, bs, pre);
    launch_scan(st, cnt, Tb, start, scan_tmp);
    launch_sort_scatter(st, E, n, bs, start, pre ? L : nullptr, T);
    // (the records' level: the output elements carry their keys' true prefixes again)
    launch_sort_tile(st, T, start, L, Tb, E, newkey, pre, pre ? split_buf : nullptr);
    return E;
}

// The merged order of R records as one sorted list: the record arrays are replaced by sorted
// copies (merges of more than TILE_TARGET / 2 streams, whose splitter bounds table would be
// tiles x streams). hi/lo/cmp_klen become dense key ranks for the merge stage; klen stays the real
// key length (descriptors, WAL split).
void sort_records(skv_ctx* ctx, uint64_t R, uint64_t*& hi, uint64_t*& lo, uint64_t*& addr, uint32_t*& klen,
                         uint32_t*& meta, const uint32_t*& cmp_klen, bool last_wins, const SElem** sorted,
                         uint32_t const_meta, const SortMerged* merged, uint64_t** d_K, bool e_ready) {
    hipStream_t st = ctx->stream;
    SElem* E = dbuf<SElem>(ctx, "sort_e", R);  // e_ready: the fixed-stride parse wrote it
    SElem* T = dbuf<SElem>(ctx, "sort_t", R);
    uint64_t* newkey = dbuf<uint64_t>(ctx, "sort_newkey", R + 1);
    uint64_t* newkey_ex = dbuf<uint64_t>(ctx, "sort_newkey_ex", R + 1);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, "sort_rank_scan", scan_tmp_words(R) + 64);
    if (!e_ready) launch_sort_load(st, R, hi, lo, addr, klen, E, last_wins);
    const SElem* S = sort_elems(ctx, E, T, R, 0, newkey);
    launch_scan(st, newkey, R, newkey_ex, scan_tmp);
    uint64_t* nhi = dbuf<uint64_t>(ctx, "srt_hi", R);
    uint64_t* nlo = dbuf<uint64_t>(ctx, "srt_lo", R);
    uint64_t* naddr = dbuf<uint64_t>(ctx, "srt_addr", R);
    uint32_t* nklen = dbuf<uint32_t>(ctx, "srt_klen", R);
    uint32_t* ncklen = dbuf<uint32_t>(ctx, "srt_cklen", R);
    uint32_t* nmeta = dbuf<uint32_t>(ctx, "srt_meta", R);
    launch_sort_store(st, R, S, meta, const_meta, newkey, newkey_ex, nhi, nlo, naddr, nklen, ncklen, nmeta, last_wins,
                      merged ? *merged : SortMerged{});
    HIPCHK(hipGetLastError());
    if (d_K) *d_K = newkey_ex + R;  // distinct keys (the survivors when merged arrays were asked for)
    if (sorted) *sorted = S;
    hi = nhi;
    lo = nlo;
    addr = naddr;
    klen = nklen;
    meta = nmeta;
    cmp_klen = ncklen;
}

void ensure_aux(skv_ctx* ctx) {  // the ctx's second stream and its two events
    if (ctx->aux_stream) return;
    HIPCHK(hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ctx->aux_ev[0], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->aux_ev[1], hipEventDisableTiming));
}

// allow_deferred: on the fixed-stride fast path, launch the merge without waiting for the parse's
// verdict (broken runs / order errors / oversized records) and check it with the final readback;
// a bad verdict discards the result and reruns the call on the exact general path.
int compact_device(skv_ctx* ctx, const Job& job, skv_result** out, bool allow_deferred) {
    hipStream_t st = ctx->stream;
    // nothing of an earlier call may still read this ctx's buffers on the aux stream
    if (ctx->aux_stream) HIPCHK(hipStreamSynchronize(ctx->aux_stream));
    ctx->syncs = 0;
    ctx->up_chunk = 0;
    ctx->up_off = 0;
    mark(ctx, PH_START);
    htrace("start");
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t my_gen = ++ctx->table_gen;
    auto tables_mine = [&]() {  // the s_* tables below are ctx storage that a nested call refills
        if (ctx->table_gen != my_gen) throw DevError("internal: host tables read after a nested rerun refilled them");
    };
    // ---- run table ------------------------------------------------------------------------
    std::vector<RunInfo>& runs = ctx->s_runs;  // (a rerun returns right after its nested call)
    runs.resize(job.run_ptr.size());  // same size as the last call: no fill
    std::vector<uint32_t>& stream_first_run = ctx->s_sfr;
    stream_first_run.resize(k + 1);
    // speculative walk length: CHUNK, doubled up to 64 KiB while a call still has >= 2^16 walks (a
    // big call spends fewer re-synchronising starts per record). Parse of config 3 shapes by walk
    // length (tools/stage_probe.py): 59 GiB 16/32/64 KiB 30.3/26.4/25.2 ms; 3.7 GiB 4/16/32/64 KiB
    // 3.59/2.27/2.14/2.34; 0.23 GiB 4/8/16 KiB 0.50/0.49/0.53; 0.06 GiB 4/16 KiB 0.38/0.47
    uint64_t chunk = CHUNK;
    if (const char* ce = test_opt("SKV_CHUNK_BYTES"))  // slot offsets are 16-bit: at most 64 KiB
        chunk = std::min<uint64_t>(65536, std::max<uint64_t>(CHUNK, strtoull(ce, nullptr, 10)));
    else
        while (chunk < 65536 && job.in_bytes / (2 * chunk) >= (1ull << 16)) chunk *= 2;
    auto n_chunks_of = [chunk](uint64_t len) { return len >= 2 ? (uint32_t)((len - 1 + chunk - 1) / chunk) : 0u; };
    uint64_t n_chunks = 0;
    // one run per stream in a monotone seq_no order, past the splitter merge's fan-in (config 5's
    // shape, the device-table calls below): the run table is built on the device (k_run_info) from
    // the caller-order pointer / length arrays, and the host table only if a host path needs it
    const bool runs_dev = k > (uint32_t)TILE_TARGET / 2 && job.one_run_each && job.caller_order != 0 && !job.scan &&
                          !job.search && !job.batch && !job.part;
    bool host_runs_built = false;
    auto build_host_runs = [&]() {  // blocks of streams (rank order) on host threads: runs and chunks before each block, then fill
        runs.resize(job.run_ptr.size());
        const unsigned nb = par_nblocks(k);
        std::vector<uint64_t> rb(nb + 1, 0), cb(nb + 1, 0);
        par_run(k, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
            uint64_t nr = 0, nc = 0;
            for (uint64_t s = lo; s < hi; ++s) {
                const InStream& S = job.ranked[s];
                nr += S.n_runs;
                for (uint32_t m = 0; m < S.n_runs; ++m) nc += n_chunks_of(job.run_len[S.first + m]);
            }
            rb[b + 1] = nr;
            cb[b + 1] = nc;
        });
        for (unsigned b = 0; b < nb; ++b) {
            rb[b + 1] += rb[b];
            cb[b + 1] += cb[b];
        }
        par_run(k, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
            uint64_t at = rb[b], nc = cb[b];
            for (uint64_t s = lo; s < hi; ++s) {
                stream_first_run[s] = (uint32_t)at;
                const InStream& S = job.ranked[s];
                for (uint32_t m = 0; m < S.n_runs; ++m, ++at) {
                    RunInfo& R = runs[at];
                    R.ptr = job.run_ptr[S.first + m];
                    R.len = job.run_len[S.first + m];
                    R.chunk_base = nc;
                    R.n_chunks = n_chunks_of(R.len);
                    R.stream = (uint32_t)s;
                    nc += R.n_chunks;
                }
            }
        });
        n_chunks = cb[nb];
        stream_first_run[k] = (uint32_t)runs.size();
        host_runs_built = true;
    };
    const uint32_t n_runs = (uint32_t)job.run_ptr.size();
    if (runs_dev) {  // chunk count only (8 MB of lengths)
        const unsigned nb = par_nblocks(n_runs);
        std::vector<uint64_t> cb(nb, 0);
        par_run(n_runs, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
            uint64_t nc = 0;
            for (uint64_t r = lo; r < hi; ++r) nc += n_chunks_of(job.run_len[r]);
            cb[b] = nc;
        });
        for (uint64_t c : cb) n_chunks += c;
    } else {
        build_host_runs();
    }
    htrace("run table built");

    RunInfo* d_runs = dbuf<RunInfo>(ctx, "runs", n_runs);
    uint32_t* d_hdr = dbuf<uint32_t>(ctx, "hdr_err", n_runs);
    uint64_t* ch_start = dbuf<uint64_t>(ctx, "ch_start", n_chunks);
    uint64_t* ch_end = dbuf<uint64_t>(ctx, "ch_end", n_chunks);
    uint32_t* ch_cnt = dbuf<uint32_t>(ctx, "ch_cnt", n_chunks);
    uint32_t* ch_err = dbuf<uint32_t>(ctx, "ch_err", n_chunks);
    unsigned long long* bad_bits = dbuf<unsigned long long>(ctx, "bad_bits", n_chunks / 64 + 1);
    uint32_t* first_bad = dbuf<uint32_t>(ctx, "first_bad", n_runs);
    uint32_t* err_chunk = dbuf<uint32_t>(ctx, "err_chunk", n_runs);
    uint64_t* cnt64 = dbuf<uint64_t>(ctx, "cnt64", n_chunks);
    uint64_t* ch_rec_base = dbuf<uint64_t>(ctx, "ch_rec_base", n_chunks + 1);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, "scan_tmp", scan_tmp_words(std::max<uint64_t>(n_chunks, 1 << 20)) + 64);
    RunSummary* d_sum = dbuf<RunSummary>(ctx, "run_sum", n_runs);
    htrace("buffers");

    if (runs_dev) {
        uint64_t* d_ptr_in = dbuf<uint64_t>(ctx, "run_ptr_in", n_runs);
        uint64_t* d_len_in = dbuf<uint64_t>(ctx, "run_len_in", n_runs);
        uint64_t* d_nch = dbuf<uint64_t>(ctx, "run_nch", n_runs);
        uint64_t* d_cbase = dbuf<uint64_t>(ctx, "run_cbase", n_runs + 1);
        h2d_up(ctx, d_ptr_in, job.run_ptr.data(), (size_t)n_runs * 8);
        h2d_up(ctx, d_len_in, job.run_len.data(), (size_t)n_runs * 8);
        uint64_t* d_tmp = dbuf<uint64_t>(ctx, "run_info_scan", scan_tmp_words(n_runs) + 64);
        launch_run_info(st, d_ptr_in, d_len_in, n_runs, job.caller_order < 0, chunk, d_nch, d_cbase, d_tmp, d_runs);
    } else {
        h2d_up(ctx, d_runs, runs.data(), n_runs * sizeof(RunInfo));
    }
    htrace("runs uploaded");
    RunFmt* d_fmt = dbuf<RunFmt>(ctx, "run_fmt", n_runs);
    uint32_t* d_broken = dbuf<uint32_t>(ctx, "run_broken", n_runs);
    uint64_t* d_recb = dbuf<uint64_t>(ctx, "run_recb", n_runs + 1);
    HIPCHK(hipMemsetAsync(d_broken, 0, (size_t)n_runs * 4, st));
    launch_run_header(st, d_runs, n_runs, d_hdr, d_fmt, job.part);

    std::vector<RunSummary>& sum = ctx->s_sum;
    sum.resize(n_runs);  // every entry is written by whichever parse runs
    std::vector<uint64_t>& stream_base = ctx->s_sbase;
    std::vector<uint64_t>& stream_valid = ctx->s_svalid;
    std::vector<uint32_t>& stream_err = ctx->s_serr;
    stream_base.resize(k + 1);  // written by stream_tables() before any read
    stream_valid.resize(k);
    stream_err.resize(k);
    bool any_err = false;
    uint64_t R = 0;
    uint64_t* rec_addr = nullptr;
    uint64_t* rec_hi = nullptr;
    uint64_t* rec_lo = nullptr;
    uint32_t* rec_klen = nullptr;
    uint32_t* rec_meta = nullptr;
    uint64_t* rec_fp = nullptr;  // fingerprints of the key bytes past 16 (written by the emit kernels)
    uint32_t* utf8_bad = dbuf<uint32_t>(ctx, "utf8_bad", 1);
    uint32_t* d_flags = dbuf<uint32_t>(ctx, "flags", 4);
    uint64_t* d_stream_base = dbuf<uint64_t>(ctx, "stream_base", k + 1);
    unsigned long long* d_first_dec = dbuf<unsigned long long>(ctx, "first_dec", k);
    std::vector<uint64_t>& first_dec = ctx->s_first_dec;
    first_dec.resize(k);  // read back, or filled with ~0 on the deferred path
    bool dec_none = false;  // no stream has a decrease (flags[1] clear): first_dec not read back, all ~0
    uint32_t hflags[4];
    // per stream (rank order): base index, valid record count n_s and the first error
    auto stream_tables = [&]() {  // blocks of streams on host threads (10^6-stream calls)
        if (!host_runs_built) build_host_runs();  // (a device-built run table: its host copy, same content)
        const unsigned nb = par_nblocks(k);
        std::vector<uint8_t> blk_err(nb, 0);
        const uint64_t acc = par_scan(
            k,
            [&](uint64_t lo, uint64_t hi) {
                uint64_t a = 0;
                for (uint32_t r = stream_first_run[lo]; r < stream_first_run[hi]; ++r) a += sum[r].records;
                return a;
            },
            [&](unsigned b, uint64_t lo, uint64_t hi, uint64_t acc) {
                for (uint64_t s = lo; s < hi; ++s) {
                    stream_base[s] = acc;
                    uint64_t valid = 0;
                    bool dead = false;
                    stream_err[s] = 0;
                    for (uint32_t r = stream_first_run[s]; r < stream_first_run[s + 1]; ++r) {
                        acc += sum[r].records;
                        if (!dead) {
                            valid += sum[r].records;
                            if (sum[r].err) {
                                stream_err[s] = sum[r].err;
                                dead = true;
                                blk_err[b] = 1;
                            }
                        }
                    }
                    stream_valid[s] = valid;
                }
            });
        for (uint8_t e : blk_err) any_err = any_err || e;
        stream_base[k] = acc;
        if (acc != R) throw DevError("internal: record count mismatch");
    };
    // Wide fixed-stride calls (config 5: 10^6 one-run streams) keep their run and stream tables on
    // the device: record counts, flags and record bases come from k_run_tables + a scan, and the host
    // copies (sum, stream_base / _valid / _err) are read back only if an error path needs them
    // (materialize_tables). dev_tables: this call's tables live on the device only.
    bool dev_tables = false;
    // zeroed verdict words: record flags, the UTF-8 flag, each stream's first decrease (none)
    auto reset_verdict = [&]() {
        HIPCHK(hipMemsetAsync(d_flags, 0, 16, st));
        HIPCHK(hipMemsetAsync(utf8_bad, 0, 4, st));
        HIPCHK(hipMemsetAsync(d_first_dec, 0xFF, (size_t)k * 8, st));
    };
    auto alloc_records = [&]() {
        rec_addr = dbuf<uint64_t>(ctx, "rec_addr", R);
        rec_hi = dbuf<uint64_t>(ctx, "rec_hi", R);
        rec_lo = dbuf<uint64_t>(ctx, "rec_lo", R);
        rec_klen = dbuf<uint32_t>(ctx, "rec_klen", R);
        rec_meta = dbuf<uint32_t>(ctx, "rec_meta", R);
        rec_fp = dbuf<uint64_t>(ctx, "rec_fp", R);
        reset_verdict();
        if (dev_tables)  // one run per stream, rank order: stream bases are the run record bases
            HIPCHK(hipMemcpyAsync(d_stream_base, d_recb, (size_t)(k + 1) * 8, hipMemcpyDeviceToDevice, st));
        else
            h2d_up(ctx, d_stream_base, stream_base.data(), (k + 1) * 8);
    };
    auto materialize_tables = [&]() {  // the host tables of a dev_tables call (error paths only)
        if (!dev_tables) return;
        std::vector<uint64_t>& recb = ctx->s_recb;
        recb.resize(n_runs + 1);
        HIPCHK(hipMemcpy(recb.data(), d_recb, (size_t)(n_runs + 1) * 8, hipMemcpyDeviceToHost));
        for (uint32_t r = 0; r < n_runs; ++r) sum[r] = RunSummary{recb[r + 1] - recb[r], 0u, 0u};
        dev_tables = false;
        stream_tables();
    };
    uint32_t utf8_flag = 0;
    // order check + readback of its result, the record flags and (fast path) the broken-run flags
    // order: ORDER_LAUNCH runs k_order_check here; ORDER_DONE the parse did it (first decreases as
    // stream-local indices)
    enum { ORDER_LAUNCH = 0, ORDER_DONE = 1 };
    auto check_and_read = [&](bool read_broken, int order = ORDER_LAUNCH) -> bool {
        // the fast path's parse kernel already did the order check
        if (!read_broken && !job.batch && order == ORDER_LAUNCH)  // a writer batch is unsorted by definition
            launch_order_check(st, R, d_stream_base, k, rec_addr, rec_hi, rec_lo, rec_klen, d_first_dec, d_flags + 1);
        HIPCHK(hipGetLastError());
        // the verdict words first; the 10^6-entry tables only when a word says they hold something:
        // every writer of first_dec also sets flags[1], every broken run also flags[2]
        uint8_t* hp = (uint8_t*)pinned(ctx, 64);
        d2h(ctx, hp, d_flags, 16);
        d2h(ctx, hp + 16, utf8_bad, 4);
        sync(ctx);
        memcpy(hflags, hp, 16);
        memcpy(&utf8_flag, hp + 16, 4);
        const bool need_dec = hflags[1] != 0, need_broken = read_broken && hflags[2] != 0;
        dec_none = !need_dec;
        bool broken = false;
        if (need_dec || need_broken) {
            uint8_t* hq = (uint8_t*)pinned(ctx, (size_t)k * 8 + (size_t)n_runs * 4 + 16);
            if (need_dec) d2h(ctx, hq, d_first_dec, (size_t)k * 8);
            if (need_broken) d2h(ctx, hq + (size_t)k * 8, d_broken, (size_t)n_runs * 4);
            sync(ctx);
            if (need_dec) memcpy(first_dec.data(), hq, (size_t)k * 8);
            const uint32_t* b = (const uint32_t*)(hq + (size_t)k * 8);
            for (uint32_t r = 0; need_broken && r < n_runs && !broken; ++r) broken = b[r] != 0;
        }
        return broken;
    };

    // ---- fast path: every run fixed-stride (one record size per run) -> one verifying pass ------
    bool parsed = false, deferred = false;
    // The merge's choice between the splitter merge and the record sort (skv_sort.hip): past
    // TILE_TARGET / 2 streams the splitter table does not fit; SKV_SORT=1 forces the sort (tests).
    // Made where the fixed-stride parse decides whether to write key fingerprints, and kept: a parse
    // that skipped them (fp_skipped) commits the call to the sort, which merges on dense ranks -- the
    // splitter merge would read unwritten fingerprints (a scan's key filter can shrink R in between).
    const char* sort_env = test_opt("SKV_SORT");
    auto sort_by_fan_in = [&](uint64_t nrec) {
        return (k > (uint32_t)TILE_TARGET / 2 && nrec > (uint64_t)TILE_CAP) || (sort_env && sort_env[0] == '1') ||
               job.batch;
    };
    bool fp_skipped = false;
    bool e_direct = false;  // the fixed-stride parse wrote the record sort's elements (sort_e)
    bool any_fixed = false;  // some run is fixed-stride: the general parse also runs k_emit_fixed
    uint32_t uniform_meta = 0;  // every record a Put of one size (the fixed path's runs, one format): its meta
    // the device-table variant: past the splitter merge's fan-in (the fused path cannot apply), one
    // run per stream, a plain compaction or WAL flush (SKV_HOST_TABLES=1: the host tables always).
    // One run per STREAM, not n_runs == k: an empty stream beside a two-member stream also gives
    // n_runs == k, and the stream bases below are the run record bases.
    const bool try_dev_tables = k > (uint32_t)TILE_TARGET / 2 && n_runs == k && job.one_run_each && !job.scan && !job.search &&
                                !job.batch && !job.part;
    if (try_dev_tables) {
        uint64_t* d_cnt = dbuf<uint64_t>(ctx, "run_cnt", n_runs + 1);
        uint32_t* d_rfl = dbuf<uint32_t>(ctx, "run_tflags", 4);
        uint64_t* tmp = dbuf<uint64_t>(ctx, "run_scan_tmp", scan_tmp_words(n_runs) + 64);
        HIPCHK(hipMemsetAsync(d_rfl, 0, 16, st));
        launch_run_tables(st, d_runs, d_fmt, n_runs, d_cnt, d_rfl);
        launch_scan(st, d_cnt, n_runs, d_recb, tmp);  // d_recb[n_runs] = R
        uint8_t* hp = (uint8_t*)pinned(ctx, 64 + sizeof(RunFmt));
        d2h(ctx, hp, d_rfl, 16);
        d2h(ctx, hp + 16, d_recb + n_runs, 8);
        d2h(ctx, hp + 32, d_fmt, sizeof(RunFmt));
        sync(ctx);
        htrace("run tables on the device");
        uint32_t fl[4];
        memcpy(fl, hp, 16);
        const uint64_t Rd = *(const uint64_t*)(hp + 16);
        if (!fl[RT_NOT_FIXED] && Rd < 0xFFFFFFFFull) {  // every run fixed-stride: the parse below
            RunFmt f0;
            memcpy(&f0, hp + 32, sizeof f0);
            any_fixed = true;
            dev_tables = true;
            R = Rd;
            any_err = false;  // (the fixed-stride parse decodes every record or marks its run broken)
            alloc_records();
            const bool will_sort = sort_by_fan_in(R);
            fp_skipped = will_sort;
            // the record sort follows: the parse writes the sort's elements itself (no k_sort_load
            // pass; the record arrays are filled from them only if a key decrease needs them)
            e_direct = will_sort && !job.batch && !job.scan && !job.search;
            launch_parse_fixed(st, d_runs, n_runs, d_fmt, d_broken, d_recb, R, rec_addr, rec_hi, rec_lo, rec_klen,
                               rec_meta, d_flags, d_stream_base, d_first_dec, will_sort ? nullptr : rec_fp,
                               dbuf<uint32_t>(ctx, "wave_run", (R + 63) / 64 + 1),
                               e_direct ? dbuf<SElem>(ctx, "sort_e", R) : nullptr);
            mark(ctx, PH_PARSE);
            if (allow_deferred && !(job.flags & SKV_SPLIT_BY_TABLE)) {
                deferred = true;  // verdict read with the result
                parsed = true;
                std::fill(first_dec.begin(), first_dec.end(), ~0ull);
                memset(hflags, 0, sizeof hflags);
            } else {
                parsed = !check_and_read(true);
                htrace("parse verdict read");
            }
            if (parsed && !deferred && !fl[RT_NOT_UNIFORM] && !(hflags[3] & 1u)) uniform_meta = (uint32_t)f0.S;
            if (parsed && e_direct && !deferred && hflags[1]) {  // a decrease: its paths read the record arrays
                launch_sort_unload(st, R, dbuf<SElem>(ctx, "sort_e", R), rec_hi, rec_lo, rec_addr, rec_klen);
                e_direct = false;
            }
            if (!parsed) {  // a run is not what its first record promised: general parse, host tables
                dev_tables = false;
                fp_skipped = false;
                e_direct = false;
                R = 0;
                any_err = false;
                std::fill(stream_err.begin(), stream_err.end(), 0u);
            }
        } else {
            any_fixed = fl[RT_ANY_FIXED] != 0;  // the general parse also runs k_emit_fixed then
        }
    }
    if (!try_dev_tables) {
        RunFmt* hf = (RunFmt*)pinned(ctx, (size_t)n_runs * sizeof(RunFmt) + 16);
        d2h(ctx, hf, d_fmt, (size_t)n_runs * sizeof(RunFmt));
        htrace("header launched");
        sync(ctx);
        htrace("header synced");
        htrace("run formats read");
        // blocks of runs on host threads: every run fixed-stride? one format everywhere?
        const unsigned nbr = par_nblocks(n_runs);
        std::vector<uint8_t> blk_fixed(nbr, 1), blk_uni(nbr, 1), blk_any(nbr, 0);
        par_run(n_runs, nbr, [&](unsigned b, uint64_t lo, uint64_t hi) {
            bool fx = true, un = true, an = false;
            for (uint64_t r = lo; r < hi; ++r) {
                fx = fx && hf[r].S != 0;
                an = an || hf[r].S != 0;
                un = un && hf[r].S == hf[0].S && hf[r].K == hf[0].K;
            }
            blk_fixed[b] = fx;
            blk_uni[b] = un;
            blk_any[b] = an;
        });
        bool all_fixed = n_runs > 0, uniform = true;
        for (unsigned b = 0; b < nbr; ++b) {
            all_fixed = all_fixed && blk_fixed[b];
            uniform = uniform && blk_uni[b];
            any_fixed = any_fixed || blk_any[b];
        }
        if (all_fixed) {
            std::vector<uint64_t>& recb = ctx->s_recb;
            recb.resize(n_runs + 1);
            recb[0] = 0;
            R = par_scan(
                n_runs,
                [&](uint64_t lo, uint64_t hi) {
                    uint64_t a = 0;
                    for (uint64_t r = lo; r < hi; ++r) a += (runs[r].len - 1) / hf[r].S;
                    return a;
                },
                [&](unsigned, uint64_t lo, uint64_t hi, uint64_t acc) {
                    for (uint64_t r = lo; r < hi; ++r) {
                        sum[r].records = (runs[r].len - 1) / hf[r].S;
                        sum[r].err = 0;
                        sum[r].pad = 0;
                        acc += sum[r].records;
                        recb[r + 1] = acc;
                    }
                });
            // one record size and one key length <= 16 everywhere: the fused stride path
            const RunFmt f0 = hf[0];
            const char* fenv = test_opt("SKV_FUSED");
            if (allow_deferred && uniform && !job.batch && !job.search && !job.scan && !job.part &&
                !(job.flags & SKV_SPLIT_BY_TABLE) &&
                !(fenv && fenv[0] == '0') &&
                f0.K <= FX_MAX_K && f0.S >= FX_MIN_S && f0.S <= FX_MAX_S && k <= (uint32_t)TILE_TARGET / 2 &&
                R < 0xFFFFFFFFull) {
                if (compact_fused(ctx, job, runs, d_runs, stream_first_run, f0, recb, out)) return SKV_OK;
                return compact_device(ctx, job, out, false);
            }
            stream_tables();
            alloc_records();
            htrace("record tables");
            h2d_up(ctx, d_recb, recb.data(), (n_runs + 1) * 8);
            // the record sort merges on dense key ranks: no key fingerprints to compute then
            const bool will_sort = sort_by_fan_in(R);
            fp_skipped = will_sort;  // then the merge below must take the record sort whatever R becomes
            launch_parse_fixed(st, d_runs, n_runs, d_fmt, d_broken, d_recb, R, rec_addr, rec_hi, rec_lo, rec_klen,
                               rec_meta, d_flags, d_stream_base, job.batch ? nullptr : d_first_dec,
                               will_sort ? nullptr : rec_fp, dbuf<uint32_t>(ctx, "wave_run", (R + 63) / 64 + 1));
            mark(ctx, PH_PARSE);
            if (allow_deferred && !(job.flags & SKV_SPLIT_BY_TABLE) && !job.search && !job.scan) {
                deferred = true;  // verdict read with the result
                parsed = true;
                std::fill(first_dec.begin(), first_dec.end(), ~0ull);
                memset(hflags, 0, sizeof hflags);
            } else {
                parsed = !check_and_read(true);
                htrace("parse verdict read");
            }
            // one size everywhere and no Delete among the records (read with the verdict): one meta
            if (parsed && !deferred && uniform && !(hflags[3] & 1u)) uniform_meta = (uint32_t)f0.S;
            if (!parsed) {  // a run is not what its first record promised: general parse
                fp_skipped = false;  // (the general parse writes every fingerprint)
                R = 0;
                any_err = false;
                std::fill(stream_err.begin(), stream_err.end(), 0u);
            }
        }
    }
    // ---- general path: speculative chunk walks ----------------------------------------------
    if (!parsed) {
        // record starts of each chunk as the walks find them (16-bit offsets), chunk / 64 per chunk:
        // k_emit parses the records of a chunk in parallel instead of walking its chain again
        const uint32_t slot_cap = (uint32_t)((chunk / 64 + 7) & ~7ull);  // rows of 16-byte groups (walk_fast)
        uint16_t* ch_slots = dbuf<uint16_t>(ctx, "ch_slots", n_chunks * slot_cap);
        // the walks' staged record arrays (32 bytes per record, chunk / 128 per chunk: a chunk of
        // shorter records is emitted from the records as before)
        const uint32_t stg_cap = (uint32_t)((chunk / 128 + 7) & ~7ull);
        StgRec* ch_stg_rec = dbuf<StgRec>(ctx, "ch_stg_rec", (n_chunks + STG_W - 1) / STG_W * STG_W * stg_cap);
        uint8_t* ch_stg = dbuf<uint8_t>(ctx, "ch_stg", n_chunks);
        HIPCHK(hipMemsetAsync(bad_bits, 0, (n_chunks / 64 + 1) * 8, st));
        HIPCHK(hipMemsetAsync(first_bad, 0xFF, n_runs * 4, st));
        HIPCHK(hipMemsetAsync(err_chunk, 0xFF, n_runs * 4, st));
        launch_spec(st, d_runs, n_runs, n_chunks, d_hdr, d_fmt, d_broken, ch_start, ch_end, ch_cnt, ch_err,
                    ctx->exact_utf8, chunk, ch_slots, slot_cap, ch_stg_rec, stg_cap, ch_stg);
        launch_validate(st, d_runs, n_runs, n_chunks, d_hdr, ch_start, ch_end, ch_err, bad_bits, first_bad);
        launch_fixup(st, d_runs, n_runs, d_hdr, first_bad, bad_bits, ch_start, ch_end, ch_cnt, ch_err,
                     ctx->exact_utf8, chunk, ch_slots, slot_cap, ch_stg);
        launch_err_chunk(st, d_runs, n_runs, n_chunks, d_hdr, ch_err, err_chunk);
        launch_mask(st, d_runs, n_runs, n_chunks, d_hdr, err_chunk, ch_cnt, cnt64);
        launch_scan(st, cnt64, n_chunks, ch_rec_base, scan_tmp);
        launch_run_summary(st, d_runs, n_runs, d_hdr, err_chunk, ch_err, ch_rec_base, d_sum, d_recb);
        HIPCHK(hipGetLastError());
        {
            RunSummary* hs = (RunSummary*)pinned(ctx, n_runs * sizeof(RunSummary) + 16);
            d2h(ctx, hs, d_sum, n_runs * sizeof(RunSummary));
            d2h(ctx, (uint8_t*)hs + n_runs * sizeof(RunSummary), ch_rec_base + n_chunks, 8);
            sync(ctx);
            memcpy(sum.data(), hs, n_runs * sizeof(RunSummary));
            memcpy(&R, (uint8_t*)hs + n_runs * sizeof(RunSummary), 8);
        }
        stream_tables();
        alloc_records();
        // the order check fused into k_emit (+ k_chunk_order at chunk edges) when every record comes from
        // it (fixed-stride runs' records, from k_emit_fixed<false>, are not checked there; a writer batch is
        // unsorted by definition)
        const bool emit_order = !any_fixed && !job.batch;
        launch_emit(st, d_runs, n_runs, n_chunks, d_fmt, d_broken, ch_start, ch_rec_base, d_recb, any_fixed ? R : 0,
                    rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_flags, rec_fp, utf8_bad, ch_slots, slot_cap, chunk,
                    ch_end, emit_order ? d_stream_base : nullptr, emit_order ? d_first_dec : nullptr, ch_stg_rec,
                    stg_cap, ch_stg, R, dbuf<uint32_t>(ctx, "blk_chunk", R / 64 + 1 + n_chunks));
        mark(ctx, PH_PARSE);
        check_and_read(false, emit_order ? ORDER_DONE : ORDER_LAUNCH);
        if (utf8_flag && !ctx->exact_utf8) {  // a key the chunk walks did not check: exact walks
            ctx->exact_utf8 = true;
            int rc;
            try {
                rc = compact_device(ctx, job, out, false);
            } catch (...) {
                ctx->exact_utf8 = false;
                throw;
            }
            ctx->exact_utf8 = false;
            return rc;
        }
    }
    mark(ctx, PH_CHECK);
    htrace("check done");
    tables_mine();
    if (dec_none && (any_err || job.search)) std::fill(first_dec.begin(), first_dec.end(), ~0ull);  // (rare paths read it)
    if (job.search) return search_stage(ctx, job, runs[0], R, stream_err[0], first_dec[0], rec_addr, rec_hi, rec_lo,
                                        rec_klen, rec_meta);
    bool any_dec = false;
    for (uint32_t s = 0; !dec_none && s < k; ++s)
        if (first_dec[s] != ~0ull) {
            materialize_tables();
            if (first_dec[s] + 1 < stream_valid[s]) any_dec = true;
        }
    // A key-range part of a pipelined host call (skv_hostpipe.hip) holds the slices a cut by key
    // gave: with a decode error or a key decrease in a slice, the cut itself is not a key range and
    // the reference's outcome depends on the whole call's pop order (heap-order mode, error order).
    // The part ends the attempt; the serial path gives the exact outcome.
    if (job.part && (any_err || any_dec)) throw ApiError{SKV_E_FORMAT, "part: error or decrease in a slice"};

    // ---- ScanFromRun (skv_scan_host.hip): the per-run key filter (cache_service.rs:125-129) on the
    // record arrays, before the merge; a run's decode error surfaces after the pop of its last kept
    // record, or, with none, at the merge's first pulls in vector order (k_way.rs:126-140) -- the
    // first such run's error ends the scan before any item
    std::vector<ScanEvent> scan_ev;
    uint8_t* d_start = nullptr;
    if (job.scan) {
        const uint32_t slen = (uint32_t)job.scan_start.size();
        d_start = dbuf<uint8_t>(ctx, "scan_start", slen + 32);  // + the aligned blocks key_cmp may read
        HIPCHK(hipMemsetAsync(d_start, 0, slen + 32, st));
        if (slen) h2d_up(ctx, d_start, job.scan_start.data(), slen);
        std::vector<ScanEvent> errs;  // read_run_iter's text needs the failing record's offset (unfiltered arrays)
        for (uint32_t s = 0; s < k; ++s) {
            if (!stream_err[s]) continue;
            const RunInfo& run = runs[stream_first_run[s]];  // one run per stream
            uint64_t err_off = 1;
            if (stream_valid[s]) {
                const uint64_t last = stream_base[s] + stream_valid[s] - 1;
                err_off = read_dev(rec_addr + last) + (read_dev(rec_meta + last) & 0x7FFFFFFFu) - run.ptr;
            }
            ScanEvent e{s, 0, 0, std::string()};
            e.code = scan_err_to_api(stream_err[s], err_off, run.len, e.msg);
            errs.push_back(e);
        }
        uint64_t* keep = dbuf<uint64_t>(ctx, "scf_keep", R + 1);
        uint64_t* keepx = dbuf<uint64_t>(ctx, "scf_keepx", R + 1);
        uint64_t* ftmp = dbuf<uint64_t>(ctx, "scf_scan_tmp", scan_tmp_words(R + 1) + 64);
        uint64_t* f_addr = dbuf<uint64_t>(ctx, "scf_addr", R);
        uint64_t* f_hi = dbuf<uint64_t>(ctx, "scf_hi", R);
        uint64_t* f_lo = dbuf<uint64_t>(ctx, "scf_lo", R);
        uint32_t* f_klen = dbuf<uint32_t>(ctx, "scf_klen", R);
        uint32_t* f_meta = dbuf<uint32_t>(ctx, "scf_meta", R);
        uint64_t* f_base = dbuf<uint64_t>(ctx, "scf_base", k + 1);
        launch_scan_filter(st, R, k, d_stream_base, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_start, slen, keep,
                           keepx, ftmp, f_addr, f_hi, f_lo, f_klen, f_meta, f_base);
        HIPCHK(hipGetLastError());
        uint8_t* hp = (uint8_t*)pinned(ctx, (size_t)(k + 1) * 8 + 16);
        d2h(ctx, hp, f_base, (size_t)(k + 1) * 8);
        sync(ctx);
        memcpy(stream_base.data(), hp, (size_t)(k + 1) * 8);
        HIPCHK(hipMemcpyAsync(d_stream_base, f_base, (size_t)(k + 1) * 8, hipMemcpyDeviceToDevice, st));
        rec_addr = f_addr;
        rec_hi = f_hi;
        rec_lo = f_lo;
        rec_klen = f_klen;
        rec_meta = f_meta;
        R = stream_base[k];
        int64_t first_v = -1;
        const ScanEvent* first_pull = nullptr;
        for (const ScanEvent& e : errs) {
            const uint64_t kept = stream_base[e.s + 1] - stream_base[e.s];
            if (kept) {
                scan_ev.push_back(e);
                scan_ev.back().after_rec = stream_base[e.s + 1] - 1;  // filtered numbering
            } else if (first_v < 0 || job.ranked[e.s].vec_idx < (uint32_t)first_v) {
                first_v = job.ranked[e.s].vec_idx;
                first_pull = &e;
            }
        }
        if (first_pull) throw ApiError{first_pull->code, first_pull->msg};
    }

    // ---- errors: which one k_way::merge surfaces first --------------------------------------
    // Heap-order mode (skv_heap.hip) where the outcome depends on the merge's exact pop sequence
    // past a stream's first key decrease or decode error: the WAL split with either, and the Delete
    // filter with a decrease. Everywhere else the first trigger record decides (below).
    const bool wal = (job.flags & SKV_SPLIT_BY_TABLE) != 0;
    const bool heap = !job.batch && ((wal && (any_err || any_dec)) || ((job.flags & SKV_DROP_TOMBSTONES) && any_dec) ||
                                     (job.scan && (any_err || any_dec)));
    HeapRes hres;
    if (any_err || any_dec) materialize_tables();
    if ((any_err || any_dec) && !job.scan) {  // (the scan resolved its first pulls above)
        // (1) first items are pulled in the caller's vector order (k_way.rs:126-140)
        std::vector<uint32_t> by_vec(k);
        for (uint32_t s = 0; s < k; ++s) by_vec[job.ranked[s].vec_idx] = s;
        for (uint32_t v = 0; v < k; ++v) {
            uint32_t s = by_vec[v];
            if (stream_valid[s] == 0 && stream_err[s]) {
                std::string msg;
                int code = derr_to_api(stream_err[s], msg);
                throw ApiError{code, msg};
            }
        }
        if (heap) {
            for (uint32_t s = 0; s < k; ++s)
                if (stream_err[s]) hres.dec.push_back({stream_base[s] + stream_valid[s] - 1, stream_err[s]});
        }
    }
    if ((any_err || any_dec) && !heap) {
        // (2) each stream's earliest trigger item; the one popped first wins
        struct Cand { uint32_t s; uint64_t idx; bool order; std::string key; };
        std::vector<Cand> cands;
        bool any_order = false;
        for (uint32_t s = 0; s < k; ++s) {
            uint64_t trig = ~0ull;
            bool order = false;
            if (first_dec[s] != ~0ull && first_dec[s] + 1 < stream_valid[s]) { trig = first_dec[s]; order = true; }
            if (stream_err[s] && stream_valid[s] > 0) {
                uint64_t t2 = stream_valid[s] - 1;
                if (t2 < trig) { trig = t2; order = false; }
            }
            if (trig == ~0ull) continue;
            any_order |= order;
            cands.push_back({s, trig, order, fetch_key(ctx, rec_addr, rec_klen, stream_base[s] + trig)});
        }
        if (cands.empty()) throw DevError("internal: error without trigger");
        // pop order: key ascending, then seq_no descending (== smaller rank)
        std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) {
            if (a.key != b.key) return a.key < b.key;
            return a.s < b.s;
        });
        const Cand& w = cands[0];
        (void)any_order;
        if (w.order) throw ApiError{SKV_E_FORMAT, "Data format error: Operations must be sorted by key"};
        std::string msg;
        int code = derr_to_api(stream_err[w.s], msg);
        throw ApiError{code, msg};
    }
    if (hflags[0]) throw ApiError{SKV_E_UNSUPPORTED, "record of 2 GiB or more: unsupported by this build"};
    if (R == 0) {  // nothing survives: build_runs yields no run (runs.rs:270-271)
        ResultBox* box = new ResultBox();
        box->pub.runs = (skv_run_desc*)malloc(sizeof(skv_run_desc));
        box->pub.bytes = dbuf<uint8_t>(ctx, "out", 16);
        box->pub.in_bytes = job.in_bytes;
        mark(ctx, PH_MERGE);
        mark(ctx, PH_CHAIN);
        mark(ctx, PH_GATHER);
        ctx->timings = skv_timings{};
        ctx->timings.host_syncs = ctx->syncs;
        *out = &box->pub;
        return SKV_OK;
    }
    if (R >= 0xFFFFFFFFull) throw ApiError{SKV_E_UNSUPPORTED, "more than 2^32-1 records in one compaction"};

    // ---- merge ------------------------------------------------------------------------------
    struct Level {
        uint64_t N = 0, S = 1;
        std::vector<uint64_t> off;  // k+1 list offsets
        uint64_t* hi = nullptr;
        uint64_t* lo = nullptr;
        uint64_t* c = nullptr;       // level > 0
        uint64_t* d_off = nullptr;
        // sorted output (level > 0)
        uint64_t* shi = nullptr;
        uint64_t* slo = nullptr;
        uint64_t* sc = nullptr;
    };
    // Past TILE_TARGET / 2 streams the records are sorted into one list first (skv_sort.hip);
    // SKV_SORT=1 forces that path (tests).
    uint32_t km = k;  // lists the splitter merge sees
    const uint32_t* cmp_klen = rec_klen;  // key lengths the merge compares (dense ranks: 0)
    // the keys the merge orders by: the records' own, or (heap-order mode with a key decrease) each
    // record's stream-prefix-maximum record's (skv_heap.hip)
    uint64_t* cmp_hi = rec_hi;
    uint64_t* cmp_lo = rec_lo;
    const uint64_t* cmp_addr = rec_addr;
    uint64_t* pop_pos = nullptr;
    if (heap) {
        // the fixed-stride parse poisons the merge on a key decrease (k_emit_fixed); here the
        // decrease is what this mode merges exactly (broken runs never get this far: they reparse)
        HIPCHK(hipMemsetAsync(d_flags + 2, 0, 4, st));
        pop_pos = dbuf<uint64_t>(ctx, "heap_pop_pos", R);
        // always the prefix-maximum keys: a stream may be unsorted past its decode error (records of
        // later member runs), which any_dec does not see, and those records are merged too
        {
            uint32_t* eff = dbuf<uint32_t>(ctx, "heap_eff", R);
            uint64_t* blk = dbuf<uint64_t>(ctx, "heap_blk", heap_key_blocks(R));
            uint32_t* carry = dbuf<uint32_t>(ctx, "heap_carry", heap_key_blocks(R));
            uint64_t* ehi = dbuf<uint64_t>(ctx, "heap_hi", R);
            uint64_t* elo = dbuf<uint64_t>(ctx, "heap_lo", R);
            uint32_t* ekl = dbuf<uint32_t>(ctx, "heap_klen", R);
            uint64_t* ead = dbuf<uint64_t>(ctx, "heap_addr", R);
            launch_heap_keys(st, R, d_stream_base, k, rec_hi, rec_lo, rec_klen, rec_addr, eff, blk, carry, ehi, elo, ekl,
                             ead);
            cmp_hi = ehi;
            cmp_lo = elo;
            cmp_klen = ekl;
            cmp_addr = ead;
        }
    }
    const bool sorting = sort_by_fan_in(R) || fp_skipped;
    bool sorted_merged = false;     // the sort emitted the merged arrays (no level-0 merge tiles)
    uint64_t* sorted_K = nullptr;   // then: the survivor count, on the device
    const SElem* sorted_S = nullptr;  // then: the sorted elements, true key prefixes (WAL table ids)
    if (!sorting) materialize_tables();  // the splitter merge's list offsets are the stream bases
    std::vector<uint64_t> list_off = sorting ? std::vector<uint64_t>{0, R} : stream_base;  // (no 10^6-entry copy)
    uint64_t* d_list_off = d_stream_base;
    {
        if (sorting) {
            if (heap) {
                // sort on the merge keys; the records' own keys, payload and meta follow in sorted
                // order, and inv maps an original record index to its sorted position
                uint64_t *h2 = cmp_hi, *l2 = cmp_lo, *a2 = (uint64_t*)cmp_addr;
                uint32_t* k2 = (uint32_t*)cmp_klen;
                uint32_t* m2 = rec_meta;
                const uint32_t* ck = nullptr;
                const SElem* S = nullptr;
                sort_records(ctx, R, h2, l2, a2, k2, m2, ck, false, &S, 0);
                uint64_t* shi = dbuf<uint64_t>(ctx, "heap_s_hi", R);
                uint64_t* slo = dbuf<uint64_t>(ctx, "heap_s_lo", R);
                uint32_t* skl = dbuf<uint32_t>(ctx, "heap_s_klen", R);
                uint64_t* sad = dbuf<uint64_t>(ctx, "heap_s_addr", R);
                uint32_t* inv = dbuf<uint32_t>(ctx, "heap_inv", R);
                launch_heap_sorted(st, R, S, rec_hi, rec_lo, rec_klen, rec_addr, shi, slo, skl, sad, inv);
                rec_hi = shi;
                rec_lo = slo;
                rec_klen = skl;
                rec_addr = sad;
                rec_meta = m2;
                cmp_hi = h2;
                cmp_lo = l2;
                cmp_addr = a2;
                cmp_klen = ck;
                hres.inv = inv;
            } else {
                // Without the Delete filter (and outside writer batches and scans) the survivors of the
                // one sorted list are the first record of each key: the sort's store emits the merged
                // arrays itself and the level-0 merge tiles are skipped
                const bool direct = !(job.flags & SKV_DROP_TOMBSTONES) && !job.batch && !job.scan;
                SortMerged M{};
                if (direct) {
                    M.m_rec = dbuf<uint32_t>(ctx, "m_rec", R + 1);
                    M.m_src = dbuf<uint64_t>(ctx, "m_src", R + 1);
                    M.size = dbuf<uint64_t>(ctx, "sm_size", R + 1);
                    M.del = dbuf<uint64_t>(ctx, "sm_del", R + 1);
                    M.mm = dbuf<uint32_t>(ctx, "tile_mm", 2 * std::max<uint64_t>(1, sort_store_blocks(R)));
                    // the WAL stage reads the merged arrays only (its error text fetches keys through
                    // m_src): no sorted record arrays
                    M.arrays = !(job.flags & SKV_SPLIT_BY_TABLE);
                }
                sort_records(ctx, R, rec_hi, rec_lo, rec_addr, rec_klen, rec_meta, cmp_klen, job.batch,
                             direct ? &sorted_S : nullptr, uniform_meta, direct ? &M : nullptr,
                             direct ? &sorted_K : nullptr, e_direct);
                sorted_merged = direct;
                cmp_hi = rec_hi;
                cmp_lo = rec_lo;
                cmp_addr = rec_addr;
            }
            htrace("sort launched");
            if (getenv("SKV_SORT_PROF_PRINT")) {  // (SKV_SORT_PROF=1 builds; zeros otherwise)
                unsigned long long pr[16];
                sort_prof_read(pr);
                fprintf(stderr, "[sort prof] bucket: load %llu top %llu group %llu slot+store %llu | tile: load %llu "
                                "bitonic %llu ties %llu out %llu | tiles %llu (100 MHz ticks, cumulative) | tie runs %llu "
                                "tie elements %llu long %llu record words %llu global %llu\n",
                        pr[0], pr[1], pr[2], pr[3], pr[4], pr[5], pr[6], pr[7], pr[15], pr[8], pr[9], pr[10], pr[11],
                        pr[12]);
            }
            km = 1;
            list_off = {0, R};
            d_list_off = dbuf<uint64_t>(ctx, "sorted_off", 2);
            h2d_up(ctx, d_list_off, list_off.data(), 16);
            ctx->timings.sorted = 1;
        }
    }
    std::vector<Level> lv(1);
    if (sorted_merged) lv[0].N = 0;  // (no sample levels: nothing below is merged again)
    else lv[0].N = R;
    lv[0].off = list_off;
    lv[0].hi = cmp_hi;
    lv[0].lo = cmp_lo;
    lv[0].d_off = d_list_off;
    const uint64_t S_step = std::max<uint64_t>(2, (uint64_t)TILE_TARGET / std::max<uint32_t>(km, 1));
    // SKV_HI_STEP=f: levels >= 2 (they only pick splitters for the sample sorts) at an f times
    // coarser step. Measured at config 3 with f = 2: one sample level fewer, but the merge phase
    // 4.02 vs 3.26 ms (the level-1 sample tiles lose their balance), so the default is 1.
    const char* hse = test_opt("SKV_HI_STEP");
    const uint64_t hi_f = hse ? std::max<uint64_t>(1, strtoull(hse, nullptr, 10)) : 1;
    // Level 1 (the level-0 tiles' splitters) at twice the step from 128 lists on: a tile's size
    // spreads by ~sqrt(k) x step / 2.4 records around TILE_TARGET, which at k >= 128 stays under
    // 1/4.6 of the TILE_CAP margin, and half the samples halve their sort (3F merge 27.3 -> 25.7 ms,
    // config 3 2.22 -> 1.92 ms; a step of 3 unbalanced the tiles: 31.4 ms).
    const uint64_t l1_f = km >= 128 ? 2 : 1;
    while (lv.back().N > (uint64_t)TILE_CAP) {
        const Level& P = lv.back();
        Level L;
        L.S = lv.size() >= 2 ? S_step * hi_f : S_step * l1_f;
        L.off.resize(km + 1);
        uint64_t acc = 0;
        for (uint32_t j = 0; j < km; ++j) {
            L.off[j] = acc;
            uint64_t nj = P.off[j + 1] - P.off[j];
            acc += (nj + L.S - 1) / L.S;
        }
        L.off[km] = acc;
        L.N = acc;
        char nm[64];
        int li = (int)lv.size();
        snprintf(nm, sizeof nm, "lv%d_hi", li); L.hi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_lo", li); L.lo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_c", li); L.c = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_off", li); L.d_off = dbuf<uint64_t>(ctx, nm, km + 1);
        h2d_up(ctx, L.d_off, L.off.data(), (km + 1) * 8);
        launch_sample(st, li == 1, P.hi, P.lo, P.c, cmp_klen, P.d_off, L.d_off, km, L.S, L.N, L.hi, L.lo, L.c);
        lv.push_back(L);
    }
    // top-down: sort each sample level, derive splitters for the level below
    uint64_t T0 = 1;
    uint32_t* m_rec = dbuf<uint32_t>(ctx, "m_rec", R + 1);
    uint64_t* m_src = dbuf<uint64_t>(ctx, "m_src", R + 1);
    uint64_t* m_P = dbuf<uint64_t>(ctx, "m_P", R + 1);
    uint64_t* m_Dp = dbuf<uint64_t>(ctx, "m_Dp", R + 1);
    uint64_t* d_Kout = dbuf<uint64_t>(ctx, "K_out", 1);
    uint32_t* tile_max = nullptr;
    // fingerprints of the key bytes past 16 for the level-0 merge rounds (SKV_FP_TEST=1: all zero,
    // so every same-length key pair with one prefix is taken as equal and the exact check must catch it)
    const uint64_t* key_fp = nullptr;
    uint32_t* fp_bad = dbuf<uint32_t>(ctx, "fp_bad", 1);
    HIPCHK(hipMemsetAsync(fp_bad, 0, 4, st));
    // k_fp_verify's inputs once the level-0 tiles are queued; it runs on the ctx stream before the
    // WAL stage, or on the aux stream beside the gather (its verdict is read with the result)
    std::pair<const unsigned long long*, const uint64_t*> verify_args{nullptr, nullptr};
    // in-gather verify of the pairs whose first record survives (TileOut::m_dup): when k_gather is the
    // output stage and no Delete filter runs (a dropped Delete survivor has no output record to check
    // against). SKV_FP_GATHER=0: every pair goes to k_fp_verify.
    uint64_t* m_dup = nullptr;
    const unsigned long long* verify_lo = nullptr;  // pairs before it verified beside the merge
    bool verify_pending = false;
    if (km > 1 && !ctx->exact_keys && !heap && !job.scan) {  // (the scan's filtered arrays carry no fingerprints)
        const char* te = test_opt("SKV_FP_TEST");
        if (te && te[0] == '1') {
            uint64_t* f = dbuf<uint64_t>(ctx, "rec_fp_test", R);
            HIPCHK(hipMemsetAsync(f, 0, R * 8, st));
            key_fp = f;
        } else {
            key_fp = rec_fp;  // written by the emit kernels with the record arrays
        }
        const char* ge = test_opt("SKV_FP_GATHER");
        if (!(ge && ge[0] == '0') && !(job.flags & (SKV_SPLIT_BY_TABLE | SKV_DROP_TOMBSTONES)))
            m_dup = dbuf<uint64_t>(ctx, "m_dup", R + 1);
    }
    if (sorted_merged) {  // m_P / m_Dp: exclusive scans of the survivors' sizes / Delete bits
        uint64_t* tmp = dbuf<uint64_t>(ctx, "sm_scan_tmp", scan_tmp_words(R + 1) + 64);
        launch_scan_dn(st, dbuf<uint64_t>(ctx, "sm_size", R + 1), sorted_K, R, m_P, tmp);
        launch_scan_dn(st, dbuf<uint64_t>(ctx, "sm_del", R + 1), sorted_K, R, m_Dp, tmp);
        HIPCHK(hipMemcpyAsync(d_Kout, sorted_K, 8, hipMemcpyDeviceToDevice, st));
        // one (min, max) pair per k_sort_store block, reduced to SORT_MM_OUT pairs for the split
        tile_max = dbuf<uint32_t>(ctx, "tile_mm2", 2 * SORT_MM_OUT);
        launch_sort_mm_reduce(st, dbuf<uint32_t>(ctx, "tile_mm", 2 * std::max<uint64_t>(1, sort_store_blocks(R))),
                              sort_store_blocks(R), tile_max);
        T0 = SORT_MM_OUT;
    }
    for (int li = sorted_merged ? -1 : (int)lv.size() - 1; li >= 0; --li) {
        Level& L = lv[li];
        const bool l0 = li == 0;
        uint64_t T = 1, m = 1;
        if (li + 1 < (int)lv.size()) {
            m = std::max<uint64_t>(1, (uint64_t)TILE_TARGET / lv[li + 1].S);
            T = std::max<uint64_t>(1, (lv[li + 1].N + m - 1) / m);
        }
        char nm[64];
        snprintf(nm, sizeof nm, "bounds%d", li);
        uint64_t* bounds = dbuf<uint64_t>(ctx, nm, (T + 1) * km);
        const Level* U = li + 1 < (int)lv.size() ? &lv[li + 1] : nullptr;
        L1Cnt C{};
        if (l0 && U && T > 1) {  // level 0: each search starts inside one level-1 sample gap
            uint32_t* posof = dbuf<uint32_t>(ctx, "l1_posof", U->N);
            uint32_t* cnt = dbuf<uint32_t>(ctx, "l1_cnt", (T + 1) * km);
            launch_l1_cnt(st, U->sc, U->N, L.d_off, U->d_off, km, U->S, m, T, posof, cnt);
            C = L1Cnt{cnt, U->d_off, U->hi, U->lo, U->c, U->S};
        }
        launch_bounds(st, l0, L.hi, L.lo, L.c, cmp_klen, L.d_off, km, U ? U->shi : nullptr, U ? U->slo : nullptr,
                      U ? U->sc : nullptr, m, T, cmp_addr, bounds, d_flags + 2, C.cnt ? &C : nullptr);
        snprintf(nm, sizeof nm, "tile_n%d", li);
        uint64_t* tile_n = dbuf<uint64_t>(ctx, nm, T);
        snprintf(nm, sizeof nm, "tile_base%d", li);
        uint64_t* tile_base = dbuf<uint64_t>(ctx, nm, T + 1);
        launch_tile_n(st, bounds, km, T, tile_n);
        launch_scan(st, tile_n, T, tile_base, scan_tmp);
        TileOut O{};
        snprintf(nm, sizeof nm, "x%d_hi", li); O.xhi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "x%d_lo", li); O.xlo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "x%d_c", li); O.xc = dbuf<uint64_t>(ctx, nm, L.N);
        if (l0) {
            O.xmeta = dbuf<uint32_t>(ctx, "x0_meta", L.N);
            O.m_rec = m_rec;
            O.m_src = m_src;
            O.m_P = m_P;
            O.m_Dp = m_Dp;
            O.Kout = d_Kout;
            O.T = T;
            tile_max = O.tile_mm = dbuf<uint32_t>(ctx, "tile_mm", 2 * T);  // (min, max) record size per tile
            O.key_fp = key_fp;
            O.fp_bad = fp_bad;
            O.m_dup = m_dup;
            if (key_fp) {  // pairs taken as equal by fingerprint, verified after the tiles
                O.vpairs = dbuf<uint64_t>(ctx, "fp_vpairs", 2 * R);
                O.vcount = dbuf<unsigned long long>(ctx, "fp_vcount", 1);
                HIPCHK(hipMemsetAsync(O.vcount, 0, 8, st));
            }
            O.tstate = dbuf<uint64_t>(ctx, "tile_state", 3 * T);
            O.tcounter = dbuf<uint32_t>(ctx, "tile_ticket", 1);
            if (heap) {
                O.pay_addr = rec_addr;
                O.act_hi = rec_hi;
                O.act_lo = rec_lo;
                O.act_klen = rec_klen;
                O.pop_pos = pop_pos;
            }
            HIPCHK(hipMemsetAsync(O.tstate, 0, 3 * T * 8, st));
            HIPCHK(hipMemsetAsync(O.tcounter, 0, 4, st));
#if SKV_TILE_PROF
            O.prof = dbuf<uint64_t>(ctx, "tile_prof", 16);
            if (!ctx->prof_init) {
                HIPCHK(hipMemsetAsync(O.prof, 0, 128, st));
                ctx->prof_init = true;
            }
#endif
        } else {
            snprintf(nm, sizeof nm, "s%d_hi", li); L.shi = O.ohi = dbuf<uint64_t>(ctx, nm, L.N);
            snprintf(nm, sizeof nm, "s%d_lo", li); L.slo = O.olo = dbuf<uint64_t>(ctx, nm, L.N);
            snprintf(nm, sizeof nm, "s%d_c", li); L.sc = O.oc = dbuf<uint64_t>(ctx, nm, L.N);
        }
        const uint32_t drop = (job.flags & SKV_DROP_TOMBSTONES) ? 1u : 0u;
        // (round 4-5 also split level 0 into pieces whose pairs k_fp_verify checked beside the next
        // piece's merge: measured neutral at 3F, 89.6 vs 89.3 ms, and removed in round 6)
        HIPCHK(launch_tile(st, l0, L.hi, L.lo, L.c, cmp_klen, bounds, km, T, tile_base, rec_meta, cmp_addr, drop, O,
                           d_flags + 2));
        if (l0 && key_fp) verify_args = {O.vcount, O.vpairs};
        if (l0) T0 = T;
    }
    HIPCHK(hipGetLastError());
    mark(ctx, PH_MERGE);
    const uint64_t* d_K = d_Kout;
    hres.pop_pos = pop_pos;
    tables_mine();
    auto fork_verify = [&]() {  // k_fp_verify on the aux stream, after what the ctx stream has queued
        if (!verify_args.first) return;
        ensure_aux(ctx);
        HIPCHK(hipEventRecord(ctx->aux_ev[0], st));
        HIPCHK(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_ev[0], 0));
        launch_fp_verify(ctx->aux_stream, verify_lo, verify_args.first, verify_args.second, R, fp_bad);
        HIPCHK(hipEventRecord(ctx->aux_ev[1], ctx->aux_stream));
        verify_args.first = nullptr;
        verify_pending = true;
    };
    auto join_verify = [&]() {  // fp_bad is read next: the ctx stream waits for k_fp_verify
        if (verify_args.first) {  // not forked: in order on the ctx stream
            launch_fp_verify(st, verify_lo, verify_args.first, verify_args.second, R, fp_bad);
            verify_args.first = nullptr;
        }
        if (verify_pending) HIPCHK(hipStreamWaitEvent(st, ctx->aux_ev[1], 0));
        verify_pending = false;
    };
    if (job.scan) {
        join_verify();
        const int rc = scan_stage(ctx, job, R, d_K, m_rec, m_src, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_start,
                                  fp_bad, heap ? &hres : nullptr, scan_ev, out);
        if (rc == RC_RETRY_EXACT) return rerun_exact(ctx, job, out);
        return rc;
    }
    if (job.flags & SKV_SPLIT_BY_TABLE) {
        join_verify();
        htrace("merge launched");
        const int rc =
            wal_stage(ctx, job, R, d_K, m_rec, m_src, m_P, m_Dp, rec_addr, rec_klen, fp_bad, heap ? &hres : nullptr, out,
                      sorted_merged ? sorted_S : nullptr);
        htrace("wal stage done");
        if (rc == RC_RETRY_EXACT) return rerun_exact(ctx, job, out);
        return rc;
    }
    if (heap) {
        // Delete filter + unsorted input: build_runs' order check on what the filter let through
        // (runs.rs:190-198, table_tree_compaction.rs:139-147), against the streams' decode errors
        unsigned long long* first_bad = dbuf<unsigned long long>(ctx, "heap_first_bad", 1);
        HIPCHK(hipMemsetAsync(first_bad, 0xFF, 8, st));
        launch_merged_order(st, d_K, R, m_rec, rec_hi, rec_lo, rec_klen, rec_addr, first_bad);
        HIPCHK(hipGetLastError());
        sync(ctx);  // (read_dev copies on the null stream, which does not wait for the ctx stream)
        const uint64_t v = read_dev((const uint64_t*)first_bad);
        std::vector<JobEvent> ev;
        if (v != ~0ull)
            ev.push_back({read_dev(pop_pos + read_dev(m_rec + v)), 0, SKV_E_FORMAT,
                          "Data format error: Operations must be sorted by key"});
        for (const HeapRes::Dec& d : hres.dec) {
            std::string msg;
            const int code = derr_to_api(d.err, msg);
            ev.push_back({hres.pos_of_original(d.rec), 2, code, msg});
        }
        throw_first(ev);
    }
    // ---- chain + stats ----------------------------------------------------------------------
    uint64_t* run_b = dbuf<uint64_t>(ctx, "run_b", R + 2);
    uint64_t* d_nruns = dbuf<uint64_t>(ctx, "n_runs", 4);  // {runs, K, P[K]} (k_chain)
    DevRunDesc* d_desc = dbuf<DevRunDesc>(ctx, "descs", R + 1);
    uint64_t* seg_r0 = dbuf<uint64_t>(ctx, "seg_r0", R / GATHER_SEG + 2);
    const uint64_t in_rec_bytes = job.in_bytes;  // bounds P[K]
    uint32_t* chain_tbl = dbuf<uint32_t>(ctx, "chain_tbl", chain_table_entries(in_rec_bytes));
    // parallel split buffers (k_split_*; the device plan falls back to k_chain where it does not fit).
    // SKV_SPLIT=serial: k_chain only; =par: no minimum run count. SKV_SPLIT_NC / SKV_SPLIT_SEG:
    // candidates per window, runs per segment (tests shrink the window to exercise the stitch's walks)
    SplitBufs sp{};
    {
        const char* mode = test_opt("SKV_SPLIT");
        const bool serial = mode && !strcmp(mode, "serial");
        sp.segr = 16;
        sp.nc = 512;
        sp.min_runs = mode && !strcmp(mode, "par") ? 0 : 1024;
        if (const char* e = test_opt("SKV_SPLIT_NC")) sp.nc = (uint32_t)std::min<uint64_t>(8192, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
        if (const char* e = test_opt("SKV_SPLIT_SEG")) sp.segr = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
        const uint64_t M = job.max_run_size;
        if (!serial && M > 8 && R < 0xFFFFFFF0ull) {
            // runs of >= 8 records (the plan's gate) hold > 7/8 (max - 1) bytes each
            const uint64_t runs_ub = in_rec_bytes / ((M - 1) - (M - 1) / 8) + 2;
            const uint64_t want = runs_ub / sp.segr + 2;
            sp.nseg_cap = (uint32_t)std::min<uint64_t>(want, 16384);
        }
        if (sp.nseg_cap) {
            sp.plan = dbuf<SplitPlan>(ctx, "split_plan", 1);
            sp.seg_w = dbuf<uint64_t>(ctx, "split_w", sp.nseg_cap);
            sp.seg_n = dbuf<uint32_t>(ctx, "split_n", sp.nseg_cap);
            sp.seg_sel = dbuf<uint32_t>(ctx, "split_sel", sp.nseg_cap);
            sp.seg_D = dbuf<uint64_t>(ctx, "split_D", sp.nseg_cap);
            sp.chain = dbuf<uint32_t>(ctx, "split_chain", (uint64_t)sp.nseg_cap * sp.segr * sp.nc);
            sp.ends = dbuf<uint32_t>(ctx, "split_ends", (uint64_t)sp.nseg_cap * sp.nc + 4);
        }
    }
    // a part of skv_compact_split (variable-length records): the split continues the open run of
    // the previous part -- records [0, e1) join it (run 0, a continuation), the rest split afresh
    uint64_t carry_c = 0, carry_e1 = 0;
    if (job.carry) {
        if (!job.carry->wait_in(job.carry_part, carry_c)) throw DevError("split stopped");
        if (carry_c) {
            uint64_t* d_cf = dbuf<uint64_t>(ctx, "carry_first", 4);
            launch_carry_first(st, d_K, m_P, job.max_run_size, carry_c, d_cf);
            uint64_t* hcf = (uint64_t*)pinned(ctx, 16);
            d2h(ctx, hcf, d_cf, 16);
            sync(ctx);
            carry_e1 = hcf[0];
            if (carry_e1) {
                const uint64_t K_all = hcf[0] + hcf[1];
                launch_chain(st, d_cf + 1, m_P + carry_e1, job.max_run_size, tile_max, T0, run_b + 1, d_nruns,
                             chain_tbl, R, in_rec_bytes, &sp);
                launch_carry_fix(st, run_b, d_nruns, m_P, carry_e1, K_all);
            }
        }
    }
    if (!carry_e1)
        launch_chain(st, d_K, m_P, job.max_run_size, tile_max, T0, run_b, d_nruns, chain_tbl, R, in_rec_bytes, &sp);
    if (job.carry) {  // the open run this part leaves, staged (handed on once the part's result is final)
        uint64_t* d_co = dbuf<uint64_t>(ctx, "carry_out", 1);
        launch_carry_out(st, run_b, d_nruns, m_P, carry_c, carry_e1 ? 1u : 0u, d_co);
        uint64_t* hco = (uint64_t*)pinned(ctx, 16);
        d2h(ctx, hco, d_co, 8);
        sync(ctx);
        job.carry->post_out(job.carry_part, hco[0], carry_e1 != 0);
    }
    if (sp.nseg_cap && test_opt("SKV_SPLIT_DEBUG")) {  // tests/test_gpu_split.py reads which split ran
        sync(ctx);
        SplitPlan pl;
        HIPCHK(hipMemcpy(&pl, sp.plan, sizeof(pl), hipMemcpyDeviceToHost));
        fprintf(stderr, "[split] mode=%u nseg=%u sel=%u walked=%u K=%llu L0=%llu cap=%u\n", pl.mode, pl.nseg,
                pl.nseg_sel, pl.n_fb, (unsigned long long)pl.K, (unsigned long long)pl.L0, sp.nseg_cap);
    }
    launch_run_stats(st, d_nruns, run_b, m_P, m_Dp, m_rec, rec_klen, d_desc, seg_r0, R);
    mark(ctx, PH_CHAIN);
    fork_verify();  // beside the gather (beside the single-wave chain it slowed the chain 3x)
    // ---- gather -----------------------------------------------------------------------------
    const uint64_t total_rec_bytes = job.in_bytes;
    // a part of a pipelined host call writes into the call's shared output buffer (job.dev_out)
    uint8_t* d_out = job.dev_out ? job.dev_out : dbuf<uint8_t>(ctx, "out", total_rec_bytes + R + 16);
    launch_gather(st, d_K, d_nruns, run_b, m_P, m_src, seg_r0, d_out, R, m_dup, fp_bad);
    HIPCHK(hipGetLastError());
    mark(ctx, PH_GATHER);
    // ---- readback: summary + descriptors in one sync (descriptor count guessed from sizes) -------
    static_assert(sizeof(skv_run_desc) == sizeof(DevRunDesc), "desc layout");
    const uint64_t guess = std::min<uint64_t>(
        R + 1, job.max_run_size > 1 ? 2 * (total_rec_bytes / (job.max_run_size - 1)) + 64 : R + 1);
    uint64_t h3[4];
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    {
        const size_t vbytes = deferred ? 16 + (size_t)n_runs * 4 : 0;  // flags + broken runs
        join_verify();
        uint8_t* hp = (uint8_t*)pinned(ctx, 64 + guess * sizeof(DevRunDesc) + vbytes);
        uint8_t* hv = hp + 64 + guess * sizeof(DevRunDesc);
        d2h(ctx, hp, d_nruns, 24);
        d2h(ctx, hp + 32, fp_bad, 4);
        d2h(ctx, hp + 64, d_desc, guess * sizeof(DevRunDesc));
        if (deferred) {
            d2h(ctx, hv, d_flags, 16);
            d2h(ctx, hv + 16, d_broken, (size_t)n_runs * 4);
        }
        sync(ctx);
        if (deferred) {
            const uint32_t* f = (const uint32_t*)hv;  // >= 2 GiB record, key decrease, poison
            bool bad = f[0] || f[1] || f[2];
            for (uint32_t r = 0; r < n_runs && !bad; ++r) bad = ((const uint32_t*)(hv + 16))[r] != 0;
            if (bad) {
                delete box;
                return compact_device(ctx, job, out, false);
            }
        }
        uint32_t fpb = 0;
        memcpy(&fpb, hp + 32, 4);
        if (fpb) {
            delete box;
            return rerun_exact(ctx, job, out);
        }
        memcpy(h3, hp, 24);
        const uint64_t n = h3[0];
        res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, n) * sizeof(skv_run_desc));
        memcpy(res->runs, hp + 64, std::min(n, guess) * sizeof(DevRunDesc));
        if (n > guess)
            HIPCHK(hipMemcpy(res->runs + guess, d_desc + guess, (n - guess) * sizeof(DevRunDesc), hipMemcpyDeviceToHost));
    }
    const uint64_t n_out_runs = h3[0], K = h3[1], kept_bytes = h3[2];
    res->n_runs = n_out_runs;
    res->bytes = d_out;
    res->n_bytes = kept_bytes + n_out_runs;
    res->in_bytes = job.in_bytes;
    res->in_records = R;
    res->out_records = K;
    res->dropped_tables = 0;
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
        t.gather_read_bytes = kept_bytes;
        t.gather_write_bytes = kept_bytes + n_out_runs;
        t.hot_ms = ms[PH_GATHER];
    }
    ctx->timings.path = parsed ? SKV_PATH_FIXED : SKV_PATH_GENERAL;
    ctx->timings.hot_read_bytes = kept_bytes;
    ctx->timings.hot_write_bytes = kept_bytes + n_out_runs;
    ctx->timings.host_syncs = ctx->syncs;
    *out = res;
    return SKV_OK;
}
// the one-run job of a writer batch (writer_service.rs:148-162)
int batch_job(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size, Job& job) {
    if (len && !ops_run) return set_err(ctx, SKV_E_INVALID_ARG, "ops_run is NULL");
    const uint8_t* runs[1] = {ops_run};
    const uint64_t lens[1] = {len};
    skv_stream st{runs, lens, 1u, 0};
    const int rc = build_job(ctx, &st, 1, max_run_size, 0, job);
    job.batch = true;
    return rc;
}

extern "C" {

int skv_compact_dev(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams, uint64_t max_run_size, uint32_t flags,
                    skv_result** out) {
    const double t_entry = now_ms();
    htrace("entry");
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;  // its tables borrow the ctx's storage for the call (no fresh 10^6-entry vectors)
    job.ranked.swap(ctx->j_ranked);
    job.run_ptr.swap(ctx->j_ptr);
    job.run_len.swap(ctx->j_len);
    int rc = build_job(ctx, streams, n_streams, max_run_size, flags, job);
    htrace("job built");
    if (!rc) rc = run_guarded(ctx, job, out, t_entry);
    job.ranked.swap(ctx->j_ranked);
    job.run_ptr.swap(ctx->j_ptr);
    job.run_len.swap(ctx->j_len);
    return rc;
}

int skv_encode_batch_dev(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size,
                         skv_result** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;
    int rc = batch_job(ctx, ops_run, len, max_run_size, job);
    if (rc) return rc;
    return run_guarded(ctx, job, out, t_entry);
}

}  // extern "C"
