// skv_split.hip — one compaction split across several GPUs by key range:
// skv_compact_split, the host-input entry (skv_compact) over G ctxs at once.
//
// The call is cut into P = G x P_g key-range parts (the cut keys and per-run bounds of the pipelined
// host call, fx_host_cuts), dealt round-robin: part p goes to ctxs[p % G]. Each ctx's worker thread
// queues, for each of its parts, the H2D of the part's slices (in_stream) and the fused stride path
// over them (the ctx stream), survivors numbered from 0 within the part, and publishes the part's
// survivor count and verdict to host-mapped words. Equal keys never straddle a cut, so each part's
// merge, dedup and record checks are exactly the whole call's restricted to its keys
// (k_way.rs:113-171; runs.rs:559-624).
//
// What does not shard is build_runs' greedy split (runs.rs:211-238): it walks the merged records
// in order. With one record size it is arithmetic in the global survivor index -- survivor i goes to
// run i / n, slot i % n (n = fx_run_records) -- so the one exchange between the GPUs is the parts'
// survivor counts C_p. The host chains them into bases B_p = C_0 + ... + C_{p-1} (the "carry" of the
// split) as they arrive; once B_p is known the worker of part p copies its survivors D2H straight to
// their global places in the one pinned output buffer (out_stream; one copy per output run the part
// touches) while its later parts are still arriving and merging. Round-robin dealing keeps the parts
// in flight on all GPUs close together in key order, so the D2H of round r overlaps the H2D of
// round r + 1 on every GPU. The host writes the version bytes and the descriptors (StatsV1,
// runs.rs:102-109) arithmetically, as k_fx_desc does.
//
// A call outside the fused shape (variable-length records, Deletes, WAL flushes), or one whose
// survivors would need more than 2^16 D2H copies, takes the split with build_runs' carry
// (compact_split_general, skv_hostpipe.hip). A poisoned part (a record the fused path does not
// take, a key decrease) runs the call as skv_compact on ctxs[0], which gives the reference's exact
// outcome. A HIP failure on any ctx is SKV_E_DEVICE on ctxs[0].
#include "skv_host.hpp"

namespace {

constexpr uint64_t NPOS = ~0ull;

// State the workers share: the parts' survivor counts as they arrive and the bases chained from them.
struct Split {
    const Job* job = nullptr;
    RunFmt f{};
    const std::vector<uint64_t>* lb = nullptr;
    uint64_t P = 0, G = 0, n = 0;
    uint8_t* h_out = nullptr;
    uint64_t out_cap = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> cnt;   // part p's survivors (NPOS: not yet known)
    std::vector<uint64_t> base;  // base[p] = survivors of parts < p, valid for p <= prefix
    uint64_t prefix = 0;         // parts [0, prefix) have posted their counts
    bool stop = false;           // a poisoned part or a failed worker: no more egress
    bool poisoned = false;
    std::string err;
    // ctxs that share a device: their parts' H2D go in part order (each waits for the previous
    // part of its device), so the first parts land first instead of all parts at once
    std::vector<int64_t> prev_on_dev;  // the part before p on p's device from another ctx, or -1
    std::vector<hipEvent_t> h2d_ev;    // part p's H2D-complete event, once its worker recorded it

    void post(uint64_t p, uint64_t c) {
        {
            std::lock_guard<std::mutex> g(mu);
            cnt[p] = c;
            while (prefix < P && cnt[prefix] != NPOS) {
                base[prefix + 1] = base[prefix] + cnt[prefix];
                ++prefix;
            }
        }
        cv.notify_all();
    }
    void halt(bool poison, const std::string& e) {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            poisoned = poisoned || poison;
            if (!e.empty() && err.empty()) err = e;
        }
        cv.notify_all();
    }
    void h2d_post(uint64_t p, hipEvent_t e) {
        {
            std::lock_guard<std::mutex> g(mu);
            h2d_ev[p] = e;
        }
        cv.notify_all();
    }
    // the H2D event of part q once recorded; null once the call has stopped
    hipEvent_t h2d_wait(uint64_t q) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || h2d_ev[q] != nullptr; });
        return stop ? nullptr : h2d_ev[q];
    }
    // B_p once every earlier part has posted; false once the call has stopped
    bool wait_base(uint64_t p, uint64_t& B) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || prefix >= p; });
        if (stop) return false;
        B = base[p];
        return true;
    }
};

// The worker of ctxs[g]: parts g, g + G, g + 2G, ...
void split_worker(Split& sp, skv_ctx* ctx, uint64_t g) {
    const Job& job = *sp.job;
    const std::vector<uint64_t>& lb = *sp.lb;
    const RunFmt& f = sp.f;
    const uint64_t nr = job.run_ptr.size(), S = f.S, W = sp.n * S + 1;
    std::vector<uint64_t> parts;
    for (uint64_t p = g; p < sp.P; p += sp.G) parts.push_back(p);
    const uint64_t np = parts.size();
    // part i's images: run m's slice [a, z) after the byte before a, at in_off[i] + img[i][m];
    // its survivors at out_off[i] + 1 + j * S (one local run of R_i records)
    std::vector<std::vector<uint64_t>> img(np), base(np);
    std::vector<uint64_t> Rp(np, 0), in_off(np + 1, 0), out_off(np + 1, 0);
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t p = parts[i];
        img[i].assign(nr + 1, 0);
        base[i].assign(nr, 0);
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t a = lb[p * nr + m], z = lb[(p + 1) * nr + m];
            base[i][m] = a;
            Rp[i] += z - a;
            img[i][m + 1] = img[i][m] + (z > a ? ((1 + (z - a) * S + 15) & ~15ull) : 0);
        }
        in_off[i + 1] = in_off[i] + ((img[i][nr] + 255) & ~255ull);
        out_off[i + 1] = out_off[i] + ((1 + Rp[i] * S + 16 + 255) & ~255ull);
    }
    hipStream_t st = ctx->stream;
    // table uploads by kernel (a DMA upload would queue behind the bulk H2D); fx_launch's own buffers
    // are sized per part and may grow mid-queue: their old allocations wait for the streams to drain
    PipeIO kio(ctx);
    ctx->syncs = 0;
    ctx->up_chunk = 0;
    ctx->up_off = 0;
    if (!ctx->in_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->in_stream, hipStreamNonBlocking));
    if (!ctx->out_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->out_stream, hipStreamNonBlocking));
    while (ctx->part_ev.size() < 2 * np) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->part_ev.push_back(e);
    }
    if (ctx->part_k_cap < 2 * np) {
        if (ctx->part_k) HIPCHK(hipHostFree(ctx->part_k));
        ctx->part_k = nullptr;
        ctx->part_k_cap = 0;
        HIPCHK(host_alloc_near(ctx->device, (void**)&ctx->part_k, std::max<uint64_t>(2 * np, 64) * 8,
                               hipHostMallocCoherent));
        ctx->part_k_cap = std::max<uint64_t>(2 * np, 64);
    }
    volatile uint64_t* hK = ctx->part_k;  // [2i] survivors of part i, [2i + 1] its verdict words
    // the call's own buffers sized before the first launch (fx_launch's per-part ones: PipeIO above)
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", in_off[np] + 16);
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", out_off[np] + 16);
    uint64_t* d_K = dbuf<uint64_t>(ctx, "hp_K", np);
    uint32_t* d_flags = dbuf<uint32_t>(ctx, "hp_flags", 4);
    RunInfo* d_runs = dbuf<RunInfo>(ctx, "hp_runs", np * nr);
    std::vector<FxPartTables> pt(np);
    std::vector<RunInfo> rows(np * nr);
    for (uint64_t i = 0; i < np; ++i) {
        fx_part_tables(job, f, parts[i], parts[i] + 1, lb, d_in + in_off[i], img[i], &base[i], pt[i]);
        std::copy(pt[i].runs.begin(), pt[i].runs.end(), rows.begin() + i * nr);
    }
    h2d_up(ctx, d_runs, rows.data(), np * nr * sizeof(RunInfo));
    HIPCHK(hipMemsetAsync(d_K, 0, np * 8, st));
    HIPCHK(hipMemsetAsync(d_flags, 0, 16, st));
    for (uint64_t i = 0; i < np; ++i) {
        hK[2 * i] = NPOS;
        hK[2 * i + 1] = NPOS;
    }
    // ---- queue every part: H2D, the fused path, the count and verdict to host-mapped words
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t p = parts[i];
        if (sp.prev_on_dev[p] >= 0) {
            const hipEvent_t e = sp.h2d_wait((uint64_t)sp.prev_on_dev[p]);
            if (!e) return;  // the call has stopped (a poisoned part or a failed worker)
            HIPCHK(hipStreamWaitEvent(ctx->in_stream, e, 0));
        }
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t a = lb[p * nr + m], z = lb[(p + 1) * nr + m];
            if (z == a) continue;
            HIPCHK(hipMemcpyAsync(d_in + in_off[i] + img[i][m], (const uint8_t*)(uintptr_t)job.run_ptr[m] + a * S,
                                  1 + (z - a) * S, hipMemcpyHostToDevice, ctx->in_stream));
        }
        HIPCHK(hipEventRecord(ctx->part_ev[2 * i], ctx->in_stream));
        sp.h2d_post(p, ctx->part_ev[2 * i]);
        HIPCHK(hipStreamWaitEvent(st, ctx->part_ev[2 * i], 0));
        if (pt[i].kp[0]) {
            FxPartIO io;
            io.gbase = nullptr;
            io.Kout = d_K + i;
            io.flags = d_flags;
            io.out = d_out + out_off[i];
            uint64_t* rb_unused = nullptr;
            (void)fx_launch(ctx, pt[i].kp[0], pt[i].np[0], d_runs + i * nr, pt[i].sfr[0], f, pt[i].recb[0], Rp[i],
                            out_off[i + 1] - out_off[i], &io, rb_unused);
        }
        launch_fx_publish(st, d_K + i, (uint64_t*)hK + 2 * i);
        launch_fx_publish(st, (const uint64_t*)(d_flags + 2), (uint64_t*)hK + 2 * i + 1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->part_ev[2 * i + 1], st));
    }
    // ---- as each part ends: post its count; once its base is known, its survivors to their places
    for (uint64_t i = 0; i < np; ++i) {
        HIPCHK(hipEventSynchronize(ctx->part_ev[2 * i + 1]));
        const uint64_t c = hK[2 * i];
        const uint32_t poison = (uint32_t)hK[2 * i + 1];  // flags[2]: cumulative over this ctx's parts
        if (poison != 0 || c > Rp[i]) {
            sp.halt(true, "");
            break;
        }
        sp.post(parts[i], c);
        uint64_t B = 0;
        if (!sp.wait_base(parts[i], B)) break;
        for (uint64_t j = 0; j < c;) {
            const uint64_t gi = B + j, q = gi / sp.n, slot = gi % sp.n;
            const uint64_t cc = std::min(sp.n - slot, c - j);
            if (q * W + 1 + (slot + cc) * S > sp.out_cap) throw DevError("internal: split egress past the output");
            HIPCHK(hipMemcpyAsync(sp.h_out + q * W + 1 + slot * S, d_out + out_off[i] + 1 + j * S, cc * S,
                                  hipMemcpyDeviceToHost, ctx->out_stream));
            j += cc;
        }
    }
    HIPCHK(hipStreamSynchronize(ctx->out_stream));
}

}  // namespace

extern "C" {

// The deal of skv_compact_split's key-range parts (include/skv.h): part p on ctxs[p % n_ctx]; ctxs that
// share a device take their parts' H2D in part order, so part p waits for the H2D of the latest
// earlier part dealt to another ctx of its device (h2d_after[p], -1: none).
int skv_split_deal(const int* ctx_device, uint32_t n_ctx, uint64_t n_parts, uint32_t* ctx_of_part,
                   int64_t* h2d_after) {
    if (!ctx_device || !n_ctx || (n_parts && (!ctx_of_part || !h2d_after))) return SKV_E_INVALID_ARG;
    std::map<int, uint64_t> last;  // device -> its latest part so far
    for (uint64_t p = 0; p < n_parts; ++p) {
        const uint32_t g = (uint32_t)(p % n_ctx);
        const int dv = ctx_device[g];
        ctx_of_part[p] = g;
        h2d_after[p] = -1;
        auto it = last.find(dv);
        if (it != last.end() && it->second % n_ctx != g) h2d_after[p] = (int64_t)it->second;
        last[dv] = p;
    }
    return SKV_OK;
}

int skv_compact_split(skv_ctx* const* ctxs, uint32_t n_ctx, const skv_stream* streams, uint32_t n_streams,
                      uint64_t max_run_size, uint32_t flags, skv_result** out) {
    const double t_entry = now_ms();
    if (!ctxs || !n_ctx || !ctxs[0]) return SKV_E_INVALID_ARG;
    skv_ctx* home = ctxs[0];
    if (!out) return set_err(home, SKV_E_INVALID_ARG, "out is NULL");
    *out = nullptr;
    for (uint32_t g = 0; g < n_ctx; ++g) {
        if (!ctxs[g]) return set_err(home, SKV_E_INVALID_ARG, "ctxs[%u] is NULL", g);
        for (uint32_t h = 0; h < g; ++h)
            if (ctxs[h] == ctxs[g]) return set_err(home, SKV_E_INVALID_ARG, "ctxs[%u] repeats ctxs[%u]", g, h);
    }
    if (n_ctx == 1) return skv_compact(home, streams, n_streams, max_run_size, flags, out);
    {
        SKV_DEVICE_SCOPE(home);
        Job job;
        if (const int rc = build_job(home, streams, n_streams, max_run_size, flags, job)) return rc;
        RunFmt f{};
        uint64_t R = 0;
        const uint64_t G = n_ctx;
        // P_g parts per ctx (a part is at most ~256 MiB of input, as in the pipelined call)
        uint64_t Pg = std::max<uint64_t>(1, std::min<uint64_t>(16, job.in_bytes / G / (256ull << 20)));
        if (const char* e = getenv("SKV_SPLIT_PARTS")) Pg = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
        const uint64_t P = G * Pg;
        std::vector<uint64_t> lb;
        // the fused shape's arithmetic split; one D2H copy per output run a part touches, so a split
        // into tiny runs takes the general split below
        const bool fused = fx_host_shape(job, f, R) && R >= P * 64 &&
                           R / fx_run_records(max_run_size, f.S, R) <= (1u << 16) && fx_host_cuts(job, f, P, lb);
        if (!fused) {  // variable-length records: the split with build_runs' carry (skv_hostpipe.hip)
            bool used = false;
            try {
                const int rc = compact_split_general(ctxs, n_ctx, job, out, t_entry, used);
                if (used) return rc;
            } catch (const DevError& e) {
                return set_err(home, SKV_E_DEVICE, "%s", e.msg.c_str());
            } catch (const std::exception& e) {
                return set_err(home, SKV_E_DEVICE, "host error: %s", e.what());
            }
        } else {
            try {
                const uint64_t n = fx_run_records(max_run_size, f.S, R), W = n * f.S + 1;
                Split sp;
                sp.job = &job;
                sp.f = f;
                sp.lb = &lb;
                sp.P = P;
                sp.G = G;
                sp.n = n;
                sp.cnt.assign(P, NPOS);
                sp.base.assign(P + 1, 0);
                sp.h2d_ev.assign(P, nullptr);
                sp.prev_on_dev.assign(P, -1);
                {
                    std::vector<int> dev(G);
                    std::vector<uint32_t> ctx_of(P);
                    for (uint64_t g = 0; g < G; ++g) dev[g] = ctxs[g]->device;
                    (void)skv_split_deal(dev.data(), (uint32_t)G, P, ctx_of.data(), sp.prev_on_dev.data());
                }
                // sized for every record surviving (the counts arrive while the copies run)
                sp.out_cap = R * f.S + (R + n - 1) / n;
                size_t cap = 0;
                sp.h_out = (uint8_t*)home->out_pool->take(std::max<uint64_t>(sp.out_cap, 1), cap);
                if (!sp.h_out) return set_err(home, SKV_E_DEVICE, "pinned host allocation of the output failed");
                WorkerSet ws;
                const bool spawned = ws.spawn((unsigned)G, [&sp, ctxs](unsigned g) {
                        skv_ctx* ctx = ctxs[g];
                        DeviceScope ds(ctx->device);
                        try {
                            if (!ds.ok) throw DevError("hipSetDevice failed");
                            split_worker(sp, ctx, g);
                        } catch (const DevError& e) {
                            sp.halt(false, e.msg);
                        } catch (const std::exception& e) {
                            sp.halt(false, std::string("host error: ") + e.what());
                        }
                        drain(ctx);  // nothing of this call still runs on the ctx (nor writes h_out)
                    }, [&sp] { sp.halt(false, "worker thread creation failed"); });
                ws.join();
                if (!spawned && sp.err.empty()) sp.halt(false, "worker thread creation failed");
                if (!sp.err.empty() || sp.poisoned) {
                    home->out_pool->give(sp.h_out, cap);
                    if (!sp.err.empty()) return set_err(home, SKV_E_DEVICE, "split: %s", sp.err.c_str());
                } else {
                    const uint64_t C = sp.base[P];
                    const uint64_t runs = (C + n - 1) / n, bytes = C * f.S + runs;
                    ResultBox* box = new ResultBox();
                    skv_result* res = &box->pub;
                    res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, runs) * sizeof(skv_run_desc));
                    for (uint64_t r = 0; r < runs; ++r) {
                        const uint64_t c = std::min(n, C - r * n);
                        skv_run_desc& d = res->runs[r];
                        sp.h_out[r * W] = 1;  // RUN_VERSION_V1 (runs.rs:241-244)
                        d.off = r * W;
                        d.len = 1 + c * f.S;
                        d.put_count = c;
                        d.delete_count = 0;
                        d.min_key_off = d.off + 1 + 5;
                        d.min_key_len = f.K;
                        d.max_key_off = d.off + 1 + (c - 1) * f.S + 5;
                        d.max_key_len = f.K;
                        d.table_id = 0;
                        d.reserved = 0;
                    }
                    res->n_runs = runs;
                    res->bytes = sp.h_out;
                    res->n_bytes = bytes;
                    res->in_bytes = job.in_bytes;
                    res->in_records = R;
                    res->out_records = C;
                    res->dropped_tables = 0;
                    box->pool = home->out_pool;
                    box->pool_cap = cap;
                    skv_timings& t = home->timings;
                    t = skv_timings{};
                    t.path = SKV_PATH_FUSED;
                    t.hot_read_bytes = R * f.S;
                    t.hot_write_bytes = bytes;
                    t.host_parts = (uint32_t)P;
                    t.host_total_ms = now_ms() - t_entry;
                    *out = res;
                    return SKV_OK;
                }
            } catch (const DevError& e) {
                return set_err(home, SKV_E_DEVICE, "%s", e.msg.c_str());
            } catch (const std::exception& e) {
                return set_err(home, SKV_E_DEVICE, "host error: %s", e.what());
            }
        }
    }
    // outside the split's shape, or a poisoned part: the whole call on ctxs[0] (exact outcome)
    return skv_compact(home, streams, n_streams, max_run_size, flags, out);
}

}  // extern "C"
