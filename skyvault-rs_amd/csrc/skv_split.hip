// skv_split.hip — one compaction split across several GPUs by key range:
// skv_compact_split, the host-input entry (skv_compact) over G ctxs at once.
//
// The call is cut into G key-range shards, each of P_g key-range parts (the cut keys and per-run
// bounds of the pipelined host call, fx_host_cuts). Shard g runs on ctxs[g]: the H2D of its slices
// and the fused stride path over its parts, survivors numbered from 0 within the shard (each
// part's numbering chained on the device through the shard's earlier parts only, FxPartIO::gbase).
// Equal keys never straddle a cut, so each shard's merge, dedup and record checks are exactly the
// whole call's restricted to its keys (k_way.rs:113-171; runs.rs:559-624).
//
// What does not shard is build_runs' greedy split (runs.rs:211-238): it walks the merged records
// in order. With one record size it is arithmetic in the global survivor index -- survivor i goes to
// run i / n, slot i % n (n = fx_run_records) -- so the one exchange between the shards is their
// survivor counts C_g. The host chains them into bases B_g = C_0 + ... + C_{g-1} (G additions, the
// "carry" of the split), and every shard copies its survivors D2H straight to their global places
// in the one pinned output buffer: one copy per output run the shard touches. The host writes the
// version bytes and the descriptors (StatsV1, runs.rs:102-109) arithmetically, as k_fx_desc does.
//
// A call outside the fused shape, a cut that a run decreases across, or a poisoned shard (a record
// the fused path does not take, a key decrease) runs as skv_compact on ctxs[0], which gives the
// reference's exact outcome. A HIP failure in any shard is SKV_E_DEVICE on ctxs[0].
#include "skv_host.hpp"

namespace {

struct Shard {
    skv_ctx* ctx = nullptr;
    uint64_t p0 = 0, p1 = 0;    // its key-range parts
    uint64_t R = 0;             // input records
    uint64_t C = 0;             // survivors
    uint64_t B = 0;             // survivors of the earlier shards
    uint8_t* d_out = nullptr;   // survivors 0..C-1 at 1 + j * S
    bool poisoned = false;
    uint32_t reason = 0;
    std::string err;
    double merge_ms = 0;
};

// Shard g up to its survivor count: H2D of its slices on in_stream, the fused path per part on the
// ctx stream, one readback of the count and the verdict. Runs on its own host thread.
void shard_merge(Shard& sh, const Job& job, const RunFmt& f, const std::vector<uint64_t>& lb) {
    skv_ctx* ctx = sh.ctx;
    const double t0 = now_ms();
    const uint64_t nr = job.run_ptr.size(), S = f.S, Pn = sh.p1 - sh.p0;
    // run m's image holds its records [a_m, z_m) of this shard, after the byte before a_m
    std::vector<uint64_t> base(nr), img(nr + 1, 0);
    sh.R = 0;
    for (uint64_t m = 0; m < nr; ++m) {
        const uint64_t a = lb[sh.p0 * nr + m], z = lb[sh.p1 * nr + m];
        base[m] = a;
        sh.R += z - a;
        img[m + 1] = img[m] + (z > a ? ((1 + (z - a) * S + 15) & ~15ull) : 0);
    }
    if (!sh.R) return;
    hipStream_t st = ctx->stream;
    struct KernelUploads {  // table uploads by kernel: a DMA upload would queue behind the bulk H2D
        skv_ctx* c;
        explicit KernelUploads(skv_ctx* x) : c(x) { c->kernel_uploads = true; }
        ~KernelUploads() { c->kernel_uploads = false; }
    } ku(ctx);
    ctx->syncs = 0;
    ctx->up_chunk = 0;
    ctx->up_off = 0;
    if (!ctx->in_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->in_stream, hipStreamNonBlocking));
    while (ctx->part_ev.size() < Pn) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->part_ev.push_back(e);
    }
    // every buffer sized before the first launch (no buffer moves under queued work)
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", img[nr] + 16);
    const uint64_t n_loc = sh.R, out_cap = 1 + sh.R * S + 16;  // one local run: survivors at 1 + j * S
    sh.d_out = dbuf<uint8_t>(ctx, "out", out_cap);
    uint64_t* d_Kp = dbuf<uint64_t>(ctx, "hp_K", Pn);
    uint32_t* d_flags = dbuf<uint32_t>(ctx, "hp_flags", 4);
    FxPartTables pt;
    fx_part_tables(job, f, sh.p0, sh.p1, lb, d_in, img, &base, pt);
    RunInfo* d_runs = dbuf<RunInfo>(ctx, "hp_runs", Pn * nr);
    uint8_t* hp = (uint8_t*)pinned(ctx, 64);
    h2d_up(ctx, d_runs, pt.runs.data(), Pn * nr * sizeof(RunInfo));
    HIPCHK(hipMemsetAsync(d_Kp, 0, Pn * 8, st));
    HIPCHK(hipMemsetAsync(d_flags, 0, 16, st));
    for (uint64_t i = 0; i < Pn; ++i) {
        const uint64_t p = sh.p0 + i;
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t a = lb[p * nr + m], z = lb[(p + 1) * nr + m];
            if (z == a) continue;
            // the byte before record a rides along with the shard's first slice of the run
            const uint64_t lo = a == base[m] ? a * S : 1 + a * S, hi = 1 + z * S;
            HIPCHK(hipMemcpyAsync(d_in + img[m] + (lo - base[m] * S), (const uint8_t*)(uintptr_t)job.run_ptr[m] + lo,
                                  hi - lo, hipMemcpyHostToDevice, ctx->in_stream));
        }
        HIPCHK(hipEventRecord(ctx->part_ev[i], ctx->in_stream));
        HIPCHK(hipStreamWaitEvent(st, ctx->part_ev[i], 0));
        if (pt.kp[i]) {
            FxPartIO io;
            io.gbase = i ? d_Kp + i - 1 : nullptr;
            io.Kout = d_Kp + i;
            io.flags = d_flags;
            io.out = sh.d_out;
            uint64_t* rb_unused = nullptr;
            (void)fx_launch(ctx, pt.kp[i], pt.np[i], d_runs + i * nr, pt.sfr[i], f, pt.recb[i], n_loc, out_cap, &io,
                            rb_unused);
        } else if (i) {
            launch_copy_bytes(st, (uint8_t*)(d_Kp + i), (const uint8_t*)(d_Kp + i - 1), 8);
        }
        HIPCHK(hipGetLastError());
    }
    d2h(ctx, hp, d_Kp + Pn - 1, 8);
    d2h(ctx, hp + 16, d_flags, 16);
    sync(ctx);
    uint32_t fl[4];
    memcpy(&sh.C, hp, 8);
    memcpy(fl, hp + 16, 16);
    sh.poisoned = fl[2] != 0 || sh.C > sh.R;
    sh.reason = fl[3];
    sh.merge_ms = now_ms() - t0;
}

// Shard g's survivors to their global places: local survivor j is global survivor B + j.
void shard_egress(Shard& sh, const RunFmt& f, uint64_t n, uint8_t* h_out) {
    skv_ctx* ctx = sh.ctx;
    const uint64_t S = f.S, W = n * S + 1;
    for (uint64_t j = 0; j < sh.C;) {
        const uint64_t g = sh.B + j, q = g / n, slot = g % n;
        const uint64_t c = std::min(n - slot, sh.C - j);
        HIPCHK(hipMemcpyAsync(h_out + q * W + 1 + slot * S, sh.d_out + 1 + j * S, c * S, hipMemcpyDeviceToHost,
                              ctx->stream));
        j += c;
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
}

// fn(shard) on one host thread per shard, on the shard's device; a throw is kept as the shard's error
template <typename F>
void on_shards(std::vector<Shard>& sh, F&& fn) {
    std::vector<std::thread> th;
    for (Shard& s : sh)
        th.emplace_back([&s, &fn] {
            try {
                DeviceScope ds(s.ctx->device);
                if (!ds.ok) throw DevError("hipSetDevice failed");
                fn(s);
            } catch (const DevError& e) {
                s.err = e.msg;
            } catch (const std::exception& e) {
                s.err = std::string("host error: ") + e.what();
            }
        });
    for (std::thread& t : th) t.join();
}

}  // namespace

extern "C" {

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
        // shards of P_g parts each (a part is at most ~256 MiB of input, as in the pipelined call)
        uint64_t Pg = std::max<uint64_t>(1, std::min<uint64_t>(16, job.in_bytes / G / (256ull << 20)));
        if (const char* e = getenv("SKV_SPLIT_PARTS")) Pg = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
        const uint64_t P = G * Pg;
        std::vector<uint64_t> lb;
        // one D2H copy per output run a shard touches: a split into tiny runs stays on one GPU
        if (fx_host_shape(job, f, R) && R >= P * 64 &&
            R / fx_run_records(max_run_size, f.S, R) <= (1u << 16) && fx_host_cuts(job, f, P, lb)) {
            try {
                std::vector<Shard> sh(G);
                for (uint64_t g = 0; g < G; ++g) {
                    sh[g].ctx = ctxs[g];
                    sh[g].p0 = g * Pg;
                    sh[g].p1 = (g + 1) * Pg;
                }
                on_shards(sh, [&](Shard& s) { shard_merge(s, job, f, lb); });
                std::string err;
                bool poisoned = false;
                uint64_t C = 0;
                for (Shard& s : sh) {
                    if (!s.err.empty() && err.empty()) err = s.err;
                    poisoned = poisoned || s.poisoned;
                    s.B = C;  // the carry of build_runs' split: survivors of the earlier shards
                    C += s.C;
                }
                if (!err.empty()) {
                    for (Shard& s : sh) {
                        DeviceScope ds(s.ctx->device);
                        drain(s.ctx);
                    }
                    return set_err(home, SKV_E_DEVICE, "split shard: %s", err.c_str());
                }
                if (!poisoned) {
                    const uint64_t n = fx_run_records(max_run_size, f.S, R), W = n * f.S + 1;
                    const uint64_t runs = (C + n - 1) / n, bytes = C * f.S + runs;
                    size_t cap = 0;
                    uint8_t* h_out = (uint8_t*)home->out_pool->take(std::max<uint64_t>(bytes, 1), cap);
                    if (!h_out) return set_err(home, SKV_E_DEVICE, "pinned host allocation of the output failed");
                    const double t_eg = now_ms();
                    on_shards(sh, [&](Shard& s) { shard_egress(s, f, n, h_out); });
                    for (Shard& s : sh)
                        if (!s.err.empty()) {
                            for (Shard& x : sh) {  // no copy still writes h_out once it is back in the pool
                                DeviceScope ds(x.ctx->device);
                                drain(x.ctx);
                            }
                            home->out_pool->give(h_out, cap);
                            return set_err(home, SKV_E_DEVICE, "split shard egress: %s", s.err.c_str());
                        }
                    ResultBox* box = new ResultBox();
                    skv_result* res = &box->pub;
                    res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, runs) * sizeof(skv_run_desc));
                    for (uint64_t r = 0; r < runs; ++r) {
                        const uint64_t c = std::min(n, C - r * n);
                        skv_run_desc& d = res->runs[r];
                        h_out[r * W] = 1;  // RUN_VERSION_V1 (runs.rs:241-244)
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
                    res->bytes = h_out;
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
                    t.merge_ms = 0;
                    for (const Shard& s : sh) t.merge_ms = std::max(t.merge_ms, s.merge_ms);
                    t.gather_ms = now_ms() - t_eg;  // the shards' D2H copies to their global places
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
    // outside the split's shape, or a poisoned shard: the whole call on ctxs[0] (exact outcome)
    return skv_compact(home, streams, n_streams, max_run_size, flags, out);
}

}  // extern "C"
