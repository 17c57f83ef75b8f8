// skv_hostpipe.hip — skv_compact with host inputs: the serial stage -> compact -> copy path and the
// pipelined key-range paths that overlap H2D, kernels and D2H.
#include "skv_host.hpp"

using namespace skv;


// ---- pipelined host calls ---------------------------------------------------------------------
// skv_compact with host inputs (the get_run -> compact -> put_run of a job, storage.rs:183-250) as
// a key-range pipeline: the call is cut into P parts by key, every part holds each stream's records
// in [B_p, B_p+1) (equal keys never straddle a cut), and three streams overlap:
//   in_stream   H2D of part p's slices (pinned host runs -> their images in HBM)
//   ctx->stream the fused path on part p (fx_launch), survivor numbering chained on the device
//               through part p-1's count (FxArgs::gbase), one shared output buffer and verdict
//   out_stream  D2H of part p's output bytes as soon as its count is published
// so the PCIe copies in both directions run at once, and the kernels hide behind them. Taken when
// the host can see that the fused path applies (one run per stream, every run fixed-stride at one
// record size, key <= 16 bytes) and the call is large; the device verifies everything as in
// compact_fused, and a poisoned call (or a stream whose records decrease across a cut) reruns as
// the serial copy -> compact -> copy of compact_host_job.
static uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }


// The fused stride path's shape as the host can see it (one run format, key <= 16 bytes, fan-in
// within one tile, member runs of a stream ascending as one stream); R = the call's records.
bool fx_host_shape(const Job& job, RunFmt& f, uint64_t& R) {
    const uint32_t k = (uint32_t)job.ranked.size();
    if ((job.flags & SKV_SPLIT_BY_TABLE) || job.batch || job.search || job.scan) return false;
    const uint64_t nr = job.run_ptr.size();
    if (k == 0 || k > (uint32_t)TILE_TARGET / 2 || nr == 0) return false;
    R = 0;
    for (uint64_t m = 0; m < nr; ++m) {
        const uint8_t* run = (const uint8_t*)(uintptr_t)job.run_ptr[m];
        const uint64_t len = job.run_len[m];
        if (len < 1 + 9 || run[0] != 1 || run[1] != 1) return false;
        const uint64_t K = be32(run + 2);
        if (K > FX_MAX_K || 1 + 5 + K + 4 > len) return false;
        const uint64_t S = 9 + K + be32(run + 6 + K);
        if (S < FX_MIN_S || S > FX_MAX_S || (len - 1) % S) return false;
        if (m == 0) {
            f.S = S;
            f.K = (uint32_t)K;
            f.V = (uint32_t)(S - 9 - K);
        } else if (S != f.S || K != f.K) {
            return false;
        }
        R += (len - 1) / S;
    }
    // member runs of one stream (an L0 / next-level concatenation) must ascend as one sorted stream:
    // member i's last key below member i + 1's first (each member's own order: the device and the cuts)
    for (const InStream& st : job.ranked)
        for (uint64_t m = st.first; m + 1 < st.first + st.n_runs; ++m) {
            const uint8_t* a = (const uint8_t*)(uintptr_t)job.run_ptr[m];
            const uint8_t* b = (const uint8_t*)(uintptr_t)job.run_ptr[m + 1];
            if (memcmp(a + job.run_len[m] - f.S + 5, b + 1 + 5, f.K) >= 0) return false;
        }
    return R < 0xFFFFFFFFull;
}

static bool pipe_eligible(const Job& job, RunFmt& f, uint64_t& R) {
    const char* pe = getenv("SKV_HOST_PIPE");
    if (pe && pe[0] == '0') return false;
    const char* me = getenv("SKV_HOST_PIPE_MIN");
    const uint64_t min_bytes = me ? strtoull(me, nullptr, 10) : (512ull << 20);
    if (job.in_bytes < min_bytes) return false;
    return fx_host_shape(job, f, R);
}

// P - 1 cut keys (quantiles of an even sample of every run) and lb[p * nr + m] = the first record of
// run m with key >= cut p (lb[m] = 0, lb[P * nr + m] = its record count). False when a run
// decreases across a cut: the device checks the order inside each part only.
bool fx_host_cuts(const Job& job, const RunFmt& f, uint64_t P, std::vector<uint64_t>& lb) {
    const uint64_t nr = job.run_ptr.size(), S = f.S, K = f.K;
    auto key_at = [&](uint64_t m, uint64_t i) { return (const uint8_t*)(uintptr_t)job.run_ptr[m] + 1 + i * S + 5; };
    auto nrec = [&](uint64_t m) { return (job.run_len[m] - 1) / S; };
    std::vector<std::array<uint8_t, 16>> smp;
    const uint64_t Q = std::max<uint64_t>(2, 4096 / nr);
    for (uint64_t m = 0; m < nr; ++m) {
        const uint64_t nm = nrec(m);
        for (uint64_t t = 0; t < Q && t < nm; ++t) {
            std::array<uint8_t, 16> a{};
            memcpy(a.data(), key_at(m, (2 * t + 1) * nm / (2 * Q)), K);
            smp.push_back(a);
        }
    }
    std::sort(smp.begin(), smp.end());
    std::vector<std::array<uint8_t, 16>> cut;  // B_1..B_{P-1}
    for (uint64_t p = 1; p < P; ++p) cut.push_back(smp[p * smp.size() / P]);
    lb.assign((P + 1) * nr, 0);
    const unsigned nb = par_nblocks(nr, 8);
    std::vector<uint8_t> ok(nb, 1);
    par_run(nr, nb, [&](unsigned b, uint64_t lo_m, uint64_t hi_m) {
        for (uint64_t m = lo_m; m < hi_m; ++m) {
            const uint64_t nm = nrec(m);
            lb[m] = 0;
            lb[P * nr + m] = nm;
            for (uint64_t p = 1; p < P; ++p) {
                uint64_t a = 0, z = nm;
                while (a < z) {
                    const uint64_t mid = (a + z) >> 1;
                    if (memcmp(key_at(m, mid), cut[p - 1].data(), K) < 0) a = mid + 1;
                    else z = mid;
                }
                lb[p * nr + m] = a;
                if (a < lb[(p - 1) * nr + m]) ok[b] = 0;
                if (a > 0 && a < nm && memcmp(key_at(m, a - 1), key_at(m, a), K) > 0) ok[b] = 0;
            }
        }
    });
    bool cuts_ok = true;
    for (uint8_t o : ok) cuts_ok = cuts_ok && o;
    return cuts_ok;
}

// Parts [p0, p1) as fused launches: part p's runs (streams in rank order, each stream's member
// slices in member order, empty slices and streams left out; rows (p - p0) * nr ...), the first run
// of each stream and the record bases. Slice (p, m) starts at d_in + img[m] + (lb[p][m] - base[m]) * S,
// the byte before its first record (run m's image holds its records from record base[m] on; no
// base: from record 0).
void fx_part_tables(const Job& job, const RunFmt& f, uint64_t p0, uint64_t p1, const std::vector<uint64_t>& lb,
                    const uint8_t* d_in, const std::vector<uint64_t>& img, const std::vector<uint64_t>* base,
                    FxPartTables& t) {
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t nr = job.run_ptr.size(), S = f.S, Pn = p1 - p0;
    t.runs.assign(Pn * nr, RunInfo{});
    t.kp.assign(Pn, 0);
    t.np.assign(Pn, 0);
    t.sfr.assign(Pn, {});
    t.recb.assign(Pn, {});
    for (uint64_t i = 0; i < Pn; ++i) {
        const uint64_t p = p0 + i;
        t.recb[i].assign(1, 0);
        for (uint32_t s = 0; s < k; ++s) {
            const InStream& st = job.ranked[s];
            const uint32_t n0 = t.np[i];
            for (uint64_t m = st.first; m < st.first + st.n_runs; ++m) {
                const uint64_t a = lb[p * nr + m], z = lb[(p + 1) * nr + m];
                if (z == a) continue;
                RunInfo& ri = t.runs[i * nr + t.np[i]++];
                ri.ptr = (uint64_t)(uintptr_t)(d_in + img[m] + (a - (base ? (*base)[m] : 0)) * S);
                ri.len = 1 + (z - a) * S;
                ri.chunk_base = 0;
                ri.n_chunks = 0;
                ri.stream = t.kp[i];
                t.recb[i].push_back(t.recb[i].back() + (z - a));
            }
            if (t.np[i] > n0) {
                t.sfr[i].push_back(n0);
                ++t.kp[i];
            }
        }
        t.sfr[i].push_back(t.np[i]);
    }
}

static int compact_host_pipelined(skv_ctx* ctx, Job& job, skv_result** out, double t_entry, bool& used) {
    used = false;
    RunFmt f{};
    uint64_t R = 0;
    if (!pipe_eligible(job, f, R)) return SKV_OK;
    const uint64_t nr = job.run_ptr.size();  // member runs (one per stream unless a stream concatenates)
    const uint64_t S = f.S;
    uint64_t P = std::max<uint64_t>(2, std::min<uint64_t>(64, job.in_bytes / (256ull << 20)));
    if (const char* pp = getenv("SKV_HOST_PARTS")) P = std::max<uint64_t>(1, std::min<uint64_t>(256, strtoull(pp, nullptr, 10)));
    if (R < P * 64) return SKV_OK;
    htrace("pipe: eligible");
    std::vector<uint64_t> lb;  // lb[p * nr + m]: first record of run m with key >= cut p
    if (!fx_host_cuts(job, f, P, lb)) return SKV_OK;
    htrace("pipe: cuts");
    used = true;
    hipStream_t st = ctx->stream;
    struct KernelUploads {  // table uploads of this call by kernel, not by a DMA engine
        skv_ctx* c;
        explicit KernelUploads(skv_ctx* x) : c(x) { c->kernel_uploads = true; }
        ~KernelUploads() { c->kernel_uploads = false; }
    } ku(ctx);
    ctx->syncs = 0;
    ctx->up_chunk = 0;  // the upload arena from its start (the last call ended with a sync)
    ctx->up_off = 0;
    if (!ctx->in_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->in_stream, hipStreamNonBlocking));
    if (!ctx->out_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->out_stream, hipStreamNonBlocking));
    while (ctx->part_ev.size() < 2 * P) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->part_ev.push_back(e);
    }
    if (ctx->part_k_cap < P) {
        if (ctx->part_k) HIPCHK(hipHostFree(ctx->part_k));
        ctx->part_k = nullptr;
        ctx->part_k_cap = 0;
        HIPCHK(host_alloc_near(ctx->device, (void**)&ctx->part_k, std::max<uint64_t>(P, 64) * 8, hipHostMallocCoherent));
        ctx->part_k_cap = std::max<uint64_t>(P, 64);
    }
    volatile uint64_t* hK = ctx->part_k;
    for (uint64_t p = 0; p < P; ++p) hK[p] = ~0ull;
    // ---- device buffers (all sized before the first launch: no buffer moves under queued work)
    std::vector<uint64_t> img(nr + 1, 0);
    for (uint64_t m = 0; m < nr; ++m) img[m + 1] = img[m] + ((job.run_len[m] + 15) & ~15ull);
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", img[nr] + 16);
    const uint64_t out_cap = job.in_bytes + R + 16;
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", out_cap);
    uint64_t* d_Kp = dbuf<uint64_t>(ctx, "hp_K", P);
    uint32_t* d_pflags = dbuf<uint32_t>(ctx, "hp_flags", 4);
    uint64_t* d_prb = dbuf<uint64_t>(ctx, "hp_rb", 4);
    const uint64_t n = fx_run_records(job.max_run_size, S, R), W = n * S + 1;
    const uint64_t max_runs = (R + n - 1) / n;
    DevRunDesc* d_desc = dbuf<DevRunDesc>(ctx, "descs", max_runs + 1);
    FxPartTables pt;
    fx_part_tables(job, f, 0, P, lb, d_in, img, nullptr, pt);
    RunInfo* d_runs = dbuf<RunInfo>(ctx, "hp_runs", P * nr);
    h2d_up(ctx, d_runs, pt.runs.data(), P * nr * sizeof(RunInfo));
    HIPCHK(hipMemsetAsync(d_Kp, 0, P * 8, st));
    HIPCHK(hipMemsetAsync(d_pflags, 0, 16, st));
    size_t cap = 0;
    uint8_t* h_out = (uint8_t*)ctx->out_pool->take(out_cap, cap);
    if (!h_out) throw DevError("pinned host allocation of the output failed");
    // Unless the result takes h_out, it goes back to the pool once no copy can touch it any more:
    // on every exit (a throw included) the three streams are drained first, so no H2D still reads
    // the caller's runs and no D2H still writes h_out after this call returns. Declared before the
    // egress thread's joiner, so it runs after the thread has been joined.
    struct OutGuard {
        skv_ctx* c;
        uint8_t*& buf;
        size_t cap;
        ~OutGuard() {
            if (c->in_stream) (void)hipStreamSynchronize(c->in_stream);
            if (c->out_stream) (void)hipStreamSynchronize(c->out_stream);
            (void)hipStreamSynchronize(c->stream);
            if (buf) c->out_pool->give(buf, cap);
        }
    } out_guard{ctx, h_out, cap};
    // ---- egress thread: D2H of part p once its count is published
    std::mutex mu;
    std::condition_variable cv;
    uint64_t issued = 0;
    bool stop = false;
    std::string d2h_err;
    uint64_t egress_end = 0;
    auto end_of = [&](uint64_t Kc) -> uint64_t {  // output bytes through survivor Kc - 1
        if (!Kc) return 0;
        const uint64_t g = Kc - 1;
        return (g / n) * W + 1 + (g % n) * S + S;
    };
    std::thread egress([&] {
        try {
            if (hipSetDevice(ctx->device) != hipSuccess) throw DevError("hipSetDevice failed (egress)");
            uint64_t E = 0, Kprev = 0;
            for (uint64_t p = 0; p < P; ++p) {
                {
                    std::unique_lock<std::mutex> g(mu);
                    cv.wait(g, [&] { return issued > p || stop; });
                    if (issued <= p) {  // stopped early: the copies already issued end first
                        (void)hipStreamSynchronize(ctx->out_stream);
                        return;
                    }
                }
                HIPCHK(hipEventSynchronize(ctx->part_ev[2 * p + 1]));
                const uint64_t Kc = hK[p];
                if (Kc < Kprev || Kc > R) break;  // a poisoned part: the verdict says so
                Kprev = Kc;
                const uint64_t E1 = std::min(end_of(Kc), out_cap);
                if (E1 > E) HIPCHK(hipMemcpyAsync(h_out + E, d_out + E, E1 - E, hipMemcpyDeviceToHost, ctx->out_stream));
                E = std::max(E, E1);
                htrace("pipe: part egress issued");
            }
            HIPCHK(hipStreamSynchronize(ctx->out_stream));
            egress_end = E;
        } catch (const DevError& e) {
            d2h_err = e.msg;
        } catch (const std::exception& e) {
            d2h_err = e.what();
        }
    });
    struct Join {  // the egress thread ends before this frame does, whatever throws
        std::thread& t;
        std::mutex& mu;
        std::condition_variable& cv;
        bool& stop;
        ~Join() {
            {
                std::lock_guard<std::mutex> g(mu);
                stop = true;
            }
            cv.notify_all();
            if (t.joinable()) t.join();
        }
    } joiner{egress, mu, cv, stop};
    // ---- ingest + kernels, part by part
    FxArgs Alast{};
    bool have_A = false;
    const char* fail_env = test_opt("SKV_TEST_FAIL_PART");  // tests: a failure after part p was queued
    const uint64_t fail_at = fail_env ? strtoull(fail_env, nullptr, 10) : ~0ull;
    for (uint64_t p = 0; p < P; ++p) {
        if (p == fail_at) throw DevError("injected failure before part " + std::to_string(p));
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t lo = p == 0 ? 0 : 1 + lb[p * nr + m] * S;
            const uint64_t hi = p + 1 == P ? job.run_len[m] : 1 + lb[(p + 1) * nr + m] * S;
            if (hi > lo)
                HIPCHK(hipMemcpyAsync(d_in + img[m] + lo, (const uint8_t*)(uintptr_t)job.run_ptr[m] + lo, hi - lo,
                                      hipMemcpyHostToDevice, ctx->in_stream));
        }
        HIPCHK(hipEventRecord(ctx->part_ev[2 * p], ctx->in_stream));
        HIPCHK(hipStreamWaitEvent(st, ctx->part_ev[2 * p], 0));
        if (pt.kp[p]) {
            FxPartIO io;
            io.gbase = p ? d_Kp + p - 1 : nullptr;
            io.Kout = d_Kp + p;
            io.flags = d_pflags;
            io.out = d_out;
            uint64_t* rb_unused = nullptr;
            Alast = fx_launch(ctx, pt.kp[p], pt.np[p], d_runs + p * nr, pt.sfr[p], f, pt.recb[p], n, out_cap, &io, rb_unused);
            have_A = true;
        } else if (p) {
            launch_copy_bytes(st, (uint8_t*)(d_Kp + p), (const uint8_t*)(d_Kp + p - 1), 8);
        }
        launch_fx_publish(st, d_Kp + p, (uint64_t*)hK + p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->part_ev[2 * p + 1], st));
        {
            std::lock_guard<std::mutex> g(mu);
            issued = p + 1;
        }
        cv.notify_one();
    }
    htrace("pipe: all parts queued");
    if (!have_A) throw DevError("internal: pipelined call without records");
    // ---- descriptors over the whole output, one readback with the verdict
    Alast.Kout = d_Kp + P - 1;
    launch_fx_desc(st, Alast, d_desc, d_prb, max_runs);
    HIPCHK(hipGetLastError());
    const uint64_t guess = std::min<uint64_t>(max_runs, 64 + job.in_bytes / (n * S));
    uint8_t* hp = (uint8_t*)pinned(ctx, 64 + guess * sizeof(DevRunDesc));
    d2h(ctx, hp, d_prb, 24);
    d2h(ctx, hp + 32, d_pflags, 16);
    d2h(ctx, hp + 64, d_desc, guess * sizeof(DevRunDesc));
    sync(ctx);
    {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
    }
    cv.notify_all();
    egress.join();
    htrace("pipe: egress done");
    uint32_t hf[4];
    memcpy(hf, hp + 32, 16);
    uint64_t h3[3];
    memcpy(h3, hp, 24);
    const uint64_t n_out = h3[0], Kt = h3[1];
    if (!d2h_err.empty()) {
        throw DevError("pipelined egress: " + d2h_err);
    }
    if (hf[2] || egress_end != h3[2] + n_out) {  // poisoned (or a part count the verdict rejects)
        used = false;
        ctx->timings.fused_reject = hf[3] ? hf[3] : 0x80000000u;
        return SKV_OK;
    }
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, n_out) * sizeof(skv_run_desc));
    memcpy(res->runs, hp + 64, std::min(n_out, guess) * sizeof(DevRunDesc));
    if (n_out > guess)
        HIPCHK(hipMemcpy(res->runs + guess, d_desc + guess, (n_out - guess) * sizeof(DevRunDesc), hipMemcpyDeviceToHost));
    res->n_runs = n_out;
    res->bytes = h_out;
    h_out = nullptr;  // the result owns it now
    res->n_bytes = h3[2] + n_out;
    res->in_bytes = job.in_bytes;
    res->in_records = R;
    res->out_records = Kt;
    res->dropped_tables = 0;
    box->pool = ctx->out_pool;
    box->pool_cap = cap;
    skv_timings& t = ctx->timings;
    t = skv_timings{};
    t.path = SKV_PATH_FUSED;
    t.hot_read_bytes = R * S;  // every input record is read once
    t.hot_write_bytes = res->n_bytes;
    t.host_syncs = ctx->syncs;
    t.host_total_ms = now_ms() - t_entry;
    t.host_parts = (uint32_t)P;
    *out = res;
    return SKV_OK;
}

// ---- the general key-range pipeline (variable-length records, Deletes) --------------------------
// skv_compact with host inputs that the fused pipeline does not take: the record framing of every
// run is walked on host threads (every G-th record start kept), P - 1 cut keys are quantiles of
// those records' keys, and each run is cut at its first record >= each cut key (equal keys never
// straddle a cut). Part p is then a compaction of its slices (compact_device in part mode: a
// slice's leading byte stands in for the version byte) on ctx->stream while the H2D of later parts
// runs on in_stream and the D2H of finished output on out_stream (its own host thread).
// build_runs' greedy split carries across parts exactly: part p also takes the previous parts'
// last (still open) output run -- a valid v1 run, already in the output buffer -- as one more input
// stream, and writes its output from that run's offset on. All open-run keys sort before part p's,
// so the merge puts them first unchanged and the split restarts at a true run boundary of the
// whole output; only the bytes before the open run are final, and those go back to the host. Any
// error, decrease across a cut or oversized open run ends the attempt; the serial path then gives
// the reference's exact outcome.
namespace {
constexpr uint64_t NPOS = ~0ull;
// the framing of one record at p (runs.rs:559-624 without the key's UTF-8, which the device checks):
// its size, or 0 when it does not decode
inline uint64_t host_rec_at(const uint8_t* b, uint64_t len, uint64_t p) {
    if (p + 5 > len) return 0;
    const uint8_t marker = b[p];
    const uint64_t klen = be32(b + p + 1), kp = p + 5;
    if (kp + klen > len) return 0;
    if (marker == 2) return 5 + klen;
    if (marker != 1 || kp + klen + 4 > len) return 0;
    const uint64_t vlen = be32(b + kp + klen);
    return kp + klen + 4 + vlen > len ? 0 : 9 + klen + vlen;
}
// Rust str Ord: bytewise, a proper prefix first
inline int host_key_cmp(const uint8_t* a, uint64_t al, const uint8_t* c, uint64_t cl) {
    const int r = memcmp(a, c, al < cl ? al : cl);
    return r ? r : (al < cl ? -1 : (al > cl ? 1 : 0));
}
inline int rec_vs(const uint8_t* b, uint64_t p, const std::string& c) {
    return host_key_cmp(b + p + 5, be32(b + p + 1), (const uint8_t*)c.data(), c.size());
}
// core::str::from_utf8 acceptance (runs.rs:585-591)
inline bool host_utf8(const uint8_t* s, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        const uint32_t c = s[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return false;
        if (n - i - 1 < need || s[i + 1] < lo || s[i + 1] > hi) return false;
        for (uint32_t q = 2; q <= need; ++q)
            if (s[i + q] < 0x80 || s[i + q] > 0xBF) return false;
        i += need + 1;
    }
    return true;
}
// A record start near byte x without walking the run from its start: the first p >= x from which
// RESYNC_N records decode with valid UTF-8 keys in strictly increasing order (or the run ends
// cleanly after fewer). The UTF-8 check matters: a value byte 1 followed by a length that fits the
// run makes one giant "record" whose end can land on a true record start, and its random-byte
// "key" sorts below the next key one time in five -- at config 3's scale such positions occur a few
// hundred times per 4 GB. A position that still passes but is not a true record start would put a
// slice boundary inside a record; the part's decode then fails and the call takes the serial path.
constexpr int RESYNC_N = 8;
constexpr uint64_t RESYNC_SPAN = 1u << 16;
inline bool plausible(const uint8_t* b, uint64_t len, uint64_t p) {
    uint64_t prev = NPOS;
    for (int i = 0; i < RESYNC_N && p < len; ++i) {
        const uint64_t sz = host_rec_at(b, len, p);
        if (!sz || !host_utf8(b + p + 5, be32(b + p + 1))) return false;
        if (prev != NPOS && host_key_cmp(b + prev + 5, be32(b + prev + 1), b + p + 5, be32(b + p + 1)) >= 0) return false;
        prev = p;
        p += sz;
    }
    return true;
}
inline uint64_t resync(const uint8_t* b, uint64_t len, uint64_t x) {
    const uint64_t e = std::min(len, x + RESYNC_SPAN);
    for (uint64_t p = x; p < e; ++p)
        if ((b[p] == 1 || b[p] == 2) && plausible(b, len, p)) return p;
    return NPOS;
}
// run m's first record with key >= c: bisection over resynced positions, then a walk of a few
// records from the last one below c. prev_ok: the record before it sorts below c.
inline uint64_t host_lower_bound(const uint8_t* b, uint64_t len, const std::string& c) {
    if (len <= 1) return len;
    if (rec_vs(b, 1, c) >= 0) return 1;
    uint64_t lo = 1, hi = len;  // lo: a record start below c; hi: at or past the bound
    while (hi - lo > 4096) {
        const uint64_t mid = lo + (hi - lo) / 2;
        const uint64_t q = resync(b, len, mid);
        if (q == NPOS || q >= hi) {
            hi = mid;
            continue;
        }
        if (rec_vs(b, q, c) < 0) lo = q;
        else hi = q;
    }
    uint64_t q = lo;
    while (q < len && rec_vs(b, q, c) < 0) {
        const uint64_t sz = host_rec_at(b, len, q);
        if (!sz) return NPOS;  // not decodable here: the serial path
        q += sz;
    }
    return q;
}
// "{id}." at the start of key k when id is a canonical Rust i64 Display text (the prefix
// wal_compaction.rs strips is format!("{id}."), :76-98): its length, else 0
inline uint64_t wal_canon_prefix(const uint8_t* k, uint64_t n) {
    uint64_t i = 0;
    if (i < n && k[i] == '-') ++i;
    const uint64_t d0 = i;
    while (i < n && k[i] >= '0' && k[i] <= '9') ++i;
    const uint64_t nd = i - d0;
    if (nd == 0 || nd > 19 || i >= n || k[i] != '.') return 0;
    if (nd > 1 && k[d0] == '0') return 0;    // leading zero
    if (d0 && nd == 1 && k[d0] == '0') return 0;  // "-0"
    if (nd == 19 && memcmp(k + d0, d0 ? "9223372036854775808" : "9223372036854775807", 19) > 0) return 0;
    return i + 1;
}
}  // namespace

// Key-range cuts of a general pipelined call: every member run m is cut at its first record >= each
// cut key. bnd[p * nr + m] is that byte offset (1 and len at the ends). Small runs are walked once
// for all cuts; large ones bisect over resynced positions (host_lower_bound). False: a run that does
// not decode where the cut search looked, or cuts that come out of order (the serial path then).
static bool cut_runs(const Job& job, const std::vector<std::string>& cut, uint64_t P, std::vector<uint64_t>& bnd) {
    const uint64_t nr = job.run_ptr.size();
    bnd.assign((P + 1) * nr, 0);
    const unsigned nb = std::max(1u, std::min<unsigned>(16, (unsigned)((nr + 63) / 64)));
    std::vector<uint8_t> ok(nb, 1);
    par_run(nr, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
        for (uint64_t m = lo; m < hi && ok[b]; ++m) {
            const uint8_t* rb = (const uint8_t*)(uintptr_t)job.run_ptr[m];
            const uint64_t len = job.run_len[m];
            bnd[m] = 1;
            bnd[P * nr + m] = len;
            if (len <= (1u << 16)) {  // one walk over the run finds every cut
                uint64_t q = 1;
                for (uint64_t p = 1; p < P; ++p) {
                    while (q < len) {
                        const uint64_t sz = host_rec_at(rb, len, q);
                        if (!sz) {
                            ok[b] = 0;
                            break;
                        }
                        if (rec_vs(rb, q, cut[p - 1]) >= 0) break;
                        q += sz;
                    }
                    bnd[p * nr + m] = q;
                }
            } else {
                for (uint64_t p = 1; p < P; ++p) {
                    const uint64_t q = host_lower_bound(rb, len, cut[p - 1]);
                    if (q == NPOS || q < bnd[(p - 1) * nr + m]) ok[b] = 0;
                    bnd[p * nr + m] = q;
                }
            }
        }
    });
    for (uint8_t o : ok)
        if (!o) return false;
    return true;
}

// A stream of several member runs (an L0 or next-level concatenation, table_buffer_compaction.rs:
// 66-100, table_tree_compaction.rs:103-135) is cut member by member; that is a key range of the
// stream only when the concatenation ascends: every record of member i below member i + 1's first
// key (checked here, empty members skipped; each member's own order is checked by the parts).
static bool members_ascend(const Job& job) {
    std::vector<std::pair<uint64_t, uint64_t>> pairs;  // (member i, member j): the next non-empty one
    for (const InStream& s : job.ranked) {
        uint64_t prev = NPOS;
        for (uint64_t r = s.first; r < s.first + s.n_runs; ++r) {
            if (job.run_len[r] <= 1) continue;
            if (prev != NPOS) pairs.emplace_back(prev, r);
            prev = r;
        }
    }
    if (pairs.empty()) return true;
    const unsigned nb = std::max(1u, std::min<unsigned>(16, (unsigned)((pairs.size() + 15) / 16)));
    std::vector<uint8_t> ok(nb, 1);
    par_run(pairs.size(), nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
        for (uint64_t x = lo; x < hi && ok[b]; ++x) {
            const uint64_t i = pairs[x].first, j = pairs[x].second;
            const uint8_t* bj = (const uint8_t*)(uintptr_t)job.run_ptr[j];
            if (!host_rec_at(bj, job.run_len[j], 1)) {
                ok[b] = 0;
                break;
            }
            const std::string f((const char*)bj + 6, be32(bj + 2));
            const uint8_t* bi = (const uint8_t*)(uintptr_t)job.run_ptr[i];
            if (host_lower_bound(bi, job.run_len[i], f) != job.run_len[i]) ok[b] = 0;
        }
    });
    for (uint8_t o : ok)
        if (!o) return false;
    return true;
}

// Cut keys of a general key-range split: quantiles of records found at evenly spaced offsets of the
// whole input (about 8192 samples whatever the fan-in: a WAL flush of 10^6 tiny runs samples a subset
// of them); P - 1 of them, fewer when samples repeat. WAL flushes cut at canonical table prefixes.
static bool sample_cuts(const Job& job, bool wal, uint64_t P, std::vector<std::string>& cut) {
    const uint64_t nr = job.run_ptr.size();
    auto run_b = [&](uint64_t m) { return (const uint8_t*)(uintptr_t)job.run_ptr[m]; };
    std::vector<uint64_t> rpre(nr + 1, 0);
    for (uint64_t m = 0; m < nr; ++m) rpre[m + 1] = rpre[m] + job.run_len[m];
    const uint64_t NS = 8192;
    std::vector<std::pair<const uint8_t*, uint64_t>> smp(NS, {nullptr, 0});
    par_run(NS, 16, [&](unsigned, uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) {
            const uint64_t g = (2 * i + 1) * rpre[nr] / (2 * NS);
            const uint64_t m = (uint64_t)(std::upper_bound(rpre.begin(), rpre.end(), g) - rpre.begin()) - 1;
            const uint8_t* rb = run_b(m);
            const uint64_t len = job.run_len[m];
            const uint64_t q = resync(rb, len, std::max<uint64_t>(1, g - rpre[m]));
            if (q == NPOS || q >= len) continue;
            const uint64_t kl = be32(rb + q + 1);
            if (wal) {
                const uint64_t pl = wal_canon_prefix(rb + q + 5, kl);
                if (pl) smp[i] = {rb + q + 5, pl};
            } else {
                smp[i] = {rb + q + 5, kl};
            }
        }
    });
    smp.erase(std::remove_if(smp.begin(), smp.end(), [](const auto& e) { return e.first == nullptr; }), smp.end());
    htrace("gpipe: sampled");
    if (smp.size() < P) {
        htrace("gpipe: too few samples");
        return false;
    }
    std::sort(smp.begin(), smp.end(), [](const auto& a, const auto& c) {
        return host_key_cmp(a.first, a.second, c.first, c.second) < 0;
    });
    cut.clear();
    for (uint64_t p = 1; p < P; ++p) {
        const auto& e = smp[p * smp.size() / P];
        std::string c((const char*)e.first, e.second);
        if (cut.empty() || cut.back() < c) cut.push_back(c);  // (Rust str order = bytewise = std::string's)
    }
    return true;
}

static int compact_host_pipelined_general(skv_ctx* ctx, Job& job, skv_result** out, double t_entry, bool& used) {
    used = false;
    const char* pe = getenv("SKV_HOST_PIPE");
    if (pe && pe[0] == '0') return SKV_OK;
    const char* me = getenv("SKV_HOST_PIPE_MIN");
    const uint64_t min_bytes = me ? strtoull(me, nullptr, 10) : (512ull << 20);
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t nr = job.run_ptr.size();
    const bool wal = (job.flags & SKV_SPLIT_BY_TABLE) != 0;
    if (job.in_bytes < min_bytes || job.batch || job.search || job.scan) return SKV_OK;
    if (k == 0 || nr == 0) return SKV_OK;
    // Past 2^16 member runs (a WAL flush of 10^6 tiny runs) the call takes the serial path: a walk of
    // every run up to its last cut costs what the transfers do (125-147 ms on 8 threads for config 5,
    // against ~80 ms for the whole H2D), and the parts' 10^6 scattered slices move at ~26-30 GB/s (the
    // GPU reading pinned memory) against ~56 GB/s for one DMA copy of the whole input. Round 5 built
    // a pipeline for them (a fixed-stride cut search, cut rows found while the GPU ingests) and
    // measured it slower (235-300 vs 169 ms, profiles/r05/c5_host.txt); round 6 removed it.
    if (nr > (1u << 16)) return SKV_OK;
    // parts of ~1 GiB: each part costs a DMA copy per slice (config 3, 3.7 GiB: 4 parts 99.8 ms, 6
    // parts 102.9, 8 parts 105.0, 10 parts 110.5)
    uint64_t P = std::max<uint64_t>(2, std::min<uint64_t>(32, job.in_bytes / (1ull << 30)));
    if (const char* pp = getenv("SKV_HOST_PARTS")) P = std::max<uint64_t>(1, std::min<uint64_t>(256, strtoull(pp, nullptr, 10)));
    // the open output run is carried into every part (not for WAL flushes, whose parts hold whole
    // tables): keep it small against a part
    if (P < 2 || (!wal && job.max_run_size > job.in_bytes / (4 * P))) return SKV_OK;
    auto run_b = [&](uint64_t m) { return (const uint8_t*)(uintptr_t)job.run_ptr[m]; };
    for (uint64_t m = 0; m < nr; ++m)  // a run without a version byte: the serial path's error
        if (job.run_len[m] == 0 || run_b(m)[0] != 1) return SKV_OK;
    // ---- cut keys: quantiles of records found at evenly spaced offsets of the whole input (about
    // 8192 samples whatever the fan-in: a WAL flush of 10^6 tiny runs samples a subset of them).
    // WAL flushes cut at canonical table prefixes "{id}.": every key of a table sorts at or after
    // its prefix and before the next table's, so a part holds whole tables (the one-run rule and the
    // prefix strip stay per table); a key that is not canonical ends the attempt in its part.
    std::vector<std::string> cut;
    if (!sample_cuts(job, wal, P, cut)) return SKV_OK;
    P = cut.size() + 1;
    if (P < 2 || (!wal && job.max_run_size > job.in_bytes / (4 * P))) return SKV_OK;
    // ---- bnd[p * nr + m]: byte offset of run m's first record >= cut p (1 / len at the ends)
    std::vector<uint64_t> bnd;
    if (!cut_runs(job, cut, P, bnd)) {
        htrace("gpipe: a cut not found");
        return SKV_OK;
    }
    if (!members_ascend(job)) {
        htrace("gpipe: member runs overlap");
        return SKV_OK;
    }
    // ---- ingest mode: one DMA copy per non-empty slice while the call has few enough of them, else
    // (and with SKV_INGEST=kernel) the GPU copies each part's slices itself from pinned, device-mapped
    // host memory (k_ingest, one launch per part). The copy kernels measured slower on config 3 (8 parts:
    // 130 vs 105 ms: part 0's kernels waited behind the later parts' ingest); a WAL flush of 10^6 tiny
    // runs has millions of slices, each a DMA descriptor with its own fixed cost.
    uint64_t n_slices = 0;
    for (uint64_t p = 0; p < P; ++p)
        for (uint64_t m = 0; m < nr; ++m) n_slices += bnd[(p + 1) * nr + m] > bnd[p * nr + m];
    std::vector<uint64_t> hdev;
    bool kernel_ingest = n_slices > (1u << 15);
    {
        const char* ie = test_opt("SKV_INGEST");
        if (ie && !strcmp(ie, "kernel")) kernel_ingest = true;
        if (kernel_ingest) {
            hdev.assign(nr, 0);
            for (uint64_t m = 0; m < nr && kernel_ingest; ++m) {
                hipPointerAttribute_t a;
                if (hipPointerGetAttributes(&a, run_b(m)) != hipSuccess) {
                    (void)hipGetLastError();
                    kernel_ingest = false;
                } else if (a.type != hipMemoryTypeHost || !a.devicePointer) {
                    kernel_ingest = false;
                } else {
                    hdev[m] = (uint64_t)(uintptr_t)a.devicePointer;
                }
            }
            if (!kernel_ingest && n_slices > (1u << 15)) {
                htrace("gpipe: too many slices for DMA copies, runs not device-mapped");
                return SKV_OK;
            }
        }
    }
    htrace("gpipe: cuts");
    used = true;
    PipeIO kio(ctx);
    if (!ctx->in_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->in_stream, hipStreamNonBlocking));
    if (!ctx->out_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->out_stream, hipStreamNonBlocking));
    while (ctx->part_ev.size() < 2 * P) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->part_ev.push_back(e);
    }
    // ---- device images of the runs (each congruent mod 16 with its host bytes); the shared output
    std::vector<uint64_t> img(nr + 1, 0);
    for (uint64_t m = 0; m < nr; ++m) img[m + 1] = img[m] + ((job.run_len[m] + 31) & ~15ull);
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", img[nr] + 16);
    for (uint64_t m = 0; m < nr; ++m) img[m] += ((uint64_t)(uintptr_t)run_b(m) & 15);  // 16-aligned base + skew
    const uint64_t R = job.in_bytes / 5 + 1;  // records: at most one per 5 bytes (sizes only)
    const uint64_t out_cap = job.in_bytes + R + 64;
    uint8_t* d_out = dbuf<uint8_t>(ctx, "gp_out", out_cap);
    size_t cap = 0;
    uint8_t* h_out = (uint8_t*)ctx->out_pool->take(out_cap, cap);
    if (!h_out) throw DevError("pinned host allocation of the output failed");
    struct OutGuard {  // as in compact_host_pipelined: drain the copies, then the buffer back
        skv_ctx* c;
        uint8_t*& buf;
        size_t cap;
        ~OutGuard() {
            if (c->in_stream) (void)hipStreamSynchronize(c->in_stream);
            if (c->out_stream) (void)hipStreamSynchronize(c->out_stream);
            (void)hipStreamSynchronize(c->stream);
            if (buf) c->out_pool->give(buf, cap);
        }
    } out_guard{ctx, h_out, cap};
    // ---- ingest: every part's slices, in part order, on in_stream. Kernel ingest: part p's slice
    // table is built on the host pool into the ctx's pinned slice arena and goes up on in_stream right
    // before part p's ingest launch.
    IngestSlice* d_sl = nullptr;
    std::vector<uint64_t> sl_base(P + 1, 0);
    IngestSlice* h_sl = nullptr;
    if (kernel_ingest) {
        // capacity: one slice per (part, run) -- part 0's slices start at the version byte, so a run
        // whose part-0 key range is empty still has one (n_slices does not count those)
        d_sl = dbuf<IngestSlice>(ctx, "gp_slices", P * nr + 1);
        const size_t need = (P * nr + 1) * sizeof(IngestSlice);
        if (ctx->sl_cap < need) {
            if (ctx->sl_host) ctx->host_graveyard.push_back(ctx->sl_host);  // (defer_free: kio above)
            ctx->sl_host = nullptr;
            ctx->sl_cap = 0;
            HIPCHK(host_alloc_near(ctx->device, &ctx->sl_host, need, hipHostMallocDefault));
            ctx->sl_cap = need;
        }
        h_sl = (IngestSlice*)ctx->sl_host;
    }
    // a few hundred ingest workgroups in all: the copies are bound by PCIe, and a grid that filled
    // every CU (8 per slice: 2,048 at config 3) held the part kernels off the GPU until the whole
    // input had landed (part 0 finished after 77 ms, parts 1-7 in 3 ms each behind it)
    const uint32_t igrid = 384;
    for (uint64_t p = 0; p < P; ++p) {
        if (kernel_ingest) {
            const unsigned nb = par_nblocks(nr, 1u << 14);
            std::vector<uint64_t> cnt(nb + 1, 0);
            auto slice = [&](uint64_t m, uint64_t& lo, uint64_t& hi) {
                lo = p == 0 ? 0 : bnd[p * nr + m];
                hi = bnd[(p + 1) * nr + m];
            };
            par_run(nr, nb, [&](unsigned b, uint64_t lo_m, uint64_t hi_m) {
                uint64_t c = 0;
                for (uint64_t m = lo_m; m < hi_m; ++m) {
                    uint64_t lo, hi;
                    slice(m, lo, hi);
                    c += hi > lo;
                }
                cnt[b + 1] = c;
            });
            for (unsigned b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
            sl_base[p + 1] = sl_base[p] + cnt[nb];
            IngestSlice* out_sl = h_sl + sl_base[p];
            par_run(nr, nb, [&](unsigned b, uint64_t lo_m, uint64_t hi_m) {
                uint64_t at = cnt[b];
                for (uint64_t m = lo_m; m < hi_m; ++m) {
                    uint64_t lo, hi;
                    slice(m, lo, hi);
                    if (hi > lo) out_sl[at++] = IngestSlice{hdev[m] + lo, (uint64_t)(uintptr_t)(d_in + img[m] + lo), hi - lo};
                }
            });
            const uint64_t ns = sl_base[p + 1] - sl_base[p];
            if (ns)
                HIPCHK(hipMemcpyAsync(d_sl + sl_base[p], out_sl, ns * sizeof(IngestSlice), hipMemcpyHostToDevice,
                                      ctx->in_stream));
            launch_ingest_slices(ctx->in_stream, d_sl + sl_base[p], ns, igrid);
            HIPCHK(hipGetLastError());
        } else {
            for (uint64_t m = 0; m < nr; ++m) {
                const uint64_t lo = p == 0 ? 0 : bnd[p * nr + m], hi = bnd[(p + 1) * nr + m];
                if (hi > lo)
                    HIPCHK(hipMemcpyAsync(d_in + img[m] + lo, run_b(m) + lo, hi - lo, hipMemcpyHostToDevice, ctx->in_stream));
            }
        }
        HIPCHK(hipEventRecord(ctx->part_ev[2 * p], ctx->in_stream));
        if (p == 0) htrace("gpipe: part 0 queued");
    }
    htrace("gpipe: ingest queued");
    // ---- egress thread: D2H of every byte range the parts finalize
    std::mutex mu;
    std::condition_variable cv;
    uint64_t final_end = 0;
    bool stop = false, done = false;
    std::string d2h_err;
    std::thread egress([&] {
        try {
            if (hipSetDevice(ctx->device) != hipSuccess) throw DevError("hipSetDevice failed (egress)");
            uint64_t E = 0;
            for (;;) {
                uint64_t F;
                bool last;
                {
                    std::unique_lock<std::mutex> g(mu);
                    cv.wait(g, [&] { return final_end > E || done || stop; });
                    if (stop) break;
                    F = final_end;
                    last = done;
                }
                if (F > E) HIPCHK(hipMemcpyAsync(h_out + E, d_out + E, F - E, hipMemcpyDeviceToHost, ctx->out_stream));
                E = F;
                if (last && E == F) break;
            }
            HIPCHK(hipStreamSynchronize(ctx->out_stream));
        } catch (const DevError& e) {
            d2h_err = e.msg;
        } catch (const std::exception& e) {
            d2h_err = e.what();
        }
    });
    struct Join {
        std::thread& t;
        std::mutex& mu;
        std::condition_variable& cv;
        bool& stop;
        ~Join() {
            {
                std::lock_guard<std::mutex> g(mu);
                stop = true;
            }
            cv.notify_all();
            if (t.joinable()) t.join();
        }
    } joiner{egress, mu, cv, stop};
    // ---- the parts, in key order, on ctx->stream
    int64_t seq_extra = INT64_MIN;  // the open run's stream: any SeqNo unused by the job
    {
        std::vector<int64_t> seqs;
        for (const InStream& S : job.ranked) seqs.push_back(S.seq);
        std::sort(seqs.begin(), seqs.end());
        while (std::binary_search(seqs.begin(), seqs.end(), seq_extra)) ++seq_extra;
    }
    std::vector<skv_run_desc> descs;
    uint64_t open_off = 0, open_len = 0, open_recs = 0, out_records = 0, in_records = 0, dropped = 0;
    uint64_t wal_off = 0;  // WAL flushes: output bytes of the parts so far (every part's tables are final)
    uint64_t syncs = 0;
    std::vector<const uint8_t*> ptrs;
    std::vector<uint64_t> lens;
    std::vector<skv_stream> sv;
    for (uint64_t p = 0; p < P; ++p) {
        // part p's streams: each stream's member slices in member order (empty ones left out), the
        // streams in rank order, then the carried open run
        ptrs.clear();
        lens.clear();
        sv.clear();
        std::vector<std::pair<int64_t, uint64_t>> sfirst;  // (seq, first slice) per non-empty stream
        for (uint32_t s = 0; s < k; ++s) {
            const InStream& S = job.ranked[s];
            const uint64_t f0 = ptrs.size();
            for (uint64_t m = S.first; m < S.first + S.n_runs; ++m) {
                const uint64_t lo = bnd[p * nr + m], hi = bnd[(p + 1) * nr + m];
                if (hi <= lo) continue;
                ptrs.push_back(d_in + img[m] + lo - 1);  // the byte before the slice: its "version byte"
                lens.push_back(1 + hi - lo);
            }
            if (ptrs.size() > f0) sfirst.emplace_back(S.seq, f0);
        }
        if (open_len) {
            sfirst.emplace_back(seq_extra, ptrs.size());
            ptrs.push_back(d_out + open_off);
            lens.push_back(open_len);
        }
        const bool last_part = p + 1 == P;
        if (sfirst.empty()) {  // no records in this key range
            if (last_part) {
                std::lock_guard<std::mutex> g(mu);
                final_end = wal ? wal_off : (descs.empty() ? 0 : descs.back().off + descs.back().len);
                done = true;
            }
            cv.notify_all();
            continue;
        }
        for (size_t i = 0; i < sfirst.size(); ++i) {
            const uint64_t a = sfirst[i].second, z = i + 1 < sfirst.size() ? sfirst[i + 1].second : ptrs.size();
            sv.push_back(skv_stream{&ptrs[a], &lens[a], (uint32_t)(z - a), sfirst[i].first});
        }
        Job pj;
        if (build_job(ctx, sv.data(), (uint32_t)sv.size(), job.max_run_size, job.flags, pj) != SKV_OK)
            throw DevError("internal: part job: " + ctx->err);
        pj.part = true;
        pj.dev_out = d_out + (wal ? wal_off : open_off);
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->part_ev[2 * p], 0));
        if (getenv("SKV_HOST_TRACE")) {  // diagnostics: when part p's slices have landed
            HIPCHK(hipEventSynchronize(ctx->part_ev[2 * p]));
            htrace("gpipe: part ingested");
        }
        skv_result* pres = nullptr;
        int rc;
        try {
            rc = compact_device(ctx, pj, &pres, true);
        } catch (const ApiError&) {
            rc = -1;  // a data error: the serial path reports it exactly
        }
        syncs += ctx->syncs;
        if (rc != SKV_OK) {
            drain(ctx);
            used = false;
            return SKV_OK;
        }
        const uint64_t n = pres->n_runs;
        if (wal) {
            // whole tables: every run of the part is final at its offset in the call's output
            for (uint64_t r = 0; r < n; ++r) {
                skv_run_desc d = pres->runs[r];
                d.off += wal_off;
                d.min_key_off += wal_off;
                d.max_key_off += wal_off;
                descs.push_back(d);
                out_records += d.put_count + d.delete_count;
            }
            in_records += pres->in_records;
            dropped += pres->dropped_tables;
            wal_off += pres->n_bytes;
            skv_result_free(pres);
            {
                std::lock_guard<std::mutex> g(mu);
                final_end = wal_off;
                done = last_part;
            }
            cv.notify_all();
            htrace("gpipe: part done");
            continue;
        }
        // Part p read the carried open run at d_out + open_off while writing its own output from that
        // same address. That is safe because the merge re-emits the open run first and unchanged --
        // every key of it sorts before every key of part p, and it is under max_run_size, so
        // build_runs keeps it whole as (the start of) part p's first run: each output byte the part
        // writes there is the byte it read. Checked: part p's first run starts at the open run's offset
        // and holds at least its bytes; anything else would mean the input was overwritten.
        if (open_len && (n == 0 || pres->runs[0].off != 0 || pres->runs[0].len < open_len)) {
            const std::string why = "internal: general pipeline part " + std::to_string(p) +
                                    " did not re-emit the open run (runs " + std::to_string(n) + ", first at " +
                                    std::to_string(n ? pres->runs[0].off : 0) + " len " +
                                    std::to_string(n ? pres->runs[0].len : 0) + ", open run " + std::to_string(open_off) +
                                    " len " + std::to_string(open_len) + ")";
            skv_result_free(pres);
            throw DevError(why);
        }
        in_records += pres->in_records - (open_len ? open_recs : 0);  // the carried run's records once
        for (uint64_t r = 0; r < n; ++r) {
            skv_run_desc d = pres->runs[r];
            d.off += open_off;
            d.min_key_off += open_off;
            d.max_key_off += open_off;
            if (!last_part && r + 1 == n) {  // still open: carried into the next part
                open_off = d.off;
                open_len = d.len;
                open_recs = d.put_count + d.delete_count;
                break;
            }
            descs.push_back(d);
            out_records += d.put_count + d.delete_count;
        }
        if (!n) open_len = 0;  // (nothing so far: no open run)
        skv_result_free(pres);
        {
            std::lock_guard<std::mutex> g(mu);
            final_end = last_part ? (descs.empty() ? 0 : descs.back().off + descs.back().len) : open_off;
            done = last_part;
        }
        cv.notify_all();
        htrace("gpipe: part done");
    }
    egress.join();
    if (!d2h_err.empty()) throw DevError("pipelined egress: " + d2h_err);
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(std::max<size_t>(1, descs.size()) * sizeof(skv_run_desc));
    if (!descs.empty()) memcpy(res->runs, descs.data(), descs.size() * sizeof(skv_run_desc));
    res->n_runs = descs.size();
    res->bytes = h_out;
    h_out = nullptr;  // the result owns it now
    res->n_bytes = wal ? wal_off : (descs.empty() ? 0 : descs.back().off + descs.back().len);
    res->in_bytes = job.in_bytes;
    res->in_records = in_records;
    res->out_records = out_records;
    res->dropped_tables = dropped;
    box->pool = ctx->out_pool;
    box->pool_cap = cap;
    skv_timings& t = ctx->timings;
    t = skv_timings{};
    t.path = SKV_PATH_GENERAL;
    t.host_syncs = syncs;
    t.host_total_ms = now_ms() - t_entry;
    t.host_parts = (uint32_t)P;
    t.wal_stage = wal ? 1 : 0;
    *out = res;
    return SKV_OK;
}

// ---- skv_compact_split for variable-length records -----------------------------
// The call is cut into P key-range parts (sample_cuts / cut_runs, as the general pipeline) dealt
// round-robin over the ctxs. Each ctx's worker stages its parts' slices (in_stream, all queued up
// front) and compacts them one by one in part mode, each into its own region of the ctx's output
// buffer. The merges run in parallel on the GPUs; build_runs' greedy split (runs.rs:211-238) does
// not, so each part's split waits inside compact_device (Job::carry) for the open run the previous
// part left, and hands its own on as soon as its split is done (the serial chain SURVEY §8(e)
// describes: one split pass per part, each a few ms, while later parts still merge). A part whose
// first run continues the carried run writes it after a version byte that is not copied out; its
// descriptor is merged into the previous part's last. Once the output bytes of every earlier part
// are known, a part's bytes go D2H to their place in the one pinned output (out_stream).
namespace {
struct GSplit : CarryHook {
    uint64_t P = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> carry;    // carry[p + 1]: the open run part p leaves (bytes; carry[0] = 0)
    std::vector<uint8_t> have_c;    // carry[p] committed (the next part may split)
    // what compact_device posts at its split (post_out) is only staged: a part can rerun after its
    // split (a deferred verification that fails, a fingerprint collision) and post again; its
    // worker commits the value once the part's result is final
    std::vector<uint64_t> carry_st;
    std::vector<uint8_t> staged;
    std::vector<uint8_t> cont;      // part p's run 0 continues the carried run
    std::vector<uint64_t> nbytes;   // part p's output bytes (after the dropped version byte)
    std::vector<uint8_t> have_b;
    std::vector<uint64_t> off;      // off[p]: output bytes of parts < p, valid for p <= prefix
    uint64_t prefix = 0;
    bool stop = false, data_err = false;
    std::string err;
    std::vector<std::vector<skv_run_desc>> descs;  // part p's runs, offsets already global
    std::vector<uint64_t> in_recs, dropped;
    bool wal = false;  // WAL flush: parts hold whole tables, nothing is carried

    bool wait_in(uint64_t part, uint64_t& c) override {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || have_c[part]; });
        if (stop) return false;
        c = carry[part];
        return true;
    }
    void post_out(uint64_t part, uint64_t c, bool is_cont) override {
        std::lock_guard<std::mutex> g(mu);
        carry_st[part + 1] = c;
        staged[part + 1] = 1;
        cont[part] = is_cont ? 1 : 0;
    }
    void commit(uint64_t part) {
        {
            std::lock_guard<std::mutex> g(mu);
            carry[part + 1] = carry_st[part + 1];
            have_c[part + 1] = 1;
        }
        cv.notify_all();
    }
    void post_bytes(uint64_t part, uint64_t n) {
        {
            std::lock_guard<std::mutex> g(mu);
            nbytes[part] = n;
            have_b[part] = 1;
            while (prefix < P && have_b[prefix]) {
                off[prefix + 1] = off[prefix] + nbytes[prefix];
                ++prefix;
            }
        }
        cv.notify_all();
    }
    bool wait_off(uint64_t part, uint64_t& o) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || prefix >= part; });
        if (stop) return false;
        o = off[part];
        return true;
    }
    void halt(bool data, const std::string& e) {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            data_err = data_err || data;
            if (!e.empty() && err.empty()) err = e;
        }
        cv.notify_all();
    }
};

void gsplit_worker(GSplit& gs, skv_ctx* ctx, uint64_t g, uint64_t G, const Job& job, const std::vector<uint64_t>& bnd,
                   uint8_t* h_out, uint64_t out_cap) {
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t nr = job.run_ptr.size(), P = gs.P;
    std::vector<uint64_t> parts;
    for (uint64_t p = g; p < P; p += G) parts.push_back(p);
    if (parts.empty()) return;
    const uint64_t np = parts.size();
    auto run_b = [&](uint64_t m) { return (const uint8_t*)(uintptr_t)job.run_ptr[m]; };
    PipeIO kio(ctx);  // as in compact_host_pipelined_general
    if (!ctx->in_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->in_stream, hipStreamNonBlocking));
    if (!ctx->out_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->out_stream, hipStreamNonBlocking));
    while (ctx->part_ev.size() < np) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->part_ev.push_back(e);
    }
    // this ctx's slices only: slice (i, m) = run m's bytes [lo - 1, hi) of part i (the byte before
    // the slice stands in for its version byte), at d_in + soff[i * nr + m], congruent mod 16 with
    // its host bytes; the output regions of its parts (a part writes at most its record bytes plus
    // a version byte per record of >= 5 bytes)
    std::vector<uint64_t> soff(np * nr, 0), ocap(np, 0);
    uint64_t in_total = 0, out_total = 0;
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t p = parts[i];
        uint64_t pb = 0;
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t lo = bnd[p * nr + m] - 1, hi = bnd[(p + 1) * nr + m];
            if (hi <= lo + 1) continue;
            in_total = ((in_total + 15) & ~15ull) + (((uint64_t)(uintptr_t)run_b(m) + lo) & 15);
            soff[i * nr + m] = in_total;
            in_total += hi - lo;
            pb += hi - lo - 1;
        }
        ocap[i] = (pb + pb / 5 + 64 + 255) & ~255ull;
        out_total += ocap[i];
    }
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", in_total + 32);
    uint8_t* d_out = dbuf<uint8_t>(ctx, "gs_out", out_total + 256);
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t p = parts[i];
        for (uint64_t m = 0; m < nr; ++m) {
            const uint64_t lo = bnd[p * nr + m] - 1, hi = bnd[(p + 1) * nr + m];
            if (hi > lo + 1)
                HIPCHK(hipMemcpyAsync(d_in + soff[i * nr + m], run_b(m) + lo, hi - lo, hipMemcpyHostToDevice,
                                      ctx->in_stream));
        }
        HIPCHK(hipEventRecord(ctx->part_ev[i], ctx->in_stream));
    }
    uint64_t dev_off = 0;
    std::vector<const uint8_t*> ptrs;
    std::vector<uint64_t> lens;
    std::vector<skv_stream> sv;
    for (uint64_t i = 0; i < np; ++i) {
        const uint64_t p = parts[i];
        ptrs.clear();
        lens.clear();
        sv.clear();
        std::vector<std::pair<int64_t, uint64_t>> sfirst;
        for (uint32_t s = 0; s < k; ++s) {
            const InStream& S = job.ranked[s];
            const uint64_t f0 = ptrs.size();
            for (uint64_t m = S.first; m < S.first + S.n_runs; ++m) {
                const uint64_t lo = bnd[p * nr + m], hi = bnd[(p + 1) * nr + m];
                if (hi <= lo) continue;
                ptrs.push_back(d_in + soff[i * nr + m]);
                lens.push_back(1 + hi - lo);
            }
            if (ptrs.size() > f0) sfirst.emplace_back(S.seq, f0);
        }
        if (sfirst.empty()) {  // no records in this key range: the carried run passes through
            uint64_t c = 0;
            if (!gs.wal) {
                if (!gs.wait_in(p, c)) return;
                gs.post_out(p, c, false);
                gs.commit(p);
            }
            gs.in_recs[p] = 0;
            gs.post_bytes(p, 0);
            continue;
        }
        for (size_t q = 0; q < sfirst.size(); ++q) {
            const uint64_t a = sfirst[q].second, z = q + 1 < sfirst.size() ? sfirst[q + 1].second : ptrs.size();
            sv.push_back(skv_stream{&ptrs[a], &lens[a], (uint32_t)(z - a), sfirst[q].first});
        }
        Job pj;
        if (build_job(ctx, sv.data(), (uint32_t)sv.size(), job.max_run_size, job.flags, pj) != SKV_OK)
            throw DevError("internal: split part job: " + ctx->err);
        pj.part = true;
        pj.dev_out = d_out + dev_off;
        pj.carry = gs.wal ? nullptr : &gs;
        pj.carry_part = p;
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->part_ev[i], 0));
        skv_result* pres = nullptr;
        int rc;
        try {
            rc = compact_device(ctx, pj, &pres, true);
        } catch (const ApiError&) {
            rc = -1;  // a data error: the serial path reports it exactly
        }
        if (rc != SKV_OK) {
            if (pres) skv_result_free(pres);
            gs.halt(true, "");
            return;
        }
        if (!gs.wal) {  // the part's result is final: its open run goes to the next part
            bool posted;
            {
                std::lock_guard<std::mutex> lk(gs.mu);
                posted = gs.staged[p + 1] != 0;
            }
            uint64_t c = 0;
            if (!posted) {  // it never reached the split (no runs): the carried run passes through
                if (!gs.wait_in(p, c)) {
                    skv_result_free(pres);
                    return;
                }
                gs.post_out(p, c, false);
            }
            gs.commit(p);
        }
        bool is_cont;
        {
            std::lock_guard<std::mutex> lk(gs.mu);
            is_cont = gs.cont[p] != 0;
        }
        const uint64_t skip = is_cont ? 1 : 0;  // the continuation's version byte stays behind
        const uint64_t n = pres->n_runs, nb = pres->n_bytes;
        if (is_cont && (n == 0 || pres->runs[0].off != 0)) {
            skv_result_free(pres);
            throw DevError("internal: split part " + std::to_string(p) + " lost its continuation run");
        }
        gs.in_recs[p] = pres->in_records;
        gs.dropped[p] = pres->dropped_tables;
        gs.post_bytes(p, nb - skip);
        uint64_t O = 0;
        if (!gs.wait_off(p, O)) {
            skv_result_free(pres);
            return;
        }
        if (O + (nb - skip) > out_cap) {
            skv_result_free(pres);
            throw DevError("internal: split output past its buffer");
        }
        if (nb > skip)
            HIPCHK(hipMemcpyAsync(h_out + O, (const uint8_t*)pres->bytes + skip, nb - skip, hipMemcpyDeviceToHost,
                                  ctx->out_stream));
        std::vector<skv_run_desc> ds(pres->runs, pres->runs + n);
        for (skv_run_desc& d : ds) {  // part-relative -> global (the dropped byte before them all)
            d.off = d.off + O - skip;
            d.min_key_off = d.min_key_off + O - skip;
            d.max_key_off = d.max_key_off + O - skip;
        }
        {
            std::lock_guard<std::mutex> lk(gs.mu);
            gs.descs[p] = std::move(ds);
        }
        skv_result_free(pres);
        dev_off += ocap[i];
    }
    HIPCHK(hipStreamSynchronize(ctx->out_stream));
}
}  // namespace

int compact_split_general(skv_ctx* const* ctxs, uint32_t G, Job& job, skv_result** out, double t_entry, bool& used) {
    used = false;
    skv_ctx* home = ctxs[0];
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t nr = job.run_ptr.size();
    const bool wal = (job.flags & SKV_SPLIT_BY_TABLE) != 0;
    if (job.batch || job.search || job.scan || k == 0 || nr == 0) return SKV_OK;
    if (nr > (1u << 16)) return SKV_OK;  // the cut walk of every run would cost what the copies do
    for (uint64_t m = 0; m < nr; ++m)  // a run without a version byte: skv_compact's error
        if (job.run_len[m] == 0 || ((const uint8_t*)(uintptr_t)job.run_ptr[m])[0] != 1) return SKV_OK;
    uint64_t Pg = std::max<uint64_t>(1, std::min<uint64_t>(16, job.in_bytes / G / (1ull << 30)));
    if (const char* e = getenv("SKV_SPLIT_PARTS")) Pg = std::max<uint64_t>(1, std::min<uint64_t>(64, strtoull(e, nullptr, 10)));
    uint64_t P = (uint64_t)G * Pg;
    std::vector<std::string> cut;
    if (!sample_cuts(job, wal, P, cut)) return SKV_OK;  // (WAL flushes: cuts at table prefixes)
    P = cut.size() + 1;
    if (P < 2) return SKV_OK;
    std::vector<uint64_t> bnd;
    if (!cut_runs(job, cut, P, bnd) || !members_ascend(job)) return SKV_OK;
    used = true;
    GSplit gs;
    gs.P = P;
    gs.carry.assign(P + 1, 0);
    gs.have_c.assign(P + 1, 0);
    gs.have_c[0] = 1;  // the first part starts a fresh run
    gs.carry_st.assign(P + 1, 0);
    gs.staged.assign(P + 1, 0);
    gs.cont.assign(P, 0);
    gs.nbytes.assign(P, 0);
    gs.have_b.assign(P, 0);
    gs.off.assign(P + 1, 0);
    gs.descs.assign(P, {});
    gs.in_recs.assign(P, 0);
    gs.dropped.assign(P, 0);
    gs.wal = wal;
    const uint64_t out_cap = job.in_bytes + job.in_bytes / 5 + 64;  // records >= 5 bytes: version bytes <= R
    size_t cap = 0;
    uint8_t* h_out = (uint8_t*)home->out_pool->take(out_cap, cap);
    if (!h_out) throw DevError("pinned host allocation of the output failed");
    WorkerSet ws;
    const bool spawned = ws.spawn(G, [&](unsigned g) {
            skv_ctx* c = ctxs[g];
            DeviceScope ds(c->device);
            try {
                if (!ds.ok) throw DevError("hipSetDevice failed");
                gsplit_worker(gs, c, g, G, job, bnd, h_out, out_cap);
            } catch (const DevError& e) {
                if (e.msg != "split stopped") gs.halt(false, e.msg);
            } catch (const std::exception& e) {
                gs.halt(false, std::string("host error: ") + e.what());
            }
            drain(c);  // nothing of this call still runs on the ctx (nor writes h_out)
        }, [&] { gs.halt(false, "worker thread creation failed"); });
    ws.join();
    if (!spawned && !gs.stop) gs.halt(false, "worker thread creation failed");
    if (gs.stop) {
        home->out_pool->give(h_out, cap);
        if (!gs.err.empty()) throw DevError("split: " + gs.err);
        used = false;  // a data error in some part: skv_compact reports it exactly
        return SKV_OK;
    }
    // the runs in order; a continuation run 0 extends the run before it
    std::vector<skv_run_desc> all;
    uint64_t in_records = 0, out_records = 0, dropped = 0;
    for (uint64_t p = 0; p < P; ++p) {
        in_records += gs.in_recs[p];
        dropped += gs.dropped[p];
        for (size_t r = 0; r < gs.descs[p].size(); ++r) {
            const skv_run_desc& d = gs.descs[p][r];
            out_records += d.put_count + d.delete_count;
            if (r == 0 && gs.cont[p]) {
                if (all.empty()) {
                    home->out_pool->give(h_out, cap);
                    throw DevError("internal: a continuation with no run before it");
                }
                skv_run_desc& b = all.back();
                b.len += d.len - 1;
                b.put_count += d.put_count;
                b.delete_count += d.delete_count;
                b.max_key_off = d.max_key_off;
                b.max_key_len = d.max_key_len;
            } else {
                all.push_back(d);
            }
        }
    }
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(std::max<size_t>(1, all.size()) * sizeof(skv_run_desc));
    if (!all.empty()) memcpy(res->runs, all.data(), all.size() * sizeof(skv_run_desc));
    res->n_runs = all.size();
    res->bytes = h_out;
    res->n_bytes = gs.off[P];
    res->in_bytes = job.in_bytes;
    res->in_records = in_records;
    res->out_records = out_records;
    res->dropped_tables = dropped;
    box->pool = home->out_pool;
    box->pool_cap = cap;
    skv_timings& t = home->timings;
    t = skv_timings{};
    t.path = SKV_PATH_GENERAL;
    t.host_total_ms = now_ms() - t_entry;
    t.host_parts = (uint32_t)P;
    t.wal_stage = wal ? 1 : 0;
    *out = res;
    return SKV_OK;
}

// host inputs: stage them into HBM, compact, return the output bytes in pinned host memory
int compact_host_job(skv_ctx* ctx, Job& job, skv_result** out, double t_entry) {
    int rc;
    try {
        // stage inputs into HBM: one copy per span of runs that tile one host range (consecutive in
        // rank order, ascending or descending in memory -- a caller's buffer of 10^6 WAL runs is one
        // span; per-run copies cost ~2.5 us each), each span 16-byte aligned, its runs at their
        // offsets inside it (the kernels take unaligned runs)
        const size_t n = job.run_ptr.size();
        std::vector<size_t>& sp_end = ctx->s_span_end;  // span s: members [sp_end[s-1], sp_end[s])
        sp_end.clear();
        uint64_t total = 0;
        for (size_t m = 0; m < n;) {
            size_t e = m + 1;
            uint64_t lo = job.run_ptr[m], hi = lo + job.run_len[m];
            if (job.run_len[m]) {
                int dir = 0;  // +1 ascending, -1 descending
                while (e < n && job.run_len[e]) {
                    const uint64_t p = job.run_ptr[e], l = job.run_len[e];
                    const int d = p == hi ? 1 : (p + l == lo ? -1 : 0);
                    if (!d || (dir && d != dir)) break;
                    dir = d;
                    if (d > 0) hi += l;
                    else lo = p;
                    ++e;
                }
            }
            total += (hi - lo + 15) & ~15ull;
            sp_end.push_back(e);
            m = e;
        }
        uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", total + 16);
        uint64_t off = 0;
        for (size_t s = 0, m = 0; s < sp_end.size(); ++s) {
            const size_t e = sp_end[s];
            uint64_t lo = job.run_ptr[m], hi = lo + job.run_len[m];
            for (size_t i = m + 1; i < e; ++i) {
                lo = std::min<uint64_t>(lo, job.run_ptr[i]);
                hi = std::max<uint64_t>(hi, job.run_ptr[i] + job.run_len[i]);
            }
            if (hi > lo) h2d(ctx, d_in + off, (const void*)lo, hi - lo);
            for (size_t i = m; i < e; ++i)
                job.run_ptr[i] = (uint64_t)(uintptr_t)(d_in + off + (job.run_len[i] ? job.run_ptr[i] - lo : 0));
            off += (hi - lo + 15) & ~15ull;
            m = e;
        }
    } catch (const DevError& e) {
        return set_err(ctx, SKV_E_DEVICE, "%s", e.msg.c_str());
    } catch (const std::exception& e) {
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
    skv_result* dres = nullptr;
    rc = run_guarded(ctx, job, &dres, t_entry);
    if (rc) return rc;
    ResultBox* box = (ResultBox*)dres;
    size_t cap = 0;
    uint8_t* hb = (uint8_t*)ctx->out_pool->take(std::max<uint64_t>(1, dres->n_bytes), cap);
    if (!hb) {
        skv_result_free(dres);
        return set_err(ctx, SKV_E_DEVICE, "pinned host allocation of %" PRIu64 " output bytes failed", dres->n_bytes);
    }
    if (dres->n_bytes && (hipMemcpyAsync(hb, dres->bytes, dres->n_bytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                          hipStreamSynchronize(ctx->stream) != hipSuccess)) {
        ctx->out_pool->give(hb, cap);
        skv_result_free(dres);
        return set_err(ctx, SKV_E_DEVICE, "device-to-host copy of the output failed");
    }
    dres->bytes = hb;
    box->pool = ctx->out_pool;
    box->pool_cap = cap;
    *out = dres;
    return SKV_OK;
}


extern "C" {

int skv_compact(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams, uint64_t max_run_size, uint32_t flags,
                skv_result** out) {
    const double t_entry = now_ms();
    htrace("entry");
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;  // lent ctx tables, as in skv_compact_dev
    job.ranked.swap(ctx->j_ranked);
    job.run_ptr.swap(ctx->j_ptr);
    job.run_len.swap(ctx->j_len);
    int rc = build_job(ctx, streams, n_streams, max_run_size, flags, job);
    if (!rc) {
        bool used = false;
        try {
            ctx->timings = skv_timings{};
            rc = compact_host_pipelined(ctx, job, out, t_entry, used);
            if (!used) rc = compact_host_pipelined_general(ctx, job, out, t_entry, used);
        } catch (const DevError& e) {
            (void)hipStreamSynchronize(ctx->stream);
            rc = set_err(ctx, SKV_E_DEVICE, "%s", e.msg.c_str());
            used = true;
        } catch (const std::exception& e) {
            (void)hipStreamSynchronize(ctx->stream);
            rc = set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
            used = true;
        }
        if (!used) rc = compact_host_job(ctx, job, out, t_entry);
    }
    job.ranked.swap(ctx->j_ranked);
    job.run_ptr.swap(ctx->j_ptr);
    job.run_len.swap(ctx->j_len);
    return rc;
}

int skv_encode_batch(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size, skv_result** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    SKV_DEVICE_SCOPE(ctx);
    Job job;
    int rc = batch_job(ctx, ops_run, len, max_run_size, job);
    if (rc) return rc;
    return compact_host_job(ctx, job, out, t_entry);
}

}  // extern "C"
