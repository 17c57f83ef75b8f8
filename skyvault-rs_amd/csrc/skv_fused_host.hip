// skv_fused_host.hip — host side of the fused stride path (skv_stride.hip): splitter levels, the
// fused tile launch and the descriptors of one compaction (compact_fused), or of one key-range part
// of a pipelined host call (fx_launch with FxPartIO).
#include "skv_host.hpp"

using namespace skv;


// The fused stride path (skv_stride.hip): every run is fixed-stride with one record size S and one
// key length K <= 16. Splitters, then one fused verify/merge/copy kernel, then the descriptors;
// one host sync reads the descriptors together with the verdict. Returns false when the device
// poisoned the call (a record or key order the run's first record did not promise, or splitter
// skew): the caller then reruns the exact path, which produces the reference's outcome.
// records per output run of the fused path (build_runs' greedy split is arithmetic at one size)
uint64_t fx_run_records(uint64_t max_run_size, uint64_t S, uint64_t R) {
    uint64_t n = max_run_size >= 1 ? (max_run_size - 1) / S : 0;  // runs.rs:211-238
    if (n < 1) n = 1;  // a record that alone exceeds max still forms its own run (runs.rs:219)
    if (n > R) n = R;
    return n;
}

// The fused stride path up to and including k_fx_tile, on ctx->stream, with no host sync:
// splitters (levels sized from host-known counts) and the fused tiles. d_rb: the blob's readback
// words {runs, K, bytes} + flags (whole-call launches).
FxArgs fx_launch(skv_ctx* ctx, uint32_t k, uint32_t n_runs, const RunInfo* d_runs,
                        const std::vector<uint32_t>& stream_first_run, const RunFmt& f,
                        const std::vector<uint64_t>& recb, uint64_t n, uint64_t out_bytes, const FxPartIO* io,
                        uint64_t*& d_rb_out) {
    hipStream_t st = ctx->stream;
    const uint64_t R = recb[n_runs];
    std::vector<uint64_t> stream_base(k + 1);
    for (uint32_t s = 0; s <= k; ++s) stream_base[s] = recb[stream_first_run[s]];

    FxArgs A{};
    A.k = k;
    A.K = f.K;
    A.V = f.V;
    A.S = f.S;
    A.n = n;
    A.inv_S = 1.0 / (double)f.S;
    A.inv_W = 1.0 / (double)(n * f.S + 1);
    A.inv_n = 1.0 / (double)n;
#if SKV_TILE_PROF
    A.prof = dbuf<uint64_t>(ctx, "tile_prof", 16);
    if (!ctx->prof_init) {
        HIPCHK(hipMemsetAsync(A.prof, 0, 128, st));
        ctx->prof_init = true;
    }
#endif

    // ---- splitters: level 1 sampled from the run bytes, higher levels as in the general path.
    // The level sizes, the tile count and every host table are known before the first launch, so
    // all tables and the zeroed state (flags, tile states, ticket) go up as ONE blob: one H2D
    // copy in place of six copies and four fills.
    struct Level {
        uint64_t N = 0, S = 1;
        std::vector<uint64_t> off;
        uint64_t *hi = nullptr, *lo = nullptr, *c = nullptr, *d_off = nullptr;
        uint64_t *shi = nullptr, *slo = nullptr, *sc = nullptr;
    };
    std::vector<Level> lv(1);
    lv[0].N = R;
    lv[0].off = stream_base;
    // level-1 sample spacing: FX_TARGET/k records gives ~k samples between splitters, whose
    // sampling noise spreads tile sizes by ~1/sqrt(k) (a few streams of a few thousand records
    // reached 1.5x the target, above FX_CAP); small inputs sample densely (>= 256 per tile),
    // where the extra samples cost nothing
    const uint64_t S_step = std::max<uint64_t>(
        2, (uint64_t)FX_TARGET / std::max<uint32_t>(R >= (1ull << 22) ? k : std::max<uint32_t>(k, 256), 1));
    while (lv.back().N > (uint64_t)FX_CAP) {
        const Level& P = lv.back();
        Level L;
        L.S = S_step;
        L.off.resize(k + 1);
        uint64_t acc = 0;
        for (uint32_t j = 0; j < k; ++j) {
            L.off[j] = acc;
            acc += (P.off[j + 1] - P.off[j] + L.S - 1) / L.S;
        }
        L.off[k] = acc;
        L.N = acc;
        lv.push_back(L);
    }
    uint64_t T0 = 1, m0 = 1;
    if (lv.size() > 1) {
        m0 = std::max<uint64_t>(1, (uint64_t)FX_TARGET / lv[1].S);
        T0 = std::max<uint64_t>(1, (lv[1].N + m0 - 1) / m0);
    }
    // the last generation of tiles (as many as are resident at once) at half size, so the grid
    // drains in half a tile time (SKV_FX_TAIL=0: uniform tiles)
    uint64_t T1 = T0, m2 = m0;
    {
        if (lv.size() > 1 && m0 >= 4) {
            const char* se = test_opt("SKV_FX_TAIL_SLOTS");  // tests: a small grid's worth of slots
            const uint64_t slots = se ? std::max<uint64_t>(1, strtoull(se, nullptr, 10)) : fx_tile_slots(k);
            const uint64_t h = m0 / 2;
            if (T0 > 3 * slots) {
                m2 = h;
                T1 = (lv[1].N - slots * h) / m0;
                T0 = T1 + (lv[1].N - T1 * m0 + h - 1) / h;
            }
        }
    }
    // blob layout (256-byte aligned pieces): readback words {runs, K, bytes} + flags[4] | K_out |
    // ticket | recb | stream_run | stream_base | level offsets | tile states
    std::vector<size_t> lv_off(lv.size(), 0);
    size_t blob_n = 0;
    auto piece = [&](size_t bytes) {
        const size_t at = blob_n;
        blob_n += (bytes + 255) & ~(size_t)255;
        return at;
    };
    const size_t o_rb = piece(64), o_K = piece(8), o_tick = piece(4), o_recb = piece((n_runs + 1) * 8),
                 o_srun = piece((k + 1) * 4), o_sbase = piece((k + 1) * 8);
    for (size_t li = 1; li < lv.size(); ++li) lv_off[li] = piece((k + 1) * 8);
    const size_t o_tstate = piece(T0 * 8);
    std::vector<uint8_t>& blob = ctx->fx_blob;
    blob.assign(blob_n, 0);
    memcpy(blob.data() + o_recb, recb.data(), (n_runs + 1) * 8);
    memcpy(blob.data() + o_srun, stream_first_run.data(), (k + 1) * 4);
    memcpy(blob.data() + o_sbase, stream_base.data(), (k + 1) * 8);
    for (size_t li = 1; li < lv.size(); ++li) memcpy(blob.data() + lv_off[li], lv[li].off.data(), (k + 1) * 8);
    uint8_t* d_blob = dbuf<uint8_t>(ctx, "fx_blob", blob_n);
    h2d_up(ctx, d_blob, blob.data(), blob_n);
    uint64_t* d_rb = (uint64_t*)(d_blob + o_rb);        // k_fx_desc: {runs, K, record bytes}
    uint32_t* d_flags = (uint32_t*)(d_blob + o_rb + 32);  // verdict flags, read back with d_rb
    A.runs = d_runs;
    A.run_recb = (uint64_t*)(d_blob + o_recb);
    A.stream_run = (uint32_t*)(d_blob + o_srun);
    A.stream_base = (uint64_t*)(d_blob + o_sbase);
    if (io && io->flags) d_flags = io->flags;
    A.flags = d_flags;
    A.Kout = io && io->Kout ? io->Kout : (uint64_t*)(d_blob + o_K);
    A.gbase = io ? io->gbase : nullptr;
    d_rb_out = d_rb;
    lv[0].d_off = (uint64_t*)(d_blob + o_sbase);
    mark(ctx, PH_PARSE);
    for (size_t li = 1; li < lv.size(); ++li) {
        Level& L = lv[li];
        char nm[64];
        snprintf(nm, sizeof nm, "lv%d_hi", (int)li); L.hi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_lo", (int)li); L.lo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_c", (int)li); L.c = dbuf<uint64_t>(ctx, nm, L.N);
        L.d_off = (uint64_t*)(d_blob + lv_off[li]);
    }
    // level 1 sampled from the run bytes; levels 2 and 3 written by the same launch (every level
    // samples the one below with the same step S_step, so level li's sample c is level 1's sample
    // c * S_step^(li-1)); any higher level from the one below it
    if (lv.size() > 1) {
        FxUpLevels up{};
        for (size_t li = 2; li < lv.size() && up.n < 2; ++li, ++up.n) {
            up.hi[up.n] = lv[li].hi;
            up.lo[up.n] = lv[li].lo;
            up.c[up.n] = lv[li].c;
            up.off[up.n] = lv[li].d_off;
        }
        launch_fx_sample(st, A, lv[1].d_off, lv[1].S, lv[1].N, lv[1].hi, lv[1].lo, lv[1].c, up);
        for (size_t li = 2 + up.n; li < lv.size(); ++li) {
            const Level& P = lv[li - 1];
            Level& L = lv[li];
            launch_sample(st, false, P.hi, P.lo, P.c, nullptr, P.d_off, L.d_off, k, L.S, L.N, L.hi, L.lo, L.c);
        }
    }
    for (int li = (int)lv.size() - 1; li >= 1; --li) {
        Level& L = lv[li];
        uint64_t T = 1, m = 1;
        if (li + 1 < (int)lv.size()) {
            m = std::max<uint64_t>(1, (uint64_t)TILE_TARGET / lv[li + 1].S);
            T = std::max<uint64_t>(1, (lv[li + 1].N + m - 1) / m);
        }
        char nm[64];
        snprintf(nm, sizeof nm, "bounds%d", li);
        uint64_t* bounds = dbuf<uint64_t>(ctx, nm, (T + 1) * k);
        const Level* U = li + 1 < (int)lv.size() ? &lv[li + 1] : nullptr;
        launch_bounds(st, false, L.hi, L.lo, L.c, nullptr, L.d_off, k, U ? U->shi : nullptr, U ? U->slo : nullptr,
                      U ? U->sc : nullptr, m, T, nullptr, bounds, d_flags + 2);
        TileOut O{};  // sample tiles find their output base from the bounds (no tile_base table)
        snprintf(nm, sizeof nm, "x%d_hi", li); O.xhi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "x%d_lo", li); O.xlo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "x%d_c", li); O.xc = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "s%d_hi", li); L.shi = O.ohi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "s%d_lo", li); L.slo = O.olo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "s%d_c", li); L.sc = O.oc = dbuf<uint64_t>(ctx, nm, L.N);
        HIPCHK(launch_tile(st, false, L.hi, L.lo, L.c, nullptr, bounds, k, T, nullptr, nullptr, nullptr, 0u, O,
                           d_flags + 2));
    }
    A.T = T0;
    const bool l1 = lv.size() > 1;
    A.shi = l1 ? lv[1].shi : nullptr;
    A.slo = l1 ? lv[1].slo : nullptr;
    A.l1hi = l1 ? lv[1].hi : nullptr;
    A.l1lo = l1 ? lv[1].lo : nullptr;
    A.l1off = l1 ? lv[1].d_off : nullptr;
    A.m = m0;
    A.T1 = T1;
    A.m2 = m2;
    A.Sstep = S_step;
    if (l1 && T0 > 1) {  // per (splitter, stream) sample counts: k_fx_bounds skips its sample search
        uint32_t* posof = dbuf<uint32_t>(ctx, "fx_posof", lv[1].N);
        uint32_t* cnt = dbuf<uint32_t>(ctx, "fx_l1cnt", (T0 + 1) * k);
        launch_fx_l1cnt(st, A, lv[1].sc, lv[1].N, posof, cnt);
        A.l1cnt = cnt;
    }
    A.bnd = dbuf<FxBound>(ctx, "fx_bnd", (T0 + 1) * k);
    launch_fx_bounds(st, A, A.shi, A.slo, m0, A.l1hi, A.l1lo, A.l1off, S_step);
    A.tstate = (uint64_t*)(d_blob + o_tstate);  // zeroed by the blob upload
    A.tcounter = (uint32_t*)(d_blob + o_tick);
    A.out = io && io->out ? io->out : dbuf<uint8_t>(ctx, "out", out_bytes);
    mark(ctx, PH_CHECK);
    // ---- the fused tiles
    HIPCHK(launch_fx_tile(st, A));
    return A;
}

// The fused stride path (whole call): fx_launch, then the descriptors; one host sync reads the
// descriptors together with the verdict. Returns false when the device poisoned the call.
bool compact_fused(skv_ctx* ctx, const Job& job, const std::vector<RunInfo>& runs, const RunInfo* d_runs,
                          const std::vector<uint32_t>& stream_first_run, const RunFmt& f,
                          const std::vector<uint64_t>& recb, skv_result** out) {
    hipStream_t st = ctx->stream;
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint32_t n_runs = (uint32_t)runs.size();
    const uint64_t R = recb[n_runs];
    const uint64_t n = fx_run_records(job.max_run_size, f.S, R);
    const uint64_t total_rec_bytes = job.in_bytes;
    uint64_t* d_rb = nullptr;
    const FxArgs A = fx_launch(ctx, k, n_runs, d_runs, stream_first_run, f, recb, n, total_rec_bytes + R + 16, nullptr,
                               d_rb);
    uint8_t* d_out = A.out;
    mark(ctx, PH_MERGE);
    const uint64_t max_runs = (R + n - 1) / n;
    DevRunDesc* d_desc = dbuf<DevRunDesc>(ctx, "descs", max_runs + 1);
    launch_fx_desc(st, A, d_desc, d_rb, max_runs);
    HIPCHK(hipGetLastError());
    mark(ctx, PH_CHAIN);
    mark(ctx, PH_GATHER);
    // ---- one readback: {runs, K, record bytes}, descriptors (count guessed from sizes), verdict
    const uint64_t guess = std::min<uint64_t>(max_runs, 64 + total_rec_bytes / (n * f.S));
    uint8_t* hp = (uint8_t*)pinned(ctx, 64 + guess * sizeof(DevRunDesc));
    uint8_t* hv = hp + 32;
    d2h(ctx, hp, d_rb, 48);  // {runs, K, bytes} and the flags
    d2h(ctx, hp + 64, d_desc, guess * sizeof(DevRunDesc));
    sync(ctx);
    uint32_t hf[4];
    memcpy(hf, hv, 16);
    if (hf[2]) {
        ctx->timings.fused_reject = hf[3] ? hf[3] : 0x80000000u;
        return false;
    }
    uint64_t h3[3];
    memcpy(h3, hp, 24);
    const uint64_t n_out = h3[0], K = h3[1];
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, n_out) * sizeof(skv_run_desc));
    memcpy(res->runs, hp + 64, std::min(n_out, guess) * sizeof(DevRunDesc));
    if (n_out > guess)
        HIPCHK(hipMemcpy(res->runs + guess, d_desc + guess, (n_out - guess) * sizeof(DevRunDesc), hipMemcpyDeviceToHost));
    res->n_runs = n_out;
    res->bytes = d_out;
    res->n_bytes = h3[2] + n_out;
    res->in_bytes = job.in_bytes;
    res->in_records = R;
    res->out_records = K;
    res->dropped_tables = 0;
    skv_timings& t = ctx->timings;
    const uint32_t reject = t.fused_reject;
    t = skv_timings{};
    t.path = SKV_PATH_FUSED;
    t.fused_reject = reject;
    t.hot_read_bytes = R * f.S;  // every input record is read (and verified) once
    t.hot_write_bytes = h3[2] + n_out;
    if (ctx->profiling) {
        HIPCHK(hipEventSynchronize(ctx->ev[PH_GATHER]));
        float ms[PH_N] = {};
        for (int p = PH_PARSE; p < PH_N; ++p) HIPCHK(hipEventElapsedTime(&ms[p], ctx->ev[p - 1], ctx->ev[p]));
        float tot = 0;
        HIPCHK(hipEventElapsedTime(&tot, ctx->ev[PH_START], ctx->ev[PH_GATHER]));
        t.total_ms = tot;
        t.parse_ms = ms[PH_PARSE];
        t.check_ms = ms[PH_CHECK];  // splitters
        t.merge_ms = ms[PH_MERGE];  // k_fx_tile: verify + merge + output bytes
        t.chain_ms = ms[PH_CHAIN];
        t.gather_ms = ms[PH_GATHER];
        t.hot_ms = ms[PH_MERGE];
    }
    t.host_syncs = ctx->syncs;
    *out = res;
    return true;
}
