// skv_index_host.hip — runs::search_run batches (runs.rs:285-398) and the cached run index of the
// cache service (cache_service.rs:52-94): skv_search_run, skv_run_index_*.
#include "skv_host.hpp"

using namespace skv;


// the lookups of one batch against parsed arrays (bsearch) or the run bytes (scan)
void search_launch(skv_ctx* ctx, const uint8_t* run, uint64_t len, bool clean, uint64_t R,
                          const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
                          const uint32_t* rec_klen, const uint32_t* rec_meta, const uint8_t* keys,
                          const uint64_t* key_offs, uint32_t n, skv_lookup* out) {
    hipStream_t st = ctx->stream;
    const uint64_t qbytes = key_offs[n];
    uint8_t* d_q = dbuf<uint8_t>(ctx, "sr_keys", qbytes + 16);
    uint64_t* d_off = dbuf<uint64_t>(ctx, "sr_offs", n + 1);
    SrResult* d_out = dbuf<SrResult>(ctx, "sr_out", n);
    if (qbytes) h2d(ctx, d_q, keys, qbytes);
    h2d(ctx, d_off, key_offs, (n + 1) * 8);
    if (clean)
        launch_search_bsearch(st, run, len, R, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_q, d_off, n, d_out);
    else
        launch_search_scan(st, run, len, d_q, d_off, n, d_out);
    HIPCHK(hipGetLastError());
    static_assert(sizeof(SrResult) == sizeof(skv_lookup), "lookup layout");
    if (n) HIPCHK(hipMemcpyAsync(out, d_out, (size_t)n * sizeof(SrResult), hipMemcpyDeviceToHost, st));
    sync(ctx);
}

// skv_search_run after the parse: a run that parsed clean with no key decrease takes one binary
// search per key over its record arrays; any other run the reference's scan (skv_search.hip).
int search_stage(skv_ctx* ctx, const Job& job, const RunInfo& run, uint64_t R, uint32_t run_err,
                        uint64_t first_dec, const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
                        const uint32_t* rec_klen, const uint32_t* rec_meta) {
    const bool clean = run_err == 0 && first_dec == ~0ull;
    if (skv_run_index* ix = job.index_out) {  // keep the parsed arrays in the index's memory
        ix->clean = clean;
        ix->R = clean ? R : 0;
        if (clean && R) {
            hipStream_t st = ctx->stream;
            uint8_t* base = (uint8_t*)ix->mem + ((ix->len + 255) & ~(uint64_t)255);
            uint64_t* a = (uint64_t*)base;
            uint64_t* h = a + R;
            uint64_t* l = h + R;
            uint32_t* kl = (uint32_t*)(l + R);
            uint32_t* m = kl + R;
            HIPCHK(hipMemcpyAsync(a, rec_addr, R * 8, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(h, rec_hi, R * 8, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(l, rec_lo, R * 8, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(kl, rec_klen, R * 4, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(m, rec_meta, R * 4, hipMemcpyDeviceToDevice, st));
            sync(ctx);
            ix->addr = a;
            ix->hi = h;
            ix->lo = l;
            ix->klen = kl;
            ix->meta = m;
        }
        ctx->timings.path = clean ? SKV_PATH_FIXED : SKV_PATH_GENERAL;
        return SKV_OK;
    }
    search_launch(ctx, (const uint8_t*)run.ptr, run.len, clean, R, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta,
                  job.sr_keys, job.sr_offs, job.sr_n, job.sr_out);
    ctx->timings.path = clean ? SKV_PATH_FIXED : SKV_PATH_GENERAL;
    return SKV_OK;
}

// runs::search_run's panic text (runs.rs:288-386)
static std::string search_panic_text(uint32_t p) {
    char buf[64];
    switch (p & 0xFF) {
        case SKV_PANIC_EMPTY: return "Empty run data";
        case SKV_PANIC_VERSION: snprintf(buf, sizeof buf, "Unsupported version: %u", p >> 8); return buf;
        case SKV_PANIC_MARKER: snprintf(buf, sizeof buf, "Invalid marker byte: %u", p >> 8); return buf;
        case SKV_PANIC_KEYLEN: return "Incomplete key length data";
        case SKV_PANIC_KEY: return "Incomplete key data";
        case SKV_PANIC_VALLEN: return "Incomplete value length data";
        case SKV_PANIC_VAL: return "Incomplete value data";
        case SKV_PANIC_VALLEN_FOUND: return "Incomplete value length data for found key";
        case SKV_PANIC_VAL_FOUND: return "Incomplete value data for found key";
        default: return "internal: unknown search panic";
    }
}

extern "C" {

int skv_search_run(skv_ctx* ctx, const uint8_t* run, uint64_t len, const uint8_t* keys, const uint64_t* key_offs,
                   uint32_t n_keys, skv_lookup* out) {
    const double t_entry = now_ms();
    if (!ctx) return SKV_E_INVALID_ARG;
    if (n_keys && (!out || !key_offs)) return set_err(ctx, SKV_E_INVALID_ARG, "out/key_offs is NULL");
    if (len && !run) return set_err(ctx, SKV_E_INVALID_ARG, "run is NULL");
    if (n_keys && key_offs[n_keys] && !keys) return set_err(ctx, SKV_E_INVALID_ARG, "keys is NULL");
    for (uint32_t i = 0; i < n_keys; ++i)
        if (key_offs[i + 1] < key_offs[i]) return set_err(ctx, SKV_E_INVALID_ARG, "key_offs not ascending at %u", i);
    if (n_keys == 0) return SKV_OK;
    if (len == 0 || run[0] != 1) {  // the panics before the scan loop (runs.rs:288-297)
        const uint32_t pc = len == 0 ? (uint32_t)SKV_PANIC_EMPTY : (SKV_PANIC_VERSION | ((uint32_t)run[0] << 8));
        for (uint32_t i = 0; i < n_keys; ++i) out[i] = skv_lookup{SKV_LOOKUP_PANIC, pc, 0, 0};
        return set_err(ctx, SKV_E_FORMAT, "%s", search_panic_text(pc).c_str());
    }
    SKV_DEVICE_SCOPE(ctx);
    Job job;
    int rc = batch_job(ctx, run, len, 1ull << 62, job);
    if (rc) return rc;
    job.batch = false;
    job.search = true;
    job.sr_keys = keys;
    job.sr_offs = key_offs;
    job.sr_n = n_keys;
    job.sr_out = out;
    try {
        uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", len + 16);
        h2d(ctx, d_in, run, len);
        job.run_ptr[0] = (uint64_t)(uintptr_t)d_in;
    } catch (const DevError& e) {
        return set_err(ctx, SKV_E_DEVICE, "%s", e.msg.c_str());
    } catch (const std::exception& e) {
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
    skv_result* none = nullptr;
    rc = run_guarded(ctx, job, &none, t_entry);
    if (rc) return rc;
    for (uint32_t i = 0; i < n_keys; ++i)
        if (out[i].kind == SKV_LOOKUP_PANIC) return set_err(ctx, SKV_E_FORMAT, "%s", search_panic_text(out[i].panic).c_str());
    return SKV_OK;
}

int skv_run_index_create(skv_ctx* ctx, const uint8_t* run, uint64_t len, skv_run_index** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    if (len && !run) return set_err(ctx, SKV_E_INVALID_ARG, "run is NULL");
    SKV_DEVICE_SCOPE(ctx);
    std::unique_ptr<skv_run_index> ix(new (std::nothrow) skv_run_index());
    if (!ix) return set_err(ctx, SKV_E_DEVICE, "host allocation failed");
    ix->device = ctx->device;
    ix->len = len;
    if (len == 0 || run[0] != 1) {  // every lookup panics before the scan loop (runs.rs:288-297)
        ix->panic_all = len == 0 ? (uint32_t)SKV_PANIC_EMPTY : (SKV_PANIC_VERSION | ((uint32_t)run[0] << 8));
        *out = ix.release();
        return SKV_OK;
    }
    // worst case: every record 5 bytes (an empty-key Delete) -> R <= len / 5
    const uint64_t maxR = len / 5 + 1;
    const size_t bytes = ((len + 255) & ~(uint64_t)255) + maxR * 32 + 256;
    if (hipMalloc(&ix->mem, bytes) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "index allocation of %zu bytes failed", bytes);
    ix->run = (const uint8_t*)ix->mem;
    if (hipMemcpy(ix->mem, run, len, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(ix->mem);
        return set_err(ctx, SKV_E_DEVICE, "index staging copy failed");
    }
    Job job;
    int rc = batch_job(ctx, ix->run, len, 1ull << 62, job);
    if (rc) {
        (void)hipFree(ix->mem);
        return rc;
    }
    job.batch = false;
    job.search = true;
    job.index_out = ix.get();
    skv_result* none = nullptr;
    rc = run_guarded(ctx, job, &none, t_entry);
    if (rc) {
        (void)hipFree(ix->mem);
        return rc;
    }
    *out = ix.release();
    return SKV_OK;
}

int skv_run_index_search(skv_ctx* ctx, const skv_run_index* ix, const uint8_t* keys, const uint64_t* key_offs,
                         uint32_t n_keys, skv_lookup* out) {
    if (!ctx || !ix) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/index is NULL");
    if (ix->device != ctx->device) return set_err(ctx, SKV_E_INVALID_ARG, "index belongs to device %d", ix->device);
    if (n_keys && (!out || !key_offs)) return set_err(ctx, SKV_E_INVALID_ARG, "out/key_offs is NULL");
    if (n_keys && key_offs[n_keys] && !keys) return set_err(ctx, SKV_E_INVALID_ARG, "keys is NULL");
    for (uint32_t i = 0; i < n_keys; ++i)
        if (key_offs[i + 1] < key_offs[i]) return set_err(ctx, SKV_E_INVALID_ARG, "key_offs not ascending at %u", i);
    if (n_keys == 0) return SKV_OK;
    if (ix->panic_all) {
        for (uint32_t i = 0; i < n_keys; ++i) out[i] = skv_lookup{SKV_LOOKUP_PANIC, ix->panic_all, 0, 0};
        return set_err(ctx, SKV_E_FORMAT, "%s", search_panic_text(ix->panic_all).c_str());
    }
    SKV_DEVICE_SCOPE(ctx);
    try {
        search_launch(ctx, ix->run, ix->len, ix->clean, ix->R, ix->addr, ix->hi, ix->lo, ix->klen, ix->meta, keys,
                      key_offs, n_keys, out);
    } catch (const DevError& e) {
        return set_err(ctx, SKV_E_DEVICE, "%s", e.msg.c_str());
    } catch (const std::exception& e) {
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
    for (uint32_t i = 0; i < n_keys; ++i)
        if (out[i].kind == SKV_LOOKUP_PANIC) return set_err(ctx, SKV_E_FORMAT, "%s", search_panic_text(out[i].panic).c_str());
    return SKV_OK;
}

void skv_run_index_free(skv_run_index* ix) {
    if (!ix) return;
    if (ix->mem) {  // on the index's device, and the caller's current device left as it was
        int prev = 0;
        const bool had = hipGetDevice(&prev) == hipSuccess;
        (void)hipSetDevice(ix->device);
        (void)hipFree(ix->mem);
        if (had) (void)hipSetDevice(prev);
    }
    delete ix;
}

}  // extern "C"
