// skv_host.hip — C ABI (include/skv.h) and host orchestration of the MI355X compaction path.
//
// One skv_compact call = the decode -> merge -> [filter] -> build_runs composition of the
// compaction jobs (table_buffer_compaction.rs:48-121, table_tree_compaction.rs:81-167). The
// device does all per-record work; the host only sequences kernels, sizes buffers and turns
// per-run / per-stream summaries into the reference's error (which error surfaces first is a
// property of k_way::merge's pull order, resolved here from a handful of candidate records).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <condition_variable>
#include <array>
#include <vector>

#include "../../include/skv.h"
#include "skv_dev.hpp"

#include "skv_launch.hpp"

using namespace skv;

// ------------------------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

enum Phase { PH_START = 0, PH_PARSE, PH_CHECK, PH_MERGE, PH_CHAIN, PH_GATHER, PH_N };

// Pinned host buffers for skv_compact outputs. Shared by the ctx and its live results, so a
// result may outlive its ctx; a freed result's buffer is kept for the next call.
struct PinnedPool {
    std::mutex mu;
    std::vector<std::pair<void*, size_t>> free_list;
    ~PinnedPool() {
        for (auto& b : free_list) (void)hipHostFree(b.first);
    }
    void* take(size_t bytes, size_t& cap) {
        {
            std::lock_guard<std::mutex> g(mu);
            for (size_t i = 0; i < free_list.size(); ++i) {
                if (free_list[i].second >= bytes) {
                    void* p = free_list[i].first;
                    cap = free_list[i].second;
                    free_list.erase(free_list.begin() + i);
                    return p;
                }
            }
        }
        void* p = nullptr;
        cap = std::max<size_t>(bytes, 1 << 20);
        if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        return p;
    }
    void give(void* p, size_t cap) {
        std::lock_guard<std::mutex> g(mu);
        free_list.emplace_back(p, cap);
    }
};

struct InStream {
    int64_t seq;
    uint32_t vec_idx;  // position in the caller's vector (merge pulls first items in this order)
    uint32_t n_runs;
    uint64_t first;    // its member runs: Job::run_ptr/run_len[first, first + n_runs)
};

struct skv_ctx {
    int device = 0;
    std::shared_ptr<PinnedPool> out_pool = std::make_shared<PinnedPool>();
    bool prof_init = false;  // SKV_TILE_PROF builds
    hipStream_t stream = nullptr;
    std::string err;
    bool profiling = false;
    skv_timings timings{};
    std::map<std::string, DevBuf> bufs;
    hipEvent_t ev[PH_N] = {};
    void* pinned = nullptr;  // small readback staging
    size_t pinned_cap = 0;
    // pinned upload arena: small host tables are staged here so their H2D copies are truly async
    // (a copy from pageable memory stalls the host); chunks live until the ctx is destroyed and
    // are reused from the start on every call (each call ends with a stream sync)
    std::vector<std::pair<uint8_t*, size_t>> up_chunks;
    size_t up_chunk = 0, up_off = 0;
    bool kernel_uploads = false;  // h2d_up by a copy kernel from the mapped arena (pipelined calls)
    std::vector<uint8_t> fx_blob;  // fused path: host image of its one table upload
    // per-call host tables kept across calls: at 10^6 runs, fresh vectors cost their page faults
    // (~15 ms per call) every time; reused ones keep their touched pages
    std::vector<RunInfo> s_runs;
    std::vector<RunSummary> s_sum;
    std::vector<uint64_t> s_sbase, s_svalid, s_first_dec, s_recb;
    std::vector<uint32_t> s_sfr, s_serr;
    std::vector<InStream> j_ranked;  // skv_compact_dev's job tables, lent to each call
    std::vector<uint64_t> j_ptr, j_len;
    uint64_t syncs = 0;
    double sync_ms = 0;
    bool exact_keys = false;  // rerun after a fingerprint shortcut misordered a tile (never in practice)
    bool exact_utf8 = false;  // rerun with UTF-8 checked in the chunk walks (a run holds a bad key)
    // compact_device calls started on this ctx: the s_* tables belong to the newest one, so a call
    // that continues after a nested rerun (none does; each returns at once) must not read them
    uint64_t table_gen = 0;
    // pipelined host calls (compact_host_pipelined): the copy streams, per-part events, and the
    // host-mapped words the parts publish their survivor counts to
    hipStream_t in_stream = nullptr, out_stream = nullptr;
    // k_fp_verify runs beside the chain and the gather (its verdict is only read with the result)
    hipStream_t aux_stream = nullptr;
    hipEvent_t aux_ev[2] = {};
    std::vector<hipEvent_t> part_ev;
    uint64_t* part_k = nullptr;
    size_t part_k_cap = 0;
};

struct ResultBox {  // skv_result + how to free it
    skv_result pub;
    std::shared_ptr<PinnedPool> pool;  // set: bytes is a pinned host buffer of pool_cap bytes
    size_t pool_cap = 0;
};

static int set_err(skv_ctx* ctx, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess)                                                                       \
            throw DevError(std::string(#x) + ": " + hipGetErrorString(e_));                         \
    } while (0)

struct DevError {
    std::string msg;
    explicit DevError(std::string m) : msg(std::move(m)) {}
};
struct ApiError {
    int code;
    std::string msg;
};

template <typename T>
static T* dbuf(skv_ctx* ctx, const char* name, size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    bytes = (bytes + 255) & ~(size_t)255;
    DevBuf& b = ctx->bufs[name];
    if (b.cap < bytes) {
        if (b.p) {  // queued work of this call (pipelined parts) may still use the old buffer
            HIPCHK(hipStreamSynchronize(ctx->stream));
            HIPCHK(hipFree(b.p));
        }
        b.p = nullptr;
        b.cap = 0;
        size_t cap = bytes + bytes / 8;
        HIPCHK(hipMalloc(&b.p, cap));
        b.cap = cap;
    }
    return (T*)b.p;
}

static void* pinned(skv_ctx* ctx, size_t bytes) {
    if (ctx->pinned_cap < bytes) {
        if (ctx->pinned) HIPCHK(hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        size_t cap = std::max<size_t>(bytes, 1 << 16);
        HIPCHK(hipHostMalloc(&ctx->pinned, cap, hipHostMallocDefault));
        ctx->pinned_cap = cap;
    }
    return ctx->pinned;
}

// host copy into pinned staging; large tables (10^6-run calls: tens of MB) on several threads
static void stage_copy(void* dst, const void* src, size_t bytes) {
    const char* pe = getenv("SKV_PAR_COPY_MIN");  // tests: split small tables too
    const size_t kPar = pe ? (size_t)strtoull(pe, nullptr, 10) : (8u << 20);
    const unsigned hw = std::thread::hardware_concurrency();
    static const unsigned cap = [] {  // SKV_HOST_THREADS: host threads for 10^6-entry tables (default 8)
        const char* e = getenv("SKV_HOST_THREADS");
        const long v = e ? atol(e) : 8;
        return (unsigned)std::max(1l, std::min(64l, v));
    }();
    const unsigned nt = std::min<unsigned>(cap, hw ? hw : 1);
    if (bytes < kPar || nt < 2) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t part = ((bytes + nt - 1) / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    th.reserve(nt);
    auto piece = [=](unsigned i) {
        memcpy((uint8_t*)dst + i * part, (const uint8_t*)src + i * part, std::min(part, bytes - i * part));
    };
    unsigned started = 1;  // pieces [1, started) run on threads
    for (unsigned i = 1; i < nt && i * part < bytes; ++i) {
        try {
            th.emplace_back(piece, i);
        } catch (...) {  // no thread: this piece and the rest are copied here
            break;
        }
        started = i + 1;
    }
    memcpy(dst, src, std::min(part, bytes));
    for (unsigned i = started; i < nt && i * part < bytes; ++i) piece(i);
    for (auto& t : th) t.join();
}

// [0, n) as nb contiguous blocks fn(b, lo, hi) on host threads: the per-run and per-stream
// table loops of a 10^6-stream call (config 5) are memory-bound at one core's bandwidth, ~10 ns
// per entry. Below min_par entries one block runs on the calling thread; a block whose thread
// cannot be started runs here too.
static unsigned par_nblocks(uint64_t n, uint64_t min_par = 1u << 16) {
    const unsigned hw = std::thread::hardware_concurrency();
    static const unsigned cap = [] {  // SKV_HOST_THREADS: host threads for 10^6-entry tables (default 8)
        const char* e = getenv("SKV_HOST_THREADS");
        const long v = e ? atol(e) : 8;
        return (unsigned)std::max(1l, std::min(64l, v));
    }();
    const unsigned nt = std::min<unsigned>(cap, hw ? hw : 1);
    return n < min_par ? 1u : nt;
}
template <typename F>
static void par_run(uint64_t n, unsigned nb, F&& fn) {
    auto lo = [&](unsigned b) { return n * b / nb; };
    std::vector<std::thread> th;
    th.reserve(nb);
    unsigned started = 1;
    for (unsigned b = 1; b < nb; ++b) {
        try {
            th.emplace_back([&, b] { fn(b, lo(b), lo(b + 1)); });
        } catch (...) {
            break;
        }
        started = b + 1;
    }
    fn(0u, lo(0), lo(1));
    for (unsigned b = started; b < nb; ++b) fn(b, lo(b), lo(b + 1));
    for (auto& t : th) t.join();
}
// two-pass block scan: count(lo, hi) -> items of the block; fill(b, lo, hi, base) with base = the
// items of all earlier blocks. Returns the total.
template <typename C, typename F>
static uint64_t par_scan(uint64_t n, C&& count, F&& fill, uint64_t min_par = 1u << 16) {
    const unsigned nb = par_nblocks(n, min_par);
    std::vector<uint64_t> base(nb + 1, 0);
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) { base[b + 1] = count(lo, hi); });
    for (unsigned b = 0; b < nb; ++b) base[b + 1] += base[b];
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) { fill(b, lo, hi, base[b]); });
    return base[nb];
}

// async H2D of a host table through the pinned upload arena
static void h2d_up(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    const size_t need = (bytes + 255) & ~(size_t)255;
    while (ctx->up_chunk < ctx->up_chunks.size() &&
           ctx->up_off + need > ctx->up_chunks[ctx->up_chunk].second) {
        ++ctx->up_chunk;
        ctx->up_off = 0;
    }
    if (ctx->up_chunk == ctx->up_chunks.size()) {
        const size_t cap = std::max<size_t>(need, 1 << 20);
        void* p = nullptr;
        HIPCHK(hipHostMalloc(&p, cap, hipHostMallocDefault));
        ctx->up_chunks.emplace_back((uint8_t*)p, cap);
        ctx->up_off = 0;
    }
    uint8_t* stage = ctx->up_chunks[ctx->up_chunk].first + ctx->up_off;
    ctx->up_off += need;
    stage_copy(stage, src, bytes);
    if (ctx->kernel_uploads) {  // a DMA copy here would queue behind the pipeline's bulk copies
        void* dptr = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dptr, stage, 0));
        launch_copy_bytes(ctx->stream, (uint8_t*)dst, (const uint8_t*)dptr, bytes);
        return;
    }
    HIPCHK(hipMemcpyAsync(dst, stage, bytes, hipMemcpyHostToDevice, ctx->stream));
}

static void d2h(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
}
static void h2d(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// SKV_HOST_TRACE=1: host-side milestones of a call on stderr (ms since the call's first one)
static void htrace(const char* what) {
    static int on = -1;
    static double t0 = 0;
    if (on < 0) {
        const char* e = getenv("SKV_HOST_TRACE");
        on = e && e[0] == '1';
    }
    if (!on) return;
    const double t = now_ms();
    if (!strcmp(what, "entry")) t0 = t;  // each API call starts the clock
    fprintf(stderr, "[skv host] %8.3f ms %s\n", t - t0, what);
}
static void sync(skv_ctx* ctx) {
    const double t0 = now_ms();
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->sync_ms += now_ms() - t0;
    ctx->syncs++;
}
static void mark(skv_ctx* ctx, Phase p) {
    if (ctx->profiling) HIPCHK(hipEventRecord(ctx->ev[p], ctx->stream));
}

// reference Display text of a device error word (runs.rs:83-95, :537-624)
static int derr_to_api(uint32_t e, std::string& msg) {
    uint32_t code = e & 0xFF, extra = e >> 8;
    char buf[128];
    switch (code) {
        case DERR_EMPTY: msg = "Input list of operations cannot be empty"; return SKV_E_EMPTY_INPUT;
        case DERR_VERSION: snprintf(buf, sizeof buf, "Unsupported run version: %u", extra); msg = buf; return SKV_E_UNSUPPORTED_VERSION;
        case DERR_IO: msg = "I/O error: failed to fill whole buffer"; return SKV_E_IO;
        case DERR_KEY: msg = "Data format error: Incomplete key data"; return SKV_E_FORMAT;
        case DERR_UTF8: msg = "Data format error: Invalid UTF-8 in key"; return SKV_E_FORMAT;
        case DERR_VAL: msg = "Data format error: Incomplete value data"; return SKV_E_FORMAT;
        case DERR_MARKER: snprintf(buf, sizeof buf, "Data format error: Invalid marker byte: %u", extra); msg = buf; return SKV_E_FORMAT;
        default: snprintf(buf, sizeof buf, "internal: unknown device error %u", e); msg = buf; return SKV_E_DEVICE;
    }
}

// ------------------------------------------------------------------------------------------
struct Job {
    std::vector<InStream> ranked;  // streams sorted by seq_no descending
    std::vector<uint64_t> run_ptr, run_len;  // member runs, caller order (flat: 10^6-stream jobs)
    uint64_t max_run_size = 0;
    uint32_t flags = 0;
    uint64_t in_bytes = 0;
    bool batch = false;  // writer batch encode (skv_encode_batch): one unsorted run, last op per key wins
    // skv_search_run: one run, the keys (host), the outcomes (host)
    const uint8_t* sr_keys = nullptr;
    const uint64_t* sr_offs = nullptr;
    uint32_t sr_n = 0;
    skv_lookup* sr_out = nullptr;
    bool search = false;
    struct skv_run_index* index_out = nullptr;  // skv_run_index_create: keep the parse, search nothing
};

// a record's key bytes (host copy) for error-trigger comparisons
static std::string fetch_key(skv_ctx* ctx, const uint64_t* d_rec_addr, const uint32_t* d_rec_klen, uint64_t rec) {
    uint64_t addr = 0;
    uint32_t klen = 0;
    HIPCHK(hipMemcpy(&addr, d_rec_addr + rec, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&klen, d_rec_klen + rec, 4, hipMemcpyDeviceToHost));
    std::string k(klen, '\0');
    if (klen) HIPCHK(hipMemcpy(&k[0], (const void*)(addr + 5), klen, hipMemcpyDeviceToHost));
    return k;
}

// JobError::InvalidInput text of a bad WAL key (wal_compaction.rs:71-79; Rust ParseIntError Display)
static std::string wal_key_error(const std::string& key) {
    size_t dot = key.find('.');
    if (dot == std::string::npos) return "Invalid input: Key does not follow 'table_id.key' format: " + key;
    const std::string pre = key.substr(0, dot);
    const char* why = nullptr;
    if (pre.empty()) why = "cannot parse integer from empty string";
    else {
        size_t i = 0;
        bool neg = false;
        if (pre[0] == '+' || pre[0] == '-') {
            neg = pre[0] == '-';
            i = 1;
            if (pre.size() == 1) why = "invalid digit found in string";
        }
        int64_t r = 0;
        for (; !why && i < pre.size(); ++i) {
            if (pre[i] < '0' || pre[i] > '9') { why = "invalid digit found in string"; break; }
            int64_t m, d = pre[i] - '0';
            if (__builtin_mul_overflow(r, (int64_t)10, &m) ||
                (neg ? __builtin_sub_overflow(m, d, &r) : __builtin_add_overflow(m, d, &r)))
                why = neg ? "number too small to fit in target type" : "number too large to fit in target type";
        }
    }
    if (!why) return "internal: WAL key flagged but parses: " + key;
    return "Invalid input: Invalid table ID '" + pre + "': " + why;
}

constexpr int RC_RETRY_EXACT = -100;  // internal: the merge's fingerprint shortcut misordered a tile

template <typename T>
static T read_dev(const T* p) {
    T v{};
    HIPCHK(hipMemcpy(&v, p, sizeof(T), hipMemcpyDeviceToHost));
    return v;
}

// Heap-order mode (skv_heap.hip): the merge reproduced k_way::merge's pop sequence for unsorted
// streams; pop_pos[r] is record r's pop position (r in the merge's numbering; inv maps original
// record indices to it after the record sort). Decode errors surface right after their stream's
// last decodable record is popped (k_way.rs:154-171).
struct HeapRes {
    const uint64_t* pop_pos = nullptr;
    const uint32_t* inv = nullptr;
    struct Dec { uint64_t rec; uint32_t err; };
    std::vector<Dec> dec;
    uint64_t pos_of_original(uint64_t rec) const {
        const uint64_t r = inv ? read_dev(inv + rec) : rec;
        return read_dev(pop_pos + r);
    }
};

// the job's first failure among events at pop positions: (position, order at one position, error)
struct JobEvent {
    uint64_t pos;
    int sub;  // 0: the op itself fails (key / order / send), 1: a send after the op, 2: the stream's
              // decode error, raised after the op at pos was handled
    int code;
    std::string msg;
};
static void throw_first(std::vector<JobEvent>& ev) {
    if (ev.empty()) return;
    std::sort(ev.begin(), ev.end(), [](const JobEvent& a, const JobEvent& b) {
        return a.pos != b.pos ? a.pos < b.pos : a.sub < b.sub;
    });
    throw ApiError{ev[0].code, ev[0].msg};
}
static int compact_device(skv_ctx* ctx, const Job& job, skv_result** out, bool allow_deferred);
// the whole call again with exact key compares in the merge rounds
static int rerun_exact(skv_ctx* ctx, const Job& job, skv_result** out) {
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

// SKV_SPLIT_BY_TABLE after the merge: table split, prefix strip, one run per kept table
// (skv_wal.hip). One extra host sync reads the surviving record count first.
static int wal_stage(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint32_t* m_rec,
                     const uint64_t* m_src, const uint64_t* m_P, const uint64_t* m_Dp, const uint64_t* rec_addr,
                     const uint32_t* rec_klen, const uint32_t* fp_bad, const HeapRes* heap, skv_result** out) {
    hipStream_t st = ctx->stream;
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
    launch_wal_keys(st, d_K, K, m_src, m_rec, rec_klen, m_P, tid, strip, wsize, canon, first_err);
    launch_wal_flags(st, d_K, K, tid, strip, canon, m_src, m_rec, rec_klen, is_new, bad, heap != nullptr);
    launch_scan(st, is_new, K, new_ex, scan_tmp);  // new_ex[K] = number of tables
    launch_wal_index(st, d_K, K, is_new, new_ex, bad, tix, tstart, tbad, tfirst);
    launch_wal_sendfail(st, new_ex + K, K, tstart, tfirst, first_err + 1);
    launch_scan(st, wsize, K, Pw, scan_tmp);       // stripped record offsets
    const uint64_t* d_NT = new_ex + K;
    launch_wal_tables(st, d_NT, K, tstart, Pw, tbad, job.max_run_size, run_len, keep);
    launch_scan_dn(st, run_len, d_NT, K, run_off, scan_tmp);  // output offset per table, total at [K]
    launch_scan_dn(st, keep, d_NT, K, keep_ex, scan_tmp);     // run index per kept table, count at [K]
    launch_wal_desc(st, d_NT, K, tstart, Pw, m_Dp, keep, keep_ex, run_off, tid, strip, m_rec, rec_klen, d_desc);
    mark(ctx, PH_CHAIN);
    launch_wal_gather(st, d_K, K, tix, tstart, keep, run_off, Pw, strip, m_src, m_rec, rec_klen, d_out);
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
                      wal_key_error(fetch_key(ctx, rec_addr, rec_klen, read_dev(m_rec + h[0])))});
    if (h[4] != ~0ull)
        ev.push_back({pos_of_survivor(h[4]), 1, SKV_E_INTERNAL, "Internal error: Failed to send operation to table channel"});
    if (heap)
        for (const HeapRes::Dec& d : heap->dec) {
            std::string msg;
            const int code = derr_to_api(d.err, msg);
            ev.push_back({heap->pos_of_original(d.rec), 2, code, msg});
        }
    if (getenv("SKV_HEAP_DEBUG")) {
        fprintf(stderr, "[wal] K=%llu heap=%d badkey=%lld sendfail=%lld\n", (unsigned long long)K, heap ? 1 : 0,
                (long long)h[0], (long long)h[4]);
        for (const JobEvent& e : ev) fprintf(stderr, "  event pos=%llu sub=%d code=%d %s\n", (unsigned long long)e.pos, e.sub, e.code, e.msg.c_str());
        if (heap)
            for (uint64_t r = 0; r < R && r < 64; ++r)
                fprintf(stderr, "  rec %llu pop=%llu\n", (unsigned long long)r, (unsigned long long)read_dev(heap->pop_pos + r));
    }
    throw_first(ev);
    const uint64_t n_tables = h[1], n_kept = h[2], n_bytes = h[3];
    ResultBox* box = new ResultBox();
    skv_result* res = &box->pub;
    res->runs = (skv_run_desc*)malloc(std::max<uint64_t>(1, n_kept) * sizeof(skv_run_desc));
    if (n_kept) HIPCHK(hipMemcpy(res->runs, d_desc, n_kept * sizeof(DevRunDesc), hipMemcpyDeviceToHost));
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
    ctx->timings.path = SKV_PATH_GENERAL;  // WAL stage: the dominant launch is k_wal_gather
    ctx->timings.hot_read_bytes = n_bytes - n_kept;
    ctx->timings.hot_write_bytes = n_bytes;
    ctx->timings.host_syncs = ctx->syncs;
    *out = res;
    return SKV_OK;
}

// The fused stride path (skv_stride.hip): every run is fixed-stride with one record size S and one
// key length K <= 16. Splitters, then one fused verify/merge/copy kernel, then the descriptors;
// one host sync reads the descriptors together with the verdict. Returns false when the device
// poisoned the call (a record or key order the run's first record did not promise, or splitter
// skew): the caller then reruns the exact path, which produces the reference's outcome.
// records per output run of the fused path (build_runs' greedy split is arithmetic at one size)
static uint64_t fx_run_records(uint64_t max_run_size, uint64_t S, uint64_t R) {
    uint64_t n = max_run_size >= 1 ? (max_run_size - 1) / S : 0;  // runs.rs:211-238
    if (n < 1) n = 1;  // a record that alone exceeds max still forms its own run (runs.rs:219)
    if (n > R) n = R;
    return n;
}

// Where a fused launch's survivors go: a key-range part of a pipelined host call chains its
// survivor numbering through device words and shares one output buffer and one verdict.
struct FxPartIO {
    const uint64_t* gbase = nullptr;  // survivors of the earlier parts (device)
    uint64_t* Kout = nullptr;         // survivors through this part (device)
    uint32_t* flags = nullptr;        // shared verdict flags (device, zeroed by the caller)
    uint8_t* out = nullptr;           // shared output bytes (device)
};

// The fused stride path up to and including k_fx_tile, on ctx->stream, with no host sync:
// splitters (levels sized from host-known counts) and the fused tiles. d_rb: the blob's readback
// words {runs, K, bytes} + flags (whole-call launches).
static FxArgs fx_launch(skv_ctx* ctx, uint32_t k, uint32_t n_runs, const RunInfo* d_runs,
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
        const char* te = getenv("SKV_FX_TAIL");
        if (lv.size() > 1 && m0 >= 4 && !(te && te[0] == '0')) {
            const char* se = getenv("SKV_FX_TAIL_SLOTS");  // tests: a small grid's worth of slots
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
        const Level& P = lv[li - 1];
        char nm[64];
        snprintf(nm, sizeof nm, "lv%d_hi", (int)li); L.hi = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_lo", (int)li); L.lo = dbuf<uint64_t>(ctx, nm, L.N);
        snprintf(nm, sizeof nm, "lv%d_c", (int)li); L.c = dbuf<uint64_t>(ctx, nm, L.N);
        L.d_off = (uint64_t*)(d_blob + lv_off[li]);
        if (li == 1) launch_fx_sample(st, A, L.d_off, L.S, L.N, L.hi, L.lo, L.c);
        else launch_sample(st, false, P.hi, P.lo, P.c, nullptr, P.d_off, L.d_off, k, L.S, L.N, L.hi, L.lo, L.c);
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
static bool compact_fused(skv_ctx* ctx, const Job& job, const std::vector<RunInfo>& runs, const RunInfo* d_runs,
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
    t.hot_read_bytes = K * f.S + (R - K) * (9 + (uint64_t)f.K);  // survivors whole, superseded: header + key
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

// Sorts n SElems by (key, record index) (skv_sort.hip); E and T are n-element buffers, the
// result is in the returned one of the two. Samples recurse with their own buffers (depth).
static SElem* sort_elems(skv_ctx* ctx, SElem* E, SElem* T, uint64_t n, int depth, uint64_t* newkey = nullptr) {
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
    // depth 0 (the records themselves): the bucket search stores each element's window from its
    // bucket's common prefix on, so the bucket sort reads no record bytes; its output keeps only
    // addr / pos / klen meaningful (sort_records reads no more). Sample levels keep their keys.
    const bool pre = depth == 0;
    launch_sort_bucket(st, E, n, Ss, SORT_OV, Tb - 1, split_buf, cnt, bs, pre ? L : nullptr);
    launch_scan(st, cnt, Tb, start, scan_tmp);
    launch_sort_scatter(st, E, n, bs, start, T);
    launch_sort_tile(st, T, start, L, Tb, E, newkey, pre);
    return E;
}

// The merged order of R records as one sorted list: the record arrays are replaced by sorted
// copies (merges of more than TILE_TARGET / 2 streams, whose splitter bounds table would be
// tiles x streams). hi/lo/cmp_klen become dense key ranks for the merge stage; klen stays the real
// key length (descriptors, WAL split).
static void sort_records(skv_ctx* ctx, uint64_t R, uint64_t*& hi, uint64_t*& lo, uint64_t*& addr, uint32_t*& klen,
                         uint32_t*& meta, const uint32_t*& cmp_klen, bool last_wins, const SElem** sorted = nullptr) {
    hipStream_t st = ctx->stream;
    SElem* E = dbuf<SElem>(ctx, "sort_e", R);
    SElem* T = dbuf<SElem>(ctx, "sort_t", R);
    uint64_t* newkey = dbuf<uint64_t>(ctx, "sort_newkey", R + 1);
    uint64_t* newkey_ex = dbuf<uint64_t>(ctx, "sort_newkey_ex", R + 1);
    uint64_t* scan_tmp = dbuf<uint64_t>(ctx, "sort_rank_scan", scan_tmp_words(R) + 64);
    launch_sort_load(st, R, hi, lo, addr, klen, E, last_wins);
    const SElem* S = sort_elems(ctx, E, T, R, 0, newkey);
    launch_scan(st, newkey, R, newkey_ex, scan_tmp);
    uint64_t* nhi = dbuf<uint64_t>(ctx, "srt_hi", R);
    uint64_t* nlo = dbuf<uint64_t>(ctx, "srt_lo", R);
    uint64_t* naddr = dbuf<uint64_t>(ctx, "srt_addr", R);
    uint32_t* nklen = dbuf<uint32_t>(ctx, "srt_klen", R);
    uint32_t* ncklen = dbuf<uint32_t>(ctx, "srt_cklen", R);
    uint32_t* nmeta = dbuf<uint32_t>(ctx, "srt_meta", R);
    launch_sort_store(st, R, S, meta, newkey, newkey_ex, nhi, nlo, naddr, nklen, ncklen, nmeta, last_wins);
    HIPCHK(hipGetLastError());
    if (sorted) *sorted = S;
    hi = nhi;
    lo = nlo;
    addr = naddr;
    klen = nklen;
    meta = nmeta;
    cmp_klen = ncklen;
}

// A run parsed once for many lookup batches (skv_run_index_create): the run bytes and its record
// arrays stay in HBM, owned by the index (the cache service keeps one per cached run,
// cache_service.rs:52-94).
struct skv_run_index {
    int device = 0;
    uint64_t len = 0;
    uint32_t panic_all = 0;  // empty run / bad version: every lookup panics (runs.rs:288-297)
    bool clean = false;      // parsed without error or key decrease: binary search, else the scan
    uint64_t R = 0;
    void* mem = nullptr;     // one allocation: run bytes | rec_addr | rec_hi | rec_lo | rec_klen | rec_meta
    const uint8_t* run = nullptr;
    const uint64_t *addr = nullptr, *hi = nullptr, *lo = nullptr;
    const uint32_t *klen = nullptr, *meta = nullptr;
};

// the lookups of one batch against parsed arrays (bsearch) or the run bytes (scan)
static void search_launch(skv_ctx* ctx, const uint8_t* run, uint64_t len, bool clean, uint64_t R,
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
static int search_stage(skv_ctx* ctx, const Job& job, const RunInfo& run, uint64_t R, uint32_t run_err,
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

static void ensure_aux(skv_ctx* ctx) {  // the ctx's second stream and its two events
    if (ctx->aux_stream) return;
    HIPCHK(hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ctx->aux_ev[0], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->aux_ev[1], hipEventDisableTiming));
}

// allow_deferred: on the fixed-stride fast path, launch the merge without waiting for the parse's
// verdict (broken runs / order errors / oversized records) and check it with the final readback;
// a bad verdict discards the result and reruns the call on the exact general path.
static int compact_device(skv_ctx* ctx, const Job& job, skv_result** out, bool allow_deferred) {
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
    // speculative walk length: CHUNK, doubled up to 4x while a call still has >= 2^20 walks (a big
    // call spends fewer re-synchronising starts per record; 4 KiB walks of 64 GB: 56 ms, 16 KiB: 44)
    uint64_t chunk = CHUNK;
    if (const char* ce = getenv("SKV_CHUNK_BYTES"))  // slot offsets are 16-bit: at most 64 KiB
        chunk = std::min<uint64_t>(65536, std::max<uint64_t>(CHUNK, strtoull(ce, nullptr, 10)));
    else
        while (chunk < 4 * CHUNK && job.in_bytes / (2 * chunk) >= (1ull << 20)) chunk *= 2;
    auto n_chunks_of = [chunk](uint64_t len) { return len >= 2 ? (uint32_t)((len - 1 + chunk - 1) / chunk) : 0u; };
    uint64_t n_chunks = 0;
    {  // blocks of streams (rank order) on host threads: runs and chunks before each block, then fill
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
    }
    stream_first_run[k] = (uint32_t)runs.size();
    const uint32_t n_runs = (uint32_t)runs.size();
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

    h2d_up(ctx, d_runs, runs.data(), n_runs * sizeof(RunInfo));
    htrace("runs uploaded");
    RunFmt* d_fmt = dbuf<RunFmt>(ctx, "run_fmt", n_runs);
    uint32_t* d_broken = dbuf<uint32_t>(ctx, "run_broken", n_runs);
    uint64_t* d_recb = dbuf<uint64_t>(ctx, "run_recb", n_runs + 1);
    HIPCHK(hipMemsetAsync(d_broken, 0, (size_t)n_runs * 4, st));
    launch_run_header(st, d_runs, n_runs, d_hdr, d_fmt);

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
    uint32_t hflags[4];
    // per stream (rank order): base index, valid record count n_s and the first error
    auto stream_tables = [&]() {  // blocks of streams on host threads (10^6-stream calls)
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
    auto alloc_records = [&]() {
        rec_addr = dbuf<uint64_t>(ctx, "rec_addr", R);
        rec_hi = dbuf<uint64_t>(ctx, "rec_hi", R);
        rec_lo = dbuf<uint64_t>(ctx, "rec_lo", R);
        rec_klen = dbuf<uint32_t>(ctx, "rec_klen", R);
        rec_meta = dbuf<uint32_t>(ctx, "rec_meta", R);
        rec_fp = dbuf<uint64_t>(ctx, "rec_fp", R);
        HIPCHK(hipMemsetAsync(d_flags, 0, 16, st));
        HIPCHK(hipMemsetAsync(utf8_bad, 0, 4, st));
        HIPCHK(hipMemsetAsync(d_first_dec, 0xFF, (size_t)k * 8, st));
        h2d_up(ctx, d_stream_base, stream_base.data(), (k + 1) * 8);
    };
    uint32_t utf8_flag = 0;
    // order check + readback of its result, the record flags and (fast path) the broken-run flags
    auto check_and_read = [&](bool read_broken) -> bool {
        // the fast path's parse kernel already did the order check
        if (!read_broken && !job.batch)  // a writer batch is unsorted by definition
            launch_order_check(st, R, d_stream_base, k, rec_addr, rec_hi, rec_lo, rec_klen, d_first_dec, d_flags + 1);
        HIPCHK(hipGetLastError());
        uint8_t* hp = (uint8_t*)pinned(ctx, k * 8 + 16 + (read_broken ? n_runs * 4 : 0) + 16);
        d2h(ctx, hp, d_first_dec, (size_t)k * 8);
        d2h(ctx, hp + (size_t)k * 8, d_flags, 16);
        uint8_t* hu = hp + k * 8 + 16 + (read_broken ? n_runs * 4 : 0);
        d2h(ctx, hu, utf8_bad, 4);
        if (read_broken) d2h(ctx, hp + (size_t)k * 8 + 16, d_broken, (size_t)n_runs * 4);
        sync(ctx);
        memcpy(first_dec.data(), hp, (size_t)k * 8);
        memcpy(hflags, hp + (size_t)k * 8, 16);
        memcpy(&utf8_flag, hu, 4);
        bool broken = false;
        if (read_broken) {
            const uint32_t* b = (const uint32_t*)(hp + (size_t)k * 8 + 16);
            for (uint32_t r = 0; r < n_runs && !broken; ++r) broken = b[r] != 0;
        }
        return broken;
    };

    // ---- fast path: every run fixed-stride (one record size per run) -> one verifying pass ------
    bool parsed = false, deferred = false;
    bool any_fixed = false;  // some run is fixed-stride: the general parse also runs k_emit_fixed
    {
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
            const char* fenv = getenv("SKV_FUSED");
            if (allow_deferred && uniform && !job.batch && !job.search && !(job.flags & SKV_SPLIT_BY_TABLE) &&
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
            launch_parse_fixed(st, d_runs, n_runs, d_fmt, d_broken, d_recb, R, rec_addr, rec_hi, rec_lo, rec_klen,
                               rec_meta, d_flags, d_stream_base, job.batch ? nullptr : d_first_dec, rec_fp,
                               dbuf<uint32_t>(ctx, "wave_run", (R + 63) / 64 + 1));
            mark(ctx, PH_PARSE);
            if (allow_deferred && !(job.flags & SKV_SPLIT_BY_TABLE) && !job.search) {
                deferred = true;  // verdict read with the result
                parsed = true;
                std::fill(first_dec.begin(), first_dec.end(), ~0ull);
                memset(hflags, 0, sizeof hflags);
            } else {
                parsed = !check_and_read(true);
                htrace("parse verdict read");
            }
            if (!parsed) {  // a run is not what its first record promised: general parse
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
        HIPCHK(hipMemsetAsync(bad_bits, 0, (n_chunks / 64 + 1) * 8, st));
        HIPCHK(hipMemsetAsync(first_bad, 0xFF, n_runs * 4, st));
        HIPCHK(hipMemsetAsync(err_chunk, 0xFF, n_runs * 4, st));
        launch_spec(st, d_runs, n_runs, n_chunks, d_hdr, d_fmt, d_broken, ch_start, ch_end, ch_cnt, ch_err,
                    ctx->exact_utf8, chunk, ch_slots, slot_cap);
        launch_validate(st, d_runs, n_runs, n_chunks, d_hdr, ch_start, ch_end, ch_err, bad_bits, first_bad);
        launch_fixup(st, d_runs, n_runs, d_hdr, first_bad, bad_bits, ch_start, ch_end, ch_cnt, ch_err,
                     ctx->exact_utf8, chunk, ch_slots, slot_cap);
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
        launch_emit(st, d_runs, n_runs, n_chunks, d_fmt, d_broken, ch_start, ch_rec_base, d_recb, any_fixed ? R : 0,
                    rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, d_flags, rec_fp, utf8_bad, ch_slots, slot_cap, chunk);
        mark(ctx, PH_PARSE);
        check_and_read(false);
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
    if (job.search) return search_stage(ctx, job, runs[0], R, stream_err[0], first_dec[0], rec_addr, rec_hi, rec_lo,
                                        rec_klen, rec_meta);
    bool any_dec = false;
    for (uint32_t s = 0; s < k; ++s)
        if (first_dec[s] != ~0ull && first_dec[s] + 1 < stream_valid[s]) any_dec = true;

    // ---- errors: which one k_way::merge surfaces first --------------------------------------
    // Heap-order mode (skv_heap.hip) where the outcome depends on the merge's exact pop sequence
    // past a stream's first key decrease or decode error: the WAL split with either, and the Delete
    // filter with a decrease. Everywhere else the first trigger record decides (below).
    const bool wal = (job.flags & SKV_SPLIT_BY_TABLE) != 0;
    const bool heap = !job.batch && ((wal && (any_err || any_dec)) || ((job.flags & SKV_DROP_TOMBSTONES) && any_dec));
    HeapRes hres;
    if (any_err || any_dec) {
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
    std::vector<uint64_t> list_off = stream_base;
    uint64_t* d_list_off = d_stream_base;
    {
        const char* se = getenv("SKV_SORT");
        if ((k > (uint32_t)TILE_TARGET / 2 && R > (uint64_t)TILE_CAP) || (se && se[0] == '1') || job.batch) {
            if (heap) {
                // sort on the merge keys; the records' own keys, payload and meta follow in sorted
                // order, and inv maps an original record index to its sorted position
                uint64_t *h2 = cmp_hi, *l2 = cmp_lo, *a2 = (uint64_t*)cmp_addr;
                uint32_t* k2 = (uint32_t*)cmp_klen;
                uint32_t* m2 = rec_meta;
                const uint32_t* ck = nullptr;
                const SElem* S = nullptr;
                sort_records(ctx, R, h2, l2, a2, k2, m2, ck, false, &S);
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
                sort_records(ctx, R, rec_hi, rec_lo, rec_addr, rec_klen, rec_meta, cmp_klen, job.batch);
                cmp_hi = rec_hi;
                cmp_lo = rec_lo;
                cmp_addr = rec_addr;
            }
            htrace("sort launched");
            km = 1;
            list_off = {0, R};
            d_list_off = dbuf<uint64_t>(ctx, "sorted_off", 2);
            h2d_up(ctx, d_list_off, list_off.data(), 16);
            ctx->timings.sorted = 1;
        }
    }
    std::vector<Level> lv(1);
    lv[0].N = R;
    lv[0].off = list_off;
    lv[0].hi = cmp_hi;
    lv[0].lo = cmp_lo;
    lv[0].d_off = d_list_off;
    const uint64_t S_step = std::max<uint64_t>(2, (uint64_t)TILE_TARGET / std::max<uint32_t>(km, 1));
    // SKV_HI_STEP=f: levels >= 2 (they only pick splitters for the sample sorts) at an f times
    // coarser step. Measured at config 3 with f = 2: one sample level fewer, but the merge phase
    // 4.02 vs 3.26 ms (the level-1 sample tiles lose their balance), so the default is 1.
    const char* hse = getenv("SKV_HI_STEP");
    const uint64_t hi_f = hse ? std::max<uint64_t>(1, strtoull(hse, nullptr, 10)) : 1;
    // Level 1 (the level-0 tiles' splitters) at twice the step from 128 lists on: a tile's size
    // spreads by ~sqrt(k) x step / 2.4 records around TILE_TARGET, which at k >= 128 stays under
    // 1/4.6 of the TILE_CAP margin, and half the samples halve their sort (3F merge 27.3 -> 25.7 ms,
    // config 3 2.22 -> 1.92 ms; a step of 3 unbalanced the tiles: 31.4 ms). SKV_L1_STEP=f overrides.
    const char* l1e = getenv("SKV_L1_STEP");
    const uint64_t l1_f = l1e ? std::max<uint64_t>(1, strtoull(l1e, nullptr, 10)) : (km >= 128 ? 2 : 1);
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
    const unsigned long long* verify_lo = nullptr;  // pairs before it verified beside the merge
    bool verify_pending = false;
    if (km > 1 && !ctx->exact_keys && !heap) {
        const char* te = getenv("SKV_FP_TEST");
        if (te && te[0] == '1') {
            uint64_t* f = dbuf<uint64_t>(ctx, "rec_fp_test", R);
            HIPCHK(hipMemsetAsync(f, 0, R * 8, st));
            key_fp = f;
        } else {
            key_fp = rec_fp;  // written by the emit kernels with the record arrays
        }
    }
    for (int li = (int)lv.size() - 1; li >= 0; --li) {
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
        // SKV_FP_PIECE_MIN=T: split level 0 from T tiles on (off by default: at 3F the verify beside
        // the merge pieces slowed the merge by what it saved beside the gather, 89.6 vs 89.3 ms)
        const char* pme = getenv("SKV_FP_PIECE_MIN");
        const uint64_t piece_min = pme ? std::max<uint64_t>(1, strtoull(pme, nullptr, 10)) : ~0ull;
        if (l0 && key_fp && T >= piece_min && T >= 4) {
            // Level 0 in FP_PIECES launches (tickets continue across them): after each piece but
            // the last, a one-lane kernel snapshots the pair count, and k_fp_verify checks that
            // piece's pairs on the aux stream while the next piece merges; the last piece's pairs
            // are checked beside the gather. Measured neutral: the verify's random record reads
            // cost the LDS-bound merge about what they cost the gather.
            constexpr int FP_PIECES = 4;
            uint64_t* snap = dbuf<uint64_t>(ctx, "fp_vsnap", FP_PIECES);
            ensure_aux(ctx);
            uint64_t done = 0;
            for (int p = 0; p < FP_PIECES; ++p) {
                const uint64_t upto = T * (uint64_t)(p + 1) / FP_PIECES;
                HIPCHK(launch_tile(st, l0, L.hi, L.lo, L.c, cmp_klen, bounds, km, T, tile_base, rec_meta, cmp_addr,
                                   drop, O, d_flags + 2, upto - done));
                done = upto;
                if (p + 1 < FP_PIECES) {
                    launch_fx_publish(st, (const uint64_t*)O.vcount, snap + p);
                    HIPCHK(hipEventRecord(ctx->aux_ev[0], st));
                    HIPCHK(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_ev[0], 0));
                    launch_fp_verify(ctx->aux_stream, p ? (const unsigned long long*)(snap + p - 1) : nullptr,
                                     (const unsigned long long*)(snap + p), O.vpairs, R, fp_bad, 1024);
                    verify_pending = true;
                }
            }
            HIPCHK(hipEventRecord(ctx->aux_ev[1], ctx->aux_stream));
            verify_lo = (const unsigned long long*)(snap + FP_PIECES - 2);
        } else {
            HIPCHK(launch_tile(st, l0, L.hi, L.lo, L.c, cmp_klen, bounds, km, T, tile_base, rec_meta, cmp_addr, drop,
                               O, d_flags + 2));
        }
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
    if (job.flags & SKV_SPLIT_BY_TABLE) {
        join_verify();
        htrace("merge launched");
        const int rc =
            wal_stage(ctx, job, R, d_K, m_rec, m_src, m_P, m_Dp, rec_addr, rec_klen, fp_bad, heap ? &hres : nullptr, out);
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
        if (getenv("SKV_HEAP_DEBUG")) {  // diagnostic: the merged sequence of heap-order mode
            const uint64_t K = read_dev(d_K);
            fprintf(stderr, "[heap] R=%llu K=%llu first_bad=%lld\n", (unsigned long long)R, (unsigned long long)K,
                    (long long)v);
            const uint32_t* effp = (const uint32_t*)ctx->bufs["heap_eff"].p;
            for (uint64_t i = 0; i < R && i < 40; ++i)
                fprintf(stderr, "  rec %llu hi=%016llx lo=%016llx klen=%u eff=%u key=%s\n", (unsigned long long)i,
                        (unsigned long long)read_dev(rec_hi + i), (unsigned long long)read_dev(rec_lo + i),
                        read_dev(rec_klen + i), effp ? read_dev(effp + i) : 0u, fetch_key(ctx, rec_addr, rec_klen, i).c_str());
            for (uint64_t g = 0; g < K && g < 200; ++g) {
                const uint32_t r = read_dev(m_rec + g);
                fprintf(stderr, "  g=%llu rec=%u pop=%llu key=%s cmpkey=%s\n", (unsigned long long)g, r,
                        (unsigned long long)read_dev(pop_pos + r), fetch_key(ctx, rec_addr, rec_klen, r).c_str(),
                        fetch_key(ctx, cmp_addr, cmp_klen, r).c_str());
            }
        }
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
        const char* mode = getenv("SKV_SPLIT");
        const bool serial = mode && !strcmp(mode, "serial");
        sp.segr = 16;
        sp.nc = 512;
        sp.min_runs = mode && !strcmp(mode, "par") ? 0 : 1024;
        if (const char* e = getenv("SKV_SPLIT_NC")) sp.nc = (uint32_t)std::min<uint64_t>(8192, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
        if (const char* e = getenv("SKV_SPLIT_SEG")) sp.segr = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, strtoull(e, nullptr, 10)));
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
    launch_chain(st, d_K, m_P, job.max_run_size, tile_max, T0, run_b, d_nruns, chain_tbl, R, in_rec_bytes, &sp);
    if (sp.nseg_cap && getenv("SKV_SPLIT_DEBUG")) {
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
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", total_rec_bytes + R + 16);
#if SKV_PAGE_GATHER
    {
        const uint64_t max_out = total_rec_bytes + R + 16;
        uint64_t* Dst = dbuf<uint64_t>(ctx, "g_dst", R + 1);
        uint32_t* page_first = dbuf<uint32_t>(ctx, "g_page_first", max_out / PAGE_BYTES + 2);
        launch_page_prep(st, d_K, d_nruns, run_b, m_P, seg_r0, Dst, page_first, R);
        mark(ctx, PH_CHAIN);
        launch_gather_pages(st, d_K, d_nruns, m_P, Dst, m_src, page_first, d_out, max_out);
    }
#else
    launch_gather(st, d_K, d_nruns, run_b, m_P, m_src, seg_r0, d_out, R);
#endif
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

// ------------------------------------------------------------------------------------------
static int build_job_impl(skv_ctx* ctx, const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags,
                     Job& job) {
    if (n && !streams) return set_err(ctx, SKV_E_INVALID_ARG, "streams is NULL");
    if (flags & ~(uint32_t)(SKV_DROP_TOMBSTONES | SKV_SPLIT_BY_TABLE))
        return set_err(ctx, SKV_E_INVALID_ARG, "unknown flags 0x%x", flags);
    if ((flags & SKV_SPLIT_BY_TABLE) && (flags & SKV_DROP_TOMBSTONES))
        return set_err(ctx, SKV_E_INVALID_ARG, "SKV_SPLIT_BY_TABLE and SKV_DROP_TOMBSTONES are exclusive");
    job.max_run_size = max_run_size;
    job.flags = flags;
    // pass 1 (blocks of streams on host threads): NULL checks, run counts, input bytes, and
    // whether the caller's order is strictly ascending / descending by seq_no
    const unsigned nb = par_nblocks(n);
    struct Blk {
        uint64_t runs = 0, bytes = 0, bad = ~0ull;
        uint32_t bad_run = ~0u;
        bool asc = true, desc = true;
    };
    std::vector<Blk> B(nb);
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
        Blk& K = B[b];
        for (uint64_t i = lo; i < hi; ++i) {
            const skv_stream& s = streams[i];
            if (s.n_runs && (!s.runs || !s.run_lens)) {
                K.bad = i;
                return;
            }
            for (uint32_t r = 0; r < s.n_runs; ++r) {
                if (s.run_lens[r] && !s.runs[r]) {
                    K.bad = i;
                    K.bad_run = r;
                    return;
                }
                K.bytes += s.run_lens[r];
            }
            K.runs += s.n_runs;
            if (i > 0) {
                K.asc = K.asc && streams[i - 1].seq_no < s.seq_no;
                K.desc = K.desc && streams[i - 1].seq_no > s.seq_no;
            }
        }
    });
    bool asc = true, desc = true;
    uint64_t total_runs = 0;
    for (unsigned b = 0; b < nb; ++b) {  // the first invalid stream in the caller's order
        if (B[b].bad != ~0ull) {
            if (B[b].bad_run == ~0u)
                return set_err(ctx, SKV_E_INVALID_ARG, "stream %u: runs/run_lens is NULL", (uint32_t)B[b].bad);
            return set_err(ctx, SKV_E_INVALID_ARG, "stream %u run %u: NULL data", (uint32_t)B[b].bad, B[b].bad_run);
        }
        const uint64_t r = B[b].runs;
        B[b].runs = total_runs;  // now the block's first run
        total_runs += r;
        job.in_bytes += B[b].bytes;
        asc = asc && B[b].asc;
        desc = desc && B[b].desc;
    }
    // pass 2: the tables, streams already in rank order (seq_no descending) when the caller's
    // order is either strict one; resize keeps a lent table's entries (no zero fill per call)
    job.run_ptr.resize(total_runs);
    job.run_len.resize(total_runs);
    job.ranked.resize(n);
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
        uint64_t at = B[b].runs;
        for (uint64_t i = lo; i < hi; ++i) {
            const skv_stream& s = streams[i];
            InStream& S = job.ranked[asc ? n - 1 - i : i];
            S.seq = s.seq_no;
            S.vec_idx = (uint32_t)i;
            S.n_runs = s.n_runs;
            S.first = at;
            for (uint32_t r = 0; r < s.n_runs; ++r, ++at) {
                job.run_ptr[at] = (uint64_t)(uintptr_t)s.runs[r];
                job.run_len[at] = s.run_lens[r];
            }
        }
    });
    if (!asc && !desc) {
        std::stable_sort(job.ranked.begin(), job.ranked.end(),
                         [](const InStream& a, const InStream& b) { return a.seq > b.seq; });
        for (size_t i = 1; i < job.ranked.size(); ++i)
            if (job.ranked[i].seq == job.ranked[i - 1].seq)
                return set_err(ctx, SKV_E_INVALID_ARG, "duplicate seq_no %" PRId64, job.ranked[i].seq);
    }
    return SKV_OK;
}

// the job tables of a call (10^6-stream calls: vectors of that size) without unwinding into C
static int build_job(skv_ctx* ctx, const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags,
                     Job& job) {
    try {
        return build_job_impl(ctx, streams, n, max_run_size, flags, job);
    } catch (const std::exception& e) {
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
}

// after an error: every stream of the ctx idle before its buffers are reused
static void drain(skv_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->aux_stream) (void)hipStreamSynchronize(ctx->aux_stream);
}

static int run_guarded(skv_ctx* ctx, const Job& job, skv_result** out, double t_entry) {
    try {
        ctx->sync_ms = 0;
        ctx->timings = skv_timings{};
        const int rc = compact_device(ctx, job, out, true);
        ctx->timings.host_total_ms = now_ms() - t_entry;
        ctx->timings.host_sync_ms = ctx->sync_ms;
        return rc;
    } catch (const ApiError& e) {
        drain(ctx);
        return set_err(ctx, e.code, "%s", e.msg.c_str());
    } catch (const DevError& e) {
        drain(ctx);
        return set_err(ctx, SKV_E_DEVICE, "%s", e.msg.c_str());
    } catch (const std::exception& e) {  // bad_alloc of a host table, system_error, ...: never unwind into C
        drain(ctx);
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
}

extern "C" {

int skv_abi_version(void) { return SKV_ABI_VERSION; }

int skv_device_count(int* out) {
    if (!out) return SKV_E_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return SKV_OK;
}

int skv_ctx_create(int device, skv_ctx** out) {
    if (!out) return SKV_E_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return SKV_E_DEVICE;
    if (device < 0 || device >= n) return SKV_E_INVALID_ARG;
    skv_ctx* ctx = new skv_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SKV_E_DEVICE;
    }
    for (int i = 0; i < PH_N; ++i) (void)hipEventCreate(&ctx->ev[i]);
    *out = ctx;
    return SKV_OK;
}

void skv_ctx_destroy(skv_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
#if SKV_TILE_PROF
    if (ctx->bufs.count("tile_prof")) {
        uint64_t pr[16] = {};
        const size_t nb = ctx->bufs["tile_prof"].cap >= 128 ? 128 : 64;
        if (hipMemcpy(pr, ctx->bufs["tile_prof"].p, nb, hipMemcpyDeviceToHost) == hipSuccess) {
            fprintf(stderr, "tile phase time (100 MHz ticks summed over tiles; [15] = tiles):");
            for (int i = 0; i < (int)(nb / 8); ++i) fprintf(stderr, " %d:%llu", i, (unsigned long long)pr[i]);
            fprintf(stderr, "\n");
        }
    }
#endif
    for (auto& kv : ctx->bufs)
        if (kv.second.p) (void)hipFree(kv.second.p);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    for (auto& c : ctx->up_chunks) (void)hipHostFree(c.first);
    for (int i = 0; i < PH_N; ++i)
        if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
    for (hipEvent_t e : ctx->part_ev) (void)hipEventDestroy(e);
    if (ctx->aux_stream) {
        (void)hipStreamSynchronize(ctx->aux_stream);
        (void)hipStreamDestroy(ctx->aux_stream);
    }
    for (hipEvent_t e : ctx->aux_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->part_k) (void)hipHostFree(ctx->part_k);
    if (ctx->in_stream) {
        (void)hipStreamSynchronize(ctx->in_stream);
        (void)hipStreamDestroy(ctx->in_stream);
    }
    if (ctx->out_stream) {
        (void)hipStreamSynchronize(ctx->out_stream);
        (void)hipStreamDestroy(ctx->out_stream);
    }
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* skv_last_error(const skv_ctx* ctx) { return ctx ? ctx->err.c_str() : "ctx is NULL"; }

int skv_ctx_set_profiling(skv_ctx* ctx, int enable) {
    if (!ctx) return SKV_E_INVALID_ARG;
    ctx->profiling = enable != 0;
    return SKV_OK;
}

int skv_ctx_get_timings(const skv_ctx* ctx, skv_timings* out) {
    if (!ctx || !out) return SKV_E_INVALID_ARG;
    *out = ctx->timings;
    return SKV_OK;
}

int skv_compact_dev(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams, uint64_t max_run_size, uint32_t flags,
                    skv_result** out) {
    const double t_entry = now_ms();
    htrace("entry");
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
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

}  // extern "C"

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

static int compact_host_job(skv_ctx* ctx, Job& job, skv_result** out, double t_entry);

static bool pipe_eligible(const Job& job, RunFmt& f, uint64_t& R) {
    const char* pe = getenv("SKV_HOST_PIPE");
    if (pe && pe[0] == '0') return false;
    const char* me = getenv("SKV_HOST_PIPE_MIN");
    const uint64_t min_bytes = me ? strtoull(me, nullptr, 10) : (512ull << 20);
    const uint32_t k = (uint32_t)job.ranked.size();
    if (job.in_bytes < min_bytes || (job.flags & SKV_SPLIT_BY_TABLE) || job.batch || job.search) return false;
    if (k == 0 || k > (uint32_t)TILE_TARGET / 2 || job.run_ptr.size() != k) return false;
    R = 0;
    for (uint32_t m = 0; m < k; ++m) {
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
    return R < 0xFFFFFFFFull;
}

static int compact_host_pipelined(skv_ctx* ctx, Job& job, skv_result** out, double t_entry, bool& used) {
    used = false;
    RunFmt f{};
    uint64_t R = 0;
    if (!pipe_eligible(job, f, R)) return SKV_OK;
    const uint32_t k = (uint32_t)job.ranked.size();
    const uint64_t S = f.S, K = f.K;
    uint64_t P = std::max<uint64_t>(2, std::min<uint64_t>(64, job.in_bytes / (256ull << 20)));
    if (const char* pp = getenv("SKV_HOST_PARTS")) P = std::max<uint64_t>(1, std::min<uint64_t>(256, strtoull(pp, nullptr, 10)));
    if (R < P * 64) return SKV_OK;
    htrace("pipe: eligible");
    auto key_at = [&](uint32_t m, uint64_t i) { return (const uint8_t*)(uintptr_t)job.run_ptr[m] + 1 + i * S + 5; };
    auto nrec = [&](uint32_t m) { return (job.run_len[m] - 1) / S; };
    // ---- cut keys: quantiles of an even sample of every run
    std::vector<std::array<uint8_t, 16>> smp;
    const uint64_t Q = std::max<uint64_t>(8, 4096 / k);
    for (uint32_t m = 0; m < k; ++m) {
        const uint64_t nm = nrec(m);
        for (uint64_t t = 0; t < Q && t < nm; ++t) {
            std::array<uint8_t, 16> a{};
            memcpy(a.data(), key_at(m, (2 * t + 1) * nm / (2 * Q)), K);
            smp.push_back(a);
        }
    }
    std::sort(smp.begin(), smp.end());
    std::vector<std::array<uint8_t, 16>> cut;  // P - 1 cut keys B_1..B_{P-1}
    for (uint64_t p = 1; p < P; ++p) cut.push_back(smp[p * smp.size() / P]);
    // ---- lb[p * k + m]: first record of run m with key >= B_p (binary search in host memory)
    std::vector<uint64_t> lb((P + 1) * k);
    bool cuts_ok = true;
    {
        const unsigned nb = par_nblocks(k, 8);
        std::vector<uint8_t> ok(nb, 1);
        par_run(k, nb, [&](unsigned b, uint64_t lo_m, uint64_t hi_m) {
            for (uint64_t m = lo_m; m < hi_m; ++m) {
                const uint64_t nm = nrec((uint32_t)m);
                lb[m] = 0;
                lb[P * k + m] = nm;
                for (uint64_t p = 1; p < P; ++p) {
                    uint64_t a = 0, z = nm;
                    while (a < z) {
                        const uint64_t mid = (a + z) >> 1;
                        if (memcmp(key_at((uint32_t)m, mid), cut[p - 1].data(), K) < 0) a = mid + 1;
                        else z = mid;
                    }
                    lb[p * k + m] = a;
                    // a stream that decreases across a cut is left to the serial path (the device
                    // checks the order inside each part only)
                    if (a < lb[(p - 1) * k + m]) ok[b] = 0;
                    if (a > 0 && a < nm && memcmp(key_at((uint32_t)m, a - 1), key_at((uint32_t)m, a), K) > 0) ok[b] = 0;
                }
            }
        });
        for (uint8_t o : ok) cuts_ok = cuts_ok && o;
    }
    if (!cuts_ok) return SKV_OK;
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
        HIPCHK(hipHostMalloc((void**)&ctx->part_k, std::max<uint64_t>(P, 64) * 8, hipHostMallocCoherent));
        ctx->part_k_cap = std::max<uint64_t>(P, 64);
    }
    volatile uint64_t* hK = ctx->part_k;
    for (uint64_t p = 0; p < P; ++p) hK[p] = ~0ull;
    // ---- device buffers (all sized before the first launch: no buffer moves under queued work)
    std::vector<uint64_t> img(k + 1, 0);
    for (uint32_t m = 0; m < k; ++m) img[m + 1] = img[m] + ((job.run_len[m] + 15) & ~15ull);
    uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", img[k] + 16);
    const uint64_t out_cap = job.in_bytes + R + 16;
    uint8_t* d_out = dbuf<uint8_t>(ctx, "out", out_cap);
    uint64_t* d_Kp = dbuf<uint64_t>(ctx, "hp_K", P);
    uint32_t* d_pflags = dbuf<uint32_t>(ctx, "hp_flags", 4);
    uint64_t* d_prb = dbuf<uint64_t>(ctx, "hp_rb", 4);
    const uint64_t n = fx_run_records(job.max_run_size, S, R), W = n * S + 1;
    const uint64_t max_runs = (R + n - 1) / n;
    DevRunDesc* d_desc = dbuf<DevRunDesc>(ctx, "descs", max_runs + 1);
    // per part: its runs (rank order, empty slices left out), record bases
    std::vector<RunInfo> hruns(P * k);
    std::vector<uint32_t> kp(P, 0);
    std::vector<std::vector<uint64_t>> recbp(P);
    for (uint64_t p = 0; p < P; ++p) {
        recbp[p].assign(1, 0);
        for (uint32_t s = 0; s < k; ++s) {
            const uint32_t m = (uint32_t)job.ranked[s].first;  // one run per stream
            const uint64_t a = lb[p * k + m], z = lb[(p + 1) * k + m];
            if (z == a) continue;
            RunInfo& ri = hruns[p * k + kp[p]];
            ri.ptr = (uint64_t)(uintptr_t)(d_in + img[m] + a * S);  // the byte before record a
            ri.len = 1 + (z - a) * S;
            ri.chunk_base = 0;
            ri.n_chunks = 0;
            ri.stream = kp[p]++;
            recbp[p].push_back(recbp[p].back() + (z - a));
        }
    }
    RunInfo* d_runs = dbuf<RunInfo>(ctx, "hp_runs", P * k);
    h2d_up(ctx, d_runs, hruns.data(), P * k * sizeof(RunInfo));
    HIPCHK(hipMemsetAsync(d_Kp, 0, P * 8, st));
    HIPCHK(hipMemsetAsync(d_pflags, 0, 16, st));
    size_t cap = 0;
    uint8_t* h_out = (uint8_t*)ctx->out_pool->take(out_cap, cap);
    if (!h_out) throw DevError("pinned host allocation of the output failed");
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
                    if (issued <= p) return;
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
    for (uint64_t p = 0; p < P; ++p) {
        for (uint32_t m = 0; m < k; ++m) {
            const uint64_t lo = p == 0 ? 0 : 1 + lb[p * k + m] * S;
            const uint64_t hi = p + 1 == P ? job.run_len[m] : 1 + lb[(p + 1) * k + m] * S;
            if (hi > lo)
                HIPCHK(hipMemcpyAsync(d_in + img[m] + lo, (const uint8_t*)(uintptr_t)job.run_ptr[m] + lo, hi - lo,
                                      hipMemcpyHostToDevice, ctx->in_stream));
        }
        HIPCHK(hipEventRecord(ctx->part_ev[2 * p], ctx->in_stream));
        HIPCHK(hipStreamWaitEvent(st, ctx->part_ev[2 * p], 0));
        if (kp[p]) {
            std::vector<uint32_t> sfr(kp[p] + 1);
            for (uint32_t s = 0; s <= kp[p]; ++s) sfr[s] = s;
            FxPartIO io;
            io.gbase = p ? d_Kp + p - 1 : nullptr;
            io.Kout = d_Kp + p;
            io.flags = d_pflags;
            io.out = d_out;
            uint64_t* rb_unused = nullptr;
            Alast = fx_launch(ctx, kp[p], kp[p], d_runs + p * k, sfr, f, recbp[p], n, out_cap, &io, rb_unused);
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
        ctx->out_pool->give(h_out, cap);
        throw DevError("pipelined egress: " + d2h_err);
    }
    if (hf[2] || egress_end != h3[2] + n_out) {  // poisoned (or a part count the verdict rejects)
        ctx->out_pool->give(h_out, cap);
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
    t.hot_read_bytes = Kt * S + (R - Kt) * (9 + K);
    t.hot_write_bytes = res->n_bytes;
    t.host_syncs = ctx->syncs;
    t.host_total_ms = now_ms() - t_entry;
    t.host_parts = (uint32_t)P;
    *out = res;
    return SKV_OK;
}

// host inputs: stage them into HBM, compact, return the output bytes in pinned host memory
static int compact_host_job(skv_ctx* ctx, Job& job, skv_result** out, double t_entry) {
    int rc;
    try {
        // stage inputs into HBM (16-byte aligned per run)
        uint64_t total = 0;
        for (uint64_t l : job.run_len) total += (l + 15) & ~15ull;
        uint8_t* d_in = dbuf<uint8_t>(ctx, "host_in", total + 16);
        uint64_t off = 0;
        for (size_t m = 0; m < job.run_ptr.size(); ++m) {
            if (job.run_len[m]) h2d(ctx, d_in + off, (const void*)job.run_ptr[m], job.run_len[m]);
            job.run_ptr[m] = (uint64_t)(uintptr_t)(d_in + off);
            off += (job.run_len[m] + 15) & ~15ull;
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

// the one-run job of a writer batch (writer_service.rs:148-162)
static int batch_job(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size, Job& job) {
    if (len && !ops_run) return set_err(ctx, SKV_E_INVALID_ARG, "ops_run is NULL");
    const uint8_t* runs[1] = {ops_run};
    const uint64_t lens[1] = {len};
    skv_stream st{runs, lens, 1u, 0};
    const int rc = build_job(ctx, &st, 1, max_run_size, 0, job);
    job.batch = true;
    return rc;
}

extern "C" {

int skv_compact(skv_ctx* ctx, const skv_stream* streams, uint32_t n_streams, uint64_t max_run_size, uint32_t flags,
                skv_result** out) {
    const double t_entry = now_ms();
    htrace("entry");
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
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
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
    Job job;
    int rc = batch_job(ctx, ops_run, len, max_run_size, job);
    if (rc) return rc;
    return compact_host_job(ctx, job, out, t_entry);
}

}  // extern "C"

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
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
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
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
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
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
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
    if (ix->mem) {
        (void)hipSetDevice(ix->device);
        (void)hipFree(ix->mem);
    }
    delete ix;
}

int skv_encode_batch_dev(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size,
                         skv_result** out) {
    const double t_entry = now_ms();
    if (!ctx || !out) return set_err(ctx, SKV_E_INVALID_ARG, "ctx/out is NULL");
    *out = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, SKV_E_DEVICE, "hipSetDevice failed");
    Job job;
    int rc = batch_job(ctx, ops_run, len, max_run_size, job);
    if (rc) return rc;
    return run_guarded(ctx, job, out, t_entry);
}

void skv_result_free(skv_result* r) {
    if (!r) return;
    ResultBox* box = (ResultBox*)r;
    if (box->pool) box->pool->give(r->bytes, box->pool_cap);
    free(r->runs);
    delete box;
}

}  // extern "C"
