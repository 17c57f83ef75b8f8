// skv_host.hpp — internal header of the host side of libskv.so (not part of the C ABI).
//
// The host code is split by path; every file below includes this header:
//   skv_ctx.hip       ctx lifetime, error text, staging helpers, job tables (build_job), run_guarded
//   skv_compact.hip   compact_device: the general / fixed-stride / record-sort / WAL device path
//   skv_fused_host.hip  the fused stride path's launches (fx_launch, compact_fused)
//   skv_hostpipe.hip  skv_compact with host inputs: the serial copy path and the key-range pipelines
//   skv_index_host.hip  runs::search_run batches and the cached run index
//   skv_scan_host.hip ScanFromRun (cache_service.rs:97-151) over read_run_iter decodes
#pragma once
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

// Pinned host memory on the NUMA node of `device`'s GPU (its node from the PCI bus via sysfs; the
// thread's memory policy prefers that node while the pages are allocated). device < 0 or an unknown
// node: a plain hipHostMalloc.
hipError_t host_alloc_near(int device, void** p, size_t bytes, unsigned flags);
int device_numa_node(int device);

// ------------------------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

enum Phase { PH_START = 0, PH_PARSE, PH_CHECK, PH_MERGE, PH_CHAIN, PH_GATHER, PH_N };

// Pinned host buffers for skv_compact outputs. Shared by the ctx and its live results, so a
// result may outlive its ctx; a freed result's buffer is kept for the next call.
struct PinnedPool {
    int device = -1;  // buffers on this GPU's NUMA node
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
        if (host_alloc_near(device, &p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
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
    std::vector<size_t> s_span_end;  // compact_host_job: the host-contiguous spans of its runs
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
    void* sl_host = nullptr;  // pinned slice tables of a pipelined call's kernel ingest
    size_t sl_cap = 0;
    // while a pipelined host call has copies queued on in_stream / out_stream, a buffer that grows
    // keeps its old allocation here until the call has drained (hipFree waits for the whole device,
    // which would serialise the pipeline behind every queued copy)
    bool defer_free = false;
    std::vector<void*> graveyard, host_graveyard;
};

struct ResultBox {  // skv_result + how to free it
    skv_result pub;
    std::shared_ptr<PinnedPool> pool;  // set: bytes is a pinned host buffer of pool_cap bytes
    size_t pool_cap = 0;
};

int set_err(skv_ctx* ctx, int code, const char* fmt, ...);

// Every C-ABI entry point runs on its ctx's device and leaves the caller's current device as it
// found it (a host thread that drives several GPUs must not find its device switched by a call).
// It also names the device whose host worker pool the call's table passes use (skv_tl_device).
extern thread_local int skv_tl_device;
struct DeviceScope {
    int prev = -1, prev_tl = -1;
    bool ok = false;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
        prev_tl = skv_tl_device;
        skv_tl_device = dev;
    }
    ~DeviceScope() {
        skv_tl_device = prev_tl;
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
#define SKV_DEVICE_SCOPE(ctx)                                                                       \
    DeviceScope dev_scope_((ctx)->device);                                                          \
    if (!dev_scope_.ok) return set_err((ctx), SKV_E_DEVICE, "hipSetDevice failed")

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
inline T* dbuf(skv_ctx* ctx, const char* name, size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    bytes = (bytes + 255) & ~(size_t)255;
    DevBuf& b = ctx->bufs[name];
    if (b.cap < bytes) {
        if (b.p && ctx->defer_free) {
            ctx->graveyard.push_back(b.p);  // queued work may still use it: freed after the call
        } else if (b.p) {  // queued work of this call (pipelined parts) may still use the old buffer
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

void* pinned(skv_ctx* ctx, size_t bytes);
void stage_copy(void* dst, const void* src, size_t bytes);
unsigned par_nblocks(uint64_t n, uint64_t min_par = 1u << 16);
// run(arg, b) for every b in [0, nb): the caller and the process's host worker pool (SKV_HOST_THREADS
// - 1 threads, started once) claim blocks from one counter. A 10^6-stream call makes ~10 such
// passes; a std::thread spawned and joined per block per pass cost ~2 ms of its host time.
void par_exec(unsigned nb, void (*run)(void*, unsigned), void* arg);
template <typename F>
inline void par_run(uint64_t n, unsigned nb, F&& fn) {
    if (nb <= 1) {
        fn(0u, (uint64_t)0, n);
        return;
    }
    struct Ctx {
        F* fn;
        uint64_t n;
        unsigned nb;
    } c{&fn, n, nb};
    par_exec(nb, [](void* a, unsigned b) {
        Ctx& x = *(Ctx*)a;
        (*x.fn)(b, x.n * b / x.nb, x.n * (b + 1) / x.nb);
    }, &c);
}
// two-pass block scan: count(lo, hi) -> items of the block; fill(b, lo, hi, base) with base = the
// items of all earlier blocks. Returns the total.
template <typename C, typename F>
inline uint64_t par_scan(uint64_t n, C&& count, F&& fill, uint64_t min_par = 1u << 16) {
    const unsigned nb = par_nblocks(n, min_par);
    std::vector<uint64_t> base(nb + 1, 0);
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) { base[b + 1] = count(lo, hi); });
    for (unsigned b = 0; b < nb; ++b) base[b + 1] += base[b];
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) { fill(b, lo, hi, base[b]); });
    return base[nb];
}

void h2d_up(skv_ctx* ctx, void* dst, const void* src, size_t bytes);
void d2h(skv_ctx* ctx, void* dst, const void* src, size_t bytes);
void h2d(skv_ctx* ctx, void* dst, const void* src, size_t bytes);
double now_ms();
void htrace(const char* what);
void sync(skv_ctx* ctx);
void mark(skv_ctx* ctx, Phase p);
int derr_to_api(uint32_t e, std::string& msg);
// ------------------------------------------------------------------------------------------
// A part of skv_compact_split's split of variable-length records (skv_hostpipe.hip): build_runs'
// greedy split continues across parts, so each part's split starts from the open run the previous
// part left (its bytes) and posts its own. wait_in blocks until that is known (false: the call
// has stopped); post_out only stages the value -- a part may rerun after its split (a deferred
// verification that fails, a fingerprint collision) and post again -- and the split hands it on
// once the part's result is final.
struct CarryHook {
    virtual ~CarryHook() = default;
    virtual bool wait_in(uint64_t part, uint64_t& c) = 0;
    virtual void post_out(uint64_t part, uint64_t c, bool cont) = 0;  // cont: run 0 continues the carried run
};

struct Job {
    std::vector<InStream> ranked;  // streams sorted by seq_no descending
    std::vector<uint64_t> run_ptr, run_len;  // member runs, caller order (flat: 10^6-stream jobs)
    // build_job's view of the caller's table: every stream holds exactly one run, and its order by
    // seq_no (1: strictly descending = rank order, -1: strictly ascending = reversed, 0: sorted here)
    bool one_run_each = false;
    int caller_order = 0;
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
    // skv_scan_runs (ScanFromRun, cache_service.rs:97-151): one run per stream at SeqNo
    // i64::MAX - index, read_run_iter's error texts, key > start filter, cut at the max-th Put
    bool scan = false;
    std::string scan_start;
    uint64_t scan_max = 0;
    // a key-range part of a pipelined host call (skv_hostpipe.hip): member runs are slices whose
    // leading byte is not a version byte, and the output goes to dev_out (the call's shared buffer)
    bool part = false;
    uint8_t* dev_out = nullptr;
    CarryHook* carry = nullptr;  // a part of skv_compact_split's variable-record split
    uint64_t carry_part = 0;
};

std::string fetch_key(skv_ctx* ctx, const uint64_t* d_rec_addr, const uint32_t* d_rec_klen, uint64_t rec);
// the key of the record at device address addr (its header read first)
std::string fetch_key_at(skv_ctx* ctx, uint64_t addr);
std::string wal_key_error(const std::string& key);

constexpr int RC_RETRY_EXACT = -100;  // internal: the merge's fingerprint shortcut misordered a tile

template <typename T>
inline T read_dev(const T* p) {
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
void throw_first(std::vector<JobEvent>& ev);
int compact_device(skv_ctx* ctx, const Job& job, skv_result** out, bool allow_deferred);
int rerun_exact(skv_ctx* ctx, const Job& job, skv_result** out);
int wal_stage(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint32_t* m_rec,
              const uint64_t* m_src, const uint64_t* m_P, const uint64_t* m_Dp, const uint64_t* rec_addr,
              const uint32_t* rec_klen, const uint32_t* fp_bad, const HeapRes* heap, skv_result** out,
              const SElem* sorted = nullptr);
uint64_t fx_run_records(uint64_t max_run_size, uint64_t S, uint64_t R);

// Where a fused launch's survivors go: a key-range part of a pipelined host call chains its
// survivor numbering through device words and shares one output buffer and one verdict.
struct FxPartIO {
    const uint64_t* gbase = nullptr;  // survivors of the earlier parts (device)
    uint64_t* Kout = nullptr;         // survivors through this part (device)
    uint32_t* flags = nullptr;        // shared verdict flags (device, zeroed by the caller)
    uint8_t* out = nullptr;           // shared output bytes (device)
};
FxArgs fx_launch(skv_ctx* ctx, uint32_t k, uint32_t n_runs, const RunInfo* d_runs,
                        const std::vector<uint32_t>& stream_first_run, const RunFmt& f,
                        const std::vector<uint64_t>& recb, uint64_t n, uint64_t out_bytes, const FxPartIO* io,
                        uint64_t*& d_rb_out);
// Key-range parts of a fused call with host inputs (skv_hostpipe.hip; the pipelined host call and
// the multi-GPU split, skv_split.hip)
bool fx_host_shape(const Job& job, RunFmt& f, uint64_t& R);
bool fx_host_cuts(const Job& job, const RunFmt& f, uint64_t P, std::vector<uint64_t>& lb);
struct FxPartTables {  // per part i of [p0, p1): runs rows i * nr.., streams, first runs, record bases
    std::vector<RunInfo> runs;
    std::vector<uint32_t> kp, np;
    std::vector<std::vector<uint32_t>> sfr;
    std::vector<std::vector<uint64_t>> recb;
};
void fx_part_tables(const Job& job, const RunFmt& f, uint64_t p0, uint64_t p1, const std::vector<uint64_t>& lb,
                    const uint8_t* d_in, const std::vector<uint64_t>& img, const std::vector<uint64_t>* base,
                    FxPartTables& t);
bool compact_fused(skv_ctx* ctx, const Job& job, const std::vector<RunInfo>& runs, const RunInfo* d_runs,
                          const std::vector<uint32_t>& stream_first_run, const RunFmt& f,
                          const std::vector<uint64_t>& recb, skv_result** out);
SElem* sort_elems(skv_ctx* ctx, SElem* E, SElem* T, uint64_t n, int depth, uint64_t* newkey = nullptr);
void sort_records(skv_ctx* ctx, uint64_t R, uint64_t*& hi, uint64_t*& lo, uint64_t*& addr, uint32_t*& klen,
                         uint32_t*& meta, const uint32_t*& cmp_klen, bool last_wins, const SElem** sorted = nullptr,
                         uint32_t const_meta = 0, const SortMerged* merged = nullptr, uint64_t** d_K = nullptr,
                         bool e_ready = false);

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
void search_launch(skv_ctx* ctx, const uint8_t* run, uint64_t len, bool clean, uint64_t R,
                          const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
                          const uint32_t* rec_klen, const uint32_t* rec_meta, const uint8_t* keys,
                          const uint64_t* key_offs, uint32_t n, skv_lookup* out);
int search_stage(skv_ctx* ctx, const Job& job, const RunInfo& run, uint64_t R, uint32_t run_err,
                        uint64_t first_dec, const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
                        const uint32_t* rec_klen, const uint32_t* rec_meta);
void ensure_aux(skv_ctx* ctx);
int build_job(skv_ctx* ctx, const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags, Job& job);
void drain(skv_ctx* ctx);

// Test hooks (include/skv.h skv_test_option): the parity suite forces rare paths through named
// values set on the library (the fused path off, the record sort on, fingerprint collisions, small
// chunks, ...). Never read from the environment: production behaviour depends only on the call.
// test_opt(name): the value set for `name`, or null (declared in skv_launch.hpp).

// A pipelined or split call on one ctx (skv_hostpipe.hip, skv_split.hip): table uploads and readbacks
// by copy kernels, not DMA copies that would queue behind the bulk copies; buffers that grow keep
// their old allocation (the graveyards) until the ctx's three streams have drained, as a hipFree in
// between would synchronise the whole device under every other ctx's queued work.
struct PipeIO {
    skv_ctx* c;
    explicit PipeIO(skv_ctx* x) : c(x) {
        c->kernel_uploads = true;
        c->defer_free = true;
    }
    ~PipeIO() {
        c->kernel_uploads = false;
        c->defer_free = false;
        if (!c->graveyard.empty() || !c->host_graveyard.empty()) {
            if (c->in_stream) (void)hipStreamSynchronize(c->in_stream);
            if (c->out_stream) (void)hipStreamSynchronize(c->out_stream);
            (void)hipStreamSynchronize(c->stream);
            for (void* q : c->graveyard) (void)hipFree(q);
            for (void* q : c->host_graveyard) (void)hipHostFree(q);
            c->graveyard.clear();
            c->host_graveyard.clear();
        }
    }
};

// Worker threads of a multi-ctx call, joined on every path: a std::thread constructor that throws
// after some workers started must not destroy joinable threads (std::terminate); the caller's
// stop() is asked to halt the started workers before they are joined.
struct WorkerSet {
    std::vector<std::thread> th;
    template <class F, class Stop>
    bool spawn(unsigned n, F&& body, Stop&& stop) {
        try {
            for (unsigned g = 0; g < n; ++g) th.emplace_back(body, g);
        } catch (...) {
            stop();
            join();
            return false;
        }
        return true;
    }
    void join() {
        for (std::thread& t : th)
            if (t.joinable()) t.join();
        th.clear();
    }
    ~WorkerSet() { join(); }
};
int run_guarded(skv_ctx* ctx, const Job& job, skv_result** out, double t_entry);
int compact_host_job(skv_ctx* ctx, Job& job, skv_result** out, double t_entry);
// skv_compact_split for inputs outside the fused shape (variable-length records, Deletes): key-range
// parts over the ctxs with build_runs' split carried from part to part (skv_hostpipe.hip). used =
// false: not taken, or a part hit a data error -- the caller runs skv_compact on ctxs[0]
int compact_split_general(skv_ctx* const* ctxs, uint32_t G, Job& job, skv_result** out, double t_entry, bool& used);
// skv_scan_host.hip: the scan's device stage after the merge, and read_run_iter's error text
struct ScanEvent {  // a run's decode error and the record it surfaces after
    uint32_t s;             // stream (rank order)
    uint64_t after_rec;     // original record index of the run's last record above the start key
    int code;
    std::string msg;
};
int scan_stage(skv_ctx* ctx, const Job& job, uint64_t R, const uint64_t* d_K, const uint32_t* m_rec,
               const uint64_t* m_src, const uint64_t* rec_addr, const uint64_t* rec_hi, const uint64_t* rec_lo,
               const uint32_t* rec_klen, const uint32_t* rec_meta, const uint8_t* d_start, const uint32_t* fp_bad,
               const HeapRes* heap, const std::vector<ScanEvent>& events, skv_result** out);
int scan_err_to_api(uint32_t derr, uint64_t err_off, uint64_t run_len, std::string& msg);
int batch_job(skv_ctx* ctx, const uint8_t* ops_run, uint64_t len, uint64_t max_run_size, Job& job);
