// skv_ctx.hip — ctx lifetime, the reference's error text, host staging helpers, the job tables of a
// call (build_job) and the guarded device call (run_guarded). C ABI: include/skv.h.
#include "skv_host.hpp"

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <deque>
#include <exception>
#include <fstream>
#include <mutex>
#include <set>
#include <sstream>

using namespace skv;

thread_local int skv_tl_device = -1;

namespace skv {
void lds_limit(const void* kernel) {
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    if (done.count({dev, kernel})) return;
    // the ceiling is the device's per-workgroup LDS opt-in limit (the CU's 160 KiB on gfx950) less
    // the kernel's static LDS (a larger value is refused); recorded only once the device took it,
    // so a refused or failed call is tried again by the next launch
    int cap = 0;
    if (hipDeviceGetAttribute(&cap, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || cap <= 0) {
        (void)hipGetLastError();
        if (hipDeviceGetAttribute(&cap, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
    }
    hipFuncAttributes fa{};
    size_t stat = 0;
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess) stat = fa.sharedSizeBytes;
    else (void)hipGetLastError();
    if ((size_t)cap <= stat) return;
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)((size_t)cap - stat)) == hipSuccess)
        done.insert({dev, kernel});
    else
        (void)hipGetLastError();
}
}  // namespace skv


int set_err(skv_ctx* ctx, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

void* pinned(skv_ctx* ctx, size_t bytes) {
    if (ctx->pinned_cap < bytes) {
        if (ctx->pinned && ctx->defer_free) ctx->host_graveyard.push_back(ctx->pinned);  // see dbuf
        else if (ctx->pinned) HIPCHK(hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        size_t cap = std::max<size_t>(bytes, 1 << 16);
        HIPCHK(host_alloc_near(ctx->device, &ctx->pinned, cap, hipHostMallocDefault));
        ctx->pinned_cap = cap;
    }
    return ctx->pinned;
}

namespace {
struct PoolBatch {
    void (*run)(void*, unsigned);
    void* arg;
    unsigned nb;
    std::atomic<unsigned> next{0};    // next block to claim
    std::atomic<unsigned> done{0};    // blocks finished
    std::atomic<unsigned> active{0};  // workers holding this batch (the caller waits them out)
    std::exception_ptr err;           // first exception of a worker's block
    std::mutex err_m;
};
struct HostPool {
    std::mutex m;
    std::condition_variable cv;
    std::deque<PoolBatch*> q;  // one token per helper wanted; a token names its batch
    // n detached workers, each bound to `cpus` (the GPU's NUMA node) when that leaves it any CPU the
    // process may run on
    HostPool(unsigned n, const std::vector<int>& cpus) {
        for (unsigned i = 0; i < n; ++i)
            std::thread([this, cpus] {
                bind_to(cpus);
                work();
            }).detach();
    }
    static void bind_to(const std::vector<int>& cpus) {
        if (cpus.empty()) return;
        cpu_set_t allowed, want;
        if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
        CPU_ZERO(&want);
        int n = 0;
        for (int c : cpus)
            if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) {
                CPU_SET(c, &want);
                ++n;
            }
        if (n) (void)pthread_setaffinity_np(pthread_self(), sizeof want, &want);
    }
    static void drain(PoolBatch* b) {
        for (;;) {
            const unsigned i = b->next.fetch_add(1);
            if (i >= b->nb) return;
            try {
                b->run(b->arg, i);
            } catch (...) {
                std::lock_guard<std::mutex> l(b->err_m);
                if (!b->err) b->err = std::current_exception();
            }
            b->done.fetch_add(1);
        }
    }
    void work() {
        for (;;) {
            PoolBatch* b;
            {
                std::unique_lock<std::mutex> l(m);
                cv.wait(l, [&] { return !q.empty(); });
                b = q.front();
                q.pop_front();
                b->active.fetch_add(1);  // under the lock: the caller's token sweep sees it
            }
            drain(b);
            b->active.fetch_sub(1);  // the last touch of b
        }
    }
};
unsigned host_threads_cap() {  // SKV_HOST_THREADS: host threads for 10^6-entry tables (default 8)
    static const unsigned cap = [] {
        const char* e = getenv("SKV_HOST_THREADS");
        const long v = e ? atol(e) : 8;
        return (unsigned)std::max(1l, std::min(64l, v));
    }();
    return cap;
}
std::string read_text(const std::string& path) {
    std::ifstream f(path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}
std::vector<int> parse_cpulist(const std::string& s) {  // "0-63,128-191"
    std::vector<int> out;
    std::stringstream ss(s);
    std::string item;
    while (std::getline(ss, item, ',')) {
        const size_t d = item.find('-');
        try {
            if (d == std::string::npos) {
                if (!item.empty() && item[0] != '\n') out.push_back(std::stoi(item));
            } else {
                const int a = std::stoi(item.substr(0, d)), b = std::stoi(item.substr(d + 1));
                for (int c = a; c <= b && c - a < 65536; ++c) out.push_back(c);
            }
        } catch (...) {
        }
    }
    return out;
}
// The host side of one GPU: its NUMA node (from the PCI bus via sysfs), that node's CPUs, and a
// host worker pool of its own. One process driving the 8 GPUs of a node (skv.multi.MultiCompactor,
// skv_pool) then runs each device's 10^6-entry table passes on threads near that device instead of
// queueing every device's passes on one shared pool. Pool size: SKV_HOST_THREADS (default 8), at
// most the machine's CPUs / devices.
struct DevHost {
    int numa = -1;
    std::vector<int> cpus;
    unsigned threads = 1;  // the caller + threads - 1 workers
    HostPool* pool = nullptr;
};
// The plan of one device's host side from sysfs (root "/sys" on a live system): its NUMA node (the PCI
// device's numa_node), that node's CPUs, and the pool size for a machine of hw CPUs and ndev GPUs.
struct HostPlan {
    int numa = -1;
    std::vector<int> cpus;
    unsigned threads = 1;
};
HostPlan host_plan(const std::string& root, const char* bus_id, int ndev, unsigned hw) {
    HostPlan p;
    if (bus_id && *bus_id) {
        std::string bus(bus_id);
        for (char& c : bus) c = (char)tolower(c);
        const std::string nn = read_text(root + "/bus/pci/devices/" + bus + "/numa_node");
        try {
            p.numa = nn.empty() ? -1 : std::stoi(nn);
        } catch (...) {
            p.numa = -1;
        }
        if (p.numa >= 0) p.cpus = parse_cpulist(read_text(root + "/devices/system/node/node" + std::to_string(p.numa) + "/cpulist"));
    }
    if (ndev < 1) ndev = 1;
    hw = std::max(1u, hw);
    p.threads = std::max(1u, std::min(host_threads_cap(), std::max(1u, hw / (unsigned)ndev)));
    return p;
}
DevHost& dev_host(int device) {  // created on first use, never torn down (like the workers)
    static std::mutex mu;
    static std::map<int, DevHost*> hosts;
    std::lock_guard<std::mutex> g(mu);
    if (device < 0) device = 0;
    auto it = hosts.find(device);
    if (it != hosts.end()) return *it->second;
    DevHost* d = new DevHost();
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) {
        (void)hipGetLastError();
        bus[0] = 0;
    }
    int ndev = 1;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) ndev = 1;
    const HostPlan p = host_plan("/sys", bus, ndev, std::thread::hardware_concurrency());
    d->numa = p.numa;
    d->cpus = p.cpus;
    d->threads = p.threads;
    d->pool = new HostPool(d->threads > 1 ? d->threads - 1 : 1, d->cpus);
    hosts[device] = d;
    return *d;
}
}  // namespace

int device_numa_node(int device) { return dev_host(device).numa; }

// the test hooks' table (skv_test_option): fixed names, values copied in under a lock; test_opt hands
// a caller a thread-local copy, so a hook set from another thread never tears a value being parsed
namespace {
struct TestOpt {
    const char* name;
    bool set;
    char value[48];
};
std::mutex& test_opt_mu() {
    static std::mutex mu;
    return mu;
}
std::vector<TestOpt>& test_opts() {
    static std::vector<TestOpt> t = [] {
        std::vector<TestOpt> v;
        for (const char* n : {"SKV_FUSED", "SKV_SORT", "SKV_FP_TEST", "SKV_FP_GATHER", "SKV_CHUNK_BYTES",
                              "SKV_WAL_FUSED", "SKV_INGEST", "SKV_TEST_FAIL_PART", "SKV_PAR_COPY_MIN", "SKV_HI_STEP",
                              "SKV_SPLIT", "SKV_SPLIT_DEBUG", "SKV_SPLIT_SEG", "SKV_SPLIT_NC", "SKV_SORT_TWO_PASS",
                              "SKV_SB_NT", "SKV_SB_GMAX", "SKV_FX_TAIL_SLOTS"})
            v.push_back(TestOpt{n, false, {}});
        return v;
    }();
    return t;
}
}  // namespace
const char* test_opt(const char* name) {
    thread_local char buf[8][48];
    thread_local unsigned next = 0;
    std::lock_guard<std::mutex> g(test_opt_mu());
    for (const TestOpt& o : test_opts()) {
        if (strcmp(o.name, name)) continue;
        if (!o.set) return nullptr;
        char* b = buf[next++ & 7];
        memcpy(b, o.value, sizeof o.value);
        return b;
    }
    return nullptr;
}

hipError_t host_alloc_near(int device, void** p, size_t bytes, unsigned flags) {
    const int node = device >= 0 ? dev_host(device).numa : -1;
    if (node < 0 || node >= 1024) return hipHostMalloc(p, bytes, flags);
    // prefer the GPU's node for this thread while the pages are allocated (and pinned), then put the
    // thread's own policy back; hipHostMallocNumaUser makes the allocation follow it
    constexpr int MPOL_PREFERRED_ = 1;
    unsigned long old_mask[16] = {}, mask[16] = {};
    int old_mode = 0;
    const bool have_old = syscall(SYS_get_mempolicy, &old_mode, old_mask, 1024ul, nullptr, 0ul) == 0;
    mask[node / 64] |= 1ul << (node % 64);
    const bool set = syscall(SYS_set_mempolicy, MPOL_PREFERRED_, mask, 1024ul) == 0;
    const hipError_t e = hipHostMalloc(p, bytes, flags | (set ? hipHostMallocNumaUser : 0u));
    if (set) {
        if (have_old) (void)syscall(SYS_set_mempolicy, old_mode, old_mode ? old_mask : nullptr, old_mode ? 1024ul : 0ul);
        else (void)syscall(SYS_set_mempolicy, 0, nullptr, 0ul);
    }
    return e;
}

void par_exec(unsigned nb, void (*run)(void*, unsigned), void* arg) {
    PoolBatch b;
    b.run = run;
    b.arg = arg;
    b.nb = nb;
    HostPool& P = *dev_host(skv_tl_device).pool;
    {
        std::lock_guard<std::mutex> l(P.m);
        for (unsigned k = 1; k < nb; ++k) P.q.push_back(&b);
    }
    P.cv.notify_all();
    HostPool::drain(&b);  // the caller claims blocks too: the call finishes even with every worker busy
    {
        std::lock_guard<std::mutex> l(P.m);  // tokens no worker took
        P.q.erase(std::remove(P.q.begin(), P.q.end(), &b), P.q.end());
    }
    while (b.done.load() != nb || b.active.load() != 0) std::this_thread::yield();
    if (b.err) std::rethrow_exception(b.err);
}

// host copy into pinned staging; large tables (10^6-run calls: tens of MB) on the host pool
void stage_copy(void* dst, const void* src, size_t bytes) {
    const char* pe = test_opt("SKV_PAR_COPY_MIN");  // tests: split small tables too
    const size_t kPar = pe ? (size_t)strtoull(pe, nullptr, 10) : (8u << 20);
    const unsigned nt = dev_host(skv_tl_device).threads;
    if (bytes < kPar || nt < 2) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t part = ((bytes + nt - 1) / nt + 4095) & ~(size_t)4095;
    const unsigned np = (unsigned)((bytes + part - 1) / part);
    par_run(np, np, [&](unsigned, uint64_t lo, uint64_t) {
        memcpy((uint8_t*)dst + lo * part, (const uint8_t*)src + lo * part, std::min(part, bytes - lo * part));
    });
}

// Blocks for par_run ([0, n) as nb contiguous blocks fn(b, lo, hi), par_exec's pool): the per-run and
// per-stream table loops of a 10^6-stream call (config 5) are memory-bound at one core's bandwidth,
// ~10 ns per entry. Below min_par entries one block runs on the calling thread.
unsigned par_nblocks(uint64_t n, uint64_t min_par) {
    return n < min_par ? 1u : dev_host(skv_tl_device).threads;
}

// async H2D of a host table through the pinned upload arena
void h2d_up(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
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
        HIPCHK(host_alloc_near(ctx->device, &p, cap, hipHostMallocDefault));
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

// async D2H of a readback into pinned staging (dst is always a pinned() / arena buffer). In a
// pipelined host call a copy kernel writes it through the mapping: a DMA copy on the ctx stream
// could wait behind the egress thread's bulk D2H copies.
void d2h(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    if (ctx->kernel_uploads) {
        void* dptr = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dptr, dst, 0));
        launch_copy_bytes(ctx->stream, (uint8_t*)dptr, (const uint8_t*)src, bytes);
        return;
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
}
void h2d(skv_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
}
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// SKV_HOST_TRACE=1: host-side milestones of a call on stderr (ms since the call's first one)
void htrace(const char* what) {
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
void sync(skv_ctx* ctx) {
    const double t0 = now_ms();
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->sync_ms += now_ms() - t0;
    ctx->syncs++;
}
void mark(skv_ctx* ctx, Phase p) {
    if (ctx->profiling) HIPCHK(hipEventRecord(ctx->ev[p], ctx->stream));
}

// reference Display text of a device error word (runs.rs:83-95, :537-624)
int derr_to_api(uint32_t e, std::string& msg) {
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


// a record's key bytes (host copy) for error-trigger comparisons
std::string fetch_key(skv_ctx* ctx, const uint64_t* d_rec_addr, const uint32_t* d_rec_klen, uint64_t rec) {
    uint64_t addr = 0;
    uint32_t klen = 0;
    HIPCHK(hipMemcpy(&addr, d_rec_addr + rec, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&klen, d_rec_klen + rec, 4, hipMemcpyDeviceToHost));
    std::string k(klen, '\0');
    if (klen) HIPCHK(hipMemcpy(&k[0], (const void*)(addr + 5), klen, hipMemcpyDeviceToHost));
    return k;
}

std::string fetch_key_at(skv_ctx* ctx, uint64_t addr) {
    uint8_t h[5] = {};
    HIPCHK(hipMemcpy(h, (const void*)addr, 5, hipMemcpyDeviceToHost));
    const uint32_t klen = ((uint32_t)h[1] << 24) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 8) | h[4];
    std::string k(klen, '\0');
    if (klen) HIPCHK(hipMemcpy(&k[0], (const void*)(addr + 5), klen, hipMemcpyDeviceToHost));
    return k;
}

// JobError::InvalidInput text of a bad WAL key (wal_compaction.rs:71-79; Rust ParseIntError Display)
std::string wal_key_error(const std::string& key) {
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
void throw_first(std::vector<JobEvent>& ev) {
    if (ev.empty()) return;
    std::sort(ev.begin(), ev.end(), [](const JobEvent& a, const JobEvent& b) {
        return a.pos != b.pos ? a.pos < b.pos : a.sub < b.sub;
    });
    throw ApiError{ev[0].code, ev[0].msg};
}

// ------------------------------------------------------------------------------------------
int build_job_impl(skv_ctx* ctx, const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags,
                     Job& job) {
    if (n && !streams) return set_err(ctx, SKV_E_INVALID_ARG, "streams is NULL");
    if (flags & ~(uint32_t)(SKV_DROP_TOMBSTONES | SKV_SPLIT_BY_TABLE))
        return set_err(ctx, SKV_E_INVALID_ARG, "unknown flags 0x%x", flags);
    if ((flags & SKV_SPLIT_BY_TABLE) && (flags & SKV_DROP_TOMBSTONES))
        return set_err(ctx, SKV_E_INVALID_ARG, "SKV_SPLIT_BY_TABLE and SKV_DROP_TOMBSTONES are exclusive");
    job.max_run_size = max_run_size;
    job.flags = flags;
    // pass 1 (blocks of streams on host threads): NULL checks, run counts, input bytes, and
    // whether the caller's order is strictly ascending / descending by seq_no. A block of one-run
    // streams in a strict order also writes its tables right away, placed as that order would put
    // them (spec = -1 ascending / 1 descending); pass 2 then redoes only the blocks whose guess the
    // whole table's order contradicts (a 10^6-stream WAL flush skips pass 2 entirely).
    const unsigned nb = par_nblocks(n);
    struct Blk {
        uint64_t runs = 0, bytes = 0, bad = ~0ull;
        uint32_t bad_run = ~0u;
        bool asc = true, desc = true, one = true;
        int spec = 0;
    };
    std::vector<Blk> B(nb);
    job.run_ptr.resize(n);  // (the one-run size; pass 2 resizes otherwise)
    job.run_len.resize(n);
    job.ranked.resize(n);
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
            K.one = K.one && s.n_runs == 1;
            if (i > 0) {
                K.asc = K.asc && streams[i - 1].seq_no < s.seq_no;
                K.desc = K.desc && streams[i - 1].seq_no > s.seq_no;
            }
        }
        const int dir = K.asc && !K.desc ? -1 : (K.desc && !K.asc ? 1 : 0);
        if (!K.one || !dir) return;
        for (uint64_t i = lo; i < hi; ++i) {  // (the block's entries are in cache)
            const skv_stream& s = streams[i];
            job.run_ptr[i] = (uint64_t)(uintptr_t)s.runs[0];
            job.run_len[i] = s.run_lens[0];
            InStream& S = job.ranked[dir < 0 ? n - 1 - i : i];
            S.seq = s.seq_no;
            S.vec_idx = (uint32_t)i;
            S.n_runs = 1;
            S.first = i;
        }
        K.spec = dir;
    });
    bool asc = true, desc = true, one = true;
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
        one = one && B[b].one;
    }
    job.one_run_each = one;
    job.caller_order = desc ? 1 : (asc ? -1 : 0);
    // pass 2: the tables, streams already in rank order (seq_no descending) when the caller's
    // order is either strict one; resize keeps a lent table's entries (no zero fill per call)
    job.run_ptr.resize(total_runs);
    job.run_len.resize(total_runs);
    const int gdir = asc ? -1 : (desc ? 1 : 0);  // (pass 2's placement below)
    par_run(n, nb, [&](unsigned b, uint64_t lo, uint64_t hi) {
        if (one && gdir && B[b].spec == gdir) return;  // written by pass 1
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
int build_job(skv_ctx* ctx, const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags,
                     Job& job) {
    try {
        return build_job_impl(ctx, streams, n, max_run_size, flags, job);
    } catch (const std::exception& e) {
        return set_err(ctx, SKV_E_DEVICE, "host error: %s", e.what());
    }
}

// after an error: every stream of the ctx idle before its buffers are reused
void drain(skv_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->aux_stream) (void)hipStreamSynchronize(ctx->aux_stream);
    if (ctx->in_stream) (void)hipStreamSynchronize(ctx->in_stream);
    if (ctx->out_stream) (void)hipStreamSynchronize(ctx->out_stream);
}

int run_guarded(skv_ctx* ctx, const Job& job, skv_result** out, double t_entry) {
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
    DeviceScope scope(device);
    skv_ctx* ctx = new skv_ctx();
    ctx->device = device;
    ctx->out_pool->device = device;
    if (!scope.ok || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SKV_E_DEVICE;
    }
    for (int i = 0; i < PH_N; ++i) (void)hipEventCreate(&ctx->ev[i]);
    *out = ctx;
    return SKV_OK;
}

void skv_ctx_destroy(skv_ctx* ctx) {
    if (!ctx) return;
    DeviceScope scope(ctx->device);
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
    if (ctx->sl_host) (void)hipHostFree(ctx->sl_host);
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

int skv_test_option(const char* name, const char* value) {
    if (!name) {  // clear every hook
        std::lock_guard<std::mutex> g(test_opt_mu());
        for (TestOpt& o : test_opts()) o.set = false;
        return SKV_OK;
    }
    std::lock_guard<std::mutex> g(test_opt_mu());
    for (TestOpt& o : test_opts()) {
        if (strcmp(o.name, name)) continue;
        if (value && strlen(value) >= sizeof o.value) return SKV_E_INVALID_ARG;
        if (value) memcpy(o.value, value, strlen(value) + 1);
        o.set = value != nullptr;
        return SKV_OK;
    }
    return SKV_E_INVALID_ARG;
}

int skv_host_plan(const char* sysfs_root, const char* pci_bus_id, int n_devices, int hw_threads, int* numa_node,
                  int* pool_threads, int* cpus, int max_cpus) {
    try {
        const HostPlan p = host_plan(sysfs_root && *sysfs_root ? sysfs_root : "/sys", pci_bus_id, n_devices,
                                     hw_threads > 0 ? (unsigned)hw_threads : 1u);
        if (numa_node) *numa_node = p.numa;
        if (pool_threads) *pool_threads = (int)p.threads;
        for (int i = 0; cpus && i < max_cpus && i < (int)p.cpus.size(); ++i) cpus[i] = p.cpus[i];
        return p.numa < 0 ? -1 : (int)p.cpus.size();
    } catch (...) {
        return -1;
    }
}

int skv_ctx_host_info(const skv_ctx* ctx, int* numa_node, int* host_threads) {
    if (!ctx) return SKV_E_INVALID_ARG;
    DeviceScope scope(ctx->device);
    if (numa_node) *numa_node = dev_host(ctx->device).numa;
    if (host_threads) *host_threads = (int)dev_host(ctx->device).threads;
    return SKV_OK;
}

int skv_ctx_get_timings(const skv_ctx* ctx, skv_timings* out) {
    if (!ctx || !out) return SKV_E_INVALID_ARG;
    *out = ctx->timings;
    return SKV_OK;
}

void skv_result_free(skv_result* r) {
    if (!r) return;
    ResultBox* box = (ResultBox*)r;
    if (box->pool) box->pool->give(r->bytes, box->pool_cap);
    free(r->runs);
    delete box;
}

}  // extern "C"
