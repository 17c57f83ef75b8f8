// skv_span.hip — one-pass parse of variable-length runs (gfx950): runs::read_run_stream
// (runs.rs:559-626) for every input run at once, reading every run byte exactly once.
//
// The chunk-walk parse (k_spec / k_emit, skv_kernels.hip) reads each record's header lines twice
// from HBM with dependent loads: 88 GB of line traffic for config 3F's 64 GB of runs. Here one
// workgroup takes one SPAN-byte span of a run and:
//   1. stages the span (+ MARGIN bytes of the next, for records that start near its end) in LDS
//      with coalesced 16-byte loads;
//   2. wave 0 walks it in LDS: lane l owns SPAN/64 bytes, finds its first record start
//      speculatively (a marker byte from which 3 records decode), walks the records starting in
//      its bytes and keeps their offsets; the lanes' walks are then checked against each other
//      (lane l must start where the nearest earlier lane with records ended);
//   3. publishes its record count (decoupled look-back over spans in ticket order) to learn the
//      global index of its first record;
//   4. parses its records again from LDS (prefix, key length, size | Delete, fingerprint of the key
//      bytes past 16, exact UTF-8) and writes the record arrays at their final indices.
// A span's speculative first start is checked against the previous span's exit by k_span_check.
// A span in which no record starts (a run's short tail, or inside a record longer than a span) is
// checked to lie inside the record that crosses it. Anything unusual -- a decode error, an invalid
// UTF-8 key, a lane that started off the record chain, more records than the arrays hold -- sets a
// fail bit, and the host runs the chunk-walk parse instead, which reproduces
// the reference's exact error. Only a clean decode of every run is taken from here.
#include "skv_dev.hpp"
#include "skv_launch.hpp"

namespace skv {

constexpr uint32_t SPAN = SPAN_BYTES;
constexpr uint32_t SPAN_MARGIN = 512;               // bytes staged past the span
constexpr uint32_t SPAN_SUB = SPAN / 64;            // bytes per walking lane
constexpr uint32_t SPAN_LCAP = 64;                  // record starts a lane keeps (multiple of 8)
constexpr uint32_t SPAN_THREADS = 256;
constexpr uint32_t SPAN_BLOCKS = (SPAN + SPAN_MARGIN) / 16 + 2;  // staged 16-byte blocks
static_assert(SPAN_SUB * 64 == SPAN && SPAN <= 65536, "u16 offsets, 64 walking lanes");
static_assert(SPAN_LCAP % 8 == 0, "walk_fast stores record starts eight at a time");

enum : uint32_t { SPF_DECODE = 1, SPF_CHAIN = 2, SPF_OVER = 8, SPF_UTF8 = 16, SPF_CAP = 32 };

// Loads of the record parsers: blocks inside the staged bytes come from LDS, others from HBM
struct SpanLoad {
    const uint4* lds;
    uintptr_t g0, g1;
    __device__ __forceinline__ uint4 operator()(uintptr_t a) const {
        return (a >= g0 && a < g1) ? lds[(a - g0) >> 4] : gblk(a);
    }
};

__device__ __forceinline__ uint64_t span_lookback(uint64_t* st, uint64_t t, uint64_t agg) {
    constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62, VM = FA - 1;
    const int lane = threadIdx.x & 63;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(&st[0], FI | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&st[t], FA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t acc = 0;
    int64_t top = (int64_t)t - 1;
    for (;;) {
        const int64_t p = top - lane;
        const uint64_t v = p >= 0 ? __hip_atomic_load(&st[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FI;
        const uint64_t f = v >> 62;
        const uint64_t incl = __ballot(f == 2), none = __ballot(f == 0);
        const int first = incl ? __builtin_ctzll(incl) : 64;
        const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
        if (none & upto) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t x = (uint64_t)lane <= (uint64_t)first ? (v & VM) : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        acc += x;
        if (first < 64) break;
        top -= 64;
    }
    if (lane == 0) __hip_atomic_store(&st[t], FI | (acc + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return acc;
}

__device__ __forceinline__ uint32_t span_run(const RunInfo* runs, uint32_t n_runs, uint64_t s) {
    uint32_t lo = 0, hi = n_runs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (runs[mid].chunk_base <= s) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(SPAN_THREADS) k_span_parse(const RunInfo* __restrict__ runs, uint32_t n_runs,
                                                             uint64_t n_spans, SpanOut O) {
    __shared__ uint4 buf[SPAN_BLOCKS];
    __shared__ __attribute__((aligned(16))) uint16_t lst[64 * SPAN_LCAP];
    __shared__ uint32_t pre[65];
    __shared__ uint64_t s_t, s_base;
    __shared__ uint32_t s_fail;
    const uint32_t tid = threadIdx.x;
    uint64_t* const tk = O.dbg ? (uint64_t*)(O.dbg + 6) : nullptr;  // phase ticks (SKV_SPAN_DBG)
    uint64_t t0 = tk ? wall_clock64() : 0, t1 = 0, t2 = 0, t3 = 0;
    if (tid == 0) {
        s_t = atomicAdd(O.ticket, 1u);
        s_fail = 0;
    }
    __syncthreads();
    const uint64_t s = s_t;
    const uint32_t r = span_run(runs, n_runs, s);
    const RunInfo R = runs[r];
    const uint8_t* run = (const uint8_t*)R.ptr;
    const uint64_t local = s - R.chunk_base;
    const uint64_t cs = 1 + local * SPAN, ce = cs + SPAN < R.len ? cs + SPAN : R.len;
    // ---- 1. stage [cs, ce + MARGIN) (whole aligned blocks, none past the run's last byte)
    const uintptr_t g0 = ((uintptr_t)run + cs) & ~(uintptr_t)15;
    const uint64_t se = ce + SPAN_MARGIN < R.len ? ce + SPAN_MARGIN : R.len;
    const uintptr_t g1 = ((uintptr_t)run + se + 15) & ~(uintptr_t)15;
    const uint32_t nb = (uint32_t)((g1 - g0) >> 4);
    {
        uint4 v[(SPAN_BLOCKS + SPAN_THREADS - 1) / SPAN_THREADS];
#pragma unroll
        for (uint32_t u = 0; u < (SPAN_BLOCKS + SPAN_THREADS - 1) / SPAN_THREADS; ++u) {
            const uint32_t b = tid + u * SPAN_THREADS;
            if (b < nb) v[u] = gblk(g0 + 16ull * b);
        }
#pragma unroll
        for (uint32_t u = 0; u < (SPAN_BLOCKS + SPAN_THREADS - 1) / SPAN_THREADS; ++u) {
            const uint32_t b = tid + u * SPAN_THREADS;
            if (b < nb) buf[b] = v[u];
        }
    }
    __syncthreads();
    const SpanLoad ld{buf, g0, g1};
    const uint8_t* bytes = (const uint8_t*)buf;
    if (tk) t1 = wall_clock64();
    // ---- 2. wave 0 walks the span, lane l the records starting in [a, b)
    uint64_t count = 0;
    if (tid < 64) {
        const uint32_t l = tid;
        const uint64_t a = cs + (uint64_t)l * SPAN_SUB, b = a + SPAN_SUB < ce ? a + SPAN_SUB : ce;
        uint32_t fail = 0;
        uint64_t st = NO_POS, e = NO_POS;  // NO_POS: at or past ce
        uint32_t n = 0;
        if (a < ce) {
            if (local == 0 && l == 0) {
                st = 1;
            } else {
                for (uint64_t p = a; p < ce; ++p) {  // the first marker from which 3 records decode
                    const uint32_t m = bytes[(uintptr_t)run + p - g0];
                    if ((m == 1 || m == 2) && walk_fast<2>(run, R.len, p, R.len, 3, ld).err == DERR_NONE) {
                        st = p;
                        break;
                    }
                }
            }
            if (st < b) {
                const WalkRes w = walk_fast<0>(run, R.len, st, b, 0xFFFFFFFFu, ld, lst + l * SPAN_LCAP, SPAN_LCAP, cs);
                if (w.err) fail |= SPF_DECODE;
                if (w.cnt > SPAN_LCAP) fail |= SPF_OVER;
                n = w.cnt;
                e = w.end;
            } else {
                e = st;
            }
        }
        // the chain check: lane l starts where the nearest earlier lane with records ended (or, with
        // none, where lane 0 started); a lane whose bytes hold no record start found none before b
        const uint64_t has = __ballot(n > 0);
        const uint64_t s0 = __shfl(st, 0, 64);
        const uint64_t below = has & ((1ull << l) - 1);
        const int j = below ? 63 - __builtin_clzll(below) : -1;
        const uint64_t ej = __shfl(e, j < 0 ? 0 : j, 64);
        const uint64_t P = j < 0 ? s0 : ej;
        if (a < ce && l > 0) {
            const bool ok = P >= b ? (st >= b) : (st == P);
            if (!ok) fail |= SPF_CHAIN;
        }
        // no record start in this span (s0 >= ce): fine when a record crosses it (k_span_check)
        // the span's exit: the end of its last record (the lane with records furthest on)
        const int jl = has ? 63 - __builtin_clzll(has) : -1;
        const uint64_t ex = __shfl(e, jl < 0 ? 0 : jl, 64);
        // lane prefix of the record counts
        uint32_t inc = n;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if (l >= (uint32_t)d) inc += o;
        }
        pre[l + 1] = inc;
        if (l == 0) pre[0] = 0;
        count = __shfl(inc, 63, 64);
        if (l == 0 && O.hdr_err[r]) fail |= SPF_DECODE;  // a bad version byte: the exact path reports it
        if (fail) atomicOr(O.fail, fail);
        if (O.dbg && fail && atomicAdd(O.dbg, 1u) < 48)
            printf("span %lu run %u local %lu cs %lu ce %lu len %lu | lane %u a %lu b %lu st %lu e %lu n %u P %lu fail %u\n",
                   (unsigned long)s, r, (unsigned long)local, (unsigned long)cs, (unsigned long)ce,
                   (unsigned long)R.len, l, (unsigned long)a, (unsigned long)b, (unsigned long)st,
                   (unsigned long)e, n, (unsigned long)P, fail);
        const bool any_fail = __ballot(fail != 0) != 0;
        if (l == 0) {
            O.first[s] = s0 < ce ? s0 : NO_POS;
            O.exit[s] = ex;
            if (any_fail) s_fail = 1;
        }
        // ---- 3. global index of the span's first record (the look-back needs every span to publish)
        if (tk) t2 = wall_clock64();
        const uint64_t base = span_lookback(O.tstate, s, count);
        if (l == 0) {
            s_base = base;
            if (local == 0) O.run_recb[r] = base;
            if (s + 1 == n_spans) O.run_recb[n_runs] = base + count;
            if (base + count > O.cap) {
                atomicOr(O.fail, SPF_CAP);
                s_fail = SPF_CAP;
            }
        }
    }
    __syncthreads();
    if (tk) t3 = wall_clock64();
    if (s_fail) return;
    count = pre[64];
    const uint64_t base = s_base;
    // ---- 4. the record arrays: thread t parses records t, t + 256, ... from LDS
    uint32_t bad = 0;
    for (uint32_t k = tid; k < count; k += SPAN_THREADS) {
        uint32_t lo = 0, hi = 64;  // lane holding record k: pre[lo] <= k < pre[lo + 1]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= k) lo = mid;
            else hi = mid;
        }
        const uint64_t p = cs + lst[lo * SPAN_LCAP + (k - pre[lo])];
        const RecHdr h = parse_rec<true, 1>(run, R.len, p, ld);
        if (h.err) {
            bad |= h.err == DERR_UTF8 ? SPF_UTF8 : SPF_DECODE;
            continue;
        }
        if (h.size >= (1ull << 31)) {
            bad |= SPF_DECODE;
            continue;
        }
        bool ascii;
        const uint64_t fpv = key_tail_fp(run + p + 5, (uint32_t)h.klen, ascii, ld);
        const uint64_t o = base + k;
        O.rec_addr[o] = (uint64_t)(run + p);
        O.rec_hi[o] = h.hi;
        O.rec_lo[o] = h.lo;
        O.rec_klen[o] = (uint32_t)h.klen;
        O.rec_meta[o] = (uint32_t)h.size | (h.marker == 2 ? 0x80000000u : 0u);
        O.rec_fp[o] = fpv;
    }
    if (bad) atomicOr(O.fail, bad);
    if (tk) {
        __syncthreads();
        if (tid == 0) {
            const uint64_t t4 = wall_clock64();
            atomicAdd((unsigned long long*)&tk[0], (unsigned long long)(t1 - t0));
            atomicAdd((unsigned long long*)&tk[1], (unsigned long long)(t2 - t1));
            atomicAdd((unsigned long long*)&tk[2], (unsigned long long)(t3 - t2));
            atomicAdd((unsigned long long*)&tk[3], (unsigned long long)(t4 - t3));
        }
    }
}

// every span after a run's first starts where the nearest earlier span with records ended; a span
// with no record start (the tail of a run, or records longer than a span) must lie inside the record
// that crosses it; a run's last record ends at the run's end
constexpr uint32_t SPAN_BACK = 64;  // spans a check looks back over (longer records: the chunk walks)
__global__ void k_span_check(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_spans, SpanOut O) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_spans) return;
    const uint32_t r = span_run(runs, n_runs, s);
    const RunInfo R = runs[r];
    const uint64_t local = s - R.chunk_base;
    const uint64_t first = O.first[s];
    bool bad = false;
    uint64_t pe = 0;  // exit of the nearest earlier span of this run with records
    if (local > 0) {
        uint64_t q = s - 1;
        uint32_t k = 0;
        while (O.first[q] == NO_POS && q > R.chunk_base && k < SPAN_BACK) --q, ++k;
        if (O.first[q] == NO_POS) bad = true;  // span 0 of a run always has records: too far back
        pe = O.exit[q];
        const uint64_t cs = 1 + local * SPAN, ce = cs + SPAN < R.len ? cs + SPAN : R.len;
        bad = bad || (first == NO_POS ? pe < ce : first != pe);
    }
    if (local + 1 == R.n_chunks) bad = bad || (first == NO_POS ? pe != R.len : O.exit[s] != R.len);
    if (bad) atomicOr(O.fail, SPF_CHAIN);
    if (O.dbg && bad && atomicAdd(O.dbg, 1u) < 64)
        printf("check span %lu run %u local %lu first %lu prev_exit %lu exit %lu len %lu\n", (unsigned long)s, r,
               (unsigned long)local, (unsigned long)first, (unsigned long)pe, (unsigned long)O.exit[s],
               (unsigned long)R.len);
}

void launch_span_parse(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_spans, const SpanOut& O) {
    if (!n_spans) return;
    k_span_parse<<<(uint32_t)n_spans, SPAN_THREADS, 0, s>>>(runs, n_runs, n_spans, O);
    k_span_check<<<(uint32_t)((n_spans + 255) / 256), 256, 0, s>>>(runs, n_runs, n_spans, O);
}

}  // namespace skv
