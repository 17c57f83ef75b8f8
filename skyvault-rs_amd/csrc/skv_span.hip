// skv_span.hip — one-pass parse of variable-length runs (gfx950): runs::read_run_stream
// (runs.rs:559-626) for every input run at once, reading every run byte exactly once.
//
// The chunk-walk parse (k_spec / k_emit, skv_kernels.hip) reads each record's header lines twice
// from HBM with dependent loads: 104 GB of line traffic for config 3F's 63 GB of runs. Here one
// workgroup (SPAN / 64 threads) takes one SPAN-byte span of a run and:
//   1. stages the span (+ MARGIN bytes of the next, for records that start near its end) in LDS
//      with coalesced 16-byte loads;
//   2. resolves its record chain in LDS with every thread: each thread marks the marker-valued
//      bytes (1 Put, 2 Delete) of its 64 staged bytes as candidate record starts; each candidate
//      decodes its header from LDS (key length, a Put's value length) into the candidate its record
//      ends on, or EXIT (the record ends past the span), or DEAD (no candidate there, or a header
//      that does not decode); pointer jumping (one jump table per power of two) gives every
//      candidate its chain length and terminal. The span's first record is its run's first byte
//      (span 0), else the first candidate whose chain reaches EXIT with at least min(3, longest)
//      records; the chain's records are listed by composing jumps (one lookup per set bit);
//   3. publishes its record count (decoupled look-back over spans in ticket order) to learn the
//      global index of its first record;
//   4. parses its records again from LDS (prefix, key length, size | Delete, fingerprint of the key
//      bytes past 16, exact UTF-8) and writes the record arrays at their final indices.
// A span's chosen first start is checked against the previous span's exit by k_span_check.
// A span in which no record starts (a run's short tail, or inside a record longer than a span) is
// checked to lie inside the record that crosses it. Anything unusual -- a decode error, an invalid
// UTF-8 key, a first start off the record chain, more candidates than a span resolves, more records
// than the arrays hold -- sets a fail bit, and the host runs the chunk-walk parse instead, which
// reproduces the reference's exact error. Only a clean decode of every run is taken from here.
// (Round 3's walk -- 64 lanes of wave 0 scanning their bytes one at a time with a 3-record decode at
// every marker-valued byte -- spent 350 us per span in lane divergence; tools/r03_spandbg.sh.)
#include "skv_dev.hpp"
#include "skv_launch.hpp"

namespace skv {

constexpr uint32_t SPAN = SPAN_BYTES;
constexpr uint32_t SPAN_MARGIN = 512;                       // bytes staged past the span
constexpr uint32_t SPAN_THREADS = SPAN / 64;               // 64 staged bytes per thread
constexpr uint32_t SPAN_PT = SPAN / SPAN_THREADS;           // staged bytes a thread scans for markers
constexpr uint32_t SPAN_BLOCKS = (SPAN + SPAN_MARGIN) / 16 + 2;  // staged 16-byte blocks
constexpr uint32_t SPAN_WORDS = SPAN / 32;                  // candidate bitmap words
constexpr uint32_t SPAN_WPT = (SPAN_WORDS + SPAN_THREADS - 1) / SPAN_THREADS;
constexpr uint32_t SPAN_CCAP = SPAN / 32;                   // candidates a span resolves (more: the chunk walks)
constexpr uint32_t SPAN_CPT = SPAN_CCAP / SPAN_THREADS;     // candidates per thread in the chain phases
constexpr uint32_t span_log2(uint32_t v) { return v <= 1 ? 0 : 1 + span_log2(v >> 1); }
constexpr uint32_t SPAN_LV = span_log2(SPAN_CCAP) + 1;     // jump levels: 2^(LV-1) >= CCAP
constexpr uint16_t SJ_EXIT = 0xFFFE, SJ_DEAD = 0xFFFF;      // jump terminals
constexpr uint32_t SNX_LONG = 0xFFFFFFFFu;                  // a record end past the staged bytes
static_assert(SPAN_PT % 16 == 0 && SPAN_PT <= 64, "a thread's marker bits fit one 64-bit mask");
static_assert(SPAN <= 65536 && SPAN_WORDS % SPAN_THREADS == 0 && SPAN_THREADS <= 1024 && SPAN_THREADS % 64 == 0,
              "u16 offsets, whole bitmap words per thread, whole waves");
static_assert((1u << (SPAN_LV - 1)) >= SPAN_CCAP && SPAN_CCAP < SJ_EXIT && SPAN_CCAP % SPAN_THREADS == 0,
              "jump levels cover the longest chain");

enum : uint32_t { SPF_DECODE = 1, SPF_CHAIN = 2, SPF_OVER = 8, SPF_UTF8 = 16, SPF_CAP = 32 };

// Loads of the record parsers: blocks inside the staged bytes come from LDS, others from HBM
struct SpanLoad {
    const uint4* lds;
    uintptr_t g0, g1;
    __device__ __forceinline__ uint4 operator()(uintptr_t a) const {
        return (a >= g0 && a < g1) ? lds[(a - g0) >> 4] : gblk(a);
    }
};

// big-endian u32 at staged byte bo (bo + 4 <= staged bytes)
__device__ __forceinline__ uint32_t span_be32(const uint4* buf, uint32_t bo) {
    const uint32_t q = bo >> 4, sh = bo & 15;
    const uint4 a = buf[q];
    const uint4 b = sh > 12 ? buf[q + 1] : make_uint4(0, 0, 0, 0);
    return __builtin_bswap32(funnel16(a, b, sh).x);
}

// Rust str Ord of two parsed keys (runs.rs:190-198's comparison), the bytes past the 16-byte
// prefixes through the span loader (LDS when staged)
__device__ inline int span_key_cmp(const RecHdr& a, const uint8_t* ka, const RecHdr& b, const uint8_t* kb,
                                   const SpanLoad& ld) {
    if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
    if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
    if (a.klen > 16 && b.klen > 16) {
        const uint64_t n = (a.klen < b.klen ? a.klen : b.klen) - 16;
        for (uint64_t i = 0; i < n; i += 16) {
            const uint32_t m = (uint32_t)(n - i < 16 ? n - i : 16);
            const uint4 x = load_window16(ka + 16 + i, m, ld), y = load_window16(kb + 16 + i, m, ld);
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t mk = dword_mask(0, m, q);
                const uint32_t xa = __builtin_bswap32(xs[q] & mk), ya = __builtin_bswap32(ys[q] & mk);
                if (xa != ya) return xa < ya ? -1 : 1;
            }
        }
    }
    return a.klen < b.klen ? -1 : (a.klen > b.klen ? 1 : 0);
}

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
    __shared__ uint32_t cbits[SPAN_WORDS];            // candidate starts, bit x
    __shared__ uint16_t crank[SPAN_WORDS];            // candidates before each bitmap word
    __shared__ uint16_t cpos[SPAN_CCAP];              // candidate i's offset x (ascending)
    __shared__ uint32_t cnx[SPAN_CCAP];               // its record's end (offset), SNX_LONG past the stage
    __shared__ uint16_t jmp[SPAN_LV * SPAN_CCAP];     // level r: the candidate 2^r records on, or a terminal
    __shared__ uint16_t lst[SPAN_CCAP];               // the chosen chain's record offsets, in order
    __shared__ uint32_t ws[SPAN_THREADS / 64];
    __shared__ uint32_t s_more[3];
    __shared__ uint64_t s_t, s_base, s_exit;
    __shared__ uint32_t s_fail, s_maxlen, s_s0, s_len, s_last;
    const uint32_t tid = threadIdx.x;
    uint64_t* const tk = O.dbg ? (uint64_t*)(O.dbg + 6) : nullptr;  // phase ticks (SKV_SPAN_DBG)
    uint64_t t0 = tk ? wall_clock64() : 0, t1 = 0, t2 = 0, t3 = 0;
    if (tid == 0) {
        s_t = atomicAdd(O.ticket, 1u);
        s_fail = 0;
        s_maxlen = 0;
        s_s0 = NO_POS32;
        s_len = 0;
        s_last = 0;
        s_exit = NO_POS;
        s_more[0] = s_more[1] = s_more[2] = 0;
    }
    for (uint32_t w = tid; w < SPAN_WORDS; w += SPAN_THREADS) cbits[w] = 0;
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
    // offsets x are relative to cs; staged byte of x: x + d0
    const uint32_t d0 = (uint32_t)((uintptr_t)run + cs - g0);
    const uint32_t nspan = (uint32_t)(ce - cs);
    const uint64_t rel = R.len - cs;                          // run bytes from x = 0
    const uint32_t avail = (uint32_t)(g1 - g0) - d0;           // staged bytes from x = 0 (>= min(rel, nspan + MARGIN))
    // ---- 2a. candidates: marker-valued bytes at x in [0, nspan); bit i of cm <-> x = xs + i
    const int32_t xs = (int32_t)(tid * SPAN_PT) - (int32_t)d0;
    uint64_t cm = 0;
#pragma unroll
    for (uint32_t q = 0; q < SPAN_PT / 16; ++q) {
        const uint32_t b = tid * (SPAN_PT / 16) + q;
        const uint4 v = b < nb ? buf[b] : make_uint4(0, 0, 0, 0);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) {
            const uint32_t by = (w4[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            if (by - 1u < 2u) cm |= 1ull << (q * 16 + i);
        }
    }
    if (xs < 0) cm &= ~0ull << (uint32_t)(-xs);  // bytes before cs (-xs <= 15)
    {
        const int32_t lim = (int32_t)nspan - xs;  // bits from lim on are past the span
        if (lim <= 0) cm = 0;
        else if (lim < 64) cm &= (1ull << (uint32_t)lim) - 1;
    }
    // the span's last d0 bytes sit in staged block SPAN / 16: the last thread scans it too
    // (bit i of cm2 <-> x = SPAN - d0 + i)
    uint32_t cm2 = 0;
    if (tid == SPAN_THREADS - 1 && d0) {
        const uint32_t b = SPAN / 16;
        const uint4 v = b < nb ? buf[b] : make_uint4(0, 0, 0, 0);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) {
            const uint32_t by = (w4[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            if (by - 1u < 2u) cm2 |= 1u << i;
        }
        const int32_t lim2 = (int32_t)nspan - (int32_t)(SPAN - d0);
        if (lim2 <= 0) cm2 = 0;
        else if (lim2 < 32) cm2 &= (1u << (uint32_t)lim2) - 1u;
    }
    for (uint64_t c = cm; c; c &= c - 1) {
        const uint32_t x = (uint32_t)(xs + (int32_t)__builtin_ctzll(c));
        atomicOr(&cbits[x >> 5], 1u << (x & 31));
    }
    for (uint32_t c = cm2; c; c &= c - 1) {
        const uint32_t x = SPAN - d0 + (uint32_t)__builtin_ctz(c);
        atomicOr(&cbits[x >> 5], 1u << (x & 31));
    }
    __syncthreads();
    // ---- 2b. candidate ranks: exclusive prefix of the bitmap's popcounts
    uint32_t m;
    {
        uint32_t pc[SPAN_WPT], mine = 0;
#pragma unroll
        for (uint32_t u = 0; u < SPAN_WPT; ++u) {
            pc[u] = __builtin_popcount(cbits[tid * SPAN_WPT + u]);
            mine += pc[u];
        }
        const uint32_t lane = tid & 63, wv = tid >> 6;
        uint32_t inc = mine;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) ws[wv] = inc;
        __syncthreads();
        uint32_t before = 0;
        m = 0;
#pragma unroll
        for (uint32_t w = 0; w < SPAN_THREADS / 64; ++w) {
            before += w < wv ? ws[w] : 0u;
            m += ws[w];
        }
        uint32_t ex = before + inc - mine;
#pragma unroll
        for (uint32_t u = 0; u < SPAN_WPT; ++u) {
            crank[tid * SPAN_WPT + u] = (uint16_t)ex;
            ex += pc[u];
        }
    }
    __syncthreads();
    auto rank_of = [&](uint32_t x) -> uint32_t {
        return crank[x >> 5] + __builtin_popcount(cbits[x >> 5] & ((1u << (x & 31)) - 1u));
    };
    const bool over = m > SPAN_CCAP;  // (uniform)
    // ---- 2c. each candidate's record: its end, and the candidate there (level-0 jump)
    auto candidate = [&](uint32_t x) {
        const uint32_t i = rank_of(x);
        cpos[i] = (uint16_t)x;
        uint16_t j0 = SJ_DEAD;
        uint32_t nx = SNX_LONG;
        if ((uint64_t)x + 5 <= rel) {  // runs.rs:570-576: the key length is in the run
            const uint64_t kend = (uint64_t)x + 5 + span_be32(buf, x + d0 + 1);
            bool ok = false, known = false;
            uint64_t e = 0;
            if (kend <= rel) {  // :580-583 the key is in the run
                if (bytes[x + d0] == 2) {  // Delete: marker, key length, key
                    ok = known = true;
                    e = kend;
                } else if (kend + 4 <= rel) {  // :598-604 the value length is in the run
                    if (kend + 4 <= avail) {
                        e = kend + 4 + span_be32(buf, (uint32_t)kend + d0);
                        ok = known = e <= rel;  // :608-611 the value is in the run
                    } else {
                        ok = true;  // ends past the staged bytes, so past the span: EXIT
                    }
                }
            }
            if (ok) {
                if (known && e < nspan) j0 = ((cbits[e >> 5] >> (e & 31)) & 1u) ? (uint16_t)rank_of((uint32_t)e) : SJ_DEAD;
                else j0 = SJ_EXIT;
                nx = known && e < SNX_LONG ? (uint32_t)e : SNX_LONG;
            }
        }
        jmp[i] = j0;
        cnx[i] = nx;
    };
    if (!over) {
        for (uint64_t c = cm; c; c &= c - 1) candidate((uint32_t)(xs + (int32_t)__builtin_ctzll(c)));
        for (uint32_t c = cm2; c; c &= c - 1) candidate(SPAN - d0 + (uint32_t)__builtin_ctz(c));
    }
    __syncthreads();
    // ---- 2d. pointer jumping: level r = level r-1 twice; stops once every chain has ended
    uint32_t lv = 1;
    if (!over && m > 0) {
        for (uint32_t rr = 1; rr < SPAN_LV; ++rr) {
            uint32_t more = 0;
            for (uint32_t i = tid; i < m; i += SPAN_THREADS) {
                const uint16_t y = jmp[(rr - 1) * SPAN_CCAP + i];
                const uint16_t z = y < SJ_EXIT ? jmp[(rr - 1) * SPAN_CCAP + y] : y;
                jmp[rr * SPAN_CCAP + i] = z;
                more |= z < SJ_EXIT ? 1u : 0u;
            }
            if (more) s_more[rr % 3] = 1;
            if (tid == 0) s_more[(rr + 1) % 3] = 0;
            __syncthreads();
            lv = rr + 1;
            if (!s_more[rr % 3]) break;  // (uniform: read between this barrier and the next clear)
        }
    }
    // ---- 2e. chain length and terminal of each candidate (binary lifting), then the first start
    uint32_t clen[SPAN_CPT], clast[SPAN_CPT];
    bool cexit[SPAN_CPT];
#pragma unroll
    for (uint32_t u = 0; u < SPAN_CPT; ++u) {
        const uint32_t i = tid + u * SPAN_THREADS;
        clen[u] = 0;
        clast[u] = 0;
        cexit[u] = false;
        if (!over && i < m) {
            uint32_t x = i, len = 1;
            for (int rr = (int)lv - 1; rr >= 0; --rr) {
                const uint16_t y = jmp[rr * SPAN_CCAP + x];
                if (y < SJ_EXIT) {
                    x = y;
                    len += 1u << rr;
                }
            }
            clen[u] = len;
            clast[u] = x;
            cexit[u] = jmp[x] == SJ_EXIT;
            if (cexit[u]) atomicMax(&s_maxlen, len);
        }
    }
    __syncthreads();
    {
        const uint32_t need = s_maxlen < 3 ? s_maxlen : 3u;
#pragma unroll
        for (uint32_t u = 0; u < SPAN_CPT; ++u) {
            const uint32_t i = tid + u * SPAN_THREADS;
            if (local == 0) {  // the run's first record starts at its byte 1 (x = 0)
                if (i == 0 && m > 0 && !over && (cbits[0] & 1u) && cexit[u]) s_s0 = 0;
            } else if (cexit[u] && clen[u] >= need) {
                atomicMin(&s_s0, i);
            }
        }
    }
    __syncthreads();
    const uint32_t s0 = s_s0;
#pragma unroll
    for (uint32_t u = 0; u < SPAN_CPT; ++u)
        if (tid + u * SPAN_THREADS == s0) {
            s_len = clen[u];
            s_last = clast[u];
        }
    __syncthreads();
    // ---- 2f. the chain's records (jumps composed by the bits of d) and its exit
    const uint32_t n0 = s0 != NO_POS32 ? s_len : 0u;
    for (uint32_t d = tid; d < n0; d += SPAN_THREADS) {
        uint32_t x = s0;
        for (uint32_t rr = 0; rr < lv; ++rr)
            if ((d >> rr) & 1u) x = jmp[rr * SPAN_CCAP + x];
        lst[d] = cpos[x];
    }
    if (tid == 0) {
        uint32_t f = 0;
        if (over) f |= SPF_OVER;
        if (local == 0 && s0 == NO_POS32) f |= SPF_DECODE;  // the run's first record does not decode
        if (O.hdr_err[r]) f |= SPF_DECODE;                 // a bad version byte: the exact path reports it
        if (n0) {
            const uint32_t L = s_last;
            if (cnx[L] != SNX_LONG) {
                s_exit = cs + cnx[L];
            } else {  // a record running past the staged bytes: its value length from HBM
                const RecHdr h = parse_rec<false, 0>(run, R.len, cs + cpos[L], ld);
                if (h.err) f |= SPF_DECODE;
                s_exit = cs + cpos[L] + h.size;
            }
        }
        if (f) s_fail = f;
    }
    __syncthreads();
    uint32_t count = s_fail ? 0u : n0;
    if (tid < 64) {
        const uint64_t first = n0 ? cs + cpos[s0] : NO_POS;
        if (tid == 0) {
            O.first[s] = first;
            O.exit[s] = s_exit;
        }
        if (O.dbg && s_fail && tid == 0 && atomicAdd(O.dbg, 1u) < 48)
            printf("span %lu run %u local %lu cs %lu ce %lu len %lu | cand %u levels %u first %lu exit %lu n %u fail %u\n",
                   (unsigned long)s, r, (unsigned long)local, (unsigned long)cs, (unsigned long)ce,
                   (unsigned long)R.len, m, lv, (unsigned long)first, (unsigned long)s_exit, n0, s_fail);
        // ---- 3. global index of the span's first record (the look-back needs every span to publish)
        if (tk) t2 = wall_clock64();
        const uint64_t base = span_lookback(O.tstate, s, count);
        if (tid == 0) {
            s_base = base;
            O.sbase[s] = base;
            if (local == 0) O.run_recb[r] = base;
            if (s + 1 == n_spans) O.run_recb[n_runs] = base + count;
            if (base + count > O.cap) s_fail |= SPF_CAP;
            if (s_fail) atomicOr(O.fail, s_fail);
        }
    }
    __syncthreads();
    if (tk) t3 = wall_clock64();
    if (s_fail) return;
    const uint64_t base = s_base;
    // ---- 4. the record arrays: thread t parses records t, t + SPAN_THREADS, ... from LDS
    uint32_t bad = 0;
    for (uint32_t d = tid; d < count; d += SPAN_THREADS) {
        const uint64_t p = cs + lst[d];
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
        const uint64_t o = base + d;
        if (O.first_dec && d > 0) {  // in-stream order against the span's record before (k_span_check: its first)
            const uint64_t q = cs + lst[d - 1];
            const RecHdr hq = parse_rec<true, 0>(run, R.len, q, ld);
            if (span_key_cmp(hq, run + q + 5, h, run + p + 5, ld) > 0) {
                atomicMin(&O.first_dec[R.stream], (unsigned long long)(o - 1));
                atomicOr(O.any_dec, 1u);
            }
        }
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
    // the order check across span edges: a span's first record against the record before it in its
    // stream (the previous span's last one, or the last one of the stream's previous member run)
    // (only when every span emitted: a failed span left its records unwritten, and the host discards
    // the arrays anyway)
    if (!bad && O.first_dec && first != NO_POS && (local > 0 || (r > 0 && runs[r - 1].stream == R.stream)) &&
        __hip_atomic_load(O.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        const uint64_t g = O.sbase[s];
        if (g > 0) {
            const int c = key_cmp(O.rec_hi[g - 1], O.rec_lo[g - 1], O.rec_klen[g - 1], (const uint8_t*)O.rec_addr[g - 1] + 5,
                                  O.rec_hi[g], O.rec_lo[g], O.rec_klen[g], (const uint8_t*)O.rec_addr[g] + 5);
            if (c > 0) {
                atomicMin(&O.first_dec[R.stream], (unsigned long long)(g - 1));
                atomicOr(O.any_dec, 1u);
            }
        }
    }
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
