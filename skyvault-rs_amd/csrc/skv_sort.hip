// skv_sort.hip — the record sort behind merges of more than TILE_TARGET / 2 streams (gfx950).
//
// k_way::merge pops records in (key ascending, seq_no descending) order (k_way.rs:14-33), and a
// stream's own records come out in stream order (its order is checked first, runs.rs:190-198).
// Records are numbered stream by stream in rank (seq_no descending) order, so the merged order is
// the order of (key bytes, record index): a sort. For up to TILE_TARGET / 2 streams the splitter
// merge of skv_kernels.hip produces it from the sorted streams; past that its (tiles x streams)
// bounds table outgrows memory (config 5: 10^6 WAL runs of 83 records), and this sample sort
// takes over:
//   1. one SElem {prefix, address, index, key length} per record (coalesced)
//   2. samples: every SORT_EVERY-th element, sorted by this same routine (recursion down to one
//      workgroup)
//   3. splitters: every SORT_OV-th sorted sample; bucket b holds the keys in (sp[b-1], sp[b]]
//      (key-only order, so equal keys share a bucket), L[b] = common prefix length of its two
//      splitters, which every key of the bucket shares
//   4. bucket of each element (binary search over the splitters), slot by atomic count, exclusive
//      scan, scatter
//   5. one workgroup per bucket: bitonic sort in LDS on the 16 key bytes after the bucket's common
//      prefix, then the key length and record index (the rest of a longer key from memory on a
//      tie); buckets above SORT_CAP sort in global memory (same order, slower)
// The sorted records then form ONE stream, and the level-0 merge machinery runs on them with
// k = 1 on dense key ranks (one per distinct key, flagged by the bucket sort): first record per
// key, Delete filter, dense output arrays (skv_compact.hip).
#include "skv_launch.hpp"

namespace skv {

// index of the first differing byte among the first n bytes (n if none)
__device__ inline uint64_t sk_bytes_diff(const uint8_t* a, const uint8_t* b, uint64_t n) {
    for (uint64_t i = 0; i < n; i += 16) {
        const uint32_t m = (uint32_t)(n - i < 16 ? n - i : 16);
        const uint4 x = load_window16(a + i, m), y = load_window16(b + i, m);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t d = (xs[q] ^ ys[q]) & dword_mask(0, m, q);
            if (d) return i + 4 * q + (__builtin_ctz(d) >> 3);
        }
    }
    return n;
}

__device__ __forceinline__ const uint8_t* sk_key(const SElem& e) { return (const uint8_t*)e.addr + 5; }

// key-only order: Rust str Ord (bytewise, a proper prefix first), as HeapItem compares keys
__device__ inline int sk_kcmp(const SElem& a, const SElem& b) {
    if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
    if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
    if (a.klen > 16 && b.klen > 16) {
        const uint32_t n = a.klen < b.klen ? a.klen : b.klen;
        const int s = bytes_cmp16(sk_key(a) + 16, sk_key(b) + 16, n - 16);
        if (s) return s;
    }
    return a.klen < b.klen ? -1 : (a.klen > b.klen ? 1 : 0);
}

// the merged order: key, then record index (== seq_no descending, then stream order)
__device__ __forceinline__ bool sk_less(const SElem& a, const SElem& b) {
    const int c = sk_kcmp(a, b);
    return c ? c < 0 : a.pos < b.pos;
}

// common prefix length of two keys
__device__ inline uint32_t sk_common(const SElem& a, const SElem& b) {
    const uint32_t n = a.klen < b.klen ? a.klen : b.klen;
    uint64_t c;
    if (a.hi != b.hi) c = __builtin_clzll(a.hi ^ b.hi) >> 3;
    else if (a.lo != b.lo) c = 8 + (__builtin_clzll(a.lo ^ b.lo) >> 3);
    else if (n > 16) c = 16 + sk_bytes_diff(sk_key(a) + 16, sk_key(b) + 16, n - 16);
    else c = 16;
    return (uint32_t)(c < n ? c : n);
}

// the 16 key bytes from byte L on (big-endian, zero past the key's end)
__device__ inline void sk_window(const SElem& e, uint32_t L, uint64_t& wh, uint64_t& wl) {
    if (L == 0) {
        wh = e.hi;
        wl = e.lo;
        return;
    }
    wh = wl = 0;
    if (e.klen <= L) return;
    const uint32_t m = e.klen - L < 16 ? e.klen - L : 16;
    const uint4 v = load_window16(sk_key(e) + L, m);
    const uint32_t d0 = v.x & dword_mask(0, m, 0), d1 = v.y & dword_mask(0, m, 1);
    const uint32_t d2 = v.z & dword_mask(0, m, 2), d3 = v.w & dword_mask(0, m, 3);
    wh = ((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1);
    wl = ((uint64_t)__builtin_bswap32(d2) << 32) | __builtin_bswap32(d3);
}

// ---------------------------------------------------------------------------------------------
// SKV_SORT_PROF=1 (diagnostic builds): per-phase wall ticks of k_sort_bucket / k_sort_tile summed by
// each workgroup's thread 0 into g_sort_prof (read with sort_prof_read)
#ifndef SKV_SORT_PROF
#define SKV_SORT_PROF 0
#endif
#if SKV_SORT_PROF
__device__ unsigned long long g_sort_prof[16];
#define SPROF_T(v) const uint64_t v = threadIdx.x == 0 ? wall_clock64() : 0
#define SPROF_ADD(i, a, b) \
    do { if (threadIdx.x == 0) atomicAdd(&g_sort_prof[i], (unsigned long long)((b) - (a))); } while (0)
#else
#define SPROF_T(v) do {} while (0)
#define SPROF_ADD(i, a, b) do {} while (0)
#endif
void sort_prof_read(unsigned long long* out16) {
#if SKV_SORT_PROF
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_sort_prof), 16 * 8);
#else
    for (int i = 0; i < 16; ++i) out16[i] = 0;
#endif
}

// pos is the tie-break: the record index (newer stream first), or for a writer batch the index
// from the end (the last op of a key wins, BTreeMap insertion in writer_service.rs:153-157)
__global__ void k_sort_load(uint64_t R, const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                            const uint64_t* __restrict__ addr, const uint32_t* __restrict__ klen, SElem* E,
                            bool last_wins) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    SElem e;
    e.hi = hi[i];
    e.lo = lo[i];
    e.addr = addr[i];
    e.pos = (uint32_t)(last_wins ? R - 1 - i : i);
    e.klen = klen[i];
    E[i] = e;
}

// The record arrays in sorted order (meta follows its record). The merge stage then compares
// dense key ranks (hi = rank of the key among the distinct keys, lo = 0, compare length 0): the
// same order and the same equal-key groups as the key bytes, with no key bytes read again.
// const_meta != 0: every record has that meta (one record format in every run, e.g. WAL flushes
// of one key/value shape) -- no gather of meta_in at the sorted element's record, a random 4-byte
// read that fetched a line of its own per record.
__global__ void k_sort_store(uint64_t R, const SElem* __restrict__ E, const uint32_t* __restrict__ meta_in,
                             uint32_t const_meta, const uint64_t* __restrict__ newkey,
                             const uint64_t* __restrict__ newkey_ex, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                             uint32_t* klen, uint32_t* cmp_klen, uint32_t* meta, bool last_wins, SortMerged M) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < R;
    uint32_t sz = 0xFFFFFFFFu, szx = 0;
    if (live) {
        const SElem e = E[i];
        const uint64_t src = last_wins ? R - 1 - e.pos : e.pos;
        const uint64_t nk = newkey[i];
        const uint32_t m = const_meta ? const_meta : meta_in[src];
        if (!M.m_rec || M.arrays) {
            hi[i] = newkey_ex[i] + nk - 1;
            lo[i] = 0;
            addr[i] = e.addr;
            klen[i] = e.klen;
            cmp_klen[i] = 0;
            meta[i] = m;
        }
        // the merged arrays of the one sorted list, straight from the sort: the first record of each
        // key is its survivor (k_way.rs:146-151), and its index among the survivors is its key's rank
        if (M.m_rec && nk) {
            const uint64_t g = newkey_ex[i];
            M.m_rec[g] = (uint32_t)i;
            M.m_src[g] = e.addr;
            M.size[g] = m & 0x7FFFFFFFu;
            M.del[g] = m >> 31;
            sz = szx = m & 0x7FFFFFFFu;
        }
    }
    if (M.m_rec) {  // (min, max) surviving record size of this block's records, for the split (k_chain)
        __shared__ uint32_t s_mm[2 * (256 / 64)];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t a = __shfl_xor(sz, d, 64), b = __shfl_xor(szx, d, 64);
            sz = a < sz ? a : sz;
            szx = b > szx ? b : szx;
        }
        const uint32_t w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            s_mm[2 * w] = sz;
            s_mm[2 * w + 1] = szx;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // one pair per block (one address for every block's atomics was 29 ms at config 5)
            for (uint32_t q = 1; q < (blockDim.x >> 6); ++q) {
                sz = s_mm[2 * q] < sz ? s_mm[2 * q] : sz;
                szx = s_mm[2 * q + 1] > szx ? s_mm[2 * q + 1] : szx;
            }
            M.mm[2 * blockIdx.x] = sz;
            M.mm[2 * blockIdx.x + 1] = szx;
        }
    }
}

// S[j] = E[j * n / Ns]  (n < 2^32)
__global__ void k_sort_sample(const SElem* __restrict__ E, uint64_t n, uint64_t Ns, SElem* S) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= Ns) return;
    S[j] = E[j * n / Ns];
}

// L[b] of the Tb buckets; splitter b (b < Tb - 1) is sorted sample (b + 1) * ov - 1
__global__ void k_sort_prefix(const SElem* __restrict__ Ss, uint64_t ov, uint64_t Tb, uint32_t* L) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= Tb) return;
    L[b] = (b == 0 || b + 1 == Tb) ? 0u : sk_common(Ss[b * ov - 1], Ss[(b + 1) * ov - 1]);
}

// A splitter for the bucket search: the 16-byte prefix plus key bytes 16..31 (big-endian, zero
// padded), so keys of up to 32 bytes compare without touching the records again.
struct SSplit {
    uint64_t hi, lo, x0, x1;
    uint64_t addr;
    uint32_t klen, pad;
};

// The key's true 16-byte prefix of an element whose (hi, lo) hold its window from byte L on (the
// bucket pass, pre): bytes [0, L) are the bucket's common prefix -- its splitter's -- and bytes
// [L, 16) the window's first 16 - L. Every key of the bucket is longer than L, so no byte of the
// splitter's part lies past the key's end; the window is zero past it.
// (shi, slo: the splitter's 16-byte prefix, read once per bucket by the caller -- read per element,
// the loads were ordered after every output store, which may alias them)
__device__ __forceinline__ void sk_restore(SElem& e, uint32_t L, uint64_t shi, uint64_t slo) {
    if (!L) return;
    if (L >= 16) {
        e.hi = shi;
        e.lo = slo;
        return;
    }
    const uint32_t sh = 8 * L;  // 8 .. 120: the window moves right by L bytes
    const uint64_t rh = sh < 64 ? e.hi >> sh : 0;
    const uint64_t rl = sh < 64 ? (e.lo >> sh) | (e.hi << (64 - sh)) : (e.hi >> (sh - 64));
    const uint64_t mh = sh >= 64 ? ~0ull : ~0ull << (64 - sh);
    const uint64_t ml = sh <= 64 ? 0ull : ~0ull << (128 - sh);
    e.hi = (shi & mh) | rh;
    e.lo = (slo & ml) | rl;
}

__device__ __forceinline__ void sk_ext(const uint8_t* key, uint32_t klen, uint64_t& x0, uint64_t& x1) {
    x0 = x1 = 0;
    if (klen <= 16) return;
    const uint32_t m = klen - 16 < 16 ? klen - 16 : 16;
    const uint4 v = load_window16(key + 16, m);
    x0 = ((uint64_t)__builtin_bswap32(v.x & dword_mask(0, m, 0)) << 32) | __builtin_bswap32(v.y & dword_mask(0, m, 1));
    x1 = ((uint64_t)__builtin_bswap32(v.z & dword_mask(0, m, 2)) << 32) | __builtin_bswap32(v.w & dword_mask(0, m, 3));
}

// The first 32 key bytes of a splitter (big-endian words, zero past the key's end). Zero-padded
// windows order as the keys do wherever they differ (a proper prefix pads with zeros, which sort
// first), so the bucket search compares windows and reads the full SSplit only on a tie. 32 bytes,
// not 16: WAL keys ("{table}." + a zero-filled decimal, gen.wal_run) share their first 16 bytes
// within a table.
struct SWin {
    uint64_t hi, lo, x0, x1;
};

__global__ void k_sort_splitters(const SElem* __restrict__ Ss, uint64_t ov, uint64_t nsp, SSplit* sp, SWin* win) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nsp) return;
    const SElem e = Ss[(b + 1) * ov - 1];
    SSplit o;
    o.hi = e.hi;
    o.lo = e.lo;
    sk_ext(sk_key(e), e.klen, o.x0, o.x1);
    o.addr = e.addr;
    o.klen = e.klen;
    o.pad = 0;
    sp[b] = o;
    win[b] = SWin{o.hi, o.lo, o.x0, o.x1};
}

// The 8 key bytes from byte c on, big-endian, zero past the key's end.
__device__ __forceinline__ uint64_t sk_word8(const uint8_t* key, uint32_t klen, uint32_t c) {
    if (klen <= c) return 0;
    const uint32_t m = klen - c < 8 ? klen - c : 8;
    const uint4 v = load_window16(key + c, m);
    return ((uint64_t)__builtin_bswap32(v.x & dword_mask(0, m, 0)) << 32) | __builtin_bswap32(v.y & dword_mask(0, m, 1));
}

// Group discriminators for the bucket search's global level. Group g holds splitters
// [g top, (g + 1) top - 1), searched after the LDS level has placed a key x strictly after
// boundary splitter g top - 1 and at or before boundary (g + 1) top - 1. Both boundaries share
// their first cp[g] bytes, so x and every splitter of the group share them too (a key that
// differed inside that prefix, or ended in it, would order outside the two boundaries).
// disc[j] = splitter j's 8 key bytes from cp[g] on: where disc differs from x's 8 bytes at cp[g],
// the zero-padded words order as the keys do (the windows' argument), so one 8-byte read decides
// the step and the 32-byte window is read only on a tie.
__global__ void k_sort_disc(const SElem* __restrict__ Ss, uint64_t ov, uint64_t nsp, uint64_t top, uint32_t* cp,
                            uint64_t* disc, ulong2* gw) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nsp) return;
    const uint64_t g = j / top, nt = nsp / top;
    uint32_t c = 0;
    if (g > 0 && g < nt) c = sk_common(Ss[(g * top) * ov - 1], Ss[((g + 1) * top) * ov - 1]);
    if (j % top == 0) cp[g] = c;
    if (j + 1 == nsp && (j + 1) % top == 0) cp[g + 1] = 0;  // a last, empty group
    const SElem e = Ss[(j + 1) * ov - 1];
    disc[j] = sk_word8(sk_key(e), e.klen, c);
    if (gw) {  // the two-pass bucket search's group level: the 16-byte window from cp[g] on
        uint64_t wh, wl;
        sk_window(e, c, wh, wl);
        gw[j] = make_ulong2(wh, wl);
    }
}

// splitter vs element key order (<0, 0, >0)
__device__ __forceinline__ int sk_scmp(const SSplit& a, const SElem& b, uint64_t bx0, uint64_t bx1) {
    if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
    if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
    if (a.klen > 16 && b.klen > 16) {
        if (a.x0 != bx0) return a.x0 < bx0 ? -1 : 1;
        if (a.x1 != bx1) return a.x1 < bx1 ? -1 : 1;
        if (a.klen > 32 && b.klen > 32) {
            const uint32_t n = a.klen < b.klen ? a.klen : b.klen;
            const int s = bytes_cmp16((const uint8_t*)a.addr + 5 + 32, sk_key(b) + 32, n - 32);
            if (s) return s;
        }
    }
    return a.klen < b.klen ? -1 : (a.klen > b.klen ? 1 : 0);
}

// does splitter j (window w) order strictly before x? The full entry only on a window tie.
__device__ __forceinline__ bool sk_sbefore(const SWin& w, const SSplit* __restrict__ sp, uint64_t j, const SElem& x,
                                           uint64_t x0, uint64_t x1) {
    int c = 0;
    if (w.hi != x.hi) c = w.hi < x.hi ? -1 : 1;
    else if (w.lo != x.lo) c = w.lo < x.lo ? -1 : 1;
    else if (w.x0 != x0) c = w.x0 < x0 ? -1 : 1;
    else if (w.x1 != x1) c = w.x1 < x1 ? -1 : 1;
    if (c == 0) c = sk_scmp(sp[j], x, x0, x1);
    return c < 0;
}

// Bucket of each element = the number of splitters ordered strictly before its key; slot by an
// atomic count (the bucket sort restores a deterministic order). Two-level search: the windows of
// every top-th splitter sit in LDS, the final < top splitters are searched in the global window
// table (32 B per splitter: 3.4 MB at config 5's 10^5 splitters, L2-resident, where the 48-byte
// SSplit table was not). Both levels are branch-free power-of-two searches with a step count
// uniform over the wave, run for SB_ILP elements at once so their loads overlap.
#define SKV_SB_THREADS 256
#define SKV_SB_PER 16
#define SKV_SB_TOP 1024
#define SKV_SB_ILP 4  // elements a thread searches at once
constexpr int SB_THREADS = SKV_SB_THREADS, SB_PER = SKV_SB_PER, SB_TOP = SKV_SB_TOP, SB_ILP = SKV_SB_ILP;
static_assert(SB_PER % SB_ILP == 0, "a workgroup's elements in whole ILP batches");
// D (SKV_SB_DIAGK builds only, timing diagnostics with scratch outputs): bit 0 skips the LDS level
// (a hashed group instead), bit 1 the global level, bit 2 the slot atomic
template <int D>
__global__ void __launch_bounds__(SB_THREADS) k_sort_bucket(const SElem* __restrict__ E, uint64_t n,
                                                            const SSplit* __restrict__ sp,
                                                            const SWin* __restrict__ win, uint64_t nsp, uint64_t top,
                                                            const uint32_t* __restrict__ gcp,
                                                            const uint64_t* __restrict__ disc,
                                                            unsigned long long* cnt, uint64_t* bs) {
    __shared__ SWin tt[SB_TOP];
    const uint32_t nt = (uint32_t)(nsp / top);  // top entry j = splitter (j + 1) * top - 1
    for (uint32_t j = threadIdx.x; j < nt; j += SB_THREADS) tt[j] = win[(uint64_t)(j + 1) * top - 1];
    __syncthreads();
    uint32_t s1 = 0;
    if (nt) {
        s1 = 1;
        while (s1 * 2 <= nt) s1 *= 2;
    }
    const uint64_t base = (uint64_t)blockIdx.x * SB_THREADS * SB_PER;
    for (int u0 = 0; u0 < SB_PER; u0 += SB_ILP) {
        SPROF_T(pa);
        SElem x[SB_ILP];
        uint64_t x0[SB_ILP], x1[SB_ILP], g[SB_ILP], len[SB_ILP], c[SB_ILP], dx[SB_ILP];
        uint32_t a[SB_ILP];
        bool live[SB_ILP];
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            const uint64_t i = base + (uint64_t)(u0 + u) * SB_THREADS + threadIdx.x;
            live[u] = i < n;
            x[u] = E[live[u] ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            sk_ext(sk_key(x[u]), x[u].klen, x0[u], x1[u]);
            a[u] = 0;
        }
        SPROF_T(pb);
        SPROF_ADD(0, pa, pb);
        if (D & 1) {
#pragma unroll
            for (int u = 0; u < SB_ILP; ++u) a[u] = (x[u].pos * 2654435761u) % (nt + 1);
        }
        for (uint32_t st = (D & 1) ? 0 : s1; st; st >>= 1) {
#pragma unroll
            for (int u = 0; u < SB_ILP; ++u) {
                const uint32_t p = a[u] + st;
                if (p <= nt) {
                    const bool before = sk_sbefore(tt[p - 1], sp, (uint64_t)p * top - 1, x[u], x0[u], x1[u]);
                    if (before) a[u] = p;
                }
            }
        }
        SPROF_T(pc);
        SPROF_ADD(1, pb, pc);
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            g[u] = (uint64_t)a[u] * top;
            len[u] = a[u] < nt ? top - 1 : nsp - (uint64_t)nt * top;
            c[u] = 0;
            dx[u] = len[u] ? sk_word8(sk_key(x[u]), x[u].klen, gcp[a[u]]) : 0;
        }
        if (D & 2) {
#pragma unroll
            for (int u = 0; u < SB_ILP; ++u) c[u] = len[u] ? dx[u] % len[u] : 0;
        }
        for (uint64_t st = (D & 2) ? 0 : top >> 1; st; st >>= 1) {
#pragma unroll
            for (int u = 0; u < SB_ILP; ++u) {
                const uint64_t p = c[u] + st;
                if (p <= len[u]) {
                    const uint64_t j = g[u] + p - 1, dj = disc[j];
                    const bool before = dj != dx[u] ? dj < dx[u] : sk_sbefore(win[j], sp, j, x[u], x0[u], x1[u]);
                    if (before) c[u] = p;
                }
            }
        }
        SPROF_T(pd);
        SPROF_ADD(2, pc, pd);
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            if (!live[u]) continue;
            const uint64_t i = base + (uint64_t)(u0 + u) * SB_THREADS + threadIdx.x;
            const uint64_t b = g[u] + c[u];
            const uint64_t slot = (D & 4) ? (i & 0xFFF) : atomicAdd(cnt + b, 1ull);
            bs[i] = (b << 32) | slot;
        }
#if SKV_SORT_PROF
        __builtin_amdgcn_s_waitcnt(0);
#endif
        SPROF_T(pe);
        SPROF_ADD(3, pd, pe);
    }
}

// ---------------------------------------------------------------------------------------------
// Two-pass bucketing (depth 0 at config-5 sizes). The one-pass search above spends its time in the
// group level's dependent probes of a global table and in one memory-side returning atomic per
// element (SKV_SB_DIAGK: 4.1 and 3.1 ms of 8 at 87 M elements). Two passes keep both in LDS:
//   A  the LDS level only: super-bucket a (group a's range of top buckets), a workgroup-local LDS
//      count per super-bucket and one global atomic per (workgroup, super-bucket); the scatter
//      then moves each element to its super-bucket with its window from the super-bucket's common
//      prefix cp[a] (records read in record order)
//   B  per chunk of the super-bucket order: the chunk's groups' 16-byte windows from cp[a] in LDS,
//      the group search there (a tie reads the two records), LDS counts per bucket and one global
//      atomic per (chunk, bucket); the second scatter then forms the buckets.
// The bucket sort compares windows from cp[a] (every key of the bucket shares them) and takes its
// 8-byte sort words from the bucket's own prefix L[b] >= cp[a] on (k_sort_tile's ks).
#define SKV_SA_PER 16
#define SKV_SBB_PER 8
constexpr int SA_PER = SKV_SA_PER;    // pass A: elements per thread (workgroup slots < 2^14)
constexpr int SBB_PER = SKV_SBB_PER;  // pass B: elements per thread (workgroup slots < 2^13)
static_assert(SA_PER * SB_THREADS <= (1 << 14) && SBB_PER * SB_THREADS <= (1 << 13), "slot bits");
constexpr uint32_t SBB_LW = 1024;     // pass B: group windows in LDS (16 KB), also its bucket bins
constexpr uint32_t SBB_GMAX = 16;     // pass B: groups a chunk may span on the LDS path

struct SplitLayout {
    SSplit* sp;
    SWin* win;
    uint64_t* disc;
    uint32_t* gcp;
    ulong2* gw;
};
static SplitLayout split_layout(void* split_buf, uint64_t nsp) {
    SplitLayout l;
    l.sp = (SSplit*)split_buf;
    l.win = (SWin*)(l.sp + nsp + 1);
    l.disc = (uint64_t*)(l.win + nsp + 1);
    l.gcp = (uint32_t*)(l.disc + nsp + 1);
    l.gw = (ulong2*)(((uintptr_t)(l.gcp + nsp + 2) + 15) & ~(uintptr_t)15);
    return l;
}

// top-level entries of the bucket search (SKV_SB_NT caps them below SB_TOP: tests reach the group
// level and the two-pass path at small sizes)
static uint64_t sb_top(uint64_t nsp) {
    const char* e = test_opt("SKV_SB_NT");
    uint64_t cap = e ? strtoull(e, nullptr, 10) : (uint64_t)SB_TOP;
    if (cap == 0 || cap > (uint64_t)SB_TOP) cap = SB_TOP;
    uint64_t top = 1;  // a power of two: the global search level is a full power-of-two search
    while (nsp / top > cap) top <<= 1;
    return top;
}

__global__ void __launch_bounds__(SB_THREADS) k_sort_pass_a(const SElem* __restrict__ E, uint64_t n,
                                                            const SSplit* __restrict__ sp,
                                                            const SWin* __restrict__ win, uint64_t nsp, uint64_t top,
                                                            unsigned long long* scnt, uint64_t* as) {
    __shared__ SWin tt[SB_TOP];
    __shared__ uint32_t hist[SB_TOP + 1];
    const uint32_t nt = (uint32_t)(nsp / top);
    for (uint32_t j = threadIdx.x; j < nt; j += SB_THREADS) tt[j] = win[(uint64_t)(j + 1) * top - 1];
    for (uint32_t j = threadIdx.x; j <= nt; j += SB_THREADS) hist[j] = 0;
    __syncthreads();
    uint32_t s1 = 0;
    if (nt) {
        s1 = 1;
        while (s1 * 2 <= nt) s1 *= 2;
    }
    const uint64_t base = (uint64_t)blockIdx.x * SB_THREADS * SA_PER;
    uint32_t pk[SA_PER];  // super-bucket << 14 | workgroup-local slot
#pragma unroll
    for (int u0 = 0; u0 < SA_PER; u0 += SB_ILP) {
        SElem x[SB_ILP];
        uint64_t x0[SB_ILP], x1[SB_ILP];
        uint32_t a[SB_ILP];
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            const uint64_t i = base + (uint64_t)(u0 + u) * SB_THREADS + threadIdx.x;
            x[u] = E[i < n ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            sk_ext(sk_key(x[u]), x[u].klen, x0[u], x1[u]);
            a[u] = 0;
        }
        for (uint32_t st = s1; st; st >>= 1) {
#pragma unroll
            for (int u = 0; u < SB_ILP; ++u) {
                const uint32_t p = a[u] + st;
                if (p <= nt && sk_sbefore(tt[p - 1], sp, (uint64_t)p * top - 1, x[u], x0[u], x1[u])) a[u] = p;
            }
        }
#pragma unroll
        for (int u = 0; u < SB_ILP; ++u) {
            const uint64_t i = base + (uint64_t)(u0 + u) * SB_THREADS + threadIdx.x;
            pk[u0 + u] = i < n ? (a[u] << 14) | atomicAdd(&hist[a[u]], 1u) : 0u;
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j <= nt; j += SB_THREADS) {
        const uint32_t h = hist[j];
        if (h) hist[j] = (uint32_t)atomicAdd(scnt + j, (unsigned long long)h);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SA_PER; ++u) {
        const uint64_t i = base + (uint64_t)u * SB_THREADS + threadIdx.x;
        if (i < n) {
            const uint32_t a = pk[u] >> 14;
            as[i] = ((uint64_t)a << 32) | (hist[a] + (pk[u] & 0x3FFFu));
        }
    }
}

// splitter s strictly before element x, given equal 16-byte windows from L (the keys share bytes
// [0, L + 16) as far as both reach): the bytes past the window, then the key length
__device__ __noinline__ bool sk_tie_before(const SSplit* __restrict__ s, const SElem& x, uint32_t L) {
    const uint32_t sk = s->klen;
    if (sk > L + 16 && x.klen > L + 16) {
        const uint32_t m = sk < x.klen ? sk : x.klen;
        const int c = bytes_cmp16((const uint8_t*)s->addr + 5 + L + 16, sk_key(x) + L + 16, m - L - 16);
        if (c) return c < 0;
    }
    return sk < x.klen;
}

// bucket count c in group a (the group's windows at w: LDS or global)
template <typename W>
__device__ __forceinline__ void sb_group_search(W w, const SSplit* __restrict__ spa, uint64_t top, uint64_t len,
                                                uint32_t L, const SElem& x, uint64_t& c) {
    c = 0;
    for (uint64_t st = top >> 1; st; st >>= 1) {
        const uint64_t p = c + st;
        if (p <= len) {
            const ulong2 v = w[p - 1];
            const bool before = v.x != x.hi ? v.x < x.hi : (v.y != x.lo ? v.y < x.lo : sk_tie_before(spa + p - 1, x, L));
            if (before) c = p;
        }
    }
}

__global__ void __launch_bounds__(SB_THREADS) k_sort_pass_b(const SElem* __restrict__ T, uint64_t n,
                                                            const uint64_t* __restrict__ sstart,
                                                            const ulong2* __restrict__ gw,
                                                            const SSplit* __restrict__ sp,
                                                            const uint32_t* __restrict__ gcp, uint64_t nsp,
                                                            uint64_t top, uint32_t gmax, unsigned long long* cnt,
                                                            uint64_t* bs) {
    __shared__ ulong2 lw[SBB_LW];
    __shared__ uint32_t hist[SBB_LW];
    __shared__ uint64_t s_st[SBB_GMAX + 1];
    __shared__ uint32_t s_a0, s_ng;
    const uint32_t nt = (uint32_t)(nsp / top);
    const uint64_t p0 = (uint64_t)blockIdx.x * SB_THREADS * SBB_PER;
    if (p0 >= n) return;
    const uint64_t p1 = p0 + (uint64_t)SB_THREADS * SBB_PER < n ? p0 + (uint64_t)SB_THREADS * SBB_PER : n;
    if (threadIdx.x == 0) {  // the chunk's first and last super-buckets (sstart: nt + 2 entries, last = n)
        uint32_t lo = 0, hi = nt + 1;  // largest a with sstart[a] <= p
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (sstart[m] <= p0) lo = m;
            else hi = m;
        }
        const uint32_t a0 = lo;
        hi = nt + 1;
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (sstart[m] <= p1 - 1) lo = m;
            else hi = m;
        }
        s_a0 = a0;
        s_ng = lo - a0 + 1;
    }
    __syncthreads();
    const uint32_t a0 = s_a0, ng = s_ng;
    const bool lds = ng <= gmax && (uint64_t)ng * top <= SBB_LW;  // (uniform; else the global windows)
    if (lds) {
        for (uint32_t k = threadIdx.x; k < ng * top; k += SB_THREADS) {
            const uint64_t j = (uint64_t)a0 * top + k;
            lw[k] = j < nsp ? gw[j] : make_ulong2(0, 0);
            hist[k] = 0;
        }
        for (uint32_t k = threadIdx.x; k <= ng; k += SB_THREADS) s_st[k] = sstart[a0 + k];
        __syncthreads();
    }
    uint32_t pk[SBB_PER];  // bin (bucket - a0 top) << 13 | workgroup-local slot
#pragma unroll
    for (int u = 0; u < SBB_PER; ++u) {
        const uint64_t p = p0 + (uint64_t)u * SB_THREADS + threadIdx.x;
        pk[u] = 0;
        if (p >= p1) continue;
        const SElem x = T[p];
        uint32_t a = a0;
        if (lds) {
            while (a + 1 < a0 + ng && s_st[a + 1 - a0] <= p) ++a;
        } else {
            uint32_t lo = a0, hi = nt + 1;
            while (hi - lo > 1) {
                const uint32_t m = (lo + hi) >> 1;
                if (sstart[m] <= p) lo = m;
                else hi = m;
            }
            a = lo;
        }
        const uint64_t len = a < nt ? top - 1 : nsp - (uint64_t)nt * top;
        uint64_t c;
        if (lds) sb_group_search(lw + (uint64_t)(a - a0) * top, sp + (uint64_t)a * top, top, len, gcp[a], x, c);
        else sb_group_search(gw + (uint64_t)a * top, sp + (uint64_t)a * top, top, len, gcp[a], x, c);
        const uint64_t b = (uint64_t)a * top + c;
        if (lds) {
            const uint32_t bin = (uint32_t)(b - (uint64_t)a0 * top);
            pk[u] = (bin << 13) | atomicAdd(&hist[bin], 1u);
        } else {
            bs[p] = (b << 32) | atomicAdd(cnt + b, 1ull);
        }
    }
    if (!lds) return;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < ng * top; k += SB_THREADS) {
        const uint32_t h = hist[k];
        if (h) hist[k] = (uint32_t)atomicAdd(cnt + (uint64_t)a0 * top + k, (unsigned long long)h);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SBB_PER; ++u) {
        const uint64_t p = p0 + (uint64_t)u * SB_THREADS + threadIdx.x;
        if (p < p1) {
            const uint32_t bin = pk[u] >> 13;
            bs[p] = (((uint64_t)a0 * top + bin) << 32) | (hist[bin] + (pk[u] & 0x1FFFu));
        }
    }
}

// With Lb (depth 0), each element's (hi, lo) is replaced by its 16-byte window from byte Lb[bucket]
// on, read while the record's key line is in cache (elements are in record order): the bucket sort
// then reads no record bytes, where it used to load one window per element from a record at random
// (~250 B of HBM lines per element). (Stored back by the bucket pass instead, the rewrite of E cost
// 1.8 of its 8 ms at config 5, SKV_SB_DIAGK.)
// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs, so each XCD takes a
// contiguous range of blocks. The elements one counting workgroup placed (k_sort_pass_a: 8,192;
// k_sort_pass_b: 4,096) own contiguous slot ranges per (super-)bucket; written from one XCD, those
// ranges' lines are completed in one L2 instead of leaving it as partial lines from eight.
__global__ void k_sort_scatter(const SElem* __restrict__ E, uint64_t n, const uint64_t* __restrict__ bs,
                               const uint64_t* __restrict__ start, const uint32_t* __restrict__ Lb, SElem* out) {
    const uint32_t nb = gridDim.x, bid = blockIdx.x;
    const uint32_t xcd = bid & 7, qn = nb >> 3, rn = nb & 7;
    const uint32_t blk = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
    const uint64_t i = (uint64_t)blk * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t v = bs[i];
    SElem e = E[i];
    if (Lb) {
        const uint32_t L = Lb[v >> 32];
        if (L) {
            uint64_t wh, wl;
            sk_window(e, L, wh, wl);
            e.hi = wh;
            e.lo = wl;
        }
    }
    out[start[v >> 32] + (v & 0xFFFFFFFFull)] = e;
}

// Bucket order: window (wh, wl), then the key bytes past the window when both keys run past it,
// then key length, then record index. Every key of the bucket shares its first L bytes.
struct SKey {
    uint64_t wh, wl;
    uint32_t klen, pos;
};
__device__ __forceinline__ bool sk_wless(const SKey& a, const SKey& b, const SElem* bk, uint32_t ia, uint32_t ib,
                                         uint32_t L) {
    if (a.wh != b.wh) return a.wh < b.wh;
    if (a.wl != b.wl) return a.wl < b.wl;
    if (a.klen > L + 16 && b.klen > L + 16) {
        const uint32_t nmin = a.klen < b.klen ? a.klen : b.klen;
        const int s = bytes_cmp16(sk_key(bk[ia]) + L + 16, sk_key(bk[ib]) + L + 16, nmin - L - 16);
        if (s) return s < 0;
    }
    if (a.klen != b.klen) return a.klen < b.klen;
    return a.pos < b.pos;
}

// One workgroup per bucket: in[start[b], start[b+1]) sorted into out[...]. Bitonic network in
// the ascending-comparator form (the second element of the first step of each merge is mirrored),
// so padding past n acts as +inf and is never touched.
// pre: the elements' (hi, lo) already hold their windows from byte L on (k_sort_scatter with Lb).
__device__ __forceinline__ SKey sk_skey(const SElem& e, uint32_t L, bool pre) {
    SKey k;
    if (pre) {
        k.wh = e.hi;
        k.wl = e.lo;
    } else {
        sk_window(e, L, k.wh, k.wl);
    }
    k.klen = e.klen;
    k.pos = e.pos;
    return k;
}
// equal keys, given equal first L bytes (the bucket's common prefix)
__device__ __forceinline__ bool sk_wsame(const SKey& a, const SKey& c, const SElem& ea, const SElem& ec, uint32_t L) {
    if (a.wh != c.wh || a.wl != c.wl || a.klen != c.klen) return false;
    return c.klen <= L + 16 || bytes_cmp16(sk_key(ea) + L + 16, sk_key(ec) + L + 16, c.klen - L - 16) == 0;
}

// The bucket sorted in global memory, in place (bitonic on the full order), then copied out:
// buckets above SORT_CAP, and LDS sorts that found a long run of equal first words.
__device__ void sk_sort_global(SElem* bk, uint64_t n, uint32_t L, bool pre, SElem* out, uint64_t s0,
                               uint64_t* newkey, const SSplit* spb) {
    uint64_t P = 1;
    while (P < n) P <<= 1;
    for (uint64_t kk = 2; kk <= P; kk <<= 1) {
        for (uint64_t jj = kk >> 1; jj >= 1; jj >>= 1) {
            for (uint64_t i = threadIdx.x; i < P / 2; i += blockDim.x) {
                const uint64_t blk = i / jj, off = i % jj;
                const bool first = jj == (kk >> 1);
                const uint64_t a = first ? blk * kk + off : blk * 2 * jj + off;
                const uint64_t c = first ? blk * kk + kk - 1 - off : a + jj;
                bool sw = false;
                if (c < n) {
                    if (pre) {
                        const SKey kc = sk_skey(bk[c], L, true), ka = sk_skey(bk[a], L, true);
                        sw = sk_wless(kc, ka, bk, (uint32_t)c, (uint32_t)a, L);
                    } else {
                        sw = sk_less(bk[c], bk[a]);
                    }
                }
                if (sw) {
                    const SElem t = bk[a];
                    bk[a] = bk[c];
                    bk[c] = t;
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
    const uint64_t shi = spb ? spb->hi : 0, slo = spb ? spb->lo : 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        SElem o = bk[i];
        if (pre && spb) sk_restore(o, L, shi, slo);
        out[s0 + i] = o;
        if (newkey) {
            bool nk = i == 0;
            if (!nk && pre) nk = !sk_wsame(sk_skey(bk[i - 1], L, true), sk_skey(bk[i], L, true), bk[i - 1], bk[i], L);
            else if (!nk) nk = sk_kcmp(bk[i - 1], bk[i]) != 0;
            newkey[s0 + i] = nk ? 1 : 0;
        }
    }
}

// full bucket order of elements x and y (indices into the bucket)
__device__ __forceinline__ bool sk_eless(const SElem* bk, uint32_t x, uint32_t y, uint32_t L, bool pre) {
    return sk_wless(sk_skey(bk[x], L, pre), sk_skey(bk[y], L, pre), bk, x, y, L);
}

#define SKV_SORT_TIE_MAX 8
constexpr uint32_t SORT_TIE_MAX = SKV_SORT_TIE_MAX;  // longest run of equal first words sorted by one thread

// One compare-exchange of the network on packed sort words: the first word's top 53 bits and the
// element id (11 bits) in one 64-bit value, so a pair moves with one 64-bit shuffle and compares
// once (ids are distinct; padding is ~0). The lower index keeps the smaller word.
__device__ __forceinline__ void sk_cx(uint64_t& k, uint64_t pk, bool lower) {
    const bool take = lower ? pk < k : pk > k;
    k = take ? pk : k;
}
constexpr uint64_t SK_ID_MASK = 0x7FFull;  // SORT_CAP = 2048 ids
// The bitonic network of k_sort_tile on P = 256 EPT elements held in registers: element
// e = w * 64 EPT + u * 64 + l (wave w, register u, lane l). A pair inside a wave's span is exchanged
// through a lane shuffle or between two registers of one lane; a pair across waves through LDS
// (xk; 3 of the 55 stages at P = 1024). The stages are template instances (LK = log2 of the merge
// block, LJ = log2 of the pair distance), so every register index is a compile-time constant.
template <int EPT, int LK, int LJ>
__device__ __forceinline__ void sk_stage(uint64_t (&k)[EPT], uint64_t* xk) {
    constexpr bool flip = LJ == LK - 1;
    constexpr uint32_t B = 1u << LK, jj = 1u << LJ, WSPAN = 64 * EPT;
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    if constexpr (flip ? B <= 64 : jj < 64) {  // partner lane l ^ mask, same register
        constexpr uint32_t mask = flip ? B - 1 : jj;
        const bool lower = (l & (flip ? (B >> 1) : jj)) == 0;
#pragma unroll
        for (int u = 0; u < EPT; ++u) sk_cx(k[u], __shfl_xor(k[u], (int)mask, 64), lower);
    } else if constexpr (!flip && jj < WSPAN) {  // same lane, register u ^ jj / 64
        constexpr int jm = (int)(jj >> 6);
#pragma unroll
        for (int u = 0; u < EPT; ++u) {
            if ((u & jm) == 0) {
                const int v = u | jm;
                const uint64_t lo = k[u] < k[v] ? k[u] : k[v], hi = k[u] < k[v] ? k[v] : k[u];
                k[u] = lo;
                k[v] = hi;
            }
        }
    } else if constexpr (flip && B <= WSPAN) {  // mirror inside the wave: lane l ^ 63, register u ^ (B / 64 - 1)
        constexpr int mm = (int)(B >> 6) - 1;
        uint64_t pk[EPT];
#pragma unroll
        for (int u = 0; u < EPT; ++u) pk[u] = __shfl_xor(k[u ^ mm], 63, 64);
#pragma unroll
        for (int u = 0; u < EPT; ++u) sk_cx(k[u], pk[u], (u & (int)(B >> 7)) == 0);
    } else {  // across waves, through LDS
#pragma unroll
        for (int u = 0; u < EPT; ++u) xk[w * WSPAN + (uint32_t)u * 64 + l] = k[u];
        __syncthreads();
        uint64_t pk[EPT];
#pragma unroll
        for (int u = 0; u < EPT; ++u) {
            const uint32_t e = w * WSPAN + (uint32_t)u * 64 + l, p = flip ? (e ^ (B - 1)) : (e ^ jj);
            pk[u] = xk[p];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < EPT; ++u) {
            const uint32_t e = w * WSPAN + (uint32_t)u * 64 + l, p = flip ? (e ^ (B - 1)) : (e ^ jj);
            sk_cx(k[u], pk[u], e < p);
        }
    }
}
template <int EPT, int LK, int LJ>
__device__ __forceinline__ void sk_bitonic_regs(uint64_t (&k)[EPT], uint64_t* xk) {
    constexpr int LP = EPT == 1 ? 8 : (EPT == 2 ? 9 : (EPT == 4 ? 10 : 11));  // log2(256 EPT)
    if constexpr (LK <= LP) {
        if constexpr (LJ >= 0) {
            sk_stage<EPT, LK, LJ>(k, xk);
            sk_bitonic_regs<EPT, LK, LJ - 1>(k, xk);
        } else {
            sk_bitonic_regs<EPT, LK + 1, LK>(k, xk);
        }
    }
}
// load the bucket's first words into registers (padding past n), sort, store them by position
// the bitonic network's 8-byte sort word: the window's first 8 bytes past the ks bytes every key of
// the bucket shares beyond L (two-pass windows start at the super-bucket's prefix L <= L[b]). Past
// 4 shared bytes the word is read from the record instead: a super-bucket that straddles two
// tables' keys ("17." / "18.") has L = 1 while its buckets share 20+ bytes, and a word of shared
// bytes would send every such bucket to the global-memory sort.
__device__ __forceinline__ uint64_t sk_kw(const SElem& e, uint32_t L, bool pre, uint32_t ks) {
    if (ks > 4) {
        uint64_t wh, wl;
        sk_window(e, L + ks, wh, wl);
        return wh;
    }
    const SKey k = sk_skey(e, L, pre);
    const uint32_t sh = 8 * ks;
    return sh ? (k.wh << sh) | (k.wl >> (64 - sh)) : k.wh;
}

template <int EPT>
__device__ void sk_sort_regs(const SElem* bk, uint32_t n, uint32_t L, bool pre, uint32_t ks, uint64_t* kw,
                             uint16_t* id, uint64_t* kwid) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t k[EPT];  // the sort word's top 53 bits | element id (runs of equal 53-bit words go to
                      // the tie pass like runs of equal words did)
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const uint32_t e = w * 64 * EPT + (uint32_t)u * 64 + l;
        k[u] = ~0ull;
        if (e < n) {
            const uint64_t w = sk_kw(bk[e], L, pre, ks);
            kwid[e] = w;  // the full word by element id: the tie pass orders equal 53-bit words by it
            k[u] = (w & ~SK_ID_MASK) | e;
        }
    }
    sk_bitonic_regs<EPT, 1, 0>(k, kw);
    __syncthreads();  // (the last cross-wave stage's reads of kw are done)
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const uint32_t e = w * 64 * EPT + (uint32_t)u * 64 + l;
        if (e < n) {
            kw[e] = k[u] & ~SK_ID_MASK;
            id[e] = (uint16_t)(k[u] & SK_ID_MASK);
        }
    }
}


// One workgroup per bucket: in[start[b], start[b+1]) sorted into out[...]. The bitonic network
// runs on the first 8 window bytes (kw) and the element ids only, 10 bytes per element where the
// full window, length and index took 26: the sort is bound by LDS traffic. Runs of equal kw are
// then put in the full order (window, bytes past it, key length, record index) by the thread
// holding the run's first position (insertion sort, elements read from the bucket in HBM/L2); a
// run longer than SORT_TIE_MAX sends the bucket to the global-memory sort instead.
// The network is the ascending-comparator form (the second element of the first step of each
// merge is mirrored), so padding past n acts as +inf and is never touched.
__global__ void __launch_bounds__(SORT_THREADS) k_sort_tile(SElem* __restrict__ in, const uint64_t* __restrict__ start,
                                                            const uint32_t* __restrict__ Lb, uint64_t Tb,
                                                            SElem* __restrict__ out, uint64_t* __restrict__ newkey,
                                                            bool pre,
                                                            const SSplit* __restrict__ sp,
                                                            const uint32_t* __restrict__ Lsup, uint64_t top) {
    __shared__ uint64_t kw[SORT_CAP];
    __shared__ uint16_t id[SORT_CAP];
    // full 64-bit sort word by element id: runs of equal 53-bit words (ASCII keys: the dropped low
    // bits carry most of a byte's information -- ~5 runs per config-5 bucket) are ordered on it in
    // LDS, and only equal full words read the elements
    __shared__ uint64_t kwid[SORT_CAP];
    __shared__ uint32_t s_long;
    const uint64_t b = blockIdx.x;
    if (b >= Tb) return;
    const uint64_t s0 = start[b], n = start[b + 1] - s0;
    // L: where the elements' windows start (Lsup: the two-pass super-bucket's prefix, else the
    // bucket's own); ks: bytes past L that every key of the bucket shares (sort words skip them)
    const uint32_t Lt = Lb ? Lb[b] : 0u;
    const uint32_t L = Lsup ? Lsup[b / top] : Lt;
    const uint32_t ks = Lt > L ? Lt - L : 0u;
#if SKV_SORT_PROF
    if (threadIdx.x == 0 && ks > 4 && start[b + 1] > start[b]) atomicAdd(&g_sort_prof[11], 1ull);
    if (threadIdx.x == 0 && start[b + 1] - start[b] > (uint64_t)SORT_CAP) atomicAdd(&g_sort_prof[12], 1ull);
#endif
    SElem* bk = in + s0;
    // sp (the records' level, pre): the output elements get their keys' true prefixes back (the WAL
    // stage reads table ids from them). L > 0 only between two splitters: splitter b bounds bucket b.
    const SSplit* spb = sp && L ? sp + b : nullptr;
    if (n == 0) return;
    const uint64_t shi = spb ? spb->hi : 0, slo = spb ? spb->lo : 0;
    if (n > (uint64_t)SORT_CAP) {
        sk_sort_global(bk, n, L, pre, out, s0, newkey, spb);
        return;
    }
    const uint32_t n32 = (uint32_t)n;
    SPROF_T(q0);
    if (threadIdx.x == 0) s_long = 0;
    static_assert(SORT_THREADS == 256 && SORT_CAP == 2048, "register network: 256 threads, <= 8 elements each");
    if (n32 <= 256) sk_sort_regs<1>(bk, n32, L, pre, ks, kw, id, kwid);
    else if (n32 <= 512) sk_sort_regs<2>(bk, n32, L, pre, ks, kw, id, kwid);
    else if (n32 <= 1024) sk_sort_regs<4>(bk, n32, L, pre, ks, kw, id, kwid);
    else sk_sort_regs<8>(bk, n32, L, pre, ks, kw, id, kwid);
    __syncthreads();
    SPROF_T(q1);
    SPROF_ADD(4, q0, q1);
    SPROF_T(q2);
    SPROF_ADD(5, q1, q2);
    // runs of equal kw into the full order
    for (uint32_t i = threadIdx.x; i < n32; i += blockDim.x) {
        const uint64_t w = kw[i];
        if ((i == 0 || kw[i - 1] != w) && i + 1 < n32 && kw[i + 1] == w) {
            uint32_t e = i + 2;
            while (e < n32 && kw[e] == w && e - i <= SORT_TIE_MAX) ++e;
            if (e - i > SORT_TIE_MAX) {
#if SKV_SORT_PROF
                atomicAdd(&g_sort_prof[10], 1ull);
#endif
                s_long = 1;
            } else {
#if SKV_SORT_PROF
                atomicAdd(&g_sort_prof[8], 1ull);
                atomicAdd(&g_sort_prof[9], (unsigned long long)(e - i));
#endif
                for (uint32_t t = i + 1; t < e; ++t) {
                    const uint32_t x = id[t];
                    uint32_t j = t;
                    while (j > i) {
                        const uint32_t y = id[j - 1];
                        const uint64_t kx = kwid[x], ky = kwid[y];
                        if (kx != ky ? kx > ky : !sk_eless(bk, x, y, L, pre)) break;
                        id[j] = id[j - 1];
                        --j;
                    }
                    id[j] = (uint16_t)x;
                }
            }
        }
    }
    __syncthreads();
    SPROF_T(q3);
    SPROF_ADD(6, q2, q3);
    if (s_long) {  // uniform: every thread read it after the barrier
        sk_sort_global(bk, n, L, pre, out, s0, newkey, spb);
        return;
    }
    for (uint32_t i = threadIdx.x; i < n32; i += blockDim.x) {
        const uint32_t c = id[i];
        SElem o = bk[c];
        if (pre && spb) sk_restore(o, L, shi, slo);
        out[s0 + i] = o;
        if (newkey) {  // a key differing from its predecessor's (buckets never share a key)
            bool nk = i == 0 || kw[i - 1] != kw[i] || kwid[id[i - 1]] != kwid[id[i]];
            if (!nk) {
                const uint32_t a = id[i - 1];
                nk = !sk_wsame(sk_skey(bk[a], L, pre), sk_skey(bk[c], L, pre), bk[a], bk[c], L);
            }
            newkey[s0 + i] = nk ? 1 : 0;
        }
    }
#if SKV_SORT_PROF
    __syncthreads();
    SPROF_T(q4);
    SPROF_ADD(7, q3, q4);
    if (threadIdx.x == 0) atomicAdd(&g_sort_prof[15], 1ull);
#endif
}

__global__ void k_sort_unload(uint64_t R, const SElem* __restrict__ E, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                              uint32_t* klen) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const SElem e = E[i];
    hi[i] = e.hi;
    lo[i] = e.lo;
    addr[i] = e.addr;
    klen[i] = e.klen;
}
void launch_sort_unload(hipStream_t s, uint64_t R, const SElem* E, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                        uint32_t* klen) {
    if (R) k_sort_unload<<<(unsigned)((R + 255) / 256), 256, 0, s>>>(R, E, hi, lo, addr, klen);
}

// (min, max) pairs of k_sort_store's blocks reduced to SORT_MM_OUT pairs (the split's tile_max
// table: k_chain reads it with one wave)
__global__ void __launch_bounds__(256) k_sort_mm_reduce(const uint32_t* __restrict__ in, uint64_t n, uint32_t* out) {
    __shared__ uint32_t s_mm[2 * (256 / 64)];
    const uint64_t b = blockIdx.x, a0 = b * n / gridDim.x, a1 = (b + 1) * n / gridDim.x;
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    for (uint64_t i = a0 + threadIdx.x; i < a1; i += 256) {
        mn = in[2 * i] < mn ? in[2 * i] : mn;
        mx = in[2 * i + 1] > mx ? in[2 * i + 1] : mx;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t x = __shfl_xor(mn, d, 64), y = __shfl_xor(mx, d, 64);
        mn = x < mn ? x : mn;
        mx = y > mx ? y : mx;
    }
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_mm[2 * w] = mn;
        s_mm[2 * w + 1] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t q = 1; q < 256 / 64; ++q) {
            mn = s_mm[2 * q] < mn ? s_mm[2 * q] : mn;
            mx = s_mm[2 * q + 1] > mx ? s_mm[2 * q + 1] : mx;
        }
        out[2 * b] = mn;
        out[2 * b + 1] = mx;
    }
}
void launch_sort_mm_reduce(hipStream_t s, const uint32_t* in, uint64_t n, uint32_t* out) {
    k_sort_mm_reduce<<<SORT_MM_OUT, 256, 0, s>>>(in, n, out);
}

static inline unsigned sk_blocks(uint64_t n) { return (unsigned)((n + 255) / 256); }
uint64_t sort_store_blocks(uint64_t R) { return sk_blocks(R); }

void launch_sort_load(hipStream_t s, uint64_t R, const uint64_t* hi, const uint64_t* lo, const uint64_t* addr,
                      const uint32_t* klen, SElem* E, bool last_wins) {
    if (R) k_sort_load<<<sk_blocks(R), 256, 0, s>>>(R, hi, lo, addr, klen, E, last_wins);
}
void launch_sort_store(hipStream_t s, uint64_t R, const SElem* E, const uint32_t* meta_in, uint32_t const_meta,
                       const uint64_t* newkey, const uint64_t* newkey_ex, uint64_t* hi, uint64_t* lo, uint64_t* addr,
                       uint32_t* klen, uint32_t* cmp_klen, uint32_t* meta, bool last_wins, SortMerged M) {
    if (R)
        k_sort_store<<<sk_blocks(R), 256, 0, s>>>(R, E, meta_in, const_meta, newkey, newkey_ex, hi, lo, addr, klen,
                                                  cmp_klen, meta, last_wins, M);
}
void launch_sort_sample(hipStream_t s, const SElem* E, uint64_t n, uint64_t Ns, SElem* S) {
    if (Ns) k_sort_sample<<<sk_blocks(Ns), 256, 0, s>>>(E, n, Ns, S);
}
void launch_sort_prefix(hipStream_t s, const SElem* Ss, uint64_t ov, uint64_t Tb, uint32_t* L) {
    if (Tb) k_sort_prefix<<<sk_blocks(Tb), 256, 0, s>>>(Ss, ov, Tb, L);
}
void launch_sort_bucket(hipStream_t s, const SElem* E, uint64_t n, const SElem* Ss, uint64_t ov, uint64_t nsp,
                        void* split_buf, uint64_t* cnt, uint64_t* bs, bool diag) {
    const SplitLayout l = split_layout(split_buf, nsp);
    SSplit* sp = l.sp;
    SWin* win = l.win;
    uint64_t* disc = l.disc;
    uint32_t* gcp = l.gcp;
    const uint64_t top = sb_top(nsp);
    if (nsp) {
        k_sort_splitters<<<sk_blocks(nsp), 256, 0, s>>>(Ss, ov, nsp, sp, win);
        k_sort_disc<<<sk_blocks(nsp), 256, 0, s>>>(Ss, ov, nsp, top, gcp, disc, nullptr);
    }
    const uint64_t per_wg = (uint64_t)SB_THREADS * SB_PER;
    const unsigned nb = (unsigned)((n + per_wg - 1) / per_wg);
    if (n) k_sort_bucket<0><<<nb, SB_THREADS, 0, s>>>(E, n, sp, win, nsp, top, gcp, disc, (unsigned long long*)cnt, bs);
}
size_t sort_split_bytes(uint64_t nsp) {
    return (size_t)(nsp + 1) * (sizeof(SSplit) + sizeof(SWin) + sizeof(uint64_t)) + (size_t)(nsp + 2) * sizeof(uint32_t) +
           16 + (size_t)(nsp + 1) * sizeof(ulong2);  // (the two-pass search's group windows, 16-aligned)
}
void launch_sort_scatter(hipStream_t s, const SElem* E, uint64_t n, const uint64_t* bs, const uint64_t* start,
                         const uint32_t* Lb, SElem* out) {
    if (n) k_sort_scatter<<<sk_blocks(n), 256, 0, s>>>(E, n, bs, start, Lb, out);
}
void launch_sort_tile(hipStream_t s, SElem* in, const uint64_t* start, const uint32_t* L, uint64_t Tb, SElem* out,
                      uint64_t* newkey, bool pre, const void* split_buf, uint64_t two_pass_top) {
    const uint32_t* Lsup = two_pass_top ? split_layout((void*)split_buf, Tb - 1).gcp : nullptr;
    if (Tb)
        k_sort_tile<<<(unsigned)Tb, SORT_THREADS, 0, s>>>(in, start, L, Tb, out, newkey, pre,
                                                         (const SSplit*)split_buf, Lsup, two_pass_top);
}

uint64_t sort_two_pass_top(uint64_t nsp) {
    const char* e = test_opt("SKV_SORT_TWO_PASS");  // 0: the one-pass search always
    if (e && e[0] == '0') return 0;
    const uint64_t top = sb_top(nsp);
    return top >= 4 && top <= SBB_LW ? top : 0;
}
uint64_t sort_two_pass_groups(uint64_t nsp) { return nsp / sb_top(nsp) + 1; }

void launch_sort_pass_a(hipStream_t s, const SElem* E, uint64_t n, const SElem* Ss, uint64_t ov, uint64_t nsp,
                        void* split_buf, uint64_t* scnt, uint64_t* as) {
    const SplitLayout l = split_layout(split_buf, nsp);
    const uint64_t top = sb_top(nsp);
    if (nsp) {
        k_sort_splitters<<<sk_blocks(nsp), 256, 0, s>>>(Ss, ov, nsp, l.sp, l.win);
        k_sort_disc<<<sk_blocks(nsp), 256, 0, s>>>(Ss, ov, nsp, top, l.gcp, l.disc, l.gw);
    }
    const uint64_t per_wg = (uint64_t)SB_THREADS * SA_PER;
    if (n)
        k_sort_pass_a<<<(unsigned)((n + per_wg - 1) / per_wg), SB_THREADS, 0, s>>>(E, n, l.sp, l.win, nsp, top,
                                                                                (unsigned long long*)scnt, as);
}
const uint32_t* sort_super_prefix(const void* split_buf, uint64_t nsp) {
    return split_layout((void*)split_buf, nsp).gcp;
}
void launch_sort_pass_b(hipStream_t s, const SElem* T, uint64_t n, const uint64_t* sstart, uint64_t nsp,
                        const void* split_buf, uint64_t* cnt, uint64_t* bs) {
    const SplitLayout l = split_layout((void*)split_buf, nsp);
    const uint64_t per_wg = (uint64_t)SB_THREADS * SBB_PER;
    const char* e = test_opt("SKV_SB_GMAX");  // groups a chunk may span on the LDS path (tests: 0)
    const uint32_t gmax = e ? (uint32_t)std::min<unsigned long>(strtoul(e, nullptr, 10), SBB_GMAX) : SBB_GMAX;
    if (n)
        k_sort_pass_b<<<(unsigned)((n + per_wg - 1) / per_wg), SB_THREADS, 0, s>>>(
            T, n, sstart, l.gw, l.sp, l.gcp, nsp, sb_top(nsp), gmax, (unsigned long long*)cnt, bs);
}

}  // namespace skv
