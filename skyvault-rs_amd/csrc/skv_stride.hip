// skv_stride.hip — the fused stride path of the compaction (gfx950).
//
// When every input record is a Put of one size S whose key has one length K <= 16 (the shape
// of BASELINE configs 1, 2 and 4), everything between the run bytes and the output bytes is
// arithmetic except the merge itself:
//   - record i of a run sits at run + 1 + i * S, so no parse pass writes record arrays: the
//     merge tiles read the 16-byte keys straight from the run bytes and verify each record
//     exactly as runs::read_run_stream would decode it (runs.rs:559-626);
//   - every survivor has size S, so build_runs' greedy split (runs.rs:211-238) closes a run
//     after n = (max - 1) / S records and survivor g lands at (g / n) * (n S + 1) + 1 + (g % n) S;
//   - hence a tile that knows its first survivor's global index (decoupled look-back) writes its
//     output bytes itself: one kernel reads every input byte once and writes every output byte
//     once, and the LDS-bound merge of one tile overlaps the HBM-bound copy of another.
// Kernels:
//   k_fx_sample  level-1 splitter samples read from the runs (+ per-stream sample order check)
//   k_fx_bounds  level-0 tile bounds: per (tile, stream) lower_bound over the run bytes
//   k_fx_tile    verify + in-stream order check + k_way::merge (k_way.rs:113-179: key asc,
//                seq_no desc, first per key) + look-back + output bytes
//   k_fx_desc    output run descriptors and StatsV1 (runs.rs:102-109, :221-228, :271-280)
// A record that is not what the run's first record promised, a key decrease inside a stream or
// a splitter tile above FX_CAP sets the poison flag; the host then discards the result and
// reruns the call on the general path, which reproduces the reference's exact outcome.
#include "skv_launch.hpp"

#include <map>
#include <mutex>

namespace skv {

static_assert(FX_HSLOTS >= 2 * FX_CAP && FX_CAP < 65535, "distinct-key set: 16-bit slots at <= 1/2 load");
static_assert((FX_HSLOTS & (FX_HSLOTS - 1)) == 0, "distinct-key set: probes wrap with & (FX_HSLOTS - 1)");
// The early survivor count takes (hi, lo) = the first 16 key bytes as the whole key: true only while
// the fused path admits keys of at most 16 bytes (and Puts only; the host's fused gate).
static_assert(FX_MAX_K <= 16, "fused keys must fit the 16-byte (hi, lo) compare key");

typedef unsigned int fx_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void fx_store16(uint8_t* p, uint4 v) {
    fx_u32x4 vv = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(vv, (fx_u32x4*)p);  // written once, never re-read here
}

// q = z / d, r = z % d from a double reciprocal and one correction step (z < 2^52)
__device__ __forceinline__ uint64_t fx_divmod(uint64_t z, uint64_t d, double inv, uint64_t& r) {
    uint64_t q = (uint64_t)((double)z * inv);
    int64_t rem = (int64_t)(z - q * d);
    if (rem < 0) {
        --q;
        rem += (int64_t)d;
    } else if ((uint64_t)rem >= d) {
        ++q;
        rem -= (int64_t)d;
    }
    r = (uint64_t)rem;
    return q;
}

template <typename T>
__device__ __forceinline__ T fx_wave_incl(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// exclusive block scan; ws >= 16 entries of LDS
template <typename T>
__device__ T fx_block_excl(T v, T* ws, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = fx_wave_incl(v);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        T w = lane < nw ? ws[lane] : (T)0;
        w = fx_wave_incl(w);
        if (lane < nw) ws[lane] = w;
    }
    __syncthreads();
    T off = wid ? ws[wid - 1] : (T)0;
    total = ws[nw - 1];
    __syncthreads();
    return off + inc - v;
}

// last s in [0, m) with cb[s] <= i
__device__ __forceinline__ uint32_t fx_seg(const uint32_t* cb, uint32_t m, uint32_t i) {
    uint32_t lo = 0, hi = m;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (cb[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

// address of record `pos` (rank-order record index) of stream j
__device__ __forceinline__ uint64_t fx_addr(const FxArgs& A, uint32_t j, uint64_t pos) {
    uint32_t lo = A.stream_run[j], hi = A.stream_run[j + 1];
    while (hi - lo > 1) {  // member runs of an L0-style concatenated stream
        uint32_t mid = (lo + hi) >> 1;
        if (A.run_recb[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return A.runs[lo].ptr + 1 + (pos - A.run_recb[lo]) * A.S;
}

// Loads through the global address space (an integer address would otherwise become a flat
// access, which also counts against lgkmcnt and so serialises with every LDS wait).
typedef unsigned int fx_v4 __attribute__((ext_vector_type(4)));
typedef unsigned int fx_v2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) fx_v4 fx_g16;
typedef const __attribute__((address_space(1))) fx_v2 fx_g8;
typedef const __attribute__((address_space(1))) uint32_t fx_g4;
__device__ __forceinline__ uint4 fx_ld16(uint64_t a) {  // unaligned: full rate on gfx950
    const fx_v4 v = *(fx_g16*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint4 fx_cld16(uint64_t a) { return fx_ld16(a); }  // the copy's loads

// One record's header pieces: marker + key_len (bytes 0..7), the 16 bytes from the key start,
// val_len (at 5 + K). All inside the record (S >= 32), issued as three independent loads.
struct FxRec {
    uint2 h;
    uint4 k;
    uint32_t v;
};
__device__ __forceinline__ void fx_issue(uint64_t a, uint32_t K, FxRec& r) {
    const fx_v2 h = *(fx_g8*)a;
    r.h = make_uint2(h.x, h.y);
    r.k = fx_ld16(a + 5);
    r.v = *(fx_g4*)(a + 5 + K);
}

// The record at a, decoded as read_run_stream does (runs.rs:559-626): marker 1 (Put), key_len
// == K, UTF-8 key (runs.rs:585-591), val_len == V, so its size is S. Returns false otherwise.
// Key -> (hi, lo) big-endian, zero padded past K.
__device__ __forceinline__ bool fx_check(const FxArgs& A, const FxRec& r, uint64_t a, uint64_t& hi, uint64_t& lo) {
    const uint32_t marker = r.h.x & 0xFFu;
    const uint32_t klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(r.h.y, r.h.x, 1));
    const uint32_t vlen = __builtin_bswap32(r.v);
    const uint32_t d0 = r.k.x & dword_mask(0, A.K, 0), d1 = r.k.y & dword_mask(0, A.K, 1);
    const uint32_t d2 = r.k.z & dword_mask(0, A.K, 2), d3 = r.k.w & dword_mask(0, A.K, 3);
    hi = ((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1);
    lo = ((uint64_t)__builtin_bswap32(d2) << 32) | __builtin_bswap32(d3);
    bool ok = marker == 1u && klen == A.K && vlen == A.V;
    if (ok && ((d0 | d1 | d2 | d3) & 0x80808080u)) ok = utf8_valid((const uint8_t*)a + 5, A.K);
    return ok;
}

__device__ __forceinline__ bool fx_key(const FxArgs& A, uint64_t a, uint64_t& hi, uint64_t& lo) {
    FxRec r;
    fx_issue(a, A.K, r);
    return fx_check(A, r, a, hi, lo);
}

__device__ __forceinline__ bool fx_gt(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah > bh || (ah == bh && al > bl);
}

__device__ __forceinline__ void fx_poison(const FxArgs& A, uint32_t why) {
    atomicOr(A.flags + 3, why);
    atomicOr(A.flags + 2, 1u);
}

// ---------------------------------------------------------------------------------------------
// splitters

// level-1 samples: every Sstep-th record of each stream, c = K << 32 | pos (the element form of
// k_tile<false>). Samples out of order inside a stream poison the call before any sample tile
// merges them (a merge of unsorted lists is not a permutation).
__global__ void k_fx_sample(FxArgs A, const uint64_t* __restrict__ off_dst, uint64_t Sstep, uint64_t n_dst,
                            uint64_t* dhi, uint64_t* dlo, uint64_t* dc, FxUpLevels up) {
    extern __shared__ uint64_t fx_offs[];  // off_dst[0..k], staged once per workgroup
    for (uint32_t x = threadIdx.x; x <= A.k; x += blockDim.x) fx_offs[x] = off_dst[x];
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = i < n_dst;
    uint32_t lo = 0, hi = A.k;
    while (act && hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (fx_offs[mid] <= i) lo = mid;
        else hi = mid;
    }
    const uint64_t pos = A.stream_base[lo] + (i - fx_offs[lo]) * Sstep;
    uint64_t h = 0, l = 0;
    if (act) {
        fx_key(A, fx_addr(A, lo, pos), h, l);
        dhi[i] = h;
        dlo[i] = l;
        dc[i] = ((uint64_t)A.K << 32) | pos;
        uint64_t c = i - fx_offs[lo];  // this stream's sample index at level 1, then 2
        for (uint32_t u = 0; u < up.n && c % Sstep == 0; ++u) {
            c /= Sstep;
            const uint64_t q = up.off[u][lo] + c;
            up.hi[u][q] = h;
            up.lo[u][q] = l;
            up.c[u][q] = ((uint64_t)A.K << 32) | pos;
        }
    }
    // per-stream sample order: sample i-1 of the same stream is the previous lane's key (one load
    // per sample; the first lane of each wave loads its predecessor itself)
    uint64_t ph = __shfl_up(h, 1, 64), pl = __shfl_up(l, 1, 64);
    if (act && i > fx_offs[lo]) {
        if ((threadIdx.x & 63) == 0) fx_key(A, fx_addr(A, lo, pos - Sstep), ph, pl);
        if (fx_gt(ph, pl, h, l)) fx_poison(A, FXR_SAMPLE);
    }
}

// sorted level-1 sample index of splitter t, and its inverse (the last splitter at or before
// sorted position p)
__device__ __forceinline__ uint64_t fx_srank(const FxArgs& A, uint64_t t) {
    return t <= A.T1 ? t * A.m : A.T1 * A.m + (t - A.T1) * A.m2;
}
__device__ __forceinline__ uint64_t fx_sinv(const FxArgs& A, uint64_t p) {
    const uint64_t b = A.T1 * A.m;
    return p < b ? p / A.m : A.T1 + (p - b) / A.m2;
}

// member run of stream j holding record pos
__device__ __forceinline__ uint32_t fx_run(const FxArgs& A, uint32_t j, uint64_t pos) {
    uint32_t lo = A.stream_run[j], hi = A.stream_run[j + 1];
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (A.run_recb[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return lo;
}

// first index in [lo, hi) whose element is not below the splitter (or hi), one thread: each round
// issues 8 independent probes and keeps the gap where the predicate flips (9-ary search), so a
// search of n elements costs ~log9(n) dependent round trips instead of log2(n)
template <typename Below>
__device__ __forceinline__ uint64_t fx_lower_bound8(uint64_t lo, uint64_t hi, Below below) {
    while (lo < hi) {
        const uint64_t n = hi - lo;
        uint64_t idx[8];
        bool p[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) idx[i] = n >= 9 ? lo + ((uint64_t)(i + 1) * n) / 9 : lo + (uint64_t)i;
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = idx[i] < hi && below(idx[i]);
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) c += p[i] ? 1u : 0u;
        if (n < 9) return lo + c;
        if (c == 0) {
            hi = idx[0];
        } else {
            uint64_t l2 = idx[0], h2 = hi;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i + 1 == (int)c) l2 = idx[i] + 1;
                if (i == (int)c) h2 = idx[i];
            }
            lo = l2;
            hi = h2;
        }
    }
    return lo;
}

template <bool FULL>
__device__ __forceinline__ FxBound fx_bound(const FxArgs& A, const uint64_t* __restrict__ shi,
                                            const uint64_t* __restrict__ slo, uint64_t m,
                                            const uint64_t* __restrict__ l1hi, const uint64_t* __restrict__ l1lo,
                                            const uint64_t* __restrict__ l1off, uint64_t Sstep, uint64_t t, uint32_t j) {
    const uint64_t s0 = A.stream_base[j], s1 = A.stream_base[j + 1];
    uint64_t a = s0;
    uint64_t pvh = 0, pvl = 0;  // key of record a - 1 when pv
    bool pv = false;
    if (t == A.T) {
        a = s1;
    } else if (t > 0 && s1 > s0) {
        if (__hip_atomic_load(A.flags + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            FxBound o{};
            o.pos = s0;
            return o;
        }
        const uint64_t sr = fx_srank(A, t);
        const uint64_t h = shi[sr], l = slo[sr];
        const uint64_t q0 = l1off[j], q1 = l1off[j + 1];
        uint64_t c;
        if (A.l1cnt) {
            // the samples of stream j sorted before the splitter, minus those equal to it (they
            // sort on either side of it; lower_bound counts only the smaller ones)
            c = A.l1cnt[t * A.k + j];
            while (c > 0 && l1hi[q0 + c - 1] == h && l1lo[q0 + c - 1] == l) --c;
        } else {
            c = fx_lower_bound8(q0, q1, [&](uint64_t i) {
                    const uint64_t eh = l1hi[i], el = l1lo[i];
                    return eh < h || (eh == h && el < l);
                }) - q0;
        }
        if (c > 0) {
            // record lo - 1 is stream j's sample c - 1: its key is the previous key until the
            // search moves past it (then the last probe below the splitter is)
            pvh = l1hi[q0 + c - 1];
            pvl = l1lo[q0 + c - 1];
            pv = true;
            const uint64_t lo = s0 + (c - 1) * Sstep + 1;
            const uint64_t hi = s0 + c * Sstep < s1 ? s0 + c * Sstep : s1;
            const uint32_t r0 = A.stream_run[j];
            const bool one_run = A.stream_run[j + 1] - r0 == 1;
            const uint64_t base = A.runs[r0].ptr + 1 - A.run_recb[r0] * A.S;  // record pos -> address (one run)
            // inside the gap (< Sstep records, each probe a random HBM line). First round: the two
            // records around the position interpolated from the gap's end keys (sample c - 1 below
            // the splitter, sample c at or above it), issued together; for keys spread evenly
            // inside a gap that brackets the bound at once. Then a plain binary search over what
            // is left, one line per round. Every probe below the splitter moves a past it and
            // carries its key as the previous record's, so that key stays exact on any input.
            auto probe = [&](uint64_t i) {
                const uint64_t ad = one_run ? base + i * A.S : fx_addr(A, j, i);
                return fx_ld16(ad + 5);
            };
            auto key_of = [&](const uint4& kk, uint64_t& eh, uint64_t& el) {
                eh = ((uint64_t)__builtin_bswap32(kk.x & dword_mask(0, A.K, 0)) << 32) |
                     __builtin_bswap32(kk.y & dword_mask(0, A.K, 1));
                el = ((uint64_t)__builtin_bswap32(kk.z & dword_mask(0, A.K, 2)) << 32) |
                     __builtin_bswap32(kk.w & dword_mask(0, A.K, 3));
            };
            uint64_t b2 = hi;
            a = lo;
            while (a < b2) {
                const uint64_t i = (a + b2) >> 1;
                uint64_t eh, el;
                key_of(probe(i), eh, el);
                if (eh < h || (eh == h && el < l)) {
                    a = i + 1;
                    pvh = eh;
                    pvl = el;
                } else {
                    b2 = i;
                }
            }
        }
    }
    FxBound o{};
    o.pos = a;
    if (!FULL) return o;
    if (a < s1) {
        const uint32_t r = fx_run(A, j, a);
        o.addr = A.runs[r].ptr + 1 + (a - A.run_recb[r]) * A.S;
        o.rem = A.run_recb[r + 1] - a;
    }
    if (a > s0 && t < A.T) {
        o.has_prev = 1;
        if (pv) {
            o.ph = pvh;
            o.pl = pvl;
        } else {
            fx_key(A, fx_addr(A, j, a - 1), o.ph, o.pl);
        }
    }
    return o;
}

// Level-1 sample counts per (splitter, stream) from the sorted samples' positions: sorted sample
// p is stream j's c-th sample (record pos = the low half of sc[p]); posof[l1off[j] + c] = p.
__global__ void k_fx_posof(FxArgs A, const uint64_t* __restrict__ sc, uint64_t N1, uint32_t* posof) {
    extern __shared__ uint64_t fx_tab[];  // stream_base[0..k] | l1off[0..k]
    for (uint32_t x = threadIdx.x; x <= A.k; x += blockDim.x) {
        fx_tab[x] = A.stream_base[x];
        fx_tab[A.k + 1 + x] = A.l1off[x];
    }
    __syncthreads();
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N1) return;
    const uint64_t pos = sc[p] & 0xFFFFFFFFull;
    uint32_t lo = 0, hi = A.k;  // stream j: stream_base[j] <= pos < stream_base[j + 1]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fx_tab[mid] <= pos) lo = mid;
        else hi = mid;
    }
    const uint64_t q = fx_tab[A.k + 1 + lo] + (pos - fx_tab[lo]) / A.Sstep;
    if (q < fx_tab[A.k + 2 + lo]) posof[q] = (uint32_t)p;
}
// cnt[t*k + j] = stream j's samples at sorted positions < t*m (splitter t is sample t*m): sample c
// at position p, next one at pn, is the last one before splitters t with p < t*m <= pn; every
// (t, j) with t in [1, T) is written exactly once (c = 0 also covers the splitters before it).
__global__ void k_fx_l1cnt(FxArgs A, const uint32_t* __restrict__ posof, uint64_t N1, uint32_t* cnt) {
    extern __shared__ uint64_t fx_l1o[];  // l1off[0..k]
    for (uint32_t x = threadIdx.x; x <= A.k; x += blockDim.x) fx_l1o[x] = A.l1off[x];
    __syncthreads();
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= N1) return;
    uint32_t lo = 0, hi = A.k;  // stream j: l1off[j] <= q < l1off[j + 1]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fx_l1o[mid] <= q) lo = mid;
        else hi = mid;
    }
    const uint32_t j = lo, k = A.k;
    const uint64_t c = q - fx_l1o[j], T = A.T;
    const uint64_t p = posof[q];
    const uint64_t tmax = T - 1;
    const uint64_t sp = fx_sinv(A, p);
    const uint64_t t_hi0 = sp < tmax ? sp : tmax;  // splitters at or before p: nothing of j's below
    if (c == 0)
        for (uint64_t t = 1; t <= t_hi0; ++t) cnt[t * k + j] = 0;
    const uint64_t pn = q + 1 < fx_l1o[j + 1] ? posof[q + 1] : ~0ull;
    const uint64_t spn = pn == ~0ull ? tmax : fx_sinv(A, pn);
    const uint64_t t_hi = spn < tmax ? spn : tmax;
    for (uint64_t t = sp + 1; t <= t_hi; ++t) cnt[t * k + j] = (uint32_t)(c + 1);
}

// bnd[t*k + j].pos = first record of stream j whose key >= splitter t (sorted level-1 samples,
// every m-th one), plus what tile t needs to start its segment without further searches: the
// record's address, the records left in its member run, and the key of the record before it
// (the in-stream order check across tile edges, runs.rs:190-198). One thread per (t, j): a 9-ary
// search over stream j's own level-1 samples (every Sstep-th record, L2-resident) narrows the
// bound to one sample gap, then a binary search over the records of that gap.
__global__ void k_fx_bounds(FxArgs A, const uint64_t* __restrict__ shi, const uint64_t* __restrict__ slo, uint64_t m,
                            const uint64_t* __restrict__ l1hi, const uint64_t* __restrict__ l1lo,
                            const uint64_t* __restrict__ l1off, uint64_t Sstep) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = A.k;
    if (g >= (A.T + 1) * k) return;
    const uint64_t t = g / k;
    const uint32_t j = (uint32_t)(g - t * k);
    A.bnd[g] = fx_bound<true>(A, shi, slo, m, l1hi, l1lo, l1off, Sstep, t, j);
}

// ---------------------------------------------------------------------------------------------
// the fused tile

// decoupled look-back over tiles with one wave (64 predecessors per probe), one 62-bit counter
// per tile (flag in bits 62-63: 1 aggregate, 2 inclusive prefix). Tiles take tickets in start
// order, so every predecessor of a waiting tile is resident or done. Called by wave 0.
// published: the tile stored its aggregate already (fx_publish_early)
__device__ __forceinline__ void fx_publish_early(uint64_t* st, uint64_t t, uint64_t agg) {
    constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62;
    __hip_atomic_store(&st[t], (t == 0 ? FI : FA) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ uint64_t fx_lookback(uint64_t* st, uint64_t t, uint64_t agg, bool published = false) {
    constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62, VM = FA - 1;
    const int lane = threadIdx.x & 63;
    if (t == 0) {
        if (lane == 0 && !published) __hip_atomic_store(&st[0], FI | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0 && !published) __hip_atomic_store(&st[t], FA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t acc = 0;
    int64_t top = (int64_t)t - 1;  // window: predecessors top, top-1, ..., top-63
    for (;;) {
        const int64_t p = top - lane;
        const uint64_t v = p >= 0 ? __hip_atomic_load(&st[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FI;
        const uint64_t f = v >> 62;
        const uint64_t incl = __ballot(f == 2), none = __ballot(f == 0);
        const int first = incl ? __builtin_ctzll(incl) : 64;       // nearest inclusive prefix
        const uint64_t upto = first == 64 ? ~0ull : (first == 63 ? ~0ull : ((2ull << first) - 1));
        if (none & upto) {  // a predecessor before it has not published yet
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

// Output bytes [x0, x1) (inside one 16-byte block B) that start at byte o of local survivor j
// (o == -1: the version byte before it; qj = j's index inside its output run). Pieces are taken
// in output order: record tail, version byte of the next run, next record, ...
__device__ uint4 fx_compose(const FxArgs& A, const uint64_t* src, uint64_t B, uint64_t x0, uint64_t x1, uint32_t j,
                            int64_t o, uint64_t qj) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint64_t x = x0;
    while (x < x1) {
        const uint32_t a = (uint32_t)(x - B);
        if (o < 0) {  // version byte (runs.rs:241-246)
            const uint32_t sh = 8 * (a & 3), q = a >> 2;
            if (q == 0) acc.x |= 1u << sh;
            else if (q == 1) acc.y |= 1u << sh;
            else if (q == 2) acc.z |= 1u << sh;
            else acc.w |= 1u << sh;
            ++x;
            o = 0;
            continue;
        }
        const uint64_t m = (A.S - (uint64_t)o) < (x1 - x) ? (A.S - (uint64_t)o) : (x1 - x);
        const uint32_t b = a + (uint32_t)m;
        uint4 w = load_window16((const uint8_t*)src[j] + o, (uint32_t)m);
        w = shl_bytes(w, a);
        acc.x |= w.x & dword_mask(a, b, 0);
        acc.y |= w.y & dword_mask(a, b, 1);
        acc.z |= w.z & dword_mask(a, b, 2);
        acc.w |= w.w & dword_mask(a, b, 3);
        x += m;
        o += (int64_t)m;
        if ((uint64_t)o == A.S) {
            ++j;
            ++qj;
            o = 0;
            if (qj == A.n) {
                qj = 0;
                o = -1;
            }
        }
    }
    return acc;
}

__device__ __forceinline__ void fx_store_bytes(uint8_t* out, uint64_t B, uint64_t x0, uint64_t x1, uint4 v) {
    for (uint64_t y = x0; y < x1; ++y) out[y] = (uint8_t)byte_of(v, (uint32_t)(y - B));
}

// key order with the left (newer seq_no) side winning ties
__device__ __forceinline__ bool fx_le(const ulong2& a, const ulong2& b) {
    return a.x < b.x || (a.x == b.x && a.y <= b.y);
}

__device__ __forceinline__ uint4 fx_vbyte_then(uint4 head) {  // version byte, then 15 record bytes
    uint4 v = shl_bytes(head, 1);
    v.x |= 1u;
    return v;
}

// x / d and x % d for x < 2^31 (double reciprocal, one correction)
__device__ __forceinline__ uint32_t fx_div32(uint32_t x, uint32_t d, double inv, uint32_t& r) {
    uint32_t q = (uint32_t)((double)x * inv);
    int32_t rem = (int32_t)(x - q * d);
    if (rem < 0) {
        --q;
        rem += (int32_t)d;
    } else if ((uint32_t)rem >= d) {
        ++q;
        rem -= (int32_t)d;
    }
    r = (uint32_t)rem;
    return q;
}

// The copy walk of one lane over its output blocks B, B + 16 FX_THREADS, ... of a tile with at
// most one run boundary: (record j, byte o) of the block's first byte, kept incrementally.
struct FxWalk {
    uint64_t B, V0, Vb;
    uint32_t j, o, jb1, S32, dq, dr;
    bool past;
};
template <int U>
struct FxBatch {
    uint64_t aL[U], aX[U];
    uint32_t mode[U], sh[U];  // 0 one record, 1 record tail + next, 2 version byte + record,
                              // 3 record tail + version byte + next
    uint4 L[U], X[U];
    uint32_t b;
};
// addresses of the batch's U blocks (b, b + FX_THREADS, ...) and their loads, issued together.
// No branches where memory is touched: blocks past nb load `safe`, and the second load (X, the
// next record's head) is exec-masked to the lanes whose block straddles a record end (~6 % at
// 281-byte records), so the waitcnt pass sees the same count on every path and can leave later
// batches in flight. Issuing X on every lane (re-reading its own address) cost 9 % of the tile.
template <int U>
__device__ __forceinline__ void fx_plan(FxBatch<U>& t, FxWalk& w, const uint64_t* src, uint32_t b, uint32_t nb,
                                        uint64_t safe) {
    t.b = b;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool valid = b + u * FX_THREADS < nb;
        const bool vb = w.B == w.V0 || w.B == w.Vb;
        const bool st = !vb && w.o + 16 > w.S32;
        uint32_t ja = vb ? (w.B == w.V0 ? 0u : w.jb1) : w.j;
        ja = ja < (uint32_t)(FX_CAP - 1) ? ja : (uint32_t)(FX_CAP - 1);
        const uint64_t s0 = src[ja], s1 = src[ja + 1];
        uint64_t aL = vb ? s0 : s0 + (st ? w.S32 - 16 : w.o);
        uint64_t aX = st ? s1 : aL;  // only a block that straddles a record end needs X
        t.aL[u] = valid ? aL : 0;
        t.aX[u] = valid ? aX : safe;
        if (!valid) aL = aX = safe;
        t.mode[u] = vb ? 2u : (st ? (w.j + 1 == w.jb1 ? 3u : 1u) : 0u);
        t.sh[u] = 16 - (w.S32 - w.o);
        w.B += 16u * FX_THREADS;  // this lane's next block
        w.o += w.dr;
        w.j += w.dq;
        const bool wrap = w.o >= w.S32;
        w.o = wrap ? w.o - w.S32 : w.o;
        w.j = wrap ? w.j + 1 : w.j;
        if (!w.past && w.B > w.Vb) {  // crossed the run boundary: one version byte earlier
            w.past = true;
            const bool z = w.o == 0;
            w.o = z ? w.S32 - 1 : w.o - 1;
            w.j = z ? w.j - 1 : w.j;
        }
        t.L[u] = fx_cld16(aL);
        // the second load only on the lanes that straddle (exec-masked)
        uint4 xv = make_uint4(0, 0, 0, 0);
        if (st && valid) xv = fx_cld16(aX);
        t.X[u] = xv;
    }
}
__device__ __forceinline__ uint4 fx_sel4(bool c, uint4 a, uint4 b) {  // c ? a : b, per dword
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
// funnel16 without the sh == 0 early exit (alignbyte by 0 is the identity): straight-line code
__device__ __forceinline__ uint4 fx_funnel16(uint4 x, uint4 y, uint32_t sh) {
    const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    const uint32_t q = sh >> 2, r = sh & 3;
    uint32_t t[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t v3 = (i + 3 < 8) ? w[i + 3] : 0u;
        t[i] = q == 0 ? w[i] : (q == 1 ? w[i + 1] : (q == 2 ? w[i + 2] : v3));
    }
    return make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                      __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
}
template <int U, bool FULL>
__device__ __forceinline__ void fx_finish(const FxBatch<U>& t, uint8_t* ob) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t m = t.mode[u];
        const uint4 xv = fx_sel4(m == 3, fx_vbyte_then(t.X[u]), t.X[u]);
        const uint4 f = fx_funnel16(t.L[u], xv, t.sh[u] & 15);
        const uint4 v = fx_sel4(m == 2, fx_vbyte_then(t.L[u]), fx_sel4(m != 0, f, t.L[u]));
        if (FULL || t.aL[u]) fx_store16(ob + 16ull * (t.b + u * FX_THREADS), v);
    }
}

#if SKV_TILE_PROF
#define FXPROF(i)                                                                               \
    do {                                                                                        \
        if (threadIdx.x == 0) {                                                                 \
            const uint64_t now_ = __builtin_amdgcn_s_memrealtime();                             \
            atomicAdd((unsigned long long*)&A.prof[i], (unsigned long long)(now_ - tp_last));  \
            tp_last = now_;                                                                     \
        }                                                                                       \
    } while (0)
#else
#define FXPROF(i) do {} while (0)
#endif

// LDS: key[FX_CAP] 16 B (by position; after the merge: source addresses by survivor, u64)
//      | prevk[k] 16 B | segaddr[k] sbase[k] u64 | cb0[k+1] cbA[k+1] cbB[k+1] u32 | id[FX_CAP] u16
//      | prevok[k] u8
__global__ void __launch_bounds__(FX_THREADS) k_fx_tile(FxArgs A) {
    constexpr int PER = FX_CAP / FX_THREADS;
    extern __shared__ __attribute__((aligned(16))) uint64_t fx_smem[];
    const uint32_t k = A.k;
    ulong2* key = (ulong2*)fx_smem;
    ulong2* prevk = key + FX_CAP;
    uint64_t* segaddr = (uint64_t*)(prevk + k);
    uint64_t* sbase = segaddr + k;
    uint32_t* cb0 = (uint32_t*)(sbase + k);
    uint32_t* cbA = cb0 + (k + 1);
    uint32_t* cbB = cbA + (k + 1);
    uint16_t* id = (uint16_t*)(cbB + (k + 1));
    uint8_t* prevok = (uint8_t*)(id + FX_CAP);
    __shared__ uint64_t ws[16];
    __shared__ uint64_t s_t, s_g0;
    __shared__ uint32_t s_dead, s_bad;
    __shared__ uint32_t hs[FX_HSLOTS / 2];  // distinct-key set: 16-bit slots (element + 1), two per word
    __shared__ uint32_t s_early;
    const uint32_t tid = threadIdx.x;
    const uint64_t S = A.S;
    for (uint32_t x = tid; x < FX_HSLOTS / 2; x += FX_THREADS) hs[x] = 0;
#if SKV_TILE_PROF
    uint64_t tp_last = __builtin_amdgcn_s_memrealtime();
#endif
    if (tid == 0) {
        s_t = atomicAdd(A.tcounter, 1u);
        s_dead = __hip_atomic_load(A.flags + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_bad = 0;
    }
    __syncthreads();
    const uint64_t t = s_t;
#if SKV_TILE_PROF
    if (tid == 0) atomicAdd((unsigned long long*)&A.prof[15], 1ull);
#endif
    do {
    // ---- segments: stream j contributes its records [bnd[t][j].pos, bnd[t+1][j].pos)
    uint64_t tot = 0;
    if (!s_dead) {
        for (uint32_t j0 = 0; j0 < k; j0 += FX_THREADS) {
            const uint32_t j = j0 + tid;
            uint64_t len = 0;
            if (j < k) {
                const FxBound b = A.bnd[t * k + j];
                uint64_t b1 = A.bnd[(t + 1) * k + j].pos;
                if (b1 < b.pos) {  // splitters over unsorted input
                    atomicOr(&s_bad, FXR_SPLIT);
                    b1 = b.pos;
                }
                len = b1 - b.pos;
                sbase[j] = b.pos;
                segaddr[j] = len <= b.rem ? b.addr : 0;  // 0: the segment spans member runs
                prevk[j] = make_ulong2(b.ph, b.pl);
                prevok[j] = (uint8_t)b.has_prev;
                if (len > FX_CAP) len = FX_CAP + 1;
            }
            uint64_t part;
            const uint64_t ex = fx_block_excl<uint64_t>(len, ws, part);
            if (j < k) cb0[j] = (uint32_t)(tot + ex < FX_CAP + 1 ? tot + ex : FX_CAP + 1);
            tot += part;
        }
        if (tid == 0) {
            cb0[k] = (uint32_t)(tot < FX_CAP + 1 ? tot : FX_CAP + 1);
            if (tot > FX_CAP) s_bad |= FXR_OVERSIZE;
        }
    }
    __syncthreads();
    FXPROF(0);
    const uint32_t n = (uint32_t)(tot <= FX_CAP ? tot : 0);
    const bool live = !s_dead && !s_bad;
    // ---- load + verify every record of the tile: addresses from LDS, all loads issued first
    uint32_t bad = 0;
    {
        uint64_t ad[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t e = tid + u * FX_THREADS;
            ad[u] = 0;
            if (live && e < n) {
                const uint32_t j = fx_seg(cb0, k + 1, e);
                const uint64_t sa = segaddr[j];
                ad[u] = sa ? sa + (uint64_t)(e - cb0[j]) * S : fx_addr(A, j, sbase[j] + (e - cb0[j]));
            }
        }
        FxRec rec[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u)
            if (ad[u]) fx_issue(ad[u], A.K, rec[u]);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            if (ad[u]) {
                const uint32_t e = tid + u * FX_THREADS;
                uint64_t h = 0, l = 0;
                if (!fx_check(A, rec[u], ad[u], h, l)) bad |= FXR_RECORD;
                key[e] = make_ulong2(h, l);
                id[e] = (uint16_t)e;
            }
        }
    }
    __syncthreads();
    FXPROF(1);
    // ---- order check inside each stream (runs.rs:190-198): against the previous record of the
    // same stream (the previous element of the segment, or the record before the segment).
    // In the same pass, the tile's survivor count before its merge: first-per-key keeps one record
    // per distinct key (k_way.rs:146-151; the fused path holds Puts only, keys <= 16 bytes, so
    // (hi, lo) is the whole key), so the count is the number of distinct keys, found with an LDS
    // hash set (16-bit slots holding element + 1, two per word, claimed by CAS). Published before
    // the merge rounds, successors' look-backs stop waiting on them; the merge's own count is
    // checked against it after the rounds.
    uint32_t distinct = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t e = tid + u * FX_THREADS;
        if (live && e < n) {
            const uint32_t j = fx_seg(cb0, k + 1, e);
            const ulong2 c = key[e];
            bool has = true;
            ulong2 pv;
            if (e > cb0[j]) pv = key[e - 1];
            else {
                pv = prevk[j];
                has = prevok[j] != 0;
            }
            if (has && !fx_le(pv, c)) bad |= FXR_ORDER;  // a strict decrease
            uint32_t h = (uint32_t)((c.x * 0x9E3779B97F4A7C15ull ^ c.y * 0xC2B2AE3D27D4EB4Full) >> 40) & (FX_HSLOTS - 1);
            for (;;) {
                const uint32_t sh = (h & 1u) * 16u;
                const uint32_t w = hs[h >> 1];
                const uint32_t cur = (w >> sh) & 0xFFFFu;
                if (cur == 0) {
                    if (atomicCAS(&hs[h >> 1], w, w | ((e + 1) << sh)) == w) {
                        ++distinct;
                        break;
                    }
                    continue;  // the word changed: look at this slot again
                }
                const ulong2 o = key[cur - 1];
                if (o.x == c.x && o.y == c.y) break;  // a duplicate of a key already in the set
                h = (h + 1) & (FX_HSLOTS - 1);
            }
        }
    }
    if (bad) atomicOr(&s_bad, bad);
    uint32_t tot_d;
    fx_block_excl<uint32_t>(distinct, (uint32_t*)ws, tot_d);  // barriers: s_bad is settled after it
    FXPROF(2);
    if (s_dead || s_bad) {  // publish an empty aggregate so later tiles never wait on this one
        if (tid == 0) {
            if (s_bad) fx_poison(A, s_bad);
            __hip_atomic_store(&A.tstate[t], (t == 0 ? 2ull : 1ull) << 62, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
    }
    if (tid == 0) {
        s_early = tot_d;
        fx_publish_early(A.tstate, t, tot_d);
    }
    // ---- k_way::merge order (k_way.rs:20-27, :113-179): pairwise merge-path rounds over the k
    // stream segments (segment s pairs with s ^ 1, the left one holds newer seq_nos and wins ties,
    // so equal keys end up seq_no-descending, and in stream order within a stream). Each thread
    // produces PER consecutive outputs of a round: one merge-path search, then a sequential merge.
    const uint32_t i0 = tid * PER;
    {
        uint32_t m = k;
        const uint32_t* cb = cb0;
        uint32_t* cbn = cbA;
        while (m > 1) {
            const uint32_t mp = (m + 1) >> 1;
            ulong2 ok_[PER];
            uint32_t oi[PER];
            uint32_t pos = i0, ia = 0, a1 = 0, ib = 0, b1 = 0;
            ulong2 hA = make_ulong2(0, 0), hB = make_ulong2(0, 0);
            bool setup = true;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                ok_[q] = make_ulong2(0, 0);
                oi[q] = 0;
                if (pos < n) {
                    if (setup || pos >= b1) {
                        uint32_t lo = 0, hi = mp;  // pair p with cb[2p] <= pos
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (cb[2 * mid] <= pos) lo = mid;
                            else hi = mid;
                        }
                        const uint32_t a0 = cb[2 * lo];
                        a1 = cb[2 * lo + 1 < m ? 2 * lo + 1 : m];
                        b1 = cb[2 * lo + 2 < m ? 2 * lo + 2 : m];
                        const uint32_t lenA = a1 - a0, lenB = b1 - a1, d = pos - a0;
                        uint32_t l = d > lenB ? d - lenB : 0, h = d < lenA ? d : lenA;
                        while (l < h) {  // how many of the first d outputs come from A
                            const uint32_t mid = (l + h) >> 1;
                            if (fx_le(key[a0 + mid], key[a1 + d - mid - 1])) l = mid + 1;
                            else h = mid;
                        }
                        ia = a0 + l;
                        ib = a1 + (d - l);
                        if (ia < a1) hA = key[ia];
                        if (ib < b1) hB = key[ib];
                        setup = false;
                    }
                    const bool takeA = ia < a1 && (ib >= b1 || fx_le(hA, hB));
                    if (takeA) {
                        ok_[q] = hA;
                        oi[q] = id[ia];
                        if (++ia < a1) hA = key[ia];
                    } else {
                        ok_[q] = hB;
                        oi[q] = id[ib];
                        if (++ib < b1) hB = key[ib];
                    }
                    ++pos;
                }
            }
            __syncthreads();  // every thread has read its inputs of this round
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                if (i0 + q < n) {
                    key[i0 + q] = ok_[q];
                    id[i0 + q] = (uint16_t)oi[q];
                }
            }
            for (uint32_t p = tid; p <= mp; p += FX_THREADS) cbn[p] = p < mp ? cb[2 * p] : cb[m];
            __syncthreads();
            cb = cbn;
            cbn = cbn == cbA ? cbB : cbA;
            m = mp;
        }
    }
    FXPROF(3);
    // ---- first record per key survives (k_way.rs:146-151); source address of each survivor
    uint32_t keep = 0;
    uint64_t sad[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = i0 + q;
        sad[q] = 0;
        if (i < n) {
            const ulong2 c = key[i];
            bool first = i == 0;
            if (!first) {
                const ulong2 p = key[i - 1];
                first = p.x != c.x || p.y != c.y;
            }
            if (first) {
                keep |= 1u << q;
                const uint32_t e = id[i];
                const uint32_t j = fx_seg(cb0, k + 1, e);
                const uint64_t sa = segaddr[j];
                sad[q] = sa ? sa + (uint64_t)(e - cb0[j]) * S : fx_addr(A, j, sbase[j] + (e - cb0[j]));
            }
        }
    }
    uint32_t total;
    uint32_t c = fx_block_excl<uint32_t>((uint32_t)__builtin_popcount(keep), (uint32_t*)ws, total);  // barriers
    uint64_t* src = (uint64_t*)key;  // source address by survivor
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if (keep & (1u << q)) src[c++] = sad[q];
    const uint32_t cnt = total;
    FXPROF(4);
    if (tid < 64) {
        const uint64_t g0 = fx_lookback(A.tstate, t, cnt, true) + (A.gbase ? *A.gbase : 0ull);
        if (tid == 0) {
            s_g0 = g0;
            if (s_early != cnt) fx_poison(A, FXR_RECORD);  // never: the merge kept another count
            if (t == A.T - 1) *A.Kout = g0 + cnt;
            s_dead = __hip_atomic_load(A.flags + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    FXPROF(5);
    if (!cnt || s_dead) break;
    // ---- output bytes of survivors g0 .. g0+cnt-1 (build_runs' bytes, runs.rs:241-267). The
    // tile's survivors form "pieces": runs of consecutive survivors inside one output run; piece 0
    // starts at survivor 0, piece i >= 1 at survivor jb1 + (i-1) n behind its run's version byte.
    const uint64_t nr = A.n, W = nr * S + 1;
    const uint64_t g0 = s_g0;
    uint64_t q0;
    const uint64_t r0 = fx_divmod(g0, nr, A.inv_n, q0);
    const uint64_t a0 = r0 * W + 1 + q0 * S;  // first survivor's record
    const uint64_t start = q0 == 0 ? a0 - 1 : a0;
    const uint64_t jb1 = nr - q0;             // first survivor (local) opening a new run
    const uint64_t V1 = a0 + jb1 * S;         // its version byte (when jb1 < cnt)
    const uint64_t jL = cnt - 1;
    uint64_t nbL = 0;
    if (jL >= jb1) {
        uint64_t rr;
        nbL = 1 + fx_divmod(jL - jb1, nr, A.inv_n, rr);
    }
    const uint64_t aL = a0 + jL * S + nbL;
    const uint64_t end = aL + S;
    uint8_t* out = A.out;
    const uint32_t S32 = (uint32_t)S;
    const uint64_t Blo = (start + 15) & ~15ull, Bhi = end & ~15ull;
    const uint32_t nb = Bhi > Blo ? (uint32_t)((Bhi - Blo) >> 4) : 0u;
    constexpr int U = SKV_FX_U;
    // At most one run boundary inside the tile (n >= cnt, e.g. 4 MiB runs): each lane walks its
    // blocks with incremental (record, offset) coordinates. Every block, including those that
    // straddle a record end or start at a version byte, is written by the wave instruction that
    // writes its neighbours, so each 128-B output line is completed at once and each input line
    // is read while the neighbouring lanes read it (no partial-line writes, no re-reads).
    // Tiles crossing several runs (small max sizes) take the generic loop.
    const bool multi = jb1 < cnt && cnt - jb1 > nr;
    if (!multi) {
        FxWalk w;
        w.V0 = q0 == 0 ? a0 - 1 : ~0ull;  // version byte before survivor 0
        w.Vb = jb1 < cnt ? V1 : ~0ull;     // version byte before survivor jb1
        w.jb1 = (uint32_t)jb1;
        w.S32 = S32;
        w.dq = (16u * FX_THREADS) / S32;
        w.dr = (16u * FX_THREADS) % S32;
        w.B = Blo + 16ull * tid;
        w.j = 0;
        w.o = 0;
        w.past = w.B > w.Vb;
        {
            const int64_t y = (int64_t)(w.B - a0) - (w.past ? 1 : 0);
            if (y < 0) {  // B is the version byte before survivor 0: y == -1
                w.j = 0xFFFFFFFFu;
                w.o = S32 - 1;
            } else if (w.B < Bhi) {
                uint32_t oo;
                w.j = fx_div32((uint32_t)y, S32, A.inv_S, oo);
                w.o = oo;
            }
        }
        // Software-pipelined over batches of U blocks: batch i+1's loads are issued before batch
        // i's stores, so waiting for a batch's loads never waits for the previous batch's stores
        // (vmcnt counts loads and stores in issue order on gfx9-family CDNA).
        FxBatch<U> P0, P1;
        uint8_t* const ob = out + Blo;
        const uint64_t safe = src[0];
        const uint32_t nfull = nb / (U * FX_THREADS);  // batches whose blocks are all < nb, every lane
        uint32_t i = 0;
        if (nfull) {
            fx_plan<U>(P0, w, src, tid, nb, safe);
            for (; i + 2 < nfull; i += 2) {  // P0 = batch i in flight
                fx_plan<U>(P1, w, src, tid + (i + 1) * U * FX_THREADS, nb, safe);
                fx_finish<U, true>(P0, ob);
                fx_plan<U>(P0, w, src, tid + (i + 2) * U * FX_THREADS, nb, safe);
                fx_finish<U, true>(P1, ob);
            }
            if (i + 1 < nfull) {
                fx_plan<U>(P1, w, src, tid + (i + 1) * U * FX_THREADS, nb, safe);
                fx_finish<U, true>(P0, ob);
                fx_finish<U, true>(P1, ob);
                i += 2;
            } else {
                fx_finish<U, true>(P0, ob);
                i += 1;
            }
        }
        for (uint32_t bb = tid + i * U * FX_THREADS; bb < nb; bb += U * FX_THREADS) {  // the partial batch
            fx_plan<U>(P0, w, src, bb, nb, safe);
            fx_finish<U, false>(P0, ob);
        }
    }
    // Per block: addresses and mode first, then every load of the U blocks, then the merges and
    // stores, so that a lane keeps U (or 2U) loads in flight instead of waiting on each.
    if (multi) for (uint32_t b = tid; b < nb; b += U * FX_THREADS) {
        uint64_t aL[U], aX[U];
        uint32_t mode[U], sh[U];  // mode 0: one record, 1: record tail + next, 2: version byte + record
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t bb = b + u * FX_THREADS;
            aL[u] = 0;
            aX[u] = 0;
            mode[u] = 0;
            sh[u] = 0;
            if (bb < nb) {
                const uint64_t B = Blo + 16ull * bb;
                uint64_t pj = 0, pend = jb1;
                int64_t rel;
                if (jb1 >= cnt || B < V1) {
                    rel = (int64_t)(B - a0);
                } else {
                    const uint64_t d = B - V1;
                    uint64_t i = 0, dr = d;
                    if (d >= W) i = fx_divmod(d, W, A.inv_W, dr);
                    pj = jb1 + i * nr;
                    pend = pj + nr;
                    rel = (int64_t)dr - 1;
                }
                if (rel < 0) {  // the block starts at a version byte
                    if (pj < cnt) {
                        aL[u] = src[pj];
                        mode[u] = 2;
                    }
                } else {
                    uint32_t o;
                    const uint32_t j = (uint32_t)pj + fx_div32((uint32_t)rel, S32, A.inv_S, o);
                    if (o + 16 <= S32) {
                        if (j < cnt) aL[u] = src[j] + o;
                    } else if (j + 1 < cnt) {  // straddles record j's end: its last 16 bytes + what follows
                        aL[u] = src[j] + S - 16;
                        aX[u] = src[j + 1];
                        mode[u] = (j + 1 == pend) ? 3 : 1;  // 3: a version byte sits between the records
                        sh[u] = 16 - (S32 - o);
                    }
                }
            }
        }
        uint4 L[U], X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            L[u] = aL[u] ? fx_cld16(aL[u]) : make_uint4(0, 0, 0, 0);
            X[u] = aX[u] ? fx_cld16(aX[u]) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!aL[u]) continue;
            uint4 v = L[u];
            if (mode[u] == 2) v = fx_vbyte_then(L[u]);
            else if (mode[u] != 0) v = funnel16(L[u], mode[u] == 3 ? fx_vbyte_then(X[u]) : X[u], sh[u]);
            fx_store16(out + Blo + 16ull * (b + u * FX_THREADS), v);
        }
    }
    FXPROF(6);
    // tile edges: blocks shared with the neighbouring tiles get this tile's bytes only
    if (tid == 0 && (start & 15)) {
        const uint64_t B = start & ~15ull, x1 = B + 16 < end ? B + 16 : end;
        fx_store_bytes(out, B, start, x1, fx_compose(A, src, B, start, x1, 0, q0 == 0 ? -1 : 0, q0));
    }
    if (tid == FX_THREADS - 1 && (end & 15)) {
        const uint64_t B = end & ~15ull;
        uint64_t qL;
        fx_divmod(q0 + jL, nr, A.inv_n, qL);
        fx_store_bytes(out, B, B, end, fx_compose(A, src, B, B, end, (uint32_t)jL, (int64_t)(B - aL), qL));
    }
    FXPROF(7);
    } while (0);
}

// descriptors + StatsV1 of the output runs: run r holds survivors [r n, min((r+1) n, K))
__global__ void k_fx_desc(FxArgs A, DevRunDesc* descs, uint64_t* n_runs_out, uint64_t max_runs) {
    const uint64_t K = *A.Kout, nr = A.n, S = A.S, W = nr * S + 1;
    uint64_t runs = (K + nr - 1) / nr;
    if (runs > max_runs) runs = max_runs;  // poisoned call: Kout is meaningless, stay in bounds
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        n_runs_out[0] = runs;
        n_runs_out[1] = K;
        n_runs_out[2] = K * S;
    }
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < runs; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = K - r * nr < nr ? K - r * nr : nr;
        DevRunDesc d;
        d.off = r * W;
        d.len = 1 + c * S;
        d.put_count = c;
        d.delete_count = 0;
        d.min_key_off = d.off + 1 + 5;
        d.min_key_len = A.K;
        d.max_key_off = d.off + 1 + (c - 1) * S + 5;
        d.max_key_len = A.K;
        d.table_id = 0;
        d.reserved = 0;
        descs[r] = d;
    }
}


// a part's survivor count to host-mapped memory (pipelined host calls): one lane, a vector
// store with system scope, so the host sees it once the part's completion event has fired
__global__ void k_fx_publish(const uint64_t* __restrict__ src, uint64_t* dst) {
    if (threadIdx.x == 0) __hip_atomic_store(dst, *src, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i + 16 <= n && !(((uintptr_t)dst | (uintptr_t)src) & 15)) {
        *(uint4*)(dst + i) = *(const uint4*)(src + i);
    } else {
        for (uint64_t b = i; b < i + 16 && b < n; ++b) dst[b] = src[b];
    }
}

// Ingest of a pipelined host call's part by the GPU itself: slice y of the part goes from pinned,
// device-mapped host memory to its run image in HBM (src and dst congruent mod 16), all slices in
// one launch -- in place of one DMA copy per slice (k slices per part, each a DMA descriptor with its
// own fixed cost). Blocks x of a slice stride over its 16-byte blocks, four loads in flight per lane.
__global__ void __launch_bounds__(256) k_ingest(const IngestSlice* __restrict__ sl) {
    const IngestSlice S = sl[blockIdx.y];
    const uint8_t* src = (const uint8_t*)S.src;
    uint8_t* dst = (uint8_t*)S.dst;
    const uint64_t head = ((16 - (S.src & 15)) & 15) < S.len ? ((16 - (S.src & 15)) & 15) : S.len;
    const uint64_t nb = (S.len - head) >> 4, tail0 = head + (nb << 4);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    if (t < head) dst[t] = src[t];
    if (t < S.len - tail0) dst[tail0 + t] = src[tail0 + t];
    const uint4* s4 = (const uint4*)(src + head);
    uint4* d4 = (uint4*)(dst + head);
    uint64_t i = t;
    for (; i + 3 * stride < nb; i += 4 * stride) {
        const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
        d4[i] = a;
        d4[i + stride] = b;
        d4[i + 2 * stride] = c;
        d4[i + 3 * stride] = d;
    }
    for (; i < nb; i += stride) d4[i] = s4[i];
}

// The same ingest for calls with many slices (a WAL flush of 10^6 tiny runs: ~1 KiB slices):
// workgroups stride over the slices one WAVE per slice (a workgroup per slice left 3 of its 4 waves
// idle), each wave copying its slice's 16-byte blocks four per lane in flight; the grid stays small
// (the copies are bound by PCIe) whatever the slice count.
__global__ void __launch_bounds__(256) k_ingest_waves(const IngestSlice* __restrict__ sl, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    for (uint64_t y = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); y < n; y += W) {
        const IngestSlice S = sl[y];
        const uint8_t* src = (const uint8_t*)S.src;
        uint8_t* dst = (uint8_t*)S.dst;
        const uint64_t head = ((16 - (S.src & 15)) & 15) < S.len ? ((16 - (S.src & 15)) & 15) : S.len;
        const uint64_t nb = (S.len - head) >> 4, tail0 = head + (nb << 4);
        if (lane < head) dst[lane] = src[lane];
        if (lane < S.len - tail0) dst[tail0 + lane] = src[tail0 + lane];
        const uint4* s4 = (const uint4*)(src + head);
        uint4* d4 = (uint4*)(dst + head);
        uint64_t i = lane;
        for (; i + 192 < nb; i += 256) {
            const uint4 a = s4[i], b = s4[i + 64], c = s4[i + 128], d = s4[i + 192];
            d4[i] = a;
            d4[i + 64] = b;
            d4[i + 128] = c;
            d4[i + 192] = d;
        }
        for (; i < nb; i += 64) d4[i] = s4[i];
    }
}

// ---------------------------------------------------------------------------------------------
static inline unsigned fx_blocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

void launch_fx_sample(hipStream_t s, const FxArgs& A, const uint64_t* off_dst, uint64_t Sstep, uint64_t n_dst,
                      uint64_t* dhi, uint64_t* dlo, uint64_t* dc, const FxUpLevels& up) {
    if (n_dst) k_fx_sample<<<fx_blocks(n_dst, 256), 256, (A.k + 1) * 8, s>>>(A, off_dst, Sstep, n_dst, dhi, dlo, dc, up);
}
void launch_fx_l1cnt(hipStream_t s, const FxArgs& A, const uint64_t* sc, uint64_t N1, uint32_t* posof, uint32_t* cnt) {
    if (!N1) return;
    k_fx_posof<<<fx_blocks(N1, 256), 256, 2 * (A.k + 1) * 8, s>>>(A, sc, N1, posof);
    k_fx_l1cnt<<<fx_blocks(N1, 256), 256, (A.k + 1) * 8, s>>>(A, posof, N1, cnt);
}
void launch_fx_bounds(hipStream_t s, const FxArgs& A, const uint64_t* shi, const uint64_t* slo, uint64_t m,
                      const uint64_t* l1hi, const uint64_t* l1lo, const uint64_t* l1off, uint64_t Sstep) {
    const uint64_t n = (A.T + 1) * A.k;
    if (n) k_fx_bounds<<<fx_blocks(n, 256), 256, 0, s>>>(A, shi, slo, m, l1hi, l1lo, l1off, Sstep);
}
size_t fx_tile_lds_bytes(uint32_t k) {
    return (size_t)FX_CAP * 16 + (size_t)k * 16 + 2 * (size_t)k * 8 + 3 * (size_t)(k + 1) * 4 + (size_t)FX_CAP * 2 + k + 16;
}
hipError_t launch_fx_tile(hipStream_t s, const FxArgs& A) {
    const size_t lds = fx_tile_lds_bytes(A.k);
    lds_limit((const void*)k_fx_tile);
    k_fx_tile<<<(unsigned)A.T, FX_THREADS, lds, s>>>(A);
    return hipGetLastError();
}
uint64_t fx_tile_slots(uint32_t k) {  // fused tiles resident at once on the current device
    // one entry per (device, k), under a lock: ctxs on other threads call this concurrently
    static std::mutex mu;
    static std::map<std::pair<int, uint32_t>, uint64_t> cache;
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({dev, k});
    if (it != cache.end()) return it->second;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_fx_tile, FX_THREADS, fx_tile_lds_bytes(k));
    const uint64_t slots = (uint64_t)(cus > 0 ? cus : 256) * (uint64_t)(per > 0 ? per : 1);
    cache[{dev, k}] = slots;
    return slots;
}
void launch_ingest(hipStream_t s, const IngestSlice* slices, uint32_t n, uint32_t blocks_per_slice) {
    if (n) k_ingest<<<dim3(blocks_per_slice, n), 256, 0, s>>>(slices);
}
void launch_ingest_slices(hipStream_t s, const IngestSlice* slices, uint64_t n, uint32_t grid) {
    // a wave per slice (a workgroup per slice, k_ingest_slices' old shape, measured 12 % slower on
    // config 5's 10^6-slice parts: profiles/r05/c5_host.txt)
    if (n) k_ingest_waves<<<(unsigned)std::min<uint64_t>((n + 3) / 4, grid ? grid : 1), 256, 0, s>>>(slices, n);
}
void launch_copy_bytes(hipStream_t s, uint8_t* dst, const uint8_t* src, uint64_t n) {
    if (n) k_copy_bytes<<<fx_blocks((n + 15) / 16, 256), 256, 0, s>>>(dst, src, n);
}
void launch_fx_publish(hipStream_t s, const uint64_t* src, uint64_t* dst) { k_fx_publish<<<1, 64, 0, s>>>(src, dst); }
void launch_fx_desc(hipStream_t s, const FxArgs& A, DevRunDesc* descs, uint64_t* n_runs_out, uint64_t max_runs) {
    unsigned blocks = fx_blocks(max_runs ? max_runs : 1, 256);
    if (blocks > 4096) blocks = 4096;
    k_fx_desc<<<blocks, 256, 0, s>>>(A, descs, n_runs_out, max_runs);
}

}  // namespace skv
