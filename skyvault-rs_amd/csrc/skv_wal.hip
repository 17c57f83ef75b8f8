// skv_wal.hip — WAL compaction's table split on the device (SKV_SPLIT_BY_TABLE).
//
// After the merge (k_finalize's dense arrays: K surviving records in key order), the reference's
// WAL loop (src/jobs/wal_compaction.rs:66-174) does, per merged op:
//   split_once('.') -> InvalidInput if missing (:71-73); prefix.parse::<i64>() -> InvalidInput
//   (:75-79); strip format!("{id}.").len() bytes (:81, :91-94); a change of table id closes the
//   table's build_runs task and opens a new one (:82-86, :96-123). Each task must produce exactly
//   one run (:126-137); a failing task (that check, or build_runs' order error) is swallowed by
//   `if let Ok(..)` (:103, :168) and the table's data is dropped.
// Here: one thread per merged record parses its key prefix; tables are the maximal runs of equal
// table id in merged order; per table the stripped sizes, order check and one-run rule decide
// keep/drop; kept tables become one output run each (version byte + rewritten records).
#include "skv_launch.hpp"

#include <algorithm>
#include <cstdlib>

namespace skv {

static inline unsigned wal_blocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Rust `str::parse::<i64>` (core::num, radix 10): returns 0 ok, else WERR_*.
__device__ __forceinline__ uint32_t parse_i64_dev(const uint8_t* s, uint64_t n, int64_t& out) {
    if (n == 0) return WERR_EMPTY;
    uint64_t i = 0;
    bool neg = false;
    uint8_t c0 = s[0];
    if (c0 == '+' || c0 == '-') {
        if (n == 1) return WERR_DIGIT;
        neg = c0 == '-';
        i = 1;
    }
    int64_t r = 0;
    for (; i < n; ++i) {
        uint32_t c = s[i];
        if (c < '0' || c > '9') return WERR_DIGIT;  // to_digit before the overflow checks
        int64_t m;
        if (__builtin_mul_overflow(r, (int64_t)10, &m)) return neg ? WERR_NEG : WERR_POS;
        int64_t d = (int64_t)(c - '0');
        if (neg ? __builtin_sub_overflow(m, d, &r) : __builtin_add_overflow(m, d, &r)) return neg ? WERR_NEG : WERR_POS;
    }
    out = r;
    return 0;
}

// parse_i64_dev over key bytes 0..n-1 (n <= 27) held in a record's first 32 bytes (key at byte 5):
// the same outcome, read from registers (unrolled, constant indices) instead of byte loads
__device__ __forceinline__ uint32_t parse_i64_win(const uint32_t hw[8], uint32_t n, int64_t& out) {
    if (n == 0) return WERR_EMPTY;
    const uint32_t c0 = (hw[1] >> 8) & 0xFFu;
    const bool sign = c0 == '+' || c0 == '-';
    if (sign && n == 1) return WERR_DIGIT;
    const bool neg = c0 == '-';
    int64_t r = 0;
    uint32_t err = 0;
#pragma unroll
    for (int i = 0; i < 27; ++i) {
        if ((uint32_t)i < n && !err && !(i == 0 && sign)) {
            const uint32_t c = (hw[(i + 5) >> 2] >> (8 * ((i + 5) & 3))) & 0xFFu;
            if (c < '0' || c > '9') {
                err = WERR_DIGIT;  // to_digit before the overflow checks
            } else {
                int64_t m;
                const int64_t d = (int64_t)(c - '0');
                if (__builtin_mul_overflow(r, (int64_t)10, &m) ||
                    (neg ? __builtin_sub_overflow(m, d, &r) : __builtin_add_overflow(m, d, &r)))
                    err = neg ? WERR_NEG : WERR_POS;
            }
        }
    }
    if (!err) out = r;
    return err;
}

// byte length of format!("{id}.")
__device__ __forceinline__ uint32_t id_prefix_len(int64_t id) {
    uint64_t u = id < 0 ? (uint64_t)0 - (uint64_t)id : (uint64_t)id;
    uint32_t d = 1;
    while (u >= 10) {
        u /= 10;
        ++d;
    }
    return d + (id < 0 ? 1u : 0u) + 1u;
}

// per merged record: table id, strip length, stripped record size; the first bad key (merged
// order) is the job's InvalidInput error. The key length and marker come from the record's own
// header (the line the key is read from), not from rec_klen[m_rec[j]]: that random 4-byte gather
// fetched a line of its own per merged record. wnk = the stripped key's length, canon bit 1 a Delete.
__global__ void k_wal_keys(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ m_src,
                           const uint64_t* __restrict__ P, int64_t* tid, uint32_t* strip, uint32_t* wnk,
                           uint64_t* wsize, uint8_t* canon, unsigned long long* first_err) {
    const uint64_t K = *Kp;
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const uint8_t* rp = (const uint8_t*)m_src[j];
    const uint64_t size = P[j + 1] - P[j];  // the record's bytes: its first min(32, size) in one round trip
    const uint4 h0 = load_window16(rp, (uint32_t)(size < 16 ? size : 16));
    const uint4 h1 = size > 16 ? load_window16(rp + 16, (uint32_t)(size - 16 < 16 ? size - 16 : 16)) : make_uint4(0, 0, 0, 0);
    const uint32_t hw[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    const uint32_t marker = hw[0] & 0xFFu;
    const uint64_t klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(hw[1], hw[0], 1));
    const uint8_t* key = rp + 5;
    // split_once('.'): the first '.' -- key bytes 0..26 from the window, then 16 per load
    uint64_t dot = klen;
    {
        const uint32_t n0 = (uint32_t)(klen < 27 ? klen : 27);
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 27; ++i)
            if (((hw[(i + 5) >> 2] >> (8 * ((i + 5) & 3))) & 0xFFu) == (uint32_t)'.' && (uint32_t)i < n0) hit |= 1u << i;
        if (hit) dot = __builtin_ctz(hit);
    }
    for (uint64_t o = 27; dot == klen && o < klen; o += 16) {
        const uint32_t m = (uint32_t)(klen - o < 16 ? klen - o : 16);
        const uint4 v = load_window16(key + o, m);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == (uint32_t)'.' && (uint32_t)i < m) hit |= 1u << i;
        if (hit) dot = o + __builtin_ctz(hit);
    }
    int64_t id = 0;
    uint32_t e = dot == klen ? WERR_NODOT : (dot <= 27 ? parse_i64_win(hw, (uint32_t)dot, id) : parse_i64_dev(key, dot, id));
    uint32_t st = 0;
    if (e) atomicMin(first_err, (unsigned long long)j);
    else st = id_prefix_len(id);
    tid[j] = id;
    strip[j] = st;
    wnk[j] = (uint32_t)(klen - st);
    canon[j] = ((!e && dot + 1 == st) ? 1 : 0) | (marker == 2 ? 2 : 0);  // the prefix is format!("{id}.") itself
    wsize[j] = size - st;
}

// stripped key of record j: bytes [src+5+strip, src+5+klen)
__device__ __forceinline__ int stripped_cmp(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
    const uint64_t n = la < lb ? la : lb;
    const int c = bytes_cmp16(a, b, n);
    if (c) return c;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// table starts (a change of table id, :82-86) and build_runs' order check between neighbours of
// one table on the stripped keys (runs.rs:190-198). Two neighbours whose prefixes are both the
// canonical "{id}." text of the same id share that prefix, so their stripped keys order like the
// merged keys (strictly ascending): only non-canonical prefixes ("007.", "+5.") compare bytes.
__global__ void k_wal_flags(const uint64_t* __restrict__ Kp, const int64_t* __restrict__ tid,
                            const uint32_t* __restrict__ strip, const uint8_t* __restrict__ canon,
                            const uint64_t* __restrict__ m_src, const uint32_t* __restrict__ wnk, uint64_t* is_new,
                            uint32_t* bad, uint32_t exact) {
    const uint64_t K = *Kp;
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const bool nw = j == 0 || tid[j] != tid[j - 1];
    is_new[j] = nw ? 1 : 0;
    uint32_t b = 0;
    // (heap-order mode, unsorted inputs: the merged keys are not ascending, compare every pair)
    if (!nw && (exact || !(canon[j - 1] & canon[j] & 1))) {
        const uint64_t sa = strip[j - 1], sb = strip[j];
        const uint8_t* ka = (const uint8_t*)m_src[j - 1] + 5 + sa;
        const uint8_t* kb = (const uint8_t*)m_src[j] + 5 + sb;
        const uint64_t la = wnk[j - 1], lb = wnk[j];
        b = stripped_cmp(ka, la, kb, lb) >= 0 ? 1u : 0u;
    }
    bad[j] = b;
}

// table index per record, table start table, failing tables and each one's first failing record
__global__ void k_wal_index(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ is_new,
                            const uint64_t* __restrict__ new_ex, const uint32_t* __restrict__ bad, uint32_t* tix,
                            uint64_t* tstart, uint32_t* tbad, unsigned long long* tfirst) {
    const uint64_t K = *Kp;
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const uint64_t t = new_ex[j] + is_new[j] - 1;
    tix[j] = (uint32_t)t;
    if (is_new[j]) tstart[t] = j;
    if (j == K - 1) tstart[t + 1] = K;
    if (bad[j]) {
        tbad[t] = 1;
        atomicMin(&tfirst[t], (unsigned long long)j);
    }
}

// keep/drop per table: no order error and exactly one run (count == 1, or 1 + bytes <= max)
__global__ void k_wal_tables(const uint64_t* __restrict__ NTp, const uint64_t* __restrict__ tstart,
                             const uint64_t* __restrict__ Pw, const uint32_t* __restrict__ tbad, uint64_t max_size,
                             uint64_t* run_len, uint64_t* keep) {
    const uint64_t NT = *NTp;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NT) return;
    const uint64_t b = tstart[t], e = tstart[t + 1];
    const uint64_t bytes = Pw[e] - Pw[b];
    const bool ok = !tbad[t] && (e - b == 1 || 1 + bytes <= max_size);
    run_len[t] = ok ? 1 + bytes : 0;
    keep[t] = ok ? 1 : 0;
}

__global__ void k_wal_desc(const uint64_t* __restrict__ NTp, const uint64_t* __restrict__ tstart,
                           const uint64_t* __restrict__ Pw, const uint64_t* __restrict__ Dp,
                           const uint64_t* __restrict__ keep, const uint64_t* __restrict__ keep_ex,
                           const uint64_t* __restrict__ run_off, const int64_t* __restrict__ tid,
                           const uint32_t* __restrict__ wnk, DevRunDesc* descs) {
    const uint64_t NT = *NTp;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NT || !keep[t]) return;
    const uint64_t b = tstart[t], e = tstart[t + 1];
    DevRunDesc d;
    d.off = run_off[t];
    d.len = 1 + Pw[e] - Pw[b];
    d.delete_count = Dp[e] - Dp[b];
    d.put_count = (e - b) - d.delete_count;
    d.min_key_off = d.off + 1 + 5;
    d.min_key_len = wnk[b];
    d.max_key_off = d.off + 1 + (Pw[e - 1] - Pw[b]) + 5;
    d.max_key_len = wnk[e - 1];
    d.table_id = tid[b];
    d.reserved = 0;
    descs[keep_ex[t]] = d;
}

// Output bytes of kept tables: a version byte per run, then every record with its key_len
// rewritten and the table prefix removed (WriteOperation::Put(key.split_off(..), value), :91-94).
// One workgroup per WAL_G merged records: the kept ones' output pieces (a synthesized head of
// [version byte,] marker, key_len and the source body after the prefix) go to LDS; the
// workgroup's output span is contiguous (kept tables are), and each lane then composes whole
// 16-byte output blocks from the pieces (bytewise only at the span's two edges).
constexpr int WAL_G = 256;  // k_wal_gather's merged records (and threads) per workgroup

// bytes [x0, x1) of output block B, starting inside kept record r
template <typename HL>
__device__ uint4 wal_compose(uint64_t B, uint64_t x0, uint64_t x1, uint32_t r, const uint64_t* os,
                             const uint64_t* src, const uint64_t* head, const HL* hl) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint64_t x = x0;
    while (x < x1) {
        const uint64_t rel = x - os[r];
        const uint64_t rlen = os[r + 1] - os[r];
        uint64_t m;
        if (rel < hl[r]) {  // synthesized head bytes (<= 6): shifted into place as one 16-byte word
            m = hl[r] - rel;
            if (m > x1 - x) m = x1 - x;
            const uint64_t hv = head[r] >> (8 * rel);
            const uint32_t a = (uint32_t)(x - B), e = a + (uint32_t)m;
            const uint4 w = shl_bytes(make_uint4((uint32_t)hv, (uint32_t)(hv >> 32), 0u, 0u), a);
            acc.x |= w.x & dword_mask(a, e, 0);
            acc.y |= w.y & dword_mask(a, e, 1);
            acc.z |= w.z & dword_mask(a, e, 2);
            acc.w |= w.w & dword_mask(a, e, 3);
        } else {
            m = rlen - rel;
            if (m > x1 - x) m = x1 - x;
            const uint32_t a = (uint32_t)(x - B), e = a + (uint32_t)m;
            uint4 w = load_window16((const uint8_t*)src[r] + (rel - hl[r]), (uint32_t)m);
            w = shl_bytes(w, a);
            acc.x |= w.x & dword_mask(a, e, 0);
            acc.y |= w.y & dword_mask(a, e, 1);
            acc.z |= w.z & dword_mask(a, e, 2);
            acc.w |= w.w & dword_mask(a, e, 3);
        }
        x += m;
        if (x - os[r] == rlen) ++r;
    }
    return acc;
}

__global__ void __launch_bounds__(WAL_G) k_wal_gather(const uint64_t* __restrict__ Kp, const uint32_t* __restrict__ tix,
                                                      const uint64_t* __restrict__ tstart,
                                                      const uint64_t* __restrict__ keep,
                                                      const uint64_t* __restrict__ run_off,
                                                      const uint64_t* __restrict__ Pw,
                                                      const uint32_t* __restrict__ strip,
                                                      const uint64_t* __restrict__ m_src,
                                                      const uint32_t* __restrict__ wnk,
                                                      const uint8_t* __restrict__ canon, uint8_t* out) {
    __shared__ uint64_t os[WAL_G + 1], src[WAL_G], head[WAL_G];
    __shared__ uint32_t hl[WAL_G];
    __shared__ uint32_t s_cnt[WAL_G / 64 + 1];
    const uint64_t K = *Kp;
    const uint64_t j0 = (uint64_t)blockIdx.x * WAL_G;
    if (j0 >= K) return;
    const uint64_t j = j0 + threadIdx.x;
    bool kept = false;
    uint64_t ostart = 0, olen = 0, body = 0, hd = 0;
    uint32_t hlen = 0;
    if (j < K) {
        const uint32_t t = tix[j];
        kept = keep[t] != 0;
        if (kept) {
            const uint64_t b = tstart[t];
            const uint8_t* sp = (const uint8_t*)m_src[j];
            const uint32_t st = strip[j];
            const uint32_t nk = wnk[j];
            const bool first = j == b;
            ostart = run_off[t] + 1 + (Pw[j] - Pw[b]) - (first ? 1 : 0);
            olen = (Pw[j + 1] - Pw[j]) + (first ? 1 : 0);
            body = (uint64_t)sp + 5 + st;
            const uint64_t h5 = (uint64_t)((canon[j] & 2) ? 2u : 1u) | ((uint64_t)(nk >> 24) << 8) | ((uint64_t)((nk >> 16) & 0xFF) << 16) |
                                ((uint64_t)((nk >> 8) & 0xFF) << 24) | ((uint64_t)(nk & 0xFF) << 32);
            hd = first ? (1ull | (h5 << 8)) : h5;  // CURRENT_VERSION (runs.rs:241-246), marker, key_len
            hlen = first ? 6u : 5u;
        }
    }
    // compact the kept records (merged order) into the piece table
    const uint64_t bal = __ballot(kept);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) s_cnt[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = 0, c = 0;
    for (int w = 0; w < WAL_G / 64; ++w) {
        if (w < wv) before += s_cnt[w];
        c += s_cnt[w];
    }
    if (kept) {
        const uint32_t i = before + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        os[i] = ostart;
        src[i] = body;
        head[i] = hd;
        hl[i] = hlen;
        if (i + 1 == c) os[c] = ostart + olen;
    }
    __syncthreads();
    if (c == 0) return;
    const uint64_t lo = os[0], hi = os[c];
    const uint64_t Blo = lo & ~15ull, Bhi = (hi + 15) & ~15ull;
    for (uint64_t B = Blo + 16ull * threadIdx.x; B < Bhi; B += 16ull * WAL_G) {
        const uint64_t x0 = B > lo ? B : lo, x1 = B + 16 < hi ? B + 16 : hi;
        uint32_t a = 0, bb = c;  // last record with os <= x0
        while (bb - a > 1) {
            const uint32_t mid = (a + bb) >> 1;
            if (os[mid] <= x0) a = mid;
            else bb = mid;
        }
        const uint4 v = wal_compose(B, x0, x1, a, os, src, head, hl);
        if (x0 == B && x1 == B + 16) {
            *(uint4*)(out + B) = v;
        } else {  // span edge: this workgroup's bytes only
            for (uint64_t y = x0; y < x1; ++y) out[y] = (uint8_t)byte_of(v, (uint32_t)(y - B));
        }
    }
}

// ---------------------------------------------------------------------------------------------
// One pass for the common case (k_wal_fused): every key has a table prefix, every table's stripped
// keys ascend, and every table fits one run -- then every table is kept and its run is simply
// [version byte, its records stripped]. Per merged record: the first min(32, size) bytes (the key's
// prefix and length), the table id, a new-table flag against the previous record, the stripped size;
// a decoupled look-back over workgroups (ticket order) gives each record's output offset W_j + N_j
// (stripped bytes before it, table starts up to it); the workgroup then composes its output blocks
// from the lines it just read (k_wal_gather's pieces). Table starts go to an unordered list that the
// host sorts into the descriptors. Anything else -- a bad key, an order error, a table over max, more
// tables than the list holds -- sets a fail bit, and the host runs the exact stage above instead.
struct WalRec {
    uint64_t size;
    int64_t tid;
    uint32_t strip, klen, marker, err;
    bool canon;
};
__device__ __forceinline__ WalRec wal_parse(const uint8_t* rp, uint64_t size) {
    WalRec r;
    r.size = size;
    const uint4 h0 = load_window16(rp, (uint32_t)(size < 16 ? size : 16));
    const uint4 h1 = size > 16 ? load_window16(rp + 16, (uint32_t)(size - 16 < 16 ? size - 16 : 16)) : make_uint4(0, 0, 0, 0);
    const uint32_t hw[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    r.marker = hw[0] & 0xFFu;
    r.klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(hw[1], hw[0], 1));
    const uint8_t* key = rp + 5;
    uint64_t dot = r.klen;
    {
        const uint32_t n0 = r.klen < 27 ? r.klen : 27;
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 27; ++i)
            if (((hw[(i + 5) >> 2] >> (8 * ((i + 5) & 3))) & 0xFFu) == (uint32_t)'.' && (uint32_t)i < n0) hit |= 1u << i;
        if (hit) dot = __builtin_ctz(hit);
    }
    for (uint64_t o = 27; dot == r.klen && o < r.klen; o += 16) {
        const uint32_t m = (uint32_t)(r.klen - o < 16 ? r.klen - o : 16);
        const uint4 v = load_window16(key + o, m);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == (uint32_t)'.' && (uint32_t)i < m) hit |= 1u << i;
        if (hit) dot = o + __builtin_ctz(hit);
    }
    r.tid = 0;
    r.err = dot == r.klen ? WERR_NODOT : (dot <= 27 ? parse_i64_win(hw, (uint32_t)dot, r.tid) : parse_i64_dev(key, dot, r.tid));
    r.strip = r.err ? 0u : id_prefix_len(r.tid);
    r.canon = !r.err && dot + 1 == r.strip;
    return r;
}

// wal_parse from a record's 16-byte key prefix (the record sort's output element: no record line
// read): the window words are rebuilt as the record's first 21 bytes (marker, key length, key bytes
// 0..15); a dot inside those 16 bytes (or a key of at most 16 bytes) decides it exactly, else the
// record itself is parsed (ok = false)
__device__ __forceinline__ WalRec wal_parse_pfx(uint64_t hi, uint64_t lo, uint32_t klen, uint32_t marker,
                                               uint64_t size, bool& ok) {
    WalRec r;
    r.size = size;
    r.marker = marker;
    r.klen = klen;
    r.tid = 0;
    uint32_t k[4] = {__builtin_bswap32((uint32_t)(hi >> 32)), __builtin_bswap32((uint32_t)hi),
                     __builtin_bswap32((uint32_t)(lo >> 32)), __builtin_bswap32((uint32_t)lo)};  // key bytes LE
    const uint32_t kb = __builtin_bswap32(klen);
    uint32_t hw[8];  // bytes: [marker, klen BE x4, key 0..15, zeros]
    hw[0] = marker | (kb << 8);
    hw[1] = (kb >> 24) | (k[0] << 8);
    hw[2] = (k[0] >> 24) | (k[1] << 8);
    hw[3] = (k[1] >> 24) | (k[2] << 8);
    hw[4] = (k[2] >> 24) | (k[3] << 8);
    hw[5] = k[3] >> 24;
    hw[6] = hw[7] = 0;
    const uint32_t n0 = klen < 16 ? klen : 16;
    uint32_t hit = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (((hw[(i + 5) >> 2] >> (8 * ((i + 5) & 3))) & 0xFFu) == (uint32_t)'.' && (uint32_t)i < n0) hit |= 1u << i;
    ok = hit || klen <= 16;
    if (!ok) return r;
    const uint32_t dot = hit ? (uint32_t)__builtin_ctz(hit) : klen;
    r.err = dot == klen ? WERR_NODOT : parse_i64_win(hw, dot, r.tid);
    r.strip = r.err ? 0u : id_prefix_len(r.tid);
    r.canon = !r.err && dot + 1 == r.strip;
    return r;
}

// SKV_WAL_PROBE (diagnostic builds, output invalid by design): phase knockouts of k_wal_fused --
// 1 no look-back wait (the predecessor's slot as read once: offsets stay in bounds), 2 no output
// bytes, 4 no key parse (the element's fields as a canonical key)
#ifndef SKV_WAL_PROBE
#define SKV_WAL_PROBE 0
#endif
constexpr uint32_t WF_BADKEY = 1, WF_ORDER = 2, WF_TABLES = 4;
// WF_R merged records per thread, strided (record k*WAL_T + tid of the workgroup's WF_G): one
// look-back per WF_G records (at one record per thread the look-back wait was 1.85 of 7.0 ms at
// config 5, profiles/r06/wal_probe.txt)
constexpr int WAL_T = 256, WF_R = (int)WAL_FUSED_RPT, WF_G = WAL_T * WF_R;
static_assert(WF_G == (int)WAL_FUSED_G, "k_wal_fused's records per workgroup (host look-back sizing)");
constexpr uint32_t WF_TBL = 4096;  // output blocks of a workgroup's span with a piece table (64 KiB)
static_assert(WF_G <= 65536, "piece ids in the block table are 16-bit");
constexpr int WF_NB = 4;                 // a body's aligned 16-byte blocks loaded before the look-back
constexpr uint32_t WF_STAGE = 64 * WF_G;  // LDS staging bytes (64 per record); the piece arrays share it
static_assert(8 * (WF_G + 1) + 16 * WF_G + 2 * WF_TBL + WF_G <= WF_STAGE, "piece arrays fit the stage area");

// bytes 0..n-1 of v (n <= 16) to LDS bytes d..d+n-1 of a zeroed area: dwords a neighbouring piece
// shares are ORed in, whole dwords stored
__device__ __forceinline__ void lds_or16(uint32_t* buf, uint32_t d, uint4 v, uint32_t n) {
    const uint32_t sh = d & 3;
    uint32_t* p = buf + (d >> 2);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t x[5];
    x[0] = w[0] << (8 * sh);
#pragma unroll
    for (int i = 1; i < 4; ++i) x[i] = (uint32_t)((((uint64_t)w[i] << 32) | w[i - 1]) >> (32 - 8 * sh));
    x[4] = sh ? w[3] >> (32 - 8 * sh) : 0u;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t m = dword_mask(sh, sh + n, (uint32_t)i);
        if (m == 0xFFFFFFFFu) p[i] = x[i];
        else if (m) atomicOr(&p[i], x[i] & m);
    }
}
struct WalPrev {
    int64_t tid;
    uint64_t size, rp;
    uint32_t strip, klen;
    bool canon;
};

// (4 waves per SIMD asked of the register allocator: 128 VGPRs with a few spills, 5.55 ms at config 5,
// against 134 VGPRs at 3 waves, 5.86 ms)
__global__ void __launch_bounds__(WAL_T) __attribute__((amdgpu_waves_per_eu(4))) k_wal_fused(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ m_src,
                                                     const uint64_t* __restrict__ P, const uint64_t* __restrict__ Dp,
                                                     uint8_t* out, uint64_t* tstate, uint32_t* ticket, uint32_t* fail,
                                                     WalTStart* tlist, uint32_t* tcount, uint32_t tcap,
                                                     uint64_t* tail, uint32_t diag,
                                                     const SElem* __restrict__ S, const uint32_t* __restrict__ m_rec) {
    constexpr int NW = WAL_T / 64;
    // the output staging area; a span too long for it composes from the pieces (arrays carved from it)
    __shared__ uint4 s_stage[WF_STAGE / 16];
    uint64_t* os = (uint64_t*)s_stage;  // [WF_G + 1]
    uint64_t* src = os + WF_G + 1;
    uint64_t* head = src + WF_G;
    uint16_t* s_tbl = (uint16_t*)(head + WF_G);  // [WF_TBL]
    uint8_t* hl = (uint8_t*)(s_tbl + WF_TBL);    // [WF_G]
    __shared__ uint64_t s_w[WF_R][NW], s_base[1];
    __shared__ WalPrev s_prev[WF_R][NW];  // each wave's last record (per k), for the next wave's lane 0
    __shared__ uint32_t s_t;
    const uint64_t K = *Kp;
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t t = s_t;
    const uint64_t j0 = t * WF_G;
    if (j0 >= K) return;  // (tickets past the last workgroup: nothing to publish)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WalRec r[WF_R];
    const uint8_t* rp[WF_R];
    uint64_t p0[WF_R], p1[WF_R], d0[WF_R], d1[WF_R];
    uint32_t bad = 0;
    // every load of the WF_R records first (independent), then the parses
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
        rp[k] = nullptr;
        p0[k] = p1[k] = d0[k] = d1[k] = 0;
        if (j < K) {
            rp[k] = (const uint8_t*)m_src[j];
            p0[k] = P[j];
            p1[k] = P[j + 1];
            d0[k] = Dp[j];
            d1[k] = Dp[j + 1];
        }
    }
    SElem e[WF_R];
    uint4 pb[WF_R][WF_NB];
    bool pre[WF_R];
    if (S) {
#pragma unroll
        for (int k = 0; k < WF_R; ++k) {
            const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
            if (j < K) e[k] = S[m_rec[j]];
        }
    }
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
        r[k] = WalRec{};
        if (j < K) {
            bool ok = false;
            if (S) {  // the record sort's element: its key prefix, no record line read for the parse
                if (SKV_WAL_PROBE & 4) {
                    r[k].size = p1[k] - p0[k];
                    r[k].marker = d1[k] != d0[k] ? 2u : 1u;
                    r[k].klen = e[k].klen;
                    r[k].tid = (int64_t)(e[k].hi >> 56);
                    r[k].strip = 2;
                    r[k].canon = true;
                    r[k].err = 0;
                    ok = true;
                } else {
                    r[k] = wal_parse_pfx(e[k].hi, e[k].lo, e[k].klen, d1[k] != d0[k] ? 2u : 1u, p1[k] - p0[k], ok);
                }
            }
            if (!ok) r[k] = wal_parse(rp[k], p1[k] - p0[k]);
            if (r[k].err || ((diag & WAL_STRICT_CANON) && !r[k].canon)) bad |= WF_BADKEY;
        }
        // the record before: the neighbouring lane; a wave's lane 0 takes the previous wave's last
        // lane (of the same k, or of k - 1 for the workgroup's thread 0) through LDS
        if (lane == 63) {
            WalPrev& q = s_prev[k][wv];
            q.tid = r[k].tid;
            q.strip = r[k].strip;
            q.klen = r[k].klen;
            q.canon = r[k].canon;
            q.size = r[k].size;
            q.rp = (uint64_t)rp[k];
        }
    }
    __syncthreads();
    uint64_t wo[WF_R], wi[WF_R];
    bool nw[WF_R];
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
        const bool live = j < K;
        int64_t ptid = __shfl_up(r[k].tid, 1, 64);
        uint32_t pstrip = __shfl_up(r[k].strip, 1, 64), pklen = __shfl_up(r[k].klen, 1, 64);
        bool pcanon = __shfl_up(r[k].canon ? 1 : 0, 1, 64) != 0;
        uint64_t psize = __shfl_up(r[k].size, 1, 64);
        const uint8_t* prp = (const uint8_t*)__shfl_up((uint64_t)rp[k], 1, 64);
        if (lane == 0 && (wv > 0 || k > 0)) {
            const WalPrev& q = wv > 0 ? s_prev[k][wv - 1] : s_prev[k > 0 ? k - 1 : 0][NW - 1];
            ptid = q.tid;
            pstrip = q.strip;
            pklen = q.klen;
            pcanon = q.canon;
            psize = q.size;
            prp = (const uint8_t*)q.rp;
        }
        if (live && threadIdx.x == 0 && k == 0 && j > 0) {  // only the workgroup's first record parses its predecessor
            prp = (const uint8_t*)m_src[j - 1];
            const WalRec q = wal_parse(prp, P[j] - P[j - 1]);
            ptid = q.tid;
            pstrip = q.strip;
            pklen = q.klen;
            pcanon = q.canon;
            psize = q.size;
            if (q.err) bad |= WF_BADKEY;
        }
        nw[k] = live && (j == 0 || ptid != r[k].tid);
        if (live && !nw[k] && !(pcanon && r[k].canon)) {  // stripped keys must ascend inside a table
            const uint8_t* ka = prp + 5 + pstrip;
            const uint8_t* kb = rp[k] + 5 + r[k].strip;
            const uint64_t la = pklen - pstrip, lb = r[k].klen - r[k].strip;
            const uint64_t n = la < lb ? la : lb;
            int c = bytes_cmp16(ka, kb, n);
            if (!c) c = la < lb ? -1 : (la > lb ? 1 : 0);
            if (c >= 0) bad |= WF_ORDER;
        }
        if (nw[k] && live) {  // table starts go to the unordered list
            const uint32_t x = atomicAdd(tcount, 1u);
            if (x < tcap) {
                WalTStart ts;
                ts.b = j;
                ts.W = 0;  // (filled below, once the output offset is known)
                ts.Dp = d0[k];
                ts.tid = r[k].tid;
                ts.nk = r[k].klen - r[k].strip;
                ts.prev_nk = j ? pklen - pstrip : 0;
                ts.prev_ws = j ? psize - pstrip : 0;
                tlist[x] = ts;
                p0[k] = x;  // (p0 no longer needed: the list slot)
            } else {
                atomicOr(fail, WF_TABLES);
                p0[k] = ~0ull;
            }
        }
        // output bytes of record j: its version byte (a table start) + its stripped record. The
        // exclusive prefix of those is where its piece starts, and a table's version byte sits where
        // its first record's piece starts, so one sum places everything (no separate table-start count).
        wo[k] = live ? r[k].size - r[k].strip + (nw[k] ? 1 : 0) : 0;
        wi[k] = wo[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t a = __shfl_up(wi[k], d, 64);
            if (lane >= d) wi[k] += a;
        }
        if (lane == 63) s_w[k][wv] = wi[k];
    }
    if (bad) atomicOr(fail, bad);
    __syncthreads();
    uint64_t wb[WF_R], wt = 0;
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        wb[k] = wt;
        for (int w = 0; w < NW; ++w) {
            if (w < wv) wb[k] += s_w[k][w];
            wt += s_w[k][w];
        }
    }
    const bool staged = wt + 32 <= WF_STAGE;
    if (staged)
        for (uint32_t i = threadIdx.x; i < WF_STAGE / 16; i += WAL_T) s_stage[i] = make_uint4(0, 0, 0, 0);
    // decoupled look-back over workgroups (ticket order); wave 0 reads 64 predecessors per step.
    // The aggregate goes out before any record body is read: a successor's look-back waits on it
    constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62, VM = FA - 1;
    if (threadIdx.x == 0) __hip_atomic_store(&tstate[t], (t == 0 ? FI : FA) | wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the bodies' aligned 16-byte blocks, loaded now so their lines arrive during the look-back (a
    // body of more than WF_NB blocks is loaded when it is written)
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
        pre[k] = false;
        if (staged && j < K) {
            const uintptr_t sa = (uintptr_t)rp[k] + 5 + r[k].strip, a0 = sa & ~(uintptr_t)15;
            const uint64_t L = r[k].size - 5 - r[k].strip;
            pre[k] = (sa & 15) + L <= 16 * WF_NB;
            if (pre[k]) {
#pragma unroll
                for (int i = 0; i < WF_NB; ++i)
                    if (a0 + 16 * i < sa + L) pb[k][i] = *(const uint4*)(a0 + 16 * i);
            }
        }
    }
    if (threadIdx.x < 64) {
        uint64_t acc = 0;
        if (t > 0) {
            int64_t top = (int64_t)t - 1;
            if (SKV_WAL_PROBE & 1) {  // one read: an inclusive, an aggregate or 0, all <= the true prefix
                acc = lane == 0 ? (__hip_atomic_load(&tstate[top], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & VM) : 0;
                acc = __shfl(acc, 0, 64);
                top = -1;
            }
            for (; top >= 0;) {
                const int64_t p = top - lane;
                const uint64_t v = p >= 0 ? __hip_atomic_load(&tstate[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FI;
                const uint64_t f = v >> 62;
                const uint64_t incl = __ballot(f == 2), none = __ballot(f == 0);
                const int first = incl ? __builtin_ctzll(incl) : 64;
                const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
                if (none & upto) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint64_t x = lane <= first ? (v & VM) : 0;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
                acc += x;
                if (first < 64) break;
                top -= 64;
            }
            if (lane == 0) __hip_atomic_store(&tstate[t], FI | (acc + wt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_base[0] = acc;
    }
    __syncthreads();
    const uint32_t c = (uint32_t)(K - j0 < (uint64_t)WF_G ? K - j0 : (uint64_t)WF_G);
    const uint64_t Blo = s_base[0] & ~15ull;
    uint32_t* stg = (uint32_t*)s_stage;
#pragma unroll
    for (int k = 0; k < WF_R; ++k) {
        const uint64_t j = j0 + (uint64_t)k * WAL_T + threadIdx.x;
        if (j >= K) continue;
        const uint32_t q = (uint32_t)k * WAL_T + threadIdx.x;
        const uint64_t ostart = s_base[0] + wb[k] + wi[k] - wo[k];  // this record's piece (version byte first if nw)
        if (j + 1 == K) {
            tail[0] = ostart + wo[k];  // output bytes of the whole call
            tail[1] = r[k].size - r[k].strip;
            tail[2] = r[k].klen - r[k].strip;
            tail[4] = d1[k];           // deletes of all records
        }
        if (nw[k] && p0[k] != ~0ull) tlist[p0[k]].W = ostart;
        // the output piece: [version byte,] marker, new key_len, then the record body past the prefix
        const uint32_t nk = r[k].klen - r[k].strip;
        const uint64_t h5 = (uint64_t)r[k].marker | ((uint64_t)(nk >> 24) << 8) | ((uint64_t)((nk >> 16) & 0xFF) << 16) |
                            ((uint64_t)((nk >> 8) & 0xFF) << 24) | ((uint64_t)(nk & 0xFF) << 32);
        const uint64_t hd = nw[k] ? (1ull | (h5 << 8)) : h5;
        const uint32_t hn = nw[k] ? 6u : 5u;
        const uintptr_t sa = (uintptr_t)rp[k] + 5 + r[k].strip;
        if (staged) {
            const uint32_t d = (uint32_t)(ostart - Blo), db = d + hn;
            const uint64_t L = r[k].size - 5 - r[k].strip;
            lds_or16(stg, d, make_uint4((uint32_t)hd, (uint32_t)(hd >> 32), 0u, 0u), hn);
            if (pre[k]) {
                const uint32_t s0 = (uint32_t)(sa & 15);
#pragma unroll
                for (int i = 0; i < WF_NB; ++i) {
                    const uint64_t gs = 16 * (uint64_t)i;  // block i's first byte, relative to sa's block
                    if (gs >= s0 + L) break;
                    const uint32_t lb = i == 0 ? s0 : 0u;
                    const uint32_t hb = (uint32_t)(s0 + L - gs < 16 ? s0 + L - gs : 16);
                    lds_or16(stg, (uint32_t)(db + gs + lb - s0), i == 0 ? funnel16(pb[k][0], make_uint4(0, 0, 0, 0), s0) : pb[k][i],
                             hb - lb);
                }
            } else {
                for (uint64_t o = 0; o < L; o += 16) {
                    const uint32_t m = (uint32_t)(L - o < 16 ? L - o : 16);
                    lds_or16(stg, (uint32_t)(db + o), load_window16((const uint8_t*)sa + o, m), m);
                }
            }
        } else {
            os[q] = ostart;
            src[q] = sa;
            head[q] = hd;
            hl[q] = (uint8_t)hn;
            if (q + 1 == c) os[q + 1] = ostart + wo[k];
        }
    }
    if (staged) {
        __syncthreads();
        if (SKV_WAL_PROBE & 2) return;
        const uint64_t lo = s_base[0], hi = lo + wt, Bhi = (hi + 15) & ~15ull;
        for (uint64_t B = Blo + 16ull * threadIdx.x; B < Bhi; B += 16ull * WAL_T) {
            const uint64_t x0 = B > lo ? B : lo, x1 = B + 16 < hi ? B + 16 : hi;
            const uint4 v = s_stage[(B - Blo) >> 4];
            if (x0 == B && x1 == B + 16) {
                *(uint4*)(out + B) = v;
            } else {  // span edge: this workgroup's bytes only
                for (uint64_t y = x0; y < x1; ++y) out[y] = (uint8_t)byte_of(v, (uint32_t)(y - B));
            }
        }
        return;
    }
    __syncthreads();
    if (SKV_WAL_PROBE & 2) return;
    // consecutive threads compose consecutive aligned output blocks (coalesced stores; a thread per
    // record instead, its blocks in a loop, measured slower: 10.1 vs 8.9 ms at config 5)
    const uint64_t lo = os[0], hi = os[c];  // (lo = s_base: Blo as above)
    const uint64_t Bhi = (hi + 15) & ~15ull;
    // block -> piece holding its first byte (lo for the first block), marked by the pieces
    // themselves when the span fits the table; else a binary search over the pieces per block
    const uint64_t q0 = Blo >> 4;
    const bool use_tbl = (Bhi >> 4) - q0 <= WF_TBL;
    if (use_tbl) {
        if (threadIdx.x == 0) s_tbl[0] = 0;
        for (uint32_t q = threadIdx.x; q < c; q += WAL_T) {
            uint64_t qs = (os[q] + 15) >> 4;
            const uint64_t qe = (os[q + 1] + 15) >> 4;
            if (qs <= q0) qs = q0 + 1;
            for (uint64_t b = qs; b < qe; ++b) s_tbl[b - q0] = (uint16_t)q;
        }
        __syncthreads();
    }
    for (uint64_t B = Blo + 16ull * threadIdx.x; B < Bhi; B += 16ull * WAL_T) {
        const uint64_t x0 = B > lo ? B : lo, x1 = B + 16 < hi ? B + 16 : hi;
        uint32_t a = 0;  // last record with os <= x0
        if (use_tbl) {
            a = s_tbl[(B >> 4) - q0];
        } else {
            uint32_t bb = c;
            while (bb - a > 1) {
                const uint32_t mid = (a + bb) >> 1;
                if (os[mid] <= x0) a = mid;
                else bb = mid;
            }
        }
        const uint4 v = wal_compose(B, x0, x1, a, os, src, head, hl);
        if (x0 == B && x1 == B + 16) {
            *(uint4*)(out + B) = v;
        } else {  // span edge: this workgroup's bytes only
            for (uint64_t y = x0; y < x1; ++y) out[y] = (uint8_t)byte_of(v, (uint32_t)(y - B));
        }
    }
}

void launch_wal_fused(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint64_t* m_src, const uint64_t* P,
                      const uint64_t* Dp, uint8_t* out, uint64_t* tstate, uint32_t* ticket, uint32_t* fail,
                      WalTStart* tlist, uint32_t* tcount, uint32_t tcap, uint64_t* tail, uint32_t diag,
                      const SElem* S, const uint32_t* m_rec) {
    if (max_K)
        k_wal_fused<<<wal_blocks(max_K, WF_G), WAL_T, 0, s>>>(Kp, m_src, P, Dp, out, tstate, ticket, fail, tlist,
                                                               tcount, tcap, tail, diag, S, m_rec);
}

void launch_wal_keys(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint64_t* m_src, const uint64_t* P,
                     int64_t* tid, uint32_t* strip, uint32_t* wnk, uint64_t* wsize, uint8_t* canon,
                     unsigned long long* first_err) {
    if (max_K)
        k_wal_keys<<<wal_blocks(max_K, 256), 256, 0, s>>>(Kp, m_src, P, tid, strip, wnk, wsize, canon, first_err);
}
void launch_wal_flags(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const int64_t* tid, const uint32_t* strip,
                      const uint8_t* canon, const uint64_t* m_src, const uint32_t* wnk, uint64_t* is_new, uint32_t* bad,
                      bool exact) {
    if (max_K)
        k_wal_flags<<<wal_blocks(max_K, 256), 256, 0, s>>>(Kp, tid, strip, canon, m_src, wnk, is_new, bad,
                                                           exact ? 1u : 0u);
}
void launch_wal_index(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint64_t* is_new, const uint64_t* new_ex,
                      const uint32_t* bad, uint32_t* tix, uint64_t* tstart, uint32_t* tbad,
                      unsigned long long* tfirst) {
    if (max_K) k_wal_index<<<wal_blocks(max_K, 256), 256, 0, s>>>(Kp, is_new, new_ex, bad, tix, tstart, tbad, tfirst);
}
void launch_wal_tables(hipStream_t s, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart, const uint64_t* Pw,
                       const uint32_t* tbad, uint64_t max_size, uint64_t* run_len, uint64_t* keep) {
    if (max_NT) k_wal_tables<<<wal_blocks(max_NT, 256), 256, 0, s>>>(NTp, tstart, Pw, tbad, max_size, run_len, keep);
}
void launch_wal_desc(hipStream_t s, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart, const uint64_t* Pw,
                     const uint64_t* Dp, const uint64_t* keep, const uint64_t* keep_ex, const uint64_t* run_off,
                     const int64_t* tid, const uint32_t* wnk, DevRunDesc* descs) {
    if (max_NT)
        k_wal_desc<<<wal_blocks(max_NT, 256), 256, 0, s>>>(NTp, tstart, Pw, Dp, keep, keep_ex, run_off, tid, wnk,
                                                           descs);
}
void launch_wal_gather(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint32_t* tix, const uint64_t* tstart,
                       const uint64_t* keep, const uint64_t* run_off, const uint64_t* Pw, const uint32_t* strip,
                       const uint64_t* m_src, const uint32_t* wnk, const uint8_t* canon, uint8_t* out) {
    if (max_K)
        k_wal_gather<<<wal_blocks(max_K, WAL_G), WAL_G, 0, s>>>(Kp, tix, tstart, keep, run_off, Pw, strip, m_src,
                                                                wnk, canon, out);
}

}  // namespace skv
