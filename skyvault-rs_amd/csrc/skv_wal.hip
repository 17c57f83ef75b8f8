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
constexpr int WAL_G = 256;
static_assert(WAL_G == (int)WAL_FUSED_G, "k_wal_fused's workgroup size (host look-back sizing)");

// bytes [x0, x1) of output block B, starting inside kept record r
__device__ uint4 wal_compose(uint64_t B, uint64_t x0, uint64_t x1, uint32_t r, const uint64_t* os,
                             const uint64_t* src, const uint64_t* head, const uint32_t* hl) {
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

constexpr uint32_t WF_BADKEY = 1, WF_ORDER = 2, WF_TABLES = 4;
constexpr uint32_t WF_TBL = 4096;  // output blocks of a workgroup's span with a piece table (64 KiB)
static_assert(WAL_G <= 256, "piece ids in the block table are bytes");
struct WalPrev {
    int64_t tid;
    uint64_t size, rp;
    uint32_t strip, klen;
    bool canon;
};

__global__ void __launch_bounds__(WAL_G) k_wal_fused(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ m_src,
                                                     const uint64_t* __restrict__ P, const uint64_t* __restrict__ Dp,
                                                     uint8_t* out, uint64_t* tstate, uint32_t* ticket, uint32_t* fail,
                                                     WalTStart* tlist, uint32_t* tcount, uint32_t tcap,
                                                     uint64_t* tail, uint32_t diag,
                                                     const SElem* __restrict__ S, const uint32_t* __restrict__ m_rec) {
    __shared__ uint64_t os[WAL_G + 1], src[WAL_G], head[WAL_G];
    __shared__ uint32_t hl[WAL_G];
    __shared__ uint64_t s_w[WAL_G / 64], s_base[1];
    __shared__ WalPrev s_prev[WAL_G / 64];  // each wave's last record, for the next wave's lane 0
    __shared__ uint8_t s_tbl[WF_TBL];
    __shared__ uint32_t s_t;
    const uint64_t K = *Kp;
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t t = s_t;
    const uint64_t j0 = t * WAL_G;
    if (j0 >= K) return;  // (tickets past the last workgroup: nothing to publish)
    const uint64_t j = j0 + threadIdx.x;
    const bool live = j < K;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WalRec r{};
    const uint8_t* rp = nullptr;
    uint32_t bad = 0;
    if (live) {
        rp = (const uint8_t*)m_src[j];
        bool ok = false;
        if (S) {  // the record sort's element: its key prefix, no record line read for the parse
            const SElem e = S[m_rec[j]];
            r = wal_parse_pfx(e.hi, e.lo, e.klen, Dp[j + 1] != Dp[j] ? 2u : 1u, P[j + 1] - P[j], ok);
        }
        if (!ok) r = wal_parse(rp, P[j + 1] - P[j]);
        if (r.err || ((diag & WAL_STRICT_CANON) && !r.canon)) bad |= WF_BADKEY;
    }
    // the record before: the neighbouring lane; a wave's lane 0 takes the previous wave's last lane
    // through LDS, and only the workgroup's first record parses its predecessor again
    if (lane == 63) {
        s_prev[wv].tid = r.tid;
        s_prev[wv].strip = r.strip;
        s_prev[wv].klen = r.klen;
        s_prev[wv].canon = r.canon;
        s_prev[wv].size = r.size;
        s_prev[wv].rp = (uint64_t)rp;
    }
    __syncthreads();
    int64_t ptid = __shfl_up(r.tid, 1, 64);
    uint32_t pstrip = __shfl_up(r.strip, 1, 64), pklen = __shfl_up(r.klen, 1, 64);
    bool pcanon = __shfl_up(r.canon ? 1 : 0, 1, 64) != 0;
    uint64_t psize = __shfl_up(r.size, 1, 64);
    const uint8_t* prp = (const uint8_t*)__shfl_up((uint64_t)rp, 1, 64);
    if (lane == 0 && wv > 0) {
        const WalPrev& q = s_prev[wv - 1];
        ptid = q.tid;
        pstrip = q.strip;
        pklen = q.klen;
        pcanon = q.canon;
        psize = q.size;
        prp = (const uint8_t*)q.rp;
    }
    if (live && threadIdx.x == 0 && j > 0) {
        prp = (const uint8_t*)m_src[j - 1];
        const WalRec q = wal_parse(prp, P[j] - P[j - 1]);
        ptid = q.tid;
        pstrip = q.strip;
        pklen = q.klen;
        pcanon = q.canon;
        psize = q.size;
        if (q.err) bad |= WF_BADKEY;
    }
    const bool nw = live && (j == 0 || ptid != r.tid);
    if (live && !nw && !(pcanon && r.canon)) {  // stripped keys must ascend inside a table
        const uint8_t* ka = prp + 5 + pstrip;
        const uint8_t* kb = rp + 5 + r.strip;
        const uint64_t la = pklen - pstrip, lb = r.klen - r.strip;
        const uint64_t n = la < lb ? la : lb;
        int c = bytes_cmp16(ka, kb, n);
        if (!c) c = la < lb ? -1 : (la > lb ? 1 : 0);
        if (c >= 0) bad |= WF_ORDER;
    }
    if (bad) atomicOr(fail, bad);
    const uint64_t ws = live ? r.size - r.strip : 0;
    // output bytes of record j: its version byte (a table start) + its stripped record. The exclusive
    // prefix of those is where its piece starts, and a table's version byte sits where its first
    // record's piece starts, so one sum places everything (no separate table-start count).
    const uint64_t wo = ws + (nw ? 1 : 0);
    uint64_t wi = wo;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t a = __shfl_up(wi, d, 64);
        if (lane >= d) wi += a;
    }
    if (lane == 63) s_w[wv] = wi;
    __syncthreads();
    uint64_t wb = 0, wt = 0;
    for (int w = 0; w < WAL_G / 64; ++w) {
        if (w < wv) wb += s_w[w];
        wt += s_w[w];
    }
    // decoupled look-back over workgroups (ticket order); wave 0 reads 64 predecessors per step --
    // workgroups are short, so chains of aggregates are long
    if (threadIdx.x < 64) {
        constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62, VM = FA - 1;
        uint64_t acc = 0;
        if (t == 0) {
            if (lane == 0) __hip_atomic_store(&tstate[0], FI | wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&tstate[t], FA | wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t top = (int64_t)t - 1;
            for (;;) {
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
    const uint64_t ostart = s_base[0] + wb + wi - wo;  // this record's piece (version byte first if nw)
    if (live && j + 1 == K) {
        tail[0] = ostart + wo;  // output bytes of the whole call
        tail[1] = ws;
        tail[2] = r.klen - r.strip;
        tail[4] = Dp[j + 1];    // deletes of all records
    }
    if (nw) {
        const uint32_t e = atomicAdd(tcount, 1u);
        if (e < tcap) {
            WalTStart x;
            x.b = j;
            x.W = ostart;
            x.Dp = Dp[j];
            x.tid = r.tid;
            x.nk = r.klen - r.strip;
            x.prev_nk = j ? pklen - pstrip : 0;
            x.prev_ws = j ? psize - pstrip : 0;
            tlist[e] = x;
        } else {
            atomicOr(fail, WF_TABLES);
        }
    }
    // the output pieces: [version byte,] marker, new key_len, then the record body past the prefix
    if (live) {
        const uint32_t nk = r.klen - r.strip;
        const uint64_t h5 = (uint64_t)r.marker | ((uint64_t)(nk >> 24) << 8) | ((uint64_t)((nk >> 16) & 0xFF) << 16) |
                            ((uint64_t)((nk >> 8) & 0xFF) << 24) | ((uint64_t)(nk & 0xFF) << 32);
        os[threadIdx.x] = ostart;
        src[threadIdx.x] = (uint64_t)rp + 5 + r.strip;
        head[threadIdx.x] = nw ? (1ull | (h5 << 8)) : h5;
        hl[threadIdx.x] = nw ? 6u : 5u;
        if (j + 1 == K || threadIdx.x + 1 == WAL_G) os[threadIdx.x + 1] = ostart + wo;
    }
    __syncthreads();
    // consecutive threads compose consecutive aligned output blocks (coalesced stores; a thread per
    // record instead, its blocks in a loop, measured slower: 10.1 vs 8.9 ms at config 5)
    const uint32_t c = (uint32_t)(K - j0 < WAL_G ? K - j0 : WAL_G);
    const uint64_t lo = os[0], hi = os[c];
    const uint64_t Blo = lo & ~15ull, Bhi = (hi + 15) & ~15ull;
    // block -> piece holding its first byte (lo for the first block), marked by the pieces
    // themselves when the span fits the table; else a binary search over the pieces per block
    const uint64_t q0 = Blo >> 4;
    const bool use_tbl = (Bhi >> 4) - q0 <= WF_TBL;
    if (use_tbl) {
        if (live) {
            uint64_t qs = (ostart + 15) >> 4;
            const uint64_t qe = (ostart + wo + 15) >> 4;
            if (threadIdx.x == 0) s_tbl[0] = 0;
            if (qs <= q0) qs = q0 + 1;
            for (uint64_t q = qs; q < qe; ++q) s_tbl[q - q0] = (uint8_t)threadIdx.x;
        }
        __syncthreads();
    }
    for (uint64_t B = Blo + 16ull * threadIdx.x; B < Bhi; B += 16ull * WAL_G) {
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
    // SKV_WAL_LDS=<bytes>: pad the workgroup's LDS request (caps workgroups per CU: a smaller set of
    // record lines in flight per XCD, so the composition's re-read can hit L2; occupancy studies)
    if (max_K)
        k_wal_fused<<<wal_blocks(max_K, WAL_G), WAL_G, 0, s>>>(Kp, m_src, P, Dp, out, tstate, ticket, fail, tlist,
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
