// skv_kernels.hip — HIP/CDNA4 (gfx950) kernels of the skyvault compaction path.
//
// Pipeline (one compaction; host orchestration in skv_compact.hip):
//   parse   k_run_header, k_spec, k_validate, k_fixup, k_err_chunk, k_mask, scan, k_run_summary,
//           k_emit           — runs::read_run_stream (runs.rs:517-628) for every input run at once
//   check   k_order_check    — first in-stream key decrease (what build_runs rejects, runs.rs:190-198)
//   merge   k_sample, k_bounds, k_tile_n, k_tile<L0> (level 0 emits the merged arrays)
//                            — k_way::merge (k_way.rs:113-179): order by (key asc, seq_no desc),
//                              keep the first record per key, drop Deletes at Level::max
//                              (table_tree_compaction.rs:139-145)
//   chain   k_chain, k_run_stats — build_runs' greedy size split + StatsV1 (runs.rs:202-280)
//   gather  k_gather         — output bytes: version byte per run + surviving records verbatim
//
// Everything is integer/byte work: no MFMA. The HBM-bound kernel is k_gather (reads the
// surviving input records once, writes the output once, 16-byte vector stores).
#include "skv_launch.hpp"

namespace skv {

// ---------------------------------------------------------------------------------------
// small helpers

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// exclusive scan across the block (blockDim multiple of 64, <= 1024); ws: >= 16 T of LDS
template <typename T>
__device__ T block_excl_scan(T v, T* ws, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_incl_scan(v);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        T w = lane < nw ? ws[lane] : (T)0;
        w = wave_incl_scan(w);
        if (lane < nw) ws[lane] = w;
    }
    __syncthreads();
    T off = wid ? ws[wid - 1] : (T)0;
    total = ws[nw - 1];
    __syncthreads();
    return off + inc - v;
}

template <typename T>
__device__ T block_reduce_sum(T v, T* ws) {
    T total;
    block_excl_scan(v, ws, total);
    return total;
}

// last index i in [0, n) with a[i] <= x (a sorted ascending, a[0] <= x assumed)
template <typename T>
__device__ __forceinline__ uint32_t upper_idx(const T* a, uint32_t n, T x) {
    uint32_t lo = 0, hi = n;  // answer in [lo, hi)
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t find_run(const RunInfo* runs, uint32_t n_runs, uint64_t c) {
    uint32_t lo = 0, hi = n_runs;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (runs[mid].chunk_base <= c) lo = mid;
        else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------------------
// parse: run headers (runs.rs:537-556)

// Header checks (runs.rs:537-556) and the run's fixed-stride hypothesis: when the first record is
// a Put of size S and the body is a whole number of S-byte records, every chunk can verify its
// records at their predicted positions with independent loads (k_spec), and the records can be
// emitted one thread per record (k_emit_fixed). The hypothesis is verified record by record.
// slices: key-range slices of runs (pipelined host calls): the byte before a slice's first record
// stands in for the version byte and is not checked (the host walked the run's framing)
__global__ void k_run_header(const RunInfo* runs, uint32_t n_runs, uint32_t* hdr_err, RunFmt* fmt, bool slices) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_runs) return;
    RunInfo R = runs[r];
    uint32_t e = 0;
    RunFmt f{0, 0, 0, 0};
    const uint8_t* run = (const uint8_t*)R.ptr;
    if (R.len == 0) e = DERR_EMPTY;
    else {
        uint32_t v = slices ? 1u : run[0];
        if (v != 1) e = DERR_VERSION | (v << 8);
        else if (R.len >= 2) {
            RecHdr h = parse_rec<false>(run, R.len, 1);
            if (!h.err) f.first = h.size;
            if (!h.err && h.marker == 1 && (R.len - 1) % h.size == 0 && h.klen <= 0xFFFFFFFFu) {
                f.S = h.size;
                f.K = (uint32_t)h.klen;
                f.V = (uint32_t)(h.size - 9 - h.klen);
            }
        }
    }
    hdr_err[r] = e;
    fmt[r] = f;
}

// Speculative start of chunk `local` (> 0): a record start must lie in [cs, ce). Scan for the
// first position whose next three records decode cleanly. Wrong guesses are caught by
// k_validate and repaired by k_fixup.
template <int UTF8, class L = GLoad>
__device__ uint64_t spec_start(const uint8_t* run, uint64_t len, uint64_t cs, uint64_t ce, L ld = L()) {
    for (uint64_t p0 = cs; p0 < ce; p0 += 16) {  // 16 bytes per load; marker candidates as a mask
        const uint32_t m = (uint32_t)(ce - p0 < 16 ? ce - p0 : 16);
        const uint4 v = load_window16(run + p0, m, ld);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t cand = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t b = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            if ((b == 1u || b == 2u) && (uint32_t)i < m) cand |= 1u << i;
        }
        while (cand) {
            const uint32_t i = __builtin_ctz(cand);
            cand &= cand - 1;
            // candidates are checked with the keys (the heuristic form in the structure-only mode),
            // which rejects random bytes taken for a record far more often than structure alone
            const WalkRes r = walk_fast<UTF8 ? 1 : 2>(run, len, p0 + i, len, 3, ld);
            if (r.err == DERR_NONE) return p0 + i;
        }
    }
    return NO_POS;
}

template <class L = GLoad>
__device__ __forceinline__ bool fixed_rec_ok(const uint8_t* run, uint64_t len, uint64_t q, const RunFmt& f,
                                             L ld = L()) {
    uint32_t w[8];
    window32(run, len, q, w, ld);
    if ((w[0] & 0xFFu) != 1u) return false;
    uint32_t klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], 1));
    if (klen != f.K) return false;
    uint32_t kd[7];
    win_key(w, kd);
    bool ok = f.K <= 27 ? ascii_prefix(kd, f.K) : false;
    if (!ok && !utf8_valid_fast(run + q + 5, f.K, ld)) return false;
    uint32_t vo = 5 + f.K;
    uint32_t vlen;
    if (vo + 4 <= 32) vlen = win_be32(w, vo);
    else vlen = __builtin_bswap32(load_window16(run + q + vo, 4, ld).x);
    return vlen == f.V;
}

template <int UTF8>
__global__ void k_spec(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                       const uint32_t* __restrict__ hdr_err, const RunFmt* __restrict__ fmt, uint32_t* run_broken,
                       uint64_t* ch_start, uint64_t* ch_end, uint32_t* ch_cnt, uint32_t* ch_err, uint64_t chunk,
                       uint16_t* slots, uint32_t cap, StgRec* stg, uint32_t scap, uint8_t* ch_stg) {
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    ch_stg[c] = 0;  // (a walked chunk's records are staged)
    uint32_t r = find_run(runs, n_runs, c);
    RunInfo R = runs[r];
    uint64_t local = c - R.chunk_base;
    const uint8_t* run = (const uint8_t*)R.ptr;
    uint64_t cs = 1 + local * chunk;
    uint64_t ce = cs + chunk < R.len ? cs + chunk : R.len;
    if (hdr_err[r]) {
        ch_start[c] = cs;
        ch_end[c] = cs;
        ch_cnt[c] = 0;
        ch_err[c] = 0;
        return;
    }
    uint64_t start;
    const RunFmt f = fmt[r];
    if (f.S) {
        // fixed stride: the records starting in this chunk sit at p0, p0+S, ...; verify each with
        // independent loads (no dependent walk)
        const uint64_t S = f.S;
        const uint64_t p0 = 1 + ((cs - 1 + S - 1) / S) * S;
        if (p0 >= ce) {
            ch_start[c] = p0;
            ch_end[c] = p0;
            ch_cnt[c] = 0;
            ch_err[c] = 0;
            return;
        }
        const uint64_t n = (ce - p0 + S - 1) / S;
        bool ok = true;
        for (uint64_t i = 0; i < n; i += 4) {
            bool o0 = fixed_rec_ok(run, R.len, p0 + i * S, f);
            bool o1 = i + 1 < n ? fixed_rec_ok(run, R.len, p0 + (i + 1) * S, f) : true;
            bool o2 = i + 2 < n ? fixed_rec_ok(run, R.len, p0 + (i + 2) * S, f) : true;
            bool o3 = i + 3 < n ? fixed_rec_ok(run, R.len, p0 + (i + 3) * S, f) : true;
            ok = ok && o0 && o1 && o2 && o3;
        }
        if (ok) {
            ch_start[c] = p0;
            ch_end[c] = p0 + n * S;
            ch_cnt[c] = (uint32_t)n;
            ch_err[c] = 0;
            // k_emit reads these when another chunk breaks the run's hypothesis
            uint16_t* sl = slots + c * cap;
            for (uint64_t i = 0; i < n && i < cap; ++i) sl[i] = (uint16_t)(p0 + i * S - cs);
            return;
        }
        // hypothesis broken: this run takes the general path, from a speculative start like any
        // variable-size run (p0 is only right for a run that is fixed-stride up to some fault; for a
        // variable run whose first record size happens to divide its body -- ~1 run in 300 of
        // config 3 -- every chunk's p0 missed the chain and k_fixup walked the whole run: 95 ms)
        atomicOr(&run_broken[r], 1u);
        start = local == 0 ? 1 : spec_start<UTF8>(run, R.len, cs, ce);
    } else {
        start = local == 0 ? 1 : spec_start<UTF8>(run, R.len, cs, ce);
    }
    if (start == NO_POS) {
        ch_start[c] = NO_POS;
        ch_end[c] = NO_POS;
        ch_cnt[c] = 0;
        ch_err[c] = 0;
        return;
    }
    const WalkRes w = walk_fast<UTF8, true>(run, R.len, start, ce, 0xFFFFFFFFu, GLoad(), slots + c * cap, cap, cs,
                                            stg + stg_base(c, scap), scap);
    ch_stg[c] = w.nst == w.cnt ? 1 : 0;
    ch_start[c] = start;
    ch_end[c] = w.end;
    ch_cnt[c] = w.cnt;
    ch_err[c] = w.err;
}

// A chunk is "bad" when its speculative start is not the exit of its predecessor.
__global__ void k_validate(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                           const uint32_t* __restrict__ hdr_err, const uint64_t* ch_start,
                           const uint64_t* ch_end, const uint32_t* ch_err, unsigned long long* bad_bits,
                           uint32_t* run_first_bad) {
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    uint32_t r = find_run(runs, n_runs, c);
    RunInfo R = runs[r];
    uint64_t local = c - R.chunk_base;
    if (local == 0 || hdr_err[r]) return;
    bool ok = ch_err[c - 1] == 0 && ch_end[c - 1] == ch_start[c];
    if (!ok) {
        atomicOr(&bad_bits[c >> 6], 1ull << (c & 63));
        atomicMin(&run_first_bad[r], (uint32_t)local);
    }
}

__device__ uint64_t next_bad(const unsigned long long* bits, uint64_t from, uint64_t to) {
    uint64_t c = from;
    while (c < to) {
        unsigned long long w = bits[c >> 6] >> (c & 63);
        if (w) {
            uint64_t r = c + __builtin_ctzll(w);
            return r < to ? r : to;
        }
        c = (c | 63) + 1;
    }
    return to;
}

// Repair of each run's bad chunks from the true chain (exact; rare on real data): one wave per run,
// its bad chunks in order. A bad chunk is re-speculated across the wave -- lane l takes 1/64 of it,
// lane 0 from the true start E, the others from a speculative start in their sub-range (as k_spec
// does over chunks) -- the links are checked in lane order (a lane whose start is not its
// predecessor's end walks again from that end), and the starts are written at their scanned
// offsets. (One lane walking a whole 64 KiB chunk took 0.8 ms at 3F for 51 bad chunks.)
template <int UTF8>
__device__ void fix_chunk(const uint8_t* run, uint64_t len, uint64_t E, uint64_t cs, uint64_t ce, uint16_t* sl,
                          uint32_t cap, uint64_t& end, uint32_t& cnt, uint32_t& err) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t sub = (ce - cs + 63) / 64;
    const uint64_t lo = cs + sub * lane < ce ? cs + sub * lane : ce;
    const uint64_t hi = lane == 63 || lo + sub > ce ? ce : lo + sub;
    uint64_t st = lane == 0 ? E : (lo < hi ? spec_start<UTF8>(run, len, lo, hi) : hi);
    WalkRes w{st, 0, 0};
    if (st != NO_POS && st < hi) w = walk_fast<UTF8>(run, len, st, hi, 0xFFFFFFFFu);
    else if (st != NO_POS) w = WalkRes{st, 0, 0};
    uint32_t last = 63;  // the last lane on the true chain
    for (uint32_t l = 1; l < 64; ++l) {  // wave-uniform: every value below is a shuffle result
        const uint32_t perr = __shfl(w.err, l - 1, 64);
        if (perr) {
            last = l - 1;
            break;
        }
        const uint64_t pe = __shfl(w.end, l - 1, 64);
        if (__shfl(st, l, 64) != pe && lane == l) {  // walk again from the true chain's position
            st = pe;
            w = pe < hi ? walk_fast<UTF8>(run, len, pe, hi, 0xFFFFFFFFu) : WalkRes{pe, 0, 0};
        }
    }
    const uint32_t mine = lane <= last ? w.cnt : 0u;
    uint32_t ex = mine;  // inclusive scan of the counts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(ex, d, 64);
        if (lane >= (uint32_t)d) ex += v;
    }
    cnt = __shfl(ex, 63, 64);
    end = __shfl(w.end, last, 64);
    err = __shfl(w.err, last, 64);
    ex -= mine;
    if (mine && ex < cap) {  // the starts of this lane's records at their chunk positions
        uint64_t p = st;
        for (uint32_t i = 0; i < mine && ex + i < cap; ++i) {
            sl[ex + i] = (uint16_t)(p - cs);
            p += parse_rec<false, UTF8>(run, len, p).size;
        }
    }
}

__global__ void __launch_bounds__(64) k_fixup(const RunInfo* __restrict__ runs, uint32_t n_runs, const uint32_t* __restrict__ hdr_err,
                        const uint32_t* __restrict__ run_first_bad, const unsigned long long* __restrict__ bad_bits,
                        uint64_t* ch_start, uint64_t* ch_end, uint32_t* ch_cnt, uint32_t* ch_err, bool utf8,
                        uint64_t chunk, uint16_t* slots, uint32_t cap, uint8_t* ch_stg) {
    const uint32_t r = blockIdx.x;  // one wave per run
    if (r >= n_runs) return;
    const uint32_t fb = run_first_bad[r];
    if (fb == NO_POS32 || hdr_err[r]) return;
    const RunInfo R = runs[r];
    const uint8_t* run = (const uint8_t*)R.ptr;
    const uint64_t n = R.n_chunks, base = R.chunk_base;
    uint64_t c = fb;
    while (c < n) {
        const uint64_t g = base + c;
        if (ch_err[g - 1]) break;  // a real error in a valid chunk ends the run
        const uint64_t E = ch_end[g - 1];
        const uint64_t cs = 1 + c * chunk;
        const uint64_t ce = cs + chunk < R.len ? cs + chunk : R.len;
        uint64_t end = E;
        uint32_t cnt = 0, err = 0;
        if (E < ce) {
            uint16_t* sl = slots + g * cap;
            if (utf8) fix_chunk<1>(run, R.len, E, cs, ce, sl, cap, end, cnt, err);
            else fix_chunk<0>(run, R.len, E, cs, ce, sl, cap, end, cnt, err);
        }
        __syncthreads();  // (every lane's reads of this chunk's old state are done)
        if (threadIdx.x == 0) {
            ch_stg[g] = 0;  // (k_emit parses a repaired chunk from its record starts)
            ch_start[g] = E;
            ch_end[g] = end;
            ch_cnt[g] = cnt;
            ch_err[g] = err;
        }
        __syncthreads();
        if (err) break;
        ++c;
        if (c >= n) break;
        if (ch_start[base + c] == end) c = next_bad(bad_bits, base + c + 1, base + n) - base;
    }
}

__global__ void k_err_chunk(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                            const uint32_t* __restrict__ hdr_err, const uint32_t* __restrict__ ch_err,
                            uint32_t* run_err_chunk) {
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    if (!ch_err[c]) return;
    uint32_t r = find_run(runs, n_runs, c);
    if (hdr_err[r]) return;
    atomicMin(&run_err_chunk[r], (uint32_t)(c - runs[r].chunk_base));
}

__global__ void k_mask(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                       const uint32_t* __restrict__ hdr_err, const uint32_t* __restrict__ run_err_chunk,
                       const uint32_t* __restrict__ ch_cnt, uint64_t* cnt64) {
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    uint32_t r = find_run(runs, n_runs, c);
    uint64_t local = c - runs[r].chunk_base;
    uint32_t ec = run_err_chunk[r];
    cnt64[c] = (hdr_err[r] || (ec != NO_POS32 && local > ec)) ? 0 : ch_cnt[c];
}

__global__ void k_run_summary(const RunInfo* __restrict__ runs, uint32_t n_runs, const uint32_t* __restrict__ hdr_err,
                              const uint32_t* __restrict__ run_err_chunk, const uint32_t* __restrict__ ch_err,
                              const uint64_t* __restrict__ ch_rec_base, RunSummary* out, uint64_t* run_recb) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_runs) return;
    RunInfo R = runs[r];
    RunSummary s;
    s.records = ch_rec_base[R.chunk_base + R.n_chunks] - ch_rec_base[R.chunk_base];
    uint32_t ec = run_err_chunk[r];
    s.err = hdr_err[r] ? hdr_err[r] : (ec != NO_POS32 ? ch_err[R.chunk_base + ec] : 0u);
    s.pad = 0;
    out[r] = s;
    run_recb[r] = ch_rec_base[R.chunk_base];
    if (r == n_runs - 1) run_recb[n_runs] = ch_rec_base[R.chunk_base + R.n_chunks];
}

__device__ __forceinline__ void put_rec(uint64_t o, const uint8_t* rp, const RecHdr& h, uint64_t* rec_addr,
                                        uint64_t* rec_hi, uint64_t* rec_lo, uint32_t* rec_klen, uint32_t* rec_meta,
                                        uint32_t* flags, uint64_t* rec_fp, uint64_t fpv) {
    rec_addr[o] = (uint64_t)rp;
    if (rec_fp) rec_fp[o] = fpv;
    rec_hi[o] = h.hi;
    rec_lo[o] = h.lo;
    rec_klen[o] = (uint32_t)h.klen;
    if (h.size >= (1ull << 31)) atomicOr(flags, 1u);  // record too large for this build
    rec_meta[o] = (uint32_t)h.size | (h.marker == 2 ? 0x80000000u : 0u);
}

// Emit the record arrays (address, 16 B key prefix, key length, meta) of every validated chunk of
// the runs that are not fixed-stride. The chunk walks (k_spec / k_fixup) left each chunk's record
// starts in its slot row, so EM_G lanes per chunk parse one record each with independent loads and
// store consecutive records side by side; a chunk with more records than slots is walked by one
// lane from its validated start.
constexpr uint32_t EM_G = 16;  // lanes per chunk
__global__ void k_emit(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                       const RunFmt* __restrict__ fmt, const uint32_t* __restrict__ run_broken,
                       const uint64_t* __restrict__ ch_start, const uint64_t* __restrict__ ch_rec_base,
                       uint64_t* __restrict__ rec_addr, uint64_t* __restrict__ rec_hi, uint64_t* __restrict__ rec_lo,
                       uint32_t* __restrict__ rec_klen, uint32_t* __restrict__ rec_meta, uint32_t* flags,
                       uint64_t* __restrict__ rec_fp, uint32_t* utf8_bad, const uint16_t* __restrict__ slots,
                       uint32_t cap, uint64_t chunk, const uint64_t* __restrict__ ch_end,
                       const uint64_t* __restrict__ stream_base, unsigned long long* first_dec,
                       const StgRec* __restrict__ stg, uint32_t scap, const uint8_t* __restrict__ ch_stg) {
    const uint64_t gi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t c = gi / EM_G;
    const uint32_t j0 = (uint32_t)(gi % EM_G);
    if (c >= n_chunks) return;
    uint64_t b0 = ch_rec_base[c], cnt = ch_rec_base[c + 1] - b0;
    if (!cnt) return;
    if (ch_stg[c] && cnt <= scap) return;  // k_emit_stg
    uint32_t r = find_run(runs, n_runs, c);
    if (fmt[r].S && !run_broken[r]) return;  // k_emit_fixed
    const uint8_t* run = (const uint8_t*)runs[r].ptr;
    const uint64_t len = runs[r].len;
    // structure validated by k_spec / k_fixup's walk; the key's UTF-8 is checked here with the
    // same loads that fingerprint it (a bad key flags the call for an exact rerun)
    auto emit = [&](uint64_t i, uint64_t p, const RecHdr& h) {
        bool ascii;
        const uint64_t fpv = key_tail_fp(run + p + 5, (uint32_t)h.klen, ascii);
        if (!(ascii && ((h.hi | h.lo) & 0x8080808080808080ull) == 0) && !utf8_valid(run + p + 5, h.klen))
            atomicOr(utf8_bad, 1u);
        put_rec(b0 + i, run + p, h, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, flags, rec_fp, fpv);
    };
    // the in-stream order check (runs.rs:190-198, k_order_check's comparison) fused in: each record
    // against the one before it in the chunk (the neighbouring lane's, through shuffles); a chunk's
    // first record against the record before it is k_chunk_order's
    const uint32_t sidx = runs[r].stream;
    const uint64_t sbase = first_dec ? stream_base[sidx] : 0;
    auto decrease = [&](uint64_t i) {  // record i - 1 of the chunk sorts after record i
        atomicMin(&first_dec[sidx], (unsigned long long)(b0 + i - 1 - sbase));
        atomicOr(flags + 1, 1u);
    };
    if (cnt > cap) {
        if (j0) return;
        uint64_t p = ch_start[c];
        RecHdr hp{};
        uint64_t pp = 0;
        for (uint64_t i = 0; i < cnt; ++i) {
            const RecHdr h = parse_rec<true, false>(run, len, p);
            emit(i, p, h);
            if (first_dec && i > 0 &&
                key_cmp(hp.hi, hp.lo, (uint32_t)hp.klen, run + pp + 5, h.hi, h.lo, (uint32_t)h.klen, run + p + 5) > 0)
                decrease(i);
            hp = h;
            pp = p;
            p += h.size;
        }
        return;
    }
    const uint64_t cs = 1 + (c - runs[r].chunk_base) * chunk;
    const uint16_t* sl = slots + c * cap;
    // A record's size is the distance to the next record start (the next slot, or the walk's end:
    // the first start past the chunk, or the failing record of an error chunk), so the emit reads
    // no value length: per record one 32-byte header window, then the key tail for the fingerprint.
    // Two records per lane per step, their loads issued together.
    const uint64_t cend = ch_end[c];
    auto hdr = [&](uint64_t p, uint64_t pn) {
        RecHdr h;
        uint32_t w[8];
        window32(run, len, p, w);
        h.marker = w[0] & 0xFFu;
        h.err = 0;
        h.klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], 1));
        uint32_t kd[7];
        win_key(w, kd);
        win_prefix(kd, h.klen, h.hi, h.lo);
        h.size = pn - p;
        return h;
    };
    // steps are uniform over the chunk's EM_G lanes (the order check shuffles inside the group)
    const uint64_t nit = (cnt + 2 * EM_G - 1) / (2 * EM_G);
    uint64_t c_hi = 0, c_lo = 0, c_ad = 0;  // lane EM_G - 1's second record of the previous step
    uint32_t c_kl = 0;
    for (uint64_t t = 0; t < nit; ++t) {
        const uint64_t i = j0 + t * 2 * EM_G, i2 = i + EM_G;
        const bool one = i < cnt, two = i2 < cnt;
        const uint64_t ia = one ? i : 0;
        const uint64_t p = cs + sl[ia];
        const uint64_t pn = ia + 1 < cnt ? cs + sl[ia + 1] : cend;
        const uint64_t q = two ? cs + sl[i2] : p;
        const uint64_t qn = two ? (i2 + 1 < cnt ? cs + sl[i2 + 1] : cend) : pn;
        const RecHdr ha = hdr(p, pn);
        const RecHdr hb = hdr(q, qn);
        if (one) emit(i, p, ha);
        if (two) emit(i2, q, hb);
        if (first_dec) {
            const uint64_t pa = (uint64_t)(uintptr_t)(run + p), pb = (uint64_t)(uintptr_t)(run + q);
            const uint32_t ka = (uint32_t)ha.klen, kb = (uint32_t)hb.klen;
            // before record i: lane j0 - 1's first record (lane 0: the carried one)
            uint64_t x_hi = __shfl_up(ha.hi, 1, EM_G), x_lo = __shfl_up(ha.lo, 1, EM_G), x_ad = __shfl_up(pa, 1, EM_G);
            uint32_t x_kl = __shfl_up(ka, 1, EM_G);
            // before record i2: lane j0 - 1's second record (lane 0: lane EM_G - 1's first record)
            uint64_t y_hi = __shfl_up(hb.hi, 1, EM_G), y_lo = __shfl_up(hb.lo, 1, EM_G), y_ad = __shfl_up(pb, 1, EM_G);
            uint32_t y_kl = __shfl_up(kb, 1, EM_G);
            const uint64_t l_hi = __shfl(ha.hi, EM_G - 1, EM_G), l_lo = __shfl(ha.lo, EM_G - 1, EM_G);
            const uint64_t l_ad = __shfl(pa, EM_G - 1, EM_G);
            const uint32_t l_kl = __shfl(ka, EM_G - 1, EM_G);
            if (j0 == 0) {
                x_hi = c_hi; x_lo = c_lo; x_ad = c_ad; x_kl = c_kl;
                y_hi = l_hi; y_lo = l_lo; y_ad = l_ad; y_kl = l_kl;
            }
            c_hi = __shfl(hb.hi, EM_G - 1, EM_G);
            c_lo = __shfl(hb.lo, EM_G - 1, EM_G);
            c_ad = __shfl(pb, EM_G - 1, EM_G);
            c_kl = __shfl(kb, EM_G - 1, EM_G);
            if (one && i > 0 &&
                key_cmp(x_hi, x_lo, x_kl, (const uint8_t*)x_ad + 5, ha.hi, ha.lo, ka, run + p + 5) > 0)
                decrease(i);
            if (two && key_cmp(y_hi, y_lo, y_kl, (const uint8_t*)y_ad + 5, hb.hi, hb.lo, kb, run + q + 5) > 0)
                decrease(i2);
        }
    }
}

// k_emit_stg: 64-record groups per wave (1 / 2 / 4 / 8 measured 3.73 / 4.12 / 4.27 / 4.90 ms at 3F)
constexpr int EMS_R = 1;
// blk_chunk[q] = the chunk holding record 64 q (k_emit_stg's starting point for a wave);
// chunk_run[c] = the run of chunk c (one search per chunk instead of one per record)
__global__ void k_blk_chunk(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                            const uint64_t* __restrict__ ch_rec_base, uint32_t* blk_chunk, uint32_t* chunk_run) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    chunk_run[c] = find_run(runs, n_runs, c);
    const uint64_t b0 = ch_rec_base[c], b1 = ch_rec_base[c + 1];
    for (uint64_t q = (b0 + 63) >> 6; (q << 6) < b1; ++q) blk_chunk[q] = (uint32_t)c;
}

// k_emit for the chunks whose walk staged every record (k_spec): the arrays are copied from the
// staged entries, one thread per record in record order, so a wave stores 64 consecutive records
// of every array (whole lines; a chunk's lanes storing 32 records each wrote 12.2 GB for 8.2 GB of
// arrays at 3F). The record itself is read only for a non-ASCII key's UTF-8 check and for the
// order check of two keys with equal prefixes.
__global__ void __launch_bounds__(256) k_emit_stg(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t R,
                           const uint64_t* __restrict__ ch_rec_base, const uint32_t* __restrict__ blk_chunk,
                           const uint32_t* __restrict__ chunk_run, uint64_t* __restrict__ rec_addr, uint64_t* __restrict__ rec_hi, uint64_t* __restrict__ rec_lo,
                           uint32_t* __restrict__ rec_klen, uint32_t* __restrict__ rec_meta, uint32_t* flags,
                           uint64_t* __restrict__ rec_fp, uint32_t* utf8_bad, const uint16_t* __restrict__ slots,
                           uint32_t cap, uint64_t chunk, const uint64_t* __restrict__ ch_end,
                           const uint64_t* __restrict__ stream_base, unsigned long long* first_dec,
                           const StgRec* __restrict__ stg, uint32_t scap, const uint8_t* __restrict__ ch_stg) {
    // XCD-aware block order (workgroup b runs on XCD b % 8): each XCD takes one contiguous eighth of
    // the records, so the staged lines a wave reads 32 bytes of (the rest: its neighbouring chunks'
    // entries) are read again from that XCD's L2 by the waves that follow (24.1 -> 7.3 GB read at 3F)
    const uint32_t nb = gridDim.x, bid = blockIdx.x, xcd = bid & 7, qn = nb >> 3, rn = nb & 7;
    const uint32_t blk = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
    // a wave takes EMS_R x 64 consecutive records
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t w0 = ((uint64_t)blk * (blockDim.x >> 6) + wv) * (64 * EMS_R);
#pragma unroll
    for (int k = 0; k < EMS_R; ++k) {
        const uint64_t o = w0 + 64 * k + lane;
        const bool inr = o < R;
        uint64_t c = 0, b0 = 0, cnt = 0;
        if (inr) {
            c = blk_chunk[o >> 6];
            while (ch_rec_base[c + 1] <= o) ++c;  // (64 consecutive records span few chunks)
            b0 = ch_rec_base[c];
            cnt = ch_rec_base[c + 1] - b0;
        }
        const bool live = inr && ch_stg[c] && cnt <= scap;  // (else k_emit / k_emit_fixed)
        const uint64_t i = o - b0;
        uint64_t hi = 0, lo = 0, ad = 0, cs = 0;
        uint32_t kl = 0, sidx = 0;
        const uint8_t* run = nullptr;
        const uint16_t* sl = nullptr;
        const StgRec* sg = nullptr;
        if (live) {
            const uint32_t r = chunk_run[c];
            run = (const uint8_t*)runs[r].ptr;
            sidx = runs[r].stream;
            cs = 1 + (c - runs[r].chunk_base) * chunk;
            sl = slots + c * cap;
            sg = stg + stg_base(c, scap);
            const uint64_t p = cs + sl[i];
            const uint64_t pn = i + 1 < cnt ? cs + sl[i + 1] : ch_end[c];
            const uint4* e = (const uint4*)(sg + i * STG_W);
            const uint4 x = e[0], y = e[1];
            hi = ((uint64_t)x.y << 32) | x.x;
            lo = ((uint64_t)x.w << 32) | x.z;
            kl = y.z & 0x7FFFFFFFu;
            ad = (uint64_t)(uintptr_t)(run + p);
            const uint64_t size = pn - p;
            rec_addr[o] = ad;
            rec_fp[o] = ((uint64_t)y.y << 32) | y.x;
            rec_hi[o] = hi;
            rec_lo[o] = lo;
            rec_klen[o] = kl;
            if (size >= (1ull << 31)) atomicOr(flags, 1u);  // record too large for this build
            rec_meta[o] = (uint32_t)size | (y.z & 0x80000000u);
            if (!y.w && !utf8_valid(run + p + 5, kl)) atomicOr(utf8_bad, 1u);
        }
        if (!first_dec) continue;
        // the in-stream order check against the record before in the chunk: the lane before holds
        // it (record o - 1), except at lane 0; a chunk's first record is k_chunk_order's
        uint64_t x_hi = __shfl_up(hi, 1, 64), x_lo = __shfl_up(lo, 1, 64), x_ad = __shfl_up(ad, 1, 64);
        uint32_t x_kl = __shfl_up(kl, 1, 64);
        if (!live || i == 0) continue;
        if (lane == 0) {
            const uint4* ep = (const uint4*)(sg + (i - 1) * STG_W);
            const uint4 x = ep[0];
            x_hi = ((uint64_t)x.y << 32) | x.x;
            x_lo = ((uint64_t)x.w << 32) | x.z;
            x_kl = ep[1].z & 0x7FFFFFFFu;
            x_ad = (uint64_t)(uintptr_t)(run + cs + sl[i - 1]);
        }
        if (key_cmp(x_hi, x_lo, x_kl, (const uint8_t*)x_ad + 5, hi, lo, kl, (const uint8_t*)ad + 5) > 0) {
            atomicMin(&first_dec[sidx], (unsigned long long)(o - 1 - stream_base[sidx]));
            atomicOr(flags + 1, 1u);
        }
    }
}

// The order check across chunk edges (k_emit's fused check): a chunk's first record against the
// record before it in its stream (records are numbered stream by stream, chunk by chunk)
__global__ void k_chunk_order(const RunInfo* __restrict__ runs, uint32_t n_runs, uint64_t n_chunks,
                              const uint64_t* __restrict__ ch_rec_base, const uint64_t* __restrict__ stream_base,
                              const uint64_t* __restrict__ rec_addr, const uint64_t* __restrict__ rec_hi,
                              const uint64_t* __restrict__ rec_lo, const uint32_t* __restrict__ rec_klen,
                              unsigned long long* first_dec, uint32_t* any_dec) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const uint64_t g = ch_rec_base[c];
    if (ch_rec_base[c + 1] == g) return;
    const uint32_t sidx = runs[find_run(runs, n_runs, c)].stream;
    if (g == stream_base[sidx]) return;  // the stream's first record
    if (key_cmp(rec_hi[g - 1], rec_lo[g - 1], rec_klen[g - 1], (const uint8_t*)rec_addr[g - 1] + 5, rec_hi[g],
                rec_lo[g], rec_klen[g], (const uint8_t*)rec_addr[g] + 5) > 0) {
        atomicMin(&first_dec[sidx], (unsigned long long)(g - 1 - stream_base[sidx]));
        atomicOr(any_dec, 1u);
    }
}

// Fixed-stride runs: one thread per record at 1 + i*S (coalesced stores, independent loads).
// VERIFY: the single-pass parse of a job whose runs are all fixed-stride — each record is parsed
// exactly as read_run_stream would (runs.rs:559-626) and must have size S, which by induction
// proves the whole run decodes to these records; any other outcome marks the run broken and
// the host reruns the general parse.
// wave_run[w] = the run holding record 64 w (the last run with run_recb <= 64 w). k_emit_fixed's
// threads then search only between their wave's first run and the next wave's: with 10^6 runs
// (config 5) a whole-table search per record was 20 dependent loads and most of the kernel.
__global__ void k_wave_run(const uint64_t* __restrict__ run_recb, uint32_t n_runs, uint64_t nw, uint32_t* wave_run) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    const uint64_t i = w << 6;
    uint32_t lo = 0, hi = n_runs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (run_recb[mid] <= i) lo = mid;
        else hi = mid;
    }
    wave_run[w] = lo;
}

template <bool VERIFY>
__global__ void k_emit_fixed(const RunInfo* __restrict__ runs, uint32_t n_runs, const uint32_t* __restrict__ wave_run,
                             uint64_t R_total,
                             const RunFmt* __restrict__ fmt, uint32_t* run_broken,
                             const uint64_t* __restrict__ run_recb, uint64_t* __restrict__ rec_addr,
                             uint64_t* __restrict__ rec_hi, uint64_t* __restrict__ rec_lo,
                             uint32_t* __restrict__ rec_klen, uint32_t* __restrict__ rec_meta, uint32_t* flags,
                             const uint64_t* __restrict__ stream_base, unsigned long long* first_dec,
                             uint64_t* __restrict__ rec_fp, SElem* __restrict__ E = nullptr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool act = i < R_total;
    // E (the record sort follows): the sort's element {prefix, address, index, key length} in place of
    // rec_hi / rec_lo / rec_addr / rec_klen -- k_sort_load's pass over them is skipped
    auto put = [&](uint64_t o, const uint8_t* rp, const RecHdr& h, uint64_t fpv) {
        if (E) {
            SElem e;
            e.hi = h.hi;
            e.lo = h.lo;
            e.addr = (uint64_t)(uintptr_t)rp;
            e.pos = (uint32_t)o;
            e.klen = (uint32_t)h.klen;
            E[o] = e;
            if (h.size >= (1ull << 31)) atomicOr(flags, 1u);
            rec_meta[o] = (uint32_t)h.size | (h.marker == 2 ? 0x80000000u : 0u);
        } else {
            put_rec(o, rp, h, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, flags, rec_fp, fpv);
        }
    };
    uint32_t lo = 0;
    RunFmt f{0, 0, 0};
    const uint8_t* run = nullptr;
    uint64_t p = 0, len = 0;
    RecHdr h{};
    if (act) {
        const uint64_t w = i >> 6, nw = (R_total + 63) >> 6;  // last run with run_recb <= i:
        uint32_t hi = n_runs;                                  // between this wave's first run
        if (wave_run) {                                        // and the next wave's
            lo = wave_run[w];
            if (w + 1 < nw) hi = wave_run[w + 1] + 1;
        }
        while (hi - lo > 1) {
            uint32_t mid = (lo + hi) >> 1;
            if (run_recb[mid] <= i) lo = mid;
            else hi = mid;
        }
        f = fmt[lo];
        if (!VERIFY && (!f.S || run_broken[lo])) act = false;
    }
    if (act) {
        run = (const uint8_t*)runs[lo].ptr;
        len = runs[lo].len;
        p = 1 + (i - run_recb[lo]) * f.S;
        h = parse_rec<true>(run, len, p);
        if (VERIFY && (h.err || h.size != f.S || h.size >= (1ull << 31))) {
            atomicOr(&run_broken[lo], 1u);
            atomicOr(flags + 2, 1u);  // poison the speculative merge
            act = false;
            // a harmless stand-in (empty key, zero size) so that the speculatively launched merge
            // never follows a garbage address; the host reruns the general parse
            RecHdr z{};
            z.marker = 1;
            put(i, run, z, 0);
        }
        if (act) {
            bool ascii;
            put(i, run + p, h, rec_fp ? key_tail_fp(run + p + 5, (uint32_t)h.klen, ascii) : 0);
        }
    }
    // a Delete of the run's record size (k_run_header's hypothesis is a Put): flags[3] bit 0, so
    // the host does not take one meta for every record (k_sort_store's const_meta)
    if (VERIFY && __ballot(act && h.marker == 2) && (threadIdx.x & 63) == 0) atomicOr(flags + 3, 1u);
    if (!VERIFY || !first_dec) return;  // (no order check for a writer batch)
    // fused order check (runs.rs:190-198 as k_order_check does it): compare with the previous
    // record of the same stream — the neighbouring lane's, or parsed here at a run / wave edge
    const int lane = threadIdx.x & 63;
    uint64_t phi = __shfl_up(h.hi, 1, 64), plo = __shfl_up(h.lo, 1, 64);
    uint64_t paddr = __shfl_up((uint64_t)(uintptr_t)(run + p), 1, 64);
    uint32_t pkl = __shfl_up((uint32_t)h.klen, 1, 64);
    uint32_t prun = __shfl_up(lo, 1, 64);
    int pact = __shfl_up(act ? 1 : 0, 1, 64);
    if (!act) return;
    const uint64_t local = i - run_recb[lo];
    if (lane == 0 || prun != lo || !pact) {
        const uint8_t* prev = nullptr;
        uint64_t pl = 0, pp = 0;
        if (local > 0) {
            prev = run;
            pl = len;
            pp = p - f.S;
        } else if (lo > 0 && runs[lo - 1].stream == runs[lo].stream) {  // L0-style concatenation
            const RunFmt pf = fmt[lo - 1];
            prev = (const uint8_t*)runs[lo - 1].ptr;
            pl = runs[lo - 1].len;
            pp = 1 + (run_recb[lo] - 1 - run_recb[lo - 1]) * pf.S;
        }
        if (!prev) return;  // first record of its stream
        RecHdr ph = parse_rec<true>(prev, pl, pp);
        phi = ph.hi;
        plo = ph.lo;
        pkl = (uint32_t)ph.klen;
        paddr = (uint64_t)(uintptr_t)(prev + pp);
    }
    const int c = key_cmp(phi, plo, pkl, (const uint8_t*)paddr + 5, h.hi, h.lo, (uint32_t)h.klen, run + p + 5);
    if (c > 0) {
        const uint32_t sidx = runs[lo].stream;
        atomicMin(&first_dec[sidx], (unsigned long long)(i - 1 - stream_base[sidx]));
        atomicOr(flags + 1, 1u);
        atomicOr(flags + 2, 1u);  // unsorted segment: poison the speculative merge
    }
}

// ---------------------------------------------------------------------------------------
// check: first key decrease inside each stream (rank order)

__global__ void k_order_check(uint64_t R, const uint64_t* __restrict__ stream_base, uint32_t k,
                              const uint64_t* __restrict__ rec_addr, const uint64_t* __restrict__ rec_hi,
                              const uint64_t* __restrict__ rec_lo, const uint32_t* __restrict__ rec_klen,
                              unsigned long long* first_dec, uint32_t* any_dec) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 || i >= R) return;
    uint32_t lo = 0, hi = k;  // stream s with base[s] <= i < base[s+1]
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (stream_base[mid] <= i) lo = mid;
        else hi = mid;
    }
    if (stream_base[lo] == i) return;
    int c = key_cmp(rec_hi[i - 1], rec_lo[i - 1], rec_klen[i - 1], (const uint8_t*)rec_addr[i - 1] + 5, rec_hi[i],
                    rec_lo[i], rec_klen[i], (const uint8_t*)rec_addr[i] + 5);
    if (c > 0) {
        atomicMin(&first_dec[lo], (unsigned long long)(i - 1 - stream_base[lo]));
        atomicOr(any_dec, 1u);
    }
}

// ---------------------------------------------------------------------------------------
// merge: recursive sampled splitters + LDS tile merge
//
// An element is (hi, lo, c) with c = key_len << 32 | rec_idx. Total order: key bytes (prefix,
// then suffix from the record when both keys exceed 16 B), key length, rec_idx — and rec_idx
// order == seq_no descending for equal keys, which is exactly HeapItem's pop order.

struct Elems {
    const uint64_t* hi;
    const uint64_t* lo;
    const uint64_t* c;       // null at level 0 (c = klen << 32 | position)
    const uint32_t* klen;    // level 0 only
    const uint32_t* poison;  // set: the speculatively parsed records are invalid (unsorted or
                             // stand-ins) -> splitter / merge kernels do nothing (see k_emit_fixed)
};

template <bool L0>
__device__ __forceinline__ void load_elem(const Elems& E, uint64_t pos, uint64_t& hi, uint64_t& lo, uint64_t& c) {
    hi = E.hi[pos];
    lo = E.lo[pos];
    c = L0 ? (((uint64_t)E.klen[pos] << 32) | pos) : E.c[pos];
}

__device__ __forceinline__ int suffix_cmp(const uint64_t* rec_addr, uint64_t ca, uint64_t cb) {
    uint32_t la = (uint32_t)(ca >> 32), lb = (uint32_t)(cb >> 32);
    if (la > 16 && lb > 16) {
        const uint8_t* a = (const uint8_t*)rec_addr[(uint32_t)ca] + 5;
        const uint8_t* b = (const uint8_t*)rec_addr[(uint32_t)cb] + 5;
        const uint32_t n = la < lb ? la : lb;
        return bytes_cmp16(a + 16, b + 16, n - 16);
    }
    return 0;
}

// key-only comparison (<0, 0, >0)
__device__ __forceinline__ int ekey_cmp(const uint64_t* rec_addr, uint64_t ha, uint64_t la_, uint64_t ca,
                                        uint64_t hb, uint64_t lb_, uint64_t cb) {
    if (ha != hb) return ha < hb ? -1 : 1;
    if (la_ != lb_) return la_ < lb_ ? -1 : 1;
    int s = suffix_cmp(rec_addr, ca, cb);
    if (s) return s;
    uint32_t la = (uint32_t)(ca >> 32), lb = (uint32_t)(cb >> 32);
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// total order (key, then rec_idx)
__device__ __forceinline__ bool elem_less(const uint64_t* rec_addr, uint64_t ha, uint64_t la_, uint64_t ca,
                                          uint64_t hb, uint64_t lb_, uint64_t cb) {
    int k = ekey_cmp(rec_addr, ha, la_, ca, hb, lb_, cb);
    if (k) return k < 0;
    return (uint32_t)ca < (uint32_t)cb;
}

// elem_less with a fingerprint shortcut (level-0 merge rounds): keys with equal prefix, length
// and fingerprint of the bytes past 16 are taken as equal (no record bytes read); both
// fingerprints come from registers / LDS. k_fp_verify checks every pair taken as equal.
__device__ __forceinline__ bool elem_less_fp(bool use_fp, uint64_t fpa, const uint64_t* rec_addr, uint64_t ha,
                                             uint64_t la_, uint64_t ca, uint64_t hb, uint64_t lb_, uint64_t cb,
                                             uint64_t fpb) {
    if (ha != hb) return ha < hb;
    if (la_ != lb_) return la_ < lb_;
    const uint32_t la = (uint32_t)(ca >> 32), lb = (uint32_t)(cb >> 32);
    if (la > 16 && lb > 16) {
        if (!(use_fp && la == lb && fpa == fpb)) {
            const int s = suffix_cmp(rec_addr, ca, cb);
            if (s) return s < 0;
        }
    }
    if (la != lb) return la < lb;
    return (uint32_t)ca < (uint32_t)cb;
}

// Key bytes 16.. of two records whose keys have one length klen (> 16): equal? 64 tail bytes of both
// per step, all eight windows loaded before any compare.
__device__ __forceinline__ bool key_tails_equal(const uint8_t* ra, const uint8_t* rb, uint32_t klen) {
    const uint8_t* ka = ra + 5 + 16;
    const uint8_t* kb = rb + 5 + 16;
    const uint32_t nt = klen > 16 ? klen - 16 : 0;
    uint32_t diff = 0;
    for (uint32_t o = 0; o < nt; o += 64) {
        uint4 x[4], y[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t m = o + 16 * w < nt ? (nt - o - 16 * w < 16 ? nt - o - 16 * w : 16) : 0;
            x[w] = m ? load_window16(ka + o + 16 * w, m) : make_uint4(0, 0, 0, 0);
            y[w] = m ? load_window16(kb + o + 16 * w, m) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t m = o + 16 * w < nt ? (nt - o - 16 * w < 16 ? nt - o - 16 * w : 16) : 0;
            diff |= ((x[w].x ^ y[w].x) & dword_mask(0, m, 0)) | ((x[w].y ^ y[w].y) & dword_mask(0, m, 1)) |
                    ((x[w].z ^ y[w].z) & dword_mask(0, m, 2)) | ((x[w].w ^ y[w].w) & dword_mask(0, m, 3));
        }
    }
    return diff == 0;
}

// The pairs k_tile<true> took as one key on equal prefix, length and fingerprint (O.vpairs: the two
// records' addresses): their bytes past 16 must be equal, else the call is rerun with exact
// compares. Every pair is independent: a grid-stride loop with all its loads in flight.
// pairs [*vlo, *vcount) (vlo null: from 0): a slice of the queue whose tiles have finished
__global__ void k_fp_verify(const unsigned long long* __restrict__ vlo, const unsigned long long* __restrict__ vcount,
                            const uint64_t* __restrict__ vpairs, uint32_t* fp_bad) {
    const uint64_t n = *vcount, n0 = vlo ? *vlo : 0;
    uint32_t bad = 0;
    for (uint64_t i = n0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* ra = (const uint8_t*)vpairs[2 * i];
        const uint8_t* rb = (const uint8_t*)vpairs[2 * i + 1];
        const uint32_t la = __builtin_bswap32(load_window16(ra + 1, 4).x);  // key_len of each record
        const uint32_t lb = __builtin_bswap32(load_window16(rb + 1, 4).x);
        bad |= la != lb || !key_tails_equal(ra, rb, la);
    }
    if (bad) atomicOr(fp_bad, 1u);
}

// fingerprints of the key bytes past 16 of the record arrays (records the emit kernels did not
// fingerprint themselves)
__global__ void k_key_fp(uint64_t R, const uint64_t* __restrict__ rec_addr, const uint32_t* __restrict__ rec_klen,
                         uint64_t* fp) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    bool ascii;
    fp[i] = key_tail_fp((const uint8_t*)rec_addr[i] + 5, rec_klen[i], ascii);
}

// samples: every S-th element of each list
template <bool L0>
__global__ void k_sample(Elems src, const uint64_t* __restrict__ off_src, const uint64_t* __restrict__ off_dst,
                         uint32_t k, uint64_t S, uint64_t n_dst, uint64_t* dhi, uint64_t* dlo, uint64_t* dc) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_dst) return;
    uint32_t lo = 0, hi = k;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (off_dst[mid] <= i) lo = mid;
        else hi = mid;
    }
    // skip empty lists sharing this offset: want the last list j with off_dst[j] <= i
    uint64_t pos = off_src[lo] + (i - off_dst[lo]) * S;
    uint64_t h, l, c;
    load_elem<L0>(src, pos, h, l, c);
    dhi[i] = h;
    dlo[i] = l;
    dc[i] = c;
}

// bounds[t*k + j] = first position of list j whose key >= splitter t's key
// Level-1 sample counts per (splitter, stream) for the level-0 bounds (the fused path's k_fx_posof /
// k_fx_l1cnt, skv_stride.hip): the level-1 samples of list j are its records off0[j] + c*S; sorted,
// splitter t is sorted sample t*m. posof[l1off[j] + c] = sorted position of list j's sample c.
__device__ __forceinline__ uint32_t last_le(const uint64_t* off, uint32_t k, uint64_t x) {
    uint32_t lo = 0, hi = k;  // the last list j with off[j] <= x (empty lists share their offset)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}
__global__ void k_l1_posof(const uint64_t* __restrict__ sc, uint64_t N1, const uint64_t* __restrict__ off0,
                           const uint64_t* __restrict__ l1off, uint32_t k, uint64_t S, uint32_t* posof) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N1) return;
    const uint64_t pos = (uint32_t)sc[p];  // level-1 c = key length << 32 | record position
    const uint32_t j = last_le(off0, k, pos);
    const uint64_t q = l1off[j] + (pos - off0[j]) / S;
    if (q < l1off[j + 1]) posof[q] = (uint32_t)p;
}
// cnt[t*k + j] = list j's samples at sorted positions < t*m, for t in [1, T): sample c at position
// p, the next one at pn, writes the splitters t with p < t*m <= pn (c = 0 also those before it)
__global__ void k_l1_cnt(const uint32_t* __restrict__ posof, uint64_t N1, const uint64_t* __restrict__ l1off,
                         uint32_t k, uint64_t m, uint64_t T, uint32_t* cnt) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= N1 || T < 2) return;
    const uint32_t j = last_le(l1off, k, q);
    const uint64_t c = q - l1off[j], p = posof[q], tmax = T - 1;
    if (c == 0) {
        const uint64_t th = p / m < tmax ? p / m : tmax;
        for (uint64_t t = 1; t <= th; ++t) cnt[t * k + j] = 0;
    }
    const uint64_t th = q + 1 < l1off[j + 1] ? (posof[q + 1] / m < tmax ? posof[q + 1] / m : tmax) : tmax;
    for (uint64_t t = p / m + 1; t <= th; ++t) cnt[t * k + j] = (uint32_t)(c + 1);
}

template <bool L0>
__global__ void k_bounds(Elems E, const uint64_t* __restrict__ off, uint32_t k, const uint64_t* __restrict__ shi,
                         const uint64_t* __restrict__ slo, const uint64_t* __restrict__ sc, uint64_t m, uint64_t T,
                         const uint64_t* __restrict__ rec_addr, uint64_t* bounds, L1Cnt C) {
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (T + 1) * k || *E.poison) return;
    uint64_t t = g / k;
    uint32_t j = (uint32_t)(g - t * k);
    uint64_t a = off[j], b = off[j + 1];
    if (t == 0) { bounds[g] = a; return; }
    if (t == T) { bounds[g] = b; return; }
    uint64_t sp = t * m;
    uint64_t h = shi[sp], l = slo[sp], c = sc[sp];
    if (C.cnt && a < b) {
        // stream j's level-1 samples sorted before the splitter (k_l1_cnt), minus those equal to it
        // (lower_bound counts only the smaller ones): the bound lies in one sample gap
        uint64_t n = C.cnt[t * k + j];
        const uint64_t q0 = C.l1off[j];
        while (n > 0 && ekey_cmp(rec_addr, C.hi[q0 + n - 1], C.lo[q0 + n - 1], C.c[q0 + n - 1], h, l, c) == 0) --n;
        const uint64_t lo = n ? a + (n - 1) * C.S + 1 : a;
        const uint64_t hi = a + n * C.S < b ? a + n * C.S : b;
        a = lo;
        b = hi;
    }
    while (a < b) {
        uint64_t mid = (a + b) >> 1;
        uint64_t eh, el, ec;
        load_elem<L0>(E, mid, eh, el, ec);
        if (ekey_cmp(rec_addr, eh, el, ec, h, l, c) < 0) a = mid + 1;
        else b = mid;
    }
    bounds[g] = a;
}

__global__ void k_tile_n(const uint64_t* __restrict__ bounds, uint32_t k, uint64_t T, uint64_t* tile_n) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    uint64_t s = 0;
    for (uint32_t j = 0; j < k; ++j) s += bounds[(t + 1) * k + j] - bounds[t * k + j];
    tile_n[t] = s;
}



// LDS layout of k_tile (dynamic): hp[CAP] el_lo[CAP] el_c[CAP] el_fp[CAP] u64 | mi[CAP] posof[CAP] u16
// | cbA[k+1] cbB[k+1] u32 | ws[16] u64 | flag
__device__ __forceinline__ uint32_t seg_of(const uint32_t* cb, uint32_t m, uint32_t i) {
    uint32_t lo = 0, hi = m;  // last s in [0, m) with cb[s] <= i
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (cb[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Output stage of a level > 0 LDS tile (sorted samples): position i has hi = hp[i] and element
// mi[i] (its lo and c in el_lo / el_c).
__device__ void tile_output_samples(uint32_t n, const uint64_t* hp, const uint16_t* mi, const uint64_t* el_lo,
                                    const uint64_t* el_c, uint64_t base, const TileOut& O) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t e = mi[i];
        O.ohi[base + i] = hp[i];
        O.olo[base + i] = el_lo[e];
        O.oc[base + i] = el_c[e];
    }
}

// Decoupled look-back over tiles (single pass, no separate scan kernel): tile t publishes its
// (kept, bytes, deletes) aggregate, adds up its predecessors' until one with an inclusive prefix,
// then publishes its own inclusive prefix. Each counter is one 64-bit word (flag in bits 62-63),
// stored and polled with 8-byte agent-scope atomics — no payload rides on the flag. Tile ids come
// from an atomic ticket, so every predecessor of a waiting tile is resident or done.
__device__ void tile_lookback(uint64_t* st, uint64_t t, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t* s_ex) {
    if (threadIdx.x < 3) {
        const uint32_t q = threadIdx.x;
        const uint64_t agg = q == 0 ? a0 : (q == 1 ? a1 : a2);
        constexpr uint64_t FA = 1ull << 62, FI = 2ull << 62, VM = FA - 1;
        uint64_t acc = 0;
        if (t == 0) {
            __hip_atomic_store(&st[q], FI | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&st[3 * t + q], FA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint64_t p = t - 1;
            for (;;) {
                const uint64_t v = __hip_atomic_load(&st[3 * p + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t f = v >> 62;
                if (f == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                acc += v & VM;
                if (f == 2) break;
                --p;
            }
            __hip_atomic_store(&st[3 * t + q], FI | (acc + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_ex[q] = acc;
    }
    __syncthreads();
}

// block-wide min / max of a record size (for k_chain's uniform-size and all-fit tests)
__device__ void tile_minmax(uint32_t mn, uint32_t mx, uint32_t* s_mm, uint32_t* out) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t o = __shfl_xor(mx, d, 64);
        mx = o > mx ? o : mx;
        o = __shfl_xor(mn, d, 64);
        mn = o < mn ? o : mn;
    }
    if ((threadIdx.x & 63) == 0) {
        s_mm[2 * (threadIdx.x >> 6)] = mn;
        s_mm[2 * (threadIdx.x >> 6) + 1] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            mn = s_mm[2 * w] < mn ? s_mm[2 * w] : mn;
            mx = s_mm[2 * w + 1] > mx ? s_mm[2 * w + 1] : mx;
        }
        out[0] = mn;
        out[1] = mx;
    }
}

// the dense merged arrays of k_way::merge's output (k_way.rs:146-151: first record per key; the
// Delete filter of table_tree_compaction.rs:139-145 when asked) at global record g:
// rec index, source address, output-byte prefix P, delete-count prefix
__device__ __forceinline__ void emit_merged(const TileOut& O, uint64_t g, uint32_t idx, uint64_t addr, uint64_t pb,
                                            uint64_t pd, uint64_t dup = 0) {
    O.m_rec[g] = idx;
    O.m_src[g] = addr;
    O.m_P[g] = pb;
    O.m_Dp[g] = pd;
    if (O.m_dup) O.m_dup[g] = dup;
}

// heap-order mode: the records' own keys (first-per-key compares them, not the merge keys)
__device__ __forceinline__ int act_key_cmp(const TileOut& O, uint32_t a, uint32_t b) {
    return key_cmp(O.act_hi[a], O.act_lo[a], O.act_klen[a], (const uint8_t*)O.pay_addr[a] + 5, O.act_hi[b],
                   O.act_lo[b], O.act_klen[b], (const uint8_t*)O.pay_addr[b] + 5);
}

// after the last tile: K, P[K], Dp[K]
__device__ __forceinline__ void emit_totals(const TileOut& O, uint64_t K, uint64_t B, uint64_t D) {
    O.Kout[0] = K;
    O.m_P[K] = B;
    O.m_Dp[K] = D;
}

// Tiles larger than TILE_CAP: bitonic sort in global scratch (ascending-comparator form, so
// virtual +inf padding never moves), then the same output stage in blocks of TILE_CAP.
template <bool L0>
__device__ void tile_big(Elems E, const uint64_t* bounds, uint32_t k, uint64_t t, uint64_t base, uint32_t n,
                         const uint32_t* sb, const uint32_t* rec_meta, const uint64_t* rec_addr, bool drop_deletes,
                         const TileOut& O, uint64_t* ws, uint32_t* s_flag) {
    uint64_t* xh = O.xhi + base;
    uint64_t* xl = O.xlo + base;
    uint64_t* xc = O.xc + base;
    uint32_t* xm = O.xmeta + base;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t j = seg_of(sb, k + 1, i);
        uint64_t pos = bounds[t * k + j] + (i - sb[j]);
        uint64_t h, l, c;
        load_elem<L0>(E, pos, h, l, c);
        xh[i] = h;
        xl[i] = l;
        xc[i] = c;
        if (L0) xm[i] = rec_meta[pos];
    }
    __syncthreads();
    uint32_t P = 1, lp = 0;
    while (P < n) {
        P <<= 1;
        ++lp;
    }
    for (uint32_t lk = 1; lk <= lp; ++lk) {
        for (int lj = (int)lk - 1; lj >= 0; --lj) {
            for (uint32_t i = threadIdx.x; i < P / 2; i += blockDim.x) {
                uint32_t a, b;
                bitonic_pair(i, lk, (uint32_t)lj, a, b);
                if (b < n) {
                    if (elem_less(rec_addr, xh[b], xl[b], xc[b], xh[a], xl[a], xc[a])) {
                        uint64_t th = xh[a], tl = xl[a], tc = xc[a];
                        xh[a] = xh[b]; xl[a] = xl[b]; xc[a] = xc[b];
                        xh[b] = th; xl[b] = tl; xc[b] = tc;
                        if (L0) { uint32_t tm = xm[a]; xm[a] = xm[b]; xm[b] = tm; }
                    }
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
    if (!L0) {
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            O.ohi[base + i] = xh[i];
            O.olo[base + i] = xl[i];
            O.oc[base + i] = xc[i];
        }
        return;
    }
    // pass 1: this tile's totals (dedup + filter), then its global prefix
    const bool heap = O.act_hi != nullptr;  // heap-order mode: first-per-key on the records' own keys
    if (heap && O.pop_pos)
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) O.pop_pos[(uint32_t)xc[i]] = base + i;
    auto keep_at = [&](uint32_t i, uint32_t& m) -> bool {
        const bool first = i == 0 || (heap ? act_key_cmp(O, (uint32_t)xc[i - 1], (uint32_t)xc[i])
                                           : ekey_cmp(rec_addr, xh[i - 1], xl[i - 1], xc[i - 1], xh[i], xl[i], xc[i])) != 0;
        m = xm[i];
        return first && !(drop_deletes && (m >> 31));
    };
    uint64_t kd = 0, bytes = 0;
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t m;
        if (keep_at(i, m)) {
            kd += 1 | ((uint64_t)(m >> 31) << 32);
            bytes += m & 0x7FFFFFFFu;
            mn = (m & 0x7FFFFFFFu) < mn ? (m & 0x7FFFFFFFu) : mn;
            mx = (m & 0x7FFFFFFFu) > mx ? (m & 0x7FFFFFFFu) : mx;
        }
    }
    const uint64_t kd_tot = block_reduce_sum<uint64_t>(kd, ws);
    const uint64_t b_tot = block_reduce_sum<uint64_t>(bytes, ws);
    tile_minmax(mn, mx, s_flag, O.tile_mm + 2 * t);
    tile_lookback(O.tstate, t, kd_tot & 0xFFFFFFFFull, b_tot, kd_tot >> 32, ws + 8);
    uint64_t g = ws[8], pb = ws[9], pd = ws[10];
    __syncthreads();
    if (t == O.T - 1 && threadIdx.x == 0) emit_totals(O, g + (kd_tot & 0xFFFFFFFFull), pb + b_tot, pd + (kd_tot >> 32));
    // pass 2: write the survivors in order
    for (uint32_t b0 = 0; b0 < n; b0 += blockDim.x) {
        const uint32_t i = b0 + threadIdx.x;
        uint32_t m = 0;
        const bool keep = i < n && keep_at(i, m);
        const uint64_t sz = keep ? (m & 0x7FFFFFFFu) : 0, dl = keep ? (m >> 31) : 0;
        uint64_t ck, cb_, cd;
        const uint64_t rk = block_excl_scan<uint64_t>(keep ? 1 : 0, ws, ck);
        const uint64_t rb = block_excl_scan<uint64_t>(sz, ws, cb_);
        const uint64_t rd = block_excl_scan<uint64_t>(dl, ws, cd);
        if (keep)
            emit_merged(O, g + rk, (uint32_t)xc[i], (heap ? O.pay_addr : rec_addr)[(uint32_t)xc[i]], pb + rb, pd + rd);
        g += ck;
        pb += cb_;
        pd += cd;
    }
}

// ---- the level-0 tile's merge as a sort of packed 64-bit words ------------------------------------
// k_way::merge's order inside a tile (key asc, then seq_no desc = rec_idx asc) is the sort of the
// tile's elements by (key, element id): ids follow (stream rank, position). Each element becomes ONE
// 64-bit word: the 52 key bits that follow the tile's common key prefix (c bytes, c <= 8, from the
// OR of every key XOR the first one: the tile is a key range, so its keys often share bytes), then
// the 12-bit id. Words order as the keys do, except inside a group of equal 52-bit windows, which
// comes out in id order: the merge order when the group's keys are equal (one 16-byte prefix, one
// length, one fingerprint past 16 bytes: the fingerprint shortcut's "equal"), and re-sorted with the
// full compare otherwise (tile_fix_groups). Equal keys across streams (config 3: a third of the
// records) are the common group; keys that differ only past the window are rare.
// Each wave sorts 256 consecutive positions in registers (a bitonic network, 4 words per lane at
// index 4 lane + r: 15 stages inside a lane, 21 across lanes over DPP / permlane swaps, no LDS, no
// barrier); then LDS merge-path rounds over the words merge the 16 sorted runs of 256 (4 rounds,
// one 8-byte read per probe, in place of log2(k) rounds over the streams' segments, 8 at k = 256,
// reading 8-byte prefixes + ids + by-id key words on ties).
template <int KK, int JJ>
__device__ __forceinline__ void wd_stage(uint64_t (&x)[4], uint32_t lane) {
    constexpr uint32_t K2 = 1u << KK, D = 1u << JJ;
    if constexpr (D < 4) {  // partners in the same lane: registers r and r | D
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            if (r & D) continue;
            const bool asc = ((4 * lane + r) & K2) == 0;
            const uint64_t a = x[r], b = x[r | D];
            const bool sw = asc ? b < a : a < b;
            x[r] = sw ? b : a;
            x[r | D] = sw ? a : b;
        }
    } else {  // partner lane ^ D / 4, same register
        constexpr int LM = (int)(D / 4);
        const bool take_min = ((lane & LM) == 0) == (((4 * lane) & K2) == 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t y = xshfl64<LM>(x[r]);
            if (take_min == (y < x[r])) x[r] = y;
        }
    }
}
template <int KK, int JJ>
__device__ __forceinline__ void wd_merge(uint64_t (&x)[4], uint32_t lane) {
    wd_stage<KK, JJ>(x, lane);
    if constexpr (JJ > 0) wd_merge<KK, JJ - 1>(x, lane);
}
template <int KK>
__device__ __forceinline__ void wd_sort(uint64_t (&x)[4], uint32_t lane) {
    if constexpr (KK > 1) wd_sort<KK - 1>(x, lane);
    wd_merge<KK, KK - 1>(x, lane);
}

constexpr uint32_t WD_ID = 12;  // id bits of a sort word (TILE_CAP <= 4096)
static_assert(TILE_CAP <= (1 << WD_ID), "element ids fit the sort word");

// the 8 key bytes that follow c common bytes (0 <= c <= 8) of a 16-byte prefix
__device__ __forceinline__ uint64_t wd_window(uint64_t hi, uint64_t lo, uint32_t c) {
    return c == 0 ? hi : (c >= 8 ? lo << (8 * (c - 8)) : (hi << (8 * c)) | (lo >> (64 - 8 * c)));
}

// key16 (by id, id == load position), n elements -> wd[] by position: runs of 256 sorted words.
// c: common prefix bytes of the tile's keys (<= 15).
__device__ void tile_sort_words(const ulong2* key16, uint64_t* wd, uint32_t n, uint32_t c) {
    static_assert(TILE_THREADS * 4 == TILE_CAP, "one 256-position run per wave");
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (256 * w < n) {  // waves past n idle (no barrier inside the sort)
        uint64_t x[4];
        const uint32_t p0 = 256 * w + 4 * lane;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t p = p0 + r;
            if (p < n) {
                const ulong2 k = key16[p];
                x[r] = (wd_window(k.x, k.y, c) >> WD_ID << WD_ID) | p;
            } else {
                x[r] = ~0ull;  // padding sorts last
            }
        }
        wd_sort<8>(x, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (p0 + r < n) wd[p0 + r] = x[r];
    }
    __syncthreads();
}
// merge-path rounds over the sorted runs of 256 words (length L, pairs of 2L; a thread's 4 outputs lie
// in one pair because 2L is a multiple of 4); words are distinct (the id), so no tie rule. ow: this
// thread's final words (positions 4 tid .. 4 tid + 3, valid below n), for the caller's epilogue.
__device__ void tile_merge_runs(uint64_t* wd, uint32_t n, uint64_t (&ow)[4]) {
    constexpr int PER = 4;
    const uint32_t o0 = threadIdx.x * PER;
    bool rounds = false;
    for (uint32_t L = 256; L < n; L <<= 1) {
        rounds = true;
        if (o0 < n) {
            const uint32_t a0 = o0 & ~(2 * L - 1);
            const uint32_t a1 = a0 + L < n ? a0 + L : n, b1 = a0 + 2 * L < n ? a0 + 2 * L : n;
            const uint32_t lenA = a1 - a0, lenB = b1 - a1, d = o0 - a0;
            uint32_t l = d > lenB ? d - lenB : 0, h = d < lenA ? d : lenA;
            while (l < h) {  // how many of the first d outputs come from A
                const uint32_t mid = (l + h) >> 1;
                if (wd[a0 + mid] < wd[a1 + d - mid - 1]) l = mid + 1;
                else h = mid;
            }
            uint32_t ia = a0 + l, ib = a1 + (d - l);
            uint64_t hA = ia < a1 ? wd[ia] : ~0ull, hB = ib < b1 ? wd[ib] : ~0ull;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const bool takeA = hA < hB;  // exhausted sides read as ~0 (above every real word)
                ow[q] = takeA ? hA : hB;
                if (takeA) hA = ++ia < a1 ? wd[ia] : ~0ull;
                else hB = ++ib < b1 ? wd[ib] : ~0ull;
            }
        }
        __syncthreads();  // every thread has read its inputs of this round
#pragma unroll
        for (int q = 0; q < PER; ++q)
            if (o0 + q < n) wd[o0 + q] = ow[q];
        __syncthreads();
    }
    if (!rounds) {
#pragma unroll
        for (int q = 0; q < PER; ++q) ow[q] = o0 + q < n ? wd[o0 + q] : ~0ull;
    }
}

// fingerprint of element e's key bytes past 16 (O.key_fp by record index), 0 in exact mode
__device__ __forceinline__ uint64_t el_fp_of(const uint64_t* kfp, uint64_t c) {
    return kfp ? kfp[(uint32_t)c] : 0;
}
// the full element order (elem_less_fp over key16 / el_c by id, fingerprints from global memory)
__device__ __forceinline__ bool el_less_full(const ulong2* key16, const uint64_t* el_c, const uint64_t* kfp,
                                             const uint64_t* rec_addr, uint32_t a, uint32_t b) {
    const ulong2 ka = key16[a], kb = key16[b];
    const uint64_t ca = el_c[a], cb = el_c[b];
    if (ka.x != kb.x) return ka.x < kb.x;
    if (ka.y != kb.y) return ka.y < kb.y;
    return elem_less_fp(kfp != nullptr, el_fp_of(kfp, ca), rec_addr, ka.x, ka.y, ca, kb.x, kb.y, cb,
                        el_fp_of(kfp, cb));
}
// two elements with the same key under the fingerprint shortcut (their id order is the merge order)
__device__ __forceinline__ bool el_same_key(const ulong2* key16, const uint64_t* el_c, const uint64_t* kfp,
                                            uint32_t a, uint32_t b) {
    const ulong2 ka = key16[a], kb = key16[b];
    const uint32_t la = (uint32_t)(el_c[a] >> 32), lb = (uint32_t)(el_c[b] >> 32);
    if (ka.x != kb.x || ka.y != kb.y || la != lb) return false;
    return la <= 16 || (kfp && el_fp_of(kfp, el_c[a]) == el_fp_of(kfp, el_c[b]));
}

// Groups of equal 52-bit windows after tile_merge_runs (wd by position) whose keys are not all one
// key: re-sorted by the full compare, one thread per group (insertion sort; groups hold a handful of
// elements). Returns false when such a group is larger than 64: the caller then merges the tile
// exactly. The rare path: the caller found a mixed pair first.
__device__ bool tile_fix_groups(const ulong2* key16, const uint64_t* wd, uint16_t* mi, uint32_t n, const uint64_t* el_c,
                                const uint64_t* kfp, const uint64_t* rec_addr, uint32_t* s_big) {
    constexpr int PER = 4;
    const uint32_t o0 = threadIdx.x * PER;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t g0 = o0 + q;
        if (g0 + 1 >= n) continue;
        const uint64_t gw = wd[g0] >> WD_ID;
        if (g0 > 0 && (wd[g0 - 1] >> WD_ID) == gw) continue;  // not a group start
        uint32_t g1 = g0 + 1;
        bool mixed = false;
        while (g1 < n && (wd[g1] >> WD_ID) == gw) {
            mixed |= !el_same_key(key16, el_c, kfp, mi[g1 - 1], mi[g1]);
            ++g1;
        }
        if (!mixed) continue;
        if (g1 - g0 > 64) {
            *s_big = 1;  // the exact merge takes the whole tile
            continue;
        }
        for (uint32_t i = g0 + 1; i < g1; ++i) {  // insertion sort of the group's ids
            const uint32_t e = mi[i];
            uint32_t j = i;
            while (j > g0 && el_less_full(key16, el_c, kfp, rec_addr, e, mi[j - 1])) {
                mi[j] = mi[j - 1];
                --j;
            }
            mi[j] = (uint16_t)e;
        }
    }
    __syncthreads();
    return *s_big == 0;
}

// The exact merge of a tile (any keys): pairwise merge-path rounds over the streams' segments (cb:
// segment starts, k + 1 entries, scratch cbn) with the full compare, elements by id through mi.
// Rare: a tile whose keys share more than the sort word sees (tile_fix_groups' large groups).
__device__ void tile_merge_exact(const ulong2* key16, const uint64_t* el_c, const uint64_t* kfp, const uint64_t* rec_addr,
                                 uint16_t* mi, uint32_t n, uint32_t k, uint32_t* cb, uint32_t* cbn) {
    constexpr int PER = 4;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) mi[i] = (uint16_t)i;
    __syncthreads();
    const uint32_t o0 = threadIdx.x * PER;
    uint32_t m = k;
    while (m > 1) {
        const uint32_t mp = (m + 1) >> 1;
        uint32_t ox[PER];
        uint32_t pos = o0, ia = 0, a1 = 0, ib = 0, b1 = 0;
        bool setup = true;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            ox[q] = 0;
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
                    while (l < h) {
                        const uint32_t mid = (l + h) >> 1;
                        if (el_less_full(key16, el_c, kfp, rec_addr, mi[a0 + mid], mi[a1 + d - mid - 1])) l = mid + 1;
                        else h = mid;
                    }
                    ia = a0 + l;
                    ib = a1 + (d - l);
                    setup = false;
                }
                const bool takeA =
                    ia < a1 && (ib >= b1 || el_less_full(key16, el_c, kfp, rec_addr, mi[ia], mi[ib]));
                ox[q] = takeA ? mi[ia++] : mi[ib++];
                ++pos;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q)
            if (o0 + q < n) mi[o0 + q] = (uint16_t)ox[q];
        for (uint32_t p = threadIdx.x; p <= mp; p += blockDim.x) cbn[p] = p < mp ? cb[2 * p] : cb[m];
        __syncthreads();
        uint32_t* t = cb;
        cb = cbn;
        cbn = t;
        m = mp;
    }
}

#if SKV_TILE_PROF
#define TPROF(i)                                                                 \
    do {                                                                         \
        if (L0 && threadIdx.x == 0) {                                            \
            const uint64_t now_ = __builtin_amdgcn_s_memrealtime();              \
            atomicAdd((unsigned long long*)&O.prof[i], (unsigned long long)(now_ - tp_last)); \
            tp_last = now_;                                                      \
        }                                                                        \
    } while (0)
#else
#define TPROF(i) do {} while (0)
#endif

template <bool L0>
__global__ void __launch_bounds__(TILE_THREADS) k_tile(Elems E, const uint64_t* __restrict__ bounds, uint32_t k,
                                                      const uint64_t* __restrict__ tile_base,
                                                      const uint32_t* __restrict__ rec_meta,
                                                      const uint64_t* __restrict__ rec_addr, uint32_t drop_deletes,
                                                      TileOut O) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // hp / mi: key bytes 0..7 and element id by merged position (permuted each merge round). By
    // element id (= load position): key bytes 8..15, length | record, fingerprint of the bytes
    // past 16, read on a prefix tie (at config 3 a third of the records share their key with
    // another stream: the fingerprint decides those without reading record bytes)
    uint64_t* hp = (uint64_t*)smem;
    uint64_t* el_lo = hp + TILE_CAP;
    uint64_t* el_c = el_lo + TILE_CAP;
    uint64_t* el_fp = el_c + TILE_CAP;
    uint16_t* mi = (uint16_t*)(el_fp + TILE_CAP);
    uint16_t* posof = mi + TILE_CAP;  // after the rounds: merged position of each element
    // level-0 tiles outside heap-order mode (tile_sort_words): hp / el_lo hold {hp, lo} by id instead
    // (key16), el_fp the sort words by position (wd; fingerprints are read from O.key_fp on ties)
    ulong2* key16 = (ulong2*)smem;
    uint64_t* wd = el_fp;
    const bool wpath = !L0 || O.act_hi == nullptr;  // (sample tiles too: level > 0, exact compares)
    uint32_t* cbA = (uint32_t*)(posof + TILE_CAP);
    uint32_t* cbB = cbA + (k + 1);
    uint64_t* ws = (uint64_t*)(((uintptr_t)(cbB + (k + 1)) + 15) & ~(uintptr_t)15);
    uint32_t* s_flag = (uint32_t*)(ws + 16);

    __shared__ uint64_t s_tk;
#if SKV_TILE_PROF
    uint64_t tp_last = __builtin_amdgcn_s_memrealtime();
#endif
    if (*E.poison) {  // a merge of unsorted segments is not a permutation: touch nothing
        if (L0 && blockIdx.x == 0 && threadIdx.x == 0) O.Kout[0] = 0;
        return;
    }
    uint64_t t = blockIdx.x;
    if (!L0 && threadIdx.x == 0) s_flag[24] = s_flag[25] = s_flag[26] = s_flag[27] = s_flag[28] = s_flag[29] = 0;
    if (L0) {  // level 0 tiles take tickets in start order (tile_lookback's progress guarantee)
        if (threadIdx.x == 0) {
            s_tk = atomicAdd(O.tcounter, 1u);
            s_flag[24] = s_flag[25] = 0;  // mixed groups / a group too large (tile_fix_groups)
            s_flag[26] = s_flag[27] = s_flag[28] = s_flag[29] = 0;  // the common-prefix ORs (tile_sort_words)
        }
        __syncthreads();
        t = s_tk;
    }
    // segment starts (and, without a tile_base table, the tile's output base: the elements of all
    // lists before bounds[t], as bounds[0] holds the list starts)
    uint64_t segtot = 0, before = 0;
    for (uint32_t j0 = 0; j0 < k; j0 += blockDim.x) {
        uint32_t j = j0 + threadIdx.x;
        uint64_t len = j < k ? bounds[(t + 1) * k + j] - bounds[t * k + j] : 0;
        uint64_t tot;
        uint64_t ex = block_excl_scan<uint64_t>(len, ws, tot);
        if (j < k) cbA[j] = (uint32_t)(segtot + ex);
        segtot += tot;
        if (!tile_base) before += block_reduce_sum<uint64_t>(j < k ? bounds[t * k + j] - bounds[j] : 0, ws);
    }
    const uint64_t base = tile_base ? tile_base[t] : before;
    const uint64_t n64 = tile_base ? tile_base[t + 1] - base : segtot;
    if (threadIdx.x == 0) cbA[k] = (uint32_t)segtot;
    __syncthreads();
    TPROF(0);
    const uint32_t n = (uint32_t)n64;
    if (n64 > TILE_CAP) {
        tile_big<L0>(E, bounds, k, t, base, n, cbA, rec_meta, rec_addr, drop_deletes != 0, O, ws, s_flag);
        return;
    }
    if (n == 0) {
        if (L0) {
            tile_minmax(0xFFFFFFFFu, 0, s_flag, O.tile_mm + 2 * t);
            tile_lookback(O.tstate, t, 0, 0, 0, ws + 8);
            if (t == O.T - 1 && threadIdx.x == 0) emit_totals(O, ws[8], ws[9], ws[10]);
        }
        return;
    }
    // Thread owns elements e = threadIdx.x + u*TILE_THREADS for the loads (payload stays in
    // registers) and output positions threadIdx.x * PER + q in the merge rounds.
    constexpr int PER = TILE_CAP / TILE_THREADS;
    uint64_t rh[PER], rl[PER], rc[PER], raddr[PER];
    uint32_t rpos[PER], rmeta[PER];
    const uint64_t* kfp = L0 ? O.key_fp : nullptr;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        uint32_t e = threadIdx.x + u * TILE_THREADS;
        rh[u] = rc[u] = raddr[u] = 0;
        rpos[u] = e;
        rmeta[u] = 0;
        if (e < n) {
            uint32_t j = seg_of(cbA, k + 1, e);
            uint64_t pos = bounds[t * k + j] + (e - cbA[j]);
            uint64_t lo, fp = 0;
            load_elem<L0>(E, pos, rh[u], lo, rc[u]);
            if (L0) {
                rmeta[u] = rec_meta[pos];
                raddr[u] = (O.pay_addr ? O.pay_addr : rec_addr)[pos];  // coalesced here, not gathered later
                if (kfp) fp = kfp[pos];
            }
            rl[u] = lo;
            if (wpath) {
                key16[e] = make_ulong2(rh[u], lo);
            } else {
                hp[e] = rh[u];
                el_lo[e] = lo;
                el_fp[e] = fp;
            }
            el_c[e] = rc[u];
            mi[e] = (uint16_t)e;
        }
    }
    __syncthreads();
    TPROF(1);
    // merge-path rounds over pairs of adjacent segments (the key order is strict: c holds the
    // record index): each thread produces PER consecutive outputs of a round with ONE merge-path
    // search, then a sequential merge. A compare reads the two prefixes by position, the ids and
    // by-id words only on a prefix tie.
    auto less_hx = [&](uint64_t ha, uint32_t xa, uint64_t hb, uint32_t xb) -> bool {
        if (ha != hb) return ha < hb;
        return L0 ? elem_less_fp(kfp != nullptr, el_fp[xa], rec_addr, ha, el_lo[xa], el_c[xa], hb, el_lo[xb],
                                 el_c[xb], el_fp[xb])
                  : elem_less(rec_addr, ha, el_lo[xa], el_c[xa], hb, el_lo[xb], el_c[xb]);
    };
    if (wpath) {
        // c = the bytes every key of the tile shares (<= 15): the OR of each key's prefix words XOR
        // element 0's, over the block (keys sharing their first 8 bytes -- 2B's zero-padded hex ids --
        // take the window from the second word: from the first, 16 ids shared one, and the sample
        // tiles went to the exact merge: 287 against 41 us)
        const ulong2 k0 = key16[0];
        uint64_t dh = 0, dl = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u)
            if (threadIdx.x + u * TILE_THREADS < n) {
                dh |= rh[u] ^ k0.x;
                dl |= rl[u] ^ k0.y;
            }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            dh |= __shfl_xor(dh, d, 64);
            dl |= __shfl_xor(dl, d, 64);
        }
        if ((threadIdx.x & 63) == 0 && (dh | dl)) {
            atomicOr(s_flag + 26, (uint32_t)(dh >> 32));
            atomicOr(s_flag + 27, (uint32_t)dh);
            atomicOr(s_flag + 28, (uint32_t)(dl >> 32));
            atomicOr(s_flag + 29, (uint32_t)dl);
        }
        __syncthreads();
        const uint64_t D = ((uint64_t)s_flag[26] << 32) | s_flag[27];
        const uint64_t DL = ((uint64_t)s_flag[28] << 32) | s_flag[29];
        const uint32_t cpx = D ? (uint32_t)__builtin_clzll(D) >> 3 : (DL ? 8u + ((uint32_t)__builtin_clzll(DL) >> 3) : 15u);
        tile_sort_words(key16, wd, n, cpx);
        TPROF(8);
        uint64_t ow[4];
        tile_merge_runs(wd, n, ow);
        TPROF(9);
        // epilogue from registers: ids by position, positions by id, and the pairs of equal windows
        // (one LDS read: the word before this thread's first); a pair whose keys differ sends the
        // tile to tile_fix_groups
        constexpr uint32_t IDM = (1u << WD_ID) - 1;
        const uint32_t o0 = threadIdx.x * 4;
        uint64_t prevw = o0 > 0 && o0 < n ? wd[o0 - 1] : ~0ull;
        bool mixed = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (o0 + q < n) {
                const uint32_t id = (uint32_t)(ow[q] & IDM);
                mi[o0 + q] = (uint16_t)id;
                posof[id] = (uint16_t)(o0 + q);
                if (prevw != ~0ull && (prevw >> WD_ID) == (ow[q] >> WD_ID))
                    mixed |= !el_same_key(key16, el_c, kfp, (uint32_t)(prevw & IDM), id);
                prevw = ow[q];
            }
        }
        if (mixed) s_flag[24] = 1;
        __syncthreads();
        if (s_flag[24]) {  // rare: re-sort the mixed groups (or the whole tile), then positions again
            if (!tile_fix_groups(key16, wd, mi, n, el_c, kfp, rec_addr, s_flag + 25))
                tile_merge_exact(key16, el_c, kfp, rec_addr, mi, n, k, cbA, cbB);
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) posof[mi[i]] = (uint16_t)i;
            __syncthreads();
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t e = threadIdx.x + u * TILE_THREADS;
            if (e < n) rpos[u] = posof[e];
        }
    } else {
        const uint32_t o0 = threadIdx.x * PER;
        uint32_t m = k;
        uint32_t* cb = cbA;
        uint32_t* cbn = cbB;
        while (m > 1) {
            const uint32_t mp = (m + 1) >> 1;
            uint64_t oh[PER];
            uint32_t ox[PER];
            uint32_t pos = o0, ia = 0, a1 = 0, ib = 0, b1 = 0, xA = 0, xB = 0;
            uint64_t hA = 0, hB = 0;
            bool setup = true;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                oh[q] = 0;
                ox[q] = 0;
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
                            const uint32_t pa = a0 + mid, pb = a1 + d - mid - 1;
                            const uint64_t ha = hp[pa], hb = hp[pb];
                            const bool lt = ha != hb ? ha < hb : less_hx(ha, mi[pa], hb, mi[pb]);
                            if (lt) l = mid + 1;
                            else h = mid;
                        }
                        ia = a0 + l;
                        ib = a1 + (d - l);
                        if (ia < a1) {
                            hA = hp[ia];
                            xA = mi[ia];
                        }
                        if (ib < b1) {
                            hB = hp[ib];
                            xB = mi[ib];
                        }
                        setup = false;
                    }
                    const bool takeA = ia < a1 && (ib >= b1 || less_hx(hA, xA, hB, xB));
                    if (takeA) {
                        oh[q] = hA;
                        ox[q] = xA;
                        if (++ia < a1) {
                            hA = hp[ia];
                            xA = mi[ia];
                        }
                    } else {
                        oh[q] = hB;
                        ox[q] = xB;
                        if (++ib < b1) {
                            hB = hp[ib];
                            xB = mi[ib];
                        }
                    }
                    ++pos;
                }
            }
            __syncthreads();  // every thread has read its inputs of this round
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                if (o0 + q < n) {
                    hp[o0 + q] = oh[q];
                    mi[o0 + q] = (uint16_t)ox[q];
                }
            }
            for (uint32_t p = threadIdx.x; p <= mp; p += blockDim.x) cbn[p] = p < mp ? cb[2 * p] : cb[m];
            __syncthreads();
            uint32_t* tp = cb;
            cb = cbn;
            cbn = tp;
            m = mp;
        }
        if (L0) {  // each element's merged position (its payload stays in the loading thread)
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) posof[mi[i]] = (uint16_t)i;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const uint32_t e = threadIdx.x + u * TILE_THREADS;
                if (e < n) rpos[u] = posof[e];
            }
        }
    }
    if (!L0) {
        if (wpath) {  // sorted samples from key16 / el_c by id
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
                const uint32_t e = mi[i];
                const ulong2 kk = key16[e];
                O.ohi[base + i] = kk.x;
                O.olo[base + i] = kk.y;
                O.oc[base + i] = el_c[e];
            }
        } else {
            tile_output_samples(n, hp, mi, el_lo, el_c, base, O);
        }
        return;
    }
    TPROF(2);
    if (O.pop_pos) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const uint32_t e = threadIdx.x + u * TILE_THREADS;
            if (e < n) O.pop_pos[(uint32_t)rc[u]] = base + rpos[u];
        }
    }
    // (a) first-per-key flags by merged position (k_way.rs:146-151). With fingerprints, a pair
    // with equal prefix, length and fingerprint is taken as one key and queued for k_fp_verify;
    // a pair whose lengths or fingerprints differ is two keys (and was ordered by exact compares
    // in the rounds). Without them (exact mode) the suffixes are compared here.
    const uint32_t i0 = threadIdx.x * PER;
    uint32_t keep_mask = 0, vmask = 0;
    uint32_t idx[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = i0 + q;
        idx[q] = 0;
        if (i < n) {
            const uint32_t e = mi[i];
            const uint64_t c = el_c[e];
            bool first = true;
            if (O.act_hi) {  // heap-order mode: adjacent pops compared on their own keys
                if (i > 0) first = act_key_cmp(O, (uint32_t)el_c[mi[i - 1]], (uint32_t)c) != 0;
            } else if (i > 0) {
                const uint32_t p = mi[i - 1];
                if (wpath ? key16[p].x == key16[e].x : hp[i - 1] == hp[i]) {
                    const uint64_t lp = wpath ? key16[p].y : el_lo[p], le = wpath ? key16[e].y : el_lo[e];
                    const uint64_t cp = el_c[p];
                    int kc = lp != le ? (lp < le ? -1 : 1) : 0;
                    const uint32_t kp = (uint32_t)(cp >> 32), ke = (uint32_t)(c >> 32);
                    if (!kc && kp > 16 && ke > 16) {
                        if (kfp) {
                            const int same = kp == ke && (wpath ? el_fp_of(kfp, cp) == el_fp_of(kfp, c)
                                                                : el_fp[p] == el_fp[e]);
                            kc = same ? 0 : 1;
                            if (same) vmask |= 1u << q;
                        } else {
                            kc = suffix_cmp(rec_addr, cp, c);
                        }
                    }
                    if (!kc) kc = kp < ke ? -1 : (kp > ke ? 1 : 0);
                    first = kc != 0;
                }
            }
            idx[q] = (uint32_t)c;
            if (first) keep_mask |= 1u << q;
        }
    }
    // in-gather verify (O.m_dup): a pair whose first record is its key's survivor is checked by
    // k_gather against the survivor's bytes; only the others are queued (qmask). Per merged
    // position in LDS (posof's bytes, free after the rounds): bit 0 first-per-key, bit 1 a pair with
    // the record before it.
    uint32_t qmask = vmask;
    uint8_t* s_f8 = (uint8_t*)posof;
    const bool dup_out = O.m_dup != nullptr && !drop_deletes;
    if (dup_out) {
        __syncthreads();  // every thread has read posof (rpos)
#pragma unroll
        for (int q = 0; q < PER; ++q)
            if (i0 + q < n) s_f8[i0 + q] = (uint8_t)(((keep_mask >> q) & 1u) | (((vmask >> q) & 1u) << 1));
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q)
            if ((vmask >> q) & 1u)
                if (s_f8[i0 + q - 1] & 1u) qmask &= ~(1u << q);
    }
    uint32_t vex = 0;
    uint64_t vb = 0;
    if (kfp) {  // slots for the pairs taken as equal (one atomic per tile), written below
        uint32_t vtot;
        vex = block_excl_scan<uint32_t>((uint32_t)__builtin_popcount(qmask), (uint32_t*)ws, vtot);
        if (threadIdx.x == 0) s_flag[31] = vtot ? (uint32_t)atomicAdd(O.vcount, (unsigned long long)vtot) : 0u;
        __syncthreads();
        vb = s_flag[31];
    }
    __syncthreads();
    TPROF(3);
    // (b) source address and meta by final position (hp / el_lo are free now)
    uint64_t* paddr = hp;
    uint32_t* pmeta = (uint32_t*)el_lo;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t e = threadIdx.x + u * TILE_THREADS;
        if (e < n) {
            paddr[rpos[u]] = raddr[u];
            pmeta[rpos[u]] = rmeta[u];
        }
    }
    __syncthreads();
    // the queued pairs as the two records' addresses (k_fp_verify then touches only their keys)
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if (qmask & (1u << q)) {
            const uint32_t i = i0 + q;
            O.vpairs[2 * (vb + vex)] = paddr[i - 1];
            O.vpairs[2 * (vb + vex) + 1] = paddr[i];
            ++vex;
        }
    TPROF(4);
    // (c) Delete filter, tile totals
    uint32_t mt[PER];
    uint64_t ad[PER];
    uint64_t kd = 0, bytes = 0;
    uint32_t smin = 0xFFFFFFFFu, smax = 0;
    const bool drop = drop_deletes != 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        mt[q] = 0;
        ad[q] = 0;
        if (keep_mask & (1u << q)) {
            const uint32_t i = i0 + q;
            mt[q] = pmeta[i];
            ad[q] = paddr[i];
            if (drop && (mt[q] >> 31)) {
                keep_mask &= ~(1u << q);
            } else {
                const uint32_t sz = mt[q] & 0x7FFFFFFFu;
                kd += 1 | ((uint64_t)(mt[q] >> 31) << 32);
                bytes += sz;
                smin = sz < smin ? sz : smin;
                smax = sz > smax ? sz : smax;
            }
        }
    }
    uint64_t kd_tot, b_tot;
    const uint64_t kd_ex = block_excl_scan<uint64_t>(kd, ws, kd_tot);
    const uint64_t b_ex = block_excl_scan<uint64_t>(bytes, ws, b_tot);
    tile_minmax(smin, smax, s_flag, O.tile_mm + 2 * t);
    // (d) global position of this tile's survivors
    TPROF(5);
    tile_lookback(O.tstate, t, kd_tot & 0xFFFFFFFFull, b_tot, kd_tot >> 32, ws + 8);
    const uint64_t K0 = ws[8], B0 = ws[9], D0 = ws[10];
    TPROF(6);
    if (t == O.T - 1 && threadIdx.x == 0)
        emit_totals(O, K0 + (kd_tot & 0xFFFFFFFFull), B0 + b_tot, D0 + (kd_tot >> 32));
    uint64_t g = K0 + (kd_ex & 0xFFFFFFFFull), pb = B0 + b_ex, pd = D0 + (kd_ex >> 32);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (keep_mask & (1u << q)) {
            const uint32_t i = i0 + q;
            const uint64_t dup = dup_out && i + 1 < n && (s_f8[i + 1] & 2u) ? paddr[i + 1] : 0;
            emit_merged(O, g, idx[q], ad[q], pb, pd, dup);
            ++g;
            pb += mt[q] & 0x7FFFFFFFu;
            pd += mt[q] >> 31;
        }
    }
    TPROF(7);
}

// ---------------------------------------------------------------------------------------
// chain: build_runs' greedy split (runs.rs:211-238). A run starting at surviving record b
// holds records b..e-1 where e is the largest index with 1 + P[e] - P[b] <= max (at least b+1).
// One wave walks the chain; each step checks a window around the predicted end first.

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint64_t o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint64_t o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    return v;
}

// Run tables of a wide fixed-stride call on the device (in place of a 10^6-entry RunFmt readback and
// host loops): cnt[r] = the records of run r under its fixed-stride hypothesis, flags[RT_*] = 1 if any
// run is not fixed-stride / differs from run 0's format / is fixed-stride / has no body (one wave
// ballot, one atomic per wave).
__global__ void k_run_tables(const RunInfo* __restrict__ runs, const RunFmt* __restrict__ fmt, uint32_t n_runs,
                             uint64_t* cnt, uint32_t* flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool nf = false, nu = false, af = false, bl = false;
    if (i < n_runs) {
        const RunFmt f = fmt[i], f0 = fmt[0];
        const uint64_t len = runs[i].len;
        cnt[i] = f.S && len >= 1 ? (len - 1) / f.S : 0;
        nf = f.S == 0;
        nu = f.S != f0.S || f.K != f0.K;
        af = f.S != 0;
        bl = runs[i].n_chunks == 0;
    }
    const uint64_t bnf = __ballot(nf), bnu = __ballot(nu), baf = __ballot(af), bbl = __ballot(bl);
    if ((threadIdx.x & 63) == 0) {
        if (bnf) atomicOr(flags + RT_NOT_FIXED, 1u);
        if (bnu) atomicOr(flags + RT_NOT_UNIFORM, 1u);
        if (baf) atomicOr(flags + RT_ANY_FIXED, 1u);
        if (bbl) atomicOr(flags + RT_BODYLESS, 1u);
    }
}
void launch_run_tables(hipStream_t s, const RunInfo* runs, const RunFmt* fmt, uint32_t n_runs, uint64_t* cnt,
                       uint32_t* flags) {
    if (n_runs) k_run_tables<<<(n_runs + 255) / 256, 256, 0, s>>>(runs, fmt, n_runs, cnt, flags);
}

// The run table of a call whose streams hold one run each, in a monotone seq_no order, built on the
// device from the caller-order pointer / length arrays (the host's pass over 10^6 runs and the
// 32-byte-per-run upload are skipped): rank r is caller stream r (descending seq_no) or n - 1 - r
// (ascending). Two launches: the chunk counts (scanned into chunk bases between them), then the
// entries.
__global__ void k_run_info(const uint64_t* __restrict__ ptr, const uint64_t* __restrict__ len, uint32_t n,
                           bool reversed, uint64_t chunk, const uint64_t* __restrict__ chunk_base, uint64_t* nch,
                           RunInfo* runs) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t c = reversed ? n - 1 - r : r;
    const uint64_t l = len[c];
    const uint64_t nc = l >= 2 ? (l - 1 + chunk - 1) / chunk : 0;
    if (!chunk_base) {
        nch[r] = nc;
        return;
    }
    RunInfo R;
    R.ptr = ptr[c];
    R.len = l;
    R.chunk_base = chunk_base[r];
    R.n_chunks = (uint32_t)nc;
    R.stream = (uint32_t)r;
    runs[r] = R;
}
void launch_run_info(hipStream_t s, const uint64_t* ptr, const uint64_t* len, uint32_t n, bool reversed, uint64_t chunk,
                     uint64_t* nch, uint64_t* chunk_base, uint64_t* scan_tmp, RunInfo* runs) {
    if (!n) return;
    k_run_info<<<(n + 255) / 256, 256, 0, s>>>(ptr, len, n, reversed, chunk, nullptr, nch, runs);
    launch_scan(s, nch, n, chunk_base, scan_tmp);
    k_run_info<<<(n + 255) / 256, 256, 0, s>>>(ptr, len, n, reversed, chunk, chunk_base, nch, runs);
}

// largest e in [lo, hi] with P[e] <= v, given P[lo] <= v (64-ary search, exact). Not inlined: k_chain
// unrolls its resolve step CH_D times, and 32 inlined copies of this rare fallback made the kernel
// ~50 KB of straight-line code, streamed through the instruction cache on every round.
__device__ __noinline__ uint64_t chain_search(const uint64_t* P, uint64_t lo, uint64_t hi, uint64_t v, int lane) {
    while (lo < hi) {
        uint64_t span = hi - lo;
        uint64_t step = (span + 63) / 64;
        uint64_t pos = lo + (uint64_t)(lane + 1) * step;
        if (pos > hi) pos = hi;
        bool f = P[pos] <= v;
        uint64_t nlo = wave_max_u64(f ? pos : lo);
        uint64_t gtpos = wave_min_u64(f ? ~0ull : pos);
        lo = nlo;
        if (gtpos != ~0ull) hi = gtpos - 1;
        if (step == 1) break;
    }
    return lo;
}

// Predicted windows in flight and entries per lane per window. With every record fitting a run,
// run d+1 from a known start ends within (d+1) x (largest record) bytes of its lower bound, so
// 32 windows of 64 consecutive P entries (one load per lane each, all independent) cover 32 run
// ends per round for records of ~300 B (config 3: 3F chain 26.6 ms with 8 x 512-entry windows,
// whose 64 loads per lane per round kept one wave latency-bound); rounds shrink to fewer
// windows when the records are small relative to the largest (see ch_d below).
constexpr int CH_D = 32;
constexpr int CH_Q = 1;
constexpr uint32_t CH_SHIFT = 10;  // byte -> record table granularity (1 KiB)

// tbl[t] = the surviving record j with P[j] <= t * 2^CH_SHIFT < P[j+1] (K past the end): lets the
// chain turn a byte position into a record index with one load
__global__ void k_chain_table(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ P, uint32_t* tbl,
                              uint64_t n_tbl, const SplitPlan* __restrict__ plan) {
    if (plan && plan->mode == SPLIT_PAR) return;
    const uint64_t K = *Kp;
    const uint64_t G = 1ull << CH_SHIFT;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= K; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t lo = P[j];
        const uint64_t hi = j < K ? P[j + 1] : lo + 1;  // past P[K] the chain clamps to K itself
        for (uint64_t t = (lo + G - 1) >> CH_SHIFT; t < ((hi + G - 1) >> CH_SHIFT) && t < n_tbl; ++t) tbl[t] = (uint32_t)j;
    }
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}
// a wave-uniform value the compiler cannot prove uniform (a shuffle reduction, a value merged from
// branches) moved to scalar registers: the chain's state then stays in SGPRs and its branches are
// scalar, instead of exec-masked VALU code on every step
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__global__ void __launch_bounds__(64) k_chain(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ P,
                                              uint64_t max_size, const uint32_t* __restrict__ tile_max,
                                              uint64_t n_tiles, uint64_t* run_b, uint64_t* n_runs_out,
                                              const uint32_t* __restrict__ tbl, uint64_t n_tbl,
                                              const SplitPlan* __restrict__ plan) {
    if (plan && plan->mode == SPLIT_PAR) return;  // k_split_* wrote run_b and n_runs_out
    const uint64_t K = *Kp;
    const int lane = threadIdx.x;
#if SKV_CHAIN_PROF
    uint64_t cp_t0 = __builtin_amdgcn_s_memrealtime(), cp_mm = 0, cp_p1 = 0, cp_p2 = 0, cp_p3 = 0, cp_fb = 0,
             cp_rounds = 0;
#endif
    // n_runs_out = {runs, K, output record bytes P[K]}: the host's single readback
    if (K == 0) {
        if (lane == 0) { run_b[0] = 0; n_runs_out[0] = 0; n_runs_out[1] = 0; n_runs_out[2] = 0; }
        return;
    }
    if (lane == 0) {
        n_runs_out[1] = K;
        n_runs_out[2] = P[K];
    }
    // smallest / largest surviving record (per-tile pairs from k_tile<true>)
    uint32_t mr = 0, mn = 0xFFFFFFFFu;
    for (uint64_t t = lane; t < n_tiles; t += 64) {
        mn = tile_max[2 * t] < mn ? tile_max[2 * t] : mn;
        mr = tile_max[2 * t + 1] > mr ? tile_max[2 * t + 1] : mr;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t o = __shfl_xor(mr, d, 64);
        mr = o > mr ? o : mr;
        o = __shfl_xor(mn, d, 64);
        mn = o < mn ? o : mn;
    }
    mr = __builtin_amdgcn_readfirstlane(mr);  // uniform from here on (see uniform_u64)
    mn = __builtin_amdgcn_readfirstlane(mn);
#if SKV_CHAIN_PROF
    cp_mm = __builtin_amdgcn_s_memrealtime() - cp_t0;
#endif
    // every record fits a run on its own when 1 + largest record <= max: no oversize probe
    const bool all_fit = max_size >= 1 && (uint64_t)mr + 1 <= max_size;
    if (all_fit && mn == mr) {
        // one record size S: the greedy split (runs.rs:211-238) closes every run after exactly
        // n = (max - 1) / S records, so the chain is arithmetic
        const uint64_t n = (max_size - 1) / mr;
        const uint64_t runs = (K + n - 1) / n;
        for (uint64_t i = lane; i <= runs; i += 64) run_b[i] = i * n < K ? i * n : K;
        if (lane == 0) *n_runs_out = runs;
        return;
    }
    uint64_t b = 0, m = 0;
    uint64_t Pb = P[0];
    const uint64_t PK = P[K];
    uint64_t L = 1;
    if (max_size > 1) {
        uint64_t avg = P[K] / K;
        if (avg == 0) avg = 1;
        L = (max_size - 1) / avg;
        if (L == 0) L = 1;
        if (L > K) L = K;
    }
    // windows per round: keep the byte uncertainty of the last one, ch_d x mr, within ~3/4 of a
    // window's records at the average record size
    int ch_d = CH_D;
    if (all_fit && tbl) {
        const uint64_t avg = PK / K > 0 ? PK / K : 1;
        const uint64_t cap = (uint64_t)(48 * CH_Q) * avg / (mr > 0 ? mr : 1);
        ch_d = cap < 1 ? 1 : (cap < (uint64_t)CH_D ? (int)cap : CH_D);
    }
    while (b < K) {
#if SKV_CHAIN_PROF
        uint64_t cp_a = __builtin_amdgcn_s_memrealtime();
        ++cp_rounds;
#endif
        // prefetch CH_D windows of P around the predicted ends of the next CH_D runs
        const uint64_t m_round = m;
        uint64_t rb = 0;
        uint64_t wv[CH_D][CH_Q];
        uint64_t wsd[CH_D];
        // window starts: with every record fitting a run, run d+1 from here ends at a record
        // starting in (Pb + (d+1)(max-1-mr), Pb + (d+1)(max-1)] bytes: the byte table gives the
        // record at the low end with one load (all CH_D loads independent); else by count
        // lane d computes window d's start (the table entries as ONE vector load: a uniform
        // address per window made them scalar loads, waited for one by one, 13 us per round)
        {
            uint64_t wl;
            if (tbl && all_fit) {
                const uint64_t step = max_size - 1 - mr;  // (saturating: max may be near 2^64)
                const uint64_t low = step > (~0ull - Pb) / (uint64_t)(lane + 1) ? ~0ull : Pb + (uint64_t)(lane + 1) * step;
                wl = (low >= PK || lane >= ch_d) ? K : (uint64_t)tbl[low >> CH_SHIFT];
            } else {
                const uint64_t c = b + (uint64_t)(lane + 1) * L;
                const uint64_t back = 16ull * CH_Q;
                wl = c > back ? c - back : 0;
            }
#pragma unroll
            for (int d = 0; d < CH_D; ++d) wsd[d] = readlane_u64(wl, d);
        }
#if SKV_CHAIN_PROF
        { uint64_t x = 0; for (int d = 0; d < CH_D; ++d) x += wsd[d]; if (x == 7) run_b[0] = x; }
        uint64_t cp_b = __builtin_amdgcn_s_memrealtime();
        cp_p1 += cp_b - cp_a;
#endif
#pragma unroll
        for (int d = 0; d < CH_D; ++d) {
            uint64_t ws = wsd[d];
            if (ws < b + 1) ws = b + 1;
            wsd[d] = ws;
#pragma unroll
            for (int q = 0; q < CH_Q; ++q) {
                uint64_t pos = ws + (uint64_t)lane * CH_Q + q;
                wv[d][q] = (pos <= K && d < ch_d) ? P[pos] : ~0ull;
            }
        }
#if SKV_CHAIN_PROF
        { uint64_t x = 0; for (int d = 0; d < CH_D; ++d) x += wv[d][0]; if (x == 7) run_b[0] = x; }
        uint64_t cp_c = __builtin_amdgcn_s_memrealtime();
        cp_p2 += cp_c - cp_b;
#endif
#pragma unroll
        for (int d = 0; d < CH_D; ++d) {
            if (b < K && d < ch_d) {  // (no break: keeps the loop fully unrolled, windows in registers)
            uint64_t e, Pe = 0;
            if (max_size == 0 || (!all_fit && P[b + 1] - Pb + 1 > max_size)) {
                e = b + 1;  // a run of one record that alone exceeds max (runs.rs:219 needs !first)
                Pe = P[e];
            } else {
                const uint64_t v = sat_add_u64(Pb, max_size - 1);  // record j fits iff P[j+1] <= v
                const uint64_t ws = wsd[d];
                // predicate P[pos] <= v is monotone in pos = ws + 4*lane + q: the last true
                // position is found from four wave ballots with scalar bit ops
                uint64_t mq[CH_Q];
#pragma unroll
                for (int q = 0; q < CH_Q; ++q) mq[q] = __ballot(wv[d][q] <= v);
                const uint64_t m0 = mq[0];
                bool found = false;
                uint64_t best = 0;
                if (m0) {
                    const int ls = 63 - __builtin_clzll(m0);
                    uint32_t qs = 0;  // true entries of lane ls past its first
#pragma unroll
                    for (int q = 1; q < CH_Q; ++q) qs += (uint32_t)((mq[q] >> ls) & 1);
                    best = ws + (uint64_t)ls * CH_Q + qs;
                    found = best == K || best < ws + CH_Q * 64 - 1;
                    if (found) {
                        uint64_t x = wv[d][0];
#pragma unroll
                        for (int q = 1; q < CH_Q; ++q) x = qs == (uint32_t)q ? wv[d][q] : x;
                        Pe = readlane_u64(x, ls);
                    }
                }
                if (found) {
                    e = best;
                } else {
                    uint64_t lo = b + 1, hi = K;
                    if (m0) lo = best;                 // window all <= v: answer at or past its end
                    // window all > v: the answer lies before it. A window predicted past the last
                    // record (its entries past K read as ~0) says nothing beyond K: the search stays
                    // inside P[0..K] (it read past the end and closed the last run too late)
                    else if (ws > b + 1) hi = ws - 1 < K ? ws - 1 : K;
                    e = chain_search(P, lo, hi, v, lane);
                    Pe = P[e];
#if SKV_CHAIN_PROF
                    ++cp_fb;
#endif
                }
            }
            e = uniform_u64(e);
            Pe = uniform_u64(Pe);
            rb = lane == d ? b : rb;  // this round's run starts, stored together below
            ++m;
            L = e - b;
            b = e;
            Pb = Pe;
            }
        }
        if ((uint64_t)lane < m - m_round) run_b[m_round + lane] = rb;
#if SKV_CHAIN_PROF
        cp_p3 += __builtin_amdgcn_s_memrealtime() - cp_c;
#endif
    }
#if SKV_CHAIN_PROF
    if (lane == 0)
        printf("[chain] total %llu ticks: minmax %llu, rounds %llu, p1 %llu p2 %llu p3 %llu, fallbacks %llu, ch_d %d, runs %llu\n",
               (unsigned long long)(__builtin_amdgcn_s_memrealtime() - cp_t0), (unsigned long long)cp_mm,
               (unsigned long long)cp_rounds, (unsigned long long)cp_p1, (unsigned long long)cp_p2,
               (unsigned long long)cp_p3, (unsigned long long)cp_fb, ch_d, (unsigned long long)m);
#endif
    if (lane == 0) {
        run_b[m] = K;
        *n_runs_out = m;
    }
}

// ---------------------------------------------------------------------------------------
// Parallel exact greedy split (build_runs' size split, runs.rs:211-238). With every record
// fitting a run, the run starting at record b ends at f(b) = the last e with P[e] <= P[b] + max - 1
// (P[K] included), and the run starts are the chain 0, f(0), f(f(0)), ... f is monotone but no
// contraction: chains from two starts a record or more apart keep their byte offset, so the chain
// cannot be guessed from anywhere but its true start. What CAN be guessed is where it is: runs are
// cut into segments of segr runs, and the byte position of segment s's first run start is the sum
// of the earlier segments' advances (segr x max minus the slack each run leaves, a sum of
// independent slacks whose spread grows as sqrt(s)). So:
//   k_split_plan   the gate (one workgroup);
//   k_split_guess  one lane per segment walks segr runs from an arbitrary record near its expected
//                  start: the advance D_s;
//   k_split_scan   G_s = the exclusive prefix of D: segment s's byte guess;
//   k_split_walk   the nc records around the record at G_s are segment s's candidate starts; one
//                  lane per candidate walks segr runs from it (all segments, all candidates at
//                  once), storing every run start and where the walk ends;
//   k_split_stitch one thread follows the true chain through the segments: its start of segment s
//                  is a candidate (index = start - window start, one LDS read of the staged ends)
//                  whose walk gives the start of segment s + 1; a start outside its window is
//                  walked by the stitch itself;
//   k_split_emit   copies the chosen candidates' run starts into run_b.
// Each f step is three rounds of eight independent probes of P (stride 64 around the previous
// run's record count, then 9-ary), no lookup table. Inputs it does not fit (runs of < 8 records,
// record sizes all equal, few runs, K >= 2^32) keep the single-wave k_chain (plan->mode).

// last j in [lo, hi) with P[j] <= v, given P[lo] <= v < P[hi]: a first round of probes at stride
// 64 around the guess g, then 9-ary rounds, each of eight independent loads
__device__ uint64_t sp_search(const uint64_t* __restrict__ P, uint64_t lo, uint64_t Plo, uint64_t hi, uint64_t v,
                              uint64_t g, uint64_t& Pe) {
    uint64_t st = 64;
    uint64_t base = g > lo + 4 * 64 ? g - 4 * 64 : lo;  // probes base + st * q, q = 1..8
    while (hi - lo > 1) {
        uint64_t x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t p = base + st * (uint64_t)(q + 1);
            x[q] = (p > lo && p < hi) ? P[p] : 0;
        }
        uint64_t nlo = lo, nPlo = Plo, nhi = hi;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t p = base + st * (uint64_t)(q + 1);
            if (p > lo && p < hi) {
                if (x[q] <= v) {
                    nlo = p;  // probes ascend: the last true one wins
                    nPlo = x[q];
                } else if (p < nhi) {
                    nhi = p;
                }
            }
        }
        lo = nlo;
        Plo = nPlo;
        hi = nhi;
        st = (hi - lo + 8) / 9;
        base = lo;
    }
    Pe = Plo;
    return lo;
}

// f(b) and P[f(b)]; every record fits a run (plan gate); Lg: guessed records in the run
__device__ __forceinline__ uint64_t sp_step(const uint64_t* __restrict__ P, uint64_t K, uint64_t PK, uint64_t M,
                                            uint64_t b, uint64_t Pb, uint64_t Lg, uint64_t& Pe) {
    if (b >= K) {
        Pe = PK;
        return K;
    }
    const uint64_t v = sat_add_u64(Pb, M - 1);  // record j fits iff P[j + 1] <= v
    if (PK <= v) {
        Pe = PK;
        return K;
    }
    uint64_t g = b + Lg;
    if (g >= K) g = K - 1;
    return sp_search(P, b, Pb, K, v, g, Pe);
}

constexpr int SPLIT_PLAN_THREADS = 1024;
constexpr int SPLIT_GUESS_SEGS = 16;  // guess walks per 64-lane workgroup: spread over CUs, each
                                      // walk's probes are cache lines of their own

// gate and constants (one workgroup): smallest / largest surviving record from k_tile<true>
__global__ void __launch_bounds__(SPLIT_PLAN_THREADS)
    k_split_plan(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ P, uint64_t M,
                 const uint32_t* __restrict__ tile_max, uint64_t n_tiles, SplitBufs B) {
    __shared__ uint32_t s_mm[2];
    const int tid = threadIdx.x;
    const uint64_t K = *Kp;
    if (tid == 0) {
        s_mm[0] = 0xFFFFFFFFu;
        s_mm[1] = 0;
    }
    __syncthreads();
    uint32_t mn = 0xFFFFFFFFu, mr = 0;
    for (uint64_t t = tid; t < n_tiles; t += SPLIT_PLAN_THREADS) {
        mn = tile_max[2 * t] < mn ? tile_max[2 * t] : mn;
        mr = tile_max[2 * t + 1] > mr ? tile_max[2 * t + 1] : mr;
    }
    atomicMin(&s_mm[0], mn);
    atomicMax(&s_mm[1], mr);
    __syncthreads();
    if (tid) return;
    mn = s_mm[0];
    mr = s_mm[1];
    SplitPlan pl{};
    pl.mode = SPLIT_SERIAL;
    // gate: every run holds >= 8 records (so no record exceeds max), record sizes differ (else
    // k_chain's arithmetic split), enough runs to pay for the passes, u32 record indices
    if (K > 0 && K < 0xFFFFFFF0ull && B.nseg_cap > 0 && M > 1 && (M - 1) >= 8 * (uint64_t)mr && mn != mr) {
        const uint64_t PK = P[K];
        const uint64_t avg = PK / K ? PK / K : 1;
        const uint64_t adv = (M - 1) - (avg / 2 < M - 1 ? avg / 2 : 0);  // expected bytes per run
        const uint64_t runs_ub = PK / ((M - 1) - mr) + 1;  // every run but the last holds > max - 1 - mr bytes
        const uint64_t nseg = (runs_ub + B.segr - 1) / B.segr + 1;
        if (nseg <= B.nseg_cap && PK / adv + 1 >= B.min_runs) {
            pl.mode = SPLIT_PAR;
            pl.nseg = (uint32_t)nseg;
            pl.K = K;
            pl.PK = PK;
            pl.L0 = (M - 1) / avg ? (M - 1) / avg : 1;
            pl.avg = avg;
            pl.adv = adv;
        }
    }
    *B.plan = pl;
}

// guess walks: segment s from the record expected at byte s * segr * adv (indexed by the average
// record size; any nearby start samples the same slack statistics): seg_D[s] = bytes advanced
__global__ void __launch_bounds__(64) k_split_guess(const uint64_t* __restrict__ P, uint64_t M, SplitBufs B) {
    const SplitPlan pl = *B.plan;
    const uint64_t s = (uint64_t)blockIdx.x * SPLIT_GUESS_SEGS + threadIdx.x;
    if (pl.mode != SPLIT_PAR || threadIdx.x >= SPLIT_GUESS_SEGS || s >= pl.nseg) return;
    const uint64_t K = pl.K, PK = pl.PK;
    const uint32_t segr = B.segr;
    uint64_t a = (uint64_t)((double)s * segr * pl.adv / pl.avg);
    if (a > K) a = K;
    uint64_t b = a, Pb = P[a], L = pl.L0;
    const uint64_t Pa = Pb;
    uint32_t k = 0;
    for (; k < segr && b < K; ++k) {
        uint64_t Pe;
        const uint64_t e = sp_step(P, K, PK, M, b, Pb, L, Pe);
        if (e < K) L = e - b;
        b = e;
        Pb = Pe;
    }
    B.seg_D[s] = k == segr ? Pb - Pa : segr * pl.adv;  // reached the end early: the expected advance
}

// seg_D becomes the exclusive prefix G_s (one workgroup; thread tid owns a block of segments)
__global__ void __launch_bounds__(SPLIT_PLAN_THREADS) k_split_scan(SplitBufs B) {
    __shared__ uint64_t ws[32];
    const SplitPlan pl = *B.plan;
    if (pl.mode != SPLIT_PAR) return;
    const uint64_t nseg = pl.nseg, tid = threadIdx.x;
    const uint64_t per = (nseg + SPLIT_PLAN_THREADS - 1) / SPLIT_PLAN_THREADS;
    const uint64_t s0 = tid * per < nseg ? tid * per : nseg, s1 = s0 + per < nseg ? s0 + per : nseg;
    uint64_t sum = 0;
    for (uint64_t s = s0; s < s1; ++s) sum += B.seg_D[s];
    uint64_t tot;
    uint64_t G = block_excl_scan(sum, ws, tot);
    for (uint64_t s = s0; s < s1; ++s) {
        const uint64_t d = B.seg_D[s];
        B.seg_D[s] = G;
        G += d;
    }
}

// grid: nseg_cap x ceil(nc / blockDim) workgroups (blockDim >= 64). Wave 0 finds the record at
// byte G_s (64-ary search over P, 64 independent probes a round); the window is the nc records
// around it; lane = candidate, walking segr runs and storing every run start
__global__ void k_split_walk(const uint64_t* __restrict__ P, uint64_t M, SplitBufs B) {
    __shared__ uint64_t s_c;
    const SplitPlan& pl = *B.plan;
    if (pl.mode != SPLIT_PAR) return;
    const uint32_t per_seg = (B.nc + blockDim.x - 1) / blockDim.x;
    const uint64_t s = blockIdx.x / per_seg;
    if (s >= pl.nseg) return;
    const uint64_t K = pl.K, PK = pl.PK;
    const uint32_t segr = B.segr, nc = B.nc;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const uint64_t G = B.seg_D[s];
        uint64_t lo = 0, hi = K;  // P[lo] <= G < P[hi]
        if (G >= PK) {
            lo = K;
            hi = K;
        }
        while (hi - lo > 1) {
            const uint64_t st = (hi - lo + 63) / 64;
            const uint64_t p = lo + st * (uint64_t)(lane + 1);
            const uint64_t m = __ballot(p < hi && P[p] <= G);  // true lanes: a prefix
            const uint64_t c = (uint64_t)__builtin_popcountll(m);
            const uint64_t nhi = lo + st * (c + 1);
            lo = lo + st * c;
            hi = nhi < hi ? nhi : hi;
        }
        if (lane == 0) s_c = lo;
    }
    __syncthreads();
    const uint64_t c = s_c;
    const uint64_t w = s == 0 ? 0 : (c > nc / 2 ? c - nc / 2 : 0);
    const uint32_t n = (uint32_t)(K + 1 - w < nc ? K + 1 - w : nc);
    const uint32_t i = (blockIdx.x % per_seg) * blockDim.x + threadIdx.x;
    if (i == 0) {
        B.seg_w[s] = w;
        B.seg_n[s] = n;
    }
    if (i >= n) return;
    uint32_t* out = B.chain + s * (uint64_t)segr * nc + i;
    uint64_t b = w + i, L = pl.L0;
    uint64_t Pb = P[b];
    for (uint32_t k = 0; k < segr; ++k) {
        out[(uint64_t)k * nc] = (uint32_t)b;
        uint64_t Pe;
        const uint64_t e = sp_step(P, K, PK, M, b, Pb, L, Pe);
        if (e < K) L = e - b;
        b = e;
        Pb = Pe;
    }
    B.ends[s * nc + i] = (uint32_t)b;  // contiguous per segment: the stitch stages whole batches
}

constexpr int SPLIT_STITCH_THREADS = 256;
constexpr uint32_t SPLIT_LDS_ENDS = 16384;  // segment ends staged per batch (64 KiB, two batches)
constexpr uint32_t SPLIT_SB = 256;          // segments per batch at most

// one workgroup: thread 0 follows the chain through batch j while waves 1-3 stage batch j + 1
__global__ void __launch_bounds__(SPLIT_STITCH_THREADS)
    k_split_stitch(const uint64_t* __restrict__ P, uint64_t M, SplitBufs B, uint64_t* run_b, uint64_t* n_runs_out) {
    __shared__ uint32_t s_end[2][SPLIT_LDS_ENDS];
    __shared__ uint64_t s_w[2][SPLIT_SB];
    __shared__ uint32_t s_n[2][SPLIT_SB];
    __shared__ uint64_t s_t;
    __shared__ uint32_t s_done;
    SplitPlan& pl = *B.plan;
    if (pl.mode != SPLIT_PAR) return;
    const uint64_t K = pl.K, PK = pl.PK;
    const uint32_t segr = B.segr, nc = B.nc, nseg = pl.nseg;
    const uint32_t sb = SPLIT_LDS_ENDS / nc < SPLIT_SB ? SPLIT_LDS_ENDS / nc : SPLIT_SB;  // segments per batch
    const uint32_t nbatch = (nseg + sb - 1) / sb;
    const int tid = threadIdx.x;
    // batch j into buffer buf by threads t0, t0 + nt, ...: eight 16-byte loads in flight per thread
    // (entries past a window's seg_n are copied but never read)
    auto stage = [&](uint32_t j, int buf, uint32_t t0, uint32_t nt) {
        const uint32_t s0 = j * sb, nb = nseg - s0 < sb ? nseg - s0 : sb;
        for (uint32_t b = t0; b < nb; b += nt) {
            s_w[buf][b] = B.seg_w[s0 + b];
            s_n[buf][b] = B.seg_n[s0 + b];
        }
        const uint32_t cnt = nb * nc;
        const uint32_t* src = B.ends + (uint64_t)s0 * nc;
        uint32_t x0 = 0;
        if ((nc & 3) == 0) {  // 16-byte aligned rows
            const uint32_t n4 = cnt / 4;
            const uint4* src4 = (const uint4*)src;
            uint4* dst4 = (uint4*)s_end[buf];
            for (uint32_t x = t0; x < n4; x += 8 * nt) {
                uint4 r[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t y = x + u * nt;
                    if (y < n4) r[u] = src4[y];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t y = x + u * nt;
                    if (y < n4) dst4[y] = r[u];
                }
            }
            x0 = n4 * 4;
        }
        for (uint32_t x = x0 + t0; x < cnt; x += nt) s_end[buf][x] = src[x];
    };
    if (tid == 0) {
        s_t = 0;
        s_done = 0;
    }
    stage(0, 0, tid, SPLIT_STITCH_THREADS);
    __syncthreads();
    uint64_t L = pl.L0;
    uint32_t n_fb = 0, sel_count = 0;
    uint32_t walked = 0;  // run starts the last walk_segment wrote
    // the stitch's own walk of segment s from t (a start outside the window): writes run_b
    auto walk_segment = [&](uint64_t s, uint64_t t) -> uint64_t {
        uint64_t Pt = P[t];
        walked = 0;
        for (uint32_t k = 0; k < segr && t < K; ++k, ++walked) {
            run_b[s * segr + k] = t;
            uint64_t Pe;
            const uint64_t e = sp_step(P, K, PK, M, t, Pt, L, Pe);
            if (e < K) L = e - t;
            t = e;
            Pt = Pe;
        }
        return t;
    };
    // the chain ended within segment s (its next start is K): count its runs, close run_b
    auto finish = [&](uint64_t s, bool by_walk, uint32_t ci) {
        uint64_t m = s * segr;
        if (by_walk) {
            m += walked;
        } else {
            const uint32_t* ch = B.chain + s * (uint64_t)segr * nc + ci;
            for (uint32_t k = 0; k < segr && ch[(uint64_t)k * nc] < K; ++k) ++m;
        }
        run_b[m] = K;
        n_runs_out[0] = m;
        n_runs_out[1] = K;
        n_runs_out[2] = PK;
    };
    for (uint32_t j = 0; j < nbatch; ++j) {
        const int buf = j & 1;
        if (tid < 64) {
            if (tid == 0 && !s_done) {
                const uint32_t s0 = j * sb, nb = nseg - s0 < sb ? nseg - s0 : sb;
                uint64_t t = s_t;
                for (uint32_t b = 0; b < nb; ++b) {
                    const uint64_t s = s0 + b;
                    const uint64_t w = s_w[buf][b];
                    const uint32_t n = s_n[buf][b];
                    sel_count = (uint32_t)s + 1;
                    bool by_walk = false;
                    uint32_t ci = 0;
                    if (t >= w && t - w < n) {
                        ci = (uint32_t)(t - w);
                        B.seg_sel[s] = ci;
                        t = s_end[buf][b * nc + ci];
                    } else {
                        B.seg_sel[s] = SPLIT_FB;
                        ++n_fb;
                        by_walk = true;
                        t = walk_segment(s, t);
                    }
                    if (t >= K) {
                        finish(s, by_walk, ci);
                        s_done = 1;
                        break;
                    }
                }
                s_t = t;
            }
        } else if (j + 1 < nbatch) {
            stage(j + 1, buf ^ 1, tid - 64, SPLIT_STITCH_THREADS - 64);
        }
        __syncthreads();
        if (s_done) break;
    }
    if (tid == 0) {
        if (!s_done) {  // past the last window (more runs than the plan's bound: cannot happen)
            uint64_t t = s_t;
            for (uint64_t s = nseg;; ++s) {
                t = walk_segment(s, t);
                if (t >= K) {
                    finish(s, true, 0);
                    break;
                }
            }
        }
        pl.nseg_sel = sel_count;
        pl.n_fb = n_fb;
    }
}

// run_b[s * segr + k] = the chosen candidate's k-th run start (segments the stitch walked are written)
__global__ void k_split_emit(SplitBufs B, uint64_t* run_b) {
    const SplitPlan& pl = *B.plan;
    if (pl.mode != SPLIT_PAR) return;
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t segr = B.segr;
    const uint64_t s = x / segr, k = x % segr;
    if (s >= pl.nseg_sel) return;
    const uint32_t ci = B.seg_sel[s];
    if (ci == SPLIT_FB) return;
    const uint32_t v = B.chain[(s * segr + k) * B.nc + ci];
    if (v < pl.K) run_b[x] = v;
}

__global__ void k_run_stats(const uint64_t* __restrict__ n_runs_p, const uint64_t* __restrict__ run_b,
                            const uint64_t* __restrict__ P, const uint64_t* __restrict__ Dp,
                            const uint32_t* __restrict__ m_rec, const uint32_t* __restrict__ rec_klen,
                            DevRunDesc* descs, uint64_t* seg_r0) {
    const uint64_t n_runs = *n_runs_p;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_runs; r += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t b = run_b[r], e = run_b[r + 1];
        // gather segments whose first record lies in this run
        for (uint64_t sg = (b + GATHER_SEG - 1) / GATHER_SEG; sg * GATHER_SEG < e; ++sg) seg_r0[sg] = r;
        DevRunDesc d;
        d.off = P[b] + r;
        d.len = 1 + P[e] - P[b];
        d.delete_count = Dp[e] - Dp[b];
        d.put_count = (e - b) - d.delete_count;
        d.min_key_off = d.off + 1 + 5;
        d.min_key_len = rec_klen[m_rec[b]];
        d.max_key_off = d.off + 1 + (P[e - 1] - P[b]) + 5;
        d.max_key_len = rec_klen[m_rec[e - 1]];
        d.table_id = 0;
        d.reserved = 0;
        descs[r] = d;
    }
}

// ---------------------------------------------------------------------------------------
// gather: workgroup per GATHER_SEG surviving records. Output byte x of the job is covered by a
// "piece": a record (copied verbatim from its input address) or a run's version byte. Record j
// of run r lands at P[j] + r + 1; run r's version byte at P[b_r] + r. Each lane produces whole
// 16-byte aligned output blocks with one vector store; blocks shared with a neighbouring
// workgroup (segment edges) are written bytewise.

// last piece whose destination starts at or before x
__device__ __forceinline__ uint32_t gather_piece(const uint64_t* s_dst, uint32_t npieces, uint64_t x) {
    uint32_t lo = 0, hi = npieces;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (s_dst[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// 16 bytes at a global address given as an integer, through the global address space (a flat
// load would also count against lgkmcnt and serialise with every LDS read)
typedef unsigned int g_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld16(uint64_t a) {
    const g_v4 v = *(const __attribute__((address_space(1))) g_v4*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// An output block covering several pieces: each piece contributes bytes [a, b) of the block,
// moved with at most two aligned 16-byte loads and merged under a byte mask. Blocks shared
// with a neighbouring workgroup (segment edges) are written bytewise, only this segment's bytes.
__device__ __noinline__ void gather_block_slow(uint64_t B, uint64_t x0, uint64_t x1, uint32_t p,
                                               const uint64_t* s_dst, const uint64_t* s_src,
                                               uint8_t* out) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint64_t x = x0;
    while (x < x1) {
        const uint64_t d = s_dst[p];
        const uint64_t src = s_src[p];
        const uint64_t e = s_dst[p + 1] < x1 ? s_dst[p + 1] : x1;  // pieces tile the output densely
        const uint32_t a = (uint32_t)(x - B), b = (uint32_t)(e - B);
        uint4 w = src ? load_window16((const uint8_t*)src + (x - d), b - a) : make_uint4(1u, 0, 0, 0);
        w = shl_bytes(w, a);
        acc.x |= w.x & dword_mask(a, b, 0);
        acc.y |= w.y & dword_mask(a, b, 1);
        acc.z |= w.z & dword_mask(a, b, 2);
        acc.w |= w.w & dword_mask(a, b, 3);
        x = e;
        ++p;
    }
    if (x0 == B && x1 == B + 16) {
        *(uint4*)(out + B) = acc;
    } else {
        for (uint64_t y = x0; y < x1; ++y) out[y] = (uint8_t)byte_of(acc, (uint32_t)(y - B));
    }
}

__global__ void __launch_bounds__(GATHER_THREADS, SKV_GATHER_WAVES) k_gather(const uint64_t* __restrict__ Kp,
                                                           const uint64_t* __restrict__ n_runs_p,
                                                           const uint64_t* __restrict__ run_b,
                                                           const uint64_t* __restrict__ P,
                                                           const uint64_t* __restrict__ m_src,
                                                           const uint64_t* __restrict__ seg_r0, uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ m_dup, uint32_t* fp_bad) {
    // 20 KB of LDS at 256 records: 8 workgroups (32 waves) per CU
    __shared__ uint64_t s_dst[2 * GATHER_SEG + 1];  // piece p = output bytes [s_dst[p], s_dst[p+1])
    __shared__ uint64_t s_src[2 * GATHER_SEG];      // 0 => version byte
    __shared__ uint64_t ws[16];
    __shared__ uint64_t s_tbl64[GATHER_TBL / 4];
    uint16_t* s_tbl = (uint16_t*)s_tbl64;  // output block -> piece covering its first byte
    uint64_t* s_rb = s_tbl64;              // run starts (setup only; dead before the table is built)
    static_assert(GATHER_TBL / 4 >= GATHER_SEG + 2, "s_rb alias");
    // XCD-aware segment order: workgroups are dealt round-robin over the 8 XCDs, so give each XCD
    // a contiguous range of segments (neighbouring segments share input lines and one L2)
    const uint32_t nb = gridDim.x, bid = blockIdx.x;
    const uint32_t xcd = bid & 7, qn = nb >> 3, rn = nb & 7;
    const uint32_t seg = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
    const uint64_t K = *Kp;
    const uint64_t j0 = (uint64_t)seg * GATHER_SEG;
    if (j0 >= K) return;
    const uint64_t j1 = j0 + GATHER_SEG < K ? j0 + GATHER_SEG : K;
    const uint32_t nrec = (uint32_t)(j1 - j0);
    // independent loads first: this lane's record (P, size, source) and the segment's first run
    const uint64_t j = j0 + threadIdx.x;
    uint64_t Pj = 0, Pj1 = 0, srcj = 0, dupj = 0;
    if (threadIdx.x < nrec) {
        Pj = P[j];
        Pj1 = P[j + 1];
        srcj = m_src[j];
        if (m_dup) dupj = m_dup[j];
    }
    const uint64_t n_runs = *n_runs_p;
    const uint64_t r0 = seg_r0[seg];  // run holding record j0 (k_run_stats)
    // run starts r0 .. r0+nrb-1 that are <= j1-1
    for (uint32_t i = threadIdx.x; i < GATHER_SEG + 1; i += blockDim.x) {
        uint64_t r = r0 + i;
        s_rb[i] = r <= n_runs ? run_b[r] : ~0ull;
    }
    __syncthreads();
    // pieces: per record 1 or 2
    uint32_t cntp = 0;
    uint64_t rr = 0;
    bool start = false;
    if (threadIdx.x < nrec) {
        uint32_t q = upper_idx<uint64_t>(s_rb, GATHER_SEG + 1, j);
        rr = r0 + q;
        start = s_rb[q] == j;
        cntp = start ? 2 : 1;
    }
    uint64_t tot;
    uint32_t pi = (uint32_t)block_excl_scan<uint64_t>(cntp, ws, tot);
    const uint32_t npieces = (uint32_t)tot;
    if (threadIdx.x < nrec) {
        uint64_t dst = Pj + rr + 1;
        if (start) {
            s_dst[pi] = dst - 1;
            s_src[pi] = 0;
            ++pi;
        }
        s_dst[pi] = dst;
        s_src[pi] = srcj;
        if (threadIdx.x == nrec - 1) s_dst[pi + 1] = dst + (Pj1 - Pj);  // end sentinel
    }
    __syncthreads();
    const uint64_t lo_b = s_dst[0];
    const uint64_t hi_b = s_dst[npieces];
    const uint64_t q0 = lo_b >> 4, q1 = (hi_b + 15) >> 4;
    const bool use_tbl = q1 - q0 <= GATHER_TBL;
    if (use_tbl) {
        // piece p covers the blocks whose first byte (lo_b for the first block, else 16q) it holds
        for (uint32_t p = threadIdx.x; p < npieces; p += blockDim.x) {
            const uint64_t d = s_dst[p], e = s_dst[p + 1];
            uint64_t qs = (d + 15) >> 4, qe = (e + 15) >> 4;  // blocks q with 16q in [d, e)
            if (d == lo_b) s_tbl[0] = (uint16_t)p;
            if (qs <= q0) qs = q0 + 1;
            for (uint64_t q = qs; q < qe; ++q) s_tbl[q - q0] = (uint16_t)p;
        }
        __syncthreads();
    }
    // Per output block, three cases (gfx950 serves unaligned 16-byte global loads at full rate):
    //  (1) inside one record: one unaligned 16-byte load + one aligned store;
    //  (2) straddling two records of >= 16 bytes: the first one's last 16 bytes and the second's
    //      first 16 bytes (both loads stay inside their records) merged by one funnel shift;
    //  (3) anything else (version bytes, records < 16 B, segment edges): gather_block_slow.
    constexpr int U = SKV_GATHER_U;  // blocks per lane per iteration, loads issued before stores
    const uint32_t step = blockDim.x;
    const uint32_t nq = (uint32_t)(q1 - q0);
    // Fast pass: cases (1) and (2) only. Slow blocks are remembered in a per-lane bit mask (block
    // it*step + lane <-> bit it) and done after the loop, so the main loop carries no call.
    const bool use_mask = nq <= 32u * step;
    uint32_t slow = 0;
    auto fast_block = [&](uint32_t qi, uint4& v) -> bool {
        const uint64_t B = (q0 + qi) << 4;
        if (!(B >= lo_b && B + 16 <= hi_b)) return false;
        const uint32_t p = use_tbl ? s_tbl[qi] : gather_piece(s_dst, npieces, B);
        const uint64_t d = s_dst[p], src = s_src[p];
        const uint64_t len = s_dst[p + 1] - d;
        if (!src) return false;
        if (d + len >= B + 16) {
            v = *(const uint4*)((const uint8_t*)src + (B - d));
            return true;
        }
        if (p + 1 < npieces && len >= 16) {
            const uint64_t src2 = s_src[p + 1];
            const uint64_t len2 = s_dst[p + 2] - s_dst[p + 1];
            if (src2 && len2 >= 16 && s_dst[p + 1] + len2 >= B + 16) {
                const uint32_t k = (uint32_t)(d + len - B);  // bytes from the first record
                const uint4 L = *(const uint4*)((const uint8_t*)src + len - 16);
                const uint4 F = *(const uint4*)((const uint8_t*)src2);
                v = funnel16(L, F, 16 - k);
                return true;
            }
        }
        return false;
    };
    // Per batch of U blocks: addresses from LDS first, then every load, then the stores — no
    // branch around a load (the second load, the next record's head, is exec-masked to the lanes
    // of case 2), so the waitcnt pass does not drain between blocks.
    const uint64_t safe = (uint64_t)run_b;  // a readable address for lanes with nothing to load
    uint32_t it = 0;
    for (uint32_t qi = threadIdx.x; qi < nq; qi += U * step, it += U) {
        uint64_t aL[U], aX[U];
        uint32_t sh[U];
        bool ok[U], two[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t qq = qi + u * step;
            const bool inq = qq < nq;
            const uint32_t qc = inq ? qq : nq - 1;
            const uint64_t B = (q0 + qc) << 4;
            const bool inr = inq && B >= lo_b && B + 16 <= hi_b;
            const uint32_t p = use_tbl ? s_tbl[qc] : gather_piece(s_dst, npieces, B);
            const uint64_t d = s_dst[p], src = s_src[p], e = s_dst[p + 1];
            const uint64_t len = e - d;
            const bool c1 = src && e >= B + 16;  // (1) inside one record
            const uint32_t pn = p + 1 < npieces ? p + 1 : p;
            const uint64_t src2 = s_src[pn], len2 = s_dst[pn + 1] - s_dst[pn];
            const bool c2 = !c1 && src && p + 1 < npieces && len >= 16 && src2 && len2 >= 16 && e + len2 >= B + 16;
            ok[u] = inr && (c1 || c2);
            two[u] = ok[u] && c2;
            aL[u] = ok[u] ? (c1 ? src + (B - d) : src + len - 16) : safe;
            aX[u] = src2;
            sh[u] = 16u - (uint32_t)(e - B);  // case 2: bytes taken from the first record = e - B
            if (inq && !ok[u] && use_mask) slow |= 1u << (it + u);
        }
        uint4 L[U], X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            L[u] = gld16(aL[u]);
            X[u] = make_uint4(0, 0, 0, 0);
            if (two[u]) X[u] = gld16(aX[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint4 v = two[u] ? funnel16(L[u], X[u], sh[u] & 15u) : L[u];
            if (ok[u]) {
                uint8_t* o = out + ((q0 + qi + u * step) << 4);
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                u32x4 vv = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(vv, (u32x4*)o);
            }
        }
    }
    // Slow pass: case (3) — version bytes, records < 16 B, segment-edge blocks.
    auto slow_block = [&](uint32_t qi) {
        const uint64_t B = (q0 + qi) << 4;
        const uint64_t x0 = B > lo_b ? B : lo_b;
        const uint32_t p = use_tbl ? s_tbl[qi] : gather_piece(s_dst, npieces, x0);
        gather_block_slow(B, x0, B + 16 < hi_b ? B + 16 : hi_b, p, s_dst, s_src, out);
    };
    if (use_mask) {
        while (slow) {
            const uint32_t b = __builtin_ctz(slow);
            slow &= slow - 1;
            slow_block(threadIdx.x + b * step);
        }
    } else {
        for (uint32_t qi = threadIdx.x; qi < nq; qi += step) {
            uint4 v;
            if (!fast_block(qi, v)) slow_block(qi);
        }
    }
    // in-gather verify: this survivor's key against the record dropped after it as fingerprint-equal
    // (same length by construction); the survivor's lines are in L2 from the copy just done
    if (dupj) {
        const uint8_t* ra = (const uint8_t*)srcj;
        const uint32_t kl = __builtin_bswap32(load_window16(ra + 1, 4).x);
        if (!key_tails_equal(ra, (const uint8_t*)dupj, kl)) atomicOr(fp_bad, 1u);
    }
}

// ---------------------------------------------------------------------------------------
// device-wide exclusive scan of u64 (reduce -> scan partials -> apply), total at out[n]

constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_PER = 4;
constexpr uint64_t SCAN_BLOCK = SCAN_THREADS * SCAN_PER;

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(const uint64_t* in, uint64_t n, uint64_t* partial) {
    __shared__ uint64_t ws[16];
    uint64_t b0 = blockIdx.x * SCAN_BLOCK;
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        if (i < n) s += in[i];
    }
    uint64_t t = block_reduce_sum<uint64_t>(s, ws);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_apply(const uint64_t* in, uint64_t n, const uint64_t* partial_ex,
                                                             uint64_t* out) {
    __shared__ uint64_t ws[16];
    uint64_t b0 = blockIdx.x * SCAN_BLOCK;
    uint64_t v[SCAN_PER];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        v[q] = i < n ? in[i] : 0;
        s += v[q];
    }
    uint64_t tot;
    uint64_t ex = block_excl_scan<uint64_t>(s, ws, tot) + partial_ex[blockIdx.x];
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        if (i < n) out[i] = ex;
        ex += v[q];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == blockDim.x - 1) out[n] = ex;
}

// ---------------------------------------------------------------------------------------
// launch wrappers (C++ linkage, used by the host files skv_*host*.hip / skv_compact.hip)

static inline unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

void launch_run_header(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint32_t* hdr_err, RunFmt* fmt, bool slices) {
    if (n_runs) k_run_header<<<blocks_for(n_runs, 256), 256, 0, s>>>(runs, n_runs, hdr_err, fmt, slices);
}
void launch_spec(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                 const RunFmt* fmt, uint32_t* run_broken, uint64_t* ch_start, uint64_t* ch_end, uint32_t* ch_cnt,
                 uint32_t* ch_err, bool utf8, uint64_t chunk, uint16_t* slots, uint32_t cap, StgRec* stg,
                 uint32_t scap, uint8_t* ch_stg) {
    if (!n_chunks) return;
    if (utf8)
        k_spec<1><<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, hdr_err, fmt, run_broken, ch_start,
                                                            ch_end, ch_cnt, ch_err, chunk, slots, cap, stg, scap, ch_stg);
    else
        k_spec<0><<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, hdr_err, fmt, run_broken, ch_start,
                                                            ch_end, ch_cnt, ch_err, chunk, slots, cap, stg, scap, ch_stg);
}
void launch_validate(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                     const uint64_t* ch_start, const uint64_t* ch_end, const uint32_t* ch_err,
                     unsigned long long* bad_bits, uint32_t* run_first_bad) {
    if (n_chunks)
        k_validate<<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, hdr_err, ch_start, ch_end, ch_err,
                                                             bad_bits, run_first_bad);
}
void launch_fixup(hipStream_t s, const RunInfo* runs, uint32_t n_runs, const uint32_t* hdr_err,
                  const uint32_t* run_first_bad, const unsigned long long* bad_bits, uint64_t* ch_start,
                  uint64_t* ch_end, uint32_t* ch_cnt, uint32_t* ch_err, bool utf8, uint64_t chunk, uint16_t* slots,
                  uint32_t cap, uint8_t* ch_stg) {
    if (n_runs)
        k_fixup<<<n_runs, 64, 0, s>>>(runs, n_runs, hdr_err, run_first_bad, bad_bits, ch_start, ch_end, ch_cnt, ch_err,
                                       utf8, chunk, slots, cap, ch_stg);
}
void launch_err_chunk(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                      const uint32_t* ch_err, uint32_t* run_err_chunk) {
    if (n_chunks) k_err_chunk<<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, hdr_err, ch_err, run_err_chunk);
}
void launch_mask(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const uint32_t* hdr_err,
                 const uint32_t* run_err_chunk, const uint32_t* ch_cnt, uint64_t* cnt64) {
    if (n_chunks) k_mask<<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, hdr_err, run_err_chunk, ch_cnt, cnt64);
}
void launch_run_summary(hipStream_t s, const RunInfo* runs, uint32_t n_runs, const uint32_t* hdr_err,
                        const uint32_t* run_err_chunk, const uint32_t* ch_err, const uint64_t* ch_rec_base,
                        RunSummary* out, uint64_t* run_recb) {
    if (n_runs)
        k_run_summary<<<blocks_for(n_runs, 256), 256, 0, s>>>(runs, n_runs, hdr_err, run_err_chunk, ch_err, ch_rec_base,
                                                              out, run_recb);
}
void launch_emit(hipStream_t s, const RunInfo* runs, uint32_t n_runs, uint64_t n_chunks, const RunFmt* fmt,
                 const uint32_t* run_broken, const uint64_t* ch_start, const uint64_t* ch_rec_base,
                 const uint64_t* run_recb, uint64_t R, uint64_t* rec_addr, uint64_t* rec_hi, uint64_t* rec_lo,
                 uint32_t* rec_klen, uint32_t* rec_meta, uint32_t* flags, uint64_t* rec_fp, uint32_t* utf8_bad,
                 const uint16_t* slots, uint32_t cap, uint64_t chunk, const uint64_t* ch_end,
                 const uint64_t* stream_base, unsigned long long* first_dec, const StgRec* stg, uint32_t scap,
                 const uint8_t* ch_stg, uint64_t R_all, uint32_t* blk_chunk) {
    if (n_chunks)
        k_emit<<<blocks_for(n_chunks * EM_G, 256), 256, 0, s>>>(runs, n_runs, n_chunks, fmt, run_broken, ch_start,
                                                                ch_rec_base, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta,
                                                                flags, rec_fp, utf8_bad, slots, cap, chunk, ch_end,
                                                                stream_base, first_dec, stg, scap, ch_stg);
    if (n_chunks && R_all) {
        uint32_t* chunk_run = blk_chunk + R_all / 64 + 1;
        k_blk_chunk<<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, ch_rec_base, blk_chunk, chunk_run);
        k_emit_stg<<<blocks_for(R_all, 256 * EMS_R), 256, 0, s>>>(runs, n_runs, R_all, ch_rec_base, blk_chunk, chunk_run, rec_addr, rec_hi,
                                                           rec_lo, rec_klen, rec_meta, flags, rec_fp, utf8_bad, slots, cap,
                                                           chunk, ch_end, stream_base, first_dec, stg, scap, ch_stg);
    }
    if (R)
        k_emit_fixed<false><<<blocks_for(R, 256), 256, 0, s>>>(runs, n_runs, nullptr, R, fmt, (uint32_t*)run_broken, run_recb,
                                                               rec_addr, rec_hi, rec_lo, rec_klen, rec_meta, flags,
                                                               nullptr, nullptr, rec_fp);
    if (n_chunks && first_dec)
        k_chunk_order<<<blocks_for(n_chunks, 256), 256, 0, s>>>(runs, n_runs, n_chunks, ch_rec_base, stream_base,
                                                                rec_addr, rec_hi, rec_lo, rec_klen, first_dec, flags + 1);
}
void launch_parse_fixed(hipStream_t s, const RunInfo* runs, uint32_t n_runs, const RunFmt* fmt, uint32_t* run_broken,
                        const uint64_t* run_recb, uint64_t R, uint64_t* rec_addr, uint64_t* rec_hi, uint64_t* rec_lo,
                        uint32_t* rec_klen, uint32_t* rec_meta, uint32_t* flags, const uint64_t* stream_base,
                        unsigned long long* first_dec, uint64_t* rec_fp, uint32_t* wave_run, SElem* E) {
    if (!R) return;
    const uint64_t nw = (R + 63) >> 6;
    k_wave_run<<<blocks_for(nw, 256), 256, 0, s>>>(run_recb, n_runs, nw, wave_run);
    k_emit_fixed<true><<<blocks_for(R, 256), 256, 0, s>>>(runs, n_runs, wave_run, R, fmt, run_broken, run_recb, rec_addr,
                                                              rec_hi, rec_lo, rec_klen, rec_meta, flags, stream_base,
                                                              first_dec, rec_fp, E);
}
void launch_order_check(hipStream_t s, uint64_t R, const uint64_t* stream_base, uint32_t k, const uint64_t* rec_addr,
                        const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen,
                        unsigned long long* first_dec, uint32_t* any_dec) {
    if (R > 1)
        k_order_check<<<blocks_for(R, 256), 256, 0, s>>>(R, stream_base, k, rec_addr, rec_hi, rec_lo, rec_klen, first_dec,
                                                         any_dec);
}
void launch_sample(hipStream_t s, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                   const uint32_t* klen, const uint64_t* off_src, const uint64_t* off_dst, uint32_t k, uint64_t S,
                   uint64_t n_dst, uint64_t* dhi, uint64_t* dlo, uint64_t* dc) {
    if (!n_dst) return;
    Elems E{hi, lo, c, klen, nullptr};
    if (l0) k_sample<true><<<blocks_for(n_dst, 256), 256, 0, s>>>(E, off_src, off_dst, k, S, n_dst, dhi, dlo, dc);
    else k_sample<false><<<blocks_for(n_dst, 256), 256, 0, s>>>(E, off_src, off_dst, k, S, n_dst, dhi, dlo, dc);
}
void launch_bounds(hipStream_t s, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                   const uint32_t* klen, const uint64_t* off, uint32_t k, const uint64_t* shi, const uint64_t* slo,
                   const uint64_t* sc, uint64_t m, uint64_t T, const uint64_t* rec_addr, uint64_t* bounds,
                   const uint32_t* poison, const L1Cnt* C) {
    Elems E{hi, lo, c, klen, poison};
    uint64_t n = (T + 1) * k;
    if (!n) return;
    const L1Cnt none{};
    const L1Cnt& cc = C ? *C : none;
    if (l0) k_bounds<true><<<blocks_for(n, 256), 256, 0, s>>>(E, off, k, shi, slo, sc, m, T, rec_addr, bounds, cc);
    else k_bounds<false><<<blocks_for(n, 256), 256, 0, s>>>(E, off, k, shi, slo, sc, m, T, rec_addr, bounds, cc);
}
void launch_l1_cnt(hipStream_t s, const uint64_t* sc, uint64_t N1, const uint64_t* off0, const uint64_t* l1off,
                   uint32_t k, uint64_t S, uint64_t m, uint64_t T, uint32_t* posof, uint32_t* cnt) {
    if (!N1) return;
    k_l1_posof<<<blocks_for(N1, 256), 256, 0, s>>>(sc, N1, off0, l1off, k, S, posof);
    k_l1_cnt<<<blocks_for(N1, 256), 256, 0, s>>>(posof, N1, l1off, k, m, T, cnt);
}
void launch_key_fp(hipStream_t s, uint64_t R, const uint64_t* rec_addr, const uint32_t* rec_klen, uint64_t* fp) {
    if (R) k_key_fp<<<blocks_for(R, 256), 256, 0, s>>>(R, rec_addr, rec_klen, fp);
}
void launch_tile_n(hipStream_t s, const uint64_t* bounds, uint32_t k, uint64_t T, uint64_t* tile_n) {
    if (!T) return;
    k_tile_n<<<blocks_for(T, 256), 256, 0, s>>>(bounds, k, T, tile_n);
}
void launch_fp_verify(hipStream_t s, const unsigned long long* vlo, const unsigned long long* vcount,
                      const uint64_t* vpairs, uint64_t cap, uint32_t* fp_bad, unsigned max_blocks) {
    unsigned blocks = blocks_for(cap ? cap : 1, 256);
    if (blocks > max_blocks) blocks = max_blocks;
    k_fp_verify<<<blocks, 256, 0, s>>>(vlo, vcount, vpairs, fp_bad);
}
size_t tile_lds_bytes(uint32_t k) {
    size_t b = (size_t)TILE_CAP * (4 * 8 + 2 + 2) + 2 * (size_t)(k + 1) * 4;
    b = (b + 15) & ~(size_t)15;
    return b + 16 * 8 + 32 * 4;  // ws[16] u64, then 32 u32 (tile_minmax)
}
hipError_t launch_tile(hipStream_t s, bool l0, const uint64_t* hi, const uint64_t* lo, const uint64_t* c,
                       const uint32_t* klen, const uint64_t* bounds, uint32_t k, uint64_t T, const uint64_t* tile_base,
                       const uint32_t* rec_meta, const uint64_t* rec_addr, uint32_t drop, TileOut O,
                       const uint32_t* poison, uint64_t grid) {
    Elems E{hi, lo, c, klen, poison};
    if (!grid) grid = T;  // level 0 takes tickets: launches of grid < T tiles continue each other
    size_t lds = tile_lds_bytes(k);
    lds_limit(l0 ? (const void*)k_tile<true> : (const void*)k_tile<false>);
    if (l0) {
        k_tile<true><<<(unsigned)grid, TILE_THREADS, lds, s>>>(E, bounds, k, tile_base, rec_meta, rec_addr, drop, O);
    } else {
        k_tile<false><<<(unsigned)T, TILE_THREADS, lds, s>>>(E, bounds, k, tile_base, rec_meta, rec_addr, drop, O);
    }
    return hipGetLastError();
}
void launch_chain(hipStream_t s, const uint64_t* Kp, const uint64_t* P, uint64_t max_size, const uint32_t* tile_max,
                  uint64_t n_tiles, uint64_t* run_b, uint64_t* n_runs, uint32_t* tbl, uint64_t max_K,
                  uint64_t max_bytes, const SplitBufs* sp) {
    const uint64_t n_tbl = tbl ? (max_bytes >> CH_SHIFT) + 2 : 0;
    const SplitPlan* plan = nullptr;
    if (sp && sp->nseg_cap) {
        plan = sp->plan;
        k_split_plan<<<1, SPLIT_PLAN_THREADS, 0, s>>>(Kp, P, max_size, tile_max, n_tiles, *sp);
        k_split_guess<<<(sp->nseg_cap + SPLIT_GUESS_SEGS - 1) / SPLIT_GUESS_SEGS, 64, 0, s>>>(P, max_size, *sp);
        k_split_scan<<<1, SPLIT_PLAN_THREADS, 0, s>>>(*sp);
        const unsigned wb = sp->nc < 64 ? 64 : (sp->nc < 256 ? sp->nc : 256);
        k_split_walk<<<sp->nseg_cap * ((sp->nc + wb - 1) / wb), wb, 0, s>>>(P, max_size, *sp);
        k_split_stitch<<<1, SPLIT_STITCH_THREADS, 0, s>>>(P, max_size, *sp, run_b, n_runs);
        k_split_emit<<<blocks_for((uint64_t)sp->nseg_cap * sp->segr, 256), 256, 0, s>>>(*sp, run_b);
    }
    if (tbl) {  // grid-stride (capped grid): with the parallel split it only reads the plan
        unsigned tb = blocks_for(max_K + 1, 256);
        if (tb > 8192) tb = 8192;
        k_chain_table<<<tb, 256, 0, s>>>(Kp, P, tbl, n_tbl, plan);
    }
    k_chain<<<1, 64, 0, s>>>(Kp, P, max_size, tile_max, n_tiles, run_b, n_runs, tbl, n_tbl, plan);
}
uint64_t chain_table_entries(uint64_t max_bytes) { return (max_bytes >> CH_SHIFT) + 2; }
// ---- carried open runs (skv_compact_split, variable-length records) -------------------------
// build_runs (runs.rs:211-238) closes the current run before a record that would take it past max;
// a run carried in with c bytes (version byte included) keeps taking this part's records while
// c + their bytes <= max. One lane: a binary search of P.
__global__ void k_carry_first(const uint64_t* __restrict__ Kp, const uint64_t* __restrict__ P, uint64_t max_size,
                              uint64_t c, uint64_t* out) {
    if (threadIdx.x) return;
    const uint64_t K = *Kp;
    uint64_t e = 0;
    if (c < max_size) {
        const uint64_t v = sat_add_u64(P[0], max_size - c);  // record j joins iff P[j + 1] <= v
        uint64_t lo = 0, hi = K;                   // largest e in [0, K] with P[e] <= v
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if (P[mid] <= v) lo = mid;
            else hi = mid - 1;
        }
        e = lo;
    }
    out[0] = e;
    out[1] = K - e;
}
__global__ void __launch_bounds__(1024) k_carry_fix(uint64_t* run_b, uint64_t* n_runs_out, const uint64_t* __restrict__ P,
                                                    uint64_t e1, uint64_t K) {
    const uint64_t m = n_runs_out[0];  // runs of the suffix; run_b[1 .. m + 1] its starts and end
    __syncthreads();
    for (uint64_t i = 1 + threadIdx.x; i <= m + 1; i += blockDim.x) run_b[i] += e1;
    if (threadIdx.x == 0) {
        run_b[0] = 0;
        n_runs_out[0] = m + 1;
        n_runs_out[1] = K;
        n_runs_out[2] = P[K];  // (an empty suffix left 0 here)
    }
}
__global__ void k_carry_out(const uint64_t* __restrict__ run_b, const uint64_t* __restrict__ n_runs_out,
                            const uint64_t* __restrict__ P, uint64_t c, uint32_t cont, uint64_t* out) {
    if (threadIdx.x) return;
    const uint64_t n = n_runs_out[0], K = n_runs_out[1];
    if (n == 0) *out = c;  // no records: the carried run stays open as it came
    else if (cont && n == 1) *out = c + (P[K] - P[0]);
    else *out = 1 + (P[K] - P[run_b[n - 1]]);
}
void launch_carry_first(hipStream_t s, const uint64_t* Kp, const uint64_t* P, uint64_t max_size, uint64_t c,
                        uint64_t* out) {
    k_carry_first<<<1, 64, 0, s>>>(Kp, P, max_size, c, out);
}
void launch_carry_fix(hipStream_t s, uint64_t* run_b, uint64_t* n_runs_out, const uint64_t* P, uint64_t e1, uint64_t K) {
    k_carry_fix<<<1, 1024, 0, s>>>(run_b, n_runs_out, P, e1, K);
}
void launch_carry_out(hipStream_t s, const uint64_t* run_b, const uint64_t* n_runs_out, const uint64_t* P, uint64_t c,
                      uint32_t cont, uint64_t* out) {
    k_carry_out<<<1, 64, 0, s>>>(run_b, n_runs_out, P, c, cont, out);
}
void launch_run_stats(hipStream_t s, const uint64_t* n_runs, const uint64_t* run_b, const uint64_t* P,
                      const uint64_t* Dp, const uint32_t* m_rec, const uint32_t* rec_klen, DevRunDesc* descs,
                      uint64_t* seg_r0, uint64_t max_runs) {
    unsigned blocks = blocks_for(max_runs ? max_runs : 1, 256);
    if (blocks > 4096) blocks = 4096;
    k_run_stats<<<blocks, 256, 0, s>>>(n_runs, run_b, P, Dp, m_rec, rec_klen, descs, seg_r0);
}
void launch_gather(hipStream_t s, const uint64_t* Kp, const uint64_t* n_runs, const uint64_t* run_b, const uint64_t* P,
                   const uint64_t* m_src, const uint64_t* seg_r0, uint8_t* out, uint64_t max_K, const uint64_t* m_dup,
                   uint32_t* fp_bad) {
    if (!max_K) return;
    k_gather<<<blocks_for(max_K, GATHER_SEG), GATHER_THREADS, 0, s>>>(Kp, n_runs, run_b, P, m_src, seg_r0, out, m_dup,
                                                                      fp_bad);
}
// small n: one workgroup walks the input in SCAN_BLOCK pieces with a running carry (one launch)
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_single(const uint64_t* in, uint64_t n, uint64_t* out) {
    __shared__ uint64_t ws[16];
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < n; b0 += SCAN_BLOCK) {
        uint64_t v[SCAN_PER];
        uint64_t s = 0;
#pragma unroll
        for (int q = 0; q < SCAN_PER; ++q) {
            uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
            v[q] = i < n ? in[i] : 0;
            s += v[q];
        }
        uint64_t tot;
        uint64_t ex = block_excl_scan<uint64_t>(s, ws, tot) + carry;
#pragma unroll
        for (int q = 0; q < SCAN_PER; ++q) {
            uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
            if (i < n) out[i] = ex;
            ex += v[q];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

// The same scan over a count known only on the device (n = min(*dn, max_n)): blocks past n do no
// memory work, and the total goes to out[n] and out[max_n] (where readers of the host-sized form
// look). Entries of `in` past n are never read. (WAL stage: per-table arrays sized by the merged
// record count, of which the first NT, the table count, are live.)
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce_dn(const uint64_t* in, const uint64_t* dn,
                                                                uint64_t max_n, uint64_t* partial) {
    __shared__ uint64_t ws[16];
    const uint64_t n = *dn < max_n ? *dn : max_n;
    const uint64_t b0 = blockIdx.x * SCAN_BLOCK;
    if (b0 >= n) {
        if (threadIdx.x == 0) partial[blockIdx.x] = 0;
        return;
    }
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        if (i < n) s += in[i];
    }
    uint64_t t = block_reduce_sum<uint64_t>(s, ws);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_apply_dn(const uint64_t* in, const uint64_t* dn, uint64_t max_n,
                                                               const uint64_t* partial_ex, uint64_t nb, uint64_t* out) {
    __shared__ uint64_t ws[16];
    const uint64_t n = *dn < max_n ? *dn : max_n;
    const uint64_t b0 = blockIdx.x * SCAN_BLOCK;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[n] = partial_ex[nb];
        out[max_n] = partial_ex[nb];
    }
    if (b0 >= n) return;
    uint64_t v[SCAN_PER];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        v[q] = i < n ? in[i] : 0;
        s += v[q];
    }
    uint64_t tot;
    uint64_t ex = block_excl_scan<uint64_t>(s, ws, tot) + partial_ex[blockIdx.x];
#pragma unroll
    for (int q = 0; q < SCAN_PER; ++q) {
        uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + q;
        if (i < n) out[i] = ex;
        ex += v[q];
    }
}
void launch_scan_dn(hipStream_t s, const uint64_t* in, const uint64_t* dn, uint64_t max_n, uint64_t* out,
                    uint64_t* tmp) {
    const uint64_t nb = (max_n + SCAN_BLOCK - 1) / SCAN_BLOCK;
    if (nb == 0) {
        (void)hipMemsetAsync(out, 0, 8, s);
        return;
    }
    uint64_t* partial = tmp;
    uint64_t* partial_ex = tmp + nb;
    k_scan_reduce_dn<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, dn, max_n, partial);
    launch_scan(s, partial, nb, partial_ex, tmp + 2 * nb + 2);
    k_scan_apply_dn<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, dn, max_n, partial_ex, nb, out);
}

// exclusive scan of n u64 values into out[0..n] (out[n] = total); tmp needs scan_tmp_words(n)
uint64_t scan_tmp_words(uint64_t n) {
    uint64_t w = 0;
    while (true) {
        uint64_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
        w += 2 * nb + 2;
        if (nb <= 1) break;
        n = nb;
    }
    return w;
}
void launch_scan(hipStream_t s, const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* tmp) {
    uint64_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
    if (nb == 0) {
        (void)hipMemsetAsync(out, 0, 8, s);
        return;
    }
    if (nb <= 16) {
        k_scan_single<<<1, SCAN_THREADS, 0, s>>>(in, n, out);
        return;
    }
    uint64_t* partial = tmp;
    uint64_t* partial_ex = tmp + nb;
    k_scan_reduce<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, n, partial);
    if (nb == 1) {
        (void)hipMemsetAsync(partial_ex, 0, 8, s);
    } else {
        launch_scan(s, partial, nb, partial_ex, tmp + 2 * nb + 2);
    }
    k_scan_apply<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, n, partial_ex, out);
}

}  // namespace skv
