// skv_dev.hpp — shared definitions of the MI355X compaction path (device + host side).
//
// Data layout in HBM (one compaction, see DESIGN.md "Data layout"):
//   runs[]          RunInfo per input member run, in "rank order": streams sorted by seq_no
//                   descending, members in stream order. Record index (rec_idx) follows the same
//                   order, so for equal keys "smaller rec_idx" == "newer seq_no" == the record
//                   k_way::merge keeps (k_way.rs:20-27, :146-151).
//   chunk arrays    per CHUNK bytes of run body: speculative walk summaries.
//   record arrays   per record (rec_idx): absolute address, 16-byte BE key prefix, key length,
//                   meta = size | is_delete<<31.
//   merged arrays   per surviving record in output order: source address, output-byte prefix P,
//                   delete-count prefix, rec_idx.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace skv {

#define SKV_CHUNK 4096
constexpr uint64_t CHUNK = SKV_CHUNK;     // bytes of run body per speculative walk lane
#define SKV_TILE_CAP 4096
#define SKV_TILE_TARGET 3072
#define SKV_TILE_THREADS 1024
constexpr int TILE_CAP = SKV_TILE_CAP;          // max elements a merge tile sorts in LDS
constexpr int TILE_TARGET = SKV_TILE_TARGET;    // target elements per merge tile
constexpr int TILE_THREADS = SKV_TILE_THREADS;
#define SKV_GATHER_SEG 256
constexpr int GATHER_SEG = SKV_GATHER_SEG;      // surviving records per gather workgroup
#define SKV_GATHER_THREADS SKV_GATHER_SEG
constexpr int GATHER_THREADS = SKV_GATHER_THREADS;  // >= GATHER_SEG: one lane per record in the setup
static_assert(SKV_GATHER_THREADS >= SKV_GATHER_SEG && SKV_GATHER_THREADS % 64 == 0, "gather block shape");
constexpr int GATHER_TBL = 23 * SKV_GATHER_SEG; // output 16-byte blocks per gather workgroup with a direct piece table
#define SKV_GATHER_U 2                   // output blocks per lane in flight in k_gather
#define SKV_GATHER_WAVES 8               // k_gather register budget: waves per SIMD (64 VGPRs at 8)
#ifndef SKV_TILE_PROF
#define SKV_TILE_PROF 0                  // 1: k_tile<true> accumulates per-phase times (diagnostic builds)
#endif
constexpr uint32_t NO_POS32 = 0xFFFFFFFFu;
constexpr uint64_t NO_POS = ~0ull;

// device-side error codes of a record walk (mapped to skv.h codes + reference text on the host)
enum : uint32_t {
    DERR_NONE = 0,
    DERR_EMPTY = 1,        // RunError::EmptyInput                     runs.rs:537-540
    DERR_VERSION = 2,      // RunError::UnsupportedVersion(v)          runs.rs:553-556
    DERR_IO = 3,           // RunError::Io (read_u32 past the end)     runs.rs:570-576, :598-604
    DERR_KEY = 4,          // Format("Incomplete key data")            runs.rs:580-583
    DERR_UTF8 = 5,         // Format("Invalid UTF-8 in key")           runs.rs:585-591
    DERR_VAL = 6,          // Format("Incomplete value data")          runs.rs:608-611
    DERR_MARKER = 7,       // Format("Invalid marker byte: {m}")       runs.rs:621-624
};
// err word = code | extra_byte << 8

struct RunInfo {
    uint64_t ptr;         // absolute device address of the run's first byte (version byte)
    uint64_t len;         // run length in bytes
    uint64_t chunk_base;  // first global chunk index of this run
    uint32_t n_chunks;
    uint32_t stream;      // stream rank (seq_no descending)
};

struct RunFmt {           // fixed-stride hypothesis of a run (S == 0: none)
    uint64_t S;           // record size
    uint32_t K, V;        // key / value length
    uint64_t first;       // size of the run's first record (0: none, or it does not decode)
};

struct RunSummary {       // per run, read back by the host after the parse
    uint64_t records;     // records decoded before the first error of the run
    uint32_t err;         // DERR_* | extra << 8 (0 = none)
    uint32_t pad;
};

// level-0 bounds narrowed by the level-1 sample counts (k_l1_cnt); cnt == null: plain searches
struct L1Cnt {
    const uint32_t* cnt;     // (T + 1) x k
    const uint64_t* l1off;   // level-1 list offsets (k + 1)
    const uint64_t *hi, *lo, *c;  // level-1 samples, list order
    uint64_t S;              // level-1 step (records)
};

// parallel greedy split (k_split_*): the plan k_split_plan leaves for the later kernels
constexpr uint32_t SPLIT_SERIAL = 0, SPLIT_PAR = 1;
constexpr uint32_t SPLIT_FB = 0xFFFFFFFFu;  // seg_sel: the stitch walked this segment itself
struct SplitPlan {
    uint32_t mode;       // SPLIT_SERIAL: k_chain splits; SPLIT_PAR: k_split_walk/stitch/emit did
    uint32_t nseg;       // segments with windows
    uint32_t nseg_sel;   // segments the stitch resolved from a window or walked (seg_sel valid)
    uint32_t n_fb;       // segments the stitch had to walk (true start outside the window)
    uint64_t K, PK, L0;  // records, output record bytes, first-run record count guess
    uint64_t avg, adv;   // average record bytes, expected bytes per run
};
struct SplitBufs {
    SplitPlan* plan;
    uint64_t* seg_w;     // window: first candidate record of segment s
    uint32_t* seg_n;     // window: candidates
    uint32_t* seg_sel;   // the true start's candidate index (SPLIT_FB: walked by the stitch)
    uint64_t* seg_D;     // guess walks: bytes advanced by segr runs, then their exclusive prefix G_s
    uint32_t* chain;     // [s][k < segr][candidate] run starts of each candidate's chain
    uint32_t* ends;      // [s][candidate] where the candidate's segr runs end (next segment's start)
    uint32_t nseg_cap, segr, nc;  // segments allocated, runs per segment, candidates per window
    uint64_t min_runs;   // fewer expected runs: SPLIT_SERIAL (the single-wave chain is as fast)
};

struct TileOut {
    // level > 0: sorted elements
    uint64_t* ohi;
    uint64_t* olo;
    uint64_t* oc;
    // level 0: the dense merged arrays (k_tile emits them directly, decoupled look-back)
    uint32_t* m_rec;      // rec index of the g-th surviving record
    uint64_t* m_src;      // its source address
    uint64_t* m_P;        // output-byte prefix (m_P[K] = total)
    uint64_t* m_Dp;       // delete-count prefix
    uint32_t* tile_mm;    // (min, max) surviving record size per tile
    uint64_t* tstate;     // look-back words, 3 per tile (zeroed per call)
    uint32_t* tcounter;   // tile ticket (zeroed per call)
    uint64_t* Kout;       // K = surviving records
    uint64_t T;           // level-0 tile count
    uint64_t* prof;       // SKV_TILE_PROF builds: per-phase time of level-0 tiles (8 counters)
    // level 0: fingerprints of the key bytes past 16 (k_key_fp); equal prefix, length and
    // fingerprint count as equal in the merge rounds and in first-per-key. Each adjacent pair taken
    // as equal that way goes to vpairs (the two records' addresses); k_fp_verify compares their
    // bytes, and a pair that differs sets *fp_bad (the host reruns with exact compares)
    const uint64_t* key_fp;
    uint32_t* fp_bad;
    uint64_t* vpairs;
    unsigned long long* vcount;
    // in-gather verify (no Delete filter, k_gather as the output stage): m_dup[g] = the address of
    // the record dropped right after the g-th survivor as fingerprint-equal to it (0: none); k_gather
    // compares the two keys while the survivor's lines are in L2 from its own copy, and only the other
    // pairs (a dropped record after a dropped one) go to vpairs. Null: every pair goes to vpairs.
    uint64_t* m_dup;
    // global scratch for tiles larger than TILE_CAP
    uint64_t* xhi;
    uint64_t* xlo;
    uint64_t* xc;
    uint32_t* xmeta;
    // heap-order mode (skv_heap.hip; unsorted input streams under the Delete filter or the WAL
    // split): the merge compares each record's stream-prefix-maximum key (which is how
    // k_way::merge's heap pops unsorted streams), while first-per-key compares the records' own
    // keys (act_*), the payload is the record itself (pay_addr) and pop_pos[rec] records every
    // record's position in the pop sequence. All null otherwise.
    const uint64_t* pay_addr;
    const uint64_t* act_hi;
    const uint64_t* act_lo;
    const uint32_t* act_klen;
    uint64_t* pop_pos;
};

// Fused stride path (skv_stride.hip): every input record is a Put of one size S with one key
// length K <= 16, so record addresses, output offsets and the greedy split are arithmetic.
#define SKV_FX_THREADS 512
#define SKV_FX_U 2                       // output blocks per lane per batch in the fused copy (two batches in flight)
#define SKV_FX_CAP 2048                  // 2048: 63 VGPRs, 4 workgroups per CU (4096: 91 VGPRs, 2 per CU; 3 % slower end to end)
constexpr int FX_HSLOTS = 2 * SKV_FX_CAP;  // distinct-key hash slots per fused tile (load <= 1/2)
constexpr int FX_CAP = SKV_FX_CAP;       // max records per fused tile
constexpr int FX_TARGET = FX_CAP / 4 * 3;  // target records per fused tile (splitter spacing)
constexpr int FX_THREADS = SKV_FX_THREADS;
constexpr uint64_t FX_MIN_S = 32;        // a 16-byte output block touches at most two records
constexpr uint64_t FX_MAX_S = 1u << 19;  // tile output spans stay below 2^31 bytes (u32 offsets)
constexpr uint32_t FX_MAX_K = 16;        // the whole key is the 16-byte compare prefix

struct FxBound {                  // per (tile boundary t, stream j), written by k_fx_bounds
    uint64_t pos;                 // first record of stream j whose key >= splitter t
    uint64_t addr;                // its address (pos < stream end)
    uint64_t rem;                 // records of its member run from pos on
    uint64_t has_prev;            // pos > stream start: ph/pl = key of record pos - 1
    uint64_t ph, pl;
};

struct FxArgs {
    const RunInfo* runs;
    const uint64_t* run_recb;     // records before run r, rank order (n_runs + 1)
    const uint32_t* stream_run;   // first run of stream j (k + 1)
    const uint64_t* stream_base;  // first record of stream j (k + 1)
    FxBound* bnd;                 // level-0 tile bounds, (T + 1) x k
    uint32_t k;
    uint32_t K, V;                // key / value length of every record
    uint32_t pad;
    uint64_t S;                   // record size
    uint64_t n;                   // records per output run (build_runs' greedy split, arithmetic)
    double inv_S, inv_W, inv_n;   // reciprocals for fx_divmod (W = n * S + 1 bytes per output run)
    uint64_t T;                   // level-0 tiles
    uint8_t* out;
    uint32_t* flags;              // [2] poison (result discarded, general path reruns), [3] reason bits
    uint64_t* tstate;             // look-back word per tile (zeroed per call)
    uint32_t* tcounter;           // tile ticket (zeroed per call)
    uint64_t* Kout;               // surviving records (through this launch's records)
    const uint64_t* gbase;        // survivors before this launch's records (a key-range part of a
                                  // pipelined host call, skv_hostpipe.hip), or null: 0
    uint64_t* prof;               // SKV_TILE_PROF builds: per-phase ticks of the fused tiles (16 counters)
    // k_fx_bounds' inputs: the sorted level-1 samples (every m-th is a splitter) and each stream's
    // own level-1 samples (every Sstep-th record, offsets l1off)
    const uint64_t *shi, *slo, *l1hi, *l1lo, *l1off;
    uint64_t m, Sstep;
    // splitter t is sorted sample t*m for t <= T1, then T1*m + (t - T1)*m2: the last generation of
    // tiles is shorter (m2 < m) so the grid drains sooner (T1 = T, m2 = m: uniform tiles)
    uint64_t T1, m2;
    const uint32_t* l1cnt;        // (T + 1) x k: stream j's level-1 samples sorted before splitter t
                                  // (k_fx_l1cnt), or null: k_fx_bounds searches them
};
// Higher sample levels written by k_fx_sample itself: level-1 sample c of stream j is also level
// 2's sample c / Sstep when Sstep divides c (and level 3's when Sstep^2 does) -- the same element
// (key, K << 32 | record) that k_sample would copy from level 1, without its launch per level
struct FxUpLevels {
    uint64_t *hi[2], *lo[2], *c[2];
    const uint64_t* off[2];  // per-stream offsets of the level (k + 1)
    uint32_t n;              // levels written (0..2)
};
// flags[3] reason bits of a poisoned fused call
enum : uint32_t { FXR_RECORD = 1, FXR_OVERSIZE = 2, FXR_SPLIT = 4, FXR_ORDER = 8, FXR_SAMPLE = 16 };

// Record sort for merges of more than TILE_TARGET / 2 streams (skv_sort.hip)
struct SElem {
    uint64_t hi, lo;              // 16-byte key prefix (big-endian, zero padded)
    uint64_t addr;                // record address (key at addr + 5)
    uint32_t pos, klen;           // record index (rank order), key length
};
constexpr int SORT_CAP = 2048;           // elements a bucket sorts in LDS
constexpr int SORT_THREADS = 256;
#define SKV_SORT_EVERY 48
constexpr uint64_t SORT_EVERY = SKV_SORT_EVERY;  // one sample per SORT_EVERY elements
#define SKV_SORT_OV 16
constexpr uint64_t SORT_OV = SKV_SORT_OV;  // samples per bucket (bucket target SORT_EVERY * SORT_OV = 768)

// Batched run lookups (skv_search.hip): same layout and codes as skv_lookup / SKV_LOOKUP_* /
// SKV_PANIC_* in include/skv.h
struct SrResult {
    uint32_t kind, panic;
    uint64_t val_off, val_len;
};
enum : uint32_t { SR_NOT_FOUND = 0, SR_FOUND = 1, SR_TOMBSTONE = 2, SR_PANIC = 3 };
enum : uint32_t {
    SRP_EMPTY = 1, SRP_VERSION = 2, SRP_MARKER = 3, SRP_KEYLEN = 4, SRP_KEY = 5, SRP_VALLEN = 6, SRP_VAL = 7,
    SRP_VALLEN_FOUND = 8, SRP_VAL_FOUND = 9
};

// WAL key errors (wal_compaction.rs:71-79): no '.', or Rust's ParseIntError kinds
enum : uint32_t { WERR_NONE = 0, WERR_NODOT, WERR_EMPTY, WERR_DIGIT, WERR_POS, WERR_NEG };

struct DevRunDesc {       // == skv_run_desc layout
    uint64_t off, len, put_count, delete_count;
    uint64_t min_key_off, min_key_len, max_key_off, max_key_len;
    int64_t table_id;
    uint64_t reserved;
};

// ------------------------------------------------------------------------------------------
#ifdef __HIPCC__

__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p) { return *p; }

__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
    return (ld_u8(p) << 24) | (ld_u8(p + 1) << 16) | (ld_u8(p + 2) << 8) | ld_u8(p + 3);
}

// core::str::from_utf8 acceptance (runs.rs:585), streaming over global memory.
__device__ inline bool utf8_valid(const uint8_t* s, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint32_t c = s[i];
        if (c < 0x80) { ++i; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEC) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c >= 0xEE && c <= 0xEF) need = 2;
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return false;
        if (n - i - 1 < need) return false;
        uint32_t c1 = s[i + 1];
        if (c1 < lo || c1 > hi) return false;
        for (uint32_t k = 2; k <= need; ++k) {
            uint32_t ck = s[i + k];
            if (ck < 0x80 || ck > 0xBF) return false;
        }
        i += need + 1;
    }
    return true;
}

// Compare-exchange i of the bitonic stage (kk = 2^lk, jj = 2^lj) in the ascending-comparator form:
// the first stage of each merge pairs mirrored positions, the others pairs jj apart. Shifts, not
// the division by jj (a 32-bit integer division is a long instruction sequence on gfx950).
__device__ __forceinline__ void bitonic_pair(uint32_t i, uint32_t lk, uint32_t lj, uint32_t& a, uint32_t& c) {
    const uint32_t off = i & ((1u << lj) - 1), blk = i >> lj;
    if (lj + 1 == lk) {
        a = (blk << lk) + off;
        c = (blk << lk) + (1u << lk) - 1 - off;
    } else {
        a = (blk << (lj + 1)) + off;
        c = a + (1u << lj);
    }
}

// v of lane (lane ^ M) inside a wave, without the LDS crossbar (ds_bpermute, which __shfl_xor
// lowers to): DPP quad permutes for 1 and 2, row rotates for 4 and 8, the gfx950 half-row / half-wave
// swaps for 16 and 32. M is a compile-time constant.
template <int M>
__device__ __forceinline__ uint32_t xshfl(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (M == 4) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
        const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);  // row_ror:12
        return (lane & 4) ? a : b;
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (M == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // odd rows <-> even rows
        return (lane & 16) ? r[0] : r[1];
    } else {
        static_assert(M == 32, "xshfl: M in {1, 2, 4, 8, 16, 32}");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // upper half <-> lower half
        return (lane & 32) ? r[0] : r[1];
    }
}
template <int M>
__device__ __forceinline__ uint64_t xshfl64(uint64_t v) {
    return ((uint64_t)xshfl<M>((uint32_t)(v >> 32)) << 32) | xshfl<M>((uint32_t)v);
}

// a + b, saturating at 2^64 - 1 (a run's byte budget P[b] + max - 1 with max near 2^64: runs.rs:219
// compares u64 sizes without overflow)
__device__ __forceinline__ uint64_t sat_add_u64(uint64_t a, uint64_t b) { return b > ~0ull - a ? ~0ull : a + b; }

struct WalkRes {
    uint64_t end;   // first record start >= stop, or the erroring record's start
    uint32_t cnt;   // records decoded
    uint32_t err;   // DERR_* | extra << 8
    uint32_t nst;   // records staged (walk_fast<.., true>): the first nst of the chunk
};
struct StgRec {  // a walked record's arrays, staged by its chunk slot (32 bytes, two 16-byte stores)
    uint64_t hi, lo;    // key prefix words
    uint64_t fp;        // fingerprint of the key bytes past 16
    uint32_t klen_del;  // key length | Delete << 31
    uint32_t ascii;     // 1: every key byte is ASCII (else k_emit checks the key's UTF-8)
};
// Staged entry i of chunk c sits at ((c / STG_W) * scap + i) * STG_W + c % STG_W: the walks of a
// wave (consecutive chunks, one record per step each) store one contiguous 2 KiB block per step.
// (A row per chunk put the lanes of a store 16 KiB apart: k_spec 1.2 s instead of 10 ms at 3F.)
// SKV_STG_PROBE (diagnostic builds, output invalid): 1 no fingerprint in the staging walk, 2 no
// staged stores (the entries computed, not written)
#ifndef SKV_STG_PROBE
#define SKV_STG_PROBE 0
#endif
constexpr uint32_t STG_W = 64;
constexpr uint64_t STG_KMAX = 144;  // longest key the walks stage (two fingerprint steps)
__device__ __forceinline__ uint64_t stg_base(uint64_t c, uint32_t scap) {
    return (c / STG_W) * scap * STG_W + c % STG_W;
}

// runs::read_run_stream's per-record loop (runs.rs:559-626) over [p, stop) of one run, in the
// reference's check order. max_recs bounds the walk (probe mode).
__device__ inline WalkRes walk_checked(const uint8_t* run, uint64_t len, uint64_t p, uint64_t stop,
                                       uint32_t max_recs) {
    uint32_t cnt = 0;
    while (p < stop && cnt < max_recs) {
        uint32_t marker = run[p];
        if (p + 5 > len) return {p, cnt, DERR_IO};
        uint64_t klen = ld_be32(run + p + 1);
        uint64_t kp = p + 5;
        if (kp + klen > len) return {p, cnt, DERR_KEY};
        if (!utf8_valid(run + kp, klen)) return {p, cnt, DERR_UTF8};
        uint64_t size;
        if (marker == 1) {
            if (kp + klen + 4 > len) return {p, cnt, DERR_IO};
            uint64_t vlen = ld_be32(run + kp + klen);
            if (kp + klen + 4 + vlen > len) return {p, cnt, DERR_VAL};
            size = 9 + klen + vlen;
        } else if (marker == 2) {
            size = 5 + klen;
        } else {
            return {p, cnt, DERR_MARKER | (marker << 8)};
        }
        ++cnt;
        p += size;
    }
    return {p, cnt, DERR_NONE};
}

// big-endian 16-byte key prefix (zero padded) of a key of klen bytes at k
__device__ inline void key_prefix(const uint8_t* k, uint64_t klen, uint64_t& hi, uint64_t& lo) {
    uint64_t h = 0, l = 0;
    uint32_t n = klen < 16 ? (uint32_t)klen : 16u;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        uint64_t b = j < n ? (uint64_t)k[j] : 0ull;
        if (j < 8) h |= b << (56 - 8 * j);
        else l |= b << (56 - 8 * (j - 8));
    }
    hi = h;
    lo = l;
}


// The aligned 16-byte block at global address a. Run bytes and every device buffer these helpers
// read live in global memory: loading through the global address space keeps the loads off
// lgkmcnt (a flat load counts against both counters and serialises with every LDS wait of the
// kernels that merge in LDS).
typedef unsigned int gblk_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gblk(uintptr_t a) {
    const gblk_v4 v = *(const __attribute__((address_space(1))) gblk_v4*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Block loader of the record parsers below (a template parameter, so a parser can be pointed at
// another copy of the bytes)
struct GLoad {
    __device__ __forceinline__ uint4 operator()(uintptr_t a) const { return gblk(a); }
};

// 16 bytes from an arbitrary (unaligned) address using two aligned 16-byte loads. The second
// aligned block contains p+15, so it holds at least one byte the caller owns and never crosses
// into an unmapped page.
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t* p) {
    uintptr_t a = (uintptr_t)p;
    const uintptr_t base = a & ~(uintptr_t)15;
    uint32_t sh = (uint32_t)(a & 15);
    uint4 x = gblk(base);
    if (sh == 0) return x;
    uint4 y = gblk(base + 16);
    uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    uint32_t q = sh >> 2, r = sh & 3;
    uint32_t s[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        uint32_t v0 = w[i], v1 = w[i + 1], v2 = w[i + 2], v3 = (i + 3 < 8) ? w[i + 3] : 0u;
        s[i] = q == 0 ? v0 : (q == 1 ? v1 : (q == 2 ? v2 : v3));
    }
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(s[1], s[0], r);
    o.y = __builtin_amdgcn_alignbyte(s[2], s[1], r);
    o.z = __builtin_amdgcn_alignbyte(s[3], s[2], r);
    o.w = __builtin_amdgcn_alignbyte(s[4], s[3], r);
    return o;
}

// bytes [sh, sh+16) of the 32-byte little-endian concatenation x|y (sh in 0..15)
__device__ __forceinline__ uint4 funnel16(uint4 x, uint4 y, uint32_t sh) {
    if (sh == 0) return x;
    uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    uint32_t q = sh >> 2, r = sh & 3;
    uint32_t s[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        uint32_t v3 = (i + 3 < 8) ? w[i + 3] : 0u;
        s[i] = q == 0 ? w[i] : (q == 1 ? w[i + 1] : (q == 2 ? w[i + 2] : v3));
    }
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(s[1], s[0], r);
    o.y = __builtin_amdgcn_alignbyte(s[2], s[1], r);
    o.z = __builtin_amdgcn_alignbyte(s[3], s[2], r);
    o.w = __builtin_amdgcn_alignbyte(s[4], s[3], r);
    return o;
}

// bytes [p, p+n) (1 <= n <= 16) at bytes 0..n-1 of the result (the rest unspecified). Only the
// aligned 16-byte blocks holding a requested byte are read, so no page beyond them is touched.
template <class L = GLoad>
__device__ __forceinline__ uint4 load_window16(const uint8_t* p, uint32_t n, L ld = L()) {
    uintptr_t a = (uintptr_t)p;
    const uintptr_t b0 = a & ~(uintptr_t)15;
    uint32_t sh = (uint32_t)(a & 15);
    uint4 x = ld(b0);
    uint4 y = make_uint4(0, 0, 0, 0);
    if (sh + n > 16) y = ld(b0 + 16);
    return funnel16(x, y, sh);
}

// move byte j to j + a (a in 0..15), zero fill
__device__ __forceinline__ uint4 shl_bytes(uint4 w, uint32_t a) {
    return a ? funnel16(make_uint4(0, 0, 0, 0), w, 16 - a) : w;
}

__device__ __forceinline__ uint32_t dword_mask(uint32_t a, uint32_t b, uint32_t i) {
    uint32_t lo = a > 4 * i ? a : 4 * i, hi = b < 4 * i + 4 ? b : 4 * i + 4;
    if (lo >= hi) return 0u;
    uint64_t m = ((1ull << (8 * (hi - lo))) - 1) << (8 * (lo - 4 * i));
    return (uint32_t)m;
}

// bytewise order of the first n bytes at a and b (<0, 0, >0), 16 bytes per step (only the
// aligned 16-byte blocks holding requested bytes are read)
__device__ inline int bytes_cmp16(const uint8_t* a, const uint8_t* b, uint64_t n) {
    for (uint64_t i = 0; i < n; i += 16) {
        const uint32_t m = (uint32_t)(n - i < 16 ? n - i : 16);
        const uint4 x = load_window16(a + i, m), y = load_window16(b + i, m);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t mk = dword_mask(0, m, q);
            const uint32_t xa = __builtin_bswap32(xs[q] & mk), ya = __builtin_bswap32(ys[q] & mk);
            if (xa != ya) return xa < ya ? -1 : 1;
        }
    }
    return 0;
}

// Ordering of two keys given their 16-byte prefixes, lengths and (for keys > 16 B) their bytes:
// bytewise lexicographic, proper prefix first (Rust str Ord). Returns <0, 0, >0.
__device__ inline int key_cmp(uint64_t ahi, uint64_t alo, uint32_t alen, const uint8_t* akey,
                              uint64_t bhi, uint64_t blo, uint32_t blen, const uint8_t* bkey) {
    if (ahi != bhi) return ahi < bhi ? -1 : 1;
    if (alo != blo) return alo < blo ? -1 : 1;
    if (alen > 16 && blen > 16) {
        const uint32_t n = (alen < blen ? alen : blen);
        const int c = bytes_cmp16(akey + 16, bkey + 16, n - 16);
        if (c) return c;
    }
    return alen < blen ? -1 : (alen > blen ? 1 : 0);
}

// ---- vectorized record headers --------------------------------------------------------------

// 32 bytes at run+p into w[0..7] (bytes at or past run+len read as zero). Only aligned 16-byte
// blocks holding a byte below run+len are loaded.
template <class L = GLoad>
__device__ __forceinline__ void window32(const uint8_t* run, uint64_t len, uint64_t p, uint32_t w[8],
                                         L ld = L()) {
    uintptr_t a = (uintptr_t)(run + p);
    uintptr_t end = (uintptr_t)(run + len);
    uintptr_t base = a & ~(uintptr_t)15;
    uint32_t sh = (uint32_t)(a & 15);
    uint4 z = make_uint4(0, 0, 0, 0);
    uint4 b0 = ld(base);
    uint4 b1 = base + 16 < end ? ld(base + 16) : z;
    uint4 b2 = (sh && base + 32 < end) ? ld(base + 32) : z;
    uint4 lo = funnel16(b0, b1, sh), hi = funnel16(b1, b2, sh);
    w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
    w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
    // zero bytes at or past the run end (the window may extend past it)
    if (p + 32 > len) {
        uint32_t valid = (uint32_t)(len - p);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] &= dword_mask(0, valid, i) | (4u * i + 4 <= valid ? 0xFFFFFFFFu : 0u);
    }
}

__device__ __forceinline__ uint32_t sel8(const uint32_t w[8], uint32_t i) {
    // the words as register values first: a select chain over the array's loads was folded into one
    // load at a variable index, which kept the window in scratch (two stores and a dependent load in
    // every walk step)
    uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4], x5 = w[5], x6 = w[6], x7 = w[7];
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    const uint32_t a = (i & 1) ? x1 : x0, b = (i & 1) ? x3 : x2, c = (i & 1) ? x5 : x4, d = (i & 1) ? x7 : x6;
    const uint32_t e = (i & 2) ? b : a, f = (i & 2) ? d : c;
    const uint32_t r = (i & 4) ? f : e;
    return i < 8 ? r : 0u;
}

// big-endian u32 at byte offset o (o <= 28) of the window
__device__ __forceinline__ uint32_t win_be32(const uint32_t w[8], uint32_t o) {
    uint32_t q = o >> 2, r = o & 3;
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(sel8(w, q + 1), sel8(w, q), r));
}

// key bytes 5.. of the window as 7 dwords (28 bytes), little-endian byte order
__device__ __forceinline__ void win_key(const uint32_t w[8], uint32_t kd[7]) {
#pragma unroll
    for (int i = 0; i < 7; ++i) kd[i] = __builtin_amdgcn_alignbyte(i + 2 < 8 ? w[i + 2] : 0u, w[i + 1], 1);
}

__device__ __forceinline__ bool ascii_prefix(const uint32_t kd[7], uint32_t n /* <= 28 */) {
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t i = 0; i < 7; ++i) acc |= kd[i] & dword_mask(0, n, i);
    return (acc & 0x80808080u) == 0;
}

// UTF-8 validity with an all-ASCII vector fast path: the aligned 16-byte blocks of the key are
// loaded 4 at a time with no dependence between them (one memory round trip per 64 bytes), their
// bytes past the key masked off; any high bit falls back to the exact scalar check.
template <class L = GLoad>
__device__ inline bool utf8_valid_fast(const uint8_t* s, uint64_t n, L ld = L()) {
    if (n == 0) return true;
    const uintptr_t a0 = (uintptr_t)s, a1 = a0 + n;  // bytes [a0, a1)
    const uintptr_t b0 = a0 & ~(uintptr_t)15, b1 = (a1 + 15) & ~(uintptr_t)15;
    for (uintptr_t b = b0; b < b1; b += 64) {
        uint4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = b + 16 * q < b1 ? ld(b + 16 * q) : make_uint4(0, 0, 0, 0);
        uint32_t acc = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uintptr_t blk = b + 16 * q;
            const uint32_t lo = a0 > blk ? (uint32_t)(a0 - blk) : 0u;
            const uint32_t hi = a1 < blk + 16 ? (uint32_t)(a1 - blk) : 16u;
            if (blk < b1 && lo < hi)
                acc |= (v[q].x & dword_mask(lo, hi, 0)) | (v[q].y & dword_mask(lo, hi, 1)) |
                       (v[q].z & dword_mask(lo, hi, 2)) | (v[q].w & dword_mask(lo, hi, 3));
        }
        if (acc & 0x80808080u) return utf8_valid(s, n);
    }
    return true;
}

// 16-byte big-endian key prefix from the window's key dwords, zero past klen
__device__ __forceinline__ void win_prefix(const uint32_t kd[7], uint64_t klen, uint64_t& hi, uint64_t& lo) {
    uint32_t n = klen < 16 ? (uint32_t)klen : 16u;
    uint32_t d0 = kd[0] & dword_mask(0, n, 0), d1 = kd[1] & dword_mask(0, n, 1);
    uint32_t d2 = kd[2] & dword_mask(0, n, 2), d3 = kd[3] & dword_mask(0, n, 3);
    hi = ((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1);
    lo = ((uint64_t)__builtin_bswap32(d2) << 32) | __builtin_bswap32(d3);
}

struct RecHdr {
    uint32_t marker;
    uint32_t err;    // DERR_* | extra << 8
    uint64_t klen;
    uint64_t size;
    uint64_t hi, lo; // key prefix
};

// One record of runs::read_run_stream (runs.rs:559-626) at p, checks in the reference's order,
// from one 32-byte window plus (only for long keys / non-ASCII keys) further loads.
// UTF8 = false: the record was already validated by a walk (k_emit re-reads records that
// k_spec / k_fixup walked with every check)
// UTF8: 0 no key check (structure only), 1 the exact check, 2 a heuristic for speculative chunk
// starts (a key whose in-window bytes are ASCII passes unchecked; any other key gets the exact
// check): random bytes taken for a record fail it, real keys cost no extra loads
template <bool PREFIX, int UTF8 = 1, class L = GLoad>
__device__ __forceinline__ RecHdr parse_rec(const uint8_t* run, uint64_t len, uint64_t p, L ld = L()) {
    RecHdr h;
    h.size = 0;
    h.hi = h.lo = 0;
    uint32_t w[8];
    window32(run, len, p, w, ld);
    h.marker = w[0] & 0xFFu;
    if (p + 5 > len) { h.err = DERR_IO; h.klen = 0; return h; }
    h.klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], 1));
    const uint64_t kp = p + 5;
    if (kp + h.klen > len) { h.err = DERR_KEY; return h; }
    // the value length past the window is loaded before the key's UTF-8 check, so that the two
    // round trips overlap (the checks keep the reference's order)
    const uint64_t vo = 5 + h.klen;
    const bool vfar = h.marker == 1 && vo + 4 > 32 && kp + h.klen + 4 <= len;
    const uint4 vv = vfar ? load_window16(run + p + vo, 4, ld) : make_uint4(0, 0, 0, 0);
    uint32_t kd[7];
    win_key(w, kd);
    bool ok = UTF8 == 0 || (UTF8 == 2 ? ascii_prefix(kd, h.klen < 27 ? (uint32_t)h.klen : 27u)
                                      : (h.klen <= 27 && ascii_prefix(kd, (uint32_t)h.klen)));
    if (!ok) ok = utf8_valid_fast(run + kp, h.klen, ld);
    if (!ok) { h.err = DERR_UTF8; return h; }
    if (PREFIX) win_prefix(kd, h.klen, h.hi, h.lo);
    if (h.marker == 1) {
        if (kp + h.klen + 4 > len) { h.err = DERR_IO; return h; }
        const uint64_t vlen = vo + 4 <= 32 ? win_be32(w, (uint32_t)vo) : __builtin_bswap32(vv.x);
        if (kp + h.klen + 4 + vlen > len) { h.err = DERR_VAL; return h; }
        h.size = 9 + h.klen + vlen;
    } else if (h.marker == 2) {
        h.size = 5 + h.klen;
    } else {
        // the key's UTF-8 check comes before the marker match (runs.rs:585-591 vs :621-624): a walk
        // that skipped it (structure only / the ASCII heuristic) does it now, at the failing record
        h.err = UTF8 != 1 && !utf8_valid_fast(run + kp, h.klen, ld) ? DERR_UTF8 : DERR_MARKER | (h.marker << 8);
        return h;
    }
    h.err = DERR_NONE;
    return h;
}

// 64-bit fingerprint of the key bytes past the 16-byte prefix (0 for keys of at most 16 bytes),
// a function of the bytes alone; ascii: those bytes have no high bit
__device__ __forceinline__ uint64_t fp_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
template <class L = GLoad>
__device__ inline uint64_t key_tail_fp(const uint8_t* key, uint32_t klen, bool& ascii, L ld = L()) {
    ascii = true;
    if (klen <= 16) return 0;
    const uint8_t* k = key + 16;
    const uint32_t n = klen - 16;
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    uint32_t acc = 0;
    // 16-byte windows at k + o, assembled from aligned blocks (an aligned block holding a key byte
    // never leaves the run's pages): five block loads per four windows, issued together
    const uintptr_t a = (uintptr_t)k;
    const uintptr_t base = a & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(a & 15);
    const uint32_t nblk = (sh + n + 15) >> 4;
    for (uint32_t o = 0; o < n; o += 64) {
        const uint32_t q0 = o >> 4;
        uint4 B[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) B[i] = q0 + i < nblk ? ld(base + 16ull * (q0 + i)) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (o + 16 * w < n) {
                const uint32_t m = n - o - 16 * w < 16 ? n - o - 16 * w : 16;
                const uint4 v = funnel16(B[w], B[w + 1], sh);
                const uint32_t a0 = v.x & dword_mask(0, m, 0), a1 = v.y & dword_mask(0, m, 1);
                const uint32_t a2 = v.z & dword_mask(0, m, 2), a3 = v.w & dword_mask(0, m, 3);
                acc |= a0 | a1 | a2 | a3;
                h = fp_mix(h ^ (((uint64_t)a1 << 32) | a0));
                h = fp_mix(h ^ (((uint64_t)a3 << 32) | a2) ^ 0x2545F4914F6CDD1Dull);
            }
        }
    }
    ascii = (acc & 0x80808080u) == 0;
    return h;
}

// uint4 b[i] for a dynamic i < N, as a select tree over register values (no array in memory)
template <int N>
__device__ __forceinline__ uint4 sel_blk(const uint4 (&b)[N], uint32_t i) {
    uint4 r = b[0];
#pragma unroll
    for (int k = 1; k < N; ++k) {
        const bool t = i == (uint32_t)k;
        r.x = t ? b[k].x : r.x;
        r.y = t ? b[k].y : r.y;
        r.z = t ? b[k].z : r.z;
        r.w = t ? b[k].w : r.w;
    }
    return r;
}

// parse_rec<true, 0> for the staging walks, reading each byte of the record's header, key and value
// length once: the header window's aligned blocks, then (past them, issued together) the blocks up
// to the value length, from which the value length and the fingerprint of the key past 16 bytes
// (key_tail_fp's function of the bytes) are taken. Keys of at most STG_KMAX bytes (longer keys end
// the chunk's staging, their fingerprint is not computed: fpv 0).
template <class L = GLoad>
__device__ __forceinline__ RecHdr parse_rec_stg(const uint8_t* run, uint64_t len, uint64_t p, uint64_t& fpv,
                                                bool& ascii, L ld = L()) {
    RecHdr h;
    h.size = 0;
    h.hi = h.lo = 0;
    fpv = 0;
    ascii = true;
    const uintptr_t a = (uintptr_t)(run + p), end = (uintptr_t)(run + len);
    const uintptr_t base = a & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(a & 15);
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 b0 = ld(base);
    const uint4 b1 = base + 16 < end ? ld(base + 16) : z;
    const bool b2ok = sh && base + 32 < end;
    const uint4 b2 = b2ok ? ld(base + 32) : z;
    uint32_t w[8];
    {
        const uint4 lo = funnel16(b0, b1, sh), hi = funnel16(b1, b2, sh);
        w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w;
        w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
        if (p + 32 > len) {
            const uint32_t valid = (uint32_t)(len - p);
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] &= dword_mask(0, valid, i) | (4u * i + 4 <= valid ? 0xFFFFFFFFu : 0u);
        }
    }
    h.marker = w[0] & 0xFFu;
    if (p + 5 > len) { h.err = DERR_IO; h.klen = 0; return h; }
    h.klen = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], 1));
    const uint64_t kp = p + 5;
    if (kp + h.klen > len) { h.err = DERR_KEY; return h; }
    const uint64_t vo = 5 + h.klen;
    const bool put = h.marker == 1;
    const bool vin = put && kp + h.klen + 4 <= len;  // (else the IO error below)
    // the region past the window: key bytes 16.. (fingerprint) and the value length, in aligned
    // blocks from tb; blocks the window already holds are taken from it
    const bool tail = h.klen > 16 && h.klen <= STG_KMAX;
    const bool vfar = vin && vo + 4 > 32 && h.klen <= STG_KMAX;
    uint4 B[10];
    const uintptr_t tb = (a + 21) & ~(uintptr_t)15;  // base + 16 or base + 32
    const uint32_t tsh = (uint32_t)((a + 21) & 15);
    const uint64_t rend = vfar ? vo + 4 : (tail ? vo : 21);  // region end, relative to p
    const uint32_t nblk = rend > 21 ? (uint32_t)((tsh + (rend - 21) + 15) >> 4) : 0u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uintptr_t ba = tb + 16ull * i;
        B[i] = (uint32_t)i >= nblk ? z : (ba == base + 16 ? b1 : (ba == base + 32 && b2ok ? b2 : ld(ba)));
    }
    uint4 vv = z;
    if (vin && vo + 4 > 32 && h.klen > STG_KMAX) vv = load_window16(run + p + vo, 4, ld);  // (unstaged key)
    if (tail && !(SKV_STG_PROBE & 1)) {
        const uint32_t n = (uint32_t)h.klen - 16;
        uint64_t hh = 0x9E3779B97F4A7C15ull ^ n;
        uint32_t acc = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (16u * q < n) {
                const uint32_t m = n - 16 * q < 16 ? n - 16 * q : 16;
                const uint4 v = funnel16(B[q], B[q + 1], tsh);
                const uint32_t a0 = v.x & dword_mask(0, m, 0), a1 = v.y & dword_mask(0, m, 1);
                const uint32_t a2 = v.z & dword_mask(0, m, 2), a3 = v.w & dword_mask(0, m, 3);
                acc |= a0 | a1 | a2 | a3;
                hh = fp_mix(hh ^ (((uint64_t)a1 << 32) | a0));
                hh = fp_mix(hh ^ (((uint64_t)a3 << 32) | a2) ^ 0x2545F4914F6CDD1Dull);
            }
        }
        ascii = (acc & 0x80808080u) == 0;
        fpv = hh;
    }
    uint32_t kd[7];
    win_key(w, kd);
    win_prefix(kd, h.klen, h.hi, h.lo);
    ascii = ascii && ((h.hi | h.lo) & 0x8080808080808080ull) == 0;
    if (put) {
        if (kp + h.klen + 4 > len) { h.err = DERR_IO; return h; }
        uint64_t vlen;
        if (vo + 4 <= 32) {
            vlen = win_be32(w, (uint32_t)vo);
        } else if (h.klen <= STG_KMAX) {
            const uint32_t off = tsh + (uint32_t)(vo - 21);  // the value length's offset from tb
            const uint4 v = funnel16(sel_blk(B, off >> 4), sel_blk(B, (off >> 4) + 1), off & 15);
            vlen = __builtin_bswap32(v.x);
        } else {
            vlen = __builtin_bswap32(vv.x);
        }
        if (kp + h.klen + 4 + vlen > len) { h.err = DERR_VAL; return h; }
        h.size = 9 + h.klen + vlen;
    } else if (h.marker == 2) {
        h.size = 5 + h.klen;
    } else {
        h.err = !utf8_valid_fast(run + kp, h.klen, ld) ? DERR_UTF8 : DERR_MARKER | (h.marker << 8);
        return h;
    }
    h.err = DERR_NONE;
    return h;
}

// walk_checked with vectorized headers: one dependent round trip per record. UTF8 = false: the
// structure only (k_spec's fast mode; k_emit checks the keys and flags a bad one for an exact rerun)
// slot (cap > 0, a multiple of 8, 16-byte aligned row): the first cap record starts, as offsets
// from cs (k_emit reads them back), stored eight at a time (one 16-byte store instead of eight
// 2-byte ones: the single-lane stores were written back as separate partial lines, 7.8 GB at 3F)
// STG: the walk also stages each record's arrays (key prefix, key length, Delete bit, fingerprint of
// the key past 16 bytes, an ASCII bit) in its chunk's StgRec row (scap entries), so that k_emit
// copies them to record order without reading the record again (the parse reads the input once)
template <int UTF8 = 1, bool STG = false, class L = GLoad>
__device__ inline WalkRes walk_fast(const uint8_t* run, uint64_t len, uint64_t p, uint64_t stop, uint32_t max_recs,
                                   L ld = L(), uint16_t* slot = nullptr, uint32_t cap = 0, uint64_t cs = 0,
                                   StgRec* stg = nullptr, uint32_t scap = 0) {
    uint32_t cnt = 0, nst = 0;
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    auto flush = [&]() {  // the group holding slot cnt - 1 (positions past cnt: unread)
        if (cap && (cnt & 7) && (cnt & ~7u) < cap) *(uint4*)(slot + (cnt & ~7u)) = make_uint4(s0, s1, s2, s3);
    };
    while (p < stop && cnt < max_recs) {
        uint64_t fpv = 0;
        bool ascii = true;
        RecHdr h;
        if (STG && UTF8 == 0) {
            h = parse_rec_stg(run, len, p, fpv, ascii, ld);
        } else {
            h = parse_rec<STG, UTF8>(run, len, p, ld);
            if (STG && h.klen <= STG_KMAX) {
                fpv = key_tail_fp(run + p + 5, (uint32_t)h.klen, ascii, ld);
                ascii = ascii && ((h.hi | h.lo) & 0x8080808080808080ull) == 0;
            }
        }
        if (h.err) {
            flush();
            return {p, cnt, h.err, nst};
        }
        // (a key past STG_KMAX bytes ends the staging: its fingerprint would lengthen the walk's
        // chain -- a wrong speculative chain can read a run-sized "key" -- and k_emit parses the chunk)
        if (STG && cnt < scap && nst == cnt && h.klen <= STG_KMAX && (!(SKV_STG_PROBE & 2) || (fpv ^ h.hi) == 42)) {
            ++nst;
            const uint32_t kd = (uint32_t)h.klen | (h.marker == 2 ? 0x80000000u : 0u);
            uint4* e = (uint4*)(stg + (uint64_t)cnt * STG_W);
            e[0] = make_uint4((uint32_t)h.hi, (uint32_t)(h.hi >> 32), (uint32_t)h.lo, (uint32_t)(h.lo >> 32));
            e[1] = make_uint4((uint32_t)fpv, (uint32_t)(fpv >> 32), kd, ascii ? 1u : 0u);
        }
        if (cnt < cap) {
            const uint32_t j = cnt & 7, v = (uint32_t)(uint16_t)(p - cs) << (16 * (j & 1)), q = j >> 1;
            s0 |= q == 0 ? v : 0u;
            s1 |= q == 1 ? v : 0u;
            s2 |= q == 2 ? v : 0u;
            s3 |= q == 3 ? v : 0u;
            if (j == 7) {
                *(uint4*)(slot + (cnt & ~7u)) = make_uint4(s0, s1, s2, s3);
                s0 = s1 = s2 = s3 = 0;
            }
        }
        ++cnt;
        p += h.size;
    }
    flush();
    return {p, cnt, DERR_NONE, nst};
}


__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t k) {
    uint32_t d = (k >> 2) == 0 ? v.x : ((k >> 2) == 1 ? v.y : ((k >> 2) == 2 ? v.z : v.w));
    return (d >> (8 * (k & 3))) & 0xFFu;
}

#endif  // __HIPCC__

}  // namespace skv
