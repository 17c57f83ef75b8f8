// skv_heap.hip — k_way::merge's exact pop order for UNSORTED input streams ("heap-order mode").
//
// k_way::merge (src/k_way.rs:113-179) keeps one head per stream in a BinaryHeap and pops the
// smallest key (ties: larger seq_no). For sorted streams that is a sorted merge. For a stream with
// a key decrease it is not, and the job's outcome then depends on that exact order wherever it is
// not simply "the first decrease fails build_runs": under the Delete filter at Level::max()
// (table_tree_compaction.rs:139-145: a decrease among filtered Deletes is never seen by
// build_runs' order check, runs.rs:190-198) and in the WAL split (wal_compaction.rs:66-174: an
// order error fails only that table's task, whose error is swallowed, or the job's next send to
// it).
//
// The heap's pop order for arbitrary streams is the stable order of (E, seq_no desc, position in
// stream) with E = the running maximum of the stream's keys up to the record: a record after a
// decrease pops right behind the stream's maximum so far (it is below every other head, all of
// which are >= that maximum), and a new maximum waits for the heads below it like in a sorted
// merge. (Checked against a literal heap on 20,000 random multi-stream cases, keys with many
// duplicates: tests/test_heap_order.py.) So the splitter merge / record sort run unchanged on the
// keys of each record's prefix-maximum record, first-per-key compares neighbouring pops on their
// own keys, and pop_pos records every record's pop position for the host's error resolution.
#include "skv_launch.hpp"

namespace skv {

static inline unsigned hp_blocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// (Compare results are taken into an int before any select: an `a || rec_cmp(..) > 0` condition
// was observed to skip its update on gfx950 at -O3.)
__device__ __forceinline__ int rec_cmp(const uint64_t* hi, const uint64_t* lo, const uint32_t* klen,
                                       const uint64_t* addr, uint32_t a, uint32_t b) {
    return key_cmp(hi[a], lo[a], klen[a], (const uint8_t*)addr[a] + 5, hi[b], lo[b], klen[b],
                   (const uint8_t*)addr[b] + 5);
}

__device__ __forceinline__ uint32_t stream_of(const uint64_t* base, uint32_t k, uint64_t i) {
    uint32_t lo = 0, hi = k;  // last s with base[s] <= i (empty streams share a base)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (base[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

constexpr int PM_T = 256, PM_PER = 4, PM_BLK = PM_T * PM_PER;
constexpr uint32_t PM_NONE = 0xFFFFFFFFu;

// Segmented prefix-maximum (segments = streams) inside each block of PM_BLK records: eff[i] = the
// record with the largest key among the stream's records in [block start or stream start, i].
// blk_agg[b] = (has a stream start, max record of the block's last segment part).
__global__ void __launch_bounds__(PM_T) k_pmax_block(uint64_t R, const uint64_t* __restrict__ base, uint32_t k,
                                                     const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                                                     const uint32_t* __restrict__ klen,
                                                     const uint64_t* __restrict__ addr, uint32_t* eff,
                                                     uint64_t* blk_agg) {
    __shared__ uint32_t s_v[2][PM_T];
    __shared__ uint32_t s_f[2][PM_T];
    const uint64_t i0 = (uint64_t)blockIdx.x * PM_BLK + (uint64_t)threadIdx.x * PM_PER;
    uint32_t v = PM_NONE, f = 0;
    uint32_t loc[PM_PER];
#pragma unroll
    for (int q = 0; q < PM_PER; ++q) {
        const uint64_t i = i0 + q;
        loc[q] = PM_NONE;
        if (i < R) {
            const uint32_t s = stream_of(base, k, i);
            const bool head = base[s] == i;  // a stream starts here
            int c = 1;
            if (!head && v != PM_NONE) c = rec_cmp(hi, lo, klen, addr, (uint32_t)i, v);
            if (head || c > 0) v = (uint32_t)i;
            if (head) f = 1;
            loc[q] = v;
        }
    }
    // block-wide inclusive segmented scan of the thread aggregates (Hillis-Steele)
    int cur = 0;
    s_v[0][threadIdx.x] = v;
    s_f[0][threadIdx.x] = f;
    __syncthreads();
    for (int d = 1; d < PM_T; d <<= 1) {
        uint32_t nv = s_v[cur][threadIdx.x], nf = s_f[cur][threadIdx.x];
        if ((int)threadIdx.x >= d) {
            const uint32_t pv = s_v[cur][threadIdx.x - d], pf = s_f[cur][threadIdx.x - d];
            if (!nf) {  // combine (pf, pv) (+) (nf, nv)
                int c = 0;
                if (nv != PM_NONE && pv != PM_NONE) c = rec_cmp(hi, lo, klen, addr, pv, nv);
                if (nv == PM_NONE || c > 0) nv = pv;
                nf = pf;
            }
        }
        s_v[cur ^ 1][threadIdx.x] = nv;
        s_f[cur ^ 1][threadIdx.x] = nf;
        cur ^= 1;
        __syncthreads();
    }
    // exclusive prefix of this thread: applies to its items before its first stream start
    const uint32_t ev = threadIdx.x ? s_v[cur][threadIdx.x - 1] : PM_NONE;
    bool open = true;
#pragma unroll
    for (int q = 0; q < PM_PER; ++q) {
        const uint64_t i = i0 + q;
        if (i >= R) break;
        if (open && base[stream_of(base, k, i)] == i) open = false;
        uint32_t w = loc[q];
        int c = 0;
        if (open && ev != PM_NONE) c = rec_cmp(hi, lo, klen, addr, ev, w);
        if (c > 0) w = ev;
        eff[i] = w;
    }
    if (threadIdx.x == PM_T - 1) blk_agg[blockIdx.x] = ((uint64_t)s_f[cur][PM_T - 1] << 32) | s_v[cur][PM_T - 1];
}

// carry into every block: the maximum of the segment running into it (one lane, blocks in order)
__global__ void k_pmax_carry(uint64_t nb, const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                             const uint32_t* __restrict__ klen, const uint64_t* __restrict__ addr,
                             const uint64_t* __restrict__ blk_agg, uint32_t* carry) {
    if (blockIdx.x || threadIdx.x) return;
    uint32_t c = PM_NONE;
    for (uint64_t b = 0; b < nb; ++b) {
        carry[b] = c;
        const uint64_t a = blk_agg[b];
        const uint32_t av = (uint32_t)a;
        int d = 1;
        if (!(a >> 32) && av != PM_NONE && c != PM_NONE) d = rec_cmp(hi, lo, klen, addr, av, c);
        if ((a >> 32) || (av != PM_NONE && d > 0)) c = av;
    }
}

// apply the carry to the records whose stream began before their block; then the merge keys:
// the key arrays of each record's prefix-maximum record
__global__ void k_pmax_apply(uint64_t R, const uint64_t* __restrict__ base, uint32_t k,
                             const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                             const uint32_t* __restrict__ klen, const uint64_t* __restrict__ addr,
                             const uint32_t* __restrict__ carry, const uint32_t* __restrict__ eff, uint64_t* ehi,
                             uint64_t* elo, uint32_t* eklen, uint64_t* eaddr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint64_t b = i / PM_BLK;
    uint32_t w = eff[i];
    const uint32_t c = carry[b];
    int d = 0;
    if (c != PM_NONE && base[stream_of(base, k, i)] < b * PM_BLK) d = rec_cmp(hi, lo, klen, addr, c, w);
    if (d > 0) w = c;
    ehi[i] = hi[w];
    elo[i] = lo[w];
    eklen[i] = klen[w];
    eaddr[i] = addr[w];
}

// Record sort path in heap-order mode: the sort ran on the merge keys; gather each sorted
// position's own key, payload and the inverse permutation (original record -> sorted position).
__global__ void k_heap_sorted(uint64_t R, const SElem* __restrict__ S, const uint64_t* __restrict__ hi,
                              const uint64_t* __restrict__ lo, const uint32_t* __restrict__ klen,
                              const uint64_t* __restrict__ addr, uint64_t* shi, uint64_t* slo, uint32_t* sklen,
                              uint64_t* saddr, uint32_t* inv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint32_t src = S[i].pos;
    shi[i] = hi[src];
    slo[i] = lo[src];
    sklen[i] = klen[src];
    saddr[i] = addr[src];
    inv[src] = (uint32_t)i;
}

// build_runs' order check (runs.rs:190-198) on the emitted, filtered sequence: the first survivor
// whose key is not above its predecessor's
__global__ void k_merged_order(const uint64_t* __restrict__ Kp, const uint32_t* __restrict__ m_rec,
                               const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                               const uint32_t* __restrict__ klen, const uint64_t* __restrict__ addr,
                               unsigned long long* first_bad) {
    const uint64_t K = *Kp;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0 || g >= K) return;
    if (rec_cmp(hi, lo, klen, addr, m_rec[g - 1], m_rec[g]) >= 0) atomicMin(first_bad, (unsigned long long)g);
}

// WAL split, heap-order mode: a table whose build_runs failed on its first order error at
// survivor v has its receiver dropped; the job's send of that table's 101st op after v then fails
// deterministically (mpsc::channel(100), wal_compaction.rs:113, :157-161). Returns the first such
// survivor over all tables.
__global__ void k_wal_sendfail(const uint64_t* __restrict__ NTp, const uint64_t* __restrict__ tstart,
                               const unsigned long long* __restrict__ tfirst, unsigned long long* first_fail) {
    const uint64_t NT = *NTp;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NT) return;
    const unsigned long long v = tfirst[t];
    if (v == ~0ull) return;
    const uint64_t f = v + 101;
    if (f < tstart[t + 1]) atomicMin(first_fail, (unsigned long long)f);
}

void launch_heap_keys(hipStream_t s, uint64_t R, const uint64_t* base, uint32_t k, const uint64_t* hi,
                      const uint64_t* lo, const uint32_t* klen, const uint64_t* addr, uint32_t* eff, uint64_t* blk_agg,
                      uint32_t* carry, uint64_t* ehi, uint64_t* elo, uint32_t* eklen, uint64_t* eaddr) {
    if (!R) return;
    const uint64_t nb = (R + PM_BLK - 1) / PM_BLK;
    k_pmax_block<<<(unsigned)nb, PM_T, 0, s>>>(R, base, k, hi, lo, klen, addr, eff, blk_agg);
    k_pmax_carry<<<1, 64, 0, s>>>(nb, hi, lo, klen, addr, blk_agg, carry);
    k_pmax_apply<<<hp_blocks(R, 256), 256, 0, s>>>(R, base, k, hi, lo, klen, addr, carry, eff, ehi, elo, eklen, eaddr);
}
uint64_t heap_key_blocks(uint64_t R) { return (R + PM_BLK - 1) / PM_BLK + 1; }
void launch_heap_sorted(hipStream_t s, uint64_t R, const SElem* S, const uint64_t* hi, const uint64_t* lo,
                        const uint32_t* klen, const uint64_t* addr, uint64_t* shi, uint64_t* slo, uint32_t* sklen,
                        uint64_t* saddr, uint32_t* inv) {
    if (R) k_heap_sorted<<<hp_blocks(R, 256), 256, 0, s>>>(R, S, hi, lo, klen, addr, shi, slo, sklen, saddr, inv);
}
void launch_merged_order(hipStream_t s, const uint64_t* Kp, uint64_t max_K, const uint32_t* m_rec, const uint64_t* hi,
                         const uint64_t* lo, const uint32_t* klen, const uint64_t* addr, unsigned long long* first_bad) {
    if (max_K > 1) k_merged_order<<<hp_blocks(max_K, 256), 256, 0, s>>>(Kp, m_rec, hi, lo, klen, addr, first_bad);
}
void launch_wal_sendfail(hipStream_t s, const uint64_t* NTp, uint64_t max_NT, const uint64_t* tstart,
                         const unsigned long long* tfirst, unsigned long long* first_fail) {
    if (max_NT) k_wal_sendfail<<<hp_blocks(max_NT, 256), 256, 0, s>>>(NTp, tstart, tfirst, first_fail);
}

}  // namespace skv
