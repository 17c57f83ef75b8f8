// skv_scan.hip — the cache service's ScanFromRun (cache_service.rs:97-151) after the device merge.
//
// The compaction's parse and merge (k_way::merge order, first record per key; heap-order mode when a
// run is unsorted or undecodable) run unchanged over the scan's runs (run i at SeqNo
// i64::MAX - i); these kernels then apply what the service does to the merged stream:
//   - the per-run filter try_filter(op.key() > exclusive_start_key) (:125-129), on the record
//     arrays before the merge (k_scan_keep / k_scan_compact);
//   - the reader's cut-off: items up to and including the max_results-th Put (:140-148);
//   - the response: the kept items, in order, as ONE v1 run (an item's record bytes are the
//     response item: Put key + value or Delete key), version byte first.
// A run's decode error surfaces right after the pop of its last record above the start key; with
// none, at the merge's first pulls (the host resolves both from the filtered stream bases).
#include "skv_launch.hpp"

namespace skv {

// key of (hi, lo, klen, bytes at addr + 5) vs the start key (device copy, its prefix words sh/sl):
// true when the record's key sorts strictly after it (Rust str >)
__device__ __forceinline__ bool scan_above(uint64_t hi, uint64_t lo, uint32_t klen, uint64_t addr, uint64_t sh,
                                           uint64_t sl, uint32_t slen, const uint8_t* start) {
    return key_cmp(hi, lo, klen, (const uint8_t*)addr + 5, sh, sl, slen, start) > 0;
}

// The per-run filter before the merge (cache_service.rs:125-129): records at or below the start key
// leave the record arrays, so the merge -- and its first-per-key, which compares consecutive pops
// (k_way.rs:146-151) -- sees exactly the filtered runs. (Filtering after the merge is not the same
// in heap order: an unsorted run's dropped record can pop between two kept records of one key.)
__global__ void k_scan_keep(uint64_t R, const uint64_t* __restrict__ rec_addr, const uint64_t* __restrict__ rec_hi,
                            const uint64_t* __restrict__ rec_lo, const uint32_t* __restrict__ rec_klen,
                            const uint8_t* __restrict__ start, uint32_t slen, uint64_t* keep) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    uint64_t sh, sl;
    key_prefix(start, slen, sh, sl);
    keep[r] = scan_above(rec_hi[r], rec_lo[r], rec_klen[r], rec_addr[r], sh, sl, slen, start) ? 1 : 0;
}

// kept records to their filtered positions (keepx: exclusive scan of keep)
__global__ void k_scan_compact(uint64_t R, const uint64_t* __restrict__ keep, const uint64_t* __restrict__ keepx,
                               const uint64_t* __restrict__ a_addr, const uint64_t* __restrict__ a_hi,
                               const uint64_t* __restrict__ a_lo, const uint32_t* __restrict__ a_klen,
                               const uint32_t* __restrict__ a_meta, uint64_t* b_addr, uint64_t* b_hi, uint64_t* b_lo,
                               uint32_t* b_klen, uint32_t* b_meta) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R || !keep[r]) return;
    const uint64_t d = keepx[r];
    b_addr[d] = a_addr[r];
    b_hi[d] = a_hi[r];
    b_lo[d] = a_lo[r];
    b_klen[d] = a_klen[r];
    b_meta[d] = a_meta[r];
}

// filtered stream bases: nb[s] = kept records before stream s's first record (s = 0..k)
__global__ void k_scan_bases(uint32_t k, const uint64_t* __restrict__ base, const uint64_t* __restrict__ keepx,
                             uint64_t* nb) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s <= k) nb[s] = keepx[base[s]];
}

// per merged survivor g < K: kept (key above the start), kept Put, kept bytes
__global__ void k_scan_mark(const uint64_t* __restrict__ d_K, const uint32_t* __restrict__ m_rec,
                            const uint64_t* __restrict__ rec_addr, const uint64_t* __restrict__ rec_hi,
                            const uint64_t* __restrict__ rec_lo, const uint32_t* __restrict__ rec_klen,
                            const uint32_t* __restrict__ rec_meta, const uint8_t* __restrict__ start, uint32_t slen,
                            uint64_t* keep, uint64_t* put, uint64_t* size) {
    const uint64_t K = *d_K;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= K) return;
    uint64_t sh, sl;
    key_prefix(start, slen, sh, sl);
    const uint32_t r = m_rec[g];
    const bool kp = scan_above(rec_hi[r], rec_lo[r], rec_klen[r], rec_addr[r], sh, sl, slen, start);
    const uint32_t m = rec_meta[r];
    keep[g] = kp ? 1 : 0;
    put[g] = kp && !(m >> 31) ? 1 : 0;
    size[g] = kp ? (m & 0x7FFFFFFFu) : 0;
}

// last g in [0, n) with a[g] <= v (a non-decreasing; a[0] <= v assumed), one thread
__device__ __forceinline__ uint64_t scan_last_le(const uint64_t* a, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The reader's cut-off (cache_service.rs:140-148) from the exclusive scans (x[g] = before g,
// x[K] = total): the response ends with the survivor whose Put is the max_results-th, or with
// the last survivor. info = {gend, items, bytes (records, no version byte), puts, first kept g,
// last kept g} (~0 for the kept g's when there is no item).
__global__ void k_scan_cut(const uint64_t* __restrict__ d_K, const uint64_t* __restrict__ putx,
                           const uint64_t* __restrict__ keepx, const uint64_t* __restrict__ offx, uint64_t max_results,
                           uint64_t* info) {
    if (threadIdx.x || blockIdx.x) return;
    const uint64_t K = *d_K;
    uint64_t gend = K;
    if (K && putx[K] >= max_results) gend = scan_last_le(putx, K + 1, max_results - 1) + 1;  // putx[gend] == max
    const uint64_t items = K ? keepx[gend] : 0;
    info[0] = gend;
    info[1] = items;
    info[2] = K ? offx[gend] : 0;
    info[3] = K ? putx[gend] : 0;
    info[4] = items ? scan_last_le(keepx, gend + 1, 0) : ~0ull;       // keepx[g] == 0 up to the first kept
    info[5] = items ? scan_last_le(keepx, gend + 1, items - 1) : ~0ull;  // the last kept's keepx == items - 1
}

// one wave per kept survivor g < gend: its record bytes to out[1 + offx[g] ..]; out[0] = version
__global__ void k_scan_gather(const uint64_t* __restrict__ info, const uint64_t* __restrict__ keep,
                              const uint64_t* __restrict__ offx, const uint64_t* __restrict__ size,
                              const uint64_t* __restrict__ m_src, uint8_t* out) {
    const uint64_t gend = info[0];
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (w0 == 0 && lane == 0 && info[1]) out[0] = 1;  // runs.rs:241-246
    for (uint64_t g = w0; g < gend; g += nw) {
        if (!keep[g]) continue;
        const uint8_t* src = (const uint8_t*)m_src[g];
        uint8_t* dst = out + 1 + offx[g];
        const uint64_t n = size[g];
        for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
    }
}

void launch_scan_filter(hipStream_t s, uint64_t R, uint32_t k, const uint64_t* stream_base, const uint64_t* a_addr,
                        const uint64_t* a_hi, const uint64_t* a_lo, const uint32_t* a_klen, const uint32_t* a_meta,
                        const uint8_t* start, uint32_t slen, uint64_t* keep, uint64_t* keepx, uint64_t* scan_tmp,
                        uint64_t* b_addr, uint64_t* b_hi, uint64_t* b_lo, uint32_t* b_klen, uint32_t* b_meta,
                        uint64_t* new_base) {
    const unsigned nb = (unsigned)((R + 255) / 256);
    if (R) k_scan_keep<<<nb, 256, 0, s>>>(R, a_addr, a_hi, a_lo, a_klen, start, slen, keep);
    launch_scan(s, keep, R, keepx, scan_tmp);  // keepx[R] = kept records
    if (R) k_scan_compact<<<nb, 256, 0, s>>>(R, keep, keepx, a_addr, a_hi, a_lo, a_klen, a_meta, b_addr, b_hi, b_lo,
                                             b_klen, b_meta);
    k_scan_bases<<<(k + 256) / 256, 256, 0, s>>>(k, stream_base, keepx, new_base);
}
void launch_scan_mark(hipStream_t s, const uint64_t* d_K, uint64_t R, const uint32_t* m_rec, const uint64_t* rec_addr,
                      const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen, const uint32_t* rec_meta,
                      const uint8_t* start, uint32_t slen, uint64_t* keep, uint64_t* put, uint64_t* size) {
    if (R) k_scan_mark<<<(unsigned)((R + 255) / 256), 256, 0, s>>>(d_K, m_rec, rec_addr, rec_hi, rec_lo, rec_klen,
                                                                  rec_meta, start, slen, keep, put, size);
}
void launch_scan_cut(hipStream_t s, const uint64_t* d_K, const uint64_t* putx, const uint64_t* keepx,
                     const uint64_t* offx, uint64_t max_results, uint64_t* info) {
    k_scan_cut<<<1, 64, 0, s>>>(d_K, putx, keepx, offx, max_results, info);
}
void launch_scan_gather(hipStream_t s, uint64_t R, const uint64_t* info, const uint64_t* keep, const uint64_t* offx,
                        const uint64_t* size, const uint64_t* m_src, uint8_t* out) {
    const uint64_t waves = R < (1u << 14) ? (R ? R : 1) : (1u << 14);  // wave-stride over g < gend <= K <= R
    k_scan_gather<<<(unsigned)((waves * 64 + 255) / 256), 256, 0, s>>>(info, keep, offx, size, m_src, out);
}

}  // namespace skv
