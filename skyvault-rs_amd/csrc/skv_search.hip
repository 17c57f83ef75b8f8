// skv_search.hip — batched point lookups in one run (the cache service's runs::search_run,
// runs.rs:285-398, called per key by cache_service.rs:52-151), on the device.
//
// search_run scans the run from its first record and stops at the first record whose key is not
// below the search key: equal -> Found(value) / Tombstone, greater -> NotFound; it panics on the
// malformed bytes it meets before stopping. Two kernels, one thread per query:
//   k_search_bsearch  the run parsed clean and its keys never decrease (every run build_runs
//                     writes): that first record is the lower bound over the parsed record
//                     arrays, one binary search per key;
//   k_search_scan     any other run (a parse error, a decrease): the reference's scan itself,
//                     with its checks in its order, so every panic and its text match.
#include "skv_launch.hpp"

namespace skv {

__device__ __forceinline__ uint32_t ld_be32_any(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// bytewise order of key (n bytes) vs query (m bytes): <0, 0, >0 (slice Ord)
__device__ __forceinline__ int sr_cmp(const uint8_t* key, uint64_t n, const uint8_t* q, uint64_t m) {
    const int c = bytes_cmp16(key, q, n < m ? n : m);
    if (c) return c;
    return n < m ? -1 : (n > m ? 1 : 0);
}

__device__ void sr_found(const uint8_t* run, uint64_t len, uint64_t p, uint32_t marker, uint64_t klen,
                         SrResult& r) {
    // the record at p is valid (parsed clean): marker, key_len, key, [val_len, value]
    if (marker == 2) {
        r.kind = SR_TOMBSTONE;
        return;
    }
    const uint64_t vp = p + 5 + klen;
    r.kind = SR_FOUND;
    r.val_len = ld_be32_any(run + vp);
    r.val_off = vp + 4;
    (void)len;
}

__global__ void k_search_bsearch(const uint8_t* __restrict__ run, uint64_t len, uint64_t R,
                                 const uint64_t* __restrict__ rec_addr, const uint64_t* __restrict__ rec_hi,
                                 const uint64_t* __restrict__ rec_lo, const uint32_t* __restrict__ rec_klen,
                                 const uint32_t* __restrict__ rec_meta, const uint8_t* __restrict__ qbytes,
                                 const uint64_t* __restrict__ qoff, uint32_t n_q, SrResult* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_q) return;
    const uint8_t* q = qbytes + qoff[i];
    const uint64_t m = qoff[i + 1] - qoff[i];
    uint64_t qh, ql;
    key_prefix(q, m, qh, ql);
    uint64_t a = 0, b = R;  // first record whose key is not below q
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        const int c = key_cmp(rec_hi[mid], rec_lo[mid], rec_klen[mid], (const uint8_t*)rec_addr[mid] + 5, qh, ql,
                              (uint32_t)m, q);
        if (c < 0) a = mid + 1;
        else b = mid;
    }
    SrResult r{};
    r.kind = SR_NOT_FOUND;
    if (a < R) {
        const uint8_t* rp = (const uint8_t*)rec_addr[a];
        const uint32_t kl = rec_klen[a];
        if (sr_cmp(rp + 5, kl, q, m) == 0)
            sr_found(run, len, (uint64_t)(rp - run), (rec_meta[a] >> 31) ? 2u : 1u, kl, r);
    }
    out[i] = r;
}

__global__ void k_search_scan(const uint8_t* __restrict__ run, uint64_t len, const uint8_t* __restrict__ qbytes,
                              const uint64_t* __restrict__ qoff, uint32_t n_q, SrResult* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_q) return;
    const uint8_t* q = qbytes + qoff[i];
    const uint64_t m = qoff[i + 1] - qoff[i];
    SrResult r{};
    r.kind = SR_NOT_FOUND;
    uint64_t p = 1;  // after the version byte (checked by the host)
    while (p < len) {
        const uint32_t marker = run[p];
        if (marker != 1 && marker != 2) {  // runs.rs:307-310
            r.kind = SR_PANIC;
            r.panic = SRP_MARKER | (marker << 8);
            break;
        }
        if (p + 1 + 4 > len) {  // :313-315
            r.kind = SR_PANIC;
            r.panic = SRP_KEYLEN;
            break;
        }
        const uint64_t klen = ld_be32_any(run + p + 1);
        const uint64_t kp = p + 5;
        if (kp + klen > len) {  // :324-326
            r.kind = SR_PANIC;
            r.panic = SRP_KEY;
            break;
        }
        const int c = sr_cmp(run + kp, klen, q, m);
        uint64_t cur = kp + klen;
        if (c < 0) {  // :331-356 skip the entry
            if (marker == 1) {
                if (cur + 4 > len) {
                    r.kind = SR_PANIC;
                    r.panic = SRP_VALLEN;
                    break;
                }
                const uint64_t vlen = ld_be32_any(run + cur);
                const uint64_t vp = cur + 4;
                if (vp + vlen > len) {
                    r.kind = SR_PANIC;
                    r.panic = SRP_VAL;
                    break;
                }
                cur = vp + vlen;
            }
            p = cur;
            continue;
        }
        if (c == 0) {  // :357-386
            if (marker == 2) {
                r.kind = SR_TOMBSTONE;
            } else if (cur + 4 > len) {
                r.kind = SR_PANIC;
                r.panic = SRP_VALLEN_FOUND;
            } else {
                const uint64_t vlen = ld_be32_any(run + cur);
                const uint64_t vp = cur + 4;
                if (vp + vlen > len) {
                    r.kind = SR_PANIC;
                    r.panic = SRP_VAL_FOUND;
                } else {
                    r.kind = SR_FOUND;
                    r.val_off = vp;
                    r.val_len = vlen;
                }
            }
        }
        break;  // equal: found; greater: NotFound (:387-391)
    }
    out[i] = r;
}

void launch_search_bsearch(hipStream_t s, const uint8_t* run, uint64_t len, uint64_t R, const uint64_t* rec_addr,
                           const uint64_t* rec_hi, const uint64_t* rec_lo, const uint32_t* rec_klen,
                           const uint32_t* rec_meta, const uint8_t* qbytes, const uint64_t* qoff, uint32_t n_q,
                           SrResult* out) {
    if (n_q)
        k_search_bsearch<<<(n_q + 255) / 256, 256, 0, s>>>(run, len, R, rec_addr, rec_hi, rec_lo, rec_klen, rec_meta,
                                                           qbytes, qoff, n_q, out);
}
void launch_search_scan(hipStream_t s, const uint8_t* run, uint64_t len, const uint8_t* qbytes, const uint64_t* qoff,
                        uint32_t n_q, SrResult* out) {
    if (n_q) k_search_scan<<<(n_q + 255) / 256, 256, 0, s>>>(run, len, qbytes, qoff, n_q, out);
}

}  // namespace skv
