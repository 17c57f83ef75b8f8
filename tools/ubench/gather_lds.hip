// Gather probe on config 3F's memory pattern ("a gather with aligned
// line-granular loads realigned in LDS" was not tried). 256 input streams of variable-length
// records (80..399 B, packed at arbitrary alignment), ~80 % of them surviving, output in merged
// (key) order, packed. Two output-order gathers over segments of survivors:
//   A  the product's k_gather fast path: per output 16-byte block one unaligned 16-byte global load
//      (two + a funnel shift where the block straddles two records), aligned store; segment edges
//      bytewise.
//   B  each segment's records first loaded as their ALIGNED 16-byte covers (line-granular, every
//      load aligned, no byte read twice inside the segment) into LDS, then every output block
//      composed from LDS (two aligned ds_read_b128 + funnel per window) and stored aligned.
//   C  input order: four lanes per input record, unaligned 16-byte loads and stores straight to
//      each survivor's output place (reads contiguous; writes scattered, partial at record edges).
// All outputs are checked against the host's expected bytes. Time: best of 5 (HIP events).
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/gl tools/ubench/gather_lds.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                      \
        }                                                                  \
    } while (0)

static uint64_t sm64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef unsigned int g_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld16(const uint8_t* a) {
    const g_v4 v = *(const __attribute__((address_space(1))) g_v4*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// bytes [s, s + 16) of the 32-byte concatenation lo ++ hi (0 <= s < 16)
__device__ __forceinline__ uint4 funnel(uint4 lo, uint4 hi, uint32_t s) {
    if (s == 0) return lo;
    uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const uint32_t q = s >> 2, r = (s & 3) * 8;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((uint32_t)j == q + i) a = w[j];
            if ((uint32_t)j == q + i + 1) b = w[j];
        }
        o[i] = r ? (a >> r) | (b << (32 - r)) : a;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

constexpr int SEG_A = 256, THR = 256, TBL_A = SEG_A * 26 + 2;

__global__ void __launch_bounds__(THR) k_gA(const uint64_t* __restrict__ P, const uint64_t* __restrict__ src,
                                            const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t K) {
    __shared__ uint64_t s_d[SEG_A + 1];
    __shared__ const uint8_t* s_s[SEG_A];
    __shared__ uint16_t s_tbl[TBL_A];
    const uint64_t j0 = (uint64_t)blockIdx.x * SEG_A;
    if (j0 >= K) return;
    const uint32_t n = (uint32_t)(K - j0 < SEG_A ? K - j0 : SEG_A);
    if (threadIdx.x < n) {
        s_d[threadIdx.x] = P[j0 + threadIdx.x];
        s_s[threadIdx.x] = in + src[j0 + threadIdx.x];
        if (threadIdx.x == n - 1) s_d[n] = P[j0 + n];
    }
    __syncthreads();
    const uint64_t lo = s_d[0], hi = s_d[n], q0 = lo >> 4, q1 = (hi + 15) >> 4;
    const uint32_t nq = (uint32_t)(q1 - q0);
    for (uint32_t p = threadIdx.x; p < n; p += THR) {
        const uint64_t d = s_d[p], e = s_d[p + 1];
        uint64_t qs = (d + 15) >> 4;
        if (d == lo) s_tbl[0] = (uint16_t)p;
        if (qs <= q0) qs = q0 + 1;
        for (uint64_t q = qs; q < (e + 15) >> 4; ++q) s_tbl[q - q0] = (uint16_t)p;
    }
    __syncthreads();
    constexpr int U = 2;
    for (uint32_t qi0 = threadIdx.x; qi0 < nq; qi0 += U * THR) {
        uint4 L[U], X[U];
        bool ok[U], two[U];
        uint32_t sh[U];
        const uint8_t *aL[U], *aX[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t qi = qi0 + u * THR;
            const uint32_t qc = qi < nq ? qi : nq - 1;
            const uint64_t B = (q0 + qc) << 4;
            const uint32_t p = s_tbl[qc];
            const uint64_t d = s_d[p], e = s_d[p + 1];
            const bool inr = qi < nq && B >= lo && B + 16 <= hi;
            const bool c1 = e >= B + 16;
            ok[u] = inr;
            two[u] = inr && !c1;
            aL[u] = c1 ? s_s[p] + (B - d) : s_s[p] + (e - d) - 16;
            aX[u] = p + 1 < n ? s_s[p + 1] : s_s[p];
            sh[u] = 16u - (uint32_t)(e - B);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            L[u] = ok[u] ? gld16(aL[u]) : make_uint4(0, 0, 0, 0);
            X[u] = two[u] ? gld16(aX[u]) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) *(uint4*)(out + ((q0 + qi0 + u * THR) << 4)) = two[u] ? funnel(L[u], X[u], sh[u] & 15u) : L[u];
    }
    // segment edges: this segment's bytes of the first / last block, bytewise
    if (threadIdx.x < 2) {
        const uint64_t B = threadIdx.x == 0 ? (q0 << 4) : ((q1 - 1) << 4);
        if (threadIdx.x == 1 && q1 - 1 == q0) return;
        if (B >= lo && B + 16 <= hi) return;
        const uint64_t y0 = B > lo ? B : lo, y1 = B + 16 < hi ? B + 16 : hi;
        uint32_t p = 0;
        for (uint64_t y = y0; y < y1; ++y) {
            while (s_d[p + 1] <= y) ++p;
            out[y] = s_s[p][y - s_d[p]];
        }
    }
}

constexpr int SEG_B = 128, LDS_B = 57344;  // 128 records of <= 399 B: covers <= 128 x 416 = 53,248 B

__global__ void __launch_bounds__(THR) k_gB(const uint64_t* __restrict__ P, const uint64_t* __restrict__ src,
                                            const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t K) {
    __shared__ uint64_t s_d[SEG_B + 1];
    __shared__ uint64_t s_c0[SEG_B];      // aligned cover start (input offset)
    __shared__ uint32_t s_lo[SEG_B + 1];  // cover's LDS offset
    __shared__ uint16_t s_bt[LDS_B / 16]; // cover block -> record
    __shared__ uint16_t s_tbl[SEG_B * 26 + 2];
    __shared__ uint32_t ws[8];
    __shared__ uint8_t s_mis[SEG_B];      // src & 15: record p's byte x sits at LDS s_lo[p] + s_mis[p] + x
    __shared__ uint4 s_buf[LDS_B / 16];
    const uint8_t* sb = (const uint8_t*)s_buf;
    const uint64_t j0 = (uint64_t)blockIdx.x * SEG_B;
    if (j0 >= K) return;
    const uint32_t n = (uint32_t)(K - j0 < SEG_B ? K - j0 : SEG_B);
    const uint32_t t = threadIdx.x;
    uint32_t clen = 0;
    uint64_t sa = 0, d = 0, e = 0;
    if (t < n) {
        d = P[j0 + t];
        e = P[j0 + t + 1];
        sa = src[j0 + t];
        s_d[t] = d;
        if (t == n - 1) s_d[n] = e;
        const uint64_t c0 = sa & ~15ull, c1 = (sa + (e - d) + 15) & ~15ull;
        s_c0[t] = c0;
        s_mis[t] = (uint8_t)(sa & 15);
        clen = (uint32_t)(c1 - c0);
    }
    // exclusive scan of clen over the block (4 waves)
    uint32_t v = clen;
    const uint32_t lane = t & 63, wv = t >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += x;
    }
    if (lane == 63) ws[wv] = v;
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wv; ++w) wpre += ws[w];
    const uint32_t lo_b = wpre + v - clen;
    const uint32_t total = ws[0] + ws[1] + ws[2] + ws[3];
    if (t < n) {
        s_lo[t] = lo_b;
        if (t == n - 1) s_lo[n] = lo_b + clen;
        for (uint32_t c = 0; c < clen / 16; ++c) s_bt[lo_b / 16 + c] = (uint16_t)t;
    }
    __syncthreads();
    // load phase: every cover block once, aligned
    const uint32_t nb = total / 16;
    constexpr int UL = 4;
    for (uint32_t b0 = t; b0 < nb; b0 += UL * THR) {
        uint4 x[UL];
#pragma unroll
        for (int u = 0; u < UL; ++u) {
            const uint32_t b = b0 + u * THR;
            if (b < nb) {
                const uint32_t p = s_bt[b];
                x[u] = gld16(in + s_c0[p] + (b * 16 - s_lo[p]));
            }
        }
#pragma unroll
        for (int u = 0; u < UL; ++u)
            if (b0 + u * THR < nb) s_buf[b0 + u * THR] = x[u];
    }
    // output block table
    const uint64_t lo = s_d[0], hi = s_d[n], q0 = lo >> 4, q1 = (hi + 15) >> 4;
    const uint32_t nq = (uint32_t)(q1 - q0);
    if (t < n) {
        uint64_t qs = (d + 15) >> 4;
        if (d == lo) s_tbl[0] = (uint16_t)t;
        if (qs <= q0) qs = q0 + 1;
        for (uint64_t q = qs; q < (e + 15) >> 4; ++q) s_tbl[q - q0] = (uint16_t)t;
    }
    __syncthreads();
    for (uint32_t qi = t; qi < nq; qi += THR) {
        const uint64_t B = (q0 + qi) << 4;
        if (!(B >= lo && B + 16 <= hi)) continue;
        const uint32_t p = s_tbl[qi];
        const uint64_t dp = s_d[p], ep = s_d[p + 1];
        const uint32_t off_p = s_lo[p] + s_mis[p];
        uint4 r;
        if (ep >= B + 16) {
            const uint32_t a = off_p + (uint32_t)(B - dp);
            const uint32_t a0 = a & ~15u;
            r = funnel(*(const uint4*)(sb + a0), *(const uint4*)(sb + a0 + 16), a & 15u);
        } else {
            const uint32_t k = (uint32_t)(ep - B);  // bytes from record p
            const uint32_t aL = off_p + (uint32_t)(ep - dp) - 16, aL0 = aL & ~15u;
            const uint4 L = funnel(*(const uint4*)(sb + aL0), *(const uint4*)(sb + aL0 + 16), aL & 15u);
            const uint32_t off_n = s_lo[p + 1] + s_mis[p + 1];
            const uint32_t aF0 = off_n & ~15u;
            const uint4 F = funnel(*(const uint4*)(sb + aF0), *(const uint4*)(sb + aF0 + 16), off_n & 15u);
            r = funnel(L, F, 16 - k);
        }
        *(uint4*)(out + B) = r;
    }
    if (t < 2) {
        const uint64_t B = t == 0 ? (q0 << 4) : ((q1 - 1) << 4);
        if (t == 1 && q1 - 1 == q0) return;
        if (B >= lo && B + 16 <= hi) return;
        const uint64_t y0 = B > lo ? B : lo, y1 = B + 16 < hi ? B + 16 : hi;
        uint32_t p = 0;
        for (uint64_t y = y0; y < y1; ++y) {
            while (s_d[p + 1] <= y) ++p;
            out[y] = sb[s_lo[p] + s_mis[p] + (y - s_d[p])];
        }
    }
}

// C: input order. Four lanes per input record (records consecutive in the input, so a wave's loads
// cover contiguous input bytes); every surviving record's 16-byte chunks go to its output place with
// unaligned 16-byte stores, its last chunk as the record's last 16 bytes (an overlapping window that
// never leaves the record, so neighbouring records written by other workgroups are not touched).
__global__ void __launch_bounds__(THR) k_gC(const uint64_t* __restrict__ dst, const uint64_t* __restrict__ off,
                                            const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t N) {
    const uint64_t r = (uint64_t)blockIdx.x * (THR / 4) + threadIdx.x / 4;
    if (r >= N) return;
    const uint64_t d = dst[r];
    if (d == ~0ull) return;
    const uint64_t s = off[r], len = off[r + 1] - s;
    const uint32_t c0 = threadIdx.x & 3;
    for (uint64_t c = c0 * 16; c < len; c += 64) {
        const uint64_t cc = c + 16 <= len ? c : len - 16;
        const uint4 v = gld16(in + s + cc);
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        u4 w = {v.x, v.y, v.z, v.w};
        *(__attribute__((address_space(1))) u4*)(out + d + cc) = w;
    }
}

int main(int argc, char** argv) {
    const uint32_t NS = 256;
    const uint64_t PER = argc > 1 ? strtoull(argv[1], nullptr, 10) : 50000;
    const uint64_t N = NS * PER;
    uint64_t seed = 42;
    std::vector<uint32_t> len(N);
    std::vector<uint64_t> off(N + 1, 0);
    for (uint64_t r = 0; r < N; ++r) {
        len[r] = 80 + (uint32_t)(sm64(seed) % 320);
        off[r + 1] = off[r] + len[r];
    }
    const uint64_t in_bytes = off[N];
    // merged order: each stream's records ascend by random key; the merge interleaves by key
    std::vector<std::pair<uint64_t, uint64_t>> kr(N);
    for (uint32_t s = 0; s < NS; ++s) {
        std::vector<uint64_t> ks(PER);
        for (auto& k : ks) k = sm64(seed);
        std::sort(ks.begin(), ks.end());
        for (uint64_t i = 0; i < PER; ++i) kr[s * PER + i] = {ks[i], s * PER + i};
    }
    std::sort(kr.begin(), kr.end());
    std::vector<uint64_t> srcv, Pv(1, 0), dstv(N, ~0ull);
    for (auto& x : kr) {
        if (sm64(seed) % 100 < 20) continue;  // superseded / deleted
        srcv.push_back(off[x.second]);
        dstv[x.second] = Pv.back();
        Pv.push_back(Pv.back() + len[x.second]);
    }
    const uint64_t K = srcv.size(), out_bytes = Pv.back();
    printf("records %llu (%.2f GB), survivors %llu (%.2f GB)\n", (unsigned long long)N, in_bytes / 1e9,
           (unsigned long long)K, out_bytes / 1e9);
    std::vector<uint8_t> hin(in_bytes);
    for (uint64_t i = 0; i < in_bytes; i += 8) {
        const uint64_t z = sm64(seed);
        memcpy(&hin[i], &z, std::min<uint64_t>(8, in_bytes - i));
    }
    uint8_t *din, *dout;
    uint64_t *dP, *dS, *dD, *dO;
    CK(hipMalloc(&din, in_bytes + 64));
    CK(hipMalloc(&dout, out_bytes + 64));
    CK(hipMalloc(&dP, (K + 1) * 8));
    CK(hipMalloc(&dS, K * 8));
    CK(hipMemcpy(din, hin.data(), in_bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(dP, Pv.data(), (K + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dS, srcv.data(), K * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&dD, N * 8));
    CK(hipMalloc(&dO, (N + 1) * 8));
    CK(hipMemcpy(dD, dstv.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dO, off.data(), (N + 1) * 8, hipMemcpyHostToDevice));
    std::vector<uint8_t> exp(out_bytes), got(out_bytes);
    for (uint64_t j = 0; j < K; ++j) memcpy(&exp[Pv[j]], &hin[srcv[j]], Pv[j + 1] - Pv[j]);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* which = argc > 2 ? argv[2] : "AB";
    for (const char* w = which; *w; ++w) {
        const bool isA = *w == 'A', isC = *w == 'C';
        const uint64_t seg = isA ? SEG_A : SEG_B;
        const unsigned grid = isC ? (unsigned)((N + THR / 4 - 1) / (THR / 4)) : (unsigned)((K + seg - 1) / seg);
        float best = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipMemset(dout, 0, out_bytes));
            CK(hipEventRecord(e0));
            if (isA) k_gA<<<grid, THR>>>(dP, dS, din, dout, K);
            else if (isC) k_gC<<<grid, THR>>>(dD, dO, din, dout, N);
            else k_gB<<<grid, THR>>>(dP, dS, din, dout, K);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) best = std::min(best, ms);
        }
        CK(hipMemcpy(got.data(), dout, out_bytes, hipMemcpyDeviceToHost));
        uint64_t bad = 0, first = ~0ull;
        for (uint64_t i = 0; i < out_bytes; ++i)
            if (got[i] != exp[i]) {
                if (!bad) first = i;
                ++bad;
            }
        printf("%c: %.3f ms  %.2f TB/s of survivor bytes read+written  mismatches %llu (first %lld)\n", *w, best,
               2.0 * out_bytes / best / 1e9, (unsigned long long)bad, bad ? (long long)first : -1ll);
    }
    return 0;
}
