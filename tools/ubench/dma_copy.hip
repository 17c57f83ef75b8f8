// dma_copy.hip — the fused tile's copy phase two ways, on the headline's access pattern (VERDICT r05
// item 2: "build the LDS-DMA tile ... if it loses, commit the probe with its PMC passes").
//
// Input: 64 runs x 238,821 records of 281 B (config 2A: 4.0 GiB) in HBM; the merged order of the
// records (random 64-bit keys, sorted on the host) as one source address per output record, i.e.
// what k_fx_tile holds after its merge. Output: the records in merged order, back to back (4.0 GiB).
// One workgroup of 512 threads per tile of TR = 1,536 output records (k_fx_tile's target), tiles in
// XCD-contiguous order:
//   direct  k_fx_tile's copy: each lane composes aligned 16-byte output blocks from unaligned
//           16-byte global loads (two and a funnel shift where a block straddles two records),
//           loads of two blocks issued before their stores, non-temporal stores;
//   dma     the same tile staged through LDS by global_load_lds_dwordx4: chunks of C records, each
//           record's aligned 16-byte cover (19 blocks) DMA'd to a slot (19 x 16 B), two chunk buffers
//           (chunk c + 1 in flight while chunk c is composed), the output blocks composed from LDS
//           (5 ds_read_b32 + alignbyte per record piece), non-temporal stores.
// Both outputs are checked against each other; times by HIP events over 20 launches; run the PMC
// passes separately (tools/r06/dma_probe.sh).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr uint32_t S = 281;        // record size (16 B key + 256 B value + 9 B framing)
constexpr uint32_t NB = 19;        // 16-byte blocks of a record's aligned cover (281 + 15 <= 19 * 16)
constexpr uint32_t TR = 1536;      // output records per tile
constexpr uint32_t THREADS = 512;
#ifndef DMA_C
#define DMA_C 32                   // records per LDS chunk
#endif
constexpr uint32_t C = DMA_C;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_nt(uint8_t* p, uint4 v) {
    v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (v4u*)p);
}
__device__ __forceinline__ uint4 ld16(uint64_t a) {
    const v4u v = *(const __attribute__((address_space(1))) v4u*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 funnel(uint4 x, uint4 y, uint32_t sh) {  // bytes sh.. of x:y
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
__device__ __forceinline__ uint32_t tile_of(uint32_t bid, uint32_t nb) {  // XCD-contiguous tile order
    const uint32_t xcd = bid & 7, qn = nb >> 3, rn = nb & 7;
    return (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (bid >> 3);
}

// ---- direct: k_fx_tile's copy (two blocks per lane per batch, loads before stores)
__global__ void __launch_bounds__(THREADS) k_direct(const uint64_t* __restrict__ src, uint32_t R, uint8_t* __restrict__ out) {
    const uint32_t t = tile_of(blockIdx.x, gridDim.x);
    const uint32_t r0 = t * TR, r1 = min(r0 + TR, R);
    if (r0 >= r1) return;
    const uint64_t o0 = (uint64_t)r0 * S, o1 = (uint64_t)r1 * S;
    const uint64_t B0 = (o0 + 15) & ~15ull, B1 = o1 & ~15ull;
    const uint32_t nb = (uint32_t)((B1 - B0) >> 4);
    constexpr int U = 2;
    for (uint32_t b = threadIdx.x; b < nb; b += U * THREADS) {
        uint64_t aL[U], aX[U];
        uint32_t sh[U];
        bool two[U], ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t bb = b + u * THREADS;
            ok[u] = bb < nb;
            const uint64_t x = B0 + 16ull * (ok[u] ? bb : 0);
            const uint64_t j = x / S, o = x - j * S;
            two[u] = o + 16 > S;
            aL[u] = two[u] ? src[j] + S - 16 : src[j] + o;
            aX[u] = two[u] ? src[j + 1] : aL[u];
            sh[u] = 16 - (uint32_t)(S - o);
        }
        uint4 L[U], X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            L[u] = ld16(aL[u]);
            X[u] = make_uint4(0, 0, 0, 0);
            if (two[u]) X[u] = ld16(aX[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) st_nt(out + B0 + 16ull * (b + u * THREADS), two[u] ? funnel(L[u], X[u], sh[u] & 15) : L[u]);
    }
    // tile edges bytewise (the blocks shared with the neighbouring tiles)
    if (threadIdx.x == 0) {
        for (uint64_t y = o0; y < B0 && y < o1; ++y) out[y] = *(const uint8_t*)(src[y / S] + y % S);
        for (uint64_t y = std::max(B1, B0); y < o1; ++y) out[y] = *(const uint8_t*)(src[y / S] + y % S);
    }
}

// ---- dma: the tile through LDS by global_load_lds_dwordx4. Issued from inline asm (the recipe of
// cdna_hip_programming.md: M0 saved and restored in the same statement): with the builtin, hipcc's
// waitcnt pass waits vmcnt(0) before every later LDS read -- the chunk in flight AND the stores queued
// behind it -- which removes the double buffering; the waits below are counted by hand instead.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_byte_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte_addr)
                 : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__global__ void __launch_bounds__(THREADS) k_dma(const uint64_t* __restrict__ src, uint32_t R, uint8_t* __restrict__ out) {
    // two chunk buffers of C slots x NB blocks (16 B): lane l of a wave-instruction writes unit base + l;
    // the tile's source addresses in LDS (the DMA issue reads them with no VMEM load, so waiting for a
    // chunk's DMAs never waits for the stores queued behind them)
    static_assert((C * S) % 16 == 0 && (TR * S) % 16 == 0, "chunk and tile edges on 16-byte boundaries");
    // every lane of a DMA wave-instruction writes its 16 bytes: a buffer holds whole instructions
    // (C * NB units rounded up to 64), or the last instruction's idle lanes would write past it
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][(C * NB + 63) / 64 * 64 * 4];
    __shared__ uint64_t s_src[TR];
    const uint32_t t = tile_of(blockIdx.x, gridDim.x);
    const uint32_t r0 = t * TR, r1 = min(r0 + TR, R);
    if (r0 >= r1) return;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr uint32_t UNITS = C * NB;                  // 16-byte units per chunk
    constexpr uint32_t INSTR = (UNITS + 63) / 64;       // wave-instructions per chunk
    constexpr uint32_t BPC = C * S / 16;                // output blocks per chunk
    for (uint32_t i = threadIdx.x; i < r1 - r0; i += THREADS) s_src[i] = src[r0 + i];
    __syncthreads();
    const uint32_t nch = (r1 - r0 + C - 1) / C;
    auto issue = [&](uint32_t c) {  // chunk c's covers -> buf[c & 1]; waves take instructions round-robin
        const uint32_t q0 = c * C;
        for (uint32_t ins = wid; ins < INSTR; ins += THREADS / 64) {
            const uint32_t u = ins * 64 + lane;
            const uint32_t slot = u / NB, blk = u - slot * NB;
            const uint32_t r = q0 + slot;
            const uint64_t a = (r0 + r < r1 && slot < C) ? ((s_src[r] & ~15ull) + 16ull * blk) : (s_src[0] & ~15ull);
            glds16((const void*)a, __builtin_amdgcn_readfirstlane(lds_addr(&buf[c & 1][ins * 64 * 4])));
        }
    };
    // store instructions this wave issues per chunk (a full chunk: BPC blocks over THREADS lanes)
    const uint32_t n_st = (BPC > 64 * wid ? (BPC - 64 * wid + THREADS - 1) / THREADS : 0);
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint32_t c = 0; c < nch; ++c) {
        if (c + 1 < nch) issue(c + 1);
        const uint32_t q0 = c * C, q1 = min(q0 + C, r1 - r0);
        const uint64_t o0 = (uint64_t)(r0 + q0) * S;
        const uint32_t nbk = (q1 - q0) * S / 16;
        const uint32_t* bb = buf[c & 1];
        for (uint32_t b = threadIdx.x; b < nbk; b += THREADS) {
            const uint32_t rel = 16 * b, j = rel / S, o = rel - j * S;
            auto read16 = [&](uint32_t jj, uint32_t oo) {  // 16 bytes of slot jj from record offset oo
                const uint32_t off = (uint32_t)(s_src[q0 + jj] & 15) + oo + jj * NB * 16;
                const uint32_t w = off >> 2, r = off & 3;
                const uint32_t d0 = bb[w], d1 = bb[w + 1], d2 = bb[w + 2], d3 = bb[w + 3], d4 = bb[w + 4];
                return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r),
                                  __builtin_amdgcn_alignbyte(d3, d2, r), __builtin_amdgcn_alignbyte(d4, d3, r));
            };
            uint4 v;
            if (o + 16 <= S) {
                v = read16(j, o);
            } else {
                const uint4 L = read16(j, S - 16), X = read16(j + 1, 0);
                v = funnel(L, X, 16 - (S - o));
            }
            st_nt(out + o0 + 16ull * b, v);
        }
        if (c + 1 < nch) {  // chunk c + 1's DMAs landed (the stores just queued may still be in flight)
            if (n_st >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else if (n_st == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // (not __syncthreads: its fence would drain the stores)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

int main(int argc, char** argv) {
    const uint32_t K = 64, N = 238821;
    const uint32_t R = K * N;
    const uint64_t run_bytes = 1 + (uint64_t)N * S;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const char* which = argc > 2 ? argv[2] : "both";
    uint8_t* d_in;
    CK(hipMalloc(&d_in, K * run_bytes + 64));
    {  // random bytes: contents do not matter to the copy
        std::vector<uint32_t> h((K * run_bytes + 64) / 4);
        std::mt19937 g(1);
        for (auto& x : h) x = g();
        CK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    std::vector<uint64_t> src(R + 1);
    {  // merged order of random keys (the merge's output order): sort (key, stream, index)
        std::vector<std::pair<uint64_t, uint32_t>> e(R);
        std::mt19937_64 g(7);
        for (uint32_t s = 0; s < K; ++s) {
            std::vector<uint64_t> keys(N);
            for (auto& x : keys) x = g();
            std::sort(keys.begin(), keys.end());
            for (uint32_t i = 0; i < N; ++i) e[(uint64_t)s * N + i] = {keys[i], s * N + i};
        }
        std::sort(e.begin(), e.end());
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t s = e[r].second / N, i = e[r].second % N;
            src[r] = (uint64_t)(uintptr_t)d_in + s * run_bytes + 1 + (uint64_t)i * S;
        }
        src[R] = src[R - 1];
    }
    uint64_t* d_src;
    CK(hipMalloc(&d_src, (R + 1) * 8));
    CK(hipMemcpy(d_src, src.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    const uint64_t out_bytes = (uint64_t)R * S;
    uint8_t *d_out_a, *d_out_b;
    CK(hipMalloc(&d_out_a, out_bytes + 64));
    CK(hipMalloc(&d_out_b, out_bytes + 64));
    const uint32_t tiles = (R + TR - 1) / TR;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 2.0 * out_bytes;  // each record read once, written once
    auto run = [&](const char* name, auto kern, uint8_t* out) {
        kern<<<tiles, THREADS>>>(d_src, R, out);  // warm-up
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) kern<<<tiles, THREADS>>>(d_src, R, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-7s %8.3f ms  %7.3f TB/s (I+O)  frac %.3f of 8 TB/s\n", name, ms, alg / ms / 1e9, alg / ms / 1e9 / 8.0);
    };
    const bool both = !strcmp(which, "both");
    if (both || !strcmp(which, "direct")) run("direct", k_direct, d_out_a);
    if (both || !strcmp(which, "dma")) run("dma", k_dma, d_out_b);
    if (!both && !strcmp(which, "dma")) return 0;
    if (both) {
        std::vector<uint8_t> a(out_bytes), b(out_bytes);
        CK(hipMemcpy(a.data(), d_out_a, out_bytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), d_out_b, out_bytes, hipMemcpyDeviceToHost));
        size_t bad = 0, first = ~(size_t)0;
        for (size_t i = 0; i < out_bytes; ++i)
            if (a[i] != b[i]) {
                if (first == ~(size_t)0) first = i;
                ++bad;
            }
        // and a spot check of the direct copy against the input bytes
        size_t bad_src = 0;
        std::vector<uint8_t> rec(S);
        for (uint32_t r = 0; r < R; r += 9973) {
            CK(hipMemcpy(rec.data(), (const void*)(uintptr_t)src[r], S, hipMemcpyDeviceToHost));
            bad_src += memcmp(rec.data(), a.data() + (uint64_t)r * S, S) != 0;
        }
        printf("outputs: %zu differing bytes (first %zd); direct vs input records: %zu bad of %u sampled\n", bad,
               bad ? (ssize_t)first : (ssize_t)-1, bad_src, (R + 9972) / 9973);
        return bad || bad_src;
    }
    return 0;
}
