// Host-side harness (plain C++, builds with g++ or hipcc): the general pipeline's cut search over 10^6
// config-5 WAL runs (83 x 49-byte records), one walk per run for all cuts vs a batched binary search.
// g++ -O2 -pthread -x c++ cut_search_host.hip -o cut_search && ./cut_search 8
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include <thread>
#include <chrono>
#include <cstdio>
#include <algorithm>
static uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
inline uint64_t host_rec_at(const uint8_t* b, uint64_t len, uint64_t p) {
    if (p + 5 > len) return 0;
    const uint8_t marker = b[p];
    const uint64_t klen = be32(b + p + 1), kp = p + 5;
    if (kp + klen > len) return 0;
    if (marker == 2) return 5 + klen;
    if (marker != 1 || kp + klen + 4 > len) return 0;
    const uint64_t vlen = be32(b + kp + klen);
    return kp + klen + 4 + vlen > len ? 0 : 9 + klen + vlen;
}
inline int host_key_cmp(const uint8_t* a, uint64_t al, const uint8_t* c, uint64_t cl) {
    const int r = memcmp(a, c, al < cl ? al : cl);
    return r ? r : (al < cl ? -1 : (al > cl ? 1 : 0));
}
int main(int argc, char** argv) {
    const uint64_t N = 1000000, R = 83, S = 49, L = 1 + R * S;
    std::vector<uint8_t> buf(N * L);
    uint64_t x = 88172645463325252ull;
    for (uint64_t i = 0; i < N; ++i) {
        uint8_t* r = buf.data() + i * L; r[0] = 1;
        std::vector<std::string> keys;
        for (uint64_t j = 0; j < R; ++j) { x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            char k[40]; int t = x % 64; snprintf(k, sizeof k, "%d.%0*llu", t, (int)(32 - (t < 10 ? 2 : 3)), (unsigned long long)((x >> 8) % 1000000000000ull)); keys.push_back(std::string(k, 32)); }
        std::sort(keys.begin(), keys.end());
        for (uint64_t j = 0; j < R; ++j) { uint8_t* p = r + 1 + j * S; p[0] = 1; p[1] = 0; p[2] = 0; p[3] = 0; p[4] = 32; memcpy(p + 5, keys[j].data(), 32); p[37] = 0; p[38] = 0; p[39] = 0; p[40] = 8; }
    }
    std::vector<std::string> cut = {"23.", "39.", "54."};
    const int T = argc > 1 ? atoi(argv[1]) : 8;
    std::vector<uint64_t> bnd(N * 4);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
        for (uint64_t m = N * t / T; m < N * (t + 1) / T; ++m) {
            const uint8_t* rb = buf.data() + m * L; uint64_t q = 1;
            for (int p = 0; p < 3; ++p) {
                while (q < L) { const uint64_t sz = host_rec_at(rb, L, q); if (!sz) break;
                    if (host_key_cmp(rb + q + 5, be32(rb + q + 1), (const uint8_t*)cut[p].data(), cut[p].size()) >= 0) break; q += sz; }
                bnd[m * 4 + p] = q;
            }
        }
    });
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    printf("walk threads %d: %.1f ms\n", T, std::chrono::duration<double, std::milli>(t1 - t0).count());
    // batched binary search: G runs at a time per thread, all their probes of one step prefetched
    std::vector<uint64_t> bnd2(N * 4);
    t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th2;
    for (int t = 0; t < T; ++t) th2.emplace_back([&, t] {
        constexpr int G = 16;
        const uint64_t m0 = N * t / T, m1 = N * (t + 1) / T;
        for (uint64_t mb = m0; mb < m1; mb += G) {
            const int g = (int)std::min<uint64_t>(G, m1 - mb);
            for (int p = 0; p < 3; ++p) {
                uint64_t lo[G], hi[G];
                for (int i = 0; i < g; ++i) { lo[i] = p ? (bnd2[(mb + i) * 4 + p - 1] - 1) / S : 0; hi[i] = R; }
                for (;;) {
                    bool any = false;
                    for (int i = 0; i < g; ++i) if (lo[i] < hi[i]) { any = true; __builtin_prefetch(buf.data() + (mb + i) * L + 1 + ((lo[i] + hi[i]) >> 1) * S + 5); }
                    if (!any) break;
                    for (int i = 0; i < g; ++i) if (lo[i] < hi[i]) {
                        const uint64_t mid = (lo[i] + hi[i]) >> 1;
                        const uint8_t* k = buf.data() + (mb + i) * L + 1 + mid * S + 5;
                        if (host_key_cmp(k, 32, (const uint8_t*)cut[p].data(), cut[p].size()) < 0) lo[i] = mid + 1; else hi[i] = mid;
                    }
                }
                for (int i = 0; i < g; ++i) bnd2[(mb + i) * 4 + p] = 1 + lo[i] * S;
            }
        }
    });
    for (auto& x : th2) x.join();
    t1 = std::chrono::steady_clock::now();
    printf("bsearch threads %d: %.1f ms\n", T, std::chrono::duration<double, std::milli>(t1 - t0).count());
    for (uint64_t m = 0; m < N; ++m) for (int p = 0; p < 3; ++p) if (bnd[m*4+p] != bnd2[m*4+p]) { printf("MISMATCH %llu %d\n", (unsigned long long)m, p); return 1; }
    printf("same\n");
}
// (appended) batched binary search variant
