/*
 * sanitize_main.c — drives the oracle restatement under ASan/UBSan (test infrastructure only,
 * tests/test_oracle_sanitize.py). Reads cases from a file:
 *   repeated { u32 n_streams; u64 max_run_size; u32 flags;
 *              n_streams x { i64 seq_no; u32 n_runs; n_runs x { u64 len; u8 bytes[len] } } }
 * and prints per case "rc <code> <fnv64 of output bytes and descriptors>" (or the error text's
 * hash), so the test can compare against the uninstrumented build.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "skv_oracle.h"

static uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    for (;;) {
        uint32_t n, flags;
        uint64_t max;
        if (!rd(f, &n, 4)) break;
        if (!rd(f, &max, 8) || !rd(f, &flags, 4)) return 3;
        skv_stream* st = (skv_stream*)calloc(n ? n : 1, sizeof(skv_stream));
        for (uint32_t i = 0; i < n; i++) {
            uint32_t nr;
            if (!rd(f, &st[i].seq_no, 8) || !rd(f, &nr, 4)) return 3;
            st[i].n_runs = nr;
            const uint8_t** runs = (const uint8_t**)calloc(nr ? nr : 1, sizeof(uint8_t*));
            uint64_t* lens = (uint64_t*)calloc(nr ? nr : 1, sizeof(uint64_t));
            for (uint32_t r = 0; r < nr; r++) {
                if (!rd(f, &lens[r], 8)) return 3;
                uint8_t* b = (uint8_t*)malloc(lens[r] ? lens[r] : 1);  /* exact-size: ASan sees overreads */
                if (lens[r] && !rd(f, b, lens[r])) return 3;
                runs[r] = b;
            }
            st[i].runs = runs;
            st[i].run_lens = lens;
        }
        skv_result* res = NULL;
        char eb[512] = {0};
        int rc = skvo_compact(st, n, max, flags, &res, eb, sizeof eb);
        uint64_t h = 0xcbf29ce484222325ull;
        if (rc == SKV_OK) {
            h = fnv(h, res->bytes, res->n_bytes);
            for (uint64_t i = 0; i < res->n_runs; i++) h = fnv(h, &res->runs[i], sizeof(skv_run_desc));
            skvo_result_free(res);
        } else {
            h = fnv(h, eb, strlen(eb));
        }
        printf("rc %d %016" PRIx64 "\n", rc, h);
        for (uint32_t i = 0; i < n; i++) {
            for (uint32_t r = 0; r < st[i].n_runs; r++) free((void*)st[i].runs[r]);
            free((void*)st[i].runs);
            free((void*)st[i].run_lens);
        }
        free(st);
    }
    fclose(f);
    return 0;
}
