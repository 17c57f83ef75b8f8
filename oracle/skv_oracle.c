/*
 * skv_oracle.c — CPU restatement of skyvault's compaction path. TEST INFRASTRUCTURE ONLY.
 *
 * This file restates, function by function, the reference algorithm of
 * dynoinc/skyvault-rs (Rust, reference snapshot 2026-04-24) that the MI355X path replaces.
 * It is the parity checker for libskv.so and the "port" CPU baseline timed by bench.py.
 * It is deliberately the *faithful* shape of the reference: a lazy per-record decoder
 * that allocates an owned key and value per record, a binary-heap k-way merge with one
 * head per stream, and a streaming encoder that clones keys as the reference does.
 *
 * Parity is pinned by the reference's own KATs (tests/golden/) and by an independent
 * Python restatement (tests/pyref.py). See skv_oracle.h.
 */
#include "skv_oracle.h"

#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* errors: Display text of RunError (runs.rs:83-95) and JobError::InvalidInput (mod.rs:26) */

static int fail(char* eb, size_t en, int code, const char* fmt, ...) {
    if (eb && en) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(eb, en, fmt, ap);
        va_end(ap);
    }
    return code;
}
#define E_EMPTY(eb, en) fail(eb, en, SKV_E_EMPTY_INPUT, "Input list of operations cannot be empty")
#define E_VERSION(eb, en, v) fail(eb, en, SKV_E_UNSUPPORTED_VERSION, "Unsupported run version: %u", (unsigned)(v))
#define E_EOF(eb, en) fail(eb, en, SKV_E_IO, "I/O error: failed to fill whole buffer")
#define E_FORMAT(eb, en, ...) fail(eb, en, SKV_E_FORMAT, "Data format error: " __VA_ARGS__)

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "skv_oracle: out of memory (%zu bytes)\n", n);
        abort();
    }
    return p;
}
static uint8_t* dup_bytes(const uint8_t* p, uint64_t n) {
    uint8_t* q = (uint8_t*)xmalloc((size_t)n);
    if (n) memcpy(q, p, (size_t)n);
    return q;
}
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

/* Rust str Ord: bytewise lexicographic, a proper prefix sorts first. */
static int key_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
    uint64_t n = al < bl ? al : bl;
    int c = n ? memcmp(a, b, (size_t)n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

/* core::str::from_utf8 validity (used by runs.rs:585). */
static int utf8_valid(const uint8_t* s, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint8_t c = s[i];
        if (c < 0x80) { i++; continue; }
        uint64_t need;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEC) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c >= 0xEE && c <= 0xEF) need = 2;
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return 0;
        if (n - i - 1 < need) return 0; /* truncated sequence */
        if (s[i + 1] < lo || s[i + 1] > hi) return 0;
        for (uint64_t k = 2; k <= need; k++)
            if (s[i + k] < 0x80 || s[i + k] > 0xBF) return 0;
        i += need + 1;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------ */
/* An owned WriteOperation (runs.rs:38-43): String key + Vec<u8> value, one allocation each,
 * as read_run_stream produces them (runs.rs:585-586, :613). */
typedef struct {
    uint32_t is_put;
    uint32_t klen;
    uint8_t* key;
    uint64_t vlen;
    uint8_t* val;
} oop;

static void oop_free(oop* o) {
    free(o->key);
    free(o->val);
    o->key = NULL;
    o->val = NULL;
}

/* ------------------------------------------------------------------------------------ */
/* runs::read_run_stream (runs.rs:517-628), one run, pulled lazily like the async stream.
 * Check order per record: marker (:561) -> key_len EOF (:570-576) -> key bounds (:580-583)
 * -> UTF-8 (:585-591) -> marker match: Put value_len EOF (:598-604), value bounds
 * (:608-611); Delete (:618-620); anything else "Invalid marker byte" (:621-624). */
typedef struct {
    const uint8_t* buf;
    uint64_t len;
    uint64_t pos;
    int started;
    int done;
    /* 1: runs::read_run_iter / RunIterator (runs.rs:400-510) instead of read_run_stream. Same
     * checks in the same order; the two EOF checks raise Format errors with their own text
     * ("Incomplete key length data" :428-430, "Incomplete value length data" :457-459) where
     * read_run_stream raises Io. Its "Unexpected end of data" (:421-423) and the two overflow
     * checks (:440-442, :469-471) cannot trigger (len == bytes.len(); u32 lengths on u64). */
    int iter;
} dec_t;

static void dec_init(dec_t* d, const uint8_t* buf, uint64_t len) {
    d->buf = buf;
    d->len = len;
    d->pos = 0;
    d->started = 0;
    d->done = 0;
    d->iter = 0;
}

/* 1 = op produced, 0 = end of run, <0 = -(error code) */
static int dec_next(dec_t* d, oop* o, char* eb, size_t en) {
    if (d->done) return 0;
    if (!d->started) {
        d->started = 1;
        if (d->len == 0) { d->done = 1; return -E_EMPTY(eb, en); }                 /* :537-540 */
        if (d->buf[0] != 1) { d->done = 1; return -E_VERSION(eb, en, d->buf[0]); } /* :553-556 */
        d->pos = 1;
    }
    if (d->pos >= d->len) { d->done = 1; return 0; } /* :559 */
    const uint8_t* b = d->buf;
    uint64_t len = d->len, p = d->pos;
    uint8_t marker = b[p];
    p += 1;
    if (p + 4 > len) {
        d->done = 1;
        return d->iter ? -E_FORMAT(eb, en, "Incomplete key length data") : -E_EOF(eb, en); /* :428-430 */
    }
    uint64_t klen = be32(b + p);
    p += 4;
    if (p + klen > len) { d->done = 1; return -E_FORMAT(eb, en, "Incomplete key data"); }
    if (!utf8_valid(b + p, klen)) { d->done = 1; return -E_FORMAT(eb, en, "Invalid UTF-8 in key"); }
    uint8_t* key = dup_bytes(b + p, klen); /* k.to_string() */
    p += klen;
    if (marker == 1) {
        if (p + 4 > len) {
            free(key);
            d->done = 1;
            return d->iter ? -E_FORMAT(eb, en, "Incomplete value length data") : -E_EOF(eb, en); /* :457-459 */
        }
        uint64_t vlen = be32(b + p);
        p += 4;
        if (p + vlen > len) { free(key); d->done = 1; return -E_FORMAT(eb, en, "Incomplete value data"); }
        o->is_put = 1;
        o->klen = (uint32_t)klen;
        o->key = key;
        o->vlen = vlen;
        o->val = dup_bytes(b + p, vlen); /* buffer[..].to_vec() */
        p += vlen;
    } else if (marker == 2) {
        o->is_put = 0;
        o->klen = (uint32_t)klen;
        o->key = key;
        o->vlen = 0;
        o->val = NULL;
    } else {
        free(key);
        d->done = 1;
        return -E_FORMAT(eb, en, "Invalid marker byte: %u", (unsigned)marker);
    }
    d->pos = p;
    return 1;
}

/* ------------------------------------------------------------------------------------ */
/* One merge input: a (SeqNo, stream) pair whose stream is the flatten of its member runs'
 * read_run_stream (table_buffer_compaction.rs:67-100, table_tree_compaction.rs:105-135).
 * The merge aborts on the first Err it pulls, so nothing past a member's error is read. */
typedef struct {
    const skv_stream* s;
    uint32_t member;
    dec_t dec;
    /* pre-decoded mode (skvo_merge_ops) */
    const skvo_op* ops;
    uint64_t n_ops, next_op;
    /* ScanFromRun's per-run filter (cache_service.rs:125-129): try_filter(op.key() > start) drops
     * Ok items with key <= start and passes errors through */
    const uint8_t* gt_key;
    uint64_t gt_len;
    int filter;
} sit_t;

static int sit_next(sit_t* it, oop* o, char* eb, size_t en) {
    if (it->ops || !it->s) {
        if (it->next_op >= it->n_ops) return 0;
        const skvo_op* src = &it->ops[it->next_op++];
        o->is_put = src->is_put;
        o->klen = src->key_len;
        o->key = dup_bytes(src->key, src->key_len);
        o->vlen = src->is_put ? src->val_len : 0;
        o->val = src->is_put ? dup_bytes(src->val, src->val_len) : NULL;
        return 1;
    }
    while (it->member < it->s->n_runs) {
        int r = dec_next(&it->dec, o, eb, en);
        if (r == 1 && it->filter && key_cmp(o->key, o->klen, it->gt_key, it->gt_len) <= 0) {
            oop_free(o);
            continue;
        }
        if (r != 0) return r;
        it->member++;
        if (it->member < it->s->n_runs)
            dec_init(&it->dec, it->s->runs[it->member], it->s->run_lens[it->member]);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* k_way::HeapItem ordering (k_way.rs:20-27): different keys -> reversed key order (the
 * smallest key is the heap maximum); equal keys -> seq_no order (the newest is the max). */
typedef struct {
    oop op;
    int64_t seq;
    uint32_t slot;
} hitem;

static int hitem_cmp(const hitem* a, const hitem* b) {
    int c = key_cmp(a->op.key, a->op.klen, b->op.key, b->op.klen);
    if (c) return -c;
    return a->seq < b->seq ? -1 : (a->seq > b->seq ? 1 : 0);
}

typedef struct {
    hitem* v;
    uint32_t n;
} heap_t;

static void heap_push(heap_t* h, hitem x) {
    uint32_t i = h->n++;
    h->v[i] = x;
    while (i) {
        uint32_t p = (i - 1) / 2;
        if (hitem_cmp(&h->v[i], &h->v[p]) <= 0) break;
        hitem t = h->v[i]; h->v[i] = h->v[p]; h->v[p] = t;
        i = p;
    }
}
static hitem heap_pop(heap_t* h) {
    hitem top = h->v[0];
    h->v[0] = h->v[--h->n];
    uint32_t i = 0;
    for (;;) {
        uint32_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && hitem_cmp(&h->v[l], &h->v[m]) > 0) m = l;
        if (r < h->n && hitem_cmp(&h->v[r], &h->v[m]) > 0) m = r;
        if (m == i) break;
        hitem t = h->v[i]; h->v[i] = h->v[m]; h->v[m] = t;
        i = m;
    }
    return top;
}

/* ------------------------------------------------------------------------------------ */
/* Growable output: the bytes of every finished run plus their descriptors. */
typedef struct {
    uint8_t* b;
    uint64_t n, cap;
    skv_run_desc* runs;
    uint64_t n_runs, runs_cap;
    uint64_t out_records;
} outbuf;

static void ob_reserve(outbuf* o, uint64_t extra) {
    if (o->n + extra <= o->cap) return;
    uint64_t c = o->cap ? o->cap : 64;
    while (c < o->n + extra) c *= 2;
    uint8_t* nb = (uint8_t*)realloc(o->b, (size_t)c);
    if (!nb) { fprintf(stderr, "skv_oracle: out of memory\n"); abort(); }
    o->b = nb;
    o->cap = c;
}
static void ob_push_run(outbuf* o, const skv_run_desc* d) {
    if (o->n_runs == o->runs_cap) {
        o->runs_cap = o->runs_cap ? 2 * o->runs_cap : 16;
        skv_run_desc* nr = (skv_run_desc*)realloc(o->runs, (size_t)o->runs_cap * sizeof(skv_run_desc));
        if (!nr) abort();
        o->runs = nr;
    }
    o->runs[o->n_runs++] = *d;
}

/* runs::build_runs (runs.rs:166-282) as a push-driven state machine. The run being built is
 * the tail of the output buffer starting at run_off. */
typedef struct {
    outbuf* out;        /* where finished runs go */
    outbuf local;       /* WAL mode: private buffer of one table's build task */
    int use_local;
    uint64_t max;
    int have_last;
    uint8_t* last_key;  /* last_key: Option<String> (:177) */
    uint64_t last_klen;
    uint8_t* min_key;   /* min_key (:171) */
    uint8_t* max_key;   /* max_key (:172) */
    int first_op_in_run;
    uint64_t cur_size, put_count, delete_count;
    uint64_t run_off, max_key_off, max_klen, min_key_off, min_klen;
    uint64_t records;
    uint64_t base;      /* bytes already drained from the output (skvo_sb_*); 0 otherwise */
} builder;

static void bld_init(builder* b, outbuf* out, uint64_t max) {
    memset(b, 0, sizeof(*b));
    b->out = out;
    b->max = max;
    b->first_op_in_run = 1;
}
static outbuf* bld_buf(builder* b) { return b->use_local ? &b->local : b->out; }

static void bld_finish_run(builder* b, int64_t table_id) {
    skv_run_desc d;
    memset(&d, 0, sizeof(d));
    d.off = b->run_off;
    d.len = b->cur_size;
    d.put_count = b->put_count;
    d.delete_count = b->delete_count;
    d.min_key_off = b->min_key_off;
    d.min_key_len = b->min_klen;
    d.max_key_off = b->max_key_off;
    d.max_key_len = b->max_klen;
    d.table_id = table_id;
    ob_push_run(bld_buf(b), &d);
    free(b->min_key);
    free(b->max_key);
    b->min_key = b->max_key = NULL;
}

/* one loop iteration of runs.rs:180-267; returns SKV_OK or the order error */
static int bld_push(builder* b, const oop* op, char* eb, size_t en) {
    uint8_t* current_key = dup_bytes(op->key, op->klen); /* :188 */
    if (b->have_last && key_cmp(current_key, op->klen, b->last_key, b->last_klen) <= 0) { /* :191-198 */
        free(current_key);
        return E_FORMAT(eb, en, "Operations must be sorted by key");
    }
    free(b->last_key);
    b->last_key = dup_bytes(current_key, op->klen); /* :199 */
    b->last_klen = op->klen;
    b->have_last = 1;

    uint64_t op_size = op->is_put ? 1 + 4 + (uint64_t)op->klen + 4 + op->vlen : 1 + 4 + (uint64_t)op->klen; /* :202-209 */
    uint64_t size_with_op = b->first_op_in_run ? b->cur_size + 1 + op_size : b->cur_size + op_size; /* :212-216 */
    if (!b->first_op_in_run && size_with_op > b->max) { /* :219-238 */
        bld_finish_run(b, 0);
        b->cur_size = 0;
        b->put_count = 0;
        b->delete_count = 0;
        b->first_op_in_run = 1;
    }
    outbuf* o = bld_buf(b);
    if (b->first_op_in_run) { /* :241-246 */
        ob_reserve(o, 1);
        b->run_off = b->base + o->n;
        o->b[o->n++] = 1; /* CURRENT_VERSION */
        b->cur_size += 1;
        b->min_key = dup_bytes(current_key, op->klen);
        b->min_key_off = b->base + o->n + 5;
        b->min_klen = op->klen;
        b->first_op_in_run = 0;
    }
    free(b->max_key);
    b->max_key = dup_bytes(current_key, op->klen); /* :248 */
    b->max_key_off = b->base + o->n + 5;
    b->max_klen = op->klen;
    b->cur_size += op_size; /* :249 */
    ob_reserve(o, op_size); /* :252-267 */
    uint8_t* w = o->b + o->n;
    w[0] = op->is_put ? 1 : 2;
    put_be32(w + 1, op->klen);
    if (op->klen) memcpy(w + 5, op->key, op->klen);
    if (op->is_put) {
        put_be32(w + 5 + op->klen, (uint32_t)op->vlen);
        if (op->vlen) memcpy(w + 9 + op->klen, op->val, (size_t)op->vlen);
        b->put_count++;
    } else {
        b->delete_count++;
    }
    o->n += op_size;
    o->out_records++;
    b->records++;
    free(current_key);
    return SKV_OK;
}

/* end of stream (runs.rs:270-280) */
static void bld_end(builder* b, int64_t table_id) {
    if (b->put_count > 0 || b->delete_count > 0) bld_finish_run(b, table_id);
}
static void bld_free(builder* b) {
    free(b->last_key);
    free(b->min_key);
    free(b->max_key);
    free(b->local.b);
    free(b->local.runs);
}

/* ------------------------------------------------------------------------------------ */
/* Rust `str::parse::<i64>()` (core::num from_str_radix): Empty, then optional sign (a lone
 * sign is InvalidDigit), then per digit: InvalidDigit before the checked mul/add overflow. */
static int parse_i64(const uint8_t* s, uint64_t n, int64_t* out, const char** err) {
    if (n == 0) { *err = "cannot parse integer from empty string"; return 0; }
    int neg = 0;
    uint64_t i = 0;
    if (s[0] == '+' || s[0] == '-') {
        if (n == 1) { *err = "invalid digit found in string"; return 0; }
        neg = s[0] == '-';
        i = 1;
    }
    int64_t r = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') { *err = "invalid digit found in string"; return 0; }
        int64_t d = s[i] - '0', m;
        if (__builtin_mul_overflow(r, (int64_t)10, &m) ||
            (neg ? __builtin_sub_overflow(m, d, &r) : __builtin_add_overflow(m, d, &r))) {
            *err = neg ? "number too small to fit in target type" : "number too large to fit in target type";
            return 0;
        }
    }
    *out = r;
    return 1;
}

/* WAL split consumer (wal_compaction.rs:66-174). One builder per table in order of
 * appearance; a failing build (order error, or != 1 run) is swallowed by `if let Ok`
 * (:103, :168) and that table's data is dropped. */
typedef struct {
    outbuf* out;
    uint64_t max;
    int have_table;
    int64_t table;
    builder cur;
    int cur_failed;
    uint64_t after_fail; /* ops sent to the table after its build_runs failed */
    uint64_t dropped;
} walc;

/* mpsc::channel(100) per table task (wal_compaction.rs:113). A task whose build_runs fails on an
 * order error drops its receiver; the job's 101st send after the failing op cannot be buffered
 * and fails with "Failed to send operation to table channel" (:157-161). Sends 1..100 after it
 * race with the task's exit; they are modelled as buffered (the task is slow). */
#define WAL_SENDS_AFTER_FAIL 101

static void wal_finish(walc* w) {
    if (!w->have_table) return;
    builder* b = &w->cur;
    if (!w->cur_failed) bld_end(b, w->table);
    /* build_runs(...).try_collect() then results.len() != 1 -> Err (:126-137) */
    if (w->cur_failed || b->local.n_runs != 1) {
        w->dropped++;
    } else {
        skv_run_desc d = b->local.runs[0];
        ob_reserve(w->out, d.len);
        uint64_t base = w->out->n;
        memcpy(w->out->b + base, b->local.b + d.off, (size_t)d.len);
        w->out->n += d.len;
        w->out->out_records += b->records;
        d.min_key_off = d.min_key_off - d.off + base;
        d.max_key_off = d.max_key_off - d.off + base;
        d.off = base;
        d.table_id = w->table;
        ob_push_run(w->out, &d);
    }
    bld_free(b);
    w->have_table = 0;
}

static int wal_push(walc* w, oop* op, char* eb, size_t en) {
    uint64_t dot = 0;
    while (dot < op->klen && op->key[dot] != '.') dot++;
    if (dot == op->klen) /* :71-73 */
        return fail(eb, en, SKV_E_INVALID_INPUT, "Invalid input: Key does not follow 'table_id.key' format: %.*s",
                    (int)op->klen, (const char*)op->key);
    int64_t id = 0;
    const char* perr = NULL;
    if (!parse_i64(op->key, dot, &id, &perr)) /* :75-79 */
        return fail(eb, en, SKV_E_INVALID_INPUT, "Invalid input: Invalid table ID '%.*s': %s", (int)dot,
                    (const char*)op->key, perr);
    char tmp[32];
    uint64_t strip = (uint64_t)snprintf(tmp, sizeof tmp, "%" PRId64 ".", id); /* :81 */
    if (!w->have_table || w->table != id) { /* :82-86, :96-123 */
        wal_finish(w);
        w->have_table = 1;
        w->table = id;
        w->cur_failed = 0;
        w->after_fail = 0;
        bld_init(&w->cur, w->out, w->max);
        w->cur.use_local = 1;
    }
    if (w->cur_failed) {
        if (++w->after_fail == WAL_SENDS_AFTER_FAIL)
            return fail(eb, en, SKV_E_INTERNAL, "Internal error: Failed to send operation to table channel");
        return SKV_OK;
    }
    oop s = *op; /* key.split_off(table_prefix_len) (:91-94) */
    s.key = op->key + strip;
    s.klen = op->klen - (uint32_t)strip;
    char e2[256];
    if (bld_push(&w->cur, &s, e2, sizeof e2) != SKV_OK) w->cur_failed = 1;
    return SKV_OK;
}

/* ------------------------------------------------------------------------------------ */
#define SCAN_STOP 1000 /* the scan's reader stopped reading: not an error, and nothing later is seen */
typedef struct {
    uint32_t flags;
    builder bld;
    walc wal;
    /* ScanFromRun's reader (cache_service.rs:137-148): every merged op goes into the response (one
     * v1 run of records here), Puts are counted, and the reader stops after the max_results-th */
    int scan;
    uint64_t scan_max, scan_puts;
    outbuf* scan_out;
    skv_run_desc scan_desc;
    /* skvo_merge_ops collection */
    int collect;
    skvo_op* col;
    uint64_t n_col, cap_col;
    uint8_t** col_bufs;
} consumer;

/* What receives each op the merge emits: the Delete filter (table_tree_compaction.rs:139-145)
 * and build_runs, or the WAL split loop. Takes ownership of op. */
static int consume(consumer* c, oop* op, char* eb, size_t en) {
    int rc = SKV_OK;
    if (c->collect) {
        if (c->n_col == c->cap_col) {
            c->cap_col = c->cap_col ? 2 * c->cap_col : 64;
            c->col = (skvo_op*)realloc(c->col, (size_t)c->cap_col * sizeof(skvo_op));
            c->col_bufs = (uint8_t**)realloc(c->col_bufs, (size_t)c->cap_col * 2 * sizeof(uint8_t*));
        }
        skvo_op* d = &c->col[c->n_col];
        d->is_put = op->is_put;
        d->key_len = op->klen;
        d->key = op->key;
        d->val_len = op->vlen;
        d->val = op->val;
        c->col_bufs[2 * c->n_col] = op->key;
        c->col_bufs[2 * c->n_col + 1] = op->val;
        c->n_col++;
        return SKV_OK; /* ownership moved */
    }
    if (c->scan) {
        outbuf* o = c->scan_out;
        const uint64_t sz = op->is_put ? 1 + 4 + (uint64_t)op->klen + 4 + op->vlen : 1 + 4 + (uint64_t)op->klen;
        ob_reserve(o, (o->n ? 0 : 1) + sz);
        if (!o->n) o->b[o->n++] = 1; /* the response as one v1 run: version byte first */
        skv_run_desc* d = &c->scan_desc;
        if (!d->put_count && !d->delete_count) {
            d->min_key_off = o->n + 5;
            d->min_key_len = op->klen;
        }
        d->max_key_off = o->n + 5;
        d->max_key_len = op->klen;
        uint8_t* w = o->b + o->n;
        w[0] = op->is_put ? 1 : 2;
        put_be32(w + 1, op->klen);
        memcpy(w + 5, op->key, op->klen);
        if (op->is_put) {
            put_be32(w + 5 + op->klen, (uint32_t)op->vlen);
            if (op->vlen) memcpy(w + 9 + op->klen, op->val, (size_t)op->vlen);
            d->put_count++;
            c->scan_puts++; /* :143 counts Puts only */
        } else {
            d->delete_count++;
        }
        o->n += sz;
        oop_free(op);
        return c->scan_puts >= c->scan_max ? SCAN_STOP : SKV_OK; /* :145-147 */
    }
    if (c->flags & SKV_SPLIT_BY_TABLE) {
        rc = wal_push(&c->wal, op, eb, en);
    } else if ((c->flags & SKV_DROP_TOMBSTONES) && !op->is_put) {
        rc = SKV_OK;
    } else {
        rc = bld_push(&c->bld, op, eb, en);
    }
    oop_free(op);
    return rc;
}

/* k_way::merge (k_way.rs:113-179) driving the consumer synchronously: the channel between
 * the merge task and its reader preserves order, so "first error in channel order" is the
 * first error either side raises in this loop. */
static int run_merge(sit_t* its, const int64_t* seqs, uint32_t n, consumer* c, char* eb, size_t en) {
    heap_t h;
    h.v = (hitem*)xmalloc((size_t)(n ? n : 1) * sizeof(hitem));
    h.n = 0;
    int rc = SKV_OK;
    for (uint32_t i = 0; i < n && rc == SKV_OK; i++) { /* :126-140, vector order */
        oop o;
        int r = sit_next(&its[i], &o, eb, en);
        if (r == 1) {
            hitem x = {o, seqs[i], i};
            heap_push(&h, x);
        } else if (r < 0) {
            rc = -r; /* first item Err: send and stop (:134-137) */
        }
    }
    uint8_t* last_key = NULL;
    uint64_t last_klen = 0;
    int have_last = 0;
    while (rc == SKV_OK && h.n) { /* :144-172 */
        hitem it = heap_pop(&h);
        uint32_t slot = it.slot;
        int64_t seq = it.seq;
        if (!have_last || key_cmp(it.op.key, it.op.klen, last_key, last_klen) != 0) { /* :146-151 */
            free(last_key);
            last_key = dup_bytes(it.op.key, it.op.klen);
            last_klen = it.op.klen;
            have_last = 1;
            rc = consume(c, &it.op, eb, en);
            if (rc != SKV_OK) break; /* an error, or SCAN_STOP: no refill is ever read */
        } else {
            oop_free(&it.op);
        }
        oop o; /* refill from the same stream (:154-171) */
        int r = sit_next(&its[slot], &o, eb, en);
        if (r == 1) {
            hitem x = {o, seq, slot};
            heap_push(&h, x);
        } else if (r < 0) {
            rc = -r;
        }
    }
    while (h.n) {
        hitem it = heap_pop(&h);
        oop_free(&it.op);
    }
    free(h.v);
    free(last_key);
    return rc;
}

typedef struct {
    int64_t seq;
    uint32_t idx;
} seq_idx;
static int seq_idx_cmp(const void* a, const void* b) {
    const seq_idx* x = (const seq_idx*)a;
    const seq_idx* y = (const seq_idx*)b;
    if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx ? 1 : 0);
}

/* API checks. Duplicate seq_nos (k_way.rs:121 keys streams by SeqNo) are found by sorting
 * (seq, index): the reported pair is the first stream i with an earlier duplicate, and that
 * duplicate's first occurrence j. */
static int check_streams(const skv_stream* streams, uint32_t n, char* eb, size_t en) {
    if (n && !streams) return fail(eb, en, SKV_E_INVALID_ARG, "streams is NULL");
    for (uint32_t i = 0; i < n; i++) {
        if (streams[i].n_runs && (!streams[i].runs || !streams[i].run_lens))
            return fail(eb, en, SKV_E_INVALID_ARG, "stream %u: runs/run_lens is NULL", i);
        for (uint32_t r = 0; r < streams[i].n_runs; r++)
            if (streams[i].run_lens[r] && !streams[i].runs[r])
                return fail(eb, en, SKV_E_INVALID_ARG, "stream %u run %u: NULL data", i, r);
    }
    if (n < 2) return SKV_OK;
    seq_idx* v = (seq_idx*)xmalloc((size_t)n * sizeof(seq_idx));
    for (uint32_t i = 0; i < n; i++) {
        v[i].seq = streams[i].seq_no;
        v[i].idx = i;
    }
    qsort(v, n, sizeof(seq_idx), seq_idx_cmp);
    uint32_t best_i = UINT32_MAX, best_j = 0;
    for (uint32_t a = 1; a < n; a++)
        if (v[a].seq == v[a - 1].seq && (a < 2 || v[a - 2].seq != v[a].seq) && v[a].idx < best_i) {
            best_i = v[a].idx;     /* the group's second occurrence */
            best_j = v[a - 1].idx; /* its first */
        }
    free(v);
    if (best_i != UINT32_MAX)
        return fail(eb, en, SKV_E_INVALID_ARG, "duplicate seq_no %" PRId64 " (streams %u and %u)",
                    streams[best_i].seq_no, best_j, best_i);
    return SKV_OK;
}

static skv_result* finish_result(outbuf* o) {
    skv_result* r = (skv_result*)calloc(1, sizeof(skv_result));
    r->bytes = o->b;
    r->n_bytes = o->n;
    r->runs = o->runs;
    r->n_runs = o->n_runs;
    r->out_records = o->out_records;
    return r;
}

int skvo_compact(const skv_stream* streams, uint32_t n, uint64_t max_run_size, uint32_t flags, skv_result** out,
                 char* eb, size_t en) {
    if (!out) return fail(eb, en, SKV_E_INVALID_ARG, "out is NULL");
    *out = NULL;
    int rc = check_streams(streams, n, eb, en);
    if (rc) return rc;
    if ((flags & SKV_SPLIT_BY_TABLE) && (flags & SKV_DROP_TOMBSTONES))
        return fail(eb, en, SKV_E_INVALID_ARG, "SKV_SPLIT_BY_TABLE and SKV_DROP_TOMBSTONES are exclusive");
    sit_t* its = (sit_t*)calloc(n ? n : 1, sizeof(sit_t));
    int64_t* seqs = (int64_t*)xmalloc((size_t)(n ? n : 1) * sizeof(int64_t));
    uint64_t in_bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        its[i].s = &streams[i];
        its[i].member = 0;
        if (streams[i].n_runs) dec_init(&its[i].dec, streams[i].runs[0], streams[i].run_lens[0]);
        seqs[i] = streams[i].seq_no;
        for (uint32_t r = 0; r < streams[i].n_runs; r++) in_bytes += streams[i].run_lens[r];
    }
    outbuf ob;
    memset(&ob, 0, sizeof ob);
    consumer c;
    memset(&c, 0, sizeof c);
    c.flags = flags;
    bld_init(&c.bld, &ob, max_run_size);
    c.wal.out = &ob;
    c.wal.max = max_run_size;
    rc = run_merge(its, seqs, n, &c, eb, en);
    if (rc == SKV_OK) {
        if (flags & SKV_SPLIT_BY_TABLE) wal_finish(&c.wal);
        else bld_end(&c.bld, 0);
    } else if (flags & SKV_SPLIT_BY_TABLE) {
        if (c.wal.have_table) bld_free(&c.wal.cur);
    }
    uint64_t dropped = c.wal.dropped;
    bld_free(&c.bld);
    free(its);
    free(seqs);
    if (rc != SKV_OK) {
        free(ob.b);
        free(ob.runs);
        return rc;
    }
    skv_result* r = finish_result(&ob);
    r->in_bytes = in_bytes;
    r->dropped_tables = dropped;
    *out = r;
    return SKV_OK;
}

/* cache_service.rs:97-151 ScanFromRun over runs already fetched: max_results in 1..=10000
 * (:101-104), run i decoded by read_run_iter (runs.rs:493-510) at SeqNo i64::MAX - i (:113-115),
 * filtered to key > exclusive_start_key (:125-129), k_way::merge (:134), read until the
 * max_results-th Put (:140-148). The response items are returned as one v1 run (records in
 * response order) with its StatsV1, or no run when there is no item. A merge error the reader
 * reaches is returned as the RunError (the service wraps it: "Merge stream error: {e}", :141). */
int skvo_scan_runs(const uint8_t* const* runs, const uint64_t* lens, uint32_t n, const uint8_t* start,
                   uint64_t start_len, uint64_t max_results, skv_result** out, char* eb, size_t en) {
    if (!out) return fail(eb, en, SKV_E_INVALID_ARG, "out is NULL");
    *out = NULL;
    if (max_results < 1 || max_results > 10000)
        return fail(eb, en, SKV_E_INVALID_ARG, "max_results must be between 1 and 10000");
    if (n && (!runs || !lens)) return fail(eb, en, SKV_E_INVALID_ARG, "runs/lens is NULL");
    if (start_len && !start) return fail(eb, en, SKV_E_INVALID_ARG, "start key is NULL");
    skv_stream* st = (skv_stream*)calloc(n ? n : 1, sizeof(skv_stream));
    sit_t* its = (sit_t*)calloc(n ? n : 1, sizeof(sit_t));
    int64_t* seqs = (int64_t*)xmalloc((size_t)(n ? n : 1) * sizeof(int64_t));
    uint64_t in_bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        st[i].runs = &runs[i];
        st[i].run_lens = &lens[i];
        st[i].n_runs = 1;
        st[i].seq_no = INT64_MAX - (int64_t)i;
        its[i].s = &st[i];
        dec_init(&its[i].dec, runs[i], lens[i]);
        its[i].dec.iter = 1;
        its[i].filter = 1;
        its[i].gt_key = start;
        its[i].gt_len = start_len;
        seqs[i] = st[i].seq_no;
        in_bytes += lens[i];
    }
    outbuf ob;
    memset(&ob, 0, sizeof ob);
    consumer c;
    memset(&c, 0, sizeof c);
    c.scan = 1;
    c.scan_max = max_results;
    c.scan_out = &ob;
    int rc = run_merge(its, seqs, n, &c, eb, en);
    if (rc == SCAN_STOP) rc = SKV_OK;
    free(its);
    free(seqs);
    free(st);
    if (rc != SKV_OK) {
        free(ob.b);
        free(ob.runs);
        return rc;
    }
    if (ob.n) {
        c.scan_desc.off = 0;
        c.scan_desc.len = ob.n;
        ob_push_run(&ob, &c.scan_desc);
        ob.out_records = c.scan_desc.put_count + c.scan_desc.delete_count;
    }
    skv_result* r = finish_result(&ob);
    r->in_bytes = in_bytes;
    *out = r;
    return SKV_OK;
}

int skvo_build_runs(const skvo_op* ops, uint64_t n, uint64_t max_run_size, skv_result** out, char* eb, size_t en) {
    if (!out) return fail(eb, en, SKV_E_INVALID_ARG, "out is NULL");
    *out = NULL;
    outbuf ob;
    memset(&ob, 0, sizeof ob);
    builder b;
    bld_init(&b, &ob, max_run_size);
    int rc = SKV_OK;
    for (uint64_t i = 0; i < n && rc == SKV_OK; i++) {
        oop o = {ops[i].is_put, ops[i].key_len, (uint8_t*)ops[i].key, ops[i].is_put ? ops[i].val_len : 0,
                 (uint8_t*)ops[i].val};
        rc = bld_push(&b, &o, eb, en);
    }
    if (rc == SKV_OK) bld_end(&b, 0);
    bld_free(&b);
    if (rc != SKV_OK) {
        free(ob.b);
        free(ob.runs);
        return rc;
    }
    *out = finish_result(&ob);
    return SKV_OK;
}

int skvo_merge_ops(const skvo_op* const* ops, const uint64_t* n_ops, const int64_t* seq_nos, uint32_t n,
                   skvo_op_list** out, char* eb, size_t en) {
    if (!out) return fail(eb, en, SKV_E_INVALID_ARG, "out is NULL");
    *out = NULL;
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t j = 0; j < i; j++)
            if (seq_nos[i] == seq_nos[j]) return fail(eb, en, SKV_E_INVALID_ARG, "duplicate seq_no");
    sit_t* its = (sit_t*)calloc(n ? n : 1, sizeof(sit_t));
    for (uint32_t i = 0; i < n; i++) {
        its[i].ops = ops[i];
        its[i].n_ops = n_ops[i];
    }
    consumer c;
    memset(&c, 0, sizeof c);
    c.collect = 1;
    int rc = run_merge(its, seq_nos, n, &c, eb, en);
    free(its);
    /* pack into one arena */
    uint64_t total = 0;
    for (uint64_t i = 0; i < c.n_col; i++) total += c.col[i].key_len + c.col[i].val_len;
    skvo_op_list* l = (skvo_op_list*)calloc(1, sizeof(skvo_op_list));
    l->ops = (skvo_op*)xmalloc((size_t)(c.n_col ? c.n_col : 1) * sizeof(skvo_op));
    l->arena = (uint8_t*)xmalloc((size_t)total);
    l->n_ops = c.n_col;
    uint64_t p = 0;
    for (uint64_t i = 0; i < c.n_col; i++) {
        skvo_op d = c.col[i];
        memcpy(l->arena + p, d.key, d.key_len);
        d.key = l->arena + p;
        p += d.key_len;
        if (d.is_put) {
            if (d.val_len) memcpy(l->arena + p, d.val, (size_t)d.val_len);
            d.val = l->arena + p;
            p += d.val_len;
        } else {
            d.val = NULL;
        }
        l->ops[i] = d;
        free(c.col_bufs[2 * i]);
        free(c.col_bufs[2 * i + 1]);
    }
    free(c.col);
    free(c.col_bufs);
    *out = l;
    return rc;
}

int skvo_decode_run(const uint8_t* run, uint64_t len, skvo_op_list** out, char* eb, size_t en) {
    if (!out) return fail(eb, en, SKV_E_INVALID_ARG, "out is NULL");
    dec_t d;
    dec_init(&d, run, len);
    skvo_op_list* l = (skvo_op_list*)calloc(1, sizeof(skvo_op_list));
    uint64_t cap = 16;
    l->ops = (skvo_op*)xmalloc(cap * sizeof(skvo_op));
    l->arena = (uint8_t*)xmalloc((size_t)(len ? len : 1));
    uint64_t ap = 0;
    int rc = SKV_OK;
    for (;;) {
        oop o;
        int r = dec_next(&d, &o, eb, en);
        if (r == 0) break;
        if (r < 0) { rc = -r; break; }
        if (l->n_ops == cap) {
            cap *= 2;
            l->ops = (skvo_op*)realloc(l->ops, cap * sizeof(skvo_op));
        }
        skvo_op* e = &l->ops[l->n_ops++];
        e->is_put = o.is_put;
        e->key_len = o.klen;
        memcpy(l->arena + ap, o.key, o.klen);
        e->key = l->arena + ap;
        ap += o.klen;
        e->val_len = o.vlen;
        if (o.is_put) {
            memcpy(l->arena + ap, o.val, (size_t)o.vlen);
            e->val = l->arena + ap;
            ap += o.vlen;
        } else {
            e->val = NULL;
        }
        oop_free(&o);
    }
    *out = l;
    return rc;
}

void skvo_op_list_free(skvo_op_list* l) {
    if (!l) return;
    free(l->ops);
    free(l->arena);
    free(l);
}

void skvo_result_free(skv_result* r) {
    if (!r) return;
    free(r->bytes);
    free(r->runs);
    free(r);
}

/* ------------------------------------------------------------------------------------ */
/* Streaming build_runs (runs.rs:166-282) for full-size checks: the merged op sequence arrives
 * as a series of v1 runs (e.g. the per-key-range outputs of skvo_compact with an unbounded
 * max), each decoded with read_run_stream (runs.rs:517-628) and pushed through ONE builder,
 * so the greedy split and the order check carry across the pieces. Output bytes are drained
 * as they are produced; descriptor offsets stay absolute. */
struct skvo_sb {
    outbuf ob;
    builder b;
    int failed;
    int finished;
};

skvo_sb* skvo_sb_new(uint64_t max_run_size) {
    skvo_sb* s = (skvo_sb*)calloc(1, sizeof(skvo_sb));
    bld_init(&s->b, &s->ob, max_run_size);
    return s;
}

int skvo_sb_feed_run(skvo_sb* s, const uint8_t* run, uint64_t len, char* eb, size_t en) {
    if (s->failed) return fail(eb, en, SKV_E_INVALID_ARG, "builder already failed");
    dec_t d;
    dec_init(&d, run, len);
    for (;;) {
        oop o;
        int r = dec_next(&d, &o, eb, en);
        if (r == 0) return SKV_OK;
        if (r < 0) { s->failed = 1; return -r; }
        int rc = bld_push(&s->b, &o, eb, en);
        oop_free(&o);
        if (rc != SKV_OK) { s->failed = 1; return rc; }
    }
}

uint64_t skvo_sb_pending(const skvo_sb* s) { return s->ob.n; }

void skvo_sb_drain(skvo_sb* s, uint8_t* dst) {
    if (s->ob.n && dst) memcpy(dst, s->ob.b, (size_t)s->ob.n);
    s->b.base += s->ob.n;
    s->ob.n = 0;
}

int skvo_sb_finish(skvo_sb* s, skv_result** out) {
    if (s->failed) return SKV_E_INVALID_ARG;
    bld_end(&s->b, 0);
    bld_free(&s->b);
    s->finished = 1;
    skv_result* r = (skv_result*)calloc(1, sizeof(skv_result));
    r->bytes = s->ob.b;           /* the undrained tail */
    r->n_bytes = s->ob.n;
    r->runs = s->ob.runs;
    r->n_runs = s->ob.n_runs;
    r->out_records = s->ob.out_records;
    r->in_bytes = s->b.base;      /* bytes drained before the tail */
    s->ob.b = NULL;
    s->ob.runs = NULL;
    *out = r;
    return SKV_OK;
}

void skvo_sb_free(skvo_sb* s) {
    if (!s) return;
    if (!s->finished) bld_free(&s->b);
    free(s->ob.b);
    free(s->ob.runs);
    free(s);
}
