/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see pj_oracle.h for who may use it and
 * how parity is pinned). Plain C restatement of
 * /root/reference/ParallelJohnson.cpp; every function cites the lines it
 * follows. No reference source is copied: the algorithm is re-expressed.
 */
#define _GNU_SOURCE
#include "pj_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* Parsing: read_webgraph :66-105                                            */
/* ------------------------------------------------------------------------ */

/* C-locale isspace minus '\n' (getline already split on it). */
static int is_ws(unsigned char c) {
    return c == ' ' || c == '\t' || c == '\v' || c == '\f' || c == '\r';
}
static int is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

#define ID_LIMIT 2147483646LL /* N = max+1 must fit the reference's int (:288, :319) */

/* One `iss >> int` extraction (:93) starting at p, line ends at e.
 * Returns 1 = value read, 0 = extraction failed on a non-space char (the
 * stream stores 0, C++11 num_get), -1 = only whitespace left (sentry fails,
 * the target is left unmodified -> reference UB), -2 = overflow. */
static int extract_int(const unsigned char** pp, const unsigned char* e, int64_t* out) {
    const unsigned char* p = *pp;
    while (p < e && is_ws(*p)) p++;
    if (p == e) { *pp = p; return -1; }
    int neg = 0;
    if (*p == '+' || *p == '-') { neg = (*p == '-'); p++; }
    if (p == e || !is_digit(*p)) { *out = 0; *pp = p; return 0; }
    int64_t acc = 0;
    int ovf = 0;
    while (p < e && is_digit(*p)) {
        acc = acc * 10 + (*p - '0');
        if (acc > 4294967295LL) { ovf = 1; acc = 4294967295LL; }
        p++;
    }
    *pp = p;
    if (ovf) return -2;
    *out = neg ? -acc : acc;
    return 1;
}

int pjo_parse_snap(const char* buf, int64_t len, int weighted, uint32_t* src, uint32_t* dst,
                   uint32_t* w, int64_t cap, int64_t* nnz_out, int64_t* max_id_out,
                   int64_t* bad_line) {
    const unsigned char* b = (const unsigned char*)buf;
    int64_t nnz = 0, max_id = -1, line = 0;
    int64_t pos = 0;
    *bad_line = 0;
    while (pos < len) {
        /* getline (:71/:89): one line = bytes up to '\n' (exclusive). */
        const unsigned char* s = b + pos;
        const unsigned char* nl = memchr(s, '\n', (size_t)(len - pos));
        const unsigned char* e = nl ? nl : b + len;
        pos = (e - b) + 1;
        line++;
        /* :73 / :91 — an edge line iff byte 0 is a decimal digit. */
        if (e == s || !is_digit(*s)) continue;
        const unsigned char* p = s;
        int64_t u = 0, v = 0, wt = 1;
        int r = extract_int(&p, e, &u); /* first byte is a digit: r is 1 or -2 */
        if (r != 1 || u > ID_LIMIT) { *bad_line = line; return -3; }
        r = extract_int(&p, e, &v);
        if (r < 0 || v < 0 || v > ID_LIMIT) { *bad_line = line; return -3; }
        if (weighted) {
            /* extension: third column = weight, same extraction rules; a
             * failed extraction stops the stream (:93 semantics) -> 0. */
            if (r == 0) wt = 0;
            else {
                r = extract_int(&p, e, &wt);
                if (r < 0 || wt < 0) { *bad_line = line; return -3; }
            }
        }
        if (src) {
            if (nnz >= cap) { *bad_line = line; return -1; }
            src[nnz] = (uint32_t)u;
            dst[nnz] = (uint32_t)v;
            if (w) w[nnz] = (uint32_t)wt;
        }
        /* :94-99 running maximum over both endpoints */
        if (u > max_id) max_id = u;
        if (v > max_id) max_id = v;
        nnz++;
    }
    *nnz_out = nnz;
    *max_id_out = max_id;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CSR: coord2csr :117-159                                                    */
/* ------------------------------------------------------------------------ */

void pjo_coo2csr(const uint32_t* src, const uint32_t* dst, const uint32_t* w, int64_t nnz,
                 int64_t n, int64_t* row_ptr, uint32_t* col, uint32_t* w_out) {
    /* :130-135 out-degree histogram, :138-141 exclusive scan */
    memset(row_ptr, 0, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t l = 0; l < nnz; l++) row_ptr[src[l] + 1]++;
    for (int64_t i = 0; i < n; i++) row_ptr[i + 1] += row_ptr[i];
    /* :143-149 stable scatter in file order (cursor copy instead of the
     * reference's in-place bump + re-scan at :151-154; same result). */
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    memcpy(cur, row_ptr, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t l = 0; l < nnz; l++) {
        int64_t k = cur[src[l]]++;
        col[k] = dst[l];
        if (w_out) w_out[k] = w ? w[l] : 1u;
    }
    free(cur);
}

/* ------------------------------------------------------------------------ */
/* R9 contract oracles                                                        */
/* ------------------------------------------------------------------------ */

void pjo_bfs(const int64_t* row_ptr, const uint32_t* col, int64_t n, int64_t source,
             int32_t* dist) {
    for (int64_t i = 0; i < n; i++) dist[i] = PJO_INT_INF;
    if (source < 0 || source >= n) return; /* :479 never matches -> all inf */
    uint32_t* q = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    int64_t head = 0, tail = 0;
    dist[source] = 0;
    q[tail++] = (uint32_t)source;
    while (head < tail) {
        uint32_t u = q[head++];
        int32_t du = dist[u];
        if (du + 1 >= PJO_INT_INF) continue; /* candidates >= INT_INF are dropped (:250-251) */
        for (int64_t e = row_ptr[u]; e < row_ptr[u + 1]; e++) {
            uint32_t v = col[e];
            if (dist[v] == PJO_INT_INF) { dist[v] = du + 1; q[tail++] = v; }
        }
    }
    free(q);
}

/* pjo_bfs for k sources on `threads` host threads (test helper for the
 * batched multi-source rows; each row is exactly pjo_bfs). */
typedef struct {
    const int64_t* row; const uint32_t* col; int64_t n;
    const int64_t* src; int64_t k; int32_t* out; int t, nt;
} bfs_job;
static void* bfs_batch_worker(void* p) {
    bfs_job* j = (bfs_job*)p;
    for (int64_t i = j->t; i < j->k; i += j->nt)
        pjo_bfs(j->row, j->col, j->n, j->src[i], j->out + (size_t)i * (size_t)j->n);
    return NULL;
}
void pjo_bfs_batch(const int64_t* row_ptr, const uint32_t* col, int64_t n, const int64_t* sources,
                   int64_t k, int threads, int32_t* dist) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    bfs_job jobs[256];
    for (int t = 0; t < threads; t++) {
        bfs_job j = {row_ptr, col, n, sources, k, dist, t, threads};
        jobs[t] = j;
        pthread_create(&th[t], NULL, bfs_batch_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* binary heap keyed by int64 distance, lazy deletion */
typedef struct { int64_t d; uint32_t v; } hent;
static void hpush(hent** h, int64_t* n, int64_t* cap, int64_t d, uint32_t v) {
    if (*n == *cap) { *cap = *cap ? *cap * 2 : 1024; *h = (hent*)realloc(*h, sizeof(hent) * (size_t)*cap); }
    int64_t i = (*n)++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if ((*h)[p].d <= d) break;
        (*h)[i] = (*h)[p];
        i = p;
    }
    (*h)[i].d = d; (*h)[i].v = v;
}
static hent hpop(hent* h, int64_t* n) {
    hent top = h[0], last = h[--(*n)];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= *n) break;
        if (c + 1 < *n && h[c + 1].d < h[c].d) c++;
        if (h[c].d >= last.d) break;
        h[i] = h[c];
        i = c;
    }
    if (*n > 0) h[i] = last;
    return top;
}

void pjo_dijkstra(const int64_t* row_ptr, const uint32_t* col, const uint32_t* w, int64_t n,
                  int64_t source, int32_t* dist) {
    for (int64_t i = 0; i < n; i++) dist[i] = PJO_INT_INF;
    if (source < 0 || source >= n) return;
    hent* h = NULL;
    int64_t hn = 0, hc = 0;
    dist[source] = 0;
    hpush(&h, &hn, &hc, 0, (uint32_t)source);
    while (hn > 0) {
        hent t = hpop(h, &hn);
        if (t.d != dist[t.v]) continue;
        for (int64_t e = row_ptr[t.v]; e < row_ptr[t.v + 1]; e++) {
            int64_t nd = t.d + (int64_t)(w ? w[e] : 1u);
            uint32_t v = col[e];
            if (nd < PJO_INT_INF && nd < dist[v]) { dist[v] = (int32_t)nd; hpush(&h, &hn, &hc, nd, v); }
        }
    }
    free(h);
}

/* ------------------------------------------------------------------------ */
/* The reference algorithm: BSP label-correcting Dijkstra, :466-594           */
/* ------------------------------------------------------------------------ */

/* nn2rank :169-176, get_Nlocal :185-192, get_start_nn :197-200 */
static int nn2rank(int64_t nn, int64_t n, int nproc) {
    int64_t quota = n / nproc;
    if (nn >= quota * nproc) return nproc - 1;
    return (int)(nn / quota);
}
static int64_t get_nlocal(int64_t n, int nproc, int rank) {
    int64_t quota = n / nproc;
    return rank == nproc - 1 ? n - (int64_t)(nproc - 1) * quota : quota;
}
static int64_t get_start(int64_t n, int nproc, int rank) { return (n / nproc) * rank; }

/* addressable min-heap over local vertex ids (the fibonacci_heap of :466 and
 * the handles of :470/:476; pq_data's inverted operator< :212-216 makes it a
 * min-heap by dist). Results are independent of the heap. */
typedef struct {
    int64_t n;
    int32_t* key;   /* key per heap slot */
    int64_t* slot_v; /* local vertex per heap slot */
    int64_t* pos;   /* heap slot per local vertex, -1 = not in heap */
} aheap;

static void ah_swap(aheap* h, int64_t a, int64_t b) {
    int32_t k = h->key[a]; h->key[a] = h->key[b]; h->key[b] = k;
    int64_t v = h->slot_v[a]; h->slot_v[a] = h->slot_v[b]; h->slot_v[b] = v;
    h->pos[h->slot_v[a]] = a; h->pos[h->slot_v[b]] = b;
}
static void ah_up(aheap* h, int64_t i) {
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (h->key[p] <= h->key[i]) break;
        ah_swap(h, p, i);
        i = p;
    }
}
static void ah_down(aheap* h, int64_t i) {
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && h->key[c + 1] < h->key[c]) c++;
        if (h->key[i] <= h->key[c]) break;
        ah_swap(h, i, c);
        i = c;
    }
}
static void ah_push(aheap* h, int64_t lv, int32_t key) {
    int64_t i = h->n++;
    h->key[i] = key; h->slot_v[i] = lv; h->pos[lv] = i;
    ah_up(h, i);
}
static void ah_decrease(aheap* h, int64_t lv, int32_t key) {
    int64_t i = h->pos[lv];
    h->key[i] = key;
    ah_up(h, i);
}
static void ah_pop(aheap* h) {
    int64_t lv = h->slot_v[0];
    h->n--;
    if (h->n > 0) {
        h->key[0] = h->key[h->n]; h->slot_v[0] = h->slot_v[h->n]; h->pos[h->slot_v[0]] = 0;
        ah_down(h, 0);
    }
    h->pos[lv] = -1;
}

typedef struct { uint32_t v; int32_t d; } msg_t;
typedef struct { msg_t* m; int64_t n, cap; } mbuf;
static void mb_push(mbuf* b, uint32_t v, int32_t d) {
    if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 256; b->m = (msg_t*)realloc(b->m, sizeof(msg_t) * (size_t)b->cap); }
    b->m[b->n].v = v; b->m[b->n].d = d; b->n++;
}

typedef struct {
    const int64_t* row_ptr; const uint32_t* col; const uint32_t* w;
    int64_t n, source; int nproc;
    int32_t* sp;            /* :443, shared; each rank touches its own slice */
    mbuf* out;              /* out[src * nproc + dst] */
    int* flags;             /* local_pq_len per rank (:579-588) */
    pthread_barrier_t bar;
    pjo_ref_stats st[64];
    double t0, t1;
    double budget_s;        /* > 0: stop after this much solve time (bounded CPU-baseline sample) */
    int stop;
} ref_shared;

typedef struct { ref_shared* sh; int rank; } ref_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* relax one candidate (v, d) into the owner's heap: the rule of :249-264 and
 * :560-572 (decrease while queued, re-insert once settled). */
static void relax_local(aheap* h, int32_t* sp, int64_t start, uint32_t v, int64_t d,
                        pjo_ref_stats* st) {
    if (sp[v] == PJO_INT_INF) {                 /* v still in the queue */
        if (h->key[h->pos[v - start]] > d) { ah_decrease(h, v - start, (int32_t)d); st->decreases++; }
    } else if (sp[v] > d) {                     /* settled, improved: re-insert */
        ah_push(h, v - start, (int32_t)d);
        sp[v] = PJO_INT_INF;
        st->reinserts++;
    }
}

static void* ref_rank(void* p) {
    ref_arg* a = (ref_arg*)p;
    ref_shared* S = a->sh;
    const int rank = a->rank, P = S->nproc;
    const int64_t n = S->n, start = get_start(n, P, rank), nl = get_nlocal(n, P, rank);
    pjo_ref_stats* st = &S->st[rank];
    memset(st, 0, sizeof(*st));
    for (int64_t i = 0; i < nl; i++) S->sp[start + i] = PJO_INT_INF; /* :445 */

    pthread_barrier_wait(&S->bar); /* :459 */
    if (rank == 0) S->t0 = now_s();

    aheap h;
    h.n = 0;
    h.key = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nl + 1));
    h.slot_v = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nl + 1));
    h.pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nl + 1));
    for (int64_t i = 0; i < nl; i++) /* :476-486 every local vertex, source key 0 */
        ah_push(&h, i, (start + i) == S->source ? 0 : PJO_INT_INF);

    for (;;) {
        mbuf* myout = S->out + (size_t)rank * P;
        for (int d = 0; d < P; d++) myout[d].n = 0;
        for (int l = 0; l < 30; l++) { /* async_iter :514-519 */
            /* extract_local_pq :226-278 */
            if (h.n == 0 || h.key[0] == PJO_INT_INF) break; /* later iterations are no-ops too */
            int64_t d = h.key[0];
            int64_t u = start + h.slot_v[0];
            ah_pop(&h);
            st->pops++;
            S->sp[u] = (int32_t)d;
            for (int64_t e = S->row_ptr[u]; e < S->row_ptr[u + 1]; e++) {
                uint32_t v = S->col[e];
                int64_t cand = d + (int64_t)(S->w ? S->w[e] : 1u);
                st->scans++;
                int owner = nn2rank(v, n, P);
                if (owner == rank) relax_local(&h, S->sp, start, v, cand, st);
                else mb_push(&myout[owner], v, cand >= PJO_INT_INF ? PJO_INT_INF : (int32_t)cand);
            }
        }
        st->rounds++;
        pthread_barrier_wait(&S->bar); /* MPI_Alltoall + MPI_Alltoallv :522-554 */
        for (int s = 0; s < P; s++) { /* :557-573, in source-rank order */
            mbuf* b = &S->out[(size_t)s * P + rank];
            st->messages += b->n;
            for (int64_t j = 0; j < b->n; j++) relax_local(&h, S->sp, start, b->m[j].v, b->m[j].d, st);
        }
        S->flags[rank] = (h.n > 0 && h.key[0] != PJO_INT_INF) ? 1 : 0; /* :579-588 */
        if (rank == 0 && S->budget_s > 0 && now_s() - S->t0 > S->budget_s) S->stop = 1;
        pthread_barrier_wait(&S->bar); /* MPI_Allreduce :589-590 */
        int total = 0;
        for (int r = 0; r < P; r++) total += S->flags[r];
        if (total == 0 || S->stop) break;
        pthread_barrier_wait(&S->bar); /* keep flags stable until every rank has summed */
    }
    pthread_barrier_wait(&S->bar); /* :597 */
    if (rank == 0) S->t1 = now_s();
    free(h.key); free(h.slot_v); free(h.pos);
    return NULL;
}

int pjo_reference_sssp(const int64_t* row_ptr, const uint32_t* col, const uint32_t* w, int64_t n,
                       int64_t source, int nproc, int32_t* dist, pjo_ref_stats* stats) {
    return pjo_reference_sssp_budget(row_ptr, col, w, n, source, nproc, 0.0, dist, stats);
}

int pjo_reference_sssp_budget(const int64_t* row_ptr, const uint32_t* col, const uint32_t* w, int64_t n,
                              int64_t source, int nproc, double budget_s, int32_t* dist,
                              pjo_ref_stats* stats) {
    if (nproc < 1 || nproc > 64) return -1;
    ref_shared* S = (ref_shared*)calloc(1, sizeof(ref_shared));
    S->budget_s = budget_s;
    S->row_ptr = row_ptr; S->col = col; S->w = w; S->n = n; S->source = source; S->nproc = nproc;
    S->sp = dist; /* MPI_Gatherv :612 is implicit: the slices are written in place */
    S->out = (mbuf*)calloc((size_t)nproc * nproc, sizeof(mbuf));
    S->flags = (int*)calloc((size_t)nproc, sizeof(int));
    pthread_barrier_init(&S->bar, NULL, (unsigned)nproc);
    pthread_t th[64];
    ref_arg args[64];
    for (int r = 0; r < nproc; r++) {
        args[r].sh = S; args[r].rank = r;
        pthread_create(&th[r], NULL, ref_rank, &args[r]);
    }
    for (int r = 0; r < nproc; r++) pthread_join(th[r], NULL);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->solve_s = S->t1 - S->t0;
        stats->truncated = S->stop;
        for (int r = 0; r < nproc; r++) {
            if (S->st[r].rounds > stats->rounds) stats->rounds = S->st[r].rounds;
            stats->pops += S->st[r].pops; stats->scans += S->st[r].scans;
            stats->decreases += S->st[r].decreases; stats->reinserts += S->st[r].reinserts;
            stats->messages += S->st[r].messages;
        }
    }
    for (int i = 0; i < nproc * nproc; i++) free(S->out[i].m);
    free(S->out); free(S->flags);
    pthread_barrier_destroy(&S->bar);
    free(S);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Output: output_vector :32-46                                               */
/* ------------------------------------------------------------------------ */

int64_t pjo_format_sol(const int32_t* dist, int64_t n, char* buf) {
    static const char hdr[] = "the vector is:\n";
    int64_t len = 0;
    if (buf) memcpy(buf, hdr, sizeof(hdr) - 1);
    len += (int64_t)sizeof(hdr) - 1;
    char tmp[16];
    for (int64_t i = 0; i < n; i++) {
        int32_t d = dist[i];
        int k = 0;
        if (d == PJO_INT_INF) { tmp[k++] = 'i'; tmp[k++] = 'n'; tmp[k++] = 'f'; }
        else {
            int64_t x = d;
            char rev[16];
            int r = 0;
            int neg = x < 0;
            if (neg) x = -x;
            do { rev[r++] = (char)('0' + x % 10); x /= 10; } while (x);
            if (neg) tmp[k++] = '-';
            while (r) tmp[k++] = rev[--r];
        }
        tmp[k++] = '\n';
        if (buf) memcpy(buf + len, tmp, (size_t)k);
        len += k;
    }
    return len;
}

/* ------------------------------------------------------------------------ */
/* Kronecker generator spec, restated for cross-checks    */
/* ------------------------------------------------------------------------ */

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static uint64_t kperm(uint64_t x, int scale, uint64_t seed) {
    if (scale == 0) return 0;
    uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    uint64_t k1 = splitmix64(seed ^ 0x243F6A8885A308D3ULL) | 1ULL;
    uint64_t k2 = splitmix64(seed ^ 0x13198A2E03707344ULL) | 1ULL;
    uint64_t c1 = splitmix64(seed ^ 0xA4093822299F31D0ULL);
    int sh = (scale + 1) / 2;
    x = (x * k1 + c1) & mask;
    x ^= x >> sh;
    x = (x * k2) & mask;
    x ^= x >> sh;
    x = (x * k1 + (c1 >> 7)) & mask;
    return x;
}

void pjo_kronecker(int scale, int edgefactor, uint64_t seed, int weighted, uint32_t* src,
                   uint32_t* dst, uint32_t* w) {
    const uint64_t M = (uint64_t)edgefactor << scale;
    const uint32_t TA = 2448131358u, TAB = 3264175144u, TABC = 4080218931u;
    for (uint64_t i = 0; i < M; i++) {
        uint64_t u = 0, v = 0;
        for (int l = 0; l < scale; l++) {
            uint32_t r = (uint32_t)(splitmix64(seed ^ ((i << 6) | (uint64_t)l)) >> 32);
            uint64_t bu = r >= TAB, bv = (r >= TA && r < TAB) || r >= TABC;
            u = (u << 1) | bu;
            v = (v << 1) | bv;
        }
        uint32_t pu = (uint32_t)kperm(u, scale, seed), pv = (uint32_t)kperm(v, scale, seed);
        src[2 * i] = pu; dst[2 * i] = pv;
        src[2 * i + 1] = pv; dst[2 * i + 1] = pu;
        if (w) {
            uint32_t wt = weighted ? 1u + (uint32_t)(splitmix64(seed ^ 0x5851F42D4C957F2DULL ^ i) % 255u) : 1u;
            w[2 * i] = wt; w[2 * i + 1] = wt;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Row digests: an order-free fingerprint of every CSR row, computed from the  */
/* generator spec directly (no sort, no CSR) and from a CSR, so a full-size    */
/* GPU build (s26w: 2^31 entries) is checked against an independent path.     */
/* digest(v) = (entries of row v, sum over them of splitmix64(col<<8 | w)).    */
/* ------------------------------------------------------------------------ */

static uint64_t entry_hash(uint32_t col, uint32_t w) {
    return splitmix64(((uint64_t)col << 8 | (uint64_t)(w & 0xffu)) ^ 0x6A09E667F3BCC909ULL);
}

typedef struct {
    int scale, weighted;
    uint64_t seed, i0, i1;
    uint32_t* deg;
    uint64_t* hsum;
} kdig_job;

static void* kdig_worker(void* arg) {
    kdig_job* J = (kdig_job*)arg;
    const uint32_t TA = 2448131358u, TAB = 3264175144u, TABC = 4080218931u;
    for (uint64_t i = J->i0; i < J->i1; i++) {
        uint64_t u = 0, v = 0;
        for (int l = 0; l < J->scale; l++) {
            uint32_t r = (uint32_t)(splitmix64(J->seed ^ ((i << 6) | (uint64_t)l)) >> 32);
            uint64_t bu = r >= TAB, bv = (r >= TA && r < TAB) || r >= TABC;
            u = (u << 1) | bu;
            v = (v << 1) | bv;
        }
        uint32_t pu = (uint32_t)kperm(u, J->scale, J->seed), pv = (uint32_t)kperm(v, J->scale, J->seed);
        uint32_t wt = J->weighted ? 1u + (uint32_t)(splitmix64(J->seed ^ 0x5851F42D4C957F2DULL ^ i) % 255u) : 1u;
        /* both directions, as pjo_kronecker writes them */
        __atomic_fetch_add(&J->deg[pu], 1u, __ATOMIC_RELAXED);
        __atomic_fetch_add(&J->hsum[pu], entry_hash(pv, wt), __ATOMIC_RELAXED);
        __atomic_fetch_add(&J->deg[pv], 1u, __ATOMIC_RELAXED);
        __atomic_fetch_add(&J->hsum[pv], entry_hash(pu, wt), __ATOMIC_RELAXED);
    }
    return NULL;
}

void pjo_kronecker_row_digest(int scale, int edgefactor, uint64_t seed, int weighted, int threads, uint32_t* deg,
                              uint64_t* hsum) {
    const uint64_t M = (uint64_t)edgefactor << scale, n = 1ULL << scale;
    memset(deg, 0, sizeof(uint32_t) * n);
    memset(hsum, 0, sizeof(uint64_t) * n);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    kdig_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (kdig_job){scale, weighted, seed, M * (uint64_t)t / (uint64_t)threads,
                             M * (uint64_t)(t + 1) / (uint64_t)threads, deg, hsum};
        pthread_create(&th[t], NULL, kdig_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

typedef struct {
    const int64_t* row;
    const uint32_t* col;
    const uint32_t* w;
    int64_t v0, v1;
    uint32_t* deg;
    uint64_t* hsum;
    int64_t unsorted;
} cdig_job;

static void* cdig_worker(void* arg) {
    cdig_job* J = (cdig_job*)arg;
    for (int64_t v = J->v0; v < J->v1; v++) {
        uint64_t h = 0;
        for (int64_t k = J->row[v]; k < J->row[v + 1]; k++) {
            const uint32_t wk = J->w ? J->w[k] : 1u;
            h += entry_hash(J->col[k], wk);
            if (J->w && k > J->row[v] && J->w[k - 1] > wk) J->unsorted++;
        }
        J->deg[v] = (uint32_t)(J->row[v + 1] - J->row[v]);
        J->hsum[v] = h;
    }
    return NULL;
}

/* returns the number of entries whose weight is below their predecessor's in the row */
int64_t pjo_csr_row_digest(const int64_t* row, const uint32_t* col, const uint32_t* w, int64_t n, int threads,
                           uint32_t* deg, uint64_t* hsum) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    cdig_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (cdig_job){row, col, w, n * t / threads, n * (t + 1) / threads, deg, hsum, 0};
        pthread_create(&th[t], NULL, cdig_worker, &jobs[t]);
    }
    int64_t bad = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        bad += jobs[t].unsorted;
    }
    return bad;
}
