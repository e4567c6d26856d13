/*
 * grf_oracle.c -- CPU restatement of the reference GRF hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline.  The product path
 * (efficient-gaussian-process-on-graphs_amd/) never links or calls it.
 *
 * Parity status: PINNED.  Every routine below is checked bit-for-bit against
 * golden vectors produced by the Python reference itself
 * (tests/golden/make_golden.py imports /root/reference in the build container).
 *
 * What it restates (reference paths relative to /root/reference):
 *   - numpy SeedSequence / PCG64 / Generator.random / Generator.integers
 *     (Lemire, 32-bit halves buffered in the bit generator) as consumed by
 *     efficient_graph_gp_sparse/random_walk_samplers_sparse/sparse_sampler.py:35-54
 *     and efficient_graph_gp/random_walk_samplers/sampler.py:35-59,148-186.
 *   - chunking np.array_split(arange(N), n_proc), seeds (seed or 42)+i
 *     (sampler.py:91,119,131; sparse_sampler.py:65,90,102).
 *   - load rules: cumulative (sampler.py:58, sparse_sampler.py:54),
 *     legacy non-cumulative (sampler.py:183), ablation (sampler.py:180-181).
 *   - per-key accumulation in walk order + normalisation value/m
 *     (sampler.py:201) or value*(1/m) (sparse_sampler.py:130, scipy _mul_scalar).
 *   - normalised Laplacians: scipy semantics
 *     (efficient_graph_gp_sparse/utils_sparse/graph_utils.py:5-30) and numpy
 *     semantics (efficient_graph_gp/graph_kernels/utils.py:6-28,
 *     efficient_graph_gp/preprocessing/laplacian_np.py:3-35).
 *   - Phi = sum_l f_l M_l with scipy CSR add semantics and K = Phi Phi^T with
 *     scipy csr_matmat summation order
 *     (efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:47-55).
 *   - Philox4x32-10 counter mode (the MI355X engine's fast RNG; not in the
 *     reference) so that the GPU walker can be checked bit-for-bit.
 *
 * Build: oracle/Makefile -> oracle/_build/libgrf_oracle.so (gcc, -ffp-contract=off).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* tiny pthread parallel-for                                                  */
/* ------------------------------------------------------------------------- */
typedef void (*range_fn)(void *ctx, int64_t begin, int64_t end);
typedef struct { range_fn fn; void *ctx; int64_t n; int64_t grain; int64_t *next; pthread_mutex_t *mu; } pf_arg;

static void *pf_worker(void *p) {
    pf_arg *a = (pf_arg *)p;
    for (;;) {
        pthread_mutex_lock(a->mu);
        int64_t b = *a->next;
        *a->next += a->grain;
        pthread_mutex_unlock(a->mu);
        if (b >= a->n) break;
        int64_t e = b + a->grain < a->n ? b + a->grain : a->n;
        a->fn(a->ctx, b, e);
    }
    return NULL;
}

static void parallel_for(int n_threads, int64_t n, int64_t grain, range_fn fn, void *ctx) {
    if (n <= 0) return;
    if (grain < 1) grain = 1;
    if (n_threads <= 1 || n <= grain) { fn(ctx, 0, n); return; }
    if (n_threads > 512) n_threads = 512;
    pthread_t th[512];
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    int64_t next = 0;
    pf_arg a = {fn, ctx, n, grain, &next, &mu};
    for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, pf_worker, &a);
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------- */
/* numpy SeedSequence (bit_generator.pyx) -> PCG64 (pcg64.c)                  */
/* ------------------------------------------------------------------------- */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

typedef unsigned __int128 u128;

typedef struct { u128 state, inc; int has_uint32; uint32_t uinteger; } pcg64_t;

static const u128 PCG_MULT = (((u128)2549297995355413924ULL) << 64) | (u128)4865540595714422341ULL;

static inline uint32_t ss_hashmix(uint32_t v, uint32_t *hc) {
    v ^= *hc;
    *hc *= SS_MULT_A;
    v *= *hc;
    v ^= v >> 16;
    return v;
}
static inline uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

/* entropy: little-endian 32-bit words of the non-negative seed integer */
static void seedseq_pcg64(const uint32_t *ent, int n_ent, pcg64_t *g) {
    uint32_t pool[4];
    uint32_t hc = SS_INIT_A;
    for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, &hc);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
    for (int s = 4; s < n_ent; ++s)
        for (int d = 0; d < 4; ++d) pool[d] = ss_mix(pool[d], ss_hashmix(ent[s], &hc));
    uint32_t hb = SS_INIT_B, w[8];
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    uint64_t s0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), s1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    uint64_t s2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), s3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
    u128 initstate = ((u128)s0 << 64) | s1, initseq = ((u128)s2 << 64) | s3;
    g->inc = (initseq << 1) | 1u;
    g->state = 0;
    g->state = g->state * PCG_MULT + g->inc;
    g->state += initstate;
    g->state = g->state * PCG_MULT + g->inc;
    g->has_uint32 = 0;
    g->uinteger = 0;
}

static inline uint64_t pcg64_next64(pcg64_t *g) {
    g->state = g->state * PCG_MULT + g->inc;
    uint64_t hi = (uint64_t)(g->state >> 64), lo = (uint64_t)g->state;
    unsigned rot = (unsigned)(g->state >> 122);
    uint64_t x = hi ^ lo;
    return (x >> rot) | (x << ((64u - rot) & 63u));
}
static inline uint32_t pcg64_next32(pcg64_t *g) {
    if (g->has_uint32) { g->has_uint32 = 0; return g->uinteger; }
    uint64_t n = pcg64_next64(g);
    g->has_uint32 = 1;
    g->uinteger = (uint32_t)(n >> 32);
    return (uint32_t)n;
}
/* Generator.random(): (next64 >> 11) * 2^-53 */
static inline double pcg64_random(pcg64_t *g) { return (double)(pcg64_next64(g) >> 11) * (1.0 / 9007199254740992.0); }
/* Generator.integers(d) for 1 <= d <= 2^32-1: buffered 32-bit Lemire; d==1 draws nothing */
static inline uint32_t pcg64_integers(pcg64_t *g, uint32_t d) {
    uint32_t rng = d - 1u;
    if (rng == 0) return 0;
    uint64_t m = (uint64_t)pcg64_next32(g) * (uint64_t)d;
    uint32_t left = (uint32_t)m;
    if (left < d) {
        uint32_t thr = (0xFFFFFFFFu - rng) % d;
        while (left < thr) {
            m = (uint64_t)pcg64_next32(g) * (uint64_t)d;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

/* exported for tests: seed -> state, and a mixed draw stream */
ORACLE_API void oracle_pcg64_init(const uint32_t *ent, int n_ent, uint64_t out[4]) {
    pcg64_t g;
    seedseq_pcg64(ent, n_ent, &g);
    out[0] = (uint64_t)(g.state >> 64); out[1] = (uint64_t)g.state;
    out[2] = (uint64_t)(g.inc >> 64);   out[3] = (uint64_t)g.inc;
}
/* ops[i] == 0 -> random(), else integers(ops[i]); results as double */
ORACLE_API void oracle_pcg64_stream(const uint32_t *ent, int n_ent, const uint32_t *ops, int64_t n, double *out) {
    pcg64_t g;
    seedseq_pcg64(ent, n_ent, &g);
    for (int64_t i = 0; i < n; ++i) out[i] = ops[i] == 0 ? pcg64_random(&g) : (double)pcg64_integers(&g, ops[i]);
}

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al. 2011)                                         */
/* ------------------------------------------------------------------------- */
static inline void philox4x32_10(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
ORACLE_API void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    philox4x32_10(ctr, key[0], key[1], out);
}

/* per-walk counter stream: block b of step l of walk (s, w) */
typedef struct { uint32_t k0, k1, step, walk, src, block; uint32_t buf[4]; int pos; } philox_stream;
static inline void ps_refill(philox_stream *p) {
    uint32_t c[4] = {p->step, p->walk, p->src, p->block};
    philox4x32_10(c, p->k0, p->k1, p->buf);
    p->block++;
    p->pos = 0;
}
static inline uint32_t ps_next(philox_stream *p) {
    if (p->pos == 4) ps_refill(p);
    return p->buf[p->pos++];
}

/* ------------------------------------------------------------------------- */
/* walk parameters (mirror of include/grf.h semantics)                        */
/* ------------------------------------------------------------------------- */
enum { LOAD_CUMULATIVE = 0, LOAD_NONCUMULATIVE = 1, LOAD_ABLATION = 2 };
enum { RNG_PCG64 = 0, RNG_PHILOX = 1 };

typedef struct {
    int64_t n;             /* nodes                                    */
    const int64_t *indptr; /* CSR of the walk matrix (Laplacian)       */
    const int32_t *indices;
    const double *data;
    int64_t m;             /* walks per node                           */
    double p_halt;
    int32_t L;             /* max walk length                          */
    int32_t load_rule;
    /* pcg64 */
    int64_t n_chunks;      /* np.array_split(arange(n), n_chunks)      */
    uint64_t seed_base;    /* chunk i seeded with seed_base + i        */
    /* philox */
    uint64_t philox_seed;
    /* output slots [n][L][m] */
    int32_t *slot_node;
    double *slot_load;
} walk_ctx;

static inline double load_update(int rule, double load, int64_t deg, double w, double p) {
    double f = ((double)deg * w) / (1.0 - p);
    if (rule == LOAD_CUMULATIVE) return load * f;
    if (rule == LOAD_NONCUMULATIVE) return f;
    return w; /* ablation */
}

static void seed_words(uint64_t seed, uint32_t *w, int *nw) {
    /* numpy _int_to_uint32_array: 0 -> [0] */
    *nw = 0;
    if (seed == 0) { w[(*nw)++] = 0; return; }
    while (seed) { w[(*nw)++] = (uint32_t)seed; seed >>= 32; }
}

/* one chunk = contiguous node range consumed by ONE sequential PCG64 stream
 * (sparse_sampler.py:35-54 / sampler.py:35-59,162-184) */
static void walk_pcg64_chunk(walk_ctx *c, int64_t chunk) {
    int64_t base = c->n / c->n_chunks, extra = c->n % c->n_chunks;
    int64_t b = chunk * base + (chunk < extra ? chunk : extra);
    int64_t e = b + base + (chunk < extra ? 1 : 0);
    uint32_t w[4];
    int nw;
    seed_words(c->seed_base + (uint64_t)chunk, w, &nw);
    pcg64_t g;
    seedseq_pcg64(w, nw, &g);
    const int64_t L = c->L, m = c->m;
    for (int64_t s = b; s < e; ++s) {
        for (int64_t wk = 0; wk < m; ++wk) {
            int64_t cur = s;
            double load = 1.0;
            int64_t l = 0;
            for (; l < L; ++l) {
                int64_t slot = (s * L + l) * m + wk;
                c->slot_node[slot] = (int32_t)cur;
                c->slot_load[slot] = load;
                int64_t rs = c->indptr[cur], deg = c->indptr[cur + 1] - rs;
                if (deg == 0 || pcg64_random(&g) < c->p_halt) { ++l; break; }
                uint32_t k = pcg64_integers(&g, (uint32_t)deg);
                double wt = c->data[rs + k];
                load = load_update(c->load_rule, load, deg, wt, c->p_halt);
                cur = c->indices[rs + k];
            }
            for (; l < L; ++l) {
                int64_t slot = (s * L + l) * m + wk;
                c->slot_node[slot] = -1;
                c->slot_load[slot] = 0.0;
            }
        }
    }
}
static void walk_pcg64_range(void *ctx, int64_t b, int64_t e) {
    for (int64_t ch = b; ch < e; ++ch) walk_pcg64_chunk((walk_ctx *)ctx, ch);
}

/* Philox walk of (s, wk), the engine's stream (csrc/grf_philox.h StepWords): one Philox4x32-10 block
 * (l / 2, wk, s, 0) serves the step pair l = 2j, 2j + 1 -- the even step halts iff x0 < ceil(p 2^32) and
 * picks its neighbour by 32-bit Lemire from x1, the odd step uses x2 and x3; a Lemire rejection of step l
 * continues on blocks (l, wk, s, 1), (l, wk, s, 2), ...; the L-th recorded visit draws nothing. */
static uint64_t halt_threshold32(double p) {
    double y = ceil(p * 4294967296.0);
    return y > 0.0 ? (y < 4294967296.0 ? (uint64_t)y : (1ull << 32)) : 0ull;
}
static void walk_philox_one(walk_ctx *c, int64_t s, int64_t wk) {
    const int64_t L = c->L, m = c->m;
    const uint32_t k0 = (uint32_t)c->philox_seed, k1 = (uint32_t)(c->philox_seed >> 32);
    const uint64_t hthr = halt_threshold32(c->p_halt);
    uint32_t x[4] = {0, 0, 0, 0};
    int64_t cur = s;
    double load = 1.0;
    int64_t l = 0;
    for (; l < L; ++l) {
        int64_t slot = (s * L + l) * m + wk;
        c->slot_node[slot] = (int32_t)cur;
        c->slot_load[slot] = load;
        if (l == L - 1) { ++l; break; }
        int64_t rs = c->indptr[cur], deg = c->indptr[cur + 1] - rs;
        if (deg == 0) { ++l; break; }
        if ((l & 1) == 0) {
            uint32_t ctr[4] = {(uint32_t)(l >> 1), (uint32_t)wk, (uint32_t)s, 0u};
            philox4x32_10(ctr, k0, k1, x);
        }
        uint32_t hw = (l & 1) ? x[2] : x[0], pw = (l & 1) ? x[3] : x[1];
        if ((uint64_t)hw < hthr) { ++l; break; }
        uint32_t d = (uint32_t)deg, k = 0;
        if (d > 1) {
            uint64_t mm = (uint64_t)pw * d;
            uint32_t left = (uint32_t)mm;
            if (left < d) {
                uint32_t thr = (uint32_t)(0u - d) % d;
                if (left < thr) {
                    philox_stream ps = {k0, k1, (uint32_t)l, (uint32_t)wk, (uint32_t)s, 1u, {0, 0, 0, 0}, 4};
                    while (left < thr) { mm = (uint64_t)ps_next(&ps) * d; left = (uint32_t)mm; }
                }
            }
            k = (uint32_t)(mm >> 32);
        }
        double wt = c->data[rs + k];
        load = load_update(c->load_rule, load, deg, wt, c->p_halt);
        cur = c->indices[rs + k];
    }
    for (; l < L; ++l) {
        int64_t slot = (s * L + l) * m + wk;
        c->slot_node[slot] = -1;
        c->slot_load[slot] = 0.0;
    }
}
static void walk_philox_range(void *ctx, int64_t b, int64_t e) {
    walk_ctx *c = (walk_ctx *)ctx;
    for (int64_t s = b; s < e; ++s)
        for (int64_t wk = 0; wk < c->m; ++wk) walk_philox_one(c, s, wk);
}

/* Walk every source in [begin, end) (philox) or every chunk in [begin, end)
 * (pcg64).  Slots are [n][L][m]. */
typedef struct { walk_ctx *c; int64_t off; int pcg; } walk_off;
static void walk_off_range(void *ctx, int64_t b, int64_t e) {
    walk_off *w = (walk_off *)ctx;
    if (w->pcg) walk_pcg64_range(w->c, b + w->off, e + w->off);
    else walk_philox_range(w->c, b + w->off, e + w->off);
}
ORACLE_API int oracle_walk_range(int64_t n, const int64_t *indptr, const int32_t *indices, const double *data,
                                 int64_t m, double p_halt, int32_t L, int32_t load_rule, int32_t rng,
                                 int64_t n_chunks, uint64_t seed, int64_t begin, int64_t end, int32_t *slot_node,
                                 double *slot_load, int n_threads) {
    walk_ctx c = {n, indptr, indices, data, m, p_halt, L, load_rule, n_chunks, seed, seed, slot_node, slot_load};
    if (rng == RNG_PCG64 && n_chunks < 1) return -1;
    walk_off w = {&c, begin, rng == RNG_PCG64};
    parallel_for(n_threads, end - begin, rng == RNG_PCG64 ? 1 : 64, walk_off_range, &w);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* slots -> per-step rows (sorted by node, sums in walk order)                */
/* ------------------------------------------------------------------------- */
typedef struct { int32_t node; int32_t walk; } nw_pair;
static int cmp_nw(const void *a, const void *b) {
    const nw_pair *x = (const nw_pair *)a, *y = (const nw_pair *)b;
    if (x->node != y->node) return x->node < y->node ? -1 : 1;
    return x->walk < y->walk ? -1 : (x->walk > y->walk);
}

enum { NORM_DIV = 0, NORM_MUL_RECIP = 1 };

typedef struct {
    int64_t n, m; int32_t L, norm;
    const int32_t *slot_node; const double *slot_load;
    int64_t *cnt;          /* [n][L] distinct nodes per (s,l) (count pass) */
    const int64_t *rowptr; /* [L][n+1] output row pointers (fill pass), NULL on count pass */
    int32_t *out_idx; double *out_val; /* [L] concatenated: step l at offset l_off[l] */
    const int64_t *l_off;
} reduce_ctx;

static void reduce_range(void *ctx, int64_t b, int64_t e) {
    reduce_ctx *r = (reduce_ctx *)ctx;
    nw_pair *buf = (nw_pair *)malloc(sizeof(nw_pair) * (size_t)(r->m > 0 ? r->m : 1));
    for (int64_t s = b; s < e; ++s) {
        for (int32_t l = 0; l < r->L; ++l) {
            const int32_t *nd = r->slot_node + (s * r->L + l) * r->m;
            const double *ld = r->slot_load + (s * r->L + l) * r->m;
            int64_t k = 0;
            for (int64_t w = 0; w < r->m; ++w)
                if (nd[w] >= 0) { buf[k].node = nd[w]; buf[k].walk = (int32_t)w; ++k; }
            qsort(buf, (size_t)k, sizeof(nw_pair), cmp_nw);
            int64_t distinct = 0;
            int64_t pos = r->rowptr ? r->l_off[l] + r->rowptr[(int64_t)l * (r->n + 1) + s] : 0;
            for (int64_t i = 0; i < k;) {
                int64_t j = i;
                double acc = 0.0; /* defaultdict(float) starts at 0.0 */
                while (j < k && buf[j].node == buf[i].node) { acc += ld[buf[j].walk]; ++j; }
                if (r->rowptr) {
                    r->out_idx[pos] = buf[i].node;
                    r->out_val[pos] = r->norm == NORM_DIV ? acc / (double)r->m : acc * (1.0 / (double)r->m);
                    ++pos;
                }
                ++distinct;
                i = j;
            }
            if (!r->rowptr) r->cnt[s * r->L + l] = distinct;
        }
    }
    free(buf);
}

/* count pass: cnt[n][L] */
ORACLE_API void oracle_reduce_count(int64_t n, int64_t m, int32_t L, const int32_t *slot_node, const double *slot_load,
                                    int64_t *cnt, int n_threads) {
    reduce_ctx r = {n, m, L, 0, slot_node, slot_load, cnt, NULL, NULL, NULL, NULL};
    parallel_for(n_threads, n, 16, reduce_range, &r);
}
/* fill pass: rowptr [L][n+1] (per-step CSR row pointers), l_off [L] (offset of
 * step l inside out_idx/out_val) */
ORACLE_API void oracle_reduce_fill(int64_t n, int64_t m, int32_t L, int32_t norm, const int32_t *slot_node,
                                   const double *slot_load, const int64_t *rowptr, const int64_t *l_off,
                                   int32_t *out_idx, double *out_val, int n_threads) {
    reduce_ctx r = {n, m, L, norm, slot_node, slot_load, NULL, rowptr, out_idx, out_val, l_off};
    parallel_for(n_threads, n, 16, reduce_range, &r);
}

/* ------------------------------------------------------------------------- */
/* Phi = sum_l f_l M_l  (scipy: empty csr, then Phi = Phi + f_l*M_l, each add */
/* drops exact zeros; fast_grf_kernel_general.py:47-52)                       */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t n; int32_t nsteps;
    const int64_t *rowptr; const int64_t *l_off; const int32_t *idx; const double *val; /* step CSRs */
    const double *f;
    const int64_t *phi_ptr; int64_t *phi_cnt; int32_t *phi_idx; double *phi_val;
} phi_ctx;

static void phi_range(void *ctx, int64_t b, int64_t e) {
    phi_ctx *p = (phi_ctx *)ctx;
    int32_t L = p->nsteps;
    int64_t pos_l[64], end_l[64];
    for (int64_t s = b; s < e; ++s) {
        for (int32_t l = 0; l < L; ++l) {
            pos_l[l] = p->l_off[l] + p->rowptr[(int64_t)l * (p->n + 1) + s];
            end_l[l] = p->l_off[l] + p->rowptr[(int64_t)l * (p->n + 1) + s + 1];
        }
        int64_t out = p->phi_ptr ? p->phi_ptr[s] : 0, cnt = 0;
        for (;;) {
            int32_t mn = INT32_MAX;
            for (int32_t l = 0; l < L; ++l)
                if (pos_l[l] < end_l[l] && p->idx[pos_l[l]] < mn) mn = p->idx[pos_l[l]];
            if (mn == INT32_MAX) break;
            double acc = 0.0;
            int present = 0;
            for (int32_t l = 0; l < L; ++l) {
                if (pos_l[l] < end_l[l] && p->idx[pos_l[l]] == mn) {
                    double t = p->f[l] * p->val[pos_l[l]];
                    acc = present ? acc + t : 0.0 + t;
                    present = 1;
                    /* scipy drops an exact zero after every add; continuing from 0 is identical */
                    if (acc == 0.0) acc = 0.0;
                    ++pos_l[l];
                }
            }
            if (acc != 0.0) {
                if (p->phi_idx) { p->phi_idx[out] = mn; p->phi_val[out] = acc; ++out; }
                ++cnt;
            }
        }
        if (p->phi_cnt) p->phi_cnt[s] = cnt;
    }
}

ORACLE_API void oracle_phi(int64_t n, int32_t nsteps, const int64_t *rowptr, const int64_t *l_off, const int32_t *idx,
                           const double *val, const double *f, const int64_t *phi_ptr, int64_t *phi_cnt,
                           int32_t *phi_idx, double *phi_val, int n_threads) {
    phi_ctx p = {n, nsteps, rowptr, l_off, idx, val, f, phi_ptr, phi_cnt, phi_idx, phi_val};
    parallel_for(n_threads, n, 64, phi_range, &p);
}

/* ------------------------------------------------------------------------- */
/* K rows [r0, r1) = Phi[r0:r1] Phi^T, scipy csr_matmat order (ascending k)    */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t n, r0;
    const int64_t *ptr; const int32_t *idx; const double *val;    /* Phi CSR (sorted) */
    const int64_t *tptr; const int32_t *tidx; const double *tval; /* Phi^T CSR (sorted) */
    double *K; /* [r1-r0][n] */
} gram_ctx;
static void gram_range(void *ctx, int64_t b, int64_t e) {
    gram_ctx *g = (gram_ctx *)ctx;
    for (int64_t r = b; r < e; ++r) {
        int64_t i = g->r0 + r;
        double *row = g->K + r * g->n;
        for (int64_t j = 0; j < g->n; ++j) row[j] = 0.0;
        for (int64_t a = g->ptr[i]; a < g->ptr[i + 1]; ++a) {
            int32_t k = g->idx[a];
            double v = g->val[a];
            for (int64_t t = g->tptr[k]; t < g->tptr[k + 1]; ++t) row[g->tidx[t]] += v * g->tval[t];
        }
    }
}
ORACLE_API void oracle_gram_rows(int64_t n, const int64_t *ptr, const int32_t *idx, const double *val,
                                 const int64_t *tptr, const int32_t *tidx, const double *tval, int64_t r0, int64_t r1,
                                 double *K, int n_threads) {
    gram_ctx g = {n, r0, ptr, idx, val, tptr, tidx, tval, K};
    parallel_for(n_threads, r1 - r0, 4, gram_range, &g);
}

/* ------------------------------------------------------------------------- */
/* Laplacians                                                                 */
/* ------------------------------------------------------------------------- */
/* numpy pairwise_sum_DOUBLE (loops_utils.h.src), used by np.sum(W, axis=1) */
static double np_pairwise(const double *a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
    }
}
/* np.add.reduceat segment (scipy csr.sum(axis=1) via _minor_reduce): a0 + pairwise(rest) */
static double np_reduceat(const double *a, int64_t n) {
    if (n <= 0) return 0.0;
    return a[0] + np_pairwise(a + 1, n - 1);
}
ORACLE_API double oracle_np_pairwise(const double *a, int64_t n) { return np_pairwise(a, n); }
ORACLE_API double oracle_np_reduceat(const double *a, int64_t n) { return np_reduceat(a, n); }

/* scipy semantics (graph_utils.py:16-30).  Input CSR must be canonical
 * (sorted, no duplicates).  out arrays sized nnz + n.  Returns nnz. */
ORACLE_API int64_t oracle_laplacian_sparse(int64_t n, const int64_t *ip, const int32_t *ix, const double *dx,
                                           int64_t *op, int32_t *ox, double *odx, double *deg_out) {
    double *dinv = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        double d = np_reduceat(dx + ip[i], ip[i + 1] - ip[i]);
        if (deg_out) deg_out[i] = d;
        double v = 1.0 / sqrt(d);
        dinv[i] = isinf(v) ? 0.0 : v;
    }
    int64_t nnz = 0;
    op[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        double d = deg_out ? deg_out[i] : np_reduceat(dx + ip[i], ip[i + 1] - ip[i]);
        int64_t a = ip[i], ae = ip[i + 1];
        int diag_done = (d == 0.0); /* diags() drops a zero diagonal entry */
        /* merge row i of D (single entry (i, d)) with row i of A: D - A, zeros dropped */
        for (;;) {
            int64_t col;
            double v;
            if (!diag_done && (a >= ae || ix[a] > i)) { col = i; v = d; diag_done = 1; }
            else if (a < ae) {
                col = ix[a];
                if (!diag_done && col == i) { v = d - dx[a]; diag_done = 1; }
                else v = 0.0 - dx[a];
                ++a;
            } else break;
            if (v == 0.0) continue;
            /* D_inv_sqrt @ (D - A): row scale (dropped if zero), then @ D_inv_sqrt */
            if (dinv[i] == 0.0) continue;
            double t = dinv[i] * v;
            if (t == 0.0) continue;
            if (dinv[col] == 0.0) continue;
            double u = t * dinv[col];
            if (u == 0.0) continue;
            ox[nnz] = (int32_t)col;
            odx[nnz] = u;
            ++nnz;
        }
        op[i + 1] = nnz;
    }
    free(dinv);
    return nnz;
}

/* numpy semantics, dense W (n x n row-major):
 *   mode 0: graph_kernels/utils.py:21-26  (dinv = 0 where deg <= 0)
 *   mode 1: preprocessing/laplacian_np.py:13-20 (safe degrees: 1 where deg <= 0)
 *   mode 2: preprocessing/laplacian_np.py:32-34 (combinatorial D - W) */
ORACLE_API void oracle_laplacian_dense(int64_t n, const double *W, int32_t mode, double *Lout) {
    double *deg = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *dinv = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        deg[i] = np_pairwise(W + i * n, n);
        if (mode == 0) dinv[i] = deg[i] > 0 ? 1.0 / sqrt(deg[i]) : 0.0;
        else dinv[i] = 1.0 / sqrt(deg[i] > 0 ? deg[i] : 1.0);
    }
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double w = W[i * n + j];
            if (mode == 2) Lout[i * n + j] = (i == j ? deg[i] : 0.0) - w;
            else Lout[i * n + j] = (i == j ? 1.0 : 0.0) - (dinv[i] * w) * dinv[j];
        }
    free(deg);
    free(dinv);
}
