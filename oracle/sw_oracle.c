/*
 * sw_oracle.c -- CPU restatement of the reference's affine-gap Smith-Waterman
 * score path.  TEST INFRASTRUCTURE ONLY: the checker for the HIP engine.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path (libswmi355.so) never links it and
 * never falls back to it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - every known-answer test and seeded golden the reference holds
 *     (main.cpp:98-108, lazySmith.cpp:84-86, cudaSmithM.cu:278-363,
 *     cudaCompareSmith.cu:122-141, testLazyGPU_CPU.cu:231-243,
 *     CPUtesting.cpp:131-142) is checked in tests/test_oracle.py;
 *   - in this container the restatement is additionally compared against the
 *     reference's own main.cpp / lazySmith.cpp compiled from /root/reference
 *     into oracle/_ref/ (oracle/Makefile target `ref`).
 *
 * Functions and the reference lines they follow:
 *   swo_full      main.cpp:40-90   (three (m+1)x(n+1) int32 matrices, 0 borders,
 *                                    full max scan)
 *   swo_linear    lazySmith.cpp:15-42 (row state H_prev/H_curr/E/F; the lazy-F
 *                                    fix-up loop :43-62 never changes H, see
 *                                    DESIGN.md, so it is omitted)
 *   swo_slab      lazySmith.cpp:15-42 over one column slab with a left edge
 *                                    (the multi-GPU column-slab checker)
 *   swo_wavefront multi-threaded linear-space restatement (column blocks
 *                                    pipelined over row blocks); same cell
 *                                    recurrence as swo_linear, used to make
 *                                    large goldens in reasonable time
 *   swo_mt64_*    std::mt19937_64 (the generator of cudaSmithM.cu:200,
 *                                    cudaCompareSmith.cu:123, CPUtesting.cpp:131)
 *   swo_gen_*     uniform_int_distribution<int>(0,3) over "ACGT" as compiled by
 *                                    libstdc++ 11 (bits/uniform_int_dist.h
 *                                    _S_nd, Lemire): for a 64-bit URNG and range
 *                                    4 it returns the top two bits of each draw.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef struct {
    int match;      /* MATCH     main.cpp:22 */
    int mismatch;   /* MISMATCH  main.cpp:23 */
    int gap_init;   /* G_INIT    main.cpp:20 */
    int gap_ext;    /* G_EXT     main.cpp:21 */
} swo_params;

static inline int imax(int a, int b) { return a > b ? a : b; }

/* score(): raw byte equality, main.cpp:28-33 */
static inline int swo_s(const swo_params* p, unsigned char a, unsigned char b) {
    return a == b ? p->match : p->mismatch;
}

/*
 * Full-matrix fill exactly as main.cpp:40-90: q = seq1 (length n, columns j),
 * d = seq2 (length m, rows i).  Returns -1 if the matrices cannot be
 * allocated.  Memory: 3*(m+1)*(n+1)*4 bytes (the reference's own layout; the
 * vector<vector<int>> rows are replaced by one contiguous row-major block).
 */
int swo_full(const unsigned char* seq1, const unsigned char* seq2, int n, int m,
             const swo_params* p) {
    if (n < 0 || m < 0) return -1;
    const size_t cols = (size_t)n + 1, rows = (size_t)m + 1;
    int* E = (int*)malloc(rows * cols * sizeof(int));
    int* F = (int*)malloc(rows * cols * sizeof(int));
    int* H = (int*)malloc(rows * cols * sizeof(int));
    if (!E || !F || !H) { free(E); free(F); free(H); return -1; }
    /* borders: main.cpp:43-52 */
    for (size_t i = 0; i < rows; ++i) { E[i * cols] = F[i * cols] = H[i * cols] = 0; }
    for (size_t j = 0; j < cols; ++j) { E[j] = F[j] = H[j] = 0; }
    /* recurrence: main.cpp:54-66 */
    for (size_t i = 1; i < rows; ++i) {
        int* Ei = E + i * cols; int* Fi = F + i * cols; int* Hi = H + i * cols;
        const int* Fu = F + (i - 1) * cols; const int* Hu = H + (i - 1) * cols;
        const unsigned char di = seq2[i - 1];
        for (size_t j = 1; j < cols; ++j) {
            Ei[j] = imax(Ei[j - 1] - p->gap_ext, Hi[j - 1] - p->gap_init);
            Fi[j] = imax(Fu[j] - p->gap_ext, Hu[j] - p->gap_init);
            int t1 = imax(Fi[j], Ei[j]);
            int t2 = imax(0, Hu[j - 1] + swo_s(p, seq1[j - 1], di));
            Hi[j] = imax(t1, t2);
        }
    }
    /* max scan over all of H including borders: main.cpp:82-87 */
    int best = 0;
    for (size_t k = 0; k < rows * cols; ++k) best = imax(best, H[k]);
    free(E); free(F); free(H);
    return best;
}

/*
 * Linear-space restatement of lazySmith.cpp:15-42 (row state of n+1 ints).
 * Rows [row0, row1) only when row0/row1 bracket a prefix (used by the CPU
 * baseline timing on a bounded sample); pass 0/m for the whole pair.
 */
int swo_linear_rows(const unsigned char* seq1, const unsigned char* seq2, int n, int m,
                    const swo_params* p, int row_count) {
    if (n <= 0 || m <= 0) return 0;
    if (row_count > m || row_count < 0) row_count = m;
    int* Hp = (int*)calloc((size_t)n + 1, sizeof(int));
    int* Hc = (int*)calloc((size_t)n + 1, sizeof(int));
    int* F = (int*)calloc((size_t)n + 1, sizeof(int));
    if (!Hp || !Hc || !F) { free(Hp); free(Hc); free(F); return -1; }
    int best = 0;
    for (int i = 1; i <= row_count; ++i) {
        const unsigned char di = seq2[i - 1];
        int e = 0;          /* E[i][0] = 0 */
        Hc[0] = 0;
        for (int j = 1; j <= n; ++j) {
            e = imax(e - p->gap_ext, Hc[j - 1] - p->gap_init);
            F[j] = imax(F[j] - p->gap_ext, Hp[j] - p->gap_init);
            int h = Hp[j - 1] + swo_s(p, seq1[j - 1], di);
            h = imax(h, e); h = imax(h, F[j]); h = imax(h, 0);
            Hc[j] = h;
            best = imax(best, h);
        }
        int* t = Hp; Hp = Hc; Hc = t;
    }
    free(Hp); free(Hc); free(F);
    return best;
}

int swo_linear(const unsigned char* seq1, const unsigned char* seq2, int n, int m,
               const swo_params* p) {
    return swo_linear_rows(seq1, seq2, n, m, p, m);
}

/*
 * One column slab of the same linear-space recurrence (lazySmith.cpp:15-42
 * with a left edge): columns seq1[0..n) of a pair whose column just left of
 * the slab ended row i with H = in_h[i-1], E = in_e[i-1] (NULL: the matrix
 * border, 0, main.cpp:43-52).  Writes the slab's last column to out_h / out_e
 * (if non-NULL) and returns the max H over the slab's cells.  Chaining slabs
 * left to right reproduces swo_linear exactly (the checker of the multi-GPU
 * column-slab path).
 */
int swo_slab(const unsigned char* seq1, const unsigned char* seq2, int n, int m, const swo_params* p,
             const int* in_h, const int* in_e, int* out_h, int* out_e) {
    if (n <= 0 || m <= 0) return 0;
    int* Hp = (int*)calloc((size_t)n + 1, sizeof(int));
    int* Hc = (int*)calloc((size_t)n + 1, sizeof(int));
    int* F = (int*)calloc((size_t)n + 1, sizeof(int));
    if (!Hp || !Hc || !F) { free(Hp); free(Hc); free(F); return -1; }
    int best = 0;
    for (int i = 1; i <= m; ++i) {
        const unsigned char di = seq2[i - 1];
        int e = in_e ? in_e[i - 1] : 0;    /* E[i][left] */
        Hc[0] = in_h ? in_h[i - 1] : 0;    /* H[i][left]; Hp[0] holds H[i-1][left] */
        for (int j = 1; j <= n; ++j) {
            e = imax(e - p->gap_ext, Hc[j - 1] - p->gap_init);
            F[j] = imax(F[j] - p->gap_ext, Hp[j] - p->gap_init);
            int h = Hp[j - 1] + swo_s(p, seq1[j - 1], di);
            h = imax(h, e); h = imax(h, F[j]); h = imax(h, 0);
            Hc[j] = h;
            best = imax(best, h);
        }
        if (out_h) out_h[i - 1] = Hc[n];
        if (out_e) out_e[i - 1] = e;
        int* t = Hp; Hp = Hc; Hc = t;
    }
    free(Hp); free(Hc); free(F);
    return best;
}

/* ---------------------------------------------------------------------------
 * Multi-threaded wavefront restatement (same recurrence as swo_linear).
 * Thread t owns column block t; the matrix is swept in row blocks of RB rows.
 * Block (rb, t) needs (rb, t-1) [left column: H,E per row] and (rb-1, t)
 * [own row state].  Progress is published per thread through a counter.
 * ------------------------------------------------------------------------- */
typedef struct {
    const unsigned char *s1, *s2;
    int n, m, nthreads, rb;
    const swo_params* p;
    volatile int* progress;      /* row blocks finished, per thread */
    int* colH;                   /* [nthreads][m] right-edge H of each block */
    int* colE;                   /* [nthreads][m] right-edge E of each block */
    int* best;                   /* per thread */
} swo_wf_shared;

typedef struct { swo_wf_shared* sh; int t; } swo_wf_arg;

static void* swo_wf_worker(void* vp) {
    swo_wf_arg* a = (swo_wf_arg*)vp;
    swo_wf_shared* sh = a->sh;
    const int t = a->t, T = sh->nthreads, n = sh->n, m = sh->m;
    const int c0 = (int)((long long)n * t / T), c1 = (int)((long long)n * (t + 1) / T);
    const int w = c1 - c0;
    const swo_params* p = sh->p;
    int* Hp = (int*)calloc((size_t)w + 1, sizeof(int));
    int* Hc = (int*)calloc((size_t)w + 1, sizeof(int));
    int* F = (int*)calloc((size_t)w + 1, sizeof(int));
    int best = 0;
    int diag_prev = 0;             /* H[i-1][c0] (left neighbour column, prev row) */
    const int nrb = (m + sh->rb - 1) / sh->rb;
    for (int b = 0; b < nrb; ++b) {
        const int r0 = b * sh->rb, r1 = (r0 + sh->rb < m) ? r0 + sh->rb : m;
        if (t > 0) { while (__atomic_load_n(&sh->progress[t - 1], __ATOMIC_ACQUIRE) <= b) { } }
        for (int i = r0 + 1; i <= r1; ++i) {
            const unsigned char di = sh->s2[i - 1];
            int hl = 0, e = 0;
            if (t > 0) { hl = sh->colH[(size_t)(t - 1) * m + (i - 1)]; e = sh->colE[(size_t)(t - 1) * m + (i - 1)]; }
            Hc[0] = hl;
            Hp[0] = diag_prev;
            for (int j = 1; j <= w; ++j) {
                e = imax(e - p->gap_ext, Hc[j - 1] - p->gap_init);
                F[j] = imax(F[j] - p->gap_ext, Hp[j] - p->gap_init);
                int h = Hp[j - 1] + swo_s(p, sh->s1[c0 + j - 1], di);
                h = imax(h, e); h = imax(h, F[j]); h = imax(h, 0);
                Hc[j] = h;
                if (h > best) best = h;
            }
            if (t < T - 1) {
                sh->colH[(size_t)t * m + (i - 1)] = Hc[w];
                sh->colE[(size_t)t * m + (i - 1)] = e;
            }
            diag_prev = hl;
            int* tmp = Hp; Hp = Hc; Hc = tmp;
        }
        __atomic_store_n(&sh->progress[t], b + 1, __ATOMIC_RELEASE);
    }
    sh->best[t] = best;
    free(Hp); free(Hc); free(F);
    return NULL;
}

int swo_wavefront(const unsigned char* seq1, const unsigned char* seq2, int n, int m,
                  const swo_params* p, int nthreads) {
    if (n <= 0 || m <= 0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n) nthreads = n;
    if (nthreads == 1) return swo_linear(seq1, seq2, n, m, p);
    swo_wf_shared sh;
    sh.s1 = seq1; sh.s2 = seq2; sh.n = n; sh.m = m; sh.nthreads = nthreads; sh.p = p;
    sh.rb = 256;
    sh.progress = (volatile int*)calloc((size_t)nthreads, sizeof(int));
    sh.colH = (int*)malloc((size_t)nthreads * (size_t)m * sizeof(int));
    sh.colE = (int*)malloc((size_t)nthreads * (size_t)m * sizeof(int));
    sh.best = (int*)calloc((size_t)nthreads, sizeof(int));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    swo_wf_arg* args = (swo_wf_arg*)malloc(sizeof(swo_wf_arg) * (size_t)nthreads);
    if (!sh.progress || !sh.colH || !sh.colE || !sh.best || !th || !args) return -1;
    for (int t = 0; t < nthreads; ++t) { args[t].sh = &sh; args[t].t = t; pthread_create(&th[t], NULL, swo_wf_worker, &args[t]); }
    int best = 0;
    for (int t = 0; t < nthreads; ++t) { pthread_join(th[t], NULL); best = imax(best, sh.best[t]); }
    free((void*)sh.progress); free(sh.colH); free(sh.colE); free(sh.best); free(th); free(args);
    return best;
}

/* Batch helper: one pair per thread (CPU baseline for the batched configs). */
typedef struct {
    const unsigned char* const* a; const int* alen;
    const unsigned char* const* b; const int* blen;
    int npairs; const swo_params* p; int* out; int next; int full;
} swo_batch_shared;

static void* swo_batch_worker(void* vp) {
    swo_batch_shared* sh = (swo_batch_shared*)vp;
    for (;;) {
        int k = __atomic_fetch_add(&sh->next, 1, __ATOMIC_RELAXED);
        if (k >= sh->npairs) break;
        sh->out[k] = sh->full ? swo_full(sh->a[k], sh->b[k], sh->alen[k], sh->blen[k], sh->p)
                              : swo_linear(sh->a[k], sh->b[k], sh->alen[k], sh->blen[k], sh->p);
    }
    return NULL;
}

int swo_batch(const unsigned char* const* a, const int* alen, const unsigned char* const* b,
              const int* blen, int npairs, const swo_params* p, int* out, int nthreads, int full) {
    swo_batch_shared sh = {a, alen, b, blen, npairs, p, out, 0, full};
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    if (!th) return -1;
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, swo_batch_worker, &sh);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
    return 0;
}

/* ---------------------------------------------------------------------------
 * std::mt19937_64 (w=64 n=312 m=156 r=31 a=0xb5026f5aa96619e9 u=29
 * d=0x5555555555555555 s=17 b=0x71d67fffeda60000 t=37 c=0xfff7eee000000000
 * l=43 f=6364136223846793005), as used by cudaSmithM.cu:200.
 * ------------------------------------------------------------------------- */
typedef struct { uint64_t mt[312]; int idx; } swo_mt64;

void swo_mt64_seed(swo_mt64* g, uint64_t seed) {
    g->mt[0] = seed;
    for (int i = 1; i < 312; ++i)
        g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
    g->idx = 312;
}

uint64_t swo_mt64_next(swo_mt64* g) {
    if (g->idx >= 312) {
        const uint64_t UM = 0xFFFFFFFF80000000ULL, LM = 0x7FFFFFFFULL, A = 0xB5026F5AA96619E9ULL;
        for (int i = 0; i < 312; ++i) {
            uint64_t x = (g->mt[i] & UM) | (g->mt[(i + 1) % 312] & LM);
            uint64_t xa = x >> 1;
            if (x & 1ULL) xa ^= A;
            g->mt[i] = g->mt[(i + 156) % 312] ^ xa;
        }
        g->idx = 0;
    }
    uint64_t x = g->mt[g->idx++];
    x ^= (x >> 29) & 0x5555555555555555ULL;
    x ^= (x << 17) & 0x71D67FFFEDA60000ULL;
    x ^= (x << 37) & 0xFFF7EEE000000000ULL;
    x ^= (x >> 43);
    return x;
}

static const char swo_nts[4] = {'A', 'C', 'G', 'T'};

/* uniform_int_distribution<int>(0,3)(mt19937_64): Lemire _S_nd with range 4
 * -> (draw * 4) >> 64 == draw >> 62 (threshold -4 % 4 == 0, never rejects). */
static inline unsigned char swo_base(swo_mt64* g) { return (unsigned char)swo_nts[swo_mt64_next(g) >> 62]; }

/* Interleaved pair generator: a[i] then b[i] per position
 * (cudaSmithM.cu:209-212, cudaCompareSmith.cu:136-139, testLazyGPU_CPU.cu:236-239). */
void swo_gen_pair(uint64_t seed, int len, unsigned char* a, unsigned char* b) {
    swo_mt64 g; swo_mt64_seed(&g, seed);
    for (int i = 0; i < len; ++i) { a[i] = swo_base(&g); b[i] = swo_base(&g); }
}

/* Continuing stream form: draws from an existing generator (multi-pair
 * generators that share one engine across lengths, e.g. cudaCompareSmith.cu:134). */
void swo_gen_pair_stream(swo_mt64* g, int len, unsigned char* a, unsigned char* b) {
    for (int i = 0; i < len; ++i) { a[i] = swo_base(g); b[i] = swo_base(g); }
}

/* Sequential generator: whole sequence from the stream (CPUtesting.cpp:122-128). */
void swo_gen_seq_stream(swo_mt64* g, int len, unsigned char* s) {
    for (int i = 0; i < len; ++i) s[i] = swo_base(g);
}

size_t swo_mt64_size(void) { return sizeof(swo_mt64); }
