/* Sanitizer driver for the oracle restatement (test infrastructure; built by
 * `make -C oracle asan` with -fsanitize=address,undefined together with
 * oracle/sw_oracle.c and run by tests/test_sanitize.py).
 *
 * stdin: one case per line, "MATCH MISMATCH G_INIT G_EXT HEX(seq1) HEX(seq2)"
 * ("-" for an empty sequence).  stdout: one line per case,
 *   "<full> <linear> <wavefront, 3 threads> <slab chain, 3 slabs> <batch, 2 threads>"
 * -- every engine of sw_oracle.c on the same pair.  Sanitizer findings abort. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int match, mismatch, gap_init, gap_ext; } swo_params;
int swo_full(const unsigned char*, const unsigned char*, int, int, const swo_params*);
int swo_linear(const unsigned char*, const unsigned char*, int, int, const swo_params*);
int swo_wavefront(const unsigned char*, const unsigned char*, int, int, const swo_params*, int);
int swo_slab(const unsigned char*, const unsigned char*, int, int, const swo_params*, const int*, const int*, int*, int*);
int swo_batch(const unsigned char* const*, const int*, const unsigned char* const*, const int*, int,
              const swo_params*, int*, int, int);

static int unhex(const char* h, unsigned char* out) {
    if (strcmp(h, "-") == 0) return 0;
    int n = (int)strlen(h) / 2;
    for (int i = 0; i < n; ++i) {
        unsigned v = 0;
        if (sscanf(h + 2 * i, "%2x", &v) != 1) return -1;
        out[i] = (unsigned char)v;
    }
    return n;
}

/* columns [0, n) cut into `k` slabs chained through their (H, E) edges */
static int slab_chain(const unsigned char* a, const unsigned char* b, int n, int m, const swo_params* p, int k) {
    if (n <= 0 || m <= 0) return 0;
    int* eh = (int*)malloc(sizeof(int) * (size_t)m);
    int* ee = (int*)malloc(sizeof(int) * (size_t)m);
    int* oh = (int*)malloc(sizeof(int) * (size_t)m);
    int* oe = (int*)malloc(sizeof(int) * (size_t)m);
    int best = 0, have = 0;
    for (int s = 0; s < k; ++s) {
        const int lo = (int)((long long)n * s / k), hi = (int)((long long)n * (s + 1) / k);
        if (hi <= lo) continue;
        const int v = swo_slab(a + lo, b, hi - lo, m, p, have ? eh : NULL, have ? ee : NULL, oh, oe);
        if (v > best) best = v;
        memcpy(eh, oh, sizeof(int) * (size_t)m);
        memcpy(ee, oe, sizeof(int) * (size_t)m);
        have = 1;
    }
    free(eh); free(ee); free(oh); free(oe);
    return best;
}

int main(void) {
    static char line[1 << 20];
    static unsigned char a[1 << 18], b[1 << 18];
    static char ha[1 << 19], hb[1 << 19];
    while (fgets(line, sizeof line, stdin)) {
        swo_params p;
        if (sscanf(line, "%d %d %d %d %524287s %524287s", &p.match, &p.mismatch, &p.gap_init, &p.gap_ext, ha, hb) != 6)
            continue;
        const int n = unhex(ha, a), m = unhex(hb, b);
        if (n < 0 || m < 0) { printf("bad\n"); continue; }
        /* exact-size heap copies, so an out-of-bounds read of a sequence is caught */
        unsigned char* A = (unsigned char*)malloc((size_t)n + 1);
        unsigned char* B = (unsigned char*)malloc((size_t)m + 1);
        memcpy(A, a, (size_t)n);
        memcpy(B, b, (size_t)m);
        const unsigned char* pa[1] = {A};
        const unsigned char* pb[1] = {B};
        int out[1] = {-7};
        swo_batch(pa, &n, pb, &m, 1, &p, out, 2, 0);
        printf("%d %d %d %d %d\n", swo_full(A, B, n, m, &p), swo_linear(A, B, n, m, &p),
               swo_wavefront(A, B, n, m, &p, 3), slab_chain(A, B, n, m, &p, 3), out[0]);
        free(A);
        free(B);
    }
    return 0;
}
