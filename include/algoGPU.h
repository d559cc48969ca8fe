/*
 * algoGPU.h -- drop-in C-ABI of the MI355X (gfx950) Smith-Waterman score engine
 * (libswmi355.so).  Link this library in place of the reference's
 * simpleGPU.o / cudaLazy.o / cudaSmithM.o (reference Makefile2:15) and keep the
 * reference's TestFileWithGPU.cpp and CPU sources unchanged.
 *
 * Semantics shared by every entry point:
 *   - the return value is the best local-alignment score max H >= 0 of the
 *     affine-gap recurrence of main.cpp:54-66 (E from the left, F from above,
 *     borders 0, score byte equality main.cpp:28-33), bit-exact;
 *   - seq1 has length n (len1), seq2 has length m (len2); the score is
 *     symmetric; any byte values are allowed (an {A,C,G,T}-only input takes
 *     the 2-bit profile path, anything else the raw-byte path);
 *   - n == 0 or m == 0 returns 0 (main.cpp:74-90 with empty loops);
 *   - the call is synchronous and re-entrant per host thread; the caller owns
 *     the host buffers, which are only read; device memory and the HIP stream
 *     are cached per (thread, device) and are not observable;
 *   - on an internal HIP failure, an invalid argument or unsupported scoring
 *     constants the return value is -1 and sw_last_error() says why (the
 *     reference had no error channel; cudaSmithM.cu:168-173 returned a
 *     partial score instead).
 *   - the scoring constants default to the reference's
 *     MATCH=1, MISMATCH=-1, G_INIT=1, G_EXT=1 (main.cpp:20-23) and can be
 *     changed with sw_set_params().
 */
#ifndef SWMI355_ALGOGPU_H
#define SWMI355_ALGOGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- the reference's algoGPU.h:5-9 surface (exact signatures) ---------------- */

/* replaces simpleGPU.cu:109-163 (reference: one launch + device sync per
 * anti-diagonal, only correct for len2 <= len1 and N < 46341). */
int SequentialSmithWatermanScoreGPU(unsigned char* seq1, unsigned char* seq2, int len1, int len2);

/* replaces cudaLazy.cu:58-99 (reference: full-matrix anti-diagonal kernel). */
int SmithWatermanLazyGPU(const unsigned char* seq1, const unsigned char* seq2, int n, int m);

/* replaces cudaSmithM.cu:128-189 (reference: full-matrix, no per-diagonal sync). */
int SmithWatermanScoreCUDA(const unsigned char* seq1, const unsigned char* seq2, int n, int m);

/* replaces SmithDiagonalGPUrefactored.cu:174-230 (extern "C" but never declared
 * in the reference's algoGPU.h).  That kernel is LINEAR-gap (gap = G_INIT per
 * residue, SmithDiagonalGPU.cu:59-66); this entry keeps its semantics: it is
 * the affine engine with G_EXT := G_INIT, which is exactly the linear model. */
int SmithDiagonalGPU(unsigned char* seq1, unsigned char* seq2, int n, int m);

/* ---- extensions (no reference counterpart) ---------------------------------- */

/* Scoring constants for later calls from ANY thread (process-wide).
 * Supported: 0 <= gap_init, gap_ext <= 1<<20; -127 <= mismatch <= 0;
 * mismatch <= match <= 127.  Returns 0, or -1 if unsupported. */
int sw_set_params(int match, int mismatch, int gap_init, int gap_ext);
void sw_get_params(int* match, int* mismatch, int* gap_init, int* gap_ext);

/* One pair with explicit constants (does not change the process-wide ones). */
int sw_score_params(const unsigned char* seq1, const unsigned char* seq2, int n, int m,
                    int match, int mismatch, int gap_init, int gap_ext);

/* Batch of independent pairs (host buffers); scores_out[k] = score(a[k], b[k]).
 * One launch for the whole batch.  Returns 0 or -1. */
int sw_score_batch(const unsigned char* const* a, const int* alen,
                   const unsigned char* const* b, const int* blen,
                   int npairs, int* scores_out);

/* The same batch over the first ngpus visible GPUs of the node (SURVEY.md 8(b), configs
 * C3/C4): pairs are cut into contiguous shards (sw_batch_shard: sizes differ by at most
 * one), each scored by its own host thread and stream on its own device, and the int32
 * scores of devices 1..ngpus-1 are gathered to device 0 over RCCL (ncclSend/ncclRecv in
 * one group; RCCL is loaded at the first call with ngpus > 1) -- the only exchange, no
 * data-path collective.  Synchronous like the reference ABI; scores_out in pair order.
 * Returns 0, or -1 with sw_last_error() (e.g. ngpus above the visible devices).
 * Callers: the reference harness's batched loops (TestFileWithGPU.cpp:82-94).
 * UNVERIFIED ON HARDWARE for ngpus > 1: the build's GPU boxes have one GPU, so the RCCL
 * branch has only run through its host-side plan (sw_batch_gather_plan, CPU-tested).
 * Lifetime: the first call starts one host worker thread per device used; the threads are
 * detached and live for the rest of the process (never joined), as do their engine contexts,
 * streams and the RCCL communicators. */
int sw_score_batch_multi(const unsigned char* const* a, const int* alen,
                         const unsigned char* const* b, const int* blen,
                         int npairs, int* scores_out, int ngpus);
/* Shard [*lo, *hi) of rank `rank` of ngpus for npairs pairs (no GPU call).  0 or -1. */
int sw_batch_shard(int npairs, int ngpus, int rank, int* lo, int* hi);
/* The gather sw_score_batch_multi runs (no GPU call): count[r] scores of device r land in
 * device 0's gather buffer at offset[r] (r = 0: the local copy; r > 0: one ncclSend from
 * device r matched by one ncclRecv on device 0, skipped when count[r] == 0).  count and
 * offset hold ngpus ints.  0 or -1. */
int sw_batch_gather_plan(int npairs, int ngpus, int* count, int* offset);

/* Batch whose sequences are already resident in device memory (one arena,
 * byte offsets per sequence).  Offsets/lengths are HOST arrays; d_scores is a
 * device array of npairs ints.  Asynchronous on `stream` (a hipStream_t; NULL =
 * the engine's own stream, and then the call is synchronous).
 * flags: SW_FLAG_DNA asserts every byte is in {A,C,G,T} (skips the alphabet
 * scan), SW_FLAG_BYTES forces the raw-byte path.  After an asynchronous call,
 * sw_stream_status(stream) synchronises and reports kernel-side failures. */
#define SW_FLAG_DNA   1
#define SW_FLAG_BYTES 2
int sw_score_batch_device(const unsigned char* d_arena,
                          const int64_t* a_off, const int* alen,
                          const int64_t* b_off, const int* blen,
                          int npairs, int* d_scores, int flags, void* stream);
int sw_stream_status(void* stream);

/* ---- one pair split into column slabs across GPUs (no reference counterpart;
 * the C5 pair N = 2^20 over the GPUs of a node) ---------
 * Rank r of R scores columns [bounds[r], bounds[r+1]) of seq1 against all of
 * seq2.  Its left edge (H - G_INIT, E - G_EXT of the previous slab's last
 * column, one 16-byte tagged granule per row) is written straight into rank
 * r's inflow buffer by rank r-1's kernel, through an IPC mapping of that
 * buffer (xGMI stores, no host staging); the pair's score is the max of the
 * R slab maxima (an all-reduce(MAX) of one int).  dist.ColumnSlabs drives it.
 *
 * sw_slab_bounds: R+1 column bounds; every slab but the last is a multiple of
 *   the kernel's column quantum (returned, > 0; 126 at two flow2 columns per lane,
 *   63 at one, 64*W for chain / flow).  flags must say
 *   SW_FLAG_DNA or SW_FLAG_BYTES (all ranks must plan the same kernel).
 * sw_score_slab_device: one slab, sequences resident in device memory:
 *   columns d_arena[col_off, col_off+n), rows d_arena[row_off, row_off+m).
 *   d_inflow / d_outflow: granule buffers of m rows (NULL = the matrix border
 *   / the pair's last column); epoch != 0, the same on every rank and fresh
 *   for every launch over the same buffers.  *d_score = this slab's max H.
 *   Asynchronous on `stream` as sw_score_batch_device.
 * sw_slab_alloc: a zeroed inflow buffer of m granules; returns 1 (fine-grained
 *   memory) or 2 (device memory), -1 on error; ipc_handle (SW_IPC_HANDLE_BYTES,
 *   may be NULL) receives its hipIpcMemHandle_t for the writing rank.  An exported
 *   buffer (ipc_handle != NULL: the edge another GPU writes) must be fine-grained:
 *   without it the call fails (-1) unless option "slab_plain" is 1.
 * sw_ipc_open / sw_ipc_close: map / unmap another process's buffer. */
#define SW_IPC_HANDLE_BYTES 64
int sw_slab_bounds(long long n, int m, int nslabs, int flags, long long* bounds);
int sw_score_slab_device(const unsigned char* d_arena, int64_t col_off, int n, int64_t row_off, int m,
                         void* d_inflow, void* d_outflow, unsigned epoch, int* d_score, int flags, void* stream);
int sw_slab_alloc(int m, void** d_buf, void* ipc_handle);
int sw_slab_free(void* d_buf);
int sw_ipc_open(const void* ipc_handle, void** d_ptr);
int sw_ipc_close(void* d_ptr);

/* ---- FASTA databases: query x database scoring (no reference counterpart;
 * SURVEY.md 8(f) f-4, the makedb / align workflow of the reference's timing.sh:3-8
 * around the external CUDASW++4 tool, Makefile_CUDASW4.mak:44-56) ------------
 * Scores are this engine's (byte equality MATCH/MISMATCH, affine gaps,
 * main.cpp:28-66), not CUDASW++'s BLOSUM62.  A database holds its residues
 * host-side and, after the first search, once in device memory (one arena,
 * per device); searches launch one batch over all of its records, longest
 * first, and return the scores in record order.
 *
 * sw_db_open: a FASTA file ('>' header lines; sequence lines of any width,
 *   whitespace and '\r' dropped, bytes otherwise kept as they are; ';' comment
 *   lines skipped; records may be empty) or a file written by sw_db_save.
 *   NULL on error (sw_last_error).
 * sw_db_from_fasta: the same parse over a buffer in memory.
 * sw_db_save: the binary database (the "makedb" step), 0 or -1.
 * sw_db_count / sw_db_residues: records, total residues.
 * sw_db_record: record i's residues, length and header (pointers owned by db).
 * sw_db_search: scores_out[i] = score(query, record i) for every record; the
 *   query is a byte string of qlen bytes.  Synchronous; 0 or -1.
 * sw_db_search_db: scores_out[q * count(db) + i] for every record q of queries.
 * sw_db_close: frees host and device memory. */
typedef struct sw_db sw_db;
sw_db* sw_db_open(const char* path);
sw_db* sw_db_from_fasta(const char* text, long long nbytes);
int sw_db_save(const sw_db* db, const char* path);
int sw_db_count(const sw_db* db);
long long sw_db_residues(const sw_db* db);
int sw_db_record(const sw_db* db, int i, const unsigned char** seq, int* len, const char** header);
int sw_db_search(sw_db* db, const unsigned char* query, int qlen, int* scores_out);
int sw_db_search_db(sw_db* db, const sw_db* queries, int* scores_out);
void sw_db_close(sw_db* db);

/* Tuning knobs (process-wide).  Keys:
 *   "W"        columns per lane: 0 = auto, 1, 2, 4, 8
 *   "C"        rows per strip hand-off chunk: 0 = auto, 16, 32, 64
 *   "bytes"    1 = force the raw-byte path
 *   "timeout"  seconds before a stalled strip hand-off gives up (default 30)
 *   "blocks"   0 = auto persistent grid, else workgroups per launch
 *   "orient"   0 = auto, 1 = seq1 spread across lanes, 2 = seq2 across lanes
 *   "mode"     -1 = auto, 0 = independent strip waves, 1 = workgroup per pair,
 *              2 = lock-step strip groups (single long pairs),
 *              3 = packed 16-bit pair duos (batches with scores < 65535: DNA, and any bytes
 *                  when MISMATCH < 0 and MATCH - MISMATCH <= 127, option duo_raw),
 *              4 = free-running strip groups, rows staged in LDS (long DNA pairs),
 *              5 = the flow2 / flow3 wavefront step (DNA, one column per lane or more, chunked
 *                  LDS / granule hand-offs; the automatic plan for single long pairs, column
 *                  slabs and batches whose scores need int32)
 *   "duo16"    1 = (default) packed duos take max3 through v_pk_maximum3_f16 when every
 *              value stays below 0x7C00 (MATCH*(min(n,m)+1) <= 31743), 0 = u16 max only
 *   "linear"   -1 = (default) the exact linear-gap step when G_INIT == G_EXT
 *              (flow2 C = 32 or 64, f16 duos), 0 = always the affine step
 *   "f2w"      flow2 columns per lane: 0 = (default) two whenever the linear-gap
 *              step runs (three in flow3 ring mode: C5, column slabs), one otherwise;
 *              1 = always one; 2 = two (linear-gap step only); 3 = three where ring mode runs;
 *              4 = four / five in ring mode for one pair, every strip group resident in one round
 *              (sw_flow3r45_kernel; measured slower than three on C5, so never automatic)
 *   "f3pool"   1 = flow3 staged launches on the loops without the I/O rotation (measured
 *              slower; default 0)
 *   "ring"     -1 = (default) ring edges for a single flow2 pair whose linear edges
 *              would exceed 1 GB, 0 = never, 1 = always (one pair per launch)
 *   "ring_rows" rows per within-round ring, a power of two in [512, 2^20] (4096)
 *   "f2_wgs"   flow2 streamed kernel: workgroups per CU, 0 = auto, 1..4 (ring mode:
 *              lowered to what the runtime reports resident for its kernel)
 *   "f2stream" 1 = flow2 streams the row codes even when they fit in LDS (tests)
 *   "f2pwg"    DNA batches whose scores need int32 (no 16-bit duos): -1 = (default) the
 *              flow2 step with a pair per workgroup when its constants fit, 0 = never
 *              (the pair-per-workgroup strip kernel), 1 = also for a forced mode 5 batch
 *   "f3"       1 = (default) a two-column linear-gap flow2 launch runs the flow3 kernel
 *              (hand-scheduled chunk loops): staged codes at C = 32 / 16 (C2), ring edges at
 *              C = 64 (C5); 0 = the compiled flow2 kernel
 *   "f3hl"     1 = (default) flow3 staged launches run 32-row chunks whose in-workgroup links
 *              hand off every half chunk (16 rows); 0 = whole-chunk links at C = 16 (auto C)
 *   "f3rhl"    1 = flow3 ring launches (C = 64) with half-chunk in-workgroup links (32 rows),
 *              0 = (default) whole-chunk links (measured faster on C5)
 *   "f3a"      1 = (default) the general affine step runs on flow3 (staged: sw_flow3a_kernel, one
 *              column per lane, C2 with G_INIT != G_EXT; ring: sw_flow3ra(3)_kernel, C5), 0 = flow2
 *   "f3pwg"    1 = (default) DNA batches on a pair-per-workgroup plan (scores that need int32, or 1-2
 *              pairs per CU) run flow3's three-column ring step (sw_flow3r3p / ra3p_kernel), 0 = flow2's
 *   "f3slab"   1 = (default) column slabs run flow3's ring kernel with slab roles
 *              (sw_flow3rs / ras / r3s / ra3s_kernel), 0 = flow2's slab kernel
 *   "duo_lds"  1 = (default) duo batches at C = 64 hand strip edges on in LDS when a round's
 *              rows fit (m <= 16384 linear-gap step, 8192 affine), 0 = through HBM granules
 *   "duo_roles" 1 = (default) the two duo LDS workgroups of a CU take complementary strip roles
 *              on each SIMD (one wave starts early, one late), 0 = roles by wave index
 *   "duo_tab"  1 = (default) the duo LDS kernel reads its row codes from an LDS table (4 or 8
 *              columns per lane, when the table and the wrap buffer fit two workgroups per CU
 *              and the duos run in one pass at that), 2 = whenever it fits, 0 = the codes travel
 *              lane to lane by DPP
 *   "hep"      1 = (default) one pair over at most seven byte values not all in {A,C,G,T} (ACGTN,
 *              lower case, RNA) runs flow3's staged kernels with 3-bit row symbols (sw_flow3h /
 *              sw_flow3ah_kernel; rows that fit in LDS, else the byte path), 0 = the byte path
 *   "duo_raw"  1 = (default) byte batches (any byte outside {A,C,G,T}: protein, N, lower case) run the
 *              duo kernels with the penalty from the bytes (one XOR and one v_pk_min_u16 per position
 *              for the DNA step's v_perm_b32; needs MISMATCH < 0, MATCH - MISMATCH <= 127), 0 = the
 *              byte-path strip kernels
 *   "duo_prio" -1 = (default) auto: 17 for the duo LDS kernel with the row-code table, else 0;
 *              k in 6..20: a CU's two duo workgroups take turns at issue priority (s_setprio) in
 *              slices of 2^k ticks (10 ns) of the clock from their start; 0 = off (timing only)
 *   "slab_plain" 1 = an exported slab buffer may fall back to plain device memory (one-GPU
 *              tests only; cross-GPU edges need fine-grained memory), 0 = (default) refuse
 *   "trace"    device address of a 16 x u64 per-strip trace buffer, 0 = off (tools)
 *   "stall_item" tests only: flow2's compute waves skip this item (its edges are never
 *              published, so its consumers' bounded waits expire: ERR_TIMEOUT); -1 = (default) none
 * Returns 0, or -1 for an unknown key / bad value. */
int sw_set_option(const char* key, long long value);
long long sw_get_option(const char* key);

/* Details of the last launch made by this thread (for the harness / bench). */
typedef struct {
    float kernel_ms;        /* HIP-event time of the score kernel alone */
    float total_ms;         /* wall time of the whole call incl. copies */
    long long cells;        /* sum of n*m over the launched pairs */
    int W, C, dna, blocks, waves_per_cu, items;
    long long boundary_bytes;
    int mode;
    int variant;            /* bit 0: duo max3 via v_pk_maximum3_f16; bit 1: flow2 streams row codes;
                               bit 2: flow2 ring edges; bit 3: the linear-gap step;
                               bit 4: flow2 two columns per lane; bit 5: flow2 pair per workgroup;
                               bit 6: the flow3 kernel (sw_flow3.hip);
                               bit 7: duo strip hand-offs in LDS (no boundary buffers);
                               bit 8: duo row codes from an LDS table;
                               bit 9: flow3 half-chunk LDS links (option f3hl);
                               bit 10: the general affine step on flow3 (sw_flow3a / sw_flow3ra kernels);
                               bit 11: a flow3 column slab (peer-edge roles, sw_flow3*s_kernel);
                               bit 12: flow3 pool loops (option f3pool);
                               bit 13: flow3 ring at three columns per lane (sw_flow3r3 / ra3 kernels);
                               bit 14: flow3 ring at four / five columns per lane (sw_flow3r45_kernel);
                               bit 15: flow3 three-column ring step with a pair per workgroup
                                       (sw_flow3r3p_kernel / sw_flow3ra3p_kernel: int32 batches);
                               bit 16: a pair over up to seven byte values on flow3's staged kernels
                                       (option hep; dna = 2 then) */
} sw_stats;
int sw_last_stats(sw_stats* out);

const char* sw_last_error(void);
int sw_version(void);

/* Synthetic {A,C,G,T} inputs (not on the score path): std::mt19937_64(seed),
 * a[i] then b[i] per position -- the generator of cudaSmithM.cu:200-212. */
void sw_gen_pair(uint64_t seed, int len, unsigned char* a, unsigned char* b);
/* npairs pairs, pair k seeded seed_base+k, laid out [a_0|b_0|a_1|b_1|...]. */
void sw_gen_batch(uint64_t seed_base, int npairs, int len, unsigned char* arena);

#ifdef __cplusplus
}
#endif

#endif /* SWMI355_ALGOGPU_H */
