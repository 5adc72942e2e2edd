/*
 * cocoa_capi.h -- C ABI of libcocoa_hip.so, the MI355X-native engine for the
 * per-round CoCoA / CoCoA+ hot path of calvinmccarter/cocoa.
 *
 * Plain pointers and sizes only (no torch / HIP types).  Every function
 * returns 0 on success or a negative COCOA_E_* code; the message of the last
 * failure is available from cocoa_last_error(ctx) (or cocoa_last_error(NULL)
 * for failures that happen before a context exists).
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repository root).  How the unchanged
 * Scala driver binds to these symbols (JNI / Panama FFM) is in INTEGRATION.md.
 *
 * Ownership: the caller owns every host buffer it passes; the engine copies
 * inputs to device memory and copies results out.  A context owns its device
 * memory, its HIP stream and its communicator; it is not thread-safe and is
 * driven from one host thread.  Multi-GPU comes in two shapes:
 *   - one context over several GPUs in one process (cocoa_create_multi): the
 *     shape of the reference's single driver JVM; the devices exchange deltaW
 *     among themselves inside cocoa_round;
 *   - one process (and one context) per GPU: rank 0 makes a communicator id
 *     (cocoa_comm_unique_id), the caller hands the 128 bytes to every rank by
 *     any means (a file, its own RPC, MPI, ...), every rank calls
 *     cocoa_comm_init, and from then on cocoa_round / cocoa_eval / cocoa_run
 *     exchange deltaW and the objective sums internally (RCCL over xGMI).
 * cocoa_round_local() / cocoa_round_apply() remain for a caller that does the
 * exchange itself.
 */
#ifndef COCOA_CAPI_H
#define COCOA_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COCOA_CAPI_VERSION 3

/* error codes */
#define COCOA_OK 0
#define COCOA_E_ARG (-1)        /* IllegalArgumentException analogue       */
#define COCOA_E_PARSE (-2)      /* NumberFormatException / MatchError       */
#define COCOA_E_RANGE (-3)      /* ArrayIndexOutOfBounds (feature index)    */
#define COCOA_E_IO (-4)         /* file not found / read error              */
#define COCOA_E_HIP (-5)        /* HIP runtime error                        */
#define COCOA_E_STATE (-6)      /* call out of order (no data, not inited)  */
#define COCOA_E_NODEV (-7)      /* no HIP device / kernels not loadable     */

/* methods: hingeDriver.scala:84-109 */
#define COCOA_METHOD_COCOA_PLUS 0 /* CoCoA.runCoCoA(plus=true)   CoCoA.scala:22   */
#define COCOA_METHOD_COCOA 1      /* CoCoA.runCoCoA(plus=false)  CoCoA.scala:22   */
#define COCOA_METHOD_MBCD 2       /* MinibatchCD.runMbCD         MinibatchCD.scala:19 */
#define COCOA_METHOD_MBSGD 3      /* SGD.runSGD(local=false)     SGD.scala:21     */
#define COCOA_METHOD_LOCALSGD 4   /* SGD.runSGD(local=true)      SGD.scala:21     */

/* Params (OptClasses.scala:21-29), minus the unused `loss` closure and with
 * wInit passed separately (cocoa_init). */
typedef struct {
    int32_t n;           /* global number of examples (Params.n)            */
    int32_t num_rounds;  /* T                                                 */
    int32_t local_iters; /* H                                                 */
    int32_t _pad;
    double lambda;
    double beta;         /* CoCoA scaling beta/K                              */
    double gamma;        /* CoCoA+ aggregation gamma (sigma' = K*gamma)       */
} cocoa_params;

/* DebugParams (OptClasses.scala:38-42); testData is set with cocoa_set_test. */
typedef struct {
    int32_t debug_iter;  /* <= 0: no per-round evaluation                     */
    int32_t seed;        /* round t uses seed + t (CoCoA.scala:45)            */
    int32_t chkpt_iter;  /* rounds between checkpoints (cocoa_set_checkpoint_dir) */
    int32_t _pad;
} cocoa_debug;

/* Evaluation record (OptUtils.scala:57-98).  Rank-local partial sums are
 * exposed so a multi-GPU caller can all-reduce them. */
typedef struct {
    double primal;        /* computePrimalObjective   OptUtils.scala:73     */
    double dual;          /* computeDualObjective     OptUtils.scala:80     */
    double gap;           /* computeDualityGap        OptUtils.scala:89     */
    double test_error;    /* computeClassificationError OptUtils.scala:95   */
    double hinge_sum;     /* sum_i max(1 - y_i x_i.w, 0) over this rank's train rows */
    double alpha_sum;     /* sum of this rank's alpha                       */
    double w_sqnorm;      /* sum_j w_j^2 (raw; norm(w) = sqrt of it)          */
    int64_t test_err_count; /* misclassified test rows on this rank         */
    int64_t test_rows;    /* test rows on this rank                         */
} cocoa_eval_result;

typedef struct cocoa_ctx cocoa_ctx;

/* ---- context ------------------------------------------------------------ */
/* device: HIP device ordinal.  strict: 1 = bit-exact mode (sequential dots in
 * stored order, no FMA contraction, exact divisions: bitwise equal to the CPU
 * restatement), 0 = fast mode (wave-tree dots, FMA; agrees within 1e-9).
 * stream: a hipStream_t to run on (NULL = a stream owned by the context). */
int cocoa_create(int device, int strict, void *stream, cocoa_ctx **out);
/* ONE context over n_devices GPUs (devices: their ordinals, NULL = 0..n-1;
 * an ordinal may repeat), driven from the caller's one thread -- the shape of
 * the reference's single driver process (hingeDriver.scala:84 ->
 * CoCoA.runCoCoA, whose deltaW reduce and `w +=` happen inside the call,
 * CoCoA.scala:45-48; SURVEY.md 8(b) `cocoa_create(n_gpus, ...)`).  Device r
 * holds the contiguous partition block [K r / n, K (r+1) / n) of
 * cocoa_set_train's data (which must be the whole problem: part_begin 0,
 * num_parts_global = num_parts) and the test rows [n_t r / n, n_t (r+1) / n).
 * Every round the devices exchange deltaW on their own streams.  Fast mode,
 * distinct devices (the default): one grouped RCCL all-reduce over xGMI
 * (ncclCommInitAll; identical bytes on every device, but the association of
 * the sum follows RCCL's algorithm and channel choice, so it is not
 * reproducible across device counts or RCCL versions).  Fast mode with a
 * repeated ordinal, COCOA_GROUP_EXCHANGE=peer, or an RCCL set-up failure: peer
 * copies, a reduce-scatter then all-gather of column slices, device r summing
 * slice r of every device's fold in device order (reproducible and identical
 * on every device).  cocoa_plan_info reports which ("exchange").  Strict: the
 * partition-order chain, so strict results stay bitwise equal to one device.
 * cocoa_eval merges the
 * objective terms; w / alpha / checkpoints are those of the whole problem (a
 * checkpoint is interchangeable with a one-device context's).  The
 * caller-driven exchange entry points (cocoa_round_local, cocoa_round_apply,
 * cocoa_dw_sum_device_ptr, cocoa_set_dw_sum_buffer, cocoa_comm_init) and the
 * solver-profile diagnostics return COCOA_E_STATE on such a context. */
int cocoa_create_multi(int32_t n_devices, const int32_t *devices, int strict, cocoa_ctx **out);
/* Devices of a context: n_devices (1 for cocoa_create), their ordinals into devices[cap]. */
int cocoa_num_devices(cocoa_ctx *ctx, int32_t *n_devices, int32_t *devices, int32_t cap);
int cocoa_destroy(cocoa_ctx *ctx);
const char *cocoa_last_error(const cocoa_ctx *ctx);
int cocoa_version(void);

/* ---- rank exchange (CoCoA.scala:45-48, OptUtils.scala:65-98) ------------ */
/* The reference sums the K partitions' deltaW with `updates.map(_._1)
 * .reduce(_ + _)` and reduces the objective terms with RDD reduces; here the
 * ranks exchange them directly.  Transports:
 *   RCCL -- over xGMI, one GPU per rank (the production path);
 *   HOST -- TCP through rank 0 (COCOA_COMM_ADDR, default 127.0.0.1), buffers
 *           staged in host memory: ranks sharing a GPU, CPU-only use.
 * With a communicator, fast mode allreduces the rank-local folds (one fixed
 * association, identical bytes on every rank); strict mode passes the running
 * partition-order fold from rank to rank (rank r continues ranks < r) and the
 * last rank broadcasts it, so strict multi-rank runs stay bitwise equal to
 * the single-process reference order. */
#define COCOA_TRANSPORT_RCCL 0
#define COCOA_TRANSPORT_HOST 1
#define COCOA_TRANSPORT_LOCAL 2 /* reported by cocoa_comm_info for a multi-device context (not for cocoa_comm_*) */
#define COCOA_COMM_UID_BYTES 128
typedef struct cocoa_comm cocoa_comm;
/* Made once, on rank 0 (HOST: opens rank 0's listening socket in this process). */
int cocoa_comm_unique_id(int transport, void *uid /* COCOA_COMM_UID_BYTES */);
/* Attach a communicator to the context (owned by it; replaces any previous). */
int cocoa_comm_init(cocoa_ctx *ctx, int transport, int32_t rank, int32_t world, const void *uid);
/* transport (-1 = none), rank and world of the context's communicator. */
int cocoa_comm_info(cocoa_ctx *ctx, int32_t *transport, int32_t *rank, int32_t *world);
/* Stand-alone communicator on host buffers (no context; device < 0 = none,
 * RCCL needs one): the two reductions the engine uses. */
int cocoa_comm_create(int transport, int32_t rank, int32_t world, const void *uid, int device, cocoa_comm **out);
int cocoa_comm_destroy(cocoa_comm *comm);
/* in place: buf = sum over ranks (HOST: ((x_0 + x_1) + x_2) + ... at rank 0). */
int cocoa_comm_allreduce(cocoa_comm *comm, double *buf, int64_t n);
/* in place: buf = ((x_0 + x_1) + ...) formed rank to rank, the strict chain. */
int cocoa_comm_ordered_sum(cocoa_comm *comm, double *buf, int64_t n);

/* ---- data (OptUtils.loadLIBSVMData result, OptUtils.scala:11-53) -------- */
/* This rank's partitions of the training set as one CSR: rows are
 * partition-contiguous, partition k owns rows [part_ptr[k], part_ptr[k+1]).
 * part_begin / num_parts_global: global index of this rank's first partition
 * and the global K (data.partitions.size, CoCoA.scala:28).  Rows keep their
 * stored entry order (dot products are summed in that order). */
int cocoa_set_train(cocoa_ctx *ctx, int32_t num_parts, const int64_t *part_ptr, const int64_t *row_ptr,
                    const int32_t *col, const double *val, const double *y, int64_t n_rows, int32_t num_features,
                    int32_t part_begin, int32_t num_parts_global);
/* This rank's share of DebugParams.testData (any row split).  Call it after
 * cocoa_set_train: cocoa_set_train drops any test set set before it (the test
 * columns are stored in the training set's device feature order). */
int cocoa_set_test(cocoa_ctx *ctx, const int64_t *row_ptr, const int32_t *col, const double *val, const double *y,
                   int64_t n_rows);
/* Dense variants (epsilon-shaped data, config C3): X is row-major
 * [n_rows][num_features] and every entry is a stored feature, as LIBSVM rows
 * listing all d features in index order are (the reference's dot products then
 * sum every entry in index order).  Equivalent to cocoa_set_train /
 * cocoa_set_test with row r holding columns 0..d-1; cocoa_set_train also
 * recognises such CSR input.  With dense rows, fast mode runs the dense local
 * solver (deltaW and w in registers, 8 B per streamed entry) and the dense
 * evaluation pass; strict mode keeps the stored-order CSR kernels. */
int cocoa_set_train_dense(cocoa_ctx *ctx, int32_t num_parts, const int64_t *part_ptr, const double *X,
                          const double *y, int64_t n_rows, int32_t num_features, int32_t part_begin,
                          int32_t num_parts_global);
int cocoa_set_test_dense(cocoa_ctx *ctx, const double *X, const double *y, int64_t n_rows);

/* ---- solver ---------------------------------------------------------------*/
/* Local solver of the SDCA methods in fast mode (strict mode always runs the
 * chain solver, which sums every dot in the reference's order):
 *   CHAIN -- each step gathers deltaW (or w) at its row and reduces the dot;
 *   GRAM  -- the dot is a lagged gather plus Gram corrections of the last 48
 *            steps, so the sequential chain does no memory access.  With
 *            2 K (MbCD) or 4 K (the others) <= CUs it runs mirrored: two
 *            workgroups per partition that wait on each other, so it assumes a
 *            device this context has to itself (a group member whose ordinal
 *            repeats, or a rank on a HOST-transport communicator, runs the
 *            one-workgroup form; COCOA_GRAM_MIRROR=0 forces it);
 *   DENSE -- dense rows (cocoa_set_train_dense, d even, d <= 4096): w and
 *            deltaW in registers across a 512-thread workgroup, rows streamed;
 *   AUTO  -- DENSE on dense rows that fit it, else GRAM on sparse rows (mean
 *            nnz/row <= 512), else CHAIN.  Takes effect at the next cocoa_init. */
#define COCOA_SOLVER_AUTO 0
#define COCOA_SOLVER_CHAIN 1
#define COCOA_SOLVER_GRAM 2
#define COCOA_SOLVER_DENSE 3
int cocoa_set_solver(cocoa_ctx *ctx, int kind);

/* Start a run: alpha = 0 (CoCoA.scala:33), w = w_init (NULL = zeros,
 * hingeDriver.scala:75), scaling per method (CoCoA.scala:37). */
int cocoa_init(cocoa_ctx *ctx, const cocoa_params *params, const cocoa_debug *debug, int method, const double *w_init);
/* Round t (1-based), local half: sampling with seed+t, K local solvers
 * (CoCoA.localSDCA, CoCoA.scala:130-192 / MinibatchCD.scala:76-132 /
 * SGD.scala:87-139), alpha update (CoCoA.scala:101) and this rank's ordered
 * deltaW fold into the device buffer returned by cocoa_dw_sum_device_ptr. */
int cocoa_round_local(cocoa_ctx *ctx, int32_t t);
/* Device pointer (double[num_features]) holding this rank's deltaW sum after
 * cocoa_round_local; a multi-GPU caller all-reduces it in place. */
int cocoa_dw_sum_device_ptr(cocoa_ctx *ctx, void **out);
/* Redirect the deltaW sum into caller-owned device memory (e.g. a tensor
 * that torch.distributed all-reduces).  NULL restores the internal buffer. */
int cocoa_set_dw_sum_buffer(cocoa_ctx *ctx, void *device_ptr);
/* w += sum * scaling (CoCoA.scala:47-48; MinibatchCD.scala:42-43;
 * SGD.scala:54-59). */
int cocoa_round_apply(cocoa_ctx *ctx);
/* One full round on a single rank = local + apply. */
int cocoa_round(cocoa_ctx *ctx, int32_t t);
/* Objectives over this rank's data (OptUtils.scala:57-98).  With one rank the
 * fields are the reference's values; with several, all-reduce hinge_sum,
 * alpha_sum and test_err_count and finish with cocoa_eval_finish. */
int cocoa_eval(cocoa_ctx *ctx, cocoa_eval_result *out);
/* The same evaluation, pipelined (one device, one rank, fast mode): enqueue
 * the objectives of the current (w, alpha) -- snapshots taken on the context's
 * stream -- on a side stream and return at once, so the next cocoa_round runs
 * beside it; cocoa_eval_wait returns exactly what cocoa_eval would have
 * returned for that state.  The reference prints these after round t before
 * starting round t+1 (CoCoA.scala:51-56); here the host learns them while
 * round t+1 is already on the GPU.  One evaluation may be pending at a time;
 * cocoa_eval refuses while one is. */
int cocoa_eval_async(cocoa_ctx *ctx);
int cocoa_eval_wait(cocoa_ctx *ctx, cocoa_eval_result *out);
/* The cocoa_eval pass with deferred read-back: cocoa_eval_begin enqueues it
 * on the context's stream behind the current round (the next round's step
 * plan still reuses its per-row x.w) and returns at once; the caller enqueues
 * the next cocoa_round and then collects with cocoa_eval_end, which returns
 * exactly what cocoa_eval would have for that state.  The reference prints
 * after round t before starting round t+1 (CoCoA.scala:51-56); here round t+1
 * is already queued while the host reads round t's gap, so the GPU does not
 * idle on the host.  Multi-rank and multi-device contexts evaluate inside
 * cocoa_eval_begin.  One evaluation may be pending at a time. */
int cocoa_eval_begin(cocoa_ctx *ctx);
int cocoa_eval_end(cocoa_ctx *ctx, cocoa_eval_result *out);
int cocoa_eval_finish(const cocoa_ctx *ctx, double hinge_sum, double alpha_sum, double w_sqnorm,
                      int64_t test_err_count, int64_t test_rows, cocoa_eval_result *out);

/* Per-round observer for cocoa_run (the reference prints at debugIter). */
typedef void (*cocoa_round_cb)(void *user, int32_t t, const cocoa_eval_result *ev);
/* CoCoA.runCoCoA / MinibatchCD.runMbCD / SGD.runSGD on one rank:
 * init + T rounds (+ eval every debug_iter rounds, reported through cb). */
int cocoa_run(cocoa_ctx *ctx, const cocoa_params *params, const cocoa_debug *debug, int method,
              const double *w_init, cocoa_round_cb cb, void *user);

int cocoa_get_w(cocoa_ctx *ctx, double *w_out);           /* num_features */
int cocoa_get_alpha(cocoa_ctx *ctx, double *alpha_out);   /* this rank's n_rows */
int cocoa_set_w(cocoa_ctx *ctx, const double *w_in);
int cocoa_set_alpha(cocoa_ctx *ctx, const double *alpha_in);

/* (t, w, alpha) checkpoint of this rank.  The reference checkpoints its alpha
 * RDD every chkptIter rounds only to truncate Spark lineage
 * (CoCoA.scala:58-62); here the round state goes to a file so that a long run
 * (config C4) can stop and resume.  Format "COCOACK1", little-endian: a
 * 96-byte header (method, n, num_features, K_glob, part_begin, K_loc, rows,
 * local_iters, lambda, beta, gamma, t, seed, strict), w[num_features] in
 * original feature order, alpha[rows], then an FNV-1a 64 checksum of
 * everything before it.  Load validates the header against the context (same
 * problem, method, partitioning, DebugParams.seed and numerics mode;
 * COCOA_E_ARG otherwise) and the checksum (COCOA_E_IO), sets w and alpha, and
 * returns the round t to resume after. */
int cocoa_checkpoint_save(cocoa_ctx *ctx, const char *path, int32_t t);
int cocoa_checkpoint_load(cocoa_ctx *ctx, const char *path, int32_t *t_out);
/* Periodic checkpoints inside cocoa_run / cocoa_resume: with a directory set
 * (hingeDriver.scala:55-59 chkptDir; NULL or "" turns them off), the state is
 * saved every debug->chkpt_iter rounds (CoCoA.scala:58-62) to
 * <dir>/cocoa_m<method>_p<part_begin>.ck, replacing the previous save.
 * cocoa_checkpoint_file writes that path (NUL-terminated) into buf[cap]. */
int cocoa_set_checkpoint_dir(cocoa_ctx *ctx, const char *dir);
int cocoa_checkpoint_file(cocoa_ctx *ctx, int method, char *buf, int64_t cap);
/* cocoa_run continued from a checkpoint: init, load (t0, w, alpha), then
 * rounds t0+1 .. num_rounds with the same per-round evaluation and saves. */
int cocoa_resume(cocoa_ctx *ctx, const cocoa_params *params, const cocoa_debug *debug, int method,
                 const char *path, cocoa_round_cb cb, void *user);

/* CoCoA.localSDCA (CoCoA.scala:130-192) for ONE partition of the loaded
 * training set, as a unit: w (in/out, mutated when plus == 0, like the
 * reference's alias), alpha (in/out), delta_w (out, num_features),
 * delta_alpha (out, rows of the partition; may be NULL). */
int cocoa_local_sdca(cocoa_ctx *ctx, int32_t part, double *w, int32_t local_iters, double lambda, int32_t n,
                     double *alpha, int32_t seed, int plus, double sigma, double *delta_w, double *delta_alpha);

/* The coordinate sample sequence partition `part` draws in round t
 * (java.util.Random(seed + t).nextInt(n_k), CoCoA.scala:144,151), computed on
 * the device; for parity tests. */
int cocoa_samples(cocoa_ctx *ctx, int32_t part, int32_t seed_plus_t, int32_t count, int32_t *out);

/* ---- profiling --------------------------------------------------------- */
/* Kernel ids for cocoa_kernel_stats. */
#define COCOA_K_SAMPLE 0
#define COCOA_K_SOLVER 1
#define COCOA_K_FOLD 2
#define COCOA_K_APPLY 3
#define COCOA_K_EVAL 4
#define COCOA_K_PLAN 5   /* per-round step plan (row offsets, x.w) of the SDCA loaders */
#define COCOA_K_GRAM 6   /* Gram rows of the round (Gram-window solver) */
#define COCOA_K_XW 7     /* x.w of the round's sampled rows, beside the Gram solver */
#define COCOA_K_COUNT 8
/* enable = 1: bracket every launch with HIP events on the context stream. */
int cocoa_stats_enable(cocoa_ctx *ctx, int enable);
/* Which kernel ids (bit i = COCOA_K_i) stats bracket when enabled; default all.
 * Each bracketed launch adds two event packets to its stream, ~5-10 us of
 * launch-to-launch latency on a short kernel. */
int cocoa_stats_kernels(cocoa_ctx *ctx, uint32_t mask);
/* total device milliseconds and launch count per kernel id since last reset */
int cocoa_kernel_stats(cocoa_ctx *ctx, int kernel, double *total_ms, int64_t *launches);
int cocoa_stats_reset(cocoa_ctx *ctx);
/* Diagnostics: per-workgroup cycle counters of the local-solver kernel
 * (uint64 [K_loc][2 waves][16]: busy cycles, barrier-wait cycles, batches,
 * then per-step phase cycles in a -DCOCOA_STEP_PROF build).  Overwritten by
 * every solver launch while enabled. */
int cocoa_solver_profile(cocoa_ctx *ctx, int enable);
int cocoa_solver_profile_read(cocoa_ctx *ctx, uint64_t *out, int64_t count);
/* Human-readable description of how the solver was planned (LDS placement), as
 * JSON into buf[len]; COCOA_E_ARG if it does not fit.  Touches no device state
 * (does not wait on the context's streams).  "gram_mirror" is 1 only when the
 * mirrored Gram solver will run: it assumes a device this context has to itself
 * (its two workgroups per partition wait on one another), so a group member
 * whose ordinal repeats or a rank on a HOST-transport communicator runs the
 * one-workgroup solver. */
int cocoa_plan_info(cocoa_ctx *ctx, char *buf, int len);
/* Diagnostics: windows the last Gram-row launch (gram_seq_kernel) handed to the
 * per-window kernel because its LDS pool overflowed; -1 when that kernel is not
 * in use.  Synchronises the context. */
int cocoa_gram_fallback_count(cocoa_ctx *ctx, int32_t *out);
/* Diagnostics (fast mode, Gram-window solver, not MbCD): the Gram rows of round
 * t's sampled steps (seed = DebugParams.seed + t) as the next cocoa_round(t)
 * would use them, into out[count]: [K_loc][ceil(H/16) * 16][48] doubles, row j
 * holding x_s . x_j at slot s % 48 for the steps s after j in its 48-step
 * window, 0 elsewhere.  Synchronises the context. */
int cocoa_debug_gram_rows(cocoa_ctx *ctx, int32_t t, double *out, int64_t count);
int cocoa_sync(cocoa_ctx *ctx);

/* ---- host-side data layer (no device needed) ---------------------------- */
/* A dataset allocated by the library; free with cocoa_dataset_free. */
typedef struct {
    int64_t n_rows;
    int32_t num_features;
    int32_t num_parts;
    int64_t nnz;
    int64_t *row_ptr;   /* n_rows + 1 */
    int32_t *col;       /* nnz, 0-based */
    double *val;        /* nnz */
    double *y;          /* n_rows */
    int64_t *part_ptr;  /* num_parts + 1 */
} cocoa_dataset;

/* OptUtils.loadLIBSVMData (OptUtils.scala:11-53): Hadoop-1.0.4 byte splits of
 * the file into num_splits partitions, label +1 iff the token contains '+'
 * or parses to 1, 1-based indices -> 0-based. */
int cocoa_load_libsvm(const char *path, int32_t num_splits, int32_t num_features, cocoa_dataset *out);
/* The same load with the tokenising and number parsing on HIP device `device`
 * (the file is copied to HBM once; line starts, labels, "index:value" tokens
 * and decimal values are found and converted by kernels, one wave per line).
 * Lines outside the device's exact fast path (tabs or other characters inside
 * a line, NaN/Infinity/hex spellings, more than 19 significant digits or a
 * decimal exponent beyond +-22, malformed or out-of-range tokens) are parsed
 * on the host by the same rules, so the dataset and the error raised are
 * those of cocoa_load_libsvm. */
int cocoa_load_libsvm_gpu(int device, const char *path, int32_t num_splits, int32_t num_features,
                          cocoa_dataset *out);
/* Seeded synthetic shapes: kind 0 = rcv1-like sparse
 * (Zipf columns, tf-idf-like values, unit rows), 1 = epsilon-like dense,
 * 2 = url-like very sparse binary-ish.  The rows are rows [first_row,
 * first_row + n_rows) of one seeded stream (first_row a multiple of 4096), so
 * ranks can generate disjoint shards of one problem (same planted separator).
 * Partitions are contiguous balanced row blocks.  threads <= 0: all cores. */
int cocoa_gen_synthetic(int32_t kind, int64_t n_rows, int32_t num_features, double mean_nnz, int32_t num_parts,
                        uint64_t seed, int64_t first_row, int32_t threads, cocoa_dataset *out);
void cocoa_dataset_free(cocoa_dataset *ds);

/* java.lang.Double.toString(x) as the reference's JVM (JDK 7/8,
 * sun.misc.FloatingDecimal) printed it -- not always the shortest digits
 * (2.0E23 -> "1.9999999999999998E23"); the driver's stdout lines use it.
 * buf: at least 32 bytes. */
int cocoa_java_double_string(double x, char *buf, int32_t cap);
/* java.util.Random(seed).nextInt(bound) x count on the host (bound <= 0:
 * nextInt()). */
int cocoa_jrandom_ints(int64_t seed, int32_t bound, int32_t count, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif /* COCOA_CAPI_H */
