// Kernel argument blocks and launcher declarations shared by the engine and
// the two kernel translation units:
//   kernels_fast.hip   -- compiled with -ffp-contract=fast (fast mode)
//   kernels_strict.hip -- compiled with -ffp-contract=off  (bit-exact mode,
//                          plus the fold/apply/sampler/strict-eval kernels)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cocoa {

// MODE_LSGD: local SGD (SGD.scala:87-139, local = true) on the Gram-window solver
enum SolverMode : int { MODE_PLUS = 0, MODE_COCOA = 1, MODE_MBCD = 2, MODE_LSGD = 3 };

constexpr int kWave = 64;
// deltaW column runs of the Gram solver (solver_gram.h).  In fast mode every
// row stores its entries in kGramRuns runs by device column c % kGramRuns
// (cocoa_set_train), with the ends of runs 0 .. kGramRuns-2 and the row length
// per row in row_zc (kGramRuns int32 a row).  A solver workgroup has one memory
// wave and one fetch wave per column class: the one-workgroup solver has 2
// classes, class lc taking the runs [lc R/2, (lc + 1) R/2); the mirrored
// solver's half h (two workgroups per partition) has R/2 classes, class lc
// taking run 2 lc + h, so half h owns the columns of parity h.
// Eight runs (the default since round 6's last tree): each mirrored half has
// four memory waves, each with half the units per batch of the four-run form.
// A diag build with half the units per memory wave had shown the solver 2.03
// -> 1.60 ms; with eight runs, the loader's per-class work vectorised and the
// counters read at once, the C2 solver measures 1.721-1.724 against
// 1.737-1.745 ms for four runs, and the step 1.975-1.977 against 1.992-1.998
// ms on one box (profiles/r06/ab_r09h.txt; with the round-6 Gram rows at 1.6
// ms the step had not moved, as they then ran into the evaluation).
// COCOA_RUNS=4 builds the four-run form.
#ifndef COCOA_RUNS
#define COCOA_RUNS 8
#endif
constexpr int kGramRuns = COCOA_RUNS;  // column runs of a fast-mode row
static_assert(kGramRuns == 4 || kGramRuns == 8, "column runs");
constexpr int kGramClasses = 2;        // classes of the one-workgroup solver
constexpr int kProfStride = 128;    // solver profile words per partition (diagnostics)
constexpr int kMetaSteps = 64;      // steps per staged batch (one per loader lane)
#ifndef COCOA_REG_CHUNKS
#define COCOA_REG_CHUNKS 4
#endif
constexpr int kRegChunks = COCOA_REG_CHUNKS;  // rows with z <= 64 * kRegChunks keep (col,val,vec) in registers
// Chain v3's short-row register-chunk count per mode (the engine picks it for
// data with short rows): MbCD 2, CoCoA+ 3; strict and CoCoA have no variant.
constexpr int short_row_chunks(int mode, bool strict) {
    return (strict || mode == 1) ? kRegChunks : (mode == 2 ? (kRegChunks < 2 ? kRegChunks : 2) : (kRegChunks < 3 ? kRegChunks : 3));
}
constexpr int kEvalTile = 4096;     // entries per fast-eval tile
constexpr int kEvalRows = 512;      // rows per fast-eval tile (their y / row_base staged in LDS up front)

// Per-batch step metadata, staged by the loader wave in LDS (SoA).
struct BatchMeta {
    int32_t r[kMetaSteps];     // row index within the partition (the sample)
    int32_t off[kMetaSteps];   // offset of the row in the staged stream, -1 = read from HBM
    int32_t z[kMetaSteps];     // nnz of the row
    int32_t flags[kMetaSteps]; // bit0: row has duplicate column indices
    int64_t beg[kMetaSteps];   // global entry offset of the row
    double y[kMetaSteps];      // label
    double q[kMetaSteps];      // Math.pow(norm(x), 2)
    double xw[kMetaSteps];     // x . w (read-only w: CoCoA+ and MbCD), summed in stored order
    double rq[kMetaSteps];     // fast mode: 1 / qii, so the chain multiplies instead of dividing
    double pq[kMetaSteps];     // private columns: y qp / (lambda n) (xw then holds x.w - sigma pq alpha^0), else 0
    int32_t m;                 // steps in this batch (0 = no more work)
    int32_t pad[3];
};

struct SolverArgs {
    const int64_t* row_ptr;   // rank-local CSR
    const int32_t* col;
    const double* val;
    const double* y;
    const double* sqn;        // per-row Math.pow(norm(x),2)
    const uint8_t* rowflags;  // per-row flags (duplicates), may be null
    const int64_t* part_ptr;  // K_loc + 1 row offsets
    const int32_t* samples;   // K_loc * H
    double* alpha;            // persistent alpha (rank-local rows)
    double* alpha_work;       // working alpha copy when not in LDS
    const double* w;          // shared w (read-only during the round)
    double* dw;               // K_loc * d private deltaW (zero on entry)
    double* wloc;             // K_loc * d task copy of w (CoCoA) when not in LDS
    // per-step plan (plan_kernel, one chip-wide pass per round) or null: the
    // loader then reads each step's row extent, y, sqn and x.w with one
    // coalesced load instead of the samples -> row_ptr -> (col, val) -> w chain
    const int64_t* plan_beg;
    const int32_t* plan_z;
    const double* plan_y;
    const double* plan_q;
    const double* plan_xw;
    // private columns (fast CoCoA+, cocoa_ctx::priv_ready): per row the private
    // entries' sum of squares (the row's dot with them is y qp (alpha - alpha^0) /
    // (lambda n)); the epilogue stores rowcoef = y (alpha - alpha^0) / (lambda n)
    // per row (the fold's tail multiplies it by each private entry's value).
    // Both null otherwise.
    const double* row_qp;
    double* rowcoef;
    int64_t d;
    int32_t H;
    int32_t stream_cap;       // staged entries per batch buffer
    int32_t any_dup;
    int32_t raw_alpha;        // 1: write the raw local alpha (unit localSDCA API)
    int32_t reg_chunks;       // chain v3: register chunks per row, kRegChunks or short_row_chunks() (engine: reg_chunks_for)
    double lam_n;             // lambda * n
    double sigma;             // sigma' = K * gamma (CoCoA+)
    double scaling;           // alpha <- alphaOld + dAlpha * scaling
    // LDS carve (byte offsets into dynamic LDS)
    int32_t lds_stream_col[2];
    int32_t lds_stream_val[2];
    int32_t lds_meta[2];
    int32_t lds_prod;         // loader scratch: stream_cap doubles
    int32_t lds_scratch;      // compute scratch: kRegChunks*64 doubles
    int32_t lds_vec;          // d doubles (deltaW, or w_loc for CoCoA) if VEC_LDS
    int32_t lds_alpha;        // rows-of-largest-partition doubles if ALPHA_LDS
    // fast CoCoA+ on compact slices: slice positions [0, hot) -- the partition's
    // most frequent columns (slices list them in device order) -- live in LDS
    // at lds_hot for the launch, written back to the slice at its end
    int32_t hot;
    int32_t lds_hot;
    uint64_t* prof;           // optional cycle counters [K][2 waves][16] (diagnostics)
};

struct PlanArgs {
    const int64_t* part_ptr;
    const int32_t* samples;
    const int64_t* row_ptr;
    const int32_t* col;
    const double* val;
    const double* y;
    const double* sqn;
    const double* w;
    int64_t steps;            // K_loc * H
    int32_t H;
    int32_t need_xw;
    const double* xw_cache;   // per-row x.w of the current w from the last fast eval, or null
    const int32_t* row_zc;    // per row: kGramRuns int32, ends of runs 0 .. kGramRuns-2 and the row length (fast mode), or null
    const int32_t* row_zs;    // private columns: per row its shared entries (the step's z), or null
    int64_t* beg;
    int32_t* z;
    int32_t* zc;              // per step: kGramRuns int32, the ends of its row's runs 0 .. kGramRuns-2 (row_zc, or
                              // all z) and its look-back (plan_impl.h), or null
    int32_t win;              // the Gram solver's window (steps) for the look-back; 0: none
    double* py;
    double* pq;
    double* xw;
};

// Gram-window local solver (solver_gram.h), fast mode
struct GramArgs {
    const int64_t* part_ptr;
    const int32_t* samples;   // K_loc * H
    const int64_t* row_ptr;
    const int32_t* col;
    const double* val;
    int32_t K, H, nbatch;     // nbatch = ceil(H / 16)
    int32_t pad;
    double* gt;               // [K][nbatch * 16][48]
    uint64_t* prof;           // optional [8] phase cycles summed over the workgroups (diagnostics)
    // sequential Gram rows (gram_seq_kernel): batch chunks per partition, and the
    // fallback list of (partition, batch) windows its pool could not hold
    // (fb: 2 int32 per window, capacity K * nbatch; fb_n: zeroed before the launch)
    int32_t chunks;
    int32_t fb_cap;           // pairs fb holds
    int32_t* fb;
    int32_t* fb_n;
    int64_t nnz, gt_len;      // (bounds of col / val and gt: the checked debug variant)
    int64_t n_rows;           // rows of row_ptr (+1 entries)
};

struct GramSolverArgs {
    const int64_t* part_ptr;
    const int32_t* samples;
    const int64_t* plan_beg;
    const int32_t* plan_z;
    const int32_t* plan_zc;   // per step: kGramRuns int32, ends of the rows' runs and the step's look-back (PlanArgs)
    const double* plan_y;
    const double* plan_q;
    const double* plan_xw;
    const int32_t* col;
    const double* val;
    double* alpha;            // alphaOld (persistent)
    double* alpha_work;       // working alpha (n + K: a sink after each partition)
    double* dw;               // K_loc * d private deltaW (zero on entry)
    const double* gt;         // Gram rows of the round (gram_kernel)
    int* status;              // set to 1 if a hand-off wait timed out (the launch then drains)
    uint64_t* prof;           // optional [K][4 waves][4]: wait cycles, total cycles (diagnostics)
    int64_t d;
    int32_t H, nbatch;
    int32_t raw_alpha;
    int32_t hot;              // columns [0, hot) of deltaW live in LDS (set by launch_solver_gram)
    int32_t diag;             // diagnostics only (COCOA_GRAM_DIAG): 1 skip scatter atomics, 2 skip gathers
    int32_t proj;             // 1: alpha may lie outside [0, 1] -- explicit projected-gradient skip (CoCoA.scala:166-172)
    double lam_n, inv_lam_n;
    double sigma;             // sigma' = K gamma (CoCoA+)
    double scaling;
    // MODE_LSGD: step_i = 1 / (lambda (t0 + i)) (SGD.scala:106); w = wInit, the
    // epilogue turns the slice's delta-v into deltaW = s (keep wInit + dv) - wInit
    const double* w;
    double lambda, t0;
    // x.w of step j of partition k at plan_xw[k * xw_stride + j]; with xw_flag the
    // values come from xw_produce_kernel beside the solver, batch b of
    // partition k published when xw_flag[k * nbatch + b] == xw_epoch
    const int32_t* xw_flag;
    const int32_t* xw_col;    // global column of each entry (x.w formed in the loader: w[xw_col])
    int32_t xw_epoch;
    int32_t xw_pad;
    int64_t xw_stride;
    // mirrored solver (two workgroups per partition, grid 2 K; half h = blockIdx /
    // K owns the deltaW columns of parity h): each half's partial bases of a
    // batch go to the other through xbase (tagged 8-byte granules, tag =
    // xtag_epoch << 20 | batch + 1), its working alpha at alpha_work + h (n + K)
    int32_t mirror;
    int32_t xtag_epoch;
    uint64_t* xbase;          // [K][kGramRuns][kXbR][kGB][2]
    int64_t alpha_work_stride;  // n + K (mirror)
    // the hot / cold run boundary of the rows' layout (COCOA_HOTRUNS, cocoa_set_train);
    // the mirrored solver specialises its memory waves when it equals hot
    int32_t hot_split;
    int32_t hot_split_pad;
};
constexpr int kXbR = 8;     // xbase ring (batches)

// x.w of the round's sampled rows, produced beside the Gram solver (its loader
// polls the flags): one 256-thread block per (batch, partition), batch-major
struct XwArgs {
    const int64_t* part_ptr;
    const int32_t* samples;   // K_loc * H
    const int64_t* row_ptr;
    const int32_t* col;
    const double* val;
    const double* w;
    double* xw;               // [K][stride], stride a multiple of 16 (one 128-byte line per batch)
    int32_t* flag;            // [K][nbatch]
    int64_t stride;
    int32_t K, H, nbatch, epoch;
};

// Dense-row local solver (solver_dense.h), fast mode: X is the CSR value array
// of rows that store all d features in index order (row r at X + r * d)
struct DenseArgs {
    const double* X;          // rank-local rows, row-major [n][d]
    const int64_t* part_ptr;
    const int32_t* samples;   // K_loc * H
    const double* plan_y;     // per step: y and ||x||^2 of the sampled row (plan kernel)
    const double* plan_q;
    double* alpha;            // persistent alpha: alphaOld in, the scaled update out
    double* dw;               // K_loc * d private deltaW (every entry written)
    const double* w;
    int64_t d;
    int32_t H;
    int32_t proj;             // 1: alpha may lie outside [0, 1] -- explicit projected-gradient skip (CoCoA.scala:166-172)
    double lam_n, inv_lam_n;
    double sigma;             // sigma' = K gamma (CoCoA+)
    double scaling;
};

struct EvalArgs {
    // train side
    const int64_t* row_ptr;
    const int32_t* col;
    const double* val;
    const double* y;
    const double* alpha;
    int64_t n;
    // test side
    const int64_t* t_row_ptr;
    const int32_t* t_col;
    const double* t_val;
    const double* t_y;
    int64_t n_test;
    const double* w;
    int64_t d;
    // partitions (strict fold order)
    const int64_t* part_ptr;
    const int32_t* perm;      // original -> device feature order (strict ||w|| order)
    int32_t K;
    int32_t pad;
    // row tiles for the fast pass: tile t covers rows [tiles[t], tiles[t+1]) whose
    // entries fit kEvalTile (or one longer row)
    const int64_t* tiles;
    int64_t n_tiles;
    const int64_t* t_tiles;
    int64_t n_t_tiles;
    // outputs
    double* partials;         // [blocks][4] fast; per-row scratch strict
    double* out;              // [4]: hinge_sum, alpha_sum, w_sq(norm^2 via sqrt), test_err_count
    double* row_scratch;      // n doubles (strict)
    double* row_xw;           // n doubles or null: eval v4 also stores each train row's x.w
    // uint16 copies of col / t_col (device feature order) when d <= 65,536, or
    // null; padded like col (the fast eval then streams 10 B per entry)
    const uint16_t* col16;
    const uint16_t* t_col16;
    // fast sparse pass: with counter (zero between launches) the last block to
    // finish sums the block partials itself (no eval_final_kernel launch) and
    // also stores the 4 sums to out_host (pinned) when set
    unsigned* counter;
    double* out_host;
    // with out_host: the Gram solver's status word (read after the rounds this
    // pass evaluates, stream order) copied to status_host (pinned), or null
    const int* status;
    int* status_host;
    // hot / cold split of the train rows (cocoa_ctx::split_ready, fast mode), or
    // row_base null: the hot entries (device column < kEvalHot) as their own CSR
    // with 16-bit columns and tiles; row_ptr / col / col16 / val / tiles above
    // then hold the cold entries, and row_base [n] the hot pass's row dots
    const int64_t* h_row_ptr;
    const uint16_t* h_col16;
    const double* h_val;
    const int64_t* h_tiles;
    int64_t n_h_tiles;
    double* row_base;
    // wide d (> kEvalHot + kEvalWarm): the warm entries (device columns [kEvalHot,
    // kEvalHot + kEvalWarm), 16-bit offsets from kEvalHot) as a third CSR, summed
    // into row_base by a pass whose w gathers stay in L2; the cold CSR then holds
    // the columns past them.  n_m_tiles 0: no warm pass
    const int64_t* m_row_ptr;
    const uint16_t* m_col16;
    const double* m_val;
    const int64_t* m_tiles;
    int64_t n_m_tiles;
    // the test rows split the same way (n_th_tiles > 0): their hot entries as a
    // CSR of their own (th_*), summed by the hot pass into row_base[n + r]; the
    // t_* arrays above then hold the test rows' cold entries
    const int64_t* th_row_ptr;
    const uint16_t* th_col16;
    const double* th_val;
    const int64_t* th_tiles;
    int64_t n_th_tiles;
};
constexpr int kEvalHot = 4096;   // w columns in LDS in the split evaluation's hot pass
constexpr int kEvalWarm = 65536; // columns of its warm pass (0.5 MB of w: L2-resident gathers)
void eval_split_tiles(int* hot_cap, int* cold_cap);  // tile entries of its hot / cold passes

// fast translation unit
void launch_solver_fast(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                        hipStream_t s);
// returns true when the sums were also stored to a.out_host (no copy needed)
bool launch_eval_fast(const EvalArgs& a, int blocks, hipStream_t s);
int eval_fast_blocks(int64_t n, int64_t n_test);
// entries per fast-eval tile (make_tiles cap).  Past kEvalWideD columns (w
// beyond the L2s, int32 columns: C4) the pass takes 2,048-entry tiles and keeps
// w's 4,096 most frequent columns in LDS, three workgroups per CU (C4, same
// box: 1.36 -> 1.21 ms; the same on C2's uint16 columns: 0.213 -> 0.220)
constexpr int64_t kEvalWideD = 65536;
int eval_tile_entries(int64_t d);
void launch_plan_fast(const PlanArgs& a, hipStream_t s);
// Gram-window solver: lds bytes for a partition of max_nl rows (alpha in LDS
// when it fits, else in alpha_work)
size_t gram_solver_lds(int64_t d, int32_t* hot, bool mirror = false);
void launch_gram(const GramArgs& a, hipStream_t s);
size_t gram_seq_lds();  // LDS bytes of gram_seq_kernel (one workgroup per CU)
int gram_window_batches();  // batches in the Gram solver's look-back window (kGNB)
bool gram_seq_supported();  // gram_seq_kernel handles this build's window (kGW)
void launch_xw_produce(const XwArgs& a, hipStream_t s);
void launch_xw_gather(const int64_t* part_ptr, const int32_t* samples, int32_t H, int64_t steps,
                      const double* row_xw, double* xw, hipStream_t s);
void launch_solver_gram(int mode, const GramSolverArgs& a, int grid, hipStream_t s);
// dense rows: whether d and the largest partition (max_nl rows) fit the kernels
bool dense_solver_fits(int64_t d, int64_t max_nl);
bool dense_eval_fits(int64_t d);
void launch_solver_dense(int mode, const DenseArgs& a, int grid, int64_t max_nl, hipStream_t s);
void launch_eval_dense(const EvalArgs& a, hipStream_t s);

// strict translation unit
void launch_plan_strict(const PlanArgs& a, hipStream_t s);
void launch_solver_strict(int mode, bool vec_lds, bool alpha_lds, const SolverArgs& a, int grid, size_t lds,
                          hipStream_t s);
void launch_eval_strict(const EvalArgs& a, hipStream_t s);
void launch_sampler(const int64_t* part_ptr, int32_t K, int32_t seed, int32_t H, int32_t* samples,
                    const uint64_t* jump_tab, hipStream_t s);
// inv (device order -> original feature index) places the unapplied sum in the
// original order, the order ranks exchange it in
void launch_zero(double* p, int64_t n, int blocks, hipStream_t s);
void launch_dense_cols(int32_t* col, uint16_t* col16, int64_t nnz, int32_t d, hipStream_t s);
void launch_sum_slices(double* own, const double* stage, int32_t n, int32_t r, int64_t len, hipStream_t s);
void launch_fold(const double* dw, int32_t K, int64_t d, double* dw_sum, double* w, double mult, bool apply,
                 const int32_t* inv, bool zero, hipStream_t s, const double* init = nullptr);
// compact deltaW slices: column j's sum is the gather of dw[fpos[fptr[j] ..
// fptr[j+1])] in partition order (each entry re-zeroed as it is read)
// fast mode, compact slices: the fold by column blocks of kFoldJ device
// columns (LDS accumulators, work items of ~kFoldItem entries); reads only
// (the double-buffered set is re-zeroed by a memset)
constexpr int64_t kFoldJ = 4096;
constexpr int64_t kFoldItem = 32768;
// the private columns' tail (cocoa_ctx::priv_ready): per (block, partition) the
// run [tbnd[b K + k], tbnd[(b+1) K + k]) of the flattened tail, each entry its
// column's offset in the block, its row and value; its deltaW is
// val * rowcoef[row] (rowcoef: the solver's epilogue)
struct FoldTail {
    const uint32_t* tbnd;
    const uint16_t* tcol16;
    const int32_t* trow;
    const double* tval;
    const double* rowcoef;
};
void launch_fold_blocks(const double* dw, const uint16_t* fcol16, const uint32_t* fbnd, const int32_t* items,
                        int32_t n_items, int32_t K, int64_t max_u, int64_t d, double* tmp, double* dw_sum, double* w,
                        double mult, bool apply, const int32_t* inv, hipStream_t s, const FoldTail* tail = nullptr);
void launch_fold_compact(double* dw, const int64_t* fptr, const uint32_t* fpos, int64_t d, double* dw_sum, double* w,
                         double mult, bool apply, const int32_t* inv, bool zero, hipStream_t s,
                         const double* init = nullptr);
void launch_apply(double* w, const double* dw_sum, int64_t d, double mult, const int32_t* inv, hipStream_t s);
// *slot = (status[0] != 0): a solver abort rides along with the deltaW all-reduce
void launch_status_slot(const int* status, double* slot, hipStream_t s);
void launch_scale(double* w, int64_t d, double scale, hipStream_t s);
void launch_row_sqnorm(const int64_t* row_ptr, const double* val, int64_t n, double* out, hipStream_t s);
void launch_sgd(bool local, const SolverArgs& a, double lambda, double t0, int grid, hipStream_t s);
void launch_sgd_fast(bool local, const SolverArgs& a, double lambda, double t0, int K, hipStream_t s);

// mb-SGD as a transposed SpMV (fast mode, kernels_fast.hip): within a round the
// driver w is fixed, so the round's deltaW is X^T c with c_r = cnt_r y_r for the
// rows r whose margin violates (cnt_r = the round's samples of r), summed column
// by column over a CSC copy of the rows instead of scattered by atomics.
constexpr int kPullTile = 4096;  // entries per tile of the mb-SGD pull
struct MbsgdPull {
    const int64_t* csc_ptr;   // [d + 1] entry offsets per device column
    const int32_t* csc_row;   // [nnz] rank-local row of each entry
    const double* csc_val;    // [nnz]
    const int64_t* tiles;     // [n_tiles][4] (e0, e1, j0, j1): whole columns [j0, j1), or j1 = -1: a slice of j0

    int64_t n_tiles;
    int32_t* row_cnt;         // [n] samples per row this round (zero on entry)
    double* row_c;            // [n] c_r
};
void launch_csc_fill(const int64_t* row_ptr, const int32_t* col, const double* val, int64_t n_rows, int64_t* cursor,
                     int32_t* csc_row, double* csc_val, hipStream_t s);
// out[j] (device order, zero on entry for split columns) = sum over column j of
// val * c[row]; xw_cache: the rows' x.w before the round's scale (null: formed
// here from the scaled w)
void launch_mbsgd_pull(const SolverArgs& a, const MbsgdPull& p, int32_t K, int64_t n_rows, const double* xw_cache,
                       double scale, double* out, hipStream_t s);

}  // namespace cocoa
