// libcocoa_hip.so engine: device context, data upload, per-round orchestration
// of the HIP kernels, and the C ABI declared in include/cocoa_capi.h.
//
// Round structure on one rank (CoCoA.scala:39-63):
//   sampler      java.util.Random(seed+t).nextInt(n_k) x H per partition
//   solver       K_loc local solvers (one 2-wave workgroup per partition)
//   fold         ordered sum of the private deltaW slices (zeroing them)
//   [caller all-reduces the sum across ranks]           (multi-GPU only)
//   apply        w += sum * scaling
// Host arithmetic in this file (objective assembly, row norms) is compiled
// with -ffp-contract=off like the strict kernels.
#include <hip/hip_runtime.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cocoa_capi.h"
#include "comm.h"
#include "common.h"
#include "jrandom.h"
#include "kernels.h"

using namespace cocoa;

static std::mutex g_err_mu;
static std::string g_err;
void cocoa_set_global_error(const std::string& msg) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = msg;
}

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess)                                                                            \
            throw Error(COCOA_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_) + " at " __FILE__ ":" + \
                                         std::to_string(__LINE__));                                      \
    } while (0)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void alloc(size_t b) {
        free();
        if (b == 0) b = 16;
        HIPCHK(hipMalloc(&p, b));
        bytes = b;
    }
    void alloc_zero(size_t b, hipStream_t s) {
        alloc(b);
        HIPCHK(hipMemsetAsync(p, 0, bytes, s));
    }
    void free() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return (T*)p;
    }
    ~DevBuf() { free(); }
};

struct Csr {
    int64_t n = 0, nnz = 0;
    DevBuf row_ptr, col, val, y;
    DevBuf col16;  // uint16 copy of col when d <= 65,536 (fast eval stream), else empty
    // dense rows set through cocoa_set_*_dense: no column array until a CSR
    // kernel needs one (ensure_cols builds it on the device)
    bool col_lazy = false;
};

// the column arrays of dense rows (entry q is column q mod d; device order is
// the identity for dense rows), built on the device when first needed
void ensure_cols(Csr& c, int32_t d, hipStream_t s) {
    if (!c.col_lazy) return;
    c.col.alloc(sizeof(int32_t) * (size_t)c.nnz + 64);
    HIPCHK(hipMemsetAsync((char*)c.col.p + sizeof(int32_t) * (size_t)c.nnz, 0, 64, s));
    if (d <= 65536) {
        c.col16.alloc(sizeof(uint16_t) * (size_t)c.nnz + 64);
        HIPCHK(hipMemsetAsync((char*)c.col16.p + sizeof(uint16_t) * (size_t)c.nnz, 0, 64, s));
    } else {
        c.col16.free();
    }
    cocoa::launch_dense_cols(c.col.as<int32_t>(), c.col16.p ? c.col16.as<uint16_t>() : nullptr, c.nnz, d, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    c.col_lazy = false;
}

// uint16 column copy for the fast eval when every device column fits 16 bits
void upload_col16(DevBuf& b, const std::vector<int32_t>& pcol, int64_t nnz, int32_t d, hipStream_t s) {
    if (d > 65536) {
        b.free();
        return;
    }
    std::vector<uint16_t> c16((size_t)std::max<int64_t>(nnz, 1));
    for (int64_t q = 0; q < nnz; ++q) c16[(size_t)q] = (uint16_t)pcol[(size_t)q];
    b.alloc(sizeof(uint16_t) * (size_t)nnz + 64);
    HIPCHK(hipMemsetAsync((char*)b.p + sizeof(uint16_t) * (size_t)nnz, 0, 64, s));
    if (nnz) HIPCHK(hipMemcpyAsync(b.p, c16.data(), sizeof(uint16_t) * (size_t)nnz, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));  // c16 is a local
}

constexpr size_t kLdsMax = 160 * 1024;
constexpr int kStreamCap = 2048;

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace

struct cocoa_comm {
    cocoa::Comm* c = nullptr;
};

struct cocoa_ctx {
    int device = 0;
    bool strict = false;
    // Multi-device context (cocoa_create_multi): one sub-context per device,
    // each holding a contiguous block of the partitions, all driven from the
    // caller's thread; the exchange between them runs on the devices' streams
    // (peer copies + an ordered sum).  The group itself holds no device data,
    // only the problem's shape (d, K, rows, params) for the objectives and
    // checkpoints.
    std::vector<cocoa_ctx*> subs;
    std::vector<int32_t> g_k0;        // first partition of each sub (+ K at the end)
    std::vector<int64_t> g_r0;        // first training row of each sub (+ n)
    std::vector<int64_t> g_t0;        // first test row of each sub (+ n_test)
    std::vector<hipEvent_t> g_ev;     // per sub: its fold (strict: its part of the chain) is ready
    std::vector<hipEvent_t> g_ev_rs;  // per sub (fast): its column slice of the total is reduced
    std::vector<hipEvent_t> g_ev_cp;  // per sub: it has copied the total (strict) / the other slices (fast)
    // as a member of a multi-device context (fast mode): slice r of the other
    // members' folds, gathered for this member's part of the reduce-scatter
    DevBuf x_stage;
    // fast exchange over distinct devices: RCCL (one communicator per device,
    // grouped all-reduce); null: the peer-copy reduce-scatter / all-gather
    cocoa::GroupComm* g_rccl = nullptr;
    std::string g_exchange;  // "rccl", "peer" or "chain" (strict), for cocoa_plan_info
    bool is_group() const { return !subs.empty(); }
    // rank exchange (cocoa_comm_init): owned; null = single rank / caller-driven
    cocoa::Comm* comm = nullptr;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    std::string ckpt_dir;  // cocoa_set_checkpoint_dir: periodic (t, w, alpha) saves in cocoa_run
    // Double-buffered deltaW slices (large K_loc * d, e.g. C4): round t works in
    // set t & 1; the set round t folded is re-zeroed by a memset on zstream
    // that starts with round t+1 (after round t's eval, so the bandwidth-bound
    // eval does not share HBM with it) and runs beside the latency-bound solver.
    DevBuf dw2;
    bool dw_dbuf = false;
    int64_t dw_slice = 0;  // doubles per partition slice (d, or max_u for compact slices)
    hipStream_t zstream = nullptr;
    hipEvent_t zdone[2] = {nullptr, nullptr}, folded = nullptr;
    bool zpending[2] = {false, false};
    int zero_owed = -1;  // set folded last round, re-zeroed once the next round starts

    // training data (this rank)
    int32_t K_loc = 0, K_glob = 0, part_begin = 0, d = 0;
    Csr tr;
    DevBuf sqn, rowflags, part_ptr;
    DevBuf row_zc;  // fast mode: per row, ends of the column runs (kGramRuns int32), see set_train_impl
    std::vector<int64_t> h_part_ptr;
    bool any_dup = false;
    bool tr_dense = false;  // every row stores columns 0..d-1 in order (val = X[n][d])
    // Compact deltaW slices (large K_loc * d, e.g. C4): partition k's slice holds
    // only the U_k distinct columns of its rows, in device order; the entries'
    // slice positions are col_local.  fptr / fpos: for every device column j the
    // flattened slice positions k * max_u + i holding it, in partition order
    // (the fold's gather list).  Built by cocoa_set_train when K_loc * d * 8 >=
    // 1 GiB; used by the fast Gram solver.
    bool compact_ready = false, dw_compact = false;
    int64_t max_u = 0, sum_u = 0;
    DevBuf col_local, fptr, fpos;
    // fast mode: the column-block fold of compact slices (fold_blocks_kernel):
    // per slice position its column's offset in its kFoldJ-column block, per
    // (block, partition) the slice's first position in the block, the work
    // items (block, partition range) and the device-order accumulator
    DevBuf fcol16, fbnd, fitems, ftmp;
    int32_t n_fitems = 0, n_fblk = 0;
    // Private columns (fast CoCoA+ on the chain solver, compact slices): a column
    // held by ONE entry of a partition never needs a deltaW slot.  Its deltaW is
    // x_rc * y_r (alpha_r - alpha_r^0) / (lambda n) (CoCoA.scala:181, summed over
    // the row's visits), so the row's dot with the private part is
    // y_r qp_r (alpha_r - alpha_r^0) / (lambda n), qp_r = the private entries'
    // sum of squares, and the fold adds the private entries' deltaW (formed by
    // the solver's epilogue).  Slices then hold the shared columns only (max_uh
    // positions; C4: ~15 k of ~60 k), each row stores its shared entries first
    // (pcol_h / pval_h, row_zs shared entries), and the private entries form a
    // per-partition tail sorted by device column (trow / tval: their deltaW is
    // tval * rowcoef[trow], rowcoef written by the solver's epilogue) beside the
    // head's fold structures (fbnd_h / fcol16_h / fitems_h; tbnd / tcol16 for
    // the tail).
    bool priv_ready = false, dw_priv = false;
    int64_t max_uh = 0, sum_uh = 0, n_tail = 0;
    DevBuf pcol_h, pval_h, row_zs, row_qp, rowcoef;
    DevBuf fcol16_h, fbnd_h, fitems_h, tbnd, tcol16, trow, tval;
    int32_t n_fitems_h = 0;
    int32_t max_nl = 0, min_nl = 0;
    // test data (this rank)
    Csr te;
    bool has_test = false, te_dense = false;
    // row tiles of the fast evaluation pass (kEvalTile entries)
    DevBuf tiles, t_tiles;
    int64_t n_tiles = 0, n_t_tiles = 0;
    // device feature order (see cocoa_set_train)
    std::vector<int32_t> perm, inv;
    std::vector<int64_t> n_hot_nnz;
    DevBuf d_perm, d_inv;

    // host <-> device order of a w-like vector
    void to_device_order(const double* orig, std::vector<double>& dev) const {
        dev.resize((size_t)d);
        for (int32_t j = 0; j < d; ++j) dev[(size_t)perm[(size_t)j]] = orig[j];
    }
    void to_host_order(const std::vector<double>& dev, double* orig) const {
        for (int32_t j = 0; j < d; ++j) orig[j] = dev[(size_t)perm[(size_t)j]];
    }

    // run state
    bool inited = false;
    int method = 0;
    cocoa_params P{};
    cocoa_debug D{};
    double scaling = 1.0, mult = 1.0;
    // alpha set from outside [0, 1] (cocoa_set_alpha / checkpoint): with it, or
    // with a scaling outside [0, 1], the fast SDCA solvers run the explicit
    // projected-gradient skip test (CoCoA.scala:166-172) instead of the clamp alone
    bool alpha_oob = false;
    bool proj_rule() const { return alpha_oob || scaling < 0.0 || scaling > 1.0; }
    DevBuf w, alpha, alpha_work, dw, wloc, samples, dw_sum_int, eval_part, eval_out, row_scratch, jump, prof;
    double* dw_sum = nullptr;
    bool dw_sum_user = false;  // dw_sum is the caller's buffer (cocoa_set_dw_sum_buffer), else dw_sum_int
    bool abort_in_sum = false; // dw_sum[d] holds the all-reduced abort flag of the last exchange
    // the solver's status word copied behind an evaluation into pinned memory:
    // [0] in-line pass (h_eval[9], cocoa_eval_end), [1] pipelined (h_eval[10], cocoa_eval_wait)
    bool status_slot[2] = {false, false};
    double* h_eval = nullptr;  // pinned [4]
    int64_t samples_cap = 0;

    // solver plan (LDS placement) and the per-step plan of the SDCA methods
    bool vec_lds = false, alpha_lds = false;
    size_t lds_bytes = 0;
    SolverArgs sa{};
    bool use_plan = false;
    // Gram-window solver (fast SDCA methods on sparse rows, solver_gram.h)
    int solver_kind = COCOA_SOLVER_AUTO;
    bool use_gram = false;
    bool use_dense = false;  // dense-row local solver (solver_dense.h)
    DevBuf gt, status;  // status: set by a Gram-solver launch whose hand-off timed out
    DevBuf status_snap;  // status as of the rounds a pipelined evaluation covers (cocoa_eval_async)
    int32_t nbatch = 0;
    // Round t+1's samples and Gram rows are computed on gstream while round t's
    // solver runs (the sample sequence depends on seed + t only, the Gram rows
    // on the samples and the data): two (samples, gt) buffers, b and 1-b.
    DevBuf samples2, gt2;
    // gram_seq_kernel's fallback windows: [0] count, then (partition, batch)
    // pairs; one per Gram-row buffer (gt, gt2): round t+1's rows are formed on
    // gstream while round t's may still be on the context's stream
    DevBuf gram_fb[2];
    int gram_chunks = 0;  // > 0: Gram rows by gram_seq_kernel, this many batch runs per partition
    bool gram_mirror = false;  // the Gram solver as two workgroups per partition (solver_gram.h MIRROR)
    // The mirrored halves of a partition wait on one another, so both must be
    // resident at once.  On a device this context owns that holds (2 K <= CUs,
    // pairs dispatched together); on one it shares -- a group member whose
    // ordinal repeats, ranks on one GPU over the HOST transport -- the other
    // users' persistent grids could hold every CU while half 0s spin, so the
    // one-workgroup solver runs instead (decided per launch: a communicator
    // may be attached after cocoa_init).
    bool shared_dev = false;   // (cocoa_create_multi: another member has this ordinal)
    bool device_shared() const;
    int32_t hot_split = 0;     // (unused: 0)
    DevBuf xbase;              //   their partial-base exchange ([K][4][kXbR][16][2] tagged granules)
    int32_t xtag_epoch = 0;    //   launch counter in the granule tags
    hipStream_t gstream = nullptr;
    hipEvent_t g_ready = nullptr, s_done[2] = {nullptr, nullptr};
    int32_t pre_t = -1, pre_buf = 0;  // round prefetched into buffer pre_buf (-1: none)
    // x.w of a round's sampled rows by xw_produce_kernel on gstream, beside the
    // solver (whose loader polls the per-batch flags), when no in-line
    // evaluation formed them: plan_xw[k * xw_stride + j], flags [K][nbatch]
    // holding the epoch of the round that published them
    bool xw_prod = false;
    bool eval_on_g = false;  // the pipelined evaluation on gstream (COCOA_EVAL_ON_GSTREAM=1)
    int ncu = 256;      // compute units of the device
    int side_res = 0;   // CUs kept off the side streams for the solver's workgroups (0: none)
    DevBuf xw_flag;
    int32_t xw_epoch = 0;
    int64_t xw_stride = 0;
    hipEvent_t e_w = nullptr, e_xw = nullptr;
    bool e_w_rec = false;  // e_w recorded behind this round's plan (side work waits on it)
    void gram_quiesce() {  // no prefetch in flight, none pending
        if (gstream) HIPCHK(hipStreamSynchronize(gstream));
        pre_t = -1;
    }
    // pipelined evaluation (cocoa_eval_async): the objectives of a snapshot of
    // (w, alpha) on estream, beside the next round; results in h_eval[4..7]
    hipStream_t estream = nullptr;
    hipEvent_t e_round = nullptr, e_done = nullptr;
    bool eval_pending = false;  // snapshots taken (cocoa_eval_async), result not yet collected
    // cocoa_eval_begin: an in-line evaluation enqueued, its sums read back by
    // cocoa_eval_end (single rank, one device); other contexts hold the finished
    // result in eval_held
    bool inl_pending = false;
    // an in-line evaluation was enqueued since the last round (cocoa_eval_begin, one
    // rank): its e_inl, recorded behind it, gates the next Gram rows on the side
    // stream in place of an e_w record behind the x.w gather (one marker packet
    // fewer on the main stream; COCOA_GATE_INL=0 restores the e_w record)
    bool inl_since_round = false;
    bool inl_ranks = false;       //   its sums all-reduced across ranks on the device (fast multi-rank)
    int64_t n_test_glob = -1;     // test rows over all ranks (-1: not yet exchanged for this test set)
    hipEvent_t e_inl = nullptr;
    cocoa_eval_result eval_held{};
    bool eval_fired = false;    //   and its kernels enqueued on estream
    DevBuf w_snap, alpha_snap, eval_part2, eval_out2;
    DevBuf eval_cnt, eval_cnt2;  // last-block counters of the fast sparse pass (in line / pipelined)
    void eval_quiesce();        // the pending evaluation (if any) runs to completion and is dropped
    DevBuf plan_beg, plan_z, plan_zc, plan_y, plan_q, plan_xw;
    // the next round's step plan (all but x.w), prefetched on gstream beside
    // this round's solver into the other set (plan set 1 = these)
    DevBuf plan_beg2, plan_z2, plan_zc2, plan_y2, plan_q2;
    bool pre_plan = false;  // the prefetched round's plan is in set pre_buf
    // x.w of every train row for the current w, written by the fast eval pass
    // (eval v4) and reused by the next round's plan; false once w moves
    DevBuf row_xw;
    bool xw_cached = false;
    // fast mb-SGD in its pull form (kernels.h MbsgdPull): a CSC copy of the rows
    // (device column order; built by cocoa_init), its tiles, and per-row counts /
    // coefficients.  csc_ready: built for the current training set.
    // fast evaluation split by column (EvalArgs::row_base): the train rows'
    // entries in device columns < kEvalHot (hot CSR, 16-bit columns) and the rest
    // (cold CSR), with tiles for each, and the hot pass's per-row dots; for d past
    // kEvalHot + kEvalWarm the warm columns in a third CSR (16-bit offsets)
    Csr hot_tr, cold_tr, warm_tr;
    DevBuf hot_tiles, cold_tiles, warm_tiles, row_base;
    int64_t n_hot_tiles = 0, n_cold_tiles = 0, n_warm_tiles = 0;
    bool split_ready = false;
    // the test rows split the same way (te_split: built by cocoa_set_test on a
    // split training set); row_base then holds n + n_test dots
    Csr hot_te, cold_te;
    DevBuf hot_t_tiles, cold_t_tiles;
    int64_t n_hot_t_tiles = 0, n_cold_t_tiles = 0;
    bool te_split = false;
    DevBuf csc_ptr, csc_row, csc_val, csc_tiles, row_cnt, row_c;
    int64_t n_csc_tiles = 0;
    bool csc_ready = false;
    bool mbsgd_pull = false;   // this round's mb-SGD runs the pull form
    int32_t max_z = 0;

    // stats
    bool stats = false;
    uint32_t stats_mask = ~0u;  // kernel ids bracketed when stats are on (cocoa_stats_kernels)
    struct Pending {
        int kid;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    double tot_ms[COCOA_K_COUNT] = {0};
    int64_t cnt[COCOA_K_COUNT] = {0};

    hipEvent_t get_ev() {
        if (!ev_pool.empty()) {
            hipEvent_t e = ev_pool.back();
            ev_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        return e;
    }
    template <class F>
    void timed(int kid, F&& f) {
        timed_on(stream, kid, f);
    }
    template <class F>
    void timed_on(hipStream_t st, int kid, F&& f) {
        if (!stats || !((stats_mask >> kid) & 1)) {
            f();
            HIPCHK(hipGetLastError());
            return;
        }
        hipEvent_t a = get_ev(), b = get_ev();
        HIPCHK(hipEventRecord(a, st));
        f();
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(b, st));
        pending.push_back({kid, a, b});
        if (pending.size() > 4096) drain();
    }
    void drain() {
        for (auto& p : pending) {
            HIPCHK(hipEventSynchronize(p.b));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
            tot_ms[p.kid] += ms;
            cnt[p.kid] += 1;
            ev_pool.push_back(p.a);
            ev_pool.push_back(p.b);
        }
        pending.clear();
    }
    ~cocoa_ctx() {
        if (g_rccl) {
            for (cocoa_ctx* sub : subs) {
                (void)hipSetDevice(sub->device);
                if (sub->stream) (void)hipStreamSynchronize(sub->stream);
            }
            delete g_rccl;
            g_rccl = nullptr;
        }
        for (size_t r = 0; r < subs.size(); ++r) {
            (void)hipSetDevice(subs[r]->device);
            if (r < g_ev.size() && g_ev[r]) (void)hipEventDestroy(g_ev[r]);
            if (r < g_ev_cp.size() && g_ev_cp[r]) (void)hipEventDestroy(g_ev_cp[r]);
            if (r < g_ev_rs.size() && g_ev_rs[r]) (void)hipEventDestroy(g_ev_rs[r]);
            delete subs[r];
        }
        if (!subs.empty()) (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (gstream) {
            (void)hipStreamSynchronize(gstream);
            (void)hipStreamDestroy(gstream);
            (void)hipEventDestroy(g_ready);
            for (auto e : s_done) (void)hipEventDestroy(e);
        }
        if (e_w) (void)hipEventDestroy(e_w);
        if (e_xw) (void)hipEventDestroy(e_xw);
        if (estream) {
            (void)hipStreamSynchronize(estream);
            (void)hipStreamDestroy(estream);
        }
        if (e_round) (void)hipEventDestroy(e_round);
        if (e_done) (void)hipEventDestroy(e_done);
        if (e_inl) {
            (void)hipEventDestroy(e_inl);
        }
        delete comm;
        if (zstream) {
            (void)hipStreamSynchronize(zstream);
            (void)hipStreamDestroy(zstream);
            for (auto e : zdone) (void)hipEventDestroy(e);
            (void)hipEventDestroy(folded);
        }
        for (auto& p : pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        if (h_eval) (void)hipHostFree(h_eval);
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }
};

bool cocoa_ctx::device_shared() const {
    return shared_dev || (comm && comm->world > 1 && comm->transport == cocoa::kTransportHost);
}

#define CAPI_BEGIN(ctx)                                             \
    if (!(ctx)) {                                                   \
        cocoa_set_global_error("null context");                     \
        return COCOA_E_ARG;                                         \
    }                                                               \
    try {                                                           \
        HIPCHK(hipSetDevice((ctx)->device));
#define CAPI_END(ctx)                                               \
    return COCOA_OK;                                                \
    }                                                               \
    catch (const Error& e) {                                        \
        (ctx)->err = e.what();                                      \
        cocoa_set_global_error(e.what());                           \
        return e.code;                                              \
    }                                                               \
    catch (const std::exception& e) {                               \
        (ctx)->err = e.what();                                      \
        cocoa_set_global_error(e.what());                           \
        return COCOA_E_ARG;                                         \
    }

static void require(bool cond, int code, const std::string& msg) {
    if (!cond) throw Error(code, msg);
}

// multi-device contexts (cocoa_create_multi): the group side of the entry points
static void group_set_train(cocoa_ctx* g, bool dense, int32_t K, const int64_t* part_ptr, const int64_t* row_ptr,
                            const int32_t* col, const double* val, const double* y, int64_t n, int32_t d,
                            int32_t part_begin, int32_t Kg);
static void group_set_test(cocoa_ctx* g, bool dense, const int64_t* row_ptr, const int32_t* col, const double* val,
                           const double* y, int64_t n_rows);
static void group_init(cocoa_ctx* g, const cocoa_params* params, const cocoa_debug* debug, int method,
                       const double* w_init);
static void group_round(cocoa_ctx* g, int32_t t);
static void group_get_state(cocoa_ctx* g, double* w, double* alpha);
static void group_set_state(cocoa_ctx* g, const double* w, const double* alpha);
static int32_t group_owner_of_part(const cocoa_ctx* g, int32_t part);
static void sub_check(int rc, const cocoa_ctx* sub);
#define GROUP_REJECT(ctx, what) \
    require(!(ctx)->is_group(), COCOA_E_STATE, what " is not available on a multi-device context (it exchanges internally)")

// after a stream synchronisation: a Gram-solver launch that had to abort
// Side streams (Gram rows and x.w on gstream, the pipelined evaluation on
// estream) may be kept off the CUs the Gram solver's workgroups need: K_loc
// workgroups of ~159 KB of LDS each wait for WHOLE free CUs, which a side
// stream's resident workgroups rarely leave (round t+2's Gram rows enqueued
// while an evaluation runs took the C2 solver 2.55 -> 2.97 ms).  With
// COCOA_CU_MASK=1 the side streams' CU mask clears bits [0, 8 ceil(K/8)): bit i
// lies on XCD i mod 8 (clearing bits 0..63 left 24 of 32 CUs on each of the 8
// XCDs, tools/ubench/cumask.hip), and the solver's blocks are dealt round
// robin over the XCDs, ceil(K/8) per XCD.
static int side_reserve(const cocoa_ctx* c, int ncu) {
    const bool on = std::getenv("COCOA_CU_MASK") && std::atoi(std::getenv("COCOA_CU_MASK"));
    if (!on || !c->use_gram || ncu % 8 != 0 || c->K_loc > ncu / 2) return 0;
    return ((c->K_loc + 7) / 8) * 8;
}
static void make_side_stream(hipStream_t* st, int reserve, int ncu, int prio) {
    if (reserve <= 0) {
        HIPCHK(hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio));
        return;
    }
    std::vector<uint32_t> m((size_t)(ncu + 31) / 32, 0xFFFFFFFFu);
    for (int i = 0; i < reserve; ++i) m[(size_t)i / 32] &= ~(1u << (i % 32));
    if (ncu % 32) m.back() &= (1u << (ncu % 32)) - 1;
    HIPCHK(hipExtStreamCreateWithCUMask(st, (uint32_t)m.size(), m.data()));
}

static void check_status(cocoa_ctx* c) {
    // (the abort slot first: a rank whose own solver is not the Gram one still
    // receives the all-reduced flag of a rank whose solver aborted)
    if (c->abort_in_sum) {  // the all-reduced abort slot of the last exchange (cocoa_round)
        double sl = 0.0;
        HIPCHK(hipMemcpyAsync(&sl, c->dw_sum + c->d, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (sl != 0.0)
            throw Error(COCOA_E_HIP, "local solver: a hand-off between the solver's waves timed out on some rank "
                                     "(launch aborted)");
    }
    if (!c->use_gram || !c->status.p) return;
    int st = 0;
    // on the context's stream (the solver's), not the null stream, which would
    // also wait for the CU-masked side streams (created blocking)
    HIPCHK(hipMemcpyAsync(&st, c->status.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (st) throw Error(COCOA_E_HIP, "local solver: a hand-off between the solver's waves timed out (launch aborted)");
}

// ---------------------------------------------------------------- context --
extern "C" int cocoa_version(void) { return COCOA_CAPI_VERSION; }

extern "C" const char* cocoa_last_error(const cocoa_ctx* ctx) {
    if (ctx) return ctx->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    static thread_local std::string copy;
    copy = g_err;
    return copy.c_str();
}

extern "C" int cocoa_create(int device, int strict, void* stream, cocoa_ctx** out) {
    if (!out) return COCOA_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        cocoa_set_global_error("no HIP device available (libcocoa_hip needs an MI355X / gfx950 GPU)");
        return COCOA_E_NODEV;
    }
    if (device < 0 || device >= ndev) {
        cocoa_set_global_error("device ordinal out of range");
        return COCOA_E_ARG;
    }
    cocoa_ctx* c = new cocoa_ctx();
    c->device = device;
    c->strict = strict != 0;
    try {
        HIPCHK(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            throw Error(COCOA_E_NODEV, std::string("libcocoa_hip is built for gfx950; device is ") + prop.gcnArchName);
        if (stream) {
            c->stream = (hipStream_t)stream;
        } else {
            // the round's own kernels (solver, fold, eval) at the highest priority:
            // the side streams' work (next round's Gram rows, re-zeroing) yields
            // dispatch slots to them
            int lo = 0, hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
            c->own_stream = true;
        }
        HIPCHK(hipHostMalloc((void**)&c->h_eval, 16 * sizeof(double), hipHostMallocDefault));
        // jump table (A_j, C_j), j = 1..256, for the sampler
        std::vector<uint64_t> jt(512);
        for (int j = 1; j <= 256; ++j) jr_jump((uint64_t)j, &jt[2 * (j - 1)], &jt[2 * (j - 1) + 1]);
        c->jump.alloc(jt.size() * sizeof(uint64_t));
        HIPCHK(hipMemcpy(c->jump.p, jt.data(), jt.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        delete c;
        return e.code;
    }
    *out = c;
    return COCOA_OK;
}

extern "C" int cocoa_destroy(cocoa_ctx* ctx) {
    if (!ctx) return COCOA_OK;
    (void)hipSetDevice(ctx->device);
    delete ctx;
    return COCOA_OK;
}

static void upload(DevBuf& b, const void* src, size_t bytes, hipStream_t s) {
    b.alloc(bytes);
    if (bytes) HIPCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s));
}

// CSR entry arrays get 64 zero bytes of tail padding: the 16-byte loads of
// eval v4 read whole 4-entry units from an aligned base, so the last unit of
// the last tile may extend up to 3 entries past nnz.
static void upload_padded(DevBuf& b, const void* src, size_t bytes, hipStream_t s) {
    b.alloc(bytes + 64);
    HIPCHK(hipMemsetAsync((char*)b.p + bytes, 0, 64, s));
    if (bytes) HIPCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s));
}

// Row tiles for the fast eval pass: whole rows, <= kEvalTile entries and rows
// per tile; a row longer than kEvalTile is a tile of its own.
static int64_t make_tiles(const int64_t* row_ptr, int64_t n, DevBuf& out, hipStream_t s, int64_t cap = kEvalTile,
                          int64_t row_cap = kEvalRows) {
    if (row_cap < 0) row_cap = cap;
    std::vector<int64_t> t{0};
    int64_t r = 0;
    while (r < n) {
        const int64_t start = r, e0 = row_ptr[r];
        if (row_ptr[r + 1] - e0 > cap) {
            ++r;
        } else {
            while (r < n && row_ptr[r + 1] - e0 <= cap && r - start < row_cap) ++r;
        }
        t.push_back(r);
    }
    // second half: entry offset of every tile boundary, so a tile's extent is
    // four independent loads (no row_ptr round trip before the data loads)
    const size_t nb = t.size();
    for (size_t i = 0; i < nb; ++i) t.push_back(row_ptr[t[i]]);
    upload(out, t.data(), sizeof(int64_t) * t.size(), s);
    HIPCHK(hipStreamSynchronize(s));
    return (int64_t)nb - 1;
}

static void check_csr(const int64_t* row_ptr, const int32_t* col, int64_t n, int32_t d) {
    require(row_ptr[0] == 0, COCOA_E_ARG, "row_ptr[0] must be 0");
    for (int64_t r = 0; r < n; ++r) require(row_ptr[r + 1] >= row_ptr[r], COCOA_E_ARG, "row_ptr not monotone");
    const int64_t nnz = row_ptr[n];
    for (int64_t q = 0; q < nnz; ++q)
        if (col[q] < 0 || col[q] >= d)
            throw Error(COCOA_E_RANGE, "ArrayIndexOutOfBoundsException: feature index " + std::to_string(col[q]) +
                                           " outside [0," + std::to_string(d) + ")");
}

// Rows that store every feature in index order: row r = columns 0..d-1 at
// entries [r d, (r + 1) d), so the value array is the row-major matrix.
static bool is_dense(const int64_t* row_ptr, const int32_t* col, int64_t n, int32_t d) {
    if (n < 1) return false;
    for (int64_t r = 0; r <= n; ++r)
        if (row_ptr[r] != r * (int64_t)d) return false;
    for (int64_t r = 0; r < n; ++r) {
        const int32_t* c = col + r * (int64_t)d;
        for (int32_t j = 0; j < d; ++j)
            if (c[j] != j) return false;
    }
    return true;
}

static void set_train_impl(cocoa_ctx* ctx, bool dense_in, int32_t num_parts, const int64_t* part_ptr,
                           const int64_t* row_ptr, const int32_t* col, const double* val, const double* y,
                           int64_t n_rows, int32_t num_features, int32_t part_begin, int32_t num_parts_global);
static void set_test_impl(cocoa_ctx* ctx, bool dense_in, const int64_t* row_ptr, const int32_t* col,
                          const double* val, const double* y, int64_t n_rows);

// Work items of the column-block fold: block b's partition range cut into
// pieces of about kFoldItem entries (cnt(b, k): the entries of partition k in
// block b); (block, k0, k1, sole), sole = the block's only item (plain stores).
template <class F>
static std::vector<int32_t> fold_items(int64_t nblk, int K, F cnt) {
    std::vector<int32_t> items;
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t acc = 0;
        int k0 = 0;
        const size_t first = items.size();
        for (int k = 0; k < K; ++k) {
            acc += cnt(b, k);
            if (acc >= kFoldItem || k == K - 1) {
                items.insert(items.end(), {(int32_t)b, k0, k + 1, 0});
                k0 = k + 1;
                acc = 0;
            }
        }
        if (items.size() - first == 4) items[first + 3] = 1;
    }
    return items;
}

// fold_items with every block's partitions in G contiguous groups, item i of a
// block covering group i % G and its items interleaved so that item index i
// runs on XCD i % 8 (round-robin dispatch): with G = 8 each XCD then folds one
// eighth of the partitions, whose rows' rowcoef (the private tail's gathers)
// stay in its L2.  Groups with fewer pieces than the block's largest get empty
// items (k0 = k1: no reads, no stores).
template <class F>
static std::vector<int32_t> fold_items_grouped(int64_t nblk, int K, int G, F cnt) {
    std::vector<int32_t> items;
    std::vector<std::vector<std::pair<int, int>>> pieces((size_t)G);
    for (int64_t b = 0; b < nblk; ++b) {
        size_t most = 0;
        for (int g = 0; g < G; ++g) {
            auto& P = pieces[(size_t)g];
            P.clear();
            const int ka = (int)((int64_t)K * g / G), kb = (int)((int64_t)K * (g + 1) / G);
            int64_t acc = 0;
            int k0 = ka;
            for (int k = ka; k < kb; ++k) {
                acc += cnt(b, k);
                if (acc >= kFoldItem || k == kb - 1) {
                    P.emplace_back(k0, k + 1);
                    k0 = k + 1;
                    acc = 0;
                }
            }
            most = std::max(most, P.size());
        }
        for (size_t r = 0; r < most; ++r)
            for (int g = 0; g < G; ++g) {
                const auto& P = pieces[(size_t)g];
                const std::pair<int, int> pc = r < P.size() ? P[r] : std::make_pair(0, 0);
                items.insert(items.end(), {(int32_t)b, pc.first, pc.second, 0});
            }
    }
    return items;
}

// Private-column layout (cocoa_ctx::priv_ready; fast mode, COCOA_DW_PRIVATE=0
// turns it off).  lists[k]: partition k's distinct device columns in device
// order; pcol / val: the rows as the fast kernels store them.
static void build_private(cocoa_ctx* c, const int64_t* row_ptr, const int32_t* pcol, const double* val,
                          const std::vector<std::vector<int32_t>>& lists) {
    c->priv_ready = false;
    for (DevBuf* b : {&c->pcol_h, &c->pval_h, &c->row_zs, &c->row_qp, &c->fcol16_h, &c->fbnd_h, &c->fitems_h, &c->tbnd,
                      &c->tcol16, &c->trow, &c->tval})
        b->free();
    c->n_fitems_h = 0;
    c->max_uh = c->sum_uh = c->n_tail = 0;
    const char* env = std::getenv("COCOA_DW_PRIVATE");
    if (c->strict || (env && !std::atoi(env))) return;
    const int K = c->K_loc;
    const int64_t d = c->d, nnz = c->tr.nnz, n = c->tr.n;
    if (n >= ((int64_t)1 << 31)) return;
    const int64_t J = kFoldJ, nblk = (d + J - 1) / J;
    std::vector<int32_t> ncol((size_t)std::max<int64_t>(nnz, 1));
    std::vector<double> nval((size_t)std::max<int64_t>(nnz, 1));
    std::vector<int32_t> zs((size_t)std::max<int64_t>(n, 1));
    std::vector<double> qp((size_t)std::max<int64_t>(n, 1));
    std::vector<std::vector<int32_t>> heads((size_t)K);
    struct TailE {
        int32_t j, r;
        double v;
    };
    std::vector<std::vector<TailE>> tails((size_t)K);
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int tix = 0; tix < T; ++tix)
        th.emplace_back([&, tix] {
            std::vector<int32_t> cnt((size_t)d, 0), idx((size_t)d, 0);
            for (int k = tix; k < K; k += T) {
                const int64_t r0 = c->h_part_ptr[(size_t)k], r1 = c->h_part_ptr[(size_t)k + 1];
                for (int64_t q = row_ptr[r0]; q < row_ptr[r1]; ++q) cnt[(size_t)pcol[q]]++;
                std::vector<int32_t>& Hd = heads[(size_t)k];
                for (int32_t j : lists[(size_t)k])
                    if (cnt[(size_t)j] >= 2) idx[(size_t)j] = (int32_t)Hd.size(), Hd.push_back(j);
                std::vector<TailE>& Tl = tails[(size_t)k];
                for (int64_t r = r0; r < r1; ++r) {
                    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
                    int64_t zsh = 0;
                    for (int64_t q = b; q < e; ++q) zsh += cnt[(size_t)pcol[q]] >= 2;
                    int64_t ds = b, dp = b + zsh;
                    double s2 = 0.0;
                    for (int64_t q = b; q < e; ++q) {  // shared entries first, each part in stored order
                        const int32_t j = pcol[q];
                        if (cnt[(size_t)j] >= 2) {
                            ncol[(size_t)ds] = idx[(size_t)j];
                            nval[(size_t)ds++] = val[q];
                        } else {
                            ncol[(size_t)dp] = 0;  // (never read: the solver stops at row_zs)
                            nval[(size_t)dp++] = val[q];
                            s2 += val[q] * val[q];
                            Tl.push_back({j, (int32_t)r, val[q]});
                        }
                    }
                    zs[(size_t)r] = (int32_t)zsh;
                    qp[(size_t)r] = s2;
                }
                std::sort(Tl.begin(), Tl.end(), [](const TailE& x, const TailE& y) { return x.j < y.j; });
                for (int32_t j : lists[(size_t)k]) cnt[(size_t)j] = 0;
            }
        });
    for (auto& t : th) t.join();
    int64_t mu = 1, su = 0, nt = 0;
    for (auto& Hd : heads) mu = std::max<int64_t>(mu, (int64_t)Hd.size()), su += (int64_t)Hd.size();
    for (auto& Tl : tails) nt += (int64_t)Tl.size();
    if ((uint64_t)K * (uint64_t)mu >= ((uint64_t)1 << 32) || nt >= ((int64_t)1 << 31)) return;
    // the head's fold structures, as build_compact's over the shared columns
    std::vector<uint32_t> bnd((size_t)(nblk + 1) * (size_t)K), tb((size_t)(nblk + 1) * (size_t)K);
    std::vector<uint16_t> fc((size_t)K * (size_t)mu, 0);
    std::vector<int32_t> trw((size_t)std::max<int64_t>(nt, 1));
    std::vector<uint16_t> tc((size_t)std::max<int64_t>(nt, 1));
    std::vector<double> tv((size_t)std::max<int64_t>(nt, 1));
    int64_t toff = 0;
    for (int k = 0; k < K; ++k) {
        const std::vector<int32_t>& L = heads[(size_t)k];
        const std::vector<TailE>& Tl = tails[(size_t)k];
        size_t i = 0, t = 0;
        for (int64_t b = 0; b <= nblk; ++b) {
            while (i < L.size() && L[i] < b * J) ++i;
            while (t < Tl.size() && Tl[t].j < b * J) ++t;
            bnd[(size_t)b * K + k] = (uint32_t)i;
            tb[(size_t)b * K + k] = (uint32_t)(toff + (int64_t)t);
        }
        for (size_t q = 0; q < L.size(); ++q) fc[(size_t)k * mu + q] = (uint16_t)(L[q] & (J - 1));
        for (size_t q = 0; q < Tl.size(); ++q) {
            trw[(size_t)toff + q] = Tl[q].r;
            tc[(size_t)toff + q] = (uint16_t)(Tl[q].j & (J - 1));
            tv[(size_t)toff + q] = Tl[q].v;
        }
        toff += (int64_t)Tl.size();
    }
    auto cnt_bk = [&](int64_t b, int k) -> int64_t {
        return (int64_t)(bnd[(size_t)(b + 1) * K + k] - bnd[(size_t)b * K + k]) +
               (int64_t)(tb[(size_t)(b + 1) * K + k] - tb[(size_t)b * K + k]);
    };
    // (COCOA_FOLD_XCD=0: the plain block-major items, A/B)
    const char* fx = std::getenv("COCOA_FOLD_XCD");
    const bool grouped = !(fx && !std::atoi(fx)) && K >= 64;
    const std::vector<int32_t> items = grouped ? fold_items_grouped(nblk, K, 8, cnt_bk) : fold_items(nblk, K, cnt_bk);
    hipStream_t s = c->stream;
    upload_padded(c->pcol_h, ncol.data(), sizeof(int32_t) * (size_t)nnz, s);
    upload_padded(c->pval_h, nval.data(), sizeof(double) * (size_t)nnz, s);
    upload(c->row_zs, zs.data(), sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1), s);
    upload(c->row_qp, qp.data(), sizeof(double) * (size_t)std::max<int64_t>(n, 1), s);
    upload(c->fbnd_h, bnd.data(), sizeof(uint32_t) * bnd.size(), s);
    upload_padded(c->fcol16_h, fc.data(), sizeof(uint16_t) * fc.size(), s);
    upload(c->fitems_h, items.data(), sizeof(int32_t) * items.size(), s);
    upload(c->tbnd, tb.data(), sizeof(uint32_t) * tb.size(), s);
    upload_padded(c->trow, trw.data(), sizeof(int32_t) * trw.size(), s);
    upload_padded(c->tcol16, tc.data(), sizeof(uint16_t) * tc.size(), s);
    upload_padded(c->tval, tv.data(), sizeof(double) * tv.size(), s);
    HIPCHK(hipStreamSynchronize(s));
    c->n_fitems_h = (int32_t)(items.size() / 4);
    c->max_uh = mu;
    c->sum_uh = su;
    c->n_tail = nt;
    c->priv_ready = true;
}

// Compact deltaW layout (see cocoa_ctx::compact_ready).  COCOA_DW_COMPACT=0 / 1
// forces it off / on (tests); on by default once K_loc * d * 8 >= 1 GiB and the
// distinct columns per partition are fewer than d / 4.
static void build_compact(cocoa_ctx* c, const int64_t* row_ptr, const int32_t* pcol, const double* val) {
    c->compact_ready = false;
    c->priv_ready = false;
    c->col_local.free();
    c->fptr.free();
    c->fpos.free();
    const int K = c->K_loc;
    const int64_t d = c->d;
    const char* env = std::getenv("COCOA_DW_COMPACT");
    if (env ? std::atoi(env) == 0 : (size_t)K * (size_t)d * sizeof(double) < ((size_t)1 << 30)) return;
    const int64_t nnz = c->tr.nnz;
    std::vector<int32_t> cl((size_t)std::max<int64_t>(nnz, 1));
    std::vector<std::vector<int32_t>> lists((size_t)K);
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int tix = 0; tix < T; ++tix)
        th.emplace_back([&, tix] {
            std::vector<int32_t> mark((size_t)d, -1), idx((size_t)d, 0);
            for (int k = tix; k < K; k += T) {
                const int64_t q0 = row_ptr[c->h_part_ptr[(size_t)k]], q1 = row_ptr[c->h_part_ptr[(size_t)k + 1]];
                std::vector<int32_t>& L = lists[(size_t)k];
                for (int64_t q = q0; q < q1; ++q) {
                    const int32_t j = pcol[q];
                    if (mark[(size_t)j] != k) mark[(size_t)j] = k, L.push_back(j);
                }
                std::sort(L.begin(), L.end());  // device order: adjacent columns, adjacent positions
                for (size_t i = 0; i < L.size(); ++i) idx[(size_t)L[i]] = (int32_t)i;
                for (int64_t q = q0; q < q1; ++q) cl[(size_t)q] = idx[(size_t)pcol[q]];
            }
        });
    for (auto& t : th) t.join();
    int64_t mu = 1, su = 0;
    for (auto& L : lists) mu = std::max<int64_t>(mu, (int64_t)L.size()), su += (int64_t)L.size();
    if (!env && mu * 4 > d) return;  // not sparse enough per partition to pay
    if ((uint64_t)K * (uint64_t)mu >= ((uint64_t)1 << 32)) return;
    std::vector<int64_t> fp((size_t)d + 1, 0);
    for (auto& L : lists)
        for (int32_t j : L) fp[(size_t)j + 1]++;
    for (int64_t j = 0; j < d; ++j) fp[(size_t)j + 1] += fp[(size_t)j];
    std::vector<uint32_t> pos((size_t)std::max<int64_t>(su, 1));
    std::vector<int64_t> cur(fp.begin(), fp.end() - 1);
    for (int k = 0; k < K; ++k) {  // partition order inside every column's list
        const std::vector<int32_t>& L = lists[(size_t)k];
        for (size_t i = 0; i < L.size(); ++i) pos[(size_t)cur[(size_t)L[i]]++] = (uint32_t)((uint64_t)k * mu + i);
    }
    hipStream_t s = c->stream;
    upload_padded(c->col_local, cl.data(), sizeof(int32_t) * (size_t)nnz, s);
    upload(c->fptr, fp.data(), sizeof(int64_t) * fp.size(), s);
    upload(c->fpos, pos.data(), sizeof(uint32_t) * pos.size(), s);
    c->fcol16.free();
    c->fbnd.free();
    c->fitems.free();
    c->ftmp.free();
    c->n_fitems = c->n_fblk = 0;
    if (!c->strict) {
        // Fast fold by column blocks (fold_blocks_kernel): block b = device
        // columns [b J, (b+1) J); each slice lists its columns in device order,
        // so block b's entries of slice k are the contiguous positions
        // [fbnd[b][k], fbnd[b+1][k]).  Work items cut each block's partition
        // range into pieces of about kFoldItem entries.
        const int64_t J = kFoldJ, nblk = (d + J - 1) / J;
        std::vector<uint32_t> bnd((size_t)(nblk + 1) * (size_t)K);
        std::vector<uint16_t> fc((size_t)K * (size_t)mu, 0);
        for (int k = 0; k < K; ++k) {
            const std::vector<int32_t>& L = lists[(size_t)k];
            size_t i = 0;
            for (int64_t b = 0; b <= nblk; ++b) {
                while (i < L.size() && L[i] < b * J) ++i;
                bnd[(size_t)b * K + k] = (uint32_t)i;
            }
            for (size_t q = 0; q < L.size(); ++q) fc[(size_t)k * mu + q] = (uint16_t)(L[q] & (J - 1));
        }
        const std::vector<int32_t> items = fold_items(nblk, K, [&](int64_t b, int k) -> int64_t {
            return (int64_t)(bnd[(size_t)(b + 1) * K + k] - bnd[(size_t)b * K + k]);
        });
        upload(c->fbnd, bnd.data(), sizeof(uint32_t) * bnd.size(), s);
        upload_padded(c->fcol16, fc.data(), sizeof(uint16_t) * fc.size(), s);
        upload(c->fitems, items.data(), sizeof(int32_t) * items.size(), s);
        c->ftmp.alloc_zero(sizeof(double) * (size_t)d, s);
        c->n_fitems = (int32_t)(items.size() / 4);
        c->n_fblk = (int32_t)nblk;
    }
    HIPCHK(hipStreamSynchronize(s));
    c->max_u = mu;
    c->sum_u = su;
    c->compact_ready = true;
    build_private(c, row_ptr, pcol, val, lists);
}

// ------------------------------------------------------------------- data --
extern "C" int cocoa_set_train_dense(cocoa_ctx* ctx, int32_t num_parts, const int64_t* part_ptr, const double* X,
                                     const double* y, int64_t n_rows, int32_t num_features, int32_t part_begin,
                                     int32_t num_parts_global) {
    if (!ctx) return COCOA_E_ARG;
    if (!X || n_rows < 0 || num_features < 1) {
        ctx->err = "cocoa_set_train_dense: bad argument";
        cocoa_set_global_error(ctx->err);
        return COCOA_E_ARG;
    }
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        group_set_train(ctx, true, num_parts, part_ptr, nullptr, nullptr, X, y, n_rows, num_features, part_begin,
                        num_parts_global);
        return COCOA_OK;
    }
    std::vector<int64_t> rp((size_t)n_rows + 1);
    for (int64_t r = 0; r <= n_rows; ++r) rp[(size_t)r] = r * (int64_t)num_features;
    set_train_impl(ctx, true, num_parts, part_ptr, rp.data(), nullptr, X, y, n_rows, num_features, part_begin,
                   num_parts_global);
    CAPI_END(ctx)
}

extern "C" int cocoa_set_test_dense(cocoa_ctx* ctx, const double* X, const double* y, int64_t n_rows) {
    if (!ctx) return COCOA_E_ARG;
    if (!X || n_rows < 0 || ctx->d < 1) {
        ctx->err = ctx->d < 1 ? "cocoa_set_test_dense: call cocoa_set_train first" : "cocoa_set_test_dense: bad argument";
        cocoa_set_global_error(ctx->err);
        return ctx->d < 1 ? COCOA_E_STATE : COCOA_E_ARG;
    }
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        group_set_test(ctx, true, nullptr, nullptr, X, y, n_rows);
        return COCOA_OK;
    }
    std::vector<int64_t> rp((size_t)n_rows + 1);
    for (int64_t r = 0; r <= n_rows; ++r) rp[(size_t)r] = r * (int64_t)ctx->d;
    set_test_impl(ctx, true, rp.data(), nullptr, X, y, n_rows);
    CAPI_END(ctx)
}

extern "C" int cocoa_set_train(cocoa_ctx* ctx, int32_t num_parts, const int64_t* part_ptr, const int64_t* row_ptr,
                               const int32_t* col, const double* val, const double* y, int64_t n_rows,
                               int32_t num_features, int32_t part_begin, int32_t num_parts_global) {
    CAPI_BEGIN(ctx)
    require(col != nullptr || (row_ptr && n_rows >= 0 && row_ptr[n_rows] == 0), COCOA_E_ARG,
            "cocoa_set_train: null column array");
    // a CSR whose rows are all empty may pass col == NULL: it stays CSR (the
    // dense layout is selected only by cocoa_set_train_dense)
    static const int32_t no_col = 0;
    if (!col) col = &no_col;
    if (ctx->is_group()) {
        group_set_train(ctx, false, num_parts, part_ptr, row_ptr, col, val, y, n_rows, num_features, part_begin,
                        num_parts_global);
        return COCOA_OK;
    }
    set_train_impl(ctx, false, num_parts, part_ptr, row_ptr, col, val, y, n_rows, num_features, part_begin,
                   num_parts_global);
    CAPI_END(ctx)
}

// dense_in: dense rows (row r = columns 0..d-1 at entries [r d, (r+1) d), col unused)
// The fast evaluation's hot / cold split of the train rows (EvalArgs::row_base):
// entries of device columns < kEvalHot into one CSR (16-bit columns), the rest
// into another, each row's entries in stored order, and eval tiles for both.
// With d > kEvalHot + kEvalWarm (C4) the columns [kEvalHot, kEvalHot +
// kEvalWarm) get a CSR of their own (16-bit offsets), the warm tier; the cold
// CSR then holds the columns past it.  Measured on C4 it gains nothing (1.107
// against 1.101-1.106 ms, profiles/r06/ab_r09j_c4_warm.txt): the cold pass is
// bound by its gather instructions, not by where w lives, so the warm tier is
// built only with COCOA_EVAL_WARM=1.  COCOA_EVAL_SPLIT=0 keeps the one-pass
// evaluation.
static void build_eval_split(cocoa_ctx* ctx, const int64_t* row_ptr, const std::vector<int32_t>& pcol,
                             const double* val, int64_t n, int32_t d, hipStream_t s) {
    const char* se = std::getenv("COCOA_EVAL_SPLIT");
    ctx->split_ready = false;
    ctx->te_split = false;  // (row_base is re-sized below; cocoa_set_test splits the test rows again)
    ctx->hot_tr = Csr{};
    ctx->cold_tr = Csr{};
    ctx->warm_tr = Csr{};
    ctx->n_warm_tiles = 0;
    if ((se && !std::atoi(se)) || ctx->strict || n < 1) return;
    const char* sw = std::getenv("COCOA_EVAL_WARM");
    // warm tier end (columns below it and past kEvalHot); kEvalHot: none
    const int32_t wend = (sw && std::atoi(sw) && d > kEvalHot + kEvalWarm) ? kEvalHot + kEvalWarm : kEvalHot;
    std::vector<int64_t> hp((size_t)n + 1), cp((size_t)n + 1), mp((size_t)n + 1);
    hp[0] = cp[0] = mp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t h = 0, m = 0;
        for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) {
            h += pcol[(size_t)q] < kEvalHot;
            m += pcol[(size_t)q] >= kEvalHot && pcol[(size_t)q] < wend;
        }
        hp[(size_t)r + 1] = hp[(size_t)r] + h;
        mp[(size_t)r + 1] = mp[(size_t)r] + m;
        cp[(size_t)r + 1] = cp[(size_t)r] + (row_ptr[r + 1] - row_ptr[r] - h - m);
    }
    const int64_t nh = hp[(size_t)n], nc = cp[(size_t)n], nm = mp[(size_t)n];
    std::vector<uint16_t> hc((size_t)std::max<int64_t>(nh, 1)), mc((size_t)std::max<int64_t>(nm, 1));
    std::vector<double> hv((size_t)std::max<int64_t>(nh, 1)), cv((size_t)std::max<int64_t>(nc, 1));
    std::vector<double> mv((size_t)std::max<int64_t>(nm, 1));
    std::vector<int32_t> cc((size_t)std::max<int64_t>(nc, 1));
    // each part of a row in ascending device column: neighbouring lanes of a gather
    // then read neighbouring words of w (fewer lines per gather instruction, fewer
    // LDS bank conflicts in the hot pass); the sums are reassociated anyway
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int tix = 0; tix < T; ++tix)
        th.emplace_back([&, tix] {
            std::vector<std::pair<int32_t, double>> tmp;
            for (int64_t r = n * tix / T; r < n * (tix + 1) / T; ++r) {
                tmp.clear();
                for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) tmp.emplace_back(pcol[(size_t)q], val[q]);
                std::stable_sort(tmp.begin(), tmp.end(),
                                 [](const std::pair<int32_t, double>& x, const std::pair<int32_t, double>& y) {
                                     return x.first < y.first;
                                 });
                int64_t a = hp[(size_t)r], b = cp[(size_t)r], m = mp[(size_t)r];
                for (const auto& cvp : tmp) {
                    if (cvp.first < kEvalHot) {
                        hc[(size_t)a] = (uint16_t)cvp.first;
                        hv[(size_t)a++] = cvp.second;
                    } else if (cvp.first < wend) {
                        mc[(size_t)m] = (uint16_t)(cvp.first - kEvalHot);
                        mv[(size_t)m++] = cvp.second;
                    } else {
                        cc[(size_t)b] = cvp.first;
                        cv[(size_t)b++] = cvp.second;
                    }
                }
            }
        });
    for (auto& t : th) t.join();
    ctx->hot_tr.n = ctx->cold_tr.n = n;
    ctx->hot_tr.nnz = nh;
    ctx->cold_tr.nnz = nc;
    upload(ctx->hot_tr.row_ptr, hp.data(), sizeof(int64_t) * (size_t)(n + 1), s);
    upload_padded(ctx->hot_tr.col16, hc.data(), sizeof(uint16_t) * (size_t)nh, s);
    upload_padded(ctx->hot_tr.val, hv.data(), sizeof(double) * (size_t)nh, s);
    upload(ctx->cold_tr.row_ptr, cp.data(), sizeof(int64_t) * (size_t)(n + 1), s);
    upload_padded(ctx->cold_tr.col, cc.data(), sizeof(int32_t) * (size_t)nc, s);
    upload_col16(ctx->cold_tr.col16, cc, nc, d, s);  // (synchronises: the host vectors may go)
    upload_padded(ctx->cold_tr.val, cv.data(), sizeof(double) * (size_t)nc, s);
    int hcap = kEvalTile, ccap = kEvalTile;
    eval_split_tiles(&hcap, &ccap);
    ctx->n_hot_tiles = make_tiles(hp.data(), n, ctx->hot_tiles, s, hcap);    // (synchronises)
    ctx->n_cold_tiles = make_tiles(cp.data(), n, ctx->cold_tiles, s, ccap);
    if (wend > kEvalHot) {
        ctx->warm_tr.n = n;
        ctx->warm_tr.nnz = nm;
        upload(ctx->warm_tr.row_ptr, mp.data(), sizeof(int64_t) * (size_t)(n + 1), s);
        upload_padded(ctx->warm_tr.col16, mc.data(), sizeof(uint16_t) * (size_t)nm, s);
        upload_padded(ctx->warm_tr.val, mv.data(), sizeof(double) * (size_t)nm, s);
        ctx->n_warm_tiles = make_tiles(mp.data(), n, ctx->warm_tiles, s, hcap);  // (synchronises)
    }
    ctx->row_base.alloc(sizeof(double) * (size_t)n);
    ctx->split_ready = true;
}

// The test rows' hot / cold split (EvalArgs::th_*), on a split training set:
// each test row's entries of device columns < kEvalHot go to the hot pass (w
// from LDS, no gather; their dot into row_base[n + r]), the rest stay in the
// cold pass's test tiles.  C2's 50,000 test rows hold 3.8 M entries, 78% of
// them hot: unsplit, the cold pass gathered w for all of them.  Each part in
// ascending device column, like the train split (the sums are reassociated).
static void build_test_split(cocoa_ctx* ctx, const int64_t* row_ptr, const std::vector<int32_t>& pcol,
                             const double* val, int64_t n, hipStream_t s) {
    ctx->te_split = false;
    const char* ts = std::getenv("COCOA_EVAL_TEST_SPLIT");  // (=0: the test rows whole in the cold pass)
    if (!ctx->split_ready || ctx->strict || n < 1 || (ts && !std::atoi(ts))) return;
    std::vector<int64_t> hp((size_t)n + 1), cp((size_t)n + 1);
    hp[0] = cp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t h = 0;
        for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) h += pcol[(size_t)q] < kEvalHot;
        hp[(size_t)r + 1] = hp[(size_t)r] + h;
        cp[(size_t)r + 1] = cp[(size_t)r] + (row_ptr[r + 1] - row_ptr[r] - h);
    }
    const int64_t nh = hp[(size_t)n], nc = cp[(size_t)n];
    std::vector<uint16_t> hc((size_t)std::max<int64_t>(nh, 1));
    std::vector<double> hv((size_t)std::max<int64_t>(nh, 1)), cv((size_t)std::max<int64_t>(nc, 1));
    std::vector<int32_t> cc((size_t)std::max<int64_t>(nc, 1));
    std::vector<std::pair<int32_t, double>> tmp;
    for (int64_t r = 0; r < n; ++r) {
        tmp.clear();
        for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) tmp.emplace_back(pcol[(size_t)q], val[q]);
        std::stable_sort(tmp.begin(), tmp.end(), [](const std::pair<int32_t, double>& x, const std::pair<int32_t, double>& y) {
            return x.first < y.first;
        });
        int64_t a = hp[(size_t)r], b = cp[(size_t)r];
        for (const auto& cvp : tmp) {
            if (cvp.first < kEvalHot) {
                hc[(size_t)a] = (uint16_t)cvp.first;
                hv[(size_t)a++] = cvp.second;
            } else {
                cc[(size_t)b] = cvp.first;
                cv[(size_t)b++] = cvp.second;
            }
        }
    }
    ctx->hot_te = Csr{};
    ctx->cold_te = Csr{};
    ctx->hot_te.n = ctx->cold_te.n = n;
    ctx->hot_te.nnz = nh;
    ctx->cold_te.nnz = nc;
    upload(ctx->hot_te.row_ptr, hp.data(), sizeof(int64_t) * (size_t)(n + 1), s);
    upload_padded(ctx->hot_te.col16, hc.data(), sizeof(uint16_t) * (size_t)nh, s);
    upload_padded(ctx->hot_te.val, hv.data(), sizeof(double) * (size_t)nh, s);
    upload(ctx->cold_te.row_ptr, cp.data(), sizeof(int64_t) * (size_t)(n + 1), s);
    upload_padded(ctx->cold_te.col, cc.data(), sizeof(int32_t) * (size_t)nc, s);
    upload_col16(ctx->cold_te.col16, cc, nc, ctx->d, s);  // (synchronises: the host vectors may go)
    upload_padded(ctx->cold_te.val, cv.data(), sizeof(double) * (size_t)nc, s);
    int hcap = kEvalTile, ccap = kEvalTile;
    eval_split_tiles(&hcap, &ccap);
    ctx->n_hot_t_tiles = make_tiles(hp.data(), n, ctx->hot_t_tiles, s, hcap);  // (synchronises)
    ctx->n_cold_t_tiles = make_tiles(cp.data(), n, ctx->cold_t_tiles, s, ccap);
    ctx->row_base.alloc(sizeof(double) * (size_t)(ctx->tr.n + n));
    ctx->te_split = ctx->n_hot_t_tiles > 0;
}

static void set_train_impl(cocoa_ctx* ctx, bool dense_in, int32_t num_parts, const int64_t* part_ptr,
                           const int64_t* row_ptr, const int32_t* col, const double* val, const double* y,
                           int64_t n_rows, int32_t num_features, int32_t part_begin, int32_t num_parts_global) {
    require(dense_in || col != nullptr, COCOA_E_ARG, "cocoa_set_train: null column array");
    ctx->gram_quiesce();  // a Gram prefetch reads the CSR being replaced
    ctx->eval_quiesce();  // so does a pending evaluation
    require(num_parts >= 1 && part_ptr && row_ptr && y && n_rows >= 0 && num_features >= 1, COCOA_E_ARG,
            "cocoa_set_train: bad argument");
    require(part_begin >= 0 && num_parts_global >= part_begin + num_parts, COCOA_E_ARG,
            "cocoa_set_train: bad partition range");
    require(part_ptr[0] == 0 && part_ptr[num_parts] == n_rows, COCOA_E_ARG, "part_ptr must span [0, n_rows]");
    for (int k = 0; k < num_parts; ++k) require(part_ptr[k + 1] >= part_ptr[k], COCOA_E_ARG, "part_ptr not monotone");
    if (!dense_in) check_csr(row_ptr, col, n_rows, num_features);
    const int64_t nnz = row_ptr[n_rows];
    require(val != nullptr || nnz == 0, COCOA_E_ARG, "cocoa_set_train: null value array");
    ctx->tr_dense = dense_in ? n_rows >= 1 : is_dense(row_ptr, col, n_rows, num_features);
    // A test set stored for the previous training set is dropped: its columns are
    // in that set's device feature order and its eval tiles were sized for that d
    // (eval_tile_entries), so keeping it could evaluate wrong columns or run
    // 4,096-entry tiles under the 2,048-entry kernel.  Call cocoa_set_test again.
    ctx->csc_ready = false;  // (the mb-SGD CSC copy is of the old rows)
    ctx->te_split = false;
    if (ctx->has_test) {
        ctx->has_test = false;
        ctx->te_dense = false;
        ctx->te.n = ctx->te.nnz = 0;
        ctx->n_t_tiles = 0;
        ctx->n_test_glob = -1;
    }
    ctx->K_loc = num_parts;
    ctx->K_glob = num_parts_global;
    ctx->part_begin = part_begin;
    ctx->d = num_features;
    ctx->tr.n = n_rows;
    ctx->tr.nnz = nnz;
    ctx->h_part_ptr.assign(part_ptr, part_ptr + num_parts + 1);
    ctx->max_nl = 0;
    ctx->min_nl = INT32_MAX;
    for (int k = 0; k < num_parts; ++k) {
        const int64_t nl = part_ptr[k + 1] - part_ptr[k];
        require(nl <= INT32_MAX, COCOA_E_ARG, "partition too large");
        ctx->max_nl = std::max<int32_t>(ctx->max_nl, (int32_t)nl);
        ctx->min_nl = std::min<int32_t>(ctx->min_nl, (int32_t)nl);
    }
    // Math.pow(x.norm(2), 2) per row (CoCoA.scala:173), in stored order; and
    // duplicate-column flags (rows whose scatter must stay sequential)
    std::vector<double> sq((size_t)std::max<int64_t>(n_rows, 1));
    std::vector<uint8_t> fl((size_t)std::max<int64_t>(n_rows, 1), 0);
    ctx->any_dup = false;
    ctx->max_z = 0;
    for (int64_t r = 0; r < n_rows; ++r) ctx->max_z = (int32_t)std::max<int64_t>(ctx->max_z, row_ptr[r + 1] - row_ptr[r]);
    std::vector<int64_t> seen_at((size_t)num_features, -1);
    for (int64_t r = 0; r < n_rows; ++r) {
        double s = 0.0;
        bool sorted = true;
        for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) {
            s += val[q] * val[q];
            if (!dense_in && q > row_ptr[r] && col[q] <= col[q - 1]) sorted = false;
        }
        const double nr = std::sqrt(s);
        sq[(size_t)r] = nr * nr;
        if (!sorted) {
            for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) {
                if (seen_at[(size_t)col[q]] == r) fl[(size_t)r] = 1;
                seen_at[(size_t)col[q]] = r;
            }
            if (fl[(size_t)r]) ctx->any_dup = true;
        }
    }
    // Device feature order: columns relabelled by descending frequency in this
    // rank's rows (ties by index) so the hottest coordinates of deltaW are the
    // first ones (the LDS-resident slice of the solver).  Entry order inside a
    // row is unchanged, so every dot product sums the same terms in the same
    // order; w crosses the C ABI in the original order.
    {
        std::vector<int64_t> freq((size_t)num_features, 0);
        if (dense_in)  // every column n_rows times: the identity order
            std::fill(freq.begin(), freq.end(), n_rows);
        else
            for (int64_t q = 0; q < nnz; ++q) freq[(size_t)col[q]]++;
        std::vector<int32_t> order((size_t)num_features);
        for (int32_t j = 0; j < num_features; ++j) order[(size_t)j] = j;
        std::stable_sort(order.begin(), order.end(),
                         [&](int32_t x, int32_t y) { return freq[(size_t)x] > freq[(size_t)y]; });
        ctx->inv.assign(order.begin(), order.end());            // new -> old
        ctx->perm.assign((size_t)num_features, 0);              // old -> new
        for (int32_t j = 0; j < num_features; ++j) ctx->perm[(size_t)order[(size_t)j]] = j;
        ctx->n_hot_nnz.assign((size_t)num_features + 1, 0);      // nnz share of the first j columns
        for (int32_t j = 0; j < num_features; ++j)
            ctx->n_hot_nnz[(size_t)j + 1] = ctx->n_hot_nnz[(size_t)j] + freq[(size_t)order[(size_t)j]];
    }
    std::vector<int32_t> pcol;
    if (!dense_in) {
        pcol.resize((size_t)std::max<int64_t>(nnz, 1));
        for (int64_t q = 0; q < nnz; ++q) pcol[(size_t)q] = ctx->perm[(size_t)col[q]];
    }
    // Fast mode: every row stores its entries in kGramRuns runs (device column
    // c % kGramRuns), each in stored order, so that each of
    // the Gram solver's memory waves (solver_gram.h) streams one contiguous run
    // per row.  Only the fast kernels see this order (their dots are
    // reassociated anyway); strict mode keeps the stored order of every row.
    std::vector<double> pval;
    std::vector<int32_t> zcv;
    const bool split_classes = !ctx->strict && !dense_in && !ctx->tr_dense && nnz > 0;  // dense rows: val is X[n][d]
    // (device column parity splits the entries evenly; a hot / cold split -- the
    // LDS-resident columns vs the rest, or the columns holding the first half of
    // the entries vs the rest -- measured 3.93 / 2.97 ms against 2.70: the first
    // class's fetch and memory waves carry most of the units; r03 A/B; the
    // mirrored halves' hot / cold runs 2.85 against 2.67 ms, r06p)
    ctx->hot_split = 0;
    if (split_classes) {
        pval.resize((size_t)nnz);
        zcv.resize((size_t)std::max<int64_t>(n_rows, 1) * kGramRuns);
        std::vector<int32_t> ncol((size_t)std::max<int64_t>(nnz, 1));
        const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (int tix = 0; tix < T; ++tix)
            th.emplace_back([&, tix] {
                for (int64_t r = n_rows * tix / T; r < n_rows * (tix + 1) / T; ++r) {
                    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
                    int64_t cnt[kGramRuns] = {}, at[kGramRuns];
                    for (int64_t q = b; q < e; ++q) ++cnt[pcol[(size_t)q] % kGramRuns];
                    int64_t run = b;
                    for (int c = 0; c < kGramRuns; ++c) {
                        at[c] = run;
                        run += cnt[c];
                    }
                    for (int c = 0; c < kGramRuns; ++c)  // ends of runs 0 .. R-2 (row-relative), then the row length
                        zcv[(size_t)r * kGramRuns + c] = (int32_t)((c < kGramRuns - 1 ? at[c] + cnt[c] : e) - b);
                    for (int64_t q = b; q < e; ++q) {
                        const int64_t dst = at[pcol[(size_t)q] % kGramRuns]++;
                        ncol[(size_t)dst] = pcol[(size_t)q];
                        pval[(size_t)dst] = val[q];
                    }
                }
            });
        for (auto& t : th) t.join();
        pcol.swap(ncol);
    }
    hipStream_t s = ctx->stream;
    upload(ctx->d_perm, ctx->perm.data(), sizeof(int32_t) * (size_t)num_features, s);
    upload(ctx->d_inv, ctx->inv.data(), sizeof(int32_t) * (size_t)num_features, s);
    upload(ctx->tr.row_ptr, row_ptr, sizeof(int64_t) * (size_t)(n_rows + 1), s);
    ctx->tr.col_lazy = dense_in;
    if (dense_in) {
        ctx->tr.col.free();
        ctx->tr.col16.free();
    } else {
        upload_padded(ctx->tr.col, pcol.data(), sizeof(int32_t) * (size_t)nnz, s);
        upload_col16(ctx->tr.col16, pcol, nnz, num_features, s);
    }
    upload_padded(ctx->tr.val, split_classes ? pval.data() : val, sizeof(double) * (size_t)nnz, s);
    if (split_classes)
        upload(ctx->row_zc, zcv.data(), sizeof(int32_t) * kGramRuns * (size_t)n_rows, s);
    else
        ctx->row_zc.free();
    upload(ctx->tr.y, y, sizeof(double) * (size_t)n_rows, s);
    upload(ctx->sqn, sq.data(), sizeof(double) * (size_t)n_rows, s);
    upload(ctx->rowflags, fl.data(), (size_t)n_rows, s);
    upload(ctx->part_ptr, part_ptr, sizeof(int64_t) * (size_t)(num_parts + 1), s);
    ctx->n_tiles = make_tiles(row_ptr, n_rows, ctx->tiles, s, eval_tile_entries(num_features));
    if (!dense_in && !ctx->tr_dense)
        build_eval_split(ctx, row_ptr, pcol, split_classes ? pval.data() : val, n_rows, num_features, s);
    else
        ctx->split_ready = false;
    if (dense_in) {
        ctx->compact_ready = false;  // dense rows touch every column: no compact slices
        ctx->priv_ready = false;
        ctx->col_local.free();
        ctx->fptr.free();
        ctx->fpos.free();
    } else {
        build_compact(ctx, row_ptr, pcol.data(), split_classes ? pval.data() : val);
    }
    HIPCHK(hipStreamSynchronize(s));
    ctx->inited = false;
}

extern "C" int cocoa_set_test(cocoa_ctx* ctx, const int64_t* row_ptr, const int32_t* col, const double* val,
                              const double* y, int64_t n_rows) {
    CAPI_BEGIN(ctx)
    require(col != nullptr || (row_ptr && n_rows >= 0 && row_ptr[n_rows] == 0), COCOA_E_ARG,
            "cocoa_set_test: null column array");
    static const int32_t no_col = 0;  // all-empty CSR with col == NULL: still CSR
    if (!col) col = &no_col;
    if (ctx->is_group()) {
        group_set_test(ctx, false, row_ptr, col, val, y, n_rows);
        return COCOA_OK;
    }
    set_test_impl(ctx, false, row_ptr, col, val, y, n_rows);
    CAPI_END(ctx)
}

// dense_in: dense rows (col unused)
static void set_test_impl(cocoa_ctx* ctx, bool dense_in, const int64_t* row_ptr, const int32_t* col,
                          const double* val, const double* y, int64_t n_rows) {
    require(dense_in || col != nullptr, COCOA_E_ARG, "cocoa_set_test: null column array");
    ctx->eval_quiesce();  // a pending evaluation reads the test rows being replaced
    ctx->te_split = false;
    require(ctx->d > 0, COCOA_E_STATE, "cocoa_set_test: call cocoa_set_train first");
    require(row_ptr && y && n_rows >= 0, COCOA_E_ARG, "cocoa_set_test: bad argument");
    if (!dense_in) check_csr(row_ptr, col, n_rows, ctx->d);
    const int64_t nnz = row_ptr[n_rows];
    require(val != nullptr || nnz == 0, COCOA_E_ARG, "cocoa_set_test: null value array");
    hipStream_t s = ctx->stream;
    ctx->te_dense = dense_in ? n_rows >= 1 : is_dense(row_ptr, col, n_rows, ctx->d);
    ctx->te.n = n_rows;
    ctx->te.nnz = nnz;
    upload(ctx->te.row_ptr, row_ptr, sizeof(int64_t) * (size_t)(n_rows + 1), s);
    ctx->te.col_lazy = dense_in;
    if (dense_in) {
        ctx->te.col.free();
        ctx->te.col16.free();
    } else {
        std::vector<int32_t> pcol((size_t)std::max<int64_t>(nnz, 1));
        for (int64_t q = 0; q < nnz; ++q) pcol[(size_t)q] = ctx->perm[(size_t)col[q]];  // device feature order
        upload_padded(ctx->te.col, pcol.data(), sizeof(int32_t) * (size_t)nnz, s);
        upload_col16(ctx->te.col16, pcol, nnz, ctx->d, s);
        build_test_split(ctx, row_ptr, pcol, val, n_rows, s);
    }
    upload_padded(ctx->te.val, val, sizeof(double) * (size_t)nnz, s);
    upload(ctx->te.y, y, sizeof(double) * (size_t)n_rows, s);
    ctx->n_t_tiles = make_tiles(row_ptr, n_rows, ctx->t_tiles, s, eval_tile_entries(ctx->d));
    HIPCHK(hipStreamSynchronize(s));
    ctx->has_test = true;
    ctx->n_test_glob = -1;  // (re-exchanged at the next multi-rank cocoa_eval_begin)
    if (ctx->inited) {
        const size_t rows = (size_t)(ctx->tr.n + ctx->te.n);
        ctx->row_scratch.alloc(sizeof(double) * std::max<size_t>(rows, 1));
    }
}

// ----------------------------------------------------------------- solver --
static bool is_sdca(int m) { return m == COCOA_METHOD_COCOA_PLUS || m == COCOA_METHOD_COCOA || m == COCOA_METHOD_MBCD; }
static int solver_mode(int m) {
    return m == COCOA_METHOD_COCOA_PLUS ? MODE_PLUS : m == COCOA_METHOD_COCOA ? MODE_COCOA : MODE_MBCD;
}
static int32_t wrap32(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }

// vec_len: length of the solver's mutable vector (d, or the compact slice)
// LDS layout of the chain solver (one workgroup per partition).  need_prod:
// the loader forms x.w itself (no step plan: the unit API), which needs the
// product buffer.  With more partitions than CUs (C4 on one GPU: 1,024 on
// 256) the workgroups queue for CUs, so the layout is sized for
// ceil(K_loc / CUs) workgroups per CU (at most 4): the stream buffers shrink
// (1,024 or 512 staged entries per batch instead of 2,048) and alpha moves to
// HBM when it does not fit.  (r03: 93.5 KB, one workgroup per CU, the 1,024
// C4 chains ran four after another.)
static void plan_solver(cocoa_ctx* c, int64_t vec_len, bool need_prod = true) {
    SolverArgs& a = c->sa;
    size_t off = 0;
    const size_t vec_bytes = align16(sizeof(double) * (size_t)vec_len);
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    const int want = (int)std::min<int64_t>(4, std::max<int64_t>(1, ((int64_t)c->K_loc + ncu - 1) / std::max(ncu, 1)));
    const size_t budget = want > 1 ? (kLdsMax / (size_t)want) & ~(size_t)1023 : kLdsMax;
    // long rows (dense data, C3: 2,000 entries) would leave one row per batch and
    // make the loader's per-batch latency the bound: double the stream instead
    // (alpha then moves to HBM when it no longer fits; the chain prefetches it)
    const double zavg = c->tr.n ? (double)c->tr.nnz / (double)c->tr.n : 0.0;
    size_t cap = zavg * 4 > (double)kStreamCap ? 2 * (size_t)kStreamCap : (size_t)kStreamCap;
    auto fixed_for = [&](size_t cp) {
        return 2 * align16(cp * 4) + 2 * align16(cp * 8) + 2 * align16(sizeof(BatchMeta)) +
               (need_prod ? align16(cp * 8) : 0) + align16(sizeof(double) * kRegChunks * 64);
    };
    // several workgroups per CU: no LDS-resident vector, stream of at least 512
    // entries (a batch still holds a few rows)
    while (want > 1 && cap > 512 && fixed_for(cap) > budget) cap /= 2;
    if (const char* e = std::getenv("COCOA_CHAIN_CAP"))  // A/B: a smaller stream, more LDS for the hot slice
        cap = std::max<size_t>(256, std::min<size_t>(cap, (size_t)std::atoi(e)));
    const size_t fixed = fixed_for(cap);
    size_t avail = (want > 1 ? budget : kLdsMax) - std::min(fixed, budget);
    c->vec_lds = is_sdca(c->method) && vec_bytes <= avail && want == 1;
    if (c->vec_lds) avail -= vec_bytes;
    const size_t al_bytes = align16(sizeof(double) * (size_t)std::max(c->max_nl, 1));
    c->alpha_lds = is_sdca(c->method) && al_bytes <= avail;
    if (c->vec_lds) {
        a.lds_vec = (int32_t)off;
        off += vec_bytes;
    }
    for (int b = 0; b < 2; ++b) {
        a.lds_stream_val[b] = (int32_t)off;
        off += align16(cap * 8);
        a.lds_stream_col[b] = (int32_t)off;
        off += align16(cap * 4);
        a.lds_meta[b] = (int32_t)off;
        off += align16(sizeof(BatchMeta));
    }
    a.lds_prod = (int32_t)off;  // (aliases the scratch when unused: never touched then)
    if (need_prod) off += align16(cap * 8);
    a.lds_scratch = (int32_t)off;
    off += align16(sizeof(double) * kRegChunks * 64);
    if (c->alpha_lds) {
        a.lds_alpha = (int32_t)off;
        off += al_bytes;
    }
    // fast CoCoA+ on compact slices (C4): the LDS left over holds each slice's
    // first positions -- the partition's most frequent columns -- so their
    // gathers and stores stay off HBM lines (COCOA_CHAIN_HOT=0: off, A/B)
    a.hot = 0;
    a.lds_hot = 0;
    const char* he = std::getenv("COCOA_CHAIN_HOT");
    if (!c->strict && c->dw_compact && c->method == COCOA_METHOD_COCOA_PLUS && !c->vec_lds &&
        !(he && !std::atoi(he))) {
        const size_t lim = want > 1 ? budget : kLdsMax;
        const int64_t h = off < lim ? std::min<int64_t>((int64_t)((lim - off) / sizeof(double)) & ~(int64_t)63,
                                                        vec_len)
                                    : 0;
        if (h >= 64) {
            a.hot = (int32_t)h;
            a.lds_hot = (int32_t)off;
            off += align16(sizeof(double) * (size_t)h);
        }
    }
    c->lds_bytes = off;
    a.stream_cap = (int32_t)cap;
}

// Register chunks of chain v3 (rows with z <= 64 * chunks keep their entries in
// registers).  Measured on MI355X (r01, profiles/r01/regchunks/), C5 MbCD
// (mean row 75.6): 6.73 ms per round with 4 chunks, 6.34 with 3, 6.09 with 2;
// C2 CoCoA+: 3 is neutral (+0.1% in a same-box A/B), 2 is +0.7%; C4 CoCoA+
// (mean 116): 3 is +2%.  So MbCD on short rows takes short_row_chunks (2) and
// everything else kRegChunks.
static int reg_chunks_for(int64_t nnz, int64_t rows, int method) {
    const int mode = method == COCOA_METHOD_MBCD ? MODE_MBCD : method == COCOA_METHOD_COCOA ? MODE_COCOA : MODE_PLUS;
    return (mode == MODE_MBCD && rows > 0 && nnz <= 96 * rows) ? short_row_chunks(mode, false) : kRegChunks;
}

static bool dw_double_buffer(size_t bytes, bool compact);

extern "C" int cocoa_set_solver(cocoa_ctx* ctx, int kind) {
    CAPI_BEGIN(ctx)
    require(kind == COCOA_SOLVER_AUTO || kind == COCOA_SOLVER_CHAIN || kind == COCOA_SOLVER_GRAM ||
                kind == COCOA_SOLVER_DENSE,
            COCOA_E_ARG, "cocoa_set_solver: unknown solver");
    ctx->solver_kind = kind;
    ctx->inited = false;  // takes effect at the next cocoa_init
    for (cocoa_ctx* sub : ctx->subs) sub_check(cocoa_set_solver(sub, kind), sub);
    CAPI_END(ctx)
}

// The rows as CSC in device column order for the mb-SGD pull (kernels.h
// MbsgdPull): column offsets are the frequency prefix set_train formed
// (n_hot_nnz), entries placed by a device fill (rows within a column in
// arrival order: fast mode), and tiles of <= kPullTile entries -- runs of whole
// columns, or slices of one longer column.
static void build_csc(cocoa_ctx* ctx, hipStream_t s) {
    const int64_t d = ctx->d, nnz = ctx->tr.nnz, n = ctx->tr.n;
    require((int64_t)ctx->n_hot_nnz.size() == d + 1 && ctx->n_hot_nnz[(size_t)d] == nnz, COCOA_E_STATE,
            "mb-SGD pull: column counts do not match the training set");
    ensure_cols(ctx->tr, ctx->d, s);
    upload(ctx->csc_ptr, ctx->n_hot_nnz.data(), sizeof(int64_t) * (size_t)(d + 1), s);
    DevBuf cursor;
    upload(cursor, ctx->n_hot_nnz.data(), sizeof(int64_t) * (size_t)(d + 1), s);
    ctx->csc_row.alloc(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1));
    ctx->csc_val.alloc(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1));
    launch_csc_fill(ctx->tr.row_ptr.as<int64_t>(), ctx->tr.col.as<int32_t>(), ctx->tr.val.as<double>(), n,
                    cursor.as<int64_t>(), ctx->csc_row.as<int32_t>(), ctx->csc_val.as<double>(), s);
    std::vector<int64_t> tl;
    const auto& cp = ctx->n_hot_nnz;
    int64_t j = 0;
    while (j < d) {
        const int64_t len = cp[(size_t)j + 1] - cp[(size_t)j];
        if (len > kPullTile) {  // a long column: slices
            for (int64_t e0 = cp[(size_t)j]; e0 < cp[(size_t)j + 1]; e0 += kPullTile)
                tl.insert(tl.end(), {e0, std::min<int64_t>(e0 + kPullTile, cp[(size_t)j + 1]), j, -1});
            ++j;
            continue;
        }
        int64_t j1 = j + 1;
        while (j1 < d && cp[(size_t)j1 + 1] - cp[(size_t)j] <= kPullTile) ++j1;
        tl.insert(tl.end(), {cp[(size_t)j], cp[(size_t)j1], j, j1});
        j = j1;
    }
    ctx->n_csc_tiles = (int64_t)tl.size() / 4;
    upload(ctx->csc_tiles, tl.data(), sizeof(int64_t) * std::max<size_t>(tl.size(), 4), s);
    ctx->row_cnt.alloc_zero(sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1), s);
    ctx->row_c.alloc(sizeof(double) * (size_t)std::max<int64_t>(n, 1));
    HIPCHK(hipStreamSynchronize(s));  // (cursor is freed on return)
    ctx->csc_ready = true;
}

extern "C" int cocoa_init(cocoa_ctx* ctx, const cocoa_params* params, const cocoa_debug* debug, int method,
                          const double* w_init) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        group_init(ctx, params, debug, method, w_init);
        return COCOA_OK;
    }
    require(params && method >= 0 && method <= 4, COCOA_E_ARG, "cocoa_init: bad argument");
    require(ctx->d > 0 && ctx->K_loc > 0, COCOA_E_STATE, "cocoa_init: no training data");
    require(params->local_iters >= 0 && params->n >= 1, COCOA_E_ARG, "cocoa_init: bad params");
    if (params->local_iters >= 1)
        require(ctx->min_nl >= 1, COCOA_E_ARG,
                "IllegalArgumentException: empty partition (java.util.Random.nextInt(0), CoCoA.scala:151)");
    ctx->P = *params;
    ctx->D = debug ? *debug : cocoa_debug{10, 0, 100, 0};
    ctx->method = method;
    const int64_t d = ctx->d, n = ctx->tr.n, K = ctx->K_loc;
    const int32_t H = params->local_iters;
    const double Kg = (double)ctx->K_glob;
    const double kh = (double)wrap32((int64_t)ctx->K_glob * H);  // Scala Int product
    switch (method) {
        case COCOA_METHOD_COCOA_PLUS: ctx->scaling = params->gamma; break;       // CoCoA.scala:37
        case COCOA_METHOD_COCOA: ctx->scaling = params->beta / Kg; break;        // CoCoA.scala:37
        case COCOA_METHOD_MBCD: ctx->scaling = params->beta / kh; break;         // MinibatchCD.scala:32
        case COCOA_METHOD_LOCALSGD: ctx->scaling = params->beta / Kg; break;     // SGD.scala:36
        case COCOA_METHOD_MBSGD: ctx->scaling = params->beta / kh; break;        // SGD.scala:38
    }
    hipStream_t s = ctx->stream;
    ctx->w.alloc(sizeof(double) * (size_t)d);
    ctx->xw_cached = false;
    ctx->row_xw.alloc(sizeof(double) * (size_t)std::max<int64_t>(ctx->tr.n, 1));
    std::vector<double> wdev;
    if (w_init) {
        ctx->to_device_order(w_init, wdev);
        HIPCHK(hipMemcpyAsync(ctx->w.p, wdev.data(), sizeof(double) * (size_t)d, hipMemcpyHostToDevice, s));
    } else
        HIPCHK(hipMemsetAsync(ctx->w.p, 0, sizeof(double) * (size_t)d, s));
    ctx->alpha.alloc_zero(sizeof(double) * (size_t)std::max<int64_t>(n, 1), s);
    ctx->alpha_oob = false;
    // + a sink per partition; two copies (the mirrored Gram solver's halves each keep their own)
    ctx->alpha_work.alloc(2 * sizeof(double) * (size_t)(std::max<int64_t>(n, 1) + K));
    if (ctx->zstream) HIPCHK(hipStreamSynchronize(ctx->zstream));  // no re-zeroing in flight
    ctx->gram_quiesce();                                            // no Gram prefetch in flight
    ctx->eval_quiesce();                                            // nor a pending evaluation
    ctx->zpending[0] = ctx->zpending[1] = false;
    ctx->zero_owed = -1;
    // the fast Gram solver on data with a compact layout: slices of max_u
    // entries, re-zeroed by the fold as it reads them (no second set needed)
    // CoCoA+ and MbCD (the chain or Gram solver, strict or fast) on data with a
    // compact layout: slices of max_u entries, re-zeroed by the fold as it reads
    // them (no second set).  CoCoA's task-local w copy is indexed by the global
    // column, so CoCoA keeps the dense slices.
    ctx->dw_compact = ctx->compact_ready && (method == COCOA_METHOD_COCOA_PLUS || method == COCOA_METHOD_MBCD) &&
                      params->local_iters >= 1 && !(ctx->tr_dense && dense_solver_fits(d, ctx->max_nl));
    // the loader of the SDCA solvers (and of local SGD on the Gram solver) is
    // fed by the per-step plan; set below, once the solver is chosen
    // fast SDCA: the Gram-window solver, unless the rows are dense-long (C3:
    // 2,000 entries per row, where the chain solver streams w / deltaW from LDS)
    const double zavg = ctx->tr.n ? (double)ctx->tr.nnz / (double)ctx->tr.n : 0.0;
    ctx->use_dense = !ctx->strict && is_sdca(method) && H >= 1 && ctx->tr_dense &&
                     dense_solver_fits(d, ctx->max_nl) &&
                     (ctx->solver_kind == COCOA_SOLVER_DENSE || ctx->solver_kind == COCOA_SOLVER_AUTO);
    require(ctx->use_dense || ctx->solver_kind != COCOA_SOLVER_DENSE || ctx->strict || !is_sdca(method), COCOA_E_ARG,
            "cocoa_init: the dense solver needs dense rows (cocoa_set_train_dense) with an even d <= 4096 and "
            "partitions of at most 19,200 rows");
    // AUTO takes the Gram solver when its side work has idle CUs to run on: at
    // most one partition per CU (C2: 64 on 256 CUs).  With more partitions than
    // CUs (C4 on one GPU: 1,024) every CU already runs chains and the Gram rows
    // (measured: 46 ms per C4 round on the side stream) only compete with them.
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device);
    ctx->ncu = ncu;
    // local SGD runs on the Gram solver too (MODE_LSGD, dense slices: its
    // epilogue reads wInit by the slice's column)
    const bool gram_method = is_sdca(method) || (method == COCOA_METHOD_LOCALSGD && !ctx->dw_compact);
    ctx->use_gram = !ctx->strict && !ctx->use_dense && gram_method && H >= 1 &&
                    (ctx->solver_kind == COCOA_SOLVER_GRAM ||
                     (ctx->solver_kind == COCOA_SOLVER_AUTO && zavg <= 512.0 && K <= ncu));
    // private columns (cocoa_ctx::priv_ready): fast CoCoA+ on the chain solver
    // over compact slices, folded by column blocks (so double-buffered)
    ctx->dw_priv = ctx->dw_compact && ctx->priv_ready && !ctx->strict && method == COCOA_METHOD_COCOA_PLUS &&
                   !ctx->use_gram && !ctx->use_dense && ctx->n_fitems_h > 0;
    int64_t slice = 0;
    for (;;) {
        slice = ctx->dw_priv ? ctx->max_uh : ctx->dw_compact ? ctx->max_u : d;
        // a second deltaW set only when it fits next to everything else (with 1 GiB
        // to spare); otherwise single buffering with the zero-in-fold path.  Compact
        // slices (C4: 1,024 x 64,847 doubles, 0.53 GB a set) take the second set
        // too: the fold then only reads, and the set it folded is re-zeroed by a
        // streaming memset beside the next round's solver instead of by 62 M
        // scattered 8-byte stores.
        ctx->dw_dbuf = dw_double_buffer((size_t)(K * slice) * sizeof(double), ctx->dw_compact);
        if (ctx->dw_dbuf) {
            ctx->dw2.free();
            size_t free_b = 0, total_b = 0;
            HIPCHK(hipMemGetInfo(&free_b, &total_b));
            if (free_b < 2 * sizeof(double) * (size_t)(K * slice) + ((size_t)1 << 30)) ctx->dw_dbuf = false;
        }
        if (ctx->dw_priv && !ctx->dw_dbuf) {  // (the gather fold has no private tail)
            ctx->dw_priv = false;
            continue;
        }
        break;
    }
    ctx->dw_slice = slice;
    ctx->dw.alloc_zero(sizeof(double) * (size_t)(K * slice), s);
    if (ctx->dw_priv)
        ctx->rowcoef.alloc(sizeof(double) * (size_t)std::max<int64_t>(n, 1));
    else
        ctx->rowcoef.free();
    if (ctx->dw_dbuf) {
        ctx->dw2.alloc_zero(sizeof(double) * (size_t)(K * slice), s);
        if (!ctx->zstream) {
            HIPCHK(hipStreamCreateWithFlags(&ctx->zstream, hipStreamNonBlocking));
            for (auto& e : ctx->zdone) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&ctx->folded, hipEventDisableTiming));
        }
    } else {
        ctx->dw2.free();
    }
    const bool need_wloc = method == COCOA_METHOD_COCOA || method == COCOA_METHOD_LOCALSGD;
    ctx->method = method;
    // every SDCA round runs the step plan (use_plan below), so the chain
    // solver's loader never forms x.w itself: no product buffer
    plan_solver(ctx, slice, !is_sdca(method));
    if (need_wloc && !(method == COCOA_METHOD_COCOA && ctx->vec_lds))
        ctx->wloc.alloc(sizeof(double) * (size_t)(K * d));
    else
        ctx->wloc.free();
    ctx->samples_cap = std::max<int64_t>((int64_t)K * H, 1);
    ctx->samples.alloc(sizeof(int32_t) * (size_t)ctx->samples_cap);
    ctx->dw_sum_int.alloc(sizeof(double) * ((size_t)d + 1));  // (+1: the abort slot of a multi-rank exchange)
    ctx->abort_in_sum = false;
    // (re-allocated on every init: a pointer kept from an earlier init would dangle)
    if (!ctx->dw_sum_user) ctx->dw_sum = ctx->dw_sum_int.as<double>();
    ctx->eval_part.alloc(sizeof(double) * (size_t)std::max<int64_t>(4 * 2048, 2 * K + 8));
    ctx->eval_out.alloc(sizeof(double) * 8);
    ctx->row_scratch.alloc(sizeof(double) * (size_t)std::max<int64_t>(n + ctx->te.n, 1));

    SolverArgs& a = ctx->sa;
    a.row_ptr = ctx->tr.row_ptr.as<int64_t>();
    // compact slices: the solvers index deltaW by the entry's slice position
    // (x.w comes from the plan, which reads the global columns)
    a.col = ctx->dw_priv ? ctx->pcol_h.as<int32_t>() : ctx->dw_compact ? ctx->col_local.as<int32_t>()
                                                                        : ctx->tr.col.as<int32_t>();
    a.val = ctx->dw_priv ? ctx->pval_h.as<double>() : ctx->tr.val.as<double>();
    a.row_qp = ctx->dw_priv ? ctx->row_qp.as<double>() : nullptr;
    a.rowcoef = ctx->dw_priv ? ctx->rowcoef.as<double>() : nullptr;
    a.y = ctx->tr.y.as<double>();
    a.sqn = ctx->sqn.as<double>();
    a.rowflags = ctx->rowflags.as<uint8_t>();
    a.part_ptr = ctx->part_ptr.as<int64_t>();
    a.samples = ctx->samples.as<int32_t>();
    a.alpha = ctx->alpha.as<double>();
    a.alpha_work = ctx->alpha_work.as<double>();
    a.w = ctx->w.as<double>();
    a.dw = ctx->dw.as<double>();
    a.wloc = ctx->wloc.p ? ctx->wloc.as<double>() : nullptr;
    a.d = slice;
    a.H = H;
    a.any_dup = ctx->any_dup ? 1 : 0;
    a.raw_alpha = 0;
    a.reg_chunks = reg_chunks_for(ctx->tr.nnz, ctx->tr.n, ctx->method);
    a.prof = nullptr;
    a.lam_n = params->lambda * (double)params->n;
    a.sigma = Kg * params->gamma;                                            // CoCoA.scala:45
    a.scaling = ctx->scaling;

    // every local solver but the dense one reads the column array (and the
    // dense rows of cocoa_set_train_dense have none yet)
    if (ctx->strict || !ctx->use_dense) {
        ensure_cols(ctx->tr, ctx->d, s);
        a.col = ctx->dw_priv ? ctx->pcol_h.as<int32_t>() : ctx->dw_compact ? ctx->col_local.as<int32_t>()
                                                                            : ctx->tr.col.as<int32_t>();
    }
    ctx->use_plan = is_sdca(method) || ctx->use_gram;
    ctx->gram_mirror = false;
    if (ctx->use_gram) {
        ctx->status.alloc_zero(sizeof(int) * 4, s);
        ctx->nbatch = (H + 15) / 16;  // kGB = 16 steps per batch (solver_gram.h)
        {
            // the mirrored solver (COCOA_GRAM_MIRROR=0 turns it off): two workgroups per
            // partition, each the whole chain and the deltaW columns of one parity, on
            // 2 K CUs -- 4 K <= CUs when the next round's Gram rows run beside it
            // (every method but MbCD), 2 K <= CUs for MbCD.  C2 CoCoA+ (r06l, one
            // box): solver 2.62 -> 2.39 ms; with the plan's look-back (round 6) 2.46
            // -> 1.79 ms against the one-workgroup solver.  Only past the window's
            // batches: the halves first trade bases at batch kGNB, and a half
            // finishing before the other starts would overwrite the alphaOld that
            // half still copies in (found as an intermittent wrong w at H = 10 with
            // four members sharing one GPU); MbCD, with no bases to trade, ties them
            // with a flag (solver_gram.h).
            const int kk = (int)std::max<int64_t>(K, 1);
            const char* me = std::getenv("COCOA_GRAM_MIRROR");
            ctx->gram_mirror = !(me && !std::atoi(me)) && (method == COCOA_METHOD_MBCD ? 2 : 4) * kk <= ncu &&
                               !ctx->dw_compact && ctx->row_zc.p && ctx->nbatch > gram_window_batches() &&
                               ctx->nbatch < (1 << 20) - 1;  // granule tag: epoch << 20 | (batch + 1)
            if (ctx->gram_mirror) ctx->xbase.alloc_zero(sizeof(uint64_t) * (size_t)kk * kGramRuns * kXbR * 32, s);
            else ctx->xbase.free();
        }
        if (method != COCOA_METHOD_MBCD) {
            const size_t gtb = sizeof(double) * (size_t)K * (size_t)ctx->nbatch * 16 * 64;
            ctx->gt.alloc(gtb);
            // Gram rows by runs of batches (gram_seq_kernel; COCOA_GRAM_SEQ=0: one
            // workgroup per window, gram_kernel): its pool records hold the column
            // in 27 bits and its links the batch in 18
            {
                const char* se = std::getenv("COCOA_GRAM_SEQ");
                const bool seq = !(se && !std::atoi(se)) && gram_seq_supported() && ctx->d < ((int64_t)1 << 27) &&
                                 ctx->nbatch < (1 << 18);
                const char* ce = std::getenv("COCOA_GRAM_CHUNKS");
                // runs per partition: one workgroup per CU on the CUs the solver's K
                // workgroups leave (C2: 3; r06h A/B beside the solver: 1 run 5.1 ms,
                // 2 runs 2.75, 3 runs 1.81, 4 runs 2.72 -- K * 4 = 256 workgroups
                // need a second pass for the 64 that find no free CU)
                const int kk = (int)std::max<int64_t>(K, 1);
                const int used = (ctx->gram_mirror ? 2 : 1) * kk;
                const int autoc = std::max(1, std::min(8, (ncu - used) / kk));
                ctx->gram_chunks = !seq ? 0 : ce ? std::max(1, std::atoi(ce)) : autoc;
                for (auto& fb : ctx->gram_fb) {
                    if (seq) fb.alloc(sizeof(int32_t) * (1 + 2 * (size_t)K * (size_t)ctx->nbatch));
                    else fb.free();
                }
            }
            // the next round's (samples, Gram rows) beside this round's, when they fit
            size_t free_b = 0, total_b = 0;
            HIPCHK(hipMemGetInfo(&free_b, &total_b));
            if (free_b > gtb + sizeof(int32_t) * (size_t)ctx->samples_cap + ((size_t)1 << 30)) {
                ctx->gt2.alloc(gtb);
                ctx->samples2.alloc(sizeof(int32_t) * (size_t)ctx->samples_cap);
                const int res = side_reserve(ctx, ncu);
                if (ctx->gstream && res != ctx->side_res) {  // another CU reservation: new side streams
                    HIPCHK(hipStreamSynchronize(ctx->gstream));
                    HIPCHK(hipStreamDestroy(ctx->gstream));
                    ctx->gstream = nullptr;
                    if (ctx->estream) {  // (re-made with the new mask by the next cocoa_eval_async)
                        HIPCHK(hipStreamSynchronize(ctx->estream));
                        HIPCHK(hipStreamDestroy(ctx->estream));
                        ctx->estream = nullptr;
                    }
                }
                ctx->side_res = res;
                if (!ctx->gstream) {
                    int lo = 0, hi = 0;  // lowest priority: fills the CUs the solver leaves idle
                    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
                    make_side_stream(&ctx->gstream, res, ncu, lo);
                    if (!ctx->g_ready) {
                        HIPCHK(hipEventCreateWithFlags(&ctx->g_ready, hipEventDisableTiming));
                        for (auto& e : ctx->s_done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                    }
                }
            } else {
                ctx->gt2.free();
                ctx->samples2.free();
            }
        } else {
            ctx->gt.free();
            ctx->gt2.free();
            ctx->samples2.free();
        }
    } else {
        ctx->gt.free();
        ctx->gt2.free();
        ctx->samples2.free();
    }
    a.plan_beg = nullptr;
    a.plan_z = nullptr;
    a.plan_y = a.plan_q = a.plan_xw = nullptr;
    if (ctx->use_plan) {
        const size_t steps = (size_t)std::max<int64_t>((int64_t)K * H, 1);
        ctx->plan_beg.alloc(steps * sizeof(int64_t));
        ctx->plan_z.alloc(steps * sizeof(int32_t));
        if (ctx->row_zc.p || ctx->use_gram)  // (the Gram solver's loader reads the step's look-back there)
            ctx->plan_zc.alloc(steps * kGramRuns * sizeof(int32_t));
        else
            ctx->plan_zc.free();
        ctx->plan_y.alloc(steps * sizeof(double));
        ctx->plan_q.alloc(steps * sizeof(double));
        // (a batch's 16 x.w on one 128-byte line for xw_produce_kernel's hand-off)
        ctx->xw_stride = ((int64_t)H + 15) & ~(int64_t)15;
        ctx->plan_xw.alloc(std::max(steps, (size_t)K * (size_t)ctx->xw_stride) * sizeof(double));
        if (ctx->use_gram && ctx->gt2.p) {  // (the Gram rows' prefetch runs the next plan too)
            ctx->plan_beg2.alloc(steps * sizeof(int64_t));
            ctx->plan_z2.alloc(steps * sizeof(int32_t));
            if (ctx->row_zc.p || ctx->use_gram)
                ctx->plan_zc2.alloc(steps * kGramRuns * sizeof(int32_t));
            else
                ctx->plan_zc2.free();
            ctx->plan_y2.alloc(steps * sizeof(double));
            ctx->plan_q2.alloc(steps * sizeof(double));
        } else {
            ctx->plan_beg2.free();
            ctx->plan_z2.free();
            ctx->plan_zc2.free();
            ctx->plan_y2.free();
            ctx->plan_q2.free();
        }
        ctx->pre_plan = false;
        // COCOA_XW_PRODUCER=0: the plan forms x.w in line instead (A/B, tests)
        const bool xw_env_off = std::getenv("COCOA_XW_PRODUCER") && !std::atoi(std::getenv("COCOA_XW_PRODUCER"));
        ctx->xw_prod = ctx->use_gram && ctx->gstream && ctx->gt2.p && !xw_env_off;
        ctx->eval_on_g = ctx->xw_prod && std::getenv("COCOA_EVAL_ON_GSTREAM") && std::atoi(std::getenv("COCOA_EVAL_ON_GSTREAM"));
        if (ctx->xw_prod) {
            ctx->xw_flag.alloc_zero(sizeof(int32_t) * (size_t)K * (size_t)ctx->nbatch, s);
            ctx->xw_epoch = 0;
            if (!ctx->e_w) HIPCHK(hipEventCreateWithFlags(&ctx->e_w, hipEventDisableTiming));
            if (!ctx->e_xw) HIPCHK(hipEventCreateWithFlags(&ctx->e_xw, hipEventDisableTiming));
        } else {
            ctx->xw_flag.free();
        }
        a.plan_beg = ctx->plan_beg.as<int64_t>();
        a.plan_z = ctx->plan_z.as<int32_t>();
        a.plan_y = ctx->plan_y.as<double>();
        a.plan_q = ctx->plan_q.as<double>();
        a.plan_xw = ctx->plan_xw.as<double>();
    } else {
        ctx->plan_beg.free();
        ctx->plan_z.free();
        ctx->plan_zc.free();
        ctx->plan_y.free();
        ctx->plan_q.free();
        ctx->plan_xw.free();
        ctx->xw_prod = false;
        ctx->xw_flag.free();
    }
    // fast mb-SGD on CSR rows with dense slices: the pull form (COCOA_MBSGD_PULL=0:
    // the atomic scatter kernel)
    {
        const char* pe = std::getenv("COCOA_MBSGD_PULL");
        ctx->mbsgd_pull = method == COCOA_METHOD_MBSGD && !ctx->strict && !ctx->tr_dense && !ctx->dw_compact &&
                          !(pe && !std::atoi(pe)) && ctx->tr.nnz < ((int64_t)1 << 40);
        if (ctx->mbsgd_pull && !ctx->csc_ready) build_csc(ctx, s);
    }
    HIPCHK(hipStreamSynchronize(s));
    ctx->inited = true;
    CAPI_END(ctx)
}

// Double-buffer the deltaW slices when a dense fold's zeroing pass is large:
// K_loc * d * 8 >= 1 GiB (C4: 1,024 x 3.23 M doubles = 26.5 GB per set).
// COCOA_DW_DBUF=0 / 1 forces it off / on (tests); cocoa_init still falls back
// to one set when the second does not fit in device memory.
static bool dw_double_buffer(size_t bytes, bool compact) {
    const char* e = std::getenv("COCOA_DW_DBUF");
    if (e) return std::atoi(e) != 0;
    return compact || bytes >= ((size_t)1 << 30);
}

// The step plan of the round whose samples are `samples` into plan set `set`
// (0: plan_*, 1: plan_*2); need_xw / xw_cache / xw as the caller sets them.
static PlanArgs plan_args(cocoa_ctx* c, const int32_t* samples, int set) {
    PlanArgs pa{};
    pa.part_ptr = c->part_ptr.as<int64_t>();
    pa.samples = samples;
    pa.row_ptr = c->tr.row_ptr.as<int64_t>();
    pa.col = c->tr.col.as<int32_t>();
    pa.val = c->tr.val.as<double>();
    pa.y = c->tr.y.as<double>();
    pa.sqn = c->sqn.as<double>();
    pa.w = c->w.as<double>();
    pa.steps = (int64_t)c->K_loc * c->P.local_iters;
    pa.H = c->P.local_iters;
    pa.row_zc = c->plan_zc.p && c->row_zc.p ? c->row_zc.as<int32_t>() : nullptr;
    pa.win = c->use_gram && c->plan_zc.p ? 16 * gram_window_batches() : 0;
    pa.row_zs = c->dw_priv ? c->row_zs.as<int32_t>() : nullptr;  // (the chain's rows: shared entries only)
    pa.zc = !c->plan_zc.p ? nullptr : set ? c->plan_zc2.as<int32_t>() : c->plan_zc.as<int32_t>();
    pa.beg = set ? c->plan_beg2.as<int64_t>() : c->plan_beg.as<int64_t>();
    pa.z = set ? c->plan_z2.as<int32_t>() : c->plan_z.as<int32_t>();
    pa.py = set ? c->plan_y2.as<double>() : c->plan_y.as<double>();
    pa.pq = set ? c->plan_q2.as<double>() : c->plan_q.as<double>();
    pa.xw = c->plan_xw.as<double>();
    return pa;
}

static GramArgs gram_args(cocoa_ctx* c, const int32_t* samples, double* gt) {
    GramArgs ga{};
    ga.part_ptr = c->part_ptr.as<int64_t>();
    ga.samples = samples;
    ga.row_ptr = c->tr.row_ptr.as<int64_t>();
    ga.col = c->tr.col.as<int32_t>();
    ga.val = c->tr.val.as<double>();
    ga.K = c->K_loc;
    ga.H = c->P.local_iters;
    ga.nbatch = c->nbatch;
    ga.gt = gt;
    ga.prof = c->sa.prof ? c->sa.prof + (size_t)c->K_loc * kProfStride : nullptr;  // phase sums of this launch
    ga.chunks = c->gram_chunks;
    ga.fb_cap = (int32_t)((size_t)c->K_loc * (size_t)c->nbatch);
    ga.nnz = c->tr.nnz;
    ga.gt_len = (int64_t)c->K_loc * c->nbatch * 16 * 64;
    ga.n_rows = c->tr.n;
    DevBuf& fb = c->gram_fb[gt == c->gt2.as<double>() ? 1 : 0];
    ga.fb_n = c->gram_chunks ? fb.as<int32_t>() : nullptr;
    ga.fb = c->gram_chunks ? fb.as<int32_t>() + 1 : nullptr;
    return ga;
}

// fuse_apply: w += sum * mult inside the fold (one rank, no exchange).
// chain_init: strict multi-rank fold, continuing the previous ranks' fold,
// which recv_init (a multi-device context's peer copy) or the communicator's
// chain_recv puts into dw_sum first.
typedef void (*recv_fn)(cocoa_ctx* c, void* user);
static void eval_fire(cocoa_ctx* ctx);
static void run_local(cocoa_ctx* c, int32_t t, bool fuse_apply, const double* chain_init = nullptr,
                      recv_fn recv_init = nullptr, void* recv_user = nullptr) {
    require(c->inited, COCOA_E_STATE, "cocoa_round: call cocoa_init first");
    const int32_t H = c->P.local_iters;
    const int32_t seed = wrap32((int64_t)c->D.seed + t);                    // debug.seed + t
    hipStream_t s = c->stream;
    const int64_t d = c->d;
    const int K = c->K_loc;
    c->mult = c->scaling;
    const int set = c->dw_dbuf ? (t & 1) : 0;
    double* dws = set ? c->dw2.as<double>() : c->dw.as<double>();
    if (c->zpending[set]) {  // this set's re-zeroing (two rounds ago) must land first
        HIPCHK(hipStreamWaitEvent(s, c->zdone[set], 0));
        c->zpending[set] = false;
    }
    c->sa.dw = dws;
    if (c->zero_owed >= 0) {
        double* zs = c->zero_owed ? c->dw2.as<double>() : c->dw.as<double>();
        HIPCHK(hipEventRecord(c->folded, s));
        HIPCHK(hipStreamWaitEvent(c->zstream, c->folded, 0));
        // hipMemsetAsync: C4 22.8-23.3 ms/round; a narrow zero_kernel grid (64-128
        // workgroups) measured 23.0 (r01), so the plain memset stays
        HIPCHK(hipMemsetAsync(zs, 0, sizeof(double) * (size_t)K * (size_t)c->dw_slice, c->zstream));
        HIPCHK(hipEventRecord(c->zdone[c->zero_owed], c->zstream));
        c->zpending[c->zero_owed] = true;
        c->zero_owed = -1;
    }
    bool produce = false;  // x.w by xw_produce_kernel beside the solver (fold waits on e_xw)
    if (H >= 1) {
        // (samples, Gram rows) of this round: prefetched during the last round's
        // solver (overlap), else computed here
        const bool gram_rows = c->use_gram && c->method != COCOA_METHOD_MBCD;
        // SGD.scala:53: t = (t-1) * localIters * parts, an Int product
        const double lsgd_t0 = (double)wrap32((int64_t)(t - 1) * H * c->K_glob);
        // COCOA_GRAM_SERIAL=1 (diagnostic A/B only): Gram rows in line, before the solver
        static const bool serial = std::getenv("COCOA_GRAM_SERIAL") && std::atoi(std::getenv("COCOA_GRAM_SERIAL"));
        const bool overlap = gram_rows && c->gstream && c->gt2.p && !serial;
        int b = 0;
        const bool plan_ready = overlap && c->pre_t == t && c->pre_plan;  // (set pre_buf)
        if (overlap && c->pre_t == t) {
            b = c->pre_buf;
            HIPCHK(hipStreamWaitEvent(s, c->g_ready, 0));
        } else {
            if (c->pre_t >= 0) HIPCHK(hipStreamWaitEvent(s, c->g_ready, 0));  // a prefetch of another round: done first
            c->timed(COCOA_K_SAMPLE, [&] {
                launch_sampler(c->part_ptr.as<int64_t>(), K, seed, H, c->samples.as<int32_t>(), c->jump.as<uint64_t>(), s);
            });
            if (gram_rows) {
                GramArgs ga = gram_args(c, c->samples.as<int32_t>(), c->gt.as<double>());
                if (ga.prof) HIPCHK(hipMemsetAsync(ga.prof, 0, 8 * sizeof(uint64_t), s));
                c->timed(COCOA_K_GRAM, [&] { launch_gram(ga, s); });
            }
        }
        c->pre_t = -1;
        c->pre_plan = false;
        int32_t* smp = b ? c->samples2.as<int32_t>() : c->samples.as<int32_t>();
        double* gtb = b ? c->gt2.as<double>() : c->gt.as<double>();
        c->sa.samples = smp;
        // the Gram solver runs this round (local SGD's wrapped-counter rounds do not)
        const bool gram_round = c->use_gram && (c->method != COCOA_METHOD_LOCALSGD || lsgd_t0 >= 0);
        bool rows = false;  // x.w gathered from the last evaluation's row cache (the rest prefetched)
        if (c->use_plan) {
            PlanArgs pa = plan_args(c, smp, b);
            // CoCoA's w moves inside the round: the chain solver forms x.w itself;
            // the Gram solver splits x.w_local = x.w + x.deltaW
            pa.need_xw = !c->use_dense && (c->method != COCOA_METHOD_COCOA || c->use_gram);
            pa.xw_cache = (c->xw_cached && !c->strict) ? c->row_xw.as<double>() : nullptr;
            rows = gram_round && overlap && pa.need_xw && pa.xw_cache;
            produce = !rows && c->xw_prod && overlap && pa.need_xw && !pa.xw_cache && gram_round;
            if (rows || produce) {  // x.w comes from elsewhere: the plan's other fields only
                pa.need_xw = 0;
                pa.xw = nullptr;
            }
            // (the prefetched plan, formed beside the last solver, is exactly that)
            if (plan_ready && rows) {
                c->timed(COCOA_K_PLAN, [&] {
                    launch_xw_gather(pa.part_ptr, smp, H, pa.steps, c->row_xw.as<double>(), c->plan_xw.as<double>(), s);
                });
            } else if (!(plan_ready && produce)) {
                if (rows) {  // one pass: the plan with x.w from the cache
                    pa.need_xw = 1;
                    pa.xw = c->plan_xw.as<double>();
                }
                c->timed(COCOA_K_PLAN, [&] {
                    if (c->strict)
                        launch_plan_strict(pa, s);
                    else
                        launch_plan_fast(pa, s);
                });
            }
        }
        // the side work of this round (x.w producer, a pipelined evaluation)
        // starts once the plan is done: begun earlier, it slowed the plan (on the
        // critical path) 0.04 -> 0.2 ms
        c->e_w_rec = false;
        // (COCOA_GATE_INL=0: the e_w record instead; 1.9632 -> 1.9584 ms per C2 step with the
        // e_inl gate, profiles/r06/ab_r10j_gate_inl.txt)
        static const bool gate_inl_env = !std::getenv("COCOA_GATE_INL") || std::atoi(std::getenv("COCOA_GATE_INL"));
        const bool gate_inl = gate_inl_env && c->inl_since_round && c->e_inl && overlap && !produce &&
                              !(c->eval_pending && !c->eval_fired);
        c->inl_since_round = false;
        if (!gate_inl && (produce || (c->eval_pending && !c->eval_fired) || overlap)) {
            if (!c->e_w) HIPCHK(hipEventCreateWithFlags(&c->e_w, hipEventDisableTiming));
            HIPCHK(hipEventRecord(c->e_w, s));
            c->e_w_rec = true;
        }
        if (produce) {
            // w and this round's samples are final in stream order here
            HIPCHK(hipStreamWaitEvent(c->gstream, c->e_w, 0));
            XwArgs xa{};
            xa.part_ptr = c->part_ptr.as<int64_t>();
            xa.samples = smp;
            xa.row_ptr = c->tr.row_ptr.as<int64_t>();
            xa.col = c->tr.col.as<int32_t>();
            xa.val = c->tr.val.as<double>();
            xa.w = c->w.as<double>();
            xa.xw = c->plan_xw.as<double>();
            xa.flag = c->xw_flag.as<int32_t>();
            xa.stride = c->xw_stride;
            xa.K = K;
            xa.H = H;
            xa.nbatch = c->nbatch;
            xa.epoch = ++c->xw_epoch;
            require(c->xw_flag.bytes >= sizeof(int32_t) * (size_t)K * (size_t)c->nbatch &&
                        c->plan_xw.bytes >= sizeof(double) * (size_t)K * (size_t)c->xw_stride,
                    COCOA_E_STATE, "x.w producer buffers");
            c->timed_on(c->gstream, COCOA_K_XW, [&] { launch_xw_produce(xa, c->gstream); });
            HIPCHK(hipEventRecord(c->e_xw, c->gstream));
            if (c->eval_on_g) eval_fire(c);  // the previous state's pipelined evaluation, next on gstream
        }
        if (c->use_dense) {
            DenseArgs g{};
            g.X = c->tr.val.as<double>();
            g.part_ptr = c->part_ptr.as<int64_t>();
            g.samples = smp;
            g.plan_y = c->plan_y.as<double>();
            g.plan_q = c->plan_q.as<double>();
            g.alpha = c->alpha.as<double>();
            g.dw = dws;
            g.w = c->w.as<double>();
            g.d = d;
            g.H = H;
            g.lam_n = c->sa.lam_n;
            g.inv_lam_n = 1.0 / c->sa.lam_n;
            g.sigma = c->method == COCOA_METHOD_COCOA_PLUS ? c->sa.sigma : 1.0;
            g.scaling = c->scaling;
            g.proj = c->proj_rule() ? 1 : 0;
            c->timed(COCOA_K_SOLVER, [&] { launch_solver_dense(solver_mode(c->method), g, K, c->max_nl, s); });
        } else if (c->use_gram && (c->method != COCOA_METHOD_LOCALSGD || lsgd_t0 >= 0)) {
            GramSolverArgs g{};
            g.part_ptr = c->part_ptr.as<int64_t>();
            g.samples = smp;
            {
                const PlanArgs ps = plan_args(c, smp, b);  // (this round's plan set)
                g.plan_beg = ps.beg;
                g.plan_z = ps.z;
                g.plan_zc = ps.zc;
                g.plan_y = ps.py;
                g.plan_q = ps.pq;
            }
            g.plan_xw = c->plan_xw.as<double>();
            g.xw_flag = produce ? c->xw_flag.as<int32_t>() : nullptr;
            g.xw_col = c->tr.col.as<int32_t>();
            g.xw_epoch = c->xw_epoch;
            g.xw_stride = produce ? c->xw_stride : H;
            g.col = c->dw_compact ? c->col_local.as<int32_t>() : c->tr.col.as<int32_t>();
            g.val = c->tr.val.as<double>();
            g.alpha = c->alpha.as<double>();
            g.alpha_work = c->alpha_work.as<double>();
            g.dw = dws;
            g.gt = gram_rows ? gtb : nullptr;
            g.status = c->status.as<int>();
            g.prof = c->sa.prof;
            g.d = c->dw_compact ? c->max_u : d;  // slice length
            g.H = H;
            g.nbatch = c->nbatch;
            g.raw_alpha = 0;
            g.lam_n = c->sa.lam_n;
            g.inv_lam_n = 1.0 / c->sa.lam_n;
            g.sigma = c->method == COCOA_METHOD_COCOA_PLUS ? c->sa.sigma : 1.0;
            g.scaling = c->scaling;
            g.proj = c->proj_rule() ? 1 : 0;
            g.w = c->w.as<double>();
            g.lambda = c->P.lambda;
            g.t0 = lsgd_t0;
            g.alpha_work_stride = c->tr.n + K;
            g.hot_split = c->hot_split;
            g.mirror = c->gram_mirror && !c->device_shared() ? 1 : 0;
            g.xbase = c->xbase.as<uint64_t>();
            if (g.mirror) c->xtag_epoch = (c->xtag_epoch % 4095) + 1;  // 1..4095 (12 tag bits, never 0)
            g.xtag_epoch = c->xtag_epoch;
            const int mode = c->method == COCOA_METHOD_LOCALSGD ? MODE_LSGD : solver_mode(c->method);
            c->timed(COCOA_K_SOLVER, [&] { launch_solver_gram(mode, g, K, s); });
            // fault injection for the abort-reporting tests: COCOA_INJECT_ABORT=t
            // marks round t's launch as aborted (the status word a timed-out
            // hand-off sets), on the stream behind it
            static const int inject_t = std::getenv("COCOA_INJECT_ABORT") ? std::atoi(std::getenv("COCOA_INJECT_ABORT")) : 0;
            if (inject_t > 0 && t == inject_t) {
                static const int one = 1;
                HIPCHK(hipMemcpyAsync(c->status.p, &one, sizeof(int), hipMemcpyHostToDevice, s));
            }
            if (overlap) {
                // round t+1's samples and Gram rows on gstream, beside this solver (its
                // buffer's last reader, round t-1's solver, is done first)
                HIPCHK(hipEventRecord(c->s_done[b], s));
                const int nb = 1 - b;
                if (t < c->P.num_rounds) {
                    HIPCHK(hipStreamWaitEvent(c->gstream, c->s_done[nb], 0));
                    // and not before this round's plan is done: with the evaluation
                    // read back after the next round is enqueued (cocoa_eval_begin /
                    // _end), the Gram rows would otherwise start during that
                    // evaluation and hold CUs the next solver's workgroups need whole
                    if (c->e_w_rec) HIPCHK(hipStreamWaitEvent(c->gstream, c->e_w, 0));
                    if (gate_inl) HIPCHK(hipStreamWaitEvent(c->gstream, c->e_inl, 0));  // (the last evaluation: done)
                    int32_t* nsmp = nb ? c->samples2.as<int32_t>() : c->samples.as<int32_t>();
                    double* ngt = nb ? c->gt2.as<double>() : c->gt.as<double>();
                    const int32_t nseed = wrap32((int64_t)c->D.seed + t + 1);
                    c->timed_on(c->gstream, COCOA_K_SAMPLE, [&] {
                        launch_sampler(c->part_ptr.as<int64_t>(), K, nseed, H, nsmp, c->jump.as<uint64_t>(), c->gstream);
                    });
                    if (c->plan_beg2.p) {  // round t+1's plan but x.w, into the other plan set
                        PlanArgs pn = plan_args(c, nsmp, nb);
                        pn.need_xw = 0;
                        pn.xw = nullptr;
                        c->timed_on(c->gstream, COCOA_K_PLAN, [&] { launch_plan_fast(pn, c->gstream); });
                        c->pre_plan = true;
                    }
                    GramArgs ga = gram_args(c, nsmp, ngt);
                    ga.prof = nullptr;
                    c->timed_on(c->gstream, COCOA_K_GRAM, [&] { launch_gram(ga, c->gstream); });
                    HIPCHK(hipEventRecord(c->g_ready, c->gstream));
                    c->pre_t = t + 1;
                    c->pre_buf = nb;
                }
            }
        } else if (is_sdca(c->method)) {
            c->timed(COCOA_K_SOLVER, [&] {
                if (c->strict)
                    launch_solver_strict(solver_mode(c->method), c->vec_lds, c->alpha_lds, c->sa, K, c->lds_bytes, s);
                else
                    launch_solver_fast(solver_mode(c->method), c->vec_lds, c->alpha_lds, c->sa, K, c->lds_bytes, s);
            });
        } else {
            const double step = 1 / (c->P.lambda * (double)t);                 // SGD.scala:44
            const bool local = c->method == COCOA_METHOD_LOCALSGD;
            if (!local) {
                const double scale = 1.0 - (step * c->P.lambda);             // SGD.scala:48-49
                c->timed(COCOA_K_APPLY, [&] { launch_scale(c->w.as<double>(), d, scale, s); });
                c->mult = step * c->scaling;                                 // SGD.scala:58
            }
            // (local SGD lands here on the strict path, or in the fast path for a
            // round whose Int step counter wrapped negative: its shrink sequence can
            // pass through 0 or blow up, which the Gram solver's scalar s does not model)
            const double t0 = lsgd_t0;
            c->timed(COCOA_K_SOLVER, [&] {
                if (c->strict) {
                    launch_sgd(local, c->sa, c->P.lambda, t0, K, s);
                } else if (!local && c->mbsgd_pull) {
                    // the round's deltaW as X^T c into slice 0 (device order), folded
                    // below as one slice
                    MbsgdPull p{c->csc_ptr.as<int64_t>(), c->csc_row.as<int32_t>(), c->csc_val.as<double>(),
                                c->csc_tiles.as<int64_t>(), c->n_csc_tiles, c->row_cnt.as<int32_t>(),
                                c->row_c.as<double>()};
                    launch_mbsgd_pull(c->sa, p, K, c->tr.n, c->xw_cached ? c->row_xw.as<double>() : nullptr,
                                      1.0 - (step * c->P.lambda), dws, s);
                } else {
                    launch_sgd_fast(local, c->sa, c->P.lambda, t0, K, s);
                }
            });
        }
    } else if (c->method == COCOA_METHOD_MBSGD) {
        const double step = 1 / (c->P.lambda * (double)t);
        c->timed(COCOA_K_APPLY, [&] { launch_scale(c->w.as<double>(), d, 1.0 - (step * c->P.lambda), s); });
        c->mult = step * c->scaling;
    }
    // a pipelined evaluation of the previous state (cocoa_eval_async) goes out
    // now, behind this round's solver launch
    eval_fire(c);
    if (chain_init) {  // the fold of ranks < rank (rank > 0)
        if (recv_init)
            recv_init(c, recv_user);
        else
            c->comm->chain_recv(c->dw_sum, d, true, s);
    }
    if (produce) HIPCHK(hipStreamWaitEvent(s, c->e_xw, 0));  // its reads of w are done
    c->timed(COCOA_K_FOLD, [&] {
        if (c->dw_priv) {
            require(!chain_init, COCOA_E_STATE, "private columns need the column-block fold");
            FoldTail tl{c->tbnd.as<uint32_t>(), c->tcol16.as<uint16_t>(), c->trow.as<int32_t>(), c->tval.as<double>(),
                        c->rowcoef.as<double>()};
            launch_fold_blocks(dws, c->fcol16_h.as<uint16_t>(), c->fbnd_h.as<uint32_t>(), c->fitems_h.as<int32_t>(),
                               c->n_fitems_h, K, c->max_uh, d, c->ftmp.as<double>(), c->dw_sum, c->w.as<double>(),
                               c->mult, fuse_apply, c->d_inv.as<int32_t>(), s, &tl);
        } else if (c->dw_compact && c->n_fitems > 0 && c->dw_dbuf && !chain_init)
            launch_fold_blocks(dws, c->fcol16.as<uint16_t>(), c->fbnd.as<uint32_t>(), c->fitems.as<int32_t>(),
                               c->n_fitems, K, c->max_u, d, c->ftmp.as<double>(), c->dw_sum, c->w.as<double>(),
                               c->mult, fuse_apply, c->d_inv.as<int32_t>(), s);
        else if (c->dw_compact)
            launch_fold_compact(dws, c->fptr.as<int64_t>(), c->fpos.as<uint32_t>(), d, c->dw_sum, c->w.as<double>(),
                                c->mult, fuse_apply, c->d_inv.as<int32_t>(), !c->dw_dbuf, s, chain_init);
        else  // (the mb-SGD pull leaves the rank's sum in slice 0 alone)
            launch_fold(dws, c->mbsgd_pull && c->method == COCOA_METHOD_MBSGD && !c->strict ? 1 : K, d, c->dw_sum,
                        c->w.as<double>(), c->mult, fuse_apply, c->d_inv.as<int32_t>(), !c->dw_dbuf, s, chain_init);
    });
    if (c->dw_dbuf) c->zero_owed = set;
    c->xw_cached = false;  // w moves this round (scale / fused apply / the caller's apply)
}

extern "C" int cocoa_round_local(cocoa_ctx* ctx, int32_t t) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_round_local");
    run_local(ctx, t, false);
    CAPI_END(ctx)
}

extern "C" int cocoa_dw_sum_device_ptr(cocoa_ctx* ctx, void** out) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_dw_sum_device_ptr");
    require(out != nullptr, COCOA_E_ARG, "null out");
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    *out = (void*)ctx->dw_sum;
    CAPI_END(ctx)
}

extern "C" int cocoa_set_dw_sum_buffer(cocoa_ctx* ctx, void* device_ptr) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_set_dw_sum_buffer");
    ctx->dw_sum = device_ptr ? (double*)device_ptr : ctx->dw_sum_int.as<double>();
    ctx->dw_sum_user = device_ptr != nullptr;
    ctx->abort_in_sum = false;  // (a caller's buffer has no abort slot)
    CAPI_END(ctx)
}

extern "C" int cocoa_round_apply(cocoa_ctx* ctx) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_round_apply");
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    ctx->timed(COCOA_K_APPLY, [&] {
        launch_apply(ctx->w.as<double>(), ctx->dw_sum, ctx->d, ctx->mult, ctx->d_inv.as<int32_t>(), ctx->stream);
    });
    ctx->xw_cached = false;
    CAPI_END(ctx)
}

// One full round.  With a communicator (cocoa_comm_init) the deltaW sum is
// exchanged between ranks before w moves (CoCoA.scala:47-48):
//   fast   -- allreduce of the rank-local folds (one fixed association, the
//             same bytes on every rank);
//   strict -- the ordered chain: rank r continues the fold of ranks < r and
//             passes it on, the last rank broadcasts the total, so the sum is
//             the single-process partition-order fold bit for bit.
extern "C" int cocoa_round(cocoa_ctx* ctx, int32_t t) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        group_round(ctx, t);
    } else if (!ctx->comm) {
        run_local(ctx, t, true);
    } else {
        cocoa::Comm& cm = *ctx->comm;
        const int64_t d = ctx->d;
        // an aborted solver launch must not send its half-updated sum to the other
        // ranks: check the status word before every exchange (the HOST transport
        // synchronises here anyway; over RCCL this costs one stream sync per round)
        auto checked = [&] {
            if (ctx->use_gram && cm.world > 1) {
                HIPCHK(hipStreamSynchronize(ctx->stream));
                check_status(ctx);
            }
        };
        if (ctx->strict && cm.world > 1) {
            run_local(ctx, t, false, cm.rank > 0 ? ctx->dw_sum : nullptr);
            cm.chain_send(ctx->dw_sum, d, true, ctx->stream);
            cm.bcast_last(ctx->dw_sum, d, true, ctx->stream);
        } else if (cm.world > 1 && !ctx->dw_sum_user) {
            // no host wait: the status word rides along with the sum (slot d), so
            // every rank sees an abort on any rank at its next synchronising call
            // (check_status), before it returns any result.  Every fast rank sends
            // d + 1 values whichever solver its own shard took (a rank without the
            // Gram solver sends 0): RCCL needs the same count on every rank.
            run_local(ctx, t, false);
            if (ctx->use_gram && ctx->status.p)
                launch_status_slot(ctx->status.as<int>(), ctx->dw_sum + d, ctx->stream);
            else
                HIPCHK(hipMemsetAsync(ctx->dw_sum + d, 0, sizeof(double), ctx->stream));
            cm.allreduce(ctx->dw_sum, d + 1, true, ctx->stream);
            ctx->abort_in_sum = true;
        } else {
            run_local(ctx, t, false);
            checked();
            cm.allreduce(ctx->dw_sum, d, true, ctx->stream);
        }
        ctx->timed(COCOA_K_APPLY, [&] {
            launch_apply(ctx->w.as<double>(), ctx->dw_sum, d, ctx->mult, ctx->d_inv.as<int32_t>(), ctx->stream);
        });
        ctx->xw_cached = false;
    }
    CAPI_END(ctx)
}

// ------------------------------------------------------------ rank exchange --
extern "C" int cocoa_comm_unique_id(int transport, void* uid) {
    try {
        require(uid != nullptr, COCOA_E_ARG, "cocoa_comm_unique_id: null uid");
        cocoa::comm_unique_id(transport, uid);
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        return e.code;
    }
    return COCOA_OK;
}

extern "C" int cocoa_comm_create(int transport, int32_t rank, int32_t world, const void* uid, int device,
                                 cocoa_comm** out) {
    if (!out) return COCOA_E_ARG;
    *out = nullptr;
    try {
        cocoa_comm* c = new cocoa_comm();
        try {
            c->c = cocoa::comm_create(transport, rank, world, uid, device);
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        return e.code;
    }
    return COCOA_OK;
}

extern "C" int cocoa_comm_destroy(cocoa_comm* comm) {
    if (comm) {
        delete comm->c;
        delete comm;
    }
    return COCOA_OK;
}

extern "C" int cocoa_comm_allreduce(cocoa_comm* comm, double* buf, int64_t n) {
    try {
        require(comm && comm->c && (buf || n == 0) && n >= 0, COCOA_E_ARG, "cocoa_comm_allreduce: bad argument");
        comm->c->allreduce(buf, n, false, nullptr);
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        return e.code;
    }
    return COCOA_OK;
}

extern "C" int cocoa_comm_ordered_sum(cocoa_comm* comm, double* buf, int64_t n) {
    try {
        require(comm && comm->c && (buf || n == 0) && n >= 0, COCOA_E_ARG, "cocoa_comm_ordered_sum: bad argument");
        cocoa::Comm& cm = *comm->c;
        std::vector<double> mine(buf, buf + n);
        if (cm.rank > 0) {
            cm.chain_recv(buf, n, false, nullptr);
            for (int64_t i = 0; i < n; ++i) buf[i] = buf[i] + mine[(size_t)i];
        }
        cm.chain_send(buf, n, false, nullptr);
        cm.bcast_last(buf, n, false, nullptr);
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        return e.code;
    }
    return COCOA_OK;
}

extern "C" int cocoa_comm_init(cocoa_ctx* ctx, int transport, int32_t rank, int32_t world, const void* uid) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_comm_init");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    delete ctx->comm;
    ctx->comm = nullptr;
    ctx->comm = cocoa::comm_create(transport, rank, world, uid, ctx->device);
    ctx->n_test_glob = -1;
    CAPI_END(ctx)
}

extern "C" int cocoa_comm_info(cocoa_ctx* ctx, int32_t* transport, int32_t* rank, int32_t* world) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {  // the devices exchange in-process
        if (transport) *transport = COCOA_TRANSPORT_LOCAL;
        if (rank) *rank = 0;
        if (world) *world = (int32_t)ctx->subs.size();
        return COCOA_OK;
    }
    if (transport) *transport = ctx->comm ? ctx->comm->transport : -1;
    if (rank) *rank = ctx->comm ? ctx->comm->rank : 0;
    if (world) *world = ctx->comm ? ctx->comm->world : 1;
    CAPI_END(ctx)
}

// ------------------------------------------------------------------- eval --
static void finish(const cocoa_ctx* c, double hinge, double alpha_sum, double w2, int64_t err, int64_t n_test,
                   cocoa_eval_result* out) {
    const double lam = c->P.lambda;
    const double n = (double)c->P.n;
    const double nw = std::sqrt(w2);                                          // w.norm(2)
    const double nw2 = nw * nw;                                               // Math.pow(., 2)
    out->hinge_sum = hinge;
    out->alpha_sum = alpha_sum;
    out->w_sqnorm = w2;                                                       // raw sum of squares
    out->primal = hinge / n + (0.5 * lam * nw2);                              // OptUtils.scala:73-75
    out->dual = (-lam / 2 * nw2) + (alpha_sum / n);                           // OptUtils.scala:80-84
    out->gap = out->primal - out->dual;                                       // OptUtils.scala:89-91
    out->test_err_count = err;
    out->test_rows = n_test;
    out->test_error = n_test > 0 ? (double)err / (double)n_test : NAN;        // OptUtils.scala:95-98
}

// The evaluation pass of one (sub-)context, enqueued: the rank-local sums land
// in h_eval (pinned) once the stream reaches them.
// async (cocoa_eval_async): on estream, from the (w, alpha) snapshots, into
// eval_part2 / eval_out2 and h_eval[4..7]; no row x.w kept (the next round's
// plan forms x.w itself)
static void eval_launch(cocoa_ctx* ctx, bool async = false, bool to_host = true) {
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    require(async || !ctx->eval_pending, COCOA_E_STATE,
            "an evaluation is pending: collect it with cocoa_eval_wait first");
    // (COCOA_EVAL_ON_GSTREAM=1: the pipelined pass on gstream, behind the x.w
    // producer and ahead of the next Gram rows, instead of beside them)
    const bool on_g = async && ctx->eval_on_g && ctx->gstream;
    hipStream_t st = on_g ? ctx->gstream : async ? ctx->estream : ctx->stream;
    const bool dense_eval = !ctx->strict && ctx->tr_dense && (!ctx->has_test || ctx->te_dense || ctx->te.n == 0) &&
                            dense_eval_fits(ctx->d);
    if (!dense_eval) {  // the CSR passes read the column arrays (on the context's stream)
        ensure_cols(ctx->tr, ctx->d, ctx->stream);
        if (ctx->has_test) ensure_cols(ctx->te, ctx->d, ctx->stream);
    }
    if (async) HIPCHK(hipStreamWaitEvent(st, ctx->e_round, 0));  // the snapshots are taken
    if (async && ctx->e_w_rec) HIPCHK(hipStreamWaitEvent(st, ctx->e_w, 0));  // behind this round's plan
    bool host_done = false;  // the sums already stored to h_eval by the pass
    // the Gram solver's status word rides behind the pass (cocoa_eval_end /
    // cocoa_eval_wait raise on an aborted launch without a stream sync)
    const bool gram_status = !ctx->strict && ctx->use_gram && ctx->status.p && (!async || ctx->status_snap.p);
    EvalArgs e{};
    e.row_ptr = ctx->tr.row_ptr.as<int64_t>();
    e.col = ctx->tr.col.as<int32_t>();
    e.val = ctx->tr.val.as<double>();
    e.y = ctx->tr.y.as<double>();
    e.alpha = async ? ctx->alpha_snap.as<double>() : ctx->alpha.as<double>();
    e.n = ctx->tr.n;
    e.t_row_ptr = ctx->has_test ? ctx->te.row_ptr.as<int64_t>() : nullptr;
    e.t_col = ctx->has_test ? ctx->te.col.as<int32_t>() : nullptr;
    e.col16 = ctx->tr.col16.p ? ctx->tr.col16.as<uint16_t>() : nullptr;
    e.t_col16 = ctx->has_test && ctx->te.col16.p ? ctx->te.col16.as<uint16_t>() : nullptr;
    e.t_val = ctx->has_test ? ctx->te.val.as<double>() : nullptr;
    e.t_y = ctx->has_test ? ctx->te.y.as<double>() : nullptr;
    e.n_test = ctx->has_test ? ctx->te.n : 0;
    e.w = async ? ctx->w_snap.as<double>() : ctx->w.as<double>();
    e.d = ctx->d;
    e.part_ptr = ctx->part_ptr.as<int64_t>();
    e.perm = ctx->d_perm.as<int32_t>();
    e.K = ctx->K_loc;
    e.partials = async ? ctx->eval_part2.as<double>() : ctx->eval_part.as<double>();
    e.out = async ? ctx->eval_out2.as<double>() : ctx->eval_out.as<double>();
    e.row_scratch = ctx->row_scratch.as<double>();
    e.tiles = ctx->tiles.as<int64_t>();
    e.n_tiles = ctx->n_tiles;
    e.t_tiles = ctx->has_test ? ctx->t_tiles.as<int64_t>() : nullptr;
    e.n_t_tiles = ctx->has_test ? ctx->n_t_tiles : 0;
    if (!ctx->strict && !dense_eval && ctx->split_ready) {
        // the split evaluation: hot pass, then the cold entries in place of the rows
        e.h_row_ptr = ctx->hot_tr.row_ptr.as<int64_t>();
        e.h_col16 = ctx->hot_tr.col16.as<uint16_t>();
        e.h_val = ctx->hot_tr.val.as<double>();
        e.h_tiles = ctx->hot_tiles.as<int64_t>();
        e.n_h_tiles = ctx->n_hot_tiles;
        e.row_base = ctx->row_base.as<double>();
        e.row_ptr = ctx->cold_tr.row_ptr.as<int64_t>();
        e.col = ctx->cold_tr.col.as<int32_t>();
        e.col16 = ctx->cold_tr.col16.p ? ctx->cold_tr.col16.as<uint16_t>() : nullptr;
        e.val = ctx->cold_tr.val.as<double>();
        e.tiles = ctx->cold_tiles.as<int64_t>();
        e.n_tiles = ctx->n_cold_tiles;
        if (ctx->has_test && ctx->te_split) {  // the test rows' cold entries here, hot ones in the hot pass
            e.t_row_ptr = ctx->cold_te.row_ptr.as<int64_t>();
            e.t_col = ctx->cold_te.col.as<int32_t>();
            e.t_col16 = ctx->cold_te.col16.p ? ctx->cold_te.col16.as<uint16_t>() : nullptr;
            e.t_val = ctx->cold_te.val.as<double>();
            e.t_tiles = ctx->cold_t_tiles.as<int64_t>();
            e.n_t_tiles = ctx->n_cold_t_tiles;
            e.th_row_ptr = ctx->hot_te.row_ptr.as<int64_t>();
            e.th_col16 = ctx->hot_te.col16.as<uint16_t>();
            e.th_val = ctx->hot_te.val.as<double>();
            e.th_tiles = ctx->hot_t_tiles.as<int64_t>();
            e.n_th_tiles = ctx->n_hot_t_tiles;
        }
        if (ctx->n_warm_tiles > 0) {
            e.m_row_ptr = ctx->warm_tr.row_ptr.as<int64_t>();
            e.m_col16 = ctx->warm_tr.col16.as<uint16_t>();
            e.m_val = ctx->warm_tr.val.as<double>();
            e.m_tiles = ctx->warm_tiles.as<int64_t>();
            e.n_m_tiles = ctx->n_warm_tiles;
        }
    }
    ctx->timed_on(st, COCOA_K_EVAL, [&] {
        if (ctx->strict)
            launch_eval_strict(e, st);
        else {
            e.row_xw = async ? nullptr : ctx->row_xw.as<double>();
            if (dense_eval) {
                launch_eval_dense(e, st);  // rows read as X[n][d]: 8 B per entry
            } else {
                // the last block sums the partials and stores them to the pinned
                // result (no final-sum launch, no copy behind it)
                DevBuf& cnt = async ? ctx->eval_cnt2 : ctx->eval_cnt;
                if (!cnt.p) cnt.alloc_zero(sizeof(unsigned), st);
                e.counter = cnt.as<unsigned>();
                e.out_host = to_host ? ctx->h_eval + (async ? 4 : 0) : nullptr;
                if (to_host && gram_status) {
                    e.status = async ? ctx->status_snap.as<int>() : ctx->status.as<int>();
                    e.status_host = (int*)(ctx->h_eval + (async ? 10 : 9));
                }
                host_done = launch_eval_fast(e, eval_fast_blocks(e.n_tiles, e.n_t_tiles), st);
            }
            ctx->xw_cached = !async;  // the next round's plan reuses these x.w (stream order)
        }
    });
    if (to_host && gram_status && !host_done)
        HIPCHK(hipMemcpyAsync(ctx->h_eval + (async ? 10 : 9), async ? ctx->status_snap.p : ctx->status.p, sizeof(int),
                              hipMemcpyDeviceToHost, st));
    ctx->status_slot[async ? 1 : 0] = to_host && gram_status;
    if (async) {
        if (!host_done)
            HIPCHK(hipMemcpyAsync(ctx->h_eval + 4, ctx->eval_out2.p, 4 * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(ctx->e_done, st));
    } else if (!host_done && to_host) {
        HIPCHK(hipMemcpyAsync(ctx->h_eval, ctx->eval_out.p, 4 * sizeof(double), hipMemcpyDeviceToHost, st));
    }
}

// the status word an evaluation carried back (eval_launch): raise on an aborted
// solver launch among the rounds it evaluated
static void check_status_slot(cocoa_ctx* ctx, int which) {
    if (!ctx->status_slot[which]) return;
    ctx->status_slot[which] = false;
    if (*(volatile int*)(ctx->h_eval + 9 + which) != 0)
        throw Error(COCOA_E_HIP, "local solver: a hand-off between the solver's waves timed out (launch aborted)");
}

struct EvalLocal {
    double hinge, alpha_sum, w2, err, n_test;
};

// wait for eval_launch's sums
static EvalLocal eval_collect(cocoa_ctx* ctx) {
    HIPCHK(hipStreamSynchronize(ctx->stream));
    check_status(ctx);
    // w is replicated: w2 is the same on every rank
    return EvalLocal{ctx->h_eval[0], ctx->h_eval[1], ctx->h_eval[2], ctx->h_eval[3],
                     (double)(ctx->has_test ? ctx->te.n : 0)};
}

// Strict multi-rank evaluation: continue the partition-order merge of the
// previous ranks (OptUtils.scala:65-84 as Spark merges partitions, in index
// order) with this rank's per-partition partials.  carry = {hinge,
// hinge-seen flag, alpha}; first: this is the first rank.
static void strict_eval_carry(cocoa_ctx* ctx, bool first, double carry[3]) {
    std::vector<double> part((size_t)2 * ctx->K_loc);
    HIPCHK(hipMemcpyAsync(part.data(), ctx->eval_part.p, sizeof(double) * part.size(), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    bool have = carry[1] != 0.0;
    double h = carry[0], al = carry[2];
    for (int32_t k = 0; k < ctx->K_loc; ++k) {
        al = (first && k == 0) ? part[2 * (size_t)k + 1] : al + part[2 * (size_t)k + 1];
        if (ctx->h_part_ptr[(size_t)k + 1] > ctx->h_part_ptr[(size_t)k]) {
            h = have ? h + part[2 * (size_t)k] : part[2 * (size_t)k];
            have = true;
        }
    }
    carry[0] = h;
    carry[1] = have ? 1.0 : 0.0;
    carry[2] = al;
}

static void group_eval(cocoa_ctx* g, cocoa_eval_result* out);

extern "C" int cocoa_eval(cocoa_ctx* ctx, cocoa_eval_result* out) {
    CAPI_BEGIN(ctx)
    require(out != nullptr, COCOA_E_ARG, "null out");
    require(!ctx->inl_pending, COCOA_E_STATE, "an evaluation is pending: collect it with cocoa_eval_end first");
    if (ctx->is_group()) {
        group_eval(ctx, out);
        return COCOA_OK;
    }
    eval_launch(ctx);
    const EvalLocal ev = eval_collect(ctx);
    double hinge = ev.hinge, alpha_sum = ev.alpha_sum;
    double w2 = ev.w2;
    double counts[2] = {ev.err, ev.n_test};
    if (ctx->comm && ctx->comm->world > 1) {
        cocoa::Comm& cm = *ctx->comm;
        if (ctx->strict) {
            double carry[3] = {0.0, 0.0, 0.0};
            cm.chain_recv(carry, 3, false, ctx->stream);
            strict_eval_carry(ctx, cm.rank == 0, carry);
            cm.chain_send(carry, 3, false, ctx->stream);
            cm.bcast_last(carry, 3, false, ctx->stream);
            hinge = carry[0];
            alpha_sum = carry[2];
        } else {
            // ||w||^2: rank 0's on every rank (each rank's pass sums the replicated w
            // over its own grid, so the last bit may differ between ranks)
            double sums[3] = {hinge, alpha_sum, cm.rank == 0 ? w2 : 0.0};
            cm.allreduce(sums, 3, false, ctx->stream);
            hinge = sums[0];
            alpha_sum = sums[1];
            w2 = sums[2];
        }
        cm.allreduce(counts, 2, false, ctx->stream);  // integers: exact in any order
    }
    finish(ctx, hinge, alpha_sum, w2, (int64_t)counts[0], (int64_t)counts[1], out);
    CAPI_END(ctx)
}

// Pipelined evaluation: one device, one rank, fast mode (the strict and
// multi-rank merges need the exchange in order; those contexts use cocoa_eval).
extern "C" int cocoa_eval_async(cocoa_ctx* ctx) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_eval_async");
    require(!ctx->strict && !(ctx->comm && ctx->comm->world > 1), COCOA_E_STATE,
            "cocoa_eval_async: fast mode on a single rank only (use cocoa_eval)");
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    require(!ctx->eval_pending, COCOA_E_STATE, "an evaluation is pending: collect it with cocoa_eval_wait first");
    require(!ctx->inl_pending, COCOA_E_STATE, "an evaluation is pending: collect it with cocoa_eval_end first");
    if (!ctx->estream) {
        make_side_stream(&ctx->estream, ctx->side_res, ctx->ncu, 0);
        if (!ctx->e_round) HIPCHK(hipEventCreateWithFlags(&ctx->e_round, hipEventDisableTiming));
        if (!ctx->e_done) HIPCHK(hipEventCreateWithFlags(&ctx->e_done, hipEventDisableTiming));
    }
    const size_t nw = sizeof(double) * (size_t)ctx->d, na = sizeof(double) * (size_t)std::max<int64_t>(ctx->tr.n, 1);
    if (ctx->w_snap.bytes < nw) ctx->w_snap.alloc(nw);
    if (ctx->alpha_snap.bytes < na) ctx->alpha_snap.alloc(na);
    const size_t np = sizeof(double) * (size_t)std::max<int64_t>(4 * 2048, 2 * ctx->K_loc + 8);
    if (ctx->eval_part2.bytes < np) ctx->eval_part2.alloc(np);
    if (ctx->eval_out2.bytes < 8 * sizeof(double)) ctx->eval_out2.alloc(8 * sizeof(double));
    // snapshots on the context's stream (the next round moves w and alpha); the
    // evaluation itself is enqueued by the next round right after its solver
    // launch (eval_fire), so the solver's workgroups hold their CUs first and the
    // evaluation fills the idle ones beside the Gram rows.  (Enqueued at once, it
    // raced the next round's plan and solver for CUs: 3.30 -> 3.74 ms per C2 step.)
    HIPCHK(hipMemcpyAsync(ctx->w_snap.p, ctx->w.p, nw, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->alpha_snap.p, ctx->alpha.p, na, hipMemcpyDeviceToDevice, ctx->stream));
    if (ctx->use_gram && ctx->status.p) {  // the status word as of the evaluated rounds (the next round may set it)
        if (!ctx->status_snap.p) ctx->status_snap.alloc(sizeof(int) * 4);
        HIPCHK(hipMemcpyAsync(ctx->status_snap.p, ctx->status.p, sizeof(int), hipMemcpyDeviceToDevice, ctx->stream));
    }
    HIPCHK(hipEventRecord(ctx->e_round, ctx->stream));
    ctx->eval_pending = true;
    ctx->eval_fired = false;
    ctx->xw_cached = false;  // the next round's plan forms x.w itself
    CAPI_END(ctx)
}

static void eval_fire(cocoa_ctx* ctx) {
    if (!ctx->eval_pending || ctx->eval_fired) return;
    eval_launch(ctx, true);
    ctx->eval_fired = true;
}

void cocoa_ctx::eval_quiesce() {
    if (inl_pending) {  // an uncollected cocoa_eval_begin: its result is dropped
        if (e_inl) HIPCHK(hipEventSynchronize(e_inl));
        inl_pending = false;
        inl_ranks = false;
    }
    if (!eval_pending) return;
    eval_fire(this);
    HIPCHK(hipEventSynchronize(e_done));
    eval_pending = false;
}

extern "C" int cocoa_eval_wait(cocoa_ctx* ctx, cocoa_eval_result* out) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_eval_wait");
    require(out != nullptr, COCOA_E_ARG, "null out");
    require(ctx->eval_pending, COCOA_E_STATE, "cocoa_eval_wait: no evaluation pending (cocoa_eval_async)");
    eval_fire(ctx);  // no round was issued after cocoa_eval_async
    HIPCHK(hipEventSynchronize(ctx->e_done));
    ctx->eval_pending = false;
    // the evaluated rounds' status word came back with the sums (h_eval[10]);
    // the next round's solver, still running, is checked by the next call that
    // synchronises ctx->stream or collects an evaluation behind it
    check_status_slot(ctx, 1);
    const double* h = ctx->h_eval + 4;
    finish(ctx, h[0], h[1], h[2], (int64_t)h[3], (int64_t)(ctx->has_test ? ctx->te.n : 0), out);
    CAPI_END(ctx)
}

// In-line evaluation with deferred read-back: the same pass as cocoa_eval,
// enqueued on the context's stream (so the next round's plan still reuses its
// row x.w), its sums copied to pinned memory behind it; the caller enqueues
// the next round before collecting them, and the GPU never idles while the
// host reads a round's gap.  Multi-rank and multi-device contexts evaluate at
// once (their merges exchange in order) and hand the result over at
// cocoa_eval_end.
extern "C" int cocoa_eval_begin(cocoa_ctx* ctx) {
    CAPI_BEGIN(ctx)
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    require(!ctx->inl_pending, COCOA_E_STATE, "an evaluation is pending: collect it with cocoa_eval_end first");
    require(!ctx->eval_pending, COCOA_E_STATE, "an evaluation is pending: collect it with cocoa_eval_wait first");
    if (!ctx->is_group() && ctx->comm && ctx->comm->world > 1 && !ctx->strict) {
        // fast multi-rank: the rank sums all-reduced on the device behind the pass
        // (hinge and alpha sums, then the error count; ||w||^2 is the same on
        // every rank), read back by cocoa_eval_end.  Over RCCL nothing here waits
        // for the GPU; the HOST transport stages through the host as always.
        cocoa::Comm& cm = *ctx->comm;
        if (ctx->n_test_glob < 0) {  // (once per test set: every rank takes this branch together)
            double nt = (double)(ctx->has_test ? ctx->te.n : 0);
            cm.allreduce(&nt, 1, false, ctx->stream);
            ctx->n_test_glob = (int64_t)nt;
        }
        if (!ctx->e_inl) HIPCHK(hipEventCreateWithFlags(&ctx->e_inl, hipEventDisableTiming));
        eval_launch(ctx, false, false);
        double* out = ctx->eval_out.as<double>();
        // ||w||^2: rank 0's everywhere (each rank sums the replicated w over its own grid)
        if (cm.rank != 0) HIPCHK(hipMemsetAsync(out + 2, 0, sizeof(double), ctx->stream));
        cm.allreduce(out, 3, true, ctx->stream);
        cm.allreduce(out + 3, 1, true, ctx->stream);
        HIPCHK(hipMemcpyAsync(ctx->h_eval, out, 4 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        if (ctx->abort_in_sum)  // the last exchange's all-reduced abort flag, read with the sums
            HIPCHK(hipMemcpyAsync(ctx->h_eval + 8, ctx->dw_sum + ctx->d, sizeof(double), hipMemcpyDeviceToHost,
                                  ctx->stream));
        HIPCHK(hipEventRecord(ctx->e_inl, ctx->stream));
        ctx->inl_ranks = true;
        ctx->inl_pending = true;
        return COCOA_OK;
    }
    if (ctx->is_group() || (ctx->comm && ctx->comm->world > 1)) {
        cocoa_eval_result r{};
        const int rc = cocoa_eval(ctx, &r);
        if (rc != COCOA_OK) return rc;
        ctx->eval_held = r;
    } else {
        if (!ctx->e_inl) HIPCHK(hipEventCreateWithFlags(&ctx->e_inl, hipEventDisableTiming));
        eval_launch(ctx);
        HIPCHK(hipEventRecord(ctx->e_inl, ctx->stream));
        ctx->inl_since_round = true;
    }
    ctx->inl_pending = true;
    CAPI_END(ctx)
}

extern "C" int cocoa_eval_end(cocoa_ctx* ctx, cocoa_eval_result* out) {
    CAPI_BEGIN(ctx)
    require(out != nullptr, COCOA_E_ARG, "null out");
    require(ctx->inl_pending, COCOA_E_STATE, "cocoa_eval_end: no evaluation pending (cocoa_eval_begin)");
    ctx->inl_pending = false;
    if (ctx->inl_ranks) {
        ctx->inl_ranks = false;
        HIPCHK(hipEventSynchronize(ctx->e_inl));
        const double* h = ctx->h_eval;
        if (ctx->abort_in_sum && h[8] != 0.0)
            throw Error(COCOA_E_HIP, "local solver: a hand-off between the solver's waves timed out on some rank "
                                     "(launch aborted)");
        finish(ctx, h[0], h[1], h[2], (int64_t)h[3], ctx->n_test_glob, out);
        return COCOA_OK;
    }
    if (ctx->is_group() || (ctx->comm && ctx->comm->world > 1)) {
        *out = ctx->eval_held;
        return COCOA_OK;
    }
    HIPCHK(hipEventSynchronize(ctx->e_inl));
    // the evaluated rounds' status word came back with the sums (h_eval[9]); a
    // round enqueued since may still run (checked at the next collection or sync)
    check_status_slot(ctx, 0);
    const double* h = ctx->h_eval;
    finish(ctx, h[0], h[1], h[2], (int64_t)h[3], (int64_t)(ctx->has_test ? ctx->te.n : 0), out);
    CAPI_END(ctx)
}

extern "C" int cocoa_eval_finish(const cocoa_ctx* ctx, double hinge_sum, double alpha_sum, double w_sqnorm,
                                 int64_t test_err_count, int64_t test_rows, cocoa_eval_result* out) {
    if (!ctx || !out) return COCOA_E_ARG;
    // w_sqnorm: the raw sum of squares of w (identical on every rank)
    finish(ctx, hinge_sum, alpha_sum, w_sqnorm, test_err_count, test_rows, out);
    return COCOA_OK;
}

static std::string checkpoint_path(const cocoa_ctx* ctx, int method = -1);

// Rounds t0+1 .. T of a started run.  With a checkpoint directory set, the
// (t, w, alpha) state is saved every chkpt_iter rounds, where the reference
// checkpoints its alpha RDD (CoCoA.scala:58-62; hingeDriver.scala:55-59 turns
// it off without a chkptDir).
static int run_rounds(cocoa_ctx* ctx, const cocoa_params* params, int32_t t0, cocoa_round_cb cb, void* user) {
    int rc = COCOA_OK;
    for (int32_t t = t0 + 1; t <= params->num_rounds; ++t) {
        rc = cocoa_round(ctx, t);
        if (rc) return rc;
        if (ctx->D.debug_iter > 0 && t % ctx->D.debug_iter == 0) {              // CoCoA.scala:51
            cocoa_eval_result ev{};
            rc = cocoa_eval(ctx, &ev);
            if (rc) return rc;
            if (cb) cb(user, t, &ev);
        }
        if (!ctx->ckpt_dir.empty() && ctx->D.chkpt_iter > 0 && t % ctx->D.chkpt_iter == 0) {  // CoCoA.scala:58
            rc = cocoa_checkpoint_save(ctx, checkpoint_path(ctx).c_str(), t);
            if (rc) return rc;
        }
    }
    return cocoa_sync(ctx);
}

extern "C" int cocoa_run(cocoa_ctx* ctx, const cocoa_params* params, const cocoa_debug* debug, int method,
                         const double* w_init, cocoa_round_cb cb, void* user) {
    const int rc = cocoa_init(ctx, params, debug, method, w_init);
    if (rc) return rc;
    return run_rounds(ctx, params, 0, cb, user);
}

// mkdir -p: sc.setCheckpointDir (hingeDriver.scala:56) creates the directory,
// so a missing one is created here, and an unusable one fails now rather than
// after chkptIter rounds of work.
static void make_dirs(const std::string& dir) {
    std::string cur;
    size_t i = 0;
    while (i <= dir.size()) {
        const size_t j = dir.find('/', i);
        const size_t e = j == std::string::npos ? dir.size() : j;
        cur = dir.substr(0, e);
        if (!cur.empty() && ::mkdir(cur.c_str(), 0777) != 0 && errno != EEXIST)
            throw Error(COCOA_E_IO, "cannot create checkpoint directory " + cur + ": " + std::strerror(errno));
        i = e + 1;
    }
    struct stat st {};
    require(::stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode) && ::access(dir.c_str(), W_OK) == 0, COCOA_E_IO,
            "checkpoint directory " + dir + " is not a writable directory");
}

extern "C" int cocoa_set_checkpoint_dir(cocoa_ctx* ctx, const char* dir) {
    CAPI_BEGIN(ctx)
    const std::string d = dir ? dir : "";
    if (!d.empty()) make_dirs(d);
    ctx->ckpt_dir = d;
    CAPI_END(ctx)
}

extern "C" int cocoa_checkpoint_file(cocoa_ctx* ctx, int method, char* buf, int64_t cap) {
    CAPI_BEGIN(ctx)
    require(buf != nullptr && cap > 0, COCOA_E_ARG, "cocoa_checkpoint_file: bad argument");
    require(!ctx->ckpt_dir.empty(), COCOA_E_STATE, "cocoa_checkpoint_file: no checkpoint directory set");
    const std::string p = checkpoint_path(ctx, method);
    require((int64_t)p.size() < cap, COCOA_E_ARG, "cocoa_checkpoint_file: buffer too small");
    std::memcpy(buf, p.c_str(), p.size() + 1);
    CAPI_END(ctx)
}

extern "C" int cocoa_resume(cocoa_ctx* ctx, const cocoa_params* params, const cocoa_debug* debug, int method,
                            const char* path, cocoa_round_cb cb, void* user) {
    int rc = cocoa_init(ctx, params, debug, method, nullptr);
    if (rc) return rc;
    int32_t t0 = 0;
    rc = cocoa_checkpoint_load(ctx, path, &t0);
    if (rc) return rc;
    return run_rounds(ctx, params, t0, cb, user);
}

extern "C" int cocoa_sync(cocoa_ctx* ctx) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        for (cocoa_ctx* sub : ctx->subs) sub_check(cocoa_sync(sub), sub);
        return COCOA_OK;
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    check_status(ctx);
    CAPI_END(ctx)
}

extern "C" int cocoa_get_w(cocoa_ctx* ctx, double* w_out) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        require(w_out != nullptr, COCOA_E_ARG, "cocoa_get_w: null output");
        group_get_state(ctx, w_out, nullptr);
        return COCOA_OK;
    }
    require(ctx->inited && w_out, COCOA_E_STATE, "cocoa_get_w: not initialised");
    std::vector<double> dev((size_t)ctx->d);
    HIPCHK(hipMemcpyAsync(dev.data(), ctx->w.p, sizeof(double) * (size_t)ctx->d, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    check_status(ctx);
    ctx->to_host_order(dev, w_out);
    CAPI_END(ctx)
}

extern "C" int cocoa_get_alpha(cocoa_ctx* ctx, double* alpha_out) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        require(alpha_out != nullptr, COCOA_E_ARG, "cocoa_get_alpha: null output");
        group_get_state(ctx, nullptr, alpha_out);
        return COCOA_OK;
    }
    require(ctx->inited && alpha_out, COCOA_E_STATE, "cocoa_get_alpha: not initialised");
    if (ctx->tr.n)
        HIPCHK(hipMemcpyAsync(alpha_out, ctx->alpha.p, sizeof(double) * (size_t)ctx->tr.n, hipMemcpyDeviceToHost,
                              ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    check_status(ctx);
    CAPI_END(ctx)
}

extern "C" int cocoa_set_w(cocoa_ctx* ctx, const double* w_in) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        require(w_in != nullptr, COCOA_E_ARG, "cocoa_set_w: null input");
        group_set_state(ctx, w_in, nullptr);
        return COCOA_OK;
    }
    require(ctx->inited && w_in, COCOA_E_STATE, "cocoa_set_w: not initialised");
    std::vector<double> dev;
    ctx->to_device_order(w_in, dev);
    HIPCHK(hipMemcpyAsync(ctx->w.p, dev.data(), sizeof(double) * (size_t)ctx->d, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->xw_cached = false;
    CAPI_END(ctx)
}

// an alpha outside [0, 1] (or NaN) switches the fast solvers to the explicit
// projected-gradient rule
static bool any_outside_unit(const double* a, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (!(a[i] >= 0.0 && a[i] <= 1.0)) return true;
    return false;
}

extern "C" int cocoa_set_alpha(cocoa_ctx* ctx, const double* alpha_in) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        require(alpha_in != nullptr, COCOA_E_ARG, "cocoa_set_alpha: null input");
        group_set_state(ctx, nullptr, alpha_in);
        return COCOA_OK;
    }
    require(ctx->inited && alpha_in, COCOA_E_STATE, "cocoa_set_alpha: not initialised");
    if (ctx->tr.n)
        HIPCHK(hipMemcpyAsync(ctx->alpha.p, alpha_in, sizeof(double) * (size_t)ctx->tr.n, hipMemcpyHostToDevice,
                              ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->alpha_oob = ctx->alpha_oob || any_outside_unit(alpha_in, ctx->tr.n);
    CAPI_END(ctx)
}

// ------------------------------------------------------------ checkpoint --
// <dir>/cocoa_m<method>_p<part_begin>.ck: one file per method and rank, the
// latest state only (each save replaces the previous one atomically).
static std::string checkpoint_path(const cocoa_ctx* ctx, int method) {
    return ctx->ckpt_dir + "/cocoa_m" + std::to_string(method < 0 ? ctx->method : method) + "_p" +
           std::to_string(ctx->part_begin) + ".ck";
}

namespace {
struct CkptHeader {
    char magic[8];
    int32_t method, num_features, k_glob, part_begin, k_loc, local_iters;
    int64_t n, rows;
    double lambda, beta, gamma;
    int32_t t, pad;
    int32_t seed, strict;  // DebugParams.seed and the numerics mode: a resume must continue the same trajectory
    int64_t reserved;
};
static_assert(sizeof(CkptHeader) == 96, "checkpoint header layout");

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ULL;
    return h;
}

CkptHeader ckpt_header(const cocoa_ctx* c, int32_t t) {
    CkptHeader h{};
    std::memcpy(h.magic, "COCOACK1", 8);
    h.method = c->method;
    h.num_features = c->d;
    h.k_glob = c->K_glob;
    h.part_begin = c->part_begin;
    h.k_loc = c->K_loc;
    h.local_iters = c->P.local_iters;
    h.n = c->P.n;
    h.rows = c->tr.n;
    h.lambda = c->P.lambda;
    h.beta = c->P.beta;
    h.gamma = c->P.gamma;
    h.t = t;
    h.seed = c->D.seed;
    h.strict = c->strict ? 1 : 0;
    return h;
}
}  // namespace

extern "C" int cocoa_checkpoint_save(cocoa_ctx* ctx, const char* path, int32_t t) {
    CAPI_BEGIN(ctx)
    require(ctx->inited, COCOA_E_STATE, "cocoa_checkpoint_save: call cocoa_init first");
    require(path != nullptr && t >= 0, COCOA_E_ARG, "cocoa_checkpoint_save: bad argument");
    std::vector<double> w((size_t)ctx->d), dev((size_t)ctx->d), al((size_t)std::max<int64_t>(ctx->tr.n, 1));
    if (ctx->is_group()) {
        // the whole problem's state: the same file a one-device run writes
        group_get_state(ctx, w.data(), al.data());  // (checks every device's solver status)
    } else {
        HIPCHK(hipMemcpyAsync(dev.data(), ctx->w.p, sizeof(double) * (size_t)ctx->d, hipMemcpyDeviceToHost,
                              ctx->stream));
        if (ctx->tr.n)
            HIPCHK(hipMemcpyAsync(al.data(), ctx->alpha.p, sizeof(double) * (size_t)ctx->tr.n, hipMemcpyDeviceToHost,
                                  ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        check_status(ctx);  // never save (with a valid checksum) the state of an aborted solver launch
        ctx->to_host_order(dev, w.data());
    }
    const CkptHeader h = ckpt_header(ctx, t);
    uint64_t sum = 1469598103934665603ULL;
    sum = fnv1a(sum, &h, sizeof h);
    sum = fnv1a(sum, w.data(), sizeof(double) * w.size());
    sum = fnv1a(sum, al.data(), sizeof(double) * (size_t)ctx->tr.n);
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    require(f != nullptr, COCOA_E_IO, std::string("cannot write checkpoint ") + tmp);
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1;
    ok = ok && std::fwrite(w.data(), sizeof(double), w.size(), f) == w.size();
    ok = ok && (ctx->tr.n == 0 ||
                std::fwrite(al.data(), sizeof(double), (size_t)ctx->tr.n, f) == (size_t)ctx->tr.n);
    ok = ok && std::fwrite(&sum, sizeof sum, 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    require(ok, COCOA_E_IO, std::string("short write on checkpoint ") + tmp);
    require(std::rename(tmp.c_str(), path) == 0, COCOA_E_IO, std::string("cannot rename checkpoint to ") + path);
    CAPI_END(ctx)
}

extern "C" int cocoa_checkpoint_load(cocoa_ctx* ctx, const char* path, int32_t* t_out) {
    CAPI_BEGIN(ctx)
    require(ctx->inited, COCOA_E_STATE, "cocoa_checkpoint_load: call cocoa_init first");
    require(path != nullptr && t_out != nullptr, COCOA_E_ARG, "cocoa_checkpoint_load: bad argument");
    FILE* f = std::fopen(path, "rb");
    require(f != nullptr, COCOA_E_IO, std::string("cannot open checkpoint ") + path);
    CkptHeader h{};
    std::vector<double> w((size_t)ctx->d), al((size_t)std::max<int64_t>(ctx->tr.n, 1));
    uint64_t stored = 0;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, "COCOACK1", 8) == 0;
    const CkptHeader want = ckpt_header(ctx, h.t);
    const bool same = ok && h.method == want.method && h.num_features == want.num_features &&
                      h.k_glob == want.k_glob && h.part_begin == want.part_begin && h.k_loc == want.k_loc &&
                      h.local_iters == want.local_iters && h.n == want.n && h.rows == want.rows &&
                      h.lambda == want.lambda && h.beta == want.beta && h.gamma == want.gamma && h.t >= 0 &&
                      h.seed == want.seed && h.strict == want.strict;
    if (same) {
        ok = std::fread(w.data(), sizeof(double), w.size(), f) == w.size();
        ok = ok && (ctx->tr.n == 0 || std::fread(al.data(), sizeof(double), (size_t)ctx->tr.n, f) == (size_t)ctx->tr.n);
        ok = ok && std::fread(&stored, sizeof stored, 1, f) == 1;
    }
    std::fclose(f);
    require(ok, COCOA_E_IO, std::string("not a COCOACK1 checkpoint or truncated: ") + path);
    require(same, COCOA_E_ARG,
            std::string("checkpoint ") + path +
                " was written for a different problem, method, partitioning, seed or numerics mode");
    uint64_t sum = 1469598103934665603ULL;
    sum = fnv1a(sum, &h, sizeof h);
    sum = fnv1a(sum, w.data(), sizeof(double) * w.size());
    sum = fnv1a(sum, al.data(), sizeof(double) * (size_t)ctx->tr.n);
    require(sum == stored, COCOA_E_IO, std::string("checkpoint checksum mismatch: ") + path);
    if (ctx->is_group()) {
        group_set_state(ctx, w.data(), al.data());
        *t_out = h.t;
        return COCOA_OK;
    }
    std::vector<double> dev;
    ctx->to_device_order(w.data(), dev);
    HIPCHK(hipMemcpyAsync(ctx->w.p, dev.data(), sizeof(double) * (size_t)ctx->d, hipMemcpyHostToDevice, ctx->stream));
    if (ctx->tr.n)
        HIPCHK(hipMemcpyAsync(ctx->alpha.p, al.data(), sizeof(double) * (size_t)ctx->tr.n, hipMemcpyHostToDevice,
                              ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->xw_cached = false;
    ctx->alpha_oob = ctx->alpha_oob || any_outside_unit(al.data(), ctx->tr.n);
    *t_out = h.t;
    CAPI_END(ctx)
}

// ------------------------------------------------- unit: CoCoA.localSDCA --
extern "C" int cocoa_local_sdca(cocoa_ctx* ctx, int32_t part, double* w, int32_t local_iters, double lambda, int32_t n,
                                double* alpha, int32_t seed, int plus, double sigma, double* delta_w,
                                double* delta_alpha) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {  // the device holding partition `part`
        require(!ctx->g_k0.empty(), COCOA_E_STATE, "cocoa_local_sdca: no training data");
        const int32_t r = group_owner_of_part(ctx, part);
        cocoa_ctx* sub = ctx->subs[(size_t)r];
        sub_check(cocoa_local_sdca(sub, part - ctx->g_k0[(size_t)r], w, local_iters, lambda, n, alpha, seed, plus,
                                   sigma, delta_w, delta_alpha),
                  sub);
        return COCOA_OK;
    }
    require(ctx->d > 0, COCOA_E_STATE, "cocoa_local_sdca: no training data");
    require(part >= 0 && part < ctx->K_loc && w && alpha && delta_w && local_iters >= 0, COCOA_E_ARG,
            "cocoa_local_sdca: bad argument");
    const int64_t p0 = ctx->h_part_ptr[(size_t)part], p1 = ctx->h_part_ptr[(size_t)part + 1];
    const int32_t nl = (int32_t)(p1 - p0);
    if (local_iters >= 1) require(nl >= 1, COCOA_E_ARG, "IllegalArgumentException: empty partition");
    ensure_cols(ctx->tr, ctx->d, ctx->stream);
    const int64_t d = ctx->d;
    hipStream_t s = ctx->stream;
    // a one-partition problem over the loaded CSR
    cocoa_ctx& c = *ctx;
    const int saved_method = c.method;
    c.method = plus ? COCOA_METHOD_COCOA_PLUS : COCOA_METHOD_COCOA;
    const int32_t saved_max = c.max_nl;
    c.max_nl = nl;
    plan_solver(&c, d);
    c.max_nl = saved_max;
    c.method = saved_method;
    DevBuf pp, smp, dwb, wb, wl, al, alw, sumb;
    const int64_t h_pp[2] = {p0, p1};
    upload(pp, h_pp, sizeof(h_pp), s);
    smp.alloc(sizeof(int32_t) * (size_t)std::max(local_iters, 1));
    dwb.alloc_zero(sizeof(double) * (size_t)d, s);
    std::vector<double> wdev;
    ctx->to_device_order(w, wdev);
    upload(wb, wdev.data(), sizeof(double) * (size_t)d, s);
    if (!plus) wl.alloc(sizeof(double) * (size_t)d);
    al.alloc_zero(sizeof(double) * (size_t)std::max<int64_t>(ctx->tr.n, 1), s);
    alw.alloc(sizeof(double) * (size_t)std::max<int64_t>(ctx->tr.n, 1));
    if (nl) HIPCHK(hipMemcpyAsync(al.as<double>() + p0, alpha, sizeof(double) * (size_t)nl, hipMemcpyHostToDevice, s));
    sumb.alloc(sizeof(double) * (size_t)d);
    SolverArgs a = c.sa;
    a.row_ptr = ctx->tr.row_ptr.as<int64_t>();
    a.col = ctx->tr.col.as<int32_t>();
    a.val = ctx->tr.val.as<double>();
    a.y = ctx->tr.y.as<double>();
    a.sqn = ctx->sqn.as<double>();
    a.rowflags = ctx->rowflags.as<uint8_t>();
    a.part_ptr = pp.as<int64_t>();
    a.samples = smp.as<int32_t>();
    a.alpha = al.as<double>();
    a.alpha_work = alw.as<double>();
    a.w = wb.as<double>();
    a.dw = dwb.as<double>();
    a.wloc = plus ? nullptr : wl.as<double>();
    a.plan_beg = nullptr;  // the unit API stages its rows itself
    a.plan_z = nullptr;
    a.plan_y = a.plan_q = a.plan_xw = nullptr;
    a.row_qp = nullptr;  // (the full rows and a dense deltaW)
    a.rowcoef = nullptr;
    a.d = d;
    a.H = local_iters;
    a.any_dup = ctx->any_dup ? 1 : 0;
    a.raw_alpha = 1;
    a.reg_chunks = reg_chunks_for(ctx->tr.nnz, ctx->tr.n, ctx->method);
    a.prof = nullptr;
    a.lam_n = lambda * (double)n;
    a.sigma = sigma;
    a.scaling = 1.0;
    if (local_iters >= 1) {
        launch_sampler(pp.as<int64_t>(), 1, seed, local_iters, smp.as<int32_t>(), ctx->jump.as<uint64_t>(), s);
        if (ctx->strict)
            launch_solver_strict(plus ? MODE_PLUS : MODE_COCOA, c.vec_lds, c.alpha_lds, a, 1, c.lds_bytes, s);
        else
            launch_solver_fast(plus ? MODE_PLUS : MODE_COCOA, c.vec_lds, c.alpha_lds, a, 1, c.lds_bytes, s);
        HIPCHK(hipGetLastError());
    }
    launch_fold(dwb.as<double>(), 1, d, sumb.as<double>(), nullptr, 1.0, false, ctx->d_inv.as<int32_t>(), true, s);
    HIPCHK(hipGetLastError());
    std::vector<double> old(alpha, alpha + nl);
    HIPCHK(hipMemcpyAsync(delta_w, sumb.p, sizeof(double) * (size_t)d, hipMemcpyDeviceToHost, s));
    if (nl) HIPCHK(hipMemcpyAsync(alpha, al.as<double>() + p0, sizeof(double) * (size_t)nl, hipMemcpyDeviceToHost, s));
    if (!plus) HIPCHK(hipMemcpyAsync(wdev.data(), wl.p, sizeof(double) * (size_t)d, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!plus) ctx->to_host_order(wdev, w);
    if (delta_alpha)
        for (int32_t i = 0; i < nl; ++i) delta_alpha[i] = alpha[i] - old[(size_t)i];  // CoCoA.scala:190
    if (ctx->inited) plan_solver(ctx, ctx->dw_slice, !is_sdca(ctx->method));
    CAPI_END(ctx)
}

extern "C" int cocoa_samples(cocoa_ctx* ctx, int32_t part, int32_t seed_plus_t, int32_t count, int32_t* out) {
    CAPI_BEGIN(ctx)
    if (ctx->is_group()) {
        require(!ctx->g_k0.empty(), COCOA_E_STATE, "cocoa_samples: no training data");
        const int32_t r = group_owner_of_part(ctx, part);
        cocoa_ctx* sub = ctx->subs[(size_t)r];
        sub_check(cocoa_samples(sub, part - ctx->g_k0[(size_t)r], seed_plus_t, count, out), sub);
        return COCOA_OK;
    }
    require(part >= 0 && part < ctx->K_loc && count >= 0 && out, COCOA_E_ARG, "cocoa_samples: bad argument");
    const int64_t h_pp[2] = {ctx->h_part_ptr[(size_t)part], ctx->h_part_ptr[(size_t)part + 1]};
    require(h_pp[1] > h_pp[0], COCOA_E_ARG, "IllegalArgumentException: empty partition");
    DevBuf pp, smp;
    upload(pp, h_pp, sizeof(h_pp), ctx->stream);
    smp.alloc(sizeof(int32_t) * (size_t)std::max(count, 1));
    if (count) {
        launch_sampler(pp.as<int64_t>(), 1, seed_plus_t, count, smp.as<int32_t>(), ctx->jump.as<uint64_t>(), ctx->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(out, smp.p, sizeof(int32_t) * (size_t)count, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    CAPI_END(ctx)
}

// ------------------------------------------------ multi-device context --
// cocoa_create_multi: ONE context over several GPUs, driven from the caller's
// one thread, for a caller that runs the whole problem in one process (the
// reference's single driver: hingeDriver.scala:84 -> CoCoA.runCoCoA, whose
// reduce and `w +=` happen inside that call, CoCoA.scala:45-48).  Device r
// holds the contiguous partition block [K r / N, K (r+1) / N) like rank r of
// a multi-process run (same part_begin / num_parts_global, so sigma' = K gamma
// and the scaling see the global K).  Per round every device runs its local
// half on its own stream; the deltaW sums then meet on the devices' streams:
//   fast   -- a reduce-scatter then all-gather of column slices by peer
//             copies over xGMI: device r sums slice r of every device's fold
//             in device order, then every device copies the other slices;
//   strict -- the ordered chain: device r's fold continues device r-1's (peer
//             copy, then the fold kernel), the last device's total goes to all,
// so strict stays bitwise equal to the single-device partition-order fold.
// No host round trip inside a round.

static void sub_check(int rc, const cocoa_ctx* sub) {
    if (rc != COCOA_OK) throw Error(rc, sub ? sub->err : std::string(cocoa_last_error(nullptr)));
}

static int32_t group_owner_of_part(const cocoa_ctx* g, int32_t part) {
    require(part >= 0 && part < g->K_loc, COCOA_E_ARG, "partition index out of range");
    int32_t r = 0;
    while (g->g_k0[(size_t)r + 1] <= part) ++r;
    return r;
}

extern "C" int cocoa_create_multi(int32_t n_devices, const int32_t* devices, int strict, cocoa_ctx** out) {
    if (!out) return COCOA_E_ARG;
    *out = nullptr;
    if (n_devices < 1 || n_devices > 64) {
        cocoa_set_global_error("cocoa_create_multi: n_devices must be in [1, 64]");
        return COCOA_E_ARG;
    }
    cocoa_ctx* g = new cocoa_ctx();
    g->strict = strict != 0;
    try {
        for (int32_t r = 0; r < n_devices; ++r) {
            const int dv = devices ? devices[r] : r;
            cocoa_ctx* sub = nullptr;
            const int rc = cocoa_create(dv, strict, nullptr, &sub);
            if (rc) throw Error(rc, std::string("cocoa_create_multi: device ") + std::to_string(dv) + ": " +
                                        cocoa_last_error(nullptr));
            g->subs.push_back(sub);
            HIPCHK(hipSetDevice(dv));
            hipEvent_t e1 = nullptr, e2 = nullptr;
            HIPCHK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
            g->g_ev.push_back(e1);
            HIPCHK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
            g->g_ev_cp.push_back(e2);
            hipEvent_t e3 = nullptr;
            HIPCHK(hipEventCreateWithFlags(&e3, hipEventDisableTiming));
            g->g_ev_rs.push_back(e3);
        }
        g->device = g->subs[0]->device;
        for (cocoa_ctx* a : g->subs)
            for (cocoa_ctx* b : g->subs)
                if (a != b && a->device == b->device) a->shared_dev = true;
        // peer access between distinct devices (xGMI); copies work without it too
        for (cocoa_ctx* a : g->subs)
            for (cocoa_ctx* b : g->subs) {
                if (a->device == b->device) continue;
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, a->device, b->device) == hipSuccess && can) {
                    HIPCHK(hipSetDevice(a->device));
                    const hipError_t e = hipDeviceEnablePeerAccess(b->device, 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
                    (void)hipGetLastError();
                }
            }
        HIPCHK(hipSetDevice(g->device));
        // fast mode over distinct devices: the deltaW sum as RCCL all-reduces
        // (COCOA_GROUP_EXCHANGE=peer keeps the peer-copy reduce-scatter); any
        // RCCL failure at set-up falls back to the peer copies
        g->g_exchange = g->strict ? "chain" : "peer";
        bool distinct = n_devices > 1 && !g->strict;
        for (int32_t a = 0; a < n_devices && distinct; ++a)
            for (int32_t b = a + 1; b < n_devices; ++b)
                if (g->subs[(size_t)a]->device == g->subs[(size_t)b]->device) distinct = false;
        const char* ge = std::getenv("COCOA_GROUP_EXCHANGE");
        if (distinct && !(ge && std::strcmp(ge, "peer") == 0)) {
            std::vector<int> devs;
            for (cocoa_ctx* sub : g->subs) devs.push_back(sub->device);
            try {
                g->g_rccl = cocoa::group_comm_create(devs);
                g->g_exchange = "rccl";
            } catch (const Error&) {
                g->g_rccl = nullptr;
            }
            HIPCHK(hipSetDevice(g->device));
        }
    } catch (const Error& e) {
        cocoa_set_global_error(e.what());
        delete g;
        return e.code;
    }
    *out = g;
    return COCOA_OK;
}

extern "C" int cocoa_num_devices(cocoa_ctx* ctx, int32_t* n_devices, int32_t* devices, int32_t cap) {
    CAPI_BEGIN(ctx)
    require(n_devices != nullptr, COCOA_E_ARG, "cocoa_num_devices: null output");
    *n_devices = ctx->is_group() ? (int32_t)ctx->subs.size() : 1;
    for (int32_t r = 0; devices && r < cap && r < *n_devices; ++r)
        devices[r] = ctx->is_group() ? ctx->subs[(size_t)r]->device : ctx->device;
    CAPI_END(ctx)
}

// dense: dense rows (val = X[n][d], col unused)
static void group_set_train(cocoa_ctx* g, bool dense, int32_t K, const int64_t* part_ptr, const int64_t* row_ptr,
                            const int32_t* col, const double* val, const double* y, int64_t n, int32_t d,
                            int32_t part_begin, int32_t Kg) {
    const int32_t N = (int32_t)g->subs.size();
    require(part_begin == 0 && Kg == K, COCOA_E_ARG,
            "a multi-device context holds the whole problem (part_begin = 0, num_parts_global = num_parts)");
    require(K >= N, COCOA_E_ARG, "cocoa_set_train: fewer partitions than devices");
    require(part_ptr && y && n >= 0 && d >= 1 && (dense || row_ptr), COCOA_E_ARG, "cocoa_set_train: bad argument");
    require(part_ptr[0] == 0 && part_ptr[K] == n, COCOA_E_ARG, "part_ptr must span [0, n_rows]");
    for (int32_t k = 0; k < K; ++k) require(part_ptr[k + 1] >= part_ptr[k], COCOA_E_ARG, "part_ptr not monotone");
    if (!dense) require(row_ptr[0] == 0, COCOA_E_ARG, "row_ptr[0] must be 0");
    g->g_k0.assign((size_t)N + 1, 0);
    g->g_r0.assign((size_t)N + 1, 0);
    for (int32_t r = 0; r <= N; ++r) {
        g->g_k0[(size_t)r] = (int32_t)((int64_t)K * r / N);  // configs.shard_bounds
        g->g_r0[(size_t)r] = part_ptr[g->g_k0[(size_t)r]];
    }
    // every device's host-side preparation (row norms, feature order, compact
    // slices) and upload in parallel, one thread per device
    std::vector<int> rcs((size_t)N, 0);
    std::vector<std::thread> th;
    for (int32_t r = 0; r < N; ++r)
        th.emplace_back([&, r] {
            cocoa_ctx* sub = g->subs[(size_t)r];
            const int32_t k0 = g->g_k0[(size_t)r], k1 = g->g_k0[(size_t)r + 1];
            const int64_t r0 = g->g_r0[(size_t)r], r1 = g->g_r0[(size_t)r + 1];
            std::vector<int64_t> pp((size_t)(k1 - k0) + 1);
            for (int32_t k = k0; k <= k1; ++k) pp[(size_t)(k - k0)] = part_ptr[k] - r0;
            if (dense) {
                rcs[(size_t)r] = cocoa_set_train_dense(sub, k1 - k0, pp.data(), val + r0 * (int64_t)d, y + r0, r1 - r0,
                                                       d, k0, K);
            } else {
                const int64_t e0 = row_ptr[r0];
                std::vector<int64_t> rp((size_t)(r1 - r0) + 1);
                for (int64_t i = r0; i <= r1; ++i) rp[(size_t)(i - r0)] = row_ptr[i] - e0;
                rcs[(size_t)r] = cocoa_set_train(sub, k1 - k0, pp.data(), rp.data(), col + e0, val + e0, y + r0,
                                                 r1 - r0, d, k0, K);
            }
        });
    for (auto& t : th) t.join();
    for (int32_t r = 0; r < N; ++r) sub_check(rcs[(size_t)r], g->subs[(size_t)r]);
    HIPCHK(hipSetDevice(g->device));
    g->d = d;
    g->K_loc = K;
    g->K_glob = K;
    g->part_begin = 0;
    g->tr.n = n;
    g->tr.nnz = dense ? n * (int64_t)d : row_ptr[n];
    g->h_part_ptr.assign(part_ptr, part_ptr + K + 1);
    g->tr_dense = g->subs[0]->tr_dense;
    g->has_test = false;
    g->te.n = 0;
    g->inited = false;
}

static void group_set_test(cocoa_ctx* g, bool dense, const int64_t* row_ptr, const int32_t* col, const double* val,
                           const double* y, int64_t n_rows) {
    const int32_t N = (int32_t)g->subs.size();
    require(g->d > 0, COCOA_E_STATE, "cocoa_set_test: call cocoa_set_train first");
    require(y && n_rows >= 0 && (dense || row_ptr), COCOA_E_ARG, "cocoa_set_test: bad argument");
    if (!dense) require(row_ptr[0] == 0, COCOA_E_ARG, "row_ptr[0] must be 0");
    g->g_t0.assign((size_t)N + 1, 0);
    for (int32_t r = 0; r <= N; ++r) g->g_t0[(size_t)r] = n_rows * r / N;  // any row split (OptUtils.scala:95-98)
    for (int32_t r = 0; r < N; ++r) {
        cocoa_ctx* sub = g->subs[(size_t)r];
        const int64_t t0 = g->g_t0[(size_t)r], t1 = g->g_t0[(size_t)r + 1];
        if (dense) {
            sub_check(cocoa_set_test_dense(sub, val + t0 * (int64_t)g->d, y + t0, t1 - t0), sub);
        } else {
            const int64_t e0 = row_ptr[t0];
            std::vector<int64_t> rp((size_t)(t1 - t0) + 1);
            for (int64_t i = t0; i <= t1; ++i) rp[(size_t)(i - t0)] = row_ptr[i] - e0;
            sub_check(cocoa_set_test(sub, rp.data(), col + e0, val + e0, y + t0, t1 - t0), sub);
        }
    }
    HIPCHK(hipSetDevice(g->device));
    g->has_test = true;
    g->te.n = n_rows;
}

// fast exchange: member r reduces the columns [slice(r), slice(r+1)) of deltaW
static int64_t group_slice(const cocoa_ctx* g, size_t r) {
    return (int64_t)g->d * (int64_t)r / (int64_t)g->subs.size();
}

static void group_init(cocoa_ctx* g, const cocoa_params* params, const cocoa_debug* debug, int method,
                       const double* w_init) {
    require(params && method >= 0 && method <= 4, COCOA_E_ARG, "cocoa_init: bad argument");
    require(g->d > 0 && !g->g_k0.empty(), COCOA_E_STATE, "cocoa_init: no training data");
    for (cocoa_ctx* sub : g->subs) sub_check(cocoa_init(sub, params, debug, method, w_init), sub);
    HIPCHK(hipSetDevice(g->device));
    g->P = *params;
    g->D = debug ? *debug : cocoa_debug{10, 0, 100, 0};
    g->method = method;
    g->scaling = g->subs[0]->scaling;
    g->alpha_oob = false;
    const size_t N = g->subs.size();
    if (!g->strict && N > 1)
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            const int64_t len = group_slice(g, r + 1) - group_slice(g, r);
            sub->x_stage.alloc(sizeof(double) * (N - 1) * (size_t)std::max<int64_t>(len, 1));
        }
    HIPCHK(hipSetDevice(g->device));
    g->inited = true;
}

namespace {
struct GroupPrev {
    cocoa_ctx* prev;
    hipEvent_t ev;
};
}  // namespace

// strict chain: this device's fold continues the previous device's
static void group_recv_prev(cocoa_ctx* c, void* user) {
    const GroupPrev* p = (const GroupPrev*)user;
    HIPCHK(hipStreamWaitEvent(c->stream, p->ev, 0));
    HIPCHK(hipMemcpyPeerAsync(c->dw_sum, c->device, p->prev->dw_sum, p->prev->device, sizeof(double) * (size_t)c->d,
                              c->stream));
}

static void group_round(cocoa_ctx* g, int32_t t) {
    require(g->inited, COCOA_E_STATE, "cocoa_round: call cocoa_init first");
    const size_t N = g->subs.size();
    const size_t bytes = sizeof(double) * (size_t)g->d;
    size_t owner = 0;  // strict: the device whose dw_sum ends up holding the total
    if (N == 1) {
        HIPCHK(hipSetDevice(g->subs[0]->device));
        run_local(g->subs[0], t, true);
        return;
    }
    if (g->strict) {
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            if (r == 0) {
                run_local(sub, t, false);
            } else {
                GroupPrev pv{g->subs[r - 1], g->g_ev[r - 1]};
                run_local(sub, t, false, sub->dw_sum, group_recv_prev, &pv);
            }
            HIPCHK(hipEventRecord(g->g_ev[r], sub->stream));
        }
        owner = N - 1;
    } else if (g->g_rccl) {
        // distinct devices: every member folds its partitions, then one grouped
        // RCCL all-reduce of the folds (each on its member's stream, behind the
        // fold), then the identical w update on every member
        std::vector<double*> bufs;
        std::vector<hipStream_t> streams;
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            run_local(sub, t, false);
            bufs.push_back(sub->dw_sum);
            streams.push_back(sub->stream);
        }
        g->g_rccl->allreduce(bufs, g->d, streams);
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            sub->timed(COCOA_K_APPLY, [&] {
                launch_apply(sub->w.as<double>(), sub->dw_sum, sub->d, sub->mult, sub->d_inv.as<int32_t>(), sub->stream);
            });
            sub->xw_cached = false;
        }
        HIPCHK(hipSetDevice(g->device));
        return;
    } else {
        // Every member folds its partitions; then a reduce-scatter and an
        // all-gather of column slices, all on the members' own streams: member
        // r gathers slice r of every other member's fold (N - 1 peer copies of
        // d / N doubles over xGMI) and sums the N pieces in member order,
        // ((x_0 + x_1) + x_2) + ..., the association the earlier gather-to-one
        // exchange used, so the total is reproducible and bitwise identical on
        // every member; then every member copies the other slices.  Per member
        // 2 (N - 1) / N * 8 d bytes cross the links, all members at once.
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            run_local(sub, t, false);
            HIPCHK(hipEventRecord(g->g_ev[r], sub->stream));
        }
        for (size_t r = 0; r < N; ++r) {  // reduce-scatter
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            const int64_t j0 = group_slice(g, r), len = group_slice(g, r + 1) - j0;
            double* stage = sub->x_stage.as<double>();
            for (size_t q = 0, i = 0; q < N; ++q) {
                if (q == r) continue;
                HIPCHK(hipStreamWaitEvent(sub->stream, g->g_ev[q], 0));
                if (len > 0)
                    HIPCHK(hipMemcpyPeerAsync(stage + i * (size_t)len, sub->device, g->subs[q]->dw_sum + j0,
                                              g->subs[q]->device, sizeof(double) * (size_t)len, sub->stream));
                ++i;
            }
            sub->timed(COCOA_K_FOLD, [&] {
                launch_sum_slices(sub->dw_sum + j0, stage, (int32_t)N, (int32_t)r, len, sub->stream);
            });
            HIPCHK(hipEventRecord(g->g_ev_rs[r], sub->stream));
        }
        for (size_t r = 0; r < N; ++r) {  // all-gather, then w += sum * scaling (CoCoA.scala:48)
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            for (size_t q = 0; q < N; ++q) {
                if (q == r) continue;
                const int64_t j0 = group_slice(g, q), len = group_slice(g, q + 1) - j0;
                HIPCHK(hipStreamWaitEvent(sub->stream, g->g_ev_rs[q], 0));
                if (len > 0)
                    HIPCHK(hipMemcpyPeerAsync(sub->dw_sum + j0, sub->device, g->subs[q]->dw_sum + j0,
                                              g->subs[q]->device, sizeof(double) * (size_t)len, sub->stream));
            }
            HIPCHK(hipEventRecord(g->g_ev_cp[r], sub->stream));
            sub->timed(COCOA_K_APPLY, [&] {
                launch_apply(sub->w.as<double>(), sub->dw_sum, sub->d, sub->mult, sub->d_inv.as<int32_t>(), sub->stream);
            });
            sub->xw_cached = false;
        }
        // a member's next fold overwrites its sum: only after every other
        // member has copied its slice of it
        for (size_t r = 0; r < N; ++r) {
            cocoa_ctx* sub = g->subs[r];
            HIPCHK(hipSetDevice(sub->device));
            for (size_t q = 0; q < N; ++q)
                if (q != r) HIPCHK(hipStreamWaitEvent(sub->stream, g->g_ev_cp[q], 0));
        }
        HIPCHK(hipSetDevice(g->device));
        return;
    }
    cocoa_ctx* src = g->subs[owner];
    for (size_t r = 0; r < N; ++r) {
        cocoa_ctx* sub = g->subs[r];
        HIPCHK(hipSetDevice(sub->device));
        if (r != owner) {
            HIPCHK(hipStreamWaitEvent(sub->stream, g->g_ev[owner], 0));
            HIPCHK(hipMemcpyPeerAsync(sub->dw_sum, sub->device, src->dw_sum, src->device, bytes, sub->stream));
            HIPCHK(hipEventRecord(g->g_ev_cp[r], sub->stream));
        }
        // w += sum * scaling (CoCoA.scala:48), identical on every device
        sub->timed(COCOA_K_APPLY, [&] {
            launch_apply(sub->w.as<double>(), sub->dw_sum, sub->d, sub->mult, sub->d_inv.as<int32_t>(), sub->stream);
        });
        sub->xw_cached = false;
    }
    // the owner's next fold overwrites its sum: only after every copy of it
    HIPCHK(hipSetDevice(src->device));
    for (size_t r = 0; r < N; ++r)
        if (r != owner) HIPCHK(hipStreamWaitEvent(src->stream, g->g_ev_cp[r], 0));
    HIPCHK(hipSetDevice(g->device));
}

static void group_eval(cocoa_ctx* g, cocoa_eval_result* out) {
    require(g->inited, COCOA_E_STATE, "call cocoa_init first");
    const size_t N = g->subs.size();
    for (cocoa_ctx* sub : g->subs) {
        HIPCHK(hipSetDevice(sub->device));
        eval_launch(sub);
    }
    double hinge = 0.0, alpha_sum = 0.0, w2 = 0.0, err = 0.0, n_test = 0.0;
    double carry[3] = {0.0, 0.0, 0.0};
    for (size_t r = 0; r < N; ++r) {
        cocoa_ctx* sub = g->subs[r];
        HIPCHK(hipSetDevice(sub->device));
        const EvalLocal ev = eval_collect(sub);
        if (g->strict) {
            strict_eval_carry(sub, r == 0, carry);  // the partition-order merge across devices
        } else {
            hinge = r == 0 ? ev.hinge : hinge + ev.hinge;  // device order
            alpha_sum = r == 0 ? ev.alpha_sum : alpha_sum + ev.alpha_sum;
        }
        if (r == 0) w2 = ev.w2;
        err += ev.err;  // integers: exact in any order
        n_test += ev.n_test;
    }
    if (g->strict) {
        hinge = carry[0];
        alpha_sum = carry[2];
    }
    HIPCHK(hipSetDevice(g->device));
    finish(g, hinge, alpha_sum, w2, (int64_t)err, (int64_t)n_test, out);
}

// (w in the original feature order, alpha of all rows) of a group
static void group_get_state(cocoa_ctx* g, double* w, double* alpha) {
    require(g->inited, COCOA_E_STATE, "not initialised");
    if (w) sub_check(cocoa_get_w(g->subs[0], w), g->subs[0]);
    for (size_t r = 0; alpha && r < g->subs.size(); ++r)
        sub_check(cocoa_get_alpha(g->subs[r], alpha + g->g_r0[r]), g->subs[r]);
    HIPCHK(hipSetDevice(g->device));
}

static void group_set_state(cocoa_ctx* g, const double* w, const double* alpha) {
    require(g->inited, COCOA_E_STATE, "not initialised");
    for (size_t r = 0; r < g->subs.size(); ++r) {
        if (w) sub_check(cocoa_set_w(g->subs[r], w), g->subs[r]);
        if (alpha) sub_check(cocoa_set_alpha(g->subs[r], alpha + g->g_r0[r]), g->subs[r]);
    }
    HIPCHK(hipSetDevice(g->device));
}

// ------------------------------------------------------------- profiling --
extern "C" int cocoa_stats_enable(cocoa_ctx* ctx, int enable) {
    CAPI_BEGIN(ctx)
    for (cocoa_ctx* sub : ctx->subs) sub_check(cocoa_stats_enable(sub, enable), sub);
    ctx->drain();
    ctx->stats = enable != 0;
    CAPI_END(ctx)
}

extern "C" int cocoa_stats_kernels(cocoa_ctx* ctx, uint32_t mask) {
    CAPI_BEGIN(ctx)
    for (cocoa_ctx* sub : ctx->subs) sub_check(cocoa_stats_kernels(sub, mask), sub);
    ctx->stats_mask = mask;
    CAPI_END(ctx)
}

extern "C" int cocoa_kernel_stats(cocoa_ctx* ctx, int kernel, double* total_ms, int64_t* launches) {
    CAPI_BEGIN(ctx)
    require(kernel >= 0 && kernel < COCOA_K_COUNT, COCOA_E_ARG, "bad kernel id");
    if (ctx->is_group()) {  // summed over the devices
        double tot = 0.0;
        int64_t cnt = 0;
        for (cocoa_ctx* sub : ctx->subs) {
            double m = 0.0;
            int64_t c = 0;
            sub_check(cocoa_kernel_stats(sub, kernel, &m, &c), sub);
            tot += m;
            cnt += c;
        }
        if (total_ms) *total_ms = tot;
        if (launches) *launches = cnt;
        return COCOA_OK;
    }
    ctx->drain();
    if (total_ms) *total_ms = ctx->tot_ms[kernel];
    if (launches) *launches = ctx->cnt[kernel];
    CAPI_END(ctx)
}

extern "C" int cocoa_stats_reset(cocoa_ctx* ctx) {
    CAPI_BEGIN(ctx)
    for (cocoa_ctx* sub : ctx->subs) sub_check(cocoa_stats_reset(sub), sub);
    ctx->drain();
    for (int i = 0; i < COCOA_K_COUNT; ++i) ctx->tot_ms[i] = 0, ctx->cnt[i] = 0;
    CAPI_END(ctx)
}

extern "C" int cocoa_solver_profile(cocoa_ctx* ctx, int enable) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_solver_profile");
    require(ctx->inited, COCOA_E_STATE, "call cocoa_init first");
    if (enable) {
        ctx->prof.alloc_zero(sizeof(uint64_t) * ((size_t)ctx->K_loc * kProfStride + 8), ctx->stream);  // + gram_kernel phases
        ctx->sa.prof = ctx->prof.as<uint64_t>();
    } else {
        ctx->sa.prof = nullptr;
    }
    CAPI_END(ctx)
}

extern "C" int cocoa_solver_profile_read(cocoa_ctx* ctx, uint64_t* out, int64_t count) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_solver_profile_read");
    require(out && ctx->prof.p, COCOA_E_STATE, "solver profiling not enabled");
    const size_t n = std::min<size_t>((size_t)count, (size_t)ctx->K_loc * kProfStride + 8);
    HIPCHK(hipMemcpyAsync(out, ctx->prof.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    CAPI_END(ctx)
}

extern "C" int cocoa_debug_gram_rows(cocoa_ctx* ctx, int32_t t, double* out, int64_t count) {
    CAPI_BEGIN(ctx)
    GROUP_REJECT(ctx, "cocoa_debug_gram_rows");
    require(ctx->inited && ctx->use_gram && ctx->gt.p, COCOA_E_STATE,
            "cocoa_debug_gram_rows: the context does not run the Gram-window solver with Gram rows");
    const int32_t H = ctx->P.local_iters;
    const int64_t need = (int64_t)ctx->K_loc * ctx->nbatch * 16 * 48;
    require(out && count >= need, COCOA_E_ARG, "cocoa_debug_gram_rows: out holds fewer than K * nbatch * 16 * 48");
    if (ctx->gstream) HIPCHK(hipStreamSynchronize(ctx->gstream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // a scratch sample / Gram buffer: the round state (and any prefetch) stays untouched
    DevBuf smp, gt;
    smp.alloc(sizeof(int32_t) * (size_t)ctx->samples_cap);
    gt.alloc(sizeof(double) * (size_t)need);
    launch_sampler(ctx->part_ptr.as<int64_t>(), ctx->K_loc, wrap32((int64_t)ctx->D.seed + t), H, smp.as<int32_t>(),
                   ctx->jump.as<uint64_t>(), ctx->stream);
    GramArgs ga = gram_args(ctx, smp.as<int32_t>(), gt.as<double>());
    ga.prof = nullptr;
    DevBuf fb;
    if (ga.chunks > 0) {
        fb.alloc(sizeof(int32_t) * (1 + 2 * (size_t)ctx->K_loc * (size_t)ctx->nbatch));
        ga.fb_n = fb.as<int32_t>();
        ga.fb = fb.as<int32_t>() + 1;
    }
    launch_gram(ga, ctx->stream);
    HIPCHK(hipMemcpyAsync(out, gt.p, sizeof(double) * (size_t)need, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    CAPI_END(ctx)
}

extern "C" int cocoa_plan_info(cocoa_ctx* ctx, char* buf, int len) {
    CAPI_BEGIN(ctx)
    require(buf && len > 0, COCOA_E_ARG, "bad buffer");
    if (ctx->is_group()) {  // device 0's plan (every device plans alike) + the device count
        sub_check(cocoa_plan_info(ctx->subs[0], buf, len), ctx->subs[0]);
        std::string p(buf);
        if (!p.empty() && p.back() == '}') p.pop_back();
        p += ",\"n_devices\":" + std::to_string(ctx->subs.size()) + ",\"exchange\":\"" + ctx->g_exchange + "\"}";
        require((int)p.size() < len, COCOA_E_ARG, "cocoa_plan_info: buffer too small");
        std::memcpy(buf, p.c_str(), p.size() + 1);
        return COCOA_OK;
    }
    // (no device access: the call never waits on the streams; the Gram-row
    // fallback count is cocoa_gram_fallback_count's)
    const int wrote = std::snprintf(buf, (size_t)len,
                  "{\"gram_chunks\":%d,\"gram_mirror\":%d,\"strict\":%d,\"method\":%d,\"K_loc\":%d,\"K_glob\":%d,\"d\":%d,\"vec_lds\":%d,\"alpha_lds\":%d,"
                  "\"lds_bytes\":%zu,\"stream_cap\":%d,\"any_dup\":%d,\"max_nl\":%d,"
                  "\"hot_nnz_frac_4096\":%.4f,\"dw_dbuf\":%d,\"solver\":\"%s\",\"dw_compact\":%d,\"max_u\":%lld,"
                  "\"sum_u\":%lld,\"fold\":\"%s\",\"xw_producer\":%d,\"side_cus_reserved\":%d,\"chain_hot\":%d,"
                  "\"dw_private\":%d,\"max_uh\":%lld,\"n_tail\":%lld,\"mbsgd_pull\":%d,\"eval_split\":%d,\"eval_warm\":%d,\"eval_test_split\":%d}",
                  ctx->use_gram ? ctx->gram_chunks : 0, ctx->gram_mirror && !ctx->device_shared() ? 1 : 0,
                  ctx->strict ? 1 : 0, ctx->method, ctx->K_loc, ctx->K_glob, ctx->d, ctx->vec_lds ? 1 : 0,
                  ctx->alpha_lds ? 1 : 0, ctx->lds_bytes, ctx->sa.stream_cap, ctx->any_dup ? 1 : 0, ctx->max_nl,
                  ctx->tr.nnz > 0 ? (double)ctx->n_hot_nnz[(size_t)std::min(ctx->d, 4096)] / (double)ctx->tr.nnz : 0.0,
                  ctx->dw_dbuf ? 1 : 0, ctx->use_dense ? "dense" : ctx->use_gram ? "gram" : "chain",
                  ctx->dw_compact ? 1 : 0, (long long)ctx->max_u, (long long)ctx->sum_u,
                  !ctx->dw_compact ? "dense" : (ctx->n_fitems > 0 && ctx->dw_dbuf) ? "blocks" : "gather",
                  ctx->xw_prod ? 1 : 0, ctx->gstream ? ctx->side_res : 0, ctx->sa.hot, ctx->dw_priv ? 1 : 0,
                  (long long)ctx->max_uh, (long long)ctx->n_tail, ctx->mbsgd_pull ? 1 : 0,
                  ctx->split_ready && !ctx->strict ? 1 : 0, ctx->split_ready && ctx->n_warm_tiles > 0 ? 1 : 0,
                  ctx->split_ready && ctx->has_test && ctx->te_split ? 1 : 0);
    require(wrote >= 0 && wrote < len, COCOA_E_ARG, "cocoa_plan_info: buffer too small");
    CAPI_END(ctx)
}

// Diagnostic: windows the last sequential Gram launch sent to the per-window
// kernel (gram_seq_kernel's pool overflows; the larger of the two Gram-row
// buffers' counts).  Waits for the context's streams.
extern "C" int cocoa_gram_fallback_count(cocoa_ctx* ctx, int32_t* out) {
    CAPI_BEGIN(ctx)
    require(out != nullptr, COCOA_E_ARG, "null output");
    if (ctx->is_group()) ctx = ctx->subs[0];
    *out = -1;
    if (ctx->use_gram && ctx->gram_chunks > 0 && ctx->gram_fb[0].p) {
        HIPCHK(hipSetDevice(ctx->device));
        if (ctx->gstream) HIPCHK(hipStreamSynchronize(ctx->gstream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        int32_t f2[2] = {0, 0};
        HIPCHK(hipMemcpy(&f2[0], ctx->gram_fb[0].p, sizeof(int32_t), hipMemcpyDeviceToHost));
        if (ctx->gram_fb[1].p) HIPCHK(hipMemcpy(&f2[1], ctx->gram_fb[1].p, sizeof(int32_t), hipMemcpyDeviceToHost));
        *out = std::max(f2[0], f2[1]);
    }
    CAPI_END(ctx)
}
