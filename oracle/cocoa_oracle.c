/*
 * cocoa_oracle.c -- CPU restatement of calvinmccarter/cocoa's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped product links, loads or
 * calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / the timed CPU
 * baseline, never as the thing measured or shipped.
 *
 * Parity status: PARITY UNPINNED at the breeze/Spark boundary.  The reference
 * (Scala 2.10 / Spark 1.3.1 / breeze 0.11.2, build.sbt:11-36) cannot be built
 * or run in this image (no JVM), and the reference repository holds no tests,
 * golden vectors or known-answer tests for this path.
 * What pins this restatement instead:
 *   - JDK java.util.Random known answers (tests/test_oracle.py),
 *   - the Hadoop-1.0.4 byte-split partition sizes of the demo data
 *     (SURVEY.md section 8, C1 row),
 *   - a second, independent pure-Python restatement that must agree bit for bit
 *     (tests/golden/make_golden.py -> tests/golden/c1_<name>.json fixtures),
 *   - the liblinear SVM optimum of the demo problem (scikit-learn), which long
 *     CoCoA+ runs must approach with a non-negative duality gap.
 * Assumptions about third-party arithmetic (breeze 0.11.2, not in the tree):
 *   sparse dot / norm / DenseVector sum are sequential left-to-right sums in
 *   stored-entry order starting from 0.0, with no fused multiply-add;
 *   norm(2) = sqrt(sum v*v);  Math.pow(r, 2) = r*r (fdlibm special case).
 *   Spark merges per-partition results in task-completion order; this
 *   restatement merges in partition-index order 0..K-1.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; x86-64 SSE2 doubles).
 * All citations are relative to /root/reference/.
 */
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* java.util.Random, as used by scala.util.Random(seed: Int)                  */
/* (CoCoA.scala:144,151; MinibatchCD.scala:91,98; SGD.scala:99,109).            */
/* JDK algorithm: 48-bit LCG, multiplier 0x5DEECE66D, addend 0xB.             */
/* ------------------------------------------------------------------------- */
#define JR_MULT 0x5DEECE66DULL
#define JR_ADD 0xBULL
#define JR_MASK ((1ULL << 48) - 1)

typedef struct {
    uint64_t seed;
} jrand_t;

static void jr_init(jrand_t *r, int64_t seed) {
    /* new Random(long seed): this.seed = (seed ^ multiplier) & mask */
    r->seed = ((uint64_t)seed ^ JR_MULT) & JR_MASK;
}

static int32_t jr_next(jrand_t *r, int bits) {
    r->seed = (r->seed * JR_MULT + JR_ADD) & JR_MASK;
    return (int32_t)(uint32_t)(r->seed >> (48 - bits));
}

/* Random.nextInt(bound): power-of-two fast path, else rejection loop with
 * Java int (32-bit wrapping) arithmetic in the test `bits - val + (bound-1) < 0`. */
static int32_t jr_next_int_bound(jrand_t *r, int32_t bound) {
    int32_t bits = jr_next(r, 31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)bits) >> 31);
    for (;;) {
        int32_t val = bits % bound;
        int32_t t = (int32_t)((uint32_t)bits - (uint32_t)val + (uint32_t)m); /* wraps like Java */
        if (t >= 0) return val;
        bits = jr_next(r, 31);
    }
}

/* ctypes helper: `count` draws of nextInt(bound) (bound > 0) or nextInt() (bound <= 0). */
void oracle_jrandom_ints(int64_t seed, int32_t bound, int32_t count, int32_t *out) {
    jrand_t r;
    jr_init(&r, seed);
    for (int32_t i = 0; i < count; ++i) out[i] = bound > 0 ? jr_next_int_bound(&r, bound) : jr_next(&r, 32);
}

/* ------------------------------------------------------------------------- */
/* Data: partitioned CSR.  Rows are kept in file order; partition k owns rows  */
/* [part_ptr[k], part_ptr[k+1]).  Entries are kept in stored order.            */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t n;          /* rows */
    int32_t d;          /* numFeatures */
    int32_t K;          /* partitions */
    int64_t *row_ptr;   /* n+1 */
    int32_t *col;       /* nnz, 0-based */
    double *val;        /* nnz */
    double *y;          /* n, +1/-1 */
    int64_t *part_ptr;  /* K+1 */
    int owns;           /* 1 if arrays were malloc'ed by the oracle */
} oracle_data;

void oracle_free_data(oracle_data *D) {
    if (D && D->owns) {
        free(D->row_ptr); free(D->col); free(D->val); free(D->y); free(D->part_ptr);
    }
    if (D) memset(D, 0, sizeof(*D));
}

/* Java String.trim(): strip chars <= ' ' from both ends. */
static void java_trim(const char **b, const char **e) {
    while (*b < *e && (unsigned char)**b <= ' ') ++*b;
    while (*e > *b && (unsigned char)(*e)[-1] <= ' ') --*e;
}

/* Integer.parseInt semantics (Scala String.toInt): [+-]?[0-9]+, int32 range. */
static int java_parse_int(const char *b, const char *e, int32_t *out) {
    if (b >= e) return -1;
    int neg = 0;
    if (*b == '+' || *b == '-') { neg = (*b == '-'); ++b; }
    if (b >= e) return -1;
    int64_t v = 0;
    for (; b < e; ++b) {
        if (*b < '0' || *b > '9') return -1;
        v = v * 10 + (*b - '0');
        if (v > 2147483648LL) return -1;
    }
    if (neg) v = -v;
    if (v > 2147483647LL || v < -2147483648LL) return -1;
    *out = (int32_t)v;
    return 0;
}

/* Double.parseDouble for the decimal forms LIBSVM files use (strtod is
 * correctly rounded, as is the JDK).  A trailing [fFdD] suffix is accepted. */
static int java_parse_double(const char *b, const char *e, double *out) {
    java_trim(&b, &e);
    if (b >= e) return -1;
    char buf[128];
    size_t len = (size_t)(e - b);
    if (len >= sizeof(buf)) return -1;
    memcpy(buf, b, len);
    buf[len] = 0;
    if (len > 1 && (buf[len - 1] == 'f' || buf[len - 1] == 'F' || buf[len - 1] == 'd' || buf[len - 1] == 'D'))
        buf[--len] = 0;
    for (size_t i = 0; i < len; ++i)  /* strtod would accept inf/nan spellings Java rejects */
        if (buf[i] == 'i' || buf[i] == 'n' || buf[i] == 'x' || buf[i] == 'X') {
            if (strcmp(buf, "NaN") && strcmp(buf, "Infinity") && strcmp(buf, "+Infinity") && strcmp(buf, "-Infinity"))
                return -1;
        }
    char *end = NULL;
    errno = 0;
    double v = strtod(buf, &end);
    if (end != buf + len) return -1;
    *out = v;
    return 0;
}

/* Hadoop 1.0.4 FileInputFormat.getSplits for one local file:
 * splitSize = max(1, min(S / numSplits, 32 MiB local block)); emit splits
 * while remaining/splitSize > 1.1 (SPLIT_SLOP), then the remainder.
 * A line belongs to the split in which its first byte lies (LineRecordReader).
 * Returns the number of splits written to starts[] (<= cap). */
static int hadoop_splits(int64_t S, int numSplits, int64_t *starts, int cap) {
    int64_t goal = S / (numSplits == 0 ? 1 : numSplits);
    int64_t block = 32LL * 1024 * 1024;
    int64_t split = goal < block ? goal : block;
    if (split < 1) split = 1;
    int ns = 0;
    int64_t rem = S;
    while ((double)rem / (double)split > 1.1) {
        if (ns < cap) starts[ns] = S - rem;
        ++ns;
        rem -= split;
    }
    if (rem != 0) {
        if (ns < cap) starts[ns] = S - rem;
        ++ns;
    }
    if (ns == 0) { starts[0] = 0; ns = 1; }
    return ns;
}

/* OptUtils.loadLIBSVMData (OptUtils.scala:11-53).
 * Returns 0 on success, negative error code on failure (with message). */
int oracle_load_libsvm(const char *path, int32_t num_splits, int32_t num_feats, oracle_data *out,
                       char *errbuf, int errlen) {
    memset(out, 0, sizeof(*out));
    FILE *f = fopen(path, "rb");
    if (!f) { snprintf(errbuf, errlen, "cannot open %s", path); return -1; }
    fseek(f, 0, SEEK_END);
    int64_t S = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)S + 1);
    if (S > 0 && fread(buf, 1, (size_t)S, f) != (size_t)S) { fclose(f); free(buf); snprintf(errbuf, errlen, "read error"); return -1; }
    fclose(f);
    buf[S] = 0;

    int64_t goal0 = S / (num_splits <= 0 ? 1 : num_splits);
    int64_t ss0 = goal0 < 32LL * 1024 * 1024 ? goal0 : 32LL * 1024 * 1024;
    int cap = (int)(S / (ss0 < 1 ? 1 : ss0)) + 4;
    int64_t *starts = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    int ns = hadoop_splits(S, num_splits, starts, cap);
    /* Spark coalesce(numSplits) with more Hadoop splits than requested only
     * happens for files > 32 MiB * numSplits; group consecutive splits
     * (CoalescedRDD no-locality rule). */
    int K = ns <= num_splits ? ns : num_splits;

    /* count lines */
    int64_t nlines = 0;
    for (int64_t p = 0; p < S;) {
        const char *nl = memchr(buf + p, '\n', (size_t)(S - p));
        int64_t e = nl ? (nl - buf) : S;
        ++nlines;
        p = e + 1;
    }
    int64_t nnz_cap = 0;
    for (int64_t p = 0; p < S; ++p) nnz_cap += (buf[p] == ':');

    out->row_ptr = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nlines + 1));
    out->col = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nnz_cap + 1));
    out->val = (double *)malloc(sizeof(double) * (size_t)(nnz_cap + 1));
    out->y = (double *)malloc(sizeof(double) * (size_t)(nlines + 1));
    out->part_ptr = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
    out->owns = 1;
    out->d = num_feats;
    out->K = K;

    int64_t row = 0, nnz = 0;
    int split_idx = 0;
    out->row_ptr[0] = 0;
    for (int64_t p = 0; p < S;) {
        const char *nl = memchr(buf + p, '\n', (size_t)(S - p));
        int64_t e = nl ? (nl - buf) : S;
        /* the Hadoop split in which this line starts */
        while (split_idx + 1 < ns && p >= starts[split_idx + 1]) ++split_idx;
        /* Spark coalesce(K): identity when ns == K; otherwise CoalescedRDD's
         * no-locality grouping, partition i <- splits [i*ns/K, (i+1)*ns/K) */
        int part = split_idx;
        if (ns > K) {
            part = 0;
            while (part + 1 < K && (int64_t)split_idx >= ((int64_t)(part + 1) * ns) / K) ++part;
        }
        out->part_ptr[part + 1] += 1;   /* row count; prefix-summed below */

        const char *b = buf + p, *le = buf + e;
        java_trim(&b, &le);
        /* parts = line.trim().split(' '): trailing empty tokens dropped */
        const char *tok = b;
        int first = 1;
        const char *scan = b;
        for (;;) {
            const char *sp = scan;
            while (sp < le && *sp != ' ') ++sp;
            const char *te = sp;
            if (first) {
                /* label: parts(0).contains("+") || parts(0).toInt == 1 */
                int has_plus = memchr(tok, '+', (size_t)(te - tok)) != NULL;
                double lab = -1.0;
                if (has_plus) lab = 1.0;
                else {
                    int32_t iv;
                    if (java_parse_int(tok, te, &iv) != 0) {
                        snprintf(errbuf, errlen, "NumberFormatException: bad label on line %lld", (long long)row + 1);
                        free(buf); free(starts); oracle_free_data(out); return -2;
                    }
                    if (iv == 1) lab = 1.0;
                }
                out->y[row] = lab;
                first = 0;
            } else {
                /* trailing empty tokens are removed by split; interior ones are errors */
                int trailing_only = 1;
                for (const char *q = tok; q < le; ++q) if (*q != ' ') { trailing_only = 0; break; }
                if (trailing_only) break;
                /* token.split(':') match { case Array(i, j) => (i.toInt - 1, j.toDouble) } */
                const char *c1 = memchr(tok, ':', (size_t)(te - tok));
                if (!c1 || c1 + 1 >= te || memchr(c1 + 1, ':', (size_t)(te - c1 - 1))) {
                    snprintf(errbuf, errlen, "MatchError: bad feature token on line %lld", (long long)row + 1);
                    free(buf); free(starts); oracle_free_data(out); return -3;
                }
                int32_t idx;
                double v;
                if (java_parse_int(tok, c1, &idx) != 0 || java_parse_double(c1 + 1, te, &v) != 0) {
                    snprintf(errbuf, errlen, "NumberFormatException: bad feature on line %lld", (long long)row + 1);
                    free(buf); free(starts); oracle_free_data(out); return -2;
                }
                int64_t j = (int64_t)idx - 1;
                if (j < 0 || j >= num_feats) {
                    /* breeze would throw ArrayIndexOutOfBounds at the first dot */
                    snprintf(errbuf, errlen, "ArrayIndexOutOfBounds: feature %d on line %lld (numFeatures=%d)", idx,
                             (long long)row + 1, num_feats);
                    free(buf); free(starts); oracle_free_data(out); return -4;
                }
                out->col[nnz] = (int32_t)j;
                out->val[nnz] = v;
                ++nnz;
            }
            if (sp >= le) break;
            tok = scan = sp + 1;
        }
        ++row;
        out->row_ptr[row] = nnz;
        p = e + 1;
    }
    out->n = row;
    for (int q = 1; q <= K; ++q) out->part_ptr[q] += out->part_ptr[q - 1];
    free(buf);
    free(starts);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* breeze arithmetic as assumed above                                          */
/* ------------------------------------------------------------------------- */
static inline double sp_dot(const int32_t *c, const double *v, int64_t z, const double *dense) {
    double s = 0.0;
    for (int64_t i = 0; i < z; ++i) s += v[i] * dense[c[i]];
    return s;
}
static inline double sp_norm2(const double *v, int64_t z) {
    double s = 0.0;
    for (int64_t i = 0; i < z; ++i) s += v[i] * v[i];
    return sqrt(s);
}
static inline double dense_norm2(const double *w, int64_t d) {
    double s = 0.0;
    for (int64_t i = 0; i < d; ++i) s += w[i] * w[i];
    return sqrt(s);
}
/* java.lang.Math.min/max on doubles (NaN-propagating, -0.0 < +0.0) */
static inline double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
    return a >= b ? a : b;
}
static inline double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return signbit(a) ? a : b;
    return a <= b ? a : b;
}

/* ------------------------------------------------------------------------- */
/* CoCoA.localSDCA  (CoCoA.scala:130-192)                                      */
/* rows: local partition CSR (row_ptr relative to col/val base).              */
/* w: the task's copy of wInit; mutated in place when !plus (:142,183).       */
/* alpha: mutated in place (:186).  delta_w: dense d, zeroed here (:145).     */
/* delta_alpha (optional, may be NULL): alpha - alphaOld (:190).               */
/* ------------------------------------------------------------------------- */
void oracle_local_sdca(const int64_t *row_ptr, const int32_t *col, const double *val, const double *y,
                       int32_t n_local, int32_t d, double *w, int32_t local_iters, double lambda, int32_t n,
                       double *alpha, const double *alpha_old, int32_t seed, int plus, double sigma,
                       double *delta_w, double *delta_alpha) {
    jrand_t r;
    jr_init(&r, (int64_t)seed);
    memset(delta_w, 0, sizeof(double) * (size_t)d);
    const double lam_n = lambda * (double)n;
    for (int32_t it = 1; it <= local_iters; ++it) {
        int32_t idx = jr_next_int_bound(&r, n_local);                 /* :151 */
        const int64_t b = row_ptr[idx], z = row_ptr[idx + 1] - b;
        const int32_t *c = col + b;
        const double *v = val + b;
        const double yy = y[idx];
        double grad;
        if (plus)                                                     /* :157-163 */
            grad = (yy * (sp_dot(c, v, z, w) + (sigma * sp_dot(c, v, z, delta_w))) - 1.0) * lam_n;
        else
            grad = (yy * (sp_dot(c, v, z, w)) - 1.0) * lam_n;
        double proj = grad;                                           /* :166-170 */
        if (alpha[idx] <= 0.0) proj = jmin(grad, 0.0);
        else if (alpha[idx] >= 1.0) proj = jmax(grad, 0.0);
        if (fabs(proj) != 0.0) {                                      /* :172 */
            double nr = sp_norm2(v, z);
            double xnorm = nr * nr;                                   /* :173 Math.pow(.,2) */
            double qii = plus ? xnorm * sigma : xnorm;                /* :174 */
            double na = 1.0;
            if (qii != 0.0) na = jmin(jmax((alpha[idx] - (grad / qii)), 0.0), 1.0); /* :175-178 */
            double coef = (yy * (na - alpha[idx])) / lam_n;          /* :181 */
            for (int64_t i = 0; i < z; ++i) {
                double u = v[i] * coef;
                if (!plus) w[c[i]] += u;                              /* :182-184 */
                delta_w[c[i]] += u;                                   /* :185 */
            }
            alpha[idx] = na;                                          /* :186 */
        }
    }
    if (delta_alpha)
        for (int32_t i = 0; i < n_local; ++i) delta_alpha[i] = alpha[i] - alpha_old[i];
}

/* MinibatchCD.partitionUpdate inner loop (MinibatchCD.scala:76-132): like
 * !plus localSDCA but with the stale w (never written) and no sigma. */
static void mbcd_local(const int64_t *row_ptr, const int32_t *col, const double *val, const double *y, int32_t n_local,
                       int32_t d, const double *w, int32_t local_iters, double lambda, int32_t n, double *alpha,
                       int32_t seed, double *delta_w) {
    jrand_t r;
    jr_init(&r, (int64_t)seed);
    memset(delta_w, 0, sizeof(double) * (size_t)d);
    const double lam_n = lambda * (double)n;
    for (int32_t it = 1; it <= local_iters; ++it) {
        int32_t idx = jr_next_int_bound(&r, n_local);
        const int64_t b = row_ptr[idx], z = row_ptr[idx + 1] - b;
        const int32_t *c = col + b;
        const double *v = val + b;
        const double yy = y[idx];
        double grad = (yy * (sp_dot(c, v, z, w)) - 1.0) * lam_n;      /* MinibatchCD.scala:104 */
        double proj = grad;
        if (alpha[idx] <= 0.0) proj = jmin(grad, 0.0);
        else if (alpha[idx] >= 1.0) proj = jmax(grad, 0.0);
        if (fabs(proj) != 0.0) {
            double nr = sp_norm2(v, z);
            double qii = nr * nr;                                     /* MinibatchCD.scala:114 */
            double na = 1.0;
            if (qii != 0.0) na = jmin(jmax((alpha[idx] - (grad / qii)), 0.0), 1.0);
            double coef = (yy * (na - alpha[idx])) / lam_n;
            for (int64_t i = 0; i < z; ++i) delta_w[c[i]] += v[i] * coef; /* MinibatchCD.scala:121-122 */
            alpha[idx] = na;
        }
    }
    (void)d;
}

/* SGD.partitionUpdate (SGD.scala:87-139). t0 is the Double parameter `t`. */
static void sgd_local(const int64_t *row_ptr, const int32_t *col, const double *val, const double *y, int32_t n_local,
                      int32_t d, const double *w_init, double lambda, double t0, int32_t local_iters, int local,
                      int32_t seed, double *w_scratch, double *delta_w) {
    jrand_t r;
    jr_init(&r, (int64_t)seed);
    memcpy(w_scratch, w_init, sizeof(double) * (size_t)d);           /* SGD.scala:100 */
    memset(delta_w, 0, sizeof(double) * (size_t)d);                   /* SGD.scala:101 */
    for (int32_t i = 1; i <= local_iters; ++i) {
        double step = 1.0 / (lambda * (t0 + (double)i));              /* SGD.scala:106 */
        int32_t idx = jr_next_int_bound(&r, n_local);                 /* SGD.scala:109 */
        const int64_t b = row_ptr[idx], z = row_ptr[idx + 1] - b;
        const int32_t *c = col + b;
        const double *v = val + b;
        const double yy = y[idx];
        double ev = 1.0 - (yy * (sp_dot(c, v, z, w_scratch)));        /* SGD.scala:115 */
        if (local) {                                                  /* SGD.scala:117-121 */
            double scale = 1.0 - (step * lambda);
            for (int32_t j = 0; j < d; ++j) w_scratch[j] *= scale;
        }
        if (ev > 0) {                                                 /* SGD.scala:124-130 */
            for (int64_t q = 0; q < z; ++q) {
                double u = v[q] * yy;
                delta_w[c[q]] += u;
                if (local) w_scratch[c[q]] += (u * step);
            }
        }
        if (local)                                                    /* SGD.scala:132-134 */
            for (int32_t j = 0; j < d; ++j) delta_w[j] = w_scratch[j] - w_init[j];
    }
}

/* ------------------------------------------------------------------------- */
/* OptUtils evaluation (OptUtils.scala:57-98)                                  */
/* ------------------------------------------------------------------------- */
/* sum of hinge losses: per-partition reduceLeft in row order, partitions
 * merged in index order (Spark RDD.reduce). */
/* Partition-parallel evaluation, as the reference's evaluation is a Spark job
 * over the partitions (local[N]: one task per partition, N at a time): every
 * partition folds its own rows, the driver merges the partition results in
 * partition order -- so the result does not depend on the thread count. */
typedef struct {
    const oracle_data *D;
    const double *w;
    double *part;      /* per-partition hinge fold */
    int64_t *cnt;      /* per-partition error count */
    int nt, tid;
} eval_arg;

static double hinge_part(const oracle_data *D, const double *w, int32_t k) {
    int64_t r0 = D->part_ptr[k], r1 = D->part_ptr[k + 1];
    double acc = 0.0;
    for (int64_t r = r0; r < r1; ++r) {
        int64_t b = D->row_ptr[r], z = D->row_ptr[r + 1] - b;
        double h = jmax(1.0 - D->y[r] * (sp_dot(D->col + b, D->val + b, z, w)), 0.0); /* :57-61 */
        acc = (r == r0) ? h : acc + h;                                /* reduceLeft */
    }
    return acc;
}

static int64_t errors_rows(const oracle_data *D, const double *w, int64_t r0, int64_t r1) {
    int64_t cnt = 0;
    for (int64_t r = r0; r < r1; ++r) {
        int64_t b = D->row_ptr[r], z = D->row_ptr[r + 1] - b;
        if (!((sp_dot(D->col + b, D->val + b, z, w)) * (D->y[r]) > 0)) ++cnt; /* OptUtils.scala:97 */
    }
    return cnt;
}

static void *eval_worker(void *p) {
    eval_arg *a = (eval_arg *)p;
    if (a->part)
        for (int32_t k = a->tid; k < a->D->K; k += a->nt) a->part[k] = hinge_part(a->D, a->w, k);
    if (a->cnt)  /* integer counts: any split of the rows gives the same total */
        a->cnt[a->tid] = errors_rows(a->D, a->w, a->D->n * a->tid / a->nt, a->D->n * (a->tid + 1) / a->nt);
    return NULL;
}

/* per-partition hinge folds (part) or per-thread error counts (cnt[thread]) */
static void eval_parts(const oracle_data *D, const double *w, double *part, int64_t *cnt, int nthreads) {
    int nt = part ? (nthreads < D->K ? nthreads : D->K) : nthreads;
    if (nt > 256) nt = 256;
    if (nt <= 1) {
        eval_arg a = {D, w, part, cnt, 1, 0};
        eval_worker(&a);
        return;
    }
    pthread_t th[256];
    eval_arg args[256];
    for (int i = 0; i < nt; ++i) {
        eval_arg a = {D, w, part, cnt, nt, i};
        args[i] = a;
        pthread_create(&th[i], NULL, eval_worker, &args[i]);
    }
    for (int i = 0; i < nt; ++i) pthread_join(th[i], NULL);
}

static double hinge_sum_mt(const oracle_data *D, const double *w, int nthreads) {
    double *part = (double *)malloc(sizeof(double) * ((size_t)D->K + 1));
    eval_parts(D, w, part, NULL, nthreads);
    double tot = 0.0;
    int have = 0;
    for (int32_t k = 0; k < D->K; ++k) {                             /* merge in partition order */
        if (D->part_ptr[k + 1] <= D->part_ptr[k]) continue;
        tot = have ? tot + part[k] : part[k];
        have = 1;
    }
    free(part);
    return tot;
}

static double hinge_sum(const oracle_data *D, const double *w) { return hinge_sum_mt(D, w, 1); }

static int64_t error_count_mt(const oracle_data *D, const double *w, int nthreads) {
    int nt = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
    int64_t *cnt = (int64_t *)calloc((size_t)nt, sizeof(int64_t));
    eval_parts(D, w, NULL, cnt, nt);
    int64_t tot = 0;
    for (int i = 0; i < nt; ++i) tot += cnt[i];
    free(cnt);
    return tot;
}

double oracle_primal(const oracle_data *D, const double *w, double lambda) {
    double avg = hinge_sum(D, w) / (double)D->n;                     /* :65-68 */
    double nw = dense_norm2(w, D->d);
    return avg + (0.5 * lambda * (nw * nw));                          /* :73-75 */
}

/* alpha: n entries, partition-contiguous like D's rows.  Per-partition
 * DenseVector.sum, merged in partition order (alpha.map(_.sum).reduce). */
static double alpha_sum_parts(const oracle_data *D, const double *alpha) {
    double tot = 0.0;
    int have = 0;
    for (int32_t k = 0; k < D->K; ++k) {
        int64_t r0 = D->part_ptr[k], r1 = D->part_ptr[k + 1];
        double s = 0.0;                                               /* DenseVector.sum */
        for (int64_t r = r0; r < r1; ++r) s += alpha[r];
        tot = have ? tot + s : s;
        have = 1;
    }
    return tot;
}

double oracle_dual(const oracle_data *D, const double *w, const double *alpha, double lambda) {
    double nw = dense_norm2(w, D->d);
    return (-lambda / 2 * (nw * nw)) + (alpha_sum_parts(D, alpha) / (double)D->n); /* :80-84 */
}

double oracle_gap(const oracle_data *D, const double *w, const double *alpha, double lambda) {
    return oracle_primal(D, w, lambda) - oracle_dual(D, w, alpha, lambda); /* :89-91 */
}

/* returns the error COUNT; the reference divides by n (OptUtils.scala:95-98) */
int64_t oracle_error_count(const oracle_data *D, const double *w) { return error_count_mt(D, w, 1); }

/* ------------------------------------------------------------------------- */
/* Round drivers: CoCoA.runCoCoA (CoCoA.scala:22-66), MinibatchCD.runMbCD      */
/* (MinibatchCD.scala:19-61), SGD.runSGD (SGD.scala:21-70).                    */
/* ------------------------------------------------------------------------- */
enum { M_PLUS = 0, M_COCOA = 1, M_MBCD = 2, M_MBSGD = 3, M_LOCALSGD = 4 };

typedef struct {
    oracle_data D;     /* borrowed arrays */
    int method;
    int32_t n, H;
    double lambda, beta, gamma;
    int32_t seed;
    int nthreads;
    double *w;         /* d */
    double *alpha;     /* n */
    double *alpha_old; /* n */
    double *dw;        /* K*d private deltaW */
    double *wloc;      /* K*d task copy of w (CoCoA / SGD) */
    double scaling;
    int32_t t_cur;
    double sgd_step;
    int32_t Kg;        /* global number of partitions (== D.K unless sharded) */
    double mult;       /* multiplier of the last local round's deltaW sum */
} oracle_run;

void oracle_run_set_scaling(oracle_run *R);

oracle_run *oracle_run_create(const oracle_data *train, int method, int32_t n, int32_t H, double lambda,
                              double beta, double gamma, int32_t seed, int nthreads) {
    oracle_run *R = (oracle_run *)calloc(1, sizeof(oracle_run));
    R->D = *train;
    R->D.owns = 0;
    R->method = method;
    R->n = n; R->H = H; R->lambda = lambda; R->beta = beta; R->gamma = gamma; R->seed = seed;
    R->nthreads = nthreads < 1 ? 1 : nthreads;
    R->Kg = train->K;
    int64_t d = train->d, K = train->K;
    R->w = (double *)calloc((size_t)d, sizeof(double));               /* wInit = zeros */
    R->alpha = (double *)calloc((size_t)train->n + 1, sizeof(double));
    R->alpha_old = (double *)calloc((size_t)train->n + 1, sizeof(double));
    R->dw = (double *)calloc((size_t)(K * d), sizeof(double));
    R->wloc = (double *)calloc((size_t)(K * d), sizeof(double));
    oracle_run_set_scaling(R);
    return R;
}

/* scaling per method from the GLOBAL partition count (CoCoA.scala:37,
 * MinibatchCD.scala:32, SGD.scala:34-39) */
void oracle_run_set_scaling(oracle_run *R) {
    const int64_t K = R->Kg;
    const int32_t H = R->H;
    const double beta = R->beta, gamma = R->gamma;
    const int method = R->method;
    /* parts * localIters is Scala Int arithmetic (wraps) */
    const double kh = (double)(int32_t)((uint32_t)K * (uint32_t)H);
    switch (method) {
        case M_PLUS: R->scaling = gamma; break;                       /* CoCoA.scala:37 */
        case M_COCOA: R->scaling = beta / (double)K; break;           /* CoCoA.scala:37 */
        case M_MBCD: R->scaling = beta / kh; break;                   /* MinibatchCD.scala:32 */
        case M_LOCALSGD: R->scaling = beta / (double)K; break;        /* SGD.scala:36 */
        case M_MBSGD: R->scaling = beta / kh; break;                  /* SGD.scala:38 */
    }
}

void oracle_run_set_global_parts(oracle_run *R, int32_t Kg) {
    R->Kg = Kg;
    oracle_run_set_scaling(R);
}

void oracle_run_destroy(oracle_run *R) {
    if (!R) return;
    free(R->w); free(R->alpha); free(R->alpha_old); free(R->dw); free(R->wloc);
    free(R);
}

typedef struct {
    oracle_run *R;
    int tid;
    int32_t t;
    double t0;
} worker_arg;

static void partition_update(oracle_run *R, int32_t k, int32_t t, double t0) {
    const oracle_data *D = &R->D;
    int64_t r0 = D->part_ptr[k], r1 = D->part_ptr[k + 1];
    int32_t nl = (int32_t)(r1 - r0);
    int64_t d = D->d;
    double *dw = R->dw + (size_t)k * d;
    double *wl = R->wloc + (size_t)k * d;
    const int64_t *rp = D->row_ptr + r0;
    double *al = R->alpha + r0, *ao = R->alpha_old + r0;
    int32_t seed = (int32_t)((uint32_t)R->seed + (uint32_t)t);       /* debug.seed + t */
    if (R->method == M_PLUS || R->method == M_COCOA || R->method == M_MBCD) {
        if (nl == 0) {  /* nextInt(0) throws in the reference; an empty partition contributes nothing */
            memset(dw, 0, sizeof(double) * (size_t)d);
            return;
        }
        memcpy(ao, al, sizeof(double) * (size_t)nl);                  /* alphaOld = alpha.copy */
        if (R->method == M_MBCD) {
            mbcd_local(rp, D->col, D->val, D->y + r0, nl, (int32_t)d, R->w, R->H, R->lambda, R->n, al, seed, dw);
        } else {
            int plus = R->method == M_PLUS;
            const double *wsrc = R->w;
            if (!plus) { memcpy(wl, R->w, sizeof(double) * (size_t)d); wsrc = wl; } /* task's private copy */
            oracle_local_sdca(rp, D->col, D->val, D->y + r0, nl, (int32_t)d, (double *)wsrc, R->H, R->lambda, R->n,
                              al, ao, seed, plus, (double)R->Kg * R->gamma, dw, NULL);
        }
        for (int32_t i = 0; i < nl; ++i) al[i] = ao[i] + ((al[i] - ao[i]) * R->scaling); /* CoCoA.scala:101 */
    } else {
        if (nl == 0) { memset(dw, 0, sizeof(double) * (size_t)d); return; }
        sgd_local(rp, D->col, D->val, D->y + r0, nl, (int32_t)d, R->w, R->lambda, t0, R->H,
                  R->method == M_LOCALSGD, seed, wl, dw);
    }
}

static void *worker(void *p) {
    worker_arg *a = (worker_arg *)p;
    for (int32_t k = a->tid; k < a->R->D.K; k += a->R->nthreads) partition_update(a->R, k, a->t, a->t0);
    return NULL;
}

/* One outer round t (1-based), local half: partition updates + ordered fold. */
void oracle_run_local(oracle_run *R, int32_t t, double *dw_sum) {
    const oracle_data *D = &R->D;
    int64_t d = D->d;
    double t0 = 0.0;
    if (R->method == M_MBSGD || R->method == M_LOCALSGD) {
        double step = 1 / (R->lambda * (double)t);                    /* SGD.scala:44 */
        R->sgd_step = step;
        if (R->method == M_MBSGD) {                                   /* SGD.scala:46-50 */
            double scale = 1.0 - (step * R->lambda);
            for (int64_t j = 0; j < d; ++j) R->w[j] *= scale;
        }
        /* ((t-1) * localIters * parts) in Scala Int arithmetic (SGD.scala:53) */
        int32_t ti = (int32_t)((uint32_t)(t - 1) * (uint32_t)R->H * (uint32_t)R->Kg);
        t0 = (double)ti;
    }
    int nt = R->nthreads < D->K ? R->nthreads : D->K;
    if (nt <= 1) {
        for (int32_t k = 0; k < D->K; ++k) partition_update(R, k, t, t0);
    } else {
        pthread_t th[256];
        worker_arg args[256];
        if (nt > 256) nt = 256;
        int saved = R->nthreads;
        R->nthreads = nt;
        for (int i = 0; i < nt; ++i) {
            args[i].R = R; args[i].tid = i; args[i].t = t; args[i].t0 = t0;
            pthread_create(&th[i], NULL, worker, &args[i]);
        }
        for (int i = 0; i < nt; ++i) pthread_join(th[i], NULL);
        R->nthreads = saved;
    }
    /* reduce(_ + _) in partition order (CoCoA.scala:47) */
    R->mult = R->scaling;
    if (R->method == M_MBSGD) R->mult = R->sgd_step * R->scaling;    /* SGD.scala:58 */
    for (int64_t j = 0; j < d; ++j) {
        double s = 0.0;
        int have = 0;
        for (int32_t k = 0; k < D->K; ++k) {
            if (D->part_ptr[k + 1] <= D->part_ptr[k]) continue;
            double v = R->dw[(size_t)k * d + j];
            s = have ? s + v : v;
            have = 1;
        }
        dw_sum[j] = s;
    }
    R->t_cur = t;
}

/* w += sum * scaling (CoCoA.scala:48) */
void oracle_run_apply(oracle_run *R, const double *dw_sum) {
    for (int64_t j = 0; j < R->D.d; ++j) R->w[j] += (dw_sum[j] * R->mult);
}

void oracle_run_round(oracle_run *R, int32_t t) {
    double *s = (double *)malloc(sizeof(double) * (size_t)R->D.d);
    oracle_run_local(R, t, s);
    oracle_run_apply(R, s);
    free(s);
}

/* out: [primal, dual, gap, test_err_count, train_hinge_sum, alpha_sum] */
/* P, D, gap with n = Params.n (data.count() of the whole RDD, OptUtils.scala:
 * 65-84): equal to D->n for a full problem; for one rank's share of a larger
 * problem the objectives are that share's terms over the global n. */
void oracle_run_eval(const oracle_run *R, const oracle_data *test, double *out) {
    const double n = (double)R->n;
    const double h = hinge_sum_mt(&R->D, R->w, R->nthreads);
    const double a = alpha_sum_parts(&R->D, R->alpha);
    const double nw = dense_norm2(R->w, R->D.d);
    out[0] = h / n + (0.5 * R->lambda * (nw * nw));                  /* :73-75 */
    out[1] = (-R->lambda / 2 * (nw * nw)) + (a / n);                  /* :80-84 */
    out[2] = out[0] - out[1];                                         /* :89-91 */
    out[3] = test ? (double)error_count_mt(test, R->w, R->nthreads) : -1.0;
    out[4] = h;
    out[5] = a;
}

void oracle_run_get_w(const oracle_run *R, double *out) { memcpy(out, R->w, sizeof(double) * (size_t)R->D.d); }
void oracle_run_get_alpha(const oracle_run *R, double *out) { memcpy(out, R->alpha, sizeof(double) * (size_t)R->D.n); }
void oracle_run_set_w(oracle_run *R, const double *in) { memcpy(R->w, in, sizeof(double) * (size_t)R->D.d); }
void oracle_run_set_alpha(oracle_run *R, const double *in) { memcpy(R->alpha, in, sizeof(double) * (size_t)R->D.n); }

/* the sample sequence partition k would draw in round t (for sampler parity) */
void oracle_samples(int32_t seed_plus_t, int32_t n_local, int32_t H, int32_t *out) {
    jrand_t r;
    jr_init(&r, (int64_t)seed_plus_t);
    for (int32_t i = 0; i < H; ++i) out[i] = jr_next_int_bound(&r, n_local);
}

/* precomputed Math.pow(x.norm(2), 2) per row, as localSDCA computes it */
void oracle_row_sqnorm(const oracle_data *D, double *out) {
    for (int64_t r = 0; r < D->n; ++r) {
        int64_t b = D->row_ptr[r], z = D->row_ptr[r + 1] - b;
        double nr = sp_norm2(D->val + b, z);
        out[r] = nr * nr;
    }
}

size_t oracle_sizeof_data(void) { return sizeof(oracle_data); }
