// cocoa_driver -- command-line drop-in for the reference's distopt.driver
// (hingeDriver.scala:9-115): same --key=value flags and defaults, same stdout
// lines, with the solvers running on the MI355X through libcocoa_hip.so's C ABI
// instead of Spark executors.  Extra flags: --device=<ordinal>,
// --strict=<bool> (bit-exact mode, default false).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "cocoa_capi.h"
#include "jdouble.h"

namespace {

// java.lang.Double.toString as JDK 7/8 printed it (csrc/jdouble.h)
std::string jstr(double x) { return cocoa::jdouble::to_string(x); }

struct Bad : std::runtime_error {
    using std::runtime_error::runtime_error;
};

int to_int(const std::string& s) {  // Integer.parseInt
    size_t i = 0;
    if (s.empty()) throw Bad("NumberFormatException: For input string: \"" + s + "\"");
    if (s[0] == '+' || s[0] == '-') i = 1;
    if (i == s.size()) throw Bad("NumberFormatException: For input string: \"" + s + "\"");
    for (size_t j = i; j < s.size(); ++j)
        if (s[j] < '0' || s[j] > '9') throw Bad("NumberFormatException: For input string: \"" + s + "\"");
    const long long v = std::strtoll(s.c_str(), nullptr, 10);
    if (v > 2147483647LL || v < -2147483648LL) throw Bad("NumberFormatException: For input string: \"" + s + "\"");
    return (int)v;
}

double to_double(const std::string& s) {
    char* e = nullptr;
    const double v = std::strtod(s.c_str(), &e);
    if (s.empty() || *e) throw Bad("NumberFormatException: For input string: \"" + s + "\"");
    return v;
}

bool to_bool(const std::string& s) {  // StringOps.toBoolean
    std::string l;
    for (char c : s) l += (char)std::tolower((unsigned char)c);
    if (l == "true") return true;
    if (l == "false") return false;
    throw Bad("IllegalArgumentException: For input string: \"" + s + "\"");
}

void check(int rc, const cocoa_ctx* ctx = nullptr) {
    if (rc != COCOA_OK) throw std::runtime_error(cocoa_last_error(ctx));
}

struct Printer {
    bool test;
    bool primal_dual;
};

void on_round(void* user, int32_t t, const cocoa_eval_result* ev) {
    const Printer* p = (const Printer*)user;
    std::printf("Iteration: %d\n", t);                                   // CoCoA.scala:52
    std::printf("primal objective: %s\n", jstr(ev->primal).c_str());     // CoCoA.scala:53
    if (p->primal_dual) std::printf("primal-dual gap: %s\n", jstr(ev->gap).c_str());
    if (p->test) std::printf("test error: %s\n", jstr(ev->test_error).c_str());
    std::fflush(stdout);
}

void summary(const char* alg, cocoa_ctx* ctx, bool primal_dual, bool test) {
    cocoa_eval_result ev{};
    check(cocoa_eval(ctx, &ev), ctx);                                      // OptUtils.scala:102-126
    std::string s = std::string(alg) + " has finished running. Summary Stats: ";
    s += "\n Total Objective Value: " + jstr(ev.primal);
    if (primal_dual) s += "\n Duality Gap: " + jstr(ev.gap);
    if (test) s += "\n Test Error: " + jstr(ev.test_error);
    std::printf("%s\n\n", s.c_str());
    std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    try {
        std::map<std::string, std::string> opt;                            // hingeDriver.scala:13-19
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            size_t b = 0;
            while (b < a.size() && a[b] == '-') ++b;
            a = a.substr(b);
            std::vector<std::string> parts;
            size_t st = 0;
            for (;;) {
                const size_t q = a.find('=', st);
                parts.push_back(a.substr(st, q == std::string::npos ? std::string::npos : q - st));
                if (q == std::string::npos) break;
                st = q + 1;
            }
            while (parts.size() > 1 && parts.back().empty()) parts.pop_back();  // split drops trailing ""
            if (parts.size() == 1) opt[parts[0]] = "true";
            else if (parts.size() == 2) opt[parts[0]] = parts[1];
            else throw Bad(std::string("IllegalArgumentException: Invalid argument: ") + argv[i]);
        }
        auto get = [&](const char* k, const char* dflt) { return opt.count(k) ? opt[k] : std::string(dflt); };
        const std::string master = get("master", "local[4]");
        const std::string trainFile = get("trainFile", "");
        const int numFeatures = to_int(get("numFeatures", "0"));
        const int numSplits = to_int(get("numSplits", "1"));
        const std::string chkptDir = get("chkptDir", "");
        int chkptIter = to_int(get("chkptIter", "100"));
        const std::string testFile = get("testFile", "");
        const bool justCoCoA = to_bool(get("justCoCoA", "true"));
        const double lambda = to_double(get("lambda", "0.01"));
        const int numRounds = to_int(get("numRounds", "200"));
        const double localIterFrac = to_double(get("localIterFrac", "1.0"));
        const double beta = to_double(get("beta", "1.0"));
        const double gamma = to_double(get("gamma", "1.0"));
        const int debugIter = to_int(get("debugIter", "10"));
        const int seed = to_int(get("seed", "0"));
        const int device = to_int(get("device", "0"));
        const bool strict = to_bool(get("strict", "false"));

        // hingeDriver.scala:41-48 (including its label quirk on line 47)
        std::printf("master:       %s\ntrainFile:    %s\n", master.c_str(), trainFile.c_str());
        std::printf("numFeatures:  %d\nnumSplits:    %d\n", numFeatures, numSplits);
        std::printf("chkptDir:     %s\nchkptIter     %d\n", chkptDir.c_str(), chkptIter);
        std::printf("testfile:     %s\njustCoCoA     %s\n", testFile.c_str(), justCoCoA ? "true" : "false");
        std::printf("lambda:       %s\nnumRounds:    %d\n", jstr(lambda).c_str(), numRounds);
        std::printf("localIterFrac:%s\nbeta          %s\n", jstr(localIterFrac).c_str(), jstr(beta).c_str());
        std::printf("gamma         %s\ndebugIter     %d\n", jstr(beta).c_str(), debugIter);
        std::printf("seed          %d\n", seed);
        std::fflush(stdout);
        if (chkptDir.empty()) chkptIter = numRounds + 1;                   // hingeDriver.scala:55-59

        cocoa_dataset train{}, test{};                                      // hingeDriver.scala:62-67
        check(cocoa_load_libsvm(trainFile.c_str(), numSplits, numFeatures, &train));
        const bool has_test = !testFile.empty();
        if (has_test) check(cocoa_load_libsvm(testFile.c_str(), numSplits, numFeatures, &test));
        const int n = (int)train.n_rows;
        const int K = train.num_parts;
        int localIters = (int)(localIterFrac * n / K);                       // hingeDriver.scala:70-71
        if (localIters < 1) localIters = 1;

        cocoa_ctx* ctx = nullptr;
        check(cocoa_create(device, strict ? 1 : 0, nullptr, &ctx));
        check(cocoa_set_train(ctx, K, train.part_ptr, train.row_ptr, train.col, train.val, train.y, train.n_rows,
                              numFeatures, 0, K), ctx);
        if (has_test) check(cocoa_set_test(ctx, test.row_ptr, test.col, test.val, test.y, test.n_rows), ctx);
        if (!chkptDir.empty()) check(cocoa_set_checkpoint_dir(ctx, chkptDir.c_str()), ctx);  // CoCoA.scala:58-62
        cocoa_params P{n, numRounds, localIters, 0, lambda, beta, gamma};
        cocoa_debug D{debugIter, seed, chkptIter, 0};

        struct M {
            int method;
            const char* banner;
            const char* summary;
            bool pd;
        };
        std::vector<M> ms = {{COCOA_METHOD_COCOA_PLUS, "CoCoA+", "CoCoA+", true},
                             {COCOA_METHOD_COCOA, "CoCoA", "CoCoA", true}};
        if (!justCoCoA) {
            ms.push_back({COCOA_METHOD_MBCD, "Mini-batch CD", "Mini-batch CD", true});
            ms.push_back({COCOA_METHOD_MBSGD, "SGD (with local updates = false)", "Mini-batch SGD", false});
            ms.push_back({COCOA_METHOD_LOCALSGD, "SGD (with local updates = true)", "Local SGD", false});
        }
        for (const M& m : ms) {
            std::printf("\nRunning %s on %d data examples, distributed over %d workers\n", m.banner, n, K);
            std::fflush(stdout);
            Printer pr{has_test, m.pd};
            check(cocoa_run(ctx, &P, &D, m.method, nullptr, on_round, &pr), ctx);
            summary(m.summary, ctx, m.pd, has_test);
        }
        if (!justCoCoA) {
            // DistGD (hingeDriver.scala:107-109) is outside this engine's scope; the
            // reference itself fails there (DistGD.scala:82 reads dataArr(nLocal)).
            std::printf("\nRunning DistGD on %d data examples, distributed over %d workers\n", n, K);
            std::fflush(stdout);
            std::fprintf(stderr, "DistGD is not provided by cocoa_driver (the reference throws "
                                 "ArrayIndexOutOfBoundsException in DistGD.partitionUpdate)\n");
            cocoa_destroy(ctx);
            cocoa_dataset_free(&train);
            cocoa_dataset_free(&test);
            return 1;
        }
        cocoa_destroy(ctx);
        cocoa_dataset_free(&train);
        cocoa_dataset_free(&test);
        return 0;
    } catch (const std::exception& e) {
        std::fflush(stdout);
        std::fprintf(stderr, "Exception in thread \"main\" %s\n", e.what());
        return 1;
    }
}
