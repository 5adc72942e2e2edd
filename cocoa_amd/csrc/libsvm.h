// Host-side LIBSVM helpers shared by the CPU loader (dataset.cpp) and the
// GPU ingest (ingest.hip): OptUtils.loadLIBSVMData (OptUtils.scala:11-53).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/cocoa_capi.h"

namespace cocoa {

// Hadoop 1.0.4 FileInputFormat.getSplits: byte offset of every split of a file
std::vector<int64_t> hadoop_split_starts(int64_t size, int num_splits);

// Partition of a line from its first byte: the split holding it, then
// CoalescedRDD's consecutive ranges when there are more splits than K.
// Lines must be visited in file order.
struct LinePartitioner {
    const std::vector<int64_t>& starts;
    int ns, K, split = 0;
    LinePartitioner(const std::vector<int64_t>& s, int k) : starts(s), ns((int)s.size()), K(k) {}
    int part(int64_t p) {
        while (split + 1 < ns && p >= starts[(size_t)split + 1]) ++split;
        if (ns <= K) return split;
        int q = 0;
        while (q + 1 < K && (int64_t)split >= ((int64_t)(q + 1) * ns) / K) ++q;
        return q;
    }
};

// One line [b, le) of the file (without its newline), line number r (0-based):
// label, entries and count, or the reference's exception kind with a message.
int libsvm_parse_line(const char* b, const char* le, int64_t r, int32_t num_features, double* y, int32_t* col,
                      double* val, int64_t* z, std::string* msg);
bool dataset_alloc(cocoa_dataset* ds, int64_t n, int64_t nnz, int32_t K);
int host_error(int code, const std::string& msg);

}  // namespace cocoa
