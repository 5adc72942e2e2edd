// Rank-to-rank exchange of the per-round deltaW sum and the objective scalars
// (CoCoA.scala:45-48: `updates.map(_._1).reduce(_ + _)` then `w += ...`;
// OptUtils.scala:65-98: the scalar reduces of the evaluation).  One process
// per GPU; the communicator belongs to the engine context (or stands alone
// for host buffers).
//
// Transports:
//   RCCL -- librccl (loaded at first use) over xGMI: ncclAllReduce for the
//           fast-mode sum, ncclSend/ncclRecv/ncclBroadcast for the ordered
//           chain of strict mode.  One GPU per rank (RCCL refuses two ranks
//           on one device).
//   HOST -- TCP (loopback or the host network), star around rank 0, buffers
//           staged through host memory.  For ranks that share a GPU (tests
//           on a one-GPU box) and for CPU-only use of the communicator.
//
// Two reductions:
//   allreduce   -- sum with a fixed association, identical bytes on every
//                  rank (fast mode);
//   chain       -- rank r receives the running left fold of ranks < r,
//                  continues it over its own partitions and passes it on;
//                  the last rank broadcasts the total.  This keeps the
//                  single-process partition-order fold ((dW_0 + dW_1) + ...)
//                  exactly, so strict mode stays bitwise across ranks.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

namespace cocoa {

constexpr int kTransportRccl = 0;
constexpr int kTransportHost = 1;
constexpr int kUidBytes = 128;

struct Comm {
    int transport = kTransportRccl;
    int rank = 0, world = 1, device = -1;
    void* nccl = nullptr;          // ncclComm_t
    std::vector<int> fds;          // HOST: root: fds[r] (r >= 1) = socket of rank r; others: fds[0] = root
    std::vector<double> host;      // HOST: staging / receive buffer
    double* dev_scratch = nullptr; // RCCL: staging for host buffers
    size_t dev_scratch_n = 0;

    ~Comm();
    // in-place sum over ranks of n doubles (device memory on `s` when device)
    void allreduce(double* buf, int64_t n, bool device, hipStream_t s);
    // ordered chain: receive the fold of ranks < rank (rank > 0) / send ours on
    void chain_recv(double* buf, int64_t n, bool device, hipStream_t s);
    void chain_send(const double* buf, int64_t n, bool device, hipStream_t s);
    // every rank gets the last rank's buffer
    void bcast_last(double* buf, int64_t n, bool device, hipStream_t s);

    // internals (also used by comm_create)
    void host_send(int fd, const void* p, size_t bytes);
    void host_recv(int fd, void* p, size_t bytes);
    double* scratch(int64_t n);
};

// One process driving several distinct devices (cocoa_create_multi): one RCCL
// communicator per device from ncclCommInitAll, and the per-round deltaW sum
// as one ncclAllReduce per device inside ncclGroupStart / ncclGroupEnd, each
// on its device's stream behind that device's fold.  RCCL reduce-scatters then
// all-gathers, so every device holds the same bytes.
struct GroupComm {
    std::vector<void*> comms;  // ncclComm_t per device, in member order
    ~GroupComm();
    void allreduce(const std::vector<double*>& bufs, int64_t n, const std::vector<hipStream_t>& streams);
};
GroupComm* group_comm_create(const std::vector<int>& devices);

// uid for `transport` (128 bytes); HOST opens the listening socket in this
// process, so rank 0 must create it.
void comm_unique_id(int transport, void* uid);
Comm* comm_create(int transport, int rank, int world, const void* uid, int device);

}  // namespace cocoa
