// Communicator of libcocoa_hip.so (see comm.h).  RCCL is loaded with dlopen
// at first use, so the library loads (and its host-side API works) on a
// machine without RCCL or a GPU.
#include "comm.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <thread>

#include "../../include/cocoa_capi.h"
#include "common.h"

namespace cocoa {

namespace {

#define HIPCHK_C(x)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) throw Error(COCOA_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- RCCL, resolved at first use -------------------------------------------
struct Rccl {
    void* so = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*bcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*err_str)(ncclResult_t) = nullptr;
    // one process over several devices (GroupComm)
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char* n : names)
            if ((r.so = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
        if (!r.so) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.so, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(r.so, "ncclCommInitRank");
        r.destroy = (decltype(r.destroy))dlsym(r.so, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(r.so, "ncclAllReduce");
        r.send = (decltype(r.send))dlsym(r.so, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(r.so, "ncclRecv");
        r.bcast = (decltype(r.bcast))dlsym(r.so, "ncclBroadcast");
        r.err_str = (decltype(r.err_str))dlsym(r.so, "ncclGetErrorString");
        r.init_all = (decltype(r.init_all))dlsym(r.so, "ncclCommInitAll");
        r.group_start = (decltype(r.group_start))dlsym(r.so, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(r.so, "ncclGroupEnd");
    });
    if (!r.so || !r.get_unique_id || !r.init_rank || !r.all_reduce || !r.send || !r.recv || !r.bcast)
        throw Error(COCOA_E_NODEV, "RCCL (librccl.so) is not available");
    return r;
}

void nccl_check(ncclResult_t rc, const char* what) {
    if (rc != ncclSuccess)
        throw Error(COCOA_E_IO, std::string(what) + ": " + (rccl().err_str ? rccl().err_str(rc) : "RCCL error"));
}

// ---- HOST transport: uid and listening sockets -----------------------------
constexpr char kHostMagic[8] = {'C', 'O', 'C', 'O', 'A', 'H', 'S', 'T'};

struct HostUid {
    char magic[8];
    uint32_t addr;   // network order
    uint16_t port;   // network order
    uint16_t pad;
    uint64_t nonce;
};
static_assert(sizeof(HostUid) <= (size_t)kUidBytes, "uid layout");

std::mutex g_listen_mu;
std::map<uint64_t, int> g_listen;  // nonce -> listening socket of this process

// Connect / handshake timeout (COCOA_COMM_TIMEOUT_MS, default 120 s).
int timeout_ms() {
    const char* e = std::getenv("COCOA_COMM_TIMEOUT_MS");
    return e ? std::atoi(e) : 120000;
}
// Exchange timeout (COCOA_COMM_EXCHANGE_TIMEOUT_MS, default 30 min; 0 = none):
// a round's recv also waits for the other ranks' work -- the strict chain,
// rank 0's relay, ranks that finish set_train / the compact layout at
// different times -- which on C4-sized data can outlast any handshake-sized
// limit, but a rank that hangs without closing its socket (a wedged GPU, a
// stuck host) must still end the others with an error instead of blocking them
// forever.
int exchange_timeout_ms() {
    const char* e = std::getenv("COCOA_COMM_EXCHANGE_TIMEOUT_MS");
    return e ? std::atoi(e) : 30 * 60 * 1000;
}

timeval to_timeval(int ms) {
    timeval tv{};
    if (ms > 0) {
        tv.tv_sec = ms / 1000;
        tv.tv_usec = (ms % 1000) * 1000;
    }
    return tv;  // {0, 0}: no timeout
}

void set_sock_timeout(int fd, int ms) {
    const timeval tv = to_timeval(ms);
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}

void set_sock_opts(int fd) {
    const int one = 1;
    (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    set_sock_timeout(fd, timeout_ms());  // the handshake; exchange_timeout_ms() once connected
}

}  // namespace

void comm_unique_id(int transport, void* uid) {
    std::memset(uid, 0, kUidBytes);
    if (transport == kTransportRccl) {
        ncclUniqueId id;
        nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId");
        std::memcpy(uid, &id, kUidBytes);
        return;
    }
    if (transport != kTransportHost) throw Error(COCOA_E_ARG, "unknown transport");
    const char* a = std::getenv("COCOA_COMM_ADDR");  // host address the other ranks reach rank 0 at
    in_addr addr{};
    if (inet_pton(AF_INET, a ? a : "127.0.0.1", &addr) != 1) throw Error(COCOA_E_ARG, "bad COCOA_COMM_ADDR");
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw Error(COCOA_E_IO, std::string("socket: ") + std::strerror(errno));
    const int one = 1;
    (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_addr = addr;
    sa.sin_port = 0;
    socklen_t len = sizeof sa;
    if (bind(fd, (sockaddr*)&sa, sizeof sa) != 0 || listen(fd, 256) != 0 || getsockname(fd, (sockaddr*)&sa, &len) != 0) {
        const std::string m = std::strerror(errno);
        close(fd);
        throw Error(COCOA_E_IO, "cannot listen for ranks: " + m);
    }
    HostUid u{};
    std::memcpy(u.magic, kHostMagic, 8);
    u.addr = addr.s_addr;
    u.port = sa.sin_port;
    std::random_device rd;
    u.nonce = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid();
    {
        std::lock_guard<std::mutex> lk(g_listen_mu);
        g_listen[u.nonce] = fd;
    }
    std::memcpy(uid, &u, sizeof u);
}

Comm* comm_create(int transport, int rank, int world, const void* uid, int device) {
    if (world < 1 || rank < 0 || rank >= world || !uid) throw Error(COCOA_E_ARG, "cocoa_comm: bad rank / world / uid");
    Comm* c = new Comm();
    c->transport = transport;
    c->rank = rank;
    c->world = world;
    c->device = device;
    try {
        if (transport == kTransportRccl) {
            if (device < 0) throw Error(COCOA_E_ARG, "the RCCL transport needs a device");
            HIPCHK_C(hipSetDevice(device));
            ncclUniqueId id;
            std::memcpy(&id, uid, kUidBytes);
            ncclComm_t nc = nullptr;
            nccl_check(rccl().init_rank(&nc, world, id, rank), "ncclCommInitRank");
            c->nccl = nc;
        } else if (transport == kTransportHost) {
            HostUid u;
            std::memcpy(&u, uid, sizeof u);
            if (std::memcmp(u.magic, kHostMagic, 8) != 0) throw Error(COCOA_E_ARG, "not a HOST-transport uid");
            if (rank == 0) {
                int lfd = -1;
                {
                    std::lock_guard<std::mutex> lk(g_listen_mu);
                    auto it = g_listen.find(u.nonce);
                    if (it != g_listen.end()) {
                        lfd = it->second;
                        g_listen.erase(it);
                    }
                }
                if (lfd < 0) throw Error(COCOA_E_ARG, "rank 0 must create the HOST uid (cocoa_comm_unique_id)");
                c->fds.assign((size_t)world, -1);
                const timeval tv = to_timeval(timeout_ms());
                (void)setsockopt(lfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
                for (int got = 1; got < world; ++got) {
                    const int fd = accept(lfd, nullptr, nullptr);
                    if (fd < 0) {
                        close(lfd);
                        throw Error(COCOA_E_IO, std::string("accept: ") + std::strerror(errno));
                    }
                    set_sock_opts(fd);
                    int32_t hello[3] = {0, 0, 0};  // rank, nonce (2 halves)
                    size_t off = 0;
                    while (off < sizeof hello) {
                        const ssize_t k = recv(fd, (char*)hello + off, sizeof hello - off, 0);
                        if (k <= 0) break;
                        off += (size_t)k;
                    }
                    const uint64_t nn = ((uint64_t)(uint32_t)hello[2] << 32) | (uint32_t)hello[1];
                    if (off != sizeof hello || nn != u.nonce || hello[0] < 1 || hello[0] >= world ||
                        c->fds[(size_t)hello[0]] >= 0) {
                        close(fd);
                        close(lfd);
                        throw Error(COCOA_E_IO, "bad rank handshake");
                    }
                    c->fds[(size_t)hello[0]] = fd;
                }
                close(lfd);
                for (int fd : c->fds)
                    if (fd >= 0) set_sock_timeout(fd, exchange_timeout_ms());
            } else {
                sockaddr_in sa{};
                sa.sin_family = AF_INET;
                sa.sin_addr.s_addr = u.addr;
                sa.sin_port = u.port;
                const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms());
                int fd = -1;
                for (;;) {
                    fd = socket(AF_INET, SOCK_STREAM, 0);
                    if (fd >= 0 && connect(fd, (sockaddr*)&sa, sizeof sa) == 0) break;
                    if (fd >= 0) close(fd);
                    fd = -1;
                    if (std::chrono::steady_clock::now() > t_end) throw Error(COCOA_E_IO, "cannot reach rank 0");
                    std::this_thread::sleep_for(std::chrono::milliseconds(20));
                }
                set_sock_opts(fd);
                const int32_t hello[3] = {rank, (int32_t)(uint32_t)u.nonce, (int32_t)(uint32_t)(u.nonce >> 32)};
                c->fds.assign(1, fd);
                c->host_send(fd, hello, sizeof hello);
                set_sock_timeout(fd, exchange_timeout_ms());
            }
        } else {
            throw Error(COCOA_E_ARG, "unknown transport");
        }
    } catch (...) {
        delete c;
        throw;
    }
    return c;
}

Comm::~Comm() {
    if (nccl && rccl().destroy) (void)rccl().destroy((ncclComm_t)nccl);
    for (int fd : fds)
        if (fd >= 0) close(fd);
    if (dev_scratch) (void)hipFree(dev_scratch);
}

void Comm::host_send(int fd, const void* p, size_t bytes) {
    const char* b = (const char*)p;
    while (bytes) {
        const ssize_t k = send(fd, b, bytes, MSG_NOSIGNAL);
        if (k <= 0) throw Error(COCOA_E_IO, std::string("rank exchange send: ") + std::strerror(errno));
        b += k;
        bytes -= (size_t)k;
    }
}

void Comm::host_recv(int fd, void* p, size_t bytes) {
    char* b = (char*)p;
    while (bytes) {
        const ssize_t k = recv(fd, b, bytes, 0);
        if (k <= 0) {
            const bool to = k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK);
            throw Error(COCOA_E_IO, std::string("rank exchange recv: ") +
                                        (k == 0 ? "peer closed"
                                         : to ? "timed out waiting for another rank (COCOA_COMM_EXCHANGE_TIMEOUT_MS, "
                                                "default 1800000 = 30 min, 0 = no limit, raises it)"
                                              : std::strerror(errno)));
        }
        b += k;
        bytes -= (size_t)k;
    }
}

double* Comm::scratch(int64_t n) {
    if ((size_t)n > dev_scratch_n) {
        if (dev_scratch) HIPCHK_C(hipFree(dev_scratch));
        dev_scratch = nullptr;
        HIPCHK_C(hipMalloc(&dev_scratch, sizeof(double) * (size_t)n));
        dev_scratch_n = (size_t)n;
    }
    return dev_scratch;
}

// HOST transport works on host memory; device buffers are staged on `s`.
// RCCL works on device memory; host buffers are staged through dev_scratch.

void Comm::allreduce(double* buf, int64_t n, bool device, hipStream_t s) {
    if (world == 1 && transport == kTransportHost) return;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (transport == kTransportRccl) {
        double* d = buf;
        if (!device) {
            d = scratch(n);
            HIPCHK_C(hipMemcpyAsync(d, buf, bytes, hipMemcpyHostToDevice, s));
        }
        nccl_check(rccl().all_reduce(d, d, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)nccl, s), "ncclAllReduce");
        if (!device) {
            HIPCHK_C(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, s));
            HIPCHK_C(hipStreamSynchronize(s));
        }
        return;
    }
    std::vector<double> mine;
    double* h = buf;
    if (device) {
        mine.resize((size_t)n);
        h = mine.data();
        HIPCHK_C(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
        HIPCHK_C(hipStreamSynchronize(s));
    }
    if (rank == 0) {
        // ((x_0 + x_1) + x_2) + ... in rank order, then the total to everyone
        host.resize((size_t)n);
        for (int r = 1; r < world; ++r) {
            host_recv(fds[(size_t)r], host.data(), bytes);
            for (int64_t i = 0; i < n; ++i) h[i] = h[i] + host[(size_t)i];
        }
        for (int r = 1; r < world; ++r) host_send(fds[(size_t)r], h, bytes);
    } else {
        host_send(fds[0], h, bytes);
        host_recv(fds[0], h, bytes);
    }
    if (device) HIPCHK_C(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
    if (device) HIPCHK_C(hipStreamSynchronize(s));
}

void Comm::chain_recv(double* buf, int64_t n, bool device, hipStream_t s) {
    if (rank == 0) return;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (transport == kTransportRccl) {
        double* d = device ? buf : scratch(n);
        nccl_check(rccl().recv(d, (size_t)n, ncclFloat64, rank - 1, (ncclComm_t)nccl, s), "ncclRecv");
        if (!device) {
            HIPCHK_C(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, s));
            HIPCHK_C(hipStreamSynchronize(s));
        }
        return;
    }
    // the fold of ranks < rank arrives from rank 0 (which relays it)
    if (device) {
        host.resize((size_t)n);
        host_recv(fds[0], host.data(), bytes);
        HIPCHK_C(hipMemcpyAsync(buf, host.data(), bytes, hipMemcpyHostToDevice, s));
        HIPCHK_C(hipStreamSynchronize(s));
    } else {
        host_recv(fds[0], buf, bytes);
    }
}

void Comm::chain_send(const double* buf, int64_t n, bool device, hipStream_t s) {
    if (rank == world - 1) return;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (transport == kTransportRccl) {
        const double* d = buf;
        if (!device) {
            double* t = scratch(n);
            HIPCHK_C(hipMemcpyAsync(t, buf, bytes, hipMemcpyHostToDevice, s));
            d = t;
        }
        nccl_check(rccl().send(d, (size_t)n, ncclFloat64, rank + 1, (ncclComm_t)nccl, s), "ncclSend");
        if (!device) HIPCHK_C(hipStreamSynchronize(s));
        return;
    }
    const double* h = buf;
    std::vector<double> tmp;
    if (device) {
        tmp.resize((size_t)n);
        HIPCHK_C(hipMemcpyAsync(tmp.data(), buf, bytes, hipMemcpyDeviceToHost, s));
        HIPCHK_C(hipStreamSynchronize(s));
        h = tmp.data();
    }
    host_send(rank == 0 ? fds[1] : fds[0], h, bytes);  // rank 0 -> rank 1 directly; later hops via rank 0
}

void Comm::bcast_last(double* buf, int64_t n, bool device, hipStream_t s) {
    if (world == 1) return;
    const size_t bytes = sizeof(double) * (size_t)n;
    const int last = world - 1;
    if (transport == kTransportRccl) {
        double* d = buf;
        if (!device) {
            d = scratch(n);
            HIPCHK_C(hipMemcpyAsync(d, buf, bytes, hipMemcpyHostToDevice, s));
        }
        nccl_check(rccl().bcast(d, d, (size_t)n, ncclFloat64, last, (ncclComm_t)nccl, s), "ncclBroadcast");
        if (!device) {
            HIPCHK_C(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, s));
            HIPCHK_C(hipStreamSynchronize(s));
        }
        return;
    }
    std::vector<double> tmp;
    double* h = buf;
    if (device) {
        tmp.resize((size_t)n);
        h = tmp.data();
        if (rank == last) {
            HIPCHK_C(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
            HIPCHK_C(hipStreamSynchronize(s));
        }
    }
    if (rank == 0) {
        // relay the chain hops 1 -> 2 -> ... -> last, then fan the total out
        std::vector<double> hop((size_t)n);
        for (int r = 1; r < last; ++r) {
            host_recv(fds[(size_t)r], hop.data(), bytes);
            host_send(fds[(size_t)r + 1], hop.data(), bytes);
        }
        host_recv(fds[(size_t)last], h, bytes);
        for (int r = 1; r < last; ++r) host_send(fds[(size_t)r], h, bytes);
    } else if (rank == last) {
        host_send(fds[0], h, bytes);
    } else {
        host_recv(fds[0], h, bytes);
    }
    if (device && rank != last) {
        HIPCHK_C(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
        HIPCHK_C(hipStreamSynchronize(s));
    }
}

// ---- one process, several devices -------------------------------------------
GroupComm* group_comm_create(const std::vector<int>& devices) {
    Rccl& r = rccl();
    if (!r.init_all || !r.group_start || !r.group_end || !r.destroy)
        throw Error(COCOA_E_NODEV, "RCCL (librccl.so) has no ncclCommInitAll / ncclGroupStart");
    GroupComm* g = new GroupComm();
    g->comms.assign(devices.size(), nullptr);
    const ncclResult_t rc = r.init_all((ncclComm_t*)g->comms.data(), (int)devices.size(), devices.data());
    if (rc != ncclSuccess) {
        delete g;
        nccl_check(rc, "ncclCommInitAll");
    }
    return g;
}

GroupComm::~GroupComm() {
    for (void* c : comms)
        if (c && rccl().destroy) (void)rccl().destroy((ncclComm_t)c);
}

void GroupComm::allreduce(const std::vector<double*>& bufs, int64_t n, const std::vector<hipStream_t>& streams) {
    Rccl& r = rccl();
    nccl_check(r.group_start(), "ncclGroupStart");
    for (size_t i = 0; i < comms.size(); ++i)
        nccl_check(r.all_reduce(bufs[i], bufs[i], (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)comms[i], streams[i]),
                   "ncclAllReduce");
    nccl_check(r.group_end(), "ncclGroupEnd");
}

}  // namespace cocoa
