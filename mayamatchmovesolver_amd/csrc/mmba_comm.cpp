// mmba_comm.cpp -- communicators of the frame-sharded solve (one process or
// thread per shard).  Every collective is an in-place all-reduce of a device
// buffer on the plan's stream:
//   RcclComm   RCCL over xGMI, one process per GPU (torch.distributed.run);
//   LocalComm  N shards driven by N host threads in one process (tests on a
//              one-GPU box run the sharded code path against the unsharded
//              one): every shard sums all shards' buffers in rank order, so
//              all shards get bitwise identical results; MMBA_PATH_LOCAL_RING
//              = 1 at creation (mmba_debug_set_path) sums in ring order instead -- the order of a ring
//              reduce-scatter (RCCL's ring all-reduce): the buffer is cut into
//              N chunks and chunk c is accumulated starting at rank c + 1 and
//              ending at rank c (mod N), so the sharded tests also see a
//              summation order other than rank order.
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mmba_plan.h"

namespace mmba {

// ---- bounded waits ----
int comm_timeout_ms() {
    const int p = path_choice(MMBA_PATH_COMM_TIMEOUT_MS);
    if (p > 0) return p;
    if (const char *e = std::getenv("MMBA_COMM_TIMEOUT_MS")) {
        const int v = std::atoi(e);
        if (v > 0) return v;
    }
    return 120000;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void comm_wait(Comm *c, hipStream_t s, hipEvent_t ev) {
    if (!c || !c->bounded()) {
        if (ev)
            MMBA_HIP(hipEventSynchronize(ev));
        else
            MMBA_HIP(hipStreamSynchronize(s));
        return;
    }
    const double t_end = now_ms() + comm_timeout_ms();
    for (unsigned spins = 0;; ++spins) {
        const hipError_t e = ev ? hipEventQuery(ev) : hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) MMBA_HIP(e);
        if ((spins & 255u) == 255u) {
            c->poll_async();  // throws on a communicator error
            if (now_ms() > t_end) {
                c->abort();
                set_error("collective timed out after " + std::to_string(comm_timeout_ms()) +
                          " ms (communicator aborted; another rank never joined)");
                throw CommError();
            }
            if (spins > 65536u) std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
}

// ---- RCCL ----
// Communicators are created non-blocking (ncclConfig_t::blocking = 0): the
// initialisation and every collective return at once (ncclInProgress while
// the communicator works) and the library polls ncclCommGetAsyncError with
// the same deadline as comm_wait, so a rank that never joins costs the others
// MMBA_ERR_COMM after comm_timeout_ms(), never a hang.
static void rccl_settle(ncclComm_t c, const char *what) {
    const double t_end = now_ms() + comm_timeout_ms();
    for (unsigned spins = 0;; ++spins) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(c, &st);
        if (r != ncclSuccess) st = r;
        if (st == ncclSuccess) return;
        if (st != ncclInProgress) {
            set_error(std::string(what) + ": " + ncclGetErrorString(st));
            throw CommError();
        }
        if (now_ms() > t_end) {
            set_error(std::string(what) + ": timed out after " +
                      std::to_string(comm_timeout_ms()) + " ms");
            throw CommError();
        }
        if (spins > 1024u) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

struct RcclComm : Comm {
    ncclComm_t c = nullptr;
    bool aborted = false;
    ~RcclComm() override {
        if (!c || aborted) return;
        // non-blocking communicator: finalize (flushes issued operations,
        // ncclInProgress until done), settled with the deadline, then free;
        // a communicator that does not settle is aborted instead
        const ncclResult_t r = ncclCommFinalize(c);
        bool ok = r == ncclSuccess || r == ncclInProgress;
        if (ok) {
            try {
                rccl_settle(c, "ncclCommFinalize");
            } catch (const CommError &) {
                ok = false;
            }
        }
        if (ok)
            (void)ncclCommDestroy(c);
        else
            (void)ncclCommAbort(c);
    }
    void abort() override {
        if (c && !aborted) (void)ncclCommAbort(c);
        aborted = true;
    }
    bool bounded() const override { return true; }
    void poll_async() override {
        if (aborted) throw CommError();
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess ||
            (st != ncclSuccess && st != ncclInProgress)) {
            set_error(std::string("RCCL asynchronous error: ") + ncclGetErrorString(st));
            abort();
            throw CommError();
        }
    }
    int count() const override {
        int n = 0;
        if (c && !aborted && ncclCommCount(c, &n) == ncclSuccess) return n;
        return nranks;
    }
    void check(ncclResult_t r, const char *what) {
        if (r == ncclInProgress) {
            try {
                rccl_settle(c, what);
            } catch (const CommError &) {
                abort();
                throw;
            }
            return;
        }
        if (r != ncclSuccess) {
            set_error(std::string(what) + ": " + ncclGetErrorString(r));
            abort();
            throw CommError();
        }
    }
    void allgather(const double *send, double *recv, size_t count, hipStream_t s) override {
        if (count == 0) return;
        if (aborted) throw CommError();
        check(ncclAllGather(send, recv, count, ncclDouble, c, s), "ncclAllGather");
    }
    void allreduce(double *buf, size_t count, ReduceOp op, hipStream_t s) override {
        if (count == 0) return;
        if (aborted) throw CommError();
        check(ncclAllReduce(buf, buf, count, ncclDouble, op == ReduceOp::Max ? ncclMax : ncclSum,
                            c, s),
              "ncclAllReduce");
    }
};

Comm *make_rccl_comm(ncclComm_t c, int rank, int nranks);

// One communicator per device of this process (the multi-device context):
// ncclCommInitRankConfig per device inside one group, non-blocking, settled
// with a deadline -- ncclCommInitAll's blocking form could hang the caller.
int rccl_init_all(const int *devices, int n, std::vector<Comm *> &out) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
        return MMBA_ERR_COMM;
    }
    std::vector<ncclComm_t> nc(n, nullptr);
    int cur = 0;
    (void)hipGetDevice(&cur);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    r = ncclGroupStart();
    for (int k = 0; k < n && (r == ncclSuccess || r == ncclInProgress); ++k) {
        if (hipSetDevice(devices[k]) != hipSuccess) {
            r = ncclUnhandledCudaError;
            break;
        }
        r = ncclCommInitRankConfig(&nc[k], n, id, k, &cfg);
    }
    const ncclResult_t re = ncclGroupEnd();
    (void)hipSetDevice(cur);
    bool ok = (r == ncclSuccess || r == ncclInProgress) &&
              (re == ncclSuccess || re == ncclInProgress);
    if (!ok) set_error(std::string("RCCL communicator group init: ") +
                       ncclGetErrorString(r != ncclSuccess && r != ncclInProgress ? r : re));
    for (int k = 0; k < n && ok; ++k) {
        try {
            if (!nc[k]) throw CommError();
            rccl_settle(nc[k], "RCCL communicator group init");
        } catch (const CommError &) {
            ok = false;
        }
    }
    if (!ok) {
        for (ncclComm_t c : nc)
            if (c) (void)ncclCommAbort(c);
        return MMBA_ERR_COMM;
    }
    for (int k = 0; k < n; ++k) out.push_back(make_rccl_comm(nc[k], k, n));
    return MMBA_OK;
}

Comm *make_rccl_comm(ncclComm_t c, int rank, int nranks) {
    auto *r = new RcclComm();
    r->c = c;
    r->rank = rank;
    r->nranks = nranks;
    return r;
}

// ---- in-process group ----
constexpr int LOCAL_MAX = 8;

struct LocalGroup {
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    bool ring = false;
    bool aborted = false;
    double *bufs[LOCAL_MAX] = {};
    const double *sends[LOCAL_MAX] = {};
    // bounded like RCCL's waits: a shard that never arrives aborts the group
    // after comm_timeout_ms() (every waiter, and the late shard when it
    // arrives, gets CommError)
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) throw CommError();
        const long g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            const bool done = cv.wait_for(lk, std::chrono::milliseconds(comm_timeout_ms()),
                                          [&] { return gen != g || aborted; });
            if (!done) {
                aborted = true;
                cv.notify_all();
                set_error("in-process shard group: collective timed out after " +
                          std::to_string(comm_timeout_ms()) + " ms (group aborted)");
                throw CommError();
            }
            if (gen == g) {
                set_error("in-process shard group aborted (another shard failed)");
                throw CommError();
            }
        }
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

struct BufSet {
    const double *p[LOCAL_MAX];
};

__global__ void k_group_reduce(BufSet b, int n, size_t count, int max_op, int ring, double *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        // ring: chunk c = floor(i n / count) starts at rank c + 1
        const int r0 = ring ? (int)((i * (size_t)n / count + 1) % n) : 0;
        double s = b.p[r0][i];
        for (int k = 1; k < n; ++k) {
            const double v = b.p[(r0 + k) % n][i];
            s = max_op ? fmax(s, v) : s + v;
        }
        out[i] = s;
    }
}

struct LocalComm : Comm {
    std::shared_ptr<LocalGroup> g;
    double *tmp = nullptr;
    size_t tmp_count = 0;
    ~LocalComm() override {
        if (tmp) (void)hipFree(tmp);
    }
    void allreduce(double *buf, size_t count, ReduceOp op, hipStream_t s) override {
        if (count == 0) return;
        if (count > tmp_count) {
            if (tmp) MMBA_HIP(hipFree(tmp));
            MMBA_HIP(hipMalloc(&tmp, count * sizeof(double)));
            tmp_count = count;
        }
        MMBA_HIP(hipStreamSynchronize(s));
        g->bufs[rank] = buf;
        g->barrier();  // every shard's buffer is final
        BufSet b{};
        for (int k = 0; k < g->n; ++k) b.p[k] = g->bufs[k];
        const int blocks = (int)std::min<size_t>((count + 255) / 256, 1024);
        k_group_reduce<<<blocks, 256, 0, s>>>(b, g->n, count, op == ReduceOp::Max,
                                              g->ring ? 1 : 0, tmp);
        MMBA_HIP(hipStreamSynchronize(s));
        g->barrier();  // nobody reads a shard's buffer any more
        MMBA_HIP(hipMemcpyAsync(buf, tmp, count * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    void allgather(const double *send, double *recv, size_t count, hipStream_t s) override {
        if (count == 0) return;
        MMBA_HIP(hipStreamSynchronize(s));
        g->sends[rank] = send;
        g->barrier();  // every shard's send buffer is final
        for (int k = 0; k < g->n; ++k)
            MMBA_HIP(hipMemcpyAsync(recv + (size_t)k * count, g->sends[k], count * sizeof(double),
                                    hipMemcpyDeviceToDevice, s));
        MMBA_HIP(hipStreamSynchronize(s));
        g->barrier();  // nobody reads a shard's send buffer any more
    }
    void abort() override { g->abort(); }
};

}  // namespace mmba

using namespace mmba;

extern "C" {

int mmba_comm_unique_id(unsigned char out_id[128]) {
    if (!out_id) return MMBA_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
        return MMBA_ERR_COMM;
    }
    std::memcpy(out_id, &id, 128);
    return MMBA_OK;
}

int mmba_comm_create_rccl(mmba_context *ctx, int rank, int nranks,
                          const unsigned char unique_id[128], mmba_comm **out) {
    if (!ctx || !unique_id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return MMBA_ERR_INVALID;
    *out = nullptr;
    if (!ctx->shards.empty()) {
        set_error("a multi-device context brings its own communicators");
        return MMBA_ERR_INVALID;
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return MMBA_ERR_DEVICE;
    auto *c = new RcclComm();
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, 128);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // bounded: rccl_settle polls with a deadline
    const ncclResult_t r = ncclCommInitRankConfig(&c->c, nranks, id, rank, &cfg);
    bool ok = r == ncclSuccess || r == ncclInProgress;
    if (!ok) set_error(std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
    if (ok && c->c) {
        try {
            rccl_settle(c->c, "ncclCommInitRankConfig");
        } catch (const CommError &) {
            ok = false;
        }
    }
    if (!ok) {
        if (c->c) (void)ncclCommAbort(c->c);
        c->c = nullptr;
        delete c;
        return MMBA_ERR_COMM;
    }
    *out = reinterpret_cast<mmba_comm *>(static_cast<Comm *>(c));
    return MMBA_OK;
}

int mmba_comm_create_local(int nranks, mmba_comm **out) {
    if (!out || nranks < 1 || nranks > LOCAL_MAX) return MMBA_ERR_INVALID;
    auto g = std::make_shared<LocalGroup>();
    g->n = nranks;
    g->ring = path_choice(MMBA_PATH_LOCAL_RING) > 0;
    for (int r = 0; r < nranks; ++r) {
        auto *c = new LocalComm();
        c->rank = r;
        c->nranks = nranks;
        c->g = g;
        out[r] = reinterpret_cast<mmba_comm *>(static_cast<Comm *>(c));
    }
    return MMBA_OK;
}

int mmba_comm_count(const mmba_comm *comm) {
    if (!comm) return MMBA_ERR_INVALID;
    return reinterpret_cast<const Comm *>(comm)->count();
}

void mmba_comm_destroy(mmba_comm *comm) {
    delete reinterpret_cast<Comm *>(comm);
}

int mmba_debug_comm_allreduce(mmba_context *ctx, mmba_comm *comm, double *buf, int count,
                              int op) {
    if (!ctx || !comm || !buf || count < 0 || op < 0 || op > 1) return MMBA_ERR_INVALID;
    if (hipSetDevice(ctx->device) != hipSuccess) return MMBA_ERR_DEVICE;
    double *d = nullptr;
    int rc = MMBA_OK;
    try {
        MMBA_HIP(hipMalloc(&d, sizeof(double) * (size_t)std::max(count, 1)));
        MMBA_HIP(hipMemcpyAsync(d, buf, sizeof(double) * (size_t)count, hipMemcpyHostToDevice,
                                ctx->stream));
        reinterpret_cast<Comm *>(comm)->allreduce(d, (size_t)count,
                                                  op ? ReduceOp::Max : ReduceOp::Sum, ctx->stream);
        MMBA_HIP(hipMemcpyAsync(buf, d, sizeof(double) * (size_t)count, hipMemcpyDeviceToHost,
                                ctx->stream));
        MMBA_HIP(hipStreamSynchronize(ctx->stream));
    } catch (const CommError &) {
        rc = MMBA_ERR_COMM;
    } catch (const DeviceError &) {
        rc = MMBA_ERR_DEVICE;
    }
    if (d) (void)hipFree(d);
    return rc;
}

}  // extern "C"
