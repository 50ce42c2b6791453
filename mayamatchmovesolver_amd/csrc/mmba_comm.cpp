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
#include <mutex>

#include "mmba_plan.h"

namespace mmba {

// ---- RCCL ----
struct RcclComm : Comm {
    ncclComm_t c = nullptr;
    bool aborted = false;
    ~RcclComm() override {
        if (c && !aborted) (void)ncclCommDestroy(c);
    }
    void abort() override {
        if (c && !aborted) (void)ncclCommAbort(c);
        aborted = true;
    }
    void check(ncclResult_t r, const char *what) {
        if (r != ncclSuccess) {
            set_error(std::string(what) + ": " + ncclGetErrorString(r));
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
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) throw CommError();
        const long g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || aborted; });
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
    const ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
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
