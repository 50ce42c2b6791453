// mmba_group.cpp -- one caller, several devices (mmba.h ABI 9), and the
// hand-back of a sharded solve's results without a full-size collective.
//
// The reference calls solveFrames once, on Maya's main thread
// (src/mmSolver/adjust/adjust_base.cpp:1174-1183); SURVEY 8(b) "Threading":
// multi-GPU fan-out stays inside the library.  mmba_context_create_multi
// makes one context (own stream) per device plus the group's communicators:
//   - distinct devices: RCCL, one communicator per device in this process
//     (non-blocking ncclCommInitRankConfig in one group, settled with a
//     deadline: rccl_init_all), each driven by its own host thread;
//   - one device named N times: the in-process transport (LocalComm), so a
//     one-GPU box runs the N-shard path through the same entry.
// mmba_plan_create over such a context builds one sharded plan per device
// (the frame partition of mmba_plan_create_sharded), and every plan entry
// point runs the N shards together: shard 0 on the caller's thread, the
// others on the group's persistent threads.  The shards' LM control flows
// stay identical through their collectives; interrupt polls are answered by
// shard 0 (PollShare); x and the per-residual outputs go straight into the
// caller's host buffers, each shard writing its own parameters and its own
// observations (no collective in the hand-back).
//
// One-process-per-GPU shards (mmba_comm_create_rccl) hand back through one
// all-gather of every shard's own rows instead (each rank returns the whole
// vectors); the step's rows after a sharded band solve are all-gathered the
// same way (each shard contributes its rows [Ra, Rb)).
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <numeric>
#include <thread>

#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

Comm *make_rccl_comm(ncclComm_t c, int rank, int nranks);  // mmba_comm.cpp
int rccl_init_all(const int *devices, int n, std::vector<Comm *> &out);  // mmba_comm.cpp

// ---------------------------------------------------------------------------
// kernels of the hand-back and the step-row gather

// send = [x at the own parameters (npar_pad) | f (2 pad) | eu (2 pad) | ed (pad)]
// (the outputs only when f2 != nullptr: count = npar_pad + 5 pad)
__global__ void k_own_pack(int n_own, int npar_pad, const int *__restrict__ own_par,
                           const double *__restrict__ x, int m_own, int pad,
                           const int *__restrict__ own_dev, const double *__restrict__ f2,
                           const double *__restrict__ eu2, const double *__restrict__ ed,
                           double *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npar_pad) out[i] = (i < n_own && x) ? x[own_par[i]] : 0.;
    if (!f2 || i >= pad) return;
    double *of = out + npar_pad, *oe = of + 2 * (size_t)pad, *od = oe + 2 * (size_t)pad;
    if (i < m_own) {
        const int d = own_dev[i];
        of[2 * i] = f2[2 * d];
        of[2 * i + 1] = f2[2 * d + 1];
        oe[2 * i] = eu2 ? eu2[2 * d] : 0.;
        oe[2 * i + 1] = eu2 ? eu2[2 * d + 1] : 0.;
        od[i] = ed ? ed[d] : 0.;
    } else {
        of[2 * i] = of[2 * i + 1] = oe[2 * i] = oe[2 * i + 1] = od[i] = 0.;
    }
}

// every rank's packed rows (recv, `count` doubles per rank) -> x (n) and the
// reference-order outputs (f / eu 2 Mg, ed Mg)
__global__ void k_own_unpack(int nr, size_t count, const double *__restrict__ recv, int npar_pad,
                             const int *__restrict__ par_all, double *__restrict__ x, int pad,
                             const int *__restrict__ ref_all, double *__restrict__ f2o,
                             double *__restrict__ eu2o, double *__restrict__ edo) {
    const int k = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr) return;
    const double *in = recv + (size_t)k * count;
    if (i < npar_pad) {
        const int p = par_all[(size_t)k * npar_pad + i];
        if (p >= 0) x[p] = in[i];
    }
    if (!f2o || i >= pad) return;
    const int r = ref_all[(size_t)k * pad + i];
    if (r < 0) return;
    const double *of = in + npar_pad, *oe = of + 2 * (size_t)pad, *od = oe + 2 * (size_t)pad;
    f2o[2 * (size_t)r] = of[2 * i];
    f2o[2 * (size_t)r + 1] = of[2 * i + 1];
    eu2o[2 * (size_t)r] = oe[2 * i];
    eu2o[2 * (size_t)r + 1] = oe[2 * i + 1];
    edo[r] = od[i];
}

// send = [xR rows [Ra, Ra + len) | 0 ... | the nG arrow rows] (pad doubles)
__global__ void k_rows_pack(const double *__restrict__ xR, int Ra, int len, int nb, int nG, int pad,
                            double *__restrict__ send) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= pad) return;
    const int ga = pad - nG;
    send[i] = i < len ? xR[Ra + i] : i >= ga ? xR[nb + (i - ga)] : 0.;
}

// xR rows of rank k from its block; the arrow rows from rank 0's
__global__ void k_rows_unpack(const double *__restrict__ recv, const int *__restrict__ Ra_all,
                              const int *__restrict__ Rb_all, int nr, int nb, int nG, int pad,
                              double *__restrict__ xR) {
    const int k = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr || i >= pad) return;
    const int a = Ra_all[k], len = Rb_all[k] - a, ga = pad - nG;
    const double v = recv[(size_t)k * pad + i];
    if (i < len) xR[a + i] = v;
    else if (k == 0 && i >= ga) xR[nb + (i - ga)] = v;
}

static int nblk(size_t n, int t) { return (int)((n + t - 1) / t); }

// ---------------------------------------------------------------------------
// Plan: sharded hand-back and step rows

// own_obs_rank[i] / par_rank[p]: every rank's ownership (global observation
// / parameter), from the frame partition every shard computes identically.
void Plan::setup_handback(const std::vector<int> &own_rank_obs_par) {
    // own_rank_obs_par = [rank of each global observation (Mg) | rank of each
    // parameter (n)]
    const int *orank = own_rank_obs_par.data(), *prank = orank + Mg;
    std::vector<int> cnt_obs(nranks, 0), cnt_par(nranks, 0);
    for (int i = 0; i < Mg; ++i) cnt_obs[orank[i]]++;
    for (int p = 0; p < n; ++p) cnt_par[prank[p]]++;
    own_pad = std::max(1, *std::max_element(cnt_obs.begin(), cnt_obs.end()));
    npar_pad = std::max(1, *std::max_element(cnt_par.begin(), cnt_par.end()));
    // every rank's lists in ascending reference / parameter order, padded
    std::vector<int> ref_all((size_t)nranks * own_pad, -1), par_all((size_t)nranks * npar_pad, -1);
    std::vector<int> fill_o(nranks, 0), fill_p(nranks, 0);
    for (int i = 0; i < Mg; ++i) {
        const int k = orank[i];
        ref_all[(size_t)k * own_pad + fill_o[k]++] = i;
    }
    for (int p = 0; p < n; ++p) {
        const int k = prank[p];
        par_all[(size_t)k * npar_pad + fill_p[k]++] = p;
    }
    M_own = cnt_obs[rank];
    n_own = cnt_par[rank];
    own_ref_h.assign(ref_all.begin() + (size_t)rank * own_pad,
                     ref_all.begin() + (size_t)rank * own_pad + M_own);
    own_par_h.assign(par_all.begin() + (size_t)rank * npar_pad,
                     par_all.begin() + (size_t)rank * npar_pad + n_own);
    // device index of each own observation (ref_of_dev's inverse)
    std::vector<int> dev_of_ref(Mg, -1);
    for (int i = 0; i < M; ++i) dev_of_ref[ref_of_dev[i]] = i;
    std::vector<int> own_dev(std::max(M_own, 1), 0);
    for (int j = 0; j < M_own; ++j) {
        own_dev[j] = dev_of_ref[own_ref_h[j]];
        if (own_dev[j] < 0) throw Invalid{"an own observation missing from the shard"};
    }
    d_own_dev = upload(own_dev);
    d_own_par = upload(own_par_h.empty() ? std::vector<int>(1, 0) : own_par_h);
    d_own_ref_all = upload(ref_all);
    d_own_par_all = upload(par_all);
    const size_t count = (size_t)npar_pad + 5 * (size_t)own_pad;
    d_pack = dalloc<double>(count);
    d_pack_all = dalloc<double>(count * nranks);
    MMBA_HIP(hipHostMalloc((void **)&h_pack, sizeof(double) * count, hipHostMallocDefault));
    // the step's rows
    rows_pad = 1;
    for (int k = 0; k < nranks; ++k) rows_pad = std::max(rows_pad, Rb_all[k] - Ra_all[k]);
    rows_pad += nG;
    d_Ra_all = upload(Ra_all);
    d_Rb_all = upload(Rb_all);
    d_rows_send = dalloc<double>(rows_pad);
    d_rows_all = dalloc<double>((size_t)rows_pad * nranks);
}

void Plan::gather_step_rows() {
    const int nb = nR - nG;
    k_rows_pack<<<nblk(rows_pad, 256), 256, 0, s>>>(d_xR, Ra, Rb - Ra, nb, nG, rows_pad,
                                                   d_rows_send);
    comm->allgather(d_rows_send, d_rows_all, rows_pad, s);
    k_rows_unpack<<<dim3(nblk(rows_pad, 256), nranks), 256, 0, s>>>(
        d_rows_all, d_Ra_all, d_Rb_all, nranks, nb, nG, rows_pad, d_xR);
}

// x (dx: n) and the per-residual outputs (device order: f2 / eu2 2 M, ed M)
// to the caller.  Group shards (host_gather): this shard's own parameters
// and observations into the caller's buffers, no collective.  Otherwise one
// all-gather of every shard's own rows: each rank returns the whole vectors.
// Attribute rows (identical on every shard) come from shard 0 / the device.
void Plan::handback_sharded(const double *dx, double *x_out, double *f_out, double *eu_out,
                            double *ed_out, const double *f2, const double *eu2,
                            const double *ed1) {
    const bool outs = f_out || eu_out || ed_out;
    const size_t count = (size_t)npar_pad + (outs ? 5 * (size_t)own_pad : 0);
    const int work = std::max(npar_pad, outs ? own_pad : 0);
    k_own_pack<<<nblk(work, 256), 256, 0, s>>>(n_own, npar_pad, d_own_par, x_out ? dx : nullptr,
                                              M_own, own_pad, d_own_dev, outs ? f2 : nullptr, eu2,
                                              ed1, d_pack);
    if (host_gather) {
        MMBA_HIP(hipMemcpyAsync(h_pack, d_pack, sizeof(double) * count, hipMemcpyDeviceToHost, s));
        if (rank == 0 && nrows > 0) {  // attribute rows: identical on every shard
            if (f_out)
                MMBA_HIP(hipMemcpyAsync(f_out + 2 * (size_t)Mg, f2 + 2 * (size_t)M,
                                        sizeof(double) * nrows, hipMemcpyDeviceToHost, s));
            if (eu_out)
                MMBA_HIP(hipMemcpyAsync(eu_out + 2 * (size_t)Mg, eu2 + 2 * (size_t)M,
                                        sizeof(double) * nrows, hipMemcpyDeviceToHost, s));
        }
        host_sync();
        if (x_out)
            for (int j = 0; j < n_own; ++j) x_out[own_par_h[j]] = h_pack[j];
        if (outs) {
            const double *of = h_pack + npar_pad, *oe = of + 2 * (size_t)own_pad,
                         *od = oe + 2 * (size_t)own_pad;
            for (int j = 0; j < M_own; ++j) {
                const size_t r = (size_t)own_ref_h[j];
                if (f_out) {
                    f_out[2 * r] = of[2 * j];
                    f_out[2 * r + 1] = of[2 * j + 1];
                }
                if (eu_out) {
                    eu_out[2 * r] = oe[2 * j];
                    eu_out[2 * r + 1] = oe[2 * j + 1];
                }
                if (ed_out) ed_out[r] = od[j];
            }
        }
        return;
    }
    comm->allgather(d_pack, d_pack_all, count, s);
    double *tf = d_gather, *te = d_gather + mg, *td = d_gather + 2 * (size_t)mg;
    double *tx = d_gather + 2 * (size_t)mg + Mg;
    k_own_unpack<<<dim3(nblk(work, 256), nranks), 256, 0, s>>>(
        nranks, count, d_pack_all, npar_pad, d_own_par_all, tx, own_pad, d_own_ref_all,
        outs ? tf : nullptr, te, td);
    if (nrows > 0 && outs) {
        MMBA_HIP(hipMemcpyAsync(tf + 2 * (size_t)Mg, f2 + 2 * (size_t)M, sizeof(double) * nrows,
                                hipMemcpyDeviceToDevice, s));
        MMBA_HIP(hipMemcpyAsync(te + 2 * (size_t)Mg, eu2 + 2 * (size_t)M, sizeof(double) * nrows,
                                hipMemcpyDeviceToDevice, s));
    }
    if (x_out) MMBA_HIP(hipMemcpyAsync(x_out, tx, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    if (f_out) MMBA_HIP(hipMemcpyAsync(f_out, tf, sizeof(double) * mg, hipMemcpyDeviceToHost, s));
    if (eu_out) MMBA_HIP(hipMemcpyAsync(eu_out, te, sizeof(double) * mg, hipMemcpyDeviceToHost, s));
    if (ed_out) MMBA_HIP(hipMemcpyAsync(ed_out, td, sizeof(double) * Mg, hipMemcpyDeviceToHost, s));
    host_sync();
}

bool Plan::poll_agree() {
    if (!pshare) return poll_interrupt();
    const int v = rank == 0 ? (poll_interrupt() ? 1 : 0) : 0;
    return pshare->agree(rank, v) != 0;
}

int Plan::poll_agree_index(int k) { return pshare ? pshare->agree(rank, k) : k; }

// ---------------------------------------------------------------------------
// the shard group

struct GroupPoll : PollShare {
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0, val = 0, out = 0;
    long gen = 0;
    bool aborted = false;
    int agree(int rank, int v) override {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) throw CommError();
        const long g = gen;
        if (rank == 0) val = v;
        if (++arrived == n) {
            arrived = 0;
            out = val;
            ++gen;
            cv.notify_all();
            return out;
        }
        cv.wait(lk, [&] { return gen != g || aborted; });
        if (gen == g) {
            set_error("shard group aborted (another shard failed)");
            throw CommError();
        }
        return out;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

struct ShardGroup {
    mmba_context *ctx = nullptr;  // the multi-device context
    int n = 0;                    // shards that run (1 when the problem was replicated)
    std::vector<mmba_plan *> plans;
    GroupPoll poll;
    bool broken = false;

    // persistent workers for shards 1 .. n-1
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done_cv;
    const std::function<int(int)> *job = nullptr;
    long gen = 0;
    int remaining = 0;
    bool stop = false;
    std::vector<int> rc;
    std::vector<std::string> err;

    void abort_all() {
        for (Comm *c : ctx->comms) c->abort();
        poll.abort();
    }

    int run_one(const std::function<int(int)> &f, int k) {
        int r;
        try {
            r = f(k);
        } catch (const CommError &) {
            r = MMBA_ERR_COMM;
        } catch (const DeviceError &) {
            r = MMBA_ERR_DEVICE;
        } catch (const std::exception &e) {
            set_error(std::string("exception: ") + e.what());
            r = MMBA_ERR_INVALID;
        }
        rc[k] = r;
        err[k] = r == MMBA_OK ? std::string() : std::string(mmba_last_error());
        // ANY failure of one shard can leave the others inside a collective
        // (an Invalid / Unsupported / bad_alloc thrown mid-solve is as fatal
        // to them as a device error): release them at once; the group is
        // unusable afterwards (run() marks it broken).  The interrupt is
        // agreed through the poll share, so every shard stops at the same
        // point and nobody waits.
        if (n > 1 && r != MMBA_OK && r != MMBA_ERR_INTERRUPTED) abort_all();
        return r;
    }

    void worker(int k) {
        (void)hipSetDevice(ctx->shards[k]->device);
        long seen = 0;
        for (;;) {
            const std::function<int(int)> *f;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                // a replicated problem runs shard 0 alone (n == 1): the
                // other workers stay idle whatever wakes them
                if (k >= n || !job) continue;
                f = job;
            }
            run_one(*f, k);
            std::lock_guard<std::mutex> lk(m);
            if (--remaining == 0) done_cv.notify_all();
        }
    }

    void start(int nthreads) {
        rc.assign(nthreads, 0);
        err.assign(nthreads, std::string());
        for (int k = 1; k < nthreads; ++k) th.emplace_back([this, k] { worker(k); });
    }

    // f(k) on every running shard; the first failing shard's code and message
    int run(const std::function<int(int)> &f) {
        if (broken) {
            set_error("shard group unusable after an earlier device / communicator failure");
            return MMBA_ERR_COMM;
        }
        {
            std::lock_guard<std::mutex> lk(m);
            job = &f;
            remaining = n - 1;
            for (int k = 0; k < n; ++k) rc[k] = MMBA_OK;
            ++gen;
        }
        if (n > 1) cv.notify_all();
        run_one(f, 0);
        {
            std::unique_lock<std::mutex> lk(m);
            done_cv.wait(lk, [&] { return remaining == 0; });
            job = nullptr;
        }
        // the first shard's failure, preferring a cause over the
        // communicator errors of the shards it released
        int out = MMBA_OK, first = -1;
        for (int k = 0; k < n; ++k) {
            if (n > 1 && rc[k] != MMBA_OK && rc[k] != MMBA_ERR_INTERRUPTED) broken = true;
            if (rc[k] == MMBA_OK) continue;
            if (first < 0 || (rc[first] == MMBA_ERR_COMM && rc[k] != MMBA_ERR_COMM)) first = k;
        }
        if (first >= 0) {
            out = rc[first];
            set_error(err[first]);
        }
        return out;
    }

    ~ShardGroup() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
        for (mmba_plan *p : plans) mmba_plan_destroy(p);
    }
};

void destroy_group(ShardGroup *g) { delete g; }

// ---- group forms of the plan entry points (mmba_api.cpp routes here) ----

int group_plan_create(mmba_context *ctx, const mmba_problem *prob, const mmba_options *opt,
                      mmba_plan **out) {
    const int N = (int)ctx->shards.size();
    auto *g = new ShardGroup();
    g->ctx = ctx;
    g->n = N;
    g->plans.assign(N, nullptr);
    g->poll.n = N;
    g->start(N);
    const std::function<int(int)> f = [&](int k) -> int {
        return mmba_plan_create_sharded(ctx->shards[k], prob, opt,
                                        reinterpret_cast<mmba_comm *>(ctx->comms[k]),
                                        &g->plans[k]);
    };
    const int rc = g->run(f);
    if (rc != MMBA_OK) {
        const std::string why = mmba_last_error();
        delete g;
        set_error(why);
        return rc;
    }
    if (g->plans[0]->impl.replicated) {
        // the problem does not shard (every shard built the whole problem):
        // shard 0 alone solves it, the group's threads stay idle
        for (int k = 1; k < N; ++k) {
            mmba_plan_destroy(g->plans[k]);
            g->plans[k] = nullptr;
        }
        g->plans.resize(1);
        g->n = 1;
    } else {
        for (int k = 0; k < N; ++k) {
            g->plans[k]->impl.pshare = &g->poll;
            g->plans[k]->impl.host_gather = true;
        }
    }
    auto *p = new mmba_plan();
    p->impl.ctx = ctx;
    p->group.reset(g);
    *out = p;
    return MMBA_OK;
}

static int dummy_interrupt(void *) { return 0; }  // never called: shard 0 answers polls

int group_plan_solve(mmba_plan *plan, double *x_inout, double *fvec_out, double *err_user_out,
                     double *err_dist_out, mmba_result *res, const mmba_callbacks *cb,
                     mmba_trace *trace) {
    ShardGroup &g = *plan->group;
    const int n = g.plans[0]->impl.n;
    // every shard starts from a private copy of x0 and writes its own
    // parameters into x_inout at the end (a replicated plan: shard 0 alone)
    std::vector<std::vector<double>> x0(g.n, std::vector<double>(x_inout, x_inout + n));
    mmba_callbacks proxy{};
    if (cb && cb->interrupt) proxy.interrupt = dummy_interrupt;
    std::vector<mmba_result> rs(g.n);
    const std::function<int(int)> f = [&](int k) -> int {
        Plan &p = g.plans[k]->impl;
        p.group_x_out = g.n > 1 ? x_inout : nullptr;
        return mmba_plan_solve(g.plans[k], g.n > 1 ? x0[k].data() : x_inout, fvec_out,
                               err_user_out, err_dist_out, &rs[k], k == 0 ? cb : &proxy,
                               k == 0 ? trace : nullptr);
    };
    const int rc = g.run(f);
    if (res) *res = rs[0];
    return rc;
}

int group_plan_measure(mmba_plan *plan, const double *x, double *fvec_out, double *err_user_out,
                       double *err_dist_out, double *avg_min_max_out) {
    ShardGroup &g = *plan->group;
    const std::function<int(int)> f = [&](int k) -> int {
        return mmba_plan_measure(g.plans[k], x, fvec_out, err_user_out, err_dist_out,
                                 k == 0 ? avg_min_max_out : nullptr);
    };
    return g.run(f);
}

int group_plan_reproject(mmba_plan *plan, const double *x, double *point_xy_out,
                         double *marker_xy_out) {
    ShardGroup &g = *plan->group;
    const std::function<int(int)> f = [&](int k) -> int {
        return mmba_plan_reproject(g.plans[k], x, point_xy_out, marker_xy_out);
    };
    return g.run(f);
}

int group_plan_jacobian(mmba_plan *plan, const double *x, double *fjac) {
    ShardGroup &g = *plan->group;
    if (g.n > 1) {
        set_error("unsupported: dense Jacobian of a sharded plan");
        return MMBA_ERR_UNSUPPORTED;
    }
    return mmba_plan_jacobian(g.plans[0], x, fjac);
}

int group_plan_outputs(mmba_plan *plan, double *fvec_out, double *err_user_out,
                       double *err_dist_out) {
    ShardGroup &g = *plan->group;
    const std::function<int(int)> f = [&](int k) -> int {
        return mmba_plan_outputs(g.plans[k], fvec_out, err_user_out, err_dist_out);
    };
    return g.run(f);
}

int group_plan_set_attr_values(mmba_plan *plan, const double *attr_values) {
    ShardGroup &g = *plan->group;
    const std::function<int(int)> f = [&](int k) -> int {
        return mmba_plan_set_attr_values(g.plans[k], attr_values);
    };
    return g.run(f);
}

int group_plan_solve_per_frame(mmba_plan *plan, double *x_inout, mmba_result *results,
                               const mmba_callbacks *cb) {
    ShardGroup &g = *plan->group;
    if (g.n > 1) {
        set_error("unsupported: per-frame batch: sharded plan");
        return MMBA_ERR_UNSUPPORTED;
    }
    return mmba_plan_solve_per_frame(g.plans[0], x_inout, results, cb);
}

// shard 0's statistics; the timing switch reaches every shard
int group_plan_kernel_stats(mmba_plan *plan, int enable_timing, mmba_kernel_stats *out) {
    ShardGroup &g = *plan->group;
    for (int k = g.n - 1; k >= 0; --k) {
        const int rc = mmba_plan_kernel_stats(g.plans[k], enable_timing, k == 0 ? out : nullptr);
        if (rc != MMBA_OK) return rc;
    }
    if (out) out->shards_replicated = (int)g.ctx->shards.size() > 1 && g.n == 1 ? 1 : 0;
    return MMBA_OK;
}

int group_num_shards(const mmba_plan *plan) { return plan->group ? plan->group->n : 1; }

}  // namespace mmba

using namespace mmba;

extern "C" {

int mmba_context_create_multi(const int *devices, int ndevices, mmba_context **out) {
    if (!out || !devices || ndevices < 1 || ndevices > 8) return MMBA_ERR_INVALID;
    *out = nullptr;
    const int visible = mmba_device_count();
    if (visible <= 0) {
        set_error("no gfx950 (MI355X) device visible");
        return MMBA_ERR_NO_DEVICE;
    }
    bool same = true, distinct = true;
    for (int k = 0; k < ndevices; ++k) {
        if (devices[k] < 0 || devices[k] >= visible) {
            set_error("device index out of range");
            return MMBA_ERR_INVALID;
        }
        same &= devices[k] == devices[0];
        for (int j = 0; j < k; ++j) distinct &= devices[j] != devices[k];
    }
    if (ndevices > 1 && !same && !distinct) {
        set_error("devices must be distinct (RCCL) or one device named N times (in-process "
                  "shards)");
        return MMBA_ERR_INVALID;
    }
    auto *c = new mmba_context();
    c->device = devices[0];
    int rc = MMBA_OK;
    for (int k = 0; k < ndevices && rc == MMBA_OK; ++k) {
        mmba_context *sub = nullptr;
        rc = mmba_context_create(devices[k], &sub);
        if (rc == MMBA_OK) c->shards.push_back(sub);
    }
    if (rc == MMBA_OK && ndevices > 1) {
        if (same) {
            std::vector<mmba_comm *> cs(ndevices, nullptr);
            rc = mmba_comm_create_local(ndevices, cs.data());
            if (rc == MMBA_OK)
                for (mmba_comm *x : cs) c->comms.push_back(reinterpret_cast<Comm *>(x));
        } else {
            rc = rccl_init_all(devices, ndevices, c->comms);
        }
    }
    if (rc != MMBA_OK) {
        const std::string why = mmba_last_error();
        mmba_context_destroy(c);
        set_error(why);
        return rc;
    }
    c->stream = c->shards[0]->stream;
    *out = c;
    return MMBA_OK;
}

int mmba_context_num_devices(const mmba_context *ctx) {
    if (!ctx) return MMBA_ERR_INVALID;
    return ctx->shards.empty() ? 1 : (int)ctx->shards.size();
}

int mmba_plan_num_shards(const mmba_plan *plan) {
    if (!plan) return MMBA_ERR_INVALID;
    if (plan->group) return group_num_shards(plan);
    return plan->impl.nranks;
}

}  // extern "C"
