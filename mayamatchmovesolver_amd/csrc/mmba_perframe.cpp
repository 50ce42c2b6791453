// mmba_perframe.cpp -- per-frame solve mode (FrameSolveMode::kPerFrame,
// src/mmSolver/adjust/adjust_base.cpp:1430-1484): one solveFrames call per
// frame, each over that frame's observations and the parameters of that frame
// (animated attributes keyed at it) plus every static parameter.
//
// The reference runs the frames one after another.  When no static parameter
// is solved the frames share nothing, so here they run concurrently: a pool
// of host threads, each with its own context (stream) and one plan per frame,
// all on the caller's device -- many small launch-bound LM solves overlap on
// the GPU instead of queueing behind each other.  With a static parameter the
// frames are chained exactly as in the reference (frame i starts from the
// static values frame i - 1 left), so they run in order.
//
// Like the reference loop (":1471-1476 Failed to solve frame, stopping
// solve"), the first frame that cannot be solved (fewer residuals than
// parameters, no parameters) stops the sequence: later frames are left
// untouched and report success = 0, reason_number = 0.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

// Every frame's solve in one launch (mmba_batch.hip).  The interrupt
// callback is polled on this (the calling) thread while the launch runs; a
// request reaches the frames through a host-mapped flag they read at the
// reference's poll points (each evaluation, each Jacobian).
int Plan::solve_frames(double *x_inout, mmba_result *results, const mmba_callbacks *cb) {
    if (!batch_ok) {
        set_error("per-frame batch: " + batch_why);
        return MMBA_ERR_UNSUPPORTED;
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (!d_bJ) {
        d_bJ = dalloc<double>((size_t)M * 2 * PCMAX);
        d_bdist = dalloc<double>((size_t)2 * M);
        d_bx = dalloc<double>(n);
        d_bpw = upload(param_weight);
        d_bout = dalloc<BatchOut>(std::max(F, 1));
        MMBA_HIP(hipHostMalloc(&h_bflag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        MMBA_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_bflag), h_bflag, 0));
    }
    const bool polls = cb && cb->interrupt;
    // a request already pending stops every frame at its first poll
    __atomic_store_n(h_bflag, polls && cb->interrupt(cb->user) ? 1 : 0, __ATOMIC_SEQ_CST);
    attrs_reset();
    // bundle records (no bundle is solved: computed once per call)
    records_enqueue(nullptr, 1);
    MMBA_HIP(hipMemcpyAsync(d_bx, x_inout, sizeof(double) * n, hipMemcpyHostToDevice, s));
    BatchArgs B{};
    B.nf = batch_nf;
    B.fr_cf_off = d_fr_cf_off;
    B.fr_par_off = d_fr_par_off;
    B.fr_par = d_fr_par;
    B.fr_last = d_fr_last;
    B.fr_nobs = d_fr_nobs;
    B.pweight = d_bpw;
    B.J = d_bJ;
    B.ed = d_ed;
    B.dist = d_bdist;
    B.x = d_bx;
    B.out = d_bout;
    B.interrupt = polls ? d_bflag : nullptr;
    B.solver_type = opt.solver_type;
    B.mode = opt.auto_param_scale == 1 ? 1 : 2;
    B.maxfev = opt.iter_max;
    B.accept_only_better = opt.accept_only_better;
    B.initial_error_given = opt.initial_error_given;
    B.delta = opt.delta;
    B.factor = opt.tau * 100.0;
    B.ftol = opt.eps1;
    B.xtol = opt.eps2;
    B.gtol = opt.eps3;
    B.initial_error_avg = opt.initial_error_avg;
    launch_batch_lm(s, P, B, batch_nfmax);
    MMBA_HIP(hipGetLastError());
    if (polls) {
        hipError_t q;
        while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
            if (!__atomic_load_n(h_bflag, __ATOMIC_RELAXED) && cb->interrupt(cb->user))
                __atomic_store_n(h_bflag, 1, __ATOMIC_SEQ_CST);
            std::this_thread::yield();
        }
        if (q != hipSuccess) MMBA_HIP(q);
    }
    std::vector<double> xo(n);
    std::vector<BatchOut> out(std::max(batch_nf, 1));
    MMBA_HIP(hipMemcpyAsync(xo.data(), d_bx, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    if (batch_nf > 0)
        MMBA_HIP(hipMemcpyAsync(out.data(), d_bout, sizeof(BatchOut) * batch_nf,
                                hipMemcpyDeviceToHost, s));
    MMBA_HIP(hipStreamSynchronize(s));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // the first frame whose damped factorisation broke down stops the loop
    // like a failed frame of the reference (adjust_base.cpp:1471-1476)
    int ef = batch_nf;
    for (int f = 0; f < batch_nf; ++f)
        if (out[f].failed) {
            ef = f;
            break;
        }
    for (int f = 0; f < F; ++f) {
        mmba_result r;
        std::memset(&r, 0, sizeof(r));
        if (f < batch_nf && f <= ef) {
            const BatchOut &o = out[f];
            r.reason_number = o.info;
            r.iterations = o.nfev;
            r.function_evals = o.func_evals;
            r.jacobian_evals = o.jac_evals;
            r.outer_iterations = o.njev;
            r.user_interrupted = o.interrupted;
            r.success = o.func_evals > 0;
            r.error_final = o.fnorm;
            r.error_avg = o.avg;
            r.error_min = o.mn;
            r.error_max = o.mx;
            r.error_rms = o.rms;
            r.error_initial_avg = o.init_avg;
            r.error_is_better = o.better;
            r.time_solve_s = dt;
        }
        results[f] = r;
    }
    for (int p = 0; p < n; ++p)
        if (param_frame_host[p] < ef) x_inout[p] = xo[p];
    if (ef < batch_nf) {
        set_error("damped normal-equation factorisation failed (frame " + std::to_string(ef) + ")");
        return MMBA_ERR_DEVICE;
    }
    return MMBA_OK;
}

}  // namespace mmba

namespace {

// The reference's per-frame mode runs solveFrames once per frame, with a
// one-frame frame list, so its lens lookups never mix indices (SURVEY B3;
// Plan::build_lens_instances): plans built for it take the plain lens
// instances.
struct LensPlain {
    bool prev;
    LensPlain() : prev(mmba::t_lens_plain) { mmba::t_lens_plain = true; }
    ~LensPlain() { mmba::t_lens_plain = prev; }
};


// The sub-problem of one frame: the caller's arrays except the observation
// and parameter lists, which are filtered (order kept: observations stay
// marker-major, parameters attr-major).
struct FrameProblem {
    std::vector<int32_t> obs_marker, obs_frame, param_attr, param_frame, param_ref;
    std::vector<double> obs_xy, obs_weight, pmin, pmax, poff, pscale;
    std::vector<int> params;  // indices into the full parameter vector
    mmba_problem p{};

    void build(const mmba_problem &full, int f) {
        p = full;
        for (int i = 0; i < full.num_obs; ++i) {
            if (full.obs_frame[i] != f) continue;
            obs_marker.push_back(full.obs_marker[i]);
            obs_frame.push_back(f);
            obs_xy.push_back(full.obs_xy[2 * i]);
            obs_xy.push_back(full.obs_xy[2 * i + 1]);
            obs_weight.push_back(full.obs_weight[i]);
        }
        for (int j = 0; j < full.num_params; ++j) {
            if (full.param_frame[j] != f && full.param_frame[j] != -1) continue;
            params.push_back(j);
            param_attr.push_back(full.param_attr[j]);
            param_frame.push_back(full.param_frame[j]);
            if (full.param_ref_attr) param_ref.push_back(full.param_ref_attr[j]);
            pmin.push_back(full.param_min[j]);
            pmax.push_back(full.param_max[j]);
            poff.push_back(full.param_offset[j]);
            pscale.push_back(full.param_scale[j]);
        }
        p.num_obs = (int32_t)obs_marker.size();
        p.obs_marker = obs_marker.data();
        p.obs_frame = obs_frame.data();
        p.obs_xy = obs_xy.data();
        p.obs_weight = obs_weight.data();
        p.num_params = (int32_t)params.size();
        p.param_attr = param_attr.data();
        p.param_frame = param_frame.data();
        if (full.param_ref_attr) p.param_ref_attr = param_ref.data();
        p.param_min = pmin.data();
        p.param_max = pmax.data();
        p.param_offset = poff.data();
        p.param_scale = pscale.data();
    }
    bool solvable() const { return p.num_params > 0 && p.num_params <= 2 * p.num_obs; }
};

// One frame: plan, solve from the current x, write the frame's parameters
// back when the error got better (solveFrames' write-back, :1231-1244).
int solve_frame(mmba_context *ctx, FrameProblem &fp, const mmba_options *opt, double *x,
                mmba_result *res, const mmba_callbacks *cb) {
    const int n = fp.p.num_params;
    const int m = 2 * fp.p.num_obs + fp.p.num_stiff + fp.p.num_smooth;
    std::vector<double> xs(n), fvec(m), eu(m), ed(fp.p.num_obs);
    for (int k = 0; k < n; ++k) xs[k] = x[fp.params[k]];
    mmba_plan *plan = nullptr;
    LensPlain plain_lenses;  // one frame per solve: no lens index mixing (B3)
    int rc = mmba_plan_create(ctx, &fp.p, opt, &plan);
    if (rc != MMBA_OK) return rc;
    rc = mmba_plan_solve(plan, xs.data(), fvec.data(), eu.data(), ed.data(), res, cb, nullptr);
    mmba_plan_destroy(plan);
    if (rc != MMBA_OK && rc != MMBA_ERR_INTERRUPTED) return rc;
    if (res->error_is_better)
        for (int k = 0; k < n; ++k) x[fp.params[k]] = xs[k];
    return MMBA_OK;
}

}  // namespace

extern "C" int mmba_solve_per_frame(mmba_context *ctx, const mmba_problem *prob,
                                    const mmba_options *opt, double *x_inout,
                                    mmba_result *results, int32_t max_concurrency,
                                    const mmba_callbacks *cb) {
    if (!ctx || !prob || !opt || !x_inout || !results || prob->num_frames <= 0)
        return MMBA_ERR_INVALID;
    if (!ctx->shards.empty()) ctx = ctx->shards[0];  // a multi-device context: its first device
    try {
        const int F = prob->num_frames;
        std::vector<FrameProblem> fr(F);
        bool chained = false;
        for (int j = 0; j < prob->num_params; ++j) chained |= prob->param_frame[j] < 0;
        int nf = F;  // frames before the first unsolvable one
        for (int f = 0; f < F; ++f) {
            results[f] = mmba_result{};
            if (f < nf) {
                fr[f].build(*prob, f);
                if (!fr[f].solvable()) nf = f;
            }
        }
        if (!chained) {
            // one launch for every frame when the plan's structure allows it
            // (MMBA_PATH_PERFRAME_BATCH = 0: the per-frame plans below)
            if (mmba::path_choice(MMBA_PATH_PERFRAME_BATCH) != 0) {
                mmba_plan *plan = nullptr;
                LensPlain plain_lenses;
                if (mmba_plan_create(ctx, prob, opt, &plan) == MMBA_OK) {
                    int rc = MMBA_ERR_UNSUPPORTED;
                    if (plan->impl.batch_ok) rc = mmba_plan_solve_per_frame(plan, x_inout, results, cb);
                    mmba_plan_destroy(plan);
                    if (rc != MMBA_ERR_UNSUPPORTED) return rc;
                }
            }
        }
        if (max_concurrency <= 0) max_concurrency = nf;
        const int workers = chained ? 1 : std::max(1, std::min<int>(max_concurrency, nf));
        if (workers == 1) {
            for (int f = 0; f < nf; ++f) {
                const int rc = solve_frame(ctx, fr[f], opt, x_inout, &results[f], cb);
                if (rc != MMBA_OK) return rc;
            }
            return MMBA_OK;
        }
        // Independent frames: disjoint parameter sets, so the workers write
        // disjoint entries of x_inout.  A worker's failure is kept with its
        // message (mmba_last_error is per thread) and re-raised on the
        // calling thread; frames after the first failed one keep their
        // starting values, as the reference loop stops there (:1473-1477).
        // The interrupt callback is only called from the calling thread (the
        // Maya main-thread contract): it is polled here before each frame is
        // handed out, and a set interrupt reaches the frames' own solves
        // through a flag.
        std::atomic<int> next{0}, first_err{MMBA_OK}, err_frame{F}, active{workers};
        std::atomic<bool> stop_flag{false};
        std::mutex mu;
        std::string err_msg;
        std::vector<std::vector<double>> xout(nf);
        std::vector<char> done(nf, 0);
        struct Sticky {
            std::atomic<bool> *flag;
        } sticky{&stop_flag};
        mmba_callbacks wcb{};
        wcb.interrupt = [](void *u) -> int {
            return static_cast<Sticky *>(u)->flag->load() ? 1 : 0;
        };
        wcb.user = &sticky;
        auto work = [&]() {
            struct Done {  // every exit of the worker counts it out
                std::atomic<int> *a;
                ~Done() { a->fetch_sub(1); }
            } done_{&active};
            mmba_context *c = nullptr;
            int rc = mmba_context_create(ctx->device, &c);
            if (rc != MMBA_OK) {
                std::lock_guard<std::mutex> lk(mu);
                int ok = MMBA_OK;
                if (first_err.compare_exchange_strong(ok, rc)) err_msg = mmba_last_error();
                return;
            }
            for (int f; (f = next.fetch_add(1)) < nf && first_err.load() == MMBA_OK;) {
                try {
                    std::vector<double> x(x_inout, x_inout + prob->num_params);
                    rc = solve_frame(c, fr[f], opt, x.data(), &results[f],
                                     cb && cb->interrupt ? &wcb : nullptr);
                    if (rc == MMBA_OK) {
                        xout[f] = std::move(x);
                        done[f] = 1;
                    }
                } catch (const std::exception &e) {
                    mmba::set_error(std::string("per-frame worker: ") + e.what());
                    rc = MMBA_ERR_INVALID;
                } catch (...) {
                    mmba::set_error("per-frame worker: unknown exception");
                    rc = MMBA_ERR_INVALID;
                }
                if (rc != MMBA_OK) {
                    std::lock_guard<std::mutex> lk(mu);
                    if (f < err_frame.load()) {
                        err_frame = f;
                        first_err = rc;
                        err_msg = mmba_last_error();
                    }
                }
            }
            mmba_context_destroy(c);
        };
        std::vector<std::thread> pool;
        for (int w = 0; w < workers; ++w) pool.emplace_back(work);
        if (cb && cb->interrupt) {
            // poll from the calling thread until every worker has finished
            // (frames still running see an interrupt requested after the last
            // frame was handed out)
            while (active.load() > 0 && first_err.load() == MMBA_OK && !stop_flag.load()) {
                if (cb->interrupt(cb->user)) stop_flag = true;
                std::this_thread::yield();
            }
        }
        for (auto &t : pool) t.join();
        const int ef = err_frame.load();
        for (int f = 0; f < nf && f < ef; ++f) {
            if (!done[f]) continue;
            for (int k : fr[f].params) x_inout[k] = xout[f][k];
        }
        for (int f = ef + 1; f < F; ++f) results[f] = mmba_result{};
        if (first_err.load() != MMBA_OK) mmba::set_error(err_msg);
        return first_err.load();
    } catch (const std::exception &e) {
        mmba::set_error(std::string("per-frame: ") + e.what());
        return MMBA_ERR_INVALID;
    }
}
