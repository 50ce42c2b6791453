// mmba_lm.cpp -- device-resident Levenberg-Marquardt, MINPACK-1 lmder/lmdif
// control flow on normal equations.
//
// Mapping to the reference (cminpack 1.3.8 lmder.c / lmpar.c as called from
// src/mmSolver/adjust/adjust_cminpack_lmder.cpp:94-184):
//   qrfac column norms acnorm_j       -> sqrt(A_jj), A = J^T J
//   R^T (Q^T f)                       -> g = J^T f
//   ||R P^T p||                       -> ||J p|| (k_jp_sumsq, exact products)
//   qrsolv(par): (A + par D^2) x = g  -> bundle-Schur + tiled Cholesky
//   ||S^-T P^T v|| in lmpar           -> sqrt(v^T (A + par D^2)^-1 v)
//                                        = ||Lb^-1 v_b|| (+) ||Ls^-1 w_R||
// Scalar control (trust region, ratio tests, info codes) runs on the host
// with the same constants and operation order as the restatement in
// oracle/refcpu.c (lm_core / lmpar).
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

static double wall_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// ---- timing spans: events recorded on the stream, read after the solve ----
hipEvent_t Plan::next_event() {
    if (ev_used == ev_pool.size()) {
        hipEvent_t e = nullptr;
        MMBA_HIP(hipEventCreate(&e));
        ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
}

// Spans are sampled: every span_stride-th span of each kind is timed (an
// event pair costs ~6 us of stream time, more than some of the kernels it
// brackets), so the timed region is barely perturbed.
void Plan::span_begin(int kind) {
    span_on = timing && (span_ctr[kind]++ % span_stride) == 0;
    if (!span_on) return;
    span_a = next_event();
    MMBA_HIP(hipEventRecord(span_a, s));
}

void Plan::span_end(int kind) {
    if (!span_on) return;
    span_on = false;
    hipEvent_t b = next_event();
    MMBA_HIP(hipEventRecord(b, s));
    spans.push_back({span_a, b, kind});
    if (ev_used > 8192) collect_spans();  // bounded pool (long solves)
}

void Plan::collect_spans() {
    if (!spans.empty()) {
        host_sync();
        for (const Span &sp : spans) {
            float ms = 0.f;
            MMBA_HIP(hipEventElapsedTime(&ms, sp.a, sp.b));
            if (sp.kind == SPAN_RESID) {
                resid_ms += ms;
                resid_n++;
            } else if (sp.kind == SPAN_JAC) {
                jac_ms += ms;
                jac_n++;
            } else {
                chol_ms += ms;
                chol_n++;
            }
        }
        spans.clear();
    }
    ev_used = 0;
}

// ---- scalar slots ----
// The trial's slots on their way to the host before anything else is
// enqueued behind them (the pre-enqueued Jacobian): the D2H copy (unless the
// reduction mirrors them) and the event read_slots waits on.
bool Plan::red_defer_ok() const {
    // the next damped solve's k_schur_init launch takes them (no bundles:
    // nothing is launched ahead of it -- no one-launch block-diagonal solve
    // at nG == 0, no shard memsets); with solved bundles k_schur_obs does
    // (the bundle factor ahead of it touches neither the partial rows nor
    // the slots)
    if (nranks != 1 || b15 || nR <= 0) return false;
    if (nB_solved > 0) return !rs_bnd;
    // nG == 0: the one-launch block-diagonal solve carries them (k_bd_direct's
    // extra workgroups); a damped solve without a norm slot takes the general
    // path, whose k_schur_init does
    return band && bs.use_bd && (nG > 0 || path_choice(MMBA_PATH_RED_BD) != 0);
}

void Plan::flush_red() {
    if (!pend_red) return;
    pend_red = false;
    launch_reduce_multi(s, d_partial, pend_rs, d_scalar);
}

void Plan::stage_slots() {
    flush_red();
    const bool mirrored = mirror_pending;
    if (!mirrored)
        MMBA_HIP(hipMemcpyAsync(h_scalar, d_scalar, sizeof(double) * (SL_LAST + 1),
                                hipMemcpyDeviceToHost, s));
    if (!(mirrored && seq_pending)) {
        if (!ev_sync) MMBA_HIP(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
        MMBA_HIP(hipEventRecord(ev_sync, s));
    }
    slots_staged = true;
}

// A host wait on the plan's stream: bounded through an RCCL communicator
// (the stream may carry a collective another rank never joins: comm_wait
// aborts it after comm_timeout_ms() and throws CommError), a plain
// synchronisation otherwise.
void Plan::host_sync() { comm_wait(nranks > 1 ? comm : nullptr, s, nullptr); }

void Plan::wait_event() {
    if (nranks > 1 && comm && comm->bounded()) {
        comm_wait(comm, s, ev_sync);
        return;
    }
    if (!spin_wait) {
        MMBA_HIP(hipEventSynchronize(ev_sync));
        return;
    }
    for (;;) {
        const hipError_t e = hipEventQuery(ev_sync);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) MMBA_HIP(e);
    }
}

void Plan::read_slots(int lo, int hi) {
    flush_red();
    const bool mirrored = mirror_pending && lo == 0 && hi == SL_LAST;
    mirror_pending = false;
    const bool by_seq = mirrored && seq_pending;
    seq_pending = false;
    if (slots_staged && lo == 0 && hi == SL_LAST) {
        slots_staged = false;
        if (!by_seq) {
            wait_event();
            return;
        }
    }
    slots_staged = false;
    if (by_seq) {
        // the reduction's last block wrote the mirror, then the sequence
        // word (system-scope release): poll page-locked memory directly --
        // a stream event query costs microseconds per call.  The stream is
        // checked now and then, so a failed launch ends the wait.
        for (unsigned spins = 1;; ++spins) {
            if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq_next) return;
            if ((spins & 4095u) == 0) {
                if (nranks > 1 && comm && comm->bounded()) {
                    // (mirrored reductions are taken unsharded only; kept
                    // bounded should that change)
                    host_sync();
                    if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq_next) return;
                }
                const hipError_t e = hipStreamQuery(s);
                if (e == hipSuccess) {
                    if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq_next) return;
                    set_error("mirrored reduction finished without its sequence word");
                    throw DeviceError();
                }
                if (e != hipErrorNotReady) MMBA_HIP(e);
            }
        }
    }
    if (!mirrored)
        MMBA_HIP(hipMemcpyAsync(h_scalar + lo, d_scalar + lo, sizeof(double) * (hi - lo + 1),
                                hipMemcpyDeviceToHost, s));
    if (!spin_wait || (nranks > 1 && comm && comm->bounded())) {
        host_sync();
        return;
    }
    // The LM control thread has nothing else to do: poll an event instead of
    // a blocking stream synchronisation (whose wake-up adds tens of us per
    // decision point).
    if (!ev_sync) MMBA_HIP(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
    MMBA_HIP(hipEventRecord(ev_sync, s));
    for (;;) {
        const hipError_t e = hipEventQuery(ev_sync);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) MMBA_HIP(e);
    }
}

// Everything enqueued so far done: poll an event (a blocking stream
// synchronisation's wake-up costs tens of microseconds).
void Plan::stream_wait() {
    if (!ev_sync) MMBA_HIP(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
    MMBA_HIP(hipEventRecord(ev_sync, s));
    wait_event();
}

double Plan::read_scalar(int slot) {
    read_slots(slot, slot);
    return h_scalar[slot];
}

// Sharded: every shard holds a partial sum (or max); sum them in place.
void Plan::allreduce(double *d, size_t count, ReduceOp op) {
    if (comm && nranks > 1) comm->allreduce(d, count, op, s);
}

double Plan::reduce_read(int slot, ReduceOp op) {
    allreduce(d_scalar + slot, 1, op);
    return read_scalar(slot);
}

// ||D v||^2 over the parameters (each counted by the shard that owns it).
void Plan::dnorm_enqueue(const double *dv, int slot) {
    launch_sumsq(s, dv, d_diag, n, d_partial, nparts, d_scalar + slot, d_p_own, d_ticket);
    allreduce(d_scalar + slot, 1);
}

double Plan::dnorm(const double *dv) {
    dnorm_enqueue(dv, SL_DNORM);
    return std::sqrt(read_scalar(SL_DNORM));
}

void Plan::records_enqueue(const double *xat, int base_only) {
    launch_records(s, P, d_var_cf, d_ext_pert, d_step, d_recs, nvar, d_brec, base_only);
    recs_full_at = base_only ? nullptr : xat;
}

// iflag = 1: setParameters + measureErrors; ||f||^2 -> SL_FNORM.
void Plan::fun_enqueue(const double *dx, double *df, double *eu, double *ed, double *dist,
                       int slot) {
    flush_red();
    // ext_pert / step with the Jacobian's eps: a Jacobian at dx that follows
    // reuses this parameter pass (params_at)
    launch_param_set(s, P, dx, d_ext, d_ext_pert, d_step, opt.solver_type, opt.delta, fd_eps());
    params_at = dx;
    // the full record set (same launch; the variants and perturbed bundle
    // positions are what a Jacobian at dx reads next)
    records_enqueue(dx, 0);
    span_begin(SPAN_RESID);
    // stiffness / smoothness rows: their partial goes after the residual blocks
    launch_rows_eval(s, P, df + 2 * (size_t)M, eu ? eu + 2 * (size_t)M : nullptr, d_partial,
                     (M + 255) / 256);
    // the ticket epilogue sums only the residual kernel's own grid: with
    // attribute rows the rows' partial would be dropped, so reduce separately
    launch_residual(s, P, d_recs, df, eu, ed, d_partial, d_scalar + slot,
                    P.nrows > 0 ? nullptr : d_ticket, dist);
    span_end(SPAN_RESID);
    allreduce(d_scalar + slot, 1);
}

double Plan::fun(const double *dx, double *df, double *eu, double *ed, double *dist) {
    const double t0 = wall_now();
    fun_enqueue(dx, df, eu, ed, dist);
    const double r = std::sqrt(read_scalar(SL_FNORM));
    t_func += wall_now() - t0;
    return r;
}

// The pre-enqueued Jacobian applies where jac() takes the fused path whose
// only launch before the host-visible epilogue is k_jac_ne_u (uniform fast
// unsharded plans, forward differences, no attribute rows), no callback can
// end the solve between the trial and the Jacobian, and no timing spans run.
bool Plan::pre_jac_ok() const {
    return pre_jac && nranks == 1 && !central && nrows == 0 && !timing && !k2_split &&
           ne_epilogue_fusable(P) && jac_ne_fusable(P, jac_ncv) && !(cbk && cbk->interrupt) &&
           !(cbk && cbk->progress);
}

void Plan::pre_jac_enqueue(const double *dx, double *eu, double *ed) {
    NeEpi epi;
    epi.on = 1;
    epi.first = 0;  // a later iteration: the first Jacobian is never enqueued ahead
    epi.mode = opt.auto_param_scale == 1 ? 1 : 2;
    epi.fnorm = 0.;
    epi.fnorm_sq = d_scalar + SL_FNORM;  // the trial's ||f||^2 = the accepted fnorm^2
    epi.do_xn = 0;
    epi.do_gn = 1;
    epi.x = dx;
    epi.diag = d_diag;
    epi.acnorm = d_acnorm;
    epi.partial = d_partial;
    epi.rstride = pw;
    epi.cf_base = 0;
    epi.bnd_base = ncf;
    epi.gate = d_gate;
    epi.probe = d_k2probe;
    launch_jac_ne(s, jb_recompute() ? P_nojb() : P, d_recs, d_step, opt.solver_type, d_J, d_jcol,
                  nloc_set ? nullptr : d_nloc, d_stale, eu, ed, d_Acc, d_g, epi);
    nloc_set = true;
    pre_jac_pending = true;
    // the bundle pass right behind it, under the same gate (round 6): the
    // GPU no longer idles between the two while the host takes its decision
    // (the 5.8 us gap of profiles/r5_final6 / r6_k2).  jac() would launch
    // it with this epilogue: the fused path's, at a later iteration (first
    // = 0, gnorm from the device slot), with the lam = 0 bundle factor
    pre_bnd_pending = false;
    if (P.nbs > 0 && P.JB != nullptr && nG == 0) {
        if (jb_recompute()) {
            epi.jb_recs = d_recs;
            epi.jb_lmder = opt.solver_type == MMBA_SOLVER_CMINPACK_LMDER ? 1 : 0;
        }
        if (fold_ok && nB_solved > 0) {
            epi.Lb = d_Lb;
            epi.tb = d_tb;
            epi.fail = d_fail;
        }
        launch_ne(s, P, d_J, d_jcol, d_nloc, d_f, d_Acc, d_Acg, d_Abb, d_Abg, d_Agg, d_g,
                  d_glob_partial, glob_chunk, epi, true);
        pre_bnd_pending = true;
    }
    // ... and (MMBA_PATH_PRE_SCHUR = 1) the next damped solve's first launch
    // (the undamped solve of the next lmpar: lam = 0 with the bundle factor
    // the pass just formed), which carries the epilogue's reduction -- the
    // rows jac() defers at a later iteration (first = 0: no XN2; gnorm).
    // Measured on C4 (profiles/r6_presch/): the 5.8 us idle gap moves from
    // before k_schur_obs to before k_schur_dest_u -- the host's launches of
    // the trial and the gated passes are what it waits for -- and the rate is
    // unchanged, so opt-in
    pre_sobs_pending = false;
    if (pre_bnd_pending && fold_ok && nB_solved > 0 && !rs_bnd && red_defer_ok() &&
        path_choice(MMBA_PATH_PRE_SCHUR) == 1) {
        const int ncol = ncf + (nB + NE_BND_TPB - 1) / NE_BND_TPB;
        RedSpec rs{};
        rs.flag_slot = -1;
        rs.row[rs.nrows++] = {0, ncol, 1, SL_ZERO};
        rs.row[rs.nrows++] = {2 * pw, ncol, 1, SL_GNORM};
        launch_schur_obs(s, P, d_J, d_Lb, d_W, &rs, d_partial, d_scalar, d_gate);
        pre_sobs_pending = true;
    }
    pre_jac_x = dx;
}

// The bundle records of the fused Jacobian pass re-evaluated by the bundle
// pass instead of stored and re-fetched (MMBA_PATH_JB_RECOMPUTE = 1; only
// where k_jac_ne_u -- jac_obs_u's arithmetic -- is the Jacobian pass).  Same
// bits (test_k2_records_and_backsub_forms_bit_identical).  Measured on C4
// (profiles/r6_b2/c4_iteration_trace.txt): k_jac_ne_u 31.5 -> 29.1 us (12.8
// MB fewer stores) but k_ne_bnd_jb 12.0 -> 19.7 us (each bundle thread
// gathers and re-projects its four observations in series) and the 5.8 us
// gap before it unchanged -- a net loss, so opt-in.
bool Plan::jb_recompute() const {
    return P.JB != nullptr && P.all_bnd_fast && path_choice(MMBA_PATH_JB_RECOMPUTE) == 1;
}

// The plan's problem without the JB records: k_jac_ne_u then stores none.
DevProblem Plan::P_nojb() const {
    DevProblem Q = P;
    Q.JB = nullptr;
    return Q;
}

// iflag = 2: FD Jacobian blocks + normal equations + column norms at x.
void Plan::jac(const double *dx, const JacLM *lm) {
    flush_red();
    const double t0 = wall_now();
    const double eps_dif = fd_eps();
    const bool lmder = opt.solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    // the accepted trial point (or the last evaluation) already set the
    // parameters at dx: external values, FD points and steps are those
    // k_param_set would write, bit for bit (same inputs, same kernel code)
    if (params_at != dx) {
        launch_param_set(s, P, dx, d_ext, d_ext_pert, d_step, opt.solver_type, opt.delta, eps_dif);
        recs_full_at = nullptr;
    }
    params_at = dx;
    if (recs_full_at != dx) records_enqueue(dx, 0);  // else built by the evaluation at dx
    CentralB CB;
    if (central) {  // the deltaB pass of the central columns
        MMBA_HIP(hipMemsetAsync(d_scalar + SL_NCENT, 0, sizeof(double), s));
        launch_param_central(s, P, dx, d_ext_pertB, d_stepB, opt.delta, d_scalar + SL_NCENT,
                             b15 ? d_c15 : nullptr);
        launch_records(s, P, d_var_cf, d_ext_pertB, d_stepB, d_recsB, nvar, d_brecB, 0);
        CB.recs = d_recsB;
        CB.brec = d_brecB;
        CB.ext_pert = d_ext_pertB;
        CB.step = d_stepB;
        if (b15) {
            launch_b15_q(s, P, d_c15, d_q15, d_kap15, d_c15r);
            CB.q15 = d_q15;
            CB.kap15 = d_kap15;
        }
    }
    span_begin(SPAN_JAC);
    // uniform unsharded plans: the lmder bookkeeping rides in the
    // normal-equation kernels (no k_jac_epilogue launch), and with one
    // block size the camera-frame normal equations ride in the Jacobian
    // pass itself (k_jac_ne_u: J is written once and not re-read)
    const bool fuse = lm && ne_epilogue_fusable(P) && nrows == 0 && !b15;
    NeEpi epi;
    if (fuse) {
        epi.on = 1;
        epi.first = lm->first;
        epi.mode = lm->mode;
        epi.fnorm = lm->fnorm;
        epi.fnorm_sq = lm->fnorm_sq;
        epi.do_xn = lm->first;
        epi.do_gn = lm->fnorm_sq || lm->fnorm != 0.;
        epi.x = dx;
        epi.diag = d_diag;
        epi.acnorm = d_acnorm;
        epi.partial = d_partial;
        epi.rstride = pw;
        epi.cf_base = 0;
        epi.bnd_base = ncf;
    }
    epi.probe = d_k2probe;
    if (fuse && path_choice(MMBA_PATH_NE_CF_SPLIT) != 0) {
        // long camera-frame segments: the camera-frame normal equations over
        // NE_CF_SPLIT workgroups each (k_ne_cf_split; launch_ne decides)
        epi.cf_part = d_cf_part;
        epi.cf_ticket = d_cf_ticket;
    }
    // unsharded plans with fast bundles: the bundle pass forms the lam = 0
    // bundle factor the undamped solve reads next (no k_bundle_factor
    // launch); with tail_reduce its last workgroup also reduces the
    // epilogue rows
    // (sharded too: every bundle a shard touches has all its observations
    // there; the others have Abb = 0 and factor as the identity)
    const bool fold = fuse && P.nbs > 0 && P.JB != nullptr && fold_ok;
    const bool tail = fold && tail_reduce && nranks == 1;
    lb0_valid = false;
    if (tail) {
        epi.fold = 1;
        epi.scalar = d_scalar;
        epi.ticket = d_mticket;
        RedSpec &rf = epi.spec;
        rf.flag_slot = -1;
        const int ncol = ncf + (nB_solved > 0 ? (nB + NE_BND_TPB - 1) / NE_BND_TPB : 0);  // as below
        rf.row[rf.nrows++] = {0, ncol, 1, SL_ZERO};
        if (epi.do_xn) rf.row[rf.nrows++] = {pw, ncol, 0, SL_XN2};
        if (epi.do_gn) rf.row[rf.nrows++] = {2 * pw, ncol, 1, SL_GNORM};
    }
    if (fold && nB_solved > 0) {
        epi.Lb = d_Lb;
        epi.tb = d_tb;
        epi.fail = d_fail;
        lb0_valid = true;
    }
    const bool k2_fused = !central && jac_ne_fusable(P, jac_ncv) && !k2_split;
    const bool pre_done = pre_jac_pending && pre_jac_x == dx && k2_fused && fuse;
    // sharded: g holds only this shard's terms -- zeroed BEFORE the fused
    // pass, which writes the camera-frame part of g itself
    if (nranks > 1) MMBA_HIP(hipMemsetAsync(d_g, 0, sizeof(double) * n, s));
    pre_jac_pending = false;
    const bool pre_bnd = pre_done && pre_bnd_pending;  // its bundle pass ran ahead too
    pre_bnd_pending = false;
    sobs_ahead = pre_done && pre_sobs_pending;  // and the next damped solve's k_schur_obs
    pre_sobs_pending = false;
    if (pre_done) {
        // k_jac_ne_u ran ahead at this x (its gate was open: the device took
        // this trial point, as the host did)
    } else if (k2_fused) {
        // the local column counts are a property of the plan: stored once
        launch_jac_ne(s, jb_recompute() ? P_nojb() : P, d_recs, d_step, opt.solver_type, d_J,
                      d_jcol, nloc_set ? nullptr : d_nloc, d_stale, d_eu, d_ed, d_Acc, d_g, epi);
        nloc_set = true;
    } else {
        launch_jacobian(s, P, d_recs, d_ext_pert, d_step, opt.solver_type, d_J, d_jcol, d_nloc,
                        d_stale, d_eu, d_ed, jac_ncv, d_f, CB);
    }
    if (k2_fused && jb_recompute()) {
        // the bundle pass re-evaluates the records k_jac_ne_u did not store
        epi.jb_recs = d_recs;
        epi.jb_lmder = lmder ? 1 : 0;
    }
    launch_rows_jac(s, P, d_ext, d_ext_pert, d_step, central ? d_ext_pertB : nullptr,
                    central ? d_stepB : nullptr, lmder ? 1 : 0, d_Jrow, d_eu + 2 * (size_t)M,
                    n - 1);
    if (!pre_bnd)
        launch_ne(s, P, d_J, d_jcol, d_nloc, d_f, d_Acc, d_Acg, d_Abb, d_Abg, d_Agg, d_g,
                  d_glob_partial, glob_chunk, epi, k2_fused);
    launch_rows_ne(s, P, d_Jrow, d_f + 2 * (size_t)M, d_p_own, d_Acc, d_Abb, d_Agg, d_g);
    if (nG > 0) allreduce(d_Agg, NGMAX * NGMAX + NGMAX);  // global block: all shards
    if (fuse) {
        span_end(SPAN_JAC);
        const int ncol = ncf + (nB_solved > 0 ? (nB + NE_BND_TPB - 1) / NE_BND_TPB : 0);
        RedSpec rs{};
        rs.flag_slot = -1;
        if (nranks > 1) {  // [ZERO, XN2, gnorm per rank]: one collective (see below)
            double *tail = d_Agg + NGMAX * NGMAX + NGMAX;
            MMBA_HIP(hipMemsetAsync(tail, 0, sizeof(double) * (2 + nranks), s));
            rs.row[rs.nrows++] = {0, ncol, 1, 0};
            if (epi.do_xn) rs.row[rs.nrows++] = {pw, ncol, 0, 1};
            if (epi.do_gn) rs.row[rs.nrows++] = {2 * pw, ncol, 1, 2 + rank};
            launch_reduce_multi(s, d_partial, rs, tail);
            allreduce(tail, 2 + nranks);
            launch_fold_ranks(s, tail, nranks, d_scalar + SL_ZERO, epi.do_xn, epi.do_gn);
        } else if (!tail) {
            rs.row[rs.nrows++] = {0, ncol, 1, SL_ZERO};
            if (epi.do_xn) rs.row[rs.nrows++] = {pw, ncol, 0, SL_XN2};
            if (epi.do_gn) rs.row[rs.nrows++] = {2 * pw, ncol, 1, SL_GNORM};
            if (sobs_ahead) {
                // carried by the k_schur_obs enqueued with the Jacobian ahead
                // of the decision (same rows: first = 0, gnorm)
            } else if (red_defer_ok() && !timing) {  // rides in the next k_schur_init launch
                pend_rs = rs;
                pend_red = true;
            } else {
                launch_reduce_multi(s, d_partial, rs, d_scalar);
            }
        }
    } else if (!lm) {
        launch_colnorms(s, P, d_Acc, d_Abb, d_Agg, d_acnorm, d_g);
        span_end(SPAN_JAC);
    } else {
        const int do_xn = lm->first, do_gn = lm->fnorm_sq || lm->fnorm != 0.;
        if (b15) {
            launch_b15_s(s, lm->fnorm_sq, lm->fnorm, d_b15k + 4);
            launch_b15_unrot(s, P, d_Acc, d_g, d_q15, d_adiag15, d_u15);
        }
        launch_jac_epilogue(s, P, d_Acc, d_Abb, d_Agg, d_acnorm, d_g, d_diag, dx, lm->first,
                            lm->mode, lm->fnorm, lm->fnorm_sq, do_xn, do_gn, d_p_own, d_partial,
                            nparts, pw, b15 ? d_c15 : nullptr, d_b15k + 4, d_g15, d_adiag15,
                            d_u15);
        span_end(SPAN_JAC);
        RedSpec rs{};
        rs.flag_slot = -1;
        rs.row[rs.nrows++] = {0, nparts, 1, SL_ZERO};
        if (do_xn) rs.row[rs.nrows++] = {pw, nparts, 0, SL_XN2};
        if (do_gn) rs.row[rs.nrows++] = {2 * pw, nparts, 1, SL_GNORM};
        if (nranks > 1) {
            // one collective for the three scalars: the gnorm max travels as
            // one slot per rank of a sum all-reduce and is folded after it
            double *tail = d_Agg + NGMAX * NGMAX + NGMAX;
            MMBA_HIP(hipMemsetAsync(tail, 0, sizeof(double) * (2 + nranks), s));
            RedSpec rj{};
            rj.flag_slot = -1;
            rj.row[rj.nrows++] = {0, nparts, 1, 0};
            if (do_xn) rj.row[rj.nrows++] = {pw, nparts, 0, 1};
            if (do_gn) rj.row[rj.nrows++] = {2 * pw, nparts, 1, 2 + rank};
            launch_reduce_multi(s, d_partial, rj, tail);
            allreduce(tail, 2 + nranks);
            launch_fold_ranks(s, tail, nranks, d_scalar + SL_ZERO, do_xn, do_gn);
        } else if (red_defer_ok() && !timing) {  // rides in the next k_schur_init launch (C5)
            pend_rs = rs;
            pend_red = true;
        } else {
            launch_reduce_multi(s, d_partial, rs, d_scalar);
        }
    }
    t_jac += wall_now() - t0;
}

// Trial point x + p, p = -xs (lmder): one parameter pass (step, norms,
// setParameters), measureErrors, ||J p||, one reduction launch.
void Plan::trial_enqueue(double *eu, double *ed, bool with_dnorm, bool fill_dnorm,
                         const LmDec *dec, bool jac_ahead) {
    flush_red();
    const double t0 = wall_now();
    double *pr = d_partial + 3 * (size_t)pw;  // rows 3..6 (0..2: jac epilogue)
    // the parameter pass ran in the damped solve's back substitution, or here
    const int tparts = trial_folded     ? trial_fold_parts(P, n_trial_other, trial_rec)
                       : trial_prep_rec ? trial_prep_rec_parts(P, n_prep_other)
                                        : nparts;
    if (!trial_folded && trial_prep_rec) {
        TrialFold T;
        T.x = d_x;
        T.diag = d_diag;
        T.wa1 = d_wa1;
        T.wa2 = d_wa2;
        T.wa3 = d_wa3;
        T.ext = d_ext;
        T.ext_pert = d_ext_pert;
        T.step = d_step;
        T.solver_type = opt.solver_type;
        T.delta = opt.delta;
        T.eps_dif = fd_eps();
        T.other = d_prep_other;
        T.nother = n_prep_other;
        T.partial = pr;
        T.rstride = pw;
        T.own = d_p_own;
        T.rec = 1;
        T.recs = d_recs;
        T.brec = d_brec;
        launch_trial_prep_rec(s, P, d_xs, T);
    } else if (!trial_folded) {
        launch_trial_prep(s, P, d_xs, d_x, d_diag, d_wa1, d_wa2, d_wa3, d_ext, d_ext_pert, d_step,
                          opt.solver_type, opt.delta, fd_eps(), d_p_own, pr, nparts, pw);
    }
    if (b15) launch_b15_rot(s, P, d_q15, d_wa1, d_p15);  // p in the rotated basis of J
    params_at = d_wa2;  // x <- wa2 on acceptance: the next Jacobian skips k_param_set
    if ((trial_folded && trial_rec) || (!trial_folded && trial_prep_rec))
        recs_full_at = d_wa2;  // built by the back substitution / the trial pass
    else
        records_enqueue(d_wa2, 0);  // ... and k_records
    span_begin(SPAN_RESID);
    launch_rows_eval(s, P, d_ftrial + 2 * (size_t)M, eu + 2 * (size_t)M, pr + 2 * (size_t)pw,
                     (M + 255) / 256, d_Jrow, d_wa1, pr + 3 * (size_t)pw);
    RedSpec rs{};
    rs.flag_slot = -1;
    rs.row[rs.nrows++] = {3 * pw, tparts, 0, SL_PNORM};
    rs.row[rs.nrows++] = {4 * pw, tparts, 0, SL_XN2T};
    rs.row[rs.nrows++] = {5 * pw, trial_blocks(P), 0, SL_FNORM};
    rs.row[rs.nrows++] = {6 * pw, trial_blocks(P), 0, SL_JP};
    if (fill_dnorm) {  // the undamped solve's ||D xs||^2 and fail flag (solve_damped_enqueue)
        rs.row[rs.nrows++] = {3 * pw, tparts, 0, SL_DNORM};
        rs.flag_slot = SL_FAIL;
    }
    // unsharded: the LM decision after this trial reads slots [0, SL_LAST],
    // which the reduction's last block mirrors to the host itself
    const bool mirror = host_mirror && nranks == 1;
    // tail_reduce (unsharded, compiled out): the residual pass's last workgroup
    // runs the reduction launch's work itself (RedTail: same rows, flag and
    // mirror) -- off by default, see Plan::tail_reduce
    RedTail T;
    if (nranks == 1 && tail_reduce) {
        T.on = 1;
        T.spec = rs;
        T.partial = d_partial;
        T.scalar = d_scalar;
        T.flag = fill_dnorm ? d_fail : nullptr;
        T.host = mirror ? h_scalar : nullptr;
        T.host_n = SL_LAST + 1;
        T.ticket = d_mticket;
    }
    launch_residual_jp(s, P, d_recs, d_ftrial, eu, ed, pr + 2 * (size_t)pw, d_J, d_jcol, d_nloc,
                       b15 ? d_p15 : d_wa1, pr + 3 * (size_t)pw, d_dist_t, T);
    span_end(SPAN_RESID);
    LmDec D;
    if (dec) {
        D = *dec;
        D.on = 1;
        D.s_pnorm = SL_PNORM;
        D.s_xn2t = SL_XN2T;
        D.s_fnorm = SL_FNORM;
        D.s_jp = SL_JP;
        D.s_dnorm = SL_DNORM;
        D.s_fail = SL_FAIL;
        D.s_xn2 = SL_XN2;
        D.s_gnorm = SL_GNORM;
        D.s_f0 = SL_F0;
        D.s_out = SL_DGO;
        D.gate = d_gate;
    }
    if (!T.on) {
        const bool sq = mirror && seq_poll;
        if (sq) ++seq_next;
        launch_reduce_multi(s, d_partial, rs, d_scalar, fill_dnorm ? d_fail : nullptr,
                            mirror ? h_scalar : nullptr, SL_LAST + 1, d_mticket,
                            sq ? h_seq : nullptr, seq_next, D);
        seq_pending = sq;
    }
    if (b15)  // ||J p||^2 of J = J_s + f c^T (no host mirror on these plans; rotated basis)
        launch_b15_jp(s, n, d_xs15r, d_g, d_c15r, d_b15k + 4, d_scalar + SL_JP);
    mirror_pending = mirror;
    pre_hb_enq = dec && pre_hb_on && !b15;
    if (pre_hb_enq)  // (the previous trial's kernel precedes it on s_hb[0]: no wait)
        MMBA_HIP(hipEventRecord(ev_hb[3], s));
    if (dec && jac_ahead) {  // the next Jacobian's first launch, gated on the device's decision
        stage_slots();
        pre_jac_enqueue(d_wa2, eu, ed);
    }
    if (pre_hb_enq) {  // behind the decision, beside the gated Jacobian
        MMBA_HIP(hipStreamWaitEvent(s_hb[0], ev_hb[3], 0));
        launch_handback_host(s_hb[0], Mg, nrows, d_dev_of_ref, d_f, eu, ed, pre_hb_map[0],
                             pre_hb_map[1], pre_hb_map[2], d_scalar + SL_DGO, d_ftrial);
        hb_used[0] = true;
        hb_pending = true;
    }
    // [PNORM, XN2T, FNORM, JP] (+ [DNORM, FAIL] of the undamped solve)
    allreduce(d_scalar + SL_PNORM, with_dnorm ? 6 : 4);
    t_func += wall_now() - t0;
}

// d_xs = (A + lam D^2)^-1 g; failure flag -> SL_FAIL (max over shards).
void Plan::solve_damped_enqueue(double lam, int dnorm_slot, bool defer, bool dnorm_by_trial) {
    if (nranks > 1 && path_choice(MMBA_PATH_FAULT_SHARD) == rank + 1)
        throw Invalid{"injected shard fault (MMBA_PATH_FAULT_SHARD)"};
    if (nranks > 1 && path_choice(MMBA_PATH_STALL_SHARD) == rank + 1 && !stall_done) {
        // test hook: this shard reaches its next collective only after its
        // peers' bounded waits have expired
        stall_done = true;
        std::this_thread::sleep_for(std::chrono::milliseconds(2 * (long long)comm_timeout_ms()));
    }
    if (!red_defer_ok()) flush_red();
    if (b15 && !b15_inner) {
        // B15: (M + U B U^T) xs = u + s c from M z_u = u and M z_c = c, the
        // same damped factorisation formed twice (the right-hand side rides
        // in every stage of the solve); the host loop never asks these plans
        // for a by-trial norm (Plan::solve)
        // (rotated basis: the camera-frame blocks carry lam Q D^2 Q)
        b15_inner = true;
        launch_b15_accl(s, P, d_Acc, d_q15, d_diag, lam, d_AccL, d_diagL);
        std::swap(d_Acc, d_AccL);
        std::swap(d_diag, d_diagL);
        solve_damped_enqueue(lam, -1, false, false);
        MMBA_HIP(hipMemcpyAsync(d_z15u, d_xs, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        MMBA_HIP(hipMemcpyAsync(d_b15k + 5, d_scalar + SL_FAIL, sizeof(double),
                                hipMemcpyDeviceToDevice, s));
        std::swap(d_g, d_c15r);
        solve_damped_enqueue(lam, -1, false, false);
        std::swap(d_g, d_c15r);
        std::swap(d_Acc, d_AccL);
        std::swap(d_diag, d_diagL);
        MMBA_HIP(hipMemcpyAsync(d_z15c, d_xs, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        b15_inner = false;
        launch_b15_combine(s, n, d_g, d_c15r, d_z15u, d_z15c, d_b15k + 4, d_xs15r, d_b15k,
                           d_scalar, SL_FAIL, d_b15k + 5);
        launch_b15_rot(s, P, d_q15, d_xs15r, d_xs);
        if (dnorm_slot >= 0) launch_b15_dnorm(s, n, d_xs, d_diag, d_scalar + dnorm_slot);
        (void)defer;
        (void)dnorm_by_trial;
        return;
    }
    const double t0 = wall_now();
    trial_folded = false;
    // d_fail is zero here: launch_flag_to_scalar clears it after every use
    if (band && bs.use_bd && nG == 0 && nranks == 1 && dnorm_slot >= 0) {
        // the whole damped solve, ||D xs||^2 and the flag in one launch
        span_begin(SPAN_CHOL);
        bd_direct(s, P, bs.bd, d_Acc, d_g, d_diag, lam, d_xR, d_xs, d_fail, d_scalar, dnorm_slot,
                  SL_FAIL, pend_red ? &pend_rs : nullptr, d_partial);
        pend_red = false;
        span_end(SPAN_CHOL);
        t_linear += wall_now() - t0;
        return;
    }
    if (nB_solved > 0) {
        // (folding the 3 x 3 factor into k_schur_obs, one factor per
        // observation, measured 34 us against 16 + 6 us: the per-observation
        // square roots and divisions lengthen the latency-bound pass)
        if (!(lam == 0. && lb0_valid))  // else formed by the Jacobian's bundle pass
            launch_bundle_factor(s, P, d_Abb, d_Abg, d_g, d_diag, lam, d_Lb, d_tb, d_Wg, d_fail);
        // W of this undamped solve already enqueued behind the gated Jacobian
        const bool ahead = sobs_ahead && lam == 0. && lb0_valid && !rs_bnd;
        sobs_ahead = false;
        lb0_valid = false;
        if (rs_bnd)  // W rows of the virtual observations
            launch_schur_obs_rs(s, PV, M, d_nloc, d_vobs, d_vcoff, d_J, d_Lb, d_W);
        else if (!ahead) {
            launch_schur_obs(s, P, d_J, d_Lb, d_W, pend_red ? &pend_rs : nullptr, d_partial,
                             d_scalar);
            pend_red = false;
        }
    }
    const DevProblem &PS = schur_problem();
    if (nR > 0) {
        const SView V = sview();
        // unsharded, every rhs row is written by k_schur_init
        if (nranks > 1) MMBA_HIP(hipMemsetAsync(d_rhs, 0, sizeof(double) * nRpad, s));
        // BCR leaves the band input untouched and every structural entry is
        // rewritten (diagonal blocks by k_schur_init, off-diagonal blocks
        // assigned by k_schur_dest, arrow rows by k_schur_init), so S is only
        // zeroed once at plan build; the partitioned path factors in place
        if (band && bs.red) {  // d_rhs is the tail of the block, zeroed above
            MMBA_HIP(hipMemsetAsync(bs.red, 0, sizeof(double) * (bs.red_count - nRpad), s));
        } else if (band && ((!bs.use_bcr && !bs.use_bd) || rs_bnd)) {
            // (rolling shutter with solved bundles: k_rs_offdiag writes the
            // coupling blocks, so k_schur_dest subtracts instead of assigning)
            const int nb = nR - nG;
            MMBA_HIP(hipMemsetAsync(bs.Bd, 0, sizeof(double) * (size_t)nb * (bw + 1), s));
            if (nG > 0) MMBA_HIP(hipMemsetAsync(bs.Ga, 0, sizeof(double) * (size_t)nG * nb, s));
            MMBA_HIP(hipMemsetAsync(bs.Gd, 0, sizeof(double) * NGMAX * NGMAX, s));
        } else if (dense) {
            MMBA_HIP(hipMemsetAsync(d_S, 0, sizeof(double) * (size_t)(nRpad + 1) * dld, s));
        } else if (!band) {
            MMBA_HIP(hipMemsetAsync(d_S, 0, sizeof(double) * (size_t)nslots * TILE * TILE, s));
        }
        const bool fold = fold_init && nB_solved > 0;
        if (!fold) {
            launch_schur_init(s, P, d_Acc, d_Acg, d_Agg, d_g, d_diag, lam, V, nRpad - nR, d_rhs,
                              pend_red ? &pend_rs : nullptr, d_partial, d_scalar);
            pend_red = false;
        }
        flush_red();
        if (nB_solved > 0) {
            if (use_dest) {
                // unsharded uniform plans fold the rhs update into the
                // diagonal destinations (and, with fold, the whole of
                // k_schur_init: one launch less per damped solve)
                SchurInitFold fi{};
                if (fold) fi = SchurInitFold{1, d_Acc, d_g, d_diag, lam};
                const bool rhs_done =
                    launch_schur_dest(s, PS, d_W, d_dest, d_dest_off, ndest, d_dpairs, V,
                                      pc_uniform, band && bs.use_bcr && !rs_bnd, d_tb, d_rhs, fi,
                                      d_dest_wave, n_dest_wave, d_dest_lane, n_dest_lane);
                if (!rhs_done) launch_schur_rhs(s, PS, d_W, d_tb, d_row_cf, d_rhs);
                launch_schur_glob(s, PS, d_W, d_Wg, d_tb, V, d_rhs);
            } else {
                launch_schur_pairs(s, PS, d_W, d_Wg, d_tb, V, d_rhs);
            }
        }
        if (dbg_keep_S && dense) {  // mmba_debug_reduced_residual: S and r before the factor
            MMBA_HIP(hipMemcpyAsync(d_Skeep, ds.A, sizeof(double) * (size_t)ds.ld * (ds.n + 1),
                                    hipMemcpyDeviceToDevice, s));
            MMBA_HIP(hipMemcpyAsync(d_rkeep, d_rhs, sizeof(double) * nRpad, hipMemcpyDeviceToDevice,
                                    s));
        }
        span_begin(SPAN_CHOL);
        if (band && bs.use_bd) {  // factor, forward and backward
            bd_factor_solve(s, bs.bd, d_fail, d_rhs, d_yR, d_xR, d_xs);
        } else if (band) {
            if (bs.red) allreduce(bs.red, bs.red_count);
            if (bs.use_pcr && !bs.df_off)  // the whole solve: x, scattered when unsharded
                pcr_solve(s, bs.pcr, d_rhs, d_xR, bs.pcr.row_param ? d_xs : nullptr, d_fail);
            else
                band_factor_forward(s, bs, d_fail, d_probe, d_rhs, d_yR);
        } else if (dense) {
            if (nranks > 1) {  // each shard's rows of S and r, summed (shard_dense)
                allreduce(d_S, (size_t)ds.ld * (ds.n + 1));
                allreduce(d_rhs, nRpad);
            }
            ds.factor_forward(s, d_rhs, d_yR, d_fail);  // y = L^-1 rhs rides along
        } else {
            for (int k = 0; k < NT; ++k) {
                const int r0 = panel_rows_off[k], nr = panel_rows_off[k + 1] - r0;
                launch_chol_panel(s, d_S, d_slot, NT, k, d_rows + r0, nr, d_Linv, d_fail);
                const int q0 = panel_pairs_off[k], nq = panel_pairs_off[k + 1] - q0;
                launch_chol_update(s, d_S, d_slot, NT, k, d_pairs + q0, nq);
            }
        }
        span_end(SPAN_CHOL);
        if (band && bs.use_bd) {
            // solved and scattered to parameter order above
        } else if (band && bs.use_pcr && !bs.df_off) {
            // solved by pcr_solve
        } else if (band) {
            band_backward(s, bs, d_yR, d_xR);
            // every shard needs its halo camera-frame rows: each shard's own
            // rows [Ra, Rb) (and shard 0's arrow rows) all-gathered
            if (nranks > 1 && !bs.use_bcr) gather_step_rows();
        } else if (dense) {
            ds.backward(s, d_yR, d_xR);
        } else if (narrow) {
            launch_trsv_fwd_all(s, d_S, d_slot, NT, d_rows_off, d_rows, d_Linv, d_rhs, d_yR);
            launch_trsv_bwd_all(s, d_S, d_slot, NT, d_cols_off, d_cols, d_Linv, d_yR, d_xR);
        } else {
            for (int k = 0; k < NT; ++k) {
                const int r0 = panel_rows_off[k], nr = panel_rows_off[k + 1] - r0;
                launch_trsv_fwd(s, d_S, d_slot, NT, k, d_rows + r0, nr, d_Linv, d_rhs, d_yR);
            }
            for (int k = NT - 1; k >= 0; --k) {
                const int c0 = panel_cols_off[k], nc = panel_cols_off[k + 1] - c0;
                launch_trsv_bwd(s, d_S, d_slot, NT, k, d_cols + c0, nc, d_Linv, d_yR, d_xR);
            }
        }
        // else done by the BCR backward solve / the block-diagonal back substitution
        const bool pcr_now = band && bs.use_pcr && !bs.df_off;
        if (!(band && ((bs.use_bcr && !pcr_now && bs.bcr.xs) || (pcr_now && bs.pcr.row_param) ||
                       bs.use_bd)))
            launch_scatter_xR(s, P, d_xR, d_xs);
    }
    trial_folded = false;
    if (nB_solved > 0) {
        if (trial_fold_ok) {
            // the trial point's parameter pass rides in the back substitution
            // (the last damped solve before a trial is the one it keeps)
            // one pass (MMBA_PATH_BACKSUB_ONEPASS = 1): the bundle threads form
            // u_i = W_i^T x_cf(i) themselves (the same sums), no k_obs_wtx --
            // measured slower on C4 (4,299 against 4,406 LM it/s, same box,
            // profiles/r6_ab2/: the gathered 144-B W rows), so opt-in
            const bool onepass = path_choice(MMBA_PATH_BACKSUB_ONEPASS) == 1;
            if (!onepass) launch_obs_wtx(s, PS, d_W, d_xR, d_U);
            TrialFold T;
            T.x = d_x;
            T.diag = d_diag;
            T.wa1 = d_wa1;
            T.wa2 = d_wa2;
            T.wa3 = d_wa3;
            T.ext = d_ext;
            T.ext_pert = d_ext_pert;
            T.step = d_step;
            T.solver_type = opt.solver_type;
            T.delta = opt.delta;
            T.eps_dif = fd_eps();
            T.other = d_trial_other;
            T.nother = n_trial_other;
            T.partial = d_partial + 3 * (size_t)pw;
            T.rstride = pw;
            T.own = d_p_own;
            T.rec = trial_rec ? 1 : 0;
            T.recs = d_recs;
            T.brec = d_brec;
            launch_backsub_trial(s, PS, onepass ? d_W : nullptr, d_Wg, d_tb, d_Lb, d_xR, d_U, d_xs, T);
            trial_folded = true;
            params_at = nullptr;  // the attribute block now holds the trial point
            recs_full_at = nullptr;
        } else {
            launch_backsub_bundle(s, PS, d_W, d_Wg, d_tb, d_Lb, d_xR, d_U, d_xs);
        }
    }
    if (dnorm_by_trial) {
        // the speculative trial's ||D p||^2 (p = -xs, same partial blocks and
        // order as k_sumsq: bit-identical) becomes ||D xs||^2, and its
        // reduction also converts the fail flag (trial_enqueue)
        t_linear += wall_now() - t0;
        return;
    }
    if (dnorm_slot < 0) {
        launch_flag_to_scalar(s, d_fail, d_scalar + SL_FAIL);
    } else {  // ||D xs||^2 and the fail flag in one reduction launch
        double *pr = d_partial + 7 * (size_t)pw;
        launch_sumsq(s, d_xs, d_diag, n, pr, nparts, nullptr, d_p_own);
        RedSpec rs{};
        rs.flag_slot = SL_FAIL;
        rs.row[rs.nrows++] = {7 * pw, nparts, 0, dnorm_slot};
        launch_reduce_multi(s, d_partial, rs, d_scalar, d_fail);
    }
    if (dnorm_slot == SL_DNORM) {
        if (!defer) allreduce(d_scalar + SL_DNORM, 2);  // [DNORM, FAIL]
    } else {
        if (dnorm_slot >= 0) allreduce(d_scalar + dnorm_slot, 1);
        allreduce(d_scalar + SL_FAIL, 1);
    }
    t_linear += wall_now() - t0;
}

bool Plan::solve_damped(double lam) {
    solve_damped_enqueue(lam);
    return read_scalar(SL_FAIL) == 0.;
}

// v^T (A + lam D^2)^-1 v with v = D^2 xs / dxnorm, using the current
// factorisation (lmpar's parl / parc denominators): bundle part -> SL_NEWT_B,
// reduced part -> SL_NEWT_R.
void Plan::newton_enqueue(double dxnorm) {
    const double t0 = wall_now();
    launch_newton_v(s, n, d_diag, d_xs, dxnorm, d_v);
    if (b15) {  // v in the rotated basis of the factorisation
        launch_b15_rot(s, P, d_q15, d_v, d_v15);
        std::swap(d_v, d_v15);
    }
    MMBA_HIP(hipMemsetAsync(d_scalar + SL_NEWT_B, 0, 2 * sizeof(double), s));
    if (nR > 0) launch_gather_R(s, P, d_v, d_wR, nRpad);
    if (nB_solved > 0) {
        launch_newton_bundle(s, schur_problem(), d_W, d_Wg, d_Lb, d_v, d_wR, d_usq, d_nu, d_ngp);
        launch_reduce_sum(s, d_usq, nB, d_scalar + SL_NEWT_B);
    }
    if (nR > 0) {
        if (band && bs.use_pcr && !bs.df_off) {
            // w^T S^-1 w (= ||L^-1 w||^2 of any Cholesky of S) from the last
            // solve's factors: per-block partials, summed in block order
            pcr_rhs_dot(s, bs.pcr, d_wR, d_ymask, d_fail);
            launch_reduce_sum(s, bs.pcr.part, bs.pcr.nblk, d_scalar + SL_NEWT_R);
        } else if (band && bs.use_bd) {
            bd_forward(s, bs.bd, d_wR, d_yR);
        } else if (band) {
            band_forward(s, bs, d_wR, d_yR);
        } else if (dense) {
            ds.forward(s, d_wR, d_yR);
        } else if (narrow) {
            launch_trsv_fwd_all(s, d_S, d_slot, NT, d_rows_off, d_rows, d_Linv, d_wR, d_yR);
        } else {
            for (int k = 0; k < NT; ++k) {
                const int r0 = panel_rows_off[k], nr = panel_rows_off[k + 1] - r0;
                launch_trsv_fwd(s, d_S, d_slot, NT, k, d_rows + r0, nr, d_Linv, d_wR, d_yR);
            }
        }
        if (band && bs.pcr_int && !bs.df_off)
            launch_sumsq_mix(s, d_yR, d_wR, nR, d_partial, nparts, d_scalar + SL_NEWT_R, d_ymask);
        else if (!(band && bs.use_pcr && !bs.df_off))
            launch_sumsq(s, d_yR, nullptr, nRpad, d_partial, nparts, d_scalar + SL_NEWT_R,
                         d_ymask, d_ticket);
    }
    // B15: v^T (M + U B U^T)^-1 v = v^T M^-1 v - w^T K^-1 w (the factor and
    // z_u, z_c of the last damped solve)
    if (b15) {
        launch_b15_newton(s, n, d_v, d_z15u, d_z15c, d_b15k, d_scalar + SL_NEWT_B);
        std::swap(d_v, d_v15);  // back to the original basis buffer
    }
    allreduce(d_scalar + SL_NEWT_B, 2);
    t_linear += wall_now() - t0;
}

// lmpar restated on normal equations (see oracle/refcpu.c lmpar).  Every
// decision point reads its scalars with one synchronisation.
// pre: the undamped solve and its ||D x|| were enqueued and read already
// (lmpar_first_enqueue); *undamped is set when lmpar returns that step.
static void lmpar_first_enqueue(Plan &pl, bool defer = false, bool by_trial = false) {
    pl.solve_damped_enqueue(0.0, Plan::SL_DNORM, defer, by_trial);
}

// A timed-out wait in a parallel-cyclic-reduction right-hand-side pass (the
// Newton term's k_pcr_rhs / k_pcr_rhs_mc) leaves NaN partials instead of
// stale ones: the plan switches to the band chains for good (the flag bit
// is cleared) and lmpar starts over from its first, undamped solve.
struct PcrRestart {};
static void check_newton(Plan &pl) {
    if (std::isfinite(pl.h_scalar[Plan::SL_NEWT_R])) return;
    if (!(pl.band && (pl.bs.use_pcr || pl.bs.pcr_int)) || pl.bs.df_off) return;
    pl.bs.df_off = true;
    launch_flag_to_scalar(pl.s, pl.d_fail, pl.d_scalar + Plan::SL_FAIL);
    throw PcrRestart{};
}

// A timed-out dataflow wait in the undamped solve (flag bit 2) switches the
// plan to the per-level launches and solves again; `pre` is cleared then, so
// the caller does not take the speculative trial built on the failed solve.
static double lmpar_ne_once(Plan &pl, double delta, double *par, bool &pre, bool *undamped) {
    const double p1 = .1, p001 = .001;
    const double dwarf = DBL_MIN;
    double *h = pl.h_scalar;
    int iter = 0;
    *undamped = false;
    if (!pre) {
        lmpar_first_enqueue(pl);
        pl.read_slots(Plan::SL_DNORM, Plan::SL_FAIL);
    }
    if (h[Plan::SL_FAIL] >= 2. && !pl.bs.df_off) {
        pl.bs.df_off = true;
        pre = false;
        lmpar_first_enqueue(pl);
        pl.read_slots(Plan::SL_DNORM, Plan::SL_FAIL);
    }
    const bool ok0 = h[Plan::SL_FAIL] == 0.;
    double dxnorm = ok0 ? std::sqrt(h[Plan::SL_DNORM]) : HUGE_VAL;
    double fp = dxnorm - delta;
    if (fp <= p1 * delta) {
        if (iter == 0) *par = 0.;
        *undamped = true;
        return dxnorm;
    }
    double parl = 0.;
    const bool newton0 = !pl.rank_deficient && ok0;
    if (newton0) pl.newton_enqueue(dxnorm);
    launch_sumsq_div(pl.s, pl.b15 ? pl.d_g15 : pl.d_g, pl.d_diag, pl.n, pl.d_partial, pl.nparts,
                     pl.d_scalar + Plan::SL_GDIV, pl.d_p_own, pl.d_ticket);
    pl.allreduce(pl.d_scalar + Plan::SL_GDIV, 1);
    pl.read_slots(Plan::SL_NEWT_B, Plan::SL_GDIV);
    if (newton0) check_newton(pl);
    if (newton0) {
        const double temp = std::sqrt(h[Plan::SL_NEWT_B] + h[Plan::SL_NEWT_R]);
        parl = fp / delta / temp / temp;
    }
    const double gnorm = std::sqrt(h[Plan::SL_GDIV]);
    double paru = gnorm / delta;
    if (paru == 0.) paru = dwarf / std::min(delta, p1);
    *par = std::max(*par, parl);
    *par = std::min(*par, paru);
    if (*par == 0.) *par = gnorm / dxnorm;
    for (;;) {
        ++iter;
        if (*par == 0.) *par = std::max(dwarf, p001 * paru);
        pl.solve_damped_enqueue(*par, Plan::SL_DNORM);
        pl.read_slots(Plan::SL_DNORM, Plan::SL_FAIL);
        // (A + par D^2) is positive definite for par > 0, so a failed damped
        // factorisation is a numerical breakdown (or, bit 2, a timed-out
        // dataflow wait in the block cyclic reduction): never use its stale
        // step.  Raise par (a larger damping is better conditioned) a few
        // times, then give up with an error.
        for (int retry = 0; h[Plan::SL_FAIL] != 0.; ++retry) {
            if (h[Plan::SL_FAIL] >= 2. && !pl.bs.df_off) {
                // a timed-out dataflow wait (bit 2): the plan switches to the
                // per-level launches for good and this damped solve runs again
                pl.bs.df_off = true;
                pl.solve_damped_enqueue(*par, Plan::SL_DNORM);
                pl.read_slots(Plan::SL_DNORM, Plan::SL_FAIL);
                continue;
            }
            if (h[Plan::SL_FAIL] >= 2. || retry == 8) {
                set_error("damped normal-equation factorisation failed (par " +
                          std::to_string(*par) + ", flag " + std::to_string(h[Plan::SL_FAIL]) +
                          ")");
                throw DeviceError();
            }
            *par *= 10.;
            pl.solve_damped_enqueue(*par, Plan::SL_DNORM);
            pl.read_slots(Plan::SL_DNORM, Plan::SL_FAIL);
        }
        dxnorm = std::sqrt(h[Plan::SL_DNORM]);
        double temp = fp;
        fp = dxnorm - delta;
        if (std::fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) || iter == 10)
            break;
        pl.newton_enqueue(dxnorm);
        pl.read_slots(Plan::SL_NEWT_B, Plan::SL_NEWT_R);
        check_newton(pl);
        temp = std::sqrt(h[Plan::SL_NEWT_B] + h[Plan::SL_NEWT_R]);
        const double parc = fp / delta / temp / temp;
        if (fp > 0.) parl = std::max(parl, *par);
        if (fp < 0.) paru = std::min(paru, *par);
        *par = std::max(parl, *par + parc);
    }
    if (iter == 0) *par = 0.;
    return dxnorm;
}

static double lmpar_ne(Plan &pl, double delta, double *par, bool &pre, bool *undamped) {
    const double par0 = *par;
    for (;;) {
        try {
            return lmpar_ne_once(pl, delta, par, pre, undamped);
        } catch (const PcrRestart &) {
            *par = par0;
            pre = false;
        }
    }
}

// Device order -> reference (errorToMarkerList) order on the host.  Sharded:
// every shard scatters the observations it owns and the shards' buffers are
// summed, so every shard returns the full vectors.
void Plan::download_ref_order(const double *d_f2, const double *d_eu2, const double *d_ed1,
                              double *f_out, double *eu_out, double *ed_out, bool sync) {
    if (nranks > 1) {  // each shard's own observations (mmba_group.cpp)
        handback_sharded(nullptr, nullptr, f_out, eu_out, ed_out, d_f2, d_eu2, d_ed1);
        return;
    }
    handback_wait();  // (a hand-back an exception left in flight still reads d_gather)
    handback_streams();
    // page-locked caller lists (hipHostMalloc / hipHostRegister, 16-B
    // aligned): one kernel stores them in reference order through their
    // host-mapped addresses, on its own stream beside whatever follows on s
    double *hmap[3] = {nullptr, nullptr, nullptr};
    if (map_outputs(f_out, eu_out, ed_out, hmap)) {
        MMBA_HIP(hipEventRecord(ev_hb[3], s));
        MMBA_HIP(hipStreamWaitEvent(s_hb[0], ev_hb[3], 0));
        launch_handback_host(s_hb[0], Mg, nrows, d_dev_of_ref, d_f2, d_eu2, d_ed1, hmap[0],
                             hmap[1], hmap[2]);
        hb_used[0] = true;
        hb_pending = true;
        if (sync) handback_wait();
        return;
    }
    double *tf = d_gather, *te = d_gather + mg, *td = d_gather + 2 * (size_t)mg;
    const size_t total = 2 * (size_t)mg + Mg;
    if (nranks > 1) MMBA_HIP(hipMemsetAsync(d_gather, 0, sizeof(double) * total, s));
    launch_unpermute(s, M, d_ref_of_dev, P.obs_own, f_out ? d_f2 : nullptr,
                     eu_out ? d_eu2 : nullptr, ed_out ? d_ed1 : nullptr, tf, te, td);
    allreduce(d_gather, total);
    if (nrows > 0) {  // stiffness / smoothness rows: identical on every shard
        if (f_out)
            MMBA_HIP(hipMemcpyAsync(tf + 2 * (size_t)Mg, d_f2 + 2 * (size_t)M,
                                    sizeof(double) * nrows, hipMemcpyDeviceToDevice, s));
        if (eu_out)
            MMBA_HIP(hipMemcpyAsync(te + 2 * (size_t)Mg, d_eu2 + 2 * (size_t)M,
                                    sizeof(double) * nrows, hipMemcpyDeviceToDevice, s));
    }
    // the three lists on three streams (measured on C2's 8 MB: one stream
    // runs the copies back to back with ~9 us between them; tools/ubench/d2h)
    MMBA_HIP(hipEventRecord(ev_hb[3], s));
    double *dst[3] = {f_out, eu_out, ed_out};
    const double *src[3] = {tf, te, td};
    const size_t cnt[3] = {(size_t)mg, (size_t)mg, (size_t)Mg};
    for (int k = 0; k < 3; ++k) {
        if (!dst[k]) continue;
        MMBA_HIP(hipStreamWaitEvent(s_hb[k], ev_hb[3], 0));
        MMBA_HIP(hipMemcpyAsync(dst[k], src[k], sizeof(double) * cnt[k], hipMemcpyDeviceToHost,
                                s_hb[k]));
        hb_used[k] = true;
    }
    hb_pending = true;
    if (sync) handback_wait();
}

void Plan::handback_streams() {
    if (s_hb[0]) return;
    for (hipStream_t &c : s_hb) MMBA_HIP(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    for (hipEvent_t &e : ev_hb) MMBA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

bool Plan::map_outputs(double *f_out, double *eu_out, double *ed_out, double *hmap[3]) {
    // opt-in (MMBA_PATH_HANDBACK_DMA = 0): on C2 the three DMA copies on their
    // own streams measured 6,498 / 6,513 LM it/s against 6,266 / 6,275 for the
    // host-mapped stores with the speculative launch and 6,338 / 6,688 without
    // it, on one box (profiles/r6_c2hb/) -- the stores' PCIe-bound waves slow
    // the kernels beside them
    if (!d_dev_of_ref || path_choice(MMBA_PATH_HANDBACK_DMA) != 0) return false;
    double *outs3[3] = {f_out, eu_out, ed_out};
    for (int k = 0; k < 3; ++k) {
        hmap[k] = nullptr;
        if (!outs3[k]) continue;
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, outs3[k]) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory: not an error of the solve
            return false;
        }
        if (a.type != hipMemoryTypeHost || !a.devicePointer ||
            (k < 2 && ((uintptr_t)a.devicePointer & 15u)))
            return false;
        hmap[k] = static_cast<double *>(a.devicePointer);
    }
    return true;
}

// The hand-back's copies done (polled events: a blocking synchronisation's
// wake-up costs tens of microseconds).
void Plan::handback_wait() {
    if (!hb_pending) return;
    hb_pending = false;
    for (int k = 0; k < 3; ++k)
        if (hb_used[k]) MMBA_HIP(hipEventRecord(ev_hb[k], s_hb[k]));
    for (int k = 0; k < 3; ++k)
        for (; hb_used[k];) {
            const hipError_t e = hipEventQuery(ev_hb[k]);
            if (e == hipSuccess) hb_used[k] = false;
            else if (e != hipErrorNotReady) MMBA_HIP(e);
        }
}

// Parameter vector of the solve on the host (sharded: owners' entries summed).
void Plan::download_params(const double *dx, double *x_out) {
    if (nranks > 1) {  // each shard's own parameters (mmba_group.cpp)
        handback_sharded(dx, x_out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
        return;
    }
    MMBA_HIP(hipMemcpyAsync(x_out, dx, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    host_sync();
}

void Plan::error_stats_enqueue(const double *ed, int base) {
    launch_dist_stats(s, P, ed, d_partial, nparts, pw, d_scalar + base);
    allreduce(d_scalar + base, 1);
    allreduce(d_scalar + base + 1, 2, ReduceOp::Max);
}

void Plan::error_stats_device(const double *ed, double *avg, double *mn, double *mx) {
    error_stats_enqueue(ed);
    read_slots(SL_ESUM, SL_EMAX);
    *avg = h_scalar[SL_ESUM] / Mg;
    *mn = -h_scalar[SL_ENMIN];
    *mx = h_scalar[SL_EMAX];
}

static void error_stats(const double *dist, int M, double *avg, double *mn, double *mx) {
    double a = 0., lo = DBL_MAX, hi = -0.0;
    for (int i = 0; i < M; ++i) {
        const double e = dist[i];
        if (!std::isfinite(e)) continue;
        a += e;
        if (e < lo) lo = e;
        if (e > hi) hi = e;
    }
    a /= M;
    *avg = a;
    *mn = lo;
    *mx = hi;
}

int Plan::measure(const double *x, double *fvec_out, double *eu_out, double *ed_out,
                  double *stats) {
    // an epilogue reduction a previous entry point deferred (pend_red) reads
    // d_partial rows this call rewrites: dropped, its slots are not read
    // outside the solve that deferred it
    pend_red = false;
    attrs_reset();
    if (x) {
        MMBA_HIP(hipMemcpyAsync(d_x, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
        fun(d_x, d_f, d_eu, d_ed);
    } else {
        records_enqueue(nullptr, 1);
        launch_rows_eval(s, P, d_f + 2 * (size_t)M, d_eu + 2 * (size_t)M, d_partial,
                         (M + 255) / 256);
        launch_residual(s, plug_problem(), d_recs, d_f, d_eu, d_ed, d_partial);
    }
    if (nranks > 1) {
        // sharded: the statistics all-reduced, the outputs handed back by
        // each shard's own observations
        double st[3];
        error_stats_device(d_ed, &st[0], &st[1], &st[2]);
        if (stats) std::memcpy(stats, st, sizeof(st));
        if (fvec_out || eu_out || ed_out)
            download_ref_order(d_f, d_eu, d_ed, fvec_out, eu_out, ed_out);
        collect_spans();
        return MMBA_OK;
    }
    std::vector<double> ed(Mg);
    download_ref_order(d_f, d_eu, d_ed, fvec_out, eu_out, ed.data());
    if (ed_out) std::memcpy(ed_out, ed.data(), sizeof(double) * Mg);
    if (stats) error_stats(ed.data(), Mg, &stats[0], &stats[1], &stats[2]);
    collect_spans();
    return MMBA_OK;
}

// Per-observation reprojected point and corrected marker at x (caller's
// observation order); the scratch trial buffers carry them (no solve runs).
int Plan::reproject(const double *x, double *point_out, double *marker_out) {
    // an epilogue reduction a previous entry point deferred (pend_red) reads
    // d_partial rows this call rewrites: dropped, its slots are not read
    // outside the solve that deferred it
    pend_red = false;
    attrs_reset();
    if (x) {
        MMBA_HIP(hipMemcpyAsync(d_x, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
        fun(d_x, d_f, d_eu, d_ed);  // parameters set, records current
        launch_reproject(s, P, d_recs, d_ftrial, d_eu_s);
    } else {
        records_enqueue(nullptr, 1);
        launch_reproject(s, plug_problem(), d_recs, d_ftrial, d_eu_s);
    }
    download_ref_order(d_ftrial, d_eu_s, d_ed_s, point_out, marker_out, nullptr);
    return MMBA_OK;
}

// Dense reference-order Jacobian at x (column-major, ldfjac = m); for tests
// and small problems only.
int Plan::dense_jacobian(const double *x, double *fjac) {
    // an epilogue reduction a previous entry point deferred (pend_red) reads
    // d_partial rows this call rewrites: dropped, its slots are not read
    // outside the solve that deferred it
    pend_red = false;
    if (nranks > 1) throw Unsupported{"dense Jacobian of a sharded plan"};
    attrs_reset();
    MMBA_HIP(hipMemcpyAsync(d_x, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
    fun(d_x, d_f, d_eu, d_ed);
    const int implicit = P.jcol_implicit;
    P.jcol_implicit = 0;  // this host-side reassembly reads jcol
    jac(d_x);
    P.jcol_implicit = implicit;
    std::vector<double> J((size_t)2 * P.lmax * M), Jr(nrows);
    std::vector<int> jc((size_t)std::max(P.lmax, 1) * M), nl(M), rp(nrows);
    if (nrows > 0) {
        MMBA_HIP(hipMemcpyAsync(Jr.data(), d_Jrow, sizeof(double) * nrows, hipMemcpyDeviceToHost,
                                s));
        MMBA_HIP(hipMemcpyAsync(rp.data(), P.row_param, sizeof(int) * nrows,
                                hipMemcpyDeviceToHost, s));
    }
    if (b15) launch_b15_unrot_J(s, P, d_J, d_q15);  // back to the original basis
    MMBA_HIP(hipMemcpyAsync(J.data(), d_J, sizeof(double) * J.size(), hipMemcpyDeviceToHost, s));
    MMBA_HIP(hipMemcpyAsync(jc.data(), d_jcol, sizeof(int) * jc.size(), hipMemcpyDeviceToHost, s));
    MMBA_HIP(hipMemcpyAsync(nl.data(), d_nloc, sizeof(int) * M, hipMemcpyDeviceToHost, s));
    host_sync();
    collect_spans();
    std::memset(fjac, 0, sizeof(double) * (size_t)m * n);
    for (int i = 0; i < M; ++i) {
        const int r = ref_of_dev[i];
        for (int l = 0; l < nl[i]; ++l) {
            const int p = jc[(size_t)l * M + i];
            fjac[(size_t)p * m + 2 * r] = J[(size_t)(2 * l) * M + i];
            fjac[(size_t)p * m + 2 * r + 1] = J[(size_t)(2 * l + 1) * M + i];
        }
    }
    for (int r = 0; r < nrows; ++r)
        if (rp[r] >= 0) fjac[(size_t)rp[r] * m + 2 * (size_t)M + r] = Jr[r];
    if (b15) {  // J = J_s + f c^T
        std::vector<double> c(n), f(2 * (size_t)M);
        MMBA_HIP(hipMemcpy(c.data(), d_c15, sizeof(double) * n, hipMemcpyDeviceToHost));
        MMBA_HIP(hipMemcpy(f.data(), d_f, sizeof(double) * f.size(), hipMemcpyDeviceToHost));
        for (int p = 0; p < n; ++p) {
            if (c[p] == 0.) continue;
            for (int i = 0; i < M; ++i) {
                const int r = ref_of_dev[i];
                fjac[(size_t)p * m + 2 * r] += f[2 * (size_t)i] * c[p];
                fjac[(size_t)p * m + 2 * r + 1] += f[2 * (size_t)i + 1] * c[p];
            }
        }
    }
    return MMBA_OK;
}

// ||S x - r||^2 and ||r||^2 of a dense symmetric S (lower triangle,
// column-major, ld): one thread per row, the lower part read down its row
// (coalesced across threads), the upper part from its own column.
__global__ void k_dense_symv_res(const double *__restrict__ A, int ld, int n,
                                 const double *__restrict__ x, const double *__restrict__ r,
                                 double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.;
    if (i < n) {
        for (int j = 0; j <= i; ++j) acc = fma(A[(size_t)j * ld + i], x[j], acc);
        for (int j = i + 1; j < n; ++j) acc = fma(A[(size_t)i * ld + j], x[j], acc);
        const double d = acc - r[i];
        atomicAdd(&out[0], d * d);
        atomicAdd(&out[1], r[i] * r[i]);
    }
}

int Plan::reduced_residual(const double *x, double lam, double *relres) {
    // an epilogue reduction a previous entry point deferred (pend_red) reads
    // d_partial rows this call rewrites: dropped, its slots are not read
    // outside the solve that deferred it
    pend_red = false;
    if (!dense) throw Unsupported{"reduced residual hook: dense reduced plans only"};
    if (!d_Skeep) {
        d_Skeep = dalloc<double>((size_t)ds.ld * (ds.n + 1));
        d_rkeep = dalloc<double>(nRpad);
    }
    attrs_reset();
    MMBA_HIP(hipMemcpyAsync(d_x, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
    MMBA_HIP(hipMemsetAsync(d_diag, 0, sizeof(double) * n, s));
    fun(d_x, d_f, d_eu, d_ed);
    const JacLM lm{1, 1, 1.0, nullptr};
    jac(d_x, &lm);
    dbg_keep_S = true;
    try {
        solve_damped_enqueue(lam, SL_DNORM);
    } catch (...) {
        dbg_keep_S = false;
        throw;
    }
    dbg_keep_S = false;
    double *acc = dalloc<double>(2);
    MMBA_HIP(hipMemsetAsync(acc, 0, 2 * sizeof(double), s));
    k_dense_symv_res<<<(nR + 255) / 256, 256, 0, s>>>(d_Skeep, ds.ld, nR, d_xR, d_rkeep, acc);
    double h[2];
    MMBA_HIP(hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, s));
    host_sync();
    read_slots(SL_DNORM, SL_FAIL);
    if (h_scalar[SL_FAIL] != 0.) throw Invalid{"reduced residual hook: the factorisation failed"};
    *relres = std::sqrt(h[0] / h[1]);
    collect_spans();
    return MMBA_OK;
}

// Columns [0, k) of an interrupted lmder Jacobian were measured: recompute
// errorList / errorDistanceList as the last of them left them (B13 with the
// stale-column table cut at k; lmdif measured every frame per column).
void Plan::jac_partial_stale(const double *dx, int k) {
    std::vector<int> st(F, -1);
    const bool lmdif = opt.solver_type == MMBA_SOLVER_CMINPACK_LMDIF;
    for (int f = 0; f < F; ++f) {
        if (lmdif) {
            st[f] = k - 1;
            continue;
        }
        for (int p = k - 1; p >= 0; --p)
            if (param_frame_host[p] < 0 || param_frame_host[p] == f ||
                (rs_on && std::abs(param_frame_host[p] - f) <= 1)) {
                st[f] = p;
                break;
            }
    }
    MMBA_HIP(hipMemcpyAsync(d_stale, st.data(), sizeof(int) * F, hipMemcpyHostToDevice, s));
    const double eps_dif = fd_eps();
    launch_param_set(s, P, dx, d_ext, d_ext_pert, d_step, opt.solver_type, opt.delta, eps_dif);
    params_at = dx;
    records_enqueue(dx, 0);
    CentralB CB;
    if (central) {
        MMBA_HIP(hipMemsetAsync(d_scalar + SL_NCENT, 0, sizeof(double), s));
        launch_param_central(s, P, dx, d_ext_pertB, d_stepB, opt.delta, d_scalar + SL_NCENT);
        launch_records(s, P, d_var_cf, d_ext_pertB, d_stepB, d_recsB, nvar, d_brecB, 0);
        CB.recs = d_recsB;
        CB.brec = d_brecB;
        CB.ext_pert = d_ext_pertB;
        CB.step = d_stepB;
    }
    // the generic kernel honours the stale table for every column
    launch_jacobian(s, P, d_recs, d_ext_pert, d_step, opt.solver_type, d_J, d_jcol, d_nloc,
                    d_stale, d_eu, d_ed, 0, d_f, CB);
    launch_rows_jac(s, P, d_ext, d_ext_pert, d_step, central ? d_ext_pertB : nullptr,
                    central ? d_stepB : nullptr, lmdif ? 0 : 1, d_Jrow, d_eu + 2 * (size_t)M,
                    k - 1);
    MMBA_HIP(hipMemcpyAsync(d_stale, stale_host.data(), sizeof(int) * F, hipMemcpyHostToDevice,
                            s));
}

// The solve; a speculative Jacobian that the host's decision does not take
// (SpecMismatch: the device's restatement of the lmder decision disagreed
// with the host's, which the kernels are written never to do) is not an
// error: the solve is replayed from x0 with the Jacobian enqueued only after
// the host's decisions (same kernels, same bits as an unspeculated solve;
// no callback can have run, pre_jac_ok requires none) and the event is
// counted in mmba_kernel_stats.spec_replays.
int Plan::solve(double *x_inout, double *fvec_out, double *eu_out, double *ed_out,
                mmba_result *res, const mmba_callbacks *cb, mmba_trace *trace) {
    try {
        return solve_once(x_inout, fvec_out, eu_out, ed_out, res, cb, trace);
    } catch (const SpecMismatch &) {
        host_sync();
        ++spec_replays;
        pre_jac_pending = false;
        pre_bnd_pending = false;
        pre_sobs_pending = false;
        sobs_ahead = false;
        seq_pending = false;
        mirror_pending = false;
        slots_staged = false;
        params_at = nullptr;
        recs_full_at = nullptr;
        const bool keep = pre_jac;
        pre_jac = false;
        int rc;
        try {
            rc = solve_once(x_inout, fvec_out, eu_out, ed_out, res, cb, trace);
        } catch (...) {
            pre_jac = keep;
            throw;
        }
        pre_jac = keep;
        return rc;
    }
}

int Plan::solve_once(double *x_inout, double *fvec_out, double *eu_out, double *ed_out,
                     mmba_result *res, const mmba_callbacks *cb, mmba_trace *trace) {
    // an epilogue reduction a previous entry point deferred (pend_red) reads
    // d_partial rows this call rewrites: dropped, its slots are not read
    // outside the solve that deferred it
    pend_red = false;
    const double t_start = wall_now();
    t_func = t_jac = t_linear = 0.;
    cbk = cb;
    pre_hb_enq = false;
    pre_sobs_pending = sobs_ahead = false;
    pre_hb_on = nranks == 1 && n > 0 && pre_jac && (fvec_out || eu_out || ed_out) &&
                path_choice(MMBA_PATH_PRE_HANDBACK) != 0 &&
                map_outputs(fvec_out, eu_out, ed_out, pre_hb_map);
    if (pre_hb_on) handback_streams();
    mmba_result r;
    std::memset(&r, 0, sizeof(r));
    bool post_trial_end = false;  // ended by the tests after a trial (lm_decide's info)
    if (trace) trace->count = 0;
    auto push_trace = [&](double fn) {
        if (trace) {
            if (trace->count < trace->capacity) trace->fnorm[trace->count] = fn;
            trace->count++;
        }
    };
    // the host's decision on a trial point against the device's (LmDec):
    // a Jacobian the device ran ahead must be one the host takes
    pre_jac_pending = false;
    auto settle_pre = [&](bool go_host) {
        if (!pre_jac_pending) return;
        const bool go_dev = h_scalar[SL_DGO] != 0.;
        if (go_dev && !go_host) {
            // the Jacobian ran ahead at a trial point the host rejects (its
            // epilogue moved diag): replay the solve without speculation
            pre_jac_pending = false;
            throw SpecMismatch{};
        }
        // !go_dev: the gated launch did nothing (jac() launches it itself)
        if (!go_dev || !go_host) pre_jac_pending = false;
    };
    // fresh attribute block (the scene's current values)
    attrs_reset();
    double init_avg = 0.;
    bool measured = false;
    if (opt.accept_only_better && !opt.initial_error_given) {
        // measureErrors before any parameter is set (adjust_base.cpp:1080-1103);
        // it writes errorList (lmder's fvec), ud->errorList and
        // errorDistanceList, which an immediate interrupt leaves in place.
        // Its ||f|| and statistics stay in device slots until the solve's
        // last synchronisation (only the accept-only-better test reads them)
        records_enqueue(nullptr, 1);
        launch_rows_eval(s, P, d_f + 2 * (size_t)M, d_eu + 2 * (size_t)M, d_partial,
                         (M + 255) / 256);
        launch_residual(s, plug_problem(), d_recs, d_f, d_eu, d_ed, d_partial, d_scalar + SL_FI,
                        nullptr, d_dist_x);
        allreduce(d_scalar + SL_FI, 1);
        error_stats_enqueue(d_ed, SL_IESUM);
        measured = true;
    } else if (opt.accept_only_better) {
        init_avg = opt.initial_error_avg;  // the caller measured it
    }

    // x0 through the pinned stage: no blocking pageable copy (the previous
    // solve's last synchronisation released the stage)
    if (n > 0) std::memcpy(h_xstage, x_inout, sizeof(double) * n);
    MMBA_HIP(hipMemcpyAsync(d_x, h_xstage, sizeof(double) * n, hipMemcpyHostToDevice, s));
    MMBA_HIP(hipMemsetAsync(d_diag, 0, sizeof(double) * n, s));

    const double p1 = .1, p5 = .5, p25 = .25, p75 = .75, p0001 = 1e-4;
    const double epsmch = DBL_EPSILON;
    const int mode = opt.auto_param_scale == 1 ? 1 : 2;
    const double factor = opt.tau * 100.0;
    const double ftol = opt.eps1, xtol = opt.eps2, gtol = opt.eps3;
    const int maxfev = opt.iter_max;
    const bool lmdif = opt.solver_type == MMBA_SOLVER_CMINPACK_LMDIF;
    const bool polls = cb && cb->interrupt;
    int info = 0, nfev = 0, njev = 0, func_evals = 0, jac_evals = 0;
    bool interrupted = false;
    bool dist_ok = false;     // d_dist_x holds the distances at d_x
    bool f0_pending = false;  // x0's ||f||^2 is in SL_F0, not yet read
    bool x0_eval = false;     // x0's evaluation was enqueued
    double delta = 0., xnorm = 0., par = 0., fnorm = 0., gnorm = 0., ratio = 0.;

    if (n <= 0 || mg < n || ftol < 0. || xtol < 0. || gtol < 0. || maxfev <= 0 || factor <= 0.)
        goto TERMINATE;
    if (mode == 2) {
        // diag = paramWeightList (adjust_cminpack_lmder.cpp:151); lmder
        // rejects a non-positive entry before the first evaluation (both
        // checked and uploaded once, at plan build)
        if (!pweight_ok) goto TERMINATE;
        MMBA_HIP(hipMemcpyAsync(d_diag, d_pweight, sizeof(double) * n, hipMemcpyDeviceToDevice,
                                s));
    }
    // iflag = 1 at x0: incrementNormalIteration, then the interrupt poll
    // (adjust_solveFunc.cpp:551-571)
    nfev = 1;
    func_evals = 1;
    if (polls && poll_agree()) {
        interrupted = true;
        info = -1;
        goto TERMINATE;
    }
    // x0's evaluation, enqueued: its ||f|| reaches the host with the first
    // decision point's slots, and the first Jacobian's gnorm reads it on the
    // device (JacLM::fnorm_sq) -- no synchronisation before the Jacobian
    fun_enqueue(d_x, d_f, d_eu, d_ed, d_dist_x, SL_F0);
    dist_ok = true;
    f0_pending = true;
    x0_eval = true;
    {
        int iter = 1;
        for (;;) {
            if (cb && cb->progress) cb->progress(cb->user, njev);
            if (polls) {
                // the Jacobian request: lmder polls at solveFunc entry and before
                // every FD column (adjust_solveFunc.cpp:321-325); every fdjac2
                // column of lmdif is a solveFunc call (counted, then polled)
                // (a group shard takes shard 0's answer: poll_agree_index)
                int k = -1;
                if (!pshare || rank == 0) {
                    if (!lmdif && poll_interrupt()) k = 0;
                    for (int j = 0; j < n && k < 0; ++j)
                        if (poll_interrupt()) k = j;
                }
                k = poll_agree_index(k);
                if (lmdif) jac_evals += k >= 0 ? k + 1 : n;
                if (k >= 0) {
                    interrupted = true;
                    info = -1;
                    if (lmdif) {
                        nfev += n;  // lmdif adds n after fdjac2 returns
                    } else {
                        ++njev;     // lmder counts the Jacobian call
                        jac_evals += k;
                        if (central && k > 0) {  // second evaluations of columns < k
                            launch_param_central(s, P, d_x, d_ext_pertB, d_stepB, opt.delta,
                                                 d_scalar + SL_NCENT);
                            std::vector<double> sb(n);
                            MMBA_HIP(hipMemcpyAsync(sb.data(), d_stepB, sizeof(double) * n,
                                                    hipMemcpyDeviceToHost, s));
                            host_sync();
                            for (int j = 0; j < k; ++j) jac_evals += sb[j] != 0. ? 1 : 0;
                        }
                    }
                    if (k > 0) jac_partial_stale(d_x, k);
                    goto TERMINATE;
                }
                if (lmdif) jac_evals -= n;  // counted below with the rest
            }
            {
                const JacLM lm{iter == 1, mode, fnorm, f0_pending ? d_scalar + SL_F0 : nullptr};
                jac(d_x, &lm);
            }
            ++njev;
            jac_evals += n;
            if (lmdif) nfev += n;
            // lmpar always starts from the undamped (Gauss-Newton) step of
            // the new Jacobian, and when that step lies inside the trust
            // region (the common case: spec_ok says the last lmpar took it)
            // the trial point is x - xs0.  Both are enqueued behind the
            // Jacobian before the host has seen gnorm / delta, so the whole
            // outer iteration needs one synchronisation; a speculative
            // trial that lmpar does not take is discarded (its errorList /
            // errorDistanceList went to d_eu_s / d_ed_s).
            // sharded: the speculative trial's all-reduce also carries the
            // undamped solve's [DNORM, FAIL] -- two scalar collectives per
            // outer iteration (Jacobian scalars, trial + step norm)
            const bool spec = spec_ok;
            // with the speculative trial behind it, the undamped solve's
            // ||D xs|| comes from the trial's ||D p|| reduction (no separate
            // norm launches), and sharded plans fold [DNORM, FAIL] into the
            // trial's all-reduce
            const bool by_trial = spec && !(band && bs.use_bd && nG == 0 && nranks == 1) && !b15;
            lmpar_first_enqueue(*this, spec && nranks > 1, by_trial);
            // the next Jacobian is enqueued behind the trial, gated on the
            // device's restatement of the decision the host takes below
            const bool pj = pre_jac_ok();
            // the device's restatement of the decision: for the Jacobian
            // enqueued ahead (pj) and for the speculative hand-back
            const bool dv = pj || pre_hb_on;
            LmDec dec;
            if (dv) {
                dec.spec = 1;
                dec.first = iter == 1;
                dec.f0 = f0_pending;
                dec.fnorm = fnorm;
                dec.delta = delta;
                dec.xnorm = xnorm;
                dec.par = par;
                dec.gnorm = gnorm;
                dec.nfev = nfev + 1;
                dec.maxfev = maxfev;
                dec.factor = factor;
                dec.ftol = ftol;
                dec.xtol = xtol;
                dec.gtol = gtol;
            }
            if (spec)
                trial_enqueue(d_eu_s, d_ed_s, nranks > 1, by_trial, dv ? &dec : nullptr, pj);
            {
                const double t0 = wall_now();
                read_slots(0, SL_LAST);
                t_jac += wall_now() - t0;
            }
            if (f0_pending) {  // lmder's fnorm at x0, first entry of the trace
                fnorm = std::sqrt(h_scalar[SL_F0]);
                push_trace(fnorm);
                f0_pending = false;
            }
            if (central) jac_evals += (int)h_scalar[SL_NCENT];
            rank_deficient = h_scalar[SL_ZERO] != 0.;
            if (iter == 1) {
                xnorm = std::sqrt(h_scalar[SL_XN2]);
                delta = factor * xnorm;
                if (delta == 0.) delta = factor;
            }
            gnorm = fnorm != 0. ? h_scalar[SL_GNORM] : 0.;
            if (gnorm <= gtol) info = 4;
            if (info != 0) {
                settle_pre(false);
                goto TERMINATE;
            }
            bool pre = true;
            do {
                bool undamped = false;
                const double dxn = lmpar_ne(*this, delta, &par, pre, &undamped);
                (void)dxn;
                if (pre) spec_ok = undamped;
                // the trial point's solveFunc call: counted, then polled
                ++nfev;
                ++func_evals;
                if (polls && poll_agree()) {
                    interrupted = true;
                    info = -1;
                    goto TERMINATE;
                }
                if (pre && spec && undamped) {
                    // the speculative trial is lmder's trial point
                    std::swap(d_eu, d_eu_s);
                    std::swap(d_ed, d_ed_s);
                } else {
                    settle_pre(false);  // a speculative trial lmpar did not take
                    LmDec dec2;
                    if (dv) {
                        dec2.spec = 0;
                        dec2.first = iter == 1;
                        dec2.fnorm = fnorm;
                        dec2.delta = delta;
                        dec2.xnorm = xnorm;
                        dec2.par = par;
                        dec2.gnorm = gnorm;
                        dec2.nfev = nfev;
                        dec2.maxfev = maxfev;
                        dec2.factor = factor;
                        dec2.ftol = ftol;
                        dec2.xtol = xtol;
                        dec2.gtol = gtol;
                    }
                    // trial point: ||D p||, f(x + p), ||J p|| and the
                    // candidate ||D x_new|| -- one synchronisation
                    trial_enqueue(d_eu, d_ed, false, false, dv ? &dec2 : nullptr, pj);
                    const double t0 = wall_now();
                    read_slots(0, SL_LAST);
                    t_func += wall_now() - t0;
                }
                pre = false;
                const double pnorm = std::sqrt(h_scalar[SL_PNORM]);
                if (iter == 1) delta = std::min(delta, pnorm);
                const double fnorm1 = std::sqrt(h_scalar[SL_FNORM]);
                push_trace(fnorm1);
                double actred = -1.;
                if (p1 * fnorm1 < fnorm) {
                    const double d1 = fnorm1 / fnorm;
                    actred = 1. - d1 * d1;
                }
                const double temp1 = std::sqrt(h_scalar[SL_JP]) / fnorm;
                const double temp2 = (std::sqrt(par) * pnorm) / fnorm;
                const double prered = temp1 * temp1 + temp2 * temp2 / p5;
                const double dirder = -(temp1 * temp1 + temp2 * temp2);
                ratio = 0.;
                if (prered != 0.) ratio = actred / prered;
                if (ratio <= p25) {
                    double temp;
                    if (actred >= 0.)
                        temp = p5;
                    else
                        temp = p5 * dirder / (dirder + p5 * actred);
                    if (p1 * fnorm1 >= fnorm || temp < p1) temp = p1;
                    delta = temp * std::min(delta, pnorm / p1);
                    par /= temp;
                } else if (par == 0. || ratio >= p75) {
                    delta = pnorm / p5;
                    par = p5 * par;
                }
                if (ratio >= p0001) {
                    std::swap(d_x, d_wa2);  // x <- wa2 (both plain n-vectors: no copy)
                    std::swap(d_f, d_ftrial);
                    std::swap(d_dist_x, d_dist_t);
                    xnorm = std::sqrt(h_scalar[SL_XN2T]);  // ||D wa2||, computed above
                    fnorm = fnorm1;
                    ++iter;
                }
                if (std::fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1.) info = 1;
                if (delta <= xtol * xnorm) info = 2;
                if (std::fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1. && info == 2)
                    info = 3;
                if (info != 0) {
                    settle_pre(false);
                    post_trial_end = true;
                    goto TERMINATE;
                }
                if (nfev >= maxfev) info = 5;
                if (std::fabs(actred) <= epsmch && prered <= epsmch && p5 * ratio <= 1.) info = 6;
                if (delta <= epsmch * xnorm) info = 7;
                if (gnorm <= epsmch) info = 8;
                if (info != 0) {
                    settle_pre(false);
                    post_trial_end = true;
                    goto TERMINATE;
                }
                settle_pre(ratio >= p0001);
            } while (ratio < p0001);
        }
    }
TERMINATE:
    cbk = nullptr;
    if (interrupted && !measured && nfev <= 1) {
        // errorList / ud->errorList / errorDistanceList were never written
        MMBA_HIP(hipMemsetAsync(d_f, 0, sizeof(double) * m, s));
        MMBA_HIP(hipMemsetAsync(d_eu, 0, sizeof(double) * m, s));
        MMBA_HIP(hipMemsetAsync(d_ed, 0, sizeof(double) * M, s));
    }
    r.reason_number = info;
    r.iterations = nfev;
    r.function_evals = func_evals;
    r.jacobian_evals = jac_evals;
    r.outer_iterations = njev;
    r.user_interrupted = interrupted ? 1 : 0;
    r.success = func_evals > 0;
    {
        // lmder leaves the solved x in paramList (adjust_cminpack_lmder.cpp:128);
        // solveFrames writes it back only when the error got better
        // (:1227-1244), which error_is_better reports
        // RMS at the returned parameters: the accepted point's distances
        if (!dist_ok) {  // stopped before the first evaluation
            fun(d_x, d_ftrial, d_J, d_J + m, d_dist_x);  // scratch user buffers
        }
        // compute_error_stats (B13: the last measured distances), the RMS
        // and x: one synchronisation.  Unsharded, the output lists' unpermute
        // and copies go first: the copies (their own streams) run beside the
        // statistics kernels
        const bool staged = nranks == 1 && n > 0;
        const bool outs = fvec_out || eu_out || ed_out;
        // the speculative hand-back behind the last trial stored the lists
        // (the device decided the solve ends there: its info slot, mirrored)
        const bool dev_handed = post_trial_end && pre_hb_enq && h_scalar[SL_DGO + 4] > 0.;
        if (dev_handed) ++pre_handbacks;
        if (staged && outs && !dev_handed)
            download_ref_order(d_f, d_eu, d_ed, fvec_out, eu_out, ed_out, false);
        error_stats_enqueue(d_ed);
        launch_sumsq(s, d_dist_x, nullptr, M, d_partial + 3 * (size_t)pw, nparts,
                     d_scalar + SL_RMS, P.obs_own);
        allreduce(d_scalar + SL_RMS, 1);
        if (staged)  // x and the slots: one wait (read_slots' event follows the copy)
            MMBA_HIP(hipMemcpyAsync(h_xstage, d_x, sizeof(double) * n, hipMemcpyDeviceToHost, s));
        read_slots(SL_RMS, SL_IEMAX);  // also x0's ||f|| and the initial measurement's
        handback_wait();
        if (f0_pending) {  // stopped between x0's evaluation and the first decision
            fnorm = std::sqrt(h_scalar[SL_F0]);
            push_trace(fnorm);
        } else if (!x0_eval) {
            fnorm = measured ? std::sqrt(h_scalar[SL_FI]) : 0.;  // no evaluation at x0
        }
        r.error_final = fnorm;  // enorm(fvec) at the returned x
        if (measured) init_avg = h_scalar[SL_IESUM] / Mg;
        r.error_initial_avg = init_avg;
        const double avg = h_scalar[SL_ESUM] / Mg;
        r.error_avg = avg;
        r.error_min = -h_scalar[SL_ENMIN];
        r.error_max = h_scalar[SL_EMAX];
        r.error_is_better = opt.accept_only_better ? (avg <= init_avg) : 1;
        r.error_rms = std::sqrt(h_scalar[SL_RMS] / Mg);
        if (staged) {
            std::memcpy(x_inout, h_xstage, sizeof(double) * n);
        } else if (nranks > 1) {
            // x and the outputs in one hand-back (a group shard writes its own
            // parameters into the caller's x, group_x_out)
            handback_sharded(d_x, host_gather ? group_x_out : x_inout, fvec_out, eu_out, ed_out,
                             d_f, d_eu, d_ed);
        } else {
            download_params(d_x, x_inout);
            if (fvec_out || eu_out || ed_out)
                download_ref_order(d_f, d_eu, d_ed, fvec_out, eu_out, ed_out);
        }
    }
    collect_spans();
    r.num_trace = trace ? trace->count : 0;
    r.time_solve_s = wall_now() - t_start;
    r.time_func_s = t_func;
    r.time_jac_s = t_jac;
    r.time_linear_s = t_linear;
    if (res) *res = r;
    return interrupted ? MMBA_ERR_INTERRUPTED : MMBA_OK;
}

}  // namespace mmba
