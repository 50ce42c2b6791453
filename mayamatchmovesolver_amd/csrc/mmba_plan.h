// mmba_plan.h -- host-side plan: problem resident in HBM + derived structure.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <memory>
#include <string>
#include <vector>

#include "mmba_internal.h"
#include "mmba_kernels.h"

struct mmba_context {
    int device = 0;
    hipStream_t stream = nullptr;
    // ABI 9, mmba_context_create_multi: one context per shard (each with its
    // own stream) and the group's communicators; device / stream above are
    // shard 0's.  Empty for a one-device context.
    std::vector<mmba_context *> shards;
    std::vector<mmba::Comm *> comms;
};

namespace mmba {

void set_error(const std::string &msg);
// mmba_debug_set_path's choice for MMBA_PATH_<key> (-1: the builder's own)
int path_choice(int key);
// set around the plan builds of the per-frame solves (mmba_perframe.cpp):
// their lens instances follow the reference's one-frame solves (no index
// mixing, Plan::build_lens_instances)
extern thread_local bool t_lens_plain;

#define MMBA_HIP(call)                                                             \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                    \
            ::mmba::set_error(std::string(#call) + ": " + hipGetErrorString(e_));  \
            throw ::mmba::DeviceError();                                           \
        }                                                                          \
    } while (0)

struct DeviceError {};
struct SpecMismatch {};  // a Jacobian enqueued ahead of a decision the host did not take
struct Unsupported {
    std::string what;
};
struct Invalid {
    std::string what;
};

void shard_layout(int F, int M, const int32_t *obs_frame, const int32_t *obs_bnd, int nB,
                  int nranks, int32_t *bounds, int32_t *bnd_owner);

// Dense reduced system (mmba_dense.hip): blocked right-looking Cholesky,
// two-wave panel kernel + fp64 MFMA GEMM/SYRK trailing updates (k_dgemm_nt),
// right-hand side carried as an extra row (fused forward solve), block
// triangular solves.
struct Plan;
// Interrupt polls of a shard group (mmba_group.cpp): shard 0 polls the
// caller's callback, every shard takes its answer, so the shards' LM control
// flows stay identical.
struct PollShare {
    virtual ~PollShare() {}
    // leader: publishes v and returns it; others: return the leader's v
    virtual int agree(int rank, int v) = 0;
};
struct DenseSolver {
    int n = 0, ld = 0;       // columns (nRpad), leading dimension (n + 64)
    double *A = nullptr, *Linv = nullptr, *ws = nullptr;
    void setup(Plan &pl, int n);
    void init(hipStream_t s);
    void block(hipStream_t s, double *A, int ld, int k0, int nb, int end, int *fail);
    void factor_forward(hipStream_t s, const double *r, double *y, int *fail);
    void forward(hipStream_t s, const double *r, double *y);
    void backward(hipStream_t s, const double *y, double *x);
};

struct Plan {
    mmba_context *ctx = nullptr;
    hipStream_t s = nullptr;
    mmba_options opt{};
    DevProblem P{};

    // sizes (M, m: observations / residuals on this shard; Mg, mg: all)
    int n = 0, M = 0, m = 0, F = 0, Mg = 0, mg = 0;
    // frame sharding (mmba_comm.cpp): shard rank of nranks owns reduced rows
    // [Ra, Rb); every shard's range is known for the partition layout
    int rank = 0, nranks = 1, Ra = 0, Rb = 0;
    std::vector<int> Ra_all, Rb_all;
    std::vector<int> p_own;        // parameters this shard owns (norms, gather)
    int *d_p_own = nullptr;        // device copy (nullptr unsharded)
    int *d_ymask = nullptr;        // rows of L^-1 v this shard counts
    int ncf = 0, nB = 0, nG = 0, nCF = 0, nR = 0, NT = 0, nRpad = 0, nvar = 0, nslots = 0;
    int nB_solved = 0;  // bundles with a B block
    bool rank_deficient = false;
    int nparts = 256;
    int glob_chunk = 512;

    // host structure
    std::vector<int> ref_of_dev;
    // lens instances (Plan::build_lens_instances, DevProblem::obs_inst ..):
    // per global observation, and the instance tables
    std::vector<int> obs_inst_g, inst_lens_h, inst_attr_h, inst_frame_h, inst_lpar_off_h,
        inst_lpar_h;
    std::vector<double> inst_val_h;
    // every instance slot at its plug value (the measurement before
    // setParameters first runs)
    int *d_inst_attr_plug = nullptr;
    void build_lens_instances(const mmba_problem *pr);
    bool sep_form(int w);
    // min over shards of pcr_max_resident(K) for K = 8 / 16 / 24, agreed by
    // mmba_plan_create_sharded BEFORE the build (a collective inside the
    // build could pair with another shard's build-status collective); -1:
    // not agreed (the separator form is then never taken)
    int shard_resident[3] = {-1, -1, -1};
    // P with every lens instance slot at its plug value: what the reference
    // measures before setParameters first runs (solveFrames' initial
    // measureErrors, adjust_base.cpp:1002-1004 then 1076-1089)
    // rolling shutter with solved bundles: the Schur complement's view of
    // the problem, over virtual observations (one per observation and
    // camera-frame block its row reaches, grouped by camera-frame):
    // obs_cf / obs_bnd / cf_obs_off / bobs / M are theirs (Plan::build)
    bool rs_bnd = false;
    int Mv = 0;
    DevProblem PV{};
    const int *d_vobs = nullptr, *d_vcoff = nullptr;
    const DevProblem &schur_problem() const { return rs_bnd ? PV : P; }
    DevProblem plug_problem() const {
        DevProblem Q = P;
        if (Q.obs_inst) Q.inst_attr = d_inst_attr_plug;
        return Q;
    }
    std::vector<int> panel_rows_off, panel_rows;    // rows(k) flattened
    std::vector<int> panel_cols_off, panel_cols;    // colsT(k) flattened
    std::vector<int> panel_pairs_off;               // pairs(k) offsets into d_pairs
    std::vector<double> host_attr0;

    // device allocations (owned)
    std::vector<void *> allocs;
    int *d_slot = nullptr;
    double *d_S = nullptr, *d_Linv = nullptr;
    int *d_rows = nullptr, *d_cols = nullptr;
    int2 *d_pairs = nullptr;
    // deterministic Schur accumulation (destination-sorted observation pairs)
    bool use_dest = false;
    int ndest = 0;
    int jac_ncv = 0;     // uniform fast Jacobian kernel (k_jacobian_u<jac_ncv>), 0: generic
    // fixed choices of earlier A/B measurements (the alternatives stay in
    // the source, compiled out): the fused Jacobian + normal-equation pass,
    // the lam = 0 bundle factor formed in the bundle pass
    static constexpr bool k2_split = false;
    static constexpr bool fold_ok = true;
    // reductions folded into their producers' last workgroup (one ticket
    // counter) instead of a k_reduce_multi launch: measured slower on C4
    // (k_residual<JP> 16.7 -> 30.5 us, k_ne_bnd_jb +7 us): 782 / 196 arrivals
    // on one device-scope counter cost more than the launch they save (MI355X
    // guide "fanin", ~12 ns per atomic)
    static constexpr bool tail_reduce = false;
    // page-locked sequence word of the mirrored reductions (read_slots
    // polls it)
    unsigned *h_seq = nullptr;
    unsigned seq_next = 0;
    bool seq_pending = false;  // the next mirrored read_slots polls h_seq
    static constexpr bool seq_poll = true;  // (stream events: measured slower)
    int pc_uniform = 0;  // common block size of the solved camera-frames (0: mixed)
    int2 *d_dest = nullptr, *d_dpairs = nullptr;
    // destination lists of the split Schur pass (k_schur_dest_u over the
    // wave list, k_schur_dest_lane over the lane list); null: one pass
    int *d_dest_wave = nullptr, *d_dest_lane = nullptr;
    int n_dest_wave = 0, n_dest_lane = 0;
    int *d_dest_off = nullptr, *d_row_cf = nullptr;
    // band + arrow layout of the reduced system (mmba_band.hip)
    bool band = false;
    int bw = 0;
    BandSolver bs;
    void setup_band(int Pforce = 0);
    SView sview() const {
        SView V{};
        V.band = band ? 1 : 0;
        V.dense = dense ? 1 : 0;
        V.ld = dld;
        V.S = d_S;
        V.slot = d_slot;
        V.NT = NT;
        V.Bd = bs.Bd;
        V.w = bw;
        V.nb = nR - nG;
        V.Ga = bs.Ga;
        V.Gd = bs.Gd;
        return V;
    }
    // dense reduced system (most tiles structurally non-zero)
    bool dense = false;
    bool shard_dense = false;  // sharded plan without a narrow band: dense S all-reduced
    int dld = 0;
    DenseSolver ds;
    long long *d_probe = nullptr;  // MMBA_PATH_PROBE = 1: band-kernel phase cycles
    long long *d_k2probe = nullptr;  // MMBA_PATH_PROBE = 2: k_jac_ne_u workgroup timeline
    bool nloc_set = false;         // d_nloc stored by a fused Jacobian pass
    // single-workgroup triangular solves for narrow (banded) structures
    bool narrow = false;
    int *d_rows_off = nullptr, *d_cols_off = nullptr;
    int *d_var_cf = nullptr, *d_stale = nullptr, *d_ref_of_dev = nullptr;
    int *d_dev_of_ref = nullptr;  // unsharded: the inverse permutation
    double *d_attr0 = nullptr;
    size_t attr_bytes = 0;

    double *d_x = nullptr, *d_ext = nullptr, *d_ext_pert = nullptr, *d_step = nullptr;
    double *d_diag = nullptr, *d_acnorm = nullptr, *d_g = nullptr;
    double *d_wa1 = nullptr, *d_wa2 = nullptr, *d_wa3 = nullptr, *d_xs = nullptr,
           *d_v = nullptr;
    // residual buffers: [2 M marker rows | nrows stiffness / smoothness rows]
    double *d_f = nullptr, *d_ftrial = nullptr, *d_eu = nullptr, *d_ed = nullptr;
    int nrows = 0;                 // attribute rows (same on every shard)
    double *d_Jrow = nullptr;      // their Jacobian entries (one column each)
    // central differences (lmder, autoDiffType central): the deltaB pass
    bool central = false;
    // B15: central differences where animated columns skip the other
    // frames' rows.  The reference's Jacobian is then J = J_s + f c^T (f at
    // the Jacobian's point, c_p = 0.5 / (|dA| + |dB|) of animated central
    // columns): J_s is the sparse Jacobian the kernels store, the rank-one
    // term rides in the epilogue (column norms, J^T f), the damped solve
    // (Woodbury over two right-hand sides, u = J_s^T f and c, with one
    // factorisation each), lmpar's Newton term and ||J p||.
    // The c f part of an animated block is one direction per camera-frame:
    // the block's columns are stored in the Householder basis Q_cf with
    // Q c_cf = kappa e_0, so the normal equations keep the accuracy of the
    // differences (in the original basis the block's columns are nearly
    // parallel and the squared condition loses ~5 digits); every
    // parameter-space vector crosses Q at the solve's boundary.
    bool b15 = false, b15_inner = false;
    double *d_c15 = nullptr;   // c (n, original basis)
    double *d_c15r = nullptr;  // c in the rotated basis
    double *d_g15 = nullptr;   // J^T f = u + s c (n, original): gnorm, lmpar's ||D^-1 g||
    double *d_q15 = nullptr, *d_kap15 = nullptr;  // Q_cf (ncf x PCMAX^2), kappa_cf
    double *d_AccL = nullptr, *d_diagL = nullptr;  // damped rotated blocks, diag off them
    double *d_z15u = nullptr, *d_z15c = nullptr;  // M^-1 u, M^-1 c (rotated) of the last solve
    double *d_xs15r = nullptr, *d_p15 = nullptr, *d_v15 = nullptr;  // xs, p, v rotated
    double *d_adiag15 = nullptr, *d_u15 = nullptr;  // A_pp, u in the original basis
    double *d_b15k = nullptr;  // [K^-1 (4), s, fail of the first solve]
    // rolling shutter (mmba.h ABI 3, mmba_rs.hip)
    bool rs_on = false;
    double *d_ext_pertB = nullptr, *d_stepB = nullptr, *d_recsB = nullptr, *d_brecB = nullptr;
    std::vector<double> param_weight;  // paramWeightList (diag in mode 2)
    double *d_pweight = nullptr;       // ... on the device
    bool pweight_ok = true;            // every weight > 0 (lmder's mode-2 check)
    std::vector<int> stale_host;       // stale-column table (B13), host copy
    std::vector<int> param_frame_host;
    // solved camera-frame blocks (reduced rows [roff, roff + pc)), for the
    // block-diagonal solver
    std::vector<int> cfblk_roff, cfblk_pc, cfblk_cf;
    double *d_recs = nullptr, *d_brec = nullptr;
    double *d_J = nullptr;
    int *d_jcol = nullptr, *d_nloc = nullptr;
    double *d_Acc = nullptr, *d_Acg = nullptr, *d_Abb = nullptr, *d_Abg = nullptr,
           *d_Agg = nullptr, *d_glob_partial = nullptr;
    double *d_Lb = nullptr, *d_tb = nullptr, *d_Wg = nullptr, *d_W = nullptr, *d_U = nullptr;
    double *d_rhs = nullptr, *d_yR = nullptr, *d_xR = nullptr, *d_wR = nullptr,
           *d_usq = nullptr, *d_nu = nullptr, *d_ngp = nullptr;  // Newton-term scratch
    double *d_partial = nullptr, *d_scalar = nullptr;
    double *d_gather = nullptr;  // outputs in reference order: f | eu | ed | x
    int *d_fail = nullptr;
    unsigned int *d_ticket = nullptr;  // single-launch reduction ticket (zero between uses)
    double *h_scalar = nullptr;  // pinned
    // host mirror: trial reductions write slots [0, SL_LAST] straight
    // into h_scalar (the last k_reduce_multi block) and read_slots skips its
    // copy launch.  With a stream-event wait it measured 3 % slower per C4
    // solve (round 2); with the page-locked sequence word the LM thread polls
    // (seq_poll) it is 4 % faster (C4 14.48 -> 13.90 ms, profiles/r3_prejac)
    unsigned *d_mticket = nullptr;
    bool host_mirror = true, mirror_pending = false;
    // every solved camera-frame has a diagonal Schur destination; fold_init:
    // k_schur_init rides in k_schur_dest_u (SchurInitFold)
    bool dest_diag_all = false, fold_init = false, dest_diag_ii = false;
    double *h_xstage = nullptr;  // pinned [n]: x in / out without a blocking pageable copy
    int *h_fail = nullptr;       // pinned

    // timing (HIP events on the plan stream, read back only at the end of a
    // solve so the hot path never waits on them)
    bool timing = false;
    enum SpanKind { SPAN_RESID = 0, SPAN_JAC = 1, SPAN_CHOL = 2 };
    struct Span {
        hipEvent_t a, b;
        int kind;
    };
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<Span> spans;
    hipEvent_t span_a = nullptr;
    hipEvent_t next_event();
    int span_ctr[3] = {0, 0, 0};
    int span_stride = 4;
    bool span_on = false;
    void span_begin(int kind);
    void span_end(int kind);
    void collect_spans();
    double jac_ms = 0., resid_ms = 0., chol_ms = 0.;
    int jac_n = 0, resid_n = 0, chol_n = 0;
    double t_func = 0., t_jac = 0., t_linear = 0.;

    // multi-GPU
    Comm *comm = nullptr;
    // shard of a group plan (one caller, several devices, mmba_group.cpp):
    // interrupt answers come from shard 0; outputs go straight to the
    // caller's host buffers (each shard its own observations and
    // parameters), no collective
    PollShare *pshare = nullptr;
    bool host_gather = false;
    // sharded hand-back: this shard's own observations in reference order
    // (device index, reference index), its own parameters
    int M_own = 0, own_pad = 0, n_own = 0, npar_pad = 0;
    std::vector<int> own_ref_h, own_par_h;
    int *d_own_dev = nullptr, *d_own_par = nullptr;
    // every shard's lists, padded (-1), for the all-gather of the
    // one-process-per-GPU path
    int *d_own_ref_all = nullptr, *d_own_par_all = nullptr;
    double *d_pack = nullptr, *d_pack_all = nullptr, *h_pack = nullptr;
    // the step's rows after a sharded band solve: each shard's rows
    // [Ra_all[k], Rb_all[k]) (+ the arrow rows, shard 0's) all-gathered
    int rows_pad = 0;
    int *d_Ra_all = nullptr, *d_Rb_all = nullptr;
    double *d_rows_send = nullptr, *d_rows_all = nullptr;
    double *group_x_out = nullptr;  // group solve: the caller's x (own parameters written)
    void gather_step_rows();
    void handback_sharded(const double *dx, double *x_out, double *f_out, double *eu_out,
                          double *ed_out, const double *f2, const double *eu2, const double *ed1);
    // [rank of each global observation (Mg) | rank of each parameter (n)]
    void setup_handback(const std::vector<int> &own_rank_obs_par);
    bool poll_agree();
    int poll_agree_index(int k);
    // a sharded plan whose problem does not shard (mmba_plan_create_sharded):
    // every shard solves the whole problem, no collectives
    bool replicated = false;
    std::string replicate_why;

    ~Plan();

    template <class T>
    T *dalloc(size_t count) {
        void *p = nullptr;
        if (count == 0) count = 1;
        MMBA_HIP(hipMalloc(&p, count * sizeof(T)));
        allocs.push_back(p);
        return static_cast<T *>(p);
    }
    template <class T>
    T *upload(const std::vector<T> &v) {
        T *d = dalloc<T>(v.size());
        if (!v.empty())
            MMBA_HIP(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
        return d;
    }
    template <class T>
    T *upload(const T *src, size_t count) {
        T *d = dalloc<T>(count);
        if (count && src)
            MMBA_HIP(hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, s));
        return d;
    }

    void build(const mmba_problem *prob, const mmba_options *o);

    // LM building blocks.  *_enqueue functions only launch work; results land
    // in device scalar slots (all-reduced across shards) and are fetched with
    // one read_slots() per decision point of the MINPACK control flow.
    enum Slot {
        // grouped so that each sharded exchange is one all-reduce:
        // trial point [PNORM..JP], damped solve [DNORM, FAIL], lmpar Newton
        // [NEWT_B, NEWT_R], Jacobian [ZERO, XN2] (sums; the flags are 0/1
        // per shard, so a sum is nonzero exactly when the max is)
        SL_PNORM = 0,   // ||D p||^2 of the trial step
        SL_XN2T = 1,    // ||D x_new||^2 of the trial point
        SL_FNORM = 2,   // ||f||^2 of the last fun_enqueue
        SL_JP = 3,      // ||J p||^2
        SL_DNORM = 4,   // ||D v||^2
        SL_FAIL = 5,    // factorisation failed (flag)
        SL_NEWT_B = 6,  // lmpar Newton term, bundle part
        SL_NEWT_R = 7,  //                    reduced-system part
        SL_GDIV = 8,    // ||D^-1 g||^2 (lmpar gnorm)
        SL_ZERO = 9,    // any exactly-zero Jacobian column (flag)
        SL_XN2 = 10,    // ||D x||^2 (first pass)
        SL_GNORM = 11,  // lmder gnorm (max)
        SL_RMS = 12,
        SL_NCENT = 13,  // central FD columns of the last Jacobian (second evaluations)
        SL_F0 = 14,     // ||f||^2 at x0 (lmder's first evaluation; read with the first decision)
        // the device's restatement of the decision after a trial point
        // (LmDec, k_reduce_multi): gate of the pre-enqueued Jacobian, then
        // ratio, delta, par, info -- the host checks its own against them
        SL_DGO = 15,
        SL_DRATIO = 16,
        SL_DDELTA = 17,
        SL_DPAR = 18,
        SL_DINFO = 19,
        SL_LAST = 19,
        SL_FI = 20,     // ||f||^2 of the initial measurement (read at the end)
        // errorDistanceList statistics (launch_dist_stats): sum, -min, max
        SL_ESUM = 21,
        SL_ENMIN = 22,
        SL_EMAX = 23,
        // ... of the initial measurement (read at the end)
        SL_IESUM = 24,
        SL_IENMIN = 25,
        SL_IEMAX = 26,
        NSLOT = 28
    };
    void read_slots(int lo, int hi);
    static constexpr bool spin_wait = true;  // (blocking synchronisation: slower)
    hipEvent_t ev_sync = nullptr;  // [lo, hi] inclusive, one D2H copy + sync
    double read_scalar(int slot = 0);
    void stream_wait();
    void allreduce(double *d, size_t count, ReduceOp op = ReduceOp::Sum);
    double reduce_read(int slot, ReduceOp op = ReduceOp::Sum);
    void fun_enqueue(const double *dx, double *df, double *eu, double *ed,
                     double *dist = nullptr, int slot = SL_FNORM);
    double fun(const double *dx, double *df, double *eu, double *ed, double *dist = nullptr);
    // errorDistanceList of the accepted x and of the pending trial point
    // (swapped on acceptance): the RMS at the returned x needs no extra
    // evaluation
    double *d_dist_x = nullptr, *d_dist_t = nullptr;
    std::vector<long long> param_vidx;  // attribute-value index of each parameter
    std::vector<double> pmin_h, pmax_h, poff_h, pscale_h;  // bound transform (host)
    // compute_error_stats of ed on the device -> avg, min, max (host)
    void error_stats_device(const double *ed, double *avg, double *mn, double *mx);
    // -> slots base .. base + 2 (sum, -min, max): SL_ESUM or SL_IESUM
    void error_stats_enqueue(const double *ed, int base = SL_ESUM);
    // with lm: the lmder bookkeeping after the normal equations is fused
    // into the column-norm launch (k_jac_epilogue); scalars -> SL_ZERO,
    // SL_XN2 (first pass), SL_GNORM (fnorm != 0)
    struct JacLM {
        int first, mode;
        double fnorm;
        // non-null: ||f||^2 in a device slot (the first Jacobian, before the
        // host has read x0's evaluation); the kernels take its square root
        const double *fnorm_sq = nullptr;
    };
    void jac(const double *dx, const JacLM *lm = nullptr);
    // interrupt polls of the reference (MComputation::isInterruptRequested):
    // true once the caller's callback asks to stop
    const mmba_callbacks *cbk = nullptr;
    bool poll_interrupt() const {
        return cbk && cbk->interrupt && cbk->interrupt(cbk->user) != 0;
    }
    // FD columns [0, k) only: errorList / errorDistanceList as an interrupted
    // Jacobian leaves them (the stale-column table restricted to k columns)
    void jac_partial_stale(const double *dx, int k);
    // trial point x - xs: setParameters, measureErrors into (d_ftrial, eu,
    // ed), ||J p||; scalars -> SL_PNORM, SL_XN2T, SL_FNORM, SL_JP
    // with_dnorm (sharded speculative trial): the undamped solve's [DNORM,
    // FAIL] ride in the trial's all-reduce (slots 0..5, one collective)
    // fill_dnorm: this trial's ||D p||^2 also fills SL_DNORM and the fail
    // flag SL_FAIL of the undamped solve enqueued with dnorm_by_trial
    void trial_enqueue(double *eu, double *ed, bool with_dnorm = false, bool fill_dnorm = false,
                       const LmDec *dec = nullptr, bool jac_ahead = false);
    // The next Jacobian's first launch (k_jac_ne_u at the trial point),
    // enqueued behind a trial whose reduction restates the host's decision
    // (LmDec): it runs only when that decision takes the trial and goes on,
    // so the GPU starts the next iteration while the host reads the trial.
    // (cleared for the replay of a SpecMismatch solve)
    // the trial point's parameter pass fused into the bundle back
    // substitution of the damped solve (launch_backsub_trial);
    // otherwise k_trial_prep
    bool trial_fold_ok = false, trial_folded = false;
    // the folded trial pass also builds the trial point's records (no
    // k_records launch; TrialFold::rec)
    bool trial_rec = false;
    // plans without a solved bundle: k_trial_prep_rec sets the trial point
    // and builds its records (no k_records launch); the parameters outside
    // every camera-frame block (globals no record reads)
    bool trial_prep_rec = false;
    int *d_prep_other = nullptr;
    int n_prep_other = 0;
    int *d_trial_other = nullptr;
    int n_trial_other = 0;
    bool pre_jac = true;
    bool pre_jac_pending = false;   // enqueued, the host has not decided yet
    const double *pre_jac_x = nullptr;
    int *d_gate = nullptr;
    bool pre_jac_ok() const;
    void pre_jac_enqueue(const double *dx, double *eu, double *ed);
    // the trial's slots staged (D2H copy unless mirrored, then an event)
    // before the pre-enqueued Jacobian: read_slots(0, SL_LAST) only waits
    bool slots_staged = false;
    void stage_slots();
    // the Jacobian epilogue's row reductions held back for the next damped
    // solve's k_schur_init launch (block diagonal + arrow plans without a
    // solved bundle, C5); flush_red launches them alone wherever anything
    // else comes first
    bool pend_red = false;
    RedSpec pend_rs{};
    bool red_defer_ok() const;
    void flush_red();
    void host_sync();
    bool jb_recompute() const;
    DevProblem P_nojb() const;
    bool stall_done = false;  // MMBA_PATH_STALL_SHARD fired
    bool pre_bnd_pending = false;
    // k_schur_obs enqueued behind the gated bundle pass too, with the
    // Jacobian epilogue's deferred reduction (pre_jac_enqueue); sobs_ahead:
    // the jac() that took the pre-enqueued pass hands it to the next damped
    // solve, which then skips that launch
    bool pre_sobs_pending = false, sobs_ahead = false;
    double *d_cf_part = nullptr;      // k_ne_cf_split partial sums
    unsigned *d_cf_ticket = nullptr;  // k_ne_cf_split tickets (monotonic)  // the bundle pass was enqueued with the pre-enqueued Jacobian
    void wait_event();
    // speculative trial (lmpar's first, undamped, step taken before the
    // host has read it): its errorList / errorDistanceList land here and are
    // swapped in when lmpar accepts that step
    double *d_eu_s = nullptr, *d_ed_s = nullptr;
    bool spec_ok = true;  // last lmpar accepted its undamped step
    // d_f / d_eu / d_ed hold the last solve's (or measure's) outputs
    // (mmba_plan_outputs); other evaluations clear it
    bool outputs_ready = false;
    // the device x vector whose parameters (attribute values, d_ext,
    // d_ext_pert, d_step) are currently set; nullptr: none
    const double *params_at = nullptr;
    // the device x vector whose FULL record set (camera-frame variants and
    // perturbed bundle positions, k_records with base_only = 0) d_recs /
    // d_brec hold: an evaluation or trial point builds the full set in its
    // one records launch, so the Jacobian at an accepted point needs none
    const double *recs_full_at = nullptr;
    // d_Lb / d_tb hold the bundle factor at lam = 0 of the current normal
    // equations, formed by the Jacobian's bundle pass (NeEpi::Lb); the next
    // undamped solve uses it instead of launching k_bundle_factor
    bool lb0_valid = false;
    void records_enqueue(const double *xat, int base_only);
    void attrs_reset() {  // the scene's own attribute values
        MMBA_HIP(hipMemcpyAsync(P.attr_val, d_attr0, attr_bytes, hipMemcpyDeviceToDevice, s));
        params_at = nullptr;
        recs_full_at = nullptr;
    }
    // forward-difference eps of lmdif's fdjac2 (unused by lmder's steps)
    double fd_eps() const { return std::sqrt(std::max(std::fabs(opt.delta), DBL_EPSILON)); }
    int pw = 0;           // partial-row stride of d_partial (8 rows)
    // dnorm_slot >= 0: also ||D xs||^2 -> that slot (one reduction launch
    // with the fail flag)
    // defer: leave [DNORM, FAIL] un-reduced (the caller's next all-reduce
    // carries them)
    void solve_damped_enqueue(double lam, int dnorm_slot = -1, bool defer = false,
                              bool dnorm_by_trial = false);
    bool solve_damped(double lam);
    void newton_enqueue(double dxnorm);
    void dnorm_enqueue(const double *dv, int slot);
    double dnorm(const double *dv);
    int solve(double *x_inout, double *fvec_out, double *eu_out, double *ed_out,
              mmba_result *res, const mmba_callbacks *cb, mmba_trace *trace);
    int solve_once(double *x_inout, double *fvec_out, double *eu_out, double *ed_out,
                   mmba_result *res, const mmba_callbacks *cb, mmba_trace *trace);
    int spec_replays = 0;  // solves replayed after a speculative Jacobian the host did not take
    // Per-frame solve mode in one launch (mmba_batch.hip), valid when every
    // parameter is a camera-frame parameter (no static parameter chains the
    // frames); frames [0, batch_nf) are solvable, batch_nfmax = most
    // parameters of one frame
    bool batch_ok = false;
    std::string batch_why;
    int batch_nf = 0, batch_nfmax = 0;
    int *d_fr_cf_off = nullptr, *d_fr_par_off = nullptr, *d_fr_par = nullptr,
        *d_fr_last = nullptr, *d_fr_nobs = nullptr;
    double *d_bJ = nullptr, *d_bdist = nullptr, *d_bx = nullptr, *d_bpw = nullptr;
    BatchOut *d_bout = nullptr;
    int *h_bflag = nullptr, *d_bflag = nullptr;  // host-mapped interrupt flag
    int solve_frames(double *x_inout, mmba_result *results, const mmba_callbacks *cb);
    int dense_jacobian(const double *x, double *fjac);
    // test hook (mmba_debug_reduced_residual): the damped reduced system at
    // x and lam, kept aside before the factorisation; its solve's relative
    // residual ||S x - r|| / ||r|| (dense plans)
    bool dbg_keep_S = false;
    double *d_Skeep = nullptr, *d_rkeep = nullptr;
    int reduced_residual(const double *x, double lam, double *relres);
    int reproject(const double *x, double *point_out, double *marker_out);
    int measure(const double *x, double *fvec_out, double *eu_out, double *ed_out,
                double *stats);
    void download_params(const double *dx, double *x_out);
    // sync = false (unsharded): the copies are only enqueued, the caller's
    // next wait covers them
    void download_ref_order(const double *d_f2, const double *d_eu2, const double *d_ed1,
                            double *f_out, double *eu_out, double *ed_out, bool sync = true);
    // unsharded hand-back: each output list's device-to-host copy on its own
    // stream (its own DMA queue) behind the unpermute, so the three copies
    // run together and beside the kernels enqueued after them on s;
    // handback_wait() polls their events
    hipStream_t s_hb[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_hb[4] = {nullptr, nullptr, nullptr, nullptr};
    bool hb_pending = false;
    bool hb_used[3] = {false, false, false};
    void handback_wait();
    void handback_streams();
    // host-mapped addresses of page-locked caller lists (all non-null lists
    // mapped and 16-B aligned, else false)
    bool map_outputs(double *f_out, double *eu_out, double *ed_out, double *hmap[3]);
    // speculative hand-back (unsharded solves into page-locked lists): every
    // trial enqueued with the device's decision also enqueues k_handback_host
    // gated on it, so the lists leave as soon as the device has decided the
    // solve ends there; the host skips its own hand-back when it ends on
    // that trial and the device's slots say the kernel stored them
    bool pre_hb_on = false, pre_hb_enq = false;
    long long pre_handbacks = 0;  // solves whose lists the speculative hand-back stored
    double *pre_hb_map[3] = {nullptr, nullptr, nullptr};
};

}  // namespace mmba

namespace mmba {
struct ShardGroup;  // mmba_group.cpp
void destroy_group(ShardGroup *g);
struct GroupDeleter {
    void operator()(ShardGroup *g) const { destroy_group(g); }
};
}  // namespace mmba

namespace mmba {
// group forms of the plan entry points (mmba_group.cpp; mmba_api.cpp routes
// a plan whose group is set, or a multi-device context, here)
int group_plan_create(mmba_context *ctx, const mmba_problem *prob, const mmba_options *opt,
                      mmba_plan **out);
int group_plan_solve(mmba_plan *plan, double *x_inout, double *fvec_out, double *err_user_out,
                     double *err_dist_out, mmba_result *res, const mmba_callbacks *cb,
                     mmba_trace *trace);
int group_plan_measure(mmba_plan *plan, const double *x, double *fvec_out, double *err_user_out,
                       double *err_dist_out, double *avg_min_max_out);
int group_plan_reproject(mmba_plan *plan, const double *x, double *point_xy_out,
                         double *marker_xy_out);
int group_plan_jacobian(mmba_plan *plan, const double *x, double *fjac);
int group_plan_outputs(mmba_plan *plan, double *fvec_out, double *err_user_out,
                       double *err_dist_out);
int group_plan_set_attr_values(mmba_plan *plan, const double *attr_values);
int group_plan_solve_per_frame(mmba_plan *plan, double *x_inout, mmba_result *results,
                               const mmba_callbacks *cb);
int group_plan_kernel_stats(mmba_plan *plan, int enable_timing, mmba_kernel_stats *out);
}  // namespace mmba

struct mmba_plan {
    mmba::Plan impl;
    // ABI 9: a plan over a multi-device context -- one sharded plan per
    // device, driven by the library's own threads (impl unused)
    std::unique_ptr<mmba::ShardGroup, mmba::GroupDeleter> group;
};
