// mmba_internal.h -- shared host/device definitions of the MI355X BA core.
//
// Data layout in HBM (all fp64 unless noted, int32 indices):
//   problem tables   attr block (offset/animated/values), transforms, cameras,
//                    lenses, bundles: small, read through L2.
//   observations     device order = sorted by camera-frame ("cf"), so every
//                    cf owns a contiguous segment; SoA arrays obs_* [M].
//   Jacobian blocks  J[(2*l + r) * M + i]: local column l (<= LMAX), residual
//                    row r (x/y) of observation i; jcol[l * M + i] = param id.
//   normal equations per-cf dense blocks Acc[cf][PCMAX][PCMAX], per-bundle
//                    Abb[b][3][3], globals Agg[NG][NG], couplings Acg/Abg.
//   reduced system   S over R = {cf params} + {globals}, stored as 64x64
//                    lower tiles (only structurally non-zero tiles allocated).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mmba.h"

namespace mmba {

constexpr int PCMAX = 12;   // params per camera-frame block
constexpr int PBMAX = 3;    // params per bundle block
constexpr int NGMAX = 48;   // global parameters (the arrow of the reduced system)
constexpr int NGLANE = 16;  // arrows up to this width ride in spare lanes of the BCR pivot chains
constexpr int NGPART = 32;  // widest arrow the partitioned band chain's LDS window carries
constexpr int LMAX = 32;    // local Jacobian columns per observation
constexpr int CF_AIDX = 16;  // camera-frame attribute table: 7 camera + 9 TRS
constexpr int TILE = 64;    // reduced-system tile edge
constexpr int CAMREC = 20;  // doubles per camera-frame record
constexpr int LENS_LAYER = 1 + MMBA_LENS_NUM_ATTRS;  // input lens layer: type, 14 slots
constexpr int LENS_CHAIN_MAX = 4;                    // input layers per lens
constexpr int BREC = 16;    // doubles per bundle record (128 B: one L2 line)

// In-place all-reduce of device buffers across the shards of a plan
// (mmba_comm.cpp: RCCL, or an in-process group for tests).
enum class ReduceOp { Sum, Max };
struct CommError {};
struct Comm {
    int rank = 0, nranks = 1;
    virtual ~Comm() {}
    virtual void allreduce(double *buf, size_t count, ReduceOp op, hipStream_t s) = 0;
    // recv[k * count .. (k + 1) * count) = rank k's send[0 .. count) on every
    // rank (send and recv distinct device buffers)
    virtual void allgather(const double *send, double *recv, size_t count, hipStream_t s) = 0;
    // a shard failed outside a collective: the others' pending and future
    // collectives fail (CommError) instead of waiting forever
    virtual void abort() {}
    // RCCL: collectives complete on the device, so a host wait on a stream
    // that carries one is bounded (comm_wait) and polls the communicator's
    // asynchronous error; the in-process group waits in its own barrier
    virtual bool bounded() const { return false; }
    virtual void poll_async() {}
    // ranks as the transport reports them (ncclCommCount)
    virtual int count() const { return nranks; }
};

// Bounded wait for every collective: milliseconds before
// a communicator is aborted and the call fails with MMBA_ERR_COMM instead of
// hanging its caller (path MMBA_PATH_COMM_TIMEOUT_MS, else the environment's
// MMBA_COMM_TIMEOUT_MS, else 120 s).
int comm_timeout_ms();
// Wait until the event (or, ev == NULL, the stream) completes; through a
// bounded communicator the wait polls and, past comm_timeout_ms(), aborts the
// communicator and throws CommError.
void comm_wait(Comm *c, hipStream_t s, hipEvent_t ev);

// Band + arrow layout of the reduced system (narrow structures): rows of
// camera-frame parameters keep w+1 entries each (columns r-w .. r), the
// global parameters are dense arrow rows (mmba_band.hip).
constexpr int WBAND_MAX = 80;    // widest half bandwidth of the band layout
constexpr int WBAND_PART = 40;   // widest half bandwidth that is partitioned

// One partition of the band rows: interior rows [r0, r1) plus its arrow
// (previous separator rows, next separator rows, global rows).
struct BandPart {
    int r0, r1;
    int na, nprev, nnext;  // arrow rows: nprev + nnext + nG
    int sprev, snext;      // first band row of the prev / next separator (-1: none)
    int zoff;              // packed lower Z_p (na rows) in zpool
    int doff;              // first NB x NB block inverse
    int coff;              // solve partial sums in cpool
    long long aoff;        // arrow rows: apool[aoff + a*(r1-r0) + (c-r0)]
};

// Block cyclic reduction of the band + arrow system (mmba_bcr.hip): K x K
// blocks (K = 8/16/24/32 >= w), per-block factor columns for the solves.
struct BcrDev {
    int K = 0, nb = 0, nG = 0, nblk = 0, w = 0;
    int NR = 0;  // root system size: K + nG rounded up to 8
    // level pivot chain (MMBA_BCR_CHOL): 0 column broadcast through LDS per
    // step, 2 blocked (8-column panels); a v_readlane-per-entry chain measured
    // 13 % slower than 0 and was dropped
    int regchol = 2;
    int mfma_upd = 1;  // even-block updates as fp64 MFMA (always; the VALU form is the K > 32 fallback)
    const double *Bd = nullptr, *Ga = nullptr, *Gd = nullptr;  // input (band layout)
    double *Dk = nullptr, *Lk0 = nullptr, *Lk1 = nullptr, *Gk = nullptr;
    double *FC = nullptr, *FU = nullptr, *FV = nullptr, *FY = nullptr, *Zc = nullptr;
    double *FT = nullptr, *gpart = nullptr, *rw = nullptr;
    // dataflow backward solve (k_bcr_bwd_all): per-block flags (epochs),
    // blocks in dependency order, the plan's fail flag (nullptr: per-level launches)
    int *flags = nullptr;
    const int *ord = nullptr;
    // dataflow factorisation (k_bcr_factor_df): one flag per level item and
    // the root (nullptr: per-level launches, MMBA_PATH_BCR_DATAFLOW = 0)
    int *fflags = nullptr;
    int *fail = nullptr;
    // item tickets of the two dataflow launches ([0] factorisation, [1]
    // backward solve): a workgroup takes its next item from the counter, so
    // items are started in dependency order whatever the residency (forward
    // progress does not assume every workgroup is resident)
    unsigned *tick = nullptr;
    // with xs: the backward solve also scatters x_R to parameter order
    // (xs[row_param[R]] = x_R, k_scatter_xR's job)
    const int *row_param = nullptr;
    double *xs = nullptr;
};

// Parallel cyclic reduction of the band system without an arrow
// (mmba_pcr.hip): K x K blocks (K <= 24), one persistent workgroup per block.
// pub[(lvl * nblk + j) * (3 K^2 + K)]: C^-1, C^-1 L, C^-1 U (column-major) and
// C^-1 r of block j's factor at level lvl (its final level: C^-1 and rho);
// wlog: the update products W1, W2 of every (level, block) (Newton pass).
// right-hand sides of one k_pcr_rhs_mc launch, at most
constexpr int PCR_NCMAX = 48;

struct PcrDev {
    int K = 0, nb = 0, w = 0, nblk = 0, nlev = 0;
    int nth = 256;  // k_pcr_solve workgroup: 512 threads when that grid is resident (same bits)
    const double *Bd = nullptr;  // band input [nb][w+1]
    // publications of k_pcr_solve / k_pcr_rhs: 16-B granules {value, epoch,
    // epoch} (zeroed at build; epochs start at 1), per [nlev][nblk]
    double *pub = nullptr, *wlog = nullptr, *rpub = nullptr, *part = nullptr;
    int *flev = nullptr;                     // final level of every block
    const int *row_param = nullptr;          // reduced row -> parameter (scatter of x)
    // several right-hand sides (k_pcr_rhs_mc): granule publications
    // [nlev][nblk][2 K PCR_NCMAX]
    double *mpub = nullptr;
};

// Block-diagonal + arrow reduced system (mmba_bdiag.hip): no solved bundle,
// so the camera-frame blocks are uncoupled; block b = reduced rows
// [roff[b], roff[b] + pc[b]), pc <= PC <= PCMAX.
struct BdDev {
    int nblk = 0, nb = 0, nG = 0, w = 0, PC = 0;
    const int *roff = nullptr, *pc = nullptr;
    const double *Bd = nullptr, *Ga = nullptr, *Gd = nullptr;  // input (band layout)
    double *FC = nullptr, *FY = nullptr, *Zc = nullptr, *gpart = nullptr, *FT = nullptr;
    const int *row_param = nullptr;  // reduced row -> parameter (scatter of x)
    // direct path (nG == 0): block -> camera-frame, single-launch reduction
    const int *cf = nullptr;
    unsigned int *ticket = nullptr;
    double *part = nullptr;
};

// Batched per-frame LM (mmba_batch.hip): one workgroup runs the whole
// lmder / lmdif solve of one frame's sub-problem (per-frame solve mode with
// no static parameter: the frames share nothing).  Frame f owns camera-frames
// [fr_cf_off[f], fr_cf_off[f + 1]) and local parameters k = reduced row -
// cf_roff of its first camera-frame (fr_par[fr_par_off[f] + k] = parameter).
constexpr int BATCH_CFMAX = 8;   // camera-frames per frame
constexpr int BATCH_NFMAX = 32;  // parameters per frame
struct BatchOut {
    double fnorm, init_avg, avg, mn, mx, rms;
    int info, nfev, njev, func_evals, jac_evals, interrupted, better, failed;
    int measured, pad;
};
struct BatchArgs {
    int nf;                      // frames solved: [0, nf)
    const int *fr_cf_off, *fr_par_off, *fr_par, *fr_last, *fr_nobs;
    const double *pweight;       // paramWeightList (mode 2)
    double *J;                   // [M][2 PCMAX] Jacobian rows of the frame's last Jacobian
    double *ed, *dist;           // errorDistanceList (last measured); distances [2][M]
    double *x;                   // internal parameters, in / out (written when better)
    BatchOut *out;
    const int *interrupt;        // host-mapped stop flag (nullptr: none)
    int solver_type, mode, maxfev, accept_only_better, initial_error_given;
    double delta, factor, ftol, xtol, gtol, initial_error_avg;
};

// The MINPACK decision after a trial point, restated on the device (the
// last k_reduce_multi block, one thread) so that the next Jacobian can be
// enqueued before the host has read the trial: *gate = 1 exactly when the
// host's lmder loop will take this trial, accept it and go on (Plan::solve
// checks its own decision against the record in slots out[0..4]).
struct LmDec {
    int on = 0;
    int spec = 0;    // the speculative trial: lmpar's undamped test decides whether it is used
    int first = 0;   // iter == 1 (delta from ||D x||, delta = min(delta, pnorm))
    int f0 = 0;      // fnorm is x0's: sqrt(scalar[s_f0])
    int nfev = 0, maxfev = 0;
    double fnorm = 0., par = 0., delta = 0., xnorm = 0., gnorm = 0.;
    double factor = 0., ftol = 0., xtol = 0., gtol = 0.;
    int s_pnorm = 0, s_xn2t = 0, s_fnorm = 0, s_jp = 0, s_dnorm = 0, s_fail = 0;
    int s_xn2 = 0, s_gnorm = 0, s_f0 = 0, s_out = 0;
    int *gate = nullptr;
};
// Device buffers of the (partitioned) band factorisation.
struct BandSolver {
    bool use_bd = false;                     // block diagonal + arrow (no solved bundle)
    BdDev bd;
    bool use_bcr = false;                    // w <= 32: block cyclic reduction
    BcrDev bcr;
    // no arrow, w <= 23, every block's workgroup resident: parallel cyclic
    // reduction (the BCR buffers stay as the fallback after a timed-out wait)
    bool use_pcr = false;
    PcrDev pcr;
    // host copies of the ticket counters (every launch draws a known count)
    // and the switch to the per-level launches after a timed-out dataflow wait
    mutable unsigned tick_f = 0, tick_b = 0;
    mutable bool df_off = false;
    // dataflow grid cap (MMBA_BCR_DF_GRID at plan build: a small grid makes
    // most items run on workgroups that already ran others -- the
    // forward-progress test)
    int df_grid = 256;
    // sharded BCR: Bd | Ga | Gd | rhs contiguous; every shard writes its own
    // Schur terms, one all-reduce (sum) assembles S, every shard factors it
    double *red = nullptr, *red_rhs = nullptr;
    size_t red_count = 0;
    int P = 1, w = 0, nb = 0, nG = 0;
    int p_lo = 0, p_hi = 1;                  // partitions this shard factors
    Comm *comm = nullptr;                    // sharded: T, rT are all-reduced
    long long max_arrow = 0;                 // max na*(r1-r0) over partitions
    double *Bd = nullptr, *Ga = nullptr, *Gd = nullptr, *Gdinv = nullptr, *Dinv = nullptr;
    BandPart *d_parts = nullptr;             // P partitions (P == 1: arrow = Ga)
    double *apool = nullptr, *zpool = nullptr, *cpool = nullptr;
    // separator system (P > 1)
    double *TBd = nullptr, *TGa = nullptr, *TGd = nullptr, *TGdinv = nullptr, *TDinv = nullptr;
    size_t tcount = 0;                       // TBd | TGa | TGd are contiguous
    BandPart *d_tpart = nullptr;
    double *rT = nullptr, *yT = nullptr, *xT = nullptr;
    // separator form of the sharded solve (one partition per shard, no
    // arrow): the shard's interior is eliminated by parallel cyclic
    // reduction (ipcr, on the interior rows of Bd) instead of a band
    // Cholesky chain; XA = S_II^-1 A_p^T (column-major, interior rows x na)
    // gives the partition's Schur term A_p XA and the back substitution,
    // y's interior rows hold S_II^-1 r (not L^-1 r)
    bool pcr_int = false;
    PcrDev ipcr;
    BandPart hpart{};                        // the shard's partition (host copy)
    double *XA = nullptr, *izero = nullptr, *ix = nullptr;
    int *fail = nullptr;                     // the plan's failure flag
};

// Where entry (R, C), R >= C, of the reduced system lives.
struct SView {
    int band;  // 0: 64x64 tiles (or dense), 1: band + arrow
    int dense, ld;  // dense: column-major lower triangle, leading dimension ld
    // tiles
    double *S;
    const int *slot;
    int NT;
    // band + arrow
    double *Bd;  // [nb][w+1]
    int w, nb;   // half bandwidth, band rows (= camera-frame parameters)
    double *Ga;  // [nG][nb]
    double *Gd;  // [NGMAX][NGMAX] lower
};

// Parameter classes.
enum ParamClass : int { PC_CF = 0, PC_B = 1, PC_G = 2 };

// Flags on camera-variant entries.
// VF_LENS: the variant is a lens coefficient of the camera-frame (an
// animated coefficient only its own camera-frame's rows read, Plan::build):
// its camera record is the base one and its column perturbs the lens
enum VarFlags : int { VF_BUNDLE_SIDE = 1, VF_LENS = 2 };

// Device view of the problem + derived structure (all device pointers).
struct DevProblem {
    int F, nA, nT, nC, nL, nB, nK, M, n, ncf, nR, nG, mode;
    int nbs;  // bundles with solved parameters (a B block)
    double image_width;
    const int64_t *attr_off;
    const int *attr_anim;
    double *attr_val;  // working copy (setParameters target)
    const int *tfm_parent, *tfm_roo, *tfm_attrs;
    const int *cam_tfm, *cam_attrs, *cam_fit, *cam_size, *cam_lens;
    const int *lens_attrs, *lens_type;
    // input layers of the cameras' lens (deepest first, LENS_LAYER doubles
    // each: type, 14 slot values), constant for the solve (mmba.h ABI 5)
    const double *lens_chain;
    int lens_chain_n;
    // the one lens model every lens instance of the plan uses (no input
    // layers), -1 when mixed or chained: k_jacobian compiles that model only
    int lens_uniform;
    const int *bnd_tfm;
    // observations (device order)
    const int *obs_cf, *obs_bnd, *obs_frame, *obs_cam;
    const double *obs_xy, *obs_sqrtw;
    // camera-frame structure
    const int *cf_cam, *cf_frame, *cf_obs_off, *cf_var_off, *cf_var_param, *cf_var_flags;
    const int *cf_pc, *cf_roff;  // CF-block size and offset in R
    int pc_uniform;              // common CF-block size of solved camera-frames (0: mixed)
    // Schur factors W_i (pc x 3 per observation) are stored per observation
    // (AoS, wst doubles each: 3 * pc_uniform, else 3 * PCMAX) so the
    // destination-sorted gathers of k_schur_dest read 2-3 cache lines per
    // observation instead of one line per entry
    int wst;
    // every pair of a diagonal Schur destination (cf, cf) is (i, i)
    // (k_schur_dest_u loads one W row for both sides)
    int dest_diag_ii;
    // bundle-side parameter lists (B-class first, then bundle-side globals)
    const int *bnd_par_off, *bnd_par;
    const int *bnd_pb;     // B-block size
    const int *bnd_xoff;   // offset of the B block in x (param ids are contiguous? no: list)
    const int *bobs_off, *bobs;  // observations grouped by bundle
    // frame-independent bundles with only B-class parameters ("fast" bundles):
    // bnd_p4[b] = {p0, p1, p2, pb} (pb = -1: generic path).  brec[b*BREC]:
    // world position (3), position with parameter a perturbed (3 x 3), FD step
    // of parameter a (3); written by k_bnd_records once per evaluation so the
    // per-observation kernels read one 128-B record instead of walking
    // bundle -> transform -> attribute tables.
    const int4 *bnd_p4;
    const double *brec;
    int all_bnd_fast;  // every bundle is fast (bnd_p4[b].w >= 0)
    int lmax;          // most local Jacobian columns of any observation (<= LMAX)
    int jcol_implicit; // uniform fast plans: jcol not stored (derived from the structure)
    // camera records through a per-camera-frame table of attribute-value
    // indices (every camera transform without a parent; nullptr otherwise)
    const int *cf_aidx;
    int no_lens;       // no camera has a (3DE classic) lens
    // position of each observation in bundle order (bobs) and the bundle
    // block records JB[8 * obs_bpos[i]] = [jx_a, jy_a] (a < 3), f_x, f_y
    // written by the Jacobian kernels in bundle order, so k_ne_bnd_jb reads
    // each bundle's records contiguously (nullptr unless every solved bundle
    // is fast and nG == 0)
    const int *obs_bpos;
    double *JB;
    // per camera lens parameter lists (the batched per-frame solve, where
    // the reference solves one frame at a time and no index mixes)
    const int *cam_lpar_off, *cam_lpar;
    // lens instances (mmba.h ABI 7): observation i is
    // distorted by instance obs_inst[i] (-1: none) of lens inst_lens[j]; slot
    // k of instance j reads attribute inst_attr[14 j + k] at frame
    // inst_frame[14 j + k] (the parameter the reference's setParameters
    // leaves in that slot), or the plug model's value inst_val[14 j + k] when
    // inst_attr is -1; the instance's lens parameters (ascending ids) are
    // inst_lpar[inst_lpar_off[j] ..)
    const int *obs_inst, *inst_lens, *inst_attr, *inst_frame, *inst_lpar_off, *inst_lpar;
    const double *inst_val;
    // parameters
    const int *p_attr, *p_frame, *p_class, *p_pos, *p_both, *p_blk;
    const double *p_min, *p_max, *p_off, *p_scale;
    const int *g_param;  // global index -> param id
    // frame sharding (nullptr / all-true when unsharded): this shard owns the
    // observations of its frame range, the camera-frames in it (reduced-system
    // rows [Ra, Rb)), the bundles whose first observation it holds, and, on
    // the root shard, the global parameters.
    const int *obs_own, *cf_own, *bnd_own;
    int root, Ra, Rb;
    // attribute stiffness / smoothness rows (mmba_rows.hip): nrows rows after
    // the 2 M marker rows, measured only in Maya DAG mode (rows_live);
    // row_param = the parameter setting the row's (attribute, frame), -1 none
    int nrows, rows_live;
    const int *row_attr, *row_frame, *row_param;
    const double *row_w, *row_var, *row_val;
    // robust loss on every residual row (applyLossFunctionToErrors), when on
    int loss_on, loss_type;
    double loss_scale;
    // rolling shutter (mmba.h ABI 3, mmba_rs.hip): every observation sees its
    // camera's translate / rotate values blended over frames f-1, f, f+1 at
    // its scanline time obs_tau[i] (device order; 0 for a global shutter).
    // cf_rs_nb[2 cf + 0/1] = camera-frame of the same camera at f-1 / f+1
    // (-1: none); cf_rs_vidx[12 cf + k / 6 + k] = attribute-value index of
    // transform attribute k (tx ty tz rx ry rz) at f-1 / f+1 (-1: absent,
    // value 0; -2: outside the frame range, the exporter's extrapolation).
    // Jacobian columns of an observation: its camera-frame's variants, then
    // the CF parameters of cf_rs_nb[0], then those of cf_rs_nb[1], then the
    // lens parameters.  rs_Aoff[(2 cf + d - 1) PCMAX^2]: the camera-frame
    // coupling blocks A(cf, next^d(cf)), d = 1, 2.
    // attribute-value index of every parameter (setParameters' target;
    // one load instead of the parameter -> attribute -> offset chain)
    const long long *p_vidx;
    // fast parentless bundles whose parameters are their own translate
    // attributes: value indices of tx ty tz (w unused) and the translate
    // component of each of the bundle's (up to 3) parameters, 2 bits each
    // (nullptr: some fast bundle needs the transform-table walk)
    const int4 *bnd_vx;
    const int *bnd_pcomp;
    int rs;
    const double *obs_tau;
    const int *cf_rs_nb, *cf_rs_vidx;
    // per camera-frame: the global-parameter columns of its observations'
    // Jacobian rows (same for every observation of the segment): count, then
    // (column, global index) pairs, NGMAX slots each
    const int *cf_rs_gcnt, *cf_rs_gcol, *cf_rs_gidx;
    double *rs_Aoff;
};

__device__ __forceinline__ size_t widx(const DevProblem &P, int k, int i) {
    return (size_t)i * P.wst + k;
}

__device__ __forceinline__ double *s_at(const SView &V, int R, int C) {
    if (V.dense) return &V.S[(size_t)C * V.ld + R];
    if (!V.band) {
        const int s = V.slot[(R / TILE) * V.NT + (C / TILE)];
        return &V.S[(size_t)s * TILE * TILE + (R % TILE) * TILE + (C % TILE)];
    }
    if (R < V.nb) return &V.Bd[(size_t)R * (V.w + 1) + (C - R + V.w)];
    if (C < V.nb) return &V.Ga[(size_t)(R - V.nb) * V.nb + C];
    return &V.Gd[(R - V.nb) * NGMAX + (C - V.nb)];
}

}  // namespace mmba
