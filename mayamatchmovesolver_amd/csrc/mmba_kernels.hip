// mmba_kernels.hip -- CDNA4 (gfx950) kernels of the bundle-adjustment core.
//
// Roofline classes:
//   k_residual, k_jacobian, k_ne_*   HBM / latency bound, one thread per
//                                    observation or per block, coalesced SoA.
//   k_chol_update                    fp64 MFMA (v_mfma_f64_16x16x4_f64),
//                                    64x64 tiles staged in LDS.
//   everything else                  small O(n) vector work.
#include <cfloat>
#include <cstdlib>

#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_red_dev.h"

namespace mmba {

// Frame-sharding ownership (all-true when unsharded).
MMBA_DEV bool own_obs(const DevProblem &P, int i) { return !P.obs_own || P.obs_own[i]; }
MMBA_DEV bool own_cf(const DevProblem &P, int cf) { return !P.cf_own || P.cf_own[cf]; }
MMBA_DEV bool own_bnd(const DevProblem &P, int b) { return !P.bnd_own || P.bnd_own[b]; }
MMBA_DEV bool own_mask(const int *m, int i) { return !m || m[i]; }

// Workgroup b of a G-workgroup grid runs on XCD b mod 8; xcd_remap(b, G) is
// the logical block it takes so that each XCD sweeps one contiguous range of
// logical blocks (a bijection of [0, G)).  Kernels that walk the
// camera-frame-sorted observations, the records they read and the Jacobian
// they write use it alike, so a producer's lines sit in the L2 of the XCD
// that reads them next.
__device__ __forceinline__ int xcd_remap(int b, int G) {
    const int x = b & 7, idx = b >> 3, q = G >> 3, r = G & 7;
    return x * q + min(x, r) + idx;
}

// Deterministic single-launch reduction epilogue (see the reductions section).
template <bool MAX>
__device__ __forceinline__ void finish_blocks(double v, double *partial, double *out,
                                              unsigned int *ticket, int blk = -1) {
    if (blk < 0) blk = blockIdx.x;
    __shared__ int last;
    __shared__ double red[256];
    if (threadIdx.x == 0) {
        if (!ticket) {
            partial[blk] = v;
        } else {
            __hip_atomic_store(&partial[blk], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __threadfence();  // release the partial before the ticket
            last = atomicAdd(ticket, 1u) == gridDim.x - 1;
        }
    }
    if (!ticket) return;
    __syncthreads();
    if (!last) return;
    __threadfence();  // acquire the other blocks' partials
    double a = 0.;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) {
        const double q = __hip_atomic_load(&partial[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a = MAX ? fmax(a, q) : a + q;
    }
    red[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            red[threadIdx.x] = MAX ? fmax(red[threadIdx.x], red[threadIdx.x + w])
                                   : red[threadIdx.x] + red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *out = red[0];
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// 3 x 3 damped bundle factor of one bundle (k_bundle_factor's arithmetic):
// A (pb x pb block, identity padding), rhs = gB (0 on padding), dd = diag of
// the bundle's parameters -> Lb, tb = Lb^-1 rhs; L / il returned for the
// arrow columns.
__device__ __forceinline__ void bundle_chol3(double (&A)[3][3], double (&rhs)[3],
                                             const double (&dd)[3], int pb, double lam, int b,
                                             double *Lb, double *tb, int *fail,
                                             double (*Lo)[3] = nullptr, double *ilo = nullptr) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (a < pb) {
            const double d = dd[a];
            A[a][a] += lam * (d * d);
            if (A[a][a] == 0.) {
                A[a][a] = 1.;
                rhs[a] = 0.;
            }
        }
    }
    double L[3][3] = {}, il[3];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double s = A[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
        if (!(s > 0.)) {
            ok = false;
            s = 1.;
        }
        L[j][j] = sqrt(s);
        il[j] = 1.0 / L[j][j];
#pragma unroll
        for (int i = j + 1; i < 3; ++i) {
            double t = A[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
            L[i][j] = t * il[j];
        }
    }
    if (!ok) atomicOr(fail, 1);
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) Lb[(size_t)b * 9 + a * 3 + c] = (a < pb) ? L[a][c] : 0.;
    double t[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double s = rhs[a];
#pragma unroll
        for (int k = 0; k < a; ++k) s -= L[a][k] * t[k];
        t[a] = s * il[a];  // zero on padding rows (rhs 0)
    }
    for (int a = 0; a < 3; ++a) tb[(size_t)b * 3 + a] = t[a];
    if (Lo) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            ilo[a] = il[a];
#pragma unroll
            for (int c = 0; c < 3; ++c) Lo[a][c] = L[a][c];
        }
    }
}

// reduce_row_block by one wave (a 64-thread workgroup of another launch):
// lane t holds the block's threads t, t + 64, t + 128 and t + 192 and combines
// them, then the lanes, in that block's tree order -- the same value.
__device__ __forceinline__ double reduce_row_w64(const double *partial, const RedRow &rw) {
    const bool mx = rw.is_max != 0;
    const int t = threadIdx.x & 63;
    double s[4];
    constexpr int JB = 6;  // rows of up to 1,536 entries (C4: 1,282): every load issued first
    if (rw.n <= 256 * JB) {
        double q[4][JB];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < JB; ++j) {
                const int i = t + 64 * k + 256 * j;
                q[k][j] = i < rw.n ? partial[rw.off + i] : 0.;
            }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double v = 0.;
#pragma unroll
            for (int j = 0; j < JB; ++j)
                if (t + 64 * k + 256 * j < rw.n) v = mx ? fmax(v, q[k][j]) : v + q[k][j];
            s[k] = v;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double v = 0.;
            for (int i = t + 64 * k; i < rw.n; i += 256) {
                const double q = partial[rw.off + i];
                v = mx ? fmax(v, q) : v + q;
            }
            s[k] = v;
        }
    }
    const double a0 = mx ? fmax(s[0], s[2]) : s[0] + s[2];  // w = 128
    const double a1 = mx ? fmax(s[1], s[3]) : s[1] + s[3];
    double r = mx ? fmax(a0, a1) : a0 + a1;                 // w = 64
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        const double o = __shfl_down(r, w);
        if (t < w) r = mx ? fmax(r, o) : r + o;
    }
    return r;  // lane 0
}

// Every row of spec at once (the last workgroup of a folded launch): each
// thread issues its loads of all rows before any sum, then one fixed tree
// per row, level by level for all rows -- per row the arithmetic of
// reduce_row_block (and so of k_reduce_multi).
constexpr int RED_ROWS = 8;
__device__ __forceinline__ void reduce_rows_sc1(const RedSpec &spec, const double *partial,
                                                double *scalar) {
    __shared__ double red[RED_ROWS][256];
    const int nr = spec.nrows;
    double sv[RED_ROWS];
#pragma unroll
    for (int r = 0; r < RED_ROWS; ++r) {
        sv[r] = 0.;
        if (r < nr) {
            const RedRow rw = spec.row[r];
            const bool mx = rw.is_max != 0;
            for (int i = threadIdx.x; i < rw.n; i += blockDim.x) {
                const double q = ld_sc1(&partial[rw.off + i]);
                sv[r] = mx ? fmax(sv[r], q) : sv[r] + q;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RED_ROWS; ++r)
        if (r < nr) red[r][threadIdx.x] = sv[r];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
#pragma unroll
            for (int r = 0; r < RED_ROWS; ++r) {
                if (r >= nr) break;
                const bool mx = spec.row[r].is_max != 0;
                red[r][threadIdx.x] = mx ? fmax(red[r][threadIdx.x], red[r][threadIdx.x + w])
                                         : red[r][threadIdx.x] + red[r][threadIdx.x + w];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < nr) scalar[spec.row[threadIdx.x].slot] = red[threadIdx.x][0];
    __syncthreads();
}

// Last-workgroup epilogue of a launch whose workgroups stored partials with
// st_sc1 (or an earlier launch stored them): every storing wave drains, one
// lane adds to the ticket (agent scope), the workgroup whose add came last
// loads every partial sc1 (MI355X guide, valid forms, first table row) and
// reduces the rows of spec into scalar; the ticket is reset for the next
// user.  256 threads per workgroup.
__device__ __forceinline__ void tail_reduce(const RedSpec &spec, const double *partial,
                                            double *scalar, unsigned *ticket) {
    __shared__ unsigned last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    reduce_rows_sc1(spec, partial, scalar);
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tail_reduce plus the rest of k_reduce_multi's work: the fail flag to its
// slot (then cleared) and the host mirror of scalar[0, host_n).
__device__ __forceinline__ void tail_reduce_full(const RedTail &T) {
    __shared__ unsigned last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(T.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    reduce_rows_sc1(T.spec, T.partial, T.scalar);
    if (threadIdx.x == 0 && T.flag && T.spec.flag_slot >= 0) {
        T.scalar[T.spec.flag_slot] = (double)*T.flag;  // bit 1 pivot, bit 2 dataflow timeout
        *T.flag = 0;
    }
    if (T.host) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int i = threadIdx.x; i < T.host_n; i += blockDim.x) T.host[i] = ld_sc1(&T.scalar[i]);
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(T.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// -------------------------------------------------------------------------
// Parameters: external values, FD perturbations (adjust_solveFunc.cpp:148-180,
// cminpack fdjac2), setParameters (adjust_setParameters.cpp:174-250).
// -------------------------------------------------------------------------
__device__ __forceinline__ void param_prep_one(const DevProblem &P, int p, double v, double *ext,
                                               double *ext_pert, double *step, int solver_type,
                                               double delta, double eps_dif) {
    const double xmin = P.p_min[p], xmax = P.p_max[p], off = P.p_off[p], sc = P.p_scale[p];
    ext[p] = int_to_ext(v, xmin, xmax, off, sc);
    double st;
    const double xp = fd_point(v, xmin, xmax, solver_type, delta, eps_dif, st);
    step[p] = st;
    ext_pert[p] = int_to_ext(xp, xmin, xmax, off, sc);
}

__device__ __forceinline__ void set_attr_one(const DevProblem &P, int p, double value) {
    P.attr_val[P.p_vidx[p]] = value;
}

__global__ void k_param_prep(DevProblem P, const double *__restrict__ x, double *ext,
                             double *ext_pert, double *step, int solver_type, double delta,
                             double eps_dif) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    param_prep_one(P, p, x[p], ext, ext_pert, step, solver_type, delta, eps_dif);
}

// Central differences, second evaluation of each column
// (solveFunc_calculateJacobianMatrixForParameter, adjust_solveFunc.cpp:405-475):
// deltaB = calculateParameterDelta(value, delta, -1); when deltaB == deltaA the
// column stays a forward difference (stepB = 0), otherwise the column is
// (f(x + deltaA) - f(x + deltaB)) * 0.5 / (|deltaA| + |deltaB|) (B8), with
// stepB holding that factor.  count += number of central columns (each one
// is a second incrementJacobianIteration).
__global__ void k_param_central(DevProblem P, const double *__restrict__ x, double *ext_pertB,
                                double *stepB, double delta, double *count, double *c15) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    const double v = x[p];
    const double xmin = P.p_min[p], xmax = P.p_max[p];
    double sa = 1., sb = -1.;
    if ((v + delta) > xmax) sa = sb = -1.;
    if ((v - delta) < xmin) sa = sb = 1.;
    const double dA = delta * sa, dB = delta * sb;
    if (dA == dB) {
        stepB[p] = 0.;
        ext_pertB[p] = 0.;
        if (c15) c15[p] = 0.;
        return;
    }
    stepB[p] = 0.5 / (fabs(dA) + fabs(dB));
    // B15: an animated column's measureErrors skips the other frames, whose
    // rows keep errorListA = errors and errorListB = 0
    // (adjust_solveFunc.cpp:331-333, 412, 468-471): J_jp = f_j c_p there
    if (c15) c15[p] = P.p_frame[p] >= 0 ? stepB[p] : 0.;
    ext_pertB[p] = int_to_ext(v + dB, xmin, xmax, P.p_off[p], P.p_scale[p]);
    atomicAdd(count, 1.0);
}

__global__ void k_set_attrs(DevProblem P, const double *__restrict__ ext) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    set_attr_one(P, p, ext[p]);
}

// setParameters in one launch: external value, FD perturbation and the
// attribute write of each parameter (k_param_prep + k_set_attrs).
__global__ void k_param_set(DevProblem P, const double *__restrict__ x, double *ext,
                            double *ext_pert, double *step, int solver_type, double delta,
                            double eps_dif) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    param_prep_one(P, p, x[p], ext, ext_pert, step, solver_type, delta, eps_dif);
    set_attr_one(P, p, ext[p]);
}

// -------------------------------------------------------------------------
// Camera-frame records: variant 0 = base, variant v = one cam-side parameter
// perturbed (K0 in SURVEY 7).
// -------------------------------------------------------------------------
__device__ __forceinline__ void cam_record_thread(const DevProblem &P, int t,
                                                  const int *__restrict__ var_cf,
                                                  const double *__restrict__ ext_pert,
                                                  double *recs, int nvar, int base_only) {
    int cf, idx;
    if (base_only) {
        if (t >= P.ncf) return;
        cf = t;
        idx = P.cf_var_off[cf];
    } else {
        if (t >= nvar) return;
        idx = t;
        cf = var_cf[t];
    }
    Override ov{-1, 0.};
    const int p = P.cf_var_param[idx];
    if (p >= 0) {
        ov.attr = P.p_attr[p];
        ov.value = ext_pert[p];
    }
    if (P.cf_aidx) {
        long long ov_idx = -1;
        if (p >= 0) ov_idx = P.p_vidx[p];  // the variant's parameter (at this frame)
        camera_record_fast(P, cf, ov_idx, ov.value, &recs[(size_t)idx * CAMREC], ov.attr);
        return;
    }
    camera_record(P, P.cf_cam[cf], P.cf_frame[cf], ov, &recs[(size_t)idx * CAMREC]);
}

// -------------------------------------------------------------------------
// Bundle records (fast bundles, see DevProblem::bnd_p4): one thread per
// bundle walks the bundle's transform/attribute tables once per evaluation.
// -------------------------------------------------------------------------
__device__ __forceinline__ void bnd_record_thread(const DevProblem &P, int b,
                                                  const double *__restrict__ ext_pert,
                                                  const double *__restrict__ step, double *brec,
                                                  int base_only) {
    if (b >= P.nB) return;
    const int4 p4 = P.bnd_p4[b];
    if (p4.w < 0) return;
    double *br = &brec[(size_t)b * BREC];
    if (P.bnd_vx) {
        // parentless: the position is (tx, ty, tz) and parameter a replaces
        // one component (bundle_position's values, without the table walk)
        const int4 vx = P.bnd_vx[b];
        const double base[3] = {vx.x >= 0 ? P.attr_val[vx.x] : 0., vx.y >= 0 ? P.attr_val[vx.y] : 0.,
                                vx.z >= 0 ? P.attr_val[vx.z] : 0.};
        br[0] = base[0];
        br[1] = base[1];
        br[2] = base[2];
        if (base_only) return;
        const int pcm = P.bnd_pcomp[b];
        for (int a = 0; a < p4.w; ++a) {
            const int p = a == 0 ? p4.x : (a == 1 ? p4.y : p4.z);
            const int comp = (pcm >> (2 * a)) & 3;
            const double v = ext_pert[p];
            br[3 + 3 * a] = comp == 0 ? v : base[0];
            br[4 + 3 * a] = comp == 1 ? v : base[1];
            br[5 + 3 * a] = comp == 2 ? v : base[2];
            br[12 + a] = step[p];
        }
        return;
    }
    const Override none{-1, 0.};
    double bp[3];
    bundle_position(P, b, 0, none, bp);  // frame-independent: any frame
    br[0] = bp[0];
    br[1] = bp[1];
    br[2] = bp[2];
    if (base_only) return;
    for (int a = 0; a < p4.w; ++a) {
        const int p = a == 0 ? p4.x : (a == 1 ? p4.y : p4.z);
        const Override ov{P.p_attr[p], ext_pert[p]};
        bundle_position(P, b, 0, ov, bp);
        br[3 + 3 * a] = bp[0];
        br[4 + 3 * a] = bp[1];
        br[5 + 3 * a] = bp[2];
        br[12 + a] = step[p];
    }
}

// Camera-frame and bundle records in one launch (both are short, latency-
// bound chains; blocks [0, ncb) are camera records, the rest bundle records).
__global__ void __launch_bounds__(64) k_records(DevProblem P, const int *__restrict__ var_cf,
                                                const double *__restrict__ ext_pert,
                                                const double *__restrict__ step, double *recs,
                                                int nvar, double *brec, int base_only, int ncb) {
    // ncb is a multiple of 8 (launch_records), so both ranges start on XCD 0
    // and each maps XCD-contiguously (the K2 and residual passes read these
    // records on the XCD that owns the same camera-frames / bundles)
    if ((int)blockIdx.x < ncb)
        cam_record_thread(P, xcd_remap(blockIdx.x, ncb) * 64 + threadIdx.x, var_cf, ext_pert,
                          recs, nvar, base_only);
    else
        bnd_record_thread(P, xcd_remap(blockIdx.x - ncb, gridDim.x - ncb) * 64 + threadIdx.x,
                          ext_pert, step, brec, base_only);
}

// -------------------------------------------------------------------------
// Residuals (measureErrors).  Writes f (device order), user deviation and
// distance, and one partial sum of squares per block.
// -------------------------------------------------------------------------
// JP: the trial-point evaluation also forms (J p)_obs = sum_l J_l p[jcol_l]
// from the Jacobian blocks of the current x (lmder's ||J p|| for prered,
// k_jp_sumsq) into a second partial row.
// FAST: every bundle is fast and no camera has a lens (the transform-chain
// and lens code, and their registers, are compiled out).
// RS: rolling shutter (mmba_rs.hip): each observation's camera record is
// its own scanline pose (camera_record_rs), not the camera-frame's.
template <bool JP, bool FAST, bool RS = false>
__global__ void __launch_bounds__(256) k_residual(DevProblem P, const double *__restrict__ recs,
                                                  double *f, double *eu, double *ed,
                                                  double *partial, double *out,
                                                  unsigned int *ticket,
                                                  const double *__restrict__ J,
                                                  const int *__restrict__ jcol,
                                                  const int *__restrict__ nloc,
                                                  const double *__restrict__ pstep,
                                                  double *partial_jp, double *dist,
                                                  const RedTail T) {
    __shared__ double red[256];
    const int lb = xcd_remap(blockIdx.x, gridDim.x);  // logical block (XCD-contiguous)
    const int i = lb * blockDim.x + threadIdx.x;
    double s = 0., sj = 0.;
    if (i < P.M) {
        const int cf = P.obs_cf[i];
        const int b = P.obs_bnd[i];
        const int fr = P.obs_frame[i];
        const Override none{-1, 0.};
        double bp[3];
        if (FAST) {
            const double *br = &P.brec[(size_t)b * BREC];
            bp[0] = br[0];
            bp[1] = br[1];
            bp[2] = br[2];
        } else {
            base_bundle(P, b, fr, bp);
        }
        double lc[MMBA_LENS_NUM_ATTRS];
        int inst = -1;
        const int hl = FAST ? MMBA_LENS_NONE : obs_lens_inst(P, i, inst);
        if (hl) inst_coeffs(P, inst, none, lc);
        const double *rec = &recs[(size_t)P.cf_var_off[cf] * CAMREC];
        double rloc[RS ? CAMREC : 1];
        if constexpr (RS) {
            camera_record_rs(P, cf, P.obs_tau[i], -1, 0., rloc);
            rec = rloc;
        }
        Resid r = residual_l(P, rec, bp, P.obs_xy[2 * i], P.obs_xy[2 * i + 1], P.obs_sqrtw[i],
                             hl, lc);
        f[2 * i] = r.ex;
        f[2 * i + 1] = r.ey;
        if (eu) {
            eu[2 * i] = r.ux;
            eu[2 * i + 1] = r.uy;
            ed[i] = r.dist;
        }
        if (dist) dist[i] = r.dist;  // errorDistanceList of this point (RMS at the accepted x)
        if (own_obs(P, i)) {
            s = r.ex * r.ex + r.ey * r.ey;
            if constexpr (JP) {
                const int M = P.M;
                double ax = 0., ay = 0.;
                const int nl = nloc[i];
                if (P.jcol_implicit) {
                    // uniform plans: column l is camera variant l (l < nv), then
                    // the bundle's parameters (k_jacobian_u's order).  Eight
                    // columns' index, step and J loads issued before their
                    // products (the sums in column order as before)
                    const int voff = P.cf_var_off[cf];
                    const int nv = P.cf_var_off[cf + 1] - voff - 1;
                    const int4 p4 = P.bnd_p4[b];
                    for (int l0 = 0; l0 < nl; l0 += 8) {
                        double jx[8], jy[8], pv[8];
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            const int l = l0 + k;
                            if (l < nl) {
                                const int a = l - nv;
                                const int p = l < nv ? P.cf_var_param[voff + 1 + l]
                                                     : (a == 0 ? p4.x : (a == 1 ? p4.y : p4.z));
                                pv[k] = pstep[p];
                                jx[k] = J[(size_t)(2 * l) * M + i];
                                jy[k] = J[(size_t)(2 * l + 1) * M + i];
                            }
                        }
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            if (l0 + k < nl) {
                                ax += jx[k] * pv[k];
                                ay += jy[k] * pv[k];
                            }
                        }
                    }
                } else {
                    for (int l = 0; l < nl; ++l) {
                        const double pv = pstep[jcol[(size_t)l * M + i]];
                        ax += J[(size_t)(2 * l) * M + i] * pv;
                        ay += J[(size_t)(2 * l + 1) * M + i] * pv;
                    }
                }
                sj = ax * ax + ay * ay;
            }
        }
    }
    if constexpr (JP) {
        red[threadIdx.x] = sj;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            if (T.on)
                st_sc1(&partial_jp[lb], red[0]);  // read by this launch's last workgroup
            else
                partial_jp[lb] = red[0];
        }
        __syncthreads();
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (T.on) {
        if (threadIdx.x == 0) st_sc1(&partial[lb], red[0]);
        tail_reduce_full(T);
        return;
    }
    finish_blocks<false>(red[0], partial, out, ticket, lb);
}

// Trial point on uniform fast plans (one workgroup per camera-frame
// segment, the plans of k_jac_ne_u): the camera-frame's base record and the
// steps p of its camera parameters are staged once in LDS, where
// k_residual<JP, FAST> reaches them per observation through three dependent
// tables (obs_cf -> cf_var_off -> cf_var_param -> p).  Per observation the
// same residual and (J p) arithmetic as k_residual<true, true>; one partial
// per camera-frame (stored at the camera-frame index), in the
// XCD-contiguous order of k_jac_ne_u, whose records and J rows it reads.
template <int PC>
__global__ void __launch_bounds__(256) k_residual_jp_cf(
    DevProblem P, const double *__restrict__ recs, double *f, double *eu, double *ed,
    double *partial, const double *__restrict__ J, const int *__restrict__ nloc,
    const double *__restrict__ pstep, double *partial_jp, double *dist) {
    __shared__ double sRec[CAMREC];
    __shared__ double sP[PC];
    __shared__ int sNv;
    __shared__ double red[2][256];
    const int cf = xcd_remap(blockIdx.x, gridDim.x);
    const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
    const int tid = threadIdx.x;
    {
        const int voff = P.cf_var_off[cf];
        const int nv = P.cf_var_off[cf + 1] - voff - 1;
        if (tid < CAMREC) sRec[tid] = recs[(size_t)voff * CAMREC + tid];
        if (tid < PC) sP[tid] = tid < nv ? pstep[P.cf_var_param[voff + 1 + tid]] : 0.;
        if (tid == 0) sNv = nv;
    }
    __syncthreads();
    const int nv = sNv;
    const int M = P.M;
    double s = 0., sj = 0.;
    for (int i = o0 + tid; i < o1; i += 256) {
        const int b = P.obs_bnd[i];
        const double *br = &P.brec[(size_t)b * BREC];
        const double bp[3] = {br[0], br[1], br[2]};
        const int4 p4 = P.bnd_p4[b];
        const int nl = nloc[i];
        const Resid r = residual_l(P, sRec, bp, P.obs_xy[2 * i], P.obs_xy[2 * i + 1],
                                   P.obs_sqrtw[i], MMBA_LENS_NONE, nullptr);
        f[2 * i] = r.ex;
        f[2 * i + 1] = r.ey;
        if (eu) {
            eu[2 * i] = r.ux;
            eu[2 * i + 1] = r.uy;
            ed[i] = r.dist;
        }
        if (dist) dist[i] = r.dist;
        if (own_obs(P, i)) {
            s += r.ex * r.ex + r.ey * r.ey;
            // column l is camera variant l (l < nv), then the bundle's
            // parameters (k_residual<JP>'s implicit-jcol order); every J row
            // and step load issued before the products (nl <= PC + 3), the
            // sums in column order as before
            constexpr int NL = PC + 3;
            double jx[NL], jy[NL], pv[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                if (l < nl) {
                    const int a = l - nv;
                    pv[l] = l < nv ? sP[l] : pstep[a == 0 ? p4.x : (a == 1 ? p4.y : p4.z)];
                    jx[l] = J[(size_t)(2 * l) * M + i];
                    jy[l] = J[(size_t)(2 * l + 1) * M + i];
                }
            }
            double ax = 0., ay = 0.;
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                if (l < nl) {
                    ax += jx[l] * pv[l];
                    ay += jy[l] * pv[l];
                }
            }
            sj += ax * ax + ay * ay;
        }
    }
    red[0][tid] = s;
    red[1][tid] = sj;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            red[0][tid] += red[0][tid + w];
            red[1][tid] += red[1][tid + w];
        }
        __syncthreads();
    }
    if (tid == 0) {
        partial[cf] = red[0][0];
        partial_jp[cf] = red[1][0];
    }
}

// -------------------------------------------------------------------------
// FD Jacobian blocks per observation (K1/K2 in SURVEY 7): same differences
// as solveFunc_calculateJacobianMatrixForParameter, evaluated only for the
// parameters that can change this observation (all other entries of the
// reference column are exactly zero).
// -------------------------------------------------------------------------
// CEN: central differences / B15 compiled in (CB.recs != nullptr).  The
// forward-difference build drops the deltaB evaluations and is held to two
// waves per SIMD (256 VGPRs, some spilled; one wave at 340 registers before):
// C5 1.21 against 1.33 ms per solve (profiles/r5_jac/).
template <bool CEN, int LT = -1>
__global__ void __launch_bounds__(128, CEN ? 1 : 2) k_jacobian(DevProblem P, const double *__restrict__ recs,
                                                  const double *__restrict__ ext_pert,
                                                  const double *__restrict__ step,
                                                  int solver_type, double *J, int *jcol,
                                                  int *nloc, const int *__restrict__ stale_param,
                                                  double *eu, double *ed, CentralB CB) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.M) return;
    const int M = P.M;
    const int cf = P.obs_cf[i];
    const int b = P.obs_bnd[i];
    const int fr = P.obs_frame[i];
    const double mx = P.obs_xy[2 * i], my = P.obs_xy[2 * i + 1], sw = P.obs_sqrtw[i];
    const Override none{-1, 0.};
    const int4 p4 = P.bnd_p4[b];
    double bp0[3];
    base_bundle(P, b, fr, bp0);
    double lc0[MMBA_LENS_NUM_ATTRS];
    int inst = -1;
    const int hl = obs_lens_inst(P, i, inst);
    if (hl) inst_coeffs(P, inst, none, lc0);
    const int voff = P.cf_var_off[cf];
    const int nvar = P.cf_var_off[cf + 1] - voff;
    const double *rec0 = &recs[(size_t)voff * CAMREC];
    const Resid r0 = residual_l<LT>(P, rec0, bp0, mx, my, sw, hl, lc0);
    const bool lmder = solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const int pstale = stale_param[fr];
    Resid rs = r0;
    int l = 0;
    double ljx = 0., ljy = 0.;  // last emitted column (bundle block record)
    // evalB: the column's second (deltaB) evaluation, run only for a central
    // column (CB.step[p] != 0)
    auto emit_s = [&](int p, const Resid &r, double st, auto &&evalB) {
        double jx, jy;
        const double sB = (CEN && lmder && CB.recs) ? CB.step[p] : 0.;
        if (sB != 0.) {  // central: (f(x + dA) - f(x + dB)) * 0.5 / (|dA| + |dB|)
            const Resid rb = evalB();
            jx = (r.ex - rb.ex) * sB;
            jy = (r.ey - rb.ey) * sB;
            if (p == pstale) rs = rb;  // the column's last measureErrors
        } else {
            if (lmder) {  // st = 1/delta, multiplied (adjust_solveFunc.cpp:395-402)
                jx = (r.ex - r0.ex) * st;
                jy = (r.ey - r0.ey) * st;
            } else {      // st = h, divided (fdjac2)
                jx = (r.ex - r0.ex) / st;
                jy = (r.ey - r0.ey) / st;
            }
            if (p == pstale) rs = r;
        }
        J[(size_t)(2 * l) * M + i] = jx;
        J[(size_t)(2 * l + 1) * M + i] = jy;
        jcol[(size_t)l * M + i] = p;
        ljx = jx;
        ljy = jy;
        ++l;
    };
    // camera-side parameters (variants 1..nvar-1)
    for (int v = 1; v < nvar && l < LMAX; ++v) {
        const int t = voff + v;
        const int p = P.cf_var_param[t];
        const bool bside = (P.cf_var_flags[t] & VF_BUNDLE_SIDE) != 0;
        if (P.cf_var_flags[t] & VF_LENS) {
            // a lens coefficient in the camera-frame block: the lens loop's
            // column (below), at its place in the block -- where this
            // observation's lens instance holds the coefficient (B3 may give
            // it an instance another frame's parameter wrote: then f - f = 0)
            bool holds = false;
            if (hl)
                for (int q = P.inst_lpar_off[inst]; q < P.inst_lpar_off[inst + 1]; ++q)
                    holds |= P.inst_lpar[q] == p;
            double lc[MMBA_LENS_NUM_ATTRS];
            if (holds) inst_coeffs(P, inst, Override{P.p_attr[p], ext_pert[p]}, lc);
            emit_s(p, residual_l<LT>(P, rec0, bp0, mx, my, sw, hl, holds ? lc : lc0), step[p], [&]() {
                double lq[MMBA_LENS_NUM_ATTRS];
                if (holds) inst_coeffs(P, inst, Override{P.p_attr[p], CB.ext_pert[p]}, lq);
                return residual_l<LT>(P, rec0, bp0, mx, my, sw, hl, holds ? lq : lc0);
            });
            continue;
        }
        double bp[3] = {bp0[0], bp0[1], bp0[2]};
        if (bside) bundle_position(P, b, fr, Override{P.p_attr[p], ext_pert[p]}, bp);
        emit_s(p, residual_l<LT>(P, &recs[(size_t)t * CAMREC], bp, mx, my, sw, hl, lc0), step[p],
               [&]() {
                   double bq[3] = {bp0[0], bp0[1], bp0[2]};
                   if (bside) bundle_position(P, b, fr, Override{P.p_attr[p], CB.ext_pert[p]}, bq);
                   return residual_l<LT>(P, &CB.recs[(size_t)t * CAMREC], bq, mx, my, sw, hl, lc0);
               });
    }
    if (CEN && CB.q15) {
        // B15 (Plan::b15): the camera-frame block's columns (the first pc
        // emitted) in the basis Q_cf (Q c = kappa e_0): J_s Q = J Q - f kappa
        // e_0^T with J the central differences of the block's own frame.  The
        // large f c part of the block lands in one column, so the block's
        // normal equations keep the accuracy of its differences.
        const int pc = P.cf_pc[cf];
        const double *Q = CB.q15 + (size_t)cf * PCMAX * PCMAX;
        const double kap = CB.kap15[cf];
        double ax[PCMAX], ay[PCMAX];
#pragma unroll
        for (int a = 0; a < PCMAX; ++a) {
            ax[a] = a < pc ? J[(size_t)(2 * a) * M + i] : 0.;
            ay[a] = a < pc ? J[(size_t)(2 * a + 1) * M + i] : 0.;
        }
#pragma unroll
        for (int a2 = 0; a2 < PCMAX; ++a2) {
            if (a2 >= pc) break;
            double sx = 0., sy = 0.;
#pragma unroll
            for (int a = 0; a < PCMAX; ++a) {
                sx = fma(ax[a], Q[a * PCMAX + a2], sx);
                sy = fma(ay[a], Q[a * PCMAX + a2], sy);
            }
            if (a2 == 0) {
                sx -= r0.ex * kap;
                sy -= r0.ey * kap;
            }
            J[(size_t)(2 * a2) * M + i] = sx;
            J[(size_t)(2 * a2 + 1) * M + i] = sy;
        }
    }
    // bundle-side parameters not already covered by a camera variant
    if (p4.w >= 0) {  // fast bundle: perturbed positions from the record
        const double *br = &P.brec[(size_t)b * BREC];
        double jb[8] = {0., 0., 0., 0., 0., 0., r0.ex, r0.ey};
        for (int a = 0; a < p4.w && l < LMAX; ++a) {
            const int p = a == 0 ? p4.x : (a == 1 ? p4.y : p4.z);
            const double bp[3] = {br[3 + 3 * a], br[4 + 3 * a], br[5 + 3 * a]};
            emit_s(p, residual_l<LT>(P, rec0, bp, mx, my, sw, hl, lc0), br[12 + a], [&]() {
                const double *bb = &CB.brec[(size_t)b * BREC];
                const double bq[3] = {bb[3 + 3 * a], bb[4 + 3 * a], bb[5 + 3 * a]};
                return residual_l<LT>(P, rec0, bq, mx, my, sw, hl, lc0);
            });
            jb[2 * a] = ljx;
            jb[2 * a + 1] = ljy;
        }
        // bundle block record, one 64-B record per observation (coalesced
        // store; k_ne_bnd_jb gathers one record per observation of a bundle
        // instead of 8 SoA rows): [jx_a, jy_a]_a, f_x, f_y
        if (P.JB) {
            double4 *dst = reinterpret_cast<double4 *>(&P.JB[(size_t)P.obs_bpos[i] * 8]);
            dst[0] = make_double4(jb[0], jb[1], jb[2], jb[3]);
            dst[1] = make_double4(jb[4], jb[5], jb[6], jb[7]);
        }
    }
    for (int q = p4.w >= 0 ? P.bnd_par_off[b + 1] : P.bnd_par_off[b];
         q < P.bnd_par_off[b + 1] && l < LMAX; ++q) {
        const int p = P.bnd_par[q];
        if (P.p_frame[p] >= 0 && P.p_frame[p] != fr) continue;
        if (P.p_both[p]) {
            bool seen = false;
            for (int v = 1; v < nvar; ++v) seen |= (P.cf_var_param[voff + v] == p);
            if (seen) continue;
        }
        double bp[3];
        bundle_position(P, b, fr, Override{P.p_attr[p], ext_pert[p]}, bp);
        emit_s(p, residual_l<LT>(P, rec0, bp, mx, my, sw, hl, lc0), step[p], [&]() {
            double bq[3];
            bundle_position(P, b, fr, Override{P.p_attr[p], CB.ext_pert[p]}, bq);
            return residual_l<LT>(P, rec0, bq, mx, my, sw, hl, lc0);
        });
    }
    // the lens parameters this observation's lens instance holds (an
    // instance slot has one attribute, so overriding by attribute moves only
    // the slot the parameter writes)
    if (hl) {
        for (int q = P.inst_lpar_off[inst]; q < P.inst_lpar_off[inst + 1] && l < LMAX; ++q) {
            const int p = P.inst_lpar[q];
            // an animated parameter's column re-measures its own frame only
            // (adjust_solveFunc.cpp frameIndexEnable): the observations of
            // other frames that read the instance it writes keep f - f = 0
            if (P.p_frame[p] >= 0 && P.p_frame[p] != fr) continue;
            if (P.p_class[p] == PC_CF) continue;  // a camera-frame block column (VF_LENS)
            double lc[MMBA_LENS_NUM_ATTRS];
            inst_coeffs(P, inst, Override{P.p_attr[p], ext_pert[p]}, lc);
            emit_s(p, residual_l<LT>(P, rec0, bp0, mx, my, sw, hl, lc), step[p], [&]() {
                double lq[MMBA_LENS_NUM_ATTRS];
                inst_coeffs(P, inst, Override{P.p_attr[p], CB.ext_pert[p]}, lq);
                return residual_l<LT>(P, rec0, bp0, mx, my, sw, hl, lq);
            });
        }
    }
    nloc[i] = l;
    // errorList / errorDistanceList as left by the last FD column (Appendix B13).
    if (eu) {
        eu[2 * i] = rs.ux;
        eu[2 * i + 1] = rs.uy;
        ed[i] = rs.dist;
    }
}

// Camera-frame-uniform inputs of one observation's fast Jacobian: the
// camera-frame's record block (base record, then variant v at (1 + v) *
// CAMREC), its variant parameters and steps, and the stale column of its
// frame.  k_jac_ne_u (one workgroup per camera-frame) stages them once in
// LDS; k_jacobian_u (one thread per observation) loads them per thread.
template <int NCV>
struct JacCf {
    const double *rcf;
    int pv[NCV];
    double st[NCV];
    int nv, fr, pstale;
};

template <int NCV>
__device__ __forceinline__ JacCf<NCV> jac_cf_load(const DevProblem &P, int cf,
                                                  const double *__restrict__ recs,
                                                  const double *__restrict__ step,
                                                  const int *__restrict__ stale_param) {
    JacCf<NCV> C;
    const int voff = P.cf_var_off[cf];
    C.nv = min(P.cf_var_off[cf + 1] - voff - 1, NCV);
#pragma unroll
    for (int v = 0; v < NCV; ++v) C.pv[v] = v < C.nv ? P.cf_var_param[voff + 1 + v] : -1;
#pragma unroll
    for (int v = 0; v < NCV; ++v) C.st[v] = v < C.nv ? step[C.pv[v]] : 1.;
    C.rcf = &recs[(size_t)voff * CAMREC];
    C.fr = P.cf_frame[cf];
    C.pstale = stale_param[C.fr];
    return C;
}

// One observation of the uniform fast Jacobian: writes its J columns (and
// jcol / the bundle block record / the stale errorList) and returns the
// camera columns and f at x for a fused normal-equation accumulation.
template <int NCV, bool GEN>  // GEN: some bundle needs the transform-chain path
__device__ __forceinline__ void jac_obs_u(const DevProblem &P, int i, const JacCf<NCV> &C,
                                          bool lmder, double *__restrict__ J,
                                          int *__restrict__ jcol, int *__restrict__ nloc,
                                          double *__restrict__ eu, double *__restrict__ ed,
                                          double (&cx)[NCV], double (&cy)[NCV], double &fx,
                                          double &fy) {
    const int M = P.M;
    const int b = P.obs_bnd[i];
    const int fr = C.fr;
    const double mx = P.obs_xy[2 * i], my = P.obs_xy[2 * i + 1], sw = P.obs_sqrtw[i];
    const int4 p4 = P.bnd_p4[b];
    const int nv = C.nv;
    const int pstale = C.pstale;
    double bp0[3];
    if (GEN) {
        base_bundle(P, b, fr, bp0);
    } else {
        const double *br0 = &P.brec[(size_t)b * BREC];
        bp0[0] = br0[0];
        bp0[1] = br0[1];
        bp0[2] = br0[2];
    }
    const int nb = p4.w > 0 ? p4.w : 0;
    const double *__restrict__ br = &P.brec[(size_t)b * BREC];
    const double *__restrict__ rec0 = C.rcf;
    const Resid r0 = residual(rec0, bp0, mx, my, sw, P.mode, P.image_width, MMBA_LENS_NONE, nullptr);
    fx = r0.ex;
    fy = r0.ey;
    int l = 0;
    // the stale column (B13): re-evaluated in full below when it moves this
    // observation; the other columns need only the weighted errors
    int hit = -1;
    const bool wcol = !P.jcol_implicit;
    double jb[8] = {0., 0., 0., 0., 0., 0., r0.ex, r0.ey};
    auto emit = [&](int p, const double2 &r, double s, int tag) {
        double jx, jy;
        if (lmder) {  // s = 1/delta, multiplied (adjust_solveFunc.cpp:395-402)
            jx = (r.x - r0.ex) * s;
            jy = (r.y - r0.ey) * s;
        } else {      // s = h, divided (fdjac2)
            jx = (r.x - r0.ex) / s;
            jy = (r.y - r0.ey) / s;
        }
        // (stored non-temporal in a round-6 A/B build: C2 +1.5 %, C4 -2 % as its
        // trial pass re-reads J from L2; profiles/r6_jnt/)
        J[(size_t)(2 * l) * M + i] = jx;
        J[(size_t)(2 * l + 1) * M + i] = jy;
        if (wcol) jcol[(size_t)l * M + i] = p;
        if (p == pstale) hit = tag;
        ++l;
        return make_double2(jx, jy);
    };
#pragma unroll
    for (int v = 0; v < NCV; ++v) {
        cx[v] = 0.;
        cy[v] = 0.;
        if (v < nv) {
            const double *__restrict__ rec = C.rcf + (1 + v) * CAMREC;
            const double2 j =
                emit(C.pv[v], residual_e(rec, bp0, mx, my, sw, P.mode, P.image_width), C.st[v], v);
            cx[v] = j.x;
            cy[v] = j.y;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (a < nb) {
            const double bq[3] = {br[3 + 3 * a], br[4 + 3 * a], br[5 + 3 * a]};
            const int p = a == 0 ? p4.x : (a == 1 ? p4.y : p4.z);
            const double2 j = emit(p, residual_e(rec0, bq, mx, my, sw, P.mode, P.image_width),
                                   br[12 + a], NCV + a);
            jb[2 * a] = j.x;
            jb[2 * a + 1] = j.y;
        }
    }
    double rsx = r0.ux, rsy = r0.uy, rsd = r0.dist;  // errorList of the stale column
    if (hit >= 0) {
        const double *rec = hit < NCV ? C.rcf + (1 + hit) * CAMREC : rec0;
        double bq[3] = {bp0[0], bp0[1], bp0[2]};
        if (hit >= NCV) {
            const int a = hit - NCV;
            bq[0] = br[3 + 3 * a];
            bq[1] = br[4 + 3 * a];
            bq[2] = br[5 + 3 * a];
        }
        const Resid r = residual(rec, bq, mx, my, sw, P.mode, P.image_width, MMBA_LENS_NONE, nullptr);
        rsx = r.ux;
        rsy = r.uy;
        rsd = r.dist;
    }
    if (p4.w >= 0 && P.JB) {
        double4 *dst = reinterpret_cast<double4 *>(&P.JB[(size_t)P.obs_bpos[i] * 8]);
        dst[0] = make_double4(jb[0], jb[1], jb[2], jb[3]);
        dst[1] = make_double4(jb[4], jb[5], jb[6], jb[7]);
    }
    if (nloc) nloc[i] = l;  // constant per plan: stored by the first pass only
    // errorList / errorDistanceList as left by the last FD column: only the
    // observations that column moves change; the others keep their values at
    // x (what d_eu / d_ed already hold from the evaluation that accepted x)
    if (eu && (hit >= 0 || !P.jcol_implicit)) {
        eu[2 * i] = rsx;
        eu[2 * i + 1] = rsy;
        ed[i] = rsd;
    }
}

// Uniform fast case of k_jacobian (every camera-frame has at most NCV
// camera-side variants, no bundle-side variants, every solved bundle is a
// fast bundle, no lens): the same residuals and differences, but every
// index and record load is issued up front and the NCV + 3 perturbed
// residuals are independent straight-line code, so their fp64 latency
// chains overlap (the generic loop serialises them behind its dependent
// variant-table loads).  Emits columns in the generic kernel's order.
template <int NCV, bool GEN, bool UNI>
__global__ void __launch_bounds__(128) k_jacobian_u(
    DevProblem P, const double *__restrict__ recs, const double *__restrict__ step,
    int solver_type, double *__restrict__ J, int *__restrict__ jcol, int *__restrict__ nloc,
    const int *__restrict__ stale_param, double *__restrict__ eu, double *__restrict__ ed) {
    const int i = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // XCD-contiguous
    if (i >= P.M) return;
    double cx[NCV], cy[NCV], fx, fy;
    const int cf = P.obs_cf[i];
    const bool lmder = solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    if (UNI) {
        // every lane of the wave in one camera-frame (C2: 1,656 observations
        // per frame): the camera-frame index is wave-uniform, so its records,
        // variant parameters and steps are scalar (broadcast) loads
        const int cfu = __builtin_amdgcn_readfirstlane(cf);
        if (__all(cf == cfu)) {
            const JacCf<NCV> C = jac_cf_load<NCV>(P, cfu, recs, step, stale_param);
            jac_obs_u<NCV, GEN>(P, i, C, lmder, J, jcol, nloc, eu, ed, cx, cy, fx, fy);
            return;
        }
    }
    const JacCf<NCV> C = jac_cf_load<NCV>(P, cf, recs, step, stale_param);
    jac_obs_u<NCV, GEN>(P, i, C, lmder, J, jcol, nloc, eu, ed, cx, cy, fx, fy);
}

// -------------------------------------------------------------------------
// Normal equations.  Per camera-frame segment (contiguous observations):
// Acc (pc x pc), gC (pc), Acg (pc x nG).  One workgroup per cf; each thread
// owns output entries; J is staged through LDS in chunks of 64 observations.
// -------------------------------------------------------------------------
constexpr int NE_CHUNK = 64;

__global__ void __launch_bounds__(256) k_ne_cf(DevProblem P, const double *__restrict__ J,
                                               const int *__restrict__ jcol,
                                               const int *__restrict__ nloc,
                                               const double *__restrict__ f, double *Acc,
                                               double *Acg, double *g) {
    __shared__ double sJ[2 * LMAX][NE_CHUNK];
    __shared__ int sG[NGMAX][NE_CHUNK];  // local column of global q in observation o (-1)
    __shared__ double sF[2][NE_CHUNK];
    const int cf = blockIdx.x;
    if (!own_cf(P, cf)) return;  // another shard owns this camera-frame
    const int pc = P.cf_pc[cf];
    const int nG = P.nG;
    const int nCF = P.nR - nG;
    const int lm = P.lmax;  // widest observation: only these J rows are staged
    const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
    const int M = P.M;
    const int ncc = pc * (pc + 1) / 2;
    const int nent = ncc + pc + pc * nG;
    const int e = threadIdx.x;
    int ea = 0, eb = 0, kind = -1;
    if (e < ncc) {
        // decode upper-triangular index
        int rem = e, r = 0;
        while (rem >= pc - r) {
            rem -= pc - r;
            ++r;
        }
        ea = r;
        eb = r + rem;
        kind = 0;
    } else if (e < ncc + pc) {
        ea = e - ncc;
        kind = 1;
    } else if (e < nent) {
        ea = (e - ncc - pc) / nG;
        eb = (e - ncc - pc) % nG;
        kind = 2;
    }
    double acc = 0.;
    for (int c0 = o0; c0 < o1; c0 += NE_CHUNK) {
        const int cnt = min(NE_CHUNK, o1 - c0);
        __syncthreads();
        for (int t = threadIdx.x; t < 2 * lm * NE_CHUNK; t += blockDim.x) {
            const int row = t / NE_CHUNK, o = t % NE_CHUNK;
            sJ[row][o] = (o < cnt) ? J[(size_t)row * M + c0 + o] : 0.;
        }
        if (nG > 0) {
            for (int t = threadIdx.x; t < NGMAX * NE_CHUNK; t += blockDim.x)
                sG[t / NE_CHUNK][t % NE_CHUNK] = -1;
            __syncthreads();
            // columns l >= pc of every observation: which global parameter
            // (the camera block's own columns come first, l < pc)
            for (int t = threadIdx.x; t < lm * NE_CHUNK; t += blockDim.x) {
                const int l = t / NE_CHUNK, o = t % NE_CHUNK;
                if (o >= cnt || l < pc || l >= nloc[c0 + o]) continue;
                const int p = jcol[(size_t)l * M + c0 + o];
                if (P.p_class[p] == PC_G) sG[P.p_pos[p] - nCF][o] = l;
            }
        }
        for (int t = threadIdx.x; t < NE_CHUNK; t += blockDim.x) {
            sF[0][t] = (t < cnt) ? f[2 * (c0 + t)] : 0.;
            sF[1][t] = (t < cnt) ? f[2 * (c0 + t) + 1] : 0.;
        }
        __syncthreads();
        if (kind == 0) {
            for (int o = 0; o < cnt; ++o)
                acc += sJ[2 * ea][o] * sJ[2 * eb][o] + sJ[2 * ea + 1][o] * sJ[2 * eb + 1][o];
        } else if (kind == 1) {
            for (int o = 0; o < cnt; ++o)
                acc += sJ[2 * ea][o] * sF[0][o] + sJ[2 * ea + 1][o] * sF[1][o];
        } else if (kind == 2) {
            for (int o = 0; o < cnt; ++o) {
                const int l = sG[eb][o];
                if (l >= 0)
                    acc += sJ[2 * ea][o] * sJ[2 * l][o] + sJ[2 * ea + 1][o] * sJ[2 * l + 1][o];
            }
        }
    }
    double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
    if (kind == 0) {
        A[ea * PCMAX + eb] = acc;
        A[eb * PCMAX + ea] = acc;
    } else if (kind == 1) {
        g[P.cf_var_param[P.cf_var_off[cf] + 1 + ea]] = acc;
    } else if (kind == 2) {
        Acg[((size_t)cf * PCMAX + ea) * NGMAX + eb] = acc;
    }
}

// Uniform block size PC and no global parameters: one wave per camera-frame,
// lane o accumulates the upper triangle of Acc and gC over the observations
// o, o + 64, ... of the (contiguous) segment in registers; the 64 partial
// sums are added through LDS in a fixed order.
// One parameter's share of the lmder bookkeeping (k_jac_epilogue, same
// operations): acnorm, diag update, and its contributions to the rank flag,
// ||D x||^2 and gnorm.
__device__ __forceinline__ double epi_param(const NeEpi &E, int p, double d, double gp, double &zf,
                                          double &xn, double &gm) {
    const double an = sqrt(d);
    E.acnorm[p] = an;
    double dg = E.diag[p];
    if (E.mode != 2) {
        if (E.first) dg = an == 0. ? 1. : an;
        dg = fmax(dg, an);
        E.diag[p] = dg;
    }
    if (an == 0.) zf = 1.;
    if (E.do_xn) {
        const double v = dg * E.x[p];
        xn += v * v;
    }
    if (E.do_gn && an != 0.) {
        // a device-side ||f||^2 (first Jacobian): gnorm only when ||f|| != 0,
        // as lmder decides on the host otherwise
        const double fn = E.fnorm_sq ? sqrt(*E.fnorm_sq) : E.fnorm;
        if (fn != 0.) gm = fmax(gm, fabs((gp / fn) / an));
    }
    return dg;  // diag[p] as stored (what k_bundle_factor reads next)
}

__device__ __forceinline__ void epi_store(const NeEpi &E, int col, double zf, double xn,
                                          double gm) {
    E.partial[col] = zf;
    E.partial[E.rstride + col] = xn;
    E.partial[2 * E.rstride + col] = gm;
}

// A camera-frame's PC parameters' bookkeeping with one wave: lane a < PC
// takes parameter a (epi_param; d / gp its diagonal and gradient sums), then
// every lane folds the PC contributions in parameter order and lane 0 stores
// them -- the serial loop's sums (xn: ((0 + t_0) + t_1) + ...; zf / gm are
// order-free), without its chain of PC dependent index / diag loads (the
// last step of k_ne_cf_u / k_ne_cf_split / k_jac_ne_u: ~10 us on C2 as one
// thread).  Called by all 64 lanes of one wave.
// The operands epi_param reads from memory, loaded by epi_preload before the
// observation loop, so the epilogue after it issues no dependent loads.
struct EpiPre {
    int p;      // the parameter of lane a (camera-frame variant a)
    double dg;  // diag[p] before this Jacobian
    double xv;  // x[p] (do_xn)
    double fn;  // ||f|| (do_gn)
};
template <int PC>
__device__ __forceinline__ EpiPre epi_preload(const DevProblem &P, const NeEpi &E, int cf,
                                              int lane) {
    EpiPre q{-1, 0., 0., 0.};
    if (!E.on || lane >= PC) return q;
    q.p = P.cf_var_param[P.cf_var_off[cf] + 1 + lane];
    q.dg = E.diag[q.p];
    if (E.do_xn) q.xv = E.x[q.p];
    if (E.do_gn) q.fn = E.fnorm_sq ? sqrt(*E.fnorm_sq) : E.fnorm;
    return q;
}
// epi_param with its loads done (same operations, same bits)
__device__ __forceinline__ void epi_param_pre(const NeEpi &E, const EpiPre &q, double d, double gp,
                                              double &zf, double &xn, double &gm) {
    const double an = sqrt(d);
    E.acnorm[q.p] = an;
    double dg = q.dg;
    if (E.mode != 2) {
        if (E.first) dg = an == 0. ? 1. : an;
        dg = fmax(dg, an);
        E.diag[q.p] = dg;
    }
    if (an == 0.) zf = 1.;
    if (E.do_xn) {
        const double v = dg * q.xv;
        xn += v * v;
    }
    if (E.do_gn && an != 0.) {
        if (q.fn != 0.) gm = fmax(gm, fabs((gp / q.fn) / an));
    }
}
template <int PC>
__device__ __forceinline__ void epi_params_wave(const DevProblem &P, const NeEpi &E, int cf,
                                                int lane, double d, double gp, const EpiPre &q) {
    double zf = 0., xn = 0., gm = 0.;
    if (lane < PC) epi_param_pre(E, q, d, gp, zf, xn, gm);
    double Z = 0., X = 0., G = 0.;
#pragma unroll
    for (int a = 0; a < PC; ++a) {
        const double za = __shfl(zf, a), xa = __shfl(xn, a), ga = __shfl(gm, a);
        if (za != 0.) Z = 1.;
        X += xa;
        G = fmax(G, ga);
    }
    if (lane == 0) epi_store(E, E.cf_base + cf, Z, X, G);
}


template <int PC, int NW, int NG>
__device__ __forceinline__ void ne_cf_u_body(const DevProblem &P, const double *__restrict__ J,
                                             const int *__restrict__ jcol,
                                             const int *__restrict__ nloc,
                                             const double *__restrict__ f, double *Acc,
                                             double *Acg, double *g, const NeEpi &E, int blk,
                                             int nblk_cf) {
    // NW waves per camera-frame (long segments: C2 has ~1,700 observations
    // per camera-frame): thread t takes observations t, t + 64 NW, ...;
    // each wave folds its partial sums with a fixed xor-shuffle tree, the NW
    // wave sums are added in wave order (deterministic).  NG > 0: the
    // couplings Acg with up to NG global parameters (lens), whose columns
    // follow the camera block in each observation (found through jcol).
    constexpr int NCC = PC * (PC + 1) / 2, NE = NCC + PC, NT = NE + PC * NG;
    __shared__ double wsum[NW][NT];
    const int cf = xcd_remap(blk, nblk_cf);  // the XCD that wrote its J rows
    if (!own_cf(P, cf) || P.cf_pc[cf] != PC) {
        if (E.on && threadIdx.x == 0) epi_store(E, E.cf_base + cf, 0., 0., 0.);
        return;
    }
    const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
    const size_t M = P.M;
    const int nCF = P.nR - P.nG;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const EpiPre epq = epi_preload<PC>(P, E, cf, lane);
    double acc[NT];
#pragma unroll
    for (int e = 0; e < NT; ++e) acc[e] = 0.;
    for (int i = o0 + tid; i < o1; i += 64 * NW) {
        double jx[PC], jy[PC];
#pragma unroll
        for (int a = 0; a < PC; ++a) {
            jx[a] = J[(2 * a) * M + i];
            jy[a] = J[(2 * a + 1) * M + i];
        }
        const double fx = f[2 * i], fy = f[2 * i + 1];
        int e = 0;
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = a; c < PC; ++c) acc[e++] += jx[a] * jx[c] + jy[a] * jy[c];
#pragma unroll
        for (int a = 0; a < PC; ++a) acc[NCC + a] += jx[a] * fx + jy[a] * fy;
        if constexpr (NG > 0) {
            double gx[NG], gy[NG];
#pragma unroll
            for (int q = 0; q < NG; ++q) gx[q] = gy[q] = 0.;
            const int nl = nloc[i];
            for (int l = PC; l < nl; ++l) {
                const int p = jcol[(size_t)l * M + i];
                if (P.p_class[p] != PC_G) continue;
                const int gi = P.p_pos[p] - nCF;
                const double ux = J[(size_t)(2 * l) * M + i], uy = J[(size_t)(2 * l + 1) * M + i];
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    gx[q] = (gi == q) ? ux : gx[q];
                    gy[q] = (gi == q) ? uy : gy[q];
                }
            }
#pragma unroll
            for (int a = 0; a < PC; ++a)
#pragma unroll
                for (int q = 0; q < NG; ++q)
                    acc[NE + a * NG + q] += jx[a] * gx[q] + jy[a] * gy[q];
        }
    }
#pragma unroll
    for (int e = 0; e < NT; ++e) {
        double v = acc[e];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wv][e] = v;
    }
    __syncthreads();
    double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
    for (int e = tid; e < NT; e += 64 * NW) {
        double v = wsum[0][e];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += wsum[w][e];
        if (e < NCC) {
            int a = 0, rem = e;
            while (rem >= PC - a) {
                rem -= PC - a;
                ++a;
            }
            const int c = a + rem;
            A[a * PCMAX + c] = v;
            A[c * PCMAX + a] = v;
        } else if (e < NE) {
            g[P.cf_var_param[P.cf_var_off[cf] + 1 + (e - NCC)]] = v;
        } else {
            constexpr int NGd = NG > 0 ? NG : 1;  // e < NE always when NG == 0
            const int a = (e - NE) / NGd, q = (e - NE) % NGd;
            if (q < P.nG) Acg[((size_t)cf * PCMAX + a) * NGMAX + q] = v;
        }
    }
    if (E.on && wv == 0) {
        // the block's parameters (sums re-formed in the same order as above)
        double d = 0., gp = 0.;
        if (lane < PC) {
            const int ed = lane * PC - lane * (lane - 1) / 2;  // upper-triangle index of (a, a)
            d = wsum[0][ed];
            gp = wsum[0][NCC + lane];
#pragma unroll
            for (int w = 1; w < NW; ++w) {
                d += wsum[w][ed];
                gp += wsum[w][NCC + lane];
            }
        }
        epi_params_wave<PC>(P, E, cf, lane, d, gp, epq);
    }
}
// k_ne_cf_u for long camera-frame segments without global parameters (C2:
// ~1,650 observations per camera-frame, 120 camera-frames -- 120 workgroups
// left half the SIMDs idle and read J at ~1 TB/s): NS workgroups per
// camera-frame (logical blocks cf * NS + part, consecutive on one XCD), part
// p takes observations o0 + 64 NW p + t, o0 + 64 NW (NS + p) + t, ...; each
// workgroup stores its NT partial sums write-through, the last to arrive
// (per camera-frame ticket: monotonic, last when old % NS == NS - 1) loads
// them sc1 and adds them in part order -- deterministic whichever arrives
// last -- then writes Acc / g and the lmder epilogue as k_ne_cf_u does.
template <int PC, int NW, int NS>
__global__ void __launch_bounds__(64 * NW) k_ne_cf_split(DevProblem P, const double *__restrict__ J,
                                                         const double *__restrict__ f, double *Acc,
                                                         double *g, NeEpi E) {
    constexpr int NCC = PC * (PC + 1) / 2, NT = NCC + PC;
    static_assert(NT <= NE_CF_NT, "partial sums per workgroup");
    __shared__ double wsum[NW][NT];
    __shared__ double fin[NT];
    __shared__ unsigned last_s;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int cf = L / NS, part = L % NS;
    if (cf >= P.ncf) return;
    if (!own_cf(P, cf) || P.cf_pc[cf] != PC) {
        if (E.on && part == 0 && threadIdx.x == 0) epi_store(E, E.cf_base + cf, 0., 0., 0.);
        return;
    }
    const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
    const size_t M = P.M;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const EpiPre epq = epi_preload<PC>(P, E, cf, lane);
    double acc[NT];
#pragma unroll
    for (int e = 0; e < NT; ++e) acc[e] = 0.;
    for (int i = o0 + 64 * NW * part + tid; i < o1; i += 64 * NW * NS) {
        double jx[PC], jy[PC];
#pragma unroll
        for (int a = 0; a < PC; ++a) {
            jx[a] = J[(2 * a) * M + i];
            jy[a] = J[(2 * a + 1) * M + i];
        }
        const double fx = f[2 * i], fy = f[2 * i + 1];
        int e = 0;
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = a; c < PC; ++c) acc[e++] += jx[a] * jx[c] + jy[a] * jy[c];
#pragma unroll
        for (int a = 0; a < PC; ++a) acc[NCC + a] += jx[a] * fx + jy[a] * fy;
    }
#pragma unroll
    for (int e = 0; e < NT; ++e) {
        double v = acc[e];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wv][e] = v;
    }
    __syncthreads();
    double *mine = E.cf_part + ((size_t)cf * NS + part) * NE_CF_NT;
    for (int e = tid; e < NT; e += 64 * NW) {
        double v = wsum[0][e];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += wsum[w][e];
        st_sc1(&mine[e], v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        last_s = (__hip_atomic_fetch_add(&E.cf_ticket[cf], 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) %
                  NS) == NS - 1;
    __syncthreads();
    if (!last_s) return;
    const double *all = E.cf_part + (size_t)cf * NS * NE_CF_NT;
    for (int e = tid; e < NT; e += 64 * NW) {
        double t[NS];  // every part's load issued before the sum
#pragma unroll
        for (int q = 0; q < NS; ++q) t[q] = ld_sc1(&all[(size_t)q * NE_CF_NT + e]);
        double v = t[0];
#pragma unroll
        for (int q = 1; q < NS; ++q) v += t[q];
        fin[e] = v;
    }
    __syncthreads();
    double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
    for (int e = tid; e < NT; e += 64 * NW) {
        const double v = fin[e];
        if (e < NCC) {
            int a = 0, rem = e;
            while (rem >= PC - a) {
                rem -= PC - a;
                ++a;
            }
            const int c = a + rem;
            A[a * PCMAX + c] = v;
            A[c * PCMAX + a] = v;
        } else {
            g[P.cf_var_param[P.cf_var_off[cf] + 1 + (e - NCC)]] = v;
        }
    }
    if (E.on && wv == 0) {
        const int ed = lane * PC - lane * (lane - 1) / 2;  // upper-triangle index of (a, a)
        epi_params_wave<PC>(P, E, cf, lane, lane < PC ? fin[ed] : 0., lane < PC ? fin[NCC + lane] : 0.,
                            epq);
    }
}

template <int PC, int NW, int NG>
__global__ void __launch_bounds__(64 * NW) k_ne_cf_u(DevProblem P, const double *__restrict__ J,
                                                     const int *__restrict__ jcol,
                                                     const int *__restrict__ nloc,
                                                     const double *__restrict__ f, double *Acc,
                                                     double *Acg, double *g, NeEpi E) {
    ne_cf_u_body<PC, NW, NG>(P, J, jcol, nloc, f, Acc, Acg, g, E, blockIdx.x, gridDim.x);
}

// Camera-frame -> XCD-contiguous order: workgroups are dispatched to the 8
// XCDs round-robin, so workgroup b runs on XCD b % 8; giving each XCD a
// contiguous range of camera-frames keeps consecutive frames (which share
// bundles) on one L2 and the bundle records they gather are fetched once.

// Fused K2 for uniform fast plans without global parameters: one workgroup
// per camera-frame segment computes the FD Jacobian of its observations
// (jac_obs_u, the k_jacobian_u arithmetic), keeps the camera columns in
// registers and reduces Acc / gC (+ the lmder epilogue of the block's
// parameters) in the same pass -- the J blocks are written once for the
// Schur / ||J p|| passes and never re-read here (k_ne_cf_u's 19 MB on C4).
// Same per-lane summation order as k_ne_cf_u with its NW.
template <int PC, int NW, bool GEN>
__global__ void __launch_bounds__(64 * NW) k_jac_ne_u(
    DevProblem P, const double *__restrict__ recs, const double *__restrict__ step,
    int solver_type, double *__restrict__ J, int *__restrict__ jcol, int *__restrict__ nloc,
    const int *__restrict__ stale_param, double *__restrict__ eu, double *__restrict__ ed,
    double *Acc, double *g, NeEpi E) {
    constexpr int NCC = PC * (PC + 1) / 2, NE = NCC + PC;
    __shared__ double wsum[NW][NE];
    // the camera-frame's records, variant parameters and steps: staged once
    // (every observation of the segment reads the same ones)
    __shared__ double sRec[(PC + 1) * CAMREC];
    __shared__ int sPv[PC];
    __shared__ double sSt[PC];
    __shared__ int sHdr[3];  // nv, frame, stale column
    // a Jacobian enqueued ahead of the host's decision runs only when the
    // device's restatement of that decision (lm_decide) let it
    if (E.gate && __hip_atomic_load(E.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        return;
    const int cf = xcd_remap(blockIdx.x, gridDim.x);
    long long *pr = (E.probe && threadIdx.x == 0) ? E.probe + 5 * (size_t)cf : nullptr;
    if (pr) pr[0] = (long long)wall_clock64();
    const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool lmder = solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const bool solved = P.cf_pc[cf] == PC && own_cf(P, cf);  // sharded: owner's blocks only
    {
        const int voff = P.cf_var_off[cf];
        const int nv = min(P.cf_var_off[cf + 1] - voff - 1, PC);
        for (int t = tid; t < (nv + 1) * CAMREC; t += 64 * NW)
            sRec[t] = recs[(size_t)voff * CAMREC + t];
        if (tid < PC) {
            const int p = tid < nv ? P.cf_var_param[voff + 1 + tid] : -1;
            sPv[tid] = p;
            sSt[tid] = tid < nv ? step[p] : 1.;
        }
        if (tid == 0) {
            const int fr = P.cf_frame[cf];
            sHdr[0] = nv;
            sHdr[1] = fr;
            sHdr[2] = stale_param[fr];
        }
    }
    __syncthreads();
    if (pr) pr[1] = (long long)wall_clock64();
    JacCf<PC> C;
    C.rcf = sRec;
#pragma unroll
    for (int v = 0; v < PC; ++v) {
        C.pv[v] = sPv[v];
        C.st[v] = sSt[v];
    }
    C.nv = sHdr[0];
    C.fr = sHdr[1];
    C.pstale = sHdr[2];
    double acc[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.;
    for (int i = o0 + tid; i < o1; i += 64 * NW) {
        double jx[PC], jy[PC], fx, fy;
        // the record reads stay inside the loop (LDS broadcasts): an opaque
        // zero offset keeps the compiler from hoisting 140 loop-invariant
        // doubles into registers
        int z = 0;
        asm volatile("" : "+s"(z));
        C.rcf = sRec + z;
        jac_obs_u<PC, GEN>(P, i, C, lmder, J, jcol, nloc, eu, ed, jx, jy, fx, fy);
        int e = 0;
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = a; c < PC; ++c) acc[e++] += jx[a] * jx[c] + jy[a] * jy[c];
#pragma unroll
        for (int a = 0; a < PC; ++a) acc[NCC + a] += jx[a] * fx + jy[a] * fy;
    }
    if (pr) pr[2] = (long long)wall_clock64();
    if (!solved) {  // no camera parameter on this camera-frame: J only
        if (E.on && tid == 0) epi_store(E, E.cf_base + cf, 0., 0., 0.);
        if (pr) pr[3] = pr[2];
        return;
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        double v = acc[e];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wv][e] = v;
    }
    __syncthreads();
    double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
    for (int e = tid; e < NE; e += 64 * NW) {
        double v = wsum[0][e];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += wsum[w][e];
        if (e < NCC) {
            int a = 0, rem = e;
            while (rem >= PC - a) {
                rem -= PC - a;
                ++a;
            }
            const int c = a + rem;
            A[a * PCMAX + c] = v;
            A[c * PCMAX + a] = v;
        } else {
            g[P.cf_var_param[P.cf_var_off[cf] + 1 + (e - NCC)]] = v;
        }
    }
    if (E.on && (tid >> 6) == 0) {
        const int ln = tid & 63;
        double d = 0., gp = 0.;
        if (ln < PC) {
            const int ed2 = ln * PC - ln * (ln - 1) / 2;
            d = wsum[0][ed2];
            gp = wsum[0][NCC + ln];
#pragma unroll
            for (int w = 1; w < NW; ++w) {
                d += wsum[w][ed2];
                gp += wsum[w][NCC + ln];
            }
        }
        // (loaded here: preloaded before the loop they cost this 232-VGPR
        // kernel its second wave per SIMD)
        epi_params_wave<PC>(P, E, cf, ln, d, gp, epi_preload<PC>(P, E, cf, ln));
    }
    if (pr) {
        pr[3] = (long long)wall_clock64();
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        pr[4] = (long long)(xcc & 0xf);
    }
}

// Fast bundles, no global parameters: Abb and gB from the per-observation
// block records, same summation order as k_ne_bnd.  One thread per bundle,
// NE_BND_TPB threads per workgroup (C4: 782 workgroups over 256 CUs, so
// several waves per CU hide the record loads); a bundle's records are loaded
// four at a time before they are accumulated (C4's bundles have four).
__global__ void __launch_bounds__(NE_BND_TPB) k_ne_bnd_jb(DevProblem P, double *Abb, double *g,
                                                          NeEpi E) {
    __shared__ double red[3][NE_BND_TPB];
    // enqueued ahead of the host's decision with its Jacobian pass (round 6):
    // runs only when the device's restatement of that decision let it
    if (E.gate && __hip_atomic_load(E.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        return;
    const int b = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // XCD-contiguous
    const int4 p4 = b < P.nB ? P.bnd_p4[b] : make_int4(-1, -1, -1, 0);
    const int pb = p4.w;
    double zf = 0., xn = 0., gm = 0.;
    if (pb > 0) {
        double A[PBMAX][PBMAX] = {};
        double gb[PBMAX] = {};
        const int q0 = P.bobs_off[b], q1 = P.bobs_off[b + 1];
        const double *__restrict__ br = &P.brec[(size_t)b * BREC];
        for (int qb = q0; qb < q1; qb += 4) {
            double4 u[4], v[4];
            if (E.jb_recs) {
                // the records' values re-evaluated: jac_obs_u's base residual
                // and bundle columns (residual_e is residual's ex / ey)
                const double bp0[3] = {br[0], br[1], br[2]};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (qb + r >= q1) break;
                    const int i = P.bobs[qb + r];
                    const double *__restrict__ rec0 = &E.jb_recs[(size_t)P.cf_var_off[P.obs_cf[i]] * CAMREC];
                    const double mx = P.obs_xy[2 * i], my = P.obs_xy[2 * i + 1], sw = P.obs_sqrtw[i];
                    const double2 f0 = residual_e(rec0, bp0, mx, my, sw, P.mode, P.image_width);
                    double jb[6] = {0., 0., 0., 0., 0., 0.};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        if (a < pb) {
                            const double bq[3] = {br[3 + 3 * a], br[4 + 3 * a], br[5 + 3 * a]};
                            const double2 rr = residual_e(rec0, bq, mx, my, sw, P.mode, P.image_width);
                            const double st = br[12 + a];
                            jb[2 * a] = E.jb_lmder ? (rr.x - f0.x) * st : (rr.x - f0.x) / st;
                            jb[2 * a + 1] = E.jb_lmder ? (rr.y - f0.y) * st : (rr.y - f0.y) / st;
                        }
                    }
                    u[r] = make_double4(jb[0], jb[1], jb[2], jb[3]);
                    v[r] = make_double4(jb[4], jb[5], f0.x, f0.y);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (qb + r < q1) {
                        const double4 *src = reinterpret_cast<const double4 *>(&P.JB[(size_t)(qb + r) * 8]);
                        u[r] = src[0];
                        v[r] = src[1];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (qb + r >= q1) break;
                const double jx[3] = {u[r].x, u[r].z, v[r].x}, jy[3] = {u[r].y, u[r].w, v[r].y};
                const double fx = v[r].z, fy = v[r].w;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) A[a][c] += jx[a] * jx[c] + jy[a] * jy[c];
                    gb[a] += jx[a] * fx + jy[a] * fy;
                }
            }
        }
        double *Ab = &Abb[(size_t)b * 9];
#pragma unroll
        for (int a = 0; a < PBMAX; ++a)
#pragma unroll
            for (int c = 0; c < PBMAX; ++c) Ab[a * 3 + c] = (a < pb && c < pb) ? A[a][c] : 0.;
        g[p4.x] = gb[0];
        if (pb > 1) g[p4.y] = gb[1];
        if (pb > 2) g[p4.z] = gb[2];
        double dd[3] = {0., 0., 0.};  // diag after the epilogue (read by the factor)
        if (E.on) {
            // sharded: every bundle of the shard gets acnorm / diag, only the
            // owned ones enter the rank-summed scalars
            double zo = 0., xo = 0., go = 0.;
            dd[0] = epi_param(E, p4.x, A[0][0], gb[0], zo, xo, go);
            if (pb > 1) dd[1] = epi_param(E, p4.y, A[1][1], gb[1], zo, xo, go);
            if (pb > 2) dd[2] = epi_param(E, p4.z, A[2][2], gb[2], zo, xo, go);
            if (own_bnd(P, b)) {
                zf = zo;
                xn = xo;
                gm = go;
            }
        }
        if (E.Lb) {
            // the undamped solve's bundle factor (k_bundle_factor at lam = 0,
            // same operands and operations: Abb and gB as stored above)
            double Af[3][3], rhs[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    Af[a][c] = (a < pb && c < pb) ? A[a][c] : (a == c ? 1. : 0.);
                rhs[a] = a < pb ? gb[a] : 0.;
            }
            bundle_chol3(Af, rhs, dd, pb, 0.0, b, E.Lb, E.tb, E.fail);
        }
    }
    if (!E.on) return;
    red[0][threadIdx.x] = zf;
    red[1][threadIdx.x] = xn;
    red[2][threadIdx.x] = gm;
    __syncthreads();
    for (int w = NE_BND_TPB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            red[0][threadIdx.x] = fmax(red[0][threadIdx.x], red[0][threadIdx.x + w]);
            red[1][threadIdx.x] += red[1][threadIdx.x + w];
            red[2][threadIdx.x] = fmax(red[2][threadIdx.x], red[2][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int col = E.bnd_base + xcd_remap(blockIdx.x, gridDim.x);
        if (E.fold) {  // read by this launch's last workgroup: write-through
            st_sc1(&E.partial[col], red[0][0]);
            st_sc1(&E.partial[E.rstride + col], red[1][0]);
            st_sc1(&E.partial[2 * E.rstride + col], red[2][0]);
        } else {
            epi_store(E, col, red[0][0], red[1][0], red[2][0]);
        }
    }
    if (E.fold) tail_reduce(E.spec, E.partial, E.scalar, E.ticket);
}

// Per bundle: Abb (pb x pb), gB, Abg (pb x nG).  One thread per bundle.
__global__ void k_ne_bnd(DevProblem P, const double *__restrict__ J,
                         const int *__restrict__ jcol, const int *__restrict__ nloc,
                         const double *__restrict__ f, double *Abb, double *Abg, double *g) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    if (pb == 0) return;
    const int M = P.M, nG = P.nG;
    double A[PBMAX][PBMAX] = {};
    double gb[PBMAX] = {};
    double G[PBMAX][NGMAX];
    for (int a = 0; a < PBMAX; ++a)
        for (int q = 0; q < NGMAX; ++q) G[a][q] = 0.;
    for (int q = P.bobs_off[b]; q < P.bobs_off[b + 1]; ++q) {
        const int i = P.bobs[q];
        const int cf = P.obs_cf[i];
        // the bundle's columns follow the camera-frame's variants, or come
        // last in a rolling-shutter row (k_jacobian_rs)
        const int s = P.rs ? nloc[i] - pb : P.cf_var_off[cf + 1] - P.cf_var_off[cf] - 1;
        double jx[PBMAX], jy[PBMAX];
        for (int a = 0; a < pb; ++a) {
            jx[a] = J[(size_t)(2 * (s + a)) * M + i];
            jy[a] = J[(size_t)(2 * (s + a) + 1) * M + i];
        }
        const double fx = f[2 * i], fy = f[2 * i + 1];
        for (int a = 0; a < pb; ++a) {
            for (int c = 0; c < pb; ++c) A[a][c] += jx[a] * jx[c] + jy[a] * jy[c];
            gb[a] += jx[a] * fx + jy[a] * fy;
        }
        if (nG > 0) {
            const int nl = nloc[i];
            for (int l = 0; l < nl; ++l) {
                const int p = jcol[(size_t)l * M + i];
                if (P.p_class[p] != PC_G) continue;
                const int gi = P.p_pos[p] - (P.nR - nG);
                const double gx = J[(size_t)(2 * l) * M + i], gy = J[(size_t)(2 * l + 1) * M + i];
                for (int a = 0; a < pb; ++a) G[a][gi] += jx[a] * gx + jy[a] * gy;
            }
        }
    }
    double *Ab = &Abb[(size_t)b * 9];
    for (int a = 0; a < PBMAX; ++a)
        for (int c = 0; c < PBMAX; ++c) Ab[a * 3 + c] = (a < pb && c < pb) ? A[a][c] : 0.;
    const int po = P.bnd_par_off[b];
    for (int a = 0; a < pb; ++a) g[P.bnd_par[po + a]] = gb[a];
    for (int a = 0; a < PBMAX; ++a)
        for (int q = 0; q < nG; ++q) Abg[((size_t)b * PBMAX + a) * NGMAX + q] = G[a][q];
}

// Globals: partial sums of Agg (nG x nG) and gG per block of observations.
// NG: compile-time bound on the number of global parameters (2, 4, 8 or
// 16): the per-thread accumulators are NG^2 + NG registers (the 272-double
// array of NG = 16 spills 2 KB per lane to scratch; wider arrows take
// k_ne_glob_wide).  Partial rows keep the
// NGMAX layout.
constexpr int NE_GLOB_L = 12;  // observations with at most this many columns: batched loads
template <int NG>
__device__ __forceinline__ void ne_glob_body(const DevProblem &P, const double *__restrict__ J,
                                             const int *__restrict__ jcol,
                                             const int *__restrict__ nloc,
                                             const double *__restrict__ f, double *partial,
                                             int chunk, int blk) {
    // One observation per thread (grid-stride over the block's chunk); each
    // thread scatters its global-parameter Jacobian entries into a dense
    // register vector, products are reduced wave -> block in a fixed order
    // (deterministic, no atomics).
    constexpr int NA = NG * NG + NG;
    __shared__ double wsum[4][NA];
    const int nG = P.nG;
    const int nCF = P.nR - nG;
    const int M = P.M;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double accv[NA];
#pragma unroll
    for (int e = 0; e < NA; ++e) accv[e] = 0.;
    const int i0 = blk * chunk;
    const int i1 = min(M, i0 + chunk);
    for (int i = i0 + (int)threadIdx.x; i < i1; i += blockDim.x) {
        if (!own_obs(P, i)) continue;
        double gx[NG], gy[NG];
#pragma unroll
        for (int q = 0; q < NG; ++q) gx[q] = gy[q] = 0.;
        const int nl = nloc[i];
        if (nl <= NE_GLOB_L) {
            // the same assignments, with every column's loads issued level by
            // level (parameter ids, then class and position, then the J
            // entries): three memory round trips instead of three per column
            int pl[NE_GLOB_L], gq[NE_GLOB_L];
#pragma unroll
            for (int l = 0; l < NE_GLOB_L; ++l) pl[l] = l < nl ? jcol[(size_t)l * M + i] : -1;
#pragma unroll
            for (int l = 0; l < NE_GLOB_L; ++l) {
                const int p = pl[l];
                gq[l] = (p >= 0 && P.p_class[p] == PC_G) ? P.p_pos[p] - nCF : -1;
            }
#pragma unroll
            for (int l = 0; l < NE_GLOB_L; ++l) {
                if (gq[l] < 0) continue;
                const double jx = J[(size_t)(2 * l) * M + i], jy = J[(size_t)(2 * l + 1) * M + i];
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    gx[q] = (gq[l] == q) ? jx : gx[q];
                    gy[q] = (gq[l] == q) ? jy : gy[q];
                }
            }
        } else {
            for (int l = 0; l < nl; ++l) {
                const int p = jcol[(size_t)l * M + i];
                if (P.p_class[p] != PC_G) continue;
                const int gi = P.p_pos[p] - nCF;
                const double jx = J[(size_t)(2 * l) * M + i], jy = J[(size_t)(2 * l + 1) * M + i];
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    gx[q] = (gi == q) ? jx : gx[q];
                    gy[q] = (gi == q) ? jy : gy[q];
                }
            }
        }
        const double fx = f[2 * i], fy = f[2 * i + 1];
#pragma unroll
        for (int a = 0; a < NG; ++a) {
#pragma unroll
            for (int b = 0; b < NG; ++b) accv[a * NG + b] += gx[a] * gx[b] + gy[a] * gy[b];
            accv[NG * NG + a] += gx[a] * fx + gy[a] * fy;
        }
    }
#pragma unroll
    for (int e = 0; e < NA; ++e) {
        double v = accv[e];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wave][e] = v;
    }
    __syncthreads();
    // the block's row of [Agg | gG] in the compact layout of the plan's nG
    // (nG^2 + nG entries, k_ne_glob_reduce)
    const int NA_ = nG * nG + nG;
    for (int t = threadIdx.x; t < NA_; t += blockDim.x) {
        const bool mat = t < nG * nG;
        const int a = mat ? t / nG : t - nG * nG, b = mat ? t % nG : 0;
        const int e = mat ? a * NG + b : NG * NG + a;
        partial[(size_t)blk * NA_ + t] = (wsum[0][e] + wsum[1][e]) + (wsum[2][e] + wsum[3][e]);
    }
}
template <int NG>
__global__ void __launch_bounds__(256) k_ne_glob(DevProblem P, const double *__restrict__ J,
                                                 const int *__restrict__ jcol,
                                                 const int *__restrict__ nloc,
                                                 const double *__restrict__ f,
                                                 double *partial, int chunk) {
    ne_glob_body<NG>(P, J, jcol, nloc, f, partial, chunk, blockIdx.x);
}

// Both in one launch (C5: camera-frame blocks of four waves and at most two
// global parameters): workgroups [0, ncf) are k_ne_cf_u<PC, 4, 2>'s, the rest
// k_ne_glob<2>'s -- the same code on the same data, so the same sums, with
// the global chunks running beside the camera-frame blocks instead of after
// them (C5: 10.9 us of k_ne_glob per Jacobian).
template <int PC>
__global__ void __launch_bounds__(256) k_ne_cf_glob(DevProblem P, const double *__restrict__ J,
                                                    const int *__restrict__ jcol,
                                                    const int *__restrict__ nloc,
                                                    const double *__restrict__ f, double *Acc,
                                                    double *Acg, double *g, NeEpi E,
                                                    double *partial, int chunk) {
    if ((int)blockIdx.x < P.ncf)
        ne_cf_u_body<PC, 4, 2>(P, J, jcol, nloc, f, Acc, Acg, g, E, blockIdx.x, P.ncf);
    else
        ne_glob_body<2>(P, J, jcol, nloc, f, partial, chunk, (int)blockIdx.x - P.ncf);
}

// Globals wider than 16 (NG^2 + NG accumulators no longer fit a thread's
// registers): the block stages the dense global Jacobian rows and residuals
// of 64 observations at a time in LDS, and thread t owns entries t, t + 256,
// ... of [Agg | gG], summed over the observations in order (deterministic,
// no atomics).  Same partial-row layout as k_ne_glob.
__global__ void __launch_bounds__(256) k_ne_glob_wide(DevProblem P, const double *__restrict__ J,
                                                      const int *__restrict__ jcol,
                                                      const int *__restrict__ nloc,
                                                      const double *__restrict__ f,
                                                      double *partial, int chunk) {
    constexpr int OB = 64;  // observations per LDS round
    constexpr int EPT = (NGMAX * NGMAX + NGMAX + 255) / 256;
    __shared__ double sg[OB][2 * NGMAX + 2];  // gx[NGMAX] | gy[NGMAX] | fx, fy
    const int nG = P.nG, nCF = P.nR - nG, M = P.M;
    const int NA = nG * nG + nG;
    const int i0 = blockIdx.x * chunk, i1 = min(M, i0 + chunk);
    double acc[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) acc[k] = 0.;
    for (int b0 = i0; b0 < i1; b0 += OB) {
        __syncthreads();  // the previous round's reads are done
        for (int t = threadIdx.x; t < OB * (2 * NGMAX + 2); t += blockDim.x) (&sg[0][0])[t] = 0.;
        __syncthreads();
        if (threadIdx.x < OB) {
            const int o = threadIdx.x, i = b0 + o;
            if (i < i1 && own_obs(P, i)) {
                const int nl = nloc[i];
                for (int l = 0; l < nl; ++l) {
                    const int p = jcol[(size_t)l * M + i];
                    if (P.p_class[p] != PC_G) continue;
                    const int gi = P.p_pos[p] - nCF;
                    sg[o][gi] = J[(size_t)(2 * l) * M + i];
                    sg[o][NGMAX + gi] = J[(size_t)(2 * l + 1) * M + i];
                }
                sg[o][2 * NGMAX] = f[2 * i];
                sg[o][2 * NGMAX + 1] = f[2 * i + 1];
            }
        }
        __syncthreads();
        const int no = min(OB, i1 - b0);
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int e = threadIdx.x + 256 * k;
            if (e >= NA) continue;
            const bool mat = e < nG * nG;
            const int a = mat ? e / nG : e - nG * nG;
            const int bx = mat ? e % nG : 2 * NGMAX, by = mat ? NGMAX + bx : 2 * NGMAX + 1;
            double v = acc[k];
            for (int o = 0; o < no; ++o)
                v += sg[o][a] * sg[o][bx] + sg[o][NGMAX + a] * sg[o][by];
            acc[k] = v;
        }
    }
    // the block's row of [Agg | gG], compact (nG^2 + nG entries, as k_ne_glob)
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const int e = threadIdx.x + 256 * k;
        if (e < NA) partial[(size_t)blockIdx.x * NA + e] = acc[k];
    }
}

// Sum of the per-block partial rows: one wave per entry (entries dealt to
// the 4 waves), lanes stride over the blocks, fixed xor-shuffle tree.
__global__ void __launch_bounds__(256) k_ne_glob_reduce(DevProblem P,
                                                        const double *__restrict__ partial,
                                                        int nblk, double *Agg, double *gG) {
    const int nG = P.nG, NA = nG * nG + nG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int t = wave; t < NA; t += 4) {
        const bool mat = t < nG * nG;
        double s = 0.;
        for (int k = lane; k < nblk; k += 64) s += partial[(size_t)k * NA + t];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) {
            if (mat)
                Agg[(t / nG) * NGMAX + t % nG] = s;
            else
                gG[t - nG * nG] = s;
        }
    }
}

// Column norms acnorm_p = sqrt(A_pp) in parameter order.
__global__ void k_colnorms(DevProblem P, const double *__restrict__ Acc,
                           const double *__restrict__ Abb, const double *__restrict__ Agg,
                           const double *__restrict__ gG, double *acnorm, double *g) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    const int cls = P.p_class[p];
    double d = 0.;
    if (cls == PC_CF) {
        const int r = P.p_pos[p];  // R index; find cf by the block table
        const int cf = P.p_blk[p];
        const int a = r - P.cf_roff[cf];
        d = Acc[(size_t)cf * PCMAX * PCMAX + a * PCMAX + a];
    } else if (cls == PC_B) {
        const int b = P.p_blk[p];
        const int a = P.p_pos[p];
        d = Abb[(size_t)b * 9 + a * 3 + a];
    } else {
        const int gi = P.p_pos[p] - (P.nR - P.nG);
        d = Agg[gi * NGMAX + gi];
        g[p] = gG[gi];
    }
    acnorm[p] = sqrt(d);
}

// Block tree reduction of one value per thread into partial[blockIdx.x]
// (the order of k_sumsq / k_gnorm / k_zero_flag: bit-identical partials).
template <bool MAX>
__device__ __forceinline__ void block_partial(double v, double *red, double *partial) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            red[threadIdx.x] = MAX ? fmax(red[threadIdx.x], red[threadIdx.x + w])
                                   : red[threadIdx.x] + red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// lmder bookkeeping after a Jacobian evaluation in one pass over the
// parameters (lmder.c after qrfac; MINPACK's rank test):
//   acnorm_p = sqrt(A_pp) and g_p of global parameters (k_colnorms);
//   partial row 0: max over owned p of [acnorm_p == 0]           (k_zero_flag)
//   diag update: mode 1, first pass diag = acnorm (1 where 0), then
//   diag = max(diag, acnorm)                                      (k_diag_init)
//   partial row 1: sum over owned p of (diag_p x_p)^2, do_xn      (xnorm)
//   partial row 2: max over owned p with acnorm_p != 0 of
//   |g_p / fnorm| / acnorm_p, do_gn                               (k_gnorm)
// Rows are rstride apart, nparts = gridDim.x blocks each; every thread
// accumulates in the grid-stride order of the separate kernels.
__global__ void __launch_bounds__(256) k_jac_epilogue(
    DevProblem P, const double *__restrict__ Acc, const double *__restrict__ Abb,
    const double *__restrict__ Agg, const double *__restrict__ gG, double *acnorm, double *g,
    double *diag, const double *__restrict__ x, int first, int mode, double fnorm,
    const double *__restrict__ fnorm_sq, int do_xn, int do_gn, const int *__restrict__ mask,
    double *partial, int rstride, const double *__restrict__ c15, const double *__restrict__ s15,
    double *gfull, const double *__restrict__ adiag15, const double *__restrict__ u15) {
    __shared__ double red[256];
    if (fnorm_sq) {
        fnorm = sqrt(*fnorm_sq);
        do_gn = do_gn && fnorm != 0.;
    }
    const double s15v = c15 ? *s15 : 0.;
    double zf = 0., xn = 0., gm = 0.;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P.n; p += gridDim.x * blockDim.x) {
        const int cls = P.p_class[p];
        double d = 0.;
        double gp;
        if (cls == PC_CF) {
            const int cf = P.p_blk[p];
            const int a = P.p_pos[p] - P.cf_roff[cf];
            d = Acc[(size_t)cf * PCMAX * PCMAX + a * PCMAX + a];
            gp = g[p];
        } else if (cls == PC_B) {
            const int b = P.p_blk[p];
            const int a = P.p_pos[p];
            d = Abb[(size_t)b * 9 + a * 3 + a];
            gp = g[p];
        } else {
            const int gi = P.p_pos[p] - (P.nR - P.nG);
            d = Agg[gi * NGMAX + gi];
            gp = gG[gi];
            g[p] = gp;
        }
        if (c15) {
            // B15: ||J_p||^2 and (J^T f)_p of J = J_s + f c^T, with
            // u = J_s^T f: A_pp + 2 c_p u_p + s c_p^2, u_p + s c_p (camera-frame
            // parameters: A_pp and u_p back from the rotated block, adiag15 / u15)
            if (cls == PC_CF) {
                d = adiag15[p];
                gp = u15[p];
            }
            const double cp = c15[p];
            d = fmax(d + 2. * cp * gp + s15v * cp * cp, 0.);
            gp = gp + s15v * cp;
            gfull[p] = gp;
        }
        const double an = sqrt(d);
        acnorm[p] = an;
        double dg = diag[p];
        if (mode != 2) {
            if (first) dg = an == 0. ? 1. : an;
            dg = fmax(dg, an);
            diag[p] = dg;
        }
        if (own_mask(mask, p)) {
            if (an == 0.) zf = 1.;
            if (do_xn) {
                const double v = dg * x[p];
                xn += v * v;
            }
            if (do_gn && an != 0.) gm = fmax(gm, fabs((gp / fnorm) / an));
        }
    }
    block_partial<true>(zf, red, partial);
    __syncthreads();
    block_partial<false>(xn, red, partial + rstride);
    __syncthreads();
    block_partial<true>(gm, red, partial + 2 * rstride);
}

// lmder trial point in one pass over the parameters: p = -xs,
// wa1 = p, wa2 = x + p, wa3 = diag p (k_lm_step); setParameters at wa2
// (k_param_prep + k_set_attrs); partial rows: 0 = sum (diag p)^2 (pnorm),
// 1 = sum (diag wa2)^2 (the candidate ||D x||), over owned p.
__global__ void __launch_bounds__(256) k_trial_prep(
    DevProblem P, const double *__restrict__ xs, const double *__restrict__ x,
    const double *__restrict__ diag, double *wa1, double *wa2, double *wa3, double *ext,
    double *ext_pert, double *step, int solver_type, double delta, double eps_dif,
    const int *__restrict__ mask, double *partial, int rstride) {
    __shared__ double red[256];
    double pn = 0., xn = 0.;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < P.n; j += gridDim.x * blockDim.x) {
        const double st = -xs[j];
        const double dj = diag[j];
        const double xj = x[j] + st;
        const double w3 = dj * st;
        wa1[j] = st;
        wa2[j] = xj;
        wa3[j] = w3;
        param_prep_one(P, j, xj, ext, ext_pert, step, solver_type, delta, eps_dif);
        set_attr_one(P, j, ext[j]);
        if (own_mask(mask, j)) {
            pn += w3 * w3;
            const double v = dj * xj;
            xn += v * v;
        }
    }
    block_partial<false>(pn, red, partial);
    __syncthreads();
    block_partial<false>(xn, red, partial + rstride);
}

// lmder after a trial point (oracle/refcpu.c lm_core; mmba_lm.cpp
// Plan::solve and lmpar_ne's undamped test), the same operations in the same
// order as the host's, from the slots this reduction just wrote.
__device__ void lm_decide(const LmDec &d, double *scalar) {
    const double p1 = .1, p5 = .5, p25 = .25, p75 = .75, p0001 = 1e-4;
    const double epsmch = DBL_EPSILON;
    double fnorm = d.f0 ? sqrt(scalar[d.s_f0]) : d.fnorm;
    double delta = d.delta, xnorm = d.xnorm, par = d.par, gnorm = d.gnorm;
    int info = 0, go = 0;
    double ratio = 0.;
    bool taken = true;
    if (d.spec) {
        if (d.first) {
            xnorm = sqrt(scalar[d.s_xn2]);
            delta = d.factor * xnorm;
            if (delta == 0.) delta = d.factor;
        }
        gnorm = fnorm != 0. ? scalar[d.s_gnorm] : 0.;
        if (gnorm <= d.gtol) {
            info = 4;
            taken = false;
        } else {
            const double fl = scalar[d.s_fail];
            const bool ok0 = fl == 0.;
            const double dxnorm = ok0 ? sqrt(scalar[d.s_dnorm]) : HUGE_VAL;
            const double fp = dxnorm - delta;
            // a dataflow timeout (flag >= 2) makes the host solve again
            taken = fl < 2. && fp <= p1 * delta;
            par = 0.;
        }
    }
    if (taken) {
        const double pnorm = sqrt(scalar[d.s_pnorm]);
        if (d.first) delta = fmin(delta, pnorm);
        const double fnorm1 = sqrt(scalar[d.s_fnorm]);
        double actred = -1.;
        if (p1 * fnorm1 < fnorm) {
            const double d1 = fnorm1 / fnorm;
            actred = 1. - d1 * d1;
        }
        const double temp1 = sqrt(scalar[d.s_jp]) / fnorm;
        const double temp2 = (sqrt(par) * pnorm) / fnorm;
        const double prered = temp1 * temp1 + temp2 * temp2 / p5;
        const double dirder = -(temp1 * temp1 + temp2 * temp2);
        if (prered != 0.) ratio = actred / prered;
        if (ratio <= p25) {
            double temp;
            if (actred >= 0.)
                temp = p5;
            else
                temp = p5 * dirder / (dirder + p5 * actred);
            if (p1 * fnorm1 >= fnorm || temp < p1) temp = p1;
            delta = temp * fmin(delta, pnorm / p1);
            par /= temp;
        } else if (par == 0. || ratio >= p75) {
            delta = pnorm / p5;
            par = p5 * par;
        }
        const bool accept = ratio >= p0001;
        if (accept) xnorm = sqrt(scalar[d.s_xn2t]);
        if (fabs(actred) <= d.ftol && prered <= d.ftol && p5 * ratio <= 1.) info = 1;
        if (delta <= d.xtol * xnorm) info = 2;
        if (fabs(actred) <= d.ftol && prered <= d.ftol && p5 * ratio <= 1. && info == 2) info = 3;
        if (info == 0) {
            if (d.nfev >= d.maxfev) info = 5;
            if (fabs(actred) <= epsmch && prered <= epsmch && p5 * ratio <= 1.) info = 6;
            if (delta <= epsmch * xnorm) info = 7;
            if (gnorm <= epsmch) info = 8;
        }
        go = (accept && info == 0) ? 1 : 0;
    }
    scalar[d.s_out] = go;
    scalar[d.s_out + 1] = ratio;
    scalar[d.s_out + 2] = delta;
    scalar[d.s_out + 3] = par;
    scalar[d.s_out + 4] = taken ? info : -100 - info;
    __hip_atomic_store(d.gate, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Several partial rows reduced in one launch, block r for row r, in the
// order of k_reduce_sum / k_reduce_max; block 0 also converts the
// factorisation fail flag to a scalar and clears it (k_flag_to_scalar).
// host (optional): the last block to finish copies scalar[0, host_n) into
// that page-locked host mirror (the LM control thread's slots), so the
// decision point needs no separate device-to-host copy launch.
__global__ void __launch_bounds__(256) k_reduce_multi(const double *__restrict__ partial,
                                                      RedSpec spec, double *scalar, int *flag,
                                                      double *host, int host_n,
                                                      unsigned *ticket, unsigned *host_seq,
                                                      unsigned seq, const LmDec dec) {
    __shared__ double red[256];
    const RedRow rw = spec.row[blockIdx.x];
    const double v = reduce_row_block<false>(partial, rw, red);
    if (threadIdx.x == 0) {
        scalar[rw.slot] = v;
        if (blockIdx.x == 0 && flag && spec.flag_slot >= 0) {
            scalar[spec.flag_slot] = (double)*flag;  // bit 1 pivot, bit 2 dataflow timeout
            *flag = 0;
        }
    }
    if (!host && !dec.on) return;
    __shared__ unsigned last;
    if (threadIdx.x == 0) {
        // release this block's slots, count it in; the last arrival acquires
        // every block's slots (agent scope: the blocks may sit on other XCDs)
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        last = t == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (dec.on) {
        if (threadIdx.x == 0) lm_decide(dec, scalar);
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    if (!host) {
        if (threadIdx.x == 0)
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // the mirror by wave 0 alone (host_n <= 64 slots: one store per lane), its
    // own system fence, then lane 0's release of the sequence word the host
    // polls -- no workgroup barrier and no fence in the other waves
    if (threadIdx.x < 64) {
        for (int i = threadIdx.x; i < host_n; i += 64)
            host[i] = __hip_atomic_load(&scalar[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (host_seq) {
            __threadfence_system();  // the wave's mirror stores visible to the host
            if (threadIdx.x == 0)
                __hip_atomic_store(host_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// -------------------------------------------------------------------------
// Damped system, bundle blocks: Abb + lam D^2 = Lb Lb^T (3x3), tb = Lb^-1 gb,
// Wg_b = Abg^T Lb^-T (nG x pb).  At lam == 0 an exactly-zero diagonal (zero
// Jacobian column) is replaced by 1 so that component solves to 0 (MINPACK's
// nsing truncation for exactly zero columns).
// -------------------------------------------------------------------------
__global__ void k_bundle_factor(DevProblem P, const double *__restrict__ Abb,
                                const double *__restrict__ Abg, const double *__restrict__ g,
                                const double *__restrict__ diag, double lam, double *Lb,
                                double *tb, double *Wg, int *fail) {
    const int b = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // XCD-contiguous
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    if (pb == 0) return;
    const int po = P.bnd_par_off[b];
    // every index static (no scratch); rows a >= pb are identity padding
    double A[3][3], rhs[3], dd[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
            A[a][c] = (a < pb && c < pb) ? Abb[(size_t)b * 9 + a * 3 + c] : (a == c ? 1. : 0.);
        rhs[a] = 0.;
        dd[a] = 0.;
        if (a < pb) {
            const int p = P.bnd_par[po + a];
            dd[a] = diag[p];
            rhs[a] = g[p];
        }
    }
    double L[3][3], il[3];
    bundle_chol3(A, rhs, dd, pb, lam, b, Lb, tb, fail, L, il);
    for (int q = 0; q < P.nG; ++q) {
        // row q of Abg^T, forward-solve against L: w L^T = a  ->  L w^T = a^T
        double w[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double s = a < pb ? Abg[((size_t)b * PBMAX + a) * NGMAX + q] : 0.;
#pragma unroll
            for (int k = 0; k < a; ++k) s -= L[a][k] * w[k];
            w[a] = s * il[a];
        }
        for (int a = 0; a < 3; ++a) Wg[((size_t)b * NGMAX + q) * 3 + a] = w[a];
    }
}

// W_i = (J_c(i)^T J_b(i)) Lb^-T per observation (pc x 3, AoS rows of wst
// doubles).  One wave per 64 consecutive observations: the rows are built in
// LDS and the wave's contiguous 64 wst-double chunk is stored coalesced
// (zeros where a row has no bundle block / no camera block).
// nob: the observation workgroups; workgroups nob + r reduce row r of red
// (the Jacobian epilogue's rows, which no W row reads: one launch less)
// PCT: the widest camera-frame block the launch carries in registers (the
// plan's pc_uniform-based bound: 8 for pose + focal plans, else PCMAX).
// gate (enqueued behind the gated Jacobian, Plan::pre_jac_enqueue): runs
// only when the device's restatement of the host's decision let the
// Jacobian run.
template <int PCT>
__global__ void __launch_bounds__(64) k_schur_obs(DevProblem P, const double *__restrict__ J,
                                                  const double *__restrict__ Lb, double *W,
                                                  int nob, const RedSpec red,
                                                  const double *__restrict__ partial,
                                                  double *scalar, const int *gate) {
    extern __shared__ double sw[];  // 64 x wst doubles (9 KB for pose-only BA)
    if (gate && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    const int lane = threadIdx.x;
    if ((int)blockIdx.x >= nob) {
        const RedRow rw = red.row[blockIdx.x - nob];
        const double v = reduce_row_w64(partial, rw);
        if (lane == 0) scalar[rw.slot] = v;
        return;
    }
    const int i0 = xcd_remap(blockIdx.x, nob) * 64;  // J rows from this XCD's L2
    const int i = i0 + lane;
    const int M = P.M, wst = P.wst;
    double *row = &sw[lane * wst];
    for (int k = 0; k < wst; ++k) row[k] = 0.;
    const int b = i < M ? P.obs_bnd[i] : 0;
    const int pb = i < M ? P.bnd_pb[b] : 0;
    if (pb > 0) {
        const int cf = P.obs_cf[i];
        const int pc = min(min(P.cf_pc[cf], wst / 3), PCT);
        const int s = P.cf_var_off[cf + 1] - P.cf_var_off[cf] - 1;
        // every index static (no scratch): bundle columns a < pb, camera rows r < pc
        double bx[3], by[3], L[3][3], il[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            bx[a] = a < pb ? J[(size_t)(2 * (s + a)) * M + i] : 0.;
            by[a] = a < pb ? J[(size_t)(2 * (s + a) + 1) * M + i] : 0.;
#pragma unroll
            for (int c = 0; c < 3; ++c) L[a][c] = Lb[(size_t)b * 9 + a * 3 + c];
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) il[a] = a < pb ? 1.0 / L[a][a] : 0.;
        double cx[PCT], cy[PCT];
#pragma unroll
        for (int r = 0; r < PCT; ++r) {  // every load issued before the solves
            cx[r] = r < pc ? J[(size_t)(2 * r) * M + i] : 0.;
            cy[r] = r < pc ? J[(size_t)(2 * r + 1) * M + i] : 0.;
        }
#pragma unroll
        for (int r = 0; r < PCT; ++r) {
            if (r < pc) {
                double w[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double t = cx[r] * bx[a] + cy[r] * by[a];
#pragma unroll
                    for (int k = 0; k < a; ++k) t -= L[a][k] * w[k];
                    w[a] = t * il[a];  // zero for a >= pb
                }
#pragma unroll
                for (int a = 0; a < 3; ++a) row[r * 3 + a] = w[a];
            }
        }
    }
    __syncthreads();
    const int nrow = min(64, M - i0);
    const size_t base = (size_t)i0 * wst;
    if (wst % 2 == 0) {
        const int nv = nrow * wst / 2;
        double2 *dst = reinterpret_cast<double2 *>(&W[base]);
        const double2 *src = reinterpret_cast<const double2 *>(sw);
        for (int k = lane; k < nv; k += 64) dst[k] = src[k];
    } else {
        for (int k = lane; k < nrow * wst; k += 64) W[base + k] = sw[k];
    }
}

// Rolling shutter with solved bundles: the W row of virtual observation v
// (real observation i = vobs[v], camera-frame block PV.obs_cf[v] whose
// columns start at vcoff[v] in i's row, the bundle's columns last:
// k_jacobian_rs) -- k_schur_obs's arithmetic, one thread per virtual
// observation.  J is indexed by the real observation count Mr.
__global__ void __launch_bounds__(64) k_schur_obs_rs(DevProblem PV, int Mr,
                                                     const int *__restrict__ nloc,
                                                     const int *__restrict__ vobs,
                                                     const int *__restrict__ vcoff,
                                                     const double *__restrict__ J,
                                                     const double *__restrict__ Lb, double *W) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= PV.M) return;
    const int wst = PV.wst;
    double *row = &W[(size_t)v * wst];
    for (int k = 0; k < wst; ++k) row[k] = 0.;
    const int b = PV.obs_bnd[v];
    const int pb = PV.bnd_pb[b];
    if (pb <= 0) return;
    const int i = vobs[v], cf = PV.obs_cf[v];
    const int pc = min(PV.cf_pc[cf], wst / 3);
    const int c0 = vcoff[v], s = nloc[i] - pb;
    double bx[3], by[3], L[3][3], il[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        bx[a] = a < pb ? J[(size_t)(2 * (s + a)) * Mr + i] : 0.;
        by[a] = a < pb ? J[(size_t)(2 * (s + a) + 1) * Mr + i] : 0.;
#pragma unroll
        for (int c = 0; c < 3; ++c) L[a][c] = Lb[(size_t)b * 9 + a * 3 + c];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) il[a] = a < pb ? 1.0 / L[a][a] : 0.;
    for (int r = 0; r < pc; ++r) {
        const double cx = J[(size_t)(2 * (c0 + r)) * Mr + i], cy = J[(size_t)(2 * (c0 + r) + 1) * Mr + i];
        double w[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double t = cx * bx[a] + cy * by[a];
#pragma unroll
            for (int k = 0; k < a; ++k) t -= L[a][k] * w[k];
            w[a] = t * il[a];
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) row[r * 3 + a] = w[a];
    }
}

// S = (Acc + lam D^2 | Acg | Agg + lam D^2), lower triangle, plus identity
// on the padded tail; rhs = g_R.
__device__ __forceinline__ void schur_init_row(
    const DevProblem &P, const double *__restrict__ Acc, const double *__restrict__ Acg,
    const double *__restrict__ Agg, const double *__restrict__ g,
    const double *__restrict__ diag, double lam, const SView &V, int npad,
    double *__restrict__ rhs, int t) {
    // one thread per reduced row: (camera-frame, row a) for t < ncf * PCMAX,
    // then the global rows, then the padding rows
    const int nG = P.nG;
    const int nCF = P.nR - nG;
    const int ncr = P.ncf * PCMAX;
    if (t < ncr) {
        const int cf = t / PCMAX, a = t % PCMAX;
        const int pc = P.cf_pc[cf];
        if (a >= pc || !own_cf(P, cf)) return;
        const int r0 = P.cf_roff[cf];
        const int v0 = P.cf_var_off[cf] + 1;
        const double *Arow = &Acc[(size_t)cf * PCMAX * PCMAX + a * PCMAX];
        double av[PCMAX];
#pragma unroll
        for (int c = 0; c < PCMAX; ++c) av[c] = c <= a ? Arow[c] : 0.;
        const int pa = P.cf_var_param[v0 + a];
        const double d = diag[pa], ga = g[pa];
#pragma unroll
        for (int c = 0; c < PCMAX; ++c) {
            if (c > a) break;
            double v = av[c];
            if (c == a) {
                v += lam * (d * d);
                if (v == 0.) v = 1.;
            }
            *s_at(V, r0 + a, r0 + c) = v;
        }
        rhs[r0 + a] = (av[a] == 0. && lam == 0.) ? 0. : ga;
        for (int q = 0; q < nG; ++q)
            *s_at(V, nCF + q, r0 + a) = Acg[((size_t)cf * PCMAX + a) * NGMAX + q];
    } else if (t < ncr + nG) {
        const int q = t - ncr;
        const int p = P.g_param[q];
        if (!P.root) {  // the global block and its rhs are added once
            rhs[nCF + q] = 0.;
            return;
        }
        for (int c = 0; c <= q; ++c) {
            double v = Agg[q * NGMAX + c];
            if (c == q) {
                const double d = diag[p];
                v += lam * (d * d);
                if (v == 0.) v = 1.;
            }
            *s_at(V, nCF + q, nCF + c) = v;
        }
        rhs[nCF + q] = (Agg[q * NGMAX + q] == 0. && lam == 0.) ? 0. : g[p];
    } else {
        const int r = P.nR + (t - ncr - nG);
        if (r < P.nR + npad) {
            *s_at(V, r, r) = 1.;
            rhs[r] = 0.;
        }
    }
}
__global__ void __launch_bounds__(256) k_schur_init(
    DevProblem P, const double *__restrict__ Acc, const double *__restrict__ Acg,
    const double *__restrict__ Agg, const double *__restrict__ g,
    const double *__restrict__ diag, double lam, const SView V, int npad,
    double *__restrict__ rhs) {
    schur_init_row(P, Acc, Acg, Agg, g, diag, lam, V, npad, rhs,
                   blockIdx.x * blockDim.x + threadIdx.x);
}
// ... with the Jacobian epilogue's row reductions beside it (C5: the
// reduction that followed the epilogue was its own launch, and k_schur_init
// does not read its slots): workgroups [0, nb) form the rows, workgroup nb + r
// reduces row r exactly as k_reduce_multi's block r does.
__global__ void __launch_bounds__(256) k_schur_init_red(
    DevProblem P, const double *__restrict__ Acc, const double *__restrict__ Acg,
    const double *__restrict__ Agg, const double *__restrict__ g,
    const double *__restrict__ diag, double lam, const SView V, int npad,
    double *__restrict__ rhs, int nb, const double *__restrict__ partial, RedSpec spec,
    double *scalar) {
    if ((int)blockIdx.x < nb) {
        schur_init_row(P, Acc, Acg, Agg, g, diag, lam, V, npad, rhs,
                       blockIdx.x * blockDim.x + threadIdx.x);
        return;
    }
    __shared__ double red[256];
    const RedRow rw = spec.row[blockIdx.x - nb];
    const double v = reduce_row_block<false>(partial, rw, red);
    if (threadIdx.x == 0) scalar[rw.slot] = v;
}

// Schur complement over bundles: S -= sum_b W_b W_b^T, rhs -= W_b tb.
__global__ void k_schur_pairs(DevProblem P, const double *__restrict__ W,
                              const double *__restrict__ Wg, const double *__restrict__ tb,
                              const SView V, double *rhs) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    if (pb == 0) return;
    const int nG = P.nG;
    const int nCF = P.nR - nG;
    const int q0 = P.bobs_off[b], q1 = P.bobs_off[b + 1];
    const double t0 = tb[(size_t)b * 3], t1 = tb[(size_t)b * 3 + 1], t2 = tb[(size_t)b * 3 + 2];
    for (int qi = q0; qi < q1; ++qi) {
        const int i = P.bobs[qi];
        const int cfi = P.obs_cf[i];
        const int pci = P.cf_pc[cfi];
        const int ri = P.cf_roff[cfi];
        for (int a = 0; a < pci; ++a) {
            const double wa0 = W[widx(P, a * 3, i)], wa1 = W[widx(P, a * 3 + 1, i)],
                         wa2 = W[widx(P, a * 3 + 2, i)];
            atomicAdd(&rhs[ri + a], -(wa0 * t0 + wa1 * t1 + wa2 * t2));
            for (int qj = q0; qj < q1; ++qj) {
                const int j = P.bobs[qj];
                const int cfj = P.obs_cf[j];
                const int pcj = P.cf_pc[cfj];
                const int rj = P.cf_roff[cfj];
                for (int c = 0; c < pcj; ++c) {
                    const int R = ri + a, C = rj + c;
                    if (R < C) continue;
                    const double v = wa0 * W[widx(P, c * 3, j)] +
                                     wa1 * W[widx(P, c * 3 + 1, j)] +
                                     wa2 * W[widx(P, c * 3 + 2, j)];
                    atomicAdd(s_at(V, R, C), -v);
                }
            }
        }
    }
    for (int q = 0; q < nG; ++q) {
        const double *wg = &Wg[((size_t)b * NGMAX + q) * 3];
        atomicAdd(&rhs[nCF + q], -(wg[0] * t0 + wg[1] * t1 + wg[2] * t2));
        for (int qj = q0; qj < q1; ++qj) {
            const int j = P.bobs[qj];
            const int cfj = P.obs_cf[j];
            const int pcj = P.cf_pc[cfj];
            const int rj = P.cf_roff[cfj];
            for (int c = 0; c < pcj; ++c) {
                const double v = wg[0] * W[widx(P, c * 3, j)] +
                                 wg[1] * W[widx(P, c * 3 + 1, j)] +
                                 wg[2] * W[widx(P, c * 3 + 2, j)];
                atomicAdd(s_at(V, nCF + q, rj + c), -v);
            }
        }
        for (int q2 = 0; q2 <= q; ++q2) {
            const double *wh = &Wg[((size_t)b * NGMAX + q2) * 3];
            atomicAdd(s_at(V, nCF + q, nCF + q2),
                      -(wg[0] * wh[0] + wg[1] * wh[1] + wg[2] * wh[2]));
        }
    }
}

// Deterministic Schur accumulation: one wave per destination block
// (cf_i >= cf_j); pairs of observations sharing a bundle are pre-sorted by
// destination on the host, so every S entry has a single writer and a fixed
// summation order (no atomics).  The pairs' W rows are staged through LDS 64
// pairs at a time: lane q loads pair q (the i of one destination are one
// camera-frame's contiguous observations, so the SoA loads coalesce), then
// lane e accumulates entries e and e + 64 of the (pci x pcj) block.
__global__ void __launch_bounds__(64) k_schur_dest(DevProblem P, const double *__restrict__ W,
                                                   const int2 *__restrict__ dest,
                                                   const int *__restrict__ dest_off,
                                                   const int2 *__restrict__ pairs,
                                                   const SView V, int assign_off) {
    __shared__ double sA[3 * PCMAX][65];
    __shared__ double sB[3 * PCMAX][65];
    const int d = blockIdx.x;
    const int2 cc = dest[d];
    const int pci = P.cf_pc[cc.x], pcj = P.cf_pc[cc.y];
    const int ri = P.cf_roff[cc.x], rj = P.cf_roff[cc.y];
    const int q0 = dest_off[d], q1 = dest_off[d + 1];
    const int lane = threadIdx.x;
    const int ne = pci * pcj;
    const int e0 = lane, e1 = lane + 64;
    const int a0 = e0 / max(pcj, 1), c0 = e0 % max(pcj, 1);
    const int a1 = e1 / max(pcj, 1), c1 = e1 % max(pcj, 1);
    const bool v0 = e0 < ne && ri + a0 >= rj + c0;
    const bool v1 = e1 < ne && ri + a1 >= rj + c1;
    double acc0 = 0., acc1 = 0.;
    for (int qb = q0; qb < q1; qb += 64) {
        const int cnt = min(64, q1 - qb);
        const int2 pr = lane < cnt ? pairs[qb + lane] : make_int2(0, 0);
        double ra[3 * PCMAX], rb[3 * PCMAX];
#pragma unroll
        for (int k = 0; k < 3 * PCMAX; ++k) {  // issue every load before the stores
            ra[k] = (lane < cnt && k < 3 * pci) ? W[widx(P, k, pr.x)] : 0.;
            rb[k] = (lane < cnt && k < 3 * pcj) ? W[widx(P, k, pr.y)] : 0.;
        }
#pragma unroll
        for (int k = 0; k < 3 * PCMAX; ++k) {
            sA[k][lane] = ra[k];
            sB[k][lane] = rb[k];
        }
        __syncthreads();
        if (v0)
            for (int q = 0; q < cnt; ++q)
                acc0 += sA[a0 * 3][q] * sB[c0 * 3][q] + sA[a0 * 3 + 1][q] * sB[c0 * 3 + 1][q] +
                        sA[a0 * 3 + 2][q] * sB[c0 * 3 + 2][q];
        if (v1)
            for (int q = 0; q < cnt; ++q)
                acc1 += sA[a1 * 3][q] * sB[c1 * 3][q] + sA[a1 * 3 + 1][q] * sB[c1 * 3 + 1][q] +
                        sA[a1 * 3 + 2][q] * sB[c1 * 3 + 2][q];
        __syncthreads();
    }
    // off-diagonal camera-frame blocks have this single writer: with
    // assign_off they are assigned (no zeroing of S needed between solves)
    const bool asg = assign_off && cc.x != cc.y;
    if (v0) {
        double *d = s_at(V, ri + a0, rj + c0);
        *d = asg ? -acc0 : *d - acc0;
    }
    if (v1) {
        double *d = s_at(V, ri + a1, rj + c1);
        *d = asg ? -acc1 : *d - acc1;
    }
}

// Uniform camera-frame block size PC (every solved camera-frame has PC
// parameters, e.g. 6 for pose-only BA): one wave per destination block; lane
// q accumulates the full PC x PC product of the pairs q, q + 64, ... in
// registers (16-B vector loads of the AoS W rows, no LDS in the loop), then
// the 64 partial blocks are summed through LDS in a fixed order
// (deterministic).  XCD-aware order: consecutive workgroups are dealt round
// robin to the 8 XCDs, so workgroup w takes destination
// (w % 8) * ceil(ndest / 8) + w / 8 -- each XCD sweeps one contiguous band of
// destinations and the W rows of its camera-frames stay in that XCD's L2.
// Two waves per SIMD: C4's 1,992 destinations are ~2 waves per SIMD anyway, and
// the 3-wave register cap spilled the prefetched W rows to scratch.
template <int PC>
__global__ void __launch_bounds__(64, 2) k_schur_dest_u(DevProblem P, const double *__restrict__ W,
                                                     const int2 *__restrict__ dest,
                                                     const int *__restrict__ dest_off,
                                                     const int2 *__restrict__ pairs,
                                                     const SView V, int assign_off, int ndest,
                                                     const double *__restrict__ tb, double *rhs,
                                                     const SchurInitFold fold,
                                                     const int *__restrict__ list) {
    // diagonal destinations (cf, cf) hold exactly the pairs (i, i) of the
    // camera-frame's observations with a bundle block, so they also form
    // rhs_R -= sum_i W_i t_b(i) (k_schur_rhs) in the same loop
    // two-step lane reduction through a half-width buffer: 11 KB of LDS per
    // one-wave workgroup (a 64-wide buffer, 22 KB, capped residency at 7
    // workgroups per CU -- 1,792 < 1,992 destinations for C4 -- and ran the
    // grid in two rounds)
    __shared__ double red[PC * PC + PC][33];
    const int per = (ndest + 7) / 8;
    int d = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (d >= ndest) return;
    if (list) d = list[d];  // the destinations k_schur_dest_lane leaves
    const int2 cc = dest[d];
    const int ri = P.cf_roff[cc.x], rj = P.cf_roff[cc.y];
    const int q0 = dest_off[d], q1 = dest_off[d + 1];
    const int lane = threadIdx.x;
    const bool diag = rhs && cc.x == cc.y && own_cf(P, cc.x);
    // pairs of a diagonal destination are (i, i) when no observation's
    // bundle is seen twice in one camera-frame (plan flag, host-checked)
    const bool same = cc.x == cc.y && P.dest_diag_ii;
    double acc[PC * PC], accr[PC];
#pragma unroll
    for (int e = 0; e < PC * PC; ++e) acc[e] = 0.;
#pragma unroll
    for (int a = 0; a < PC; ++a) accr[a] = 0.;
    // pair indices of up to 8 rounds are loaded first (independent loads);
    // the unrolled rounds then let the W gathers of round k + 1 overlap the
    // products of round k
    constexpr int NPF = 4;
    for (int qb = q0; qb < q1; qb += 64 * NPF) {
        int2 prk[NPF];
#pragma unroll
        for (int k = 0; k < NPF; ++k) {
            const int q = qb + lane + 64 * k;
            prk[k] = q < q1 ? pairs[q] : make_int2(-1, -1);
        }
#pragma unroll
        for (int k = 0; k < NPF; ++k) {
        const int2 pr = prk[k];
        if (pr.x < 0) continue;
        double wi[3 * PC], wj[3 * PC];
        if (same) {
            // diagonal destination: every pair is (i, i) (a bundle is seen
            // once per camera-frame), so one W row is loaded for both sides
            if constexpr ((3 * PC) % 2 == 0) {
                const double2 *pi = reinterpret_cast<const double2 *>(&W[widx(P, 0, pr.x)]);
#pragma unroll
                for (int k = 0; k < 3 * PC / 2; ++k) {
                    const double2 a = pi[k];
                    wi[2 * k] = wj[2 * k] = a.x;
                    wi[2 * k + 1] = wj[2 * k + 1] = a.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 3 * PC; ++k) wi[k] = wj[k] = W[widx(P, k, pr.x)];
            }
        } else if constexpr ((3 * PC) % 2 == 0) {  // wst = 3 PC: 16-B aligned records
            const double2 *pi = reinterpret_cast<const double2 *>(&W[widx(P, 0, pr.x)]);
            const double2 *pj = reinterpret_cast<const double2 *>(&W[widx(P, 0, pr.y)]);
#pragma unroll
            for (int k = 0; k < 3 * PC / 2; ++k) {
                const double2 a = pi[k], b = pj[k];
                wi[2 * k] = a.x;
                wi[2 * k + 1] = a.y;
                wj[2 * k] = b.x;
                wj[2 * k + 1] = b.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3 * PC; ++k) {
                wi[k] = W[widx(P, k, pr.x)];
                wj[k] = W[widx(P, k, pr.y)];
            }
        }
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = 0; c < PC; ++c)
                acc[a * PC + c] += wi[a * 3] * wj[c * 3] + wi[a * 3 + 1] * wj[c * 3 + 1] +
                                   wi[a * 3 + 2] * wj[c * 3 + 2];
        // rhs_R -= W_i t_b(i) once per observation: from its pair (i, i)
        // only (a diagonal destination also holds pairs (i, j) of two
        // observations of one bundle in one camera-frame, or of two
        // rolling-shutter virtual observations)
        if (diag && pr.x == pr.y) {
            const int b = P.obs_bnd[pr.x];
            const double t0 = tb[(size_t)b * 3], t1 = tb[(size_t)b * 3 + 1],
                         t2 = tb[(size_t)b * 3 + 2];
#pragma unroll
            for (int a = 0; a < PC; ++a)
                accr[a] += wi[a * 3] * t0 + wi[a * 3 + 1] * t1 + wi[a * 3 + 2] * t2;
        }
        }
    }
    if (lane >= 32) {
#pragma unroll
        for (int e = 0; e < PC * PC; ++e) red[e][lane - 32] = acc[e];
        if (diag)
#pragma unroll
            for (int a = 0; a < PC; ++a) red[PC * PC + a][lane - 32] = accr[a];
    }
    __syncthreads();
    if (lane < 32) {
#pragma unroll
        for (int e = 0; e < PC * PC; ++e) red[e][lane] += acc[e];
        if (diag)
#pragma unroll
            for (int a = 0; a < PC; ++a) red[PC * PC + a][lane] += accr[a];
    }
    __syncthreads();
    // folded k_schur_init (diagonal destinations): the entries it would have
    // written, with its operations, then the same subtraction
    const bool init = fold.on && cc.x == cc.y;
    const double *Ablk = &fold.Acc[(size_t)cc.x * PCMAX * PCMAX];
    const int v0 = P.cf_var_off[cc.x] + 1;
    for (int e = lane; e < PC * PC + (diag ? PC : 0); e += 64) {
        double v = 0.;
        for (int l = 0; l < 32; ++l) v += red[e][l];
        if (e >= PC * PC) {
            const int a = e - PC * PC;
            if (init) {
                const double ga = fold.g[P.cf_var_param[v0 + a]];
                rhs[ri + a] = ((Ablk[a * PCMAX + a] == 0. && fold.lam == 0.) ? 0. : ga) - v;
            } else {
                rhs[ri + a] -= v;
            }
            continue;
        }
        const int a = e / PC, c = e % PC;
        if (ri + a >= rj + c) {
            double *dd = s_at(V, ri + a, rj + c);
            if (init) {
                double b = Ablk[a * PCMAX + c];
                if (c == a) {
                    const double d = fold.diag[P.cf_var_param[v0 + a]];
                    b += fold.lam * (d * d);
                    if (b == 0.) b = 1.;
                }
                *dd = b - v;
            } else {
                *dd = (assign_off && cc.x != cc.y) ? -v : *dd - v;  // see k_schur_dest
            }
        }
    }
}

// Off-diagonal destinations of at most 32 pairs (C3: 9.3M destinations, 5.5
// pairs on average, where a wave per destination idles 59 of its 64 lanes
// and then reduces 36 sums through LDS): one lane per destination, its
// pairs in order.  k_schur_dest_u's lane l holds pair l alone for such a
// destination and its fixed-order lane sum adds them in pair order, so
// every entry is the same sum, bit for bit.  list: the destinations (XCD-
// contiguous runs of 256 per workgroup).
template <int PC>
__global__ void __launch_bounds__(256) k_schur_dest_lane(DevProblem P, const double *__restrict__ W,
                                                         const int2 *__restrict__ dest,
                                                         const int *__restrict__ dest_off,
                                                         const int2 *__restrict__ pairs,
                                                         const SView V, int assign_off,
                                                         const int *__restrict__ list, int nlist) {
    const int per = (int)(gridDim.x + 7) / 8;
    const int wg = (int)(blockIdx.x % 8) * per + (int)blockIdx.x / 8;
    const int k = wg * 256 + (int)threadIdx.x;
    if (k >= nlist) return;
    const int d = list[k];
    const int2 cc = dest[d];
    const int ri = P.cf_roff[cc.x], rj = P.cf_roff[cc.y];
    const int q0 = dest_off[d], q1 = dest_off[d + 1];
    double acc[PC * PC];
#pragma unroll
    for (int e = 0; e < PC * PC; ++e) acc[e] = 0.;
    for (int q = q0; q < q1; ++q) {
        const int2 pr = pairs[q];
        double wi[3 * PC], wj[3 * PC];
        if constexpr ((3 * PC) % 2 == 0) {
            const double2 *pi = reinterpret_cast<const double2 *>(&W[widx(P, 0, pr.x)]);
            const double2 *pj = reinterpret_cast<const double2 *>(&W[widx(P, 0, pr.y)]);
#pragma unroll
            for (int u = 0; u < 3 * PC / 2; ++u) {
                const double2 a = pi[u], b = pj[u];
                wi[2 * u] = a.x;
                wi[2 * u + 1] = a.y;
                wj[2 * u] = b.x;
                wj[2 * u + 1] = b.y;
            }
        } else {
#pragma unroll
            for (int u = 0; u < 3 * PC; ++u) {
                wi[u] = W[widx(P, u, pr.x)];
                wj[u] = W[widx(P, u, pr.y)];
            }
        }
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = 0; c < PC; ++c)
                acc[a * PC + c] += wi[a * 3] * wj[c * 3] + wi[a * 3 + 1] * wj[c * 3 + 1] +
                                   wi[a * 3 + 2] * wj[c * 3 + 2];
    }
#pragma unroll
    for (int a = 0; a < PC; ++a)
#pragma unroll
        for (int c = 0; c < PC; ++c)
            if (ri + a >= rj + c) {
                double *dd = s_at(V, ri + a, rj + c);
                *dd = assign_off ? -acc[a * PC + c] : *dd - acc[a * PC + c];  // see k_schur_dest
            }
}

// rhs_R -= sum_{i in cf} W_i t_b(i): one wave per camera-frame, lanes stride
// over the cf's contiguous observations (coalesced W reads), fixed-order wave
// reduction per row.
__global__ void __launch_bounds__(64) k_schur_rhs(DevProblem P, const double *__restrict__ W,
                                                  const double *__restrict__ tb, double *rhs) {
    const int cf = blockIdx.x;
    const int pc = P.cf_pc[cf];
    if (pc == 0 || !own_cf(P, cf)) return;
    const int r0 = P.cf_roff[cf];
    double acc[PCMAX];
#pragma unroll
    for (int a = 0; a < PCMAX; ++a) acc[a] = 0.;
    for (int i = P.cf_obs_off[cf] + (int)threadIdx.x; i < P.cf_obs_off[cf + 1]; i += 64) {
        const int b = P.obs_bnd[i];
        if (P.bnd_pb[b] == 0) continue;
        const double t0 = tb[(size_t)b * 3], t1 = tb[(size_t)b * 3 + 1], t2 = tb[(size_t)b * 3 + 2];
#pragma unroll
        for (int a = 0; a < PCMAX; ++a)
            if (a < pc)
                acc[a] += W[widx(P, a * 3, i)] * t0 + W[widx(P, a * 3 + 1, i)] * t1 +
                          W[widx(P, a * 3 + 2, i)] * t2;
    }
#pragma unroll
    for (int a = 0; a < PCMAX; ++a) {
        if (a >= pc) break;
        double v = acc[a];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (threadIdx.x == 0) rhs[r0 + a] -= v;
    }
}

// Global-parameter rows of the Schur complement (atomics; nG is small).
__global__ void k_schur_glob(DevProblem P, const double *__restrict__ W,
                             const double *__restrict__ Wg, const double *__restrict__ tb,
                             const SView V, double *rhs) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    const int nG = P.nG;
    if (pb == 0 || nG == 0) return;
    const int nCF = P.nR - nG;
    const bool ownb = own_bnd(P, b);
    const int q0 = P.bobs_off[b], q1 = P.bobs_off[b + 1];
    const double t0 = tb[(size_t)b * 3], t1 = tb[(size_t)b * 3 + 1], t2 = tb[(size_t)b * 3 + 2];
    for (int q = 0; q < nG; ++q) {
        const double *wg = &Wg[((size_t)b * NGMAX + q) * 3];
        if (ownb) atomicAdd(&rhs[nCF + q], -(wg[0] * t0 + wg[1] * t1 + wg[2] * t2));
        for (int qj = q0; qj < q1; ++qj) {
            const int j = P.bobs[qj];
            const int cfj = P.obs_cf[j];
            if (!own_cf(P, cfj)) continue;  // S rows/columns of own camera-frames
            const int pcj = P.cf_pc[cfj];
            const int rj = P.cf_roff[cfj];
            for (int c = 0; c < pcj; ++c) {
                const double v = wg[0] * W[widx(P, c * 3, j)] +
                                 wg[1] * W[widx(P, c * 3 + 1, j)] +
                                 wg[2] * W[widx(P, c * 3 + 2, j)];
                atomicAdd(s_at(V, nCF + q, rj + c), -v);
            }
        }
        if (!ownb) continue;
        for (int q2 = 0; q2 <= q; ++q2) {
            const double *wh = &Wg[((size_t)b * NGMAX + q2) * 3];
            atomicAdd(s_at(V, nCF + q, nCF + q2),
                      -(wg[0] * wh[0] + wg[1] * wh[1] + wg[2] * wh[2]));
        }
    }
}

// u_i = W_i^T x_cf(i) per observation, so the per-bundle back substitution
// gathers 3 values per observation instead of the 3 x pc of W_i.  One wave
// per 64 consecutive observations: their contiguous W rows are loaded
// coalesced into LDS first.
__global__ void __launch_bounds__(64) k_obs_wtx(DevProblem P, const double *__restrict__ W,
                                                const double *__restrict__ xR, double *U) {
    extern __shared__ double sw[];  // 64 x wst doubles
    const int lane = threadIdx.x;
    const int i0 = xcd_remap(blockIdx.x, gridDim.x) * 64;  // W rows from this XCD's L2
    const int i = i0 + lane;
    const int M = P.M, wst = P.wst;
    const int nrow = min(64, M - i0);
    const size_t base = (size_t)i0 * wst;
    if (wst % 2 == 0) {
        const int nv = nrow * wst / 2;
        const double2 *src = reinterpret_cast<const double2 *>(&W[base]);
        double2 *dst = reinterpret_cast<double2 *>(sw);
        for (int k = lane; k < nv; k += 64) dst[k] = src[k];
    } else {
        for (int k = lane; k < nrow * wst; k += 64) sw[k] = W[base + k];
    }
    __syncthreads();
    if (i >= M) return;
    const int cf = P.obs_cf[i];
    const int pc = min(P.cf_pc[cf], wst / 3);
    const int r0 = P.cf_roff[cf];
    const double *row = &sw[lane * wst];
    double u[3] = {0., 0., 0.};
    for (int a = 0; a < pc; ++a) {
        const double xv = xR[r0 + a];
        for (int c = 0; c < 3; ++c) u[c] += row[a * 3 + c] * xv;
    }
    // one 32-B record per observation (coalesced; gathered per bundle)
    reinterpret_cast<double4 *>(U)[i] = make_double4(u[0], u[1], u[2], 0.);
}

// x_b = Lb^-T (tb - sum_i u_i - Wg_b^T x_G), scatter to parameter order.
__global__ void k_backsub_bundle(DevProblem P, const double *__restrict__ W,
                                 const double *__restrict__ U,
                                 const double *__restrict__ Wg, const double *__restrict__ tb,
                                 const double *__restrict__ Lb, const double *__restrict__ xR,
                                 double *x) {
    const int b = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // XCD-contiguous
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    if (pb == 0) return;
    const int nG = P.nG;
    const int nCF = P.nR - nG;
    double s[3] = {tb[(size_t)b * 3], tb[(size_t)b * 3 + 1], tb[(size_t)b * 3 + 2]};
    for (int q = P.bobs_off[b]; q < P.bobs_off[b + 1]; ++q) {
        double u[3];
        if (W) {  // u_i = W_i^T x_cf(i) here (k_obs_wtx's arithmetic), no U round trip
            const int i = P.bobs[q];
            const int cf = P.obs_cf[i];
            const int pc = min(P.cf_pc[cf], P.wst / 3);
            const int r0 = P.cf_roff[cf];
            const double *row = &W[widx(P, 0, i)];
            u[0] = u[1] = u[2] = 0.;
            for (int a = 0; a < pc; ++a) {
                const double xv = xR[r0 + a];
                for (int c = 0; c < 3; ++c) u[c] += row[a * 3 + c] * xv;
            }
        } else {
            const double4 uu = reinterpret_cast<const double4 *>(U)[P.bobs[q]];
            u[0] = uu.x;
            u[1] = uu.y;
            u[2] = uu.z;
        }
        s[0] -= u[0];
        s[1] -= u[1];
        s[2] -= u[2];
    }
    for (int q = 0; q < nG; ++q) {
        const double xv = xR[nCF + q];
        for (int c = 0; c < 3; ++c) s[c] -= Wg[((size_t)b * NGMAX + q) * 3 + c] * xv;
    }
    double L[3][3];
    for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) L[a][c] = Lb[(size_t)b * 9 + a * 3 + c];
    // compile-time indices under pb guards (same operation order): s, L and
    // xb stay in registers instead of scratch
    double xb[3] = {0., 0., 0.};
#pragma unroll
    for (int a = 2; a >= 0; --a) {
        if (a >= pb) continue;
        double t = s[a];
#pragma unroll
        for (int k = a + 1; k < 3; ++k)
            if (k < pb) t -= L[k][a] * xb[k];
        xb[a] = t / L[a][a];
    }
    const int po = P.bnd_par_off[b];
#pragma unroll
    for (int a = 0; a < 3; ++a)
        if (a < pb) x[P.bnd_par[po + a]] = xb[a];
}

// k_trial_prep's operations for parameter j with step xs_j; dj = diag[j] and
// x0 = x[j] already loaded.
__device__ __forceinline__ void trial_one_pre(const DevProblem &P, const TrialFold &T, int j,
                                              double xsj, double dj, double x0, double &pn,
                                              double &xn) {
    const double st = -xsj;
    const double xj = x0 + st;
    const double w3 = dj * st;
    T.wa1[j] = st;
    T.wa2[j] = xj;
    T.wa3[j] = w3;
    param_prep_one(P, j, xj, T.ext, T.ext_pert, T.step, T.solver_type, T.delta, T.eps_dif);
    set_attr_one(P, j, T.ext[j]);
    if (own_mask(T.own, j)) {  // sharded: each parameter counted by its owner
        pn += w3 * w3;
        const double v = dj * xj;
        xn += v * v;
    }
}

// k_trial_prep's operations for parameter j with step xs_j.
__device__ __forceinline__ void trial_one(const DevProblem &P, const TrialFold &T, int j,
                                          double xsj, double &pn, double &xn) {
    const double st = -xsj;
    const double dj = T.diag[j];
    const double xj = T.x[j] + st;
    const double w3 = dj * st;
    T.wa1[j] = st;
    T.wa2[j] = xj;
    T.wa3[j] = w3;
    param_prep_one(P, j, xj, T.ext, T.ext_pert, T.step, T.solver_type, T.delta, T.eps_dif);
    set_attr_one(P, j, T.ext[j]);
    if (own_mask(T.own, j)) {  // sharded: each parameter counted by its owner
        pn += w3 * w3;
        const double v = dj * xj;
        xn += v * v;
    }
}

// k_backsub_bundle (two-pass form: u_i from k_obs_wtx) + the trial point's
// parameter pass: workgroups [0, nbb) back-substitute their bundles and
// prepare those parameters from the step just formed; workgroups [nbb, ..)
// prepare the other parameters from xs (the reduced solve's scatter).
// Sharded plans count only their own parameters in the sums (TrialFold::own).
__global__ void __launch_bounds__(64) k_backsub_trial(DevProblem P, const double *__restrict__ U,
                                                      const double *__restrict__ W,
                                                      const double *__restrict__ Wg,
                                                      const double *__restrict__ tb,
                                                      const double *__restrict__ Lb,
                                                      const double *__restrict__ xR, double *x,
                                                      int nbb, TrialFold T) {
    __shared__ double red[256];
    double pn = 0., xn = 0.;
    if ((int)blockIdx.x < nbb) {
        const int b = xcd_remap(blockIdx.x, nbb) * blockDim.x + threadIdx.x;
        const int pb = b < P.nB ? P.bnd_pb[b] : 0;
        if (pb > 0) {
            const int nG = P.nG;
            const int nCF = P.nR - nG;
            double s[3] = {tb[(size_t)b * 3], tb[(size_t)b * 3 + 1], tb[(size_t)b * 3 + 2]};
            const int q0 = P.bobs_off[b], q1 = P.bobs_off[b + 1];
            // the operands of the bundle's three parameters, loaded before the
            // gather (independent of it): trial_one's reads, issued together
            const int po = P.bnd_par_off[b];
            int jj[3] = {-1, -1, -1};
            double dgj[3] = {0., 0., 0.}, x0j[3] = {0., 0., 0.};
#pragma unroll
            for (int a = 0; a < 3; ++a)
                if (a < pb) jj[a] = P.bnd_par[po + a];
#pragma unroll
            for (int a = 0; a < 3; ++a)
                if (a < pb) {
                    dgj[a] = T.diag[jj[a]];
                    x0j[a] = T.x[jj[a]];
                }
            if (W) {
                for (int q = q0; q < q1; ++q) {
                    // one pass (MMBA_PATH_BACKSUB_ONEPASS): k_obs_wtx's arithmetic here
                    double u[3];
                    const int i = P.bobs[q];
                    const int cf = P.obs_cf[i];
                    const int pc = min(P.cf_pc[cf], P.wst / 3);
                    const int r0 = P.cf_roff[cf];
                    const double *row = &W[widx(P, 0, i)];
                    u[0] = u[1] = u[2] = 0.;
                    for (int a = 0; a < pc; ++a) {
                        const double xv = xR[r0 + a];
                        for (int c = 0; c < 3; ++c) u[c] += row[a * 3 + c] * xv;
                    }
                    s[0] -= u[0];
                    s[1] -= u[1];
                    s[2] -= u[2];
                }
            } else {
                // u_i = W_i^T x from k_obs_wtx, four observations' loads issued
                // before their (in-order) subtractions: two memory round trips
                // per four observations instead of two per observation
                const double4 *U4 = reinterpret_cast<const double4 *>(U);
                for (int qb = q0; qb < q1; qb += 4) {
                    double4 uu[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (qb + k < q1) uu[k] = U4[P.bobs[qb + k]];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (qb + k < q1) {
                            s[0] -= uu[k].x;
                            s[1] -= uu[k].y;
                            s[2] -= uu[k].z;
                        }
                }
            }
            for (int q = 0; q < nG; ++q) {
                const double xv = xR[nCF + q];
                for (int c = 0; c < 3; ++c) s[c] -= Wg[((size_t)b * NGMAX + q) * 3 + c] * xv;
            }
            double L[3][3];
            for (int a = 0; a < 3; ++a)
                for (int c = 0; c < 3; ++c) L[a][c] = Lb[(size_t)b * 9 + a * 3 + c];
            double xb[3] = {0., 0., 0.};
#pragma unroll
            for (int a = 2; a >= 0; --a) {
                if (a >= pb) continue;
                double t = s[a];
#pragma unroll
                for (int k = a + 1; k < 3; ++k)
                    if (k < pb) t -= L[k][a] * xb[k];
                xb[a] = t / L[a][a];
            }
#pragma unroll
            for (int a = 0; a < 3; ++a)
                if (a < pb) {
                    const int j = jj[a];
                    x[j] = xb[a];
                    trial_one_pre(P, T, j, xb[a], dgj[a], x0j[a], pn, xn);
                }
        }
        // the bundle's record at the trial point (k_records' arithmetic; this
        // thread just set its parameters)
        if (T.rec && b < P.nB) bnd_record_thread(P, b, T.ext_pert, T.step, T.brec, 0);
    } else if (T.rec) {
        // four camera-frames per workgroup, 16 threads each: the trial values
        // of the camera-frame's parameters, then (after the barrier) its base
        // and variant records, as k_records builds them (measured: these
        // workgroups first in the grid, 18.4-19.1 us against 17.4-17.9 us)
        const int cf = ((int)blockIdx.x - nbb) * 4 + (int)(threadIdx.x >> 4);
        const int v = threadIdx.x & 15;
        int off = 0, nv = -1;
        if (cf < P.ncf) {
            off = P.cf_var_off[cf];
            nv = P.cf_var_off[cf + 1] - off - 1;
        }
        if (v < nv) {
            const int j = P.cf_var_param[off + 1 + v];
            trial_one(P, T, j, x[j], pn, xn);
        }
        __syncthreads();
        if (v <= nv) {
            const int p = P.cf_var_param[off + v];  // -1: the base record
            const long long ov_idx = p >= 0 ? P.p_vidx[p] : -1;
            const double ov_val = p >= 0 ? T.ext_pert[p] : 0.;
            camera_record_fast(P, cf, ov_idx, ov_val, &T.recs[(size_t)(off + v) * CAMREC],
                               p >= 0 ? P.p_attr[p] : -1);
        }
    } else {
        const int k = (blockIdx.x - nbb) * blockDim.x + threadIdx.x;
        if (k < T.nother) {
            const int j = T.other[k];
            trial_one(P, T, j, x[j], pn, xn);
        }
    }
    // one partial per workgroup, 64-lane fixed tree
    red[threadIdx.x] = pn;
    red[64 + threadIdx.x] = xn;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[threadIdx.x] += red[threadIdx.x + w];
            red[64 + threadIdx.x] += red[64 + threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        T.partial[blockIdx.x] = red[0];
        T.partial[T.rstride + blockIdx.x] = red[64];
    }
}

// The trial point's parameter pass with its records, for plans without a
// solved bundle (C5): workgroups [0, ncfb) take four camera-frames each (16
// lanes per camera-frame: its parameters' trial values, then after the
// barrier its base and variant records, as k_records builds them);
// workgroups [ncfb, ..) the other parameters, T.other (global parameters no
// camera or bundle record reads).  k_trial_prep + k_records in one launch.
__global__ void __launch_bounds__(64) k_trial_prep_rec(DevProblem P, const double *__restrict__ xs,
                                                       int ncfb, TrialFold T) {
    __shared__ double red[128];
    double pn = 0., xn = 0.;
    if ((int)blockIdx.x < ncfb) {
        const int cf = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 4);
        const int v = threadIdx.x & 15;
        int off = 0, nv = -1;
        if (cf < P.ncf) {
            off = P.cf_var_off[cf];
            nv = P.cf_var_off[cf + 1] - off - 1;
        }
        if (v < nv) {
            const int j = P.cf_var_param[off + 1 + v];
            trial_one(P, T, j, xs[j], pn, xn);
        }
        __syncthreads();
        if (v <= nv) {
            const int p = P.cf_var_param[off + v];  // -1: the base record
            const long long ov_idx = p >= 0 ? P.p_vidx[p] : -1;
            const double ov_val = p >= 0 ? T.ext_pert[p] : 0.;
            camera_record_fast(P, cf, ov_idx, ov_val, &T.recs[(size_t)(off + v) * CAMREC],
                               p >= 0 ? P.p_attr[p] : -1);
        }
    } else {
        const int k = ((int)blockIdx.x - ncfb) * 64 + (int)threadIdx.x;
        if (k < T.nother) {
            const int j = T.other[k];
            trial_one(P, T, j, xs[j], pn, xn);
        }
    }
    red[threadIdx.x] = pn;
    red[64 + threadIdx.x] = xn;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[threadIdx.x] += red[threadIdx.x + w];
            red[64 + threadIdx.x] += red[64 + threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        T.partial[blockIdx.x] = red[0];
        T.partial[T.rstride + blockIdx.x] = red[64];
    }
}

// Reduced-system solution (R order) -> parameter order.
__global__ void k_scatter_xR(DevProblem P, const double *__restrict__ xR, double *x) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    if (P.p_class[p] != PC_B) x[p] = xR[P.p_pos[p]];
}

// Newton-correction helpers: u_b = Lb^-1 v_b per bundle (|u_b|^2 into
// usq[b], u_b into un[3 b], and the bundle's global-row terms Wg_b u_b into
// gp[q nB + b]); the camera-frame rows w_R -= sum_b W_b u_b are then the
// fixed-order per-camera-frame gather of k_schur_rhs and the global rows a
// fixed-order reduction (k_newton_glob): no floating-point atomics, so the
// solve is bit-for-bit repeatable.
__global__ void k_newton_bundle(DevProblem P, const double *__restrict__ Wg,
                                const double *__restrict__ Lb, const double *__restrict__ v,
                                double *un, double *gp, double *usq) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= P.nB) return;
    const int pb = P.bnd_pb[b];
    const int nG = P.nG;
    double u[3] = {0., 0., 0.};
    if (pb > 0) {
        const int po = P.bnd_par_off[b];
        double L[3][3];
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) L[a][c] = Lb[(size_t)b * 9 + a * 3 + c];
        for (int a = 0; a < pb; ++a) {
            double t = v[P.bnd_par[po + a]];
            for (int k = 0; k < a; ++k) t -= L[a][k] * u[k];
            u[a] = t / L[a][a];
        }
    }
    const bool ownb = pb > 0 && own_bnd(P, b);
    usq[b] = ownb ? u[0] * u[0] + u[1] * u[1] + u[2] * u[2] : 0.;
    for (int c = 0; c < 3; ++c) un[(size_t)b * 3 + c] = u[c];
    for (int q = 0; q < nG; ++q) {
        double g = 0.;
        if (ownb)
            for (int c = 0; c < 3; ++c) g += Wg[((size_t)b * NGMAX + q) * 3 + c] * u[c];
        gp[(size_t)q * P.nB + b] = g;
    }
}

// w_R[nCF + q] -= sum_b gp[q nB + b], one workgroup per global row, fixed order.
__global__ void __launch_bounds__(256) k_newton_glob(DevProblem P, const double *__restrict__ gp,
                                                     double *wR) {
    const int q = blockIdx.x;
    __shared__ double red[4];
    double acc = 0.;
    for (int b = threadIdx.x; b < P.nB; b += 256) acc += gp[(size_t)q * P.nB + b];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) wR[P.nR - P.nG + q] -= (red[0] + red[1]) + (red[2] + red[3]);
}

// v (parameter order) -> R order (non-bundle parameters); padded tail zero.
__global__ void k_gather_R(DevProblem P, const double *__restrict__ v, double *vR, int nRpad) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P.n && P.p_class[p] != PC_B) {
        // this shard's rows, the global rows on the root shard, zero elsewhere
        const int R = P.p_pos[p];
        const bool mine = (R >= P.nR - P.nG) ? P.root != 0 : (R >= P.Ra && R < P.Rb);
        vR[R] = mine ? v[p] : 0.;
    }
    const int r = P.nR + p;
    if (r < nRpad && p < nRpad) vR[r] = 0.;
}

// -------------------------------------------------------------------------
// Vector helpers and deterministic reductions.  With a ticket the reduction
// finishes in the same launch: every block publishes its partial (release),
// takes a ticket, and the last block to arrive (acquire) combines all
// partials in the same fixed order as the separate k_reduce_* kernel, then
// resets the ticket (so the result is bit-identical to the two-launch form).
// -------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_sumsq(const double *__restrict__ a,
                                               const double *__restrict__ d, int n,
                                               const int *__restrict__ mask, double *partial,
                                               double *out, unsigned int *ticket) {
    __shared__ double red[256];
    double s = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (!own_mask(mask, i)) continue;
        double v = d ? d[i] * a[i] : a[i];
        s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    finish_blocks<false>(red[0], partial, out, ticket);
}

// Newton term of the separator form (BandSolver::pcr_int): mask 1 rows add
// y^2 (||L_T^-1 ..||^2 of the separator system), mask 2 rows y v (the
// interior's v^T S_II^-1 v, y = S_II^-1 v there).
__global__ void __launch_bounds__(256) k_sumsq_mix(const double *__restrict__ y,
                                                   const double *__restrict__ v, int n,
                                                   const int *__restrict__ mask, double *partial) {
    __shared__ double red[256];
    double s = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int m = mask[i];
        if (m == 1) s += y[i] * y[i];
        else if (m == 2) s += y[i] * v[i];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_sumsq_div(const double *__restrict__ a,
                                                   const double *__restrict__ d, int n,
                                                   const int *__restrict__ mask, double *partial,
                                                   double *out, unsigned int *ticket) {
    __shared__ double red[256];
    double s = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (!own_mask(mask, i)) continue;
        double v = a[i] / d[i];
        s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    finish_blocks<false>(red[0], partial, out, ticket);
}

__global__ void __launch_bounds__(256) k_reduce_sum(const double *__restrict__ partial, int n,
                                                    double *out) {
    __shared__ double red[256];
    double s = 0.;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

// gnorm (lmder.c): max_l |g_l / fnorm| / acnorm_l over acnorm_l != 0.
__global__ void __launch_bounds__(256) k_gnorm(const double *__restrict__ g,
                                               const double *__restrict__ acnorm, int n,
                                               double fnorm, const int *__restrict__ mask,
                                               double *partial, double *out,
                                               unsigned int *ticket) {
    __shared__ double red[256];
    double m = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (own_mask(mask, i) && acnorm[i] != 0.) m = fmax(m, fabs((g[i] / fnorm) / acnorm[i]));
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    finish_blocks<true>(red[0], partial, out, ticket);
}

__global__ void k_reduce_max(const double *__restrict__ partial, int n, double *out) {
    __shared__ double red[256];
    double m = 0.;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, partial[i]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

// ||J p||^2 partial sums (prered in lmder): (J p)_obs = sum_l J_l p[jcol_l].
__global__ void __launch_bounds__(256) k_jp_sumsq(DevProblem P, const double *__restrict__ J,
                                                  const int *__restrict__ jcol,
                                                  const int *__restrict__ nloc,
                                                  const double *__restrict__ p,
                                                  double *partial, double *out,
                                                  unsigned int *ticket) {
    __shared__ double red[256];
    const int M = P.M;
    double s = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
        if (!own_obs(P, i)) continue;
        double ax = 0., ay = 0.;
        const int nl = nloc[i];
        for (int l = 0; l < nl; ++l) {
            const double pv = p[jcol[(size_t)l * M + i]];
            ax += J[(size_t)(2 * l) * M + i] * pv;
            ay += J[(size_t)(2 * l + 1) * M + i] * pv;
        }
        s += ax * ax + ay * ay;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    finish_blocks<false>(red[0], partial, out, ticket);
}

// max over owned entries of [acnorm_j == 0] (MINPACK's rank test, nsing < n).
__global__ void __launch_bounds__(256) k_zero_flag(const double *__restrict__ acnorm, int n,
                                                   const int *__restrict__ mask,
                                                   double *partial, double *out,
                                                   unsigned int *ticket) {
    __shared__ double red[256];
    double m = 0.;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        if (own_mask(mask, i) && acnorm[i] == 0.) m = 1.;
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    finish_blocks<true>(red[0], partial, out, ticket);
}

// Keep this shard's reduced-system rows [lo, hi) (and the global rows on the
// root shard) before the rows are summed across shards.
__global__ void k_keep_rows(double *v, int lo, int hi, int nCF, int nR, int root) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nR) return;
    const bool keep = (r >= nCF) ? root != 0 : (r >= lo && r < hi);
    if (!keep) v[r] = 0.;
}

// dst = mask ? src : 0
__global__ void k_keep_mask(const double *__restrict__ src, const int *__restrict__ mask, int n,
                            double *dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = own_mask(mask, i) ? src[i] : 0.;
}

// Elementwise LM vector updates.
__global__ void k_lm_step(int n, const double *__restrict__ xs, const double *__restrict__ x,
                          const double *__restrict__ diag, double *wa1, double *wa2,
                          double *wa3) {
    // wa1 = -xs (step), wa2 = x + wa1, wa3 = diag * wa1
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const double s = -xs[j];
    wa1[j] = s;
    wa2[j] = x[j] + s;
    wa3[j] = diag[j] * s;
}

__global__ void k_diag_init(int n, const double *__restrict__ acnorm, double *diag, int first,
                            int mode) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (first && mode != 2) diag[j] = acnorm[j] == 0. ? 1. : acnorm[j];
    if (mode != 2) diag[j] = fmax(diag[j], acnorm[j]);
}

__global__ void k_newton_v(int n, const double *__restrict__ diag, const double *__restrict__ x,
                           double dxnorm, double *v) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    v[j] = diag[j] * ((diag[j] * x[j]) / dxnorm);
}

// Device order -> reference (errorToMarkerList) order.
__global__ void k_unpermute(int M, const int *__restrict__ ref_of_dev,
                            const int *__restrict__ obs_own,
                            const double *__restrict__ f2, const double *__restrict__ eu2,
                            const double *__restrict__ ed, double *f2o, double *eu2o,
                            double *edo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M || (obs_own && !obs_own[i])) return;
    const int r = ref_of_dev[i];
    if (f2) {
        f2o[2 * r] = f2[2 * i];
        f2o[2 * r + 1] = f2[2 * i + 1];
    }
    if (eu2) {
        eu2o[2 * r] = eu2[2 * i];
        eu2o[2 * r + 1] = eu2[2 * i + 1];
    }
    if (ed) edo[r] = ed[i];
}

// Unsharded hand-back straight into the caller's page-locked lists (their
// host-mapped addresses): thread r takes reference position r, gathers
// device position dev_of_ref[r] and stores 16 + 16 + 8 B, so consecutive
// threads write consecutive host bytes (full PCIe write requests); positions
// [Mg, Mg + nrows) copy the stiffness / smoothness rows that follow the
// observations in errorList / ud->errorList.  One launch replaces k_unpermute
// and the three DMA copies (tools/ubench/d2h: 163 against 192 us for C2's
// 8 MB).
// dec (the speculative form, enqueued behind a trial on its own stream):
// the device's LM decision on that trial (LmDec slots from SL_DGO: [1] the
// ratio, [4] info when the trial was taken) -- the lists are stored only when
// the solve ends on it (info > 0), errorList from the trial's f when lmder
// accepts it (ratio >= 1e-4, lm_decide) and from the accepted f otherwise.
__global__ void __launch_bounds__(256) k_handback_host(int Mg, int nrows,
                                                       const int *__restrict__ dev_of_ref,
                                                       const double *__restrict__ f2,
                                                       const double *__restrict__ eu2,
                                                       const double *__restrict__ ed,
                                                       double *hf, double *heu, double *hed,
                                                       const double *__restrict__ dec,
                                                       const double *__restrict__ f2_trial) {
    if (dec) {
        if (!(dec[4] > 0.)) return;
        if (dec[1] >= 1e-4) f2 = f2_trial;
    }
    const int stride = gridDim.x * blockDim.x;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < Mg + nrows; r += stride) {
        if (r < Mg) {
            const int d = dev_of_ref[r];
            if (hf) reinterpret_cast<double2 *>(hf)[r] = reinterpret_cast<const double2 *>(f2)[d];
            if (heu)
                reinterpret_cast<double2 *>(heu)[r] = reinterpret_cast<const double2 *>(eu2)[d];
            if (hed) hed[r] = ed[d];
        } else {
            const int k = r - Mg;  // rows: device and reference order agree
            if (hf) hf[2 * (size_t)Mg + k] = f2[2 * (size_t)Mg + k];
            if (heu) heu[2 * (size_t)Mg + k] = eu2[2 * (size_t)Mg + k];
        }
    }
}

}  // namespace mmba

// =========================================================================
// Host launch wrappers (declared in mmba_kernels.h).
// =========================================================================
namespace mmba {

static inline int nblk(long n, int bs) { return (int)((n + bs - 1) / bs); }
bool trial_records_ok(const DevProblem &P) {
    return P.nG == 0 && P.cf_aidx != nullptr && !P.rs && P.ncf > 0;
}

int trial_prep_rec_parts(const DevProblem &P, int nother) {
    return (P.ncf + 3) / 4 + nblk(nother, 64);
}
void launch_trial_prep_rec(hipStream_t s, const DevProblem &P, const double *xs, const TrialFold &T) {
    k_trial_prep_rec<<<trial_prep_rec_parts(P, T.nother), 64, 0, s>>>(P, xs, (P.ncf + 3) / 4, T);
}
int trial_fold_parts(const DevProblem &P, int nother, bool rec) {
    return nblk(P.nB, 64) + (rec ? (P.ncf + 3) / 4 : nblk(nother, 64));
}

void launch_backsub_trial(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                          const double *tb, const double *Lb, const double *xR, const double *U,
                          double *x, const TrialFold &T) {
    const int nbb = nblk(P.nB, 64);
    const int g = trial_fold_parts(P, T.nother, T.rec != 0);
    if (g > 0) k_backsub_trial<<<g, 64, 0, s>>>(P, U, W, Wg, tb, Lb, xR, x, nbb, T);
}

void launch_obs_wtx(hipStream_t s, const DevProblem &P, const double *W, const double *xR,
                    double *U) {
    if (P.nB == 0) return;
    k_obs_wtx<<<nblk(P.M, 64), 64, sizeof(double) * 64 * P.wst, s>>>(P, W, xR, U);
}

void launch_param_prep(hipStream_t s, const DevProblem &P, const double *x, double *ext,
                       double *ext_pert, double *step, int solver_type, double delta,
                       double eps_dif) {
    if (P.n == 0) return;
    k_param_prep<<<nblk(P.n, 256), 256, 0, s>>>(P, x, ext, ext_pert, step, solver_type, delta,
                                                 eps_dif);
}
void launch_records(hipStream_t s, const DevProblem &P, const int *var_cf,
                    const double *ext_pert, const double *step, double *recs, int nvar,
                    double *brec, int base_only) {
    const int ncb = (nblk(base_only ? P.ncf : nvar, 64) + 7) / 8 * 8;  // see k_records
    const int nbb = nblk(P.nB, 64);
    if (ncb + nbb > 0)
        k_records<<<ncb + nbb, 64, 0, s>>>(P, var_cf, ext_pert, step, recs, nvar, brec, base_only,
                                           ncb);
}
void launch_param_set(hipStream_t s, const DevProblem &P, const double *x, double *ext,
                      double *ext_pert, double *step, int solver_type, double delta,
                      double eps_dif) {
    if (P.n == 0) return;
    k_param_set<<<nblk(P.n, 256), 256, 0, s>>>(P, x, ext, ext_pert, step, solver_type, delta,
                                                eps_dif);
}
void launch_jac_epilogue(hipStream_t s, const DevProblem &P, const double *Acc,
                         const double *Abb, const double *aggbuf, double *acnorm, double *g,
                         double *diag, const double *x, int first, int mode, double fnorm,
                         const double *fnorm_sq, int do_xn, int do_gn, const int *mask,
                         double *partial, int nparts, int rstride, const double *c15,
                         const double *s15, double *gfull, const double *adiag15,
                         const double *u15) {
    k_jac_epilogue<<<nparts, 256, 0, s>>>(P, Acc, Abb, aggbuf, aggbuf + NGMAX * NGMAX, acnorm,
                                          g, diag, x, first, mode, fnorm, fnorm_sq, do_xn, do_gn,
                                          mask, partial, rstride, c15, s15, gfull, adiag15, u15);
}
void launch_trial_prep(hipStream_t s, const DevProblem &P, const double *xs, const double *x,
                       const double *diag, double *wa1, double *wa2, double *wa3, double *ext,
                       double *ext_pert, double *step, int solver_type, double delta,
                       double eps_dif, const int *mask, double *partial, int nparts,
                       int rstride) {
    k_trial_prep<<<nparts, 256, 0, s>>>(P, xs, x, diag, wa1, wa2, wa3, ext, ext_pert, step,
                                        solver_type, delta, eps_dif, mask, partial, rstride);
}
void launch_reduce_multi(hipStream_t s, const double *partial, const RedSpec &spec,
                         double *scalar, int *flag, double *host, int host_n, unsigned *ticket,
                         unsigned *host_seq, unsigned seq, const LmDec &dec) {
    if (spec.nrows > 0)
        k_reduce_multi<<<spec.nrows, 256, 0, s>>>(partial, spec, scalar, flag, host, host_n,
                                                   ticket, host_seq, seq, dec);
}
void launch_set_attrs(hipStream_t s, const DevProblem &P, const double *ext) {
    k_set_attrs<<<nblk(P.n, 256), 256, 0, s>>>(P, ext);
}
// Partial sums of a residual evaluation: one per 256 observations, plus one
// for the attribute rows (k_rows_eval writes entry nblk(M, 256)).
int residual_blocks(const DevProblem &P) { return nblk(P.M, 256) + (P.nrows > 0 ? 1 : 0); }
// The trial point's residual pass runs per camera-frame (k_residual_jp_cf)
// on the uniform fast plans of the fused K2: no attribute rows, no lens, no
// rolling shutter, implicit Jacobian columns.
bool trial_cf_fusable(const DevProblem &P) {
    return jac_ne_fusable(P, P.pc_uniform) && P.all_bnd_fast && P.no_lens && P.jcol_implicit &&
           !trial_cf_off();
}
bool &trial_cf_off() {  // the per-256-observation kernel instead (tests set it)
    static bool off = false;
    return off;
}
int trial_blocks(const DevProblem &P) { return trial_cf_fusable(P) ? P.ncf : residual_blocks(P); }
void launch_residual(hipStream_t s, const DevProblem &P, const double *recs, double *f, double *eu,
                     double *ed, double *partial, double *out, unsigned int *ticket, double *dist) {
    // the ticket epilogue sums the residual kernel's own nblk(M) partials
    // only: with stiffness / smoothness rows (one more partial, k_rows_eval)
    // the two-launch reduction runs
    if (ticket && residual_blocks(P) != nblk(P.M, 256)) ticket = nullptr;
    if (P.rs)
        k_residual<false, false, true><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, out, ticket, nullptr, nullptr, nullptr, nullptr, nullptr,
            dist, RedTail());
    else if (P.all_bnd_fast && P.no_lens)
        k_residual<false, true><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, out, ticket, nullptr, nullptr, nullptr, nullptr, nullptr,
            dist, RedTail());
    else
        k_residual<false, false><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, out, ticket, nullptr, nullptr, nullptr, nullptr, nullptr,
            dist, RedTail());
    if (!ticket && out) k_reduce_sum<<<1, 256, 0, s>>>(partial, residual_blocks(P), out);
}
// Per-observation reprojection (FlatScene::evaluate's out_point_list /
// out_marker_list, the pair measureErrors compares): the lens-distorted point
// and the film-fit corrected marker, device order.  Records must be current.
__global__ void __launch_bounds__(256) k_reproject(DevProblem P, const double *__restrict__ recs,
                                                   double *pts, double *mkr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.M) return;
    const int cf = P.obs_cf[i], b = P.obs_bnd[i], fr = P.obs_frame[i];
    const Override none{-1, 0.};
    double bp[3];
    base_bundle(P, b, fr, bp);
    double lc[MMBA_LENS_NUM_ATTRS];
    int inst = -1;
    const int hl = obs_lens_inst(P, i, inst);
    if (hl) inst_coeffs(P, inst, none, lc);
    const double *rec = &recs[(size_t)P.cf_var_off[cf] * CAMREC];
    double rloc[CAMREC];
    if (P.rs) {  // this observation's scanline pose
        camera_record_rs(P, cf, P.obs_tau[i], -1, 0., rloc);
        rec = rloc;
    }
    double px, py;
    project_point(rec, bp, px, py);
    distort_point(hl, lc, px, py, P.lens_chain, P.lens_chain_n);
    pts[2 * i] = px;
    pts[2 * i + 1] = py;
    mkr[2 * i] = P.obs_xy[2 * i] * rec[18];
    mkr[2 * i + 1] = P.obs_xy[2 * i + 1] * rec[19];
}
void launch_reproject(hipStream_t s, const DevProblem &P, const double *recs, double *pts,
                      double *mkr) {
    if (P.M > 0) k_reproject<<<nblk(P.M, 256), 256, 0, s>>>(P, recs, pts, mkr);
}
void launch_residual_jp(hipStream_t s, const DevProblem &P, const double *recs, double *f,
                        double *eu, double *ed, double *partial, const double *J,
                        const int *jcol, const int *nloc, const double *pstep,
                        double *partial_jp, double *dist, const RedTail &T) {
    if (!T.on && trial_cf_fusable(P)) {  // partials per camera-frame (trial_blocks)
        if (P.pc_uniform == 6)
            k_residual_jp_cf<6><<<P.ncf, 256, 0, s>>>(P, recs, f, eu, ed, partial, J, nloc, pstep,
                                                      partial_jp, dist);
        else
            k_residual_jp_cf<7><<<P.ncf, 256, 0, s>>>(P, recs, f, eu, ed, partial, J, nloc, pstep,
                                                      partial_jp, dist);
        return;
    }
    if (P.rs)
        k_residual<true, false, true><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, nullptr, nullptr, J, jcol, nloc, pstep, partial_jp, dist, T);
    else if (P.all_bnd_fast && P.no_lens)
        k_residual<true, true><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, nullptr, nullptr, J, jcol, nloc, pstep, partial_jp, dist, T);
    else
        k_residual<true, false><<<nblk(P.M, 256), 256, 0, s>>>(
            P, recs, f, eu, ed, partial, nullptr, nullptr, J, jcol, nloc, pstep, partial_jp, dist, T);
}

// compute_error_stats (adjust_base.cpp:346-372) on the device: per block the
// sum, minimum and maximum of the finite entries of errorDistanceList (own
// observations) -> partial rows 0 / 1 / 2 (1 holds -min so every row folds
// with max or sum); k_dist_stats_fin folds them into out[0..2] = sum, -min,
// max.  The average is sum / M over every observation, as the reference
// divides by the marker-error count.
__global__ void __launch_bounds__(256) k_dist_stats(DevProblem P, const double *__restrict__ ed,
                                                    double *partial, int rstride) {
    __shared__ double red[3][256];
    double sm = 0., nmn = -DBL_MAX, mx = -0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P.M; i += gridDim.x * blockDim.x) {
        if (!own_obs(P, i)) continue;
        const double e = ed[i];
        if (!isfinite(e)) continue;
        sm += e;
        nmn = fmax(nmn, -e);
        mx = fmax(mx, e);
    }
    red[0][threadIdx.x] = sm;
    red[1][threadIdx.x] = nmn;
    red[2][threadIdx.x] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[0][threadIdx.x] += red[0][threadIdx.x + w];
            red[1][threadIdx.x] = fmax(red[1][threadIdx.x], red[1][threadIdx.x + w]);
            red[2][threadIdx.x] = fmax(red[2][threadIdx.x], red[2][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = red[0][0];
        partial[rstride + blockIdx.x] = red[1][0];
        partial[2 * rstride + blockIdx.x] = red[2][0];
    }
}

__global__ void __launch_bounds__(256) k_dist_stats_fin(const double *__restrict__ partial,
                                                        int n, int rstride, double *out) {
    __shared__ double red[3][256];
    double sm = 0., nmn = -DBL_MAX, mx = -0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        sm += partial[i];
        nmn = fmax(nmn, partial[rstride + i]);
        mx = fmax(mx, partial[2 * rstride + i]);
    }
    red[0][threadIdx.x] = sm;
    red[1][threadIdx.x] = nmn;
    red[2][threadIdx.x] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[0][threadIdx.x] += red[0][threadIdx.x + w];
            red[1][threadIdx.x] = fmax(red[1][threadIdx.x], red[1][threadIdx.x + w]);
            red[2][threadIdx.x] = fmax(red[2][threadIdx.x], red[2][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = red[0][0];
        out[1] = red[1][0];
        out[2] = red[2][0];
    }
}

void launch_dist_stats(hipStream_t s, const DevProblem &P, const double *ed, double *partial,
                       int nparts, int rstride, double *out) {
    k_dist_stats<<<nparts, 256, 0, s>>>(P, ed, partial, rstride);
    k_dist_stats_fin<<<1, 256, 0, s>>>(partial, nparts, rstride, out);
}
void launch_jacobian(hipStream_t s, const DevProblem &P, const double *recs,
                     const double *ext_pert, const double *step, int solver_type, double *J,
                     int *jcol, int *nloc, const int *stale_param, double *eu, double *ed,
                     int ncv, const double *f, const CentralB &CB) {
    (void)f;
    if (P.rs) {  // rolling shutter: three camera-frame blocks per row (mmba_rs.hip)
        launch_jacobian_rs(s, P, ext_pert, step, solver_type, J, jcol, nloc, stale_param, eu, ed);
        return;
    }
    // wave-uniform record loads (per-lane loads only: measured slower)
    constexpr bool uni = true;
#define MMBA_JAC_U(NCV, GEN)                                                                \
    do {                                                                                    \
        if (uni)                                                                            \
            k_jacobian_u<NCV, GEN, true><<<nblk(P.M, 128), 128, 0, s>>>(                    \
                P, recs, step, solver_type, J, jcol, nloc, stale_param, eu, ed);            \
        else                                                                                \
            k_jacobian_u<NCV, GEN, false><<<nblk(P.M, 128), 128, 0, s>>>(                   \
                P, recs, step, solver_type, J, jcol, nloc, stale_param, eu, ed);            \
    } while (0)
    if (ncv == 6 || ncv == 7) {
        if (ncv == 6) {
            if (P.all_bnd_fast) MMBA_JAC_U(6, false); else MMBA_JAC_U(6, true);
        } else {
            if (P.all_bnd_fast) MMBA_JAC_U(7, false); else MMBA_JAC_U(7, true);
        }
        return;
    }
#undef MMBA_JAC_U
    if (CB.recs)
        k_jacobian<true><<<nblk(P.M, 128), 128, 0, s>>>(P, recs, ext_pert, step, solver_type, J,
                                                      jcol, nloc, stale_param, eu, ed, CB);
    else if (P.lens_uniform == MMBA_LENS_3DE_CLASSIC)  // C5: the classic model only
        k_jacobian<false, MMBA_LENS_3DE_CLASSIC><<<nblk(P.M, 128), 128, 0, s>>>(
            P, recs, ext_pert, step, solver_type, J, jcol, nloc, stale_param, eu, ed, CB);
    else
        k_jacobian<false><<<nblk(P.M, 128), 128, 0, s>>>(P, recs, ext_pert, step, solver_type, J,
                                                       jcol, nloc, stale_param, eu, ed, CB);
}
// One workgroup per camera-frame only fills the chip with enough
// camera-frames (C4: 500 x 400 observations); a few long segments (C2: 120 x
// 1,650) keep the split passes, whose Jacobian kernel spreads every
// observation over the whole GPU.
bool jac_ne_fusable(const DevProblem &P, int ncv) {
    return P.nG == 0 && P.pc_uniform == ncv && (ncv == 6 || ncv == 7) &&
           P.nrows == 0 && !P.loss_on && P.ncf >= 256 && !P.rs;
}
void launch_jac_ne(hipStream_t s, const DevProblem &P, const double *recs, const double *step,
                   int solver_type, double *J, int *jcol, int *nloc, const int *stale_param,
                   double *eu, double *ed, double *Acc, double *g, const NeEpi &E) {
    if (P.ncf == 0) return;
    // the 232-VGPR kernel runs 2 waves per SIMD, so 4-wave workgroups fill
    // the chip with C4's 500 segments in one round (400 observations per
    // segment: 2 waves 41.7 us, 4 waves 34.6 us, 8 waves 45.7 us)
    const long long per = (P.M + P.ncf - 1) / P.ncf;
    int nw = per > 1024 ? 8 : (per > 256 ? 4 : 2);
#define MMBA_JN(PC, NW, GEN)                                                                  \
    k_jac_ne_u<PC, NW, GEN><<<P.ncf, 64 * NW, 0, s>>>(P, recs, step, solver_type, J, jcol, nloc, \
                                                        stale_param, eu, ed, Acc, g, E)
#define MMBA_JN_NW(PC, GEN)                                         \
    do {                                                            \
        if (nw == 8) MMBA_JN(PC, 8, GEN);                           \
        else if (nw == 4) MMBA_JN(PC, 4, GEN);                      \
        else MMBA_JN(PC, 2, GEN);                                   \
    } while (0)
#define MMBA_JN_PC(PC)                                              \
    do {                                                            \
        if (P.all_bnd_fast) MMBA_JN_NW(PC, false);                  \
        else MMBA_JN_NW(PC, true);                                  \
    } while (0)
    if (P.pc_uniform == 6)
        MMBA_JN_PC(6);
    else
        MMBA_JN_PC(7);
#undef MMBA_JN_PC
#undef MMBA_JN_NW
#undef MMBA_JN
}
// [ZERO, XN2, gnorm_0 .. gnorm_{n-1}] after the sum all-reduce -> the
// ZERO / XN2 / GNORM slots (gnorm = max over ranks)
__global__ void k_fold_ranks(const double *__restrict__ t, int nranks, double *out, int do_xn,
                             int do_gn) {
    if (threadIdx.x != 0) return;
    out[0] = t[0];
    if (do_xn) out[1] = t[1];
    if (do_gn) {
        double g = 0.;
        for (int r = 0; r < nranks; ++r) g = fmax(g, t[2 + r]);
        out[2] = g;
    }
}
void launch_fold_ranks(hipStream_t s, const double *t, int nranks, double *out, int do_xn,
                       int do_gn) {
    k_fold_ranks<<<1, 64, 0, s>>>(t, nranks, out, do_xn, do_gn);
}
void launch_param_central(hipStream_t s, const DevProblem &P, const double *x, double *ext_pertB,
                          double *stepB, double delta, double *count, double *c15) {
    if (P.n > 0)
        k_param_central<<<nblk(P.n, 256), 256, 0, s>>>(P, x, ext_pertB, stepB, delta, count,
                                                        c15);
}

// ---------------------------------------------------------------------------
// B15: the reference's central Jacobian of animated parameters over several
// frames is J = J_s + f c^T (Plan::b15).  Its normal matrix is
// A = M + U B U^T with M = J_s^T J_s (+ lam D^2), U = [u c], u = J_s^T f,
// B = [0 1; 1 s], s = ||f||^2, and J^T f = u + s c.  One workgroup per call,
// fixed-order sums (bit-reproducible); the vectors are n long.
// ---------------------------------------------------------------------------
template <int NV>
__device__ __forceinline__ void b15_block_sum(double (&v)[NV], double (*red)[1024]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NV; ++k) red[k][tid] = v[k];
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (tid < w) {
#pragma unroll
            for (int k = 0; k < NV; ++k) red[k][tid] += red[k][tid + w];
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = red[k][0];
    __syncthreads();
}

__global__ void k_b15_s(const double *fsq, double fn, double *out) {
    if (threadIdx.x == 0) *out = fsq ? *fsq : fn * fn;
}

__global__ void __launch_bounds__(1024) k_b15_combine(
    int n, const double *__restrict__ u, const double *__restrict__ c,
    const double *__restrict__ zu, const double *__restrict__ zc, const double *__restrict__ sp,
    double *xs, double *kinv, double *scalar, int fail_slot, const double *__restrict__ fail_prev) {
    __shared__ double red[4][1024];
    double d[4] = {0., 0., 0., 0.};
    for (int j = threadIdx.x; j < n; j += 1024) {
        d[0] += u[j] * zu[j];
        d[1] += u[j] * zc[j];
        d[2] += c[j] * zu[j];
        d[3] += c[j] * zc[j];
    }
    b15_block_sum<4>(d, red);
    const double s = *sp;
    // K = B^-1 + U^T M^-1 U, B^-1 = [-s 1; 1 0]
    const double k00 = d[0] - s, k01 = 1. + d[1], k10 = 1. + d[2], k11 = d[3];
    const double det = k00 * k11 - k01 * k10;
    const bool sing = !(fabs(det) > 0.) || !isfinite(det);
    const double i00 = k11 / det, i01 = -k01 / det, i10 = -k10 / det, i11 = k00 / det;
    // U^T M^-1 g, g = u + s c, M^-1 g = z_u + s z_c
    const double r0 = d[0] + s * d[1], r1 = d[2] + s * d[3];
    const double al = i00 * r0 + i01 * r1, be = i10 * r0 + i11 * r1;
    const double cu = 1. - al, cc = s - be;
    for (int j = threadIdx.x; j < n; j += 1024) xs[j] = cu * zu[j] + cc * zc[j];
    if (threadIdx.x == 0) {
        kinv[0] = i00;
        kinv[1] = i01;
        kinv[2] = i10;
        kinv[3] = i11;
        double f = fmax(scalar[fail_slot], *fail_prev);
        if (sing) f = fmax(f, 1.);
        scalar[fail_slot] = f;
    }
}

__global__ void __launch_bounds__(1024) k_b15_newton(int n, const double *__restrict__ v,
                                                     const double *__restrict__ zu,
                                                     const double *__restrict__ zc,
                                                     const double *__restrict__ kinv, double *out) {
    __shared__ double red[2][1024];
    double w[2] = {0., 0.};
    for (int j = threadIdx.x; j < n; j += 1024) {
        w[0] += zu[j] * v[j];
        w[1] += zc[j] * v[j];
    }
    b15_block_sum<2>(w, red);
    if (threadIdx.x == 0)
        *out -= w[0] * (kinv[0] * w[0] + kinv[1] * w[1]) + w[1] * (kinv[2] * w[0] + kinv[3] * w[1]);
}

__global__ void __launch_bounds__(1024) k_b15_jp(int n, const double *__restrict__ xs,
                                                 const double *__restrict__ u,
                                                 const double *__restrict__ c,
                                                 const double *__restrict__ sp, double *out) {
    __shared__ double red[2][1024];
    double w[2] = {0., 0.};
    for (int j = threadIdx.x; j < n; j += 1024) {
        w[0] += c[j] * xs[j];
        w[1] += u[j] * xs[j];
    }
    b15_block_sum<2>(w, red);
    if (threadIdx.x == 0) *out += 2. * w[0] * w[1] + *sp * w[0] * w[0];
}

void launch_b15_s(hipStream_t s, const double *fsq, double fn, double *out) {
    k_b15_s<<<1, 64, 0, s>>>(fsq, fn, out);
}
void launch_b15_combine(hipStream_t s, int n, const double *u, const double *c, const double *zu,
                        const double *zc, const double *sp, double *xs, double *kinv,
                        double *scalar, int fail_slot, const double *fail_prev) {
    k_b15_combine<<<1, 1024, 0, s>>>(n, u, c, zu, zc, sp, xs, kinv, scalar, fail_slot, fail_prev);
}

// Q_cf = I - beta v v^T with v = c_cf + sign(c_0) |c_cf| e_0 (Householder:
// Q c_cf = kappa e_0, kappa = -sign(c_0) |c_cf|; Q = I where c_cf = 0), and
// c in that basis (kappa at the block's first parameter, 0 elsewhere).
__global__ void k_b15_q(DevProblem P, const double *__restrict__ c, double *q15, double *kap15,
                        double *cr) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < P.n) {
        double v = c[t];
        if (P.p_class[t] == PC_CF) {  // kappa at the block's first parameter, else 0
            const int cf = P.p_blk[t], pc = P.cf_pc[cf], voff = P.cf_var_off[cf];
            v = 0.;
            if (P.p_pos[t] == P.cf_roff[cf]) {
                double n2 = 0.;
                for (int a = 0; a < pc; ++a) {
                    const double ca = c[P.cf_var_param[voff + 1 + a]];
                    n2 += ca * ca;
                }
                if (n2 > 0.) v = (c[t] < 0. ? 1. : -1.) * sqrt(n2);
            }
        }
        cr[t] = v;
    }
    if (t >= P.ncf) return;
    const int cf = t, pc = P.cf_pc[cf], voff = P.cf_var_off[cf];
    double v[PCMAX];
    double nrm2 = 0.;
#pragma unroll
    for (int a = 0; a < PCMAX; ++a) {
        v[a] = a < pc ? c[P.cf_var_param[voff + 1 + a]] : 0.;
        nrm2 += v[a] * v[a];
    }
    double *Q = q15 + (size_t)cf * PCMAX * PCMAX;
    double kap = 0.;
    if (nrm2 > 0.) {
        const double nrm = sqrt(nrm2), sg = v[0] < 0. ? -1. : 1.;
        kap = -sg * nrm;
        v[0] += sg * nrm;
        double vv = 0.;
#pragma unroll
        for (int a = 0; a < PCMAX; ++a) vv += v[a] * v[a];
        const double beta = 2. / vv;
#pragma unroll
        for (int a = 0; a < PCMAX; ++a)
#pragma unroll
            for (int b = 0; b < PCMAX; ++b) Q[a * PCMAX + b] = (a == b ? 1. : 0.) - beta * v[a] * v[b];
    } else {
#pragma unroll
        for (int a = 0; a < PCMAX; ++a)
#pragma unroll
            for (int b = 0; b < PCMAX; ++b) Q[a * PCMAX + b] = a == b ? 1. : 0.;
    }
    kap15[cf] = kap;
}

// out = Q x per camera-frame block (Q symmetric orthogonal: its own inverse),
// other parameters copied
__global__ void k_b15_rot(DevProblem P, const double *__restrict__ q15,
                          const double *__restrict__ x, double *out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    if (P.p_class[p] != PC_CF) {
        out[p] = x[p];
        return;
    }
    const int cf = P.p_blk[p], a = P.p_pos[p] - P.cf_roff[cf];
    const int pc = P.cf_pc[cf], voff = P.cf_var_off[cf];
    const double *Q = q15 + (size_t)cf * PCMAX * PCMAX + a * PCMAX;
    double acc = 0.;
    for (int b = 0; b < pc; ++b) acc = fma(Q[b], x[P.cf_var_param[voff + 1 + b]], acc);
    out[p] = acc;
}

// Damped block of the rotated system: AccL = Acc + lam Q D^2 Q per camera-frame
// (the solve then adds nothing there: diagL = 0 on camera-frame parameters)
__global__ void k_b15_accl(DevProblem P, const double *__restrict__ Acc,
                           const double *__restrict__ q15, const double *__restrict__ diag,
                           double lam, double *AccL, double *diagL) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < P.n) diagL[t] = P.p_class[t] == PC_CF ? 0. : diag[t];
    if (t >= P.ncf) return;
    const int cf = t, pc = P.cf_pc[cf], voff = P.cf_var_off[cf];
    const double *Q = q15 + (size_t)cf * PCMAX * PCMAX;
    const double *A = Acc + (size_t)cf * PCMAX * PCMAX;
    double *AL = AccL + (size_t)cf * PCMAX * PCMAX;
    double d2[PCMAX];
    for (int k = 0; k < pc; ++k) {
        const double d = diag[P.cf_var_param[voff + 1 + k]];
        d2[k] = d * d;
    }
    for (int a = 0; a < PCMAX; ++a)
        for (int b = 0; b < PCMAX; ++b) {
            double v = A[a * PCMAX + b];
            if (a < pc && b < pc) {
                double w = 0.;
                for (int k = 0; k < pc; ++k) w = fma(Q[k * PCMAX + a] * d2[k], Q[k * PCMAX + b], w);
                v += lam * w;
            }
            AL[a * PCMAX + b] = v;
        }
}

// The camera-frame parameters' A_pp and u_p in the original basis:
// diag(Q A Q), Q u (epilogue of a rotated Jacobian)
__global__ void k_b15_unrot(DevProblem P, const double *__restrict__ Acc,
                            const double *__restrict__ g, const double *__restrict__ q15,
                            double *adiag, double *u) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.n) return;
    if (P.p_class[p] != PC_CF) {
        u[p] = g[p];
        adiag[p] = 0.;
        return;
    }
    const int cf = P.p_blk[p], a = P.p_pos[p] - P.cf_roff[cf];
    const int pc = P.cf_pc[cf], voff = P.cf_var_off[cf];
    const double *Q = q15 + (size_t)cf * PCMAX * PCMAX + a * PCMAX;
    const double *A = Acc + (size_t)cf * PCMAX * PCMAX;
    double ua = 0., da = 0.;
    for (int k = 0; k < pc; ++k) {
        ua = fma(Q[k], g[P.cf_var_param[voff + 1 + k]], ua);
        double r = 0.;
        for (int l = 0; l < pc; ++l) {
            const int hi = k > l ? k : l, lo = k > l ? l : k;  // lower triangle
            r = fma(A[hi * PCMAX + lo], Q[l], r);
        }
        da = fma(Q[k], r, da);
    }
    u[p] = ua;
    adiag[p] = da;
}

// Dense-Jacobian readback of a rotated J: the camera-frame block's first pc
// columns back to the original basis (J_s = (J_s Q) Q)
__global__ void k_b15_unrot_J(DevProblem P, double *J, const double *__restrict__ q15) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.M) return;
    const int M = P.M, cf = P.obs_cf[i], pc = P.cf_pc[cf];
    const double *Q = q15 + (size_t)cf * PCMAX * PCMAX;
    double ax[PCMAX], ay[PCMAX];
#pragma unroll
    for (int a = 0; a < PCMAX; ++a) {
        ax[a] = a < pc ? J[(size_t)(2 * a) * M + i] : 0.;
        ay[a] = a < pc ? J[(size_t)(2 * a + 1) * M + i] : 0.;
    }
#pragma unroll
    for (int a2 = 0; a2 < PCMAX; ++a2) {
        if (a2 >= pc) break;
        double sx = 0., sy = 0.;
#pragma unroll
        for (int a = 0; a < PCMAX; ++a) {
            sx = fma(ax[a], Q[a * PCMAX + a2], sx);
            sy = fma(ay[a], Q[a * PCMAX + a2], sy);
        }
        J[(size_t)(2 * a2) * M + i] = sx;
        J[(size_t)(2 * a2 + 1) * M + i] = sy;
    }
}

__global__ void __launch_bounds__(1024) k_b15_dnorm(int n, const double *__restrict__ x,
                                                    const double *__restrict__ diag, double *out) {
    __shared__ double red[1][1024];
    double v[1] = {0.};
    for (int j = threadIdx.x; j < n; j += 1024) {
        const double w = diag[j] * x[j];
        v[0] += w * w;
    }
    b15_block_sum<1>(v, red);
    if (threadIdx.x == 0) *out = v[0];
}

void launch_b15_q(hipStream_t s, const DevProblem &P, const double *c, double *q15, double *kap15,
                  double *cr) {
    const int nt = P.n > P.ncf ? P.n : P.ncf;
    if (nt > 0) k_b15_q<<<nblk(nt, 256), 256, 0, s>>>(P, c, q15, kap15, cr);
}
void launch_b15_rot(hipStream_t s, const DevProblem &P, const double *q15, const double *x,
                    double *out) {
    if (P.n > 0) k_b15_rot<<<nblk(P.n, 256), 256, 0, s>>>(P, q15, x, out);
}
void launch_b15_accl(hipStream_t s, const DevProblem &P, const double *Acc, const double *q15,
                     const double *diag, double lam, double *AccL, double *diagL) {
    const int nt = P.n > P.ncf ? P.n : P.ncf;
    if (nt > 0) k_b15_accl<<<nblk(nt, 256), 256, 0, s>>>(P, Acc, q15, diag, lam, AccL, diagL);
}
void launch_b15_unrot(hipStream_t s, const DevProblem &P, const double *Acc, const double *g,
                      const double *q15, double *adiag, double *u) {
    if (P.n > 0) k_b15_unrot<<<nblk(P.n, 256), 256, 0, s>>>(P, Acc, g, q15, adiag, u);
}
void launch_b15_unrot_J(hipStream_t s, const DevProblem &P, double *J, const double *q15) {
    if (P.M > 0) k_b15_unrot_J<<<nblk(P.M, 128), 128, 0, s>>>(P, J, q15);
}
void launch_b15_dnorm(hipStream_t s, int n, const double *x, const double *diag, double *out) {
    k_b15_dnorm<<<1, 1024, 0, s>>>(n, x, diag, out);
}
void launch_b15_newton(hipStream_t s, int n, const double *v, const double *zu, const double *zc,
                       const double *kinv, double *out) {
    k_b15_newton<<<1, 1024, 0, s>>>(n, v, zu, zc, kinv, out);
}
void launch_b15_jp(hipStream_t s, int n, const double *xs, const double *u, const double *c,
                   const double *sp, double *out) {
    k_b15_jp<<<1, 1024, 0, s>>>(n, xs, u, c, sp, out);
}
bool ne_epilogue_fusable(const DevProblem &P) {
    return P.nG == 0 && (P.JB || P.nbs == 0) && (P.pc_uniform == 6 || P.pc_uniform == 7) &&
           !P.rs;
}
void launch_ne(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
               const int *nloc, const double *f, double *Acc, double *Acg, double *Abb,
               double *Abg, double *aggbuf, double *g, double *glob_partial, int glob_chunk,
               const NeEpi &epi, bool cf_done) {
    const NeEpi E = ne_epilogue_fusable(P) ? epi : NeEpi();
    double *Agg = aggbuf, *gG = aggbuf + NGMAX * NGMAX;
    bool glob_done = false;  // the global chunks ran in the camera-frame launch
    if (P.rs) {  // coupled camera-frame blocks (mmba_rs.hip)
        launch_ne_rs(s, P, J, jcol, nloc, f, Acc, Acg, g);
    } else if (P.ncf > 0 && !cf_done) {
        // long camera-frame segments (C2), or segments of a few hundred
        // observations on fewer camera-frames than SIMDs (C5): 4 waves each
        const bool wide = P.M > 1024 * P.ncf || (P.M > 128 * P.ncf && P.ncf < 1024);
#define MMBA_NE_U(PC, NW, NG)                                                              \
    k_ne_cf_u<PC, NW, NG><<<P.ncf, 64 * NW, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, E)
        const int pcu = P.pc_uniform;
        if ((pcu == 6 || pcu == 7) && wide && P.nG > 0 && P.nG <= 2) {
            // camera-frame blocks and global chunks in one launch
            const int nbg = nblk(P.M, glob_chunk);
            if (pcu == 6)
                k_ne_cf_glob<6><<<P.ncf + nbg, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, E,
                                                           glob_partial, glob_chunk);
            else
                k_ne_cf_glob<7><<<P.ncf + nbg, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, E,
                                                           glob_partial, glob_chunk);
            glob_done = true;
        } else if ((pcu == 6 || pcu == 7) && (P.nG == 0 || P.nG <= 2)) {
            if (P.nG == 0) {
                const bool split = wide && E.cf_part && E.cf_ticket && P.M > 1024 * P.ncf;
                if (split) {  // long segments: NE_CF_SPLIT workgroups per camera-frame
                    const int gs = P.ncf * NE_CF_SPLIT;
                    if (pcu == 6)
                        k_ne_cf_split<6, 4, NE_CF_SPLIT><<<gs, 256, 0, s>>>(P, J, f, Acc, g, E);
                    else
                        k_ne_cf_split<7, 4, NE_CF_SPLIT><<<gs, 256, 0, s>>>(P, J, f, Acc, g, E);
                } else if (pcu == 6) {
                    if (wide) MMBA_NE_U(6, 4, 0); else MMBA_NE_U(6, 1, 0);
                } else {
                    if (wide) MMBA_NE_U(7, 4, 0); else MMBA_NE_U(7, 1, 0);
                }
            } else {
                if (pcu == 6) {
                    if (wide) MMBA_NE_U(6, 4, 2); else MMBA_NE_U(6, 1, 2);
                } else {
                    if (wide) MMBA_NE_U(7, 4, 2); else MMBA_NE_U(7, 1, 2);
                }
            }
        } else {
            k_ne_cf<<<P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g);
        }
#undef MMBA_NE_U
    }
    if (P.nbs > 0) {
        if (P.JB)  // every solved bundle fast and no global parameters
            k_ne_bnd_jb<<<nblk(P.nB, NE_BND_TPB), NE_BND_TPB, 0, s>>>(P, Abb, g, E);
        else
            k_ne_bnd<<<nblk(P.nB, 64), 64, 0, s>>>(P, J, jcol, nloc, f, Abb, Abg, g);
    }
    if (P.nG > 0) {
        const int nb = nblk(P.M, glob_chunk);
        if (glob_done)
            ;
        else if (P.nG <= 2)
            k_ne_glob<2><<<nb, 256, 0, s>>>(P, J, jcol, nloc, f, glob_partial, glob_chunk);
        else if (P.nG <= 4)
            k_ne_glob<4><<<nb, 256, 0, s>>>(P, J, jcol, nloc, f, glob_partial, glob_chunk);
        else if (P.nG <= 8)
            k_ne_glob<8><<<nb, 256, 0, s>>>(P, J, jcol, nloc, f, glob_partial, glob_chunk);
        else if (P.nG <= 16)
            k_ne_glob<16><<<nb, 256, 0, s>>>(P, J, jcol, nloc, f, glob_partial, glob_chunk);
        else
            k_ne_glob_wide<<<nb, 256, 0, s>>>(P, J, jcol, nloc, f, glob_partial, glob_chunk);
        k_ne_glob_reduce<<<1, 256, 0, s>>>(P, glob_partial, nb, Agg, gG);
    }
}
void launch_colnorms(hipStream_t s, const DevProblem &P, const double *Acc, const double *Abb,
                     const double *aggbuf, double *acnorm, double *g) {
    k_colnorms<<<nblk(P.n, 256), 256, 0, s>>>(P, Acc, Abb, aggbuf, aggbuf + NGMAX * NGMAX,
                                               acnorm, g);
}
void launch_bundle_factor(hipStream_t s, const DevProblem &P, const double *Abb,
                          const double *Abg, const double *g, const double *diag, double lam,
                          double *Lb, double *tb, double *Wg, int *fail) {
    if (P.nB == 0) return;
    k_bundle_factor<<<nblk(P.nB, 64), 64, 0, s>>>(P, Abb, Abg, g, diag, lam, Lb, tb, Wg, fail);
}
void launch_schur_obs(hipStream_t s, const DevProblem &P, const double *J, const double *Lb,
                      double *W, const RedSpec *red, const double *partial, double *scalar,
                      const int *gate) {
    const int nob = nblk(P.M, 64), nr = red ? red->nrows : 0;
    if (nob + nr > 0) {
        if (P.wst / 3 <= 8)
            k_schur_obs<8><<<nob + nr, 64, sizeof(double) * 64 * P.wst, s>>>(
                P, J, Lb, W, nob, red ? *red : RedSpec{}, partial, scalar, gate);
        else
            k_schur_obs<PCMAX><<<nob + nr, 64, sizeof(double) * 64 * P.wst, s>>>(
                P, J, Lb, W, nob, red ? *red : RedSpec{}, partial, scalar, gate);
    }
}
void launch_schur_obs_rs(hipStream_t s, const DevProblem &PV, int Mr, const int *nloc,
                         const int *vobs, const int *vcoff, const double *J, const double *Lb,
                         double *W) {
    if (PV.M > 0)
        k_schur_obs_rs<<<nblk(PV.M, 64), 64, 0, s>>>(PV, Mr, nloc, vobs, vcoff, J, Lb, W);
}
void launch_schur_init(hipStream_t s, const DevProblem &P, const double *Acc, const double *Acg,
                       const double *Agg, const double *g, const double *diag, double lam,
                       const SView &V, int npad, double *rhs, const RedSpec *red,
                       const double *partial, double *scalar) {
    const int n = P.ncf * PCMAX + P.nG + npad;
    if (red && red->nrows > 0)
        k_schur_init_red<<<nblk(n, 256) + red->nrows, 256, 0, s>>>(
            P, Acc, Acg, Agg, g, diag, lam, V, npad, rhs, nblk(n, 256), partial, *red, scalar);
    else
        k_schur_init<<<nblk(n, 256), 256, 0, s>>>(P, Acc, Acg, Agg, g, diag, lam, V, npad, rhs);
    if (P.rs) launch_rs_offdiag(s, P, V);  // camera-frame coupling blocks
}
void launch_schur_pairs(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                        const double *tb, const SView &V, double *rhs) {
    if (P.nB == 0) return;
    k_schur_pairs<<<nblk(P.nB, 64), 64, 0, s>>>(P, W, Wg, tb, V, rhs);
}
bool launch_schur_dest(hipStream_t s, const DevProblem &P, const double *W, const int2 *dest,
                       const int *dest_off, int ndest, const int2 *pairs, const SView &V,
                       int pc_uniform, int assign_off, const double *tb, double *rhs,
                       SchurInitFold fold, const int *wave_list, int n_wave,
                       const int *lane_list, int n_lane) {
    if (ndest <= 0) return false;
    // split pass: the wave kernel over its list, the lane kernel over the rest
    const int nw = lane_list ? n_wave : ndest;
    const int *wl = lane_list ? wave_list : nullptr;
    const int lg = 8 * ((nblk(n_lane, 256) + 7) / 8);
    // fold.on only comes with rhs and pc_uniform 6 / 7 (Plan::fold_init)
    if (pc_uniform == 6) {
        if (nw > 0)
            k_schur_dest_u<6><<<8 * ((nw + 7) / 8), 64, 0, s>>>(P, W, dest, dest_off, pairs, V,
                                                                assign_off, nw, tb, rhs, fold, wl);
        if (lane_list)
            k_schur_dest_lane<6><<<lg, 256, 0, s>>>(P, W, dest, dest_off, pairs, V, assign_off,
                                                    lane_list, n_lane);
        return rhs != nullptr;
    }
    if (pc_uniform == 7) {
        if (nw > 0)
            k_schur_dest_u<7><<<8 * ((nw + 7) / 8), 64, 0, s>>>(P, W, dest, dest_off, pairs, V,
                                                                assign_off, nw, tb, rhs, fold, wl);
        if (lane_list)
            k_schur_dest_lane<7><<<lg, 256, 0, s>>>(P, W, dest, dest_off, pairs, V, assign_off,
                                                    lane_list, n_lane);
        return rhs != nullptr;
    }
    k_schur_dest<<<ndest, 64, 0, s>>>(P, W, dest, dest_off, pairs, V, assign_off);
    return false;
}
void launch_schur_rhs(hipStream_t s, const DevProblem &P, const double *W, const double *tb,
                      const int *row_cf, double *rhs) {
    (void)row_cf;
    if (P.ncf > 0) k_schur_rhs<<<P.ncf, 64, 0, s>>>(P, W, tb, rhs);
}
void launch_schur_glob(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                       const double *tb, const SView &V, double *rhs) {
    if (P.nG > 0 && P.nB > 0)
        k_schur_glob<<<nblk(P.nB, 64), 64, 0, s>>>(P, W, Wg, tb, V, rhs);
}
void launch_backsub_bundle(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                           const double *tb, const double *Lb, const double *xR, double *U,
                           double *x) {
    if (P.nB == 0) return;
    // two passes (coalesced per-observation u_i, then the bundle gather)
    // measured faster than one per-bundle pass gathering W rows (21.6 vs
    // 25.4 us on C4)
    constexpr bool two_pass = true;
    if (two_pass) {  // per-observation u_i pass, then the bundle gather
        k_obs_wtx<<<nblk(P.M, 64), 64, sizeof(double) * 64 * P.wst, s>>>(P, W, xR, U);
        k_backsub_bundle<<<nblk(P.nB, 64), 64, 0, s>>>(P, nullptr, U, Wg, tb, Lb, xR, x);
    } else {
        k_backsub_bundle<<<nblk(P.nB, 64), 64, 0, s>>>(P, W, nullptr, Wg, tb, Lb, xR, x);
    }
}
void launch_scatter_xR(hipStream_t s, const DevProblem &P, const double *xR, double *x) {
    k_scatter_xR<<<nblk(P.n, 256), 256, 0, s>>>(P, xR, x);
}
void launch_newton_bundle(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                          const double *Lb, const double *v, double *wR, double *usq,
                          double *un, double *gp) {
    if (P.nB == 0) return;
    k_newton_bundle<<<nblk(P.nB, 64), 64, 0, s>>>(P, Wg, Lb, v, un, gp, usq);
    if (P.ncf > 0) k_schur_rhs<<<P.ncf, 64, 0, s>>>(P, W, un, wR);
    if (P.nG > 0) k_newton_glob<<<P.nG, 256, 0, s>>>(P, gp, wR);
}
void launch_gather_R(hipStream_t s, const DevProblem &P, const double *v, double *vR, int nRpad) {
    const int n = P.n > nRpad ? P.n : nRpad;
    k_gather_R<<<nblk(n, 256), 256, 0, s>>>(P, v, vR, nRpad);
}
void launch_sumsq(hipStream_t s, const double *a, const double *d, int n, double *partial,
                  int nparts, double *out, const int *mask, unsigned int *ticket) {
    k_sumsq<<<nparts, 256, 0, s>>>(a, d, n, mask, partial, out, ticket);
    if (!ticket && out) k_reduce_sum<<<1, 256, 0, s>>>(partial, nparts, out);
}
void launch_sumsq_div(hipStream_t s, const double *a, const double *d, int n, double *partial,
                      int nparts, double *out, const int *mask, unsigned int *ticket) {
    k_sumsq_div<<<nparts, 256, 0, s>>>(a, d, n, mask, partial, out, ticket);
    if (!ticket) k_reduce_sum<<<1, 256, 0, s>>>(partial, nparts, out);
}
void launch_sumsq_mix(hipStream_t s, const double *y, const double *v, int n, double *partial,
                      int nparts, double *out, const int *mask) {
    k_sumsq_mix<<<nparts, 256, 0, s>>>(y, v, n, mask, partial);
    k_reduce_sum<<<1, 256, 0, s>>>(partial, nparts, out);
}
void launch_reduce_sum(hipStream_t s, const double *partial, int n, double *out) {
    k_reduce_sum<<<1, 256, 0, s>>>(partial, n, out);
}
void launch_gnorm(hipStream_t s, const double *g, const double *acnorm, int n, double fnorm,
                  double *partial, int nparts, double *out, const int *mask,
                  unsigned int *ticket) {
    k_gnorm<<<nparts, 256, 0, s>>>(g, acnorm, n, fnorm, mask, partial, out, ticket);
    if (!ticket) k_reduce_max<<<1, 256, 0, s>>>(partial, nparts, out);
}
void launch_jp_sumsq(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
                     const int *nloc, const double *p, double *partial, int nparts,
                     double *out, unsigned int *ticket) {
    k_jp_sumsq<<<nparts, 256, 0, s>>>(P, J, jcol, nloc, p, partial, out, ticket);
    if (!ticket && out) k_reduce_sum<<<1, 256, 0, s>>>(partial, nparts, out);
}
void launch_zero_flag(hipStream_t s, const double *acnorm, int n, const int *mask,
                      double *partial, int nparts, double *out, unsigned int *ticket) {
    k_zero_flag<<<nparts, 256, 0, s>>>(acnorm, n, mask, partial, out, ticket);
    if (!ticket) k_reduce_max<<<1, 256, 0, s>>>(partial, nparts, out);
}
__global__ void k_flag_to_scalar(int *flag, double *out) {
    if (threadIdx.x == 0) {
        *out = (double)*flag;
        *flag = 0;  // read-and-clear: ready for the next factorisation
    }
}
void launch_flag_to_scalar(hipStream_t s, int *flag, double *out) {
    k_flag_to_scalar<<<1, 64, 0, s>>>(flag, out);
}
void launch_keep_rows(hipStream_t s, double *v, int lo, int hi, int nCF, int nR, int root) {
    if (nR > 0) k_keep_rows<<<nblk(nR, 256), 256, 0, s>>>(v, lo, hi, nCF, nR, root);
}
void launch_keep_mask(hipStream_t s, const double *src, const int *mask, int n, double *dst) {
    if (n > 0) k_keep_mask<<<nblk(n, 256), 256, 0, s>>>(src, mask, n, dst);
}
void launch_lm_step(hipStream_t s, int n, const double *xs, const double *x, const double *diag,
                    double *wa1, double *wa2, double *wa3) {
    k_lm_step<<<nblk(n, 256), 256, 0, s>>>(n, xs, x, diag, wa1, wa2, wa3);
}
void launch_diag_init(hipStream_t s, int n, const double *acnorm, double *diag, int first,
                      int mode) {
    k_diag_init<<<nblk(n, 256), 256, 0, s>>>(n, acnorm, diag, first, mode);
}
void launch_newton_v(hipStream_t s, int n, const double *diag, const double *x, double dxnorm,
                     double *v) {
    k_newton_v<<<nblk(n, 256), 256, 0, s>>>(n, diag, x, dxnorm, v);
}
void launch_unpermute(hipStream_t s, int M, const int *ref_of_dev, const int *obs_own,
                      const double *f2,
                      const double *eu2, const double *ed, double *f2o, double *eu2o,
                      double *edo) {
    k_unpermute<<<nblk(M, 256), 256, 0, s>>>(M, ref_of_dev, obs_own, f2, eu2, ed, f2o, eu2o,
                                             edo);
}
void launch_handback_host(hipStream_t s, int Mg, int nrows, const int *dev_of_ref,
                          const double *f2, const double *eu2, const double *ed, double *hf,
                          double *heu, double *hed, const double *dec, const double *f2_trial) {
    const int n = Mg + nrows;
    if (n <= 0) return;
    // PCIe, not the grid, bounds it: 128 workgroups (half the CUs, one each)
    // keep ~1 MB of stores in flight and leave the other CUs' memory pipes to
    // the statistics kernels running beside it (2,048 / 512 held them behind
    // its PCIe-bound stores for ~50 us)
    k_handback_host<<<std::min(nblk(n, 256), 128), 256, 0, s>>>(Mg, nrows, dev_of_ref, f2, eu2,
                                                                 ed, hf, heu, hed, dec, f2_trial);
}

}  // namespace mmba
