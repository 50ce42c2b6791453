// mmba_pcr.hip -- parallel cyclic reduction (PCR) of the band reduced camera
// system, fp64, for CDNA4 (gfx950): the damped solve (S + lam D^2) x = r of
// lmpar's qrsolv in ONE persistent launch, no backward pass.
//
// The band system (half bandwidth w <= 23, no arrow) is block tridiagonal in
// K x K blocks (K = 8 / 16 / 24 >= w).  PCR eliminates, at level l (stride
// s = 2^l), the couplings of EVERY block j to its neighbours p = j - s and
// q = j + s:
//
//   D_j <- D_j - A_jp D_p^-1 A_pj - A_jq D_q^-1 A_qj
//   A_j,p-s <- -A_jp D_p^-1 A_p,p-s,   A_j,q+s <- -A_jq D_q^-1 A_q,q+s
//   r_j <- r_j - A_jp D_p^-1 r_p - A_jq D_q^-1 r_q
//
// (block Gaussian elimination of an SPD matrix: every D stays SPD).  After
// ceil(log2 nblk) levels every block is uncoupled and x_j = D_j^-1 r_j: the
// solution comes out of the last level, where block cyclic reduction
// (mmba_bcr.hip) needs a root and a backward pass of as many dependent hops
// again.  The critical path per level is one 24-step pivot chain, two fp64
// MFMA products and one hand-off.
//
// Layout: workgroup j owns block j for the whole solve (its D_j, couplings
// L_j = A_j,j-s, U_j = A_j,j+s and r_j stay in LDS).  Right after its update
// a block factors its new D_j = C_j C_j^T ONCE, by augmented pivot chains
// (mmba_bcr_dev.h) whose right-hand-side lanes carry the identity, L_j, U_j
// and r_j (P_j = C_j^-1 L_j, Q_j = C_j^-1 U_j, rho_j = C_j^-1 r_j), and
// because A_(j-s),j = L_j^T and A_(j+s),j = U_j^T it can form everything its
// two consumers subtract itself (fp64 MFMA), before it publishes:
//
//   left consumer j - s:   P_j^T P_j, P_j^T rho_j, -(Q_j^T P_j)^T (its new U)
//   right consumer j + s:  Q_j^T Q_j, Q_j^T rho_j, -Q_j^T P_j     (its new L)
//
// so a consumer's update is loads and subtractions only:
//
//   D_j -= Q_p^T Q_p + P_q^T P_q,  L_j <- -Q_p^T P_p,  U_j <- -(Q_q^T P_q)^T,
//   r_j -= Q_p^T rho_p + P_q^T rho_q.
//
// Hand-off (round 5): data-tagged 16-B granules, MI355X guide handoff-1to1 /
// Guideline 16 R2 -- every published double is one granule {value, epoch,
// epoch} written by one 16-B sc1 store; a consumer issues 16-B sc1 loads of
// exactly the granules it needs, accepts each when its tags equal the
// launch's epoch and re-polls the others (bounded: a timeout sets bit 1 of
// *fail and the plan falls back to block cyclic reduction).  No store drain,
// flag or barrier between producer and consumer: 7.5 instead of 9.5 us per
// level on the C4 system (profiles/r5_gran/).  Every block's workgroup must
// be resident at once: the plan uses PCR only when the occupancy calculator
// admits nblk workgroups on the device.
//
// lmpar's Newton term v^T (S + lam D^2)^-1 v (the BCR path's ||L^-1 v||^2)
// reruns the elimination on a right-hand side only (k_pcr_rhs): C_j^-1, P_j
// and Q_j of every level are logged (plain stores, issued after the level's
// granule stores so their drain is off the critical path).
#include <atomic>
#include <mutex>

#include "mmba_bcr_dev.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

typedef double pcr_d4 __attribute__((ext_vector_type(4)));

// panel width of the 2 x 2-pivot chain (bcr_ldl2_aug_blk, deferred trailing
// updates): one wave, 24 x 24 augmented factorisation 2.32 us at 4, 2.44 at
// 6, 2.39 at 8 against the one-pivot chain's 2.75 (tools/ubench/chain2.hip,
// profiles/r6_pcr/chain2.txt)
#ifndef PCR_PW
#define PCR_PW 4
#endif
// threads per k_pcr_solve workgroup: the pivot chains use three waves, the
// products (12 MFMA tiles), the granule loads of the update and the log
// spread over all of them
#ifndef PCR_NTH
#define PCR_NTH 256
#endif
typedef unsigned int pcr_u4 __attribute__((ext_vector_type(4)));

// Data-tagged 16-B granules (MI355X guide: handoff-1to1, Guideline 16 R2):
// one published double per granule {lo, hi, epoch, epoch}, stored by ONE
// 16-B sc1 store, loaded by ONE 16-B sc1 load; the consumer accepts it when
// both tag words equal the launch's epoch (no drain, no flag, no barrier
// between producer and consumer).  Granule g of a view at byte 16 g.
__device__ __forceinline__ void gran_st(__amdgpu_buffer_rsrc_t r, int g, double v, unsigned ep) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const pcr_u4 w = {(unsigned)b, (unsigned)(b >> 32), ep, ep};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, g * 16, 0, 16);
}
__device__ __forceinline__ pcr_u4 gran_ld(__amdgpu_buffer_rsrc_t r, int g) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, g * 16, 0, 16);
}
__device__ __forceinline__ bool gran_ok(const pcr_u4 &w, unsigned ep) {
    return w.z == ep && w.w == ep;
}
__device__ __forceinline__ double gran_val(const pcr_u4 &w) {
    return __longlong_as_double((long long)(((unsigned long long)w.y << 32) | w.x));
}

// doubles of one (level, block) publication: X1 = P^T [P | rho], X2 =
// Q^T [Q | rho] (K x (K + 1), row-major) and X3 = Q^T P (K x K)
template <int K>
__host__ __device__ constexpr int pcr_pub_size() {
    return 2 * K * (K + 1) + K * K;
}
// ... and of one (level, block) log: C^-1, P, Q (row-major K x K)
template <int K>
__host__ __device__ constexpr int pcr_log_size() {
    return 3 * K * K;
}

// ---------------------------------------------------------------------------
// The damped solve.  blockIdx.x = block j.  r_in / x_out: reduced-order
// vectors (nb rows); x is also scattered to parameter order (xs[row_param]).
// ---------------------------------------------------------------------------
template <int K, int CH = 0, int NTH = PCR_NTH>
__global__ void __launch_bounds__(NTH) k_pcr_solve(PcrDev P, const double *__restrict__ r_in,
                                                   double *__restrict__ x_out, double *xs,
                                                   unsigned epoch, int *fail,
                                                   long long *probe = nullptr) {
    constexpr int KS = K + 1;  // LDS row stride (odd: a lane-per-row read is conflict-free)
    constexpr int K1 = K + 1;  // row stride of X1 / X2 (the rho column)
    constexpr int PS = pcr_pub_size<K>(), LS = pcr_log_size<K>();
    constexpr int NT = K / 4;  // MFMA k-steps
    constexpr int NE = (K * K + NTH - 1) / NTH;  // update entries per thread
    constexpr int NW = NTH / 64;                // waves
    __shared__ double sD[K * KS], sL[K * KS], sU[K * KS];  // own block (row-major)
    // factor images (row-major): C^-1, P, Q, and rho
    __shared__ double sCi[K * KS], sP[K * KS], sQ[K * KS];
    __shared__ double sr[K], srho[K];
    __shared__ double sI[K * KS];   // the identity (right-hand sides of the C^-1 chain)
    __shared__ double sZ[2 * K];    // a zero row, then scratch for lanes without an operand
    // pivot-chain panel images + pair constants, waves 0..2
    __shared__ double pl[3][2 * 64 * PCR_PW + 64];
    __shared__ int bad_s, ok_s;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    // XCD-aware placement (round 6): workgroup b runs on XCD b % 8; block
    // j = (b % 8) * per + b / 8 keeps the neighbours of the first four levels
    // (strides 1..8) on one XCD; the grid is 8 * per workgroups (pcr_grid),
    // the extra ones exit at once (60.8 against 62.3 us on the C4 system,
    // profiles/r6_pcr/)
    const int per = (P.nblk + 7) / 8;
    const int j = (blockIdx.x % 8) * per + blockIdx.x / 8, nblk = P.nblk, nb = P.nb, W1 = P.w + 1;
    if (j >= nblk) return;
    if (tid == 0) {
        bad_s = 0;
        ok_s = 1;
    }
    // probe (tools/ubench/pcr_probe.hip): thread 0 of every block stores the
    // wall clock (100 MHz) at the phase ends of every level (block j's slots
    // at probe[64 j ..])
    long long *pr = (probe && tid == 0) ? probe + (size_t)j * 64 : nullptr;
    auto stamp = [&](int lvl, int ph) {
        if (pr) pr[lvl * 8 + ph] = (long long)wall_clock64();
    };
    // ---- level-0 state from the band layout: D_j (lower), L_j = S[j, j-1],
    // U_j = S[j, j+1] = S[j+1, j]^T, r_j; padding rows: identity, uncoupled
    for (int q = tid; q < K * K; q += NTH) {
        const int i = q / K, c = q % K, R = j * K + i;
        double dv = 0., lv = 0., uv = 0.;
        if (R < nb) {
            const int C = j * K + c;
            if (c <= i && R - C <= P.w) dv = P.Bd[(size_t)R * W1 + (C - R + P.w)];
            const int Cl = (j - 1) * K + c;
            if (j > 0 && R - Cl <= P.w) lv = P.Bd[(size_t)R * W1 + (Cl - R + P.w)];
            const int R2 = (j + 1) * K + c;  // U_j[i][c] = S[R2, R]
            if (R2 < nb && R2 - R <= P.w) uv = P.Bd[(size_t)R2 * W1 + (R - R2 + P.w)];
        } else if (i == c) {
            dv = 1.;
        }
        sD[i * KS + c] = dv;
        sL[i * KS + c] = lv;
        sU[i * KS + c] = uv;
    }
    if (tid < K) sr[tid] = (j * K + tid < nb) ? r_in[j * K + tid] : 0.;
    for (int q = tid; q < K * KS; q += NTH) sI[q] = (q / KS == q % KS) ? 1. : 0.;
    if (tid < K) sZ[tid] = 0.;
    __syncthreads();
    int s = 1;
    for (int lvl = 0;; ++lvl, s *= 2) {
        const bool hp = j - s >= 0, hq = j + s < nblk;
        stamp(lvl, 0);
        // ---- factor D_j once: C^-1 with rho (wave 0), P = C^-1 L (wave 1),
        // Q = C^-1 U (wave 2): the three chains are the same bits; their
        // right-hand-side lanes write the column images
        int bad = 0;
        if (wv < 3 && (wv == 0 || (wv == 1 && hp) || (wv == 2 && hq))) {
            // one LDS source / destination per lane (no divergent paths):
            // rows of D (its upper part is zero), columns of the identity / L
            // / U, r; the other lanes read a zero row and write scratch
            const double *src = sZ;
            int st = 0;
            double *dst = sZ + K;
            int dt = 0;
            if (lane < K) {
                src = sD + lane * KS;
                st = 1;
            } else if (lane < 2 * K) {
                const int c = lane - K;
                src = (wv == 0 ? sI : (wv == 1 ? sL : sU)) + c;
                st = KS;
                dst = (wv == 0 ? sCi : (wv == 1 ? sP : sQ)) + c;
                dt = KS;
            } else if (wv == 0 && lane == 2 * K) {
                src = sr;
                st = 1;
                dst = srho;
                dt = 1;
            }
            double a[K];
#pragma unroll
            for (int c = 0; c < K; ++c) a[c] = src[c * st];
            stamp(lvl, 5);
            if constexpr (CH == 1)
                bcr_ldl2_aug_blk<K, PCR_PW, 2>(a, pl[wv], bad);
            else if constexpr (CH == 2)
                bcr_ldl1_aug_blk<K, PCR_PW>(a, pl[wv], bad);
            else
                bcr_chol_aug_blk<K, MMBA_BCR_PW>(a, nullptr, pl[wv], bad);
            stamp(lvl, 6);
#pragma unroll
            for (int i = 0; i < K; ++i) dst[i * dt] = a[i];
        }
        if (bad) atomicOr(&bad_s, 1);
        __syncthreads();
        stamp(lvl, 1);
        double *log = P.wlog + ((size_t)lvl * nblk + j) * LS;
        if (!hp && !hq) {
            // uncoupled: x_j = C^-T rho; C^-1 logged for the Newton pass
            if (tid < K) {
                double acc = 0.;
#pragma unroll
                for (int i = 0; i < K; ++i) acc = fma(sCi[i * KS + tid], srho[i], acc);
                const int R = j * K + tid;
                if (R < nb) {
                    x_out[R] = acc;
                    if (xs && P.row_param[R] >= 0) xs[P.row_param[R]] = acc;
                }
            }
            for (int q = tid; q < K * K; q += NTH) log[q] = sCi[(q / K) * KS + q % K];
            if (tid == 0) {
                P.flev[j] = lvl;
                if (bad_s) atomicOr(fail, 1);
            }
            return;
        }
        // ---- what the consumers subtract: X1 = P^T [P | rho] (left, hp),
        // X2 = Q^T [Q | rho] (right, hq), X3 = Q^T P (both): 32 x 32 padded
        // products, 12 tiles over the NW waves (tile t: product t / 4, 16 x 16
        // tile t % 4), stored write-through from the accumulators
        const auto gpub = sc1_view(P.pub + ((size_t)lvl * nblk + j) * PS * 2, PS * 16u);
        {
            // the wave's three tiles interleaved (independent accumulators);
            // a product nobody reads runs on zero operands and is not stored
            const int i16 = lane & 15, k4 = lane >> 4;
            constexpr int TT = (12 + NW - 1) / NW;  // tiles per wave
            pcr_d4 acc[TT];
            // per lane and tile one LDS operand base and stride each: A(i, u)
            // = Y(u, i) (Y = P or Q), B(u, c) = Z(u, c) with column K = rho
            // (X1, X2); padding rows / columns and unneeded products read the
            // zero row
            const double *pa[TT], *pb[TT];
            int sa[TT], sb[TT], bc[TT], cmax[TT];
            bool need[TT];
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) {
                const int t = wv + NW * tt, prod = t >> 2, ti = (t >> 1) & 1, tc = t & 1;
                need[tt] = t < 12 && (prod == 0 ? hp : (prod == 1 ? hq : (hp && hq)));
                cmax[tt] = prod == 2 ? K : K + 1;
                const int ai = ti * 16 + i16;
                bc[tt] = tc * 16 + i16;
                const double *ia = prod == 0 ? sP : sQ, *ib = prod == 1 ? sQ : sP;
                const bool av = need[tt] && ai < K;
                pa[tt] = av ? ia + ai : sZ;
                sa[tt] = av ? KS : 0;
                const bool bv = need[tt] && bc[tt] < cmax[tt];
                pb[tt] = !bv ? sZ : (bc[tt] < K ? ib + bc[tt] : srho);
                sb[tt] = !bv ? 0 : (bc[tt] < K ? KS : 1);
                acc[tt] = pcr_d4{0., 0., 0., 0.};
            }
#pragma unroll
            for (int st = 0; st < NT; ++st) {
                const int u = 4 * st + k4;
#pragma unroll
                for (int tt = 0; tt < TT; ++tt)
                    acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[tt][u * sa[tt]], pb[tt][u * sb[tt]],
                                                                   acc[tt], 0, 0, 0);
            }
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) {
                if (!need[tt]) continue;
                const int t = wv + NW * tt, prod = t >> 2, ti = (t >> 1) & 1;
                const int g0 = prod == 0 ? 0 : (prod == 1 ? K * K1 : 2 * K * K1);
                const int ld = prod == 2 ? K : K1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = ti * 16 + k4 + 4 * r;
                    if (row < K && bc[tt] < cmax[tt])
                        gran_st(gpub, g0 + row * ld + bc[tt], acc[tt][r], epoch);
                }
            }
        }
        stamp(lvl, 2);
        // ---- the Newton pass's log (later launches read it: plain stores;
        // issued during the granule wait instead: 66.7 against 65.0 us)
#ifndef PCR_NOLOG
        for (int q = tid; q < K * K; q += NTH) {
            const int x = (q / K) * KS + q % K;
            log[q] = sCi[x];
            log[K * K + q] = sP[x];
            log[2 * K * K + q] = sQ[x];
        }
#endif
        stamp(lvl, 3);
        // ---- the update from the neighbours' granules of this level: loads
        // and subtractions only
        //   D_j -= X2_p + X1_q (lower), L_j = -X3_p, U_j = -X3_q^T,
        //   r_j -= X2_p(:, K) + X1_q(:, K)
        {
            const bool hpp = hp && j - 2 * s >= 0, hqq = hq && j + 2 * s < nblk;
            const auto vp = sc1_view(P.pub + ((size_t)lvl * nblk + (hp ? j - s : j)) * PS * 2,
                                     hp ? PS * 16u : 0u);
            const auto vq = sc1_view(P.pub + ((size_t)lvl * nblk + (hq ? j + s : j)) * PS * 2,
                                     hq ? PS * 16u : 0u);
            // granules this thread needs: per entry e (X2_p, X3_p | X1_q,
            // X3_q), then the rho column; -1 = none (an absent neighbour or
            // an entry outside the block / above the diagonal)
            constexpr int NG = 2 * NE + 1;
            int gi[2][NG];
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int q = tid + NTH * e, i = q / K, c = q % K;
                const bool in = q < K * K;
                gi[0][2 * e] = (hp && in && c <= i) ? K * K1 + i * K1 + c : -1;
                // X3 is published only by a block with neighbours on both
                // sides: X3_p where p = j - s has j - 2s, X3_q where j + 2s
                gi[0][2 * e + 1] = (hpp && in) ? 2 * K * K1 + q : -1;
                gi[1][2 * e] = (hq && in && c <= i) ? i * K1 + c : -1;
                gi[1][2 * e + 1] = (hqq && in) ? 2 * K * K1 + q : -1;
            }
            gi[0][2 * NE] = (hp && tid < K) ? K * K1 + tid * K1 + K : -1;
            gi[1][2 * NE] = (hq && tid < K) ? tid * K1 + K : -1;
            pcr_u4 g[2][NG];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < NG; ++k)
                    if (gi[h][k] >= 0) g[h][k] = gran_ld(h ? vq : vp, gi[h][k]);
            int late = 0;
            for (unsigned spins = 0;; ++spins) {
                bool all = true;
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int k = 0; k < NG; ++k)
                        if (gi[h][k] >= 0 && !gran_ok(g[h][k], epoch)) all = false;
                if (all) break;
                if (spins > (1u << 20)) {
                    late = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int k = 0; k < NG; ++k)
                        if (gi[h][k] >= 0 && !gran_ok(g[h][k], epoch))
                            g[h][k] = gran_ld(h ? vq : vp, gi[h][k]);
            }
            stamp(lvl, 7);
            if (late) ok_s = 0;  // (ok_s = 1 was set before this level's chain)
            auto val = [&](int h, int k) { return gi[h][k] >= 0 ? gran_val(g[h][k]) : 0.; };
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int q = tid + NTH * e, i = q / K, c = q % K;
                if (q < K * K) {
                    if (c <= i) sD[i * KS + c] -= val(0, 2 * e) + val(1, 2 * e);
                    sL[i * KS + c] = -val(0, 2 * e + 1);  // 0 without j - 2s
                    sU[c * KS + i] = -val(1, 2 * e + 1);  // X3_q(i, c) -> U_j(c, i); 0 without j + 2s
                }
            }
            if (tid < K) sr[tid] -= val(0, 2 * NE) + val(1, 2 * NE);
        }
        __syncthreads();
        if (!ok_s) {
            if (tid == 0) atomicOr(fail, 2);
            return;  // the blocks waiting on this one time out as well
        }
        stamp(lvl, 4);
    }
}

// ---------------------------------------------------------------------------
// Right-hand side only (lmpar's Newton term): z = (S + lam D^2)^-1 w with the
// factors of the last k_pcr_solve, then part[j] = sum over this block's rows
// (mask) of w z.  One 64-lane workgroup per block.  Per level: rho = C^-1 r,
// publish Q^T rho (right consumer) and P^T rho (left consumer), subtract the
// neighbours'.
// ---------------------------------------------------------------------------
template <int K>
__global__ void __launch_bounds__(64) k_pcr_rhs(PcrDev P, const double *__restrict__ w,
                                                const int *__restrict__ mask, double *part,
                                                unsigned epoch, int *fail) {
    constexpr int LS = pcr_log_size<K>();
    __shared__ double sr[K], srho[K];
    __shared__ int late_s;
    const int lane = threadIdx.x, j = blockIdx.x, nblk = P.nblk, nb = P.nb;
    if (lane == 0) late_s = 0;
    const int R = j * K + lane;
    const double w0 = (lane < K && R < nb) ? w[R] : 0.;
    double r = w0;
    const int L = min(max(P.flev[j], 0), P.nlev);  // (flev is zeroed at plan build)
    int s = 1;
    for (int lvl = 0; lvl < L; ++lvl, s *= 2) {
        const bool hp = j - s >= 0, hq = j + s < nblk;
        const double *lg = P.wlog + ((size_t)lvl * nblk + j) * LS;
        if (lane < K) sr[lane] = r;
        __syncthreads();
        if (lane < K) {  // rho_i = sum_c C^-1(i, c) r_c
            double rho = 0.;
#pragma unroll
            for (int c = 0; c < K; ++c) rho = fma(lg[lane * K + c], sr[c], rho);
            srho[lane] = rho;
        }
        __syncthreads();
        // publications: 2 K granules per (level, block) (k_pcr_solve's
        // data-tagged hand-off): (Q^T rho)_c for the right consumer, (P^T
        // rho)_c for the left one
        const auto gpub = sc1_view(P.rpub + ((size_t)lvl * nblk + j) * 4 * K, 2 * K * 16u);
        if (lane < K) {
            double a = 0., b = 0.;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                a = fma(lg[2 * K * K + i * K + lane], srho[i], a);
                b = fma(lg[K * K + i * K + lane], srho[i], b);
            }
            if (hq) gran_st(gpub, lane, a, epoch);
            if (hp) gran_st(gpub, K + lane, b, epoch);
        }
        if (lane < K) {  // r -= Q_p^T rho_p + P_q^T rho_q, from the neighbours' granules
            const auto vp = sc1_view(P.rpub + ((size_t)lvl * nblk + (hp ? j - s : j)) * 4 * K,
                                     hp ? 2 * K * 16u : 0u);
            const auto vq = sc1_view(P.rpub + ((size_t)lvl * nblk + (hq ? j + s : j)) * 4 * K,
                                     hq ? 2 * K * 16u : 0u);
            pcr_u4 gp{}, gq{};
            if (hp) gp = gran_ld(vp, lane);
            if (hq) gq = gran_ld(vq, K + lane);
            for (unsigned spins = 0;; ++spins) {
                const bool okp = !hp || gran_ok(gp, epoch), okq = !hq || gran_ok(gq, epoch);
                if (okp && okq) break;
                if (spins > (1u << 20)) {
                    late_s = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if (!okp) gp = gran_ld(vp, lane);
                if (!okq) gq = gran_ld(vq, K + lane);
            }
            double sub = 0.;
            if (hp) sub += gran_val(gp);
            if (hq) sub += gran_val(gq);
            r -= sub;
        }
        __syncthreads();
        if (late_s) {
            // a timed-out wait: the partial is NaN, so the Newton term that
            // sums it cannot pass for a number (lmpar_ne restarts on it)
            if (lane == 0) {
                atomicOr(fail, 2);
                part[j] = __builtin_nan("");
            }
            return;
        }
    }
    // z = C^-T C^-1 r with the final level's factor
    const double *lg = P.wlog + ((size_t)L * nblk + j) * LS;
    if (lane < K) sr[lane] = r;
    __syncthreads();
    if (lane < K) {
        double rho = 0.;
#pragma unroll
        for (int c = 0; c < K; ++c) rho = fma(lg[lane * K + c], sr[c], rho);
        srho[lane] = rho;
    }
    __syncthreads();
    double z = 0.;
    if (lane < K) {
#pragma unroll
        for (int i = 0; i < K; ++i) z = fma(lg[i * K + lane], srho[i], z);
    }
    double v = (lane < K && R < nb && mask[R]) ? w0 * z : 0.;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) part[j] = v;
}

// ---------------------------------------------------------------------------
// Several right-hand sides at once: Z = (S)^-1 R with the factors (logs) of
// the last k_pcr_solve, R and Z column-major (element (row r, column c) at
// R[c * ldr + r], nc <= PCR_NCMAX columns).  The separator form of the
// sharded solve (mmba_band.hip, Plan::setup_band) applies a shard interior's
// inverse to its boundary couplings and to its right-hand side this way.  One
// 256-thread workgroup per block; per level: rho = C^-1 R, publish Q^T rho
// (right consumer) and P^T rho (left consumer), subtract the neighbours'; at
// the block's last level Z = C^-T C^-1 R.
// ---------------------------------------------------------------------------
template <int K>
__global__ void __launch_bounds__(256) k_pcr_rhs_mc(PcrDev P, const double *__restrict__ R,
                                                    int ldr, int nc, double *Z, int ldz,
                                                    double *mpub, unsigned epoch,
                                                    int *fail) {
    constexpr int LS = pcr_log_size<K>();
    constexpr int NS = PCR_NCMAX + 1;  // LDS row stride
    constexpr int QN = (K * PCR_NCMAX + 255) / 256;  // entries per thread
    __shared__ double sr[K * NS], srho[K * NS], sl[3 * K * K];
    __shared__ int ok_s;
    const int tid = threadIdx.x, j = blockIdx.x, nblk = P.nblk, nb = P.nb;
    if (tid == 0) ok_s = 1;
    const int ne = K * nc;  // entries (row i, column c) of the block's right-hand sides
    for (int q = tid; q < ne; q += 256) {
        const int i = q / nc, c = q % nc, row = j * K + i;
        sr[i * NS + c] = row < nb ? R[(size_t)c * ldr + row] : 0.;
    }
    const int L = min(max(P.flev[j], 0), P.nlev);
    // one (level, block) publication: 2 K PCR_NCMAX granules (k_pcr_solve's
    // data-tagged hand-off), 4 K PCR_NCMAX doubles
    const size_t pst = (size_t)4 * K * PCR_NCMAX;
    int s = 1;
    for (int lvl = 0;; ++lvl, s *= 2) {
        const double *lg = P.wlog + ((size_t)lvl * nblk + j) * LS;
        for (int q = tid; q < (lvl < L ? 3 : 1) * K * K; q += 256) sl[q] = lg[q];
        __syncthreads();
        // rho = C^-1 R
        for (int q = tid; q < ne; q += 256) {
            const int i = q / nc, c = q % nc;
            double a = 0.;
#pragma unroll 8
            for (int k = 0; k < K; ++k) a = fma(sl[i * K + k], sr[k * NS + c], a);
            srho[i * NS + c] = a;
        }
        __syncthreads();
        if (lvl == L) {  // uncoupled: Z = C^-T rho
            for (int q = tid; q < ne; q += 256) {
                const int i = q / nc, c = q % nc, row = j * K + i;
                double a = 0.;
#pragma unroll 8
                for (int k = 0; k < K; ++k) a = fma(sl[k * K + i], srho[k * NS + c], a);
                if (row < nb) Z[(size_t)c * ldz + row] = a;
            }
            return;
        }
        const bool hp = j - s >= 0, hq = j + s < nblk;
        const auto gmp = sc1_view(mpub + ((size_t)lvl * nblk + j) * pst, 2 * K * PCR_NCMAX * 16u);
        // (Q^T rho) for the right consumer, (P^T rho) for the left one
        for (int q = tid; q < ne; q += 256) {
            const int i = q / nc, c = q % nc;
            double a = 0., b = 0.;
#pragma unroll 8
            for (int k = 0; k < K; ++k) {
                a = fma(sl[2 * K * K + k * K + i], srho[k * NS + c], a);
                b = fma(sl[K * K + k * K + i], srho[k * NS + c], b);
            }
            if (hq) gran_st(gmp, q, a, epoch);
            if (hp) gran_st(gmp, K * PCR_NCMAX + q, b, epoch);
        }
        // R -= Q_p^T rho_p + P_q^T rho_q, from the neighbours' granules
        const auto vp = sc1_view(mpub + ((size_t)lvl * nblk + (hp ? j - s : j)) * pst,
                                 hp ? 2 * K * PCR_NCMAX * 16u : 0u);
        const auto vq = sc1_view(mpub + ((size_t)lvl * nblk + (hq ? j + s : j)) * pst,
                                 hq ? 2 * K * PCR_NCMAX * 16u : 0u);
        {
            pcr_u4 gp[QN], gq[QN];
#pragma unroll
            for (int e = 0; e < QN; ++e) {
                const int q = tid + 256 * e;
                if (q < ne && hp) gp[e] = gran_ld(vp, q);
                if (q < ne && hq) gq[e] = gran_ld(vq, K * PCR_NCMAX + q);
            }
            for (unsigned spins = 0;; ++spins) {
                bool all = true;
#pragma unroll
                for (int e = 0; e < QN; ++e) {
                    const int q = tid + 256 * e;
                    if (q < ne && ((hp && !gran_ok(gp[e], epoch)) || (hq && !gran_ok(gq[e], epoch))))
                        all = false;
                }
                if (all) break;
                if (spins > (1u << 20)) {
                    ok_s = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int e = 0; e < QN; ++e) {
                    const int q = tid + 256 * e;
                    if (q < ne && hp && !gran_ok(gp[e], epoch)) gp[e] = gran_ld(vp, q);
                    if (q < ne && hq && !gran_ok(gq[e], epoch)) gq[e] = gran_ld(vq, K * PCR_NCMAX + q);
                }
            }
#pragma unroll
            for (int e = 0; e < QN; ++e) {
                const int q = tid + 256 * e;
                if (q >= ne) continue;
                double sub = 0.;
                if (hp) sub += gran_val(gp[e]);
                if (hq) sub += gran_val(gq[e]);
                sr[(q / nc) * NS + q % nc] -= sub;
            }
        }
        __syncthreads();
        if (!ok_s) {
            // timed out: this block's rows of Z are NaN (never a stale number)
            if (tid == 0) atomicOr(fail, 2);
            for (int q = tid; q < ne; q += 256) {
                const int i = q / nc, c = q % nc, row = j * K + i;
                if (row < nb) Z[(size_t)c * ldz + row] = __builtin_nan("");
            }
            return;
        }
    }
}

static std::atomic<unsigned> g_pcr_epoch{0};

static unsigned pcr_next_epoch() {
    unsigned ep = ++g_pcr_epoch;
    if (ep == 0) ep = ++g_pcr_epoch;  // zeroed granules: never use epoch 0
    return ep;
}

// Two PCR launches running at once on one device can deadlock each other:
// each may hold part of its workgroups resident, spinning, while the rest wait
// for CU slots the other holds (until the bounded waits time out and the
// plans fall back).  So the PCR launches of one process on one device are
// ordered across streams: every launch waits, device-side, for the previous
// PCR launch when that one was issued on another stream (an event recorded
// after each launch).  Plans of one stream are ordered by the stream already,
// and an event record costs several microseconds of stream time, so events
// are used only while more than one context (stream) is open on the device;
// the context that makes it two drains the device first, so every launch
// before the switch has finished.  Other processes sharing the device are
// not covered (their launches time out and fall back to block cyclic
// reduction).
namespace {
struct PcrOrder {
    std::mutex mu;
    hipStream_t last = nullptr;
    hipEvent_t ev = nullptr;
    bool recorded = false;  // ev marks `last`'s latest PCR launch
    int contexts = 0;
};
PcrOrder g_pcr_order[64];
}  // namespace

void pcr_note_context(int dev, int delta) {
    PcrOrder &o = g_pcr_order[dev & 63];
    std::lock_guard<std::mutex> g(o.mu);
    const int before = o.contexts;
    o.contexts += delta;
    if (delta > 0 && before == 1) {
        // one -> two streams: drain what the first one launched unordered
        (void)hipDeviceSynchronize();
        o.recorded = false;
    }
}

template <class Launch>
static void pcr_ordered(hipStream_t s, Launch &&launch) {
    int dev = 0;
    MMBA_HIP(hipGetDevice(&dev));
    PcrOrder &o = g_pcr_order[dev & 63];
    std::lock_guard<std::mutex> g(o.mu);
    if (o.contexts <= 1) {
        launch();
        o.last = s;
        o.recorded = false;
        return;
    }
    if (!o.ev) MMBA_HIP(hipEventCreateWithFlags(&o.ev, hipEventDisableTiming));
    if (o.recorded && o.last != s) MMBA_HIP(hipStreamWaitEvent(s, o.ev, 0));
    launch();
    MMBA_HIP(hipEventRecord(o.ev, s));
    o.last = s;
    o.recorded = true;
}

// The pivot chain of k_pcr_solve's block factorisations (MMBA_PATH_PCR_CHAIN):
// 0 the one-pivot Cholesky chain (default), 1 the 2 x 2-pivot chain, 2 LDL^T
// with 1 x 1 pivots (no square root on the chain).
static int pcr_chain_choice() {
    const int v = path_choice(MMBA_PATH_PCR_CHAIN);
    return (v == 1 || v == 2) ? v : 0;
}

// k_pcr_solve's grid: 8 workgroups per block-row of the XCD map
int pcr_grid(int nblk) { return 8 * ((nblk + 7) / 8); }

void pcr_solve(hipStream_t s, const PcrDev &P, const double *r, double *x, double *xs, int *fail) {
    const int g = pcr_grid(P.nblk);
    // the one-pivot Cholesky chain by default: the 2 x 2-pivot chain is
    // faster (2.32 against 2.75 us per factorisation, tools/ubench/chain2.hip)
    // but measured less accurate on an ill-conditioned C4-spec step
    // (tools/pcr_chain_diag.py, profiles/r6_pcr/pcr_chain_diag.txt): opt-in
    const int ch = pcr_chain_choice();
    const bool wide = P.nth == 512;
    pcr_ordered(s, [&] {
        const unsigned ep = pcr_next_epoch();
#define MMBA_PCR_GO(KK, L2V, NT) k_pcr_solve<KK, L2V, NT><<<g, NT, 0, s>>>(P, r, x, xs, ep, fail)
#define MMBA_PCR_K(L2V, NT)                          \
    switch (P.K) {                                   \
        case 8: MMBA_PCR_GO(8, L2V, NT); break;      \
        case 16: MMBA_PCR_GO(16, L2V, NT); break;    \
        default: MMBA_PCR_GO(24, L2V, NT); break;    \
    }
        if (ch == 1) {
            if (wide) { MMBA_PCR_K(1, 512) } else { MMBA_PCR_K(1, 256) }
        } else if (ch == 2) {
            if (wide) { MMBA_PCR_K(2, 512) } else { MMBA_PCR_K(2, 256) }
        } else {
            if (wide) { MMBA_PCR_K(0, 512) } else { MMBA_PCR_K(0, 256) }
        }
#undef MMBA_PCR_K
#undef MMBA_PCR_GO
    });
}

void pcr_rhs_dot(hipStream_t s, const PcrDev &P, const double *w, const int *mask, int *fail) {
    pcr_ordered(s, [&] {
        const unsigned ep = pcr_next_epoch();
        switch (P.K) {
            case 8: k_pcr_rhs<8><<<P.nblk, 64, 0, s>>>(P, w, mask, P.part, ep, fail); break;
            case 16: k_pcr_rhs<16><<<P.nblk, 64, 0, s>>>(P, w, mask, P.part, ep, fail); break;
            default: k_pcr_rhs<24><<<P.nblk, 64, 0, s>>>(P, w, mask, P.part, ep, fail); break;
        }
    });
}

void pcr_rhs_mc(hipStream_t s, const PcrDev &P, const double *R, int ldr, int nc, double *Z,
                int ldz, int *fail) {
    if (nc <= 0 || nc > PCR_NCMAX) throw Invalid{"pcr_rhs_mc: 1..48 right-hand sides"};
    pcr_ordered(s, [&] {
        const unsigned ep = pcr_next_epoch();
        switch (P.K) {
            case 8: k_pcr_rhs_mc<8><<<P.nblk, 256, 0, s>>>(P, R, ldr, nc, Z, ldz, P.mpub, ep, fail); break;
            case 16: k_pcr_rhs_mc<16><<<P.nblk, 256, 0, s>>>(P, R, ldr, nc, Z, ldz, P.mpub, ep, fail); break;
            default: k_pcr_rhs_mc<24><<<P.nblk, 256, 0, s>>>(P, R, ldr, nc, Z, ldz, P.mpub, ep, fail); break;
        }
    });
}

// Workgroups of the 512-thread k_pcr_solve<K> the device keeps resident at
// once: the plan takes that form (8 waves: the products and the update's
// granule loads over twice the waves; 62.6 against 65.5 us on the C4 system,
// profiles/r6_pcr/) when its whole grid fits, the 256-thread one otherwise.
int pcr_resident_wide(int K) {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    hipError_t e;
    switch (K) {
        case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<8, 0, 512>, 512, 0); break;
        case 16: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<16, 0, 512>, 512, 0); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<24, 0, 512>, 512, 0); break;
    }
    if (e != hipSuccess) return 0;
    return per_cu * cus;
}

// Workgroups of k_pcr_solve<K> (256 threads) the device keeps resident at
// once (every block's workgroup must be: the plan takes PCR only when nblk
// fits).
int pcr_max_resident(int K) {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    hipError_t e;
    switch (K) {
        case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<8, 0, 256>, 256, 0); break;
        case 16: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<16, 0, 256>, 256, 0); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pcr_solve<24, 0, 256>, 256, 0); break;
    }
    if (e != hipSuccess) return 0;
    return per_cu * cus;
}

}  // namespace mmba
