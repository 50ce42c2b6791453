// Microbenchmark: k_pcr_solve<24> (mmba_pcr.hip) on a C4-sized band system
// (nb = 2994, w = 23: 125 blocks, 7 levels), warm, with the phase probe of
// block nblk / 2: per level, the 100 MHz wall-clock time of the pivot chain,
// the publication, the wait for the neighbours, staging, the W products and
// the update; plus HIP-event time per launch.  Build (from this directory):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../mayamatchmovesolver_amd/csrc \
//     pcr_probe.hip -o pcr_probe
#include "mmba_pcr.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace mmba {
void set_error(const std::string &) {}  // (the library's; unused here)
int path_choice(int) { return -1; }       // (the library's; defaults here)
}  // namespace mmba

using namespace mmba;

int main(int argc, char **argv) {
    const int nb = argc > 1 ? std::atoi(argv[1]) : 2994, w = 23, K = 24;
    const int W1 = w + 1;
    std::vector<double> Bd((size_t)nb * W1, 0.);
    for (int i = 0; i < nb; ++i)
        for (int k = 0; k < W1; ++k) {
            const int c = i - w + k;
            if (c < 0) continue;
            Bd[(size_t)i * W1 + k] = (c == i) ? 3.0 * w : 0.5 * std::sin(0.37 * i + 1.3 * c);
        }
    PcrDev P;
    P.K = K;
    P.nb = nb;
    P.w = w;
    P.nblk = (nb + K - 1) / K;
    int L = 0;
    while ((1 << L) < P.nblk) ++L;
    P.nlev = L;
    double *dBd, *r, *x;
    hipMalloc(&dBd, Bd.size() * 8);
    hipMemcpy(dBd, Bd.data(), Bd.size() * 8, hipMemcpyHostToDevice);
    P.Bd = dBd;
    const size_t ps = (size_t)2 * K * (K + 1) + K * K;
    hipMalloc(&P.pub, (size_t)2 * L * P.nblk * ps * 8);  // 16-B granules
    hipMemset(P.pub, 0, (size_t)2 * L * P.nblk * ps * 8);
    hipMalloc(&P.wlog, (size_t)(L + 1) * P.nblk * 3 * K * K * 8);
    hipMalloc(&P.rpub, (size_t)L * P.nblk * 4 * K * 8);  // 16-B granules
    hipMemset(P.rpub, 0, (size_t)L * P.nblk * 4 * K * 8);
    hipMalloc(&P.part, P.nblk * 8);
    hipMalloc(&P.flev, P.nblk * 4);
    hipMalloc(&r, nb * 8);
    hipMalloc(&x, nb * 8);
    std::vector<double> hr(nb, 1.0);
    hipMemcpy(r, hr.data(), nb * 8, hipMemcpyHostToDevice);
    int *fail;
    hipMalloc(&fail, 4);
    hipMemset(fail, 0, 4);
    long long *probe;
    const size_t probe_n = (size_t)64 * P.nblk;
    hipMalloc(&probe, probe_n * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 20;
    float best = 1e30f, sum = 0.f;
    for (int it = 0; it < reps; ++it) {
        hipMemset(probe, 0, probe_n * 8);
        hipEventRecord(a);
        k_pcr_solve<24><<<pcr_grid(P.nblk), PCR_NTH>>>(P, r, x, nullptr, 1000u + it, fail, probe);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        if (it >= 2) {
            best = std::min(best, ms);
            sum += ms;
        }
    }
    int hf = 0;
    hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost);
    {  // residual of the solve: max |S x - r| / max |r| (S symmetric, band lower)
        std::vector<double> hx(nb), res(nb, 0.);
        hipMemcpy(hx.data(), x, nb * 8, hipMemcpyDeviceToHost);
        for (int i = 0; i < nb; ++i)
            for (int k = 0; k < W1; ++k) {
                const int c = i - w + k;
                if (c < 0) continue;
                const double v = Bd[(size_t)i * W1 + k];
                res[i] += v * hx[c];
                if (c != i) res[c] += v * hx[i];
            }
        double mr = 0.;
        for (int i = 0; i < nb; ++i) mr = std::max(mr, std::fabs(res[i] - hr[i]));
        std::printf("max |S x - r| = %.3e\n", mr);
    }
    std::printf("nb %d nblk %d levels %d: k_pcr_solve<24> best %.1f us, mean %.1f us (fail %d)\n",
                nb, P.nblk, L, best * 1e3, sum / (reps - 2) * 1e3, hf);
    std::vector<long long> tall(probe_n);
    hipMemcpy(tall.data(), probe, probe_n * 8, hipMemcpyDeviceToHost);
    const long long *t = tall.data() + (size_t)64 * (P.nblk / 2);
    const long long t00 = t[0];
    std::printf("block %d, us from its level-0 start (chain | products | publish+log+wait | update):\n",
                P.nblk / 2);
    for (int l = 0; l <= L; ++l) {
        const long long *q = &t[l * 8];
        if (!q[0]) break;
        std::printf("  level %d start %6.2f:", l, (q[0] - t00) / 100.);
        for (int ph = 1; ph <= 4 && q[ph]; ++ph) std::printf(" %5.2f", (q[ph] - q[ph - 1]) / 100.);
        if (q[5] && q[6])  // inside the chain phase (wave 0): load | chain | stores + barrier
            std::printf("   [load %4.2f chain %4.2f rest %4.2f]", (q[5] - q[0]) / 100.,
                        (q[6] - q[5]) / 100., q[1] ? (q[1] - q[6]) / 100. : 0.);
        if (q[7] && q[4])  // thread 0's granules all in -> update done
            std::printf(" [arrived->ready %4.2f]", (q[4] - q[7]) / 100.);
        std::printf("\n");
    }
    // every block: level-start skew and the hand-off -- per level, the
    // spread of level starts, and per coupled block the time from the LATER
    // neighbour's publication (phase 2 end) to this block's update end
    long long g0 = tall[0];
    for (int j = 0; j < P.nblk; ++j)
        if (tall[(size_t)64 * j] && tall[(size_t)64 * j] < g0) g0 = tall[(size_t)64 * j];
    std::printf("all blocks (us from the first block's start): level | start min med max | "
                "later neighbour's publish -> thread 0's granules in min med max | own publish -> later neighbour's publish med max\n");
    for (int l = 0; l < L; ++l) {
        std::vector<double> st, ho, lag;
        const int s = 1 << l;
        for (int j = 0; j < P.nblk; ++j) {
            const long long *q = &tall[(size_t)64 * j + l * 8];
            if (!q[0]) continue;
            st.push_back((q[0] - g0) / 100.);
            long long late = 0;
            for (int nb = -1; nb <= 1; nb += 2) {
                const int k = j + nb * s;
                if (k < 0 || k >= P.nblk) continue;
                const long long pk = tall[(size_t)64 * k + l * 8 + 2];
                if (pk > late) late = pk;
            }
            if (late && q[4]) {
                ho.push_back((q[7] ? q[7] - late : q[4] - late) / 100.);
                if (q[2]) lag.push_back((late - q[2]) / 100.);
            }
        }
        auto mmm = [](std::vector<double> v, double &a, double &m, double &b) {
            if (v.empty()) { a = m = b = 0; return; }
            std::sort(v.begin(), v.end());
            a = v.front(); m = v[v.size() / 2]; b = v.back();
        };
        double a, m, b, c, d, e, f, g, h;
        mmm(st, a, m, b);
        mmm(ho, c, d, e);
        mmm(lag, f, g, h);
        std::printf("  %d | %6.2f %6.2f %6.2f | %5.2f %5.2f %5.2f | %5.2f %5.2f\n", l, a, m, b, c, d, e, g, h);
    }
    // the right-hand-side pass
    float rbest = 1e30f;
    int *mask;
    hipMalloc(&mask, nb * 4);
    std::vector<int> ones(nb, 1);
    hipMemcpy(mask, ones.data(), nb * 4, hipMemcpyHostToDevice);
    for (int it = 0; it < 10; ++it) {
        hipEventRecord(a);
        k_pcr_rhs<24><<<P.nblk, 64>>>(P, r, mask, P.part, 5000u + it, fail);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        if (it >= 2) rbest = std::min(rbest, ms);
    }
    std::printf("k_pcr_rhs<24> best %.1f us\n", rbest * 1e3);
    return 0;
}
