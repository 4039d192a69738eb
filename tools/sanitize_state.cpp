// sanitize_state.cpp -- the host code of libwce.so that runs without a GPU
// (wce_state.cpp: F, the reference's cofactor invF on a thread pool, H_LT,
// the REF / TEXTBOOK / COV covariances, the sinc table) driven under
// AddressSanitizer + UndefinedBehaviorSanitizer, or ThreadSanitizer for the
// invF thread pool (race detection / sanitizers on host code).
// Built and run by tests/test_sanitize.py; exit 0 = clean and finite.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/wce.h"
#include "../include/wce_debug.h"

static int finite_all(const double *p, size_t n)
{
    for (size_t i = 0; i < n; i++)
        if (!std::isfinite(p[i])) return 0;
    return 1;
}

int main()
{
    const double A = 8.8753, ow2 = 9.6172e-08;
    wce_complex tx_pre[WCE_NSC], rx_pre[WCE_NSC], Rhh[WCE_NSC * WCE_NSC] = {};
    for (int k = 0; k < WCE_NSC; k++) {   // BPSK long training symbol through a 3-tap channel (tools/wce_cli.c)
        double s = ((k * 7 + 3) % 5 < 2) ? -A : A;
        double th = -2 * M_PI * (k - 26) / 64.0;
        double hr = 0.009 + 0.003 * cos(th) + 0.001 * cos(2 * th), hi = 0.003 * sin(th) + 0.001 * sin(2 * th);
        tx_pre[k].re = k == WCE_DC ? 0 : s;
        tx_pre[k].im = 0;
        rx_pre[k].re = tx_pre[k].re * hr;
        rx_pre[k].im = tx_pre[k].re * hi;
        Rhh[k * WCE_NSC + k].re = exp(-0.12 * k) * 1e-5;   // power-delay-profile model
    }
    std::vector<long double> F(WCE_NSC * WCE_NSC * 2), invF(WCE_NSC * WCE_NSC * 2);
    if (wce_debug_reference_F(F.data()) || wce_debug_reference_invF(invF.data())) return 2;
    for (size_t i = 0; i < invF.size(); i++)
        if (!std::isfinite((double)invF[i]) || !std::isfinite((double)F[i])) return 3;
    const size_t n = wce_state_size();
    std::vector<unsigned char> blob(n);
    for (int mode = WCE_MMSE_REF; mode <= WCE_MMSE_TEXTBOOK; mode++)
        if (wce_state_build(blob.data(), n, tx_pre, rx_pre, ow2, mode)) return 4;
    if (wce_state_build_cov(blob.data(), n, tx_pre, rx_pre, Rhh, ow2)) return 5;
    if (wce_state_build(blob.data(), n - 1, tx_pre, rx_pre, ow2, WCE_MMSE_REF) == 0) return 6;   // size check
    std::vector<double> C(WCE_NSC * WCE_NSC * 2), h(WCE_NSC * 2), sinc(4 * WCE_NSC), ab(2);
    unsigned long long xm = 0;
    for (int mode = WCE_MMSE_REF; mode <= WCE_MMSE_TEXTBOOK; mode++) {
        if (wce_debug_build_state(&tx_pre[0].re, &rx_pre[0].re, ow2, mode, C.data(), h.data(), sinc.data(),
                                  ab.data(), &xm))
            return 7;
        if (!finite_all(C.data(), C.size()) || !finite_all(h.data(), h.size()) || !finite_all(sinc.data(), sinc.size()))
            return 8;
    }
    std::printf("sanitize_state ok: F, invF, REF/TEXTBOOK/COV states (%zu B)\n", n);
    return 0;
}
