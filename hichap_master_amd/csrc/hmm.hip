// Viterbi decoding of the TAD HMM (StructureFind.viterbipath,
// StructureFind.py:1113-1123, which calls ghmm's `model.viterbi` on every DI
// segment).  Host code: one sequential dynamic program per segment over 3-6
// states -- microseconds per segment, nothing for a GPU to do -- kept native
// (C-ABI) so the Python mirror stays a thin caller.
//
// Model: continuous HMM with Gaussian-mixture emissions in ghmm's
// parameterisation (B[i] = [means, variances, weights]).  ghmm is a
// third-party C library absent from /root/reference and from this image
// (pinned version unknown): the recursion below is the textbook log-space
// Viterbi ghmm documents, with impossible transitions at -inf and ties to the
// lowest state index; parity is pinned by exhaustive path enumeration on short
// sequences (tests/test_tads.py), not by ghmm itself.
#include <cmath>
#include <limits>
#include <vector>

#include "hh_common.hpp"

namespace hh {
namespace {

constexpr double kNegInf = -std::numeric_limits<double>::infinity();

inline double log0(double p) { return p > 0.0 ? std::log(p) : kNegInf; }

// log sum_m w_m N(x; mu_m, v_m), by log-sum-exp (no underflow to log 0 for
// observations far in a component's tail)
inline double log_gmm(double x, int M, const double* mu, const double* var, const double* w) {
    double t[64];
    double mx = kNegInf;
    for (int m = 0; m < M; ++m) {
        if (!(w[m] > 0.0)) {
            t[m] = kNegInf;
            continue;
        }
        const double d = x - mu[m];
        t[m] = std::log(w[m]) - 0.5 * std::log(2.0 * M_PI * var[m]) - 0.5 * d * d / var[m];
        if (t[m] > mx) mx = t[m];
    }
    if (mx == kNegInf) return kNegInf;
    double s = 0.0;
    for (int m = 0; m < M; ++m) s += std::exp(t[m] - mx);
    return mx + std::log(s);
}

}  // namespace
}  // namespace hh

using namespace hh;

extern "C" int hh_viterbi_gmm(const double* obs, int64_t n, int32_t S, int32_t M, const double* A, const double* pi,
                              const double* mean, const double* var, const double* weight, int32_t* path,
                              double* logp) {
    return guard([&] {
        HH_REQUIRE(obs && A && pi && mean && var && weight && path && logp, "null argument");
        HH_REQUIRE(n >= 1, "empty sequence");
        HH_REQUIRE(S >= 1 && S <= 64 && M >= 1 && M <= 64, "1 <= states, components <= 64");
        for (int64_t k = 0; k < (int64_t)S * M; ++k)
            HH_REQUIRE(var[k] > 0.0 && weight[k] >= 0.0, "variances must be > 0, weights >= 0");
        std::vector<double> la((size_t)S * S), lpi(S), cur(S), nxt(S);
        for (int64_t k = 0; k < (int64_t)S * S; ++k) la[k] = log0(A[k]);
        for (int i = 0; i < S; ++i) lpi[i] = log0(pi[i]);
        std::vector<int32_t> back((size_t)n * S, 0);
        auto emit = [&](int i, double x) { return log_gmm(x, M, mean + (size_t)i * M, var + (size_t)i * M,
                                                          weight + (size_t)i * M); };
        for (int i = 0; i < S; ++i) cur[i] = lpi[i] + emit(i, obs[0]);
        for (int64_t t = 1; t < n; ++t) {
            for (int j = 0; j < S; ++j) {
                double best = kNegInf;
                int arg = 0;
                for (int i = 0; i < S; ++i) {
                    const double v = cur[i] + la[(size_t)i * S + j];
                    if (v > best) {
                        best = v;
                        arg = i;
                    }
                }
                back[(size_t)t * S + j] = arg;
                nxt[j] = best + emit(j, obs[t]);
            }
            cur.swap(nxt);
        }
        double best = kNegInf;
        int arg = 0;
        for (int i = 0; i < S; ++i)
            if (cur[i] > best) {
                best = cur[i];
                arg = i;
            }
        HH_REQUIRE(best > kNegInf, "no path has nonzero probability under the model");
        for (int64_t t = n - 1; t >= 0; --t) {
            path[t] = arg;
            if (t > 0) arg = back[(size_t)t * S + arg];
        }
        *logp = best;
    });
}
