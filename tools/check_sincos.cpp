// Checks that rtdd::sincos_cr (the device fast path) returns the same bits as
// the plain double-double definitions rtdd::sin_cr / rtdd::cos_cr.
//   g++ -O2 -ffp-contract=off -I ppo-radiotherapy_amd/csrc tools/check_sincos.cpp -o /tmp/check_sincos
//   /tmp/check_sincos [n_uniform]        (exit 0 = identical)
#define __host__
#define __device__
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "rt_ddmath.h"

int main(int argc, char** argv) {
    const long n_uniform = argc > 1 ? std::atol(argv[1]) : 40000000L;
    std::mt19937_64 rng(1);
    std::uniform_real_distribution<double> U(0.0, 1.6), E(-30.0, 0.4);
    long bad = 0, n = 0;
    auto check = [&](double x) {
        double s1, c1;
        rtdd::sincos_cr(x, &s1, &c1);
        const double s0 = rtdd::sin_cr(x), c0 = rtdd::cos_cr(x);
        ++n;
        if (std::memcmp(&s0, &s1, 8) || std::memcmp(&c0, &c1, 8)) {
            if (bad < 10) std::printf("x=%.17g sin %.17g %.17g cos %.17g %.17g\n", x, s0, s1, c0, c1);
            ++bad;
        }
    };
    for (double x : {0.0, 1e-300, 1e-20, 1e-10, 1e-5, 0.001, 0.5, 1.0, 1.3610, 1.5, 1.6}) check(x);
    for (long i = 0; i < n_uniform; ++i) check(U(rng));
    for (long i = 0; i < n_uniform / 4; ++i) check(std::pow(2.0, E(rng)));
    std::printf("n=%ld mismatches=%ld\n", n, bad);
    return bad != 0;
}
