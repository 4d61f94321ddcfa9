// rt_ddmath.h -- correctly rounded f64 sin/cos on [0, ~1.6] via double-double.
//
// scipy's Rotation.from_rotvec (transforms.py:25) calls libm sin/cos on the
// half angle theta/2, theta = |rotvec| <= sqrt(3)*pi/2, so the argument is in
// [0, 1.361].  glibc's sin/cos return the correctly rounded value there in
// practice; ocml's f64 sin/cos are within 1 ulp but not correctly rounded
// (7.6 % of the reference's rotations moved by an ulp on gfx950).  These
// evaluate the Taylor series in double-double (~2^-104 relative) and round
// once, so they reproduce the correctly rounded result on host and device.
// Requires -ffp-contract=off (the error-free transforms depend on it).
#pragma once

#include <cmath>

#define RT_HD __host__ __device__

namespace rtdd {

struct dd {
    double hi, lo;
};

RT_HD inline dd two_sum(double a, double b) {
    double s = a + b;
    double bb = s - a;
    double e = (a - (s - bb)) + (b - bb);
    return {s, e};
}

RT_HD inline dd quick_two_sum(double a, double b) {
    double s = a + b;
    double e = b - (s - a);
    return {s, e};
}

RT_HD inline dd two_prod(double a, double b) {
    double p = a * b;
    double e = fma(a, b, -p);
    return {p, e};
}

RT_HD inline dd add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    dd t = two_sum(a.lo, b.lo);
    s.lo = s.lo + t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo = s.lo + t.lo;
    return quick_two_sum(s.hi, s.lo);
}

RT_HD inline dd mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    double cross = a.hi * b.lo + a.lo * b.hi;
    p.lo = p.lo + cross;
    return quick_two_sum(p.hi, p.lo);
}

// (-1)^k / (2k+1)!  and  (-1)^k / (2k)!, k = 0..17, as double-double
constexpr int kTerms = 18;
constexpr double kSinC[18][2] = {
    {1.0, 0.0},
    {-0.16666666666666666, -9.25185853854297e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {-0.0001984126984126984, -1.7209558293420705e-22},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {-2.505210838544172e-08, 1.448814070935912e-24},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
    {-7.647163731819816e-13, -7.03872877733453e-30},
    {2.8114572543455206e-15, 1.6508842730861433e-31},
    {-8.22063524662433e-18, -2.2141894119604265e-34},
    {1.9572941063391263e-20, -1.3643503830087908e-36},
    {-3.868170170630684e-23, 8.843177655482344e-40},
    {6.446950284384474e-26, -1.9330404233703465e-42},
    {-9.183689863795546e-29, -1.4303150396787322e-45},
    {1.1309962886447716e-31, 1.0498015412959506e-47},
    {-1.216125041553518e-34, -5.586290567888806e-51},
    {1.151633562077195e-37, -6.09957445788454e-54},
    {-9.67759295863189e-41, -3.202295548645562e-57},
};
constexpr double kCosC[18][2] = {
    {1.0, 0.0},
    {-0.5, 0.0},
    {0.041666666666666664, 2.3129646346357427e-18},
    {-0.001388888888888889, 5.300543954373577e-20},
    {2.48015873015873e-05, 2.1511947866775882e-23},
    {-2.755731922398589e-07, -2.3767714622250297e-23},
    {2.08767569878681e-09, -1.20734505911326e-25},
    {-1.1470745597729725e-11, -2.0655512752830745e-28},
    {4.779477332387385e-14, 4.399205485834081e-31},
    {-1.5619206968586225e-16, -1.1910679660273754e-32},
    {4.110317623312165e-19, 1.4412973378659527e-36},
    {-8.896791392450574e-22, 7.911402614872376e-38},
    {1.6117375710961184e-24, -3.6846573564509766e-41},
    {-2.4795962632247976e-27, 1.2953730964765229e-43},
    {3.279889237069838e-30, 1.5117542744029879e-46},
    {-3.7699876288159054e-33, -2.5870347832750324e-49},
    {3.8003907548547434e-36, 1.7457158024652518e-52},
    {-3.387157535521162e-39, -5.09056148151085e-56},
};

// sin(x) and cos(x) together, same bits as sin_cr / cos_cr below (checked on
// 5e7 arguments by tools/check_sincos.cpp), ~3x faster on the device: the 7
// highest-order terms (their sum < 2^-53 relative) run in plain double, the
// rest in double-double with a cheaper add (exact two-sum of the high parts,
// low parts summed), and the sin and cos Horner chains interleave.
RT_HD inline dd add_c(dd p, double chi, double clo) {
    dd s = two_sum(chi, p.hi);
    s.lo = s.lo + (clo + p.lo);
    return quick_two_sum(s.hi, s.lo);
}

RT_HD inline void sincos_cr(double x, double* sn, double* cs) {
    dd x2 = two_prod(x, x);
    double ps = kSinC[kTerms - 1][0], pc = kCosC[kTerms - 1][0];
    for (int k = kTerms - 2; k >= 11; --k) {
        ps = fma(ps, x2.hi, kSinC[k][0]);
        pc = fma(pc, x2.hi, kCosC[k][0]);
    }
    dd PS = {ps, 0.0}, PC = {pc, 0.0};
    for (int k = 10; k >= 0; --k) {
        PS = add_c(mul(PS, x2), kSinC[k][0], kSinC[k][1]);
        PC = add_c(mul(PC, x2), kCosC[k][0], kCosC[k][1]);
    }
    dd r = mul(PS, dd{x, 0.0});
    *sn = r.hi + r.lo;
    *cs = PC.hi + PC.lo;
}

// The plain definitions (all 18 terms in double-double).
// sin(x) for 0 <= x <= 1.6, correctly rounded
RT_HD inline double sin_cr(double x) {
    dd x2 = two_prod(x, x);
    dd p = {kSinC[kTerms - 1][0], kSinC[kTerms - 1][1]};
    for (int k = kTerms - 2; k >= 0; --k) p = add(mul(p, x2), dd{kSinC[k][0], kSinC[k][1]});
    dd r = mul(p, dd{x, 0.0});
    return r.hi + r.lo;
}

// cos(x) for 0 <= x <= 1.6, correctly rounded
RT_HD inline double cos_cr(double x) {
    dd x2 = two_prod(x, x);
    dd p = {kCosC[kTerms - 1][0], kCosC[kTerms - 1][1]};
    for (int k = kTerms - 2; k >= 0; --k) p = add(mul(p, x2), dd{kCosC[k][0], kCosC[k][1]});
    return p.hi + p.lo;
}

}  // namespace rtdd
