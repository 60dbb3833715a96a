// ttrl_math.h — float64 elementary functions for the fused simulate kernel.
//
// The vehicle model calls sin/cos (heading, steering), atan / asin (steering_control,
// controller.py:145-187), and pow = exp(y log x) (the IDM free-road term, behavior.py:172-183)
// several times per vehicle-frame.  ocml's float64 versions are generic (Payne-Hanek argument
// reduction, extra-precision paths): 90-210 instructions each, and the kernel had to call them
// out of line to keep its register budget.  These are short, branch-free (selects), inline
// restatements of the classic fdlibm algorithms -- Cody-Waite reduction + the __kernel_sin /
// __kernel_cos polynomials, the atan polynomial on |u| <= tan(pi/8), the asin rational form,
// log via atanh(f / (2 + f)), exp via the Remez rational form -- accurate to ~1-2 ulp over the
// argument ranges the simulator produces (tests/test_math.py measures the error against numpy
// over those ranges on the host build of this same header).
//
// Every operation is an explicit fma or a single rounded IEEE op (the kernels build with
// -ffp-contract=off), so the host and device builds return identical bits.
#pragma once

#include <math.h>

#ifndef TTRL_HD
#if defined(__HIPCC__)
#define TTRL_HD __host__ __device__ __forceinline__
#else
#define TTRL_HD static inline
#endif
#endif

namespace ttrl_math {

// |x| above this: the sine / cosine argument reduction falls back to a two-constant step of
// 2*pi (headings are angles of a vehicle; they never get near this in a simulation)
constexpr double SINCOS_CW_MAX = 8.0e5;

// sin and cos on the reduced argument r, |r| <= pi/4 (fdlibm __kernel_sin / __kernel_cos)
TTRL_HD void kernel_sincos(double r, double& s, double& c) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2), S1);
  s = fma(z * r, ps, r);
  const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  c = w + (((1.0 - w) - hz) + z * pc);
}

// sin(x) and cos(x)
TTRL_HD void sincos_d(double x, double& s, double& c) {
  const double PIO2_1 = 1.5707963267948966e+00, PIO2_2 = 6.123233995736766e-17,
               PIO2_3 = -1.4973849048591698e-33;
  double xr = x;
  if (fabs(x) > SINCOS_CW_MAX) {  // out of the simulator's range: reduce mod 2 pi first
    const double TWO_PI_1 = 6.283185307179586, TWO_PI_2 = 2.4492935982947064e-16;
    const double n = rint(x * 0.15915494309189535);
    xr = fma(-n, TWO_PI_2, fma(-n, TWO_PI_1, x));
  }
  const double k = rint(xr * 6.36619772367581382433e-01);
  double r = fma(-k, PIO2_1, xr);
  r = fma(-k, PIO2_2, r);
  r = fma(-k, PIO2_3, r);
  double ks, kc;
  kernel_sincos(r, ks, kc);
  const int q = ((int)k) & 3;
  const double ss = (q & 1) ? kc : ks, cc = (q & 1) ? ks : kc;
  s = (q & 2) ? -ss : ss;
  c = ((q + 1) & 2) ? -cc : cc;
}

// atan(x): |x| is mapped onto |u| <= tan(pi/8) with one division, then fdlibm's atan polynomial
TTRL_HD double atan_d(double x) {
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const double a = fabs(x);
  const bool lo = a <= 0.41421356237309503, hi = a > 2.4142135623730949;
  // atan(a) = 0 + atan(a) | pi/4 + atan((a-1)/(a+1)) | pi/2 + atan(-1/a)
  const double num = lo ? a : (hi ? -1.0 : a - 1.0);
  const double den = lo ? 1.0 : (hi ? a : a + 1.0);
  const double u = num / den;
  const double bh = lo ? 0.0 : (hi ? 1.57079632679489655800e+00 : 7.85398163397448278999e-01);
  const double bl = lo ? 0.0 : (hi ? 6.12323399573676603587e-17 : 3.06161699786838301793e-17);
  const double z = u * u, w = z * z;
  const double s1 = z * fma(w, fma(w, fma(w, fma(w, fma(w, aT10, aT8), aT6), aT4), aT2), aT0);
  const double s2 = w * fma(w, fma(w, fma(w, fma(w, aT9, aT7), aT5), aT3), aT1);
  const double r = bh - ((u * (s1 + s2) - bl) - u);
  return copysign(r, x);  // odd function; a NaN x has made r NaN
}

// asin(x), |x| <= 1 (fdlibm's rational form; |x| >= 1/2 through asin = pi/2 - 2 asin(sqrt((1-|x|)/2)))
TTRL_HD double asin_d(double x) {
  const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
               pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
               pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05;
  const double qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
               qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
  const double a = fabs(x);
  const bool small = a < 0.5;
  const double t = small ? a * a : (1.0 - a) * 0.5;
  const double p = t * fma(t, fma(t, fma(t, fma(t, fma(t, pS5, pS4), pS3), pS2), pS1), pS0);
  const double q = fma(t, fma(t, fma(t, fma(t, qS4, qS3), qS2), qS1), 1.0);
  const double w = p / q;
  const double sq = sqrt(small ? 0.0 : t);
  const double r_small = a + a * w;
  const double r_big = 1.57079632679489655800e+00 - (2.0 * (sq + sq * w) - 6.12323399573676603587e-17);
  const double r = small ? r_small : r_big;
  return copysign(r, x);  // odd function; a NaN x has made r NaN
}

// log(x), x >= 0 (fdlibm: x = 2^k (1 + f), log(1 + f) = f - f^2/2 + s (f^2/2 + R(s^2)), s = f / (2 + f))
TTRL_HD double log_d(double x) {
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  int e;
  double m = frexp(x, &e);  // m in [0.5, 1)
  const bool up = m < 0.70710678118654752440;
  m = up ? m + m : m;
  const double k = (double)(up ? e - 1 : e);
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double r = k * LN2_HI - ((hfsq - (s * (hfsq + R) + k * LN2_LO)) - f);
  // special values: log(0) = -inf, log(inf) = inf, log(<0) / log(nan) = nan
  return x > 0.0 && x < __builtin_inf() ? r : (x == 0.0 ? -__builtin_inf() : (x == x && x > 0.0 ? x : __builtin_nan("")));
}

// exp(y) (fdlibm: y = k ln2 + r, |r| <= ln2/2, exp(r) = 1 + 2r / (R(r^2) - r))
TTRL_HD double exp_d(double y) {
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  // the clamp only keeps k in range (|k| <= 1075); inside (-745.14, 709.79) yc == y
  const double yc = y > 709.8 ? 709.8 : (y < -745.2 ? -745.2 : (y == y ? y : 0.0));
  const double k = rint(yc * 1.44269504088896338700e+00);
  const double hi = fma(-k, LN2_HI, yc);
  const double lo = k * LN2_LO;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * fma(t, fma(t, fma(t, fma(t, P5, P4), P3), P2), P1);
  const double e = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  // 2^k in two exact halves: e * 2^1024 (top binade, e < 1) and the subnormal tail (one rounding,
  // in the second step) stay correct where a single ldexp would overflow or underflow its exponent
  const int k1 = (int)k / 2;
  const double res = ldexp(ldexp(e, k1), (int)k - k1);
  return y > 709.782712893384 ? __builtin_inf() : (y < -745.1332191019412 ? 0.0 : (y == y ? res : y));
}

// x^y = exp(y log x) for x >= 0 (the IDM free-road term's (v / v0)^DELTA)
TTRL_HD double pow_d(double x, double y) { return exp_d(y * log_d(x)); }

}  // namespace ttrl_math
