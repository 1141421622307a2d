/*
 * rt_libm.h — portable fp64 transcendentals, compiled identically for the host (C, gcc) and the
 * device (HIP, gfx950): sin, cos, log, atan, asin and the x ** 5 of schlick.
 *
 * Why: the reference evaluates sin/cos/log/atan/asin in glibc's libm (GHC calls libm; SURVEY.md
 * App. A), the device in OCML. The two differ in the last bit for 2-6 % of arguments (and glibc is not
 * correctly rounded either: 0.1-0.2 % of these functions' arguments are misrounded). In tier B such an
 * ulp only moves one sample; in tier A (RT_RNG_EXACT) one column threads a single generator through
 * every row, sample and bounce, so an ulp that later flips any branch (a medium's hit distance, a
 * grazing intersection after a chaotic path) changes how many draws the column consumes and with it
 * every pixel below. With RT_FLAG_SHARED_LIBM both the device (render_exact) and the oracle evaluate
 * these functions here, with the same operations in the same order (IEEE +, -, *, /, sqrt and fma,
 * no contraction), so the two agree bit for bit and the rest of the path — draw order, media, motion
 * time, textures — is checked exactly on every scene.
 *
 * Accuracy: within about 1 ulp (sin/cos: Cody-Waite reduction by pi/2 in three parts and Taylor
 * kernels on [-pi/4, pi/4] carried with the reduced argument's low part; log: fdlibm's
 * f - (hfsq - s(hfsq + R)) form with the atanh series; atan: a table of atan(j/8) and a series in
 * t = (y - j/8) / (1 + y j/8); asin via atan). Constants are the mathematical values rounded to double
 * (generated with mpmath at 300 bits). Arguments beyond 2^20 pi/2 lose reduction accuracy but stay
 * deterministic on both sides.
 */
#ifndef RT_LIBM_H
#define RT_LIBM_H

#include <math.h>

#if defined(__HIPCC__)
#define RTLM_FN __host__ __device__ static inline
#else
#define RTLM_FN static inline
#endif

/* --------------------------------------------------------------- sin / cos */
/* x = k pi/2 + (hi + lo), |hi| <= pi/4 (about); returns k mod 4. pi/2 = P1 + P2 + P3, P1 and P2 with
   33 significant bits, so k P1 and k P2 are exact for |k| < 2^20. */
RTLM_FN int rtlm_rem_pio2(double x, double* hi, double* lo) {
  const double P1 = 0x1.921fb54400000p+0, P2 = 0x1.0b4611a600000p-34, P3 = 0x1.3198a2e037073p-69;
  const double k = rint(x * 0x1.45f306dc9c883p-1);
  const double t = x - k * P1;
  const double w = k * P2;
  const double r = t - w; /* TwoSum(t, -w) */
  const double bp = r - t;
  double e = (t - (r - bp)) + (-w - bp);
  e = e - k * P3;
  const double h = r + e;
  *hi = h;
  *lo = (r - h) + e;
  const double kk = k - 4.0 * floor(k * 0.25); /* k mod 4 in [0, 4) (k is an integer or not finite) */
  return kk == kk ? (int)kk : 0;
}
RTLM_FN double rtlm_sin_k(double hi, double lo) { /* sin(hi + lo), |hi| <= pi/4 */
  const double z = hi * hi;
  const double p = -0x1.5555555555555p-3 +
                   z * (0x1.1111111111111p-7 +
                        z * (-0x1.a01a01a01a01ap-13 +
                             z * (0x1.71de3a556c734p-19 +
                                  z * (-0x1.ae64567f544e4p-26 +
                                       z * (0x1.6124613a86d09p-33 +
                                            z * (-0x1.ae7f3e733b81fp-41 + z * 0x1.952c77030ad4ap-49))))));
  return hi + (hi * z * p + lo * (1.0 - 0.5 * z));
}
RTLM_FN double rtlm_cos_k(double hi, double lo) { /* cos(hi + lo), |hi| <= pi/4 */
  const double z = hi * hi;
  const double zl = fma(hi, hi, -z); /* z's rounding error, exactly */
  const double q = 0x1.5555555555555p-5 +
                   z * (-0x1.6c16c16c16c17p-10 +
                        z * (0x1.a01a01a01a01ap-16 +
                             z * (-0x1.27e4fb7789f5cp-22 +
                                  z * (0x1.1eed8eff8d898p-29 +
                                       z * (-0x1.93974a8c07c9dp-37 +
                                            z * (0x1.ae7f3e733b81fp-45 +
                                                 z * (-0x1.6827863b97d97p-53 + z * 0x1.e542ba4020225p-62)))))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + ((((1.0 - w) - hz) - 0.5 * zl) + (z * z * q - hi * lo));
}
RTLM_FN double rtlm_sin(double x) {
  if (fabs(x) < 0x1p-27) return x;
  double h, l;
  const int q = rtlm_rem_pio2(x, &h, &l);
  switch (q) {
    case 0: return rtlm_sin_k(h, l);
    case 1: return rtlm_cos_k(h, l);
    case 2: return -rtlm_sin_k(h, l);
    default: return -rtlm_cos_k(h, l);
  }
}
RTLM_FN double rtlm_cos(double x) {
  if (fabs(x) < 0x1p-27) return 1.0;
  double h, l;
  const int q = rtlm_rem_pio2(x, &h, &l);
  switch (q) {
    case 0: return rtlm_cos_k(h, l);
    case 1: return -rtlm_sin_k(h, l);
    case 2: return -rtlm_cos_k(h, l);
    default: return rtlm_sin_k(h, l);
  }
}

/* --------------------------------------------------------------- log */
RTLM_FN double rtlm_log(double x) {
  if (x != x) return x;
  if (x <= 0.0) return x == 0.0 ? -INFINITY : NAN;
  if (x == INFINITY) return x;
  int e;
  double m = frexp(x, &e); /* x = m 2^e, m in [0.5, 1) (exact, subnormals included) */
  if (m < 0x1.6a09e667f3bcdp-1) {
    m = m * 2.0;
    e = e - 1;
  }
  const double f = m - 1.0; /* exact: m in [sqrt(1/2), sqrt(2)) */
  const double k = (double)e;
  const double s = f / (2.0 + f);
  const double z = s * s;
  /* R = sum_{i=1..11} 2/(2i+1) z^i: log(1+f) = f - (hfsq - s (hfsq + R)) */
  const double r = z * (0x1.5555555555555p-1 +
                   z * (0x1.999999999999ap-2 +
                   z * (0x1.2492492492492p-2 +
                   z * (0x1.c71c71c71c71cp-3 +
                   z * (0x1.745d1745d1746p-3 +
                   z * (0x1.3b13b13b13b14p-3 +
                   z * (0x1.1111111111111p-3 +
                   z * (0x1.e1e1e1e1e1e1ep-4 +
                   z * (0x1.af286bca1af28p-4 +
                   z * (0x1.8618618618618p-4 + z * 0x1.642c8590b2164p-4))))))))));
  const double hfsq = 0.5 * f * f;
  /* ln 2 = LN2_HI + LN2_LO, LN2_HI with 32 significant bits (k LN2_HI exact) */
  return k * 0x1.62e42ff000000p-1 - ((hfsq - (s * (hfsq + r) + k * -0x1.718432a1b0e26p-35)) - f);
}

/* --------------------------------------------------------------- atan / asin */
RTLM_FN double rtlm_atan(double x) {
  if (x != x) return x;
  const double ax = fabs(x);
  const int inv = ax > 1.0;
  const double y = inv ? 1.0 / ax : ax; /* (x = +-inf: y = 0) */
  const int j = (int)rint(y * 8.0);     /* 0..8 */
  const double c = 0.125 * (double)j;
  const double t = (y - c) / fma(y, c, 1.0); /* atan y = atan c + atan t, |t| <= 1/16 about */
  const double z = t * t;
  const double p = t * z * (-0x1.5555555555555p-2 +
                   z * (0x1.999999999999ap-3 +
                   z * (-0x1.2492492492492p-3 +
                   z * (0x1.c71c71c71c71cp-4 +
                   z * (-0x1.745d1745d1746p-4 +
                   z * (0x1.3b13b13b13b14p-4 +
                   z * (-0x1.1111111111111p-4 + z * (0x1.e1e1e1e1e1e1ep-5 + z * -0x1.af286bca1af28p-5))))))));
  /* atan(j/8) = AH[j] + AL[j] */
  static const double AH[9] = {0.0, 0x1.fd5ba9aac2f6ep-4, 0x1.f5b75f92c80ddp-3, 0x1.6f61941e4def1p-2,
                               0x1.dac670561bb4fp-2, 0x1.1e00babdefeb4p-1, 0x1.4978fa3269ee1p-1,
                               0x1.700a7c5784634p-1, 0x1.921fb54442d18p-1};
  static const double AL[9] = {0.0, -0x1.cd37686760c17p-59, 0x1.8ab6e3cf7afbdp-57, -0x1.c63aae6f6e918p-56,
                               0x1.a2b7f222f65e2p-56, -0x1.928df287a668fp-58, 0x1.2419a87f2a458p-56,
                               -0x1.8c34d25aadef6p-56, 0x1.1a62633145c07p-55};
  double r;
  if (!inv) r = AH[j] + (AL[j] + (t + p));
  else r = (0x1.921fb54442d18p+0 - AH[j]) + ((0x1.1a62633145c07p-54 - AL[j]) - (t + p)); /* pi/2 - atan y */
  return signbit(x) ? -r : r;
}
RTLM_FN double rtlm_asin(double x) {
  if (!(fabs(x) <= 1.0)) return x != x ? x : NAN;
  const double d = (1.0 - x) * (1.0 + x);
  return rtlm_atan(x / sqrt(d)); /* (x = +-1: x / 0 = +-inf, atan = +-pi/2; x = -0: -0) */
}

/* --------------------------------------------------------------- x ** 5 */
/* schlick's (1 - cos) ** 5 (src/Lib.hs:903). x^2, x^4 and x^5 carried as unevaluated sums hi + lo
   (each product's rounding error recovered exactly by an FMA): one final rounding, the correctly
   rounded x^5 except within ~2^-100 relative of a midpoint. Zeros, NaN, infinities and magnitudes
   outside [2^-200, 2^200] take the plain product. */
RTLM_FN double rtlm_pow5(double x) {
  const double ax = fabs(x);
  if (!(ax >= 0x1p-200 && ax <= 0x1p200)) return x * x * x * x * x;
  const double h2 = x * x, l2 = fma(x, x, -h2);
  double h4 = h2 * h2, l4 = fma(h2, h2, -h4);
  l4 = fma(2.0 * h2, l2, l4); /* (h2 + l2)^2 = h2^2 + 2 h2 l2 (+ l2^2, below 2^-104 relative) */
  const double s4 = h4 + l4;
  l4 = l4 - (s4 - h4);
  h4 = s4;
  const double h5 = h4 * x;
  double l5 = fma(h4, x, -h5);
  l5 = fma(l4, x, l5);
  return h5 + l5;
}

#endif /* RT_LIBM_H */
