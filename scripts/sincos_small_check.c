/* Host check of nco_math.h sincos_f64_small (the same operations, explicit fma): rounded to float it
 * must equal glibc double sin/cos.  gcc -O2 -ffp-contract=off scripts/sincos_small_check.c -lm */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
/* fdlibm-style double sincos for |x| < ~1e5: Cody-Waite reduction by pi/2 in three parts, then the
   __kernel_sin / __kernel_cos polynomials with the reduction tail. */
static void sincos_small(double x, double* s, double* c)
{
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double k = rint(x * invpio2);
    const double r0 = fma(-k, pio2_1, x);          /* exact: k small, pio2_1 has 33 bits */
    const double w = k * pio2_2;                     /* exact: pio2_2 has 33 bits */
    const double r1 = r0 - w;
    const double wt = fma(k, pio2_2t, -((r0 - r1) - w)); /* the part of w the subtraction dropped, plus the next term */
    const double y0 = r1 - wt;
    const double y1 = (r1 - y0) - wt;
    /* __kernel_sin(y0, y1) */
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = y0 * y0, v = z * y0;
    const double rs = fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2);
    const double sn = y0 - ((z * (0.5 * y1 - v * rs) - y1) - v * S1);
    /* __kernel_cos(y0, y1) */
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double rc = z * fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
    const double hz = 0.5 * z, ww = 1.0 - hz;
    const double cs = ww + (((1.0 - ww) - hz) + (z * rc - y0 * y1));
    const int q = ((int)k) & 3;
    *s = q == 0 ? sn : q == 1 ? cs : q == 2 ? -sn : -cs;
    *c = q == 0 ? cs : q == 1 ? -sn : q == 2 ? -cs : sn;
}
int main(void)
{
    srand(1);
    long bad = 0, badd = 0; double maxe = 0;
    for (long i = 0; i < 20000000; i++) {
        float xf = (float)((rand() / (double)RAND_MAX) * 14.0 - 7.0);
        if (i % 3 == 0) xf = (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0) * 1e-3f;
        double s, c;
        sincos_small((double)xf, &s, &c);
        double rs = sin((double)xf), rc = cos((double)xf);
        if ((float)s != (float)rs || (float)c != (float)rc) bad++;
        double e1 = fabs(s - rs) / fmax(fabs(rs), 1e-300), e2 = fabs(c - rc) / fmax(fabs(rc), 1e-300);
        if (e1 > maxe) maxe = e1; if (e2 > maxe) maxe = e2;
        if (s != rs || c != rc) badd++;
    }
    printf("float mismatches %ld / 20M, double mismatches %ld, max rel err %.3g\n", bad, badd, maxe);
    return 0;
}
