/* Host check of the kernel's div_pi (pt_kernel.hpp): RN(x/PI) == fma-corrected RN(x*RN(1/PI)) on 4e8 doubles in (0,1]. gcc -O2 -ffp-contract=off div_pi.c -lm */
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static uint64_t xr(void){ s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(void){
  const double P = 3.14159265358979323846; const double y = 1.0 / P;
  long bad = 0, n = 0;
  for (long k = 0; k < 400000000L; ++k) {
    double c;
    uint64_t r = xr();
    if (k & 1) { c = (double)(r >> 11) * 0x1p-53; }             /* uniform in [0,1) */
    else { uint64_t m = (r >> 12) | 0x3ff0000000000000ull; memcpy(&c, &m, 8); c = ldexp(c, -(int)(xr() % 60)) ; } /* random mantissa, exponents down to 2^-60 */
    if (c <= 0) continue;
    double q0 = c * y;
    double rr = fma(-q0, P, c);
    double q1 = fma(rr, y, q0);
    double ref = c / P;
    ++n; if (q1 != ref) { if (bad < 5) printf("mismatch c=%a ref=%a got=%a\n", c, ref, q1); ++bad; }
  }
  printf("tested %ld, mismatches %ld\n", n, bad);
  return 0;
}
