/* The exact-blend mode's expf (gsr_tile.hpp glibc_expf) against the host libm's expf on every
 * float in [-104, 8]: the table from long double exp2, the __expf_fma contractions written out.
 *   gcc -O2 -ffp-contract=off tools/check_glibc_expf.c -o /tmp/check_expf -lm && /tmp/check_expf
 * Prints the table (as gsr_tile.hpp GEXP_TAB holds it) and the mismatch count (0 on this image). */
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
#define N 32
static uint64_t TAB[N];
static inline uint64_t asu(double x){uint64_t u; memcpy(&u,&x,8); return u;}
static inline double asd(uint64_t u){double x; memcpy(&x,&u,8); return x;}
static const double C0 = 0x1.c6af84b912394p-5/N/N/N, C1 = 0x1.ebfce50fac4f3p-3/N/N, C2 = 0x1.62e42ff0c52d6p-1/N;
static const double InvLn2N = 0x1.71547652b82fep+0 * N;
static const double SHIFT = 0x1.8p+52;
float myexpf(float x) {
  if (x < -0x1.9fe368p6f) return 0.0f;
  double xd = (double)x, kd = fma(xd, InvLn2N, SHIFT);
  uint64_t ki = asu(kd); kd -= SHIFT; double r = fma(xd, InvLn2N, -kd);
  uint64_t t = TAB[ki % N]; t += ki << (52 - 5);
  double s = asd(t), zz = fma(C0, r, C1), r2 = r*r, y = fma(r, C2, 1.0); y = fma(zz, r2, y); y = y * s;
  return (float)y;
}
int main(){
  for (int i=0;i<N;i++){ long double v = exp2l((long double)i/N); double d=(double)v; TAB[i] = asu(d) - (((uint64_t)i << 52)/N); }
  printf("TAB:"); for (int i=0;i<N;i++) printf(" 0x%016llxull,", (unsigned long long)TAB[i]); printf("\n");
  printf("C0 %a C1 %a C2 %a InvLn2N %a\n", C0, C1, C2, InvLn2N);
  long n=0,bad=0;
  for (uint64_t b = 0x80000000u; b <= 0xC2D00000u; b++) {   // -0 .. -104
    uint32_t bb=(uint32_t)b; float x; memcpy(&x,&bb,4);
    float a = expf(x), c = myexpf(x); n++; if (memcmp(&a,&c,4)) { if (bad<3) printf("%a %a %a\n", x, a, c); bad++; }
  }
  for (uint32_t b = 0x00000000u; b <= 0x41000000u; b++) {  // 0 .. 8
    float x; memcpy(&x,&b,4); float a = expf(x), c = myexpf(x); n++; if (memcmp(&a,&c,4)) { if (bad<6) printf("%a %a %a\n", x, a, c); bad++; }
  }
  printf("n=%ld bad=%ld\n", n, bad);
}
