/* CPU check of the reciprocal-form division (ssq_common.h div_fast) against the IEEE
 * fp32 divide on random (x, d) pairs over +-30 binades, all-ones/power-of-two mantissas
 * of d, zeros and subnormals.  gcc -O2 -ffp-contract=off tools/divcheck.c -lm */
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float bf(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static float recip(float d){float a=fabsf(d); return (a>=0x1p-60f&&a<=0x1p60f)?1.0f/d:0.0f;}
static float div_rn(float x,float d,float r){
  float q0=x*r; float q1=fmaf(fmaf(-q0,d,x),r,q0); float q2=fmaf(fmaf(-q1,d,x),r,q1);
  float ax=fabsf(x);
  if(r==0.0f||!(ax<=0x1p60f)||(ax<0x1p-60f&&ax!=0.0f)) return x/d;
  return ax==0.0f?q0:q2;
}
static uint64_t s=88172645463325252ull; static uint32_t rnd(){s^=s<<13;s^=s>>7;s^=s<<17;return (uint32_t)s;}
int main(int argc,char**argv){
  long bad=0,tot=0;
  for(int t=0;t<400;t++){
    uint32_t du=(rnd()&0x7fffffu)|((uint32_t)(60+rnd()%130)<<23);
    if(t<8) du=0x7fffffu|((uint32_t)(110+t*5)<<23);
    if(t>=8&&t<16) du=((uint32_t)(110+t*2)<<23);
    if(rnd()&1) du|=0x80000000u;
    float d=bf(du), r=recip(d);
    int ed=(du>>23)&0xff;
    for(uint32_t k=0;k<(1u<<23);k++){
      uint32_t xe = ed - 30 + (rnd()%62);
      if(xe<1) xe=1; if(xe>254) xe=254;
      uint32_t xu=(rnd()&0x7fffffu)|(xe<<23)|(rnd()&0x80000000u);
      if((k&1023)==0) xu = rnd()&0x807fffffu; // subnormals/zero
      float x=bf(xu);
      float q=x/d, q2=div_rn(x,d,r);
      tot++;
      uint32_t a,b; memcpy(&a,&q,4); memcpy(&b,&q2,4);
      if(a!=b && !(isnan(q)&&isnan(q2))){ if(bad<10) printf("d=%a x=%a q=%a q2=%a\n",d,x,q,q2); bad++;}
    }
  }
  printf("bad %ld of %ld\n",bad,tot);
}
