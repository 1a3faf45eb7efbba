// Exhaustive accuracy check of gsr_expf over every fp32 in [-87, 0]: the degree-7 Taylor form (e7) vs a
// candidate degree-6 polynomial (e6, coefficients c2..c6 on the command line; tools/exp_poly_fit.py).
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
static float C2,C3,C4,C5,C6;
static inline float e7(float x){ // current
  float xc=fminf(fmaxf(x,-87.f),88.f); float kf=fmaf(xc,1.44269502f,12582912.0f); float k=kf-12582912.0f;
  float r=fmaf(-k,0.693145751953125f,xc); r=fmaf(-k,1.42860677e-06f,r);
  float p=1.98412701e-04f; p=fmaf(p,r,1.38888892e-03f); p=fmaf(p,r,8.33333377e-03f); p=fmaf(p,r,4.16666679e-02f);
  p=fmaf(p,r,1.66666672e-01f); p=fmaf(p,r,0.5f); p=fmaf(p,r,1.0f); p=fmaf(p,r,1.0f);
  uint32_t kb; memcpy(&kb,&kf,4); uint32_t sb=(kb<<23)+0x3f800000u; float s; memcpy(&s,&sb,4); return p*s; }
static inline float e6(float x){
  float xc=fminf(fmaxf(x,-87.f),88.f); float kf=fmaf(xc,1.44269502f,12582912.0f); float k=kf-12582912.0f;
  float r=fmaf(-k,0.693145751953125f,xc); r=fmaf(-k,1.42860677e-06f,r);
  float p=C6; p=fmaf(p,r,C5); p=fmaf(p,r,C4); p=fmaf(p,r,C3); p=fmaf(p,r,C2); p=fmaf(p,r,1.0f); p=fmaf(p,r,1.0f);
  uint32_t kb; memcpy(&kb,&kf,4); uint32_t sb=(kb<<23)+0x3f800000u; float s; memcpy(&s,&sb,4); return p*s; }
int main(int argc,char**argv){
  C2=atof(argv[1]);C3=atof(argv[2]);C4=atof(argv[3]);C5=atof(argv[4]);C6=atof(argv[5]);
  double m7=0,m6=0; long n=0,cr7=0,cr6=0;
  float lo = -87.0f; uint32_t lob; memcpy(&lob,&lo,4);
  #pragma omp parallel for reduction(max:m7,m6) reduction(+:n,cr7,cr6) schedule(static)
  for (long b=0x80000001L; b<=(long)lob; b+=1) {
    uint32_t u=(uint32_t)b; float x; memcpy(&x,&u,4);
    double ref=exp((double)x); float rf=(float)ref; double ulp=nextafterf(rf,INFINITY)-rf;
    float a=e7(x), c=e6(x);
    double d7=fabs(a-ref)/ulp, d6=fabs(c-ref)/ulp;
    if(d7>m7)m7=d7; if(d6>m6)m6=d6; n++; cr7+=(a==rf); cr6+=(c==rf);
  }
  printf("n=%ld deg7: max %.3f ulp, CR %.4f%% | deg6: max %.3f ulp, CR %.4f%%\n",n,m7,100.0*cr7/n,m6,100.0*cr6/n);
}
