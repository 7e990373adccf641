// PC (S7 by guess and verify) simulator on real d sequences: phase A (certified float rounds) then
// phase B (exact rounds); prints rounds per iteration.  Input: the file written by the C oracle's
// N4_DUMP_D hook (each iteration: int64 n, n floats d in raster order).
// build: gcc -O2 -ffp-contract=off -o /tmp/pc_sim scripts/dev/pc_sim.c -lm;  run: /tmp/pc_sim D.bin NBLOCKS
// Phase A: approximate float steps (cheap), rounds to their own fixed point; Phase B: exact rounds.
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
static int NB; float *gmt; int64_t gL; static int64_t n, L; static float *p; static double *A,*Bx,*C;
static inline void step_exact(int64_t k, float *mu, float *sg){ if(k>1){float q=p[k]-*mu; *sg=(float)fma((double)(q*q),C[k],(double)*sg);} *mu=(float)fma((double)*mu,A[k],Bx[k]); }
static float MUG=1.0f; static long NUNC=0;
static inline void step_apx(int64_t k, float *mu, float *sg){ float kf=(float)k; float r0=1.0f/kf; float e=fmaf(-kf,r0,1.0f); float rl=r0*e;
  float pk=p[k]; float B=fmaf(pk,r0,pk*rl); float B2=fmaf(-MUG,rl,B); float ch=1.0f-r0; float cl=((-r0)-(ch-1.0f))-rl;
  if(k>1){ float q=pk-*mu; float q2=q*q; float y=fmaf(q2,ch,*sg); float rho=fmaf(q2,ch,*sg-y); float w=fmaf(q2,cl,rho); *sg=y+w; }
  float t=fmaf(-*mu,r0,B)-MUG*rl; float y=*mu+t; float rho=t-(y-*mu); float E=fabsf(t)*1.2e-7f+fabsf(*mu)*1e-12f;
  uint32_t yb; memcpy(&yb,&y,4); float ul; uint32_t ub=(yb&0x7f800000u)-(23u<<23); memcpy(&ul,&ub,4); if((yb&0x7fffffu)==0) ul*=0.5f;
  if(fabsf(rho)+E < 0.5f*ul) *mu=y; else { NUNC++; double kd=k; double r=1.0/kd; *mu=(float)fma((double)*mu,1.0-r,(double)(float)((double)pk*r)); } }
static int rounds(int exact, float *g, float *gs, int cap){
  static float e[65536], es[65536], gold[65536], eold[65536]; int havold=0;
  for(int r=0;r<cap;r++){
    for(int j=0;j<NB;j++){ int64_t a=(int64_t)j*L+1,b=a+L-1; if(b>n)b=n; float mu=g[j],sg=gs[j]; for(int64_t k=a;k<=b;k++){ if(exact) step_exact(k,&mu,&sg); else step_apx(k,&mu,&sg);} e[j]=mu; es[j]=sg; }
    int bad=0; for(int j=0;j+1<NB && (int64_t)(j+1)*L<n;j++) if(e[j]!=g[j+1]||es[j]!=gs[j+1]) bad++;
    if(getenv("DBG")&&exact){ extern float *gmt; extern int64_t gL; long me=0; for(int j=0;j<NB&&(int64_t)j*L<=n;j++){ long ee=(long)(fabs((double)g[j]-(double)gmt[(int64_t)j*L])/6e-8+0.5); if(ee>me)me=ee;} int bm=0,bs=0; long fs=-1; double rs=0; for(int j=0;j+1<NB && (int64_t)(j+1)*L<n;j++){ if(e[j]!=g[j+1])bm++; if(es[j]!=gs[j+1]){ if(fs<0){fs=j; rs=((double)es[j]-gs[j+1]);} bs++;} } fprintf(stderr,"  r%d bad %d (mu %d sig %d, first sig %ld resid %g ulp %g) maxerr %ld\n",r,bad,bm,bs,fs,rs, fs>=0? (double)nextafterf(gs[fs+1],1e30f)-gs[fs+1]:0.0, me);} 
    if(!bad) return r+1;
    double dl=0, ds=0; float gn[65536], gsn[65536]; gn[0]=g[0]; gsn[0]=gs[0];
    for(int j=0;j+1<NB;j++){ int64_t a=(int64_t)j*L+1,b=a+L-1; if(b>n)b=n; double sl=(double)(a-1)/(double)b;
      if(havold && g[j]!=gold[j]){ double s=((double)e[j]-eold[j])/((double)g[j]-gold[j]); if(s>=0&&s<=1) sl=s; }
      gn[j+1]= dl==0? e[j] : (float)((double)e[j]+sl*dl); gsn[j+1]= ds==0? es[j] : (float)((double)es[j]+ds);
      dl = sl*dl + ((double)e[j]-g[j+1]); ds = ds + ((double)es[j]-gs[j+1]); }
    memcpy(gold,g,4*NB); memcpy(eold,e,4*NB); havold=1; memcpy(g,gn,4*NB); memcpy(gs,gsn,4*NB);
  }
  return -1;
}
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); NB=atoi(argv[2]); int it=0;
  float *d=malloc(4*30000000); p=malloc(4*30000001); A=malloc(8*30000001);Bx=malloc(8*30000001);C=malloc(8*30000001);
  float *mt=malloc(4*30000001),*st=malloc(4*30000001); static float g[65536],gs[65536];
  long sa=0,sb=0;
  while(fread(&n,8,1,f)==1){ if(fread(d,4,n,f)!=(size_t)n)break; it++;
    for(int64_t k=1;k<=n;k++){ p[k]=(float)exp((double)d[k-1]); double kd=k; A[k]=1.0-1.0/kd; Bx[k]=(double)(p[k]/(float)k); C[k]=(kd-1.0)/kd; }
    gmt=mt; mt[0]=0; st[0]=0; float mu=0,sg=0; for(int64_t k=1;k<=n;k++){ step_exact(k,&mu,&sg); mt[k]=mu; st[k]=sg; }
    L=(n+NB-1)/NB;
    double m=0,s2=0; for(int64_t k=1;k<=n;k++){ if((k-1)%L==0){ g[(k-1)/L]=(float)m; gs[(k-1)/L]=(float)s2; } double dd=(double)p[k]-m; m+=dd/(double)k; s2+=dd*dd*(k-1)/(double)k; }
    g[0]=0; gs[0]=0;
    int ra=rounds(0,g,gs,60); int rb=rounds(1,g,gs,60);
    int ok = g[NB-1]==mt[(NB-1)*L] ; // loose check
    int ok2=1; for(int j=0;j<NB && (int64_t)j*L<=n;j++) if(g[j]!=mt[(int64_t)j*L]||gs[j]!=st[(int64_t)j*L]) ok2=0;
    printf("it %2d: approx rounds %d exact rounds %d exact-ok %d\n",it,ra,rb,ok2); sa+=ra; sb+=rb; (void)ok;
  }
  printf("uncertain steps per iteration %.2f\n",(double)NUNC/it); printf("mean approx %.1f exact %.1f\n",(double)sa/it,(double)sb/it);
}
