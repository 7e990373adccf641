// PC (S7 by guess and verify) simulator, faithful to n4_shared.h pcw_run: NB blocks of consecutive
// steps, pass-0 guesses from the double running mean / variance, phase A stage 0 (mu alone,
// certified float steps), stage 1 (mu and sig), phase B (exact rounds), the affine guess update of
// pcw_update.  S7 arithmetic: ITK's roundings with the float counter frozen at 2^24
// (oracle/n4_oracle.c conv_welford).  Input: the file the C oracle's N4_DUMP_D hook writes (per
// iteration: int64 n, n floats d in raster order).  Prints rounds per iteration and stage.
// build: gcc -O2 -ffp-contract=off -o /tmp/pc_sim2 scripts/dev/pc_sim2.c -lm
// run:   /tmp/pc_sim2 D.bin [NB=1024] [GUESS=0]
//   GUESS 0: double running mean (the GPU's); 1: the previous iteration's exact float block starts
//   shifted by the change of the double running mean ("drift carried over")
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int NB, GUESS;
static int64_t n;
static float *p;
static double *Nd;   // ITK's N per step (1-based)
static float *MT;    // exact float mu after step k (debug)
static int DIT, CUR_IT;
static double *DR;
static long NOCAND;

static inline void step_exact(int64_t k, float *mu, float *sg) {
    const double N = Nd[k], r = 1.0 / N;
    if (k > 1) {
        const float q = p[k] - *mu;
        *sg = (float)((double)*sg + ((double)(q * q) * (N - 1.0)) / N);
    }
    *mu = (float)((double)*mu * (1.0 - r) + (double)(p[k] / (float)N));
}
static long NUNC;
// phase-A step (float-float constants, certified mu; sig uncertified), as pc_apx_step
static inline int step_apx(int64_t k, float e0, float *mu, float *sg, int sig) {
    const float kf = (float)Nd[k];
    const float r0 = 1.0f / kf, rl = r0 * fmaf(-kf, r0, 1.0f);
    const float pk = p[k], B = fmaf(pk, r0, pk * rl), ch = 1.0f - r0, cl = ((-r0) - (ch - 1.0f)) - rl;
    if (sig && k > 1) {
        const float q = pk - *mu, q2 = q * q;
        const float y = fmaf(q2, ch, *sg), rho = fmaf(q2, ch, *sg - y);
        *sg = y + fmaf(q2, cl, rho);
    }
    const float t1 = fmaf(-*mu, r0, B), t = fmaf(-*mu, rl, t1);
    const float E = fmaf(fabsf(t), 0x1p-21f, e0);
    const float ya = *mu + (t - E), yb = *mu + (t + E);
    *mu = ya;
    return ya == yb;
}

typedef struct { float g, gs, e, es, go, eo, lg, lgs; int64_t k0, len; } Blk;
static long NEVAL[3];
// ---- faithful emulation of n4_shared.h pcx_tpass + pcx_scan (run right after stage 0) ----------------
static int binade_f(float f) { uint32_t u; memcpy(&u, &f, 4); int be = (u >> 23) & 0xff; return (f > 0.0f && be > 0 && be < 255) ? be - 127 : -200; }
typedef struct { double C[3]; int tie[3]; int e0, cand, slot; float emu; } GX;
static int gpu_pcx(Blk *B, int nbe, int64_t L, float *sig_out, int *walks_out, const char **why) {
    static GX X[1 << 16];
    static double *TB = NULL; if (!TB) TB = malloc(8 * 40000000);
    const int64_t tcap = n / 2;
    int slots = 0;
    static double QS[1 << 16];
    for (int j = 0; j < nbe; ++j) {   // stage 0's per-block sum (p - mu)^2 (here along the exact mu)
        float mu = B[j].g; float qs = 0.0f;
        for (int64_t s2 = 0; s2 < B[j].len; ++s2) {
            const int64_t k = B[j].k0 + s2; const double N = Nd[k];
            const float dq = p[k] - mu; if (k > 1) qs = fmaf(dq, dq, qs);
            mu = (float)((double)mu * (1.0 - 1.0 / N) + (double)(p[k] / (float)N));
        }
        QS[j] = qs;
    }
    double pref = 0.0;
    for (int j = 0; j < nbe; ++j) {
        Blk *b = &B[j];
        const float gs = b->gs, gsn = j + 1 < nbe ? B[j + 1].gs : gs;
        const int e0 = binade_f((float)pref);
        pref += QS[j];
        double C[3] = {0, 0, 0}; int tie[3] = {0, 0, 0};
        float mu = b->g;
        for (int64_t s2 = 0; s2 < b->len; ++s2) {
            const int64_t k = b->k0 + s2; const double N = Nd[k];
            double t = 0.0;
            if (k > 1) { const float q = p[k] - mu; t = ((double)(q * q) * (N - 1.0)) / N; }
            if (e0 >= -125) for (int i = 0; i < 3; ++i) {
                const double Y = rint(ldexp(t, 52 - (e0 - 1 + i)));
                const double hi = floor(Y * 0x1p-29), rem = Y - hi * 0x1p29;
                tie[i] |= rem == 0x1p28; C[i] += hi + (rem > 0x1p28 ? 1.0 : 0.0);
            }
            mu = (float)((double)mu * (1.0 - 1.0 / N) + (double)(p[k] / (float)N));
        }
        X[j].emu = mu;
        const int cand = 0; (void)gsn;
        int slot = -1;
        if (cand) { int sl = slots++; if ((sl + 1) * (L + 1) <= tcap) slot = sl; }
        if (slot >= 0) {   // second pass: store t
            float mu2 = b->g;
            for (int64_t s2 = 0; s2 < b->len; ++s2) {
                const int64_t k = b->k0 + s2; const double N = Nd[k];
                double t = 0.0;
                if (k > 1) { const float q = p[k] - mu2; t = ((double)(q * q) * (N - 1.0)) / N; }
                TB[slot * (L + 1) + s2] = t;
                mu2 = (float)((double)mu2 * (1.0 - 1.0 / N) + (double)(p[k] / (float)N));
            }
        }
        for (int i = 0; i < 3; ++i) { X[j].C[i] = fmin(C[i], 1073741824.0); X[j].tie[i] = tie[i]; }
        X[j].e0 = e0; X[j].cand = cand; X[j].slot = slot;
    }
    for (int j = 0; j < nbe - 1; ++j) if (X[j].emu != B[j + 1].g) { *why = "mu verify"; return 0; }
    float s = 0.0f; int j = 0, walks = 0;
    while (j < nbe) {
        const int e = binade_f(s);
        double pre = 0.0; int first = 64; double endv[64];
        for (int l = 0; l < 64; ++l) {
            const int jj = j + l; const int have = jj < nbe;
            int ok = 0; double inc = 0.0;
            if (have && e >= -125) {
                const int c = e - X[jj].e0 + 1;
                ok = !X[jj].cand && c >= 0 && c < 3 && !X[jj].tie[c];
                inc = ok ? (double)(int32_t)X[jj].C[c] : 0.0;
            }
            pre += inc;
            const double ulp = ldexp(1.0, e - 23), lim = ldexp(1.0, e + 1) - ulp;
            endv[l] = (double)s + pre * ulp;
            ok = ok && endv[l] < lim;
            if (!(ok || !have) && first == 64) first = l;
        }
        if (first > 0) { int last = (first < nbe - j ? first : nbe - j) - 1; s = (float)endv[last]; j += last + 1; continue; }
        if (j > 0 && e >= -125 && !(e - X[j].e0 + 1 >= 0 && e - X[j].e0 + 1 < 3)) {
            static char buf[200];
            const int c = e - X[j].e0 + 1;
            snprintf(buf, sizeof buf, "walk of non-candidate j %d (s %.9g binade %d, e0 %d, c %d, C %.0f tie %d, gs %.9g gsn %.9g)", j, s, e, X[j].e0, c,
                     (c >= 0 && c < 3) ? X[j].C[c] : -1.0, (c >= 0 && c < 3) ? X[j].tie[c] : -1, B[j].gs, j + 1 < nbe ? B[j + 1].gs : 0.0f);
            *why = buf; return 0;
        }
        {   // recompute the block's mu trajectory and t exactly
            float mu2 = B[j].g;
            for (int64_t s2 = 0; s2 < B[j].len; ++s2) {
                const int64_t k = B[j].k0 + s2; const double N = Nd[k];
                double t = 0.0;
                if (k > 1) { const float q = p[k] - mu2; t = ((double)(q * q) * (N - 1.0)) / N; }
                s = (float)((double)s + t);
                mu2 = (float)((double)mu2 * (1.0 - 1.0 / N) + (double)(p[k] / (float)N));
            }
        }
        walks++; j++;
    }
    *sig_out = s; *walks_out = walks; *why = "ok";
    return 1;
}


static void run_block(Blk *b, int mode /* 0 apx mu, 1 apx both, 2 exact */) {
    if (mode < 2 && b->lg == b->g && b->lgs == b->gs) return;   // unchanged start: keep the end
    NEVAL[mode]++;
    b->lg = b->g;
    b->lgs = b->gs;
    float mu = b->g, sg = b->gs;
    const float sg_in = sg;
    if (mode == 2) {
        for (int64_t s = 0; s < b->len; ++s) step_exact(b->k0 + s, &mu, &sg);
    } else {
        const float e0 = fmaf(1.0f / (float)Nd[b->k0], 0x1p-39f, 0x1p-44f);
        int64_t s = 0;
        for (; s + 8 <= b->len; s += 8) {
            float m0 = mu, s0 = sg;
            int ok = 1;
            for (int i = 0; i < 8; ++i) ok &= step_apx(b->k0 + s + i, e0, &mu, &sg, mode == 1);
            if (!ok) {
                NUNC++;
                mu = m0;
                sg = s0;
                for (int i = 0; i < 8; ++i) step_exact(b->k0 + s + i, &mu, &sg);
            }
        }
        for (; s < b->len; ++s) step_exact(b->k0 + s, &mu, &sg);
        if (mode == 0) sg = sg_in;
    }
    b->e = mu;
    b->es = sg;
}

// one check/update (pcw_update); returns 1 when every transition matched
static int update(Blk *B, int nbe, int round, int use_sig) {
    int bad = 0;
    double dm = 0.0, ds = 0.0;
    static float ng[1 << 16], ngs[1 << 16], AF[1 << 16], GO[1 << 16], EO[1 << 16];
    for (int j = 0; j < nbe - 1; ++j) {
        Blk *b = &B[j];
        const int mm = b->e != B[j + 1].g || (use_sig && b->es != B[j + 1].gs);
        bad += mm;
        const double bm = (double)b->e - B[j + 1].g, bs = use_sig ? (double)b->es - B[j + 1].gs : 0.0;
        float af = (float)(b->k0 - 1) / (float)(b->k0 + b->len - 1);
        GO[j] = b->go; EO[j] = b->eo;
        static int SL = -1;
        if (SL < 0) SL = getenv("SLOPE") ? atoi(getenv("SLOPE")) : 0;
        if (SL == 1) af = 1.0f;
        else if (round > 0 && b->g != b->go) {
            const float sl = (b->e - b->eo) / (b->g - b->go);
            if (sl >= 0.0f && sl <= 1.0f) af = sl;
            else if (SL == 2 && sl > 1.0f) af = 1.0f;
            else if (SL == 3 && sl > 1.0f && sl < 1.5f) af = 1.0f;
        }
        AF[j] = af;
        b->go = b->g;
        b->eo = b->e;
        ng[j + 1] = dm == 0.0 ? b->e : (float)((double)b->e + af * dm);
        ngs[j + 1] = ds == 0.0 ? b->es : (float)((double)b->es + ds);
        dm = af * dm + bm;
        ds = ds + bs;
    }
    if (getenv("DBG")) {
        int bmu = 0, bsg = 0, fmu = -1, fsg = -1, binx = 0;
        for (int j = 0; j < nbe - 1; ++j) {
            if (B[j].e != B[j + 1].g) { bmu++; if (fmu < 0) fmu = j; }
            if (B[j].es != B[j + 1].gs) { bsg++; if (fsg < 0) fsg = j; }
        }
        fprintf(stderr, "   round %d sig %d: mu bad %d (first %d) sig bad %d (first %d)\n", round, use_sig, bmu, fmu, bsg, fsg);
        if (CUR_IT == DIT && !use_sig && fmu >= 0) {
            for (int j = fmu; j < fmu + 48 && j < nbe - 1; ++j) {
                const Blk *b = &B[j];
                const double u = 5.96e-8;
                fprintf(stderr, "      j %4d gerr %8.1f eerr %8.1f next-gerr %8.1f g-go %8.1f e-eo %8.1f af %.6f\n", j,
                        ((double)b->g - MT[b->k0 - 1]) / u, ((double)b->e - MT[b->k0 + b->len - 1]) / u,
                        ((double)B[j + 1].g - MT[B[j + 1].k0 - 1]) / u, ((double)b->g - GO[j]) / u, ((double)b->e - EO[j]) / u, AF[j]);
            }
        }
        (void)binx;
    }
    if (!bad) return 1;
    for (int j = 1; j < nbe; ++j) {
        B[j].g = ng[j];
        if (use_sig) B[j].gs = ngs[j];
    }
    return 0;
}

int main(int argc, char **argv) {
    setvbuf(stdout, NULL, _IONBF, 0);
    FILE *f = fopen(argv[1], "rb");
    NB = argc > 2 ? atoi(argv[2]) : 1024;
    GUESS = argc > 3 ? atoi(argv[3]) : 0;
    DIT = getenv("DIT") ? atoi(getenv("DIT")) : -1;
    const int64_t CAP = 40000000;
    float *d = malloc(4 * CAP);
    p = malloc(4 * (CAP + 1));
    Nd = malloc(8 * (CAP + 1));
    float *mt = malloc(4 * (CAP + 1)), *st = malloc(4 * (CAP + 1));
    MT = mt;
    DR = malloc(8 * (CAP + 1));
    double *dmean = malloc(8 * (CAP + 1)), *pmean = malloc(8 * (CAP + 1));
    float *pmt = malloc(4 * (CAP + 1));
    int have_prev = 0;
    int64_t nprev = 0;
    Blk *B = calloc(NB, sizeof(Blk));
    int it = 0;
    double tA0 = 0, tA1 = 0, tB = 0, terr = 0;
    while (fread(&n, 8, 1, f) == 1) {
        if (fread(d, 4, n, f) != (size_t)n) break;
        it++;
        CUR_IT = it;
        float N = 0.0f;
        for (int64_t k = 1; k <= n; ++k) {
            p[k] = (float)exp((double)d[k - 1]);
            N = (float)((double)N + 1.0);
            Nd[k] = N;
        }
        float mu = 0, sg = 0;
        double m = 0;
        mt[0] = st[0] = 0;
        dmean[0] = 0;
        for (int64_t k = 1; k <= n; ++k) {
            step_exact(k, &mu, &sg);
            mt[k] = mu;
            st[k] = sg;
            m += ((double)p[k] - m) / (double)k;
            dmean[k] = m;
        }
        if (GUESS == 2) {   // predicted float drift: quantised increments against the exact mean
            double D = 0.0, mm = 0.0;
            DR[0] = 0.0;
            for (int64_t k = 1; k <= n; ++k) {
                const double N = Nd[k];
                const double inc = ((double)p[k] - mm) / N;
                const float mf = (float)(mm + D);            // float estimate of mu before the step
                const double ulp = (double)nextafterf(mf, 2.0f) - (double)mf;
                const double rinc = ulp * rint(inc / ulp);   // the float step moves by whole ulps
                D = D * (1.0 - 1.0 / N) + (rinc - inc);
                mm += inc;
                DR[k] = D;
            }
        }
        const int64_t L = n / NB, rem = n % NB;
        const int nbe = L ? NB : (int)rem;
        double S1 = 0, S2 = 0;
        int64_t k0 = 1;
        double maxerr = 0;
        for (int j = 0; j < nbe; ++j) {
            Blk *b = &B[j];
            b->k0 = k0;
            b->len = L + (j < rem);
            const double K = (double)(k0 - 1);
            float g = 0, gs = 0;
            if (K > 0) {
                g = (float)(1.0 + S1 / K);
                const double v = S2 - S1 * (S1 / K);
                gs = (float)(v > 0 ? v : 0);
            }
            if (GUESS == 2 && K > 0) g = (float)(1.0 + S1 / K + DR[k0 - 1]);
            if (GUESS == 1 && have_prev && K > 0) {
                // previous iteration's float drift at the same relative position
                const int64_t kp = (int64_t)((double)(k0 - 1) * (double)nprev / (double)n);
                if (kp > 0) g = (float)((double)g + ((double)pmt[kp] - pmean[kp]));
            }
            b->g = g;
            b->gs = gs;
            b->go = b->eo = NAN;
            b->lg = b->lgs = NAN;
            const double err = fabs((double)g - mt[k0 - 1]) / 5.96e-8;
            if (err > maxerr) maxerr = err;
            for (int64_t s = 0; s < b->len; ++s) {
                const double e = (double)p[k0 + s] - 1.0;
                S1 += e;
                S2 = fma(e, e, S2);
            }
            k0 += b->len;
        }
        terr += maxerr;
        int ra[2] = {0, 0}, rb = 0, round = 0;
        static int XS = -1;
        if (XS < 0) XS = getenv("XSIG") ? atoi(getenv("XSIG")) : 0;
        for (int stage = 0; stage < 2; ++stage) {
            if (stage == 1 && getenv("GPX")) {
                float sg; int w; const char *why;
                const int ok = gpu_pcx(B, nbe, L, &sg, &w, &why);
                printf("   gpu-pcx: %s walks %d %s\n", ok ? "OK" : "FAIL", ok ? w : -1, ok ? (sg == st[n] ? "EXACT" : "WRONG") : why);
            }
            for (int j = 0; j < nbe; ++j) B[j].lg = NAN;   // a new stage re-evaluates every block
            for (int r = 0; r < 40; ++r, ++round) {
                for (int j = 0; j < nbe; ++j) run_block(&B[j], stage);
                ra[stage]++;
                if (update(B, nbe, round, stage == 1)) break;
            }
        }
        if (XS) {   // exact sig: stage 0 done; T pass (exact mu verify, t_k, per-binade integer sums) + scan
            static double *T = NULL;
            if (!T) T = malloc(8 * (CAP + 1));
            int mubad = 0;
            typedef struct { int e0; int64_t C[3]; int tie[3]; } Xs;
            static Xs X[1 << 16];
            for (int j = 0; j < nbe; ++j) {
                Blk *b = &B[j];
                float mu = b->g;
                for (int64_t st2 = 0; st2 < b->len; ++st2) {
                    const int64_t k = b->k0 + st2;
                    const double N = Nd[k];
                    if (k > 1) {
                        const float q = p[k] - mu;
                        T[k] = ((double)(q * q) * (N - 1.0)) / N;
                    } else T[k] = 0.0;
                    mu = (float)((double)mu * (1.0 - 1.0 / N) + (double)(p[k] / (float)N));
                }
                if (j + 1 < nbe && mu != B[j + 1].g) mubad++;
                if (j + 1 == nbe && mu != mt[n]) mubad++;
                int e0;
                frexpf(b->gs > 0 ? b->gs : 1e-30f, &e0);
                e0 -= 1;   // gs in [2^e0, 2^(e0+1))
                X[j].e0 = e0;
                for (int c = 0; c < 3; ++c) {
                    const int e = e0 - 1 + c;
                    int64_t Cs = 0; int tie = 0;
                    for (int64_t st2 = 0; st2 < b->len; ++st2) {
                        const double t = T[b->k0 + st2];
                        const double Y = rint(ldexp(t, 52 - e));           // RN_d grid units
                        const double q29 = ldexp(Y, -29);
                        const double fl = floor(q29), rem = Y - ldexp(fl, 29);
                        if (rem == 268435456.0) tie = 1;
                        Cs += (int64_t)fl + (rem > 268435456.0 ? 1 : 0);
                    }
                    X[j].C[c] = Cs; X[j].tie[c] = tie;
                }
            }
            // scan (sequential here; segments of equal binade are parallel integer prefix sums on the GPU)
            float sg = 0.0f;
            int walks = 0, ties = 0, binmiss = 0;
            for (int j = 0; j < nbe; ++j) {
                Blk *b = &B[j];
                int e; frexpf(sg, &e); e -= 1;
                const int c = e - (X[j].e0 - 1);
                int ok = j > 0 && sg > 0.0f && c >= 0 && c < 3 && !X[j].tie[c];
                if (j > 0 && sg > 0.0f && !(c >= 0 && c < 3)) binmiss++;
                if (ok && X[j].tie[c]) ties++;
                double ulp = ldexp(1.0, e - 23);
                if (ok) {
                    const double v = (double)sg + (double)X[j].C[c] * ulp;
                    if (v < ldexp(1.0, e + 1) - ulp) sg = (float)v; else ok = 0;
                }
                if (!ok) {   // walk the block exactly
                    walks++;
                    {
                        int eg, eg1;
                        frexpf(B[j].gs, &eg);
                        frexpf(j + 1 < nbe ? B[j + 1].gs : B[j].gs, &eg1);
                        const int cand = j == 0 || j == nbe - 1 || !(B[j].gs > 0) || eg != eg1;
                        if (!cand) {
                            NOCAND++;
                            if (getenv("XDBG2")) fprintf(stderr, "uncovered j %d start %.9g end-guess %.9g gs %.9g gs1 %.9g true-end %.9g\n", j, sg, 0.0, B[j].gs, j + 1 < nbe ? B[j + 1].gs : 0.0f, 0.0);
                        }
                    }
                    if (getenv("XDBG")) {
                        int eg, eg1; frexpf(B[j].gs, &eg); frexpf(j + 1 < nbe ? B[j + 1].gs : 1e30f, &eg1);
                        fprintf(stderr, "      walk j %d start %.6g binade %d guess-binades %d %d\n", j, sg, e, eg - 1, eg1 - 1);
                    }
                    for (int64_t st2 = 0; st2 < b->len; ++st2) {
                        const int64_t k = b->k0 + st2;
                        if (k > 1) sg = (float)((double)sg + T[k]);
                    }
                }
            }
            const int sok = sg == st[n];
            printf("   xsig: mu verify bad %d, walks %d, binade misses %d, ties %d, sig %s, uncovered walks so far %ld\n", mubad, walks, binmiss, ties, sok ? "EXACT" : "WRONG", NOCAND);
        }
        for (int r = 0; r < 48; ++r) {
            ++round;
            for (int j = 0; j < nbe; ++j) run_block(&B[j], 2);
            rb++;
            if (update(B, nbe, round, 1)) break;
        }
        int ok = B[nbe - 1].e == mt[n] && B[nbe - 1].es == st[n];
        printf("it %2d n %lld: guess maxerr %.0f ulp, stage0 %d stage1 %d exact %d %s\n", it, (long long)n,
               maxerr, ra[0], ra[1], rb, ok ? "ok" : "MISMATCH");
        tA0 += ra[0];
        tA1 += ra[1];
        tB += rb;
        memcpy(pmt, mt, 4 * (n + 1));
        memcpy(pmean, dmean, 8 * (n + 1));
        nprev = n;
        have_prev = 1;
    }
    printf("mean rounds: stage0 %.2f stage1 %.2f exact %.2f; guess maxerr %.0f ulp; uncertified groups/it %.1f\n",
           tA0 / it, tA1 / it, tB / it, terr / it, (double)NUNC / it);
    printf("block evaluations per iteration (in units of all %d blocks): stage0 %.2f stage1 %.2f exact %.2f\n", NB,
           (double)NEVAL[0] / it / NB, (double)NEVAL[1] / it / NB, (double)NEVAL[2] / it / NB);
    return 0;
}
