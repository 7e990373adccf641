// S7 decision by interval enclosure (design study for the study kernel's PC, round 5).
// For each iteration's d sequence (the C oracle's N4_DUMP_D file: int64 n, n floats d in raster
// order), with NL blocks of consecutive steps (the GPU's layout):
//   1. exact serial float Welford (the spec's roundings): block starts, mu_n, sig_n, conv;
//   2. guesses: the double running mean at each block start + the previous iteration's drift;
//   3. R point rounds with exact steps and the GPU's affine update (pcw_update);
//   4. interval rounds: each block runs a lower and an upper trajectory from [L_j, H_j] with the
//      float-float step t = B - m (r0 + rl) and its error bound E (pc_apx_step): lower end
//      RN(m + RN(t - E)), upper RN(m + RN(t + E)).  Each step map is monotone, so if every block's
//      end interval lies inside the next block's start interval, the true trajectory is enclosed
//      (block 0 starts exactly at 0);
//   5. decision: sig >= lo from sums of q_lo^2 (q_lo = distance of p to [lo, hi]), the measure at
//      (mu_hi one float up, RD(lo)) > threshold certifies "continue".
// Reports per iteration: rounds, interval widths, whether the decision certified, and what the
// current scheme (exact mu after stage 0, the same sig bound from the exact trajectory) gives.
// build: gcc -O2 -ffp-contract=off -o /tmp/pcis scripts/dev/pc_interval_sim.c -lm
// run:   /tmp/pcis D.bin [NL=1024] [RPRE=2] [SLACK=2] [THRESH=0.001]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NMAX 16777216.0
static int NL = 1024, RPRE = 2;
static double SLACK = 2.0, THRESH = 0.001;

static inline double Nd(int64_t k) { return k < NMAX ? (double)k : NMAX; }
static inline float ulpf(float x) { return nextafterf(fabsf(x), INFINITY) - fabsf(x); }

static inline void step_exact(int64_t k, float p, float *mu, float *sig) {
    const double N = Nd(k), r = 1.0 / N;
    if (k > 1) {
        const float d = p - *mu;
        const double q = ((double)(d * d) * (N - 1.0)) / N;
        *sig = (float)((double)*sig + q);
    }
    const double A = 1.0 - r, B = (double)(float)((double)p * r);
    *mu = (float)((double)*mu * A + B);
}

typedef struct { float r0, rl, B; } Kf;
static inline Kf kf_of(float k, float p) {
    Kf q;
    q.r0 = 1.0f / k;
    q.rl = q.r0 * fmaf(-k, q.r0, 1.0f);
    q.B = fmaf(p, q.r0, p * q.rl);
    return q;
}
// one interval step: [lo, hi] -> enclosure of f([lo, hi]); q_lo^2 summed into *s
static inline void step_iv(float kf, float e0, float p, int first, float *lo, float *hi, float *s) {
    if (!first) {
        float q = 0.0f;
        if (p > *hi) q = p - *hi;
        else if (p < *lo) q = *lo - p;
        *s = fmaf(q, q, *s);
    }
    const Kf c = kf_of(kf, p);
    float t = fmaf(-*lo, c.r0, c.B);
    t = fmaf(-*lo, c.rl, t);
    float E = fmaf(fabsf(t), 0x1p-21f, e0);
    *lo = *lo + (t - E);
    t = fmaf(-*hi, c.r0, c.B);
    t = fmaf(-*hi, c.rl, t);
    E = fmaf(fabsf(t), 0x1p-21f, e0);
    *hi = *hi + (t + E);
}

int main(int argc, char **argv) {
    if (argc < 2) return 1;
    if (argc > 2) NL = atoi(argv[2]);
    if (argc > 3) RPRE = atoi(argv[3]);
    if (argc > 4) SLACK = atof(argv[4]);
    if (argc > 5) THRESH = atof(argv[5]);
    FILE *f = fopen(argv[1], "rb");
    int64_t n;
    float *drift = calloc(NL, sizeof(float));
    int have_drift = 0, it = 0;
    int tot_cert = 0, tot_cur = 0, tot_above = 0, tot_iv_ok = 0, tot_it = 0, tot_ivr = 0;
    int tot_fix = 0, tot_fix_cert = 0, tot_new = 0, tot_adapt = 0;
    while (fread(&n, sizeof n, 1, f) == 1) {
        float *d = malloc(sizeof(float) * n), *p = malloc(sizeof(float) * n);
        if (fread(d, sizeof(float), n, f) != (size_t)n) return 2;
        for (int64_t i = 0; i < n; ++i) p[i] = (float)exp((double)d[i]);
        const int64_t L = n / NL, rem = n % NL;
        int64_t *k0 = malloc(sizeof(int64_t) * NL), *len = malloc(sizeof(int64_t) * NL);
        for (int j = 0; j < NL; ++j) {
            len[j] = L + (j < rem);
            k0[j] = (int64_t)j * L + (j < rem ? j : rem) + 1;
        }
        const int nbe = L ? NL : (int)rem;
        // 1. exact
        float *S = malloc(sizeof(float) * NL), *SS = malloc(sizeof(float) * NL);
        float mu = 0, sig = 0;
        for (int j = 0; j < nbe; ++j) {
            S[j] = mu;
            SS[j] = sig;
            for (int64_t s = 0; s < len[j]; ++s) step_exact(k0[j] + s, p[k0[j] - 1 + s], &mu, &sig);
        }
        const float conv = (float)sqrt((double)sig / (Nd(n) - 1.0)) / mu;
        // current scheme's bound: the exact trajectory's q^2 block sums
        double wb_cur = 0;
        for (int j = 0; j < nbe; ++j) {
            float m = S[j], sg = 0, bs = 0;
            for (int64_t s = 0; s < len[j]; ++s) {
                const int64_t k = k0[j] + s;
                const float pp = p[k - 1];
                if (k > 1) { const float q = pp - m; bs = fmaf(q, q, bs); }
                step_exact(k, pp, &m, &sg);
            }
            if (k0[j] > 1) wb_cur += (double)bs * (1.0 - 1.0 / fmin((double)k0[j], NMAX));
        }
        const double fct = 1.0 - ((double)n + (double)L + 8.0) * 0x1p-24;
        float sl_cur = (float)(wb_cur * fct);
        if ((double)sl_cur > wb_cur * fct) sl_cur = nextafterf(sl_cur, 0);
        const float muh_cur = nextafterf(mu, INFINITY);
        const int cur = (float)sqrt((double)sl_cur / (Nd(n) - 1.0)) / muh_cur > THRESH;
        // 2. guesses
        float *g = malloc(sizeof(float) * NL), *e = malloc(sizeof(float) * NL), *go = malloc(sizeof(float) * NL),
              *eo = malloc(sizeof(float) * NL);
        double *gd = malloc(sizeof(double) * NL);
        double cum = 0;
        for (int j = 0; j < nbe; ++j) {
            const double K = (double)(k0[j] - 1);
            gd[j] = K > 0 ? 1.0 + cum / K : 0.0;
            g[j] = K > 0 ? (float)(gd[j] + (have_drift ? (double)drift[j] : 0.0)) : 0.0f;
            for (int64_t s = 0; s < len[j]; ++s) cum += (double)p[k0[j] - 1 + s] - 1.0;
        }
        // 3. point rounds (exact steps, affine update)
        int r;
        const int ADAPT = getenv("ADAPT") ? atoi(getenv("ADAPT")) : 0;
        const double WLIM = getenv("WLIM") ? atof(getenv("WLIM")) : 4000;
        int adapt_done = 0, adapt_round = -1, fixed_round = -1, adapt_tries = 0;
        float *ael = malloc(sizeof(float) * NL), *aeh = malloc(sizeof(float) * NL), *abs_ = malloc(sizeof(float) * NL);
        for (r = 0; r < (ADAPT ? 64 : RPRE); ++r) {
            for (int j = 0; j < nbe; ++j) {
                float m = g[j], sg = 0;
                for (int64_t s = 0; s < len[j]; ++s) step_exact(k0[j] + s, p[k0[j] - 1 + s], &m, &sg);
                e[j] = m;
            }
            if (ADAPT && !adapt_done) {   // predicted widths: W_{j+1} = a W_j + |e_j - g_{j+1}| + slack
                double Wp = 0, wmx = 0;
                float *alo = malloc(sizeof(float) * NL), *ahi = malloc(sizeof(float) * NL);
                alo[0] = ahi[0] = 0.0f;
                for (int j = 0; j < nbe - 1; ++j) {
                    const double a = (double)(k0[j] - 1) / (double)(k0[j] + len[j] - 1);
                    Wp = a * Wp + fabs((double)e[j] - (double)g[j + 1]) + SLACK * ulpf(g[j + 1]);
                    alo[j + 1] = (float)((double)g[j + 1] - Wp);
                    ahi[j + 1] = (float)((double)g[j + 1] + Wp);
                    wmx = fmax(wmx, Wp / ulpf(g[j + 1]));
                }
                if (wmx < WLIM) {
                    adapt_tries++;
                    int okk = 1;
                    for (int j = 0; j < nbe; ++j) {
                        float l = alo[j], h = ahi[j], sm = 0;
                        const float kf0 = (float)(k0[j] < NMAX ? k0[j] : NMAX);
                        const float e0 = fmaf(1.0f / kf0, 0x1p-39f, 0x1p-44f);
                        for (int64_t st = 0; st < len[j]; ++st) {
                            const int64_t k = k0[j] + st;
                            step_iv((float)(k < NMAX ? k : NMAX), e0, p[k - 1], k == 1, &l, &h, &sm);
                        }
                        ael[j] = l; aeh[j] = h; abs_[j] = sm;
                        if (j + 1 < nbe && (l < alo[j + 1] || h > ahi[j + 1])) okk = 0;
                        if (!(alo[j] <= S[j] && S[j] <= ahi[j]) && okk) printf("  ADAPT ENCLOSURE VIOLATED\n");
                    }
                    if (okk) {
                        double wb = 0;
                        for (int j = 0; j < nbe; ++j)
                            if (k0[j] > 1) wb += (double)abs_[j] * (1.0 - 1.0 / fmin((double)k0[j], NMAX));
                        float sl = (float)(wb * fct);
                        if ((double)sl > wb * fct) sl = nextafterf(sl, 0);
                        if (sl > sig) printf("  ADAPT SIG BOUND VIOLATED\n");
                        const float mh = nextafterf(aeh[nbe - 1], INFINITY);
                        if ((float)sqrt((double)sl / (Nd(n) - 1.0)) / mh > THRESH) { adapt_done = 1; adapt_round = r; }
                    }
                }
                free(alo); free(ahi);
            }
            double dm = 0;
            int any = 0;
            float *gr = malloc(sizeof(float) * NL);   // this round's guesses (read before any write)
            memcpy(gr, g, sizeof(float) * NL);
            for (int j = 0; j < nbe - 1; ++j) {
                const double bm = (double)e[j] - (double)gr[j + 1];
                any |= e[j] != gr[j + 1];
                float af = (float)(k0[j] - 1) / (float)(k0[j] + len[j] - 1);
                if (r > 0 && gr[j] != go[j]) {
                    const float sl = (e[j] - eo[j]) / (gr[j] - go[j]);
                    if (sl >= 0.0f && sl <= 1.0f) af = sl;
                }
                go[j] = gr[j];
                eo[j] = e[j];
                const float newg = dm == 0.0 ? e[j] : (float)((double)e[j] + (double)af * dm);
                dm = (double)af * dm + bm;
                g[j + 1] = newg;
            }
            go[nbe - 1] = gr[nbe - 1];
            free(gr);
            if (!any) { fixed_round = r; ++r; break; }
        }
        {   // diagnostics: the point guesses' true errors and last corrections, in ulps
            double emax = 0, emean = 0, cmax = 0, cmean = 0;
            int nz = 0;
            for (int j = 1; j < nbe; ++j) {
                const double u = ulpf(S[j] > 0 ? S[j] : 1.0f);
                const double er = fabs((double)g[j] - S[j]) / u, co = fabs((double)g[j] - (double)go[j]) / u;
                emax = fmax(emax, er); emean += er; cmax = fmax(cmax, co); cmean += co; nz += er > 0;
            }
            if (getenv("DIAG")) printf("  guesses: err max %.0f mean %.1f ulp (%d nonzero) | last corr max %.0f mean %.1f\n",
                   emax, emean / nbe, nz, cmax, cmean / nbe);
        }
        // 4. intervals around the current guesses: widths from the last correction's size
        float *lo = malloc(sizeof(float) * NL), *hi = malloc(sizeof(float) * NL), *el = malloc(sizeof(float) * NL),
              *eh = malloc(sizeof(float) * NL), *bsum = malloc(sizeof(float) * NL);
        double W = 0;
        lo[0] = hi[0] = 0.0f;
        const int MAXRULE = getenv("MAXRULE") ? atoi(getenv("MAXRULE")) : 1;
        const double CW = getenv("CW") ? atof(getenv("CW")) : 2.0;
        for (int j = 1; j < nbe; ++j) {
            const double corr = fabs((double)g[j] - (double)(r > 0 ? go[j] : g[j]));
            const double a = (double)(k0[j - 1] - 1) / (double)(k0[j - 1] + len[j - 1] - 1);
            W = MAXRULE ? fmax(a * W, CW * corr) + SLACK * ulpf(g[j]) : a * W + CW * corr + SLACK * ulpf(g[j]);
            lo[j] = (float)((double)g[j] - W);
            hi[j] = (float)((double)g[j] + W);
        }
        int ivr = 0, ok = 0;
        for (ivr = 1; ivr <= 3; ++ivr) {
            for (int j = 0; j < nbe; ++j) {
                float l = lo[j], h = hi[j], s = 0;
                const float kf0 = (float)(k0[j] < NMAX ? k0[j] : NMAX);
                const float e0 = fmaf(1.0f / kf0, 0x1p-39f, 0x1p-44f);
                for (int64_t st = 0; st < len[j]; ++st) {
                    const int64_t k = k0[j] + st;
                    step_iv((float)(k < NMAX ? k : NMAX), e0, p[k - 1], k == 1, &l, &h, &s);
                }
                el[j] = l;
                eh[j] = h;
                bsum[j] = s;
            }
            ok = 1;
            double ext_l = 0, ext_h = 0;
            for (int j = 0; j < nbe - 1; ++j) {
                const double a = (double)(k0[j] - 1) / (double)(k0[j] + len[j] - 1);
                const double vl = el[j] < lo[j + 1] ? (double)lo[j + 1] - el[j] : 0.0;
                const double vh = eh[j] > hi[j + 1] ? (double)eh[j] - hi[j + 1] : 0.0;
                if (vl > 0 || vh > 0) ok = 0;
                if (MAXRULE) {
                    ext_l = fmax(a * ext_l, vl > 0 ? 2 * vl + SLACK * ulpf(lo[j + 1]) : 0);
                    ext_h = fmax(a * ext_h, vh > 0 ? 2 * vh + SLACK * ulpf(hi[j + 1]) : 0);
                } else {
                    ext_l = a * ext_l + (vl > 0 ? 2 * vl + SLACK * ulpf(lo[j + 1]) : 0);
                    ext_h = a * ext_h + (vh > 0 ? 2 * vh + SLACK * ulpf(hi[j + 1]) : 0);
                }
                if (ext_l > 0) lo[j + 1] = (float)((double)lo[j + 1] - ext_l);
                if (ext_h > 0) hi[j + 1] = (float)((double)hi[j + 1] + ext_h);
            }
            if (getenv("DIAG2")) {
                int nv = 0; double mv = 0; int first = -1;
                for (int j = 0; j < nbe - 1; ++j) {
                    const double u = ulpf(hi[j + 1] > 0 ? hi[j + 1] : 1.0f);
                    const double v = fmax(el[j] < lo[j + 1] ? 0 : 0, 0);
                    (void)v;
                    if (!(S[j + 1] >= lo[j + 1] && S[j + 1] <= hi[j + 1])) { if (first < 0) first = j + 1; }
                    const double w = ((double)hi[j + 1] - lo[j + 1]) / u;
                    if (w > mv) mv = w;
                    nv += 0;
                }
                printf("    iv round %d: ok %d, first block not enclosing the truth (after widening) %d, max width %.0f ulp\n",
                       ivr, ok, first, mv);
            }
            if (ok) break;
        }
        int cert = 0;
        double wmax = 0;
        if (ok) {
            double wb = 0;
            for (int j = 0; j < nbe; ++j) {
                if (k0[j] > 1) wb += (double)bsum[j] * (1.0 - 1.0 / fmin((double)k0[j], NMAX));
                const double w = ((double)hi[j] - lo[j]) / ulpf(hi[j] > 0 ? hi[j] : 1.0f);
                if (w > wmax) wmax = w;
                if (!(lo[j] <= S[j] && S[j] <= hi[j])) printf("  ENCLOSURE VIOLATED j %d\n", j);
            }
            float sl = (float)(wb * fct);
            if ((double)sl > wb * fct) sl = nextafterf(sl, 0);
            const float mh = nextafterf(eh[nbe - 1], INFINITY);
            if (!(el[nbe - 1] <= mu && mu <= eh[nbe - 1])) printf("  END VIOLATED\n");
            if (sl > sig) printf("  SIG BOUND VIOLATED %g > %g\n", sl, sig);
            cert = fct > 0.5 && wb > 0 && eh[nbe - 1] > 0 && (float)sqrt((double)sl / (Nd(n) - 1.0)) / mh > THRESH;
        }
        if (ADAPT) {
            printf("it %2d conv %.6f %s | fixed point after %d rounds | interval cert after round %d (%d tries) | cur %d\n",
                   it, conv, conv > THRESH ? "above" : "BELOW", fixed_round + 1, adapt_done ? adapt_round + 1 : -1,
                   adapt_tries, cur);
            tot_fix += fixed_round + 1;
            if (cur) tot_fix_cert += fixed_round + 1;
            tot_new += adapt_done ? adapt_round + 1 + adapt_tries : fixed_round + 1 + adapt_tries;
            tot_adapt += adapt_done;
        }
        free(ael); free(aeh); free(abs_);
        printf("it %2d n %6lld conv %.6f %s | point rounds %d iv rounds %d %s maxw %.0f ulp | cert %d cur %d\n", it,
               (long long)n, conv, conv > THRESH ? "above" : "BELOW", r, ivr, ok ? "ok" : "FAIL", wmax, cert, cur);
        tot_it++;
        tot_above += conv > THRESH;
        tot_cert += cert;
        tot_cur += cur;
        tot_iv_ok += ok;
        tot_ivr += ok ? ivr : 0;
        // drift for the next iteration: exact starts minus the double mean
        for (int j = 0; j < nbe; ++j) drift[j] = (float)((double)S[j] - gd[j]);
        have_drift = 1;
        ++it;
        free(d); free(p); free(k0); free(len); free(S); free(SS); free(g); free(e); free(go); free(eo); free(gd);
        free(lo); free(hi); free(el); free(eh); free(bsum);
    }
    if (getenv("ADAPT"))
        printf("ADAPT: rounds to the fixed point %d; with interval attempts (each counted as a round) %d; certified by interval %d\n",
               tot_fix, tot_new, tot_adapt);
    printf("TOTAL its %d above %d | interval ok %d (mean rounds %.2f) cert %d | current scheme cert %d\n", tot_it,
           tot_above, tot_iv_ok, tot_iv_ok ? (double)tot_ivr / tot_iv_ok : 0.0, tot_cert, tot_cur);
    return 0;
}
