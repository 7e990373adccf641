// PC stage 0 (mu alone) round counts: the GPU's affine guess update (pcw_update: secant slopes in
// value space) against "certified translation windows": each block also returns the window
// [-Tm, Tp] (in ulps of its start) over which its map is an exact translation -- no step's rounding
// decision changes for any start shifted by delta inside it: the step's exact value shifts by
// delta (1 - 1/N) ulps, i.e. by delta ulps minus delta / N, so the rounding is kept while delta / N
// stays inside the step's distance to the rounding boundary, and no binade edge lies within delta
// of the trajectory.  The update then composes the blocks exactly (D_{j+1} = D_j + e_j - g_{j+1}
// in float ordinals) as long as every D_j lies in its block's window; past the first block where
// it does not, the translation is the guess.  Exact steps throughout (rounds only).
// Input: the C oracle's N4_DUMP_D file (per iteration: int64 n, n floats d in raster order).
// build: gcc -O2 -ffp-contract=off -o /tmp/pc_sim4 scripts/dev/pc_sim4.c -lm
// run:   /tmp/pc_sim4 D.bin [NB=1024] [MODE=0 affine | 1 windows | 2 windows, affine past the frontier | 3 as 2 with one crossing]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int64_t n;
static float *p;
static double *Nd;
static inline int32_t ford(float f) { int32_t i; memcpy(&i, &f, 4); return i; }   // f > 0
static inline float ffrom(int32_t i) { float f; memcpy(&f, &i, 4); return f; }

// one exact step (the spec's roundings: mu * RN(1 - RN(1/N)) + RN_f(p / N) in double, then float)
static inline float mu_step(int64_t k, float mu, double *phi_out, double *ulp_out) {
    const double N = Nd[k], r = 1.0 / N;
    const double z = (double)mu * (1.0 - r) + (double)(p[k] / (float)N);
    const float m1 = (float)z;
    if (phi_out) {
        int e;
        frexpf(m1 > 0 ? m1 : 1.0f, &e);
        const double u = ldexp(1.0, e - 24);   // ulp of m1's binade
        *ulp_out = u;
        *phi_out = (z - (double)m1) / u;       // in [-0.5, 0.5]
    }
    return m1;
}

#define KL 16
typedef struct { float g, e, go, eo; int64_t k0, len; double Tp, Tm, Tp2, Tm2;
                 double lp[KL], lm[KL]; int np, nm; double capp, capm; } Blk;
static double DMAX = 64;

static float run(Blk *b, float mu, int win) {
    double Tp = 1e30, Tm = 1e30, Tp2 = 1e30, Tm2 = 1e30, Bp = 1e30, Bm = 1e30;
    b->np = b->nm = 0;
    b->capp = b->capm = 1e30;
    for (int64_t s = 0; s < b->len; ++s) {
        const int64_t k = b->k0 + s;
        double phi = 0, u = 0;
        const float m0 = mu;
        mu = mu_step(k, mu, win ? &phi : NULL, &u);
        if (win) {
            const double N = Nd[k];
            // shift +delta: the value moves by -delta/N relative to the shifted grid
            const double tp = (phi + 0.5) * N, tm = (0.5 - phi) * N;
            if (tp < DMAX) { if (b->np < KL) b->lp[b->np++] = tp; else if (tp < b->capp) b->capp = tp; }
            if (tm < DMAX) { if (b->nm < KL) b->lm[b->nm++] = tm; else if (tm < b->capm) b->capm = tm; }
            if (tp < Tp) { Tp2 = Tp; Tp = tp; } else if (tp < Tp2) Tp2 = tp;
            if (tm < Tm) { Tm2 = Tm; Tm = tm; } else if (tm < Tm2) Tm2 = tm;
            // binade edges around the start and the result (ordinal shifts stay uniform inside)
            int e0;
            frexpf(m0 > 0 ? m0 : 1.0f, &e0);
            const double lo0 = ldexp(1.0, e0 - 1), hi0 = ldexp(1.0, e0), u0 = ldexp(1.0, e0 - 24);
            if (m0 > 0) {
                const double up = (hi0 - m0) / u0 - 1, dn = (m0 - lo0) / u0;
                if (up < Bp) Bp = up;
                if (dn < Bm) Bm = dn;
            } else {
                Bp = Bm = 0;
            }
            int e1;
            frexpf(mu > 0 ? mu : 1.0f, &e1);
            const double lo1 = ldexp(1.0, e1 - 1), hi1 = ldexp(1.0, e1);
            if (mu > 0) {
                const double up = (hi1 - mu) / u - 1, dn = (mu - lo1) / u;
                if (up < Bp) Bp = up;
                if (dn < Bm) Bm = dn;
            }
        }
    }
    // binade edges bound every shift; rounding thresholds: the first crossing moves D one toward 0
    b->Tp = fmin(Tp, Bp);   // real thresholds: a shift |D| crosses iff |D| > T
    b->Tm = fmin(Tm, Bm);
    b->Tp2 = fmin(Tp2, Bp);
    b->Tm2 = fmin(Tm2, Bm);
    if (Tp > Bp) b->Tp2 = b->Tp;   // the binade bound is hit first: no known map past it
    if (Tm > Bm) b->Tm2 = b->Tm;
    b->capp = fmin(fmin(b->capp, Bp), DMAX);
    b->capm = fmin(fmin(b->capm, Bm), DMAX);
    return mu;
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    const int NB = argc > 2 ? atoi(argv[2]) : 1024;
    const int MODE = argc > 3 ? atoi(argv[3]) : 0;
    if (argc > 4) DMAX = atof(argv[4]);
    const int64_t CAP = 40000000;
    float *d = malloc(4 * CAP);
    p = malloc(4 * (CAP + 1));
    Nd = malloc(8 * (CAP + 1));
    float *mt = malloc(4 * (CAP + 1));
    Blk *B = calloc(NB, sizeof(Blk));
    float *ng = malloc(4 * NB);
    int it = 0;
    double tot = 0, evals = 0;
    int hist[64] = {0};
    while (fread(&n, 8, 1, f) == 1) {
        if (fread(d, 4, n, f) != (size_t)n) break;
        it++;
        float N = 0.0f;
        for (int64_t k = 1; k <= n; ++k) {
            p[k] = (float)exp((double)d[k - 1]);
            N = (float)((double)N + 1.0);
            Nd[k] = N;
        }
        float mu = 0;
        mt[0] = 0;
        for (int64_t k = 1; k <= n; ++k) mt[k] = mu = mu_step(k, mu, NULL, NULL);
        const int64_t L = n / NB, rem = n % NB;
        const int nbe = L ? NB : (int)rem;
        double S1 = 0;
        int64_t k0 = 1;
        for (int j = 0; j < nbe; ++j) {
            Blk *b = &B[j];
            b->k0 = k0;
            b->len = L + (j < rem);
            const double K = (double)(k0 - 1);
            b->g = K > 0 ? (float)(1.0 + S1 / K) : 0.0f;
            b->go = b->eo = NAN;
            b->e = NAN;
            for (int64_t s = 0; s < b->len; ++s) S1 += (double)p[k0 + s] - 1.0;
            k0 += b->len;
        }
        int rounds = 0;
        float *lastg = malloc(4 * NB);
        for (int j = 0; j < nbe; ++j) lastg[j] = NAN;
        for (int r = 0; r < 60; ++r) {
            rounds++;
            for (int j = 0; j < nbe; ++j) {
                Blk *b = &B[j];
                if (b->g == lastg[j] && r > 0) continue;   // start unchanged: keep the end
                b->e = run(b, b->g, MODE != 0);
                lastg[j] = b->g;
                evals += 1.0 / nbe;
            }
            int bad = 0, fb = -1;
            double maxerr = 0;
            for (int j = 0; j + 1 < nbe; ++j) { if (B[j].e != B[j + 1].g) { bad++; if (fb < 0) fb = j; }
                double er = fabs((double)B[j+1].g - (double)mt[B[j+1].k0 - 1]) / 1.19e-7; if (er > maxerr) maxerr = er; }
            if (getenv("DBGIT") && it == atoi(getenv("DBGIT"))) fprintf(stderr, "round %d: mismatches %d first %d max guess err %.1f ulp\n", r, bad, fb, maxerr);
            if (!bad) break;
            if (MODE == 0) {   // pcw_update: affine model, secant slopes
                double dm = 0.0;
                for (int j = 0; j + 1 < nbe; ++j) {
                    Blk *b = &B[j];
                    const double bj = (double)b->e - (double)B[j + 1].g;
                    double a = (double)(b->k0 - 1) / (double)(b->k0 + b->len - 1);
                    if (r > 0 && b->g != b->go) {
                        const double sl = ((double)b->e - b->eo) / ((double)b->g - b->go);
                        if (sl >= 0.0 && sl <= 1.0) a = sl;
                    }
                    ng[j + 1] = dm == 0.0 ? b->e : (float)((double)b->e + a * dm);
                    b->go = b->g;
                    b->eo = b->e;
                    dm = a * dm + bj;
                }
            } else {   // windows: exact composition while D_j is inside block j's window
                int64_t D = 0;   // ordinal correction of block j's guess
                int certain = 1;
                double dm = 0.0;   // MODE 2: affine past the frontier
                for (int j = 0; j + 1 < nbe; ++j) {
                    Blk *b = &B[j];
                    int64_t c = 0;   // MODE 3: one crossing past the first threshold
                    int inside = (double)D <= b->Tp && (double)-D <= b->Tm;
                    if (MODE == 4) {   // threshold lists in step order: each crossing moves D one toward 0
                        const int64_t a = D < 0 ? -D : D;
                        inside = (double)a <= (D > 0 ? b->capp : b->capm);
                        if (inside && a > 0) {
                            int64_t sft = a;
                            const double *lst = D > 0 ? b->lp : b->lm;
                            const int cnt = D > 0 ? b->np : b->nm;
                            for (int q = 0; q < cnt; ++q) if ((double)sft > lst[q]) sft--;
                            c = D > 0 ? sft - a : a - sft;
                        }
                    }
                    if (!inside && MODE == 3) {
                        if (D > 0 && (double)D <= b->Tp2 && (double)D <= b->Tp + 1e30 && b->Tp < b->Tp2) { inside = 1; c = -1; }
                        if (D < 0 && (double)-D <= b->Tm2 && b->Tm < b->Tm2) { inside = 1; c = 1; }
                    }
                    if (certain && !inside) {
                        certain = 0;
                        if (getenv("DBG") && it == atoi(getenv("DBG")))
                            fprintf(stderr, "round %d frontier j %d k0 %lld D %lld Tp %.0f Tm %.0f (true start err %d)\n", r, j,
                                    (long long)b->k0, (long long)D, b->Tp, b->Tm, ford(b->g) - ford(mt[b->k0 - 1]));
                    }
                    if (certain || MODE == 1) {
                        const int64_t endo = (int64_t)ford(b->e) + D + c;   // translated end
                        ng[j + 1] = ffrom((int32_t)endo);
                        D = endo - ford(B[j + 1].g);
                        dm = (double)ng[j + 1] - (double)B[j + 1].g;
                    } else {
                        const double bj = (double)b->e - (double)B[j + 1].g;
                        double a = (double)(b->k0 - 1) / (double)(b->k0 + b->len - 1);
                        if (r > 0 && b->g != b->go) {
                            const double sl = ((double)b->e - b->eo) / ((double)b->g - b->go);
                            if (sl >= 0.0 && sl <= 1.0) a = sl;
                        }
                        ng[j + 1] = dm == 0.0 ? b->e : (float)((double)b->e + a * dm);
                        dm = a * dm + bj;
                        D = (int64_t)ford(ng[j + 1]) - ford(B[j + 1].g);
                    }
                    b->go = b->g;
                    b->eo = b->e;
                }
            }
            for (int j = 1; j < nbe; ++j) B[j].g = ng[j];
        }
        free(lastg);
        const int ok = B[nbe - 1].e == mt[n];
        tot += rounds;
        if (rounds < 64) hist[rounds]++;
        if (getenv("V")) printf("it %2d n %lld: rounds %d %s\n", it, (long long)n, rounds, ok ? "ok" : "MISMATCH");
        if (!ok) printf("it %d MISMATCH\n", it);
    }
    printf("MODE %d NB %d: mean stage-0 rounds %.2f, block evaluations per iteration %.2f; rounds histogram:", MODE,
           NB, tot / it, evals / it);
    for (int i = 0; i < 64; ++i)
        if (hist[i]) printf(" %d:%d", i, hist[i]);
    printf("\n");
    return 0;
}
