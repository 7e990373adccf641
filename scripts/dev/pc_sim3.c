// PC stage-0 (mu alone) round counts: the affine guess update of pcw_update against "window maps":
// every block also knows its map on the 2W + 1 floats around its guess (how many ulps each start
// offset keeps at the block end), so an upstream correction that lands inside the window
// propagates exactly instead of through the secant model.  Exact steps throughout (rounds only).
// Input: the C oracle's N4_DUMP_D file (per iteration: int64 n, n floats d in raster order).
// build: gcc -O2 -ffp-contract=off -o /tmp/pc_sim3 scripts/dev/pc_sim3.c -lm
// run:   /tmp/pc_sim3 D.bin [NB=1024] [W=0 (old model) | W>0 window half-width]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int64_t n;
static float *p;
static double *Nd;
static inline float mu_step(int64_t k, float mu) {
    const double N = Nd[k], r = 1.0 / N;
    return (float)((double)mu * (1.0 - r) + (double)(p[k] / (float)N));
}
static inline int32_t fidx(float f) { int32_t i; memcpy(&i, &f, 4); return i; }   // f >= 0
static inline float ffrom(int32_t i) { float f; memcpy(&f, &i, 4); return f; }

typedef struct { float g, e, go, eo; int64_t k0, len; int F[129]; } Blk;
static int W;

static float run(const Blk *b, float mu) {
    for (int64_t s = 0; s < b->len; ++s) mu = mu_step(b->k0 + s, mu);
    return mu;
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    const int NB = argc > 2 ? atoi(argv[2]) : 1024;
    W = argc > 3 ? atoi(argv[3]) : 0;
    const int64_t CAP = 40000000;
    float *d = malloc(4 * CAP);
    p = malloc(4 * (CAP + 1));
    Nd = malloc(8 * (CAP + 1));
    float *mt = malloc(4 * (CAP + 1));
    Blk *B = calloc(NB, sizeof(Blk));
    int it = 0;
    double tot = 0, totev = 0;
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
        for (int64_t k = 1; k <= n; ++k) mt[k] = mu = mu_step(k, mu);
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
            for (int64_t s = 0; s < b->len; ++s) S1 += (double)p[k0 + s] - 1.0;
            k0 += b->len;
        }
        int rounds = 0, ev = 0;
        for (int r = 0; r < 60; ++r) {
            rounds++;
            for (int j = 0; j < nbe; ++j) {
                Blk *b = &B[j];
                b->e = run(b, b->g);
                if (W > 0 && j > 0) {
                    const int32_t gi = fidx(b->g), ei = fidx(b->e);
                    int shift = 1;
                    for (int i = -W; i <= W; ++i) {
                        b->F[i + W] = fidx(run(b, ffrom(gi + i))) - ei;
                        shift &= b->F[i + W] == i;
                    }
                    ev += !shift;
                }
            }
            int bad = 0;
            for (int j = 0; j + 1 < nbe; ++j) bad += B[j].e != B[j + 1].g;
            if (!bad) break;
            if (getenv("DBG") && it == atoi(getenv("DBG"))) {
                int shown = 0, tb = 0;
                for (int j = 0; j + 1 < nbe; ++j) tb += B[j].e != B[j + 1].g;
                fprintf(stderr, "round %d bad %d\n", r, tb);
                for (int j = 0; j + 1 < nbe && shown < 12; ++j) {
                    const Blk *b = &B[j];
                    const int ge = fidx(b->g) - fidx(mt[b->k0 - 1]), ee = fidx(b->e) - fidx(mt[b->k0 + b->len - 1]);
                    const int ne = fidx(B[j + 1].g) - fidx(mt[B[j + 1].k0 - 1]);
                    if (ge || ee || ne) {
                        fprintf(stderr, "  j %4d k0 %6lld gerr %5d eerr %5d next-gerr %5d g %.9g F:", j, (long long)b->k0, ge, ee, ne, b->g);
                        for (int i = 0; i < 2 * W + 1; ++i) if (b->F[i] != i - W) fprintf(stderr, " %d:%d", i - W, b->F[i]);
                        fprintf(stderr, "\n");
                        shown++;
                    }
                }
            }
            // update: dm = correction of block j's guess (index units; exact integer when known)
            double dm = 0.0;
            int exact = 1;
            static float ng[1 << 16];
            for (int j = 0; j + 1 < nbe; ++j) {
                Blk *b = &B[j];
                const double bj = (double)fidx(b->e) - (double)fidx(B[j + 1].g);
                double T;
                static int LOOSE = -1;
                if (LOOSE < 0) LOOSE = getenv("LOOSE") ? 1 : 0;
                if (W > 0 && (exact || LOOSE) && fabs(dm) <= W + 0.5 && j > 0) {
                    const int di = (int)lrint(dm);
                    T = b->F[(di < -W ? -W : di > W ? W : di) + W];
                } else if (dm == 0.0) {
                    T = 0.0;
                } else {
                    double a = (double)(b->k0 - 1) / (double)(b->k0 + b->len - 1);
                    static int SMIN = -1;
                    if (SMIN < 0) SMIN = getenv("SMIN") ? atoi(getenv("SMIN")) : 1;
                    if (r > 0 && b->g != b->go && fabs((double)fidx(b->g) - fidx(b->go)) >= SMIN) {
                        const double sl = ((double)fidx(b->e) - fidx(b->eo)) / ((double)fidx(b->g) - fidx(b->go));
                        if (sl >= 0.0 && sl <= 1.0) a = sl;
                    }
                    static int A1 = -1;
                    if (A1 < 0) A1 = getenv("A1") ? atoi(getenv("A1")) : 0;
                    if (A1 == 1) a = 1.0;
                    if (A1 == 3 && W > 0) a = (double)(b->F[2 * W] - b->F[0]) / (2.0 * W);
                    if (A1 == 2 && b->g != b->go && fabs((double)fidx(b->g) - fidx(b->go)) >= fabs(dm) * 0.5) {
                        const double sl = ((double)fidx(b->e) - fidx(b->eo)) / ((double)fidx(b->g) - fidx(b->go));
                        a = (sl >= 0.0 && sl <= 1.0) ? sl : 1.0;
                    } else if (A1 == 2) a = 1.0;
                    T = a * dm;
                    exact = 0;
                }
                b->go = b->g;
                b->eo = b->e;
                ng[j + 1] = ffrom(fidx(b->e) + (int32_t)llrint(T));
                dm = T + bj;
            }
            for (int j = 1; j < nbe; ++j) B[j].g = ng[j];
            // a new exact run starts wherever the guesses became exact again: the simulation only
            // needs the rounds, the GPU resets `exact` at every matched block (dm == 0 exactly)
        }
        const int ok = B[nbe - 1].e == mt[n];
        printf("it %2d n %lld: stage0 rounds %d window-event blocks/round %.1f %s\n", it, (long long)n, rounds,
               (double)ev / rounds, ok ? "ok" : "MISMATCH");
        tot += rounds;
        totev += (double)ev / rounds;
    }
    printf("W %d mean stage-0 rounds %.2f, window-event blocks per round %.1f\n", W, tot / it, totev / it);
    return 0;
}
