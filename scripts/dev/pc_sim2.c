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

typedef struct { float g, gs, e, es, go, eo; int64_t k0, len; } Blk;

static void run_block(Blk *b, int mode /* 0 apx mu, 1 apx both, 2 exact */) {
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
            if (GUESS == 1 && have_prev && K > 0) {
                // previous iteration's float drift at the same relative position
                const int64_t kp = (int64_t)((double)(k0 - 1) * (double)nprev / (double)n);
                if (kp > 0) g = (float)((double)g + ((double)pmt[kp] - pmean[kp]));
            }
            b->g = g;
            b->gs = gs;
            b->go = b->eo = NAN;
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
        for (int stage = 0; stage < 2; ++stage) {
            for (int r = 0; r < 40; ++r, ++round) {
                for (int j = 0; j < nbe; ++j) run_block(&B[j], stage);
                ra[stage]++;
                if (update(B, nbe, round, stage == 1)) break;
            }
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
    return 0;
}
