// CPU reference point for the S7 step latency: (double)(float)fma(mu, A, B) as a dependent chain.
// gcc -O2 -march=native -ffp-contract=off chain_cpu.c -o chain_cpu -lm  (build container: 4.8 ns/step)
#include <stdio.h>
#include <math.h>
#include <time.h>
int main(void) {
    const int N = 100000000;
    volatile double a = 0.9999, b = 1.0e-5;
    double A = a, B = b, mu = 0.3;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int k = 0; k < N; ++k) mu = (double)(float)fma(mu, A, B);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double ns = (t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec);
    printf("%.3f ns/step (mu %g)\n", ns / N, mu);
    return 0;
}
