/* ORACLE -- test infrastructure only.  CPU restatement of the cluster-index map
 * (CI.py:87-145 calculate_CV / calculate_CI).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  Pinned bit-for-bit against CI.py run on the same inputs
 * (tests/golden/vdp_*.npz, keys ci_values / CI; see tests/golden/make_goldens.py).
 *
 * Restated semantics:
 *   - defect voxels are visited in C order (multi_which, CI.py:10-30);
 *   - px2vec (CI.py:65-68) makes the sphere-row index L = (i+dx) + (j+dy) s0 + (k+dz) s0 s1 on the
 *     Fortran-order ravel: rows/cols outside the array ALIAS into neighbouring columns/slices,
 *     only 0 <= L < N is required for a hit;
 *   - np.intersect1d uniques its inputs: a row whose linear offset repeats an earlier row's never
 *     counts again (dup[] flags, only possible when s0 or s1 <= 100);
 *   - at each shell boundary b (CI.py:79-85, in order) the test C = hits/b < 0.5 <=> 2*hits < b;
 *     the first failing b gives CI = r[b-1] * min(vox) (CI.py:100,141);  the last shell is never
 *     tested and no break raises ValueError (CI.py:101-103) -> return code 2.
 */
#include <stdint.h>
#include <stdlib.h>

int ci_oracle(const uint8_t *defect, int64_t s0, int64_t s1, int64_t s2,
              const int16_t *offs, const uint8_t *dup, int64_t rows,
              const int32_t *bounds, const double *radii, int64_t nb, double minvox,
              double *ci_out, int32_t *shell_out)
{
    const int64_t N = s0 * s1 * s2;
    uint8_t *fdef = (uint8_t *)malloc((size_t)N);
    if (!fdef) return 1;
    for (int64_t i = 0; i < s0; ++i)
        for (int64_t j = 0; j < s1; ++j)
            for (int64_t k = 0; k < s2; ++k)
                fdef[i + j * s0 + k * s0 * s1] = defect[(i * s1 + j) * s2 + k] != 0;
    int rc = 0;
    for (int64_t i = 0; i < s0 && !rc; ++i)
        for (int64_t j = 0; j < s1 && !rc; ++j)
            for (int64_t k = 0; k < s2 && !rc; ++k) {
                const int64_t c = (i * s1 + j) * s2 + k;
                ci_out[c] = 0.0;
                if (shell_out) shell_out[c] = -1;
                if (!defect[c]) continue;
                const int64_t base = i + j * s0 + k * s0 * s1;
                int64_t hits = 0, row = 0, q = 0;
                for (; q < nb; ++q) {
                    const int64_t b = bounds[q];
                    for (; row < b; ++row) {
                        if (dup[row]) continue;
                        const int64_t L = base + offs[3 * row] + offs[3 * row + 1] * s0 +
                                          offs[3 * row + 2] * s0 * s1;
                        if (L >= 0 && L < N && fdef[L]) ++hits;
                    }
                    if (2 * hits < b) break;
                }
                if (q == nb) { rc = 2; break; }
                ci_out[c] = radii[q] * minvox;
                if (shell_out) shell_out[c] = (int32_t)q;
            }
    free(fdef);
    return rc;
}
