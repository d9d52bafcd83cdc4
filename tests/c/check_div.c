/* Checks dm_div_recip (include/eslam_detmath.h) against the IEEE division it replaces on
 * the device.  Test infrastructure: built and run by tests/test_detmath.py.
 *
 *   check_div uniform <stride>   x = 1, 1 + stride, ... < 2^31: dm_minstd_uniform_fast(x)
 *                                == dm_minstd_uniform(x) bit for bit (stride 1: all 2^31 - 1)
 *   check_div draws <count>      (k + u) / N for random N (all magnitudes, powers of two and
 *                                their neighbours), k in [0, N), u a minstd uniform, plus the
 *                                k = 0 and k = N - 1 edges
 * Prints the number of mismatches; exit status 1 if any.                                    */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "eslam_detmath.h"

static uint64_t sm_state = 0x9E3779B97F4A7C15ull;
static uint64_t splitmix(void)
{
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t bad = 0, checked = 0;

static void check_draw(uint64_t k, uint32_t x, uint64_t N)
{
    const double dN = (double)N, y = 1.0 / dN;
    const double a = (double)k + dm_minstd_uniform(x);
    const double ref = a / dN, got = dm_div_recip(a, dN, y);
    ++checked;
    if (dm_bits(ref) != dm_bits(got)) {
        if (bad < 10) fprintf(stderr, "draw mismatch k=%llu x=%u N=%llu: %a vs %a\n", (unsigned long long)k, x,
                              (unsigned long long)N, ref, got);
        ++bad;
    }
}

int main(int argc, char** argv)
{
    if (argc < 3) { fprintf(stderr, "usage: check_div uniform|draws <n>\n"); return 2; }
    const uint64_t n = strtoull(argv[2], NULL, 10);
    if (!strcmp(argv[1], "uniform")) {
        const uint64_t stride = n ? n : 1;
        for (uint64_t x = 1; x < 2147483648ull; x += stride) {
            ++checked;
            if (dm_bits(dm_minstd_uniform((uint32_t)x)) != dm_bits(dm_minstd_uniform_fast((uint32_t)x))) {
                if (bad < 10) fprintf(stderr, "uniform mismatch x=%llu\n", (unsigned long long)x);
                ++bad;
            }
        }
        /* the last value and its neighbours, whatever the stride */
        for (uint32_t x = 2147483640u; x < 2147483648u; ++x) {
            ++checked;
            if (dm_bits(dm_minstd_uniform(x)) != dm_bits(dm_minstd_uniform_fast(x))) ++bad;
        }
    } else if (!strcmp(argv[1], "draws")) {
        for (uint64_t t = 0; t < n; ++t) {
            const uint64_t r = splitmix();
            uint64_t N;
            switch (r & 3) {
            case 0: N = 1 + (splitmix() >> (64 - 1 - (int)(splitmix() % 40))); break;     /* any magnitude */
            case 1: N = (1ull << (splitmix() % 40)) + (uint64_t)((int)(splitmix() % 5) - 2); break;
            case 2: N = 1 + splitmix() % 100000; break;
            default: N = 4000000 + splitmix() % 20000000; break;
            }
            if (N == 0 || N > (1ull << 40)) N = 1;
            const uint32_t x = 1 + (uint32_t)(splitmix() % 2147483646u);
            check_draw(splitmix() % N, x, N);
            check_draw(0, x, N);
            check_draw(N - 1, x, N);
            check_draw(N - 1, 2147483646u, N);     /* u = 1 - 1/(2^31 - 2) */
        }
    } else {
        return 2;
    }
    printf("%llu checked, %llu mismatches\n", (unsigned long long)checked, (unsigned long long)bad);
    return bad ? 1 : 0;
}
