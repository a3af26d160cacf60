// Host-only check of lcfir::fft_unit (csrc/fir_fft.hpp), built by
// tests/test_fft_layout.py with `hipcc --offload-host-only`: for every
// (units, grid) pair, each round maps the grid's workgroups one-to-one onto
// that round's units, full rounds keep the XCD-aware order, and the last,
// partial round gives unit i g + b to workgroup b.  Prints the error count.
#include "fir_fft.hpp"

#include <cstdio>
#include <vector>

int main() {
    long bad = 0, cases = 0;
    for (long units = 1; units <= 5000; units += (units < 300 ? 1 : 37)) {
        for (int g : {1, 7, 8, 16, 64, 248, 256, 512}) {
            if (g > units) continue;
            ++cases;
            std::vector<int> seen((size_t)units, 0);
            for (int b = 0; b < g; ++b) {
                for (long i = 0;; ++i) {
                    const long u = lcfir::fft_unit(i, b, g, units);
                    if (u >= units) break;
                    if (u < i * g || u >= (i + 1) * g) ++bad;           // stays in its round
                    if ((i + 1) * g > units && u != i * g + b) ++bad;   // partial round: identity
                    if ((i + 1) * g <= units && g % 8 == 0 &&
                        u != i * g + (b % 8) * (g / 8) + b / 8) ++bad; // full round: XCD order
                    ++seen[(size_t)u];
                }
            }
            for (long u = 0; u < units; ++u) bad += seen[(size_t)u] != 1;
        }
    }
    // the 32-bit map the kernels run agrees with the 64-bit one
    for (int units = 1; units <= 5000; units += (units < 300 ? 1 : 37))
        for (int g : {1, 7, 8, 16, 64, 248, 256, 512}) {
            if (g > units) continue;
            ++cases;
            for (int b = 0; b < g; ++b)
                for (int i = 0; i * g < units; ++i)
                    bad += lcfir::fft_unit32(i, b, g, units) != (int)lcfir::fft_unit(i, b, g, units);
        }
    // fft_grid / fft_div: u / nseg by multiply-shift, exact for u < 2^31
    {
        std::vector<long> ds = {1, 2, 3, 5, 7, 8, 100, 2325, 2326, 4095, 4096, 4097, 65535, 131071, 131072,
                                1000003, (1L << 30) - 1, 1L << 30, (1L << 30) + 1, (1L << 31) - 1};
        unsigned long long st = 88172645463325252ULL;
        for (long d : ds) {
            ++cases;
            const lcfir::FftGrid gd = lcfir::fft_grid(d, d);
            auto chk = [&](long u) { bad += lcfir::fft_div((int)u, gd) != (int)(u / d); };
            for (long u = 0; u < 70000; ++u) chk(u);
            for (long u = (1L << 31) - 70000; u < (1L << 31); ++u) chk(u);
            for (long k = 1; k <= 3000; ++k) { // around multiples of d
                const long m = (long)(((1L << 31) - 1) / d) * k / 3000 * d;
                for (long u = m - 2; u <= m + 2; ++u)
                    if (u >= 0 && u < (1L << 31)) chk(u);
            }
            for (int r = 0; r < 200000; ++r) { // xorshift64
                st ^= st << 13; st ^= st >> 7; st ^= st << 17;
                chk((long)(st % (1ULL << 31)));
            }
        }
    }
    std::printf("cases %ld errors %ld\n", cases, bad);
    return bad != 0;
}
