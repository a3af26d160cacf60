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
    std::printf("cases %ld errors %ld\n", cases, bad);
    return bad != 0;
}
