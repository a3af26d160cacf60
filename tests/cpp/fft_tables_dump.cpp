// Writes the host-side FFT plan tables (lcfir::fft_plan_tables, fir_fft.hpp)
// for a tap file, so a CPU test can emulate the kernels' pair step on them
// (scripts/fft32_model.py).  No device is touched.
//
// usage: fft_tables_dump taps.f64 seg_len zero_phase out_prefix [family]
// (seg_len 0: the library's own choice for the taps, fft_choose_seg_len;
// family: FftTuning::family, 0 default, 1 LDS kernels)
// writes <out_prefix>.meta (L halves parts tp sym reg32, text), .pair .c8 .tw
// (complex double pairs) and .task (uint32).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "fir_fft.hpp"

template <class T>
static void dump(const std::string &path, const std::vector<T> &v) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
}

int main(int argc, char **argv) {
    if (argc != 5 && argc != 6) {
        std::fprintf(stderr, "usage: %s taps.f64 seg_len zero_phase out_prefix [family]\n", argv[0]);
        return 2;
    }
    std::ifstream f(argv[1], std::ios::binary | std::ios::ate);
    if (!f) return 2;
    const size_t bytes = (size_t)f.tellg();
    std::vector<double> taps(bytes / sizeof(double));
    f.seekg(0);
    f.read(reinterpret_cast<char *>(taps.data()), (std::streamsize)bytes);
    lcfir::FftTuning tune;
    tune.seg_len = std::atoi(argv[2]);
    tune.zero_phase = std::atoi(argv[3]);
    if (argc == 6) tune.family = std::atoi(argv[5]);
    const lcfir::FftTables T = lcfir::fft_plan_tables(taps, tune);
    const std::string out = argv[4];
    std::ofstream m(out + ".meta");
    m << T.L << " " << T.halves << " " << T.parts << " " << T.tp << " " << (T.sym ? 1 : 0) << " "
      << (T.reg32 ? 1 : 0) << "\n";
    dump(out + ".pair", T.pair);
    dump(out + ".task", T.task);
    dump(out + ".c8", T.c8);
    dump(out + ".tw", T.tw);
    return 0;
}
