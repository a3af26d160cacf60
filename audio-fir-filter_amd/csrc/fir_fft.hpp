// fir_fft.hpp -- f64 overlap-save FFT convolution (placeholder until the
// kernel lands; AUTO never selects it while fft_preferred() is false).
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include "fir_direct.hpp"

namespace lcfir {

struct FftPlan {
    bool ready = false;
};

inline bool fft_preferred(int /*ntaps*/) { return false; }

inline bool fft_plan_build(FftPlan &, const double *, int, hipStream_t, std::string &err) {
    err = "FFT method not built in this version";
    return false;
}

inline bool fft_launch(const FftPlan &, const DirectParams &, int, hipStream_t, std::string &err) {
    err = "FFT method not built in this version";
    return false;
}

inline void fft_plan_free(FftPlan &) {}

} // namespace lcfir
