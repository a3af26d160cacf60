// lcfir/FilterCore.h -- drop-in replacement for the reference's FilterCore.h.
//
// Declares, in namespace Diskerror, the NON-template function of
// FilterCore.h:20-27 with the reference's exact parameter types:
//
//   inline void apply_filter_range(const VectorMath<float32_t>& channel,
//                                  const WindowedSinc<float64_t>& sinc,
//                                  VectorMath<float32_t>& temp_output,
//                                  int_fast64_t startIdx, int_fast64_t endIdx,
//                                  ThreadSafeProgress* progress);
//
// so ProcessFile.cp:71-78 can keep passing it BY NAME to std::thread:
//
//   threads.emplace_back(apply_filter_range, std::cref(buf[ch]), std::cref(sinc),
//                        std::ref(temp_output), start, end, &safe_progress);
//
// (a function template cannot be deduced there; tests/cpp/dropin_processfile.cpp
// compiles exactly that call shape).  The body evaluates the range on an
// MI355X through the C ABI (lcfir/FilterCore.hpp -> lcfir.h); float32_t and
// float64_t are boost's typedefs for float and double, so the parameter types
// are the reference's own.
//
// Like the reference header it pulls in c_lib's VectorMath.h / WindowedSinc.h
// and ProgressBar.h (FilterCore.h:10-14).  A translation unit that has declared
// those types itself defines LCFIR_DROPIN_TYPES_DECLARED first.  The include
// guard is the reference's (DISKERROR_FILTERCORE_H), so the two headers never
// both define the function.
#ifndef DISKERROR_FILTERCORE_H
#define DISKERROR_FILTERCORE_H

#include <cstdint>

#ifndef LCFIR_DROPIN_TYPES_DECLARED
#include <VectorMath.h>
#include <WindowedSinc.h>
#include "ProgressBar.h"
#endif

#include "lcfir/FilterCore.hpp"

namespace Diskerror {

// FIR filtering for a range of samples on a single deinterleaved channel
// (FilterCore.h:19-79), on the GPU.  Writes temp_output[startIdx, endIdx) only;
// reports endIdx - startIdx to progress (nullable) once the range is done.
inline void apply_filter_range(const VectorMath<float>& channel, const WindowedSinc<double>& sinc,
                               VectorMath<float>& temp_output, int_fast64_t startIdx,
                               int_fast64_t endIdx, ThreadSafeProgress* progress) {
    lcfir::apply_filter_range(channel, sinc, temp_output, startIdx, endIdx, progress);
}

} // namespace Diskerror

#endif // DISKERROR_FILTERCORE_H
