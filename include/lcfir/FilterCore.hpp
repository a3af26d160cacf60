// lcfir/FilterCore.hpp -- C++ drop-in for the reference's FilterCore.h.
//
// The reference declares (FilterCore.h:20-27):
//
//   inline void apply_filter_range(const VectorMath<float32_t>& channel,
//                                  const WindowedSinc<float64_t>& sinc,
//                                  VectorMath<float32_t>& temp_output,
//                                  int_fast64_t startIdx, int_fast64_t endIdx,
//                                  ThreadSafeProgress* progress);
//
// This header provides the same function, same argument meaning, same
// "void, no throw on the hot path" contract, but evaluated on an MI355X through
// the C ABI of lcfir.h.  VectorMath and WindowedSinc live in the un-vendored
// c_lib, so the wrapper is a template over any contiguous float container
// (std::data / std::size, or .data()/.size()) and any tap container; a
// WindowedSinc whose taps are not reachable that way specialises
// lcfir::SincTraits.  ThreadSafeProgress is anything with report(size_t).
//
// Each distinct tap set is uploaded once per process and device (the cache
// below keys on the tap bytes), as the reference builds its WindowedSinc once
// per file (ProcessFile.cp:47-50).  Hot-path failures cannot be reported
// through a void function; they go to lcfir::last_failure() and std::abort()
// unless LCFIR_FILTERCORE_NO_ABORT is defined, in which case the output range
// is left untouched.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "lcfir.h"

namespace lcfir {

// ---- error type for the RAII layer ---------------------------------------
class Error : public std::runtime_error {
public:
    Error(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char *where) {
    if (rc != LCFIR_OK) throw Error(rc, std::string(where) + ": " + lcfir_last_error());
}

// ---- RAII filter context ----------------------------------------------------
class Filter {
public:
    Filter(const double *taps, int32_t ntaps, int device = 0, int method = LCFIR_METHOD_AUTO) {
        check(lcfir_ctx_create(device, taps, ntaps, &ctx_), "lcfir_ctx_create");
        int rc = lcfir_ctx_set_method(ctx_, method);
        if (rc != LCFIR_OK) {
            std::string msg = lcfir_last_error();
            lcfir_ctx_destroy(ctx_);
            ctx_ = nullptr;
            throw Error(rc, "lcfir_ctx_set_method: " + msg);
        }
        device_ = device;
    }
    Filter(const Filter &) = delete;
    Filter &operator=(const Filter &) = delete;
    ~Filter() {
        if (ctx_) lcfir_ctx_destroy(ctx_);
    }
    lcfir_ctx *get() const { return ctx_; }
    int device() const { return device_; }
    int32_t half() const {
        int32_t h = 0;
        check(lcfir_ctx_half(ctx_, &h), "lcfir_ctx_half");
        return h;
    }
    int32_t getMo2() const { return half(); }

    // apply_filter_range on host buffers (throws on failure)
    template <class Progress>
    void apply_range(const float *x, int64_t n, float *y, int64_t start, int64_t end,
                     Progress *progress) const {
        lcfir_progress_fn fn = nullptr;
        if (progress) fn = [](void *u, uint64_t c) { static_cast<Progress *>(u)->report((size_t)c); };
        check(lcfir_apply_range(ctx_, x, n, y, start, end, fn, progress), "lcfir_apply_range");
    }

private:
    lcfir_ctx *ctx_ = nullptr;
    int device_ = 0;
};

// ---- how to reach the taps of a WindowedSinc-like object ---------------------
template <class Sinc, class = void>
struct SincTraits {
    static const double *data(const Sinc &s) { return std::data(s); }
    static size_t size(const Sinc &s) { return std::size(s); }
};

// ---- per-process filter cache (one upload per tap set and device) -------------
class FilterCache {
public:
    static FilterCache &instance() {
        static FilterCache *c = new FilterCache; // never destroyed: outlives static dtors
        return *c;
    }
    std::shared_ptr<Filter> get(const double *taps, size_t ntaps, int device) {
        std::string key((const char *)taps, ntaps * sizeof(double));
        key.append((const char *)&device, sizeof device);
        std::lock_guard<std::mutex> lk(mu_);
        auto it = map_.find(key);
        if (it != map_.end()) return it->second;
        auto f = std::make_shared<Filter>(taps, (int32_t)ntaps, device);
        map_.emplace(std::move(key), f);
        return f;
    }
    void clear() {
        std::lock_guard<std::mutex> lk(mu_);
        map_.clear();
    }

private:
    std::mutex mu_;
    std::map<std::string, std::shared_ptr<Filter>> map_;
};

inline int &default_device() {
    static int d = 0;
    return d;
}

inline std::string &last_failure() {
    static thread_local std::string s;
    return s;
}

// ---- the drop-in ------------------------------------------------------------------
// Same signature and meaning as FilterCore.h:20-27; any number of threads may
// call it concurrently on disjoint [startIdx, endIdx) of one channel
// (ProcessFile.cp:71-78).
template <class Channel, class Sinc, class Progress>
inline void apply_filter_range(const Channel &channel, const Sinc &sinc, Channel &temp_output,
                               int_fast64_t startIdx, int_fast64_t endIdx, Progress *progress) {
    try {
        auto flt = FilterCache::instance().get(SincTraits<Sinc>::data(sinc),
                                               SincTraits<Sinc>::size(sinc), default_device());
        flt->apply_range(std::data(channel), (int64_t)std::size(channel), std::data(temp_output),
                         (int64_t)startIdx, (int64_t)endIdx, progress);
    } catch (const std::exception &e) {
        last_failure() = e.what();
#ifndef LCFIR_FILTERCORE_NO_ABORT
        std::fprintf(stderr, "lcfir apply_filter_range: %s\n", e.what());
        std::abort();
#endif
    }
}

} // namespace lcfir
