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
// the C ABI of lcfir.h, as a template over the channel, sinc and progress
// types (lcfir::apply_filter_range).  The non-template function with the
// reference's exact parameter types -- the one ProcessFile.cp:71-78 passes by
// name to std::thread -- is in lcfir/FilterCore.h on top of this one.
//
// The wrapper touches its arguments only through what FilterCore.h itself
// uses: channel.size() / channel.begin() (:28,59,67,74), temp_output[i]
// (:59,67,74), sinc.getMo2() / sinc.fms(it) (:29,67), progress->report(n)
// (:44,51) -- plus VectorMath's size constructor (ProcessFile.cp:58).  The
// taps of a WindowedSinc are read through data()/size() when it has them
// (or through a lcfir::SincTraits specialisation); otherwise they are recovered
// exactly from fms() itself: fms over a unit impulse at k is h[k] (every
// other product is an exact zero), one probe per tap, once per sinc object.
//
// Each distinct tap set is uploaded once per process and device (the cache
// below keys on the tap bytes), as the reference builds its WindowedSinc once
// per file (ProcessFile.cp:47-50).  Hot-path failures cannot be reported
// through a void function; they go to lcfir::last_failure() and std::abort()
// unless LCFIR_FILTERCORE_NO_ABORT is defined, in which case the output range
// is left untouched.
#pragma once

#include <cmath>
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
#include <type_traits>
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
// Specialise (data(), size()) for a sinc type whose taps are reachable but not
// through std::data / std::size.  Without either, the taps are probed with
// fms() (probe_taps below).
template <class Sinc, class = void>
struct SincTraits {
    static constexpr bool direct = false;
};
template <class Sinc>
struct SincTraits<Sinc, std::void_t<decltype(std::data(std::declval<const Sinc &>())),
                                    decltype(std::size(std::declval<const Sinc &>()))>> {
    static constexpr bool direct =
        std::is_same_v<std::decay_t<decltype(*std::data(std::declval<const Sinc &>()))>, double>;
    static const double *data(const Sinc &s) { return std::data(s); }
    static size_t size(const Sinc &s) { return std::size(s); }
};
template <class Sinc, class = void>
struct sinc_traits_direct : std::false_type {};
template <class Sinc>
struct sinc_traits_direct<Sinc, std::enable_if_t<SincTraits<Sinc>::direct>> : std::true_type {};
// does Sinc have getMo2() (FilterCore.h:29)?
template <class Sinc, class = void>
struct sinc_has_getmo2 : std::false_type {};
template <class Sinc>
struct sinc_has_getmo2<Sinc, std::void_t<decltype(std::declval<const Sinc &>().getMo2())>> : std::true_type {};
// does Sinc have fms(Channel::const_iterator) (FilterCore.h:67)?
template <class Channel, class Sinc, class = void>
struct sinc_has_fms : std::false_type {};
template <class Channel, class Sinc>
struct sinc_has_fms<Channel, Sinc,
                    std::void_t<decltype(std::declval<const Sinc &>().fms(std::declval<const Channel &>().begin()))>>
    : std::true_type {};

namespace detail {
// A channel's samples as a pointer, through the interfaces FilterCore.h uses
// (begin() for the input, operator[] for the output).
template <class Channel>
inline const float *in_ptr(const Channel &c) {
    return std::size(c) ? &*c.begin() : nullptr;
}
template <class Channel>
inline float *out_ptr(Channel &c) {
    return std::size(c) ? &c[0] : nullptr;
}

// Taps of a sinc that exposes only getMo2() and fms(it): T = 2 getMo2() + 1
// probes of fms over a unit impulse.  fms(p) = sum_k h[k] p[k]; with
// p = impulse + (T-1-k) every product but h[k] * 1 is an exact zero, so the
// recovered tap is bit-exact whatever fms's accumulation order.  Cached per
// sinc object, validated on reuse by getMo2() and one fms() fingerprint over a
// fixed pseudo-random window (an object rebuilt at the same address with other
// taps misses).
// the fixed pseudo-random fingerprint window of T samples in [-1, 1)
template <class Channel>
Channel fingerprint_window(int64_t T) {
    Channel fp((size_t)T);
    uint32_t s = 0x9e3779b9u;
    for (int64_t i = 0; i < T; ++i) {
        s = s * 1664525u + 1013904223u;
        fp[(size_t)i] = (float)((int32_t)(s >> 8) - (1 << 23)) * 0x1p-23f;
    }
    return fp;
}

// The direct path reads the taps through std::data / std::size; c_lib's
// WindowedSinc is not vendored, so that those are exactly the 2 getMo2() + 1
// taps in fms() order is unpinned.  Use them only if the count matches
// getMo2() and, where fms() exists, one fms() fingerprint agrees with the
// same dot product over data() (to 1e-12 of sum |h|: fms's accumulation
// order is unknown); otherwise the taps are probed through fms().
template <class Channel, class Sinc>
bool direct_taps_valid(const Sinc &sinc, const double *h, size_t T) {
    if (!h || T == 0) return false;
    if constexpr (sinc_has_getmo2<Sinc>::value) {
        const int64_t half = (int64_t)sinc.getMo2();
        if (half < 0 || (int64_t)T != 2 * half + 1) return false;
    }
    if constexpr (sinc_has_fms<Channel, Sinc>::value) {
        const Channel fp = fingerprint_window<Channel>((int64_t)T);
        long double dot = 0.0L, norm = 0.0L;
        for (size_t k = 0; k < T; ++k) {
            dot += (long double)h[k] * (long double)fp[k];
            norm += fabsl((long double)h[k]);
        }
        const long double got = (long double)sinc.fms(fp.begin());
        return fabsl(got - dot) <= 1e-12L * norm;
    }
    return true;
}

// Entries of the per-object sinc caches below: the reference builds one
// WindowedSinc per file, usually at the same address, so a few suffice; past
// the cap a cache starts over instead of growing with every object seen.
constexpr size_t kSincCacheCap = 64;

template <class Channel, class Sinc>
std::shared_ptr<const std::vector<double>> probe_taps(const Sinc &sinc) {
    const int64_t half = (int64_t)sinc.getMo2();
    if (half < 0 || half > (1 << 24)) throw Error(LCFIR_EINVAL, "sinc.getMo2() out of range");
    const int64_t T = 2 * half + 1;
    const Channel fp = fingerprint_window<Channel>(T);
    const double finger = (double)sinc.fms(fp.begin());
    struct Entry {
        int64_t half;
        double finger;
        std::shared_ptr<const std::vector<double>> taps;
    };
    static std::mutex mu;
    static std::map<const void *, Entry> *cache = new std::map<const void *, Entry>; // never destroyed
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache->find(&sinc);
    if (it != cache->end() && it->second.half == half &&
        std::memcmp(&it->second.finger, &finger, sizeof finger) == 0)
        return it->second.taps;
    if (cache->size() >= kSincCacheCap && !cache->count(&sinc)) cache->clear(); // bounded: sinc objects come and go
    Channel imp((size_t)(2 * T - 1));
    for (int64_t i = 0; i < 2 * T - 1; ++i) imp[(size_t)i] = 0.0f;
    imp[(size_t)(T - 1)] = 1.0f;
    auto taps = std::make_shared<std::vector<double>>((size_t)T);
    for (int64_t k = 0; k < T; ++k) (*taps)[(size_t)k] = (double)sinc.fms(imp.begin() + (T - 1 - k));
    (*cache)[&sinc] = Entry{half, finger, taps};
    return taps;
}
} // namespace detail

// ---- per-process filter cache (one upload per tap set and device) -------------
// Bounded like the sinc caches: past kCap distinct tap sets the map starts over
// (a Filter still in use elsewhere lives on through its shared_ptr).
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
        if (map_.size() >= kCap) map_.clear();
        map_.emplace(std::move(key), f);
        return f;
    }
    void clear() {
        std::lock_guard<std::mutex> lk(mu_);
        map_.clear();
    }

    size_t size() {
        std::lock_guard<std::mutex> lk(mu_);
        return map_.size();
    }
    static constexpr size_t kCap = 16;

private:
    std::mutex mu_;
    std::map<std::string, std::shared_ptr<Filter>> map_;
};

inline int &default_device() {
    static int d = 0;
    return d;
}

namespace detail {
// The filter of a sinc whose taps are reachable through data() / size(),
// validated once per (sinc object, tap pointer, count, device) instead of on
// every call: the reference calls apply_filter_range once per thread and
// channel (ProcessFile.cp:71-78), and a fingerprint fms() plus a long-double
// dot product over all T taps per call is host work growing with T (ADVICE
// r03).  A hit costs one memcmp of the taps against the validated copy, so a
// WindowedSinc rebuilt at the same address with other taps (the next file's)
// misses.  nullptr when data() / size() are not consistent with getMo2() /
// fms() (the caller then probes through fms()).
template <class Channel, class Sinc>
std::shared_ptr<Filter> direct_filter(const Sinc &sinc, const double *h, size_t T, int device) {
    struct Entry {
        const double *h;
        size_t T;
        int device;
        std::vector<double> taps;
        std::shared_ptr<Filter> flt;
    };
    static std::mutex mu;
    static std::map<const void *, Entry> *cache = new std::map<const void *, Entry>; // never destroyed
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache->find(&sinc);
        if (it != cache->end() && it->second.h == h && it->second.T == T && it->second.device == device &&
            std::memcmp(it->second.taps.data(), h, T * sizeof(double)) == 0)
            return it->second.flt;
    }
    if (!direct_taps_valid<Channel>(sinc, h, T)) return nullptr;
    auto flt = FilterCache::instance().get(h, T, device);
    std::lock_guard<std::mutex> lk(mu);
    if (cache->size() >= kSincCacheCap && !cache->count(&sinc)) cache->clear(); // bounded: sinc objects come and go
    (*cache)[&sinc] = Entry{h, T, device, std::vector<double>(h, h + T), flt};
    return flt;
}
} // namespace detail

inline std::string &last_failure() {
    static thread_local std::string s;
    return s;
}

// The taps of a WindowedSinc-like object as the drop-in sees them: data() /
// size() when those are consistent with getMo2() / fms() (direct_taps_valid),
// otherwise recovered through fms() (probe_taps).  For hosts that build an
// lcfir::Filter themselves (process_buffer_device): c_lib need not expose
// data() / size().
template <class Channel, class Sinc>
std::vector<double> sinc_taps(const Sinc &sinc) {
    if constexpr (sinc_traits_direct<Sinc>::value) {
        const double *h = SincTraits<Sinc>::data(sinc);
        const size_t T = SincTraits<Sinc>::size(sinc);
        if (detail::direct_taps_valid<Channel>(sinc, h, T)) return std::vector<double>(h, h + T);
    }
    if constexpr (sinc_has_fms<Channel, Sinc>::value) {
        return *detail::probe_taps<Channel>(sinc);
    } else {
        throw Error(LCFIR_EINVAL, "sinc exposes neither getMo2()-consistent data()/size() nor fms()");
    }
}

// ---- the drop-in ------------------------------------------------------------------
// Same signature and meaning as FilterCore.h:20-27; any number of threads may
// call it concurrently on disjoint [startIdx, endIdx) of one channel
// (ProcessFile.cp:71-78).
template <class Channel, class Sinc, class Progress>
inline void apply_filter_range(const Channel &channel, const Sinc &sinc, Channel &temp_output,
                               int_fast64_t startIdx, int_fast64_t endIdx, Progress *progress) {
    try {
        std::shared_ptr<Filter> flt;
        if constexpr (sinc_traits_direct<Sinc>::value)
            flt = detail::direct_filter<Channel>(sinc, SincTraits<Sinc>::data(sinc), SincTraits<Sinc>::size(sinc),
                                                 default_device());
        if (!flt) {
            if constexpr (sinc_has_fms<Channel, Sinc>::value) {
                const auto taps = detail::probe_taps<Channel>(sinc);
                flt = FilterCache::instance().get(taps->data(), taps->size(), default_device());
            } else {
                throw Error(LCFIR_EINVAL, "sinc exposes neither getMo2()-consistent data()/size() nor fms()");
            }
        }
        flt->apply_range(detail::in_ptr(channel), (int64_t)std::size(channel), detail::out_ptr(temp_output),
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
