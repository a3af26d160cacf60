// Stand-ins for the reference's un-vendored c_lib / ProgressBar.h types, as
// ProcessFile.cp and FilterCore.h use them: VectorMath(size), size(),
// begin(), operator[], max_mag(); WindowedSinc's getMo2() and fms(it[, count])
// (no data()/size(), so the drop-in must recover the taps through fms itself);
// ThreadSafeProgress::report(size_t).  Shared by dropin_processfile.cpp and
// dropin_bench.cpp.
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <mutex>
#include <new>
#include <set>
#include <vector>

#include "lcfir.h"

namespace Diskerror {

// Where the stand-in VectorMath keeps its samples: pageable memory (the
// default, as c_lib's std::vector-backed type would) or, for
// tests/cpp/dropin_bench's pinned mode, page-locked memory from
// lcfir_host_malloc (a host that pins its sample buffers; lcfir_apply_range
// then DMAs them directly).  Per thread: the buffers the ProcessFile loop's
// own thread makes (channels, temp_output) follow it, while the small
// VectorMath temporaries the drop-in builds on the worker threads (the tap
// fingerprint window) stay pageable -- a pinned allocation per call costs
// ~0.3 ms of driver time.
inline bool &vectormath_pinned() {
    static thread_local bool pinned = false;
    return pinned;
}
struct PinnedBlocks { // the blocks lcfir_host_malloc gave out (freed by lcfir_host_free)
    std::mutex mu;
    std::set<void *> live;
    static PinnedBlocks &get() {
        static PinnedBlocks *b = new PinnedBlocks;
        return *b;
    }
};
template <class T>
struct SampleAlloc {
    using value_type = T;
    SampleAlloc() = default;
    template <class U>
    SampleAlloc(const SampleAlloc<U> &) {}
    T *allocate(size_t n) {
        void *p = nullptr;
        if (vectormath_pinned()) {
            if (lcfir_host_malloc(n * sizeof(T), &p) != LCFIR_OK) throw std::bad_alloc();
            std::lock_guard<std::mutex> lk(PinnedBlocks::get().mu);
            PinnedBlocks::get().live.insert(p);
        } else if (!(p = std::malloc(n * sizeof(T)))) {
            throw std::bad_alloc();
        }
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t) {
        {
            std::lock_guard<std::mutex> lk(PinnedBlocks::get().mu);
            if (PinnedBlocks::get().live.erase(p)) {
                lcfir_host_free(p);
                return;
            }
        }
        std::free(p);
    }
    bool operator==(const SampleAlloc &) const { return true; }
    bool operator!=(const SampleAlloc &) const { return false; }
};

template <class T>
class VectorMath {
public:
    VectorMath() = default;
    explicit VectorMath(size_t n) : v_(n) {}
    size_t size() const { return v_.size(); }
    typename std::vector<T, SampleAlloc<T>>::const_iterator begin() const { return v_.begin(); }
    typename std::vector<T, SampleAlloc<T>>::iterator begin() { return v_.begin(); }
    T &operator[](size_t i) { return v_[i]; }
    const T &operator[](size_t i) const { return v_[i]; }
    T max_mag() const {
        T m = 0;
        for (T x : v_) m = std::max(m, std::abs(x));
        return m;
    }

private:
    std::vector<T, SampleAlloc<T>> v_;
};

// fms semantics as FilterCore.h calls it: fms(p) = all taps,
// fms(p, -k) = the LAST k taps against p[0..k), fms(p, +k) = the FIRST k taps.
template <class T>
class WindowedSinc {
public:
    explicit WindowedSinc(std::vector<T> h) : h_(std::move(h)) {}
    int getMo2() const { return (int)(h_.size() - 1) / 2; }
    template <class It>
    T fms(It p) const {
        return fms(p, (int)h_.size());
    }
    template <class It>
    T fms(It p, int count) const {
        T acc = 0;
        if (count >= 0) {
            for (int k = 0; k < count; ++k) acc += h_[(size_t)k] * (T)p[k];
        } else {
            const size_t off = h_.size() - (size_t)(-count);
            for (int k = 0; k < -count; ++k) acc += h_[off + (size_t)k] * (T)p[k];
        }
        return acc;
    }

private:
    std::vector<T> h_;
};

class ThreadSafeProgress {
public:
    void report(size_t count) { counter_.fetch_add(count, std::memory_order_relaxed); }
    size_t count() const { return counter_.load(); }

private:
    std::atomic<size_t> counter_{0};
};

} // namespace Diskerror
