// register_alias.hip -- what HIP reports for a hipHostRegister'd sub-range of
// a pageable buffer, and whether copies through hipHostMalloc'd buffers stay
// correct beside it (development tool, not part of the product).
//
// Written while building the REGISTER staging variant
// (scripts/variants/register_staging/): its first version moved the unaligned
// ends of a call through the slot's bounce buffers and, with a one-tap
// identity filter, got the pinned interior's bytes there.  This tool showed
// the runtime copies correctly and found the cause: hipMemGetAddressRange on a
// registered range returns its size but a NULL base, so lcfir's host_pinned()
// took the registration for pageable memory and sent the interior through the
// same bounce buffers, overwriting the ends' bytes before their DMAs ran.
// Prints the pointer attributes, the address-range query, and the check of
// every copy (profiles/r06_dropin/register_probe.log).
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 register_alias.hip -o register_alias
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static void attrs(const char *what, const void *p) {
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        std::printf("  %-22s %p: no attributes (%s)\n", what, p, hipGetErrorString(e));
        return;
    }
    std::printf("  %-22s %p: type %d device %d devicePointer %p hostPointer %p\n", what, p, (int)a.type, a.device,
                a.devicePointer, a.hostPointer);
}

static int check(const char *what, const float *got, const float *want, size_t n) {
    size_t bad = 0, first = n;
    for (size_t i = 0; i < n; ++i)
        if (got[i] != want[i]) {
            if (first == n) first = i;
            ++bad;
        }
    if (bad)
        std::printf("%-40s WRONG: %zu of %zu floats, first at %zu: got %.1f want %.1f\n", what, bad, n, first,
                    got[first], want[first]);
    else
        std::printf("%-40s ok (%zu floats)\n", what, n);
    return bad ? 1 : 0;
}

int main() {
    const size_t n = 12000003, bytes = n * sizeof(float);
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<float> x(n), y(n);
    for (size_t i = 0; i < n; ++i) x[i] = (float)i + 0.5f;
    float *d = nullptr;
    CK(hipMalloc(&d, bytes));
    constexpr size_t kB = (size_t)4 << 20;
    void *bounce[2];
    CK(hipHostMalloc(&bounce[0], kB, hipHostMallocDefault));
    CK(hipHostMalloc(&bounce[1], kB, hipHostMallocDefault));
    // a "call" over x[start, end): pin the interior, head and tail by bounce
    const size_t start = 700001, end = 2238641;
    const auto b0 = reinterpret_cast<uintptr_t>(x.data() + start);
    const uintptr_t p0 = (b0 + 4095) & ~(uintptr_t)4095, p1 = reinterpret_cast<uintptr_t>(x.data() + end) & ~(uintptr_t)4095;
    std::printf("x %p, interior [%#lx, %#lx) = %zu B; bounce %p %p\n", (void *)x.data(), (unsigned long)p0,
                (unsigned long)p1, (size_t)(p1 - p0), bounce[0], bounce[1]);
    attrs("bounce[0] before", bounce[0]);
    attrs("bounce[1] before", bounce[1]);
    CK(hipHostRegister(reinterpret_cast<void *>(p0), p1 - p0, hipHostRegisterDefault));
    attrs("interior", reinterpret_cast<void *>(p0));
    attrs("interior + 4 MiB", reinterpret_cast<void *>(p0 + kB));
    {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        const hipError_t e = hipMemGetAddressRange(&base, &size, reinterpret_cast<void *>(p0 + 4096));
        std::printf("  hipMemGetAddressRange(interior + 4 KiB): %s, base %p size %zu\n", hipGetErrorString(e),
                    (void *)base, size);
        (void)hipGetLastError();
    }
    attrs("bounce[0] after", bounce[0]);
    attrs("bounce[1] after", bounce[1]);
    const size_t head = p0 - b0, tail = reinterpret_cast<uintptr_t>(x.data() + end) - p1;
    int bad = 0;
    // H2D: head via bounce[0], interior direct, tail via bounce[1]
    CK(hipMemset(d, 0, bytes));
    std::memcpy(bounce[0], x.data() + start, head);
    CK(hipMemcpyAsync(d + start, bounce[0], head, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(reinterpret_cast<char *>(d + start) + head, reinterpret_cast<void *>(p0), p1 - p0,
                      hipMemcpyHostToDevice, s));
    std::memcpy(bounce[1], reinterpret_cast<void *>(p1), tail);
    CK(hipMemcpyAsync(reinterpret_cast<char *>(d + end) - tail, bounce[1], tail, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(y.data() + start, d + start, (end - start) * 4, hipMemcpyDeviceToHost));
    bad += check("H2D head (bounce[0])", y.data() + start, x.data() + start, head / 4);
    bad += check("H2D interior (registered)", y.data() + start + head / 4, x.data() + start + head / 4,
                 (p1 - p0) / 4);
    bad += check("H2D tail (bounce[1])", y.data() + end - tail / 4, x.data() + end - tail / 4, tail / 4);
    // the same small copies with a plain hipMemcpy (synchronous)
    CK(hipMemset(d, 0, bytes));
    CK(hipMemcpy(d + start, bounce[0], head, hipMemcpyHostToDevice));
    CK(hipMemcpy(y.data() + start, d + start, head, hipMemcpyDeviceToHost));
    bad += check("hipMemcpy head from bounce[0]", y.data() + start, x.data() + start, head / 4);
    // D2H into the bounce buffers
    std::memset(bounce[0], 0, kB);
    std::memset(bounce[1], 0, kB);
    CK(hipMemcpy(d, x.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpyAsync(bounce[0], d + start, head, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(bounce[1], reinterpret_cast<char *>(d + end) - tail, tail, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    bad += check("D2H head into bounce[0]", static_cast<float *>(bounce[0]), x.data() + start, head / 4);
    bad += check("D2H tail into bounce[1]", static_cast<float *>(bounce[1]), x.data() + end - tail / 4, tail / 4);
    CK(hipHostUnregister(reinterpret_cast<void *>(p0)));
    // after unregistering: the head copy again
    CK(hipMemset(d, 0, bytes));
    CK(hipMemcpy(d + start, bounce[0], head, hipMemcpyHostToDevice));
    CK(hipMemcpy(y.data() + start, d + start, head, hipMemcpyDeviceToHost));
    std::memcpy(bounce[0], x.data() + start, head);
    CK(hipMemcpy(d + start, bounce[0], head, hipMemcpyHostToDevice));
    CK(hipMemcpy(y.data() + start, d + start, head, hipMemcpyDeviceToHost));
    bad += check("after unregister: head via bounce[0]", y.data() + start, x.data() + start, head / 4);
    std::printf("%s\n", bad ? "COPIES WRONG" : "all copies correct");
    return 0;
}
