// common.h -- shared definitions for libmpss (MI355X-native multipole subsurface path).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <stdexcept>

namespace mpss {

constexpr int NB = 30;      // nSpectralSamples (reference src/core/spectrum.h:46)
constexpr int ROW = 32;     // padded spectral row: 30 bands + 2 pad lanes, 128 B per row

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define MPSS_HIP(expr)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            throw ::mpss::Error(-3, std::string("HIP error ") + hipGetErrorString(e_) + " at " \
                                        + __FILE__ + ":" + std::to_string(__LINE__));         \
    } while (0)

template <class T>
struct DevBuf {
    T *ptr = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        release();
        if (count == 0) return;
        MPSS_HIP(hipMalloc(&ptr, count * sizeof(T)));
        n = count;
    }
    void upload(const T *host, size_t count) {
        if (count > n) alloc(count);
        if (count) MPSS_HIP(hipMemcpy(ptr, host, count * sizeof(T), hipMemcpyHostToDevice));
    }
};

}  // namespace mpss
