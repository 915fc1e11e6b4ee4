// Host-side helpers shared by the POA batch and the aligner (C++ API + C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#define GWAMD_HIP_CHECK(expr)                                                                                  \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e__) + " at " #expr);       \
    } while (0)

namespace gwamd
{
namespace host
{

// Tuning and diagnostic switches (GWAMD_POA_KERNEL, GWAMD_TB_WALK,
// GWAMD_BAND_FWD, ...): read only when GWAMD_DIAG=1 is set, so a drop-in
// user's environment never changes which kernel runs.  The parity tests set
// GWAMD_DIAG=1 (tests/conftest.py).  GWAMD_SPOA_ACCURATE is not one of them:
// it is the runtime form of the reference's spoa_accurate build option.
inline bool diag_enabled()
{
    const char* d = std::getenv("GWAMD_DIAG");
    return d && d[0] == '1' && d[1] == '\0';
}
inline const char* diag_env(const char* name) { return diag_enabled() ? std::getenv(name) : nullptr; }

// Per-thread message of the last failed C ABI call (gwamd_last_error()).
inline std::string& last_error()
{
    thread_local std::string s;
    return s;
}

struct ScopedDevice
{
    int prev = -1;
    explicit ScopedDevice(int dev)
    {
        GWAMD_HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev)
            GWAMD_HIP_CHECK(hipSetDevice(dev));
    }
    ~ScopedDevice()
    {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0)
            (void)hipSetDevice(prev);
    }
};

class PinnedBuf
{
public:
    ~PinnedBuf() { release(); }
    void reserve(size_t bytes, hipStream_t stream)
    {
        if (bytes <= cap_)
            return;
        size_t ncap = std::max(bytes, cap_ * 2);
        void* np    = nullptr;
        GWAMD_HIP_CHECK(hipHostMalloc(&np, ncap, hipHostMallocDefault));
        if (p_)
        {
            // an async H2D copy may still read the old buffer
            GWAMD_HIP_CHECK(hipStreamSynchronize(stream));
            std::memcpy(np, p_, used_);
            (void)hipHostFree(p_);
        }
        p_   = np;
        cap_ = ncap;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p_); }
    size_t used_ = 0;

private:
    void release()
    {
        if (p_)
            (void)hipHostFree(p_);
        p_ = nullptr;
    }
    void* p_    = nullptr;
    size_t cap_ = 0;
};

} // namespace host
} // namespace gwamd
