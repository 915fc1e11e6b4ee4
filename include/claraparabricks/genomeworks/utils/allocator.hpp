// Device allocator handle accepted by create_aligner (the reference's
// common/base/include/claraparabricks/genomeworks/utils/allocator.hpp:282-298).
// The MI355X aligner allocates its own device slabs with hipMalloc; this type
// only carries the caller's caching budget so the reference signature is kept.
#pragma once

#include <cstdint>

namespace claraparabricks
{
namespace genomeworks
{

class DefaultDeviceAllocator
{
public:
    DefaultDeviceAllocator() = default;
    explicit DefaultDeviceAllocator(int64_t max_cached_bytes)
        : max_cached_bytes_(max_cached_bytes)
    {
    }
    int64_t max_cached_bytes() const { return max_cached_bytes_; }

private:
    int64_t max_cached_bytes_ = -1;
};

inline DefaultDeviceAllocator create_default_device_allocator(int64_t max_cached_bytes = -1)
{
    return DefaultDeviceAllocator(max_cached_bytes);
}

} // namespace genomeworks
} // namespace claraparabricks
