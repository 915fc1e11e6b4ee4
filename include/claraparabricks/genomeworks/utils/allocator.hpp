// Device allocator handle accepted by create_aligner (the reference's
// common/base/include/claraparabricks/genomeworks/utils/allocator.hpp:282-305).
// The reference's DefaultDeviceAllocator (GW_ENABLE_CACHING_ALLOCATOR, ON by
// default, CMakeLists.txt:33) is a caching allocator over one preallocated
// pool whose shared_ptr<MemoryResource> is shared by every copy
// (allocator.hpp:274-279): aligners created from copies of one allocator draw
// on one pool and jointly cannot exceed it.  The MI355X aligner allocates its
// own device slabs with hipMalloc; this handle carries the pool's byte budget,
// shared the same way (copies share one DeviceBudget), and each aligner
// reserves its device bytes from it for its lifetime.
#pragma once

#include <algorithm>
#include <cstdint>
#include <memory>
#include <mutex>

namespace claraparabricks
{
namespace genomeworks
{

// Byte budget of one pool (capacity < 0: all available device memory).
class DeviceBudget
{
public:
    explicit DeviceBudget(int64_t capacity)
        : capacity_(capacity)
    {
    }
    int64_t capacity() const { return capacity_; }
    int64_t used() const
    {
        std::lock_guard<std::mutex> lk(mu_);
        return used_;
    }
    // Reserves up to `want` bytes and at least `at_least`; returns the bytes
    // reserved, or -1 (nothing reserved) when fewer than `at_least` are left.
    int64_t reserve(int64_t at_least, int64_t want)
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (capacity_ < 0)
        {
            used_ += want;
            return want;
        }
        const int64_t left = capacity_ - used_;
        if (left < at_least)
            return -1;
        const int64_t r = std::min(want, left);
        used_ += r;
        return r;
    }
    void release(int64_t bytes)
    {
        std::lock_guard<std::mutex> lk(mu_);
        used_ -= bytes;
    }

private:
    const int64_t capacity_;
    int64_t used_ = 0;
    mutable std::mutex mu_;
};

class DefaultDeviceAllocator
{
public:
    // default construction: no pool of its own, the aligner may use all
    // available device memory
    DefaultDeviceAllocator() = default;
    explicit DefaultDeviceAllocator(int64_t max_cached_bytes)
        : budget_(std::make_shared<DeviceBudget>(max_cached_bytes))
    {
    }
    int64_t max_cached_bytes() const { return budget_ ? budget_->capacity() : -1; }
    // the pool shared by every copy of this allocator (null: unlimited)
    const std::shared_ptr<DeviceBudget>& budget() const { return budget_; }

private:
    std::shared_ptr<DeviceBudget> budget_;
};

// allocator.hpp:297-305: a 2 GiB pool unless told otherwise (-1: all
// available device memory)
inline DefaultDeviceAllocator create_default_device_allocator(int64_t max_caching_size = int64_t(2) << 30)
{
    return DefaultDeviceAllocator(max_caching_size);
}

} // namespace genomeworks
} // namespace claraparabricks
