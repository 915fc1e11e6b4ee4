// MI355X drop-in for cudaaligner/include/claraparabricks/genomeworks/cudaaligner/aligner.hpp.
// The only signature change: hipStream_t instead of cudaStream_t.
#pragma once

#include <claraparabricks/genomeworks/cudaaligner/alignment.hpp>
#include <claraparabricks/genomeworks/cudaaligner/cudaaligner.hpp>
#include <claraparabricks/genomeworks/utils/allocator.hpp>

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudaaligner
{

/// Batched aligner (aligner.hpp:42-77).
class Aligner
{
public:
    virtual ~Aligner() = default;
    /// Launch alignment of every pair added so far (asynchronous).
    virtual StatusType align_all() = 0;
    /// Wait for align_all() and fill the Alignment objects.
    virtual StatusType sync_alignments() = 0;
    /// Copy a pair into the batch (optionally reverse-complemented).
    virtual StatusType add_alignment(const char* query, int32_t query_length, const char* target,
                                     int32_t target_length, bool reverse_complement_query = false,
                                     bool reverse_complement_target = false) = 0;
    virtual const std::vector<std::shared_ptr<Alignment>>& get_alignments() const = 0;
    virtual void reset() = 0;
};

/// Global aligner (Hirschberg + Myers) on device_id / stream (aligner.hpp:90).
std::unique_ptr<Aligner> create_aligner(int32_t max_query_length, int32_t max_target_length,
                                        int32_t max_alignments, AlignmentType type,
                                        DefaultDeviceAllocator allocator, hipStream_t stream, int32_t device_id);

/// Same, with the caching budget of the reference's allocator (aligner.hpp:103).
std::unique_ptr<Aligner> create_aligner(int32_t max_query_length, int32_t max_target_length,
                                        int32_t max_alignments, AlignmentType type, hipStream_t stream,
                                        int32_t device_id, int64_t max_device_memory_allocator_caching_size = -1);

/// The reference's other global aligners, which its tests construct directly
/// (cudaaligner/src/aligner_global_{myers,myers_banded,ukkonen}.hpp;
/// Test_AlignerGlobal.cpp:181-216).  create_aligner() keeps returning the
/// Hirschberg + Myers aligner, as in the reference.
enum class GlobalAlgorithm : int32_t
{
    hirschberg_myers = 0, ///< AlignerGlobalHirschbergMyers (create_aligner's choice)
    myers            = 1, ///< AlignerGlobalMyers: full bit-vector matrix + backtrace
    myers_banded     = 2, ///< AlignerGlobalMyersBanded: Ukkonen-banded Myers with band doubling
    ukkonen          = 3, ///< AlignerGlobalUkkonen: banded NW, p = 100, |q - t| <= 10% of max_target_length
};

std::unique_ptr<Aligner> create_global_aligner(int32_t max_query_length, int32_t max_target_length,
                                               int32_t max_alignments, GlobalAlgorithm algorithm,
                                               hipStream_t stream, int32_t device_id);

} // namespace cudaaligner
} // namespace genomeworks
} // namespace claraparabricks
