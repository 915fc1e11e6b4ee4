// Internal hooks of the HIP Batch implementation (poa_batch.cpp) used by the
// multi-batch driver (poa_multibatch.cpp).  Not part of the drop-in API.
#pragma once

#include <claraparabricks/genomeworks/cudapoa/batch.hpp>

#include <hip/hip_runtime.h>

#include <cstdint>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{
namespace detail
{

/// Records `start` / `stop` on the batch's stream around every kernel launch
/// of `batch` (nullptr events switch it off).  `batch` must come from create_batch.
void set_launch_events(Batch* batch, hipEvent_t start, hipEvent_t stop);

/// Sum of the DP cells (SURVEY 8(d) priced cells) of the last launch's
/// windows; synchronises the batch's stream.
int64_t last_launch_cells(Batch* batch);

/// max_sequence_size of the batch (the longest read it accepts).
int32_t max_sequence_size(const Batch* batch);

} // namespace detail
} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks
