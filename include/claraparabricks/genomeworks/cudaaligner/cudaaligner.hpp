// MI355X drop-in for cudaaligner/include/claraparabricks/genomeworks/cudaaligner/cudaaligner.hpp.
// Enum values are ABI (cudaaligner.hpp:26-53 of the reference).
#pragma once

#include <cstdint>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudaaligner
{

/// Aligner status (reference cudaaligner.hpp:27-35).
enum StatusType
{
    success = 0,
    uninitialized,
    exceeded_max_alignments,
    exceeded_max_length,
    exceeded_max_alignment_difference,
    generic_error
};

/// Alignment type (cudaaligner.hpp:38-42).
enum AlignmentType
{
    global_alignment = 0,
    unset
};

/// One position of an alignment (cudaaligner.hpp:45-52).
enum AlignmentState : int8_t
{
    match = 0,
    mismatch,
    insertion, // absent in query, present in target
    deletion   // present in query, absent in target
};

/// Initialise the aligner context (cudaaligner.cpp:24-30).
StatusType Init();

} // namespace cudaaligner
} // namespace genomeworks
} // namespace claraparabricks

namespace claragenomics = claraparabricks::genomeworks;
