// Drop-in replacement for the reference's cudapoa/cudapoa.hpp
// (cudapoa/include/claraparabricks/genomeworks/cudapoa/cudapoa.hpp:26-48).
// Enum values are ABI and identical to the reference.
#pragma once

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

/// POA status / error type (cudapoa.hpp:26-38).
enum StatusType
{
    success = 0,
    exceeded_maximum_poas,
    exceeded_maximum_sequence_size,
    exceeded_maximum_sequences_per_poa,
    node_count_exceeded_maximum_graph_size,
    edge_count_exceeded_maximum_graph_size,
    seq_len_exceeded_maximum_nodes_per_window,
    loop_count_exceeded_upper_bound,
    output_type_unavailable,
    generic_error
};

/// Initialize the POA context (cudapoa.hpp:41): loads the HIP code object.
StatusType Init();

/// Output selection bit mask (cudapoa.hpp:44-48).
enum OutputType
{
    consensus = 0x1,
    msa       = 0x1 << 1
};

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks

/// Legacy namespace named by the north star (docs/cpp snapshot).
namespace claragenomics = claraparabricks::genomeworks;
