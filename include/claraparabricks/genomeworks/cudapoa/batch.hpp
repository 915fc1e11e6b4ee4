// Drop-in replacement for the reference's cudapoa/batch.hpp
// (cudapoa/include/claraparabricks/genomeworks/cudapoa/batch.hpp:39-228).
// Same types, members, defaults and validation; the only signature change is
// hipStream_t for cudaStream_t.
#pragma once

#include <claraparabricks/genomeworks/cudapoa/cudapoa.hpp>
#include <claraparabricks/genomeworks/utils/graph.hpp>

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

namespace detail
{
inline int32_t align_up(int32_t v, int32_t a) { return ((v + a - 1) / a) * a; }
inline int32_t check_non_negative(int32_t v, const char* msg)
{
    if (v < 0)
        throw std::invalid_argument(msg);
    return v;
}
} // namespace detail

/// A sequence entry (batch.hpp:39-47).
struct Entry
{
    const char* seq;
    const int8_t* weights;
    int32_t length;
};

/// Set and order of entries processed as one POA (batch.hpp:50).
typedef std::vector<Entry> Group;

/// Upper limits of a POA batch (batch.hpp:53-129).
struct BatchSize
{
    int32_t max_sequence_size;
    int32_t max_consensus_size;
    int32_t max_nodes_per_window;
    int32_t max_nodes_per_window_banded;
    int32_t max_matrix_graph_dimension        = max_nodes_per_window;
    int32_t max_matrix_graph_dimension_banded = max_nodes_per_window_banded;
    int32_t max_matrix_sequence_dimension     = max_sequence_size;
    int32_t alignment_band_width;
    int32_t max_sequences_per_poa;

    BatchSize(int32_t max_seq_sz = 1024, int32_t max_seq_per_poa = 100, int32_t band_width = 256)
        : max_sequence_size(max_seq_sz)
        , max_consensus_size(2 * max_sequence_size)
        , max_nodes_per_window(detail::align_up(3 * max_sequence_size, 4))
        , max_nodes_per_window_banded(detail::align_up(4 * max_sequence_size, 4))
        , max_matrix_graph_dimension(detail::align_up(max_nodes_per_window, 4))
        , max_matrix_graph_dimension_banded(detail::align_up(max_nodes_per_window_banded, 4))
        , max_matrix_sequence_dimension(detail::align_up(max_sequence_size, 4))
        , alignment_band_width(detail::align_up(band_width, 128))
        , max_sequences_per_poa(max_seq_per_poa)
    {
        detail::check_non_negative(max_seq_sz, "max_sequence_size cannot be negative.");
        detail::check_non_negative(max_seq_per_poa, "max_sequences_per_poa cannot be negative.");
        detail::check_non_negative(band_width, "alignment_band_width cannot be negative.");
        if (alignment_band_width != band_width)
            std::cerr << "Band-width should be multiple of 128. The input was changed from " << band_width << " to "
                      << alignment_band_width << std::endl;
    }

    BatchSize(int32_t max_seq_sz, int32_t max_consensus_sz, int32_t max_nodes_per_w, int32_t max_nodes_per_w_banded,
              int32_t band_width, int32_t max_seq_per_poa)
        : max_sequence_size(max_seq_sz)
        , max_consensus_size(max_consensus_sz)
        , max_nodes_per_window(detail::align_up(max_nodes_per_w, 4))
        , max_nodes_per_window_banded(detail::align_up(max_nodes_per_w_banded, 4))
        , max_matrix_graph_dimension(detail::align_up(max_nodes_per_window, 4))
        , max_matrix_graph_dimension_banded(detail::align_up(max_nodes_per_window_banded, 4))
        , max_matrix_sequence_dimension(detail::align_up(max_sequence_size, 4))
        , alignment_band_width(detail::align_up(band_width, 128))
        , max_sequences_per_poa(max_seq_per_poa)
    {
        detail::check_non_negative(max_seq_sz, "max_sequence_size cannot be negative.");
        detail::check_non_negative(max_consensus_sz, "max_consensus_size cannot be negative.");
        detail::check_non_negative(max_nodes_per_w, "max_nodes_per_window cannot be negative.");
        detail::check_non_negative(max_nodes_per_w_banded, "max_nodes_per_window_banded cannot be negative.");
        detail::check_non_negative(max_seq_per_poa, "max_sequences_per_poa cannot be negative.");
        detail::check_non_negative(band_width, "alignment_band_width cannot be negative.");
        if (max_nodes_per_window < max_sequence_size)
            throw std::invalid_argument("max_nodes_per_window should be greater than or equal to max_sequence_size.");
        if (max_nodes_per_window_banded < max_sequence_size)
            throw std::invalid_argument("max_nodes_per_window should be greater than or equal to max_sequence_size.");
        if (max_consensus_size < max_sequence_size)
            throw std::invalid_argument("max_consensus_size should be greater than or equal to max_sequence_size.");
        if (max_sequence_size < alignment_band_width)
            throw std::invalid_argument("alignment_band_width should not be greater than max_sequence_size.");
    }
};

/// Batched POA object (batch.hpp:133-205).
class Batch
{
public:
    virtual ~Batch() = default;

    /// Adds a group (one window); per_seq_status is cleared and filled per entry.
    virtual StatusType add_poa_group(std::vector<StatusType>& per_seq_status, const Group& poa_group) = 0;

    /// Number of POAs (windows) in the batch.
    virtual int32_t get_total_poas() const = 0;

    /// Runs POA over all windows (asynchronous on the batch stream).
    virtual void generate_poa() = 0;

    /// Consensus and per-base coverage per window; blocks on the stream.
    virtual StatusType get_consensus(std::vector<std::string>& consensus, std::vector<std::vector<uint16_t>>& coverage,
                                     std::vector<StatusType>& output_status) = 0;

    /// Multiple sequence alignment rows per window; blocks on the stream.
    virtual StatusType get_msa(std::vector<std::vector<std::string>>& msa, std::vector<StatusType>& output_status) = 0;

    /// Final POA graph per window.
    virtual void get_graphs(std::vector<DirectedGraph>& graphs, std::vector<StatusType>& output_status) = 0;

    virtual int32_t batch_id() const = 0;

    /// Rewinds the batch for re-use.
    virtual void reset() = 0;
};

/// Creates a batch (batch.hpp:220-228).  Throws std::runtime_error when max_mem
/// cannot hold one window and std::invalid_argument on negative arguments.
std::unique_ptr<Batch> create_batch(int32_t device_id, hipStream_t stream, size_t max_mem, int8_t output_mask,
                                    const BatchSize& batch_size, int16_t gap_score, int16_t mismatch_score,
                                    int16_t match_score, bool cuda_banded_alignment);

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks
