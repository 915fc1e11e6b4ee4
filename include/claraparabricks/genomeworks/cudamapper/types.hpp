// Overlap record of the cudamapper overlap-alignment caller
// (reference cudamapper/include/claraparabricks/genomeworks/cudamapper/types.hpp:40-89).
// Field order, types and the strand characters are kept, so an Overlap array
// produced by the reference's overlapper can be handed over as is.
#pragma once

#include <claraparabricks/genomeworks/types.hpp>

#include <cstdint>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudamapper
{

/// Whether query and target lie on the same DNA strand.
enum class RelativeStrand : unsigned char
{
    Forward = '+',
    Reverse = '-',
};

/// One overlap: [start, end) ranges on a query read and a target read.
typedef struct Overlap
{
    read_id_t query_read_id_;
    read_id_t target_read_id_;
    position_in_read_t query_start_position_in_read_;
    position_in_read_t target_start_position_in_read_;
    position_in_read_t query_end_position_in_read_;
    position_in_read_t target_end_position_in_read_;
    RelativeStrand relative_strand;
    std::uint32_t num_residues_ = 0; ///< anchors chained into the overlap
    bool overlap_complete       = false;
} Overlap;

} // namespace cudamapper
} // namespace genomeworks
} // namespace claraparabricks
