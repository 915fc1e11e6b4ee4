// Basic id/position types (reference common/base/include/claraparabricks/genomeworks/types.hpp:30-39).
#pragma once

#include <cstdint>

namespace claraparabricks
{
namespace genomeworks
{

using read_id_t             = std::uint32_t; ///< read index within a parser
using number_of_reads_t     = read_id_t;
using position_in_read_t    = std::uint32_t; ///< base position within a read
using number_of_basepairs_t = position_in_read_t;

} // namespace genomeworks
} // namespace claraparabricks
