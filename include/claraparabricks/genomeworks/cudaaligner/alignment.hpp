// MI355X drop-in for cudaaligner/include/claraparabricks/genomeworks/cudaaligner/alignment.hpp.
#pragma once

#include <claraparabricks/genomeworks/cudaaligner/cudaaligner.hpp>

#include <cstdint>
#include <ostream>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudaaligner
{

/// Formatted alignment strings (alignment.hpp:33-43).
typedef struct FormattedAlignment
{
    std::string query;
    std::string pairing;
    std::string target;
    uint32_t linebreak_after = 80;
} FormattedAlignment;

/// Writes the three rows, wrapped at linebreak_after (alignment.cpp:22-41).
std::ostream& operator<<(std::ostream& os, const FormattedAlignment& formatted_alignment);

/// One alignment between a query and a target (alignment.hpp:50-85).
class Alignment
{
public:
    virtual ~Alignment() = default;
    virtual const std::string& get_query_sequence() const = 0;
    virtual const std::string& get_target_sequence() const = 0;
    /// Run-length CIGAR with M (match or mismatch), I and D.
    virtual std::string convert_to_cigar() const = 0;
    virtual AlignmentType get_alignment_type() const = 0;
    virtual StatusType get_status() const = 0;
    virtual const std::vector<AlignmentState>& get_alignment() const = 0;
    virtual FormattedAlignment format_alignment(int32_t maximal_line_length = 80) const = 0;
};

} // namespace cudaaligner
} // namespace genomeworks
} // namespace claraparabricks
