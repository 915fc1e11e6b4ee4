// FASTA reader interface used by the overlap-alignment caller
// (reference common/io/include/claraparabricks/genomeworks/io/fasta_parser.hpp:26-74,
// common/io/src/kseqpp_fasta_parser.cpp:31-72).  Same names and semantics:
// records keep the first word of the header as the name, records shorter than
// min_sequence_length are dropped, and shuffle reorders them with
// std::shuffle(std::mt19937(0)) for a deterministic order.
#pragma once

#include <claraparabricks/genomeworks/types.hpp>

#include <memory>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace io
{

typedef struct
{
    std::string name; ///< header up to the first whitespace
    std::string seq;  ///< bases, all lines joined
} FastaSequence;

class FastaParser
{
public:
    virtual ~FastaParser() = default;
    /// Number of records (the reference's spelling is kept).
    virtual number_of_reads_t get_num_seqences() const = 0;
    /// Record by index; throws std::out_of_range for an index beyond the last record.
    virtual const FastaSequence& get_sequence_by_id(read_id_t sequence_id) const = 0;
};

/// Parses a FASTA (or FASTQ) file.  Throws std::invalid_argument for a missing or empty file.
std::unique_ptr<FastaParser> create_kseq_fasta_parser(const std::string& fasta_file,
                                                      number_of_basepairs_t min_sequence_length = 0,
                                                      bool shuffle                              = true);

/// In-memory parser over records already read (this build's addition; used by the C ABI).
std::unique_ptr<FastaParser> create_fasta_parser_from_sequences(std::vector<FastaSequence> records);

} // namespace io
} // namespace genomeworks
} // namespace claraparabricks
