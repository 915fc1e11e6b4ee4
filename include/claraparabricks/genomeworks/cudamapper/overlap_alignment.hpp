// The cudamapper caller of the global aligner: base-level alignment of overlap
// regions and PAF output (reference cudamapper/src/main.cu:48-175,
// cudamapper/src/cudamapper_utils.cpp:30-112).  The rest of cudamapper
// (indexing, matching, overlapping) is outside this build.
#pragma once

#include <claraparabricks/genomeworks/cudamapper/types.hpp>
#include <claraparabricks/genomeworks/io/fasta_parser.hpp>
#include <claraparabricks/genomeworks/utils/allocator.hpp>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudamapper
{

/// Globally aligns the overlapped region of every overlap (Hirschberg-Myers,
/// create_aligner's global aligner) on the current device and writes one CIGAR
/// per overlap into cigars (resized to overlaps.size()).  A Reverse overlap
/// aligns the query region against the reverse complement of the target
/// region.  num_alignment_engines host threads each drive one aligner on its own
/// stream and take batches of overlaps from a shared counter
/// (main.cu:48-122,132-175).  Throws std::runtime_error when an overlap cannot
/// be added ("Experienced error type N") or num_alignment_engines < 1.
void align_overlaps(DefaultDeviceAllocator allocator, std::vector<Overlap>& overlaps,
                    const io::FastaParser& query_parser, const io::FastaParser& target_parser,
                    int32_t num_alignment_engines, std::vector<std::string>& cigars);

/// Overlaps in PAF, one line each, with "\tcg:Z:<cigar>" when cigars is not
/// empty (cudamapper_utils.cpp:30-112).  Column 10 is num_residues_ x
/// kmer_size, column 11 the longer of the two overlap spans, column 12 is 255.
std::string format_paf(const std::vector<Overlap>& overlaps, const std::vector<std::string>& cigars,
                       const io::FastaParser& query_parser, const io::FastaParser& target_parser,
                       int32_t kmer_size);

/// format_paf written to stdout under write_output_mutex (the reference's print_paf).
void print_paf(const std::vector<Overlap>& overlaps, const std::vector<std::string>& cigars,
               const io::FastaParser& query_parser, const io::FastaParser& target_parser, int32_t kmer_size,
               std::mutex& write_output_mutex);

} // namespace cudamapper
} // namespace genomeworks
} // namespace claraparabricks
