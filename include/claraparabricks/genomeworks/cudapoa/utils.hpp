// Window input formats and multi-batch sizing for the cudapoa drop-in API
// (reference: cudapoa/include/claraparabricks/genomeworks/cudapoa/utils.hpp:48-175,
// cudapoa/src/utils.cu:24-138).  Same names, argument meaning and defaults.
#pragma once

#include <claraparabricks/genomeworks/cudapoa/batch.hpp>

#include <cassert>
#include <cstdint>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

/// Bins POA groups by how many of them fit one batch and returns a small set
/// of BatchSize values covering all groups (reference utils.cu:24-138).
/// The per-group capacity is the reference's BatchBlock::estimate_max_poas
/// (allocate_block.hpp:364-401): gpu_memory_usage_quota x free device memory
/// over (device bytes per POA + score matrix bytes).
void get_multi_batch_sizes(std::vector<BatchSize>& list_of_batch_sizes,
                           std::vector<std::vector<int32_t>>& list_of_groups_per_batch,
                           const std::vector<Group>& poa_groups,
                           bool banded_alignment               = true,
                           bool msa_flag                       = false,
                           int32_t band_width                  = 256,
                           std::vector<int32_t>* bins_capacity = nullptr,
                           float gpu_memory_usage_quota        = 0.9,
                           int32_t mismatch_score              = -6,
                           int32_t gap_score                   = -8,
                           int32_t match_score                 = 8);

/// As get_multi_batch_sizes, with the free device memory given instead of
/// queried (host-side tests and planning for another device).
void get_multi_batch_sizes_for_memory(std::vector<BatchSize>& list_of_batch_sizes,
                                      std::vector<std::vector<int32_t>>& list_of_groups_per_batch,
                                      const std::vector<Group>& poa_groups, size_t free_device_memory,
                                      bool banded_alignment = true, bool msa_flag = false, int32_t band_width = 256,
                                      std::vector<int32_t>* bins_capacity = nullptr,
                                      float gpu_memory_usage_quota = 0.9, int32_t mismatch_score = -6,
                                      int32_t gap_score = -8, int32_t match_score = 8);

/// Maximum POAs of one batch (reference BatchBlock::estimate_max_poas).
int64_t estimate_max_poas(const BatchSize& batch_size, bool banded_alignment, bool msa_flag,
                          size_t free_device_memory, float memory_usage_quota, int32_t mismatch_score,
                          int32_t gap_score, int32_t match_score);

/// Truncates or cyclically repeats the windows to total_windows (-1: keep all).
inline void resize_windows(std::vector<std::vector<std::string>>& windows, const int32_t total_windows)
{
    if (total_windows < 0)
        return;
    if (int32_t(windows.size()) > total_windows)
        windows.erase(windows.begin() + total_windows, windows.end());
    else if (int32_t(windows.size()) < total_windows)
    {
        const size_t read = windows.size();
        if (read == 0)
            throw std::runtime_error("resize_windows: no windows to repeat");
        while (int32_t(windows.size()) != total_windows)
            windows.push_back(windows[windows.size() - read]);
    }
    assert(int32_t(windows.size()) == total_windows);
}

/// Parses the cudapoa window format: a line with the number of sequences of
/// the window, then that many sequence lines, repeated.
inline void parse_cudapoa_file(std::vector<std::vector<std::string>>& windows, const std::string& filename,
                               int32_t total_windows)
{
    std::ifstream infile(filename);
    if (!infile.good())
        throw std::runtime_error("Cannot read file " + filename);
    std::string line;
    int32_t num_sequences = 0;
    while (std::getline(infile, line))
    {
        if (num_sequences == 0)
        {
            std::istringstream iss(line);
            iss >> num_sequences;
            windows.emplace_back();
        }
        else
        {
            windows.back().push_back(line);
            num_sequences--;
        }
    }
    resize_windows(windows, total_windows);
}

/// Reads all records of a (multi-line) FASTA file, in file order.
inline std::vector<std::string> read_fasta_sequences(const std::string& path)
{
    std::ifstream infile(path);
    if (!infile.good())
        throw std::runtime_error("Cannot read file " + path);
    std::vector<std::string> seqs;
    std::string line;
    bool in_record = false;
    while (std::getline(infile, line))
    {
        if (!line.empty() && line.back() == '\r')
            line.pop_back();
        if (!line.empty() && line[0] == '>')
        {
            seqs.emplace_back();
            in_record = true;
        }
        else if (in_record)
            seqs.back() += line;
    }
    return seqs;
}

/// One window per FASTA file (every record of the file is a read of the window).
inline void parse_fasta_files(std::vector<std::vector<std::string>>& windows,
                              const std::vector<std::string>& input_paths, const int32_t total_windows)
{
    windows.resize(input_paths.size());
    for (size_t i = 0; i < input_paths.size(); i++)
        windows[i] = read_fasta_sequences(input_paths[i]);
    resize_windows(windows, total_windows);
}

/// First line of a golden-value file.
inline std::string parse_golden_value_file(const std::string& filename)
{
    std::ifstream infile(filename);
    if (!infile.good())
        throw std::runtime_error("Cannot read file " + filename);
    std::string line;
    std::getline(infile, line);
    return line;
}

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks
