// cudapoa command-line tool on the MI355X batch (reference: cudapoa/src/main.cpp:30-289,
// application_parameters.cpp:30-210).  Same options, defaults and output:
// consensus (or MSA rows) per window on stdout, progress on stderr, optional
// graphs in DOT format.  Windows come from one cudapoa-format file or one or
// more FASTA files (one window per file), are binned by get_multi_batch_sizes
// and processed batch by batch.
#include <claraparabricks/genomeworks/cudapoa/batch.hpp>
#include <claraparabricks/genomeworks/cudapoa/cudapoa.hpp>
#include <claraparabricks/genomeworks/cudapoa/utils.hpp>

#include <hip/hip_runtime.h>

#include <getopt.h>

#include <cstdio>
#include <fstream>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

using namespace claraparabricks::genomeworks;
using namespace claraparabricks::genomeworks::cudapoa;

namespace
{

struct Parameters
{
    std::vector<std::string> input_paths;
    std::string graph_output_path;
    bool all_fasta            = true;
    bool msa                  = false;
    bool banded               = true;
    int32_t band_width        = 256;
    int32_t max_groups        = -1;
    double gpu_mem_allocation = 0.9;
    int32_t match_score       = 8;
    int32_t mismatch_score    = -6;
    int32_t gap_score         = -8;
};

[[noreturn]] void help(int code)
{
    std::cerr << R"(Usage: cudapoa [options ...]
     options:
        -i, --input <file>
            input in fasta/cudapoa format, can be used multiple times for multiple fasta files, but supports only one cudapoa file
        -a, --msa
            generates msa if this flag is passed [default: consensus]
        -f, --full-alignment
            uses full alignment if this flag is passed [banded alignment]
        -b, --band-width <int>
            band-width for banded alignment (must be multiple of 128) [256]
        -d, --dot <file>
            output path for printing graph in DOT format [disabled]
        -M, --max-groups  <int>
            maximum number of POA groups to create from file (-1 for all, > 0 for limited) [-1]
            repeats groups if less groups are present than specified
        -R, --gpu-mem-alloc <double>
            fraction of available GPU memory to be used for cudapoa [0.9]
        -m, --match  <int>
            score for matching bases (must be positive) [8]
        -n, --mismatch  <int>
            score for mismatching bases (must be non-positive) [-6]
        -g, --gap  <int>
            score for gaps (must be non-positive) [-8]
        -v, --version
            version information
        -h, --help
            prints usage
)";
    std::exit(code);
}

Parameters parse(int argc, char* argv[])
{
    Parameters p;
    const option options[] = {
        {"input", required_argument, 0, 'i'},      {"msa", no_argument, 0, 'a'},
        {"full-alignment", no_argument, 0, 'f'},   {"band-width", required_argument, 0, 'b'},
        {"dot", required_argument, 0, 'd'},        {"max-groups", required_argument, 0, 'M'},
        {"gpu-mem-alloc", required_argument, 0, 'R'}, {"match", required_argument, 0, 'm'},
        {"mismatch", required_argument, 0, 'n'},   {"gap", required_argument, 0, 'g'},
        {"version", no_argument, 0, 'v'},          {"help", no_argument, 0, 'h'},
        {0, 0, 0, 0},
    };
    int a = 0;
    while ((a = getopt_long(argc, argv, "i:afb:d:M:R:m:n:g:vh", options, nullptr)) != -1)
    {
        switch (a)
        {
        case 'i': p.input_paths.push_back(optarg); break;
        case 'a': p.msa = true; break;
        case 'f': p.banded = false; break;
        case 'b': p.band_width = std::stoi(optarg); break;
        case 'd': p.graph_output_path = optarg; break;
        case 'M': p.max_groups = std::stoi(optarg); break;
        case 'R': p.gpu_mem_allocation = std::stod(optarg); break;
        case 'm': p.match_score = std::stoi(optarg); break;
        case 'g': p.gap_score = std::stoi(optarg); break;
        case 'n': p.mismatch_score = std::stoi(optarg); break;
        case 'v': std::cerr << "claragenomicsanalysis_amd cudapoa (MI355X)" << std::endl; std::exit(1);
        case 'h': help(0);
        default: std::exit(1);
        }
    }
    // application_parameters.cpp:93-121
    if (p.gpu_mem_allocation <= 0 || p.gpu_mem_allocation > 1.0)
        throw std::runtime_error("gpu-mem-alloc should be greater than 0 and less than or equal to 1.0");
    if (p.banded && p.band_width < 1)
        throw std::runtime_error("band-width must be positive");
    if (p.match_score < 0)
        throw std::runtime_error("match score must be positive");
    if (p.max_groups == 0)
        throw std::runtime_error("max-groups cannot be 0");
    if (p.mismatch_score > 0)
        throw std::runtime_error("mismatch score must be non-positive");
    if (p.gap_score > 0)
        throw std::runtime_error("gap score must be non-positive");
    // application_parameters.cpp:124-147: all fasta, or exactly one cudapoa file
    for (const auto& path : p.input_paths)
    {
        std::ifstream in(path);
        if (!in.good())
            throw std::runtime_error("Invalid input file: " + path);
        std::string first;
        std::getline(in, first);
        if (first.empty() || first[0] != '>')
            p.all_fasta = false;
    }
    if (p.input_paths.empty() || (!p.all_fasta && p.input_paths.size() > 1))
    {
        std::cerr << "Invalid input. cudapoa needs input in either one cudapoa format file or in one/multiple fasta files."
                  << std::endl;
        help(1);
    }
    return p;
}

void process_batch(Batch* batch, bool msa, bool print)
{
    batch->generate_poa();
    if (msa)
    {
        std::vector<std::vector<std::string>> rows;
        std::vector<StatusType> status;
        if (batch->get_msa(rows, status) != StatusType::success)
            std::cerr << "Could not generate MSA for batch" << std::endl;
        for (size_t g = 0; g < rows.size(); g++)
        {
            if (status[g] != StatusType::success)
                std::cerr << "Error generating  MSA for POA group " << g << ". Error type " << int(status[g]) << std::endl;
            else if (print)
                for (const auto& r : rows[g])
                    std::cout << r << std::endl;
        }
    }
    else
    {
        std::vector<std::string> consensus;
        std::vector<std::vector<uint16_t>> coverage;
        std::vector<StatusType> status;
        if (batch->get_consensus(consensus, coverage, status) != StatusType::success)
            std::cerr << "Could not generate consensus for batch" << std::endl;
        for (size_t g = 0; g < consensus.size(); g++)
        {
            if (status[g] != StatusType::success)
                std::cerr << "Error generating consensus for POA group " << g << ". Error type " << int(status[g])
                          << std::endl;
            else if (print)
                std::cout << consensus[g] << std::endl;
        }
    }
}

int run(int argc, char* argv[])
{
    const Parameters prm = parse(argc, argv);
    std::vector<std::vector<std::string>> windows;
    if (prm.all_fasta)
        parse_fasta_files(windows, prm.input_paths, prm.max_groups);
    else
        parse_cudapoa_file(windows, prm.input_paths[0], prm.max_groups);

    std::ofstream graph_output;
    if (!prm.graph_output_path.empty())
    {
        graph_output.open(prm.graph_output_path);
        if (!graph_output)
        {
            std::cerr << "Error opening " << prm.graph_output_path << " for graph output" << std::endl;
            return -1;
        }
    }

    std::vector<Group> groups(windows.size());
    for (size_t i = 0; i < windows.size(); i++)
        for (const auto& s : windows[i])
            groups[i].push_back(Entry{s.c_str(), nullptr, int32_t(s.size())});

    std::vector<BatchSize> sizes;
    std::vector<std::vector<int32_t>> per_batch;
    get_multi_batch_sizes(sizes, per_batch, groups, prm.banded, prm.msa, prm.band_width, nullptr,
                          float(prm.gpu_mem_allocation), prm.mismatch_score, prm.gap_score, prm.match_score);

    if (Init() != StatusType::success)
        throw std::runtime_error("no HIP device");
    int32_t offset = 0;
    for (size_t b = 0; b < sizes.size(); b++)
    {
        // main.cpp:27-61: one batch on device 0, default stream, a fraction of free memory
        size_t free_mem = 0, total = 0;
        (void)hipSetDevice(0);
        (void)hipMemGetInfo(&free_mem, &total);
        const size_t mem = size_t(prm.gpu_mem_allocation * double(free_mem));
        std::unique_ptr<Batch> batch =
            create_batch(0, nullptr, mem, prm.msa ? OutputType::msa : OutputType::consensus, sizes[b],
                         int16_t(prm.gap_score), int16_t(prm.mismatch_score), int16_t(prm.match_score), prm.banded);
        const auto& ids = per_batch[b];
        int32_t group_count = 0;
        for (int32_t i = 0; i < int32_t(ids.size());)
        {
            std::vector<StatusType> seq_status;
            const StatusType st = batch->add_poa_group(seq_status, groups[ids[i]]);
            if (st == StatusType::exceeded_maximum_poas || i == int32_t(ids.size()) - 1)
            {
                if (batch->get_total_poas() > 0)
                {
                    process_batch(batch.get(), prm.msa, true);
                    if (graph_output.is_open())
                    {
                        if (!graph_output.good())
                            throw std::runtime_error("Error writing dot file");
                        std::vector<DirectedGraph> graphs;
                        std::vector<StatusType> gst;
                        batch->get_graphs(graphs, gst);
                        for (auto& g : graphs)
                            graph_output << g.serialize_to_dot() << std::endl;
                    }
                    batch->reset();
                    std::cerr << "Processed groups " << group_count + offset << " - "
                              << (st == StatusType::success ? i : i - 1) + offset << " (batch " << b << ")"
                              << std::endl;
                }
                else
                {
                    std::cerr << "Could not add POA group " << ids[i] << " to batch " << b << std::endl;
                    i++;
                }
                group_count = i;
            }
            if (st == StatusType::success)
            {
                for (const auto& s : seq_status)
                    if (s == StatusType::exceeded_maximum_sequence_size)
                        std::cerr << "Dropping sequence because sequence exceeded maximum size" << std::endl;
                i++;
            }
            if (st != StatusType::exceeded_maximum_poas && st != StatusType::success)
            {
                std::cerr << "Could not add POA group " << ids[i] << " to batch " << b << ". Error code " << int(st)
                          << std::endl;
                i++;
            }
        }
        offset += int32_t(ids.size());
    }
    return 0;
}

} // namespace

int main(int argc, char* argv[])
{
    try
    {
        return run(argc, argv);
    }
    catch (const std::exception& e)
    {
        std::cerr << "cudapoa: " << e.what() << std::endl;
        return 1;
    }
}
