// Overlap-alignment caller of the global aligner (reference
// cudamapper/src/main.cu:48-175) with PAF output (cudamapper_utils.cpp:30-112)
// and the FASTA reader it reads reads through (common/io/src/kseqpp_fasta_parser.cpp:31-72).
//
// Engines: num_alignment_engines host threads, each with its own HIP stream and
// aligner, pull [start, start + batch) ranges of the overlap list from a shared
// counter, add the overlap regions (target reverse-complemented for Reverse
// overlaps), align, and store the CIGARs at the overlaps' indices, so the
// output order is the overlap order whatever the thread interleaving.
#include <claraparabricks/genomeworks/cudaaligner/aligner.hpp>
#include <claraparabricks/genomeworks/cudamapper/overlap_alignment.hpp>
#include <claraparabricks/genomeworks/io/fasta_parser.hpp>

#include "../../include/gwamd_cudaaligner.h"
#include "../../include/gwamd_cudamapper.h"
#include "host_common.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <functional>
#include <iostream>
#include <mutex>
#include <random>
#include <stdexcept>
#include <thread>

namespace claraparabricks
{
namespace genomeworks
{
namespace io
{
namespace
{

class FastaParserMem : public FastaParser
{
public:
    explicit FastaParserMem(std::vector<FastaSequence> reads)
        : reads_(std::move(reads))
    {
    }
    number_of_reads_t get_num_seqences() const override { return number_of_reads_t(reads_.size()); }
    const FastaSequence& get_sequence_by_id(read_id_t sequence_id) const override
    {
        return reads_.at(sequence_id);
    }

private:
    std::vector<FastaSequence> reads_;
};

std::string first_word(const std::string& header)
{
    const size_t end = header.find_first_of(" \t\r");
    return header.substr(1, end == std::string::npos ? std::string::npos : end - 1);
}

// FASTA and FASTQ records as kseq reads them: '>' or '@' header, sequence
// lines up to the next header ('+' separator and quality lines for FASTQ)
std::vector<FastaSequence> read_records(const std::string& path)
{
    std::ifstream in(path);
    if (!in.good())
        throw std::invalid_argument("Error: non-existent or empty file " + path + " !");
    std::vector<FastaSequence> out;
    std::string line;
    bool fastq = false;
    while (std::getline(in, line))
    {
        if (!line.empty() && line.back() == '\r')
            line.pop_back();
        if (line.empty())
            continue;
        if (line[0] == '>' || line[0] == '@')
        {
            fastq = line[0] == '@';
            out.push_back(FastaSequence{first_word(line), std::string()});
            if (fastq)
            {
                // sequence lines up to '+', then as many quality characters
                while (std::getline(in, line) && !(line.size() && line[0] == '+'))
                {
                    if (!line.empty() && line.back() == '\r')
                        line.pop_back();
                    out.back().seq += line;
                }
                size_t qual = 0;
                while (qual < out.back().seq.size() && std::getline(in, line))
                    qual += line.size() - (line.size() && line.back() == '\r' ? 1 : 0);
            }
        }
        else if (!out.empty() && !fastq)
            out.back().seq += line;
    }
    if (out.empty())
        throw std::invalid_argument("Error: non-existent or empty file " + path + " !");
    return out;
}

} // namespace

std::unique_ptr<FastaParser> create_kseq_fasta_parser(const std::string& fasta_file,
                                                      number_of_basepairs_t min_sequence_length, bool shuffle)
{
    std::vector<FastaSequence> all = read_records(fasta_file);
    std::vector<FastaSequence> kept;
    kept.reserve(all.size());
    for (auto& r : all)
        if (number_of_basepairs_t(r.seq.size()) >= min_sequence_length)
            kept.push_back(std::move(r));
    if (shuffle) // kseqpp_fasta_parser.cpp:58-63: deterministic order
    {
        std::mt19937 g(0);
        std::shuffle(kept.begin(), kept.end(), g);
    }
    return std::make_unique<FastaParserMem>(std::move(kept));
}

std::unique_ptr<FastaParser> create_fasta_parser_from_sequences(std::vector<FastaSequence> records)
{
    return std::make_unique<FastaParserMem>(std::move(records));
}

} // namespace io

namespace cudamapper
{
namespace
{

// Bound on the host staging of one engine's batch (the aligner keeps pinned
// copies of every pair it holds): overlaps per batch are capped so an engine
// stages at most this many bytes.  The batch size has no effect on results.
constexpr int64_t kMaxStagingBytes = int64_t(1) << 30;

struct Region
{
    const char* query;
    int32_t query_length;
    const char* target;
    int32_t target_length;
    bool reverse;
};

using RegionFn = std::function<Region(int32_t)>;

void run_engines_on(int32_t n, int32_t max_query_size, int32_t max_target_size, int32_t num_alignment_engines,
                    const RegionFn& region, std::vector<std::string>& cigars);

// Overlaps longer than the aligner's limits (gwamd_aligner_max_lengths; the
// reference has none) are left without a CIGAR, with a warning on stderr, so
// one long overlap does not fail the whole call; the others are aligned by an
// aligner sized for them (main.cu:125-175 sizes it by the longest overlap).
void run_engines(int32_t n, int32_t num_alignment_engines, const RegionFn& region, std::vector<std::string>& cigars)
{
    if (num_alignment_engines < 1)
        throw std::runtime_error("num_alignment_engines must be at least 1");
    int32_t lim_q = 0, lim_t = 0;
    gwamd_aligner_max_lengths(GWAMD_ALIGNER_HIRSCHBERG_MYERS, &lim_q, &lim_t);
    int32_t max_q = 0, max_t = 0;
    std::vector<int32_t> kept;
    kept.reserve(size_t(n));
    for (int32_t i = 0; i < n; i++)
    {
        const Region r = region(i);
        if (r.query_length > lim_q || r.target_length > lim_t)
            continue;
        kept.push_back(i);
        max_q = std::max(max_q, r.query_length);
        max_t = std::max(max_t, r.target_length);
    }
    if (int32_t(kept.size()) != n)
        std::cerr << "align_overlaps: " << n - int32_t(kept.size())
                  << " overlap(s) longer than the aligner's limits (query " << lim_q << ", target " << lim_t
                  << " bases) left without a CIGAR" << std::endl;
    std::vector<std::string> kept_cigars;
    run_engines_on(int32_t(kept.size()), max_q, max_t, num_alignment_engines,
                   [&](int32_t k) { return region(kept[size_t(k)]); }, kept_cigars);
    cigars.assign(size_t(n), std::string());
    for (size_t k = 0; k < kept.size(); k++)
        cigars[size_t(kept[k])] = std::move(kept_cigars[k]);
}

void run_engines_on(int32_t n, int32_t max_query_size, int32_t max_target_size, int32_t num_alignment_engines,
                    const RegionFn& region, std::vector<std::string>& cigars)
{
    cigars.assign(size_t(n), std::string());
    if (n == 0)
        return;
    int device_id = 0;
    GWAMD_HIP_CHECK(hipGetDevice(&device_id));

    // main.cu:150-156: 0.03 B per cell of the largest overlap pair, 85% of free memory
    const float memory_per_base      = 0.03f;
    const float memory_per_alignment = std::max(1.0f, memory_per_base * float(max_query_size) * float(max_target_size));
    size_t free_mem = 0, total_mem = 0;
    GWAMD_HIP_CHECK(hipMemGetInfo(&free_mem, &total_mem));
    const size_t max_alignments = size_t((float(free_mem) * 85 / 100) / memory_per_alignment);
    int64_t batch_size = std::min<int64_t>(n, int64_t(std::min<size_t>(max_alignments, INT32_MAX))) /
                         num_alignment_engines;
    const int64_t per_pair = 2 * int64_t(std::max(max_query_size, max_target_size)) + max_query_size +
                             max_target_size + 16;
    batch_size = std::min<int64_t>(batch_size, std::max<int64_t>(1, kMaxStagingBytes / per_pair));
    // the reference loops forever on a zero batch size (fewer overlaps than engines)
    batch_size = std::max<int64_t>(batch_size, 1);
    std::cerr << "Aligning " << n << " overlaps (" << max_query_size << "x" << max_target_size
              << ") with batch size " << batch_size << std::endl;

    std::mutex idx_mtx;
    int32_t next = 0;
    std::vector<std::exception_ptr> errors(static_cast<size_t>(num_alignment_engines));
    auto engine = [&](int32_t e) {
        try
        {
            gwamd::host::ScopedDevice dev(device_id);
            hipStream_t stream = nullptr;
            GWAMD_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
            struct StreamGuard
            {
                hipStream_t s;
                ~StreamGuard() { (void)hipStreamDestroy(s); }
            } guard{stream};
            auto aligner = cudaaligner::create_aligner(max_query_size, max_target_size, int32_t(batch_size),
                                                       cudaaligner::AlignmentType::global_alignment,
                                                       DefaultDeviceAllocator(), stream, device_id);
            while (true)
            {
                int32_t start = 0, end = 0;
                {
                    std::lock_guard<std::mutex> lk(idx_mtx);
                    if (next == n)
                        break;
                    start = next;
                    end   = int32_t(std::min<int64_t>(int64_t(start) + batch_size, n));
                    next  = end;
                }
                for (int32_t i = start; i < end; i++)
                {
                    const Region r = region(i);
                    const cudaaligner::StatusType st =
                        aligner->add_alignment(r.query, r.query_length, r.target, r.target_length, false, r.reverse);
                    if (st != cudaaligner::StatusType::success)
                        throw std::runtime_error("Experienced error type " + std::to_string(int(st)));
                }
                aligner->align_all();
                aligner->sync_alignments();
                const auto& alignments = aligner->get_alignments();
                for (int32_t i = 0; i < int32_t(alignments.size()); i++)
                    cigars[size_t(start + i)] = alignments[size_t(i)]->convert_to_cigar();
                aligner->reset();
            }
        }
        catch (...)
        {
            errors[size_t(e)] = std::current_exception();
            std::lock_guard<std::mutex> lk(idx_mtx);
            next = n; // stop the other engines
        }
    };
    std::vector<std::thread> threads;
    for (int32_t e = 0; e < num_alignment_engines; e++)
        threads.emplace_back(engine, e);
    for (auto& t : threads)
        t.join();
    for (auto& ep : errors)
        if (ep)
            std::rethrow_exception(ep);
}

void check_range(uint32_t start, uint32_t end, size_t length, const char* what)
{
    if (start > end || end > length)
        throw std::invalid_argument(std::string("overlap ") + what + " range outside its read");
}

template <typename NameFn, typename LenFn>
std::string format_paf_impl(const std::vector<Overlap>& overlaps, const std::vector<std::string>& cigars,
                            NameFn qname, LenFn qlen, NameFn tname, LenFn tlen, int32_t kmer_size)
{
    if (!cigars.empty() && cigars.size() != overlaps.size())
        throw std::invalid_argument("print_paf: one CIGAR per overlap expected");
    std::string out;
    out.reserve(overlaps.size() * 150);
    char buf[256];
    for (size_t i = 0; i < overlaps.size(); i++)
    {
        const Overlap& o = overlaps[i];
        // cudamapper_utils.cpp:74-89: name, length, start, end, strand, name,
        // length, start, end, residues x k, longer span, mapping quality 255
        const int64_t span = std::max(std::abs(int64_t(o.target_start_position_in_read_) -
                                               int64_t(o.target_end_position_in_read_)),
                                      std::abs(int64_t(o.query_start_position_in_read_) -
                                               int64_t(o.query_end_position_in_read_)));
        out += qname(o.query_read_id_);
        std::snprintf(buf, sizeof(buf), "\t%lu\t%i\t%i\t%c\t", (unsigned long)qlen(o.query_read_id_),
                      int(o.query_start_position_in_read_), int(o.query_end_position_in_read_),
                      static_cast<unsigned char>(o.relative_strand));
        out += buf;
        out += tname(o.target_read_id_);
        std::snprintf(buf, sizeof(buf), "\t%lu\t%i\t%i\t%i\t%" PRId64 "\t%i", (unsigned long)tlen(o.target_read_id_),
                      int(o.target_start_position_in_read_), int(o.target_end_position_in_read_),
                      int(o.num_residues_ * uint32_t(kmer_size)), span, 255);
        out += buf;
        if (!cigars.empty() && !cigars[i].empty()) // no CIGAR: overlap not aligned
        {
            out += "\tcg:Z:";
            out += cigars[i];
        }
        out += '\n';
    }
    return out;
}

} // namespace

void align_overlaps(DefaultDeviceAllocator /*allocator*/, std::vector<Overlap>& overlaps,
                    const io::FastaParser& query_parser, const io::FastaParser& target_parser,
                    int32_t num_alignment_engines, std::vector<std::string>& cigars)
{
    if (overlaps.size() > size_t(INT32_MAX))
        throw std::invalid_argument("too many overlaps for one call");
    for (const Overlap& o : overlaps)
    {
        check_range(o.query_start_position_in_read_, o.query_end_position_in_read_,
                    query_parser.get_sequence_by_id(o.query_read_id_).seq.size(), "query");
        check_range(o.target_start_position_in_read_, o.target_end_position_in_read_,
                    target_parser.get_sequence_by_id(o.target_read_id_).seq.size(), "target");
    }
    run_engines(int32_t(overlaps.size()), num_alignment_engines,
                [&](int32_t i) {
                    const Overlap& o = overlaps[size_t(i)];
                    const std::string& q = query_parser.get_sequence_by_id(o.query_read_id_).seq;
                    const std::string& t = target_parser.get_sequence_by_id(o.target_read_id_).seq;
                    return Region{q.data() + o.query_start_position_in_read_,
                                  int32_t(o.query_end_position_in_read_ - o.query_start_position_in_read_),
                                  t.data() + o.target_start_position_in_read_,
                                  int32_t(o.target_end_position_in_read_ - o.target_start_position_in_read_),
                                  o.relative_strand == RelativeStrand::Reverse};
                },
                cigars);
}

std::string format_paf(const std::vector<Overlap>& overlaps, const std::vector<std::string>& cigars,
                       const io::FastaParser& query_parser, const io::FastaParser& target_parser,
                       int32_t kmer_size)
{
    using NameFn = std::function<const std::string&(read_id_t)>;
    using LenFn  = std::function<size_t(read_id_t)>;
    return format_paf_impl<NameFn, LenFn>(
        overlaps, cigars,
        [&](read_id_t id) -> const std::string& { return query_parser.get_sequence_by_id(id).name; },
        [&](read_id_t id) { return query_parser.get_sequence_by_id(id).seq.size(); },
        [&](read_id_t id) -> const std::string& { return target_parser.get_sequence_by_id(id).name; },
        [&](read_id_t id) { return target_parser.get_sequence_by_id(id).seq.size(); }, kmer_size);
}

void print_paf(const std::vector<Overlap>& overlaps, const std::vector<std::string>& cigars,
               const io::FastaParser& query_parser, const io::FastaParser& target_parser, int32_t kmer_size,
               std::mutex& write_output_mutex)
{
    const std::string text = format_paf(overlaps, cigars, query_parser, target_parser, kmer_size);
    std::lock_guard<std::mutex> lg(write_output_mutex);
    std::fwrite(text.data(), 1, text.size(), stdout);
}

} // namespace cudamapper
} // namespace genomeworks
} // namespace claraparabricks

// ---- C ABI ------------------------------------------------------------------

namespace cm = claraparabricks::genomeworks::cudamapper;

struct gwamd_text_list
{
    std::vector<std::string> items;
};

static_assert(sizeof(gwamd_overlap) == sizeof(cm::Overlap), "gwamd_overlap must match cudamapper::Overlap");
static_assert(offsetof(gwamd_overlap, relative_strand) == offsetof(cm::Overlap, relative_strand), "layout");
static_assert(offsetof(gwamd_overlap, num_residues) == offsetof(cm::Overlap, num_residues_), "layout");
static_assert(offsetof(gwamd_overlap, overlap_complete) == offsetof(cm::Overlap, overlap_complete), "layout");

namespace
{

template <typename F>
int32_t guarded_cm(F&& f)
{
    try
    {
        gwamd::host::last_error().clear();
        return f();
    }
    catch (const std::invalid_argument& e)
    {
        gwamd::host::last_error() = e.what();
        return GWAMD_E_INVALID_ARGUMENT;
    }
    catch (const std::exception& e)
    {
        gwamd::host::last_error() = e.what();
        return std::string(e.what()).rfind("HIP error", 0) == 0 ? GWAMD_E_HIP : GWAMD_E_RUNTIME;
    }
}

std::vector<cm::Overlap> to_overlaps(const gwamd_overlap* o, int32_t n)
{
    std::vector<cm::Overlap> v(static_cast<size_t>(std::max(n, 0)));
    if (n > 0)
        std::memcpy(v.data(), o, sizeof(cm::Overlap) * size_t(n));
    for (const auto& x : v)
        if (x.relative_strand != cm::RelativeStrand::Forward && x.relative_strand != cm::RelativeStrand::Reverse)
            throw std::invalid_argument("relative_strand must be '+' or '-'");
    return v;
}

void check_offsets(const int64_t* off, int32_t n, const char* what)
{
    if (n < 0 || (n > 0 && !off))
        throw std::invalid_argument(std::string(what) + ": bad read count or offsets");
    for (int32_t i = 0; i < n; i++)
        if (off[i] > off[i + 1] || off[i] < 0)
            throw std::invalid_argument(std::string(what) + ": offsets must be non-decreasing");
}

} // namespace

extern "C" {

int32_t gwamd_align_overlaps(const char* query_bases, const int64_t* query_offsets, int32_t num_queries,
                             const char* target_bases, const int64_t* target_offsets, int32_t num_targets,
                             const gwamd_overlap* overlaps, int32_t num_overlaps, int32_t num_alignment_engines,
                             int32_t device_id, gwamd_text_list** cigars)
{
    *cigars = nullptr;
    return guarded_cm([&] {
        check_offsets(query_offsets, num_queries, "queries");
        check_offsets(target_offsets, num_targets, "targets");
        std::vector<cm::Overlap> ov = to_overlaps(overlaps, num_overlaps);
        for (const auto& o : ov)
        {
            if (o.query_read_id_ >= uint32_t(num_queries) || o.target_read_id_ >= uint32_t(num_targets))
                throw std::invalid_argument("overlap read id out of range");
            const int64_t ql = query_offsets[o.query_read_id_ + 1] - query_offsets[o.query_read_id_];
            const int64_t tl = target_offsets[o.target_read_id_ + 1] - target_offsets[o.target_read_id_];
            if (o.query_start_position_in_read_ > o.query_end_position_in_read_ || o.query_end_position_in_read_ > ql)
                throw std::invalid_argument("overlap query range outside its read");
            if (o.target_start_position_in_read_ > o.target_end_position_in_read_ ||
                o.target_end_position_in_read_ > tl)
                throw std::invalid_argument("overlap target range outside its read");
        }
        auto list = std::make_unique<gwamd_text_list>();
        if (num_overlaps == 0)
        {
            *cigars = list.release();
            return 0;
        }
        gwamd::host::ScopedDevice dev(device_id);
        cm::run_engines(num_overlaps, num_alignment_engines,
                        [&](int32_t i) {
                            const cm::Overlap& o = ov[size_t(i)];
                            return cm::Region{query_bases + query_offsets[o.query_read_id_] +
                                                  o.query_start_position_in_read_,
                                              int32_t(o.query_end_position_in_read_ - o.query_start_position_in_read_),
                                              target_bases + target_offsets[o.target_read_id_] +
                                                  o.target_start_position_in_read_,
                                              int32_t(o.target_end_position_in_read_ -
                                                      o.target_start_position_in_read_),
                                              o.relative_strand == cm::RelativeStrand::Reverse};
                        },
                        list->items);
        *cigars = list.release();
        return 0;
    });
}

int32_t gwamd_format_paf(const char* query_names, const int64_t* query_name_offsets, const int64_t* query_lengths,
                         int32_t num_queries, const char* target_names, const int64_t* target_name_offsets,
                         const int64_t* target_lengths, int32_t num_targets, const gwamd_overlap* overlaps,
                         int32_t num_overlaps, const gwamd_text_list* cigars, int32_t kmer_size,
                         gwamd_text_list** paf)
{
    *paf = nullptr;
    return guarded_cm([&] {
        check_offsets(query_name_offsets, num_queries, "query names");
        check_offsets(target_name_offsets, num_targets, "target names");
        std::vector<cm::Overlap> ov = to_overlaps(overlaps, num_overlaps);
        for (const auto& o : ov)
            if (o.query_read_id_ >= uint32_t(num_queries) || o.target_read_id_ >= uint32_t(num_targets))
                throw std::invalid_argument("overlap read id out of range");
        auto names = [](const char* base, const int64_t* off, int32_t n) {
            std::vector<std::string> v(static_cast<size_t>(n));
            for (int32_t i = 0; i < n; i++)
                v[size_t(i)].assign(base + off[i], size_t(off[i + 1] - off[i]));
            return v;
        };
        const auto qn = names(query_names, query_name_offsets, num_queries);
        const auto tn = names(target_names, target_name_offsets, num_targets);
        static const std::vector<std::string> none;
        const std::vector<std::string>& cg = cigars ? cigars->items : none;
        using NameFn = std::function<const std::string&(claraparabricks::genomeworks::read_id_t)>;
        using LenFn  = std::function<size_t(claraparabricks::genomeworks::read_id_t)>;
        auto list    = std::make_unique<gwamd_text_list>();
        list->items.push_back(cm::format_paf_impl<NameFn, LenFn>(
            ov, cg, [&](claraparabricks::genomeworks::read_id_t i) -> const std::string& { return qn[i]; },
            [&](claraparabricks::genomeworks::read_id_t i) { return size_t(query_lengths[i]); },
            [&](claraparabricks::genomeworks::read_id_t i) -> const std::string& { return tn[i]; },
            [&](claraparabricks::genomeworks::read_id_t i) { return size_t(target_lengths[i]); }, kmer_size));
        *paf = list.release();
        return 0;
    });
}

int32_t gwamd_read_fasta(const char* path, uint32_t min_sequence_length, int32_t shuffle, gwamd_text_list** names,
                         gwamd_text_list** sequences)
{
    *names     = nullptr;
    *sequences = nullptr;
    return guarded_cm([&] {
        namespace io = claraparabricks::genomeworks::io;
        auto parser  = io::create_kseq_fasta_parser(path ? path : "", min_sequence_length, shuffle != 0);
        auto nl      = std::make_unique<gwamd_text_list>();
        auto sl      = std::make_unique<gwamd_text_list>();
        for (uint32_t i = 0; i < parser->get_num_seqences(); i++)
        {
            const auto& r = parser->get_sequence_by_id(i);
            nl->items.push_back(r.name);
            sl->items.push_back(r.seq);
        }
        *names     = nl.release();
        *sequences = sl.release();
        return 0;
    });
}

int32_t gwamd_text_list_create(const char* const* texts, const int64_t* lengths, int32_t n, gwamd_text_list** out)
{
    *out = nullptr;
    return guarded_cm([&] {
        if (n < 0 || (n > 0 && (!texts || !lengths)))
            throw std::invalid_argument("text list: bad count or pointers");
        auto list = std::make_unique<gwamd_text_list>();
        list->items.resize(static_cast<size_t>(n));
        for (int32_t i = 0; i < n; i++)
        {
            if (lengths[i] < 0)
                throw std::invalid_argument("text list: negative length");
            list->items[size_t(i)].assign(texts[i], size_t(lengths[i]));
        }
        *out = list.release();
        return 0;
    });
}

int32_t gwamd_text_list_size(const gwamd_text_list* list) { return list ? int32_t(list->items.size()) : 0; }

int32_t gwamd_text_list_get(const gwamd_text_list* list, int32_t i, const char** text, int64_t* length)
{
    if (!list || i < 0 || i >= int32_t(list->items.size()))
        return GWAMD_E_INVALID_ARGUMENT;
    *text   = list->items[size_t(i)].data();
    *length = int64_t(list->items[size_t(i)].size());
    return 0;
}

void gwamd_text_list_free(gwamd_text_list* list) { delete list; }

} // extern "C"
