// Host side of the MI355X global aligner: the reference's C++ API
// (create_aligner / Aligner / Alignment, cudaaligner/src/aligner.cpp,
// aligner_global.cpp, alignment_impl.cpp) and the C ABI of
// include/gwamd_cudaaligner.h.  Device work is in aligner_kernels.hip.
#include <claraparabricks/genomeworks/cudaaligner/aligner.hpp>
#include <claraparabricks/genomeworks/cudaaligner/alignment.hpp>
#include <claraparabricks/genomeworks/cudaaligner/cudaaligner.hpp>

#include "aligner_common.hpp"
#include "gwamd_cudaaligner.h"
#include "host_common.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace gwamd
{
namespace host
{
// long mode: target letter codes in LDS up to kHmLdsTarget bases, in HBM beyond
constexpr int32_t kHmMaxQuery  = 1 << 24;
constexpr int32_t kHmMaxTarget = 1 << 24;
constexpr int32_t kHmLdsTarget = 131072;
// full Myers: one pair's (word, column) state (0.375 B per cell) per slot
constexpr int64_t kMyersMaxSlot   = int64_t(32) << 30;
constexpr int64_t kMyersWorkspace = int64_t(64) << 30; // resident slots within 64 GiB of the 288 GB HBM
// Hirschberg-Myers takes the LDS-resident kernel (hm_kernel<false>, patterns in
// LDS, register-resident sweeps of up to 4 blocks per half) up to these sizes
constexpr int32_t kHmShortQuery  = 16384;
constexpr int32_t kHmShortTarget = 65535;
// Workspace slot of the full Myers aligner (always long mode): the padded
// (word, column) matrix of pv / mv / score (128-B rows), the stripes'
// per-column deltas, the query patterns and, past kHmLdsTarget, the target
// letter codes; slots start on 256-B lines.
inline int64_t myers_slot_layout(int32_t max_q, int32_t max_t, int64_t* hbuf_off, int64_t* pat_off,
                                 int64_t* tcod_off)
{
    auto a16             = [](int64_t v) { return (v + 15) & ~int64_t(15); };
    const int64_t pw     = (int64_t(max_q) + gwamd::aln::kWordBits - 1) / gwamd::aln::kWordBits;
    const int64_t nwp    = (pw + 31) & ~int64_t(31);
    const bool tcod_hbm  = max_t > kHmLdsTarget;
    const int64_t hb     = a16(nwp * (int64_t(max_t) + 1) * 12 + 64);
    const int64_t po     = a16(hb + int64_t(max_t) + 1 + gwamd::aln::kWave + 64);
    const int64_t to     = a16(po + pw * 32 + 64);
    const int64_t slot   = a16(to + (tcod_hbm ? (int64_t(max_t) + 15) / 16 * 4 + 64 : 0));
    if (hbuf_off)
        *hbuf_off = hb, *pat_off = po, *tcod_off = to;
    return (slot + 255) & ~int64_t(255);
}

// Length limits of this implementation (include/gwamd_cudaaligner.h).
inline void aligner_max_lengths(int32_t algo, int32_t& max_query, int32_t& max_target)
{
    max_target = 65535; // 16-bit segment coordinates, LDS target codes
    switch (algo)
    {
    case GWAMD_ALIGNER_HIRSCHBERG_MYERS:
        // long mode (hm_kernel<true>): query patterns in HBM, striped sweeps;
        // the target's 2-bit letter codes stay in LDS
        max_query  = kHmMaxQuery;
        max_target = kHmMaxTarget;
        break;
    case GWAMD_ALIGNER_MYERS:
        // stripes of 8,192 rows; the (word, column) state of the largest pair
        // must fit one workspace slot (kMyersMaxSlot)
        max_query  = kHmMaxQuery;
        max_target = kHmMaxTarget;
        break;
    case GWAMD_ALIGNER_MYERS_BANDED:
        // patterns (Q / 2 bytes) and target codes (T / 4 bytes) in LDS
        max_query  = 65536;
        max_target = 65536;
        break;
    default:
        // Ukkonen: both sequences in LDS (ukkonen_wide_kernel: up to 2 x 64 KiB
        // of its 160 KiB), (1 + int(0.1f * T) + 2p + 1) / 2 = 3,377 band rows
        // at 65,536, within kUkWideChunks x 1,024; the reference benchmark's
        // largest size (cudaaligner/benchmarks/main.cpp:140-143)
        max_query  = 65536;
        max_target = 65536;
    }
}
} // namespace host
} // namespace gwamd

extern "C" hipError_t gwamd_internal_align_launch(const gwamd::aln::Args* a, int algo, int grid, hipStream_t stream);
extern "C" hipError_t gwamd_internal_align_occupancy(int algo, int lds_bytes, int* blocks_per_cu);
extern "C" hipError_t gwamd_internal_banded_launch(const gwamd::aln::Args* a, int algo, int grid, hipStream_t stream);
extern "C" hipError_t gwamd_internal_banded_occupancy(int algo, int lds_bytes, int band_waves, int* blocks_per_cu);
extern "C" hipError_t gwamd_internal_ukkonen_wide_occupancy(int threads, int lds_bytes, int* blocks_per_cu);

namespace claraparabricks
{
namespace genomeworks
{
namespace cudaaligner
{

using gwamd::host::PinnedBuf;
using gwamd::host::ScopedDevice;

StatusType Init() { return StatusType::success; }

std::ostream& operator<<(std::ostream& os, const FormattedAlignment& f)
{
    // alignment.cpp:24-35
    const std::size_t line = (f.linebreak_after == 0) ? f.query.size() : f.linebreak_after;
    for (std::size_t i = 0; i < f.query.size(); i += line)
        os << f.query.substr(i, line) << '\n' << f.pairing.substr(i, line) << '\n' << f.target.substr(i, line) << '\n';
    os << std::endl;
    return os;
}

namespace
{

int32_t throw_on_negative(int32_t v, const char* msg)
{
    if (v < 0)
        throw std::invalid_argument(msg);
    return v;
}

// genomeutils::reverse_complement (genomeutils.hpp:137-150)
void reverse_complement(const char* src, int32_t n, char* dst)
{
    for (int32_t p = 0; p < n; p++)
    {
        const char c = src[n - 1 - p];
        dst[p]       = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
    }
}

char cigar_state(AlignmentState s)
{
    switch (s)
    {
    case AlignmentState::match:
    case AlignmentState::mismatch: return 'M';
    case AlignmentState::insertion: return 'I';
    case AlignmentState::deletion: return 'D';
    default: throw std::runtime_error("Unrecognized alignment state.");
    }
}

} // namespace

// AlignmentImpl (alignment_impl.cpp:24-112)
class AlignmentImpl : public Alignment
{
public:
    AlignmentImpl(const char* query, int32_t query_length, const char* target, int32_t target_length)
        : query_(query, query + throw_on_negative(query_length, "query_length has to be non-negative."))
        , target_(target, target + throw_on_negative(target_length, "target_length has to be non-negative."))
    {
    }
    const std::string& get_query_sequence() const override { return query_; }
    const std::string& get_target_sequence() const override { return target_; }
    AlignmentType get_alignment_type() const override { return type_; }
    StatusType get_status() const override { return status_; }
    const std::vector<AlignmentState>& get_alignment() const override { return alignment_; }
    void set_alignment_type(AlignmentType t) { type_ = t; }
    void set_status(StatusType s) { status_ = s; }
    void set_alignment(std::vector<AlignmentState>&& a) { alignment_ = std::move(a); }
    // the result storage, refilled in place by sync_alignments (an aligner
    // that aligns its batch again reuses the vectors' capacity)
    std::vector<AlignmentState>& alignment_storage() { return alignment_; }

    std::string convert_to_cigar() const override
    {
        if (alignment_.empty())
            return std::string();
        std::string cigar;
        char last   = cigar_state(alignment_[0]);
        int32_t cnt = 0;
        for (AlignmentState x : alignment_)
        {
            const char c = cigar_state(x);
            if (c == last)
                cnt++;
            else
            {
                cigar += std::to_string(cnt) + last;
                cnt  = 1;
                last = c;
            }
        }
        cigar += std::to_string(cnt) + last;
        return cigar;
    }

    FormattedAlignment format_alignment(int32_t maximal_line_length) const override
    {
        int64_t t = 0, q = 0;
        FormattedAlignment r;
        r.linebreak_after = (maximal_line_length < 0) ? 0 : maximal_line_length;
        for (AlignmentState x : alignment_)
        {
            switch (x)
            {
            case AlignmentState::match:
                r.target += target_[t++];
                r.query += query_[q++];
                r.pairing += '|';
                break;
            case AlignmentState::mismatch:
                r.target += target_[t++];
                r.query += query_[q++];
                r.pairing += 'x';
                break;
            case AlignmentState::deletion:
                r.target += '-';
                r.query += query_[q++];
                r.pairing += ' ';
                break;
            case AlignmentState::insertion:
                r.target += target_[t++];
                r.query += '-';
                r.pairing += ' ';
                break;
            default: throw std::runtime_error("Unknown alignment state");
            }
        }
        return r;
    }

private:
    std::string query_, target_;
    StatusType status_ = StatusType::uninitialized;
    AlignmentType type_ = AlignmentType::unset;
    std::vector<AlignmentState> alignment_;
};

// AlignerGlobal (aligner_global.cpp) with the HIP kernels of aligner_kernels.hip.
class AlignerGlobalHip : public Aligner
{
public:
    // budget: the pool of the caller's DefaultDeviceAllocator (null or a
    // negative capacity: all available memory, allocator.hpp:282-305), shared
    // by every aligner made from copies of that allocator.  The reference
    // serves every device buffer of the aligner from that pool; here the
    // fixed buffers (sequences, paths, lengths) come first and the workspace
    // gets as many persistent-grid slots as what is left of the pool holds;
    // less than the fixed buffers plus one slot throws, as the reference's
    // pool does when an allocation does not fit.  The bytes stay reserved
    // until the aligner is destroyed.
    AlignerGlobalHip(int32_t max_query_length, int32_t max_target_length, int32_t max_alignments, int algorithm,
                     hipStream_t stream, int32_t device_id, std::shared_ptr<DeviceBudget> budget = nullptr)
        : max_q_(throw_on_negative(max_query_length, "max_query_length must be non-negative."))
        , max_t_(throw_on_negative(max_target_length, "max_target_length must be non-negative."))
        , max_n_(throw_on_negative(max_alignments, "max_alignments must be non-negative."))
        , algo_(algorithm)
        , stream_(stream)
        , device_id_(device_id)
    {
        if (max_alignments < 1)
            throw std::runtime_error("Max alignments must be at least 1.");
        // limits of this implementation (aligner_max_lengths; the reference has
        // none): the Myers state of a query segment is register-resident
        // (4 blocks of 64x32 bits), segment coordinates and split scores are
        // 16-bit, the Ukkonen band has at most 4,096 diagonals
        int32_t lim_q = 0, lim_t = 0;
        gwamd::host::aligner_max_lengths(algo_, lim_q, lim_t);
        if (max_q_ > lim_q)
            throw std::invalid_argument("max_query_length above " + std::to_string(lim_q) +
                                        " is not supported by this aligner.");
        if (algo_ == GWAMD_ALIGNER_UKKONEN && ukkonen_band_rows() > gwamd::aln::kUkWideChunks * 1024)
            throw std::invalid_argument("max_target_length too large for the Ukkonen aligner's band.");
        if (max_t_ > lim_t)
            throw std::invalid_argument("max_target_length above " + std::to_string(lim_t) +
                                        " is not supported by this aligner.");
        stride_     = std::max(max_q_, max_t_);
        max_result_ = (max_q_ + max_t_ + 3) / 4 * 4; // calc_max_result_length (aligner_global.cpp:26-31)
        ScopedDevice dev(device_id_);
        plan();
        if (budget && budget->capacity() >= 0)
        {
            const int64_t fixed = int64_t(2) * stride_ * max_n_ + 16 + int64_t(2) * max_n_ * 4 +
                                  int64_t(max_result_) * max_n_ + 16 + int64_t(max_n_) * 4 + 32 +
                                  (algo_ == GWAMD_ALIGNER_MYERS_BANDED ? int64_t(max_n_) * kMaxSpecSweeps * 4 : 0);
            const int64_t sb    = std::max<int64_t>(1, slot_bytes_);
            const int64_t got   = budget->reserve(fixed + sb, fixed + int64_t(slots_) * sb);
            if (got < 0)
                throw std::runtime_error("The aligner needs " + std::to_string(fixed + sb) +
                                         " device bytes, more than its allocator has left (" +
                                         std::to_string(budget->capacity() - budget->used()) + " of " +
                                         std::to_string(budget->capacity()) + ").");
            slots_    = int32_t(std::min<int64_t>(slots_, (got - fixed) / sb));
            // keep exactly what this aligner uses
            const int64_t used = fixed + int64_t(slots_) * sb;
            budget->release(got - used);
            budget_   = std::move(budget);
            reserved_ = used;
        }
        auto dalloc = [&](void** p, size_t bytes, bool zero = true) {
            GWAMD_HIP_CHECK(hipMalloc(p, std::max<size_t>(bytes, 16)));
            if (zero)
                GWAMD_HIP_CHECK(hipMemsetAsync(*p, 0, std::max<size_t>(bytes, 16), stream_));
            device_bytes_ += int64_t(bytes);
        };
        dalloc(reinterpret_cast<void**>(&d_seqs_), size_t(2) * stride_ * max_n_ + 16);
        dalloc(reinterpret_cast<void**>(&d_lens_), size_t(2) * max_n_ * 4);
        dalloc(reinterpret_cast<void**>(&d_paths_), size_t(max_result_) * max_n_ + 16);
        dalloc(reinterpret_cast<void**>(&d_plen_), size_t(max_n_) * 4);
        dalloc(reinterpret_cast<void**>(&d_stats_), 32);
        if (algo_ == GWAMD_ALIGNER_MYERS_BANDED)
            dalloc(reinterpret_cast<void**>(&d_spec_ed_), size_t(max_n_) * kMaxSpecSweeps * 4, false);
        // workspace: every slot entry is written before it is read
        dalloc(reinterpret_cast<void**>(&d_ws_), size_t(slots_) * size_t(slot_bytes_), false);
        h_seqs_.reserve(size_t(2) * stride_ * max_n_ + 16, stream_);
        h_lens_.reserve(size_t(2) * max_n_ * 4, stream_);
        h_paths_.reserve(size_t(max_result_) * max_n_ + 16, stream_);
        h_plen_.reserve(size_t(max_n_) * 4, stream_);
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
        // second stream and the events of the pipelined align_all()
        for (hipStream_t* st : {&stream2_, &s_in_, &s_out_})
            GWAMD_HIP_CHECK(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
        for (hipEvent_t* e : {&ev_fork_, &ev_join_})
            GWAMD_HIP_CHECK(hipEventCreate(e));
        for (int k = 0; k < kMaxStages; k++)
            for (hipEvent_t* e : {&ev_d_[k], &ev_h_[k], &ev_k_[2 * k], &ev_k_[2 * k + 1]})
                GWAMD_HIP_CHECK(hipEventCreateWithFlags(e, e == &ev_k_[2 * k] || e == &ev_k_[2 * k + 1]
                                                               ? hipEventDefault
                                                               : hipEventDisableTiming));
    }

    ~AlignerGlobalHip() override
    {
        if (budget_)
            budget_->release(reserved_);
        (void)hipSetDevice(device_id_);
        for (hipStream_t st : {stream2_, s_in_, s_out_})
            if (st)
            {
                (void)hipStreamSynchronize(st);
                (void)hipStreamDestroy(st);
            }
        for (hipEvent_t e : {ev_fork_, ev_join_})
            if (e)
                (void)hipEventDestroy(e);
        for (int k = 0; k < kMaxStages; k++)
            for (hipEvent_t e : {ev_d_[k], ev_h_[k], ev_k_[2 * k], ev_k_[2 * k + 1]})
                if (e)
                    (void)hipEventDestroy(e);
        for (void* p : {static_cast<void*>(d_seqs_), static_cast<void*>(d_lens_), static_cast<void*>(d_paths_),
                        static_cast<void*>(d_plen_), static_cast<void*>(d_ws_), static_cast<void*>(d_stats_),
                        static_cast<void*>(d_spec_ed_)})
            if (p)
                (void)hipFree(p);
    }

    StatusType add_alignment(const char* query, int32_t query_length, const char* target, int32_t target_length,
                             bool rc_query, bool rc_target) override
    {
        // AlignerGlobalUkkonen::add_alignment (aligner_global_ukkonen.cpp:47-57)
        if (algo_ == GWAMD_ALIGNER_UKKONEN && std::abs(query_length - target_length) > ukkonen_max_difference())
            return StatusType::exceeded_max_alignment_difference;
        // aligner_global.cpp:60-118
        if (query_length < 0 || target_length < 0)
            return StatusType::generic_error;
        const int32_t n = int32_t(alignments_.size());
        if (n >= max_n_)
            return StatusType::exceeded_max_alignments;
        if (query_length > max_q_)
            return StatusType::exceeded_max_length;
        if (target_length > max_t_)
            return StatusType::exceeded_max_length;
        char* qd = h_seqs_.as<char>() + size_t(2 * n) * stride_;
        char* td = h_seqs_.as<char>() + size_t(2 * n + 1) * stride_;
        if (rc_query)
            reverse_complement(query, query_length, qd);
        else if (query_length > 0)
            std::memcpy(qd, query, size_t(query_length));
        if (rc_target)
            reverse_complement(target, target_length, td);
        else if (target_length > 0)
            std::memcpy(td, target, size_t(target_length));
        h_lens_.as<int32_t>()[2 * n]     = query_length;
        h_lens_.as<int32_t>()[2 * n + 1] = target_length;
        max_diff_ = std::max(max_diff_, std::abs(query_length - target_length));
        auto a = std::make_shared<AlignmentImpl>(qd, query_length, td, target_length);
        a->set_alignment_type(AlignmentType::global_alignment);
        alignments_.push_back(a);
        return StatusType::success;
    }

    // aligner_global.cpp:131-159 (H2D, kernel, D2H on the aligner's stream).
    // Batches of many grids' worth of pairs run as a pipeline of stages: the
    // pairs are cut into K consecutive chunks; all uploads go back to back on
    // a copy-in stream, chunk k's kernel runs on half of the workspace slots
    // (k % 2, one compute stream per half) once its upload is in, and its
    // download follows on a copy-out stream, so copies overlap the kernels
    // and sync_alignments fills each chunk's results on the host while later
    // chunks are still aligning.  Results are the same pair by pair; the
    // aligner's stream waits for every stage.
    StatusType align_all() override
    {
        if (alignments_.empty())
            return StatusType::success;
        ScopedDevice dev(device_id_);
        const int32_t n = int32_t(alignments_.size());
        stages_         = pipeline_stages(n);
        if (stages_ <= 1)
        {
            stages_ = 1;
            chunk0_[0] = 0, chunk0_[1] = n;
            upload();
            launch(); // records ev_k_[0] / ev_k_[1] around the kernel
            download();
            GWAMD_HIP_CHECK(hipEventRecord(ev_d_[0], stream_));
            return StatusType::success;
        }
        GWAMD_HIP_CHECK(hipEventRecord(ev_fork_, stream_));
        for (hipStream_t st : {s_in_, stream2_, s_out_})
            GWAMD_HIP_CHECK(hipStreamWaitEvent(st, ev_fork_, 0));
        const int32_t half_slots = slots_ / 2;
        for (int k = 0; k < stages_; k++)
        {
            const int32_t i0 = int32_t(int64_t(n) * k / stages_);
            const int32_t c  = int32_t(int64_t(n) * (k + 1) / stages_) - i0;
            chunk0_[k]       = i0;
            chunk0_[k + 1]   = i0 + c;
            GWAMD_HIP_CHECK(hipMemcpyAsync(d_lens_ + 2 * size_t(i0), h_lens_.as<int32_t>() + 2 * size_t(i0),
                                           2 * size_t(c) * 4, hipMemcpyHostToDevice, s_in_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(d_seqs_ + 2 * size_t(i0) * stride_,
                                           h_seqs_.as<char>() + 2 * size_t(i0) * stride_, 2 * size_t(c) * stride_,
                                           hipMemcpyHostToDevice, s_in_));
            GWAMD_HIP_CHECK(hipEventRecord(ev_h_[k], s_in_));
        }
        for (int k = 0; k < stages_; k++)
        {
            hipStream_t st   = (k & 1) ? stream2_ : stream_;
            const int32_t i0 = chunk0_[k], c = chunk0_[k + 1] - chunk0_[k];
            GWAMD_HIP_CHECK(hipStreamWaitEvent(st, ev_h_[k], 0));
            GWAMD_HIP_CHECK(hipEventRecord(ev_k_[2 * k], st));
            launch_range(i0, c, (k & 1) * half_slots, (k & 1) ? slots_ - half_slots : half_slots, st);
            GWAMD_HIP_CHECK(hipEventRecord(ev_k_[2 * k + 1], st));
            GWAMD_HIP_CHECK(hipStreamWaitEvent(s_out_, ev_k_[2 * k + 1], 0));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_paths_.as<int8_t>() + size_t(i0) * max_result_,
                                           d_paths_ + size_t(i0) * max_result_, size_t(c) * max_result_,
                                           hipMemcpyDeviceToHost, s_out_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_plen_.as<int32_t>() + i0, d_plen_ + i0, size_t(c) * 4,
                                           hipMemcpyDeviceToHost, s_out_));
            GWAMD_HIP_CHECK(hipEventRecord(ev_d_[k], s_out_));
        }
        GWAMD_HIP_CHECK(hipEventRecord(ev_join_, s_out_)); // after every kernel and download
        GWAMD_HIP_CHECK(hipStreamWaitEvent(stream_, ev_join_, 0));
        return StatusType::success;
    }

    // Kernel time of the last align_all(): the union of its launches'
    // intervals (HIP events on their streams), ms.
    double last_kernel_ms()
    {
        ScopedDevice dev(device_id_);
        if (stages_ == 0)
            return 0.0;
        std::vector<std::pair<double, double>> iv;
        for (int k = 0; k < stages_; k++)
        {
            GWAMD_HIP_CHECK(hipEventSynchronize(ev_k_[2 * k + 1]));
            float a = 0.f, b = 0.f;
            GWAMD_HIP_CHECK(hipEventElapsedTime(&a, ev_k_[0], ev_k_[2 * k]));
            GWAMD_HIP_CHECK(hipEventElapsedTime(&b, ev_k_[0], ev_k_[2 * k + 1]));
            iv.emplace_back(double(a), double(b));
        }
        std::sort(iv.begin(), iv.end());
        double total = 0.0, lo = iv[0].first, hi = iv[0].second;
        for (size_t k = 1; k < iv.size(); k++)
        {
            if (iv[k].first > hi)
            {
                total += hi - lo;
                lo = iv[k].first;
            }
            hi = std::max(hi, iv[k].second);
        }
        return total + (hi - lo);
    }

    StatusType sync_alignments() override
    {
        // aligner_global.cpp:161-189: paths come out end -> start
        ScopedDevice dev(device_id_);
        const int32_t n = int32_t(alignments_.size());
        auto fill       = [&](int32_t i0, int32_t i1) {
            for (int32_t i = i0; i < i1; i++)
            {
                const int32_t len = h_plen_.as<int32_t>()[i];
                const int8_t* p   = h_paths_.as<int8_t>() + size_t(i) * max_result_;
                auto* a           = static_cast<AlignmentImpl*>(alignments_[size_t(i)].get());
                std::vector<AlignmentState>& st = a->alignment_storage();
                st.resize(size_t(std::max(len, 0)));
                for (int32_t k = 0; k < len; k++)
                    st[size_t(len - 1 - k)] = static_cast<AlignmentState>(p[k]);
                a->set_status(StatusType::success);
            }
        };
        // the alignments are independent: large batches are filled by a few
        // host threads (each alignment object is touched by one thread)
        auto fill_range = [&](int32_t b0, int32_t b1) {
            const int32_t m   = b1 - b0;
            const int32_t nth = m < 4096 ? 1 : int32_t(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
            if (nth <= 1)
            {
                fill(b0, b1);
                return;
            }
            std::vector<std::thread> th;
            const int32_t per = (m + nth - 1) / nth;
            for (int32_t t = 0; t < nth; t++)
                th.emplace_back(fill, b0 + std::min(m, t * per), b0 + std::min(m, (t + 1) * per));
            for (auto& t : th)
                t.join();
        };
        if (stages_ > 1 && chunk0_[stages_] == n)
        {
            // each stage's paths reach the host while later stages are still
            // aligning: fill them as they arrive
            for (int k = 0; k < stages_; k++)
            {
                GWAMD_HIP_CHECK(hipEventSynchronize(ev_d_[k]));
                fill_range(chunk0_[k], chunk0_[k + 1]);
            }
            GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
        }
        else
        {
            GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
            fill_range(0, n);
        }
        return StatusType::success;
    }

    const std::vector<std::shared_ptr<Alignment>>& get_alignments() const override { return alignments_; }
    void reset() override
    {
        alignments_.clear();
        max_diff_ = 0;
        stages_   = 0; // no launch of this batch yet
    }

    // bench / C ABI helpers: the split path (upload, launch, download) runs
    // one stage on stream_, so sync_alignments waits for stream_ before it
    // fills and last_kernel_ms times that launch (the state of an
    // earlier pipelined align_all() must not survive into a split launch)
    void upload()
    {
        ScopedDevice dev(device_id_);
        const size_t n = alignments_.size();
        stages_        = 1;
        chunk0_[0]     = 0;
        chunk0_[1]     = int32_t(n);
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_lens_, h_lens_.as<int32_t>(), 2 * n * 4, hipMemcpyHostToDevice, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_seqs_, h_seqs_.as<char>(), 2 * n * size_t(stride_), hipMemcpyHostToDevice,
                                       stream_));
    }
    void launch()
    {
        ScopedDevice dev(device_id_);
        stages_    = 1;
        chunk0_[0] = 0;
        chunk0_[1] = int32_t(alignments_.size());
        GWAMD_HIP_CHECK(hipEventRecord(ev_k_[0], stream_));
        launch_range(0, int32_t(alignments_.size()), 0, slots_, stream_);
        GWAMD_HIP_CHECK(hipEventRecord(ev_k_[1], stream_));
    }
    // Pairs [i0, i0 + count) on workspace slots [slot0, slot0 + nslots).
    void launch_range(int32_t i0, int32_t count, int32_t slot0, int32_t nslots, hipStream_t s)
    {
        ScopedDevice dev(device_id_);
        gwamd::aln::Args a = args();
        a.seqs     = d_seqs_ + 2 * size_t(i0) * stride_;
        a.lens     = d_lens_ + 2 * size_t(i0);
        a.paths    = d_paths_ + size_t(i0) * max_result_;
        a.path_len = d_plen_ + i0;
        a.n        = count;
        // run-ahead distances of this stage's pairs: stages on the two compute
        // streams must not share [0, count * sweeps)
        if (a.spec_ed)
            a.spec_ed = a.spec_ed + size_t(i0) * kMaxSpecSweeps;
        a.ws       = d_ws_ + size_t(slot0) * size_t(slot_bytes_);
        if (algo_ == GWAMD_ALIGNER_UKKONEN)
        {
            // the widest band of this batch decides the Ukkonen kernel (plan_banded)
            const int rows = (1 + max_diff_ + 2 * gwamd::aln::kUkkonenP + 1) / 2;
            if (rows > gwamd::aln::kUkChunks * gwamd::aln::kWave)
            {
                a.uk_threads   = std::min(1024, (rows + gwamd::aln::kWave - 1) / gwamd::aln::kWave * gwamd::aln::kWave);
                a.lds_bytes    = uk_wide_lds_;
                a.lds_tile_off = 0;
                a.tile_bytes   = gwamd::aln::kUkTileRows * gwamd::aln::kUkTileCols * 2;
            }
        }
        if (algo_ == GWAMD_ALIGNER_MYERS_BANDED && band_waves_ > 1 && !band_waves_forced_)
        {
            // an aligner planned for long queries (8 waves per pair) runs a
            // launch whose queries are all short with one wave per pair: the
            // one-wave kernel is the default plan for such queries (short
            // bands leave most of 8 waves idle, and one wave per pair keeps
            // more pairs resident)
            int32_t mq = 0;
            for (int32_t k = i0; k < i0 + count; k++)
                mq = std::max(mq, h_lens_.as<int32_t>()[2 * size_t(k)]);
            if (mq <= kLongBandQuery)
                a.band_waves = 1;
        }
        const int grid     = std::min<int>(count, nslots);
        const int ks       = spec_sweeps(count, nslots, a.band_waves);
        if (ks > 0)
        {
            // band doubling run ahead: every (pair, sweep) on its own
            // workgroup, then one workgroup per pair on its own slot
            a.spec_sweeps = ks;
            a.spec_phase  = 1;
            GWAMD_HIP_CHECK(gwamd_internal_banded_launch(&a, algo_, std::min(count * ks, resident_), s));
            a.spec_phase = 2;
            GWAMD_HIP_CHECK(gwamd_internal_banded_launch(&a, algo_, count, s));
        }
        else if (algo_ == GWAMD_ALIGNER_MYERS_BANDED || algo_ == GWAMD_ALIGNER_UKKONEN)
            GWAMD_HIP_CHECK(gwamd_internal_banded_launch(&a, algo_, grid, s));
        else
            GWAMD_HIP_CHECK(gwamd_internal_align_launch(&a, algo_, grid, s));
    }
    // banded Myers: sweeps of the band doubling run ahead on their own
    // workgroups when a launch's pairs leave most of the GPU idle (few long
    // pairs: every pair on its own slot, all (pair, sweep) items resident) and
    // every band's chunk state fits LDS; 0 = the plain loop.
    // GWAMD_BAND_SPEC=k forces k (0..kMaxSpecSweeps, diagnostic)
    int spec_sweeps(int32_t count, int32_t nslots, int32_t waves) const
    {
        if (algo_ != GWAMD_ALIGNER_MYERS_BANDED || count <= 0)
            return 0;
        int k = waves > 1 ? kDefaultSpecSweeps : 0;
        if (const char* e = gwamd::host::diag_env("GWAMD_BAND_SPEC"))
        {
            k = std::atoi(e);
            if (k < 0 || k > kMaxSpecSweeps)
                throw std::invalid_argument("GWAMD_BAND_SPEC must be 0..8 sweeps");
        }
        const bool fits = count <= nslots && int64_t(count) * k <= resident_ && 2 * count <= cus_ &&
                          pat_words_ <= tile_bytes_ / 16;
        return fits ? k : 0;
    }
    // pipeline stages of align_all(): as many (up to kMaxStages) as keep
    // each stage's half of the slots busy four times over; 1 = one stage
    // (GWAMD_ALIGNER_PIPELINE=k forces k stages, 1..kMaxStages, diagnostic)
    int pipeline_stages(int32_t n) const
    {
        if (const char* e = gwamd::host::diag_env("GWAMD_ALIGNER_PIPELINE"))
        {
            const int k = std::atoi(e);
            if (k < 0 || k > kMaxStages)
                throw std::invalid_argument("GWAMD_ALIGNER_PIPELINE must be 0..8 stages");
            return slots_ < 2 ? 1 : std::max(1, std::min(k, n));
        }
        if (slots_ < 2)
            return 1;
        const int64_t per = int64_t(4) * (slots_ / 2); // pairs per stage
        // (config D, 100k pairs on 3,328 slots: 1 / 2 / 4 / 8 stages measured
        // 365 / 348 / 320 / 309 ms per step, gpurun_out/r5g)
        return int(std::max<int64_t>(1, std::min<int64_t>(kMaxStages, n / per)));
    }
    void download()
    {
        ScopedDevice dev(device_id_);
        const size_t n = alignments_.size();
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_paths_.as<int8_t>(), d_paths_, n * size_t(max_result_),
                                       hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_plen_.as<int32_t>(), d_plen_, n * 4, hipMemcpyDeviceToHost, stream_));
    }
    void synchronize()
    {
        ScopedDevice dev(device_id_);
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    const int8_t* host_paths() const { return h_paths_.as<int8_t>(); }
    const int32_t* host_path_lengths() const { return h_plen_.as<int32_t>(); }
    int32_t max_result_length() const { return max_result_; }
    int32_t grid() const { return slots_; }
    void path_stats(int64_t* out)
    {
        ScopedDevice dev(device_id_);
        unsigned long long v[3] = {0, 0, 0};
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
        GWAMD_HIP_CHECK(hipMemcpy(v, d_stats_, sizeof(v), hipMemcpyDeviceToHost));
        for (int i = 0; i < 3; i++)
            out[i] = int64_t(v[i]);
    }
    int64_t device_bytes() const { return device_bytes_; }

private:
    static int64_t a16(int64_t v) { return (v + 15) & ~int64_t(15); }

    // aligner_global_ukkonen.cpp:23,32: float 0.1 times max_target_length, truncated
    int32_t ukkonen_max_difference() const
    {
        return int32_t(float(max_t_) * 0.1f);
    }
    // ukkonen_max_score_matrix_size (ukkonen_gpu.cu:313-324): band rows for the
    // largest allowed length difference
    int32_t ukkonen_band_rows() const
    {
        return (1 + ukkonen_max_difference() + 2 * gwamd::aln::kUkkonenP + 1) / 2;
    }

    // GWAMD_ALIGNER_GRID (diagnostic): resident workgroups per CU instead of
    // the occupancy query's answer
    void apply_grid_override()
    {
        const char* env = gwamd::host::diag_env("GWAMD_ALIGNER_GRID");
        if (!env || !*env)
            return;
        const int per_cu = std::atoi(env);
        if (per_cu < 1 || per_cu > 32)
            throw std::invalid_argument("GWAMD_ALIGNER_GRID must be 1..32 workgroups per CU");
        int cus = 1;
        GWAMD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
        slots_ = per_cu * cus;
    }

    void plan_banded()
    {
        using namespace gwamd::aln;
        const int pat_words = (max_q_ + kWordBits - 1) / kWordBits;
        if (algo_ == GWAMD_ALIGNER_MYERS_BANDED)
        {
            // target as 2-bit letter codes, letter-major query patterns, and a
            // 4 KiB chunk-state / backtrace tile
            lds_target_off_  = 0;
            lds_pat_off_     = int32_t(a16((max_t_ + 15) / 16 * 4 + 16));
            lds_tile_off_    = int32_t(lds_pat_off_ + a16(int64_t(pat_words) * 16 + 16));
            // at least 128 16-byte band entries (two columns of 64 words, or
            // 128 chunk words: a smaller LDS image keeps more short pairs
            // resident, D_banded 372.8k -> 451.7k alignments/s with 2 KiB
            // against 4 KiB, gpurun_out/r4o); up to the whole band's chunk state while the
            // workgroup's LDS stays within the CU's 160 KiB (a 65,536 bp query:
            // 16 KiB target + 32 KiB patterns + 32 KiB state; wider bands keep
            // the state in HBM and wait on it every column)
            tile_bytes_      = 2048;
            int64_t want     = a16(int64_t(pat_words) * 16);
            want             = std::min<int64_t>(want, (163840 - 512 - lds_tile_off_) & ~int64_t(511)); // static LDS
            if (const char* tb = gwamd::host::diag_env("GWAMD_BAND_TILE_BYTES")) // parity tests: HBM chunk state
            {
                // LDS bytes for the chunk state / backtrace tile: 2048 (128
                // words) up to 48 KiB, in whole 512-byte steps; anything else
                // is a typo that would silently keep the default plan
                char* end     = nullptr;
                const long v  = std::strtol(tb, &end, 10);
                if (end == tb || *end != '\0' || v < 2048 || v > (48 << 10) || v % 512 != 0)
                    throw std::invalid_argument("GWAMD_BAND_TILE_BYTES must be 2048..49152 in steps of 512");
                tile_bytes_ = int32_t(v);
                want        = v;
            }
            if (want > tile_bytes_)
                tile_bytes_ = int32_t(want);
            // long queries (bands of many 32-word chunks) run 8 waves per pair,
            // 16 target columns in flight; short ones keep one wave per pair
            // and their occupancy
            band_waves_ = max_q_ > kLongBandQuery ? 8 : 1;
            if (const char* bwv = gwamd::host::diag_env("GWAMD_BAND_WAVES"))
            {
                const std::string v(bwv);
                if (v != "1" && v != "4" && v != "8" && v != "16")
                    throw std::invalid_argument("GWAMD_BAND_WAVES must be 1, 4, 8 or 16");
                band_waves_        = std::stoi(v);
                band_waves_forced_ = true;
            }
            lds_bytes_       = lds_tile_off_ + tile_bytes_;
            // band entries (pv, mv, score, pad) of the widest band (the whole query)
            slot_bytes_ = a16(int64_t(pat_words) * (max_t_ + 1) * 16 + 64);
        }
        else
        {
            // Ukkonen.  The band of a pair is (1 + |n - m| + 2p + 1) / 2 rows;
            // the workspace is sized for the largest allowed difference, but
            // each launch runs the single-wave kernel (ukkonen_kernel, up to
            // kUkChunks * 64 rows) when every pair of the batch fits it, and
            // the workgroup kernel (ukkonen_wide_kernel, up to 1,024 threads
            // of kUkWideChunks rows, as calc_good_blockdim, ukkonen_gpu.cu:
            // 268-273) otherwise.  Both keep the sequences in LDS; the wide
            // kernel's backtrace tile reuses them.
            const int rows      = ukkonen_band_rows();
            lds_target_off_     = 0;
            lds_seq2_off_       = int32_t(a16(stride_ + 16));
            const int64_t seqs  = lds_seq2_off_ + a16(stride_ + 16);
            uk_narrow_tile_off_ = int32_t(seqs);
            // ukkonen_kernel's backtrace tile (the narrow kernel's only use of
            // it; any size is correct, reads outside it go to HBM).  Pairs up
            // to 8 kb: 5 KiB, 10 workgroups per CU at 5 kb (8 KiB: 8; measured
            // 653-658k against 611k alignments/s on D_ukkonen, profiles/
            // r5an_bench); up to 32 kb: 8 KiB, which keeps the window walk
            // for bands up to 255 rows; pairs of 32 kb and more (few per
            // batch, one workgroup per CU already) take what the CU's LDS has
            // left, up to 48 KiB, so the walk refills every ~100 columns
            // instead of every ~22 (one HBM latency each)
            int32_t uk_tile     = stride_ <= 8192 ? 5120 : 8192;
            if (stride_ >= 32768)
                uk_tile = int32_t(std::max<int64_t>(8192, std::min<int64_t>(49152, (163840 - 64 - seqs) & ~int64_t(511))));
            if (const char* tb = gwamd::host::diag_env("GWAMD_UK_TILE_BYTES"))
            {
                char* end    = nullptr;
                const long v = std::strtol(tb, &end, 10);
                if (end == tb || *end != '\0' || v < 1024 || v > 65536 || v % 512 != 0)
                    throw std::invalid_argument("GWAMD_UK_TILE_BYTES must be 1024..65536 in steps of 512");
                uk_tile = int32_t(v);
            }
            uk_narrow_lds_      = int32_t(seqs + uk_tile);
            lds_edge_off_       = int32_t(std::max<int64_t>(seqs, kUkTileRows * kUkTileCols * 2));
            uk_wide_lds_        = lds_edge_off_ + 4 * kUkWideChunks * 16 * 4;
            slot_bytes_         = a16(int64_t(rows) * (int64_t(max_q_) + max_t_ + 2) * 2 + 64);
            lds_bytes_          = uk_narrow_lds_;
            tile_bytes_         = uk_tile;
            lds_tile_off_       = uk_narrow_tile_off_;
        }
        if (lds_bytes_ > 163840 ||
            (algo_ == GWAMD_ALIGNER_UKKONEN && uk_wide_lds_ > 163840))
            throw std::invalid_argument("aligner problem size does not fit in LDS");
        pat_words_ = pat_words;
        int per_cu = 1, cus = 1;
        GWAMD_HIP_CHECK(gwamd_internal_banded_occupancy(algo_, lds_bytes_, band_waves_, &per_cu));
        if (algo_ == GWAMD_ALIGNER_UKKONEN && ukkonen_band_rows() > kUkChunks * kWave)
        {
            // batches with wide bands run one workgroup per pair
            int wide = 1;
            GWAMD_HIP_CHECK(gwamd_internal_ukkonen_wide_occupancy(1024, uk_wide_lds_, &wide));
            per_cu = std::max(per_cu, wide);
        }
        GWAMD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
        slots_    = std::max(1, per_cu * cus);
        resident_ = slots_;
        cus_      = cus;
        // resident workspace slots within 64 GiB of the 288 GB HBM; only a
        // batch whose slots need more (32 pairs of 65,536 bp: 32 band-matrix
        // slots of 2.15 GB, and one slot fewer than pairs doubles the kernel)
        // may take up to 96 GiB, and at most 3/4 of the free memory, so short-
        // pair aligners keep a plan that does not depend on what else the
        // process has allocated
        int64_t ws_cap        = int64_t(64) << 30;
        const int64_t want_ws = int64_t(std::min(slots_, max_n_)) * slot_bytes_;
        if (want_ws > ws_cap)
        {
            size_t free_b = 0, total_b = 0;
            GWAMD_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            ws_cap = std::max<int64_t>(ws_cap, std::min<int64_t>({int64_t(96) << 30, want_ws,
                                                                  int64_t(free_b / 4 * 3)}));
        }
        slots_ = int32_t(std::max<int64_t>(1, std::min<int64_t>(slots_, ws_cap / slot_bytes_)));
        apply_grid_override();
        slots_ = std::min(slots_, max_n_);
    }

    void plan()
    {
        using namespace gwamd::aln;
        if (algo_ == GWAMD_ALIGNER_MYERS_BANDED || algo_ == GWAMD_ALIGNER_UKKONEN)
        {
            plan_banded();
            return;
        }
        const int pat_words = (max_q_ + kWordBits - 1) / kWordBits;
        const bool hm       = algo_ == GWAMD_ALIGNER_HIRSCHBERG_MYERS;
        // long mode: patterns in HBM, target codes through a generic pointer;
        // full Myers takes it past 8,192 x 65,535 (its stripes work either way)
        // full Myers always: its patterns are read only when a stripe starts,
        // and with them in HBM a wave needs ~4 KiB of LDS instead of ~10 KiB,
        // so the occupancy query allows twice the waves (config D_myers:
        // 353 -> 241 ms per 100k pairs, profiles/r3e_bench)
        long_mode_ = hm ? (max_q_ > gwamd::host::kHmShortQuery || max_t_ > gwamd::host::kHmShortTarget) : true;
        // GWAMD_HM_STRIPE_BLOCKS=1..4 (parity tests): long mode at any size, with
        // stripes of that many blocks, so short pairs take the striped sweeps
        stripe_blocks_ = kMaxChunks;
        if (const char* sb = gwamd::host::diag_env("GWAMD_HM_STRIPE_BLOCKS"))
            if (hm && std::atoi(sb) >= 1 && std::atoi(sb) <= kMaxChunks)
            {
                stripe_blocks_ = std::atoi(sb);
                long_mode_     = true;
            }
        const int sc_bytes  = long_mode_ ? 4 : 2; // split scores
        lds_target_off_     = 0;
        // target as 2-bit letter codes (long mode: in HBM past kHmLdsTarget)
        tcod_hbm_           = long_mode_ && max_t_ > gwamd::host::kHmLdsTarget;
        lds_pat_off_        = int32_t(tcod_hbm_ ? 0 : a16((max_t_ + 15) / 16 * 4 + 16));
        // long mode: the patterns live in the HBM slot
        lds_scratch_off_    = int32_t(lds_pat_off_ + (long_mode_ ? 0 : a16(int64_t(pat_words) * 32 + 16)));
        scratch_bytes_      = 0;
        if (hm) // LDS split scores of segments up to kSplitLds columns
            scratch_bytes_ = int32_t(a16(int64_t(2) * kSplitLds * sc_bytes));
        else // full Myers: the backtrace tile (kTbW words x 64 columns of pv, mv, score)
            scratch_bytes_ = 4 * 64 * 12;
        lds_stack_off_ = lds_scratch_off_ + scratch_bytes_;
        lds_bytes_     = lds_stack_off_ + (hm ? kStackSize * 16 : 0);
        if (lds_bytes_ > 65536)
            throw std::invalid_argument("aligner problem size does not fit in LDS");
        pat_words_ = pat_words;
        int per_cu = 1, cus = 1;
        GWAMD_HIP_CHECK(gwamd_internal_align_occupancy(algo_ + (long_mode_ ? 100 : 0), lds_bytes_, &per_cu));
        GWAMD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
        slots_ = std::max(1, per_cu * cus);
        if (hm)
        {
            // slot: split scores of wide segments (forward, reverse), the
            // breadth-first frontier (two buffers of (qb, qe, tb, te) + one
            // split column per entry; at most 2 * (query + 1) segments: every
            // leaf has a query row or is one of the target-only halves of a
            // split), per-lane base cases (columns of every segment: target +
            // one per segment; (offset, length) per segment; paths), and in
            // long mode the query patterns and the striped sweeps' deltas
            split_off_  = 0;
            front_cap_  = 2 * (max_q_ + 2);
            front_off_  = a16(int64_t(2) * (stride_ + 1 + kWave) * sc_bytes + 64);
            leaf_cols_  = max_t_ + front_cap_ + 2;
            leaf_off_   = a16(front_off_ + int64_t(front_cap_) * (2 * 16 + 4) + 64);
            int64_t end = a16(leaf_off_ + int64_t(leaf_cols_) * kLeafColBytes + 16 + int64_t(front_cap_) * 8 +
                              max_q_ + max_t_ + 64);
            pat_off_  = end;
            hbuf_off_ = a16(pat_off_ + (long_mode_ ? int64_t(pat_words) * 32 + 64 : 0));
            tcod_off_ = a16(hbuf_off_ + (long_mode_ ? int64_t(max_t_) + 1 + kWave + 64 : 0));
            slot_bytes_ = a16(tcod_off_ + (tcod_hbm_ ? int64_t(max_t_ + 15) / 16 * 4 + 64 : 0));
            const int64_t cap = int64_t(16) << 30; // resident slots within 16 GiB of the 288 GB HBM
            slots_            = int32_t(std::max<int64_t>(1, std::min<int64_t>(slots_, cap / slot_bytes_)));
        }
        else
        {
            // full matrix: pv, mv, score per (word, column), then the stripes'
            // per-column deltas, and in long mode the patterns and target codes
            slot_bytes_ = gwamd::host::myers_slot_layout(max_q_, max_t_, &hbuf_off_, &pat_off_, &tcod_off_);
            if (slot_bytes_ > gwamd::host::kMyersMaxSlot)
                throw std::invalid_argument("max_query_length x max_target_length too large for the full Myers "
                                            "aligner's score matrix (" + std::to_string(slot_bytes_) + " bytes)");
            // resident slots within kMyersWorkspace (or a single slot)
            slots_ = int32_t(std::max<int64_t>(1, std::min<int64_t>(slots_, gwamd::host::kMyersWorkspace / slot_bytes_)));
        }
        apply_grid_override();
        slots_ = std::min(slots_, max_n_);
    }

    gwamd::aln::Args args() const
    {
        gwamd::aln::Args a{};
        a.seqs             = d_seqs_;
        a.lens             = d_lens_;
        a.stride           = stride_;
        a.paths            = d_paths_;
        a.path_len         = d_plen_;
        a.max_path_length  = max_result_;
        a.n                = int32_t(alignments_.size());
        a.max_query_length = max_q_;
        a.max_matrix_elems = int64_t((max_q_ + 3) / 4) * (gwamd::aln::kFullMyers + 1);
        a.ws               = d_ws_;
        a.ws_slot_bytes    = slot_bytes_;
        a.ws_front_off     = front_off_;
        a.front_cap        = front_cap_;
        a.ws_leaf_off      = leaf_off_;
        a.leaf_cols        = leaf_cols_;
        a.ws_split_off     = split_off_;
        a.ws_pat_off       = pat_off_;
        a.ws_hbuf_off      = hbuf_off_;
        a.ws_tcod_off      = tcod_hbm_ ? tcod_off_ : -1;
        a.long_mode        = long_mode_ ? 1 : 0;
        a.stripe_blocks    = stripe_blocks_;
        a.lds_target_off   = lds_target_off_;
        a.lds_pat_off      = lds_pat_off_;
        a.lds_scratch_off  = lds_scratch_off_;
        a.lds_stack_off    = lds_stack_off_;
        a.lds_bytes        = lds_bytes_;
        a.pat_words        = pat_words_;
        a.scratch_bytes    = scratch_bytes_;
        a.lds_seq2_off     = lds_seq2_off_;
        a.lds_tile_off     = lds_tile_off_;
        a.tile_bytes       = tile_bytes_;
        a.ukkonen_p        = gwamd::aln::kUkkonenP;
        a.uk_threads       = 0; // launch(): the batch's widest band may need ukkonen_wide_kernel
        a.band_waves       = band_waves_;
        a.spec_phase       = 0;
        a.spec_sweeps      = 0;
        a.spec_ed          = d_spec_ed_;
        a.lds_edge_off     = lds_edge_off_;
        a.stats            = d_stats_;
        return a;
    }

    int32_t max_q_, max_t_, max_n_;
    int algo_;
    hipStream_t stream_;
    int32_t device_id_;
    int32_t stride_ = 0, max_result_ = 0;
    int32_t lds_target_off_ = 0, lds_pat_off_ = 0, lds_scratch_off_ = 0, lds_stack_off_ = 0, lds_bytes_ = 0;
    int32_t pat_words_ = 0, scratch_bytes_ = 0;
    int64_t front_off_ = 0;
    int32_t front_cap_ = 0;
    int64_t leaf_off_  = 0;
    int32_t leaf_cols_ = 0;
    int64_t split_off_ = 0, pat_off_ = 0, hbuf_off_ = 0, tcod_off_ = 0;
    bool tcod_hbm_     = false;
    bool long_mode_    = false;
    int32_t stripe_blocks_ = gwamd::aln::kMaxChunks;
    int32_t lds_seq2_off_ = 0, lds_tile_off_ = 0, tile_bytes_ = 0, band_waves_ = 1;
    int32_t lds_edge_off_ = 0, uk_narrow_tile_off_ = 0, uk_narrow_lds_ = 0, uk_wide_lds_ = 0;
    int32_t max_diff_ = 0; // largest |query - target| of the batch
    // pipelined align_all(): the second compute stream, the copy-in and
    // copy-out streams, fork / join events, per stage the upload-done and
    // download-done events and the kernel's start / stop events; stages_ of
    // the last align_all() (0: none yet) and their first pairs
    static constexpr int kMaxStages = 8;
    static constexpr int kLongBandQuery     = 8192; // banded Myers: longer queries run 8 waves per pair
    bool band_waves_forced_                 = false; // GWAMD_BAND_WAVES (diagnostic)
    static constexpr int kMaxSpecSweeps     = 8; // banded Myers sweeps run ahead, at most
    static constexpr int kDefaultSpecSweeps = 5; // est x 1 .. x 16
    hipStream_t stream2_ = nullptr, s_in_ = nullptr, s_out_ = nullptr;
    hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
    hipEvent_t ev_d_[kMaxStages]     = {};
    hipEvent_t ev_h_[kMaxStages]     = {};
    hipEvent_t ev_k_[2 * kMaxStages] = {};
    int stages_                      = 0;
    int32_t chunk0_[kMaxStages + 1]  = {};
    int32_t slots_ = 1;
    int64_t slot_bytes_ = 0, device_bytes_ = 0;
    char* d_seqs_     = nullptr;
    int32_t* d_lens_  = nullptr;
    int8_t* d_paths_  = nullptr;
    int32_t* d_plen_  = nullptr;
    uint8_t* d_ws_    = nullptr;
    unsigned long long* d_stats_ = nullptr;
    int32_t* d_spec_ed_          = nullptr; // banded Myers: distances of the sweeps run ahead
    int32_t resident_ = 1, cus_ = 1;        // workgroups resident at once, CUs
    std::shared_ptr<DeviceBudget> budget_;  // the allocator pool this aligner reserved from
    int64_t reserved_ = 0;
    PinnedBuf h_seqs_, h_lens_, h_paths_, h_plen_;
    std::vector<std::shared_ptr<Alignment>> alignments_;
};

std::unique_ptr<Aligner> create_aligner(int32_t max_query_length, int32_t max_target_length, int32_t max_alignments,
                                        AlignmentType type, DefaultDeviceAllocator allocator, hipStream_t stream,
                                        int32_t device_id)
{
    // aligner.cpp:30-38
    if (type == AlignmentType::global_alignment)
        return std::make_unique<AlignerGlobalHip>(max_query_length, max_target_length, max_alignments,
                                                  GWAMD_ALIGNER_HIRSCHBERG_MYERS, stream, device_id,
                                                  allocator.budget());
    throw std::runtime_error("Aligner for specified type not implemented yet.");
}

std::unique_ptr<Aligner> create_global_aligner(int32_t max_query_length, int32_t max_target_length,
                                               int32_t max_alignments, GlobalAlgorithm algorithm, hipStream_t stream,
                                               int32_t device_id)
{
    const int algo = int(algorithm);
    if (algo < GWAMD_ALIGNER_HIRSCHBERG_MYERS || algo > GWAMD_ALIGNER_UKKONEN)
        throw std::invalid_argument("unknown aligner algorithm");
    return std::make_unique<AlignerGlobalHip>(max_query_length, max_target_length, max_alignments, algo, stream,
                                              device_id);
}

std::unique_ptr<Aligner> create_aligner(int32_t max_query_length, int32_t max_target_length, int32_t max_alignments,
                                        AlignmentType type, hipStream_t stream, int32_t device_id,
                                        int64_t max_device_memory_allocator_caching_size)
{
    // aligner.cpp:40-63
    if (max_device_memory_allocator_caching_size < -1)
        throw std::invalid_argument("max_device_memory_allocator_caching_size has to be either -1 (=all available "
                                    "GPU memory) or greater or equal than 0.");
    return create_aligner(max_query_length, max_target_length, max_alignments, type,
                          DefaultDeviceAllocator(max_device_memory_allocator_caching_size), stream, device_id);
}

} // namespace cudaaligner
} // namespace genomeworks
} // namespace claraparabricks

// ===========================================================================
// C ABI (include/gwamd_cudaaligner.h)
// ===========================================================================
namespace ca = claraparabricks::genomeworks::cudaaligner;

namespace
{
template <typename F>
int32_t guarded_aln(F&& f)
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
    catch (const std::runtime_error& e)
    {
        gwamd::host::last_error() = e.what();
        return std::string(e.what()).rfind("HIP error", 0) == 0 ? GWAMD_E_HIP : GWAMD_E_RUNTIME;
    }
    catch (const std::exception& e)
    {
        gwamd::host::last_error() = e.what();
        return GWAMD_E_RUNTIME;
    }
}
} // namespace

struct gwamd_aligner
{
    std::unique_ptr<ca::AlignerGlobalHip> impl;
};

struct gwamd_device_allocator
{
    claraparabricks::genomeworks::DefaultDeviceAllocator alloc;
};

extern "C" {

int32_t gwamd_aligner_create(gwamd_aligner** out, int32_t max_query_length, int32_t max_target_length,
                             int32_t max_alignments, int32_t alignment_type, int32_t algorithm, void* stream,
                             int32_t device_id, int64_t max_caching)
{
    return guarded_aln([&] {
        if (!out)
            throw std::invalid_argument("out is NULL");
        if (max_caching < -1)
            throw std::invalid_argument("max_device_memory_allocator_caching_size has to be either -1 (=all "
                                        "available GPU memory) or greater or equal than 0.");
        if (alignment_type != ca::AlignmentType::global_alignment)
            throw std::runtime_error("Aligner for specified type not implemented yet.");
        if (algorithm < GWAMD_ALIGNER_HIRSCHBERG_MYERS || algorithm > GWAMD_ALIGNER_UKKONEN)
            throw std::invalid_argument("unknown aligner algorithm");
        auto h  = std::make_unique<gwamd_aligner>();
        h->impl = std::make_unique<ca::AlignerGlobalHip>(
            max_query_length, max_target_length, max_alignments, algorithm, static_cast<hipStream_t>(stream),
            device_id, max_caching >= 0 ? std::make_shared<claraparabricks::genomeworks::DeviceBudget>(max_caching)
                                        : nullptr);
        *out    = h.release();
        return int32_t(0);
    });
}

void gwamd_aligner_destroy(gwamd_aligner* a) { delete a; }

int32_t gwamd_device_allocator_create(gwamd_device_allocator** out, int64_t max_caching_size)
{
    return guarded_aln([&] {
        if (!out)
            throw std::invalid_argument("out is NULL");
        if (max_caching_size < -1)
            throw std::invalid_argument("max_caching_size has to be either -1 (=all available GPU memory) or "
                                        "greater or equal than 0.");
        auto h   = std::make_unique<gwamd_device_allocator>();
        h->alloc = claraparabricks::genomeworks::create_default_device_allocator(max_caching_size);
        *out     = h.release();
        return int32_t(0);
    });
}

void gwamd_device_allocator_destroy(gwamd_device_allocator* a) { delete a; }

int64_t gwamd_device_allocator_capacity(const gwamd_device_allocator* a)
{
    return a ? a->alloc.max_cached_bytes() : -1;
}

int64_t gwamd_device_allocator_used(const gwamd_device_allocator* a)
{
    return a && a->alloc.budget() ? a->alloc.budget()->used() : 0;
}

int64_t gwamd_device_allocator_default_size(void)
{
    return claraparabricks::genomeworks::create_default_device_allocator().max_cached_bytes();
}

int32_t gwamd_aligner_create_with_allocator(gwamd_aligner** out, int32_t max_query_length, int32_t max_target_length,
                                            int32_t max_alignments, int32_t alignment_type, int32_t algorithm,
                                            void* stream, int32_t device_id, gwamd_device_allocator* allocator)
{
    return guarded_aln([&] {
        if (!out || !allocator)
            throw std::invalid_argument("out or allocator is NULL");
        if (alignment_type != ca::AlignmentType::global_alignment)
            throw std::runtime_error("Aligner for specified type not implemented yet.");
        if (algorithm < GWAMD_ALIGNER_HIRSCHBERG_MYERS || algorithm > GWAMD_ALIGNER_UKKONEN)
            throw std::invalid_argument("unknown aligner algorithm");
        auto h  = std::make_unique<gwamd_aligner>();
        h->impl = std::make_unique<ca::AlignerGlobalHip>(max_query_length, max_target_length, max_alignments,
                                                         algorithm, static_cast<hipStream_t>(stream), device_id,
                                                         allocator->alloc.budget());
        *out    = h.release();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_add_alignment(gwamd_aligner* a, const char* q, int32_t qlen, const char* t, int32_t tlen,
                                    int32_t rc_q, int32_t rc_t)
{
    return guarded_aln([&] { return int32_t(a->impl->add_alignment(q, qlen, t, tlen, rc_q != 0, rc_t != 0)); });
}

int32_t gwamd_aligner_align_all(gwamd_aligner* a)
{
    return guarded_aln([&] { return int32_t(a->impl->align_all()); });
}

int32_t gwamd_aligner_sync_alignments(gwamd_aligner* a)
{
    return guarded_aln([&] { return int32_t(a->impl->sync_alignments()); });
}

int32_t gwamd_aligner_num_alignments(const gwamd_aligner* a) { return int32_t(a->impl->get_alignments().size()); }

int32_t gwamd_aligner_get_alignment(gwamd_aligner* a, int32_t i, int8_t* states, int32_t cap, int32_t* status)
{
    return guarded_aln([&] {
        const auto& al = a->impl->get_alignments();
        if (i < 0 || i >= int32_t(al.size()))
            throw std::invalid_argument("alignment index out of range");
        const auto& st = al[size_t(i)]->get_alignment();
        if (status)
            *status = int32_t(al[size_t(i)]->get_status());
        if (states && int32_t(st.size()) <= cap)
            for (size_t k = 0; k < st.size(); k++)
                states[k] = int8_t(st[k]);
        return int32_t(st.size());
    });
}

int32_t gwamd_aligner_get_sequences(gwamd_aligner* a, int32_t i, const char** q, int32_t* qlen, const char** t,
                                    int32_t* tlen)
{
    return guarded_aln([&] {
        const auto& al = a->impl->get_alignments();
        if (i < 0 || i >= int32_t(al.size()))
            throw std::invalid_argument("alignment index out of range");
        const std::string& qs = al[size_t(i)]->get_query_sequence();
        const std::string& ts = al[size_t(i)]->get_target_sequence();
        *q                    = qs.data();
        *qlen                 = int32_t(qs.size());
        *t                    = ts.data();
        *tlen                 = int32_t(ts.size());
        return int32_t(0);
    });
}

int32_t gwamd_aligner_get_cigar(gwamd_aligner* a, int32_t i, char* buf, int32_t cap)
{
    return guarded_aln([&] {
        const auto& al = a->impl->get_alignments();
        if (i < 0 || i >= int32_t(al.size()))
            throw std::invalid_argument("alignment index out of range");
        const std::string c = al[size_t(i)]->convert_to_cigar();
        if (buf && int32_t(c.size()) < cap)
            std::memcpy(buf, c.c_str(), c.size() + 1);
        return int32_t(c.size());
    });
}

void gwamd_aligner_reset(gwamd_aligner* a) { a->impl->reset(); }

int32_t gwamd_alignment_format(const char* query, int32_t query_length, const char* target, int32_t target_length,
                               const int8_t* states, int32_t num_states, int32_t maximal_line_length,
                               char* query_out, char* pairing_out, char* target_out, int32_t cap,
                               int32_t* linebreak_after)
{
    return guarded_aln([&] {
        ca::AlignmentImpl al(query, query_length, target, target_length);
        std::vector<ca::AlignmentState> st(size_t(std::max(num_states, 0)));
        for (int32_t k = 0; k < num_states; k++)
            st[size_t(k)] = static_cast<ca::AlignmentState>(states[k]);
        al.set_alignment(std::move(st));
        const ca::FormattedAlignment f = al.format_alignment(maximal_line_length);
        if (linebreak_after)
            *linebreak_after = f.linebreak_after;
        const int32_t n = int32_t(f.query.size());
        if (n < cap)
        {
            for (auto pr : {std::make_pair(query_out, &f.query), std::make_pair(pairing_out, &f.pairing),
                            std::make_pair(target_out, &f.target)})
                if (pr.first)
                    std::memcpy(pr.first, pr.second->c_str(), pr.second->size() + 1);
        }
        return n;
    });
}

int32_t gwamd_alignment_cigar(const int8_t* states, int32_t num_states, char* buf, int32_t cap)
{
    return guarded_aln([&] {
        ca::AlignmentImpl al("", 0, "", 0);
        std::vector<ca::AlignmentState> st(size_t(std::max(num_states, 0)));
        for (int32_t k = 0; k < num_states; k++)
            st[size_t(k)] = static_cast<ca::AlignmentState>(states[k]);
        al.set_alignment(std::move(st));
        const std::string c = al.convert_to_cigar();
        if (buf && int32_t(c.size()) < cap)
            std::memcpy(buf, c.c_str(), c.size() + 1);
        return int32_t(c.size());
    });
}

int32_t gwamd_aligner_upload(gwamd_aligner* a)
{
    return guarded_aln([&] {
        a->impl->upload();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_launch(gwamd_aligner* a)
{
    return guarded_aln([&] {
        a->impl->launch();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_download(gwamd_aligner* a)
{
    return guarded_aln([&] {
        a->impl->download();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_synchronize(gwamd_aligner* a)
{
    return guarded_aln([&] {
        a->impl->synchronize();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_get_paths(gwamd_aligner* a, const int8_t** paths, const int32_t** lengths, int32_t* stride)
{
    *paths   = a->impl->host_paths();
    *lengths = a->impl->host_path_lengths();
    *stride  = a->impl->max_result_length();
    return 0;
}

int32_t gwamd_aligner_get_config(const gwamd_aligner* a, int32_t* grid, int64_t* device_bytes)
{
    *grid         = a->impl->grid();
    *device_bytes = a->impl->device_bytes();
    return 0;
}

int32_t gwamd_aligner_last_kernel_ms(gwamd_aligner* a, double* ms)
{
    if (!a || !ms)
    {
        gwamd::host::last_error() = "gwamd_aligner_last_kernel_ms: null argument";
        return GWAMD_E_INVALID_ARGUMENT;
    }
    return guarded_aln([&] {
        *ms = a->impl->last_kernel_ms();
        return int32_t(0);
    });
}

int32_t gwamd_aligner_get_stats(gwamd_aligner* a, int64_t* hbm_state_sweeps, int64_t* ukkonen_wide_pairs,
                                int64_t* ukkonen_max_rows_per_thread)
{
    if (!a || !hbm_state_sweeps || !ukkonen_wide_pairs || !ukkonen_max_rows_per_thread)
    {
        gwamd::host::last_error() = "gwamd_aligner_get_stats: null argument";
        return GWAMD_E_INVALID_ARGUMENT;
    }
    return guarded_aln([&] {
        int64_t v[3];
        a->impl->path_stats(v);
        *hbm_state_sweeps            = v[0];
        *ukkonen_wide_pairs          = v[1];
        *ukkonen_max_rows_per_thread = v[2];
        return int32_t(0);
    });
}

int32_t gwamd_aligner_pair_fits(int32_t algorithm, int32_t max_query_length, int32_t max_target_length)
{
    if (algorithm < GWAMD_ALIGNER_HIRSCHBERG_MYERS || algorithm > GWAMD_ALIGNER_UKKONEN || max_query_length < 0 ||
        max_target_length < 0)
    {
        gwamd::host::last_error() = "gwamd_aligner_pair_fits: bad algorithm or negative length";
        return GWAMD_E_INVALID_ARGUMENT;
    }
    int32_t lq = 0, lt = 0;
    gwamd::host::aligner_max_lengths(algorithm, lq, lt);
    if (max_query_length > lq || max_target_length > lt)
        return 0;
    if (algorithm == GWAMD_ALIGNER_MYERS &&
        gwamd::host::myers_slot_layout(max_query_length, max_target_length, nullptr, nullptr, nullptr) >
            gwamd::host::kMyersMaxSlot)
        return 0;
    if (algorithm == GWAMD_ALIGNER_UKKONEN &&
        (1 + int32_t(float(max_target_length) * 0.1f) + 2 * gwamd::aln::kUkkonenP + 1) / 2 >
            gwamd::aln::kUkWideChunks * 1024)
        return 0;
    return 1;
}

int32_t gwamd_aligner_max_lengths(int32_t algorithm, int32_t* max_query, int32_t* max_target)
{
    if (max_query == nullptr || max_target == nullptr || algorithm < GWAMD_ALIGNER_HIRSCHBERG_MYERS ||
        algorithm > GWAMD_ALIGNER_UKKONEN)
    {
        gwamd::host::last_error() = "gwamd_aligner_max_lengths: bad algorithm or NULL output";
        return GWAMD_E_INVALID_ARGUMENT;
    }
    gwamd::host::aligner_max_lengths(algorithm, *max_query, *max_target);
    return 0;
}

} // extern "C"
