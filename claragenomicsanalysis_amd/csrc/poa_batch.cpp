// Host side of the MI355X POA path: the reference's cudapoa::Batch API
// (cudapoa/include/.../batch.hpp:133-228) implemented over HIP, plus the plain
// C ABI declared in include/gwamd_cudapoa.h.
//
// Host semantics follow the reference's CudapoaBatch (cudapoa_batch.cuh:56-632)
// and BatchBlock (allocate_block.hpp:47-460): the same score/size type choice,
// the same window capacity (max_poas) and score-buffer budget accounting, the
// same per-entry status codes, and the same error behaviour (throws where the
// reference throws).  Device memory is laid out for the HIP kernels
// (poa_kernels.hip), not the reference's slab.
#include <claraparabricks/genomeworks/cudapoa/batch.hpp>
#include <claraparabricks/genomeworks/cudapoa/utils.hpp>

#include "gwamd_cudapoa.h"
#include "host_common.hpp"
#include "poa_batch_internal.hpp"
#include "poa_common.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <sstream>
#include <string>

extern "C" hipError_t gwamd_internal_poa_launch(const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d,
                                       const gwamd::poa::Scores* sc, int score_bits, int size_bits, int banded,
                                       int msa, hipStream_t stream);
extern "C" int gwamd_internal_poa_blocks_per_cu(const gwamd::poa::Dims* d, int score_bits, int size_bits, int banded,
                                                int msa);

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

using gwamd::host::PinnedBuf;
using gwamd::host::ScopedDevice;

namespace
{

// use32bitScore / use32bitSize (cudapoa_limits.hpp:28-53)
bool use32bit_score(const BatchSize& bs, int16_t gap, int16_t mismatch, int16_t match)
{
    int32_t upper = bs.max_sequence_size * match;
    int32_t lower = bs.max_sequence_size * std::max(gap, mismatch) +
                    (bs.max_matrix_graph_dimension - bs.max_sequence_size) * gap;
    return upper > INT16_MAX || (-lower) > (INT16_MAX + 1);
}

bool use32bit_size(const BatchSize& bs, bool banded)
{
    int32_t m = bs.max_consensus_size;
    m         = std::max(m, banded ? bs.max_matrix_graph_dimension_banded : bs.max_matrix_graph_dimension);
    m         = std::max(m, bs.max_matrix_sequence_dimension);
    return m > INT16_MAX;
}

inline int64_t align8(int64_t v) { return (v + 7) & ~int64_t(7); }

// Device bytes per window as accounted by the reference
// (allocate_block.hpp:292-338); sizes of SizeT/ScoreT are the chosen types.
int64_t reference_device_bytes_per_poa(const BatchSize& bs, bool banded, bool msa, int size_bytes)
{
    const int64_t gdim  = banded ? bs.max_matrix_graph_dimension_banded : bs.max_matrix_graph_dimension;
    const int64_t nodes = banded ? bs.max_nodes_per_window_banded : bs.max_nodes_per_window;
    const int64_t E = gwamd::poa::kMaxEdges, A = gwamd::poa::kMaxAlignments, S = bs.max_sequences_per_poa;
    int64_t b = 0;
    b += bs.max_consensus_size;                                   // consensus
    b += !msa ? bs.max_consensus_size * 2 : 0;                    // coverage
    b += msa ? bs.max_consensus_size * S : 0;                     // msa
    b += S * bs.max_sequence_size * 2;                            // sequences + weights
    b += S * size_bytes;                                          // sequence lengths
    b += 32;                                                      // WindowDetails
    b += msa ? S * size_bytes : 0;                                // sequence_begin_nodes_ids
    b += nodes;                                                   // nodes
    b += nodes * A * size_bytes + nodes * 2;                      // node_alignments (+count)
    b += nodes * E * size_bytes + nodes * 2;                      // incoming edges (+count)
    b += nodes * E * size_bytes + nodes * 2;                      // outgoing edges (+count)
    b += nodes * E * 2 * 2;                                       // in/out edge weights
    b += nodes * size_bytes * 2 + nodes * 2;                      // sorted, node map, local count
    b += !msa ? nodes * 4 + nodes * size_bytes : 0;               // consensus scores / predecessors
    b += nodes + nodes + nodes * size_bytes;                      // marks, check, nodes_to_visit
    b += nodes * 2;                                               // node coverage
    b += msa ? nodes * E * S * 2 + nodes * E * 2 + nodes * size_bytes : 0; // edge coverage, msa pos
    b += gdim * size_bytes * 2;                                   // alignment graph/read
    return b;
}

struct DevBuf
{
    void* p = nullptr;
    size_t n = 0;
};

} // namespace

class PoaBatch : public Batch
{
public:
    PoaBatch(int32_t device_id, hipStream_t stream, size_t max_mem, int8_t output_mask, const BatchSize& bs,
             int16_t gap, int16_t mismatch, int16_t match, bool banded)
        : device_id_(detail::check_non_negative(device_id, "Device ID has to be non-negative"))
        , stream_(stream)
        , output_mask_(output_mask)
        , bs_(bs)
        , gap_(gap)
        , mismatch_(mismatch)
        , match_(match)
        , banded_(banded)
    {
        detail::check_non_negative(bs.max_sequences_per_poa, "Maximum sequences per POA has to be non-negative");
        ScopedDevice dev(device_id_);
        score_bits_ = use32bit_score(bs_, gap_, mismatch_, match_) ? 32 : 16;
        size_bits_  = (score_bits_ == 32 && use32bit_size(bs_, banded_)) ? 32 : 16;
        // batch.cu:45-73: 16-bit score implies 16-bit size
        const int sz      = size_bits_ / 8;
        const int sbytes  = score_bits_ / 8;
        const bool msa    = (output_mask_ & OutputType::msa) != 0;
        const int64_t gdim = banded_ ? bs_.max_matrix_graph_dimension_banded : bs_.max_matrix_graph_dimension;
        const int64_t ref_seq_dim = banded_ ? bs_.alignment_band_width + gwamd::poa::kBandPad : bs_.max_matrix_sequence_dimension;

        // BatchBlock ctor (allocate_block.hpp:51-91)
        const int64_t per_poa = reference_device_bytes_per_poa(bs_, banded_, msa, sz);
        if (int64_t(max_mem) < per_poa)
        {
            throw std::runtime_error(std::string("Require at least ") + std::to_string(per_poa) +
                                     " bytes of device memory per CUDAPOA batch to process correctly.");
        }
        const int64_t ref_score_matrix = ref_seq_dim * gdim * sbytes;
        int64_t max_poas               = int64_t(max_mem) / (per_poa + ref_score_matrix);

        // this build's own per-window footprint
        dims_.max_nodes     = banded_ ? bs_.max_nodes_per_window_banded : bs_.max_nodes_per_window;
        dims_.max_seqs      = bs_.max_sequences_per_poa;
        dims_.max_seq_len   = bs_.max_sequence_size;
        dims_.max_consensus = bs_.max_consensus_size;
        dims_.band_width    = bs_.alignment_band_width;
        dims_.score_stride  = banded_ ? bs_.alignment_band_width + gwamd::poa::kBandPad
                                      : int32_t(align8(int64_t(bs_.max_sequence_size) + 48));
        dims_.score_rows    = dims_.max_nodes + 2;
        dims_.aln_cap       = dims_.max_nodes + bs_.max_sequence_size + 4;
        dims_.want_consensus = (output_mask_ & OutputType::consensus) ? 1 : 0;
        // the reference's spoa_accurate build option (CMakeLists.txt:23-30) as a
        // process-wide default; gwamd_poa_set_spoa_accurate switches one batch
        if (const char* sa = std::getenv("GWAMD_SPOA_ACCURATE"))
            dims_.spoa_accurate = std::atoi(sa) != 0 ? 1 : 0;
        plan_lds_kernel();
        plan_band_kernel();
        dims_.diag = diag_bits();
        // this build's footprint: graph + inputs + outputs per window, and the
        // forward/traceback scratch per slot.  The LDS and banded kernels run
        // a persistent grid of as many workgroups as are resident at once, so
        // they need only that many slots however many windows the batch holds.
        const int64_t wbytes = window_bytes(sz, msa);
        const int64_t sbytes_slot = slot_bytes(sz, sbytes);
        int64_t own_cap = int64_t(max_mem) / (wbytes + sbytes_slot); // a slot per window
        int64_t resident = 0;
        if (dims_.lds_kernel)
        {
            int cus = 0;
            GWAMD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
            resident = int64_t(gwamd_internal_poa_blocks_per_cu(&dims_, score_bits_, size_bits_, banded_ ? 1 : 0,
                                                                msa ? 1 : 0)) * cus;
            if (const char* ev = gwamd::host::diag_env("GWAMD_POA_SLOTS")) // diagnostic: a smaller persistent grid
                if (std::atoi(ev) > 0)
                    resident = std::min<int64_t>(resident > 0 ? resident : INT32_MAX, std::atoi(ev));
            if (resident > 0 && own_cap > resident)
                own_cap = std::max(own_cap, (int64_t(max_mem) - resident * sbytes_slot) / wbytes);
        }
        max_poas = std::min<int64_t>(max_poas, own_cap);
        if (max_poas < 1)
            throw std::runtime_error("Require more device memory per CUDAPOA batch to process correctly.");
        max_poas_ = int32_t(std::min<int64_t>(max_poas, INT32_MAX));
        slots_    = resident > 0 ? int32_t(std::min<int64_t>(resident, max_poas_)) : max_poas_;
        blocks_per_cu_ = resident > 0 ? int32_t(resident) : 0;

        // score budget (allocate_block.hpp:196-201): what the reference's slab
        // leaves for the variable-width score matrices
        scorebuf_alloc_ = int64_t(max_mem) - reference_fixed_slab(sz, msa);
        if (scorebuf_alloc_ < 0)
            scorebuf_alloc_ = 0;

        allocate(sz, sbytes, msa);
        // pinned host staging for a full batch, as the reference's BatchBlock
        // allocates it up front (allocate_block.hpp:84-118), so filling a
        // batch never re-pins memory (capped; beyond the cap it grows)
        {
            const size_t cap_b = size_t(2) << 30;
            const size_t in_b  = std::min(cap_b, size_t(max_poas_) * size_t(bs_.max_sequences_per_poa) *
                                                    size_t(bs_.max_sequence_size) + 16);
            h_seqs_.reserve(in_b, stream_);
            h_wts_.reserve(in_b, stream_);
            const size_t nseq = std::min(cap_b / 8, size_t(max_poas_) * size_t(bs_.max_sequences_per_poa));
            h_len_.reserve(nseq * 4, stream_);
            h_off_.reserve(nseq * 8, stream_);
            h_win_.reserve(size_t(max_poas_) * sizeof(gwamd::poa::WindowDesc), stream_);
        }
        bid_ = batches_++;
        reset();
    }

    ~PoaBatch() override
    {
        (void)hipSetDevice(device_id_);
        for (auto* b : {&d_seqs_, &d_wts_, &d_len_, &d_off_, &d_win_, &d_slab_, &d_codes_})
            if (b->p)
                (void)hipFree(b->p);
    }

    StatusType add_poa_group(std::vector<StatusType>& per_seq_status, const Group& poa_group) override
    {
        int32_t max_len = 0;
        for (const auto& e : poa_group)
            max_len = std::max(max_len, e.length);
        if (!reserve_buf(max_len))
            return StatusType::exceeded_maximum_poas;
        per_seq_status.clear();
        StatusType st = add_poa();
        if (st != StatusType::success)
            return st;
        for (const auto& e : poa_group)
            per_seq_status.push_back(add_seq_to_poa(e.seq, e.weights, e.length));
        return StatusType::success;
    }

    int32_t get_total_poas() const override { return poa_count_; }

    void generate_poa() override
    {
        if (poa_count_ == 0)
            return;
        upload();
        launch();
    }

    void upload()
    {
        ScopedDevice dev(device_id_);
        const size_t nb = num_bases_;
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_seqs_.p, h_seqs_.as<uint8_t>(), nb + 16, hipMemcpyHostToDevice, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_wts_.p, h_wts_.as<int8_t>(), nb + 16, hipMemcpyHostToDevice, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_len_.p, h_len_.as<int32_t>(), size_t(num_seqs_) * 4, hipMemcpyHostToDevice,
                                       stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_off_.p, h_off_.as<int64_t>(), size_t(num_seqs_) * 8, hipMemcpyHostToDevice,
                                       stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_win_.p, h_win_.as<gwamd::poa::WindowDesc>(),
                                       size_t(poa_count_) * sizeof(gwamd::poa::WindowDesc), hipMemcpyHostToDevice,
                                       stream_));
        plan_launch_order();
    }

    // Queue order of the windows.  Workgroups i, i + C, i + 2C, ... (C =
    // CUs) share a CU; windows are ranked by estimated DP cells and the
    // first grid's worth is dealt to those rounds in snake order, so every CU
    // gets a mix of heavy and light windows.  When the batch holds more
    // windows than the persistent grid has slots, the rest follow heaviest
    // first and are dequeued by whichever workgroup finishes first (longest
    // processing time first).  Outputs stay indexed by window.
    void plan_launch_order()
    {
        bufs_.order = nullptr;
        bufs_.head  = nullptr;
        int cus     = 0;
        GWAMD_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
        if (const char* ev = gwamd::host::diag_env("GWAMD_LAUNCH_ORDER_CUS")) // diagnostic: plan for fewer CUs
            if (std::atoi(ev) > 0)
                cus = std::atoi(ev);
        const int n           = poa_count_;
        const bool persistent = dims_.lds_kernel != 0 && n > slots_;
        if (!persistent && (cus <= 0 || n <= cus))
            return;
        const auto* wd = h_win_.as<gwamd::poa::WindowDesc>();
        const auto* ln = h_len_.as<int32_t>();
        std::vector<std::pair<int64_t, int32_t>> cost(static_cast<size_t>(n));
        for (int w = 0; w < n; w++)
        {
            int64_t sum = 0, mx = 0;
            for (int s = 0; s < wd[w].num_seqs; s++)
            {
                const int64_t l = ln[wd[w].first_seq + s];
                mx              = std::max(mx, l);
                if (s > 0)
                    sum += l;
            }
            cost[size_t(w)] = {-sum * mx, w}; // heaviest first, ties by window
        }
        std::sort(cost.begin(), cost.end());
        // pinned, so the copy stays asynchronous (generate_poa does not block)
        h_order_.reserve(size_t(n) * 4, stream_);
        int32_t* order = h_order_.as<int32_t>();
        const int m    = persistent ? slots_ : n; // positions placed statically
        for (int k = 0; k < m; k++)
        {
            if (cus <= 0)
            {
                order[k] = cost[size_t(k)].second;
                continue;
            }
            const int t = k / cus, pos = k % cus;
            const int r = std::min(cus, m - t * cus); // workgroups in this round
            const int j = (t % 2 == 0) ? pos : r - 1 - pos;
            order[t * cus + j] = cost[size_t(k)].second;
        }
        for (int k = m; k < n; k++)
            order[k] = cost[size_t(k)].second;
        const size_t order_off = (size_t(max_poas_) * sizeof(gwamd::poa::WindowDesc) + 15) & ~size_t(15);
        int32_t* d_order       = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(d_win_.p) + order_off);
        GWAMD_HIP_CHECK(hipMemcpyAsync(d_order, order, size_t(n) * 4, hipMemcpyHostToDevice, stream_));
        bufs_.order = d_order;
        if (persistent)
            bufs_.head = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(d_win_.p) +
                                                    ((order_off + size_t(max_poas_) * 4 + 15) & ~size_t(15)));
    }

    void launch()
    {
        if (poa_count_ == 0)
            return;
        ScopedDevice dev(device_id_);
        gwamd::poa::Buffers b = bufs_;
        b.num_windows         = poa_count_;
        b.num_slots           = slots_;
        if (b.head) // the dequeue counter starts at 0 for every launch
            GWAMD_HIP_CHECK(hipMemsetAsync(b.head, 0, sizeof(int32_t), stream_));
        gwamd::poa::Scores sc{gap_, mismatch_, match_};
        const bool msa = (output_mask_ & OutputType::msa) != 0;
        if (ev_start_)
            GWAMD_HIP_CHECK(hipEventRecord(ev_start_, stream_));
        GWAMD_HIP_CHECK(gwamd_internal_poa_launch(&b, &dims_, &sc, score_bits_, size_bits_, banded_ ? 1 : 0, msa ? 1 : 0,
                                         stream_));
        if (ev_stop_)
            GWAMD_HIP_CHECK(hipEventRecord(ev_stop_, stream_));
        generated_ = true;
    }

    // instrumentation for the multi-batch driver (poa_batch_internal.hpp)
    void set_launch_events(hipEvent_t start, hipEvent_t stop)
    {
        ev_start_ = start;
        ev_stop_  = stop;
    }

    int64_t last_launch_cells()
    {
        if (poa_count_ == 0 || !generated_)
            return 0;
        std::vector<int64_t> cells(static_cast<size_t>(poa_count_));
        std::vector<int32_t> fn(static_cast<size_t>(poa_count_));
        get_stats(cells.data(), fn.data());
        int64_t s = 0;
        for (int64_t c : cells)
            s += c;
        return s;
    }

    void synchronize()
    {
        ScopedDevice dev(device_id_);
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }

    // Copies per-window outputs of the last launch to host staging.
    void fetch(bool consensus, bool msa)
    {
        ScopedDevice dev(device_id_);
        const size_t n = size_t(poa_count_);
        h_status_.resize(n);
        h_msa_status_.resize(n);
        h_len_out_.resize(n);
        h_msa_len_.resize(n);
        if (consensus)
        {
            h_cons_.resize(n * dims_.max_consensus);
            h_cov_.resize(n * dims_.max_consensus);
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_cons_.data(), bufs_.cons, n * dims_.max_consensus, hipMemcpyDeviceToHost,
                                           stream_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_cov_.data(), bufs_.cov, n * dims_.max_consensus * 2,
                                           hipMemcpyDeviceToHost, stream_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_len_out_.data(), bufs_.cons_len, n * 4, hipMemcpyDeviceToHost, stream_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_status_.data(), bufs_.status, n, hipMemcpyDeviceToHost, stream_));
        }
        if (msa)
        {
            h_msa_.resize(n * size_t(dims_.max_seqs) * dims_.max_consensus);
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_msa_.data(), bufs_.msa, h_msa_.size(), hipMemcpyDeviceToHost, stream_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_msa_len_.data(), bufs_.msa_len, n * 4, hipMemcpyDeviceToHost, stream_));
            GWAMD_HIP_CHECK(hipMemcpyAsync(h_msa_status_.data(), bufs_.msa_status, n, hipMemcpyDeviceToHost, stream_));
        }
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }

    StatusType get_consensus(std::vector<std::string>& consensus, std::vector<std::vector<uint16_t>>& coverage,
                             std::vector<StatusType>& output_status) override
    {
        if (!(output_mask_ & OutputType::consensus))
            return StatusType::output_type_unavailable;
        fetch(true, false);
        for (int32_t w = 0; w < poa_count_; w++)
        {
            const StatusType st = StatusType(h_status_[w]);
            if (!generated_ || st != StatusType::success)
            {
                output_status.push_back(generated_ ? st : StatusType::generic_error);
                consensus.emplace_back();
                coverage.emplace_back();
                continue;
            }
            output_status.push_back(StatusType::success);
            const char* c = reinterpret_cast<const char*>(&h_cons_[size_t(w) * dims_.max_consensus]);
            consensus.emplace_back(c, size_t(h_len_out_[w]));
            const uint16_t* v = &h_cov_[size_t(w) * dims_.max_consensus];
            coverage.emplace_back(v, v + h_len_out_[w]);
        }
        return StatusType::success;
    }

    StatusType get_msa(std::vector<std::vector<std::string>>& msa, std::vector<StatusType>& output_status) override
    {
        if (!(output_mask_ & OutputType::msa))
            return StatusType::output_type_unavailable;
        fetch(false, true);
        for (int32_t w = 0; w < poa_count_; w++)
        {
            msa.emplace_back();
            const StatusType st = StatusType(h_msa_status_[w]);
            if (!generated_ || st != StatusType::success)
            {
                output_status.push_back(generated_ ? st : StatusType::generic_error);
                continue;
            }
            output_status.push_back(StatusType::success);
            const int nseq = h_win_.as<gwamd::poa::WindowDesc>()[w].num_seqs;
            for (int s = 0; s < nseq; s++)
            {
                const char* row = reinterpret_cast<const char*>(
                    &h_msa_[(size_t(w) * dims_.max_seqs + s) * dims_.max_consensus]);
                msa[w].emplace_back(row, size_t(h_msa_len_[w]));
            }
        }
        return StatusType::success;
    }

    void fetch_graphs()
    {
        ScopedDevice dev(device_id_);
        const size_t n  = size_t(poa_count_);
        const size_t mn = size_t(dims_.max_nodes);
        h_g_bases_.resize(n * mn);
        h_g_in_cnt_.resize(n * mn);
        h_g_in_w_.resize(n * mn * gwamd::poa::kMaxEdges);
        h_g_in_e_raw_.resize(n * mn * gwamd::poa::kMaxEdges * (size_bits_ / 8));
        h_final_nodes_.resize(n);
        h_status_.resize(n);
        h_msa_status_.resize(n);
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_g_bases_.data(), bufs_.base, n * mn, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_g_in_cnt_.data(), bufs_.in_cnt, n * mn * 2, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_g_in_w_.data(), bufs_.in_w, h_g_in_w_.size() * 2, hipMemcpyDeviceToHost,
                                       stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_g_in_e_raw_.data(), bufs_.in_e, h_g_in_e_raw_.size(), hipMemcpyDeviceToHost,
                                       stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_final_nodes_.data(), bufs_.final_nodes, n * 4, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_status_.data(), bufs_.status, n, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(h_msa_status_.data(), bufs_.msa_status, n, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
        h_g_in_e_.resize(h_g_in_w_.size());
        if (size_bits_ == 16)
        {
            const int16_t* s = reinterpret_cast<const int16_t*>(h_g_in_e_raw_.data());
            for (size_t i = 0; i < h_g_in_e_.size(); i++)
                h_g_in_e_[i] = s[i];
        }
        else
            std::memcpy(h_g_in_e_.data(), h_g_in_e_raw_.data(), h_g_in_e_raw_.size());
    }

    // Graph status: the consensus status when consensus is produced, else MSA's.
    StatusType graph_status(int32_t w) const
    {
        if (!generated_)
            return StatusType::generic_error;
        return StatusType((output_mask_ & OutputType::consensus) ? h_status_[w] : h_msa_status_[w]);
    }

    void get_graphs(std::vector<DirectedGraph>& graphs, std::vector<StatusType>& output_status) override
    {
        fetch_graphs();
        graphs.resize(poa_count_);
        const size_t mn = size_t(dims_.max_nodes);
        for (int32_t w = 0; w < poa_count_; w++)
        {
            StatusType st = graph_status(w);
            output_status.push_back(st);
            if (st != StatusType::success)
                continue;
            DirectedGraph& g = graphs[w];
            for (int32_t v = 0; v < h_final_nodes_[w]; v++)
            {
                g.set_node_label(v, std::string(1, char(h_g_bases_[w * mn + v])));
                const int ne = h_g_in_cnt_[w * mn + v];
                for (int e = 0; e < ne; e++)
                {
                    size_t idx = (w * mn + v) * gwamd::poa::kMaxEdges + e;
                    g.add_edge(h_g_in_e_[idx], v, h_g_in_w_[idx]);
                }
            }
        }
    }

    int32_t batch_id() const override { return bid_; }

    void reset() override
    {
        poa_count_          = 0;
        num_bases_          = 0;
        num_seqs_           = 0;
        next_scores_offset_ = 0;
        avail_scorebuf_     = scorebuf_alloc_;
        generated_          = false;
    }

    // --- C ABI support ------------------------------------------------------
    int32_t score_bits() const { return score_bits_; }
    int32_t size_bits() const { return size_bits_; }
    const gwamd::poa::Dims& dims() const { return dims_; }
    const std::vector<uint8_t>& host_cons() const { return h_cons_; }
    const std::vector<uint16_t>& host_cov() const { return h_cov_; }
    const std::vector<int32_t>& host_cons_len() const { return h_len_out_; }
    const std::vector<uint8_t>& host_status() const { return h_status_; }
    const std::vector<uint8_t>& host_msa() const { return h_msa_; }
    const std::vector<int32_t>& host_msa_len() const { return h_msa_len_; }
    const std::vector<uint8_t>& host_msa_status() const { return h_msa_status_; }
    const std::vector<uint8_t>& host_g_bases() const { return h_g_bases_; }
    const std::vector<uint16_t>& host_g_in_cnt() const { return h_g_in_cnt_; }
    const std::vector<int32_t>& host_g_in_e() const { return h_g_in_e_; }
    const std::vector<uint16_t>& host_g_in_w() const { return h_g_in_w_; }
    const std::vector<int32_t>& host_final_nodes() const { return h_final_nodes_; }
    int32_t window_num_seqs(int32_t w) const { return h_win_.as<const gwamd::poa::WindowDesc>()[w].num_seqs; }
    int8_t output_mask() const { return output_mask_; }
    int64_t device_bytes() const { return int64_t(d_slab_.n + d_codes_.n + d_seqs_.n + d_wts_.n + d_len_.n + d_off_.n + d_win_.n); }
    int32_t kernel_kind() const
    {
        return dims_.lds_kernel == 3 ? (dims_.band_ad ? 4 : 3) : (dims_.lds_kernel ? 2 : 1);
    }
    int32_t max_poas() const { return max_poas_; }
    int32_t max_sequence_size() const { return bs_.max_sequence_size; }
    int32_t slots() const { return slots_; }
    int32_t resident_slots() const { return blocks_per_cu_; }
    void set_spoa_accurate(bool on) { dims_.spoa_accurate = on ? 1 : 0; }
    bool spoa_accurate() const { return dims_.spoa_accurate != 0; }

    void get_phases(int64_t* out)
    {
        ScopedDevice dev(device_id_);
        if (poa_count_ == 0)
            return;
        GWAMD_HIP_CHECK(hipMemcpyAsync(out, bufs_.phase, size_t(poa_count_) * 8 * gwamd::poa::kPhases,
                                       hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }

    void get_stats(int64_t* cells, int32_t* final_nodes)
    {
        ScopedDevice dev(device_id_);
        if (poa_count_ == 0)
            return;
        GWAMD_HIP_CHECK(hipMemcpyAsync(cells, bufs_.cells, size_t(poa_count_) * 8, hipMemcpyDeviceToHost, stream_));
        GWAMD_HIP_CHECK(hipMemcpyAsync(final_nodes, bufs_.final_nodes, size_t(poa_count_) * 4, hipMemcpyDeviceToHost,
                                       stream_));
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }

private:
    // Graph, inputs and outputs of one window.
    int64_t window_bytes(int sz, bool msa) const
    {
        const int64_t mn = dims_.max_nodes, E = gwamd::poa::kMaxEdges, S = dims_.max_seqs;
        int64_t b        = 0;
        b += align8(mn) + 4 * align8(mn * 2) + align8(mn * E * 2);   // base, counts, coverage, in_w
        b += 3 * align8(mn * E * sz) + 2 * align8(mn * sz);           // in_e, out_e, aln, sorted, pos
        b += align8(dims_.max_consensus) + align8(int64_t(dims_.max_consensus) * 2) + 32; // outputs
        b += int64_t(S) * dims_.max_seq_len * 2 + S * 12;             // inputs
        if (msa)
            b += align8(mn * E * S * 2) + align8(mn * E * 2) + align8(S * sz) +
                 align8(S * int64_t(dims_.max_consensus));
        return b;
    }

    // Forward-pass / traceback / consensus scratch of one slot.
    int64_t slot_bytes(int sz, int sbytes) const
    {
        const int64_t mn = dims_.max_nodes;
        int64_t b        = 0;
        b += 2 * align8(int64_t(dims_.aln_cap) * sz);                 // ag, ar
        b += int64_t(dims_.score_rows) * dims_.score_stride * sbytes; // scores (LDS kernel: spill rows)
        if (dims_.lds_kernel)
            b += dims_.aux_stride; // traceback codes, row program, predecessor lists, carries
        b += align8(mn * 4) + align8(mn * 4 * sz);                    // cscore, cpred
        return b;
    }

    // LDS-resident kernel (poa_window_kernel_lds): full alignment with 16-bit
    // scores and node ids.  LDS image per window: read | ring of E rows (also
    // the traceback tile and the add-alignment scratch) | row program |
    // predecessor lists | shared words; the topological sort reuses everything
    // below the shared words.  Span carries of multi-sweep reads live in HBM
    // next to the traceback codes.
    void plan_lds_kernel()
    {
        dims_.lds_kernel = 0;
        const char* env  = gwamd::host::diag_env("GWAMD_POA_KERNEL");
        if (env && std::string(env) == "v1")
            return;
        // 16-bit node ids; 16-bit scores, or 32-bit ones (the reference's
        // use32bitScore batches: nw_forward_lds_w)
        if (banded_ || size_bits_ != 16 || (score_bits_ != 16 && score_bits_ != 32))
            return;
        const bool wide      = score_bits_ == 32;
        auto a16             = [](int64_t v) { return (v + 15) & ~int64_t(15); };
        int ring_rows        = 8;
        const int64_t read_b = a16(int64_t(dims_.max_seq_len) + 48);
        // forward pass shape: CPL columns per lane on NW waves; a sweep covers
        // NW*64*CPL read columns, longer reads take several sweeps
        // (GWAMD_POA_LDS_SHAPE="cpl,waves").  32-bit scores: one sweep up to
        // 4,096 columns (8 waves), 8,192 with 16 columns per lane
        int cpl = 8, nw = 1;
        const int ms = dims_.max_seq_len;
        if (!wide && ms > 512)
            nw = 2;
        if (wide)
        {
            nw  = ms <= 512 ? 1 : (ms <= 1024 ? 2 : (ms <= 2048 ? 4 : 8));
            cpl = ms <= 4096 ? 8 : 16;
        }
        if (const char* sh = gwamd::host::diag_env("GWAMD_POA_LDS_SHAPE"))
        {
            int c = 0, n = 0;
            if (std::sscanf(sh, "%d,%d", &c, &n) == 2)
            {
                const bool known =
                    wide ? ((c == 8 && (n == 1 || n == 2 || n == 4 || n == 8)) || (c == 16 && n == 8))
                         : ((n == 1 && (c == 8 || c == 16 || c == 24 || c == 32)) || (c == 8 && n >= 2 && n <= 4) ||
                            (c == 16 && n == 4) || (c == 4 && n == 4));
                if (!known)
                    throw std::invalid_argument("GWAMD_POA_LDS_SHAPE: unsupported columns/waves pair");
                cpl = c, nw = n;
            }
        }
        const int ebytes     = wide ? 4 : 2;
        const int64_t add_b  = 5 * a16(dims_.max_seq_len + 16) + 2 * (int64_t(dims_.max_nodes) + dims_.max_seq_len);
        const int64_t tile_b = int64_t(gwamd::poa::kTileRows) * gwamd::poa::kTileCols + gwamd::poa::kTbRankBytes;
        const int64_t rec_b  = a16(int64_t(dims_.max_nodes + 2) * 4);
        const int64_t sh_b   = a16(wide ? gwamd::poa::kShBytesW(nw) : gwamd::poa::kShBytes(nw));
        auto ring_bytes      = [&](int rows) {
            return a16(std::max<int64_t>({int64_t(rows) * dims_.score_stride * ebytes, tile_b, add_b}));
        };
        int64_t ring_b       = ring_bytes(ring_rows);
        int64_t fixed        = read_b + ring_b + rec_b + sh_b;
        int64_t target       = 40960 - 16; // 4 workgroups per CU incl. static LDS: one batch of
                                           // 1024 windows is resident on the 256 CUs at once
        if (wide)
        {
            // 32-bit rows are twice as wide: two windows per CU when their
            // images fit, else one; an 8-row ring when it fits, else 4 rows
            // (predecessors farther back go through the HBM spill rows)
            int64_t chosen = 0;
            for (int64_t budget : {int64_t(81920 - 16), int64_t(163840 - 64)})
            {
                for (int rows : {8, 4})
                {
                    const int64_t rb = ring_bytes(rows);
                    const int64_t fx = read_b + rb + rec_b + sh_b;
                    if (fx + 2048 <= budget)
                    {
                        ring_rows = rows, ring_b = rb, fixed = fx, chosen = budget;
                        break;
                    }
                }
                if (chosen)
                    break;
            }
            if (!chosen)
                return;
            target = chosen;
        }
        int64_t xl_cap       = std::max<int64_t>(1024, (target - fixed) / 2);
        xl_cap               = std::min<int64_t>(xl_cap, 65535);
        int64_t total        = fixed + a16(xl_cap * 2);
        if (const char* pad = gwamd::host::diag_env("GWAMD_POA_LDS_PAD")) // diagnostic: fewer windows per CU
            total += a16(std::atoi(pad));
        if (total > (wide ? 163840 - 64 : 65536))
            return;
        dims_.lds_kernel    = 1;
        dims_.tb_rank       = tb_rank_default();
        dims_.lds_ring_off  = int32_t(read_b);
        dims_.lds_ring_rows = ring_rows;
        dims_.lds_rec_off   = int32_t(read_b + ring_b);
        dims_.lds_xl_off    = int32_t(read_b + ring_b + rec_b);
        dims_.lds_xl_cap    = int32_t(xl_cap);
        dims_.lds_sh_off    = int32_t(read_b + ring_b + rec_b + a16(xl_cap * 2));
        dims_.lds_bytes     = int32_t(total);
        dims_.lds_cpl       = cpl;
        dims_.lds_waves     = nw;
        dims_.code_stride   = int32_t(a16(int64_t(dims_.max_seq_len) + 48));
        // HBM side buffer per window: traceback codes, span carries
        const int64_t code_b = int64_t(dims_.score_rows) * dims_.code_stride;
        const int64_t cr_b   = a16(int64_t(dims_.max_nodes + 2) * ebytes);
        dims_.aux_carry_off  = int32_t(code_b);
        dims_.aux_stride     = code_b + cr_b;
    }

    // Banded kernel (poa_window_kernel_band, poa_band.hip): band widths 128 to
    // 1,024 in steps of 128 (2 to 16 cells per lane), gap <= 0.  LDS image per window: staged
    // read | work region (row-program flags, the 16-row ring of band rows, the
    // traceback tile, the add-alignment scratch; the topological sort also
    // reuses the read) | shared words.  Windows per CU: 4, 2 or 1, the most
    // that leave room for the work region at this batch's maximum sizes.
    // traceback move windows (TbWin, poa_wave.hpp): bit 0 walks them by
    // pointer doubling (else the scalar walk), bit 1 shapes them as strips
    // along the path (else 16 x 8 rectangles), bit 2 makes the strips 32
    // columns x 4 rows (else 16 x 8).  Default: pointer doubling over 16 x 8
    // strips; GWAMD_TB_WALK=scalar | rect | scalar_rect | strip32 |
    // scalar_strip32 for parity tests and A/B runs.
public:
    static int tb_rank_default()
    {
        // GWAMD_TB_ABOVE=k (0-6): strip rows above the slope line (A/B runs;
        // default 3)
        int above_bits = 0;
        if (const char* ab = gwamd::host::diag_env("GWAMD_TB_ABOVE"))
            above_bits = (std::min(std::max(std::atoi(ab), 0), 6) + 1) << 3;
        return tb_walk_bits() | above_bits;
    }
    // Dims::diag: bit 0 forces the Kahn sort's ring of queued words
    // (GWAMD_TOPSORT_RING=1, ring-mode parity tests); bit 1 keeps the LDS
    // kernel on the round-3 forward pass (GWAMD_POA_FWD=v1, A/B runs); bit 2
    // keeps the LDS and banded kernels on the FIFO Kahn sort instead of the
    // level-keyed one (GWAMD_TOPSORT=fifo, cross-check tests and A/B runs);
    // bit 3 keeps the MSA's racon sort on the round-5 DFS step (GWAMD_RACON=v1)
    static int diag_bits()
    {
        const char* r = gwamd::host::diag_env("GWAMD_TOPSORT_RING");
        const char* f = gwamd::host::diag_env("GWAMD_POA_FWD");
        const char* t = gwamd::host::diag_env("GWAMD_TOPSORT");
        const char* d = gwamd::host::diag_env("GWAMD_RACON");
        return ((r && std::atoi(r) != 0) ? 1 : 0) | ((f && std::string(f) == "v1") ? 2 : 0) |
               ((t && std::string(t) == "fifo") ? 4 : 0) | ((d && std::string(d) == "v1") ? 8 : 0);
    }
    static int tb_walk_bits()
    {
        const char* ev = gwamd::host::diag_env("GWAMD_TB_WALK");
        const std::string v = ev ? ev : "";
        if (v == "scalar")
            return 2;
        if (v == "rect")
            return 1;
        if (v == "scalar_rect")
            return 0;
        if (v == "strip32")
            return 7;
        if (v == "scalar_strip32")
            return 6;
        return 3;
    }

private:
    void plan_band_kernel()
    {
        if (!banded_ || dims_.lds_kernel)
            return;
        const char* env = gwamd::host::diag_env("GWAMD_POA_KERNEL");
        if (env && std::string(env) == "v1")
            return;
        const int bw = dims_.band_width;
        // every band width the reference accepts up to 1,024 (multiples of
        // 128, batch.hpp:85-94): CPL = bw / 64 cells per lane, one translation
        // unit per CPL (poa_band_c<CPL>.hip)
        if (bw % 128 != 0 || bw < 128 || bw > 1024 || gap_ > 0)
            return;
        auto a16          = [](int64_t v) { return (v + 15) & ~int64_t(15); };
        const int cpl     = bw / 64;
        const int sbytes  = score_bits_ / 8;
        // band row: position idx + cpl - 1, whole cpl-cell groups (66-67 of them)
        const int rowsz   = (bw + gwamd::poa::kBandPad + cpl + cpl - 1) / cpl * cpl;
        const int64_t ms  = dims_.max_seq_len, mn = dims_.max_nodes;
        const int64_t read_b  = a16(gwamd::poa::kReadGuard + ms + bw + 48);
        const int64_t sh_b    = 64;
        const int ring_rows   = gwamd::poa::band_ring_rows(cpl), tile_rows = gwamd::poa::band_tile_rows(cpl);
        const int64_t ring_b  = a16(int64_t(ring_rows) * rowsz * sbytes) + 4 * 256 * 4 + 1024 * 4; // + record staging
        const int64_t tile_b  = a16(int64_t(tile_rows) * bw + 64 * 16 + 512 + gwamd::poa::kTbRankBytes); // codes +
                                                                      // per-row decode info + walk tables
        const int64_t flags_b = 2 * a16(mn + 2); // row program: spill and far flags
        const int64_t add_b   = 7 * a16(ms + 16) + a16(2 * (mn + ms + 16)); // + the edge-slot bytes
        // anti-diagonal forward pass (poa_band_ad.hpp): a kAdRing-row ring and
        // one dummy word per lane.  Default: whenever the windows-per-CU
        // choice below leaves room for it (large windows, one or two per CU);
        // GWAMD_BAND_FWD=ad|row forces it on (planning for it) or off.
        const int64_t ad_b    = a16(int64_t(gwamd::poa::kAdRing) * rowsz * sbytes + gwamd::poa::kWave * sbytes) +
                             a16(mn / 8 + 64); // + the real-row bitmap
        const char* fwd_env   = gwamd::host::diag_env("GWAMD_BAND_FWD");
        // (band widths 128 / 256 only: its ring of kAdRing rows is too large beyond)
        const bool force_ad   = fwd_env && std::string(fwd_env) == "ad" && cpl <= 4;
        const bool no_ad      = fwd_env && std::string(fwd_env) == "row";
        const int64_t min_w   = std::max({ring_b, tile_b, flags_b, force_ad ? ad_b : int64_t(0)});
        const int64_t want_w  = std::max(min_w, add_b);
        const int64_t kStatic = 256; // static __shared__ bytes of the kernel
        int64_t total         = 0;
        int chosen_per_cu     = 1;
        for (int per_cu : {4, 2, 1})
        {
            const int64_t budget = (163840 / per_cu - kStatic) & ~int64_t(15);
            if ((!force_ad && read_b + want_w + sh_b <= budget) || per_cu == 1)
            {
                total         = budget;
                chosen_per_cu = per_cu;
                break;
            }
        }
        const int64_t work = total - read_b - sh_b;
        if (work < min_w)
            return;
        dims_.lds_kernel     = 3;
        // the pass runs kAdMaxWaves waves per window: one window per CU
        int ad_waves = gwamd::poa::kAdMaxWaves;
        if (const char* ev = gwamd::host::diag_env("GWAMD_BAND_AD_WAVES")) // diagnostic: fewer waves per window
            ad_waves = std::max(1, std::min(gwamd::poa::kAdMaxWaves, std::atoi(ev)));
        dims_.band_ad        = (!no_ad && cpl <= 4 && chosen_per_cu == 1 && work >= ad_b) ? ad_waves : 0;
        dims_.tb_rank        = tb_rank_default();
        dims_.lds_cpl        = cpl;
        dims_.lds_waves      = 1;
        dims_.lds_bytes      = int32_t(total);
        dims_.lds_ring_off   = int32_t(read_b);
        dims_.lds_ring_rows  = ring_rows;
        dims_.lds_work_bytes = int32_t(work);
        dims_.lds_sh_off     = int32_t(read_b + work);
        dims_.score_stride   = rowsz; // spill rows: band row at position idx + cpl - 1
        dims_.code_stride    = bw;
        const int64_t rows   = dims_.score_rows;
        int64_t o            = a16(rows * bw); // codes
        dims_.aux_reca_off   = int32_t(o);
        o += a16(rows * 4);
        dims_.aux_recb_off = int32_t(o);
        o += a16(rows * 4);
        dims_.aux_col0_off = int32_t(o);
        o += a16(rows * 4);
        dims_.aux_flag_off = int32_t(o);
        o += a16(rows);
        dims_.aux_xl_off = int32_t(o);
        dims_.aux_xl_cap = int32_t(2 * mn + 64);
        o += a16(int64_t(dims_.aux_xl_cap) * 4);
        dims_.aux_bx_off = int32_t(o);
        o += a16((rows / 256 + 2) * 4);
        dims_.aux_recc_off = int32_t(o);
        o += a16(rows * 4);
        dims_.aux_rece_off = int32_t(o);
        o += a16(rows * 4);
        dims_.aux_stride = o;
    }

    // Non-score bytes of the reference slab for max_poas windows
    // (allocate_block.hpp:121-285, each buffer aligned to 8 B).
    int64_t reference_fixed_slab(int sz, bool msa) const
    {
        const int64_t P = max_poas_, S = bs_.max_sequences_per_poa, E = gwamd::poa::kMaxEdges;
        const int64_t nodes = banded_ ? bs_.max_nodes_per_window_banded : bs_.max_nodes_per_window;
        const int64_t gdim  = banded_ ? bs_.max_matrix_graph_dimension_banded : bs_.max_matrix_graph_dimension;
        const bool cons     = (output_mask_ & OutputType::consensus) != 0;
        int64_t o           = 0;
        o += align8(P * bs_.max_consensus_size);
        o += cons ? align8(P * bs_.max_consensus_size * 2) : 0;
        o += msa ? align8(P * bs_.max_consensus_size * S) : 0;
        o += 2 * align8(P * S * bs_.max_sequence_size);
        o += align8(P * S * sz) + align8(P * 32);
        o += msa ? align8(P * S * sz) : 0;
        o += 2 * align8(P * gdim * sz); // alignment graph / read
        o += align8(P * nodes) + align8(P * nodes * E * sz) + align8(P * nodes * 2);
        o += align8(P * nodes * E * sz) + align8(P * nodes * 2);
        o += align8(P * nodes * E * sz) + align8(P * nodes * 2);
        o += 2 * align8(P * nodes * E * 2);
        o += 2 * align8(P * nodes * sz) + align8(P * nodes * 2);
        o += cons ? align8(P * nodes * 4) + align8(P * nodes * sz) : 0;
        o += 2 * align8(P * nodes) + align8(P * nodes * sz) + align8(P * nodes * 2);
        o += msa ? align8(P * nodes * E * S * 2) + align8(P * nodes * E * 2) + align8(P * nodes * sz) : 0;
        return o;
    }

    void allocate(int sz, int sbytes, bool msa)
    {
        const int64_t P = max_poas_, mn = dims_.max_nodes, E = gwamd::poa::kMaxEdges, S = dims_.max_seqs;
        const int64_t Z = slots_; // scratch slots
        struct Item
        {
            void** dst;
            int64_t bytes;
        };
        void* dummy = nullptr;
        std::vector<Item> items = {
            {reinterpret_cast<void**>(&bufs_.base), align8(P * mn)},
            {reinterpret_cast<void**>(&bufs_.in_cnt), align8(P * mn * 2)},
            {reinterpret_cast<void**>(&bufs_.out_cnt), align8(P * mn * 2)},
            {reinterpret_cast<void**>(&bufs_.aln_cnt), align8(P * mn * 2)},
            {reinterpret_cast<void**>(&bufs_.node_cov), align8(P * mn * 2)},
            {reinterpret_cast<void**>(&bufs_.in_w), align8(P * mn * E * 2)},
            {&bufs_.in_e, align8(P * mn * E * sz)},
            {&bufs_.out_e, align8(P * mn * E * sz)},
            {&bufs_.aln, align8(P * mn * E * sz)},
            {&bufs_.sorted, align8(P * mn * sz)},
            {&bufs_.pos, align8(P * mn * sz)},
            {&bufs_.ag, align8(Z * dims_.aln_cap * sz)},
            {&bufs_.ar, align8(Z * dims_.aln_cap * sz)},
            {reinterpret_cast<void**>(&bufs_.cscore), align8(Z * mn * 4)},
            {&bufs_.cpred, align8(Z * mn * 4 * sz)},
            {reinterpret_cast<void**>(&bufs_.cons), align8(P * dims_.max_consensus)},
            {reinterpret_cast<void**>(&bufs_.cov), align8(P * dims_.max_consensus * 2)},
            {reinterpret_cast<void**>(&bufs_.cons_len), align8(P * 4)},
            {reinterpret_cast<void**>(&bufs_.status), align8(P)},
            {reinterpret_cast<void**>(&bufs_.msa_status), align8(P)},
            {reinterpret_cast<void**>(&bufs_.msa_len), align8(P * 4)},
            {reinterpret_cast<void**>(&bufs_.final_nodes), align8(P * 4)},
            {reinterpret_cast<void**>(&bufs_.cells), align8(P * 8)},
            {reinterpret_cast<void**>(&bufs_.phase), align8(P * 8 * gwamd::poa::kPhases)},
            {msa ? reinterpret_cast<void**>(&bufs_.edge_cov) : &dummy, msa ? align8(P * mn * E * S * 2) : 0},
            {msa ? reinterpret_cast<void**>(&bufs_.edge_cov_cnt) : &dummy, msa ? align8(P * mn * E * 2) : 0},
            {msa ? &bufs_.seq_begin : &dummy, msa ? align8(P * S * sz) : 0},
            {msa ? reinterpret_cast<void**>(&bufs_.msa) : &dummy, msa ? align8(P * S * dims_.max_consensus) : 0},
        };
        // the score matrices go last, 256-B aligned
        int64_t off = 0;
        for (auto& it : items)
            off += it.bytes;
        off                   = (off + 255) & ~int64_t(255);
        const int64_t sc_off  = off;
        const int64_t sc_size = Z * int64_t(dims_.score_rows) * dims_.score_stride * sbytes;
        d_slab_.n             = size_t(off + sc_size);
        GWAMD_HIP_CHECK(hipMalloc(&d_slab_.p, d_slab_.n));
        uint8_t* base = static_cast<uint8_t*>(d_slab_.p);
        int64_t cur   = 0;
        for (auto& it : items)
        {
            if (it.bytes > 0)
                *it.dst = base + cur;
            cur += it.bytes;
        }
        bufs_.scores = base + sc_off;
        if (dims_.lds_kernel)
        {
            const size_t code_bytes = size_t(Z) * size_t(dims_.aux_stride);
            GWAMD_HIP_CHECK(hipMalloc(&d_codes_.p, code_bytes));
            d_codes_.n   = code_bytes;
            bufs_.codes = static_cast<uint8_t*>(d_codes_.p);
        }
        // inputs (allocate_block.hpp:84: max_poas * max_seqs * max_seq bytes)
        const int64_t in_bytes = P * S * dims_.max_seq_len + 64;
        d_seqs_.n              = size_t(in_bytes);
        d_wts_.n               = size_t(in_bytes);
        d_len_.n               = size_t(P * S * 4 + 8);
        d_off_.n               = size_t(P * S * 8 + 8);
        d_win_.n               = size_t(P * (sizeof(gwamd::poa::WindowDesc) + 4) + 64); // + order, dequeue head
        for (auto* b : {&d_seqs_, &d_wts_, &d_len_, &d_off_, &d_win_})
            GWAMD_HIP_CHECK(hipMalloc(&b->p, b->n));
        bufs_.seqs    = static_cast<const uint8_t*>(d_seqs_.p);
        bufs_.wts     = static_cast<const int8_t*>(d_wts_.p);
        bufs_.seq_len = static_cast<const int32_t*>(d_len_.p);
        bufs_.seq_off = static_cast<const int64_t*>(d_off_.p);
        bufs_.windows = static_cast<const gwamd::poa::WindowDesc*>(d_win_.p);
        // status defaults so that reading before generate is defined
        GWAMD_HIP_CHECK(hipMemsetAsync(bufs_.status, int(StatusType::generic_error), size_t(P), stream_));
        GWAMD_HIP_CHECK(hipMemsetAsync(bufs_.msa_status, int(StatusType::generic_error), size_t(P), stream_));
        GWAMD_HIP_CHECK(hipStreamSynchronize(stream_));
    }

    // cudapoa_batch.cuh:542-564
    bool reserve_buf(int32_t max_seq_length)
    {
        const int64_t gdim  = banded_ ? bs_.max_matrix_graph_dimension_banded : bs_.max_matrix_graph_dimension;
        const int64_t width = banded_ ? bs_.alignment_band_width + gwamd::poa::kBandPad
                                      : detail::align_up(max_seq_length + 1 + 4, 4);
        const int64_t need  = width * gdim * (score_bits_ / 8);
        if (need > avail_scorebuf_)
        {
            if (poa_count_ == 0)
            {
                std::cout << "Memory available " << std::fixed << std::setprecision(2)
                          << double(avail_scorebuf_) / 1024. / 1024. / 1024.;
                std::cout << "GB, Memory required " << double(need) / 1024. / 1024. / 1024.;
                std::cout << "GB (sequence length " << max_seq_length << ", graph length " << gdim << ")" << std::endl;
            }
            return false;
        }
        avail_scorebuf_ -= need;
        return true;
    }

    // cudapoa_batch.cuh:471-487
    StatusType add_poa()
    {
        if (poa_count_ == max_poas_)
            return StatusType::exceeded_maximum_poas;
        h_win_.reserve(size_t(poa_count_ + 1) * sizeof(gwamd::poa::WindowDesc), stream_);
        gwamd::poa::WindowDesc& wd = h_win_.as<gwamd::poa::WindowDesc>()[poa_count_];
        wd.first_seq               = num_seqs_;
        wd.num_seqs                = 0;
        h_win_.used_               = size_t(poa_count_ + 1) * sizeof(gwamd::poa::WindowDesc);
        poa_count_++;
        generated_ = false;
        return StatusType::success;
    }

    // cudapoa_batch.cuh:490-539
    StatusType add_seq_to_poa(const char* seq, const int8_t* weights, int32_t seq_len)
    {
        if (seq_len > bs_.max_sequence_size)
            return StatusType::exceeded_maximum_sequence_size;
        gwamd::poa::WindowDesc& wd = h_win_.as<gwamd::poa::WindowDesc>()[poa_count_ - 1];
        if (wd.num_seqs >= bs_.max_sequences_per_poa)
            return StatusType::exceeded_maximum_sequences_per_poa;
        if (weights != nullptr)
            for (int32_t i = 0; i < seq_len; i++)
                detail::check_non_negative(weights[i], "Base weights need to be non-negative");
        wd.num_seqs++;
        const size_t need = num_bases_ + size_t(seq_len) + 16;
        h_seqs_.reserve(need, stream_);
        h_wts_.reserve(need, stream_);
        if (seq_len > 0)
            std::memcpy(h_seqs_.as<uint8_t>() + num_bases_, seq, size_t(seq_len));
        if (weights == nullptr)
            std::memset(h_wts_.as<int8_t>() + num_bases_, 1, size_t(seq_len));
        else if (seq_len > 0)
            std::memcpy(h_wts_.as<int8_t>() + num_bases_, weights, size_t(seq_len));
        std::memset(h_seqs_.as<uint8_t>() + num_bases_ + seq_len, 0, 16);
        std::memset(h_wts_.as<int8_t>() + num_bases_ + seq_len, 0, 16);
        h_len_.reserve(size_t(num_seqs_ + 1) * 4, stream_);
        h_off_.reserve(size_t(num_seqs_ + 1) * 8, stream_);
        h_len_.as<int32_t>()[num_seqs_] = seq_len;
        h_off_.as<int64_t>()[num_seqs_] = int64_t(num_bases_);
        num_bases_ += size_t(seq_len);
        h_seqs_.used_ = h_wts_.used_ = num_bases_ + 16;
        num_seqs_++;
        h_len_.used_ = size_t(num_seqs_) * 4;
        h_off_.used_ = size_t(num_seqs_) * 8;
        return StatusType::success;
    }

    int32_t device_id_;
    hipStream_t stream_;
    int8_t output_mask_;
    BatchSize bs_;
    int16_t gap_, mismatch_, match_;
    bool banded_;
    int32_t score_bits_ = 16, size_bits_ = 16;
    int32_t max_poas_   = 0;
    int32_t slots_      = 0; // scratch slots (persistent grid size for the LDS / banded kernels)
    int32_t blocks_per_cu_ = 0; // resident workgroups on the device (0: v1 kernel)
    int64_t scorebuf_alloc_ = 0, avail_scorebuf_ = 0, next_scores_offset_ = 0;
    int32_t poa_count_  = 0;
    int32_t num_seqs_   = 0;
    size_t num_bases_   = 0;
    bool generated_     = false;
    int32_t bid_        = 0;
    hipEvent_t ev_start_ = nullptr, ev_stop_ = nullptr; // set_launch_events (multi-batch driver)
    gwamd::poa::Dims dims_{};
    PinnedBuf h_order_; // workgroup -> window (plan_launch_order)
    gwamd::poa::Buffers bufs_{};
    DevBuf d_seqs_, d_wts_, d_len_, d_off_, d_win_, d_slab_, d_codes_;
    PinnedBuf h_seqs_, h_wts_, h_len_, h_off_, h_win_;
    std::vector<uint8_t> h_cons_, h_status_, h_msa_, h_msa_status_, h_g_bases_, h_g_in_e_raw_;
    std::vector<uint16_t> h_cov_, h_g_in_cnt_, h_g_in_w_;
    std::vector<int32_t> h_len_out_, h_msa_len_, h_g_in_e_, h_final_nodes_;
    static int32_t batches_; // batch id counter (cudapoa_batch.cuh:631-635)
};

int32_t PoaBatch::batches_ = 0;

StatusType Init()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return StatusType::generic_error;
    return StatusType::success;
}

// BatchBlock::estimate_max_poas (allocate_block.hpp:364-401)
int64_t estimate_max_poas(const BatchSize& batch_size, bool banded_alignment, bool msa_flag,
                          size_t free_device_memory, float memory_usage_quota, int32_t mismatch_score,
                          int32_t gap_score, int32_t match_score)
{
    const size_t mem_per_batch = size_t(memory_usage_quota * double(free_device_memory));
    int64_t sizeof_score       = 2;
    int64_t per_poa            = 0;
    if (use32bit_score(batch_size, int16_t(gap_score), int16_t(mismatch_score), int16_t(match_score)))
    {
        sizeof_score = 4;
        per_poa      = reference_device_bytes_per_poa(batch_size, banded_alignment, msa_flag,
                                                 use32bit_size(batch_size, banded_alignment) ? 4 : 2);
    }
    else
        per_poa = reference_device_bytes_per_poa(batch_size, banded_alignment, msa_flag, 2);
    const int64_t seq_dim = banded_alignment ? batch_size.alignment_band_width + gwamd::poa::kBandPad
                                             : batch_size.max_matrix_sequence_dimension;
    const int64_t graph_dim = banded_alignment ? batch_size.max_matrix_graph_dimension_banded
                                               : batch_size.max_matrix_graph_dimension;
    return int64_t(mem_per_batch) / (per_poa + seq_dim * graph_dim * sizeof_score);
}

// get_multi_batch_sizes (utils.cu:24-138): groups are binned by their batch
// capacity (bins 1, 2, 4, ... 2^19 unless given), each non-empty bin becomes
// one BatchSize sized by its largest group (max read length x reads), and the
// following bins are merged into it while their group count fits its capacity.
void get_multi_batch_sizes_for_memory(std::vector<BatchSize>& list_of_batch_sizes,
                                      std::vector<std::vector<int32_t>>& list_of_groups_per_batch,
                                      const std::vector<Group>& poa_groups, size_t free_device_memory,
                                      bool banded_alignment, bool msa_flag, int32_t band_width,
                                      std::vector<int32_t>* bins_capacity, float gpu_memory_usage_quota,
                                      int32_t mismatch_score, int32_t gap_score, int32_t match_score)
{
    const int32_t num_groups = int32_t(poa_groups.size());
    std::vector<int64_t> max_poas(num_groups);
    std::vector<int32_t> max_lengths(num_groups);
    for (int32_t i = 0; i < num_groups; i++)
    {
        int32_t max_read_length = 0;
        for (const auto& e : poa_groups[i])
            max_read_length = std::max(max_read_length, e.length);
        max_poas[i] = estimate_max_poas(BatchSize(max_read_length, int32_t(poa_groups[i].size()), band_width),
                                        banded_alignment, msa_flag, free_device_memory, gpu_memory_usage_quota,
                                        mismatch_score, gap_score, match_score);
        max_lengths[i] = max_read_length;
    }
    std::vector<int32_t> default_bins(20, 1);
    for (size_t j = 1; j < default_bins.size(); j++)
        default_bins[j] = default_bins[j - 1] * 2;
    const std::vector<int32_t>& bins = bins_capacity ? *bins_capacity : default_bins;
    const int32_t num_bins           = int32_t(bins.size());
    std::vector<int32_t> freq(num_bins, 0), bin_len(num_bins, 0), bin_reads(num_bins, 0);
    std::vector<std::vector<int32_t>> bin_groups(num_bins);
    for (int32_t i = 0; i < num_groups; i++)
    {
        const int32_t current = max_lengths[i] * int32_t(poa_groups[i].size());
        for (int32_t j = 0; j < num_bins; j++)
        {
            if (max_poas[i] <= bins[j] || j == num_bins - 1)
            {
                freq[j]++;
                bin_groups[j].push_back(i);
                if (bin_len[j] * bin_reads[j] < current)
                {
                    bin_len[j]   = max_lengths[i];
                    bin_reads[j] = int32_t(poa_groups[i].size());
                }
                break;
            }
        }
    }
    for (int32_t j = 0; j < num_bins; j++)
    {
        if (freq[j] == 0)
            continue;
        list_of_batch_sizes.emplace_back(bin_len[j], bin_reads[j], band_width);
        list_of_groups_per_batch.push_back(bin_groups[j]);
        for (int32_t k = j + 1; k < num_bins; k++)
        {
            if (freq[k] == 0)
                continue;
            if (bins[j] >= freq[k])
            {
                auto& cur = list_of_groups_per_batch.back();
                cur.insert(cur.end(), bin_groups[k].begin(), bin_groups[k].end());
                freq[k] = 0;
            }
            else
                break;
        }
    }
}

void get_multi_batch_sizes(std::vector<BatchSize>& list_of_batch_sizes,
                           std::vector<std::vector<int32_t>>& list_of_groups_per_batch,
                           const std::vector<Group>& poa_groups, bool banded_alignment, bool msa_flag,
                           int32_t band_width, std::vector<int32_t>* bins_capacity, float gpu_memory_usage_quota,
                           int32_t mismatch_score, int32_t gap_score, int32_t match_score)
{
    size_t free_mem = 0, total = 0;
    if (hipMemGetInfo(&free_mem, &total) != hipSuccess)
        throw std::runtime_error("get_multi_batch_sizes: hipMemGetInfo failed");
    get_multi_batch_sizes_for_memory(list_of_batch_sizes, list_of_groups_per_batch, poa_groups, free_mem,
                                     banded_alignment, msa_flag, band_width, bins_capacity, gpu_memory_usage_quota,
                                     mismatch_score, gap_score, match_score);
}

std::unique_ptr<Batch> create_batch(int32_t device_id, hipStream_t stream, size_t max_mem, int8_t output_mask,
                                    const BatchSize& batch_size, int16_t gap_score, int16_t mismatch_score,
                                    int16_t match_score, bool cuda_banded_alignment)
{
    detail::check_non_negative(batch_size.max_sequences_per_poa, "Maximum sequences per POA has to be non-negative");
    return std::unique_ptr<Batch>(new PoaBatch(device_id, stream, max_mem, output_mask, batch_size, gap_score,
                                               mismatch_score, match_score, cuda_banded_alignment));
}

namespace detail
{
void set_launch_events(Batch* batch, hipEvent_t start, hipEvent_t stop)
{
    static_cast<PoaBatch*>(batch)->set_launch_events(start, stop);
}

int64_t last_launch_cells(Batch* batch) { return static_cast<PoaBatch*>(batch)->last_launch_cells(); }

int32_t max_sequence_size(const Batch* batch) { return static_cast<const PoaBatch*>(batch)->max_sequence_size(); }
} // namespace detail

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks

// ===========================================================================
// C ABI (include/gwamd_cudapoa.h)
// ===========================================================================
namespace cp = claraparabricks::genomeworks::cudapoa;

namespace
{

template <typename F>
int32_t guarded(F&& f)
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

void to_c(const cp::BatchSize& b, gwamd_poa_batch_size* o)
{
    o->max_sequence_size                 = b.max_sequence_size;
    o->max_consensus_size                = b.max_consensus_size;
    o->max_nodes_per_window              = b.max_nodes_per_window;
    o->max_nodes_per_window_banded       = b.max_nodes_per_window_banded;
    o->max_matrix_graph_dimension        = b.max_matrix_graph_dimension;
    o->max_matrix_graph_dimension_banded = b.max_matrix_graph_dimension_banded;
    o->max_matrix_sequence_dimension     = b.max_matrix_sequence_dimension;
    o->alignment_band_width              = b.alignment_band_width;
    o->max_sequences_per_poa             = b.max_sequences_per_poa;
}

cp::BatchSize from_c(const gwamd_poa_batch_size* i)
{
    cp::BatchSize b;
    b.max_sequence_size                 = i->max_sequence_size;
    b.max_consensus_size                = i->max_consensus_size;
    b.max_nodes_per_window              = i->max_nodes_per_window;
    b.max_nodes_per_window_banded       = i->max_nodes_per_window_banded;
    b.max_matrix_graph_dimension        = i->max_matrix_graph_dimension;
    b.max_matrix_graph_dimension_banded = i->max_matrix_graph_dimension_banded;
    b.max_matrix_sequence_dimension     = i->max_matrix_sequence_dimension;
    b.alignment_band_width              = i->alignment_band_width;
    b.max_sequences_per_poa             = i->max_sequences_per_poa;
    return b;
}
} // namespace

struct gwamd_poa_batch
{
    std::unique_ptr<cp::PoaBatch> impl;
};

extern "C" {

const char* gwamd_last_error(void) { return gwamd::host::last_error().c_str(); }

int32_t gwamd_poa_batch_size_init(gwamd_poa_batch_size* out, int32_t max_seq_sz, int32_t max_seq_per_poa,
                                  int32_t band_width)
{
    return guarded([&] {
        to_c(cp::BatchSize(max_seq_sz, max_seq_per_poa, band_width), out);
        return 0;
    });
}

int32_t gwamd_poa_batch_size_init_full(gwamd_poa_batch_size* out, int32_t max_seq_sz, int32_t max_consensus_sz,
                                       int32_t max_nodes_per_w, int32_t max_nodes_per_w_banded, int32_t band_width,
                                       int32_t max_seq_per_poa)
{
    return guarded([&] {
        to_c(cp::BatchSize(max_seq_sz, max_consensus_sz, max_nodes_per_w, max_nodes_per_w_banded, band_width,
                           max_seq_per_poa),
             out);
        return 0;
    });
}

int32_t gwamd_poa_create_batch(gwamd_poa_batch** out, int32_t device_id, void* stream, size_t max_mem,
                               int8_t output_mask, const gwamd_poa_batch_size* batch_size, int16_t gap_score,
                               int16_t mismatch_score, int16_t match_score, int32_t cuda_banded_alignment)
{
    *out = nullptr;
    return guarded([&] {
        auto* h = new gwamd_poa_batch;
        try
        {
            h->impl.reset(new cp::PoaBatch(device_id, static_cast<hipStream_t>(stream), max_mem, output_mask,
                                           from_c(batch_size), gap_score, mismatch_score, match_score,
                                           cuda_banded_alignment != 0));
        }
        catch (...)
        {
            delete h;
            throw;
        }
        *out = h;
        return 0;
    });
}

void gwamd_poa_destroy_batch(gwamd_poa_batch* batch) { delete batch; }

int32_t gwamd_poa_add_poa_group(gwamd_poa_batch* batch, const char* const* seqs, const int8_t* const* weights,
                                const int32_t* lengths, int32_t n, int32_t* per_seq_status)
{
    return guarded([&] {
        cp::Group group;
        for (int32_t i = 0; i < n; i++)
            group.push_back(cp::Entry{seqs[i], weights ? weights[i] : nullptr, lengths[i]});
        std::vector<cp::StatusType> st;
        cp::StatusType rc = batch->impl->add_poa_group(st, group);
        for (size_t i = 0; i < st.size(); i++)
            per_seq_status[i] = int32_t(st[i]);
        for (size_t i = st.size(); i < size_t(n); i++)
            per_seq_status[i] = int32_t(rc);
        return int32_t(rc);
    });
}

int32_t gwamd_poa_get_total_poas(const gwamd_poa_batch* batch) { return batch->impl->get_total_poas(); }

int32_t gwamd_poa_generate_poa(gwamd_poa_batch* batch)
{
    return guarded([&] {
        batch->impl->generate_poa();
        return 0;
    });
}

int32_t gwamd_poa_upload(gwamd_poa_batch* batch)
{
    return guarded([&] {
        batch->impl->upload();
        return 0;
    });
}

int32_t gwamd_poa_launch(gwamd_poa_batch* batch)
{
    return guarded([&] {
        batch->impl->launch();
        return 0;
    });
}

int32_t gwamd_poa_synchronize(gwamd_poa_batch* batch)
{
    return guarded([&] {
        batch->impl->synchronize();
        return 0;
    });
}

int32_t gwamd_poa_get_consensus(gwamd_poa_batch* batch, int32_t* status, int32_t* lengths, const char** cons_base,
                                const uint16_t** cov_base, int32_t* stride)
{
    return guarded([&] {
        std::vector<std::string> cons;
        std::vector<std::vector<uint16_t>> cov;
        std::vector<cp::StatusType> st;
        cp::StatusType rc = batch->impl->get_consensus(cons, cov, st);
        if (rc != cp::StatusType::success)
            return int32_t(rc);
        for (size_t i = 0; i < st.size(); i++)
        {
            status[i]  = int32_t(st[i]);
            lengths[i] = int32_t(cons[i].size());
        }
        *cons_base = reinterpret_cast<const char*>(batch->impl->host_cons().data());
        *cov_base  = batch->impl->host_cov().data();
        *stride    = batch->impl->dims().max_consensus;
        return int32_t(rc);
    });
}

int32_t gwamd_poa_get_msa(gwamd_poa_batch* batch, int32_t* status, int32_t* num_rows, const char** msa_base,
                          int32_t* row_stride, int32_t* max_seqs)
{
    return guarded([&] {
        std::vector<std::vector<std::string>> msa;
        std::vector<cp::StatusType> st;
        cp::StatusType rc = batch->impl->get_msa(msa, st);
        if (rc != cp::StatusType::success)
            return int32_t(rc);
        for (size_t i = 0; i < st.size(); i++)
        {
            status[i]   = int32_t(st[i]);
            num_rows[i] = int32_t(msa[i].size());
        }
        *msa_base   = reinterpret_cast<const char*>(batch->impl->host_msa().data());
        *row_stride = batch->impl->dims().max_consensus;
        *max_seqs   = batch->impl->dims().max_seqs;
        return int32_t(rc);
    });
}

int32_t gwamd_poa_get_graphs(gwamd_poa_batch* batch, int32_t* status, int32_t* num_nodes, const uint8_t** bases,
                             const uint16_t** in_count, const int32_t** in_edges, const uint16_t** in_weights,
                             int32_t* max_nodes)
{
    return guarded([&] {
        batch->impl->fetch_graphs();
        const int32_t n = batch->impl->get_total_poas();
        for (int32_t w = 0; w < n; w++)
        {
            status[w]    = int32_t(batch->impl->graph_status(w));
            num_nodes[w] = batch->impl->host_final_nodes()[w];
        }
        *bases      = batch->impl->host_g_bases().data();
        *in_count   = batch->impl->host_g_in_cnt().data();
        *in_edges   = batch->impl->host_g_in_e().data();
        *in_weights = batch->impl->host_g_in_w().data();
        *max_nodes  = batch->impl->dims().max_nodes;
        return 0;
    });
}

int32_t gwamd_poa_batch_id(const gwamd_poa_batch* batch) { return batch->impl->batch_id(); }

void gwamd_poa_reset(gwamd_poa_batch* batch) { batch->impl->reset(); }

int32_t gwamd_poa_get_stats(gwamd_poa_batch* batch, int64_t* cells, int32_t* final_nodes)
{
    return guarded([&] {
        batch->impl->get_stats(cells, final_nodes);
        return 0;
    });
}

int32_t gwamd_poa_get_phase_ticks(gwamd_poa_batch* batch, int64_t* ticks)
{
    return guarded([&] {
        batch->impl->get_phases(ticks);
        return int32_t(gwamd::poa::kPhases);
    });
}

int32_t gwamd_poa_get_types(const gwamd_poa_batch* batch, int32_t* score_bits, int32_t* size_bits)
{
    *score_bits = batch->impl->score_bits();
    *size_bits  = batch->impl->size_bits();
    return batch->impl->kernel_kind();
}

int32_t gwamd_poa_env_tuning(int32_t* tb_rank, int32_t* band_fwd, int32_t* force_v1, int32_t* diag)
{
    if (!tb_rank || !band_fwd || !force_v1 || !diag)
    {
        gwamd::host::last_error() = "gwamd_poa_env_tuning: NULL output";
        return GWAMD_E_INVALID_ARGUMENT;
    }
    *tb_rank            = claraparabricks::genomeworks::cudapoa::PoaBatch::tb_rank_default();
    const char* fwd     = gwamd::host::diag_env("GWAMD_BAND_FWD");
    *band_fwd           = !fwd ? 0 : (std::string(fwd) == "ad" ? 1 : (std::string(fwd) == "row" ? 2 : 0));
    const char* kern    = gwamd::host::diag_env("GWAMD_POA_KERNEL");
    *force_v1           = kern && std::string(kern) == "v1" ? 1 : 0;
    *diag               = claraparabricks::genomeworks::cudapoa::PoaBatch::diag_bits();
    return 0;
}

int32_t gwamd_poa_set_spoa_accurate(gwamd_poa_batch* batch, int32_t on)
{
    const int32_t was = batch->impl->spoa_accurate() ? 1 : 0;
    batch->impl->set_spoa_accurate(on != 0);
    return was;
}

int32_t gwamd_poa_get_capacity(const gwamd_poa_batch* batch, int64_t* device_bytes, int32_t* max_poas)
{
    *device_bytes = batch->impl->device_bytes();
    *max_poas     = batch->impl->max_poas();
    return 0;
}

int32_t gwamd_poa_get_grid(const gwamd_poa_batch* batch, int32_t* slots, int32_t* resident)
{
    *slots    = batch->impl->slots();
    *resident = batch->impl->resident_slots();
    return 0;
}

static size_t query_free_memory(uint64_t given)
{
    if (given != 0)
        return size_t(given);
    size_t free_mem = 0, total = 0;
    if (hipMemGetInfo(&free_mem, &total) != hipSuccess)
        throw std::runtime_error("hipMemGetInfo failed");
    return free_mem;
}

int64_t gwamd_poa_estimate_max_poas(int32_t max_seq_sz, int32_t max_seq_per_poa, int32_t band_width, int32_t banded,
                                    int32_t msa, uint64_t free_device_memory, float quota, int32_t mismatch,
                                    int32_t gap, int32_t match)
{
    int64_t r = 0;
    const int32_t rc = guarded([&]() -> int32_t {
        r = cp::estimate_max_poas(cp::BatchSize(max_seq_sz, max_seq_per_poa, band_width), banded != 0, msa != 0,
                                  query_free_memory(free_device_memory), quota, mismatch, gap, match);
        return 0;
    });
    return rc != 0 ? int64_t(rc) : r;
}

int32_t gwamd_poa_get_multi_batch_sizes(const int32_t* group_max_len, const int32_t* group_num_reads,
                                        int32_t num_groups, uint64_t free_device_memory, int32_t banded,
                                        int32_t msa, int32_t band_width, const int32_t* bins, int32_t num_bins,
                                        float quota, int32_t mismatch, int32_t gap, int32_t match,
                                        int32_t* num_batches, int32_t* batch_max_seq, int32_t* batch_num_reads,
                                        int32_t* group_batch, int32_t* group_rank)
{
    return guarded([&]() -> int32_t {
        // groups as Entry lists: only the longest read and the read count matter
        std::vector<cp::Group> groups(size_t(std::max(num_groups, 0)));
        for (int32_t i = 0; i < num_groups; i++)
        {
            groups[i].resize(size_t(std::max(group_num_reads[i], 1)));
            for (auto& e : groups[i])
                e = cp::Entry{nullptr, nullptr, 0};
            groups[i][0].length = group_max_len[i];
        }
        std::vector<int32_t> bin_vec;
        if (bins && num_bins > 0)
            bin_vec.assign(bins, bins + num_bins);
        std::vector<cp::BatchSize> sizes;
        std::vector<std::vector<int32_t>> per_batch;
        cp::get_multi_batch_sizes_for_memory(sizes, per_batch, groups, query_free_memory(free_device_memory),
                                         banded != 0, msa != 0, band_width, bin_vec.empty() ? nullptr : &bin_vec,
                                         quota, mismatch, gap, match);
        *num_batches = int32_t(sizes.size());
        for (size_t b = 0; b < sizes.size(); b++)
        {
            batch_max_seq[b]   = sizes[b].max_sequence_size;
            batch_num_reads[b] = sizes[b].max_sequences_per_poa;
            for (size_t r = 0; r < per_batch[b].size(); r++)
            {
                group_batch[per_batch[b][r]] = int32_t(b);
                group_rank[per_batch[b][r]]  = int32_t(r);
            }
        }
        return 0;
    });
}

} // extern "C"
