// Concurrent multi-batch POA driver (include/.../cudapoa/multi_batch.hpp) and
// its C ABI (include/gwamd_cudapoa.h, gwamd_poa_multibatch_*).
//
// Reference: cudapoa/benchmarks/multi_batch.hpp:30-215.  One host thread per
// batch, each batch on its own non-blocking HIP stream; windows are handed out
// under one mutex in window order; results are stored by window index.  The
// batches' kernels use a persistent grid (poa_batch.cpp plan_launch_order), so
// a kernel queued on another stream fills the CUs that the running kernel's
// last windows leave idle.
#include <claraparabricks/genomeworks/cudapoa/multi_batch.hpp>
#include <claraparabricks/genomeworks/cudapoa/utils.hpp>

#include "gwamd_cudapoa.h"
#include "host_common.hpp"
#include "poa_batch_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <thread>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

using gwamd::host::ScopedDevice;

MultiBatch::MultiBatch(int32_t num_batches, const std::string& filename, int32_t total_windows)
{
    parse_cudapoa_file(owned_windows_, filename, total_windows);
    if (owned_windows_.empty())
        throw std::runtime_error("MultiBatch: no windows in " + filename);
    std::vector<Group> groups(owned_windows_.size());
    for (size_t w = 0; w < owned_windows_.size(); w++)
        for (const auto& seq : owned_windows_[w])
            groups[w].push_back(Entry{seq.c_str(), nullptr, int32_t(seq.length())});
    set_groups(groups);
    // multi_batch.hpp:43-56
    create(num_batches, 0, 0, OutputType::consensus, BatchSize(1024, 200), -8, -6, 8, false);
}

MultiBatch::MultiBatch(int32_t num_batches, const std::vector<Group>& groups, int32_t device_id, size_t mem_per_batch,
                       int8_t output_mask, const BatchSize& batch_size, int16_t gap_score, int16_t mismatch_score,
                       int16_t match_score, bool cuda_banded_alignment)
{
    set_groups(groups);
    create(num_batches, device_id, mem_per_batch, output_mask, batch_size, gap_score, mismatch_score, match_score,
           cuda_banded_alignment);
}

void MultiBatch::create(int32_t num_batches, int32_t device_id, size_t mem_per_batch, int8_t output_mask,
                        const BatchSize& batch_size, int16_t gap_score, int16_t mismatch_score, int16_t match_score,
                        bool banded)
{
    if (num_batches < 1)
        throw std::invalid_argument("MultiBatch: number of batches has to be positive");
    if (!(output_mask & OutputType::consensus))
        throw std::invalid_argument("MultiBatch: the output mask has to include consensus");
    device_id_ = device_id;
    ScopedDevice dev(device_id_);
    if (mem_per_batch == 0)
    {
        size_t free_mem = 0, total = 0;
        GWAMD_HIP_CHECK(hipMemGetInfo(&free_mem, &total));
        mem_per_batch = size_t(0.9 * double(free_mem) / num_batches);
    }
    for (int32_t b = 0; b < num_batches; b++)
    {
        hipStream_t s = nullptr;
        GWAMD_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        streams_.push_back(s);
        batches_.emplace_back(create_batch(device_id_, s, mem_per_batch, output_mask, batch_size, gap_score,
                                           mismatch_score, match_score, banded));
    }
}

MultiBatch::~MultiBatch()
{
    batches_.clear();
    (void)hipSetDevice(device_id_);
    for (void* s : streams_)
        (void)hipStreamDestroy(static_cast<hipStream_t>(s));
}

void MultiBatch::set_groups(const std::vector<Group>& groups) { groups_ = groups; }

void MultiBatch::process_batches()
{
    const int32_t count = int32_t(groups_.size());
    if (!use_sink_)
    {
        consensus_.assign(size_t(count), std::string());
        coverages_.assign(size_t(count), std::vector<uint16_t>());
    }
    else
    {
        // a window that never reaches a batch (the threads stopped on an
        // error) must not keep the caller's earlier status / length
        for (int32_t w = 0; w < count; w++)
        {
            if (sink_.status)
                sink_.status[w] = int32_t(StatusType::generic_error);
            if (sink_.len)
                sink_.len[w] = 0;
        }
    }
    status_.assign(size_t(count), StatusType::generic_error);
    rounds_   = 0;
    max_poas_ = 0;
    skipped_  = 0;
    launches_.clear();

    std::mutex mutex_windows;
    int32_t next_window_index = 0;

    // Launch timing (set_launch_timing): one start/stop event pair per batch
    // and a reference event, so every launch becomes an interval on one clock.
    const size_t nb = batches_.size();
    std::vector<hipEvent_t> ev_start(nb, nullptr), ev_stop(nb, nullptr);
    hipEvent_t ev_ref = nullptr;
    struct EventGuard
    {
        std::vector<hipEvent_t>* a;
        std::vector<hipEvent_t>* b;
        hipEvent_t* r;
        std::vector<std::unique_ptr<Batch>>* batches;
        ~EventGuard()
        {
            for (auto& bt : *batches)
                detail::set_launch_events(bt.get(), nullptr, nullptr);
            for (auto* v : {a, b})
                for (hipEvent_t e : *v)
                    if (e)
                        (void)hipEventDestroy(e);
            if (*r)
                (void)hipEventDestroy(*r);
        }
    } guard_events{&ev_start, &ev_stop, &ev_ref, &batches_};
    if (time_launches_)
    {
        ScopedDevice dev(device_id_);
        for (size_t b = 0; b < nb; b++)
        {
            GWAMD_HIP_CHECK(hipEventCreate(&ev_start[b]));
            GWAMD_HIP_CHECK(hipEventCreate(&ev_stop[b]));
            detail::set_launch_events(batches_[b].get(), ev_start[b], ev_stop[b]);
        }
        GWAMD_HIP_CHECK(hipEventCreate(&ev_ref));
        GWAMD_HIP_CHECK(hipEventRecord(ev_ref, static_cast<hipStream_t>(streams_[0])));
        GWAMD_HIP_CHECK(hipEventSynchronize(ev_ref));
    }
    std::mutex mutex_launches;

    // multi_batch.hpp:79-115: reset, then add windows until the batch is full.
    // A window that does not fit an empty batch (a read longer than the
    // batch's max_sequence_size, too many reads) would stop every thread in
    // the reference, leaving the rest of the windows unprocessed; here it
    // gets its add_poa_group status and the batch moves past it.
    auto fill_next_batch = [&](Batch* batch) -> std::pair<int32_t, int32_t> {
        batch->reset();
        std::lock_guard<std::mutex> guard(mutex_windows);
        int32_t initial = next_window_index;
        std::vector<StatusType> s;
        while (next_window_index < count)
        {
            const StatusType st = batch->add_poa_group(s, groups_[size_t(next_window_index)]);
            if (st == StatusType::success)
            {
                next_window_index++;
                continue;
            }
            if (batch->get_total_poas() > 0)
                break;
            // nothing fits an empty batch: this window cannot be processed
            StatusType why = st;
            for (const StatusType e : s)
                if (e != StatusType::success)
                {
                    why = e;
                    break;
                }
            if (why == StatusType::exceeded_maximum_poas)
            {
                int32_t longest = 0;
                for (const auto& e : groups_[size_t(next_window_index)])
                    longest = std::max(longest, e.length);
                if (longest > detail::max_sequence_size(batch))
                    why = StatusType::exceeded_maximum_sequence_size;
            }
            const size_t w = size_t(next_window_index);
            status_[w]     = why;
            if (use_sink_ && sink_.status)
                sink_.status[w] = int32_t(why);
            skipped_++;
            batch->reset();
            initial = ++next_window_index;
        }
        if (next_window_index > initial)
        {
            rounds_++;
            max_poas_ = std::max(max_poas_, next_window_index - initial);
        }
        return {initial, next_window_index};
    };

    // multi_batch.hpp:118-155
    auto process_batch = [&](size_t b) {
        Batch* batch = batches_[b].get();
        std::vector<std::string> cons;
        std::vector<std::vector<uint16_t>> cov;
        std::vector<StatusType> st;
        while (true)
        {
            const std::pair<int32_t, int32_t> range = fill_next_batch(batch);
            if (batch->get_total_poas() == 0)
                break;
            cons.clear();
            cov.clear();
            st.clear();
            batch->generate_poa();
            batch->get_consensus(cons, cov, st);
            const int32_t n = range.second - range.first;
            if (int32_t(cons.size()) != n || int32_t(cov.size()) != n)
                throw std::runtime_error("Consensus processed doesn't match range of windows passed to batch");
            if (time_launches_)
            {
                LaunchRecord rec;
                GWAMD_HIP_CHECK(hipEventElapsedTime(&rec.start_ms, ev_ref, ev_start[b]));
                GWAMD_HIP_CHECK(hipEventElapsedTime(&rec.stop_ms, ev_ref, ev_stop[b]));
                rec.cells   = detail::last_launch_cells(batch);
                rec.windows = n;
                rec.batch   = int32_t(b);
                std::lock_guard<std::mutex> g(mutex_launches);
                launches_.push_back(rec);
            }
            for (int32_t i = 0; i < n; i++)
            {
                const size_t w = size_t(range.first + i);
                status_[w]     = st[size_t(i)];
                if (!use_sink_)
                {
                    consensus_[w] = std::move(cons[size_t(i)]);
                    coverages_[w] = std::move(cov[size_t(i)]);
                    continue;
                }
                const int32_t len = int32_t(cons[size_t(i)].size());
                if (len > sink_.stride)
                    throw std::runtime_error("MultiBatch: consensus longer than the output stride");
                if (sink_.len)
                    sink_.len[w] = len;
                if (sink_.status)
                    sink_.status[w] = int32_t(st[size_t(i)]);
                if (sink_.cons && len > 0)
                    std::memcpy(sink_.cons + w * size_t(sink_.stride), cons[size_t(i)].data(), size_t(len));
                if (sink_.cov && len > 0)
                    std::memcpy(sink_.cov + w * size_t(sink_.stride), cov[size_t(i)].data(), size_t(len) * 2);
            }
        }
    };

    // multi_batch.hpp:158-170: one thread per batch
    std::vector<std::thread> threads;
    std::vector<std::exception_ptr> errors(batches_.size());
    for (size_t b = 0; b < batches_.size(); b++)
    {
        threads.emplace_back([&, b] {
            try
            {
                ScopedDevice dev(device_id_);
                process_batch(b);
            }
            catch (...)
            {
                errors[b] = std::current_exception();
                // stop the other threads from taking more windows
                std::lock_guard<std::mutex> guard(mutex_windows);
                next_window_index = count;
            }
        });
    }
    for (auto& t : threads)
        t.join();
    for (auto& e : errors)
        if (e)
            std::rethrow_exception(e);
    std::sort(launches_.begin(), launches_.end(),
              [](const LaunchRecord& a, const LaunchRecord& b) { return a.start_ms < b.start_ms; });
}

// multi_batch.hpp:176-207
std::string MultiBatch::assembly() const
{
    std::string genome;
    for (size_t w = 0; w < consensus_.size(); w++)
    {
        const auto& cov = coverages_[w];
        if (cov.empty())
            continue;
        const int32_t average = int32_t(std::accumulate(cov.begin(), cov.end(), 0) / int32_t(cov.size()));
        int32_t begin = 0, end = int32_t(consensus_[w].length()) - 1;
        for (; begin < int32_t(cov.size()); ++begin)
            if (cov[size_t(begin)] >= average)
                break;
        for (; end >= 0; --end)
            if (cov[size_t(end)] >= average)
                break;
        if (begin < end)
            genome += consensus_[w].substr(size_t(begin), size_t(end - begin + 1));
    }
    return genome;
}

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks

// ===========================================================================
// C ABI
// ===========================================================================
namespace cp = claraparabricks::genomeworks::cudapoa;

struct gwamd_poa_multibatch
{
    std::unique_ptr<cp::MultiBatch> impl;
};

namespace
{
template <typename F>
int32_t mb_guarded(F&& f)
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

cp::BatchSize batch_size_from_c(const gwamd_poa_batch_size* i)
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

extern "C" {

int32_t gwamd_poa_multibatch_create(gwamd_poa_multibatch** out, int32_t device_id, int32_t num_batches,
                                    size_t mem_per_batch, int8_t output_mask, const gwamd_poa_batch_size* batch_size,
                                    int16_t gap_score, int16_t mismatch_score, int16_t match_score,
                                    int32_t cuda_banded_alignment)
{
    *out = nullptr;
    return mb_guarded([&] {
        auto* h = new gwamd_poa_multibatch;
        try
        {
            h->impl.reset(new cp::MultiBatch(num_batches, std::vector<cp::Group>(), device_id, mem_per_batch,
                                             output_mask, batch_size_from_c(batch_size), gap_score, mismatch_score,
                                             match_score, cuda_banded_alignment != 0));
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

void gwamd_poa_multibatch_destroy(gwamd_poa_multibatch* mb) { delete mb; }

int32_t gwamd_poa_multibatch_process(gwamd_poa_multibatch* mb, const char* bases, const int64_t* read_off,
                                     const int32_t* read_len, const int64_t* first_read, int32_t num_windows,
                                     int32_t* status, int32_t* cons_len, char* cons, uint16_t* cov, int32_t stride)
{
    return mb_guarded([&] {
        if (num_windows < 0 || (num_windows > 0 && (!bases || !read_off || !read_len || !first_read)))
            throw std::invalid_argument("gwamd_poa_multibatch_process: missing input arrays");
        std::vector<cp::Group> groups(static_cast<size_t>(num_windows));
        for (int32_t w = 0; w < num_windows; w++)
        {
            const int64_t r0 = first_read[w], r1 = first_read[w + 1];
            if (r1 < r0)
                throw std::invalid_argument("gwamd_poa_multibatch_process: first_read is not ascending");
            groups[size_t(w)].reserve(size_t(r1 - r0));
            for (int64_t r = r0; r < r1; r++)
                groups[size_t(w)].push_back(cp::Entry{bases + read_off[r], nullptr, read_len[r]});
        }
        cp::MultiBatch::Sink sink;
        sink.cons   = cons;
        sink.cov    = cov;
        sink.len    = cons_len;
        sink.status = status;
        sink.stride = stride;
        mb->impl->set_groups(groups);
        mb->impl->set_sink(sink);
        mb->impl->process_batches();
        return 0;
    });
}

int32_t gwamd_poa_multibatch_info(const gwamd_poa_multibatch* mb, int32_t* num_batches, int32_t* max_poas_per_batch,
                                  int32_t* rounds)
{
    *num_batches        = mb->impl->num_batches();
    *max_poas_per_batch = mb->impl->max_poas_per_batch();
    *rounds             = mb->impl->rounds();
    return 0;
}

int32_t gwamd_poa_multibatch_set_launch_timing(gwamd_poa_multibatch* mb, int32_t on)
{
    const int32_t was = mb->impl->launch_timing() ? 1 : 0;
    mb->impl->set_launch_timing(on != 0);
    return was;
}

int32_t gwamd_poa_multibatch_launches(const gwamd_poa_multibatch* mb, float* start_ms, float* stop_ms, int64_t* cells,
                                      int32_t* windows, int32_t* batch, int32_t capacity)
{
    const auto& l = mb->impl->launches();
    const int32_t n = int32_t(l.size());
    for (int32_t i = 0; i < std::min(n, capacity); i++)
    {
        if (start_ms)
            start_ms[i] = l[size_t(i)].start_ms;
        if (stop_ms)
            stop_ms[i] = l[size_t(i)].stop_ms;
        if (cells)
            cells[i] = l[size_t(i)].cells;
        if (windows)
            windows[i] = l[size_t(i)].windows;
        if (batch)
            batch[i] = l[size_t(i)].batch;
    }
    return n;
}

int32_t gwamd_poa_multibatch_skipped(const gwamd_poa_multibatch* mb) { return mb->impl->skipped_windows(); }

int32_t gwamd_poa_multibatch_run_file(const char* filename, int32_t num_batches, int32_t total_windows,
                                      char* assembly, int64_t capacity, int64_t* length)
{
    return mb_guarded([&] {
        cp::MultiBatch mb(num_batches, std::string(filename), total_windows);
        mb.process_batches();
        const std::string g = mb.assembly();
        *length             = int64_t(g.size());
        if (assembly && capacity > 0)
            std::memcpy(assembly, g.data(), size_t(std::min<int64_t>(capacity, int64_t(g.size()))));
        return 0;
    });
}

} // extern "C"
