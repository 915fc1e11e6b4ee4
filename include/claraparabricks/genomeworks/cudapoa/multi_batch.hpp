// Concurrent multi-batch POA driver for the cudapoa drop-in API.
//
// Reference: cudapoa/benchmarks/multi_batch.hpp:30-215 (class MultiBatch, used
// by BM_MultiBatchTest, cudapoa/benchmarks/main.cpp:52-61, and by the
// end-to-end test Test_CudapoaBatchEnd2End.cu:33-85).  Same names and
// behaviour: num_batches Batch objects, each on its own stream and host
// thread; a thread resets its batch, fills it under a mutex with the next
// windows until add_poa_group reports exceeded_maximum_poas, runs
// generate_poa + get_consensus, stores the results by window index and goes
// again until the windows run out.  While one thread packs and uploads its
// batch, the others' kernels keep the GPU busy.
#pragma once

#include <claraparabricks/genomeworks/cudapoa/batch.hpp>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{
namespace cudapoa
{

class MultiBatch
{
public:
    /// Reference constructor (multi_batch.hpp:36-58): windows from a
    /// cudapoa-format file (parse_cudapoa_file, total_windows < 0 keeps all),
    /// BatchSize(1024, 200), consensus output, scores -8 / -6 / 8, full
    /// alignment, 0.9 x free device memory of device 0 split over the batches.
    MultiBatch(int32_t num_batches, const std::string& filename, int32_t total_windows = -1);

    /// General form: caller-supplied groups (their bytes must stay valid until
    /// process_batches returns), batch limits, device memory per batch
    /// (0: 0.9 x free memory / num_batches), output mask (must include
    /// consensus), scores and alignment mode.
    MultiBatch(int32_t num_batches, const std::vector<Group>& groups, int32_t device_id, size_t mem_per_batch,
               int8_t output_mask, const BatchSize& batch_size, int16_t gap_score = -8, int16_t mismatch_score = -6,
               int16_t match_score = 8, bool cuda_banded_alignment = false);

    ~MultiBatch();

    MultiBatch(const MultiBatch&) = delete;
    MultiBatch& operator=(const MultiBatch&) = delete;

    /// Runs every window through the batches (multi_batch.hpp:64-171).
    /// Throws std::runtime_error if a batch returns a different number of
    /// consensus sequences than the windows it was given.
    void process_batches();

    /// Concatenated consensus trimmed per window to the bases whose coverage
    /// is at least the window's mean coverage (multi_batch.hpp:176-207).
    std::string assembly() const;

    /// Replaces the groups (same batches and streams) for the next process_batches.
    void set_groups(const std::vector<Group>& groups);

    /// Results of the last process_batches, by window.
    const std::vector<std::string>& consensus() const { return consensus_; }
    const std::vector<std::vector<uint16_t>>& coverages() const { return coverages_; }
    const std::vector<StatusType>& output_status() const { return status_; }

    /// Optional direct output (C ABI): window w's consensus is written to
    /// cons + w * stride and its coverage to cov + w * stride instead of the
    /// vectors above; lengths and statuses to len[w] / status[w].
    struct Sink
    {
        char* cons       = nullptr;
        uint16_t* cov    = nullptr;
        int32_t* len     = nullptr;
        int32_t* status  = nullptr;
        int32_t stride   = 0;
    };
    void set_sink(const Sink& sink) { sink_ = sink; use_sink_ = true; }

    int32_t num_batches() const { return int32_t(batches_.size()); }
    /// Window capacity of each batch (max_poas).
    int32_t max_poas_per_batch() const { return max_poas_; }
    /// generate_poa calls of the last process_batches (all batches together).
    int32_t rounds() const { return rounds_; }
    /// Windows of the last process_batches that fit no empty batch (they keep
    /// the add_poa_group status; the reference stops every thread there).
    int32_t skipped_windows() const { return skipped_; }

    /// Kernel launch records of the last process_batches when launch timing is
    /// on: start / stop of each batch's kernel in ms after the call began (HIP
    /// events on the batch's stream), the DP cells and the windows it ran.
    struct LaunchRecord
    {
        float start_ms  = 0.f;
        float stop_ms   = 0.f;
        int64_t cells   = 0;
        int32_t windows = 0;
        int32_t batch   = 0;
    };
    void set_launch_timing(bool on) { time_launches_ = on; }
    bool launch_timing() const { return time_launches_; }
    const std::vector<LaunchRecord>& launches() const { return launches_; }

private:
    void create(int32_t num_batches, int32_t device_id, size_t mem_per_batch, int8_t output_mask,
                const BatchSize& batch_size, int16_t gap_score, int16_t mismatch_score, int16_t match_score,
                bool banded);

    int32_t device_id_ = 0;
    std::vector<void*> streams_; // hipStream_t, one per batch
    std::vector<std::unique_ptr<Batch>> batches_;
    std::vector<std::vector<std::string>> owned_windows_; // reference constructor only
    std::vector<Group> groups_;
    std::vector<std::string> consensus_;
    std::vector<std::vector<uint16_t>> coverages_;
    std::vector<StatusType> status_;
    Sink sink_;
    bool use_sink_   = false;
    int32_t max_poas_ = 0;
    int32_t rounds_   = 0;
    int32_t skipped_  = 0;
    bool time_launches_ = false;
    std::vector<LaunchRecord> launches_;
};

} // namespace cudapoa
} // namespace genomeworks
} // namespace claraparabricks
