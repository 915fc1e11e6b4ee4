/*
 * gwamd_cudapoa.h -- C ABI of the MI355X POA path (libgwamd.so).
 *
 * Plain C: opaque handles, plain pointers and sizes, no C++ or torch types.
 * Each entry point replaces one method of the reference's C++ POA API, which
 * is what the reference's own FFI (pygenomeworks Cython,
 * pygenomeworks/genomeworks/cudapoa/cudapoa.pxd) binds:
 *
 *   gwamd_poa_batch_size_init       BatchSize(max_seq, max_seq_per_poa, band)      batch.hpp:74-95
 *   gwamd_poa_batch_size_init_full  BatchSize(6 args)                              batch.hpp:97-128
 *   gwamd_poa_create_batch          create_batch(...)                              batch.hpp:220-228
 *   gwamd_poa_destroy_batch         ~Batch                                         batch.hpp:137
 *   gwamd_poa_add_poa_group         Batch::add_poa_group                           batch.hpp:153-154
 *   gwamd_poa_get_total_poas        Batch::get_total_poas                          batch.hpp:159
 *   gwamd_poa_generate_poa          Batch::generate_poa                            batch.hpp:162
 *   gwamd_poa_get_consensus         Batch::get_consensus                           batch.hpp:174-176
 *   gwamd_poa_get_msa               Batch::get_msa                                 batch.hpp:186-187
 *   gwamd_poa_get_graphs            Batch::get_graphs                              batch.hpp:195-196
 *   gwamd_poa_batch_id              Batch::batch_id                                batch.hpp:201
 *   gwamd_poa_reset                 Batch::reset                                   batch.hpp:204
 *   gwamd_poa_multibatch_create     MultiBatch(num_batches, ...)     benchmarks/multi_batch.hpp:36-58
 *   gwamd_poa_multibatch_process    MultiBatch::process_batches      benchmarks/multi_batch.hpp:64-171
 *   gwamd_poa_multibatch_run_file   MultiBatch(file) + process_batches + assembly
 *                                                                    Test_CudapoaBatchEnd2End.cu:55-69
 *
 * Extra entry points (no reference counterpart; used by bench.py): split
 * generate_poa into its H2D copy and its kernel launch, and read per-window
 * work counters.
 *
 * Error convention: functions returning int32_t return a StatusType value
 * (cudapoa.hpp:26-38) >= 0, or a negative GWAMD_E_* code when the reference
 * would have thrown (message in gwamd_last_error()).
 */
#ifndef GWAMD_CUDAPOA_H
#define GWAMD_CUDAPOA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWAMD_E_INVALID_ARGUMENT (-1) /* reference: std::invalid_argument */
#define GWAMD_E_RUNTIME (-2)          /* reference: std::runtime_error    */
#define GWAMD_E_HIP (-3)              /* HIP runtime failure              */

typedef struct gwamd_poa_batch gwamd_poa_batch;

/* Mirror of cudapoa::BatchSize (batch.hpp:53-71), same field order. */
typedef struct gwamd_poa_batch_size
{
    int32_t max_sequence_size;
    int32_t max_consensus_size;
    int32_t max_nodes_per_window;
    int32_t max_nodes_per_window_banded;
    int32_t max_matrix_graph_dimension;
    int32_t max_matrix_graph_dimension_banded;
    int32_t max_matrix_sequence_dimension;
    int32_t alignment_band_width;
    int32_t max_sequences_per_poa;
} gwamd_poa_batch_size;

/* Last error message of the calling thread ("" if none). */
const char* gwamd_last_error(void);

int32_t gwamd_poa_batch_size_init(gwamd_poa_batch_size* out, int32_t max_seq_sz, int32_t max_seq_per_poa,
                                  int32_t band_width);
int32_t gwamd_poa_batch_size_init_full(gwamd_poa_batch_size* out, int32_t max_seq_sz, int32_t max_consensus_sz,
                                       int32_t max_nodes_per_w, int32_t max_nodes_per_w_banded, int32_t band_width,
                                       int32_t max_seq_per_poa);

/* stream: a hipStream_t (NULL = default stream). */
int32_t gwamd_poa_create_batch(gwamd_poa_batch** out, int32_t device_id, void* stream, size_t max_mem,
                               int8_t output_mask, const gwamd_poa_batch_size* batch_size, int16_t gap_score,
                               int16_t mismatch_score, int16_t match_score, int32_t cuda_banded_alignment);
void gwamd_poa_destroy_batch(gwamd_poa_batch* batch);

/* One group = n entries; weights[i] may be NULL (all ones).  per_seq_status
 * receives n StatusType values.  Returns the group's StatusType. */
int32_t gwamd_poa_add_poa_group(gwamd_poa_batch* batch, const char* const* seqs, const int8_t* const* weights,
                                const int32_t* lengths, int32_t n, int32_t* per_seq_status);
int32_t gwamd_poa_get_total_poas(const gwamd_poa_batch* batch);
int32_t gwamd_poa_generate_poa(gwamd_poa_batch* batch);

/* Blocks on the stream.  status/lengths receive get_total_poas() entries; the
 * consensus of window i is cons_base[i*stride .. +lengths[i]) and its coverage
 * cov_base[i*stride ..].  Buffers stay valid until the next generate/reset. */
int32_t gwamd_poa_get_consensus(gwamd_poa_batch* batch, int32_t* status, int32_t* lengths, const char** cons_base,
                                const uint16_t** cov_base, int32_t* stride);

/* Blocks on the stream.  Row s of window i is the NUL-terminated string at
 * msa_base + (i*max_seqs + s)*row_stride; num_rows[i] = reads in window i. */
int32_t gwamd_poa_get_msa(gwamd_poa_batch* batch, int32_t* status, int32_t* num_rows, const char** msa_base,
                          int32_t* row_stride, int32_t* max_seqs);

/* Blocks on the stream.  Window i has num_nodes[i] nodes; node v's label is
 * bases[i*max_nodes + v]; its incoming edges (src, weight) are
 * in_edges/in_weights[(i*max_nodes + v)*50 + e] for e < in_count[i*max_nodes+v].
 * Caller arrays: status, num_nodes sized get_total_poas(); the rest are
 * returned as pointers to batch-owned host memory. */
int32_t gwamd_poa_get_graphs(gwamd_poa_batch* batch, int32_t* status, int32_t* num_nodes, const uint8_t** bases,
                             const uint16_t** in_count, const int32_t** in_edges, const uint16_t** in_weights,
                             int32_t* max_nodes);

int32_t gwamd_poa_batch_id(const gwamd_poa_batch* batch);
void gwamd_poa_reset(gwamd_poa_batch* batch);

/* bench.py helpers: generate_poa == upload + launch. */
int32_t gwamd_poa_upload(gwamd_poa_batch* batch);
int32_t gwamd_poa_launch(gwamd_poa_batch* batch);
int32_t gwamd_poa_synchronize(gwamd_poa_batch* batch);
/* Per-window DP cells (sum over reads of (|V|+1)*(|r|+1), banded: band cells)
 * and final node counts of the last generate; arrays sized get_total_poas(). */
int32_t gwamd_poa_get_stats(gwamd_poa_batch* batch, int64_t* cells, int32_t* final_nodes);
/* Per-window phase timers of the last launch (s_memrealtime ticks, 100 MHz):
 * backbone, forward DP, traceback, add, topsort, output, total; ticks receives
 * 7 * get_total_poas() values.  Returns the number of phases. */
int32_t gwamd_poa_get_phase_ticks(gwamd_poa_batch* batch, int64_t* ticks);
/* Score/size types chosen by create_batch (16 or 32 bits each); returns the
 * kernel variant (1: global-memory kernel, 2: LDS-resident kernel). */
int32_t gwamd_poa_get_types(const gwamd_poa_batch* batch, int32_t* score_bits, int32_t* size_bits);
/* SPOA_ACCURATE mode (reference build option spoa_accurate, CMakeLists.txt:23-30;
 * cudapoa_kernels.cuh:324-337): after each read the graph is re-sorted with the
 * racon/SPOA DFS (cudapoa_topsort.cuh:94-189) instead of Kahn's order, which
 * matches SPOA's consensus order at a lower speed.  Takes effect at the next
 * generate_poa; returns the previous setting.  Default: the GWAMD_SPOA_ACCURATE
 * environment variable at create time (off when unset). */
int32_t gwamd_poa_set_spoa_accurate(gwamd_poa_batch* batch, int32_t on);
/* Kernel tuning a batch created now would take from the environment (no
 * reference counterpart).  The GWAMD_* tuning variables are read only when
 * GWAMD_DIAG=1; otherwise this reports the defaults: *tb_rank = traceback
 * walk bits (3: pointer doubling over strips), *band_fwd = 0 (plan decides;
 * 1 anti-diagonal forced, 2 row-parallel forced), *force_v1 = 0, *diag = 0.
 * Host only, needs no GPU. */
int32_t gwamd_poa_env_tuning(int32_t* tb_rank, int32_t* band_fwd, int32_t* force_v1, int32_t* diag);
/* Device bytes allocated by the batch and its window capacity (max_poas). */
int32_t gwamd_poa_get_capacity(const gwamd_poa_batch* batch, int64_t* device_bytes, int32_t* max_poas);

/* Persistent grid of the batch: scratch slots (= workgroups launched when the
 * batch holds more windows than slots; each workgroup then dequeues windows
 * heaviest first) and the device's resident workgroup count for the planned
 * kernel (0: global-memory kernel, one workgroup per window, slots = max_poas). */
int32_t gwamd_poa_get_grid(const gwamd_poa_batch* batch, int32_t* slots, int32_t* resident);

/* BatchBlock::estimate_max_poas (allocate_block.hpp:364-401) for a
 * BatchSize(max_seq_sz, max_seq_per_poa, band_width); free_device_memory 0
 * queries the current device. */
int64_t gwamd_poa_estimate_max_poas(int32_t max_seq_sz, int32_t max_seq_per_poa, int32_t band_width,
                                    int32_t banded, int32_t msa, uint64_t free_device_memory, float quota,
                                    int32_t mismatch, int32_t gap, int32_t match);

/* get_multi_batch_sizes (utils.hpp:48-66, utils.cu:24-138) over groups given
 * by their longest read and read count.  Outputs: *num_batches, per batch its
 * BatchSize(max_sequence_size, max_sequences_per_poa) in batch_max_seq /
 * batch_num_reads (capacity num_groups), and per group its batch index and its
 * rank inside that batch's group list.  bins (num_bins > 0) replaces the
 * default capacities 1, 2, 4, ... 2^19.  free_device_memory 0 queries the
 * current device.  Returns 0 or GWAMD_E_INVALID_ARGUMENT. */
int32_t gwamd_poa_get_multi_batch_sizes(const int32_t* group_max_len, const int32_t* group_num_reads,
                                        int32_t num_groups, uint64_t free_device_memory, int32_t banded,
                                        int32_t msa, int32_t band_width, const int32_t* bins, int32_t num_bins,
                                        float quota, int32_t mismatch, int32_t gap, int32_t match,
                                        int32_t* num_batches, int32_t* batch_max_seq, int32_t* batch_num_reads,
                                        int32_t* group_batch, int32_t* group_rank);

/* ---- Concurrent multi-batch driver (cudapoa/benchmarks/multi_batch.hpp) ----
 * num_batches batches of the given BatchSize, each on its own HIP stream and
 * host thread, mem_per_batch device bytes each (0: 0.9 x free / num_batches).
 * output_mask must include consensus. */
typedef struct gwamd_poa_multibatch gwamd_poa_multibatch;
int32_t gwamd_poa_multibatch_create(gwamd_poa_multibatch** out, int32_t device_id, int32_t num_batches,
                                    size_t mem_per_batch, int8_t output_mask, const gwamd_poa_batch_size* batch_size,
                                    int16_t gap_score, int16_t mismatch_score, int16_t match_score,
                                    int32_t cuda_banded_alignment);
void gwamd_poa_multibatch_destroy(gwamd_poa_multibatch* mb);
/* Runs num_windows windows through the batches.  Window w holds reads
 * first_read[w] .. first_read[w+1]-1 (first_read has num_windows+1 entries);
 * read r is bases[read_off[r] .. read_off[r]+read_len[r]).  Host bytes are
 * read while the call runs only.  Outputs per window (NULL arrays are
 * skipped): status[w] (StatusType), cons_len[w], consensus at
 * cons + w*stride, coverage at cov + w*stride.  Blocks until done. */
int32_t gwamd_poa_multibatch_process(gwamd_poa_multibatch* mb, const char* bases, const int64_t* read_off,
                                     const int32_t* read_len, const int64_t* first_read, int32_t num_windows,
                                     int32_t* status, int32_t* cons_len, char* cons, uint16_t* cov, int32_t stride);
/* Batches, the most windows one batch took, generate_poa calls of the last process. */
int32_t gwamd_poa_multibatch_info(const gwamd_poa_multibatch* mb, int32_t* num_batches, int32_t* max_poas_per_batch,
                                  int32_t* rounds);
/* Extra (no reference counterpart; bench.py config E roofline): when on,
 * process records HIP events around every kernel launch.  Returns the previous
 * setting. */
int32_t gwamd_poa_multibatch_set_launch_timing(gwamd_poa_multibatch* mb, int32_t on);
/* Launch records of the last process (sorted by start): kernel start / stop in
 * ms after the call began, DP cells, windows, batch index.  Fills at most
 * capacity entries (NULL arrays skipped); returns the number of launches. */
int32_t gwamd_poa_multibatch_launches(const gwamd_poa_multibatch* mb, float* start_ms, float* stop_ms, int64_t* cells,
                                      int32_t* windows, int32_t* batch, int32_t capacity);
/* Windows of the last process that fit no empty batch (status = the
 * add_poa_group status, e.g. exceeded_maximum_sequence_size). */
int32_t gwamd_poa_multibatch_skipped(const gwamd_poa_multibatch* mb);
/* The reference's end-to-end flow: MultiBatch(num_batches, filename,
 * total_windows), process_batches(), assembly().  Writes up to capacity bytes
 * of the assembly and its full length to *length. */
int32_t gwamd_poa_multibatch_run_file(const char* filename, int32_t num_batches, int32_t total_windows,
                                      char* assembly, int64_t capacity, int64_t* length);

#ifdef __cplusplus
}
#endif

#endif /* GWAMD_CUDAPOA_H */
