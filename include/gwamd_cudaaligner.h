/*
 * gwamd_cudaaligner.h -- C ABI of the MI355X global aligner (libgwamd.so).
 *
 * Plain C: opaque handle, plain pointers and sizes.  Each entry point replaces
 * one method of the reference's C++ aligner API, which is what the reference's
 * own FFI (pygenomeworks/genomeworks/cudaaligner/cudaaligner.pxd) binds:
 *
 *   gwamd_aligner_create          create_aligner(...)                      aligner.hpp:90,103
 *                                 (algorithm 1: AlignerGlobalMyers,        aligner_global_myers.hpp:24
 *                                  algorithm 2: AlignerGlobalMyersBanded,  aligner_global_myers_banded.hpp:24
 *                                  algorithm 3: AlignerGlobalUkkonen)      aligner_global_ukkonen.hpp:28
 *   gwamd_aligner_create_with_allocator
 *                                 create_aligner(..., DefaultDeviceAllocator, aligner.hpp:90
 *                                 stream, device_id)
 *   gwamd_device_allocator_create create_default_device_allocator(size)    allocator.hpp:297-305
 *                                 (copies share one pool: a handle here)   allocator.hpp:274-279
 *   gwamd_device_allocator_destroy / _capacity / _used / _default_size
 *   gwamd_aligner_destroy         ~Aligner                                 aligner.hpp:45
 *   gwamd_aligner_add_alignment   Aligner::add_alignment                   aligner.hpp:70-71
 *   gwamd_aligner_align_all       Aligner::align_all                       aligner.hpp:55
 *   gwamd_aligner_sync_alignments Aligner::sync_alignments                 aligner.hpp:61
 *   gwamd_aligner_num_alignments  get_alignments().size()                  aligner.hpp:76
 *   gwamd_aligner_get_alignment   Alignment::get_alignment / get_status    alignment.hpp:72-80
 *   gwamd_aligner_get_sequences   Alignment::get_query/target_sequence     alignment.hpp:53-56
 *   gwamd_aligner_get_cigar       Alignment::convert_to_cigar              alignment.hpp:62
 *   gwamd_aligner_reset           Aligner::reset                           aligner.hpp:79
 *   gwamd_alignment_format        Alignment::format_alignment              alignment.hpp:82-85
 *                                 (AlignmentImpl over given states,        alignment_impl.cpp:75-112)
 *   gwamd_alignment_cigar         Alignment::convert_to_cigar              alignment_impl.cpp:47-73
 *   gwamd_aligner_max_lengths     (none: this implementation's length limits)
 *   gwamd_aligner_pair_fits       (none: whether a (query, target) limit pair is accepted)
 *   gwamd_aligner_get_stats       (none: path counters for the parity tests)
 *   gwamd_aligner_last_kernel_ms  (none: kernel time of the last align_all, bench.py)
 *
 * Extra entry points (bench.py): split align_all into upload / launch /
 * download and read the raw device paths.
 *
 * Error convention: StatusType values (cudaaligner.hpp:27-35) >= 0, or a
 * negative GWAMD_E_* code where the reference throws (gwamd_last_error()).
 */
#ifndef GWAMD_CUDAALIGNER_H
#define GWAMD_CUDAALIGNER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef GWAMD_E_INVALID_ARGUMENT
#define GWAMD_E_INVALID_ARGUMENT (-1)
#define GWAMD_E_RUNTIME (-2)
#define GWAMD_E_HIP (-3)
#endif

#define GWAMD_ALIGNER_HIRSCHBERG_MYERS 0 /* create_aligner(global_alignment) */
#define GWAMD_ALIGNER_MYERS 1            /* AlignerGlobalMyers (full matrix) */
#define GWAMD_ALIGNER_MYERS_BANDED 2     /* AlignerGlobalMyersBanded */
#define GWAMD_ALIGNER_UKKONEN 3          /* AlignerGlobalUkkonen (p = 100) */

typedef struct gwamd_aligner gwamd_aligner;
typedef struct gwamd_device_allocator gwamd_device_allocator;

const char* gwamd_last_error(void);

/* alignment_type: 0 = global_alignment (the only type the reference
 * implements); stream: a hipStream_t (NULL = default stream). */
int32_t gwamd_aligner_create(gwamd_aligner** out, int32_t max_query_length, int32_t max_target_length,
                             int32_t max_alignments, int32_t alignment_type, int32_t algorithm, void* stream,
                             int32_t device_id, int64_t max_device_memory_allocator_caching_size);
void gwamd_aligner_destroy(gwamd_aligner* aligner);

/* DefaultDeviceAllocator pool (create_default_device_allocator): a byte budget
 * of max_caching_size (-1: all available device memory) shared by every
 * aligner created with it; each aligner reserves its device bytes (fixed
 * buffers + as many workspace slots as fit) until it is destroyed, and
 * creation fails (GWAMD_E_RUNTIME) when the fixed buffers and one slot do not
 * fit what is left.  The handle may be destroyed while aligners still use
 * the pool (they keep it alive). */
int32_t gwamd_device_allocator_create(gwamd_device_allocator** out, int64_t max_caching_size);
void gwamd_device_allocator_destroy(gwamd_device_allocator* allocator);
int64_t gwamd_device_allocator_capacity(const gwamd_device_allocator* allocator);
int64_t gwamd_device_allocator_used(const gwamd_device_allocator* allocator);
/* the default max_caching_size of create_default_device_allocator (2 GiB) */
int64_t gwamd_device_allocator_default_size(void);
int32_t gwamd_aligner_create_with_allocator(gwamd_aligner** out, int32_t max_query_length, int32_t max_target_length,
                                            int32_t max_alignments, int32_t alignment_type, int32_t algorithm,
                                            void* stream, int32_t device_id, gwamd_device_allocator* allocator);

int32_t gwamd_aligner_add_alignment(gwamd_aligner* aligner, const char* query, int32_t query_length,
                                    const char* target, int32_t target_length, int32_t reverse_complement_query,
                                    int32_t reverse_complement_target);
int32_t gwamd_aligner_align_all(gwamd_aligner* aligner);
int32_t gwamd_aligner_sync_alignments(gwamd_aligner* aligner);
int32_t gwamd_aligner_num_alignments(const gwamd_aligner* aligner);

/* Alignment i after sync: states (AlignmentState, start -> end) into
 * states[0..cap); returns the alignment length (states untouched if cap is
 * too small); *status receives the alignment's StatusType. */
int32_t gwamd_aligner_get_alignment(gwamd_aligner* aligner, int32_t i, int8_t* states, int32_t cap,
                                    int32_t* status);
/* Query and target of alignment i as stored by add_alignment (reverse-
 * complemented when requested): Alignment::get_query_sequence /
 * get_target_sequence (alignment.hpp:53-56).  Pointers stay valid until reset. */
int32_t gwamd_aligner_get_sequences(gwamd_aligner* aligner, int32_t i, const char** query, int32_t* query_length,
                                    const char** target, int32_t* target_length);
/* CIGAR of alignment i, NUL-terminated if it fits; returns its length. */
int32_t gwamd_aligner_get_cigar(gwamd_aligner* aligner, int32_t i, char* buf, int32_t cap);
void gwamd_aligner_reset(gwamd_aligner* aligner);

/* AlignmentImpl(query, target) with the given AlignmentState sequence (start ->
 * end): format_alignment(maximal_line_length) writes the three NUL-terminated
 * rows (query with '-', pairing '|'/'x'/' ', target with '-') when their
 * length is below cap; returns that length.  No device work. */
int32_t gwamd_alignment_format(const char* query, int32_t query_length, const char* target, int32_t target_length,
                               const int8_t* states, int32_t num_states, int32_t maximal_line_length,
                               char* query_out, char* pairing_out, char* target_out, int32_t cap,
                               int32_t* linebreak_after);
/* convert_to_cigar of the given AlignmentState sequence; returns its length. */
int32_t gwamd_alignment_cigar(const int8_t* states, int32_t num_states, char* buf, int32_t cap);

/* bench.py helpers: align_all == upload + launch + download. */
int32_t gwamd_aligner_upload(gwamd_aligner* aligner);
int32_t gwamd_aligner_launch(gwamd_aligner* aligner);
int32_t gwamd_aligner_download(gwamd_aligner* aligner);
int32_t gwamd_aligner_synchronize(gwamd_aligner* aligner);
/* Raw device results (copied to host by download): path i (emitted end ->
 * start) at paths + i * stride, length lengths[i]. */
int32_t gwamd_aligner_get_paths(gwamd_aligner* aligner, const int8_t** paths, const int32_t** lengths,
                                int32_t* stride);
/* Resident workgroups of the kernel (persistent grid) and device bytes. */
int32_t gwamd_aligner_get_config(const gwamd_aligner* aligner, int32_t* grid, int64_t* device_bytes);

/* Length limits of this implementation (the reference has none,
 * aligner_global_hirschberg_myers.cpp:47-51): gwamd_aligner_create throws
 * std::invalid_argument (GWAMD_E_INVALID_ARGUMENT) above them.  Hirschberg-
 * Myers and full Myers: 2^24 bases each (full Myers also needs one pair's
 * score matrix, 0.375 B per cell, within a 32 GiB workspace slot); banded
 * Myers and Ukkonen: 65,536 each (sequences, or patterns and target codes,
 * in LDS; Ukkonen bands up to 4,096 rows).  *max_query and *max_target
 * receive the query and target limits. */
int32_t gwamd_aligner_max_lengths(int32_t algorithm, int32_t* max_query, int32_t* max_target);

/* Whether gwamd_aligner_create(algorithm, max_query_length,
 * max_target_length, ...) passes this implementation's length checks: the
 * two limits of gwamd_aligner_max_lengths are not jointly valid for full
 * Myers (its (word, column) matrix of one pair must fit a 32 GiB slot, about
 * Q * T <= 9e10) nor for Ukkonen (band rows).  1 fits, 0 does not, or
 * GWAMD_E_INVALID_ARGUMENT. */
int32_t gwamd_aligner_pair_fits(int32_t algorithm, int32_t max_query_length, int32_t max_target_length);

/* Kernel time of the last gwamd_aligner_align_all (ms; waits for it): the
 * union of its launches' intervals, measured with HIP events on the streams
 * they ran on (large batches run as up to 8 pipelined stages whose kernels
 * alternate between two streams; banded Myers batches of a few long pairs run
 * their band doubling ahead in a first launch).
 * NULL arguments: GWAMD_E_INVALID_ARGUMENT. */
int32_t gwamd_aligner_last_kernel_ms(gwamd_aligner* aligner, double* ms);

/* Path counters of this aligner, accumulated over its launches:
 * *hbm_state_sweeps = banded Myers band sweeps whose 32-word chunk state went
 * through HBM (bands wider than the LDS chunk-state region);
 * *ukkonen_wide_pairs = Ukkonen pairs aligned by the workgroup kernel (batches
 * whose widest band exceeds one wave's 512 rows);
 * *ukkonen_max_rows_per_thread = the most band rows one thread of that kernel
 * held (1-4).  Counters are 64-bit on the device.  NULL outputs:
 * GWAMD_E_INVALID_ARGUMENT. */
int32_t gwamd_aligner_get_stats(gwamd_aligner* aligner, int64_t* hbm_state_sweeps, int64_t* ukkonen_wide_pairs,
                                int64_t* ukkonen_max_rows_per_thread);

#ifdef __cplusplus
}
#endif

#endif /* GWAMD_CUDAALIGNER_H */
