/*
 * gwamd_cudamapper.h -- C ABI of the overlap-alignment caller (libgwamd.so).
 *
 * The reference aligns cudamapper overlaps inside its cudamapper executable
 * (cudamapper/src/main.cu:48-175: run_alignment_batch / align_overlaps) and
 * prints them with print_paf (cudamapper/src/cudamapper_utils.cpp:30-112).
 * A reference-side binding would call these in place of those two functions:
 *
 *   gwamd_align_overlaps   align_overlaps(allocator, overlaps, query_parser,
 *                          target_parser, num_alignment_engines, cigars)   main.cu:125-175
 *   gwamd_read_fasta       io::create_kseq_fasta_parser(path, min_len, shuffle) fasta_parser.hpp:62-64
 *   gwamd_format_paf       print_paf(overlaps, cigars, query_parser,
 *                          target_parser, kmer_size, mutex)                cudamapper_utils.cpp:30-112
 *
 * Reads are passed as one byte array per side with n+1 offsets (read i is
 * bases[offsets[i], offsets[i+1])); names as NUL-separated strings with n+1
 * offsets.  gwamd_overlap has the layout of cudamapper::Overlap
 * (cudamapper/include/.../types.hpp:68-89).  Results are returned in a
 * gwamd_text_list owned by the library (free with gwamd_text_list_free).
 *
 * Error convention: 0 on success, or a negative GWAMD_E_* code where the
 * reference throws (message in gwamd_last_error()).
 */
#ifndef GWAMD_CUDAMAPPER_H
#define GWAMD_CUDAMAPPER_H

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

/* cudamapper::Overlap; relative_strand is '+' (Forward) or '-' (Reverse). */
typedef struct gwamd_overlap
{
    uint32_t query_read_id;
    uint32_t target_read_id;
    uint32_t query_start;
    uint32_t target_start;
    uint32_t query_end;
    uint32_t target_end;
    unsigned char relative_strand;
    uint32_t num_residues;
    uint8_t overlap_complete;
} gwamd_overlap;

typedef struct gwamd_text_list gwamd_text_list;

const char* gwamd_last_error(void);

/* One CIGAR per overlap, in overlap order.  num_alignment_engines host threads
 * (>= 1) share the overlaps; device_id selects the GPU. */
int32_t gwamd_align_overlaps(const char* query_bases, const int64_t* query_offsets, int32_t num_queries,
                             const char* target_bases, const int64_t* target_offsets, int32_t num_targets,
                             const gwamd_overlap* overlaps, int32_t num_overlaps, int32_t num_alignment_engines,
                             int32_t device_id, gwamd_text_list** cigars);

/* The PAF text of print_paf as one entry; cigars may be NULL (no cg:Z: tag). */
int32_t gwamd_format_paf(const char* query_names, const int64_t* query_name_offsets, const int64_t* query_lengths,
                         int32_t num_queries, const char* target_names, const int64_t* target_name_offsets,
                         const int64_t* target_lengths, int32_t num_targets, const gwamd_overlap* overlaps,
                         int32_t num_overlaps, const gwamd_text_list* cigars, int32_t kmer_size,
                         gwamd_text_list** paf);

/* Reads of a FASTA/FASTQ file as io::create_kseq_fasta_parser(path, min_sequence_length,
 * shuffle) holds them (fasta_parser.hpp:62-64; kseqpp_fasta_parser.cpp:31-72): names and
 * sequences in parser order (shuffled with std::mt19937(0) when shuffle != 0). */
int32_t gwamd_read_fasta(const char* path, uint32_t min_sequence_length, int32_t shuffle, gwamd_text_list** names,
                         gwamd_text_list** sequences);
/* A list holding copies of n texts (e.g. CIGARs from another aligner run for gwamd_format_paf). */
int32_t gwamd_text_list_create(const char* const* texts, const int64_t* lengths, int32_t n, gwamd_text_list** out);
/* Entry i of a list (text and length, not NUL terminated beyond length). */
int32_t gwamd_text_list_size(const gwamd_text_list* list);
int32_t gwamd_text_list_get(const gwamd_text_list* list, int32_t i, const char** text, int64_t* length);
void gwamd_text_list_free(gwamd_text_list* list);

#ifdef __cplusplus
}
#endif

#endif /* GWAMD_CUDAMAPPER_H */
