/* sfs2d_ingest.h -- native VCF(.gz / BGZF) + popmap ingest (host code, C ABI).
 *
 * Replaces the reference's `LikelihoodInference_jointSFS.make_data_dict_vcf(vcf_filename,
 * popinfo_filename)` (uricchio/2DSFS-scan scripts/src/twoDSFS_class.py:36-138; duplicated as
 * scripts/sims_scan.py:18-120), the first step of every scan, which reads the VCF line by line in
 * Python.  Same semantics:
 *   - popmap: `line.strip().split("\t")`, lines with >= 2 columns map column 0 -> column 1 (57-64);
 *   - header `#CHROM` line: every sample found in the popmap appends its population to `poplist`
 *     (81-85); `poplist` is then zipped POSITIONALLY against the sample columns (118);
 *   - records: annotation = 2nd '|' field of INFO else "No annotation" (92-97); FILTER must be
 *     PASS or '.' (101-102); REF and ALT upper-cased must be one of A/C/G/T (104-109); GT index from
 *     FORMAT (115); per sample `gt[::2].count('0')` / `.count('1')` added to its population (120-130);
 *   - records are keyed "CHROM-POS" (89): a repeated key keeps its first position in the dict and
 *     the values of the last record that passed the filters (dict assignment, 134).
 * Errors mirror the reference's exceptions: IndexError (too few columns / GT subfields),
 * ValueError ('GT' not in FORMAT).  Files are read as gzip (one or many members; BGZF blocks are
 * inflated in parallel) or, when the gzip magic is absent, as plain text (the reference would
 * refuse those).  Lines end at "\n", "\r\n" or "\r" (Python text mode).
 *
 * The parse is multithreaded (nthreads <= 0: all hardware threads); results do not depend on the
 * thread count.  Output arrays are borrowed views valid until sfs2d_vcf_free.
 */
#ifndef SFS2D_INGEST_H
#define SFS2D_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFS2D_VCF_OK 0
#define SFS2D_VCF_E_IO -1       /* cannot open / read a file */
#define SFS2D_VCF_E_GZIP -2     /* corrupt gzip stream */
#define SFS2D_VCF_E_INDEX -3    /* reference: IndexError */
#define SFS2D_VCF_E_VALUE -4    /* reference: ValueError */
#define SFS2D_VCF_E_ARG -5
#define SFS2D_VCF_E_MEM -6

typedef struct sfs2d_vcf sfs2d_vcf;

int sfs2d_vcf_read(const char* vcf_path, const char* popmap_path, int nthreads, sfs2d_vcf** out);
void sfs2d_vcf_free(sfs2d_vcf* v);
/* message of the last failed sfs2d_vcf_read on this thread (file line number included) */
const char* sfs2d_vcf_last_error(void);

/* records (= dict keys) in dict insertion order */
int64_t sfs2d_vcf_num_records(const sfs2d_vcf* v);
/* populations in order of first appearance in poplist (= the calls dicts' key order) */
int32_t sfs2d_vcf_num_pops(const sfs2d_vcf* v);
const char* sfs2d_vcf_pop_name(const sfs2d_vcf* v, int32_t i);
/* distinct CHROM strings / annotations, in order of first appearance among the records */
int32_t sfs2d_vcf_num_chroms(const sfs2d_vcf* v);
const char* sfs2d_vcf_chrom_name(const sfs2d_vcf* v, int32_t i);
int32_t sfs2d_vcf_num_annotations(const sfs2d_vcf* v);
const char* sfs2d_vcf_annotation(const sfs2d_vcf* v, int32_t i);

/* per-record columns:
 *   chrom[n]      index into the chromosome names
 *   pos[n]        POS as an integer, or INT64_MIN when the text is not a plain decimal number
 *   pos_text      POS text of record i = pos_blob[pos_off[i] .. pos_off[i+1]) (the key is
 *                 chrom + "-" + that text; it differs from str(pos) e.g. with leading zeros)
 *   ann[n]        index into the annotations
 *   alleles[2n]   upper-case REF, ALT characters
 *   calls[n*P*2]  (ref, alt) allele counts per population, -1 where the population is absent from
 *                 the record's calls dict (records with fewer sample columns than poplist) */
int sfs2d_vcf_columns(const sfs2d_vcf* v, const int32_t** chrom, const int64_t** pos, const char** pos_blob,
                      const int64_t** pos_off, const int32_t** ann, const uint8_t** alleles, const int32_t** calls);

/* The scan-ready packed arrays of two populations straight from the table -- pack_snp_dict(
 * make_data_dict_vcf(...), pop1, pop2) without the dict (twoDSFS_class.py:828-835 order: chromosome
 * name, then integer position) -- for the common file already in that order:
 *   chrom_rank[c]  the rank of chromosome c's name among the sorted names (the caller's sort)
 *   pop1, pop2     population indices, or -1 for a population absent from the popmap (counts 0)
 *   counts[n]      ref1 | alt1 << 8 | ref2 << 16 | alt2 << 24 (a population missing from a record: 0)
 *   pos[n]         POS as uint32;  ann[n]: annotation index as uint16
 * Returns 0 when packed; 1 when the fast path does not apply -- the records are not in scan order,
 * a POS is not a plain decimal or does not fit uint32, an allele count exceeds 255 or there are more
 * than 65535 annotations -- and the caller then packs in its general path (which raises the
 * reference's errors); SFS2D_VCF_E_ARG for bad arguments. */
int sfs2d_vcf_pack(const sfs2d_vcf* v, const int32_t* chrom_rank, int32_t pop1, int32_t pop2, uint32_t* counts,
                   uint32_t* pos, uint16_t* ann);

/* statistics of the last read: bytes of text, data lines, seconds in inflate / parse / merge */
int sfs2d_vcf_stats(const sfs2d_vcf* v, int64_t* text_bytes, int64_t* lines, double* t_inflate, double* t_parse,
                    double* t_merge);

#ifdef __cplusplus
}
#endif

#endif
