/*
 * tsg_corpus.h — the bench / test corpus generator (bench_gen/libtsg_corpus.so).
 *
 * NOT part of the product C ABI (include/trivy_secret_gpu.h): bench.py and the
 * tests load this library on its own to build seeded synthetic corpora in HBM
 *  and their host twins for oracle spot checks.
 */
#ifndef TSG_CORPUS_H
#define TSG_CORPUS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- synthetic corpus (bench / test utility, not the scan path) ----------
 * SURVEY.md §8(d) text model with planted builtin-rule secrets.  The device
 * generator and the host twin produce identical bytes for a (seed, file). */
int tsg_gen_corpus_device(uint8_t* d_data, const uint64_t* d_offsets, const uint64_t* d_chunk_ids,
                          uint64_t n_chunks, uint8_t* d_paths, uint64_t* d_path_offsets, uint64_t n_files,
                          uint64_t seed, double density, void* d_plants, uint64_t plant_cap,
                          unsigned long long* d_nplants);
int tsg_gen_file(uint64_t seed, uint32_t file, uint64_t len, double density, uint8_t* out);
/* As tsg_gen_file, plus the file's plant records (tsg_gen_plant_record_size
 * bytes each: file, template, start, end, kind 0 real / 1 one-char-short
 * decoy / 2 EXAMPLE decoy / 3 K-or-ſ-spelled instance) into plants[0..cap). */
int tsg_gen_file_plants(uint64_t seed, uint32_t file, uint64_t len, double density, uint8_t* out, void* plants,
                        size_t plant_cap, size_t* n_plants);
/* 1 if file `file` of corpus `seed` is one of the 0.1 % carrying non-ASCII runes. */
int tsg_gen_file_nonascii(uint64_t seed, uint32_t file);
/* The planted-secret templates: one per builtin rule; the rule ID of template i. */
size_t tsg_gen_template_count(void);
const char* tsg_gen_template_rule(size_t i);
size_t tsg_gen_plant_record_size(void);
uint32_t tsg_gen_chunk_bytes(void);

#ifdef __cplusplus
}
#endif

#endif /* TSG_CORPUS_H */
