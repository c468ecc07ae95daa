/*
 * trivy_secret_gpu.h — C ABI of the MI355X secret-scanning engine.
 *
 * Drop-in backend for Trivy's secret scanner hot path:
 *   pkg/fanal/secret/scanner.go:315  func NewScanner(config *Config) Scanner
 *   pkg/fanal/secret/scanner.go:371  func (s *Scanner) Scan(args ScanArgs) types.Secret
 *   pkg/fanal/analyzer/secret/secret.go:79  (*SecretAnalyzer).Analyze  (batched caller)
 *
 * Plain C types only (no torch / HIP types in signatures) so that a cgo shim
 *  can bind it directly.  Conventions:
 *   - every entry point returns an int status (TSG_OK = 0) and never aborts;
 *     tsg_last_error() returns a thread-local message for the last failure;
 *   - caller memory is never retained after a call returns;
 *   - a compiled tsg_ruleset is immutable and may be shared across threads;
 *     a tsg_engine serialises calls made on it (one HIP stream per engine).
 */
#ifndef TRIVY_SECRET_GPU_H
#define TRIVY_SECRET_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_OK 0
#define TSG_ERR_INVALID_ARG 1
#define TSG_ERR_REGEX 2       /* "regexp compile error" (scanner.go:77) */
#define TSG_ERR_DEVICE 3      /* HIP runtime failure */
#define TSG_ERR_NO_DEVICE 4   /* no MI355X visible: the product path does not fall back to CPU */
#define TSG_ERR_UNSUPPORTED 5 /* rule feature outside this engine's coverage (e.g. a non-ASCII keyword) */
#define TSG_ERR_INTERNAL 6
#define TSG_ERR_PANIC 7       /* input on which the Go reference panics (secret group did not participate) */
#define TSG_ERR_FULL 8        /* tsg_staging_add: the staging buffer has no room for the file */

/* AllowRule — pkg/fanal/secret/scanner.go:191-196 (Description stays host-side). */
typedef struct tsg_allow_rule {
  const char* id;
  const char* regex; /* Go RE2 syntax applied to the whole match text, or NULL */
  const char* path;  /* Go RE2 syntax applied to the file path, or NULL */
} tsg_allow_rule;

/* Rule — pkg/fanal/secret/scanner.go:84-95.  Category/Title/Severity are
 * report metadata the host keeps; the engine needs only these fields. */
typedef struct tsg_rule {
  const char* id;
  const char* regex; /* NULL => FindLocations returns nothing (scanner.go:98-100) */
  const char* const* keywords;
  size_t n_keywords;
  const char* path;              /* NULL => every path (scanner.go:165-167) */
  const char* secret_group_name; /* NULL or "" => whole match (scanner.go:102-104) */
  const tsg_allow_rule* allow_rules;
  size_t n_allow_rules;
  const char* const* exclude_regexes; /* Rule.ExcludeBlock.Regexes */
  size_t n_exclude_regexes;
} tsg_rule;

typedef struct tsg_ruleset tsg_ruleset;
typedef struct tsg_engine tsg_engine;
typedef struct tsg_result tsg_result;

/* ScanArgs — scanner.go:361-364 (Content already CR-stripped by the caller,
 * as analyzer/secret/secret.go:91 does). */
typedef struct tsg_file {
  const uint8_t* data;
  uint64_t len;
  const char* path;
} tsg_file;

/* One kept Location (scanner.go:223-226) after allow + exclude filtering. */
typedef struct tsg_loc {
  uint32_t file;       /* index into the batch */
  uint32_t rule;       /* index into the ruleset's rules (config order) */
  uint64_t start, end; /* byte offsets into the file content */
  uint32_t start_line; /* findLocation (scanner.go:481-537), 1-based */
  uint32_t end_line;
} tsg_loc;

/* One types.Line (pkg/fanal/types/misconf.go:53-62); Highlighted == Content. */
typedef struct tsg_line {
  uint32_t number;
  const char* content;
  size_t content_len;
  uint8_t is_cause, first_cause, last_cause;
} tsg_line;

/* One types.SecretFinding (pkg/fanal/types/secret.go:10-20) minus the rule
 * metadata the host owns (look it up by `rule`). */
typedef struct tsg_finding {
  uint32_t file;
  uint32_t rule;
  uint32_t start_line, end_line;
  const char* match; /* censored line window */
  size_t match_len;
  const tsg_line* lines;
  size_t n_lines;
  uint64_t start, end;
} tsg_finding;

/* Per-file flags in a result. */
#define TSG_FILE_PATH_ALLOWED 1u /* Global.AllowPath matched: Secret{FilePath} without findings (scanner.go:375-379) */
#define TSG_FILE_SPECIAL 2u      /* content holds U+0130/U+017F/U+212A: keywords and anchor literals spelled
                                    with them were re-checked around each occurrence (k_fold_windows) */
#define TSG_FILE_BINARY 4u       /* tsg_analyze: utils.IsBinary (utils.go:77-95) -> skipped, Analyze returns nil */

const char* tsg_version(void);
const char* tsg_last_error(void);

/* NewScanner: compile rules (builtin ∪ custom, already filtered by the caller
 * exactly as scanner.go:315-359 does), global allow rules and the global
 * exclude block. */
int tsg_ruleset_compile(const tsg_rule* rules, size_t n_rules, const tsg_allow_rule* allow_rules,
                        size_t n_allow_rules, const char* const* exclude_regexes,
                        size_t n_exclude_regexes, tsg_ruleset** out, char* err, size_t errlen);
void tsg_ruleset_free(tsg_ruleset* rs);
size_t tsg_ruleset_rule_count(const tsg_ruleset* rs);
/* Engine bound to one GPU (one process per GPU; `device` is the HIP ordinal). */
int tsg_engine_create(int device, tsg_engine** out);
void tsg_engine_free(tsg_engine* e);

/* Scan a batch of host files: pack -> H2D -> kernels -> D2H -> findings. */
int tsg_scan(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files,
             tsg_result** out);

/* Scan a batch already resident in HBM (device pointers).  Layout: files are
 * stored back to back, each followed by ONE NUL separator byte:
 *   content of file i = d_data[d_offsets[i] .. d_offsets[i+1] - 1), d_data[d_offsets[i+1] - 1] == 0,
 *   path of file i    = d_paths[d_path_offsets[i] .. d_path_offsets[i+1]).
 * (The separator resets the keyword automaton so no literal spans two files;
 * NUL bytes inside content are fine.)  Produces locs with line numbers and
 * the full findings: censoring, Match and Code (scanner.go:425-537) are cut
 * from the batch on the device, and only the records and their strings come
 * back (tsg_result_findings). */
int tsg_scan_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data,
                    const uint64_t* d_offsets, const uint8_t* d_paths,
                    const uint64_t* d_path_offsets, size_t n_files, tsg_result** out);

size_t tsg_result_loc_count(const tsg_result* r);
const tsg_loc* tsg_result_locs(const tsg_result* r);
size_t tsg_result_file_count(const tsg_result* r);
const uint8_t* tsg_result_file_flags(const tsg_result* r);
/* Findings of file i in Scan order (sorted by RuleID, then Match). */
size_t tsg_result_findings(const tsg_result* r, size_t file, const tsg_finding** out);
/* Per-stage device timings of the last scan, milliseconds. */
int tsg_result_timings(const tsg_result* r, double* ms, size_t n, size_t* n_out);
void tsg_result_free(tsg_result* r);

/* SecretAnalyzer.Analyze (pkg/fanal/analyzer/secret/secret.go:79-113) over a
 * batch of RAW files, the per-file work on the GPU: the utils.IsBinary gate on
 * the first min(len, 300) bytes (utils.go:77-95; binary files get
 * TSG_FILE_BINARY and no locations), deletion of every '\r'
 * (secret.go:91, bytes.ReplaceAll) by stream compaction in HBM, then the scan.
 * files[i].path is the FilePath the findings carry: the caller applies
 * secret.go:95-98 (the '/' prefix when AnalysisInput.Dir is empty).  Offsets
 * and line numbers of the result refer to the CR-stripped content, exactly as
 * Analyze hands it to Scan; findings are built from it. */
int tsg_analyze(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files, tsg_result** out);

/* Caller-filled staging: a page-locked batch buffer the caller reads files
 * straight into (read(2) / io.ReadFull into *dst), so a batch costs one host
 * write per byte and one H2D, with no intermediate copy or pack (tsg_scan /
 * tsg_analyze pack the caller's buffers into the engine's own staging).
 * tsg_staging_add reserves `len` bytes for one file (its NUL separator is
 * written by the library) and returns where to put them; TSG_ERR_FULL when
 * the buffer has no room -- run the batch, tsg_staging_reset, add again (a
 * file larger than the whole buffer needs a larger staging or tsg_scan).
 * A staging belongs to its caller and may be used with any engine; it must
 * not be written while a staged call on it runs.  tsg_analyze_staged is
 * tsg_analyze over the staged RAW files (IsBinary, '\r' strip, Scan),
 * tsg_scan_staged is tsg_scan over CR-stripped ones; file i of the result is
 * the i-th file added since the last reset. */
typedef struct tsg_staging tsg_staging;
int tsg_staging_create(size_t capacity_bytes, tsg_staging** out);
int tsg_staging_add(tsg_staging* st, const char* path, uint64_t len, uint8_t** dst);
size_t tsg_staging_count(const tsg_staging* st);
size_t tsg_staging_bytes(const tsg_staging* st); /* contents + one separator per file */
void tsg_staging_reset(tsg_staging* st);
void tsg_staging_free(tsg_staging* st);
int tsg_analyze_staged(tsg_engine* e, const tsg_ruleset* rs, const tsg_staging* st, tsg_result** out);
int tsg_scan_staged(tsg_engine* e, const tsg_ruleset* rs, const tsg_staging* st, tsg_result** out);

/* Byte-range split of ONE large file across GPUs (the reference
 * scans a file of any size whole, scanner.go:371-452, and the walker spools
 * tar entries >= 100 MiB to disk and still scans them, walker/cached_file.go:36-52).
 * Every rank runs the scan pass over its byte range [own_lo, own_hi) and
 * exports that range's scan state (keyword bits, the anchor hits whose
 * literal starts inside it, per-4 KiB newline counts); the file's owner
 * merges the parts and runs candidates / FindAll / exclude / lines / findings
 * over the whole file, so the result equals tsg_scan_device on the whole file.
 *
 * tsg_part_halo: the view a part must see, *left bytes before own_lo (clipped
 * at 0) and *right bytes after own_hi (clipped at the file end). */
int tsg_part_halo(const tsg_ruleset* rs, uint64_t* left, uint64_t* right);

/* d_text = file bytes [text_base, text_base + text_len) in HBM, plus one more
 * readable byte: the file's next byte, or the NUL separator when the view
 * reaches the file end (checked: TSG_ERR_INVALID_ARG otherwise; only literals
 * starting past own_hi touch it, and the next part owns those).  text_base and
 * own_lo are multiples of 4096; own_hi is too unless it is file_len.  *blob
 * (free with tsg_part_free) is opaque and position-independent: ship it to the
 * owner with any transport. */
int tsg_scan_part_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_text, uint64_t text_base,
                         uint64_t text_len, uint64_t own_lo, uint64_t own_hi, uint64_t file_len,
                         const char* path, uint8_t** blob, size_t* blob_len);
void tsg_part_free(uint8_t* blob);

/* The owner: d_file = the whole file in HBM followed by its NUL separator
 * (d_file[file_len] == 0); the parts must tile [0, file_len) (any order).
 * The result is a one-file result (file index 0), as tsg_scan_device's.
 * Files of any size up to the batch limit (2^44 bytes) merge: the match search
 * runs 64-bit positions for files past 2^31 - 1 bytes.  The one limit, as for
 * every entry point that verifies: a single match of 4 GiB or more (its allow
 * regexes run on 32-bit match strings) returns TSG_ERR_UNSUPPORTED. */
int tsg_scan_merge_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_file, uint64_t file_len,
                          const char* path, const uint8_t* const* blobs, const size_t* blob_lens, size_t n_parts,
                          tsg_result** out);

/* Prefilter-only pass (BASELINE.json configs[1]): per-file rule gate bitmasks
 * (rule i passes iff bit i set), exactly MatchKeywords (scanner.go:169-181). */
int tsg_gate_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data,
                    const uint64_t* d_offsets, size_t n_files, uint32_t* h_gates_out,
                    size_t gate_words_per_file);

/* Timings of the engine's last tsg_gate_device call, milliseconds, in the
 * tsg_result_timings layout: [0] scan + report + special gate, [7] generic scan
 * kernel, [17] k_scan_fast alone, [15] whole call (host clock). */
int tsg_engine_gate_timings(const tsg_engine* e, double* ms, size_t n, size_t* n_out);

/* ---- container-image layers (walker.LayerTar.Walk, pkg/fanal/walker/tar.go:35-103) ----
 * Walks a layer tar already in host memory without copying it: opaque-dir
 * markers and whiteouts are collected (tar.go:51-61), SkipDirs/SkipFiles are
 * doublestar globs (walk.go:28-53, CleanSkipPaths applied here), and every
 * remaining directory and regular file is an entry in archive order whose
 * content is tar[offset .. offset+size).  Regular-file entries go straight to
 * tsg_analyze as tsg_file spans (path "/" + entry path: the image artifact
 * calls AnalyzeFile with Dir "", secret.go:95-98).  A malformed archive
 * returns -1 with "failed to extract the archive: ..." (tar.go:43). */
typedef struct tsg_tar_entry {
  const char* path; /* path.Clean'd, leading '/' trimmed (tar.go:47-49) */
  size_t path_len;
  uint64_t offset; /* content start in the caller's tar (0 for directories) */
  uint64_t size;
  uint32_t mode;
  uint8_t is_dir;
} tsg_tar_entry;
typedef struct tsg_tar_walk tsg_tar_walk;

int tsg_layer_tar_walk(const uint8_t* tar, size_t len, const char* const* skip_files, size_t n_skip_files,
                       const char* const* skip_dirs, size_t n_skip_dirs, tsg_tar_walk** out);
size_t tsg_tar_walk_entry_count(const tsg_tar_walk* w);
const tsg_tar_entry* tsg_tar_walk_entries(const tsg_tar_walk* w);
size_t tsg_tar_walk_opq_count(const tsg_tar_walk* w);
const char* tsg_tar_walk_opq_dir(const tsg_tar_walk* w, size_t i);
size_t tsg_tar_walk_wh_count(const tsg_tar_walk* w);
const char* tsg_tar_walk_wh_file(const tsg_tar_walk* w, size_t i);
void tsg_tar_walk_free(tsg_tar_walk* w);
/* One walked layer through the secret analyzer in ONE tsg_analyze call:
 * directories dropped (AnalyzerGroup.AnalyzeFile, analyzer.go:398-400),
 * SecretAnalyzer.Required per regular file (secret.go:115-153: size, skip
 * dirs/files/extensions, the config file's base name, global AllowPath with
 * the ruleset's allow-path regexes on the host), content handed over as spans
 * of `tar`, paths "/"-prefixed.  Result file k is walk entry kept[k]
 * (kept: capacity tsg_tar_walk_entry_count; may be NULL). */
int tsg_analyze_layer(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* tar, size_t len,
                      const tsg_tar_walk* w, const char* config_path, uint32_t* kept, size_t* n_kept,
                      tsg_result** out);
/* Global AllowRules.AllowPath (scanner.go:200-207) on the host, per file. */
int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t len, int* allowed);
/* doublestar.Match (bmatcuk/doublestar v4, walk.go:43): 1/0 in *matched; -1 on a bad pattern. */
int tsg_glob_match(const char* pattern, const char* path, int* matched);

#ifdef __cplusplus
}
#endif

#endif /* TRIVY_SECRET_GPU_H */
