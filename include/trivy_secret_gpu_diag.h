/* trivy_secret_gpu_diag.h -- diagnostic and test hooks of libtrivy_secret_gpu.so.
 *
 * NOT part of the drop-in ABI (include/trivy_secret_gpu.h): these entry points
 * expose the compiled rule tables (anchors, scan automaton, verify DFAs / NFAs,
 * path DFAs, k_scan_big's blob) and the host Go-regexp VM so that the tests and
 * tools can check them against the oracle on the CPU.  A Trivy integration never
 * calls them; they follow the same conventions (TSG_OK / error codes,
 * tsg_last_error, no aborts).
 */
#ifndef TRIVY_SECRET_GPU_DIAG_H
#define TRIVY_SECRET_GPU_DIAG_H

#include "trivy_secret_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Anchor diagnostics for rule i: mode 0 = never matches, 1 = anchored, 2 = full scan. */
int tsg_ruleset_rule_info(const tsg_ruleset* rs, size_t i, int* mode, uint32_t* anchor_min,
                          uint32_t* anchor_max, size_t* n_literals);

/* Anchor literal k (< n_literals) of rule i: ASCII-lowercased bytes and the
 * per-byte case requirement (0 = either case), each *len bytes (<= cap). */
int tsg_ruleset_rule_literal(const tsg_ruleset* rs, size_t i, size_t k, char* lower, char* req, size_t cap,
                             size_t* len);

/* Scan-automaton pattern k (k < n_patterns of tsg_ruleset_stats): its
 * lowercased literal (*len bytes into `lower`), the class positions the
 * k_scan_fast automaton requires right after it (*ext <= 8) with their 6-bit
 * fold-column masks (cols[0..ext)), and the automaton's state count. */
int tsg_ruleset_scan_pattern(const tsg_ruleset* rs, size_t k, char* lower, size_t cap, size_t* len, uint32_t* ext,
                             uint64_t* cols, uint32_t* fast_states);

/* k_scan_fast's LDS image: up to cap bytes into buf, *len = its size (0 when
 * the ruleset has no fast image), *out_entry = the first output state's entry. */
int tsg_ruleset_scan_image(const tsg_ruleset* rs, uint8_t* buf, size_t cap, size_t* len, uint32_t* out_entry);

/* k_scan_fast's keyword states: output states whose every output is a
 * keyword-only pattern the scan resolves itself (no k_report event), and the
 * keywords they set (lowercased, each NUL-terminated, into buf up to cap). */
int tsg_ruleset_kw_states(const tsg_ruleset* rs, uint32_t* n_states, uint32_t* n_keywords, char* buf, size_t cap);

/* Instruction count and capture slots of rule i's compiled regex. */
int tsg_ruleset_rule_prog(const tsg_ruleset* rs, size_t i, uint32_t* n_inst, uint32_t* n_cap);

/* Secret-group span rule of rule i: when *valid, the group of every ASCII
 * match [ms, me) is [ms + *pre, me - *suf), *len filling a side that is -1
 * (k_verify then skips the capture search); *valid = 0: the search decides. */
int tsg_ruleset_group_span(const tsg_ruleset* rs, size_t i, int* valid, int* pre, int* len, int* suf);
/* Byte-run secret-group rule of rule i, used when tsg_ruleset_group_span is
 * not valid (diagnostics / tests): on an ASCII match [ms, me) the group ends
 * where the trailing run of s_alpha bytes begins and starts *len bytes before
 * that (a group of fixed length) or, with *len == -1, where the run of b_alpha
 * bytes before its end begins (never below ms).  s_alpha / b_alpha: 4 u32
 * words each (bit b = ASCII byte b).  Replaces the capture search of
 * getMatchSubgroupsLocations (pkg/fanal/secret/scanner.go:150-163) for such
 * rules. */
int tsg_ruleset_group_run(const tsg_ruleset* rs, size_t i, int* valid, int* len, uint32_t* s_alpha,
                          uint32_t* b_alpha);
/* MatchString of rule i's path regex (which = 0), its first allow-path regex
 * (which = 1) or the i-th global allow path (which = 2) through the DFA the
 * path gate walks (diagnostics / tests):
 * *result 1 = match, 0 = none, 2 = no DFA or undecidable (the Pike VM
 * decides).  Replaces regexp.MatchString in Rule.MatchPath / AllowPath
 * (pkg/fanal/secret/scanner.go:391,397). */
int tsg_ruleset_path_dfa_check(const tsg_ruleset* rs, size_t i, int which, const uint8_t* path, size_t len,
                               int* result);

/* k_scan_big's LDS blob replayed on the CPU (diagnostics / tests): the text
 * walked through the keyword/anchor automaton's table and through the blob
 * (dense rows + cold-state records, frequency or, bfs != 0, breadth-first
 * state numbering); *mismatches = steps where they disagree (state or output
 * bit), *cold_hops = cold records read, *n_dense = dense rows.
 * TSG_ERR_UNSUPPORTED when the automaton has no blob shape. */
int tsg_ruleset_big_check(const tsg_ruleset* rs, const uint8_t* text, size_t len, int bfs, uint64_t* mismatches,
                          uint64_t* cold_hops, uint32_t* n_dense);

/* The k_scan_big blob validator (run before every upload and at
 * tsg_ruleset_compile) on this ruleset's blob with one invariant broken:
 * kind 1 = a failure-link cycle, 2 = an unterminated overflow list, 3 = a dense
 * entry past the last state, 4 = a cold record class past the class count,
 * 0 = unmodified.  *rc = TSG_OK (accepted) or TSG_ERR_INTERNAL (rejected). */
int tsg_ruleset_big_forge_check(const tsg_ruleset* rs, int kind, int* rc);

/* Visits per state of the keyword / anchor automaton walked over a host text
 * (dense-row selection studies for k_scan_big): counts[n >= states], in the
 * k_scan_big blob's numbering when blob != 0 (*n_dense = its dense rows: the
 * ids at or past it are cold states), else in the automaton's own. */
int tsg_ruleset_ac_visits(const tsg_ruleset* rs, const uint8_t* text, size_t len, int blob, uint64_t* counts,
                          size_t n, uint32_t* n_dense);

/* k_scan_big's blob keeps at least n cold-state records in LDS (default
 * 4096); the rest are read from global memory.  Applies to blobs built after
 * the call (rulesets compiled / first uploaded later); *previous = the old
 * floor.  A GPU test sets 0 to send nearly every cold record to global. */
int tsg_big_cold_lds_floor(uint32_t n, uint32_t* previous);

/* Candidate filter of rule i, run on host text from anchor position h:
 * *accept = 0 only when no match of the rule can contain an anchor hit at h
 * (k_expand drops such hits); *n_states = its DFA size (0 = no filter). */
int tsg_ruleset_follow_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t h,
                             int* accept, uint32_t* n_states);

/* Verify DFA of rule i, anchored at s on host text: *result = 1 (match
 * [s, *me)), 0 (none) or 2 (undecidable by the DFA: the Pike VM decides);
 * *n_states = its size (0 = the rule always uses the VM). */
int tsg_ruleset_dfa_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s,
                          int* result, size_t* me, uint32_t* n_states);

/* The same anchored walk with k_verify's run acceleration (a state whose
 * entry is the same on all but <= 3 ASCII bytes skips runs of the others with
 * vector compares), restated on the host: *result / *me as
 * tsg_ruleset_dfa_check's, *skipped = bytes stepped over by skips. */
int tsg_ruleset_dfa_accel_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s,
                                int* result, size_t* me, uint64_t* skipped);

/* Bit-parallel Glushkov NFA of rule i (the verify fallback for rules whose
 * DFA state count explodes, or with \b / (?m) assertions), on host text with
 * threads started at every boundary in [s, inj_hi]: *result = 1 (anchored,
 * inj_hi == s: the match from s ends at *me and nowhere else; unanchored: a
 * match ends at *me first), 0 (none) or 2 (undecidable: the Pike VM decides);
 * *n_pos = its positions (0 = the rule has no NFA). */
int tsg_ruleset_nfa_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s, size_t inj_hi,
                          int* result, size_t* me, uint32_t* n_pos);

/* Automaton diagnostics: states/classes of the keyword+anchor automaton and
 * whether it fits k_scan_fast's LDS image (fast_path = 1). */
int tsg_ruleset_stats(const tsg_ruleset* rs, uint32_t* n_states, uint32_t* n_classes, uint32_t* n_patterns,
                      uint32_t* n_keywords, int* fast_path);

/* Host-side path regex evaluation (per-file, not per-byte): Go MatchString. */
int tsg_regex_match(const char* pattern, const uint8_t* text, size_t len, int* matched);
/* Host-side FindAllIndex for diagnostics/tests of the compiler + VM: writes
 * up to cap (start,end) pairs. */
int tsg_regex_find_all(const char* pattern, const uint8_t* text, size_t len, int64_t* pairs,
                       size_t cap, size_t* n_out);

/* Route every verify job list through k_verify_fast / k_verify_slow /
 * k_allow (on != 0), not only long lists (tests of the split on small
 * batches); 0 restores the default. */
int tsg_engine_force_verify_split(tsg_engine* e, int on);

/* The engine's post-scan key-value sort (sort_pairs) on host arrays: n
 * (key, value) pairs ordered by key bits [0, end_bit), stable --
 * hipcub::DeviceRadixSort::SortPairs' contract; small != 0 takes the
 * two-launch LDS sort up to 64 K pairs (measured slower, not the product's
 * path; tests/test_gpu_small_sort.py checks both). */
int tsg_diag_sort_pairs(tsg_engine* e, const uint64_t* keys, const uint32_t* vals, size_t n, int end_bit,
                        uint64_t* out_keys, uint32_t* out_vals, int small);

#ifdef __cplusplus
}
#endif

#endif /* TRIVY_SECRET_GPU_DIAG_H */
