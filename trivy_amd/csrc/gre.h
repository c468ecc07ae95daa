// gre — a Go-RE2-syntax regex compiler for the MI355X secret engine.
//
// Parses Go regexp/syntax patterns (the `Perl` flag set regexp.Compile uses:
// ClassNL | OneLine | PerlX | UnicodeGroups) and compiles them into a
// rune-level instruction program with Go's priorities (regexp/syntax
// compile.go + simplify.go semantics), executed by the Pike VM in pikevm.h on
// the GPU.  It also derives, per pattern, the literal "anchor" factor the
// batched scanner uses to localise candidate match starts.
//
// Reference call sites whose behaviour this must reproduce:
//   pkg/fanal/secret/scanner.go:70-82   (regexp.Compile of custom rules)
//   pkg/fanal/secret/scanner.go:65-67   (MustCompile of builtin rules)
//   pkg/fanal/secret/scanner.go:107,125,166,202,211,259 (Find*/MatchString)
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "gre_prog.h"

namespace gre {

struct Bitmap256 {
  uint64_t w[4] = {0, 0, 0, 0};
  void set(int b) { w[b >> 6] |= 1ull << (b & 63); }
  bool has(int b) const { return (w[b >> 6] >> (b & 63)) & 1; }
  void set_range(int lo, int hi) { for (int b = lo; b <= hi; ++b) set(b); }
  void merge(const Bitmap256& o) { for (int i = 0; i < 4; ++i) w[i] |= o.w[i]; }
  int count() const { int c = 0; for (int i = 0; i < 4; ++i) c += __builtin_popcountll(w[i]); return c; }
};

constexpr uint32_t kInf = 0xFFFFFFFFu;

// One string of an exact literal set, in the scanner's ASCII-lowercased view.
// `lower` is the lowercased byte string; `req[k]` is 0 when position k matches
// either case, else the exact (original-case) byte required there.
struct Lit {
  std::string lower;
  std::string req;
  bool operator==(const Lit& o) const { return lower == o.lower && req == o.req; }
};

// The anchor factor of a pattern: every match m = [s,e) of the pattern (on a
// file without the special fold bytes C4B0/C5BF/E284AA) contains, at some
// h with a <= h-s <= b, an occurrence of one of `lits` (ASCII-lowercased
// compare + req check), and every byte of [s,h) is in `alpha`.
struct Anchor {
  bool valid = false;
  std::vector<Lit> lits;
  uint32_t off_min = 0, off_max = 0;  // a, b (b may be kInf)
  Bitmap256 alpha;
  double score = -1e9;
};

struct Compiled {
  Prog prog;
  Anchor anchor;
  bool can_match_empty = false;
  uint32_t min_len = 0, max_len = 0;  // bytes
  // The language is exactly the anchor's literal set (no assertions, no other
  // constraint): on ASCII text, MatchString == "some anchor literal occurs".
  bool literal_exact = false;
};

// Compile a Go regexp.  On syntax error returns false and sets *err to a
// message in the style of Go's regexp/syntax errors.
bool compile(const std::string& pattern, Compiled* out, std::string* err);

// Where capture group `slot` sits inside ANY match of the program, from the
// match span alone: on a match [ms, me) whose bytes are all ASCII (one byte
// per rune) the group is [ms + pre, me - suf), with len filling in a missing
// side.  Valid only when the group's CAP pair is unique, on no cycle, and on
// every path to MATCH (it always participates), and each side is fixed: every
// program path gives the same rune count (-1 = not fixed).  Lets k_verify skip
// the capture search for the `(?P<key>..){0,25}..(?P<secret>[..]{N})['"]`
// family of builtin rules (builtin-rules.go), whose group ends one rune before
// the match end.
struct GroupSpan {
  bool valid = false;
  int pre = -1, len = -1, suf = -1;
};
GroupSpan group_span(const Prog& p, uint32_t slot);

// Capture-group span from byte runs at the match's end (the secret-group
// shortcut for groups between variable-length parts, gitleaks' shape
// `kw[..]{0,25}(=|:).{0,5}['"](?P<secret>[0-9a-f]{32})['"]?(\s|$)`): on an
// ASCII match [ms, me), ge = me minus the run of s_alpha bytes ending at me,
// gs = ge minus the run of b_alpha bytes ending at ge (not below ms), or
// ge - len for a group of fixed length len (fixed_len: group_span's len, or
// -1).  Valid when that is exact for every parse (gre.cpp group_run).
struct GroupRun {
  bool valid = false;
  int len = -1;
  uint32_t s_alpha[4] = {0, 0, 0, 0};  // ASCII bytes the program can consume after the group
  uint32_t b_alpha[4] = {0, 0, 0, 0};  // ASCII bytes the group can consume
};
GroupRun group_run(const Prog& p, uint32_t slot, int fixed_len);

// Unicode simple-fold orbit lookup (next member, or r itself when trivial).
uint32_t simple_fold(uint32_t r);

}  // namespace gre
