// Internal structures of the MI355X secret engine (not part of the C ABI).
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "gre.h"
#include "trivy_secret_gpu_diag.h"  // (includes trivy_secret_gpu.h)

namespace tsg {

constexpr int kAcMaxLit = 8;   // trie depth; longer patterns are confirmed on hit
constexpr int kFastExtTo = 6;  // scan automaton: short anchor literals extended by classes up to this length
constexpr uint32_t kNlBlock = 4096;  // newline-count granularity (bytes) = one k_scan_fast chain span
constexpr uint32_t kNoKw = 0xFFFFFFFFu;

constexpr uint32_t kFastCols = 64;             // k_scan_fast columns (6-bit folded bytes, engine.hip fold6)
constexpr uint32_t kFastRowBytes = 134;       // 64 u16 columns + 6 B: consecutive rows rotate LDS banks
constexpr uint32_t kFastMaxRows = 1008;
constexpr uint32_t kFastImgMax = kFastMaxRows * kFastRowBytes;  // k_scan_fast image budget (LDS)
constexpr uint32_t kLdsMax = 160 * 1024;      // LDS per CU
constexpr uint32_t kFastSpecialEv = 0xFFFF;   // event tag: U+0130/U+017F/U+212A sequence ends here
constexpr uint32_t kFollowMaxStates = 1024;  // follow-DFA subset-construction budget
constexpr uint32_t kFollowDepth = 96;        // bytes a candidate filter reads past the hit
constexpr uint32_t kNoFollow = 0xFFFFFFFFu;
constexpr uint32_t kDfaMaxStates = 4096;     // verify-DFA budget per rule (else the Pike VM)
constexpr uint32_t kDfaStateMask = 0x1FFF;  // verify-DFA entry: bit15 end-match, bit14 match state
constexpr uint32_t kDfaAccel = 0x2000;      // (device copy) bit13: the entry's state is accelerable (dfa_accel_off)
constexpr uint32_t kDfaRuneSyms = 5;        // verify-DFA rune symbols: K, ſ, İ, U+FFFD, other non-ASCII

enum RuleMode : uint8_t { MODE_NEVER = 0, MODE_ANCHORED = 1, MODE_FULL = 2 };

// ---- device-visible POD records ------------------------------------------
struct RuleDev {
  uint32_t prog;        // program index
  uint32_t kw_off, kw_n;  // keyword ids (kw_n == 0 => no gate)
  uint32_t gate_always;   // empty keyword present => gate passes
  uint32_t mode;
  uint32_t off_min, off_max;  // anchor offset range
  uint64_t alpha[4];          // anchor prefix alphabet
  uint32_t group_off, group_n;  // capture slots of groups named SecretGroupName
  uint32_t allow_off, allow_n;  // per-rule allow regex progs
  uint32_t use_groups;          // SecretGroupName != ""
  uint32_t max_len;             // longest possible match in bytes (gre::kInf if unbounded)
  uint32_t follow_off;          // candidate filter: first u16 of its table (kNoFollow = none)
  uint32_t follow_ncls;         // its byte classes; class map at follow_cls_off (128 B)
  uint32_t follow_cls_off;
  uint32_t gate_implied;        // every anchor literal contains a keyword: on files without fold-special
                                // bytes a match implies the MatchKeywords gate (scanner.go:169-181)
  uint32_t dfa_off;             // verify DFA (dfa.cpp): first u16 of its table (kNoFollow = none)
  uint32_t dfa_ncls, dfa_cls_off, dfa_match_off;
  uint32_t dfa_accel_off;   // per state u32 index of its run-acceleration record (~0: none), in dfa_bytes
  uint32_t dfa_accel_recs;  // the 32-byte records (stay bitmap, stay class), 16-aligned in dfa_bytes
  uint32_t dfa_start0, dfa_start1;  // start state at s > 0 / s == 0 (BeginText)
  uint32_t dfa_first[4];        // ASCII bytes on which a start state does not die (k_verify start skip)
  uint32_t dfa_size;            // u16 entries of its table (k_verify stages it in LDS when it fits)
  uint32_t dfa_smatch;          // bit 0/1: start0/start1 is a match state
  uint32_t dfa_sym;             // first rune-symbol column | 0x80000000 when other non-ASCII runes are one symbol
  // secret group from the match span alone (gre::group_span; one group, ASCII
  // matches): group = [ms + grp_pre, me - grp_suf), grp_len filling a missing
  // side; grp_fast = 0 -> the capture search (k_captures)
  uint32_t grp_fast;
  int32_t grp_pre, grp_len, grp_suf;
  // else, by byte runs (gre::group_run; one group, ASCII matches): ge = me
  // minus the run of grp_s bytes ending at me, gs = ge minus the run of grp_b
  // bytes ending at ge; grp_run = 0 -> the capture search
  uint32_t grp_run;
  int32_t grp_run_len;  // >= 0: a group of fixed length (gs = ge - len)
  uint32_t grp_s[4], grp_b[4];
  uint32_t id_rank;  // position of the rule ID in sorted (ID, index) order: findings sort (scanner.go:441-446)
  uint32_t no_nl;    // no instruction of the program consumes '\n': every match lies inside one line
  uint32_t nfa_off;  // bit-parallel NFA (nfa.cpp): byte offset of its NfaDev record (kNoFollow = none)
  uint32_t nfa_bytes;
};

struct PatDev {
  uint32_t len;        // full (lowercased) length
  uint32_t kw;         // keyword id or kNoKw
  uint32_t bytes_off;  // full lowercased bytes
  uint32_t req_off;    // required-case bytes (0 = either case), valid if confirm
  uint32_t rule_off, rule_n;  // rules anchored on this pattern
  uint8_t special;
  uint8_t confirm;     // anchor roles need a case check
  uint8_t trunc;       // len > trie depth
  uint8_t kw_needed;   // some rule whose gate is not implied uses this keyword
  uint8_t ext;         // scan-automaton class positions after the literal (k_scan_fast image only)
  uint8_t pad[7];
  // k_report's branch-free confirm of the first min(len, depth) bytes against
  // the last 8 bytes (byte 7 = the pattern's last automaton byte)
  uint64_t lo64, m64;    // lowered pattern bytes / their mask, top-aligned
  uint64_t rq64, rqm64;  // case requirement bytes / their mask (0 = none)
};

struct AcDev {
  const uint16_t* delta;  // [nstates * nclasses], bit15 = output state
  const uint8_t* cls;     // [256]
  const uint32_t* out_off;  // [nstates + 1]
  const uint16_t* out_pat;  // pattern ids
  const PatDev* pats;
  const uint8_t* pat_bytes;
  const uint32_t* pat_rules;
  uint32_t nstates, nclasses;
  const uint8_t* fast_lds;   // LDS image for k_scan_fast (AcHost::fast); null => generic kernel
  uint32_t fast_bytes;       // image size
  uint32_t fast_out_entry;   // entries >= this are output states
  uint32_t fast_ev_entry;    // ... and from this one on k_report events (below: keyword states, AcHost)
  uint32_t fast_kw_n;        // keyword states (fast_ev_entry - fast_out_entry)
  const uint8_t* fast_kw;    // their FastKwRec records (kFastKwPer each), then the local bits' keyword ids (u16)
  uint32_t depth;            // trie depth
  // k_report's LDS blob = fast image | out_off | out_pat | pats | pat_bytes
  // (fast_lds is its start; offsets in bytes)
  uint32_t rep_bytes, o_out_off, o_out_pat, o_pats, o_pat_bytes;
  uint32_t o_pair;  // the pair table's offset in the blob (0: none)
};

constexpr uint32_t kLitRec = 36;  // prefilter literal record: len, lower[16], req[16], exact, pad
constexpr uint32_t kLitExactByte = 33;  // 1 in every record of a literal-exact program (gre::Compiled)
constexpr uint32_t kLitFoldByte = 34;   // 1 in every record of a program with a case-free k / s literal byte

struct RuleSetDev {
  const uint16_t* follow_delta;  // all rules' candidate-filter tables (follow.cpp)
  const uint8_t* follow_cls;
  const uint16_t* dfa_delta;     // all rules' verify DFAs (dfa.cpp)
  const uint8_t* dfa_bytes;      // their class maps and match flags
  const uint8_t* nfa_bytes;      // all rules' bit-parallel NFAs (nfa.cpp), 16-byte aligned records
  const gre::ProgView* progs;
  const uint32_t* prog_lit_off;  // per program: range of prefilter literals (n_progs + 1)
  const uint8_t* prog_lits;      // kLitRec-byte records
  const RuleDev* rules;
  const uint32_t* kw_ids;
  const uint32_t* group_slots;
  const uint32_t* allow_progs;   // per-rule allow lists
  const uint32_t* global_allow;  // global allow regex progs
  const uint32_t* pdfa;          // per program: its MatchString DFA record (kPathDfaRec u32; valid flag last)
  uint32_t n_global_allow;
  uint32_t n_rules;
  uint32_t kw_words;       // uint32 words of keyword bits per file
  uint32_t max_ninst;      // for VM scratch sizing (all programs)
  uint32_t max_ncap;       // capture VM: slots of the largest SecretGroupName regex
  uint32_t max_ninst_cap;  // capture VM: instructions of the largest SecretGroupName regex
  AcDev ac;
};

// ---- host-side compiled ruleset -------------------------------------------
struct RegexHost {
  std::string src;
  gre::Compiled c;
};

// Per-rule candidate filter (follow.cpp): states 0 = DEAD, 1 = ACCEPT, 2 = start.
struct FollowDfa {
  bool valid = false;
  uint32_t ncls = 0, nstates = 0;
  uint8_t cls[128] = {};
  std::vector<uint16_t> delta;  // [nstates][ncls]
};
bool build_follow(const gre::Compiled& c, FollowDfa* out);
// Fold-column sets required right after anchor literal `lit` (follow.cpp).
std::vector<uint64_t> follow_ext(const gre::Compiled& c, const gre::Lit& lit, int max_ext);

// Anchored leftmost-first DFA over ASCII for k_verify (dfa.cpp): state 0 =
// dead; entry = next state | 0x8000 when that byte, as the text's last,
// completes a match ($ satisfied); match[state] = a match ends here.
struct DfaHost {
  bool valid = false;
  uint32_t ncls = 0, nstates = 0;
  uint32_t sym_base = 0;  // first rune symbol column (after the ASCII classes)
  bool na_ok = false;     // "other non-ASCII rune" is one symbol for this program
  uint32_t start[2] = {0, 0};
  uint32_t first[4] = {0, 0, 0, 0};  // ASCII first bytes that keep some start state alive
  uint8_t cls[128] = {};
  std::vector<uint16_t> delta;
  std::vector<uint8_t> match;
};
bool build_dfa(const gre::Compiled& c, DfaHost* out);
int dfa_anchored(const DfaHost& d, const uint8_t* text, size_t n, size_t s, size_t* me);
int dfa_rune_sym(const DfaHost& d, const uint8_t* text, size_t n, size_t q, uint32_t* w);
bool follow_accepts(const FollowDfa& f, const uint8_t* text, size_t n, size_t h);

// Bit-parallel Glushkov NFA (nfa.cpp), the fallback for rules whose verify
// DFA explodes past kDfaMaxStates or that use assertions the DFA does not
// model (\b, \B, (?m)^ / $).  Positions = the program's consuming
// instructions (<= kNfaMaxPos, two 64-bit words); the Glushkov follow relation
// is stored LimEx-style: up to kNfaShifts (delta, mask) pairs cover the edges
// p -> p + delta, and the few positions with other edges (or edges through an
// assertion) are exceptions with explicit follow masks.
constexpr uint32_t kNfaMaxPos = 128;
constexpr uint32_t kNfaShifts = 6;
constexpr uint32_t kNfaMaxCond = 4;    // conditional start / accept masks (edges through assertions)
constexpr uint32_t kNfaMaxExc = 48;    // exception positions
constexpr uint32_t kNfaExcCond = 2;    // conditional follows per exception
constexpr uint32_t kNfaNoExc = 0xFF;
constexpr uint32_t kNfaWalkMax = 8192; // bytes an NFA walk may take before the Pike VM decides

struct U128 {
  uint64_t lo, hi;
};

// The device record of one rule's NFA: this header, then reach[ncls], then
// exc[n_exc] (nfa_blob lays them out 16-byte aligned).
struct NfaDev {
  uint32_t npos, nshift, ncls, n_exc;
  int32_t shift[kNfaShifts];
  uint32_t n_first_c, n_last_c;
  U128 smask[kNfaShifts];
  U128 first_u, last_u, exc_mask;
  U128 first_c[kNfaMaxCond], last_c[kNfaMaxCond];
  uint32_t first_r[kNfaMaxCond], last_r[kNfaMaxCond];  // required EmptyOp flags of each conditional mask
  uint32_t has_cond, bytes, o_reach, o_exc;             // bytes: the whole record
  // decoded non-ASCII runes (utf8.DecodeRune; an invalid byte is U+FFFD of
  // width 1) as dfa.cpp's five rune symbols: K, ſ, İ, U+FFFD, any other --
  // the last only when every position treats all other runes alike (na_ok)
  U128 reach_sym[kDfaRuneSyms];
  uint32_t na_ok, pad_[3];
  uint8_t cls[128];                                      // ASCII byte -> reach class
  uint8_t exc_of[kNfaMaxPos];                            // position -> exception record (kNfaNoExc: none)
};
struct NfaExc {
  U128 follow_u;                // unconditional follow
  U128 follow_c[kNfaExcCond];   // follow through assertions
  uint32_t r[kNfaExcCond];      // their required flags
  uint32_t n_c, pad;
};

struct NfaHost {
  bool valid = false;
  uint32_t npos = 0, n_exc = 0;
  std::vector<uint8_t> blob;  // NfaDev | reach | exc
};
bool build_nfa(const gre::Compiled& c, NfaHost* out);
// Host mirror of the device walk (tests / diagnostics).  From s, threads
// injected at every position in [s, inj_hi]; anchored (inj_hi == s): 1 = the
// only match end *me, 0 = no match, 2 = undecidable (the Pike VM decides: a
// byte >= 0x80, two match ends, or kNfaWalkMax); unanchored: 1 = some match.
int nfa_walk_host(const NfaHost& d, const uint8_t* text, size_t n, size_t s, size_t inj_hi, size_t* me);

struct RuleHost {
  std::string id;
  int regex = -1;  // index into regexes, -1 => never matches
  std::vector<std::string> keywords;
  int path = -1;
  std::string group_name;
  std::vector<int> allow_regex;  // rule allow rules: regex
  std::vector<int> allow_path;   // rule allow rules: path
  std::vector<int> exclude;
  RuleMode mode = MODE_NEVER;
  FollowDfa follow;  // MODE_ANCHORED only
  DfaHost dfa;       // MODE_ANCHORED only
  NfaHost nfa;       // MODE_ANCHORED without a verify DFA
  bool gate_implied = false;  // every anchor literal contains one of the keywords
  gre::GroupSpan grp;         // secret-group span rule (valid: k_verify skips the capture search)
  gre::GroupRun grun;         // else the byte-run rule (valid: likewise)
  bool fold_gate = false;     // an anchor literal has a case-free k / s: K/ſ spellings of it
                              // (k_fold_windows) are gated exactly, so its keyword bits are kept
};

struct AcHost {
  std::vector<uint16_t> delta;  // generic: next state | 0x8000 output bit
  std::vector<uint16_t> fail;   // Aho-Corasick failure link per state (same numbering)
  std::vector<uint8_t> fast;    // k_scan_fast image: nstates rows of kFastRowBytes, empty if not representable
  uint32_t fast_out_entry = 0;
  uint8_t cls[256];
  std::vector<uint32_t> out_off;
  std::vector<uint16_t> out_pat;
  uint32_t nstates = 0, nclasses = 0;
  uint32_t depth = kAcMaxLit;  // trie depth (patterns longer than this are confirmed on hit)
  // k_scan_fast image's own automaton (fold columns, literal + class
  // extensions): per-state outputs and, per pattern, the extension it carries
  std::vector<uint32_t> fast_out_off;
  std::vector<uint16_t> fast_out_pat;
  std::vector<uint8_t> fast_ext;
  uint32_t fast_states = 0;
  // k_scan_fast pair table: the state two bytes after the root, per column
  // pair (64 x 64 u16); empty when a state one byte from the root has outputs
  std::vector<uint16_t> fast_pair;
  // keyword states (build_fast): the output states whose every output is a
  // keyword-only pattern the scan resolves itself (FastKwRec, kFastKwPer per
  // state), numbered [fast_out_entry, fast_ev_entry); states from
  // fast_ev_entry on become k_report events.  fast_kw_map: local keyword bit
  // -> keyword id.
  uint32_t fast_ev_entry = 0;
  std::vector<uint8_t> fast_kw;
  std::vector<uint16_t> fast_kw_map;
};

// One keyword pattern of a k_scan_fast keyword state: the lowered bytes and
// their mask, top-aligned in the 8 bytes ending at the output byte (as
// PatDev::lo64 / m64), and the keyword's local bit (< kFastKwBits).
constexpr uint32_t kFastKwPer = 2;     // patterns per keyword state (an unused record: m64 = 0, lo64 = 1, never matches)
constexpr uint32_t kFastKwBits = 32;   // local keyword bits a scan lane accumulates
constexpr uint32_t kFastKwStates = 32; // keyword states at most (the LDS table's size; a lane's seen mask is 32 bits)
struct FastKwRec {
  uint64_t lo64, m64;
  uint32_t bit;
  uint32_t used;  // 1: a pattern of the state (0: padding)
};

struct PatternHost {
  std::string lower;   // full lowercased pattern
  std::string req;     // confirm spec (same length), '\0' = any case
  int kw = -1;
  bool kw_needed = false;  // its keyword is one some non-implied gate needs (engine.hip's kw_needed)
  bool special = false;
  bool confirm = false;
  bool any_anchor = false;
  std::vector<uint32_t> rules;
  std::vector<uint64_t> ext_cols;  // fold columns every anchored use requires after the literal
};

}  // namespace tsg

struct tsg_ruleset {
  std::vector<tsg::RegexHost> regexes;
  std::map<std::string, int> regex_ids;  // source -> regexes index
  // MatchString DFAs of the path regexes (k_path_gate): the DFA of
  // (?s:.)*?(?:src), anchored at 0, per regexes index (invalid: Pike VM)
  std::vector<tsg::DfaHost> path_dfa;
  std::vector<tsg::RuleHost> rules;
  std::vector<int> global_allow_regex;  // AllowRules with Regex
  std::vector<int> global_allow_path;   // AllowRules with Path
  tsg::DfaHost allow_path_union;        // MatchString of any of them, one DFA walk (host Required)
  std::vector<int> global_exclude;
  std::vector<std::string> keywords;     // unique lowercased keywords
  std::vector<uint8_t> kw_uni;           // per keyword: 1 = holds a non-ASCII rune (k_uni_keywords, not the automaton)
  std::vector<tsg::PatternHost> patterns;
  tsg::AcHost ac;
  bool any_path_rules = false;  // some rule has Path or per-rule allow paths
  bool any_exclude = false;
  uint64_t id = 0;  // unique id for device-image caching
  // keyword-only shadow for tsg_gate_device (configs[1]): same rules and
  // keywords, no regex, so no gate is implied by an anchor and every keyword
  // is a scan pattern of its own.  Built on first use.
  mutable std::mutex gate_mu;
  mutable tsg_ruleset* gate_rs = nullptr;
  ~tsg_ruleset();
};

namespace tsg {
bool build_ac(tsg_ruleset* rs, std::string* err);
// k_scan_big's blob for this automaton (engine.hip), when the engine would use
// one, built and checked against the invariants that make its device walk end:
// TSG_OK, or TSG_ERR_INTERNAL with *err naming the violated invariant.
int big_blob_precheck(const AcHost& ac, std::string* err);
// The keyword-only shadow of rs (owned by rs), or nullptr with *err set.
const tsg_ruleset* gate_ruleset(const tsg_ruleset* rs, std::string* err);
}

namespace tsg {
constexpr uint32_t kMaxCap = 64;  // capture slots of a SecretGroupName rule's regex

// Device-built findings (engine.hip k_censor / k_find_spans / k_find_copy),
// records shared by the device and the host copy of a result.
constexpr uint32_t kCodeLines = 4;  // Code window: lines [StartLine - 2, EndLine + 2), EndLine == StartLine

// FindRec::m_off / c_off: bit 62 set = an offset into the dense files'
// region (ResultImpl::dense), else into the string arena (strs).
constexpr uint64_t kArenaDense = 1ull << 62;

// One finding: the location, its Match window and its Code lines.  The Code
// lines [StartLine - 2, EndLine + 2) (EndLine == StartLine: a censored secret
// holds no newline) are consecutive in the arena: in the dense region the
// file's own bytes ('\n' between lines), else distinct-line segments in
// (file, line start) order, adjacent with no separator.  So line k starts at
// c_off + sum of the earlier lines' lengths (+ 1 each in the dense region),
// its Number is first + k + 1 with first = max(StartLine - 3, 0), and it is
// the cause line (IsCause, FirstCause, LastCause) iff that is StartLine.
// (The rule, start and end are the location's: ResultImpl::locs[loc].)
struct FindRec {
  uint32_t file, line, n_lines, loc;  // line = StartLine = EndLine (1-based, censored buffer); loc: its location
  uint64_t m_off, c_off;              // arena offsets: Match window, first Code line
  uint32_t m_len, rank;               // Match length / RuleDev::id_rank of the rule
  uint32_t c_len[kCodeLines];         // Code line lengths
};

// Page-locked host blocks for the findings' string arena, recycled across
// results (a result keeps its block; freeing the result returns it).
struct PinnedPool {
  std::mutex mu;
  std::vector<std::pair<void*, size_t>> free_blocks;
  ~PinnedPool();
};
struct PinnedBlock {
  void* p = nullptr;
  size_t n = 0;
  std::shared_ptr<PinnedPool> pool;
  ~PinnedBlock();
};
std::shared_ptr<PinnedBlock> pinned_get(const std::shared_ptr<PinnedPool>& pool, size_t bytes);

struct ResultImpl {
  // findings in Scan order per file (sorted by file, then RuleID, then Match)
  // (records, code lines and strings share one page-locked block: the D2H
  // copies run at full PCIe rate)
  template <class T>
  struct View {
    T* p = nullptr;
    size_t n = 0;
    T* begin() const { return p; }
    T* end() const { return p + n; }
    size_t size() const { return n; }
    T* data() const { return p; }
    T& operator[](size_t i) const { return p[i]; }
  };
  // everything lives in ONE page-locked block (arena): the kept locations as
  // tsg_loc records and the per-file flags next to the findings, all written
  // by the device and copied back with the call's final synchronisation
  View<tsg_loc> locs;
  View<uint8_t> file_flags;
  View<uint32_t> ties;        // findings equal to their predecessor in (file, RuleID, Match prefix)
  size_t ties_cap = 0, ctrl_off = 0;  // (the block also holds a copy of the device counters)
  View<FindRec> frec;
  const char* strs = nullptr;
  std::shared_ptr<PinnedBlock> arena;
  // the censored contents of the dense files (build_findings_dev), copied
  // back early in a block of their own: arena offsets with kArenaDense set
  // point here (arena_at)
  const char* dense = nullptr;
  std::shared_ptr<PinnedBlock> dense_block;
  mutable std::mutex fmu;     // tsg_result_findings materialises a file's views once
  mutable std::unordered_map<uint32_t, std::pair<std::vector<tsg_finding>, std::vector<tsg_line>>> fcache;
  std::vector<double> timings;
  bool have_findings = false;
};
}  // namespace tsg

namespace tsg {
inline const char* arena_at(const ResultImpl& R, uint64_t off) {
  return (off & kArenaDense) ? R.dense + (off & ~kArenaDense) : R.strs + off;
}
}  // namespace tsg

struct tsg_result {
  tsg::ResultImpl impl;
};
