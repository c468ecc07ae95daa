// engine.hip — MI355X (gfx950) secret-scanning pipeline + C ABI.
//
// Replaces the per-file loop of Scanner.Scan (pkg/fanal/secret/scanner.go:371-452)
// with a batched device pipeline over a packed multi-file buffer in HBM:
//
//   k_path_gate   Global.AllowPath / Rule.MatchPath / Rule.AllowPath per file     (scanner.go:375,391,397)
//   k_scan        one HBM pass: Aho-Corasick over ASCII-lowercased bytes of every
//                 keyword (MatchKeywords gate bits, scanner.go:169-181), every rule's
//                 anchor literal (hit records) and the fold-special sequences
//   k_expand      anchor hits -> (rule, position) candidates for gated files
//   k_fold_windows  keywords / anchor literals spelled with İ, K, ſ around each such rune
//   k_full_jobs   rules without an anchor -> full-scan jobs
//   radix sort    candidates by (rule, position)
//   k_verify      one lane per (file, rule) job: Go leftmost-first Pike VM restricted to
//                 the anchor windows, FindAll iteration, allow rules, secret groups
//                 (FindLocations / FindSubmatchLocations / AllowLocation, scanner.go:97-163)
//   k_exclude_tags exclude-block FindAll per (file, scope) group of the kept locations, then
//                 the containment filter on the device (scanner.go:232-270)
//   k_lines       StartLine / EndLine of every kept location (findLocation, scanner.go:481-503)
//
// Host code (findings.cpp) then censors and cuts Match/Code from the caller's
// content exactly like censorLocation/toFinding (scanner.go:425-537).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "engine.h"
#include "gre_lower_table.h"
#include "nfa_walk.h"
#include "pikevm.h"

namespace tsg {
void set_last_error(const std::string& m);
}  // namespace tsg

using namespace tsg;

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      set_last_error(std::string(#expr " failed: ") + hipGetErrorString(_e));         \
      return TSG_ERR_DEVICE;                                                          \
    }                                                                                 \
  } while (0)

namespace {

constexpr uint32_t kFileAllowed = 1u;
constexpr uint32_t kFileSpecial = 2u;
constexpr uint32_t kFullFlag = 0x80000000u;
constexpr int kPosBits = 44;
constexpr uint64_t kPosMask = (1ull << kPosBits) - 1;
// (file, file-relative position) sort keys: files below 1 TiB, batches below 2^24 files
constexpr int kKeyPosBits = 40;
constexpr uint64_t kKeyPosMask = (1ull << kKeyPosBits) - 1;
constexpr uint64_t kMaxFileBytes = 1ull << kKeyPosBits;
constexpr uint64_t kMaxBatchFiles = 1ull << (64 - kKeyPosBits);
// The match search runs on 32-bit file-relative positions (verify DFA, NFA
// walk, Pike VM) with signed 32-bit capture slots for files up to this length;
// the jobs of longer files run the same kernels instantiated on 64-bit
// positions and slots (a second launch, only when the batch holds such a file).
constexpr uint64_t kMaxVerifyFile = 0x7FFFFFFFull;

// k_scan geometry: 256 threads = 4 waves; each lane owns a 128-byte chunk,
// stored in LDS as a 144-byte row (16-byte halo of the previous chunk first).
constexpr int kScanThreads = 256;
constexpr int kChunk = 128;
constexpr int kRow = kChunk + 16;
constexpr int kBlockBytes = kScanThreads * kChunk;        // 32 KiB per block step
constexpr int kSegsPerLane = kBlockBytes / 16 / kScanThreads;  // 8 x 16-byte loads
constexpr int kTileLds = kScanThreads * kRow;              // 36 KiB
constexpr int kLdsTableMax = 96 * 1024;

struct Ctrl {
  unsigned long long hits;
  unsigned long long cands;
  unsigned long long locs;
  unsigned long long excl;
  unsigned int err;
  unsigned int pad;
  unsigned long long ev_overflow;
  unsigned long long outputs;  // patterns k_report resolved (diagnostics)
  unsigned long long n_fold;     // fold-special rune occurrences recorded (ScanParams::fold_pos)
  unsigned long long events;     // k_scan_fast events in the wave segments (diagnostics, summed by k_report)
  unsigned long long find_bytes; // string arena bytes of the findings (k_find_copy)
  unsigned long long rep_next;   // k_report: next wave segment to claim
  unsigned long long n_caps;     // matches whose secret-group spans k_captures resolves
  unsigned long long n_caps_big; // ... and those too long for its arenas (k_captures_big)
  unsigned long long long_files; // files longer than kMaxVerifyFile (k_region_fill)
  unsigned long long n_panic;    // kept locations whose secret group did not participate (k_out_locs)
  unsigned long long n_ties;     // findings whose (file, RuleID, Match prefix) equals the previous one's
  unsigned long long n_redo;     // speculative job chains re-run from a conflict (k_chain_fix)
  unsigned long long n_dropped;  // locations of the conflicting speculative jobs (k_drop_spec)
  unsigned long long n_caps_run; // matches whose secret group k_group_runs cuts by byte runs
  unsigned long long n_defer;    // jobs k_verify_fast handed to k_verify_slow
  unsigned long long n_match;    // matches k_verify_fast found (k_allow's list)
  unsigned long long match_bytes;  // the Match windows' share of find_bytes (diagnostics)
  unsigned long long dense_bytes;  // the dense files' region (k_dense_at) ...
  unsigned long long dense_groups; // ... and the location file groups (dense or not) ...
  unsigned long long sparse_locs;  // ... and the locations outside dense files (their Code slots are sorted)
  unsigned long long n_long_spans; // locations k_find_spans_lane left to the wave search (long lines)
};

struct DevLoc {
  uint32_t file;
  uint32_t rule;
  uint64_t start, end;
  uint32_t start_line, end_line;
  uint32_t flags;  // 1 = secret group did not participate (reference panics)
  uint32_t job;    // the verify job that found it (kJobRedo | job: a re-run chain's)
};

// k_scan_big's LDS blob (automata too large for one LDS table): the byte
// class map, dense rows of the n_dense shallowest states, and for every
// deeper ("cold") state only the classes on which it differs from its
// failure state, plus the failure link -- delta(s, c) = its own entry, else
// delta(fail(s), c), ending in a dense row.  A cold state is one 8-byte
// record (one ds_read_b64): classes c1, c2 (kBigNone = unused), their entries
// and the failure link; a state with more than two own classes has
// c1 = c2 = kBigMore and its list (u32 class << 16 | entry, ended by
// 0xFFFFFFFF) at the 32-bit offset held in the entry fields.  Most cold
// states are trie nodes whose only own class is the next literal byte.
constexpr uint32_t kBigNone = 0xFF, kBigMore = 0xFE;  // (classes < kBigMore)

// Text byte model that orders k_scan_big's states (relative weights: English
// letter frequencies, lowercase ten times uppercase; space, newline, digits
// and the punctuation of code and config files).
static double big_byte_weight(uint8_t b) {
  static const double kLetter[26] = {8.2, 1.5, 2.8, 4.3, 12.7, 2.2, 2.0, 6.1, 7.0, 0.15, 0.8, 4.0, 2.4,
                                     6.7, 7.5, 1.9, 0.1, 6.0, 6.3, 9.1, 2.8, 1.0, 2.4, 0.15, 2.0, 0.07};
  if (b >= 'a' && b <= 'z') return 0.6 * kLetter[b - 'a'];
  if (b >= 'A' && b <= 'Z') return 0.06 * kLetter[b - 'A'];
  if (b >= '0' && b <= '9') return 0.5;
  switch (b) {
    case ' ': return 15.0;
    case '\n': return 3.0;
    case '_': case '.': case '=': case '"': case '-': case '/': case ',': case ':': case '\'':
    case '(': case ')': case ';': return 0.8;
    default: return b >= 0x20 && b < 0x7F ? 0.1 : 0.02;
  }
}
inline const char* experiment_env(const char* name);
struct BigDev {
  const uint8_t* blob;  // global copy
  uint32_t blob_bytes, n_dense, n_cold;
  uint32_t o_cold, o_eval;  // byte offsets: uint2 [n_cold] records, u32 lists (before the records)
  uint32_t lds_bytes, n_cold_lds;  // the prefix staged in LDS: every list and the first n_cold_lds records
  const uint16_t* ac_of;    // blob state id -> the automaton's (AcDev) state id
};

struct ScanParams {
  uint32_t report_mode;
  BigDev big;  // timing experiments only (TSG_REPORT_MODE): 1 = no file lookups in k_report
  uint32_t gen_lds_rows;  // k_scan_generic<false>: automaton rows staged in LDS (the shallow ones)
  const uint8_t* data;
  const uint64_t* off;  // n_files + 1
  uint64_t nbytes;
  uint32_t n_files;
  RuleSetDev rs;
  uint32_t* file_kw;     // n_files * kw_words
  uint32_t* file_flags;  // n_files
  uint64_t* hits;
  uint64_t hit_cap;
  uint64_t nl_big;  // lazy newline counts: the scan counts the spans of files this big (0: none)
  uint64_t kw_plain;  // report_event: files below this many bytes set keyword bits with plain atomics (else read first)
  uint32_t kw_drain_at;  // k_scan_fast: drain the wave's keyword queue after a step once it holds this many (0: span ends only)
  uint32_t kw_off;       // exp A/B (TSG_KW_OFF): keyword states resolved as k_report events
  // k_report: each report wave's own hit region (hit_seg_cap records at
  // hit_seg + wave * hit_seg_cap; counts in hit_seg_n), packed into `hits` by
  // k_hits_pack -- null: flushes reserve on ctrl->hits
  uint64_t* hit_seg;
  uint32_t* hit_seg_n;
  uint32_t hit_seg_cap;
  uint64_t* big_outs;  // k_big_walk -> k_big_resolve: output records (position << 16 | state)
  uint64_t big_out_cap;
  Ctrl* ctrl;
  uint32_t* nl_blocks;  // newline count per kNlBlock bytes of the batch
  const uint8_t* tail;  // virtual base of a zero-padded copy of data[tail_base-8, nbytes)
  uint64_t tail_base;   // first byte of the final partial fast region
  const uint32_t* region_file;  // file containing byte r*kNlBlock, for r in [0, n_regions]
  uint64_t n_regions;
  struct FastEvent* events;       // k_scan_fast events, one segment per wave
  uint32_t* ev_counts;            // events per wave
  uint64_t ev_cap_per_wave;
  struct FastEvent* ev_overflow;  // events beyond a wave's segment
  uint64_t ev_overflow_cap;
  uint8_t* span_hi;               // per kNlBlock span: a byte >= 0x80 occurs (k_fold_special)
  uint64_t* fold_pos;             // fold-special runes: position << 2 | kind (FoldKind), ctrl->n_fold of them
  uint64_t fold_cap;
};

// Fold-special runes (the only non-ASCII runes that Go's case rules tie to
// ASCII letters): U+0130 İ lowers to 'i' and U+212A K to 'k' in bytes.ToLower
// (the MatchKeywords gate, scanner.go:175); U+212A K and U+017F ſ match 'k' /
// 's' under (?i) simple folding (regexp/syntax).  Every occurrence is
// recorded (position of its lead byte + kind); k_fold_windows then examines
// only the bytes around each one (keywords / anchor literals spelled with it).
enum FoldKind : uint32_t { FOLD_I = 0, FOLD_S = 1, FOLD_K = 2 };

__device__ inline void mark_special(const ScanParams& P, uint32_t fi) {
  if (!(P.file_flags[fi] & kFileSpecial)) atomicOr(&P.file_flags[fi], kFileSpecial);
}

__device__ inline void note_fold(const ScanParams& P, uint64_t pos, uint32_t kind) {
  const unsigned long long k = atomicAdd(&P.ctrl->n_fold, 1ull);
  if (k < P.fold_cap) P.fold_pos[k] = (pos << 2) | kind;
}


// region_file[r] = index of the file holding byte r * kNlBlock = the largest f
// with off[f] <= r * kNlBlock.
// Written directly: file f holds the region starts
// [ceil(off[f] / B), ceil(off[f + 1] / B)) (the last file: through n_regions).
// A lane writes its file's first kRegionDirect regions; the wave then writes
// the rest of each longer file of its lanes together (coalesced, one file at a
// time).  No memset, no mark pass, no max-scan -- and no list of long files:
// an append to one counter serialised at L2 (0.75 ms for ~160 K long files of
// configs[2], profiles/r06c_ab).
constexpr uint64_t kRegionDirect = 16;
__global__ __launch_bounds__(256) void k_region_fill(const uint64_t* off, uint32_t n_files, uint64_t n_regions,
                                                     uint32_t* region_file, Ctrl* ctrl) {
  const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t rd = 0, r1 = 0;
  if (f < n_files) {
    const uint64_t o0 = off[f], o1 = off[f + 1];
    if (o1 - o0 - 1 > kMaxVerifyFile) atomicAdd(&ctrl->long_files, 1ull);
    const uint64_t r0 = (o0 + kNlBlock - 1) / kNlBlock;
    r1 = f + 1 == n_files ? n_regions : std::min<uint64_t>((o1 + kNlBlock - 1) / kNlBlock, n_regions);
    rd = std::min(r1, r0 + kRegionDirect);
    for (uint64_t r = r0; r < rd; ++r) region_file[r] = (uint32_t)f;
  }
  uint64_t m = __ballot(r1 > rd);
  while (m) {
    const uint32_t k = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    const uint64_t lo = __shfl(rd, k), hi = __shfl(r1, k);
    const uint32_t fk = (uint32_t)__shfl((uint32_t)f, k);
    for (uint64_t r = lo + lane; r < hi; r += 64) region_file[r] = fk;
  }
}

__device__ inline uint32_t find_file(const uint64_t* off, uint32_t lo, uint32_t hi, uint64_t pos) {
  // largest f in [lo, hi) with off[f] <= pos
  while (hi - lo > 1) {
    uint32_t m = (lo + hi) >> 1;
    if (off[m] <= pos) lo = m; else hi = m;
  }
  return lo;
}

__device__ inline uint8_t lower_ascii(uint8_t b) { return (b >= 'A' && b <= 'Z') ? b + 32 : b; }

// Global / LDS address spaces spelled out: through generic pointers the
// compiler emits flat loads that wait on both counters.
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const uint16_t gu16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ inline T* as_global(const void* p) { return reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(p)); }

// Report every pattern ending at global position p (AC state st has outputs).
// Files are NUL-separated, so the pattern lies inside file fi.
// Where the generic kernel's anchor hit records go: the global list.
struct GlobalHitSink {
  __device__ void push(const ScanParams& P, uint64_t rec) {
    unsigned long long idx = atomicAdd(&P.ctrl->hits, 1ull);
    if (idx < P.hit_cap) P.hits[idx] = rec;
  }
};

// kConfirm: the automaton ran on 7-bit aliased bytes (k_scan_fast), so each
// reported pattern is re-checked on the real bytes first.
// The file holding p, with a one-entry cache (*fc: file, [*fs, *fe) its
// bytes incl. the separator) for the outputs of one event.
__device__ inline uint32_t file_at(const ScanParams& P, uint64_t p, uint32_t* fc, uint64_t* fs, uint64_t* fe) {
  if (*fc != 0xFFFFFFFFu && p >= *fs && p < *fe) return *fc;
  uint32_t lo = 0, hi = P.n_files;
  if (P.region_file) {
    const uint64_t r = p / kNlBlock;
    lo = P.region_file[r];
    hi = r + 1 < P.n_regions ? P.region_file[r + 1] + 1 : P.n_files;
    if (hi > P.n_files) hi = P.n_files;
  }
  const uint32_t fi = find_file(P.off, lo, hi, p);
  *fc = fi;
  *fs = P.off[fi];
  *fe = P.off[fi + 1];
  return fi;
}

template <bool kConfirm, class Sink>
__device__ inline void report_t(const ScanParams& P, uint32_t st, uint64_t p, uint64_t* last_kw, Sink& sink,
                                uint32_t* fc = nullptr, uint64_t* fcs = nullptr, uint64_t* fce = nullptr) {
  const AcDev& ac = P.rs.ac;
  uint32_t fc0 = 0xFFFFFFFFu;
  uint64_t fs0 = 0, fe0 = 0;
  const uint32_t fi = fc ? file_at(P, p, fc, fcs, fce) : file_at(P, p, &fc0, &fs0, &fe0);
  const uint64_t fend = P.off[fi + 1] - 1;  // content end (separator excluded)
  uint32_t o0 = ac.out_off[st], o1 = ac.out_off[st + 1];
  for (uint32_t o = o0; o < o1; ++o) {
    uint32_t pid = ac.out_pat[o];
    PatDev pd = ac.pats[pid];
    uint32_t tl = pd.len < ac.depth ? pd.len : ac.depth;
    uint64_t start = p + 1 - tl;
    if (kConfirm) {
      const uint8_t* pb = ac.pat_bytes + pd.bytes_off;
      bool ok = true;
      for (uint32_t k = 0; k < tl && ok; ++k) ok = lower_ascii(P.data[start + k]) == pb[k];
      if (!ok) continue;
    }
    // (the byte checks below have no early exit: each chunk of 8 loads is
    // issued before any compare, one memory latency instead of a chain)
    if (pd.trunc) {
      if (start + pd.len > fend) continue;
      uint32_t bad = 0;
      const uint8_t* pb = ac.pat_bytes + pd.bytes_off;
      for (uint32_t k0 = ac.depth; k0 < pd.len && !bad; k0 += 8) {
#pragma unroll
        for (uint32_t k = k0; k < k0 + 8; ++k)
          if (k < pd.len) bad |= lower_ascii(P.data[start + k]) ^ pb[k];
      }
      if (bad) continue;
    }
    if (pd.special) {
      mark_special(P, fi);
      const uint8_t b0 = ac.pat_bytes[pd.bytes_off];
      note_fold(P, start, b0 == 0xC4 ? FOLD_I : b0 == 0xC5 ? FOLD_S : FOLD_K);
    }
    if (pd.kw != kNoKw) {
      const uint64_t key = ((uint64_t)fi << 32) | pd.kw;  // per-lane dedupe of repeated keywords
      if (*last_kw != key) {
        *last_kw = key;
        uint32_t* wp = &P.file_kw[(size_t)fi * P.rs.kw_words + (pd.kw >> 5)];
        const uint32_t bit = 1u << (pd.kw & 31);
        // (read first: configs[4]'s C5 files repeat a keyword thousands of
        // times, and plain atomics on those words slowed k_big_resolve's path
        // by ~0.25 ms, profiles/r04ai; k_report's plain atomics are quicker)
        if (!(__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(wp, bit);
      }
    }
    if (pd.rule_n) {
      if (pd.confirm) {
        const uint8_t* rq = ac.pat_bytes + pd.req_off;
        bool bad = false;
        for (uint32_t k0 = 0; k0 < pd.len && !bad; k0 += 8) {
#pragma unroll
          for (uint32_t k = k0; k < k0 + 8; ++k)
            if (k < pd.len) {
              const uint8_t r = rq[k], d = P.data[start + k];
              bad |= (r != 0) & (d != r);
            }
        }
        if (bad) continue;
      }
      sink.push(P, (start << 16) | pid);
    }
  }
}

__device__ __noinline__ void report(const ScanParams& P, uint32_t st, uint64_t p, uint64_t* last_kw) {
  GlobalHitSink g;
  report_t<false>(P, st, p, last_kw, g);
}

// Generic scan (any automaton size): one 128-byte chunk per lane, byte
// loads from a padded LDS tile, transitions from LDS (or global when the
// table exceeds the LDS budget).  Used for large custom rule sets.
template <bool kLdsTable>
__global__ __launch_bounds__(kScanThreads) void k_scan_generic(ScanParams P) {
  extern __shared__ __align__(16) uint8_t smem[];
  uint8_t* cls = smem;         // 256
  uint8_t* tile = smem + 256;  // kTileLds
  uint16_t* dl = (uint16_t*)(smem + 256 + kTileLds);
  const AcDev& ac = P.rs.ac;
  const uint32_t K = ac.nclasses;
  for (int i = threadIdx.x; i < 256; i += kScanThreads) cls[i] = ac.cls[i];
  // kLdsTable: the whole table in LDS; else its first gen_lds_rows rows (states
  // are numbered breadth-first, so those are where text keeps the automaton)
  // and the deep rest from global memory (L2-resident)
  const uint32_t lds_rows = kLdsTable ? ac.nstates : P.gen_lds_rows;
  {
    const uint32_t n = lds_rows * K;
    for (uint32_t i = threadIdx.x; i < n; i += kScanThreads) dl[i] = ac.delta[i];
  }
  auto next = [&](uint32_t st, uint32_t c) -> uint32_t {
    const uint32_t i = st * K + c;
    if (kLdsTable) return dl[i];
    return st < lds_rows ? (uint32_t)dl[i] : (uint32_t)ac.delta[i];
  };
  const uint32_t tid = threadIdx.x;
  const uint64_t nsteps = (P.nbytes + kBlockBytes - 1) / kBlockBytes;
  uint64_t last_kw = ~0ull;
  for (uint64_t step = blockIdx.x; step < nsteps; step += gridDim.x) {
    const uint64_t base = step * kBlockBytes;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSegsPerLane; ++k) {
      const uint32_t seg = k * kScanThreads + tid;
      const uint64_t g = base + (uint64_t)seg * 16;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (g + 16 <= P.nbytes) {
        v = *(const uint4*)(P.data + g);
      } else if (g < P.nbytes) {
        uint8_t tmp[16] = {0};
        for (uint64_t q = g; q < P.nbytes; ++q) tmp[q - g] = P.data[q];
        memcpy(&v, tmp, 16);
      }
      const uint32_t row = seg >> 3, col = seg & 7;
      *(uint4*)(tile + row * kRow + 16 + col * 16) = v;
      if (col == 7 && row + 1 < (uint32_t)kScanThreads) *(uint4*)(tile + (row + 1) * kRow) = v;
    }
    if (tid == 0) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (base >= 16) v = *(const uint4*)(P.data + base - 16);
      *(uint4*)(tile) = v;
    }
    __syncthreads();
    const uint64_t p0 = base + (uint64_t)tid * kChunk;
    if (p0 >= P.nbytes) continue;
    const uint64_t pend = p0 + kChunk < P.nbytes ? p0 + kChunk : P.nbytes;
    const uint8_t* row = tile + tid * kRow + 16;
    uint32_t st = 0;
    // warm-up: the automaton restarted kAcMaxLit-1 bytes earlier (a NUL
    // separator inside the window resets it, so files never leak)
    const uint64_t w0 = p0 >= (uint64_t)(kAcMaxLit - 1) ? p0 - (kAcMaxLit - 1) : 0;
    for (uint64_t p = w0; p < p0; ++p) st = next(st, cls[row[(int64_t)p - (int64_t)p0]]) & 0x7FFFu;
    uint32_t nl = 0;
    for (uint64_t p = p0; p < pend; ++p) {
      const uint8_t b = row[p - p0];
      nl += b == '\n';
      const uint32_t nx = next(st, cls[b]);
      st = nx & 0x7FFFu;
      if (nx & 0x8000u) report(P, st, p, &last_kw);
    }
    atomicAdd(&P.nl_blocks[p0 / kNlBlock], nl);
  }
}

// Fast scan: the HBM-bound hot loop — one pass of the keyword/anchor
// Aho-Corasick automaton over the whole batch (MatchKeywords, scanner.go:169-181).
//  * 1024-thread blocks, one LDS image of the automaton per CU (AcHost::fast):
//    rows of 128 u16 columns indexed by the byte's low 7 bits (upper case
//    shares the lower-case column), kFastRowBytes stride so consecutive rows
//    rotate the LDS banks; an entry is the next row's byte offset / 4, so one
//    step is  e = T[4e + 2(b & 0x7F)]  (one ds_read_u16, no class lookup),
//    and output states are numbered last: one max() per byte flags outputs
//  * every lane runs kFastChains independent chains (ILP against the LDS
//    latency); a chain walks one kNlBlock-byte span per work unit with 7 bytes
//    of warm-up (automaton depth <= kAcMaxLit), so spans need no stitching
//  * each chain streams its span through a 128-byte register ring: a 16-byte
//    vector is reloaded with the chain's next 128 bytes (or the next unit's
//    first ones) as soon as it is consumed, so HBM latency hides behind a
//    full ring of automaton work
//  * per 8-byte group: an output (max >= fast_out_entry) or a byte >= 0x80
//    flags the group; after each step a chain with flagged groups appends
//    ONE event (first flagged group, group count, entry state) to the wave's
//    segment with ballot/popcount (no atomics, no global reads in the scan);
//    k_report replays those bytes.  Bytes >= 0x80 alias ASCII columns, so
//    k_report confirms every pattern on the real bytes, and its replay finds
//    the fold-special sequences C4B0 / C5BF / E284AA exactly
//  * the newline count of each span goes straight to nl_blocks (one owner,
//    plain store) and feeds StartLine/EndLine.
// Variant in use (chains per lane, 16-byte vectors per chain step); the
// other shapes stay compilable for A/B runs (TSG_FAST_VARIANT).
constexpr int kFastChains = 1;
constexpr int kFastVecs = 8;
constexpr int kFastEventWin = 4;  // 8-byte groups per wave-level event check
constexpr uint32_t kFastUnitMax = 2 * kNlBlock;  // largest chains * span (tail buffer size)

__device__ inline uint32_t nl_count_dword(uint32_t w) {
  const uint32_t t = w ^ 0x0A0A0A0Au;
  const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
  return __builtin_popcount(z);
}

// 6-bit column fold, four bytes at once, each byte = 2 x column (the byte
// offset of its u16 entry in a row): column = bits 0-4 kept, bit 6 moved to
// bit 5.  Both letter cases share columns 32-58, digits and punctuation sit
// in 0-31, and a row's 64 entries cover the 32 LDS banks once (two columns
// per dword), so lanes in one state never collide on a bank.  Control bytes
// alias space/punctuation, `{|}~ and DEL alias @[\]^_, bytes >= 0x80 alias
// ASCII: k_report re-checks every pattern on the real bytes.
__device__ inline uint32_t fold6(uint32_t w) { return ((w << 1) & 0x3E3E3E3Eu) | (w & 0x40404040u); }

// fold6 in three VALU (shift, and, and_or) for k_scan_fast's step: written
// as C the compiler emitted four plus a fused byte-0 op.  Full-ruleset scan
// 11.39 -> 11.28 ms on configs[2]; in the prefilter-only kernel (kScanKwMid)
// its register allocation went the other way, 5.74 -> 6.36 ms on configs[1]
// (same-box A/B, profiles/r06zo_ab), so that kernel keeps the C form.
__device__ inline uint32_t fold6_ao(uint32_t w) {
  const uint32_t t = w << 1, m = w & 0x40404040u;
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(t), "s"(0x3E3E3E3Eu), "v"(m));
  return r;
}

// One automaton step on byte j of a folded dword w: e = T[e * row + 2 col].
// Entries are row indices and rows are kFastRowBytes apart (a stride an LDS
// bank-conflict simulation of the scan picked: 134 B conflicts ~13 % less
// than packed 130 B rows); the address is one v_mad_u32_u24 on the chain.
__device__ inline uint32_t fstep(const uint8_t* T, uint32_t e, uint32_t w, int j) {
  uint32_t c2;  // byte j (one VALU; the compiler splits a masked shift in two)
  if (j == 0) c2 = w & 0xFFu;
  else if (j == 3) c2 = w >> 24;
  else asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(c2) : "v"(w), "i"(8 * j));
  return *(const uint16_t*)(T + (e * kFastRowBytes + c2));
}


// Two bytes (j, j + 1 of the folded dword w, j even) from entry e: a lane at
// the root reads the state after both from the pair table (at kFastImgMax in
// LDS), the others walk two rows (the root lanes sit the second read out, so
// the LDS serves fewer lanes).  Returns the larger of the states passed; the
// skipped middle state of a root pair is never an output (ruleset.cpp).
__device__ inline uint32_t fstep2(const uint8_t* T, uint32_t& e, uint32_t w, int j) {
  uint32_t c1, c2;
  if (j == 0) c1 = w & 0xFFu;
  else asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(c1) : "v"(w), "i"(8 * j));
  if (j + 1 == 3) c2 = w >> 24;
  else asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(c2) : "v"(w), "i"(8 * (j + 1)));
  const uint32_t a = e == 0 ? kFastImgMax + c1 * 64u + c2 : e * kFastRowBytes + c1;
  uint32_t x = *(const uint16_t*)(T + a);
  uint32_t m = x;
  if (e != 0) {
    x = *(const uint16_t*)(T + (x * kFastRowBytes + c2));
    m = m > x ? m : x;
  }
  e = x;
  return m;
}

// `src` for a position: the batch, or for the final partial unit the
// zero-padded copy addressed with the same offsets (ScanParams::tail).
__device__ inline const uint8_t* fast_src(const ScanParams& P, uint64_t pos) {
  return pos >= P.tail_base ? P.tail : P.data;
}

// A k_scan_fast event: one 8-byte group in which the automaton reached an
// output state, with everything k_report needs to resolve it without touching
// the batch again (32 bytes: two dwordx4 stores).
struct FastEvent {
  uint64_t pos;    // first byte of the group
  uint32_t entry;  // automaton entry before the group
  uint32_t pad;
  uint2 prev;      // the 8 raw bytes before the group
  uint2 cur;       // the group's 8 raw bytes
};
static_assert(sizeof(FastEvent) == 32, "two dwordx4");

template <int V>
struct FastChain {
  uint4 cur[V];
  uint64_t pos;  // first byte of the V*16 bytes in `cur`
  uint32_t e;    // automaton entry
  uint32_t nl;   // newlines of the current span
  uint32_t hi;   // OR of the span's dwords: bit 7 of a byte = a byte >= 0x80
  uint2 prev;    // the 8 raw bytes before the next group
  bool cnt = false;  // kMode 2: wave-uniform -- count this round's newlines anyway
};

// ASCII lowercase of 8 bytes at once (bytes 'A'-'Z' gain 0x20)
__device__ inline uint64_t lower64(uint64_t x) {
  const uint64_t t = x & 0x7F7F7F7F7F7F7F7Full;
  const uint64_t up = ((t + 0x3F3F3F3F3F3F3F3Full) ^ (t + 0x2525252525252525ull)) & ~x & 0x8080808080808080ull;
  return x | (up >> 2);
}

// Keyword states (AcHost::fast_kw): a group whose automaton max is a keyword
// state -- in [fast_out_entry, fast_ev_entry) -- holds only keyword-only
// outputs, which the scan resolves itself instead of handing k_report an event
// (the 2-3 letter keywords jwt / lob / key of the builtin rules were most of
// configs[2]'s 6.3 M events; 'sk' once per KiB of configs[1]).  The lane
// appends the group (a 16-byte KwRec) to its wave's queue in LDS; the wave
// drains the queue after a step once it holds kw_drain_at records and at the
// end of each span, one record per lane: replay of the 8 bytes from the entry
// state (8 LDS steps, as k_report), each keyword state's patterns confirmed on
// the real bytes (lowered window: FastKwRec lo64 / m64; the 8 bytes before the
// group re-read from the batch), the file found from the span's region (a
// span inside one file needs no search) and the keyword's bit set (one
// atomic, read-first in files of kw_plain bytes or more, whose words every
// lane hits).  Repeats: in a span inside one file, a state whose patterns all
// confirmed is marked in the owning lane's seen mask (LDS); the lane then
// skips a group whose max m has every keyword state <= m seen (the group's
// states all lie in [fast_out_entry, m]; states are numbered shortest keyword
// first, so 'sk' / jwt are the low ones).  A full queue turns the group into
// an event.  Per-drain latency dominates the cost (threshold 8 / 16 / 32 of a
// 48 x 32 B queue: k_scan_fast +2.9 / +1.9 / +0.9 ms on configs[1],
// profiles/r06f): hence the small records and the dedupe.  The drain sits
// outside the scan's unrolled step (inlined per group it doubled the loop's
// code, which the compiler then no longer unrolled: the register ring went to
// scratch).
constexpr uint32_t kFastKwQ = 88;    // queue records per wave (16 waves x 88 x 16 B of LDS)
constexpr uint32_t kKwDrainAt = 64;  // ScanParams::kw_drain_at
constexpr int kScanKwMid = 64;       // k_scan_fast kMode bit: keyword queue drains after steps too (the gate scan)
constexpr int kScanNoCount = 128;    // k_scan_fast kMode bit: the scan never counts newlines (no per-group test)

struct KwRec {
  uint32_t span;  // the group's span (position / kNlBlock)
  uint32_t meta;  // entry state (10 bits) | group in the span (9 bits) << 10 | queuing lane << 19
  uint2 cur;      // the group's 8 bytes
};
static_assert(kFastMaxRows <= 1024 && kNlBlock / 8 <= 512, "KwRec::meta fields");

struct KwScan {
  const FastKwRec* rec;
  const uint16_t* map;
  KwRec* q;        // this wave's queue (LDS)
  uint32_t* seen;  // this wave's lanes' seen masks (LDS)
  uint32_t ev_e;   // first event state (== fast_out_entry: no keyword states)
};

__device__ inline bool kw_scan_ok(const ScanParams& P) { return P.nbytes / kNlBlock < (1ull << 32); }

__device__ inline void kw_resolve(const ScanParams& P, const uint8_t* T, const KwScan& kw, uint32_t out_e,
                                  const KwRec& rq) {
  const uint32_t meta = rq.meta;
  const uint64_t gp = (uint64_t)rq.span * kNlBlock + 8 * ((meta >> 10) & 511u);
  const uint2 pv = gp >= 8 ? *(const uint2*)(fast_src(P, gp - 8) + gp - 8) : make_uint2(0, 0);
  const uint64_t rg = rq.span;
  const uint32_t rf0 = P.region_file[rg];
  const uint32_t rf1 = rg + 1 < P.n_regions ? P.region_file[rg + 1] : 0xFFFFFFFFu;
  const bool single = rf0 == rf1;  // the span lies in one file
  const uint2 cur = rq.cur;
  uint64_t hlow = lower64(((uint64_t)pv.y << 32) | pv.x);
  uint32_t e = meta & 1023u;
  const uint32_t f0 = fold6(cur.x), f1 = fold6(cur.y);
  uint32_t fi = 0xFFFFFFFFu, seen = 0;
  bool read_first = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    e = fstep(T, e, j < 4 ? f0 : f1, j & 3);
    const uint32_t c = ((j < 4 ? cur.x : cur.y) >> (8 * (j & 3))) & 0xFFu;
    hlow = (hlow >> 8) | ((uint64_t)lower_ascii((uint8_t)c) << 56);
    if (e < out_e) continue;
    const FastKwRec* r = kw.rec + (size_t)(e - out_e) * kFastKwPer;
    uint32_t bits = 0;
    bool full = true;
#pragma unroll
    for (uint32_t q = 0; q < kFastKwPer; ++q) {
      const bool hit = (hlow & r[q].m64) == r[q].lo64;
      bits |= hit ? 1u << r[q].bit : 0u;
      full &= hit || !r[q].used;
    }
    if (!bits) continue;
    if (full) seen |= 1u << (e - out_e);
    // (a file separator resets the automaton: every pattern lies in one file)
    const uint64_t pos = gp + j;
    if (fi == 0xFFFFFFFFu || (!single && pos >= P.off[fi + 1])) {
      fi = single ? rf0 : find_file(P.off, rf0, rf1 == 0xFFFFFFFFu ? P.n_files : min(rf1 + 1, P.n_files), pos);
      read_first = P.off[fi + 1] - P.off[fi] >= P.kw_plain;
    }
    while (bits) {
      const uint32_t b = (uint32_t)__builtin_ctz(bits);
      bits &= bits - 1;
      const uint32_t g = kw.map[b];
      uint32_t* wp = &P.file_kw[(size_t)fi * P.rs.kw_words + (g >> 5)];
      const uint32_t bit = 1u << (g & 31);
      if (!read_first || !(__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(wp, bit);
    }
  }
  if (single && seen) atomicOr(&kw.seen[meta >> 19], seen);
}

// The wave's queued keyword groups, one per lane (wave-uniform count); then
// each lane takes its seen mask back.
__device__ inline void kw_drain(const ScanParams& P, const uint8_t* T, const KwScan& kw, uint32_t out_e,
                                uint32_t& kwn, uint32_t& kseen, uint32_t lane) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the queue's stores before its loads
  for (uint32_t q0 = 0; q0 < kwn; q0 += 64)
    if (q0 + lane < kwn) kw_resolve(P, T, kw, out_e, kw.q[q0 + lane]);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the loads and seen bits before the queue is refilled
  kseen = kw.seen[lane];
  kwn = 0;
}

// Append an event for a group whose automaton max reached an output state
// (ballot + popcount into the wave's segment, no atomics; every lane calls
// this, so ev_count stays wave-uniform).
template <int V>
__device__ inline void fast_event(const ScanParams& P, uint32_t out_e, const FastChain<V>& C, uint32_t m, uint32_t gs,
                                  uint32_t d0, uint32_t d1, uint64_t gpos, bool live, uint64_t lanes_lt,
                                  FastEvent* ev_seg, uint32_t* ev_count) {
  // lane mask straight from the compare (uge), live lanes only
  const uint64_t b = __builtin_amdgcn_uicmp(m, out_e, 35) & __ballot(live);
  if (b) {
    if ((b >> __lane_id()) & 1) {
      FastEvent r;
      r.pos = gpos;
      r.entry = gs;
      r.pad = 0;
      r.prev = C.prev;
      r.cur = make_uint2(d0, d1);
      const uint32_t slot = *ev_count + (uint32_t)__popcll(b & lanes_lt);
      if (slot < P.ev_cap_per_wave) {
        ev_seg[slot] = r;
      } else {
        unsigned long long ov = atomicAdd(&P.ctrl->ev_overflow, 1ull);
        if (ov < P.ev_overflow_cap) P.ev_overflow[ov] = r;
      }
    }
    *ev_count += (uint32_t)__popcll(b);
  }
}

// Walk one 8-byte group (d0, d1) of a chain and report it if it hit an output.
// kMode: 2 = no newline counts (the product's default: k_nl_spans counts the
// spans of files with locations afterwards); timing experiments only
// (TSG_SCAN_MODE, wrong results): 1 = no events, 4 = loads from the batch's
// first MiB (L2-resident: takes HBM out of the picture).
template <int V, int kMode = 0>
__device__ inline void fast_group(const ScanParams& P, const uint8_t* T, uint32_t out_e, FastChain<V>& C, uint32_t d0,
                                  uint32_t d1, uint64_t gpos, bool live, uint64_t lanes_lt, FastEvent* ev_seg,
                                  uint32_t* ev_count) {
  if (!(kMode & 2) || (!(kMode & kScanNoCount) && C.cnt)) C.nl += nl_count_dword(d0) + nl_count_dword(d1);
  C.hi |= d0 | d1;
  const uint32_t f0 = fold6(d0), f1 = fold6(d1);
  const uint32_t gs = C.e;
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    C.e = fstep(T, C.e, j < 4 ? f0 : f1, j & 3);
    m = m > C.e ? m : C.e;
  }
  if (!(kMode & 1)) fast_event(P, out_e, C, m, gs, d0, d1, gpos, live, lanes_lt, ev_seg, ev_count);
  C.prev = make_uint2(d0, d1);
}

// Two chains' groups walked in lock-step, so their LDS lookups overlap.
template <int V>
__device__ inline void fast_group2(const ScanParams& P, const uint8_t* T, uint32_t out_e, FastChain<V>& A,
                                   FastChain<V>& B, uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint64_t apos,
                                   uint64_t bpos, bool live, uint64_t lanes_lt, FastEvent* ev_seg,
                                   uint32_t* ev_count) {
  A.nl += nl_count_dword(a0) + nl_count_dword(a1);
  B.nl += nl_count_dword(b0) + nl_count_dword(b1);
  A.hi |= a0 | a1;
  B.hi |= b0 | b1;
  const uint32_t fa0 = fold6(a0), fa1 = fold6(a1), fb0 = fold6(b0), fb1 = fold6(b1);
  const uint32_t ga = A.e, gb = B.e;
  uint32_t ma = 0, mb = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A.e = fstep(T, A.e, j < 4 ? fa0 : fa1, j & 3);
    B.e = fstep(T, B.e, j < 4 ? fb0 : fb1, j & 3);
    ma = ma > A.e ? ma : A.e;
    mb = mb > B.e ? mb : B.e;
  }
  fast_event(P, out_e, A, ma, ga, a0, a1, apos, live, lanes_lt, ev_seg, ev_count);
  fast_event(P, out_e, B, mb, gb, b0, b1, bpos, live, lanes_lt, ev_seg, ev_count);
  A.prev = make_uint2(a0, a1);
  B.prev = make_uint2(b0, b1);
}

// G consecutive 8-byte groups of a chain with ONE wave-level event check:
// the per-group maxima are kept, and only when some live lane reached an
// output state anywhere in the window (rare: ~one group in 10^3) are the
// groups' events appended in order.  Cuts the compare / ballot / branch per
// group that otherwise sits on every chain step.
// kw: keyword groups go to the wave's queue (kwn: its wave-uniform count);
// without, every output state is an event.
template <int V, int kMode, int G, bool kPair = false>
__device__ inline void fast_window(const ScanParams& P, const uint8_t* T, uint32_t out_e, FastChain<V>& C,
                                   const uint32_t (&d)[2 * G], uint64_t gpos, bool live, uint64_t lanes_lt,
                                   FastEvent* ev_seg, uint32_t* ev_count, const KwScan* kw = nullptr,
                                   uint32_t* kwn = nullptr, uint32_t kseen = 0) {
  uint32_t gs[G], m[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t d0 = d[2 * g], d1 = d[2 * g + 1];
    if (!(kMode & 2) || (!(kMode & kScanNoCount) && C.cnt)) C.nl += nl_count_dword(d0) + nl_count_dword(d1);
    C.hi |= d0 | d1;
    const uint32_t f0 = (kMode & kScanKwMid) ? fold6(d0) : fold6_ao(d0);
    const uint32_t f1 = (kMode & kScanKwMid) ? fold6(d1) : fold6_ao(d1);
    gs[g] = C.e;
    uint32_t mm = 0;
    if (kPair) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const uint32_t x = fstep2(T, C.e, j < 4 ? f0 : f1, j & 3);
        mm = mm > x ? mm : x;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        C.e = fstep(T, C.e, j < 4 ? f0 : f1, j & 3);
        mm = mm > C.e ? mm : C.e;
      }
    }
    m[g] = mm;
  }
  if (!(kMode & 1)) {
    uint32_t mx = m[0];
#pragma unroll
    for (int g = 1; g < G; ++g) mx = mx > m[g] ? mx : m[g];
    if (__builtin_amdgcn_uicmp(mx, out_e, 35) & __ballot(live)) {
      const uint32_t ev_e = kw ? kw->ev_e : out_e;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        uint32_t mg = m[g];
        if (kw) {  // keyword groups into the queue; a full queue makes them events
          const bool kg = live && mg >= out_e && mg < ev_e;
          // (every keyword state <= mg seen: nothing new in this group)
          const bool kl = kg && (((2u << (mg - out_e)) - 1u) & ~kseen) != 0;
          const uint64_t kb = __ballot(kl);
          if (kb) {
            const uint32_t nq = (uint32_t)__popcll(kb);
            if (*kwn + nq <= kFastKwQ) {
              if (kl) {
                KwRec r;
                const uint64_t q = gpos + 8 * g;
                r.span = (uint32_t)(q / kNlBlock);
                r.meta = gs[g] | (uint32_t)((q % kNlBlock) / 8) << 10 | __lane_id() << 19;
                r.cur = make_uint2(d[2 * g], d[2 * g + 1]);
                kw->q[*kwn + (uint32_t)__popcll(kb & lanes_lt)] = r;
              }
              *kwn += nq;
            } else if (kl) {
              mg = ev_e;
            }
          }
        }
        fast_event(P, ev_e, C, mg, gs[g], d[2 * g], d[2 * g + 1], gpos + 8 * g, live, lanes_lt, ev_seg, ev_count);
        C.prev = make_uint2(d[2 * g], d[2 * g + 1]);
      }
    }
  }
  C.prev = make_uint2(d[2 * G - 2], d[2 * G - 1]);
}

// ---- event resolution (k_report, and the fused scan's own segments)
constexpr uint32_t kReportThreads = 1024;
constexpr uint32_t kReportHitCap = 1024;
constexpr uint32_t kReportLds = kLdsMax - kReportHitCap * 8 - 64;
constexpr uint32_t kReportWaveHits = kReportHitCap / (kReportThreads / 64);  // LDS hit slots per wave
constexpr uint32_t kHitSegCap = 4096;  // hit records in each report wave's own region (32 KiB)

__device__ inline uint32_t file_of_pos(const ScanParams& P, uint64_t pos) {
  const uint64_t r = pos / kNlBlock;
  const uint32_t hi = r + 1 < P.n_regions ? min(P.region_file[r + 1] + 1, P.n_files) : P.n_files;
  return find_file(P.off, P.region_file[r], hi, pos);
}


// The report blob's tables (LDS, or global memory when the blob is too big).
struct RepView {
  const uint8_t* B;  // blob base: the scan image first
  const uint32_t* out_off;
  const uint16_t* out_pat;
  const PatDev* pats;
  const uint8_t* pbytes;
};

__device__ inline RepView rep_view(const AcDev& ac, const uint8_t* B) {
  return RepView{B, (const uint32_t*)(B + ac.o_out_off), (const uint16_t*)(B + ac.o_out_pat),
                 (const PatDev*)(B + ac.o_pats), B + ac.o_pat_bytes};
}

constexpr uint64_t kKwReadFirst = 1ull << 20;  // (report_event's keyword bits)

// The file of an output at pos, given the file of the event's previous output
// (or ~0): one 8-byte group can hold the end of one file, its NUL separator(s)
// and the start of the next, so a cached index is kept only while pos stays
// inside that file.
__device__ inline uint32_t event_file(const ScanParams& P, uint32_t fi, uint64_t pos) {
  if (P.report_mode & 1) return (uint32_t)((pos >> 12) % P.n_files);
  if (fi != 0xFFFFFFFFu && pos < P.off[fi + 1]) return fi;
  return file_of_pos(P, pos);
}

// One event on one lane: replay its 8 bytes on the image, and per output
// confirm the pattern on the real bytes, set the file's keyword gate bit and
// stage the anchor hit in the wave's LDS slots (wbuf / *hcnt_w).
__device__ inline void report_event(const ScanParams& P, const AcDev& ac, const RepView& R, const FastEvent& ev,
                                    uint64_t* wbuf, uint32_t* hcnt_w, uint32_t& my_out, uint64_t& last_kw) {
  const uint32_t out_e = ac.fast_out_entry;
  uint64_t hist = ((uint64_t)ev.prev.y << 32) | ev.prev.x;  // the 8 raw bytes before (oldest low)
  uint64_t hlow = lower64(hist);
  uint32_t e = ev.entry;
  const uint32_t fx = fold6(ev.cur.x), fy = fold6(ev.cur.y);
  uint32_t fi = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    e = fstep(R.B, e, j < 4 ? fx : fy, j & 3);
    const uint32_t c = ((j < 4 ? ev.cur.x : ev.cur.y) >> (8 * (j & 3))) & 0xFFu;
    hist = (hist >> 8) | ((uint64_t)c << 56);  // hist byte 7 = c
    hlow = (hlow >> 8) | ((uint64_t)lower_ascii((uint8_t)c) << 56);
    if (e < out_e || c >= 0x80) continue;  // an output ending on a byte >= 0x80 is an alias
    const uint64_t pos = ev.pos + j;
    const uint32_t st = e;
    for (uint32_t o = R.out_off[st]; o < R.out_off[st + 1]; ++o) {
      const uint32_t pid = R.out_pat[o];
      const PatDev& pd = R.pats[pid];
      // the automaton's prefix on the real bytes (it ran on folded ones)
      if ((hlow & pd.m64) != pd.lo64) continue;
      const bool want_kw = pd.kw_needed != 0;
      bool want_hit = pd.rule_n != 0 && (hist & pd.rqm64) == pd.rq64;
      if (!want_kw && !want_hit) continue;
      const uint32_t tl = pd.len < ac.depth ? pd.len : ac.depth;
      const uint64_t start = pos + 1 - tl - pd.ext;
      if (pd.trunc) {  // the rest of a long pattern, on the batch (rare)
        fi = event_file(P, fi, pos);
        const uint64_t fend = P.off[fi + 1] - 1;
        if (start + pd.len > fend) continue;
        // chunks of 8 batch bytes issued before any compare (one memory
        // latency per chunk; a byte-by-byte early-exit loop was a chain of
        // dependent loads)
        uint32_t bad = 0, req_bad = 0;
        const uint8_t* pb = R.pbytes + pd.bytes_off;
        for (uint32_t k0 = tl; k0 < pd.len && !bad; k0 += 8) {
#pragma unroll
          for (uint32_t k = k0; k < k0 + 8; ++k)
            if (k < pd.len) {
              const uint8_t b = P.data[start + k];
              bad |= lower_ascii(b) ^ pb[k];
              if (want_hit && pd.confirm) {
                const uint8_t r = R.pbytes[pd.req_off + k];
                req_bad |= (r != 0) & (b != r);
              }
            }
        }
        if (bad) continue;
        if (req_bad) want_hit = false;
      }
      ++my_out;
      if (want_kw) {
        fi = event_file(P, fi, pos);
        const uint64_t key = ((uint64_t)fi << 32) | pd.kw;  // per-lane dedupe of repeated keywords
        if (last_kw != key) {
          last_kw = key;
          // fire-and-forget atomic: reading the word first to skip the
          // atomics of repeated keywords put an L2 round trip on the lane's
          // chain (k_report 650 -> 618 us on configs[2] without it,
          // profiles/r04ac) -- except in files of kKwReadFirst bytes or more,
          // whose keyword words every wave hits: atomics on one address
          // serialise in its L2 channel (one 20 GB file: k_report 11.3 ms
          // for a 5.5 ms scan, profiles/r05f)
          uint32_t* wp = &P.file_kw[(size_t)fi * P.rs.kw_words + (pd.kw >> 5)];
          const uint32_t bit = 1u << (pd.kw & 31);
          if (P.off[fi + 1] - P.off[fi] < P.kw_plain ||
              !(__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
            atomicOr(wp, bit);
        }
      }
      if (want_hit) {
        const uint32_t slot = atomicAdd(hcnt_w, 1u);  // (this wave's slots only)
        const uint64_t hrec = (start << 16) | pid;
        if (slot < kReportWaveHits) {
          wbuf[slot] = hrec;
        } else {
          unsigned long long idx = atomicAdd(&P.ctrl->hits, 1ull);
          if (idx < P.hit_cap) P.hits[idx] = hrec;
        }
      }
    }
  }
}

// The wave's staged hits -> its own hit region (P.hit_seg, `seg`; *cursor
// records used: no atomic at all) or, without one or once it is full, P.hits
// with one global reservation -- when half full or `force`; the fences order
// the wave's LDS stores before the reads.  (A returning atomic on one word
// serialises chip-wide at ~90 per us: ~30 K flush reservations were half of
// k_report's time on configs[2].)
__device__ inline void report_flush(const ScanParams& P, uint64_t* wbuf, uint32_t* hcnt_w, uint32_t lane, bool force,
                                    uint64_t* seg = nullptr, uint32_t* cursor = nullptr) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t hc = __shfl(atomicAdd(hcnt_w, 0u), 0);
  if (hc >= kReportWaveHits / 2 || (force && hc)) {
    const uint32_t nh = hc < kReportWaveHits ? hc : kReportWaveHits;
    if (seg && *cursor + nh <= P.hit_seg_cap) {
      for (uint32_t q = lane; q < nh; q += 64) seg[*cursor + q] = wbuf[q];
      *cursor += nh;
    } else {
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(&P.ctrl->hits, (unsigned long long)nh);
      base = __shfl(base, 0);
      for (uint32_t q = lane; q < nh; q += 64)
        if (base + q < P.hit_cap) P.hits[base + q] = wbuf[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane == 0) *hcnt_w = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// The fused scan's resolution of its own segment's events [from, lim) (kept
// out of line: the scan's streaming loop keeps its registers).
__device__ __noinline__ void resolve_segment(const ScanParams& P, const AcDev& ac, const RepView& R,
                                             const FastEvent* ev_seg, uint32_t from, uint32_t lim, uint64_t* wbuf,
                                             uint32_t* hcnt_w, uint32_t lane, uint32_t& my_out, uint64_t& last_kw) {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the wave's event stores before its loads
  for (uint32_t d = from; d < lim; d += 64) {
    const uint32_t i = d + lane;
    if (i < lim) report_event(P, ac, R, ev_seg[i], wbuf, hcnt_w, my_out, last_kw);
    report_flush(P, wbuf, hcnt_w, lane, false);
  }
}

// 64 MiB: on configs[2] a 256 KiB threshold moved 0.43 ms into the scan for
// 0.33 ms less verify / lazy count (step +0.1 ms, profiles/r05g); for one
// 20 GB file the lazy count would read the whole file after the scan.
constexpr uint64_t kNlBig = 64ull << 20;  // (tools/ab_env.sh, TSG_NL_BIG)
// Span sp's newline count comes from the scan (not the lazy k_nl_spans) when
// a file of nl_big bytes or more overlaps it: only the files holding its first
// and its last byte can (the others lie inside the span).  The batch's big
// files are most of the bytes the lazy count would read (every plant file of
// several MB, counted up to its last candidate), and in the scan their count
// costs VALU beside the LDS-bound walk instead of HBM time under k_verify.
__device__ inline bool span_scan_counted(const uint64_t* off, const uint32_t* region_file, uint64_t n_regions,
                                         uint32_t n_files, uint64_t sp, uint64_t nl_big) {
  if (!nl_big || !n_files) return false;
  const uint32_t f0 = region_file[sp];
  uint32_t f1 = sp + 1 < n_regions ? region_file[sp + 1] : n_files - 1;
  if (f1 >= n_files) f1 = n_files - 1;
  auto big = [&](uint32_t f) { return off[f + 1] - off[f] - 1 >= nl_big; };
  return big(f0) || (f1 != f0 && off[f1] < (sp + 1) * kNlBlock && big(f1));
}

// kFuse: the scan resolves its own events (k_report's work, report_event) --
// the whole report blob (the image followed by the output tables) sits in
// LDS, and whenever a wave's segment holds 64 unresolved events the wave
// replays them at a span boundary, one per lane (their global reads --
// file lookups, keyword atomics -- are latency the wave's 15 siblings cover
// by keeping the LDS busy); the rest after the wave's last span.  Only the
// overflow bucket is left to k_report.
template <int CH, int V, int kFastThreads, int kMode = 0, int kWin = 1, bool kPair = false, bool kFuse = false>
__global__ __launch_bounds__(kFastThreads) void k_scan_fast(ScanParams P) {
  constexpr uint32_t kUnit = CH * kNlBlock;          // bytes per lane per work unit
  constexpr int kStep = V * 16;                      // bytes per chain step
  constexpr int kSteps = kNlBlock / kStep;           // steps per span
  // static: LDS base folds to 0 in the step (kPair: the pair table follows the image)
  __shared__ __align__(16) uint8_t smem[kFuse ? kReportLds : kFastImgMax + (kPair ? kFastCols * kFastCols * 2 : 0)];
  __shared__ uint64_t hbuf[kFuse ? kReportHitCap : 1];
  __shared__ uint32_t hcnt[kFuse ? kFastThreads / 64 : 1];
  // keyword states' records and local bits (kw_resolve; not in the exp shapes)
  constexpr bool kKw = !kFuse && !kPair && CH == 1 && kWin != 1 && !(kMode & 4);
  constexpr bool kKwMid = kKw && (kMode & kScanKwMid);
  __shared__ __align__(16) FastKwRec kwrec[kKw ? kFastKwStates * kFastKwPer : 1];
  __shared__ uint16_t kwmap[kKw ? kFastKwBits : 1];
  __shared__ __align__(16) KwRec kwq[kKw ? kFastThreads / 64 * kFastKwQ : 1];
  __shared__ uint32_t kwseen[kKw ? kFastThreads : 1];
  const AcDev& ac = P.rs.ac;
  {
    const uint32_t words = (kFuse ? ac.rep_bytes : ac.fast_bytes) / 4;
    const uint32_t* src = (const uint32_t*)ac.fast_lds;
    for (uint32_t i = threadIdx.x; i < words; i += kFastThreads) ((uint32_t*)smem)[i] = src[i];
    if (kKw && ac.fast_kw_n) {
      const uint32_t rw = ac.fast_kw_n * kFastKwPer * (uint32_t)sizeof(FastKwRec) / 4;
      for (uint32_t i = threadIdx.x; i < rw; i += kFastThreads) ((uint32_t*)kwrec)[i] = ((const uint32_t*)ac.fast_kw)[i];
      const uint16_t* mp = (const uint16_t*)(ac.fast_kw + (size_t)ac.fast_kw_n * kFastKwPer * sizeof(FastKwRec));
      for (uint32_t i = threadIdx.x; i < kFastKwBits; i += kFastThreads) kwmap[i] = mp[i];
    }
    if (kPair) {
      const uint32_t* ps = (const uint32_t*)(ac.fast_lds + ac.o_pair);
      for (uint32_t i = threadIdx.x; i < kFastCols * kFastCols / 2; i += kFastThreads)
        ((uint32_t*)(smem + kFastImgMax))[i] = ps[i];
    }
    if (kFuse && (threadIdx.x & 63) == 0) hcnt[threadIdx.x >> 6] = 0;
    if (kKw) kwseen[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint8_t* T = smem;
  const uint32_t out_e = ac.fast_out_entry;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_lt = (1ull << lane) - 1;
  const uint32_t wave = (blockIdx.x * (kFastThreads / 64)) + (threadIdx.x >> 6);
  const uint64_t nlanes = (uint64_t)gridDim.x * kFastThreads;
  const uint64_t units = (P.nbytes + kUnit - 1) / kUnit;
  FastEvent* ev_seg = P.events + (uint64_t)wave * P.ev_cap_per_wave;
  uint32_t ev_count = 0;  // wave-uniform
  // kFuse: events [0, ev_done) of the segment are resolved (wave-uniform)
  uint32_t ev_done = 0, my_out = 0;
  uint64_t last_kw = ~0ull;
  const RepView R = rep_view(ac, smem);
  uint64_t* wbuf = hbuf + (threadIdx.x >> 6) * (kFuse ? kReportWaveHits : 0);
  uint32_t* hcnt_w = hcnt + (kFuse ? threadIdx.x >> 6 : 0);
  auto resolve = [&](uint32_t lim) {  // events [ev_done, lim), one per lane, 64 at a time
    resolve_segment(P, ac, R, ev_seg, ev_done, lim, wbuf, hcnt_w, lane, my_out, last_kw);
    ev_done = lim;
  };
  uint64_t u = (uint64_t)blockIdx.x * kFastThreads + threadIdx.x;
  FastChain<V> C[CH];
  uint4 nxt[CH][V];
  const KwScan kws{kwrec, kwmap, kwq + (kKw ? (threadIdx.x >> 6) * kFastKwQ : 0), kwseen + (kKw ? threadIdx.x & ~63u : 0),
                   kKw && kw_scan_ok(P) && !P.kw_off ? ac.fast_ev_entry : out_e};
  uint32_t kwn = 0;    // wave-uniform: records in this wave's keyword queue
  uint32_t kseen = 0;  // keyword states (bit: state - out_e) of this span's file already set
  if (u < units) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      C[c].pos = u * kUnit + (uint64_t)c * kNlBlock;
      const uint8_t* src = fast_src(P, C[c].pos);
#pragma unroll
      for (int k = 0; k < V; ++k) nxt[c][k] = *(const uint4*)(src + C[c].pos + 16 * k);
    }
  }
  // uniform per lane, not per wave: finished lanes walk stale bytes silently
  while (__ballot(u < units)) {
    const bool live = u < units;
    const uint64_t un = u + nlanes;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      // warm-up: the 7 bytes before the span (automaton depth <= kAcMaxLit)
      const uint64_t s0 = C[c].pos;
      const uint2 h = live && s0 >= 8 ? *(const uint2*)(fast_src(P, s0 - 8) + s0 - 8) : make_uint2(0, 0);
      uint32_t e = 0;
#pragma unroll
      for (int j = 1; j < 8; ++j) e = fstep(T, e, j < 4 ? fold6(h.x) : fold6(h.y), j & 3);
      C[c].e = e;
      C[c].prev = h;
      C[c].nl = 0;
      C[c].hi = 0;
    }
    // lazy newline counts (kMode 2) except in the spans of files of nl_big
    // bytes or more (span_scan_counted): those this scan counts -- the wave
    // takes the counting loop when any of its lanes' spans needs it
    bool count_nl = false;
    if ((kMode & 2) && P.nl_big && live) {
#pragma unroll
      for (int c = 0; c < CH; ++c)
        count_nl |= C[c].pos < P.nbytes &&
                    span_scan_counted(P.off, P.region_file, P.n_regions, P.n_files, C[c].pos / kNlBlock, P.nl_big);
    }
    {
      const bool cnt = (kMode & 2) && __builtin_amdgcn_readfirstlane((uint32_t)(__ballot(count_nl) != 0));
#pragma unroll
      for (int c = 0; c < CH; ++c) C[c].cnt = cnt;
    }
    for (int step = 0; step < kSteps; ++step) {
      // take the prefetched bytes, then prefetch the chain's next step (same
      // span, or the first step of the lane's next unit)
      uint64_t np[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
#pragma unroll
        for (int k = 0; k < V; ++k) C[c].cur[k] = nxt[c][k];
        np[c] = step + 1 < kSteps ? C[c].pos + kStep : un * kUnit + (uint64_t)c * kNlBlock;
      }
      if (live && (step + 1 < kSteps || un < units)) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const uint8_t* src = fast_src(P, np[c]);
#pragma unroll
          for (int k = 0; k < V; ++k) {
            if (kMode & 4) nxt[c][k] = *(const uint4*)(P.data + ((np[c] + 16 * k) & 0xFFFF0ull));
            else nxt[c][k] = *(const uint4*)(src + np[c] + 16 * k);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        if (CH == 2) {
          const uint4 v = C[0].cur[k], w = C[CH - 1].cur[k];
          fast_group2(P, T, out_e, C[0], C[CH - 1], v.x, v.y, w.x, w.y, C[0].pos + 16 * k, C[CH - 1].pos + 16 * k, live,
                      lanes_lt, ev_seg, &ev_count);
          fast_group2(P, T, out_e, C[0], C[CH - 1], v.z, v.w, w.z, w.w, C[0].pos + 16 * k + 8,
                      C[CH - 1].pos + 16 * k + 8, live, lanes_lt, ev_seg, &ev_count);
        } else if (kWin == 2) {
          const uint4 v = C[0].cur[k];
          const uint32_t d[4] = {v.x, v.y, v.z, v.w};
          fast_window<V, kMode, 2>(P, T, out_e, C[0], d, C[0].pos + 16 * k, live, lanes_lt, ev_seg, &ev_count,
                                   kKw ? &kws : nullptr, &kwn, kseen);
        } else if (kWin == 8) {
          if (k % 4 == 0) {
            const uint4 a = C[0].cur[k], b = C[0].cur[k + 1 < V ? k + 1 : k];
            const uint4 c2 = C[0].cur[k + 2 < V ? k + 2 : k], d2 = C[0].cur[k + 3 < V ? k + 3 : k];
            const uint32_t d[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c2.x, c2.y, c2.z, c2.w, d2.x, d2.y, d2.z, d2.w};
            fast_window<V, kMode, 8>(P, T, out_e, C[0], d, C[0].pos + 16 * k, live, lanes_lt, ev_seg, &ev_count,
                                     kKw ? &kws : nullptr, &kwn, kseen);
          }
        } else if (kWin == 4) {
          if (k % 2 == 0) {
            const uint4 v = C[0].cur[k], w = C[0].cur[k + 1 < V ? k + 1 : k];
            const uint32_t d[8] = {v.x, v.y, v.z, v.w, w.x, w.y, w.z, w.w};
            fast_window<V, kMode, 4, kPair>(P, T, out_e, C[0], d, C[0].pos + 16 * k, live, lanes_lt, ev_seg,
                                            &ev_count, kKw ? &kws : nullptr, &kwn, kseen);
          }
        } else {
          const uint4 v = C[0].cur[k];
          fast_group<V, kMode>(P, T, out_e, C[0], v.x, v.y, C[0].pos + 16 * k, live, lanes_lt, ev_seg, &ev_count);
          fast_group<V, kMode>(P, T, out_e, C[0], v.z, v.w, C[0].pos + 16 * k + 8, live, lanes_lt, ev_seg, &ev_count);
        }
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) C[c].pos = np[c];
      // a step of a wave can queue ~8 groups on keyword-dense text (configs[1]:
      // 'sk' once per KiB), a span ~256: drained after a step before it fills
      // -- kKwMid only (the prefilter-only scan): the drain's code inside the
      // step loop cost the full ruleset's scan 0.5 ms on configs[2] even where
      // it never ran (same-box A/B, profiles/r06k), span-end drains none
      if (kKwMid && P.kw_drain_at && kwn >= P.kw_drain_at) kw_drain(P, T, kws, out_e, kwn, kseen, lane);  // (wave-uniform)
    }
    if (live) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const uint64_t s0 = u * kUnit + (uint64_t)c * kNlBlock;
        if (s0 < P.nbytes) {
          if (!(kMode & 2) || count_nl) P.nl_blocks[s0 / kNlBlock] = C[c].nl;
          P.span_hi[s0 / kNlBlock] = (C[c].hi & 0x80808080u) ? 1 : 0;
        }
      }
    }
    if (kKw && kwn) kw_drain(P, T, kws, out_e, kwn, kseen, lane);  // (wave-uniform)
    if (kKw) {  // the next span's file: nothing seen
      kseen = 0;
      kws.seen[lane] = 0;
    }
    u = un;
    if (kFuse && !(P.report_mode & 4)) {  // whole rounds of 64 only: the wave goes back to streaming after them
      const uint32_t lim = ev_count < P.ev_cap_per_wave ? ev_count : (uint32_t)P.ev_cap_per_wave;
      if (lim - ev_done >= 64) resolve(ev_done + (lim - ev_done) / 64 * 64);
    }
  }
  if (lane == 0) P.ev_counts[wave] = ev_count < P.ev_cap_per_wave ? ev_count : P.ev_cap_per_wave;
  if (kFuse) {
    const uint32_t lim = ev_count < P.ev_cap_per_wave ? ev_count : (uint32_t)P.ev_cap_per_wave;
    resolve(lim);
    report_flush(P, wbuf, hcnt_w, lane, true);
    for (uint32_t d = 32; d; d >>= 1) my_out += __shfl_xor(my_out, d);
    if (lane == 0) {
      if (my_out) atomicAdd(&P.ctrl->outputs, (unsigned long long)my_out);
      if (lim) atomicAdd(&P.ctrl->events, (unsigned long long)lim);
    }
  }
}

#ifdef TSG_EXPERIMENTS
// Timing bound of a stride-2 trigram front filter (exp
// build, WRONG results): k_scan_fast's load shape (one 4 KiB span per lane,
// 128-byte register ring), but instead of one DFA step per byte, per even
// position one ds_read_b64 of a 64-bit mask indexed by the fold columns of
// bytes p, p + 1 (32 KiB: 4096 pairs) and a test of bit column(p + 2) -- 0.5
// LDS gathers per byte, no dependent chain, no replay of flagged groups and
// no events (a ballot per window keeps the work).  Whatever this costs is a
// floor for a filter-then-replay design on this load shape.
__global__ __launch_bounds__(1024) void k_scan_tri(ScanParams P) {
  __shared__ __align__(16) uint64_t tri[4096];
  for (uint32_t i = threadIdx.x; i < 4096; i += 1024) tri[i] = (i * 0x9E3779B97F4A7C15ull) & 0x0000010000000101ull;
  __syncthreads();
  const uint64_t nlanes = (uint64_t)gridDim.x * 1024;
  const uint64_t units = (P.nbytes + kNlBlock - 1) / kNlBlock;
  uint64_t u = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  uint4 nxt[8];
  uint64_t pos = u * kNlBlock;
  if (u < units) {
    const uint8_t* src = fast_src(P, pos);
#pragma unroll
    for (int k = 0; k < 8; ++k) nxt[k] = *(const uint4*)(src + pos + 16 * k);
  }
  uint32_t found = 0;
  while (__ballot(u < units)) {
    const bool live = u < units;
    const uint64_t un = u + nlanes;
    for (int step = 0; step < (int)(kNlBlock / 128); ++step) {
      uint4 cur[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
      const uint64_t np = step + 1 < (int)(kNlBlock / 128) ? pos + 128 : un * kNlBlock;
      if (live && (step + 1 < (int)(kNlBlock / 128) || un < units)) {
        const uint8_t* src = fast_src(P, np);
#pragma unroll
        for (int k = 0; k < 8; ++k) nxt[k] = *(const uint4*)(src + np + 16 * k);
      }
      uint32_t flag = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t w[5] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w, k + 1 < 8 ? cur[k + 1].x : cur[k].x};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t f = fold6(w[q]), fn = fold6(w[q + 1]);  // bytes = 2 x column
#pragma unroll
          for (int j = 0; j < 4; j += 2) {  // positions 4q + j, j even
            const uint32_t b0 = (f >> (8 * j)) & 0xFFu, b1 = j + 1 < 4 ? (f >> (8 * (j + 1))) & 0xFFu : fn & 0xFFu;
            const uint32_t b2 = j + 2 < 4 ? (f >> (8 * (j + 2))) & 0xFFu : (fn >> (8 * (j - 2))) & 0xFFu;
            const uint64_t m = tri[(b0 << 5) | (b1 >> 1)];
            flag |= (uint32_t)(m >> (b2 >> 1)) & 1u;
          }
        }
        if ((k & 3) == 3) {  // one wave-level check per 64 bytes (as k_scan_fast's event window)
          if (__ballot(flag & (live ? 1u : 0u))) found += flag;
          flag = 0;
        }
      }
      pos = np;
    }
    u = un;
  }
  if (found == 0xFFFFFFFFu) P.ctrl->err = found;  // (keeps the work observable)
}
#endif

// Scan with an automaton too large for k_scan_fast's image (configs[4]: 1000+
// custom rules), in k_scan_fast's shape: 4 KiB spans (7 bytes of warm-up)
// streamed through register rings, 1024 threads and ONE LDS copy of the
// automaton per CU (BigDev: byte classes, dense rows of the first states,
// 8-byte cold-state records + failure links for the rest).  The byte
// class lookups do not depend on the state, so only the row lookup sits on the
// dependent chain.  Outputs: entries carry bit 15; the OR over an 8-byte group
// flags it, and a flagged group becomes a FastEvent (ballot/popcount into the
// wave's segment) that k_big_walk replays -- no per-byte output branch, no
// global atomics, newlines counted SWAR and stored once per span.
constexpr uint32_t kBigThreads = 1024;
// k_scan_big's product shape (tools/big_ab.sh, profiles/r03l): two chains
// per lane, each with a 2 x 16-byte ring, every chain's dense row read issued
// before any cold walk -- 8.87 vs 9.63 ms (one chain, 8 x 16 B) on configs[4]
constexpr int kBigMode = 8, kBigChains = 2;
[[maybe_unused]] constexpr int kBigRing = 2;  // (k_scan_big, exp build only)
constexpr int kBigNoNl = 32;  // kMode bit: no per-span newline counts (the engine's nl_lazy)
constexpr uint32_t kBigLdsMax = 160 * 1024 - 256;  // the blob's LDS part (k_big_walk adds 80 B of its own)
// Cold records kept in LDS at least (the rest of the blob's cold records
// are read from global memory, L2-resident): more dense rows pay more than
// LDS records of deep states -- on the bench text, cold-state visits per
// byte are 0.0033 past 1202 dense rows and 0.0011 past 1400, 0.0003 past
// 2445 (tools/big_visits.py, profiles/r04j/big_visits.txt).
constexpr uint32_t kBigColdLdsMin = 4096;
// (tsg_big_cold_lds_floor, diagnostics: a GPU test sets 0 to read nearly
// every cold record from global memory)
static std::atomic<uint32_t> g_big_cold_floor{kBigColdLdsMin};

struct BigLds {
  const uint8_t* cls;
  const uint16_t* dense;
  const uint2* cold;   // LDS: records [0, CL)
  __attribute__((address_space(1))) const uint32_t* gcold;  // global: every record, as dword pairs (read past CL)
  const uint32_t* eval;
  uint32_t K, ND, CL;
};

__device__ inline BigLds big_lds(const BigDev& B, const uint8_t* smem, uint32_t K) {
  return BigLds{smem, (const uint16_t*)(smem + 256), (const uint2*)(smem + B.o_cold),
                (__attribute__((address_space(1))) const uint32_t*)(B.blob + B.o_cold),
                (const uint32_t*)(smem + B.o_eval), K, B.n_dense, B.n_cold_lds};
}

// delta(st, c): a cold state's own entry (where it differs from its first
// dense ancestor), else the ancestor's dense entry.  Entry bit 15 = output
// state.  The records of the deepest (rarely visited) cold states are read
// from global memory.
__device__ inline uint2 big_rec(const BigLds& L, uint32_t j) {
  uint2 r;  // x: c1 | c2 << 8 | entry1 << 16, y: entry2 | dense ancestor << 16
  if (j < L.CL) {
    r = L.cold[j];
  } else {  // (a global load of its own: a generic one would wait for the batch prefetches too)
    r.x = L.gcold[2 * j];
    r.y = L.gcold[2 * j + 1];
  }
  return r;
}
__device__ inline uint32_t big_list(const BigLds& L, uint2 r, uint32_t c) {  // 0xFFFFFFFF: not listed
  for (uint32_t k = (r.x >> 16) | ((r.y & 0xFFFFu) << 16);; ++k) {
    const uint32_t v = L.eval[k];
    if (v == 0xFFFFFFFFu || (v >> 16) == c) return v == 0xFFFFFFFFu ? v : (v & 0xFFFFu);
  }
}
__device__ inline uint32_t big_next(const BigLds& L, uint32_t st, uint32_t c) {
  if (st >= L.ND) {
    const uint2 r = big_rec(L, st - L.ND);
    if (c == (r.x & 0xFFu)) return r.x >> 16;
    if (c == ((r.x >> 8) & 0xFFu)) return r.y & 0xFFFFu;
    if ((r.x & 0xFFu) == kBigMore) {
      const uint32_t v = big_list(L, r, c);
      if (v != 0xFFFFFFFFu) return v;
    }
    st = r.y >> 16;
  }
  return L.dense[__umul24(st, L.K) + c];
}

// 8 bytes (two dwords) of each of CH chains through the automaton from their
// entries e[c]; acc[c] = the OR of a chain's entries (bit 15 = some output
// state was reached).  The chains are independent, so their row lookups
// overlap in one lane.  kMode != 0 only in the -DTSG_EXPERIMENTS build
// (TSG_BIG_VARIANT; bits 0/1/4 are timing bounds with wrong results): bit 0 =
// class from ALU instead of LDS, bit 1 = dense rows only, bit 3 = every
// chain's dense row read issued before any cold walk, bit 4 (with 3) = the
// per-byte cold test and branch without the cold walk.
template <int kMode, int CH>
__device__ inline void big_group(const BigLds& L, uint32_t (&e)[CH], const uint32_t (&d)[2 * CH],
                                 uint32_t (&acc)[CH]) {
  uint32_t c[CH][8];
#pragma unroll
  for (int h = 0; h < CH; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t b = (d[2 * h + (j >> 2)] >> (8 * (j & 3))) & 0xFFu;
      c[h][j] = (kMode & 1) ? (b & 31u) : L.cls[b];
    }
#pragma unroll
  for (int h = 0; h < CH; ++h) acc[h] = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t nx[CH];
    if (kMode & 10) {
#pragma unroll
      for (int h = 0; h < CH; ++h)  // (byte offset: one v_mad_u32_u24)
        nx[h] = *(const uint16_t*)((const uint8_t*)L.dense + (__umul24(min(e[h], L.ND - 1), 2 * L.K) + 2 * c[h][j]));
    }
    if ((kMode & 10) == 8) {
      // one wave-uniform test for every chain (a divergent if per chain cost
      // three scalar exec-mask instructions per byte each)
      bool cold = false;
#pragma unroll
      for (int h = 0; h < CH; ++h) cold |= e[h] >= L.ND;
      if (__ballot(cold)) {
        if (kMode & 16) {  // timing bound (wrong results): the test and branch without the cold walk
#pragma unroll
          for (int h = 0; h < CH; ++h) nx[h] ^= e[h] >= L.ND ? 1u : 0u;
        } else {
          // every lane, both chains: record, then the row (own entry or the
          // dense ancestor's), two LDS round trips per chain set; global
          // records and overflow lists only for the lanes that have them
          uint2 r[CH];
          bool isc[CH];
#pragma unroll
          for (int h = 0; h < CH; ++h) {
            isc[h] = e[h] >= L.ND;
            const uint32_t jj = isc[h] ? e[h] - L.ND : 0u;
            r[h] = L.cold[min(jj, L.CL - 1)];
            if (jj >= L.CL) r[h] = big_rec(L, jj);
          }
          uint32_t dn[CH];
#pragma unroll
          for (int h = 0; h < CH; ++h) dn[h] = L.dense[__umul24(isc[h] ? r[h].y >> 16 : 0u, L.K) + c[h][j]];
#pragma unroll
          for (int h = 0; h < CH; ++h) {
            const uint32_t cc = c[h][j], c1 = r[h].x & 0xFFu, c2 = (r[h].x >> 8) & 0xFFu;
            uint32_t v = cc == c1 ? r[h].x >> 16 : cc == c2 ? r[h].y & 0xFFFFu : dn[h];
            if (c1 == kBigMore && isc[h]) {
              const uint32_t w = big_list(L, r[h], cc);
              if (w != 0xFFFFFFFFu) v = w;
            }
            if (isc[h]) nx[h] = v;
          }
        }
      }
    } else if (!(kMode & 2)) {
#pragma unroll
      for (int h = 0; h < CH; ++h) nx[h] = big_next(L, e[h], c[h][j]);
    }
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      acc[h] |= nx[h];
      e[h] = nx[h] & 0x7FFFu;
    }
  }
}

__device__ inline void big_event(const ScanParams& P, uint64_t b, uint32_t lane, uint64_t lanes_lt, uint64_t pos,
                                 uint32_t entry, uint2 prev, uint32_t d0, uint32_t d1, FastEvent* ev_seg,
                                 uint32_t ev_count) {
  if ((b >> lane) & 1) {
    FastEvent r;
    r.pos = pos;
    r.entry = entry;
    r.pad = 0;
    r.prev = prev;
    r.cur = make_uint2(d0, d1);
    const uint32_t slot = ev_count + (uint32_t)__popcll(b & lanes_lt);
    if (slot < P.ev_cap_per_wave) {
      ev_seg[slot] = r;
    } else {
      unsigned long long ov = atomicAdd(&P.ctrl->ev_overflow, 1ull);
      if (ov < P.ev_overflow_cap) P.ev_overflow[ov] = r;
    }
  }
}

// CH chains per lane: lane unit u covers the CH consecutive 4 KiB spans
// u * CH .. u * CH + CH - 1, each walked by its own chain (kBigRing bytes of
// register ring per chain).  Bit 2 of kMode: one event ballot per 16 bytes
// (both groups of a dword quad) instead of per group.
template <int kMode = 0, int CH = 1, int V = 8 / CH>
__global__ __launch_bounds__(kBigThreads) void k_scan_big(ScanParams P) {
  extern __shared__ __align__(16) uint8_t smem[];
  const BigDev& B = P.big;
  for (uint32_t i = threadIdx.x; i < B.lds_bytes / 4; i += kBigThreads)
    ((uint32_t*)smem)[i] = ((const uint32_t*)B.blob)[i];
  __syncthreads();
  const BigLds L = big_lds(B, smem, P.rs.ac.nclasses);
  constexpr int kStep = V * 16;
  constexpr int kSteps = kNlBlock / kStep;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_lt = (1ull << lane) - 1;
  const uint32_t wave = blockIdx.x * (kBigThreads / 64) + (threadIdx.x >> 6);
  const uint64_t nlanes = (uint64_t)gridDim.x * kBigThreads;
  const uint64_t spans = (P.nbytes + kNlBlock - 1) / kNlBlock;
  const uint64_t units = (spans + CH - 1) / CH;
  FastEvent* ev_seg = P.events + (uint64_t)wave * P.ev_cap_per_wave;
  uint32_t ev_count = 0;  // wave-uniform
  uint64_t u = (uint64_t)blockIdx.x * kBigThreads + threadIdx.x;
  uint4 cur[CH][V], nxt[CH][V];
  uint64_t pos[CH];
  bool live[CH];
#pragma unroll
  for (int h = 0; h < CH; ++h) {
    pos[h] = (u * CH + h) * kNlBlock;
    live[h] = u * CH + h < spans;
    if (live[h]) {
      const uint8_t* src = fast_src(P, pos[h]);
#pragma unroll
      for (int k = 0; k < V; ++k) nxt[h][k] = *(const uint4*)(src + pos[h] + 16 * k);
    }
  }
  while (__ballot(u < units)) {
    const uint64_t un = u + nlanes;
    uint64_t s0[CH];
    uint32_t e[CH], nl[CH], hi[CH];
    uint2 prev[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      s0[h] = pos[h];
      live[h] = u * CH + h < spans;
      const uint2 w = live[h] && s0[h] >= 8 ? *(const uint2*)(fast_src(P, s0[h] - 8) + s0[h] - 8) : make_uint2(0, 0);
      e[h] = 0;
      // warm-up: the 7 bytes before the span (automaton depth <= kAcMaxLit)
#pragma unroll
      for (int j = 1; j < 8; ++j)
        e[h] = big_next(L, e[h], L.cls[((j < 4 ? w.x : w.y) >> (8 * (j & 3))) & 0xFFu]) & 0x7FFFu;
      prev[h] = w;
      nl[h] = 0;
      hi[h] = 0;
    }
    for (int step = 0; step < kSteps; ++step) {
      uint64_t np[CH];
#pragma unroll
      for (int h = 0; h < CH; ++h) {
#pragma unroll
        for (int k = 0; k < V; ++k) cur[h][k] = nxt[h][k];
        np[h] = step + 1 < kSteps ? pos[h] + kStep : (un * CH + h) * kNlBlock;
        if (live[h] && (step + 1 < kSteps || un * CH + h < spans)) {
          const uint8_t* src = fast_src(P, np[h]);
#pragma unroll
          for (int k = 0; k < V; ++k) nxt[h][k] = *(const uint4*)(src + np[h] + 16 * k);
        }
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        uint32_t gs[2][CH], acc[2][CH];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          uint32_t d[2 * CH];
#pragma unroll
          for (int h = 0; h < CH; ++h) {
            d[2 * h] = g ? cur[h][k].z : cur[h][k].x;
            d[2 * h + 1] = g ? cur[h][k].w : cur[h][k].y;
            if (!(kMode & kBigNoNl)) nl[h] += nl_count_dword(d[2 * h]) + nl_count_dword(d[2 * h + 1]);
            hi[h] |= d[2 * h] | d[2 * h + 1];
            gs[g][h] = e[h];
          }
          big_group<kMode, CH>(L, e, d, acc[g]);
          if (!(kMode & 4)) {
#pragma unroll
            for (int h = 0; h < CH; ++h) {
              const uint64_t b = __ballot(live[h] && (acc[g][h] & 0x8000u));
              if (b) {
                big_event(P, b, lane, lanes_lt, pos[h] + 16 * k + 8 * g, gs[g][h], prev[h], d[2 * h], d[2 * h + 1],
                          ev_seg, ev_count);
                ev_count += (uint32_t)__popcll(b);
              }
              prev[h] = make_uint2(d[2 * h], d[2 * h + 1]);
            }
          }
        }
        if (kMode & 4) {
          uint32_t any = 0;
#pragma unroll
          for (int h = 0; h < CH; ++h) any |= live[h] ? (acc[0][h] | acc[1][h]) : 0u;
          if (__ballot(any & 0x8000u)) {
#pragma unroll
            for (int h = 0; h < CH; ++h)
#pragma unroll
              for (int g = 0; g < 2; ++g) {
                const uint32_t d0 = g ? cur[h][k].z : cur[h][k].x, d1 = g ? cur[h][k].w : cur[h][k].y;
                const uint64_t b = __ballot(live[h] && (acc[g][h] & 0x8000u));
                if (b) {
                  big_event(P, b, lane, lanes_lt, pos[h] + 16 * k + 8 * g, gs[g][h], prev[h], d0, d1, ev_seg,
                            ev_count);
                  ev_count += (uint32_t)__popcll(b);
                }
                prev[h] = make_uint2(d0, d1);
              }
          }
#pragma unroll
          for (int h = 0; h < CH; ++h) prev[h] = make_uint2(cur[h][k].z, cur[h][k].w);
        }
      }
#pragma unroll
      for (int h = 0; h < CH; ++h) pos[h] = np[h];
    }
#pragma unroll
    for (int h = 0; h < CH; ++h)
      if (live[h]) {
        P.nl_blocks[s0[h] / kNlBlock] = nl[h];
        P.span_hi[s0[h] / kNlBlock] = (hi[h] & 0x80808080u) ? 1 : 0;
      }
    u = un;
  }
  if (lane == 0) P.ev_counts[wave] = ev_count < P.ev_cap_per_wave ? ev_count : P.ev_cap_per_wave;
}

// k_scan_big with coalesced whole-line loads: the unit of a chain is ONE
// 128-byte line, and lane l's chain h takes line base + 64 h + l, so a wave
// reads 64 consecutive lines per chain with eight back-to-back dwordx4 loads
// each (every line fetched once: the span-per-lane shape re-fetched each
// line from L2 / MALL once per 32-byte ring step, 3.6x its bytes,
// profiles/r04w_c4).  The price: every line restarts the automaton from the
// root over the 7 bytes before it (kAcMaxLit - 1), 5.5 % more steps; those
// bytes are the previous lane's (or chain's) last ones, passed by shuffle.
// Per-span newline counts and >= 0x80 flags are summed over the 32 lanes of
// a span.  Events as k_scan_big's (k_big_walk replays them).
template <int kMode = 8, int CH = 2>
__global__ __launch_bounds__(kBigThreads) void k_scan_lines(ScanParams P) {
  extern __shared__ __align__(16) uint8_t smem[];
  const BigDev& B = P.big;
  for (uint32_t i = threadIdx.x; i < B.lds_bytes / 4; i += kBigThreads)
    ((uint32_t*)smem)[i] = ((const uint32_t*)B.blob)[i];
  __syncthreads();
  const BigLds L = big_lds(B, smem, P.rs.ac.nclasses);
  constexpr uint32_t kLine = 128;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_lt = (1ull << lane) - 1;
  const uint32_t wave = blockIdx.x * (kBigThreads / 64) + (threadIdx.x >> 6);
  const uint64_t n_waves = (uint64_t)gridDim.x * (kBigThreads / 64);
  const uint64_t n_lines = (P.nbytes + kLine - 1) / kLine;
  FastEvent* ev_seg = P.events + (uint64_t)wave * P.ev_cap_per_wave;
  uint32_t ev_count = 0;  // wave-uniform
  for (uint64_t base = (uint64_t)wave * 64 * CH; base < n_lines; base += n_waves * 64 * CH) {
    uint4 cur[CH][8];
    uint64_t pos[CH];
    bool live[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      pos[h] = (base + 64 * h + lane) * kLine;
      live[h] = pos[h] < P.nbytes;
      const uint8_t* src = fast_src(P, pos[h]) + pos[h];
#pragma unroll
      for (int k = 0; k < 8; ++k) cur[h][k] = live[h] ? *(const uint4*)(src + 16 * k) : make_uint4(0, 0, 0, 0);
    }
    // the 8 bytes before each line: the previous lane's last 8, for lane 0 the
    // previous chain's lane 63, for chain 0's lane 0 the batch
    uint2 prev[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      uint32_t pz = __shfl_up(cur[h][7].z, 1), pw = __shfl_up(cur[h][7].w, 1);
      if (h > 0) {
        const uint32_t qz = __shfl(cur[h - 1][7].z, 63), qw = __shfl(cur[h - 1][7].w, 63);
        if (lane == 0) pz = qz, pw = qw;
      } else if (lane == 0) {
        const uint2 w = live[0] && pos[0] >= 8 ? *(const uint2*)(fast_src(P, pos[0] - 8) + pos[0] - 8) : make_uint2(0, 0);
        pz = w.x, pw = w.y;
      }
      prev[h] = make_uint2(pz, pw);
    }
    uint32_t e[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) {  // warm-up: the 7 bytes before the line (automaton depth <= kAcMaxLit)
      e[h] = 0;
#pragma unroll
      for (int j = 1; j < 8; ++j)
        e[h] = big_next(L, e[h], L.cls[((j < 4 ? prev[h].x : prev[h].y) >> (8 * (j & 3))) & 0xFFu]) & 0x7FFFu;
    }
    uint32_t nl[CH], hi[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) nl[h] = hi[h] = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        uint32_t d[2 * CH], gs[CH], acc[CH];
#pragma unroll
        for (int h = 0; h < CH; ++h) {
          d[2 * h] = g ? cur[h][k].z : cur[h][k].x;
          d[2 * h + 1] = g ? cur[h][k].w : cur[h][k].y;
          if (!(kMode & kBigNoNl)) nl[h] += nl_count_dword(d[2 * h]) + nl_count_dword(d[2 * h + 1]);
          hi[h] |= d[2 * h] | d[2 * h + 1];
          gs[h] = e[h];
        }
        big_group<kMode, CH>(L, e, d, acc);
#pragma unroll
        for (int h = 0; h < CH; ++h) {
          const uint64_t b = __ballot(live[h] && (acc[h] & 0x8000u));
          if (b) {
            big_event(P, b, lane, lanes_lt, pos[h] + 16 * k + 8 * g, gs[h], prev[h], d[2 * h], d[2 * h + 1], ev_seg,
                      ev_count);
            ev_count += (uint32_t)__popcll(b);
          }
          prev[h] = make_uint2(d[2 * h], d[2 * h + 1]);
        }
      }
    }
    // per 4 KiB span (32 lanes of a chain): newline count and the >= 0x80 flag
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      uint32_t n = nl[h], f = (hi[h] & 0x80808080u) ? 1u : 0u;
#pragma unroll
      for (int d = 1; d < 32; d <<= 1) {
        n += __shfl_xor(n, d);
        f |= __shfl_xor(f, d);
      }
      if ((lane & 31) == 0 && live[h]) {
        const uint64_t sp = pos[h] / kNlBlock;
        if (!(kMode & kBigNoNl)) P.nl_blocks[sp] = n;
        P.span_hi[sp] = f;
      }
    }
  }
  if (lane == 0) P.ev_counts[wave] = ev_count < P.ev_cap_per_wave ? ev_count : P.ev_cap_per_wave;
}

// Anchor hits of k_big_resolve are staged in LDS and appended to P.hits with
// one global atomic per block round (a global atomic per hit on the one
// counter serialised at L2: 2.3 M hits cost 27 ms on configs[4]); overflow
// past the stage goes straight to global.
template <uint32_t kCap>
struct LdsStageSink {
  uint64_t* buf;
  uint32_t* cnt;
  __device__ void push(const ScanParams& P, uint64_t rec) {
    const uint32_t i = atomicAdd(cnt, 1u);
    if (i < kCap) {
      buf[i] = rec;
    } else {
      GlobalHitSink g;
      g.push(P, rec);
    }
  }
};

__device__ inline uint32_t wave_incl_sum32(uint32_t v, uint32_t lane) {
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  return v;
}
__device__ inline uint32_t block_incl_sum32(uint32_t v, uint32_t* lds16, uint32_t* tot) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_incl_sum32(v, lane);
  if (lane == 63) lds16[wv] = v;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
    if (k < wv) before += lds16[k];
    all += lds16[k];
  }
  __syncthreads();
  *tot = all;
  return v + before;
}

// Event resolution, part 1 (k_big_walk): each event's 8-byte group is replayed from its entry
// state (blob in LDS) and every output state reached becomes one record
// (position << 16 | state) in P.big_outs -- one block-wide prefix sum and one
// global reservation (Ctrl::outputs) per 1024 events.  Only LDS work: the
// outputs' global lookups are left to k_big_resolve, which runs without the
// blob at full occupancy (resolving them here, one event per lane in
// lock-step rounds, left the block waiting on each round's slowest chain of
// dependent global reads: 3.0 ms on configs[4]).
__global__ __launch_bounds__(1024) void k_big_walk(ScanParams P, uint32_t n_waves) {
  extern __shared__ __align__(16) uint8_t smem[];
  const BigDev& B = P.big;
  for (uint32_t i = threadIdx.x; i < B.lds_bytes / 4; i += blockDim.x)
    ((uint32_t*)smem)[i] = ((const uint32_t*)B.blob)[i];
  __shared__ uint32_t s32[16];
  __shared__ unsigned long long obase;
  __syncthreads();
  const BigLds L = big_lds(B, smem, P.rs.ac.nclasses);
  for (uint32_t w = blockIdx.x; w < n_waves + 1; w += gridDim.x) {
    const FastEvent* seg;
    uint64_t n;
    if (w < n_waves) {
      seg = P.events + (uint64_t)w * P.ev_cap_per_wave;
      n = P.ev_counts[w];
      if (threadIdx.x == 0 && n) atomicAdd(&P.ctrl->events, (unsigned long long)n);
    } else {  // overflow bucket
      seg = P.ev_overflow;
      n = P.ctrl->ev_overflow < P.ev_overflow_cap ? P.ctrl->ev_overflow : P.ev_overflow_cap;
    }
    for (uint64_t r0 = 0; r0 < n; r0 += blockDim.x) {
      const uint64_t i = r0 + threadIdx.x;
      uint32_t st[8], cnt = 0;
      uint64_t pos = 0;
      if (i < n) {
        const FastEvent ev = seg[i];
        pos = ev.pos;
        uint32_t e = ev.entry;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t nx = big_next(L, e, L.cls[((j < 4 ? ev.cur.x : ev.cur.y) >> (8 * (j & 3))) & 0xFFu]);
          e = nx & 0x7FFFu;
          st[j] = (nx & 0x8000u) ? e : 0xFFFFu;
          cnt += nx >> 15;
        }
      }
      uint32_t tot;
      const uint32_t incl = block_incl_sum32(cnt, s32, &tot);
      if (threadIdx.x == 0) obase = atomicAdd(&P.ctrl->outputs, (unsigned long long)tot);
      __syncthreads();  // (the next round's scan barriers order this read before obase's next write)
      if (cnt) {
        uint64_t k = obase + incl - cnt;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (st[j] != 0xFFFFu) {
            if (k < P.big_out_cap) P.big_outs[k] = ((pos + j) << 16) | B.ac_of[st[j]];
            ++k;
          }
      }
    }
  }
}

// Event resolution, part 2 (k_big_resolve): one output record per lane (grid-stride), resolved by
// report_t (file lookup, truncated-literal and case checks on the real bytes,
// keyword gate bits, anchor hits); hits staged in LDS, one global
// reservation per block round.
constexpr uint32_t kResolveThreads = 256, kResolveStage = 2048;
__global__ __launch_bounds__(kResolveThreads) void k_big_resolve(ScanParams P) {
  __shared__ uint64_t stage[kResolveStage];
  __shared__ uint32_t n_stage;
  __shared__ unsigned long long base;
  const uint64_t n = P.ctrl->outputs < P.big_out_cap ? P.ctrl->outputs : P.big_out_cap;
  uint64_t last_kw = ~0ull;
  const uint64_t stride = (uint64_t)gridDim.x * kResolveThreads;
  if (threadIdx.x == 0) n_stage = 0;
  __syncthreads();
  for (uint64_t r0 = (uint64_t)blockIdx.x * kResolveThreads; r0 < n; r0 += stride) {
    const uint64_t i = r0 + threadIdx.x;
    LdsStageSink<kResolveStage> sink{stage, &n_stage};
    if (i < n) {
      const uint64_t rec = P.big_outs[i];
      report_t<false>(P, (uint32_t)(rec & 0xFFFFu), rec >> 16, &last_kw, sink);
    }
    __syncthreads();
    const uint32_t m = n_stage < kResolveStage ? n_stage : kResolveStage;
    if (threadIdx.x == 0) base = m ? atomicAdd(&P.ctrl->hits, (unsigned long long)m) : 0ull;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < m; k += kResolveThreads)
      if (base + k < P.hit_cap) P.hits[base + k] = stage[k];
    __syncthreads();
    if (threadIdx.x == 0) n_stage = 0;
    __syncthreads();
  }
}

#ifdef TSG_EXPERIMENTS  // A/B shapes measured slower; not in the product library
// Deep-prefetch shape of k_scan_fast (one chain per lane): the lane's span
// streams through a ring of R = D + 1 register sets of V 16-byte vectors, and
// step s issues the loads of step s + D before walking set s mod R — so every
// load has D steps of automaton work to land in, for the same registers as
// the 1x8 cur/nxt pair when R * V = 16.  The ring runs on across the lane's
// units (kSteps is a multiple of R), so a unit's first steps were prefetched
// during the previous unit.
template <int V, int D, int kFastThreads, int kMode = 0>
__global__ __launch_bounds__(kFastThreads) void k_scan_deep(ScanParams P) {
  constexpr uint32_t kUnit = kNlBlock;
  constexpr int kStep = V * 16;
  constexpr int kSteps = kNlBlock / kStep;
  constexpr int R = D + 1;
  static_assert(kSteps % R == 0 && D < kSteps, "ring must tile the span");
  __shared__ __align__(16) uint8_t smem[kFastImgMax];
  const AcDev& ac = P.rs.ac;
  {
    const uint32_t words = ac.fast_bytes / 4;
    const uint32_t* src = (const uint32_t*)ac.fast_lds;
    for (uint32_t i = threadIdx.x; i < words; i += kFastThreads) ((uint32_t*)smem)[i] = src[i];
  }
  __syncthreads();
  const uint8_t* T = smem;
  const uint32_t out_e = ac.fast_out_entry;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_lt = (1ull << lane) - 1;
  const uint32_t wave = (blockIdx.x * (kFastThreads / 64)) + (threadIdx.x >> 6);
  const uint64_t nlanes = (uint64_t)gridDim.x * kFastThreads;
  const uint64_t units = (P.nbytes + kUnit - 1) / kUnit;
  FastEvent* ev_seg = P.events + (uint64_t)wave * P.ev_cap_per_wave;
  uint32_t ev_count = 0;  // wave-uniform
  uint64_t u = (uint64_t)blockIdx.x * kFastThreads + threadIdx.x;
  FastChain<V> C;
  uint4 buf[R][V];
  auto load = [&](uint4(&b)[V], uint64_t pos) {
    const uint8_t* src = fast_src(P, pos);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (kMode & 4) b[k] = *(const uint4*)(P.data + ((pos + 16 * k) & 0xFFFF0ull));
      else b[k] = *(const uint4*)(src + pos + 16 * k);
    }
  };
  if (u < units) {
#pragma unroll
    for (int r = 0; r < D; ++r) load(buf[r], u * kUnit + (uint64_t)r * kStep);
  }
  // uniform per lane, not per wave: finished lanes walk stale bytes silently
  while (__ballot(u < units)) {
    const bool live = u < units;
    const uint64_t un = u + nlanes;
    const uint64_t base = u * kUnit;
    {
      // warm-up: the 7 bytes before the span (automaton depth <= kAcMaxLit)
      const uint2 h = live && base >= 8 ? *(const uint2*)(fast_src(P, base - 8) + base - 8) : make_uint2(0, 0);
      uint32_t e = 0;
#pragma unroll
      for (int j = 1; j < 8; ++j) e = fstep(T, e, j < 4 ? fold6(h.x) : fold6(h.y), j & 3);
      C.e = e;
      C.prev = h;
      C.nl = 0;
      C.hi = 0;
    }
    for (int s0 = 0; s0 < kSteps; s0 += R) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int st = s0 + r;
        const int ps = st + D;  // the step whose loads go out now
        if (live && (ps < kSteps || un < units))
          load(buf[(r + D) % R], ps < kSteps ? base + (uint64_t)ps * kStep : un * kUnit + (uint64_t)(ps - kSteps) * kStep);
        const uint64_t pos = base + (uint64_t)st * kStep;
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const uint4 v = buf[r][k];
          fast_group<V, kMode>(P, T, out_e, C, v.x, v.y, pos + 16 * k, live, lanes_lt, ev_seg, &ev_count);
          fast_group<V, kMode>(P, T, out_e, C, v.z, v.w, pos + 16 * k + 8, live, lanes_lt, ev_seg, &ev_count);
        }
        __builtin_amdgcn_sched_barrier(0);  // no hoisting across steps (register pressure)
      }
    }
    if (live && base < P.nbytes) {
      P.nl_blocks[base / kNlBlock] = C.nl;
      P.span_hi[base / kNlBlock] = (C.hi & 0x80808080u) ? 1 : 0;
    }
    u = un;
  }
  if (lane == 0) P.ev_counts[wave] = ev_count < P.ev_cap_per_wave ? ev_count : P.ev_cap_per_wave;
}

// Ring variant: every lane walks TWO chains in lock-step (ILP against the LDS
// latency): chain c covers half c of the lane's kNlBlock span.  Each chain
// streams through a 128-byte register ring — a 16-byte vector is reloaded
// with the chain's next 128 bytes right after it is consumed, always (a
// finished lane reloads its own bytes), so the compiler can count vmcnt
// exactly across the loop and the HBM latency hides behind a full ring of
// automaton work; every load completes whole 128-byte lines.
constexpr uint32_t kRingHalf = kNlBlock / 2;

__global__ __launch_bounds__(1024) void k_scan_ring(ScanParams P) {
  constexpr int kSteps = kRingHalf / 128;
  __shared__ __align__(16) uint8_t smem[kFastImgMax];
  const AcDev& ac = P.rs.ac;
  {
    const uint32_t words = ac.fast_bytes / 4;
    const uint32_t* src = (const uint32_t*)ac.fast_lds;
    for (uint32_t i = threadIdx.x; i < words; i += 1024) ((uint32_t*)smem)[i] = src[i];
  }
  __syncthreads();
  const uint8_t* T = smem;
  const uint32_t out_e = ac.fast_out_entry;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_lt = (1ull << lane) - 1;
  const uint32_t wave = (blockIdx.x * 16) + (threadIdx.x >> 6);
  const uint64_t nlanes = (uint64_t)gridDim.x * 1024;
  const uint64_t units = (P.nbytes + kNlBlock - 1) / kNlBlock;
  FastEvent* ev_seg = P.events + (uint64_t)wave * P.ev_cap_per_wave;
  uint32_t ev_count = 0;  // wave-uniform
  uint64_t u = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  FastChain<8> A, B;
  // ring fill: the lane's first span (a lane with no span reloads span 0)
  {
    const uint64_t s0 = (u < units ? u : 0) * kNlBlock;
    A.pos = s0;
    B.pos = s0 + kRingHalf;
    const uint8_t* sa = fast_src(P, A.pos);
    const uint8_t* sb = fast_src(P, B.pos);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      A.cur[k] = *(const uint4*)(sa + A.pos + 16 * k);
      B.cur[k] = *(const uint4*)(sb + B.pos + 16 * k);
    }
  }
  while (__ballot(u < units)) {
    const bool live = u < units;
    const uint64_t un = u + nlanes;
    const uint64_t s0 = A.pos;  // == u * kNlBlock for a live lane
    {
      // warm-up: the 7 bytes before each half (automaton depth <= kAcMaxLit)
      const uint2 ha = s0 >= 8 ? *(const uint2*)(fast_src(P, s0 - 8) + s0 - 8) : make_uint2(0, 0);
      const uint2 hb = *(const uint2*)(fast_src(P, B.pos - 8) + B.pos - 8);
      uint32_t ea = 0, eb = 0;
#pragma unroll
      for (int j = 1; j < 8; ++j) {
        ea = fstep(T, ea, j < 4 ? fold6(ha.x) : fold6(ha.y), j & 3);
        eb = fstep(T, eb, j < 4 ? fold6(hb.x) : fold6(hb.y), j & 3);
      }
      A.e = ea;
      B.e = eb;
      A.prev = ha;
      B.prev = hb;
      A.nl = B.nl = 0;
      A.hi = B.hi = 0;
    }
    // the unit after this one (or this one again: reloads stay unconditional)
    const uint64_t nbase = (un < units ? un : (live ? u : 0)) * kNlBlock;
    for (int step = 0; step < kSteps; ++step) {
      const bool last = step + 1 == kSteps;
      const uint64_t na = last ? nbase : A.pos + 128;
      const uint64_t nb = last ? nbase + kRingHalf : B.pos + 128;
      const uint8_t* sa = fast_src(P, na);
      const uint8_t* sb = fast_src(P, nb);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4 v = A.cur[k], w = B.cur[k];
        A.cur[k] = *(const uint4*)(sa + na + 16 * k);
        B.cur[k] = *(const uint4*)(sb + nb + 16 * k);
        fast_group2(P, T, out_e, A, B, v.x, v.y, w.x, w.y, A.pos + 16 * k, B.pos + 16 * k, live, lanes_lt, ev_seg,
                    &ev_count);
        fast_group2(P, T, out_e, A, B, v.z, v.w, w.z, w.w, A.pos + 16 * k + 8, B.pos + 16 * k + 8, live, lanes_lt,
                    ev_seg, &ev_count);
      }
      A.pos = na;
      B.pos = nb;
    }
    if (live) {
      const uint64_t sp = s0 / kNlBlock;
      P.nl_blocks[sp] = A.nl + B.nl;
      P.span_hi[sp] = ((A.hi | B.hi) & 0x80808080u) ? 1 : 0;
    }
    u = un;
  }
  if (lane == 0) P.ev_counts[wave] = ev_count < P.ev_cap_per_wave ? ev_count : P.ev_cap_per_wave;
}

#endif  // TSG_EXPERIMENTS

// Resolve k_scan_fast's events.  Each event is replayed on an LDS copy of the
// scan image with the output tables (out_off/out_pat/pats/pat_bytes) behind
// it; the event carries the group's bytes and the 8 before them, so a
// pattern is confirmed on the real bytes (the scan folds/aliases bytes),
// case requirement included, without touching the batch.  Per output:
// keyword gate bit (only keywords some non-implied gate needs; fire-and-forget
// atomic, file looked up once per event) and anchor hit (LDS-staged, one
// global reservation per block step).
// The events of all wave segments (and the overflow bucket after them) form
// one index space through ev_pre (the exclusive prefix of the segments'
// counts, ev_pre[n_waves] = their total); report wave r takes the r-th equal
// share of it, 64 events (one per lane) per round.  (Whole segments per wave
// left the kernel as long as its densest segment: waves lived 22 % of the
// kernel's 0.66 ms on average on configs[2], profiles/r04w_c2.)  Each wave
// stages its anchor hits in its own LDS slots and flushes them to its own
// hit region; with n_waves == 0 only the overflow bucket is left (the fused
// scan resolved the segments) -- and nothing, not even the image load,
// without one.
__global__ __launch_bounds__(kReportThreads) void k_report(ScanParams P, uint32_t n_waves, const uint64_t* ev_pre) {
  __shared__ __align__(16) uint8_t L[kReportLds];
  __shared__ uint64_t hbuf[kReportHitCap];
  __shared__ uint32_t hcnt[kReportThreads / 64];
  const uint64_t e_reg = n_waves ? ev_pre[n_waves] : 0;
  const uint64_t n_ovf = P.ctrl->ev_overflow < P.ev_overflow_cap ? P.ctrl->ev_overflow : P.ev_overflow_cap;
  const uint64_t E = e_reg + n_ovf;
  if (E == 0) return;
  const AcDev& ac = P.rs.ac;
  const bool in_lds = ac.rep_bytes <= kReportLds;
  if (in_lds) {
    const uint32_t words = ac.rep_bytes / 4;
    const uint32_t* src = (const uint32_t*)ac.fast_lds;
    for (uint32_t i = threadIdx.x; i < words; i += kReportThreads) ((uint32_t*)L)[i] = src[i];
  }
  const RepView R = rep_view(ac, in_lds ? L : ac.fast_lds);  // (LDS, or global when too big)
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* wbuf = hbuf + wv * kReportWaveHits;
  if (lane == 0) hcnt[wv] = 0;
  __syncthreads();
  uint32_t my_out = 0;
  uint64_t last_kw = ~0ull;
  const uint32_t rw = blockIdx.x * (kReportThreads / 64) + wv;
  const uint32_t n_rw = gridDim.x * (kReportThreads / 64);
  uint64_t* hseg = P.hit_seg ? P.hit_seg + (uint64_t)rw * P.hit_seg_cap : nullptr;
  uint32_t hcur = 0;
  uint64_t lo = E * rw / n_rw, hi = E * (rw + 1) / n_rw;
  if ((P.report_mode & 8) && n_waves <= n_rw) {  // (A/B, exp: whole segment rw per wave; the last wave also
    lo = rw < n_waves ? ev_pre[rw] : E;           //  takes the overflow bucket)
    hi = rw + 1 == n_rw ? E : rw < n_waves ? ev_pre[rw + 1] : E;
  }
  // the segment of event lo (s == n_waves: the overflow bucket)
  uint32_t s = n_waves;
  if (lo < e_reg) {
    uint32_t a = 0, b = n_waves;  // largest a with ev_pre[a] <= lo
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (ev_pre[m] <= lo) a = m;
      else b = m;
    }
    s = a;
  }
  // Each lane takes events lo + lane, lo + lane + 64, ...; its segment index
  // only moves forward (empty segments skipped; past e_reg: the bucket).  The
  // next round's event is loaded before this round's is resolved, so its HBM
  // latency runs under the replay instead of in front of it.
  uint32_t sl = s;
  const auto ev_at = [&](uint64_t g) -> const FastEvent* {
    while (sl < n_waves && ev_pre[sl + 1] <= g) ++sl;
    return sl < n_waves ? P.events + (uint64_t)sl * P.ev_cap_per_wave + (g - ev_pre[sl]) : P.ev_overflow + (g - e_reg);
  };
  FastEvent nxt{}, nxt2{};  // (two rounds ahead)
  if (lo + lane < hi) nxt = *ev_at(lo + lane);
  if (lo + lane + 64 < hi) nxt2 = *ev_at(lo + lane + 64);
  for (uint64_t g0 = lo; g0 < hi; g0 += 64) {
    const uint64_t g = g0 + lane;
    const FastEvent cur = nxt;
    nxt = nxt2;
    if (g + 128 < hi) nxt2 = *ev_at(g + 128);
    if (g < hi) report_event(P, ac, R, cur, wbuf, &hcnt[wv], my_out, last_kw);
    report_flush(P, wbuf, &hcnt[wv], lane, g0 + 64 >= hi, hseg, &hcur);
  }
  if (hseg && lane == 0) P.hit_seg_n[rw] = hcur;
  // per-wave totals: one atomic each
  for (uint32_t d = 32; d; d >>= 1) my_out += __shfl_xor(my_out, d);
  if (lane == 0) {
    if (my_out) atomicAdd(&P.ctrl->outputs, (unsigned long long)my_out);
    if (rw == 0 && e_reg) atomicAdd(&P.ctrl->events, (unsigned long long)e_reg);
  }
}

// The report waves' hit regions -> P.hits: one reservation on ctrl->hits for
// all of them (k_hits_reserve, after an exclusive scan of the counts into
// hit_pre), then one block per region copies it to its place.
__global__ void k_hits_reserve(ScanParams P, uint32_t n_rw, const uint64_t* hit_pre, unsigned long long* base) {
  const uint64_t total = hit_pre[n_rw - 1] + P.hit_seg_n[n_rw - 1];
  *base = atomicAdd(&P.ctrl->hits, (unsigned long long)total);
}

__global__ __launch_bounds__(256) void k_hits_pack(ScanParams P, const uint64_t* hit_pre,
                                                   const unsigned long long* base) {
  const uint32_t r = blockIdx.x;
  const uint32_t n = P.hit_seg_n[r];
  const uint64_t at = *base + hit_pre[r];
  const uint64_t* src = P.hit_seg + (uint64_t)r * P.hit_seg_cap;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (at + i < P.hit_cap) P.hits[at + i] = src[i];
}

// Fold-special sequences (C4B0 U+0130, C5BF U+017F, E284AA U+212A) in the
// spans k_scan_fast saw a byte >= 0x80 in: one wave per span, 64 bytes per
// lane, flag the file and record each occurrence for k_fold_windows.
__global__ __launch_bounds__(256) void k_fold_special(ScanParams P, uint64_t n_spans) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  constexpr uint32_t kPer = kNlBlock / 64;  // 64 bytes per lane: four 16-byte loads
  static_assert(kPer == 64, "one lane = four dwordx4");
  for (uint64_t g = w0 * 64; g < n_spans; g += nw * 64) {  // 64 spans per wave step
    uint64_t m = __ballot(g + lane < n_spans && P.span_hi[g + lane]);
    while (m) {
      const uint64_t sp = g + (uint64_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      const uint64_t a = sp * kNlBlock + (uint64_t)lane * kPer;
      uint32_t w[16];
      uint32_t hi = 0;
      if (a < P.nbytes) {  // (the last span reads the zero-padded tail copy)
        const uint8_t* src = fast_src(P, a) + a;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint4 v = *(const uint4*)(src + 16 * k);
          w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
          hi |= v.x | v.y | v.z | v.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = 0;
      }
      // the two bytes before the lane's first: the previous lane's last dword
      // (lane 0: the batch, or none at its start)
      uint32_t before = __shfl_up(w[15], 1);
      if (lane == 0) before = a >= 4 ? *(const uint32_t*)(fast_src(P, a - 4) + a - 4) : 0;
      if (!((hi | (before & 0x80800000u)) & 0x80808080u)) continue;  // no byte >= 0x80 near this lane
      uint32_t b1 = before >> 24, b2 = (before >> 16) & 0xFFu;
#pragma unroll
      for (uint32_t k = 0; k < kPer; ++k) {  // (unrolled: w stays in registers)
        const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint64_t q = a + k;
        const bool fi = c == 0xB0 && b1 == 0xC4, fs = c == 0xBF && b1 == 0xC5, fk = c == 0xAA && b1 == 0x84 && b2 == 0xE2;
        if ((fi || fs || fk) && q < P.nbytes) {
          mark_special(P, file_of_pos(P, q));
          note_fold(P, fk ? q - 2 : q - 1, fi ? FOLD_I : fs ? FOLD_S : FOLD_K);
        }
        b2 = b1;
        b1 = c;
      }
    }
  }
}

// Keywords whose lowercase holds a non-ASCII rune (MatchKeywords over
// bytes.ToLower(content), scanner.go:169-181): such an occurrence holds a
// content byte >= 0x80 (ToLower keeps ASCII ASCII; invalid bytes become
// U+FFFD), so only the spans k_scan_fast / k_scan_big flagged (span_hi), or
// every span when no flag exists, are searched, from uni_back bytes before
// the span on.  One wave per span, a 64th of the starts per lane: at each
// rune start the content is lowered rune by rune (unicode.ToLower,
// kLowerMap) and compared with the keyword's bytes.
struct UniKw {
  const uint8_t* bytes;
  const uint32_t* meta;  // 3 per keyword: offset, length, keyword id
  uint32_t n;
  uint32_t back;
  const uint32_t* lower;  // {rune, lowercase} pairs, sorted
  uint32_t n_lower;
};

__device__ inline uint32_t go_lower_rune(const UniKw& U, uint32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  uint32_t lo = 0, hi = U.n_lower;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (U.lower[2 * m] < r) lo = m + 1;
    else hi = m;
  }
  return lo < U.n_lower && U.lower[2 * lo] == r ? U.lower[2 * lo + 1] : r;
}

__device__ inline uint32_t utf8_encode(uint32_t r, uint8_t* e) {
  if (r < 0x80) { e[0] = (uint8_t)r; return 1; }
  if (r < 0x800) { e[0] = (uint8_t)(0xC0 | (r >> 6)); e[1] = (uint8_t)(0x80 | (r & 0x3F)); return 2; }
  if (r < 0x10000) {
    e[0] = (uint8_t)(0xE0 | (r >> 12)); e[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); e[2] = (uint8_t)(0x80 | (r & 0x3F));
    return 3;
  }
  e[0] = (uint8_t)(0xF0 | (r >> 18)); e[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
  e[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); e[3] = (uint8_t)(0x80 | (r & 0x3F));
  return 4;
}

__global__ __launch_bounds__(256) void k_uni_keywords(ScanParams P, UniKw U, uint64_t n_spans) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t g = w0 * 64; g < n_spans; g += nw * 64) {
    uint64_t m = __ballot(g + lane < n_spans && (!P.span_hi || P.span_hi[g + lane]));
    while (m) {
      const uint64_t sp = g + (uint64_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      const uint64_t a0 = sp * kNlBlock >= U.back ? sp * kNlBlock - U.back : 0;
      const uint64_t a1 = (sp + 1) * kNlBlock < P.nbytes ? (sp + 1) * kNlBlock : P.nbytes;
      const uint64_t per = (a1 - a0 + 63) / 64;
      const uint64_t qa = a0 + lane * per, qb = qa + per < a1 ? qa + per : a1;
      for (uint64_t q = qa; q < qb; ++q) {
        const uint64_t b0 = q >= 3 ? q - 3 : 0;
        const uint64_t avail = P.nbytes - b0;
        const uint32_t nb = (uint32_t)(avail < (1u << 30) ? avail : (1u << 30));
        if (!gre::is_rune_start(P.data + b0, nb, (uint32_t)(q - b0))) continue;
        for (uint32_t u = 0; u < U.n; ++u) {
          const uint8_t* kw = U.bytes + U.meta[3 * u];
          const uint32_t len = U.meta[3 * u + 1];
          uint64_t j = q;
          uint32_t k = 0;
          bool ok = true;
          while (ok && k < len) {
            const uint64_t rem = P.nbytes - j;
            uint32_t w = 0;
            const int r = gre::decode_rune(P.data + j, (uint32_t)(rem < 4 ? rem : 4), 0, &w);
            if (r < 0) {
              ok = false;
              break;
            }
            uint8_t e[4];
            const uint32_t el = utf8_encode(go_lower_rune(U, (uint32_t)r), e);
            if (k + el > len) {
              ok = false;
              break;
            }
            for (uint32_t t = 0; t < el; ++t) ok = ok && e[t] == kw[k + t];
            k += el;
            j += w;
          }
          if (ok) {
            const uint32_t fi = file_of_pos(P, q);
            const uint32_t id = U.meta[3 * u + 2];
            atomicOr(&P.file_kw[(size_t)fi * P.rs.kw_words + (id >> 5)], 1u << (id & 31));
          }
        }
      }
    }
  }
}

// Fold windows: around each fold-special rune occurrence q (k_fold_special,
// report_t), every work item (a pattern) is tried at every start h whose
// occurrence would contain q, so no file is ever rescanned whole:
//  * gate items (keywords holding 'i' or 'k'): MatchKeywords lowers the whole
//    file (bytes.ToLower, scanner.go:175) and İ -> 'i', K -> 'k' are the only
//    non-ASCII runes that lower to ASCII; a keyword spelled with one sets the
//    file's keyword bit (ASCII spellings were set by the scan already)
//  * hit items (anchor literals with a case-free 'k' or 's'): the literal
//    spelled with K / ſ ((?i) simple folding) is an anchor hit the ASCII scan
//    cannot see; it is appended with kFoldHit so that k_expand applies the
//    rule's keyword gate itself (ToLower(ſ) is ſ: such a match does not
//    imply the gate).  Every other match of the file still holds an ASCII
//    literal hit; gre's anchor offsets and prefix alphabets already count
//    K / ſ bytes, so those windows stay exact.
// An occurrence is taken only at its FIRST fold rune (each once).
constexpr uint64_t kFoldHit = 1ull << 63;
constexpr uint32_t kFoldItemGate = 1u << 31, kFoldItemHit = 1u << 30;

struct FoldItems {
  const uint32_t* items;  // pattern id | kFoldItemGate | kFoldItemHit
  uint32_t n;
  uint32_t with_hits;     // 0 for the prefilter-only pass (no anchor hits)
};

// Does pattern (lowered L, case requirement R or null, m bytes) occur at h?
// gate: the bytes.ToLower view (İ -> i, K -> k); else the (?i) view (K, ſ on
// case-free k / s).  *first = its first fold rune (~0 when spelled in ASCII),
// *end = the byte after it.
__device__ inline bool fold_match(const uint8_t* d, uint64_t nbytes, uint64_t h, const uint8_t* L, const uint8_t* R,
                                  uint32_t m, bool gate, uint64_t* first, uint64_t* end) {
  uint64_t t = h;
  *first = ~0ull;
  for (uint32_t i = 0; i < m; ++i) {
    if (t >= nbytes) return false;
    const uint32_t c = d[t];
    const uint8_t l = L[i];
    if (c >= 0x80) {
      uint32_t w = 0;
      if (c == 0xE2 && t + 2 < nbytes && d[t + 1] == 0x84 && d[t + 2] == 0xAA && l == 'k' && (gate || !R || !R[i])) w = 3;
      else if (!gate && c == 0xC5 && t + 1 < nbytes && d[t + 1] == 0xBF && l == 's' && (!R || !R[i])) w = 2;
      else if (gate && c == 0xC4 && t + 1 < nbytes && d[t + 1] == 0xB0 && l == 'i') w = 2;
      if (!w) return false;
      if (*first == ~0ull) *first = t;
      t += w;
      continue;
    }
    if (lower_ascii((uint8_t)c) != l) return false;
    if (!gate && R && R[i] && c != R[i]) return false;
    ++t;
  }
  *end = t;
  return true;
}

// Width of the fold-special rune at t (İ, ſ: 2, K: 3), 0 if none.
__device__ inline uint32_t fold_rune_at(const uint8_t* d, uint64_t nbytes, uint64_t t) {
  const uint32_t c = d[t];
  if (c == 0xE2) return t + 2 < nbytes && d[t + 1] == 0x84 && d[t + 2] == 0xAA ? 3 : 0;
  if (c == 0xC4 || c == 0xC5) return t + 1 < nbytes && d[t + 1] == (c == 0xC4 ? 0xB0 : 0xBF) ? 2 : 0;
  return 0;
}

__device__ __noinline__ void fold_window(const ScanParams& P, const FoldItems& F, uint64_t tid) {
  const AcDev& ac = P.rs.ac;
  const uint64_t rec = P.fold_pos[tid / F.n];
  const uint32_t it = F.items[tid % F.n];
  const uint64_t q = rec >> 2;
  const uint32_t kind = (uint32_t)(rec & 3);
  const uint32_t pid = it & 0xFFFFu;
  const PatDev pd = ac.pats[pid];
  const bool want_gate = (it & kFoldItemGate) && kind != FOLD_S;
  // a literal spelled with K / ſ, or an ASCII literal whose scan-automaton
  // extension (classes the rule requires next, follow_ext) meets the rune:
  // the extended pattern cannot fire there, so the hit is made here
  const bool want_hit = (it & kFoldItemHit) && F.with_hits && (kind != FOLD_I || pd.ext);
  if (!want_gate && !want_hit) return;
  const uint8_t* L = ac.pat_bytes + pd.bytes_off;
  const uint8_t* R = pd.confirm ? ac.pat_bytes + pd.req_off : nullptr;
  const uint32_t m = pd.len;
  if (!m) return;
  const uint64_t span = max(3ull * (m - 1), (uint64_t)m + 3ull * pd.ext);
  uint32_t fi = 0xFFFFFFFFu;
  for (uint64_t h = q > span ? q - span : 0; h <= q; ++h) {
    uint64_t first, end;
    if (want_gate && fold_match(P.data, P.nbytes, h, L, R, m, true, &first, &end) && first == q) {
      if (fi == 0xFFFFFFFFu) fi = file_of_pos(P, q);
      atomicOr(&P.file_kw[(size_t)fi * P.rs.kw_words + (pd.kw >> 5)], 1u << (pd.kw & 31));
    }
    if (!want_hit || !fold_match(P.data, P.nbytes, h, L, R, m, false, &first, &end)) continue;
    uint64_t rec_hit = ~0ull;
    if (first != ~0ull) {
      if (first == q && kind != FOLD_I) rec_hit = kFoldHit | (h << 16) | pid;  // k_expand gates it exactly
    } else if (pd.ext) {
      // ASCII literal: the first fold rune within its ext following characters
      uint64_t t = end;
      for (uint32_t j = 0; j < pd.ext && t < P.nbytes; ++j) {
        const uint32_t w = fold_rune_at(P.data, P.nbytes, t);
        if (w) {
          if (t == q) rec_hit = (h << 16) | pid;  // an ordinary anchor hit (gate implied as usual)
          break;
        }
        if (P.data[t] >= 0x80) break;
        ++t;
      }
    }
    if (rec_hit != ~0ull) {
      const unsigned long long idx = atomicAdd(&P.ctrl->hits, 1ull);
      if (idx < P.hit_cap) P.hits[idx] = rec_hit;
    }
  }
}

// One thread per (recorded fold-special rune, fold item); the rune count is
// read on the device (the scan's count, capped), so no host round trip sits
// between the scan and this pass.
__global__ __launch_bounds__(256) void k_fold_windows(ScanParams P, FoldItems F) {
  const uint64_t nf = P.ctrl->n_fold < P.fold_cap ? P.ctrl->n_fold : P.fold_cap;
  const uint64_t total = nf * F.n;
  for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total; tid += (uint64_t)gridDim.x * blockDim.x)
    fold_window(P, F, tid);
}

// ---------------------------------------------------------------- gating --
constexpr uint32_t kPathDfaRec = 8;  // u32 per program: off, ncls, cls_off, start0, start1, smatch, sym, valid

__device__ inline uint32_t zero_bytes(uint32_t x) {  // 0x80 in every byte of x that is 0 (and maybe above one)
  return (x - 0x01010101u) & ~x & 0x80808080u;
}

struct DfaRef {
  const uint16_t* T;
  const uint8_t* cls;
  uint32_t K, start0, start1, smatch, sym;
  const uint32_t* accel = nullptr;  // per-state accel record index (entries flagged kDfaAccel), global memory
  const uint4* accel_recs = nullptr;  // the 32-byte records: stay bitmap, stay class
};

// From q: the first position whose byte is not in the 128-bit stay set bm
// (every byte >= 0x80 is not), else n -- 16 bytes per load, one bitmap test
// per byte, no table lookups.  The batch is padded past every file end.
[[maybe_unused]] constexpr uint32_t kAccelRun = 8;  // (used by the TSG_EXPERIMENTS build)
template <class Pos>
__device__ inline Pos dfa_accel_skip(const uint8_t* text, Pos n, Pos q, const uint4 bm) {
  const uintptr_t base = reinterpret_cast<uintptr_t>(text);
  uintptr_t a = (base + q) & ~(uintptr_t)15;
  uint32_t i = (uint32_t)((base + q) & 15);  // first byte of the first block
  for (; a < base + n; a += 16, i = 0) {
    const u32x4 v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(a));
    for (; i < 16; ++i) {
      const uint32_t wd = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
      const uint32_t c = (wd >> (8 * (i & 3))) & 0xFFu;
      const uint32_t w = c < 64 ? (c < 32 ? bm.x : bm.y) : (c < 96 ? bm.z : bm.w);
      if (c >= 0x80 || !((w >> (c & 31)) & 1)) {
        const Pos p = (Pos)(a + i - base);
        return p < n ? p : n;
      }
    }
  }
  return n;
}

// kLds: d.T / d.cls are the block's LDS copy (k_verify stages the wave's rule).
template <bool kLds, class Pos>
__device__ inline int dfa_anchored_dev(const DfaRef d, const uint8_t* text, Pos n, Pos s, Pos* me,
                                       uint32_t* steps) {
  typedef __attribute__((address_space(3))) const uint16_t lu16;
  typedef __attribute__((address_space(3))) const uint8_t lu8;
  gu16* Tg = as_global<gu16>(d.T);
  gu8* cg = as_global<gu8>(d.cls);
  lu16* Tl = (lu16*)d.T;  // addrspacecast: only meaningful (and only read) when kLds
  lu8* cl = (lu8*)d.cls;
  uint32_t st = s == 0 ? d.start1 : d.start0;
  int64_t last = ((d.smatch >> (s == 0 ? 1 : 0)) & 1) ? (int64_t)s : -1;
  const uint32_t K = d.K;
  // the text in aligned 16-byte blocks, one dwordx4 load each (a byte load per
  // step cost a TLB lookup per lane per byte; the batch is padded past its
  // end, so a block holding a content byte never leaves the allocation)
  const uintptr_t base = reinterpret_cast<uintptr_t>(text);
  Pos q = s;
#ifdef TSG_EXPERIMENTS
  uint32_t same = 0;  // consecutive steps that kept the state (the skip engages only on a run)
#endif
  while (q < n && st) {
    const uintptr_t addr = (base + q) & ~(uintptr_t)15;
    const u32x4 v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(addr));
    uint32_t i = (uint32_t)((base + q) & 15);
    while (i < 16 && q < n && st) {
      const uint32_t wd = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);  // no dynamically indexed array
      const uint32_t c = (wd >> (8 * (i & 3))) & 0xFFu;
      uint32_t k, w = 1;
      if (c < 0x80) {
        k = kLds ? cl[c] : cg[c];
      } else {
        // a decoded rune: K, ſ, İ, U+FFFD or any other non-ASCII rune (dfa.cpp
        // symbols after the ASCII classes); the VM decides only when this
        // program tells other non-ASCII runes apart
        const int r = gre::decode_rune(text, n, q, &w);
        const uint32_t j = r == 0x212A ? 0u : r == 0x17F ? 1u : r == 0x130 ? 2u : r == 0xFFFD ? 3u : 4u;
        if (j == 4 && !(d.sym >> 31)) return 2;
        k = (d.sym & 0x7FFFFFFFu) + j;
      }
      const uint32_t e = kLds ? Tl[st * K + k] : Tg[st * K + k];
      ++*steps;
      if (q + w == n) {
        if (e & 0x8000u) last = n;
        st = 0;
        break;
      }
#ifdef TSG_EXPERIMENTS
      const uint32_t prev_st = st;
#endif
      st = e & kDfaStateMask;
      q += w;
      i += w;
      if (e & 0x4000u) last = q;
#ifdef TSG_EXPERIMENTS
      same = st == prev_st ? same + 1 : 0;
      // the record is a global read: taken only once the state has kept
      // itself for kAccelRun steps (a short run costs less walked)
      if (same >= kAccelRun && (e & kDfaAccel) && d.accel) {
        same = 0;
        // st keeps itself (same flags) on every byte of its stay set: skip
        // the run as the byte steps would take it
        const uint4* rec = d.accel_recs + 2 * d.accel[st];
        const Pos q2 = dfa_accel_skip<Pos>(text, n, q, rec[0]);
        if (q2 > q) {
          const uint32_t sc = rec[1].x;
          const uint32_t es = kLds ? Tl[st * K + sc] : Tg[st * K + sc];
          *steps += (uint32_t)(q2 - q);
          if (q2 == n) {  // the run reaches the end: bytes q .. n-2 as steps, n-1 as the last one
            if (n - 1 > q && (es & 0x4000u)) last = n - 1;
            if (es & 0x8000u) last = n;
            st = 0;
            break;
          }
          if (es & 0x4000u) last = q2;
          q = q2;
          break;  // reload the block at q
        }
      }
#endif
    }
  }
  if (last < 0) return 0;
  *me = (Pos)last;
  return 1;
}

struct GateParams {
  const uint64_t* off;
  const uint8_t* paths;
  const uint64_t* path_off;
  uint32_t n_files;
  RuleSetDev rs;
  const uint32_t* gpath;  // global allow path progs
  uint32_t n_gpath;
  const int32_t* rule_path;       // per rule: path prog or -1
  const uint32_t* rule_apath_off;  // per rule: offset into rule_apath (n_rules+1)
  const uint32_t* rule_apath;
  const uint32_t* path_rules;  // rules with a Path or allow paths, config order
  uint32_t n_path_rules;
  uint32_t any_rule_paths;
  uint32_t* file_flags;
  uint32_t* path_mask;  // n_files * rule_words: bit set => rule skipped by path
  uint32_t rule_words;
  uint8_t* scratch;
  uint64_t scratch_stride;
  // path literal automaton (PathAcHost): null => every path prog runs its VM
  const uint8_t* pac;
  uint32_t pac_states, pac_classes, pac_bytes;
  uint32_t o_pac_cls, o_pac_out_off, o_pac_out, o_pac_lits, o_pac_req, o_pac_bit;
  uint64_t pac_always;  // path progs without a literal filter
  uint32_t n_progs;
  const uint32_t* pdfa;  // per program: its MatchString DFA record (kPathDfaRec u32; valid flag last)
  uint32_t* defer;       // k_path_gate kPass 1: files a path program may match ([0] = count), for kPass 2
  uint32_t pac_lds;      // dynamic LDS bytes of the launch (0: the automaton stays in global memory)
  // kPass 1's test, without a per-program loop: the literal-mask bits of the
  // global allow paths / of the rules' paths and allow paths, and whether one
  // of them has no bit (it may always match)
  uint64_t gpath_bits, rpath_bits;
  uint32_t gpath_nobit, rpath_nobit;
};

__device__ inline gre::VmScratch make_scratch(uint8_t* base, const RuleSetDev& rs) {
  const uint32_t P = rs.max_ninst, ncap = rs.max_ncap, PC = rs.max_ninst_cap;
  gre::VmScratch sc;
  uint8_t* q = base;
  auto take = [&](size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
  };
  sc.sparse[0] = (uint16_t*)take(2ull * P);
  sc.sparse[1] = (uint16_t*)take(2ull * P);
  sc.dense[0] = (uint16_t*)take(2ull * P);
  sc.dense[1] = (uint16_t*)take(2ull * P);
  // position / capture-slot arrays sized for the 64-bit instantiation (files
  // of 4 GiB and more); the 32-bit one uses the first half of each
  sc.start[0] = take(8ull * P);
  sc.start[1] = take(8ull * P);
  sc.stack = (uint16_t*)take(2ull * (P + 1));
  sc.cur = take(8ull * ncap);
  sc.capstack = take(16ull * (P + 1));
  sc.caps[0] = take(8ull * PC * ncap);  // capture VM runs only group rules
  sc.caps[1] = take(8ull * PC * ncap);
  return sc;
}

__host__ inline uint64_t scratch_bytes(uint32_t P, uint32_t ncap, uint32_t PC) {
  auto r = [](uint64_t b) { return (b + 15) & ~15ull; };
  return r(2ull * P) * 4 + r(8ull * P) * 2 + r(2ull * (P + 1)) + r(8ull * ncap) + r(16ull * (P + 1)) +
         r(8ull * PC * ncap) * 2 + 256;
}

__device__ inline bool match_string(const gre::ProgView& pv, const uint8_t* s, uint32_t n,
                                    gre::VmScratch& sc) {
  uint32_t ms, me;
  return gre::vm_search(pv, s, n, 0, n, true, sc, &ms, &me);
}

// Literal prefilter for MatchString on match texts inside the batch: a
// pattern with an anchor factor can only match a string that contains one of
// its literals (case rules as in the scan).  Strings with bytes >= 0x80 skip
// the filter when a literal holds a case-free k or s (U+212A / U+017F match
// those); otherwise such bytes simply match nothing.  SWAR over aligned 16-byte blocks (one
// dwordx4 load each; the batch is padded past its end): per 4-byte word and
// literal, a zero-byte test on (lowered pair) ^ (literal's first two bytes),
// with `| 0x20` as the lowering (a superset for every byte: c == L implies
// c | 0x20 == L | 0x20); only the rare surviving positions re-read the literal
// from memory.  Returns kMayNo, kMayHit (a literal occurs) or kMayMaybe
// (a byte >= 0x80 was seen).
constexpr uint32_t kMayLits = 4;  // literals whose first bytes stay in registers
enum MayResult : uint32_t { kMayNo = 0, kMayHit = 1, kMayMaybe = 2 };


__device__ inline uint32_t may_match(const RuleSetDev& rs, uint32_t prog, const uint8_t* s, uint32_t n) {
  const uint32_t l0 = rs.prog_lit_off[prog], l1 = rs.prog_lit_off[prog + 1];
  if (l0 == l1) return kMayMaybe;
  const uint32_t nl = l1 - l0 < kMayLits ? l1 - l0 : kMayLits;
  uint32_t f1[kMayLits], f2[kMayLits];  // (lowered | 0x20) first / second byte, broadcast
  bool one[kMayLits];
  const bool fold = rs.prog_lits[(size_t)l0 * kLitRec + kLitFoldByte] != 0;
#pragma unroll
  for (uint32_t l = 0; l < kMayLits; ++l) {
    const uint8_t* rec = rs.prog_lits + (size_t)(l0 + (l < nl ? l : 0)) * kLitRec;
    one[l] = rec[0] < 2;
    f1[l] = (uint32_t)(rec[1] | 0x20) * 0x01010101u;
    f2[l] = (uint32_t)(rec[one[l] ? 1 : 2] | 0x20) * 0x01010101u;
  }
  auto full_check = [&](uint32_t l, int64_t i) {
    const uint8_t* rec = rs.prog_lits + (size_t)l * kLitRec;
    const uint32_t len = rec[0];
    if (i < 0 || (uint64_t)i + len > n) return false;
    for (uint32_t k = 0; k < len; ++k) {
      const uint8_t c = s[i + k];
      if (lower_ascii(c) != rec[1 + k] || (rec[17 + k] && c != rec[17 + k])) return false;
    }
    return true;
  };
  const uintptr_t base = reinterpret_cast<uintptr_t>(s);
  const uintptr_t a0 = base & ~(uintptr_t)15;
  uint32_t prev = 0;  // the previous word (lowered; bytes outside [0, n) are 0)
  for (uintptr_t a = a0; a < base + n; a += 16) {
    const u32x4 v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(a));
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t wi = 0; wi < 4; ++wi) {
      const int64_t q = (int64_t)(a + 4 * wi) - (int64_t)base;  // offset of the word's byte 0 in s
      uint32_t w = wv[wi];
      if (q < 0 || q + 4 > (int64_t)n) {  // keep bytes [max(0,-q), min(4, n-q))
        const int64_t lo = q < 0 ? -q : 0, hi = (int64_t)n - q;
        uint32_t keep = 0;
        for (int64_t k = lo; k < 4 && k < hi; ++k) keep |= 0xFFu << (8 * k);
        w &= keep;
      }
      if (fold && (w & 0x80808080u)) return kMayMaybe;  // (c | 0x20 >= 0xA0 never equals a literal byte)
      // bytes outside the string read 0x20 here: a candidate there fails full_check's bounds
      const uint32_t lwx = w | 0x20202020u;
      const uint32_t pw = (lwx << 8) | (prev >> 24);  // byte k: the byte before position q + k
#pragma unroll
      for (uint32_t l = 0; l < kMayLits; ++l) {
        if (l >= nl) break;
        uint32_t m = one[l] ? zero_bytes(lwx ^ f1[l]) : (zero_bytes(pw ^ f1[l]) & zero_bytes(lwx ^ f2[l]));
        while (m) {
          const uint32_t k = (uint32_t)__builtin_ctz(m) >> 3;
          m &= m - 1;
          if (full_check(l0 + l, q + k - (one[l] ? 0 : 1))) return kMayHit;
        }
      }
      prev = lwx;
    }
  }
  for (uint32_t l = l0 + nl; l < l1; ++l)  // literals past the register set (rare)
    for (uint32_t i = 0; i < n; ++i)
      if (full_check(l, i)) return kMayHit;
  return kMayNo;
}

__device__ inline bool match_string_pf(const RuleSetDev& rs, uint32_t prog, const uint8_t* s, uint32_t n,
                                       gre::VmScratch& sc) {
  const uint32_t mm = may_match(rs, prog, s, n);
  if (mm == kMayNo) return false;
  // a literal-exact program (e.g. the builtin "(?i)example") matches iff a literal occurs
  if (mm == kMayHit && rs.prog_lits[(size_t)rs.prog_lit_off[prog] * kLitRec + kLitExactByte]) return true;
  return match_string(rs.progs[prog], s, n, sc);
}

// Path gates (Global.AllowPath / Rule.MatchPath / Rule.AllowPath,
// scanner.go:375,391,397): one lane per file walks its path once through an
// Aho-Corasick automaton over every path regex's anchor literals (LDS), and
// only the regexes whose literal was seen (or that have none, or any path
// with a byte >= 0x80) run the Pike VM.
struct PacLit {
  uint32_t bit;      // path-prog bit
  uint32_t len;
  uint32_t req_off;  // case requirement bytes (0 = either case)
};

// kLds: the literal automaton staged in LDS; without (the launch after the
// scan) it is read from global memory (L2), so the gate's blocks fit beside
// k_report's, which take a CU's whole LDS.
// kPass 0: every file, the MatchString DFA / Pike VM where a literal occurs
// (one VM scratch slot per lane: the grid is capped at vm_threads).
// kPass 1: every file, at full occupancy (no VM scratch): a file for which
// some path program may match (a literal occurs, a byte >= 0x80, a program
// without literals) is appended to G.defer and left alone; every other file
// is decided here -- no program can match its path.  kPass 2: the deferred
// files, as kPass 0.  (kPass 0's grid -- two blocks per CU -- left the AC walk
// latency-bound: 0.23 ms for 2.25 M paths that no literal occurs in.)
// (kLds: the automaton in dynamic LDS of G.pac_lds bytes, 0 = global memory;
// the builtin rules' blob is ~20 KiB, which a static 16 KiB array missed:
// every AC step was an L2 round trip)
template <bool kLds, int kPass = 0>
__global__ __launch_bounds__(256) void k_path_gate(GateParams G) {
  extern __shared__ __align__(16) uint8_t pl[];
  const bool lds = kLds && G.pac && G.pac_bytes <= G.pac_lds;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < G.pac_bytes / 4; i += blockDim.x) ((uint32_t*)pl)[i] = ((const uint32_t*)G.pac)[i];
    __syncthreads();
  }
  const uint8_t* A = lds ? pl : G.pac;
  const uint16_t* delta = (const uint16_t*)A;
  const uint8_t* cls = A + G.o_pac_cls;
  const uint32_t* out_off = (const uint32_t*)(A + G.o_pac_out_off);
  const uint16_t* outs = (const uint16_t*)(A + G.o_pac_out);
  const PacLit* lits = (const PacLit*)(A + G.o_pac_lits);
  const uint8_t* req = A + G.o_pac_req;
  const uint8_t* pbit = A + G.o_pac_bit;
  const uint32_t nthreads = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(G.scratch + (uint64_t)t * G.scratch_stride, G.rs);
  // the next file's path offsets are loaded a file ahead, and a path is read
  // with aligned 16-byte loads (the next block before the current one is
  // walked): a byte load per step was a chain of dependent global reads
  // (0.21 ms for 2.25 M paths)
  const uint32_t n_items = kPass == 2 ? G.defer[0] : G.n_files;
  auto file_at = [&](uint32_t q) { return kPass == 2 ? G.defer[1 + q] : q; };
  uint64_t po0 = 0, po1 = 0;
  if (t < n_items) {
    const uint32_t f0 = file_at(t);
    po0 = G.path_off[f0];
    po1 = G.path_off[f0 + 1];
  }
  for (uint32_t q = t; q < n_items; q += nthreads) {
    const uint32_t f = file_at(q);
    const uint8_t* path = G.paths + po0;
    const uint32_t plen = (uint32_t)(po1 - po0);
    if (q + nthreads < n_items) {
      const uint32_t fn = file_at(q + nthreads);
      po0 = G.path_off[fn];
      po1 = G.path_off[fn + 1];
    }
    uint64_t mask = ~0ull;
    if (G.pac) {
      mask = G.pac_always;
      uint32_t st = 0;
      bool hi = false;
      const uintptr_t pbase = reinterpret_cast<uintptr_t>(path), pend = pbase + plen;
      uintptr_t blk = pbase & ~(uintptr_t)15;
      auto load16 = [](uintptr_t a) {
        return *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(a));
      };
      u32x4 v{0, 0, 0, 0}, nv{0, 0, 0, 0};
      if (plen) v = load16(blk);
      if (blk + 16 < pend) nv = load16(blk + 16);
      uint32_t k = (uint32_t)(pbase - blk);  // byte of v (0..15)
      for (uint32_t i = 0; i < plen; ++i, ++k) {
        if (k == 16) {  // the prefetched block; the one after it is issued now
          blk += 16;
          v = nv;
          if (blk + 16 < pend) nv = load16(blk + 16);
          k = 0;
        }
        const uint32_t wd = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
        const uint8_t b = (uint8_t)(wd >> (8 * (k & 3)));
        hi |= b >= 0x80;
        const uint32_t nx = delta[st * G.pac_classes + cls[b]];
        st = nx & 0x7FFFu;
        if (nx & 0x8000u) {
          for (uint32_t o = out_off[st]; o < out_off[st + 1]; ++o) {
            const PacLit L = lits[outs[o]];
            bool ok = true;
            for (uint32_t k = 0; k < L.len && ok; ++k) {
              const uint8_t r = req[L.req_off + k];
              ok = r == 0 || path[i + 1 - L.len + k] == r;
            }
            if (ok) mask |= 1ull << L.bit;
          }
        }
      }
      if (hi) mask = ~0ull;  // fold-special runes: no literal filter (as may_match)
    }
    auto may = [&](uint32_t prog) {
      if (!G.pac) return true;  // no literal prefilter (e.g. > 64 path programs)
      const uint32_t b = prog < G.n_progs ? pbit[prog] : 0xFFu;
      return b == 0xFFu || ((mask >> b) & 1);
    };
    if (kPass == 1) {  // a program that may match: the file goes to kPass 2 whole
      const bool any = !G.pac || G.gpath_nobit || (mask & G.gpath_bits) ||
                       (G.any_rule_paths && (G.rpath_nobit || (mask & G.rpath_bits)));
      if (any) {
        G.defer[1 + atomicAdd(&G.defer[0], 1u)] = f;
        continue;
      }
      if (!G.any_rule_paths) continue;  // no global allow path can match, and no rule has a path
    }
    // MatchString: the program's (?s:.)*?(?:re) DFA walked once over the path
    // (ruleset.cpp path_dfa), the Pike VM when there is none or a rune the DFA
    // cannot decide
    auto path_matches = [&](uint32_t prog) {
      const uint32_t* q = G.pdfa + (size_t)prog * kPathDfaRec;
      if (q[7]) {
        const DfaRef d{G.rs.dfa_delta + q[0], G.rs.dfa_bytes + q[2], q[1], q[3], q[4], q[5], q[6]};
        uint32_t me = 0, steps = 0;
        const int r = dfa_anchored_dev<false, uint32_t>(d, path, plen, 0u, &me, &steps);
        if (r != 2) return r == 1;
      }
      return match_string(G.rs.progs[prog], path, plen, sc);
    };
    bool allowed = false;
    for (uint32_t k = 0; k < G.n_gpath && !allowed; ++k) allowed = may(G.gpath[k]) && path_matches(G.gpath[k]);
    if (allowed) {
      atomicOr(&G.file_flags[f], kFileAllowed);  // the scan flags files concurrently (side stream)
      continue;
    }
    if (!G.any_rule_paths) continue;
    // rules share path programs (identical sources compile once): the last
    // evaluated program's answer is reused for the runs of rules naming it
    uint32_t memo_prog = 0xFFFFFFFFu;
    bool memo_res = false;
    auto path_match = [&](uint32_t prog) {
      if (prog != memo_prog) {
        memo_prog = prog;
        memo_res = may(prog) && path_matches(prog);
      }
      return memo_res;
    };
    // path_rules ascend: a mask word is gathered in a register and stored once
    // (a read-modify-write per skipped rule cost 1.7 ms for 1000 rules x 0.5 M files)
    uint32_t cur_w = 0xFFFFFFFFu, bits = 0;
    for (uint32_t q = 0; q < G.n_path_rules; ++q) {  // only rules a path can skip
      const uint32_t r = G.path_rules[q];
      bool skip = false;
      if (G.rule_path[r] >= 0) skip = !path_match((uint32_t)G.rule_path[r]);
      for (uint32_t k = G.rule_apath_off[r]; k < G.rule_apath_off[r + 1] && !skip; ++k)
        skip = path_match(G.rule_apath[k]);
      if (!skip) continue;
      if ((r >> 5) != cur_w) {
        if (bits) G.path_mask[(size_t)f * G.rule_words + cur_w] = bits;
        cur_w = r >> 5;
        bits = 0;
      }
      bits |= 1u << (r & 31);
    }
    if (bits) G.path_mask[(size_t)f * G.rule_words + cur_w] = bits;
  }
}

// Lazy newline counts reach this far past a file's last candidate (k_nl_spans phase 0).
constexpr uint64_t kNlCandReach = 16384;

struct ExpandParams {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* region_file;  // launch_scan's region -> file index
  uint64_t n_regions;
  uint32_t n_files;
  RuleSetDev rs;
  const uint32_t* file_kw;
  const uint32_t* file_flags;
  const uint32_t* path_mask;  // may be null
  uint32_t rule_words;
  const uint64_t* hits;
  uint64_t n_hits;
  const unsigned long long* n_hits_dev;  // or the count on the device (clamped to hit_cap): the speculative launch
  uint64_t hit_cap;
  uint64_t* keys;
  uint32_t* vals;
  uint64_t cand_cap;
  Ctrl* ctrl;
  const uint32_t* full_rules;  // rules in MODE_FULL
  uint32_t n_full_rules;
  unsigned long long* nl_last;  // lazy newline counts: per file, 1 + the last byte a candidate's count needs (or null)
};

__device__ inline bool rule_gate(const RuleSetDev& rs, const RuleDev& r, const uint32_t* kw) {
  if (r.kw_n == 0 || r.gate_always) return true;  // (gate_implied is applied by the callers that may use it)
  for (uint32_t k = 0; k < r.kw_n; ++k) {
    const uint32_t id = rs.kw_ids[r.kw_off + k];
    if ((kw[id >> 5] >> (id & 31)) & 1) return true;
  }
  return false;
}

// The text of a job read in aligned 16-byte blocks (one dwordx4 load per
// block; the batch is padded past its end), for the NFA walk's byte stream.
struct VecText {
  const uint8_t* base;
  uintptr_t blk;
  u32x4 v;
  __device__ explicit VecText(const uint8_t* b) : base(b), blk(~(uintptr_t)0), v{0, 0, 0, 0} {}
  template <class Pos>
  __device__ uint32_t operator[](Pos i) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(base) + i;
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != blk) {
      blk = b;
      v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(b));
    }
    const uint32_t o = (uint32_t)(a & 15);
    const uint32_t wd = o < 8 ? (o < 4 ? v.x : v.y) : (o < 12 ? v.z : v.w);  // no dynamically indexed array
    return (wd >> (8 * (o & 3))) & 0xFFu;
  }
};

// Candidate filter (follow.cpp): may a match of rule `rd` contain the anchor
// hit at text[h]?  false only when provably not.
__device__ inline bool follow_accepts_dev(const RuleSetDev& rs, const RuleDev& rd, const uint8_t* data, uint64_t h,
                                          uint64_t fend) {
  if (rd.follow_off == kNoFollow) return true;
  const uint16_t* T = rs.follow_delta + rd.follow_off;
  const uint8_t* cls = rs.follow_cls + rd.follow_cls_off;
  const uint32_t K = rd.follow_ncls;
  uint32_t st = 2;
  VecText D(data);  // (16 bytes per load: only the table walk is a dependent chain)
  for (uint32_t i = 0; i < kFollowDepth; ++i) {
    if (h + i >= fend) return false;
    const uint32_t c = D[h + i];
    if (c >= 0x80) return true;
    st = T[st * K + cls[c]];
    if (st < 2) return st == 1;
  }
  return true;
}

// The backward half of the candidate filter: every match [s, e) holding the
// anchor literal at h has h - s >= off_min and [s, h) inside the anchor
// alphabet (gre::Anchor), so the off_min bytes right before a hit must all be
// alphabet bytes (and lie in the file) -- else no match can contain it.  (The
// explosion-rule family `(?:x|y)*x(?:x|y){k}lit` anchors on lit with
// off_min = k + 1: almost every occurrence of lit fails this.)  The first
// kPrecedeMax bytes are checked.
constexpr uint32_t kPrecedeMax = 64;
__device__ inline bool precede_accepts_dev(const RuleDev& rd, const uint8_t* data, uint64_t h, uint64_t fstart) {
  const uint32_t a = rd.off_min;
  if (a == 0) return true;
  if (h - fstart < a) return false;
  const uint32_t k = a < kPrecedeMax ? a : kPrecedeMax;
  VecText D(data);
  for (uint32_t i = 1; i <= k; ++i) {
    const uint32_t c = D[h - i];
    if (!((rd.alpha[c >> 6] >> (c & 63)) & 1)) return false;
  }
  return true;
}

__device__ inline void emit_cand(const ExpandParams& E, uint32_t rule, uint64_t gpos, uint32_t val) {
  unsigned long long idx = atomicAdd(&E.ctrl->cands, 1ull);
  if (idx < E.cand_cap) {
    E.keys[idx] = ((uint64_t)rule << kPosBits) | gpos;
    E.vals[idx] = val;
  }
}

// One thread per anchor hit; the candidates of a block are reserved with ONE
// atomic on the candidate counter (a returning atomic on one word serialises
// chip-wide at ~90 per us: per wave it was ~14 K of them on configs[2]).
// Rules 32+ of a pattern (large custom rule sets) take a per-candidate atomic.
// Launched before the host knows the hit count (n_hits_dev: beside the scan's
// counter read), the grid strides over it.
__global__ __launch_bounds__(256) void k_expand(ExpandParams E) {
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long bbase;
  const uint64_t n_hits = E.n_hits_dev ? min((uint64_t)*E.n_hits_dev, E.hit_cap) : E.n_hits;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n_hits; i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t acc = 0;  // accepted rules k < 32 of the hit's pattern
    uint64_t gpos = 0;
    uint32_t fi = 0, rule_off = 0;
    if (i < n_hits) {
      const uint64_t h = E.hits[i];
      const bool fold = (h & kFoldHit) != 0;  // literal spelled with K / ſ (k_fold_windows)
      gpos = (h & ~kFoldHit) >> 16;
      const uint32_t pid = (uint32_t)(h & 0xFFFF);
      const uint64_t rg = gpos / kNlBlock;
      const uint32_t fhi = rg + 1 < E.n_regions ? min(E.region_file[rg + 1] + 1, E.n_files) : E.n_files;
      fi = find_file(E.off, E.region_file[rg], fhi, gpos);
      const uint32_t fl = E.file_flags[fi];
      if (!(fl & kFileAllowed)) {
        const PatDev pd = E.rs.ac.pats[pid];
        rule_off = pd.rule_off;
        const uint32_t* kw = E.file_kw + (size_t)fi * E.rs.kw_words;
        const uint64_t fend = E.off[fi + 1] - 1;
        for (uint32_t k = 0; k < pd.rule_n; ++k) {
          const uint32_t r = E.rs.ac.pat_rules[pd.rule_off + k];
          if (E.path_mask && ((E.path_mask[(size_t)fi * E.rule_words + (r >> 5)] >> (r & 31)) & 1)) continue;
          const RuleDev& rd = E.rs.rules[r];
          // an ASCII literal hit that holds a keyword proves the gate (gate_implied);
          // a K/ſ spelling does not (ToLower(ſ) == ſ)
          if ((fold || !rd.gate_implied) && !rule_gate(E.rs, rd, kw)) continue;
          if (!follow_accepts_dev(E.rs, rd, E.data, gpos, fend)) continue;
          if (!precede_accepts_dev(rd, E.data, gpos, E.off[fi])) continue;
          if (k < 32) {
            acc |= 1u << k;
          } else {
            emit_cand(E, r, gpos, fi);
            if (E.nl_last) atomicMax(&E.nl_last[fi], (unsigned long long)(gpos + kNlCandReach + 1));
          }
        }
      }
    }
    // block-wide exclusive prefix of the accepted counts, one reservation
    const uint32_t cnt = (uint32_t)__popc(acc);
    uint32_t incl = cnt;
  #pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) {
      before += w < wv ? wsum[w] : 0;
      total += wsum[w];
    }
    if (threadIdx.x == 0) bbase = total ? atomicAdd(&E.ctrl->cands, (unsigned long long)total) : 0ull;
    __syncthreads();
    uint64_t idx = bbase + before + incl - cnt;
    if (acc && E.nl_last) atomicMax(&E.nl_last[fi], (unsigned long long)(gpos + kNlCandReach + 1));
    while (acc) {
      const uint32_t k = (uint32_t)__ffs(acc) - 1;
      acc &= acc - 1;
      if (idx < E.cand_cap) {
        E.keys[idx] = ((uint64_t)E.rs.ac.pat_rules[rule_off + k] << kPosBits) | gpos;
        E.vals[idx] = fi;
      }
      ++idx;
    }
    __syncthreads();  // (wsum / bbase are rewritten by the next round)
  }
}

__global__ __launch_bounds__(256) void k_full_jobs(ExpandParams E) {
  const uint32_t fi = blockIdx.x * blockDim.x + threadIdx.x;
  if (fi >= E.n_files) return;
  const uint32_t fl = E.file_flags[fi];
  if (fl & kFileAllowed) return;
  const uint32_t* kw = E.file_kw + (size_t)fi * E.rs.kw_words;
  const uint64_t fstart = E.off[fi];
  for (uint32_t k = 0; k < E.n_full_rules; ++k) {
    const uint32_t r = E.full_rules[k];
    if (E.path_mask && ((E.path_mask[(size_t)fi * E.rule_words + (r >> 5)] >> (r & 31)) & 1)) continue;
    if (!rule_gate(E.rs, E.rs.rules[r], kw)) continue;
    emit_cand(E, r, fstart, fi | kFullFlag);
    if (E.nl_last) atomicMax(&E.nl_last[fi], (unsigned long long)(E.off[fi + 1] + 1));  // a full-file job: the file
  }
}

// Job boundaries over the sorted candidates: a new (file, rule) pair starts a
// job; inside a pair, a run of anchored candidates is split where the gap to
// the previous candidate exceeds max_len + (off_max - off_min) and a 4 KiB
// line is crossed — no match found before the split can reach a start
// window after it, so the pieces replay Go's sequential FindAll exactly and
// long files no longer serialise on one lane.  A rule whose program consumes
// no '\n' (unbounded ones too: JWTs, `{17,}` tokens) keeps every match inside
// one line, so a run is also split where a newline lies between the previous
// hit and the next hit's start window (found within kNlSplitScan bytes).
constexpr uint8_t kSplitHard = 1, kSplitSoft = 2;
// Every other gap between candidates whose start windows cannot overlap is a
// soft split (kSplitSoft): the jobs on both sides run in parallel and
// k_chain_fix checks that FindAll's sequence was not broken there.
constexpr uint32_t kNlSplitScan = 512;
constexpr uint32_t kSoftGapUnbounded = 64;  // soft-split gap for rules with an unbounded window
__global__ void k_mark_jobs(const uint64_t* keys, const uint32_t* vals, uint64_t n, const RuleDev* rules,
                            const uint8_t* data, uint8_t* flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t f = kSplitHard;
  if (i > 0) {
    const uint32_t r = (uint32_t)(keys[i] >> kPosBits);
    f = (r != (uint32_t)(keys[i - 1] >> kPosBits)) || ((vals[i] & ~kFullFlag) != (vals[i - 1] & ~kFullFlag));
    if (!f && !(vals[i] & kFullFlag) && !(vals[i - 1] & kFullFlag)) {
      const RuleDev& rd = rules[r];
      const uint64_t h0 = keys[i - 1] & kPosMask, h1 = keys[i] & kPosMask;
      if (rd.max_len != gre::kInf && rd.off_max != gre::kInf && (h0 >> 12) != (h1 >> 12)) {
        const uint64_t need = (uint64_t)rd.max_len + (rd.off_max - rd.off_min) + 8;
        f = h1 - h0 > need;
      }
      if (!f && rd.no_nl && rd.off_max != gre::kInf && (h0 >> 12) != (h1 >> 12) && h1 > h0 + rd.off_max) {
        const uint64_t lim = h1 - rd.off_max;  // the next hit's earliest match start
        const uint64_t end = lim < h0 + kNlSplitScan ? lim : h0 + kNlSplitScan;
        for (uint64_t q = h0; q < end && !f; ++q) f = data[q] == '\n';
      }
      if (!f) {
        const uint64_t gap = rd.off_max == gre::kInf ? kSoftGapUnbounded : (uint64_t)(rd.off_max - rd.off_min) + 8;
        if (h1 - h0 > gap) f = kSplitSoft;
      }
    }
  }
  flags[i] = f;
}

// ----------------------------------------------------------------- verify --
// A secret-group capture job (k_captures): a kept match [ms, me) of a group
// rule, with the verify job that found it (speculative-job bookkeeping).
struct CapJob {
  uint32_t file, rule, job, pad;
  uint64_t ms, me;
};

// Speculative job chains: a run of candidates of one (file, rule) is cut into
// jobs that are verified in parallel, each as if FindAll began at its first
// window; k_chain_fix then checks, job by job in order, that a job's first
// match starts at or after the previous match's end -- then the job's result
// equals the sequential one (FindAll would have tested the same starts) --
// and re-runs a chain sequentially from the first job where that fails.
constexpr uint32_t kJobRedo = 0x80000000u;  // DevLoc::job / CapJob::job of a re-run chain's output
constexpr uint32_t kJobFast = 0x40000000u;  // ... of k_verify_fast's output (void when the job was deferred)
constexpr uint32_t kJobMask = 0x3FFFFFFFu;
// Is an output of `job` void?  A re-run chain's never is; k_verify_fast's is
// when its job was later deferred (bit 1) or conflicts (bit 0); the others'
// when their job conflicts.
__device__ inline bool job_void(const uint8_t* job_bad, uint32_t job) {
  if (job & kJobRedo) return false;
  return (job_bad[job & kJobMask] & ((job & kJobFast) ? 3u : 1u)) != 0;
}
struct RedoRec {
  uint32_t job, last;  // jobs [job, last] of one chain, re-run in order
  uint64_t pos;        // FindAll's search position at `job` (file-relative)
};

struct VerifyParams {
  const uint8_t* data;
  const uint64_t* off;
  RuleSetDev rs;
  const uint64_t* keys;
  const uint32_t* vals;
  uint64_t n_cands;
  const uint32_t* job_start;
  const uint32_t* n_jobs_dev;  // job count, written by the job-segmentation select (no host read)
  DevLoc* locs;
  uint64_t loc_cap;
  unsigned long long* loc_shards;  // per-shard location counts (kLocShards; null: one counter, ctrl->locs)
  uint64_t loc_shard_cap;          // locations per shard region of `locs` (loc_cap / kLocShards)
  Ctrl* ctrl;
  uint8_t* scratch;
  uint64_t scratch_stride;
  uint64_t* prof;  // diagnostics (TSG_PROFILE_VERIFY): per job {duration | end (100 MHz), rule << 32 | full}
  uint32_t* tck;   // diagnostics: per job, 100 MHz ticks spent in DFA walks / in emit_match
  CapJob* caps;     // capture jobs for k_captures
  uint64_t cap_cap;
  CapJob* caps_big; // those too long for its arenas, for k_captures_big
  uint64_t cap_big_cap;
  CapJob* caps_run; // ASCII matches of byte-run group rules (gre::group_run), for k_group_runs
  uint64_t cap_run_cap;
  const uint8_t* span_hi;  // k_scan_fast's per-span ">= 0x80 occurs" flags (nullptr: not computed)
  // speculative jobs: per job the first match start / last match end
  // (file-relative; ~0 / 0 = no match), the split kind at each job start
  // (flags8 of its first candidate), the conflicting jobs, the re-runs
  uint64_t* job_fms;
  uint64_t* job_lme;
  const uint8_t* split;
  uint8_t* job_bad;  // bit 0: a conflicting speculative job; bit 1: deferred by k_verify_fast
  RedoRec* redo;
  uint64_t redo_cap;
  uint32_t* defer;   // jobs k_verify_fast handed to k_verify_slow (capacity >= jobs)
  CapJob* matches;   // k_verify_fast's matches, for k_allow
  uint64_t match_cap;
  uint32_t no_accel;  // 1 but in the exp build with TSG_ACCEL: DFA run acceleration (measured slower)
  uint32_t jpw;       // k_verify: jobs per wave (64 = every lane; fewer = lanes [0, jpw) of each wave)
};


// Candidate start windows of one (file, rule) job, in increasing order
// (DESIGN.md "anchor windows").
// (Pos: uint32_t, or uint64_t for the jobs of files of 4 GiB and more)
template <class Pos>
struct IvIter {
  const uint64_t* keys;
  uint64_t ci, c1;
  uint64_t fstart;
  const uint8_t* text;
  Pos n;
  uint32_t a, b;
  uint64_t al0, al1, al2, al3;  // the anchor prefix alphabet, in registers
  Pos h_prev, p_prev;
  bool have_prev;
  // current merged view
  bool have;
  Pos cs, ce;

  __device__ bool in_alpha(uint32_t c) const {
    const uint64_t w = c < 128 ? (c < 64 ? al0 : al1) : (c < 192 ? al2 : al3);  // (no dynamic index)
    return (w >> (c & 63)) & 1;
  }
  // Start of the run of alphabet bytes ending at h, never below lo: aligned
  // 16-byte loads backwards (a byte load per step was a dependent global read)
  __device__ Pos alpha_back(Pos lo, Pos h) const {
    Pos q = h;
    while (q > lo) {
      const uintptr_t last = reinterpret_cast<uintptr_t>(text) + (q - 1);
      const uintptr_t blk = last & ~(uintptr_t)15;
      const u32x4 v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(blk));
      for (int i = (int)(last - blk); i >= 0 && q > lo; --i, --q) {
        const uint32_t wd = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
        if (!in_alpha((wd >> (8 * (i & 3))) & 0xFFu)) return q;
      }
    }
    return q;
  }

  __device__ bool next_raw(Pos* ws, Pos* we) {
    while (ci < c1) {
      const Pos h = (Pos)((keys[ci++] & kPosMask) - fstart);
      if (h < a) continue;
      const Pos lo = (b == gre::kInf || h < b) ? (Pos)0 : h - b;
      // window start: the alpha run before h, never walked below lo = h - b
      // (a run reaching the previous hit joins that hit's window).  Walking to
      // the previous hit when it lies below lo re-read whole minified lines.
      Pos p;
      if (have_prev && h_prev <= h && h_prev >= lo) {
        const Pos q = alpha_back(h_prev, h);
        p = (q == h_prev) ? (p_prev > lo ? p_prev : lo) : q;
      } else {
        p = alpha_back(lo, h);
      }
      if (p < lo) p = lo;
      have_prev = true;
      h_prev = h;
      p_prev = p;
      const Pos wend = h - a;
      while (p <= wend && !gre::is_rune_start(text, n, p)) ++p;
      if (p > wend) continue;
      *ws = p;
      *we = wend;
      return true;
    }
    return false;
  }
  __device__ void advance() { have = next_raw(&cs, &ce); }
  // Start-permission protocol used by vm_search_starts.
  __device__ bool skip_to(Pos pos, Pos* np) {
    while (have && ce < pos) advance();
    if (!have) return false;
    *np = pos < cs ? cs : pos;
    return true;
  }
  __device__ bool allowed(Pos pos) {
    while (have && ce < pos) advance();
    return have && cs <= pos && pos <= ce;
  }
};

// Exactly one permitted start: an anchored leftmost-first match at s.
template <class Pos>
struct OneStart {
  Pos s;
  __device__ bool skip_to(Pos pos, Pos* np) {
    if (pos > s) return false;
    *np = s;
    return true;
  }
  __device__ bool allowed(Pos pos) { return pos == s; }
};

template <class Pos>
struct LimitStarts {
  Pos limit;
  __device__ bool skip_to(Pos pos, Pos* np) {
    if (pos > limit) return false;
    *np = pos;
    return true;
  }
  __device__ bool allowed(Pos pos) { return pos <= limit; }
};

// vm_search with a start-position oracle (anchor windows or a plain limit);
// when no thread is alive the VM jumps to the next permitted start.
template <class Pos, class Starts>
__device__ bool vm_search_starts(const gre::ProgView& p, const uint8_t* text, Pos n, Pos pos0,
                                 Starts& S, gre::VmScratch& sc, Pos* ms, Pos* me) {
  gre::Queue<Pos> q[2] = {{sc.sparse[0], sc.dense[0], (Pos*)sc.start[0], nullptr, 0},
                          {sc.sparse[1], sc.dense[1], (Pos*)sc.start[1], nullptr, 0}};
  int cur = 0;
  bool matched = false;
  Pos pos = pos0;
  uint32_t w = 0, w1 = 0;
  int r = gre::decode_rune(text, n, pos, &w);
  int r1 = r >= 0 ? gre::decode_rune(text, n, pos + w, &w1) : -1;
  uint8_t ctx = gre::empty_ctx(gre::prev_ctx_rune(text, pos), r);
  for (;;) {
    gre::Queue<Pos>& runq = q[cur];
    gre::Queue<Pos>& nextq = q[cur ^ 1];
    if (runq.n == 0) {
      if (matched) break;
      Pos np;
      if (!S.skip_to(pos, &np)) break;
      if (np != pos) {
        pos = np;
        r = gre::decode_rune(text, n, pos, &w);
        r1 = r >= 0 ? gre::decode_rune(text, n, pos + w, &w1) : -1;
        ctx = gre::empty_ctx(gre::prev_ctx_rune(text, pos), r);
      }
    }
    if (!matched && S.allowed(pos)) gre::vm_add(p, runq, sc.stack, p.start, pos, ctx);
    const uint8_t nctx = gre::empty_ctx(r, r1);
    nextq.n = 0;
    for (uint32_t j = 0; j < runq.n; ++j) {
      const gre::Inst in = p.inst[runq.dense[j]];
      if (in.op == gre::I_MATCH) {
        *ms = runq.start[j];
        *me = pos;
        matched = true;
        break;
      }
      if (gre::inst_consumes(in, p, r)) gre::vm_add(p, nextq, sc.stack, in.out, runq.start[j], nctx);
    }
    runq.n = 0;
    if (w == 0) break;
    pos += w;
    r = r1;
    w = w1;
    r1 = r >= 0 ? gre::decode_rune(text, n, pos + w, &w1) : -1;
    ctx = nctx;
    cur ^= 1;
  }
  return matched;
}

// Anchored leftmost-first DFA walk from s (dfa.cpp): 1 = match [s, *me),
// 0 = none, 2 = undecidable here (byte >= 0x80) -> the Pike VM decides.
// T / cls: the rule's table and class map, in global memory or staged in LDS.
// Plain scalars (no RuleDev reference: a by-reference struct lands in scratch
// and its fields get reloaded inside the walk).
// Bit-state backtracker (go1.22 regexp/backtrack.go semantics: depth-first in
// priority order, each (pc, pos) visited once, so the first MATCH reached is
// the leftmost-first match and its captures are Go's) for the secret-group
// spans of a match [ms, me) the DFA or VM already found.  Visited bits, job
// stack and the tracked capture slots live in the lane's LDS arena; only the
// SecretGroupName slots are tracked (captures never steer the search).
// Returns false when the match does not fit the arena (`words` LDS words; the
// caller then defers it to a larger arena, or runs the Pike capture VM) —
// never a different answer.
constexpr uint32_t kBsWords = 560;        // k_verify: LDS words per lane (140 KiB per block)
constexpr uint32_t kCapActive = 8;        // k_captures: searching lanes per 64-lane block (8 blocks per CU)
constexpr uint32_t kBigBsWords = 9216;    // and their arenas (36 KiB: P x W <= 294 K (pc, pos) bits)

// Slots: the tracked capture slots' type (int32_t, int64_t for files of 4 GiB
// and more); they take the arena's last kSlotWords words.
template <class Pos>
struct CapSlots {
  typedef typename gre::SlotOf<Pos>::type Slot;
  static constexpr uint32_t kWords = 8 * sizeof(Slot) / 4;
};

template <class Pos>
__device__ bool bitstate_captures(const gre::ProgView& p, const uint8_t* text, Pos n, Pos ms, Pos me,
                                  const uint32_t* gnum, uint32_t ng, uint32_t* area, uint32_t words,
                                  typename gre::SlotOf<Pos>::type* gcap) {
  typedef typename gre::SlotOf<Pos>::type Slot;
  constexpr uint32_t kSlotWords = CapSlots<Pos>::kWords;
  // visited rows for the join points only (Inst::vis); a path that consumes
  // past me can never end at me, so positions stay in [ms, me]
  const uint32_t P = p.nvis;
  const Pos end = me;
  if (end - ms + 1 >= 0xFFFF) return false;
  const uint32_t W = (uint32_t)(end - ms + 1);
  const uint32_t vis_words = (P * W + 31) / 32;
  // arena: visited bits | job stack | the 8 tracked capture slots (gcap, the last words)
  if (2 * ng > 8 || P >= 0x4000 || vis_words + kSlotWords + 32 > words) return false;
  uint32_t* vis = area;
  uint32_t* stk = area + vis_words;
  const uint32_t stk_cap = words - kSlotWords - vis_words;
  for (uint32_t i = 0; i < vis_words; ++i) vis[i] = 0;
  for (uint32_t k = 0; k < 2 * ng; ++k) gcap[k] = -1;
  auto local = [&](uint32_t slot) -> int {  // tracked index of capture slot, or -1
    for (uint32_t g = 0; g < ng; ++g)
      if (slot == 2 * gnum[g] || slot == 2 * gnum[g] + 1) return (int)(2 * g + (slot & 1));
    return -1;
  };
  uint32_t sp = 0;
  stk[sp++] = (p.start << 16);
  while (sp) {
    const uint32_t j = stk[--sp];
    const uint32_t kind = j >> 30, pc0 = (j >> 16) & 0x3FFFu, v = j & 0xFFFFu;
    if (kind == 2) {  // capture restore
      const int l = local(p.inst[pc0].arg);
      if (l >= 0) gcap[l] = v == 0xFFFFu ? (Slot)-1 : (Slot)(ms + v);
      continue;
    }
    Pos pos = ms + v;
    uint32_t pc = kind == 1 ? p.inst[pc0].arg : pc0;  // ALT: the second branch
    for (;;) {
      if (pc == 0 || pos > end) break;
      const gre::Inst in = p.inst[pc];
      if (in.vis != gre::kNoVis) {
        const uint32_t bit = in.vis * W + (uint32_t)(pos - ms);
        if (vis[bit >> 5] & (1u << (bit & 31))) break;
        vis[bit >> 5] |= 1u << (bit & 31);
      }
      if (in.op == gre::I_ALT) {
        if (sp >= stk_cap) return false;
        stk[sp++] = (1u << 30) | (pc << 16) | (uint32_t)(pos - ms);
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_CAP) {
        const int l = local(in.arg);
        if (l >= 0) {
          if (sp >= stk_cap) return false;
          const Slot old = gcap[l];
          stk[sp++] = (2u << 30) | (pc << 16) | (old < 0 ? 0xFFFFu : (uint32_t)(old - (Slot)ms));
          gcap[l] = (Slot)pos;
        }
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_EMPTY) {
        uint32_t w;
        const int r = gre::decode_rune(text, n, pos, &w);
        if ((in.empty & ~gre::empty_ctx(gre::prev_ctx_rune(text, pos), r)) != 0) break;
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_NOP) {
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_MATCH) return pos == me;
      uint32_t w;
      const int r = gre::decode_rune(text, n, pos, &w);
      if (!gre::inst_consumes(in, p, r)) break;
      pos += w;
      pc = in.out;
    }
  }
  return false;
}

// A kept location.  The locations are reserved from kLocShards counters
// (by block and wave), each owning a region of `locs` (loc_shard_cap
// slots), past which a shard spills into a shared overflow region (counter
// kLocShards); k_loc_compact packs everything densely afterwards.  One
// returning atomic on one word serialises chip-wide at ~90 per us, which was
// most of k_verify's time on configs[2] (29 K locations, one atomic each from
// divergent lanes).
constexpr uint32_t kLocShards = 64;
__device__ inline void loc_emit(const VerifyParams& V, const DevLoc& L) {
  if (V.loc_shards) {
    const uint32_t sh = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kLocShards - 1);
    const unsigned long long k = atomicAdd(&V.loc_shards[sh], 1ull);
    if (k < V.loc_shard_cap) {
      V.locs[(uint64_t)sh * V.loc_shard_cap + k] = L;
      return;
    }
    const unsigned long long o = atomicAdd(&V.loc_shards[kLocShards], 1ull);
    const uint64_t at = (uint64_t)kLocShards * V.loc_shard_cap + o;
    if (at < V.loc_cap) V.locs[at] = L;
    return;
  }
  const unsigned long long idx = atomicAdd(&V.ctrl->locs, 1ull);
  if (idx < V.loc_cap) V.locs[idx] = L;
}

// Block b < kLocShards copies shard b's region, block kLocShards the
// overflow region, to their dense place in `out`; block 0 sets ctrl->locs
// to the total (when the overflow region overflowed: capacity + emitted,
// above every capacity, so the host grows the lists and re-runs).
__global__ __launch_bounds__(256) void k_loc_compact(VerifyParams V, DevLoc* out) {
  __shared__ unsigned long long cnt[kLocShards + 1];
  if (threadIdx.x <= kLocShards) cnt[threadIdx.x] = V.loc_shards[threadIdx.x];
  __syncthreads();
  const uint64_t sc = V.loc_shard_cap, ocap = V.loc_cap - (uint64_t)kLocShards * sc;
  uint64_t start = 0, total = 0, emitted = cnt[kLocShards];
  for (uint32_t k = 0; k <= kLocShards; ++k) {
    const uint64_t c = k < kLocShards ? (cnt[k] < sc ? cnt[k] : sc) : (cnt[k] < ocap ? cnt[k] : ocap);
    if (k < blockIdx.x) start += c;
    total += c;
    if (k < kLocShards) emitted += cnt[k] < sc ? cnt[k] : sc;
  }
  const uint64_t b = blockIdx.x;
  const uint64_t n = b < kLocShards ? (cnt[b] < sc ? cnt[b] : sc) : (cnt[b] < ocap ? cnt[b] : ocap);
  const DevLoc* src = V.locs + b * sc;  // (b == kLocShards: the overflow region)
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) out[start + i] = src[i];
  if (b == 0 && threadIdx.x == 0) V.ctrl->locs = emitted > total ? V.loc_cap + emitted : total;
}

// Secret-group spans of one kept match (getMatchSubgroupsLocations,
// scanner.go:150-163) with the bit-state backtracker in the lane's LDS arena
// of `words` words; a match too long for it goes on to the next stage's list
// (`next`, k_captures -> k_captures_big), and only past the last arena does
// the capture VM run.
template <class Pos>
__device__ void emit_groups(const VerifyParams& V, const RuleDev& rd, uint32_t rule, uint32_t fi, uint32_t job,
                            const uint8_t* text, Pos n, Pos ms, Pos me, gre::VmScratch& sc,
                            uint32_t* bs_area, uint32_t words, CapJob* next, uint64_t next_cap,
                            unsigned long long* next_n) {
  typedef typename gre::SlotOf<Pos>::type Slot;
  const gre::ProgView& pv = V.rs.progs[rd.prog];
  const uint32_t* gnum = V.rs.group_slots + rd.group_off;
  Slot* gcap = (Slot*)(bs_area + words - CapSlots<Pos>::kWords);  // tracked slots (the arena's last words)
  const bool bs_ok = bitstate_captures<Pos>(pv, text, n, ms, me, gnum, rd.group_n, bs_area, words, gcap);
  if (!bs_ok && next) {
    const unsigned long long idx = atomicAdd(next_n, 1ull);
    if (idx < next_cap) next[idx] = CapJob{fi, rule, job, 0, ms, me};
    return;
  }
  if (bs_ok) {
    for (uint32_t g = 0; g < rd.group_n; ++g) {
      const Slot s = gcap[2 * g], e = gcap[2 * g + 1];
      if (s < 0 || e < 0) loc_emit(V, DevLoc{fi, rule, 0, 0, 0, 0, 1, job});
      else loc_emit(V, DevLoc{fi, rule, (uint64_t)s, (uint64_t)e, 0, 0, 0, job});
    }
    return;
  }
  Slot out[kMaxCap];  // ncap <= kMaxCap is enforced by the rule compiler
  bool ok = gre::vm_captures<Pos>(pv, text, n, ms, sc, out);
  if (!ok || (Pos)out[1] != me) atomicOr(&V.ctrl->err, 1u);
  for (uint32_t g = 0; g < rd.group_n; ++g) {
    const uint32_t slot = gnum[g];
    const Slot s = out[2 * slot], e = out[2 * slot + 1];
    if (s < 0 || e < 0) loc_emit(V, DevLoc{fi, rule, 0, 0, 0, 0, 1, job});
    else loc_emit(V, DevLoc{fi, rule, (uint64_t)s, (uint64_t)e, 0, 0, 0, job});
  }
}

// Start of the run of bytes in the ASCII set m that ends at e (never below lo):
// aligned 16-byte loads backwards, the bytes tested in registers.
template <class Pos>
__device__ inline Pos run_back(const uint8_t* text, Pos lo, Pos e, const uint32_t (&m)[4]) {
  Pos q = e;
  while (q > lo) {
    const uintptr_t last = reinterpret_cast<uintptr_t>(text) + (q - 1);
    const uintptr_t blk = last & ~(uintptr_t)15;
    const u32x4 v = *as_global<__attribute__((address_space(1))) const u32x4>(reinterpret_cast<const void*>(blk));
    for (int i = (int)(last - blk); i >= 0 && q > lo; --i, --q) {
      const uint32_t wd = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
      const uint32_t c = (wd >> (8 * (i & 3))) & 0xFFu;
      const uint32_t mw = c < 64 ? (c < 32 ? m[0] : m[1]) : (c < 96 ? m[2] : m[3]);  // (no dynamic index)
      if (c >= 0x80 || !((mw >> (c & 31)) & 1u)) return q;
    }
  }
  return q;
}

// A kept match: the whole-match location or, for rules with a secret group,
// its span (ASCII shortcuts) or a capture job for k_captures (whose
// bit-state arenas take LDS that would cap the search at one wave per CU).
template <class Pos>
__device__ inline void emit_kept(const VerifyParams& V, const RuleDev& rd, uint32_t rule, uint32_t fi, uint32_t job,
                                 const uint8_t* text, Pos ms, Pos me) {
  if (!rd.use_groups) {
    loc_emit(V, DevLoc{fi, rule, ms, me, 0, 0, 0, job});
    return;
  }
  if (rd.grp_fast || rd.grp_run) {  // the group's span follows from [ms, me) on ASCII text (gre::group_span / group_run)
    // ASCII: the scan's per-4 KiB-span flags, byte by byte only in a flagged span
    bool ascii = true;
    if (V.span_hi && me > ms) {  // (an empty match holds no byte: nothing to check)
      const uint64_t a = (uint64_t)(text - V.data) + ms, b = (uint64_t)(text - V.data) + me;
      for (uint64_t sp = a / kNlBlock; sp < (b + kNlBlock - 1) / kNlBlock && ascii; ++sp) ascii = V.span_hi[sp] == 0;
    }
    if (!ascii || (!V.span_hi && me > ms)) {
      ascii = true;
      for (Pos q = ms; q < me && ascii; ++q) ascii = as_global<gu8>(text)[q] < 0x80;
    }
    if (ascii && rd.grp_fast) {
      const int64_t gs = rd.grp_pre >= 0 ? (int64_t)ms + rd.grp_pre : (int64_t)me - rd.grp_suf - rd.grp_len;
      const int64_t ge = rd.grp_suf >= 0 ? (int64_t)me - rd.grp_suf : gs + rd.grp_len;
      if (gs >= (int64_t)ms && gs <= ge && ge <= (int64_t)me) {
        loc_emit(V, DevLoc{fi, rule, (uint64_t)gs, (uint64_t)ge, 0, 0, 0, job});
        return;
      }
      // (unreachable for a real match of the rule; the capture search decides)
    } else if (ascii) {  // byte runs back from the match end (gre::group_run): k_group_runs
      const unsigned long long idx = atomicAdd(&V.ctrl->n_caps_run, 1ull);
      if (idx < V.cap_run_cap) V.caps_run[idx] = CapJob{fi, rule, job, 0, (uint64_t)ms, (uint64_t)me};
      return;
    }
  }
  unsigned long long idx = atomicAdd(&V.ctrl->n_caps, 1ull);
  if (idx < V.cap_cap) V.caps[idx] = CapJob{fi, rule, job, 0, ms, me};
}

// A match k_verify found: allow rules (scanner.go:145-148), then emit_kept.
template <class Pos>
__device__ __noinline__ void emit_match(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                        const uint8_t* text, Pos n, Pos ms, Pos me, gre::VmScratch& sc,
                                        uint32_t* tck = nullptr) {
  const uint64_t t0 = tck ? __builtin_amdgcn_s_memrealtime() : 0;
  const RuleDev& rd = V.rs.rules[rule];
  if (sizeof(Pos) > 4 && me - ms > (Pos)0xFFFFFFFFu) {  // allow regexes run on 32-bit match strings
    atomicOr(&V.ctrl->err, 2u);
    return;
  }
  // AllowLocation (scanner.go:145-148): global then rule allow regexes on the whole match
  for (uint32_t k = 0; k < V.rs.n_global_allow; ++k) {
    const bool al = match_string_pf(V.rs, V.rs.global_allow[k], text + ms, (uint32_t)(me - ms), sc);
    if (tck) tck[2] += (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
    if (al) return;
  }
  const uint32_t allow_off = rd.allow_off, allow_n = rd.allow_n;
  for (uint32_t k = 0; k < allow_n; ++k)
    if (match_string_pf(V.rs, V.rs.allow_progs[allow_off + k], text + ms, (uint32_t)(me - ms), sc)) return;
  emit_kept<Pos>(V, rd, rule, fi, job, text, ms, me);
}

// Zeroes what a verify attempt counts into: the Ctrl counters (locs, n_caps /
// n_caps_big, n_redo / n_dropped / n_caps_run, n_defer / n_match), the
// location shard counters and the per-job flag bytes.
__global__ __launch_bounds__(256) void k_verify_reset(Ctrl* ctrl, unsigned long long* loc_cnt, uint8_t* job_bad,
                                                      uint64_t n_jobs) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) {
    ctrl->locs = 0;
    ctrl->n_caps = ctrl->n_caps_big = 0;
    ctrl->n_redo = ctrl->n_dropped = ctrl->n_caps_run = 0;
    ctrl->n_defer = ctrl->n_match = 0;
  }
  if (loc_cnt && t <= kLocShards) loc_cnt[t] = 0;
  const uint64_t n16 = n_jobs / 16;
  for (uint64_t i = t; i < n16; i += (uint64_t)gridDim.x * blockDim.x) ((uint4*)job_bad)[i] = make_uint4(0, 0, 0, 0);
  for (uint64_t i = n16 * 16 + t; i < n_jobs; i += (uint64_t)gridDim.x * blockDim.x) job_bad[i] = 0;
}

// emit_match for k_verify_fast: the match goes to the raw match list; the
// allow rules (which may need the Pike VM) run in k_allow, a kernel of its
// own.  false (the job is deferred) only for a match of 4 GiB or more.
template <class Pos>
__device__ inline bool emit_match_fast(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                       const uint8_t* text, Pos ms, Pos me) {
  (void)text;
  if (sizeof(Pos) > 4 && me - ms > (Pos)0xFFFFFFFFu) return false;  // (the slow kernel reports it)
  const unsigned long long idx = atomicAdd(&V.ctrl->n_match, 1ull);
  if (idx < V.match_cap) V.matches[idx] = CapJob{fi, rule, job | kJobFast, 0, (uint64_t)ms, (uint64_t)me};
  return true;
}

// AllowLocation (scanner.go:145-148) for k_verify_fast's matches, one lane
// per match (the Pike VM's registers stay out of the search kernel), then the
// location / group stage as emit_match.  A match of a job deferred after it
// was found is void (k_verify_slow re-finds it).
__global__ __launch_bounds__(64) void k_allow(VerifyParams V) {
  const unsigned long long cnt = V.ctrl->n_match;
  const uint64_t n = cnt < V.match_cap ? cnt : V.match_cap;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(V.scratch + (uint64_t)t * V.scratch_stride, V.rs);
  for (uint64_t i = t; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const CapJob M = V.matches[i];
    if (job_void(V.job_bad, M.job)) continue;
    const RuleDev& rd = V.rs.rules[M.rule];
    const uint8_t* text = V.data + V.off[M.file];
    const uint8_t* m = text + M.ms;
    const uint32_t len = (uint32_t)(M.me - M.ms);
    bool allowed = false;
    for (uint32_t k = 0; k < V.rs.n_global_allow && !allowed; ++k)
      allowed = match_string_pf(V.rs, V.rs.global_allow[k], m, len, sc);
    for (uint32_t k = 0; k < rd.allow_n && !allowed; ++k)
      allowed = match_string_pf(V.rs, V.rs.allow_progs[rd.allow_off + k], m, len, sc);
    if (!allowed) emit_kept<uint64_t>(V, rd, M.rule, M.file, M.job, text, M.ms, M.me);
  }
}

// Capture stages: a fixed grid walks the list the previous stage filled,
// its length read on the device (no host round trip between the stages).
// Only kActive lanes of each 64-lane block search (each with its own arena):
// the backtracker's control flow differs per job, so jobs sharing a wave run
// one after another; few active lanes per wave and many waves per CU keep
// each wave to about one job and let the CU overlap their load latencies.
// Secret groups by byte runs (gre::group_run), one lane per match: the
// group ends where the trailing run of the rule's after-group bytes begins and
// starts at its fixed length or the run of group bytes before that.
template <class Pos>
__global__ __launch_bounds__(256) void k_group_runs(VerifyParams V);

// Files longer than 2^31 - 1 bytes (kMaxVerifyFile: the 32-bit instantiations
// keep capture slots in int32): true when the job / location of file fi belongs to
// the 64-bit instantiation of the search kernels (each kernel is launched
// twice when the batch holds such a file; every lane skips the other's work).
__device__ inline bool is_long_file(const uint64_t* off, uint32_t fi) { return off[fi + 1] - 1 - off[fi] > kMaxVerifyFile; }

template <uint32_t kLanes, uint32_t kActive, uint32_t kWords, bool kLast, class Pos>
__global__ __launch_bounds__(kLanes) void k_captures(VerifyParams V) {
  __shared__ uint32_t bs_lds[kActive * kWords];
  if (threadIdx.x >= kActive) return;
  uint32_t* bs_area = bs_lds + threadIdx.x * kWords;
  const uint32_t nthreads = gridDim.x * kActive;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(V.scratch + (uint64_t)t * V.scratch_stride, V.rs);
  const CapJob* list = kLast ? V.caps_big : V.caps;
  const unsigned long long cnt = kLast ? V.ctrl->n_caps_big : V.ctrl->n_caps;
  const uint64_t cap = kLast ? V.cap_big_cap : V.cap_cap;
  const uint64_t n_caps = cnt < cap ? cnt : cap;
  // job i -> block i % grid, lane i / grid: a short list spreads over every CU
  // (few divergent lanes per wave) instead of filling the first waves
  for (uint64_t i = blockIdx.x + (uint64_t)threadIdx.x * gridDim.x; i < n_caps; i += nthreads) {
    const CapJob c = list[i];
    if (job_void(V.job_bad, c.job)) continue;  // a conflicting speculative job's (or a deferred fast job's) match
    if (is_long_file(V.off, c.file) != (sizeof(Pos) > 4)) continue;
    const RuleDev rd = V.rs.rules[c.rule];
    const uint64_t fstart = V.off[c.file];
    const Pos n = (Pos)(V.off[c.file + 1] - 1 - fstart);
    emit_groups<Pos>(V, rd, c.rule, c.file, c.job, V.data + fstart, n, (Pos)c.ms, (Pos)c.me, sc, bs_area, kWords,
                     kLast ? nullptr : V.caps_big, V.cap_big_cap, &V.ctrl->n_caps_big);
  }
}

template <class Pos>
__global__ __launch_bounds__(256) void k_group_runs(VerifyParams V) {
  const unsigned long long cnt = V.ctrl->n_caps_run;
  const uint64_t n = cnt < V.cap_run_cap ? cnt : V.cap_run_cap;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const CapJob c = V.caps_run[i];
    if (job_void(V.job_bad, c.job)) continue;  // a conflicting speculative job's (or a deferred fast job's) match
    if (is_long_file(V.off, c.file) != (sizeof(Pos) > 4)) continue;
    const RuleDev& rd = V.rs.rules[c.rule];
    const uint8_t* text = V.data + V.off[c.file];
    const Pos ms = (Pos)c.ms, me = (Pos)c.me;
    const uint32_t sm[4] = {rd.grp_s[0], rd.grp_s[1], rd.grp_s[2], rd.grp_s[3]};
    const Pos ge = run_back<Pos>(text, ms, me, sm);
    Pos gs;
    if (rd.grp_run_len >= 0) {
      if (ge < ms || ge - ms < (Pos)rd.grp_run_len) {  // (not for a real match of the rule: the capture search decides)
        const unsigned long long ci = atomicAdd(&V.ctrl->n_caps, 1ull);
        if (ci < V.cap_cap) V.caps[ci] = c;
        continue;
      }
      gs = ge - (Pos)rd.grp_run_len;
    } else {
      const uint32_t bm[4] = {rd.grp_b[0], rd.grp_b[1], rd.grp_b[2], rd.grp_b[3]};
      gs = run_back<Pos>(text, ms, ge, bm);
    }
    loc_emit(V, DevLoc{c.file, c.rule, (uint64_t)gs, (uint64_t)ge, 0, 0, 0, c.job});
  }
}

// Pull the rule tables k_verify walks (programs, classes, verify DFAs, rule
// records) back into every XCD's L2 after the scan streamed the batch through
// it: k_verify's walks are chains of dependent loads, and a cold line there
// costs an HBM round trip per step.  Block b serves XCD b % 8 (round-robin
// dispatch), part b / 8 of each range; nothing is written.
struct WarmRanges {
  const uint8_t* p[10];
  uint64_t n[10];
  uint32_t k;
};
constexpr uint32_t kWarmParts = 8;

__global__ __launch_bounds__(256) void k_warm(WarmRanges R, uint32_t* sink) {
  const uint32_t part = blockIdx.x / 8;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < R.k; ++r) {
    const uint64_t lines = (R.n[r] + 127) / 128;
    const uint64_t per = (lines + kWarmParts - 1) / kWarmParts;
    const uint64_t l0 = part * per, l1 = l0 + per < lines ? l0 + per : lines;
    for (uint64_t l = l0 + threadIdx.x; l < l1; l += blockDim.x) acc = acc * 31u + R.p[r][l * 128];
  }
  if (acc == 0x5EED1234u) sink[0] = acc;  // keeps the loads alive
}

// The match search: no LDS, so occupancy hides the dependent global reads of
// the DFA / VM walks; secret-group captures are left to k_captures.  Each job
// kind runs in a function of its own: the Pike VM takes its start oracle by
// reference, which would otherwise put the DFA path's IvIter (read on every
// start) in scratch memory -- 35 K lanes of scratch thrash L2 and made each
// dependent DFA step an HBM round trip (k_verify 1.96 ms at 50 GB).
// Block shapes: 64 lanes (one wave) spreads a short job list over every CU
// (UTCL1 reach per CU); a long list (findings-heavy corpora: millions of
// jobs) takes 256-lane blocks -- four waves share one staged DFA, so the
// 64 KiB of LDS per block no longer caps a CU at two resident waves.
constexpr uint32_t kVerifyBlock = 64;
constexpr uint32_t kVerifyBlockWide = 256;

// regexp.go allMatches over the whole file (rules without an anchor)
template <class Pos>
__device__ __noinline__ void verify_full_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                             const uint8_t* text, Pos n, gre::VmScratch& sc) {
  const gre::ProgView& pv = V.rs.progs[V.rs.rules[rule].prog];
  Pos pos = 0, ms, me;
  int64_t prev_end = -1;
  while (pos <= n) {
    LimitStarts<Pos> ls{n};
    if (!vm_search_starts(pv, text, n, pos, ls, sc, &ms, &me)) break;
    bool accept = true;
    if (me == pos) {
      if ((int64_t)ms == prev_end) accept = false;
      uint32_t w;
      gre::decode_rune(text, n, pos, &w);
      pos = w > 0 ? pos + w : n + 1;
    } else {
      pos = me;
    }
    prev_end = me;
    if (accept) emit_match(V, rule, fi, job, text, n, ms, me, sc);
  }
}

// A job's first match start and last match end (every match FindAll took,
// allow-listed ones included: they move its position all the same), for
// k_chain_fix; a re-run chain (kJobRedo) records nothing.
// (fms == ~Pos(0): the job found no match)
template <class Pos>
__device__ inline void job_record(const VerifyParams& V, uint32_t job, Pos fms, Pos lme) {
  if (job & kJobRedo) return;
  job &= kJobMask;
  V.job_fms[job] = fms == ~(Pos)0 ? ~0ull : (uint64_t)fms;
  V.job_lme[job] = lme;
}

template <class Pos>
__device__ inline void iv_init(IvIter<Pos>& it, const VerifyParams& V, uint32_t rule, uint64_t c0, uint64_t c1,
                               uint64_t fstart, const uint8_t* text, Pos n) {
  const RuleDev& rd = V.rs.rules[rule];
  it.keys = V.keys;
  it.ci = c0;
  it.c1 = c1;
  it.fstart = fstart;
  it.text = text;
  it.n = n;
  it.a = rd.off_min;
  it.b = rd.off_max;
  it.al0 = rd.alpha[0];
  it.al1 = rd.alpha[1];
  it.al2 = rd.alpha[2];
  it.al3 = rd.alpha[3];
  it.have_prev = false;
  it.h_prev = it.p_prev = 0;
  it.advance();
}

// FindAll over the anchor windows with the verify DFA: the first permitted
// start (>= pos) that matches is Go's leftmost match; a start the DFA cannot
// decide (byte >= 0x80) is decided by the Pike VM alone, anchored there.
template <bool kLds, class Pos>
__device__ __noinline__ uint32_t verify_dfa_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                                Pos pos0, uint64_t c0, uint64_t c1, uint64_t fstart,
                                                const uint8_t* text, Pos n, gre::VmScratch& sc,
                                                const uint16_t* lds_T, const uint8_t* lds_cls, uint32_t* tck) {
  uint32_t steps = 0;  // DFA transitions taken (diagnostics)
  uint32_t tck_dfa = 0, tck_emit = 0;
  const RuleDev& rd = V.rs.rules[rule];
  const DfaRef dref{kLds ? lds_T : V.rs.dfa_delta + rd.dfa_off, kLds ? lds_cls : V.rs.dfa_bytes + rd.dfa_cls_off,
                    rd.dfa_ncls, rd.dfa_start0, rd.dfa_start1, rd.dfa_smatch, rd.dfa_sym,
                    V.no_accel ? nullptr : (const uint32_t*)(V.rs.dfa_bytes + rd.dfa_accel_off),
                    (const uint4*)(V.rs.dfa_bytes + rd.dfa_accel_recs)};
  const uint32_t fm0 = rd.dfa_first[0], fm1 = rd.dfa_first[1], fm2 = rd.dfa_first[2], fm3 = rd.dfa_first[3];
  const uint32_t prog = rd.prog;
  IvIter<Pos> it;
  iv_init(it, V, rule, c0, c1, fstart, text, n);
  Pos pos = pos0, ms, me, fms = ~(Pos)0, lme = 0;
  while (it.have && it.ce < pos) it.advance();
  while (it.have) {
    bool found = false;
    const Pos s0 = it.cs > pos ? it.cs : pos;
    VecText TS(text);  // the window's bytes, one 16-byte load per block
    for (Pos sp = s0; sp <= it.ce && sp < n; ++sp) {
      const uint32_t b0 = TS[sp];  // first-byte skip (no dependent table loads)
      if (b0 >= 0x80 && !gre::is_rune_start(text, n, sp)) continue;  // (an ASCII byte starts a rune)
      const uint32_t fw = b0 < 32 ? fm0 : b0 < 64 ? fm1 : b0 < 96 ? fm2 : fm3;
      if (b0 < 0x80 && !((fw >> (b0 & 31)) & 1)) continue;
      const uint64_t ta = tck ? __builtin_amdgcn_s_memrealtime() : 0;
      int r = dfa_anchored_dev<kLds, Pos>(dref, text, n, sp, &me, &steps);
      if (tck) tck_dfa += (uint32_t)(__builtin_amdgcn_s_memrealtime() - ta);
      if (r == 2) {
        OneStart<Pos> one{sp};
        r = vm_search_starts<Pos>(V.rs.progs[prog], text, n, sp, one, sc, &ms, &me) ? 1 : 0;
      }
      if (r == 1) {
        const uint64_t tb = tck ? __builtin_amdgcn_s_memrealtime() : 0;
        emit_match<Pos>(V, rule, fi, job, text, n, sp, me, sc, tck);
        if (tck) tck_emit += (uint32_t)(__builtin_amdgcn_s_memrealtime() - tb);
        if (fms == ~(Pos)0) fms = sp;
        lme = me;
        pos = me;
        found = true;
        break;
      }
    }
    if (!found) it.advance();
    else while (it.have && it.ce < pos) it.advance();
  }
  if (tck) { tck[0] = tck_dfa; tck[1] = tck_emit; }
  job_record(V, job, fms, lme);
  return steps;
}

// The same FindAll with the Pike VM (rules without a verify DFA)
template <class Pos>
__device__ __noinline__ void verify_vm_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                           Pos pos0, uint64_t c0, uint64_t c1, uint64_t fstart,
                                           const uint8_t* text, Pos n, gre::VmScratch& sc) {
  const gre::ProgView& pv = V.rs.progs[V.rs.rules[rule].prog];
  IvIter<Pos> it;
  iv_init(it, V, rule, c0, c1, fstart, text, n);
  Pos pos = pos0, ms, me, fms = ~(Pos)0, lme = 0;
  while (it.have) {
    if (!vm_search_starts<Pos>(pv, text, n, pos, it, sc, &ms, &me)) break;
    emit_match<Pos>(V, rule, fi, job, text, n, ms, me, sc);
    if (fms == ~(Pos)0) fms = ms;
    lme = me;
    if (me == ms) break;  // cannot happen for anchored rules (non-empty literal)
    pos = me;
  }
  job_record(V, job, fms, lme);
}

// FindAll over the anchor windows with the bit-parallel NFA (nfa.cpp; rules
// whose verify DFA exploded or that use \b / (?m) assertions): one walk
// with a thread started at every permitted start of the window tells whether
// any of them matches (most windows: no -- done); then the starts in order,
// each with an anchored walk, the first that matches is Go's leftmost match,
// and its end is the walk's when that is the only end a match from that start
// can have.  A start the walk cannot decide (a byte >= 0x80, two possible
// ends -- Go's priorities choose -- or a walk past kNfaWalkMax) is decided by
// the Pike VM anchored there.
template <bool kWide, class Pos>
__device__ __noinline__ uint32_t verify_nfa_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job,
                                                Pos pos0, uint64_t c0, uint64_t c1, uint64_t fstart,
                                                const uint8_t* text, Pos n, gre::VmScratch& sc,
                                                const uint8_t* nfa) {
  const NfaDev& N = *(const NfaDev*)nfa;
  const U128* reach = (const U128*)(nfa + N.o_reach);
  const NfaExc* exc = (const NfaExc*)(nfa + N.o_exc);
  const uint32_t prog = V.rs.rules[rule].prog;
  uint32_t steps = 0;
  IvIter<Pos> it;
  iv_init(it, V, rule, c0, c1, fstart, text, n);
  Pos pos = pos0, ms, me, fms = ~(Pos)0, lme = 0;
  while (it.have && it.ce < pos) it.advance();
  while (it.have) {
    bool found = false;
    const Pos s0 = it.cs > pos ? it.cs : pos;
    const Pos s1 = it.ce < n ? it.ce : n;
    int any = 0;
    if (s0 <= s1) {
      VecText T(text);
      any = nfa_walk<kWide>(N, reach, exc, T, n, s0, s1, &me, &steps);
    }
    for (Pos sp = s0; any && sp <= s1 && sp < n; ++sp) {
      if (!gre::is_rune_start(text, n, sp)) continue;
      const uint32_t b0 = as_global<gu8>(text)[sp];
      if (b0 < 0x80 && !nfa_first_ok(N, reach, b0)) continue;  // first-byte skip
      VecText T(text);
      int r = nfa_walk<kWide>(N, reach, exc, T, n, sp, sp, &me, &steps);
      if (r == 2) {
        OneStart<Pos> one{sp};
        r = vm_search_starts<Pos>(V.rs.progs[prog], text, n, sp, one, sc, &ms, &me) ? 1 : 0;
      }
      if (r == 1) {
        emit_match<Pos>(V, rule, fi, job, text, n, sp, me, sc);
        if (fms == ~(Pos)0) fms = sp;
        lme = me;
        pos = me;
        found = true;
        break;
      }
    }
    if (!found) it.advance();
    else while (it.have && it.ce < pos) it.advance();
  }
  job_record(V, job, fms, lme);
  return steps;
}

// k_verify_fast's job paths: the verify DFA / NFA walks of verify_dfa_job /
// verify_nfa_job with every Pike VM call replaced by a deferral (return 0):
// a start the walk cannot decide, or an allow rule the DFA cannot decide.
// Matches found before a deferral are tagged kJobFast and voided with the job.
template <bool kLds, class Pos>
__device__ __forceinline__ int fast_dfa_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job, uint64_t c0,
                                         uint64_t c1, uint64_t fstart, const uint8_t* text, Pos n,
                                         const uint16_t* lds_T, const uint8_t* lds_cls) {
  uint32_t steps = 0;
  const RuleDev& rd = V.rs.rules[rule];
  const DfaRef dref{kLds ? lds_T : V.rs.dfa_delta + rd.dfa_off, kLds ? lds_cls : V.rs.dfa_bytes + rd.dfa_cls_off,
                    rd.dfa_ncls, rd.dfa_start0, rd.dfa_start1, rd.dfa_smatch, rd.dfa_sym,
                    V.no_accel ? nullptr : (const uint32_t*)(V.rs.dfa_bytes + rd.dfa_accel_off),
                    (const uint4*)(V.rs.dfa_bytes + rd.dfa_accel_recs)};
  const uint32_t fm0 = rd.dfa_first[0], fm1 = rd.dfa_first[1], fm2 = rd.dfa_first[2], fm3 = rd.dfa_first[3];
  IvIter<Pos> it;
  iv_init(it, V, rule, c0, c1, fstart, text, n);
  Pos pos = 0, me, fms = ~(Pos)0, lme = 0;
  while (it.have) {
    bool found = false;
    const Pos s0 = it.cs > pos ? it.cs : pos;
    VecText TS(text);
    for (Pos sp = s0; sp <= it.ce && sp < n; ++sp) {
      const uint32_t b0 = TS[sp];
      if (b0 >= 0x80 && !gre::is_rune_start(text, n, sp)) continue;
      const uint32_t fw = b0 < 32 ? fm0 : b0 < 64 ? fm1 : b0 < 96 ? fm2 : fm3;
      if (b0 < 0x80 && !((fw >> (b0 & 31)) & 1)) continue;
      const int r = dfa_anchored_dev<kLds, Pos>(dref, text, n, sp, &me, &steps);
      if (r == 2) return 0;
      if (r == 1) {
        if (!emit_match_fast<Pos>(V, rule, fi, job, text, sp, me)) return 0;
        if (fms == ~(Pos)0) fms = sp;
        lme = me;
        pos = me;
        found = true;
        break;
      }
    }
    if (!found) it.advance();
    else while (it.have && it.ce < pos) it.advance();
  }
  job_record(V, job, fms, lme);
  return 1;
}

template <bool kWide, class Pos>
__device__ __forceinline__ int fast_nfa_job(const VerifyParams& V, uint32_t rule, uint32_t fi, uint32_t job, uint64_t c0,
                                         uint64_t c1, uint64_t fstart, const uint8_t* text, Pos n, const uint8_t* nfa) {
  const NfaDev& N = *(const NfaDev*)nfa;
  const U128* reach = (const U128*)(nfa + N.o_reach);
  const NfaExc* exc = (const NfaExc*)(nfa + N.o_exc);
  uint32_t steps = 0;
  IvIter<Pos> it;
  iv_init(it, V, rule, c0, c1, fstart, text, n);
  Pos pos = 0, me, fms = ~(Pos)0, lme = 0;
  while (it.have) {
    bool found = false;
    const Pos s0 = it.cs > pos ? it.cs : pos;
    const Pos s1 = it.ce < n ? it.ce : n;
    int any = 0;
    if (s0 <= s1) {
      VecText T(text);
      any = nfa_walk<kWide>(N, reach, exc, T, n, s0, s1, &me, &steps);  // (2: the starts one by one decide)
    }
    for (Pos sp = s0; any && sp <= s1 && sp < n; ++sp) {
      if (!gre::is_rune_start(text, n, sp)) continue;
      const uint32_t b0 = as_global<gu8>(text)[sp];
      if (b0 < 0x80 && !nfa_first_ok(N, reach, b0)) continue;
      VecText T(text);
      const int r = nfa_walk<kWide>(N, reach, exc, T, n, sp, sp, &me, &steps);
      if (r == 2) return 0;
      if (r == 1) {
        if (!emit_match_fast<Pos>(V, rule, fi, job, text, sp, me)) return 0;
        if (fms == ~(Pos)0) fms = sp;
        lme = me;
        pos = me;
        found = true;
        break;
      }
    }
    if (!found) it.advance();
    else while (it.have && it.ce < pos) it.advance();
  }
  job_record(V, job, fms, lme);
  return 1;
}

// One job without the Pike VM: 1 = done, 0 = deferred to k_verify_slow
// (full-scan jobs and rules with neither a verify DFA nor an NFA at once).
template <class Pos>
__device__ inline int run_job_fast(const VerifyParams& V, uint32_t job, uint64_t c0, uint64_t c1,
                                   const uint16_t* lds_dfa, const uint8_t* lds_cls, const uint8_t* lds_nfa) {
  const uint32_t rule = (uint32_t)(V.keys[c0] >> kPosBits);
  const uint32_t fi = V.vals[c0] & ~kFullFlag;
  for (uint64_t c = c0; c < c1; ++c)
    if (V.vals[c] & kFullFlag) return 0;
  const uint64_t fstart = V.off[fi];
  const uint8_t* text = V.data + fstart;
  const Pos n = (Pos)(V.off[fi + 1] - 1 - fstart);
  const RuleDev& rd = V.rs.rules[rule];
  if (lds_dfa) return fast_dfa_job<true, Pos>(V, rule, fi, job, c0, c1, fstart, text, n, lds_dfa, lds_cls);
  if (rd.dfa_off != kNoFollow) return fast_dfa_job<false, Pos>(V, rule, fi, job, c0, c1, fstart, text, n, nullptr, nullptr);
  if (rd.nfa_off != kNoFollow) {
    const uint8_t* nfa = lds_nfa ? lds_nfa : V.rs.nfa_bytes + rd.nfa_off;
    return ((const NfaDev*)nfa)->npos > 64 ? fast_nfa_job<true, Pos>(V, rule, fi, job, c0, c1, fstart, text, n, nfa)
                                            : fast_nfa_job<false, Pos>(V, rule, fi, job, c0, c1, fstart, text, n, nfa);
  }
  return 0;
}

// The block (one wave) stages the verify DFA of its first job's rule in LDS:
// jobs are sorted by rule, so nearly every lane walks that table, and an LDS
// step costs no L2 round trip and no TLB lookup (the random text pages the
// lanes touch evict the table's translations from the small per-CU TLB).
constexpr uint32_t kVerifyDfaLds = 64 * 1024;

// One job's FindAll over candidates [c0, c1) from search position pos0, with
// the rule's verify DFA, else its NFA, else the Pike VM; full-scan jobs run
// the VM over the whole file.  lds_dfa / lds_nfa: the block's staged table
// when this job's rule is the one staged (else null: global tables).
template <class Pos>
__device__ inline uint32_t run_job(const VerifyParams& V, uint32_t job, Pos pos0, uint64_t c0, uint64_t c1,
                                   gre::VmScratch& sc, const uint16_t* lds_dfa, const uint8_t* lds_cls,
                                   const uint8_t* lds_nfa, bool* full_out) {
  const uint32_t rule = (uint32_t)(V.keys[c0] >> kPosBits);
  const uint32_t fi = V.vals[c0] & ~kFullFlag;
  bool full = false;
  for (uint64_t c = c0; c < c1 && !full; ++c) full = (V.vals[c] & kFullFlag) != 0;
  *full_out = full;
  const uint64_t fstart = V.off[fi];
  const uint8_t* text = V.data + fstart;
  const Pos n = (Pos)(V.off[fi + 1] - 1 - fstart);  // NUL separator excluded
  uint32_t* tck = V.tck && !(job & kJobRedo) ? V.tck + 4 * job : nullptr;
  const RuleDev& rd = V.rs.rules[rule];
  if (full) {
    verify_full_job<Pos>(V, rule, fi, job, text, n, sc);
    return 0;
  }
  if (lds_dfa)
    return verify_dfa_job<true, Pos>(V, rule, fi, job, pos0, c0, c1, fstart, text, n, sc, lds_dfa, lds_cls, tck);
  if (rd.dfa_off != kNoFollow)
    return verify_dfa_job<false, Pos>(V, rule, fi, job, pos0, c0, c1, fstart, text, n, sc, nullptr, nullptr, tck);
  if (rd.nfa_off != kNoFollow) {
    const uint8_t* nfa = lds_nfa ? lds_nfa : V.rs.nfa_bytes + rd.nfa_off;
    return ((const NfaDev*)nfa)->npos > 64
               ? verify_nfa_job<true, Pos>(V, rule, fi, job, pos0, c0, c1, fstart, text, n, sc, nfa)
               : verify_nfa_job<false, Pos>(V, rule, fi, job, pos0, c0, c1, fstart, text, n, sc, nfa);
  }
  verify_vm_job<Pos>(V, rule, fi, job, pos0, c0, c1, fstart, text, n, sc);
  return 0;
}

// Lanes of one wave run their jobs in lock-step: a wave whose 64 jobs walk
// different windows, DFA paths and emits executes the union of them, so on a
// short job list (a few waves per CU: configs[2]) the wave's time grows with
// its job count.  V.jpw < 64 gives each wave only jpw jobs (lanes [0, jpw))
// and the list more waves.
template <uint32_t kBlock, class Pos>
__global__ __launch_bounds__(kBlock) void k_verify(VerifyParams V) {
  __shared__ __align__(16) uint16_t dfa_lds[kVerifyDfaLds / 2];
  __shared__ __align__(16) uint8_t cls_lds[128];
  const uint32_t jpw = V.jpw;
  const uint32_t per_block = (kBlock / 64) * jpw;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t jslot = (threadIdx.x >> 6) * jpw + lane;  // this lane's job in the block's group
  // (VM scratch per active lane: grid x per_block <= vm_threads, checked by the launch)
  gre::VmScratch sc = make_scratch(V.scratch + ((uint64_t)blockIdx.x * per_block + jslot) * V.scratch_stride, V.rs);
  const uint32_t n_jobs = *V.n_jobs_dev;
  for (uint32_t jb = blockIdx.x * per_block; jb < n_jobs; jb += gridDim.x * per_block) {  // block-uniform
    const uint32_t r0 = (uint32_t)(V.keys[V.job_start[jb]] >> kPosBits);
    const RuleDev& rd0 = V.rs.rules[r0];
    const bool staged = rd0.dfa_off != kNoFollow && rd0.dfa_size * 2 <= kVerifyDfaLds;
    // (or its bit-parallel NFA record, rules without a DFA)
    const bool staged_nfa = !staged && rd0.dfa_off == kNoFollow && rd0.nfa_off != kNoFollow &&
                            rd0.nfa_bytes <= kVerifyDfaLds;
    __syncthreads();  // the previous group's walks are done with the table
    if (staged) {
      const uint32_t* src = (const uint32_t*)(V.rs.dfa_delta + rd0.dfa_off);  // dfa_off is even (build pads)
      for (uint32_t i = threadIdx.x; i < (rd0.dfa_size + 1) / 2; i += blockDim.x) ((uint32_t*)dfa_lds)[i] = src[i];
      for (uint32_t i = threadIdx.x; i < 128; i += blockDim.x) cls_lds[i] = V.rs.dfa_bytes[rd0.dfa_cls_off + i];
    } else if (staged_nfa) {
      const uint32_t* src = (const uint32_t*)(V.rs.nfa_bytes + rd0.nfa_off);  // 16-byte aligned records
      for (uint32_t i = threadIdx.x; i < rd0.nfa_bytes / 4; i += blockDim.x) ((uint32_t*)dfa_lds)[i] = src[i];
    }
    __syncthreads();
    const uint32_t j = jb + jslot;
    if (lane >= jpw || j >= n_jobs) continue;
    const uint64_t t0 = V.prof ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz wall clock
    const uint64_t c0 = V.job_start[j];
    const uint64_t c1 = (j + 1 < n_jobs) ? V.job_start[j + 1] : V.n_cands;
    if (is_long_file(V.off, V.vals[c0] & ~kFullFlag) != (sizeof(Pos) > 4)) continue;
    const uint32_t rule = (uint32_t)(V.keys[c0] >> kPosBits);
    bool full = false;
    const uint32_t steps = run_job<Pos>(V, j, 0, c0, c1, sc, staged && rule == r0 ? dfa_lds : nullptr, cls_lds,
                                        staged_nfa && rule == r0 ? (const uint8_t*)dfa_lds : nullptr, &full);
    if (V.prof) {  // diagnostics (TSG_PROFILE_VERIFY): duration | end, rule | full
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      V.prof[2 * j] = (t1 - t0) | ((t1 & 0xFFFFFFFFull) << 32);
      V.prof[2 * j + 1] = ((uint64_t)rule << 32) | (steps << 1) | (full ? 1u : 0u);
    }
  }
}

// The match search in two kernels.  k_verify_fast runs every job on the
// verify DFA / NFA paths, which never reach the Pike VM, so it compiles to a
// register budget of its own (the VM's ~250 VGPRs and private stack capped
// k_verify at two waves per SIMD); a job that needs the VM (a start the walk
// cannot decide, an allow rule its DFA cannot decide, full-scan jobs, rules
// with neither table) is flagged (job_bad bit 1, its fast output void) and
// listed for k_verify_slow, which runs it whole with the VM-capable paths.
constexpr uint32_t kVerifyFastLds = 32 * 1024;  // staged table: five 256-lane blocks per CU
template <uint32_t kBlock, class Pos>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_verify_fast(VerifyParams V) {
  __shared__ __align__(16) uint16_t dfa_lds[kVerifyFastLds / 2];
  __shared__ __align__(16) uint8_t cls_lds[128];
  const uint32_t nthreads = gridDim.x * blockDim.x;
  const uint32_t n_jobs = *V.n_jobs_dev;
  for (uint32_t jb = blockIdx.x * blockDim.x; jb < n_jobs; jb += nthreads) {  // block-uniform
    const uint32_t r0 = (uint32_t)(V.keys[V.job_start[jb]] >> kPosBits);
    const RuleDev& rd0 = V.rs.rules[r0];
    const bool staged = rd0.dfa_off != kNoFollow && rd0.dfa_size * 2 <= kVerifyFastLds;
    const bool staged_nfa = !staged && rd0.dfa_off == kNoFollow && rd0.nfa_off != kNoFollow &&
                            rd0.nfa_bytes <= kVerifyFastLds;
    __syncthreads();  // the previous group's walks are done with the table
    if (staged) {
      const uint32_t* src = (const uint32_t*)(V.rs.dfa_delta + rd0.dfa_off);
      for (uint32_t i = threadIdx.x; i < (rd0.dfa_size + 1) / 2; i += blockDim.x) ((uint32_t*)dfa_lds)[i] = src[i];
      for (uint32_t i = threadIdx.x; i < 128; i += blockDim.x) cls_lds[i] = V.rs.dfa_bytes[rd0.dfa_cls_off + i];
    } else if (staged_nfa) {
      const uint32_t* src = (const uint32_t*)(V.rs.nfa_bytes + rd0.nfa_off);
      for (uint32_t i = threadIdx.x; i < rd0.nfa_bytes / 4; i += blockDim.x) ((uint32_t*)dfa_lds)[i] = src[i];
    }
    __syncthreads();
    const uint32_t j = jb + threadIdx.x;
    if (j >= n_jobs) continue;
    const uint64_t c0 = V.job_start[j];
    const uint64_t c1 = (j + 1 < n_jobs) ? V.job_start[j + 1] : V.n_cands;
    if (is_long_file(V.off, V.vals[c0] & ~kFullFlag) != (sizeof(Pos) > 4)) continue;
    const uint32_t rule = (uint32_t)(V.keys[c0] >> kPosBits);
    if (!run_job_fast<Pos>(V, j, c0, c1, staged && rule == r0 ? dfa_lds : nullptr, cls_lds,
                           staged_nfa && rule == r0 ? (const uint8_t*)dfa_lds : nullptr)) {
      V.job_bad[j] |= 2;
      const unsigned long long k = atomicAdd(&V.ctrl->n_defer, 1ull);
      V.defer[k] = j;  // (capacity: every job)
    }
  }
}

template <class Pos>
__global__ __launch_bounds__(64) void k_verify_slow(VerifyParams V) {
  const uint64_t n = V.ctrl->n_defer;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(V.scratch + (uint64_t)t * V.scratch_stride, V.rs);
  const uint32_t n_jobs = *V.n_jobs_dev;
  // job i -> block i % grid, lane i / grid: a short list spreads over every CU
  for (uint64_t i = blockIdx.x + (uint64_t)threadIdx.x * gridDim.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = V.defer[i];
    const uint64_t c0 = V.job_start[j];
    const uint64_t c1 = (j + 1 < n_jobs) ? V.job_start[j + 1] : V.n_cands;
    if (is_long_file(V.off, V.vals[c0] & ~kFullFlag) != (sizeof(Pos) > 4)) continue;
    bool full;
    run_job<Pos>(V, j, 0, c0, c1, sc, nullptr, nullptr, nullptr, &full);
  }
}

// The speculative chains (one lane per chain head -- a job whose first
// candidate starts a hard split -- over the soft-split jobs after it): the
// first job whose first match starts before the previous match's end is a
// conflict; that job and the rest of its chain are re-run in order from that
// end (k_verify_redo), and their speculative output is dropped.
__global__ void k_chain_fix(VerifyParams V) {
  const uint32_t n_jobs = *V.n_jobs_dev;
  const uint32_t j0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (j0 >= n_jobs || V.split[V.job_start[j0]] != kSplitHard) return;
  if (j0 + 1 >= n_jobs || V.split[V.job_start[j0 + 1]] != kSplitSoft) return;  // a chain of one
  uint32_t last = j0 + 1;
  while (last + 1 < n_jobs && V.split[V.job_start[last + 1]] == kSplitSoft) ++last;
  uint64_t end = V.job_fms[j0] != ~0ull ? V.job_lme[j0] : 0;
  for (uint32_t j = j0 + 1; j <= last; ++j) {
    const uint64_t f = V.job_fms[j];
    if (f == ~0ull) continue;
    if (f < end) {
      for (uint32_t q = j; q <= last; ++q) V.job_bad[q] |= 1;
      const unsigned long long k = atomicAdd(&V.ctrl->n_redo, 1ull);
      if (k < V.redo_cap) V.redo[k] = RedoRec{j, last, end};
      return;
    }
    end = V.job_lme[j];
  }
}

// One lane per conflict: the chain's remaining jobs in order, as ONE job
// (their candidates are consecutive), from the conflict's search position.
template <class Pos>
__global__ __launch_bounds__(64) void k_verify_redo(VerifyParams V) {
  const uint64_t n = V.ctrl->n_redo < V.redo_cap ? V.ctrl->n_redo : V.redo_cap;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(V.scratch + (uint64_t)t * V.scratch_stride, V.rs);
  const uint32_t n_jobs = *V.n_jobs_dev;
  for (uint64_t i = t; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const RedoRec R = V.redo[i];
    const uint64_t c0 = V.job_start[R.job];
    const uint64_t c1 = R.last + 1 < n_jobs ? V.job_start[R.last + 1] : V.n_cands;
    if (is_long_file(V.off, V.vals[c0] & ~kFullFlag) != (sizeof(Pos) > 4)) continue;
    bool full;
    run_job<Pos>(V, kJobRedo | R.job, (Pos)R.pos, c0, c1, sc, nullptr, nullptr, nullptr, &full);
  }
}

// Locations of conflicting speculative jobs are flagged dropped (flags bit
// 2) and counted; the host compacts them away.
__global__ void k_drop_spec(VerifyParams V) {
  const uint64_t n_locs = V.ctrl->locs < V.loc_cap ? V.ctrl->locs : V.loc_cap;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_locs; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t job = V.locs[i].job;
    if (job_void(V.job_bad, job)) {
      V.locs[i].flags |= 2;
      atomicAdd(&V.ctrl->n_dropped, 1ull);
    }
  }
}

__global__ void k_keep_flags(const DevLoc* locs, uint64_t n, uint8_t* keep) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keep[i] = (locs[i].flags & 2) ? 0 : 1;
}

// --------------------------------------------------------------- exclude --
struct ExclRange {
  uint32_t tag;
  uint32_t pad;
  uint64_t s, e;
};

// Exclude blocks on the device (Blocks.Match / find, scanner.go:232-270,413-419):
// a kept location needs the FindAll ranges of its file's global blocks (scope
// 0) and of its rule's blocks (scope rule + 1).  The (file, scope) groups are
// the unique keys of k_excl_keys (sorted, ~0 = none); k_exclude_tags runs the
// FindAll of every (group, exclude regex) pair; the ranges sorted by (group,
// start) with a running maximum of their ends per group (k_excl_pmax) answer
// "some range of the group contains [start, end)" with one binary search
// (k_excl_filter) -- no location leaves the device.
struct ExclDev {
  const uint32_t* xoff;   // per rule: its exclude regexes xprog[xoff[r], xoff[r + 1])
  const uint32_t* xprog;
  const uint32_t* gx;     // global exclude regexes
  uint32_t n_gx, max_x;   // max_x: most regexes of one scope
};

__global__ void k_excl_keys(const DevLoc* locs, uint64_t n, ExclDev X, uint64_t* keys, uint32_t* idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DevLoc L = locs[i];
  keys[2 * i] = X.n_gx ? ((uint64_t)L.file << 32) : ~0ull;
  keys[2 * i + 1] = X.xoff[L.rule + 1] > X.xoff[L.rule] ? (((uint64_t)L.file << 32) | (L.rule + 1)) : ~0ull;
  idx[2 * i] = (uint32_t)(2 * i);
  idx[2 * i + 1] = (uint32_t)(2 * i + 1);
}

__global__ void k_excl_uniq(const uint64_t* keys, uint64_t n, uint8_t* flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = keys[i] != ~0ull && (i == 0 || keys[i] != keys[i - 1]);
}

__global__ __launch_bounds__(256) void k_exclude_tags(const uint8_t* data, const uint64_t* off, RuleSetDev rs,
                                                      ExclDev X, const uint64_t* skeys, const uint32_t* tidx,
                                                      const uint32_t* n_tags_dev,
                                                      ExclRange* out, uint64_t cap, Ctrl* ctrl, uint8_t* scratch,
                                                      uint64_t stride) {
  const uint32_t nthreads = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  gre::VmScratch sc = make_scratch(scratch + (uint64_t)t * stride, rs);
  const uint64_t n_jobs = (uint64_t)*n_tags_dev * X.max_x;
  for (uint64_t j = t; j < n_jobs; j += nthreads) {
    const uint32_t tag = (uint32_t)(j / X.max_x), k = (uint32_t)(j % X.max_x);
    const uint64_t key = skeys[tidx[tag]];
    const uint32_t file = (uint32_t)(key >> 32), scope = (uint32_t)key;
    const uint32_t nx = scope == 0 ? X.n_gx : X.xoff[scope] - X.xoff[scope - 1];
    if (k >= nx) continue;
    const uint32_t prog = scope == 0 ? X.gx[k] : X.xprog[X.xoff[scope - 1] + k];
    const uint8_t* text = data + off[file];
    const uint64_t n = off[file + 1] - 1 - off[file];  // (rare path: 64-bit positions for every file)
    const gre::ProgView& pv = rs.progs[prog];
    uint64_t pos = 0, ms, me;
    int64_t prev_end = -1;
    while (pos <= n) {  // FindAllIndex iteration (regexp.go allMatches)
      LimitStarts<uint64_t> ls{n};
      if (!vm_search_starts(pv, text, n, pos, ls, sc, &ms, &me)) break;
      bool accept = true;
      if (me == pos) {
        if ((int64_t)ms == prev_end) accept = false;
        uint32_t w;
        gre::decode_rune(text, n, pos, &w);
        pos = w > 0 ? pos + w : n + 1;
      } else {
        pos = me;
      }
      prev_end = me;
      if (accept) {
        unsigned long long idx = atomicAdd(&ctrl->excl, 1ull);
        if (idx < cap) out[idx] = ExclRange{tag, 0, ms, me};
      }
    }
  }
}

// (group, start) keys of the ranges (start < 2^40: kMaxFileBytes)
__global__ void k_excl_rkeys(const ExclRange* r, uint64_t n, uint64_t* keys, uint32_t* idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = ((uint64_t)r[i].tag << kKeyPosBits) | r[i].s;
  idx[i] = (uint32_t)i;
}

// running maximum of the ends inside each group's run, in (group, start)
// order (one lane per run)
__global__ void k_excl_pmax(const uint64_t* keys, const uint32_t* idx, const ExclRange* r, uint64_t* pmax,
                            uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (i > 0 && (keys[i] >> kKeyPosBits) == (keys[i - 1] >> kKeyPosBits))) return;
  const uint64_t g = keys[i] >> kKeyPosBits;
  uint64_t m = 0;
  for (uint64_t j = i; j < n && (keys[j] >> kKeyPosBits) == g; ++j) {
    const uint64_t e = r[idx[j]].e;
    m = e > m ? e : m;
    pmax[j] = m;
  }
}

__device__ inline bool excl_contains(const uint64_t* skeys, const uint32_t* tidx, uint32_t n_tags,
                                     const uint64_t* rkeys, const uint64_t* pmax, uint64_t n_r, uint64_t key,
                                     uint64_t s, uint64_t e) {
  uint32_t lo = 0, hi = n_tags;  // the group's index
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (skeys[tidx[m]] < key) lo = m + 1; else hi = m;
  }
  if (lo >= n_tags || skeys[tidx[lo]] != key) return false;
  // last range of the group starting at or before s
  const uint64_t want = ((uint64_t)lo << kKeyPosBits) | s;
  uint64_t a = 0, b = n_r;
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (rkeys[m] <= want) a = m + 1; else b = m;
  }
  return a > 0 && (rkeys[a - 1] >> kKeyPosBits) == lo && pmax[a - 1] >= e;
}

__global__ void k_excl_filter(const DevLoc* locs, uint64_t n, ExclDev X, const uint64_t* skeys, const uint32_t* tidx,
                              const uint32_t* n_tags_dev, const uint64_t* rkeys, const uint64_t* pmax, uint64_t n_r,
                              uint8_t* keep) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DevLoc L = locs[i];
  const uint32_t nt = *n_tags_dev;
  bool ex = X.n_gx && excl_contains(skeys, tidx, nt, rkeys, pmax, n_r, (uint64_t)L.file << 32, L.start, L.end);
  if (!ex && X.xoff[L.rule + 1] > X.xoff[L.rule])
    ex = excl_contains(skeys, tidx, nt, rkeys, pmax, n_r, ((uint64_t)L.file << 32) | (L.rule + 1), L.start, L.end);
  keep[i] = !ex;
}

// (file, start) sort keys of the kept locations
__global__ void k_loc_keys(const DevLoc* locs, uint64_t n, uint64_t* keys, uint32_t* idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = ((uint64_t)locs[i].file << kKeyPosBits) | locs[i].start;
  idx[i] = (uint32_t)i;
}

__global__ void k_loc_gather(const DevLoc* locs, const uint32_t* idx, uint64_t n, DevLoc* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = locs[idx[i]];
}

__global__ void k_flags8(const uint32_t* flags, uint8_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (uint8_t)flags[i];
}

// ----------------------------------------------------------------- lines --
// Global newline prefix G(x) = count('\n' in data[0,x)) from the per-8KiB
// block counts k_scan produced (nl_pre = their exclusive prefix sum) plus one
// wave-cooperative count inside x's block (<= 8 KiB, 128 B per lane).
__device__ inline uint32_t wave_nl_prefix(const uint8_t* data, const uint32_t* nl_pre, uint64_t x,
                                          uint32_t lane) {
  const uint64_t b0 = x & ~(uint64_t)(kNlBlock - 1);
  uint32_t c = 0;
  constexpr uint32_t kPer = kNlBlock / 64;  // bytes per lane
  const uint64_t s = b0 + (uint64_t)lane * kPer;
  // 16-byte vectors wholly before x (SWAR count), bytes for the partial one;
  // nothing at or past x is read
#pragma unroll
  for (uint32_t k = 0; k < kPer; k += 16) {
    const uint64_t p = s + k;
    if (p + 16 <= x) {
      const uint4 v = *(const uint4*)(data + p);
      c += nl_count_dword(v.x) + nl_count_dword(v.y) + nl_count_dword(v.z) + nl_count_dword(v.w);
    } else {
      for (uint64_t i = p; i < x && i < p + 16; ++i) c += data[i] == '\n';
    }
  }
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  return nl_pre[x / kNlBlock] + c;
}

// bit k set <=> byte k of the 16 is '\n'
__device__ inline uint32_t nl_mask16(uint4 v) {
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = d[k] ^ 0x0A0A0A0Au;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);  // 0x80 per '\n' byte
    m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
  }
  return m;
}

// wave_nl_prefix of x0 <= x1 <= x2 with one read of each distinct 4 KiB
// block (the lane's 64-byte slice: whole 16-byte vectors before the block's
// largest x, bytes for the partial one -- nothing at or past it is read).
__device__ inline void wave_nl_prefix3(const uint8_t* data, const uint32_t* nl_pre, uint64_t x0, uint64_t x1,
                                       uint64_t x2, uint32_t lane, uint32_t* out) {
  constexpr uint32_t kPer = kNlBlock / 64;  // bytes per lane
  const uint64_t xs[3] = {x0, x1, x2};
  uint64_t packed = 0;  // 21 bits per count (<= 4096 per block)
  int k = 0;
  while (k < 3) {
    const uint64_t b0 = xs[k] & ~(uint64_t)(kNlBlock - 1);
    int e = k;  // xs[k..e] share this block; xs[e] is the largest
    while (e + 1 < 3 && (xs[e + 1] & ~(uint64_t)(kNlBlock - 1)) == b0) ++e;
    const uint64_t xmax = xs[e];
    const uint64_t s0 = b0 + (uint64_t)lane * kPer;
    uint32_t m[kPer / 16];  // '\n' bit masks of the slice's vectors (bytes before xmax)
#pragma unroll
    for (uint32_t v = 0; v < kPer / 16; ++v) {
      const uint64_t p = s0 + 16 * v;
      if (p + 16 <= xmax) {
        m[v] = nl_mask16(*(const uint4*)(data + p));
      } else {
        uint32_t mm = 0;
        for (uint64_t i = p; i < xmax && i < p + 16; ++i) mm |= (data[i] == '\n' ? 1u : 0u) << (uint32_t)(i - p);
        m[v] = mm;
      }
    }
    for (int q = k; q <= e; ++q) {
      uint32_t c = 0;
#pragma unroll
      for (uint32_t v = 0; v < kPer / 16; ++v) {
        const uint64_t p = s0 + 16 * v;
        const uint32_t keep = p + 16 <= xs[q] ? 0xFFFFu : (xs[q] > p ? (1u << (uint32_t)(xs[q] - p)) - 1u : 0u);
        c += __builtin_popcount(m[v] & keep);
      }
      packed |= (uint64_t)c << (21 * q);
    }
    k = e + 1;
  }
  for (int d = 32; d > 0; d >>= 1) packed += __shfl_xor(packed, d);
  for (int q = 0; q < 3; ++q) out[q] = nl_pre[xs[q] / kNlBlock] + (uint32_t)((packed >> (21 * q)) & 0x1FFFFFu);
}

// Lazy newline counts.  Only the line searches after the locations are
// known (k_lines: findLocation's bytes.Count, scanner.go:482-503; k_find_spans:
// the Match line and the Code lines around it, :484-526) read the per-span
// newline counts, and only inside files that have a location, so the scan
// kernels skip them (a tenth of k_scan_fast's time: 11.95 -> 10.6 ms on
// configs[2]) and these kernels count what those searches can reach:
// k_nl_cands bounds each candidate file's counting (below); k_nl_spans
// (phase 0) counts the file's spans from its first through the span after
// that bound; k_nl_check / k_nl_tail send a file to phase 1 (the rest of its
// spans) when a location ends past the bound or the span after it holds
// fewer than kNlTailMin newlines (a forward search past the last location
// could otherwise jump over uncounted spans).  A span is counted whole,
// neighbouring files' bytes included, exactly as the scan would have, so
// every prefix difference inside a file reads the same counts.  Each wave
// takes 64 consecutive spans, ballots the ones it needs and counts each with
// the whole wave (64 bytes per lane, SWAR).
constexpr uint32_t kNlTailMin = 4;   // newlines of the span after the last location: Code's 2 lines + the end line's
constexpr uint64_t kNlFull = 1ull << 63;  // nl_last flag: count the whole file

// The counting starts before the locations exist: right after the
// candidates (k_expand / k_full_jobs mark each file's reach), on the side
// stream under the candidate sort and k_verify (latency-bound, so the HBM
// is free), each candidate's file is counted through kNlCandReach bytes past
// its last candidate (a full-file rule's: to the file's end).  When the
// locations are known, k_nl_check sends a file whose last location ends past
// that bound to phase 1 (which then also covers what k_nl_tail asks for).
__global__ __launch_bounds__(256) void k_nl_check(const DevLoc* locs, uint64_t n, const uint64_t* off,
                                                  unsigned long long* nl_last) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = locs[i].file;
  const uint64_t l = nl_last[f] & ~kNlFull;
  if (!l || (off[f] + locs[i].end) / kNlBlock > (l - 1) / kNlBlock) atomicOr(&nl_last[f], (unsigned long long)kNlFull);
}

__global__ __launch_bounds__(256) void k_nl_tail(const uint64_t* off, uint32_t n_files, const uint32_t* nl_blocks,
                                                 uint64_t n_spans, unsigned long long* nl_last) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_files || !(nl_last[f] & ~kNlFull) || (nl_last[f] & kNlFull)) return;
  const uint64_t next = ((nl_last[f] & ~kNlFull) - 1) / kNlBlock + 1;  // the span after the counted bound's
  if (next * kNlBlock < off[f + 1] && next < n_spans && nl_blocks[next] < kNlTailMin) nl_last[f] |= kNlFull;
}

__global__ __launch_bounds__(256) void k_nl_spans(const uint8_t* data, uint64_t nbytes, const uint64_t* off,
                                                  const uint32_t* region_file, uint64_t n_regions, uint32_t n_files,
                                                  const unsigned long long* nl_last, uint32_t* nl_blocks,
                                                  uint32_t phase, uint64_t nl_big) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t n_spans = (nbytes + kNlBlock - 1) / kNlBlock;
  const uint64_t n_waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t sp0 = ((uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 64; sp0 < n_spans;
       sp0 += n_waves * 64) {
  const uint64_t sp = sp0 + lane;
  bool need = false;
  if (sp < n_spans && !span_scan_counted(off, region_file, n_regions, n_files, sp, nl_big)) {
    // files overlapping span sp: the one holding its first byte through the
    // one holding the next span's first byte
    const uint32_t f0 = region_file[sp];
    uint32_t f1 = sp + 1 < n_regions ? region_file[sp + 1] : n_files - 1;
    if (f1 >= n_files) f1 = n_files - 1;
    for (uint32_t f = f0; f <= f1 && !need; ++f) {
      const uint64_t l = nl_last[f];
      if (!l || off[f + 1] <= sp * kNlBlock) continue;  // (no location / an empty file before the span)
      // spans counted in phase 0: [first, next]; phase 1 counts the rest of a
      // kNlFull file (all of it when phase 0 counted none)
      const uint64_t lim = l & ~kNlFull;
      const uint64_t next = lim ? (lim - 1) / kNlBlock + 1 : 0;
      need = phase == 0 ? sp <= next : ((l & kNlFull) && (!lim || sp > next));
    }
  }
  // the needed spans four at a time: their 16 KiB of loads are issued
  // before any count, so a wave keeps four spans in flight instead of one
  // (one span per round left the kernel latency-bound: a wave inside a big
  // candidate file walked its 64 spans one load latency each)
  uint64_t m = __ballot(need);
  while (m) {
    uint32_t ks[4];
    uint32_t nk = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ks[t] = m ? (uint32_t)__builtin_ctzll(m) : 64u;
      if (m) {
        m &= m - 1;
        ++nk;
      }
    }
    uint4 v[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t b = (sp0 + ks[t]) * kNlBlock + 64ull * lane;
      const bool full = (uint32_t)t < nk && b + 64 <= nbytes;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[t][q] = full ? *(const uint4*)(data + b + 16 * q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if ((uint32_t)t >= nk) break;
      const uint64_t b = (sp0 + ks[t]) * kNlBlock + 64ull * lane;
      uint32_t cnt = 0;
      if (b + 64 <= nbytes) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          cnt += nl_count_dword(v[t][q].x) + nl_count_dword(v[t][q].y) + nl_count_dword(v[t][q].z) +
                 nl_count_dword(v[t][q].w);
      } else {
        for (uint64_t x = b; x < b + 64 && x < nbytes; ++x) cnt += data[x] == '\n';
      }
      for (uint32_t d = 32; d; d >>= 1) cnt += __shfl_xor(cnt, d);
      if (lane == 0) nl_blocks[sp0 + ks[t]] = cnt;
    }
  }
  }
}

// The newline prefix at each location file's start, once per file: one wave
// per location of the (file, start)-sorted list, the first of each file
// counts (a file with thousands of locations -- minified lines full of rule
// instances -- read its first block once per location before).
__global__ __launch_bounds__(256) void k_file_base(const uint8_t* data, const uint64_t* off, const uint32_t* nl_pre,
                                                   const DevLoc* locs, uint64_t n_locs, uint32_t* fbase) {
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= n_locs) return;
  const uint32_t f = locs[w].file;
  if (w > 0 && locs[w - 1].file == f) return;
  const uint32_t g = wave_nl_prefix(data, nl_pre, off[f], lane);
  if (lane == 0) fbase[f] = g;
}

// One wave per location (sorted by (file, start)): P(start), P(end)
// relative to the file start (k_file_base) on the uncensored content;
// censored_lines() turns them into findLocation's numbers.
__global__ __launch_bounds__(256) void k_lines(const uint8_t* data, const uint64_t* off, const uint32_t* nl_pre,
                                               const uint32_t* fbase, DevLoc* locs, uint64_t n_locs) {
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= n_locs) return;
  const DevLoc L = locs[w];
  if (L.flags) return;
  const uint64_t fs = off[L.file];
  if (L.start > L.end || fs + L.end >= off[L.file + 1]) return;  // never read outside the file
  // both prefixes in one wave pass (a 4 KiB block they share is read once)
  uint32_t g[3];
  wave_nl_prefix3(data, nl_pre, fs + L.start, fs + L.start, fs + L.end, lane, g);
  if (lane == 0) {  // raw prefix counts P(start), P(end); see censored_lines()
    const uint32_t b = fbase[L.file];
    locs[w].start_line = g[1] - b;
    locs[w].end_line = g[2] - b;
  }
}

// ------------------------------------------------------------- findings --
// toFinding / findLocation over the FINAL censored buffer (scanner.go:425-537)
// on the device: the censored buffer is the batch plus, per file, the merged
// kept locations read as '*' (never materialised), so a '\n' inside one is no
// line break.  Per kept location (ordered by (file, start)):
//   k_censor      one lane per file group: merged censor intervals + the
//                 censored StartLine (= EndLine) from k_lines' raw counts
//   k_find_spans  one wave per location: Match window (the line, or 30 / 20
//                 bytes around the secret when the line exceeds 100 bytes)
//                 and up to 5 Code lines (secretHighlightRadius 2), found with
//                 wave-wide 1 KiB newline searches that skip 4 KiB blocks
//                 without '\n' (nl_blocks); byte counts for the arena
//   k_find_copy   one wave per location: the spans into the string arena,
//                 censored bytes written as '*'
// The records are then ordered by (file, RuleID rank) on the device; the host
// only breaks (file, RuleID) ties by Match (scanner.go:441-446).
struct FindParams {
  const uint8_t* data;
  uint64_t data_end;  // bytes of the batch buffer (reads stay below it)
  const uint64_t* off;
  const uint32_t* nl_blocks;
  const uint32_t* nl_pre;  // exclusive prefix of nl_blocks (n_nlb entries): newlines before each 4 KiB block
  uint64_t n_nlb;
  const RuleDev* rules;
  DevLoc* locs;        // sorted by (file, start); lines rewritten by k_censor
  uint64_t n_locs;
  uint64_t* iv;        // merged censor intervals, 2 u64 per slot, at the group's slots
  uint2* grp;          // per location: (first slot of its file group, intervals in it)
  FindRec* rec;
  uint64_t* line_key;  // per code slot: file << kKeyPosBits | line start (~0: unused slot); sorted with slot ids
  uint32_t* line_slot;
  uint32_t* line_head; // per sorted slot: 1 at the first slot of each distinct line, then its inclusive prefix
  uint32_t* line_uid;  // per code slot: index of its distinct line
  // segments of the string arena: [0, n_locs) the Match windows, then one per
  // distinct Code line (a line shared by several findings is stored once)
  uint32_t* seg_file;
  uint2* seg_grp;
  uint64_t* seg_src;
  uint64_t* seg_len;   // then, after the exclusive scan, seg_off
  uint64_t* seg_off;
  uint64_t n_seg_cap;  // n_locs + kCodeLines * n_locs
  // arena granules (kArenaGran bytes): gran_seg[g] = the segment covering
  // byte g * kArenaGran after k_arena_gran_scan, up to the maximum carried in
  // from earlier blocks of 1024 granules (gran_carry)
  uint32_t* gran_seg;
  uint32_t* gran_carry;
  uint64_t n_gran;
  uint8_t* arena;
  uint64_t arena_cap;  // bytes of `arena` (sized before find_bytes is known; a larger need redoes the stage)
  uint64_t* sort_key;
  uint32_t* sort_idx;
  uint32_t rank_bits;  // bits of RuleDev::id_rank: sort key = file << rank_bits | rank
  Ctrl* ctrl;
  const uint64_t* dense_at;  // per location: its file's offset in the dense region, ~0 (sparse); may be null
  const uint32_t* slot_base; // with dense_at: per sparse location its index among them (its line keys' place)
  uint32_t* long_list;       // k_find_spans_lane -> k_find_spans: the locations left to the wave search (may be null)
};

// Wave-wide scans (inclusive) over the 64 lanes.
__device__ inline uint64_t wave_incl_max64(uint64_t v, uint32_t lane) {
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d);
    if (lane >= d) v = v > o ? v : o;
  }
  return v;
}

// One wave per file group (the wave of the group's first location; the rest
// exit), 64 locations per step with carries: (1) merged censor intervals --
// a location opens one when it starts past the running maximum end, the
// interval's end is that running maximum (packed end << 32 | P(end), so the
// raw newline count travels with it); (2) the exclusive prefix of censored
// newlines per interval, P(b) - P(a); (3) each location's censored line:
// P(a) of its interval minus the newlines censored before it, + 1 (every
// location of one interval shares it; EndLine == StartLine).  Scratch:
// sort_key / sort_idx hold P(a) / P(b) per interval slot, line_uid the
// location's interval, line_head the prefix (all reused later).
// Files with kCensorBig or more locations (a minified line full of rule
// instances) are merged by k_censor_big, a 1024-lane block per file, instead:
// one wave would walk them 64 locations at a time.
constexpr uint32_t kCensorBig = 4096;

__device__ inline bool censor_big_group(const FindParams& F, uint64_t i) {
  return i + kCensorBig - 1 < F.n_locs && F.locs[i + kCensorBig - 1].file == F.locs[i].file;
}

__global__ __launch_bounds__(256) void k_censor(FindParams F) {
  const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (i >= F.n_locs || (i > 0 && F.locs[i - 1].file == F.locs[i].file)) return;  // wave-uniform
  if (censor_big_group(F, i)) return;  // k_censor_big's
  const uint32_t file = F.locs[i].file;
  uint64_t j = i + 1;  // group end: wave-wide probe 64 at a time
  for (;;) {
    const uint64_t k = j + lane;
    const bool same = k < F.n_locs && F.locs[k].file == file;
    const uint64_t m = __ballot(!same);
    if (m) {
      j += __builtin_ctzll(m);
      break;
    }
    j += 64;
  }
  const uint64_t lanes_lt = (1ull << lane) - 1;
  // running max of end and of P(end) over the file's valid locations so far
  // (P is monotone in the position, so the two maxima belong together)
  uint64_t carry = 0, carry_p = 0;
  uint32_t m_cnt = 0;  // intervals opened so far
  bool have = false;
  for (uint64_t k0 = i; k0 < j; k0 += 64) {
    const uint64_t k = k0 + lane;
    DevLoc L{};
    if (k < j) L = F.locs[k];
    const bool valid = k < j && !L.flags;
    uint64_t incl = wave_incl_max64(valid ? L.end : 0, lane);
    uint64_t incl_p = wave_incl_max64(valid ? (uint64_t)L.end_line : 0, lane);
    incl_p = incl_p > carry_p ? incl_p : carry_p;
    uint64_t excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0;
    excl = excl > carry ? excl : carry;
    incl = incl > carry ? incl : carry;
    const uint64_t vmask = __ballot(valid);
    const bool before = have || (vmask & lanes_lt) != 0;
    const bool opens = valid && (!before || L.start > excl);
    const uint64_t omask = __ballot(opens);
    const uint32_t id = m_cnt + (uint32_t)__popcll(omask & (lanes_lt | (1ull << lane))) - 1;
    if (valid) {
      F.line_uid[k] = id;
      if (opens) {
        F.iv[2 * (i + id)] = L.start;
        F.sort_key[i + id] = L.start_line;  // P(a)
      }
      // last valid location of its interval in this step: write the interval's end
      const uint64_t later = vmask & ~(lanes_lt | (1ull << lane));
      const bool last = !later || ((omask >> __builtin_ctzll(later)) & 1);
      if (last) {
        F.iv[2 * (i + id) + 1] = incl;
        F.sort_idx[i + id] = (uint32_t)incl_p;  // P(b)
      }
    }
    carry = __shfl(incl, 63);
    carry_p = __shfl(incl_p, 63);
    m_cnt += (uint32_t)__popcll(omask);
    have = have || vmask != 0;
  }
  // exclusive prefix of censored newlines over the intervals
  uint32_t run = 0;
  for (uint32_t q0 = 0; q0 < m_cnt; q0 += 64) {
    const uint32_t q = q0 + lane;
    const uint32_t d = q < m_cnt ? F.sort_idx[i + q] - (uint32_t)F.sort_key[i + q] : 0u;
    const uint32_t inc = wave_incl_sum32(d, lane);
    if (q < m_cnt) F.line_head[i + q] = run + inc - d;
    run += __shfl(inc, 63);
  }
  for (uint64_t k = i + lane; k < j; k += 64) {
    F.grp[k] = make_uint2((uint32_t)i, m_cnt);
    DevLoc& L = F.locs[k];
    if (L.flags) continue;
    const uint32_t id = F.line_uid[k];
    const uint32_t line = (uint32_t)F.sort_key[i + id] - F.line_head[i + id] + 1;
    L.start_line = line;
    L.end_line = line;
  }
}

// Block-wide inclusive scans over 1024 lanes (16 waves): wave scans, then
// the wave totals through LDS.  `tot` receives the block total.
__device__ inline uint64_t block_incl_max64(uint64_t v, uint64_t* lds16, uint64_t* tot) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_incl_max64(v, lane);
  if (lane == 63) lds16[wv] = v;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
    const uint64_t x = lds16[k];
    if (k < wv) before = before > x ? before : x;
    all = all > x ? all : x;
  }
  __syncthreads();
  *tot = all;
  return v > before ? v : before;
}

// k_censor for one file group of >= kCensorBig locations per 1024-lane block
// (block b takes the big group whose first location lies in [b, b + 1) x
// kCensorBig: two big groups cannot start that close).  Same results as
// k_censor; an interval's end is the running maximum just before the location
// that opens the next one (the maxima are monotone), the last one's the final
// maximum.
__global__ __launch_bounds__(1024) void k_censor_big(FindParams F) {
  __shared__ uint64_t s64[16], s64b[16];
  __shared__ uint32_t s32[16];
  __shared__ unsigned long long first;
  __shared__ unsigned long long gend;
  __shared__ uint64_t prev_incl[1024], prev_incl_p[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t w0 = (uint64_t)blockIdx.x * kCensorBig;
  if (t == 0) {
    first = ~0ull;
    gend = ~0ull;
  }
  __syncthreads();
  for (uint64_t k = w0 + t; k < w0 + kCensorBig && k < F.n_locs; k += blockDim.x)
    if ((k == 0 || F.locs[k - 1].file != F.locs[k].file) && censor_big_group(F, k)) atomicMin(&first, k);
  __syncthreads();
  if (first == ~0ull) return;  // block-uniform
  const uint64_t i = first;
  const uint32_t file = F.locs[i].file;
  for (uint64_t j0 = i + kCensorBig;; j0 += blockDim.x) {  // group end
    const uint64_t k = j0 + t;
    if (k >= F.n_locs || F.locs[k].file != file) atomicMin(&gend, k);
    __syncthreads();
    if (gend != ~0ull) break;
    __syncthreads();
  }
  const uint64_t j = gend;
  uint64_t carry = 0, carry_p = 0;
  uint32_t m_cnt = 0, n_valid = 0;
  for (uint64_t k0 = i; k0 < j; k0 += blockDim.x) {
    const uint64_t k = k0 + t;
    DevLoc L{};
    if (k < j) L = F.locs[k];
    const bool valid = k < j && !L.flags;
    uint64_t tot, tot_p;
    uint64_t incl = block_incl_max64(valid ? L.end : 0, s64, &tot);
    uint64_t incl_p = block_incl_max64(valid ? (uint64_t)L.end_line : 0, s64b, &tot_p);
    incl = incl > carry ? incl : carry;
    incl_p = incl_p > carry_p ? incl_p : carry_p;
    prev_incl[t] = incl;
    prev_incl_p[t] = incl_p;
    uint32_t vtot;
    const uint32_t vincl = block_incl_sum32(valid ? 1u : 0u, s32, &vtot);
    // (block_incl_sum32's barriers order the prev_incl writes before these reads)
    const uint64_t excl = t ? prev_incl[t - 1] : carry;
    const uint64_t excl_p = t ? prev_incl_p[t - 1] : carry_p;
    const bool before = n_valid + vincl - (valid ? 1u : 0u) > 0;
    const bool opens = valid && (!before || L.start > excl);
    uint32_t otot;
    const uint32_t oincl = block_incl_sum32(opens ? 1u : 0u, s32, &otot);
    const uint32_t id = m_cnt + oincl - 1;  // (valid locations only)
    if (valid) {
      F.line_uid[k] = id;
      if (opens) {
        F.iv[2 * (i + id)] = L.start;
        F.sort_key[i + id] = L.start_line;  // P(a)
        if (id > 0) {  // the previous interval ends at the running maximum before this one
          F.iv[2 * (i + id - 1) + 1] = excl;
          F.sort_idx[i + id - 1] = (uint32_t)excl_p;  // P(b)
        }
      }
    }
    carry = carry > tot ? carry : tot;
    carry_p = carry_p > tot_p ? carry_p : tot_p;
    m_cnt += otot;
    n_valid += vtot;
    __syncthreads();  // prev_incl reused by the next step
  }
  if (t == 0 && m_cnt) {
    F.iv[2 * (i + m_cnt - 1) + 1] = carry;
    F.sort_idx[i + m_cnt - 1] = (uint32_t)carry_p;
  }
  __threadfence_block();
  __syncthreads();
  // exclusive prefix of censored newlines over the intervals
  uint32_t run = 0;
  for (uint32_t q0 = 0; q0 < m_cnt; q0 += blockDim.x) {
    const uint32_t q = q0 + t;
    const uint32_t d = q < m_cnt ? F.sort_idx[i + q] - (uint32_t)F.sort_key[i + q] : 0u;
    uint32_t tot;
    const uint32_t inc = block_incl_sum32(d, s32, &tot);
    if (q < m_cnt) F.line_head[i + q] = run + inc - d;
    run += tot;
  }
  __threadfence_block();
  __syncthreads();
  for (uint64_t k = i + t; k < j; k += blockDim.x) {
    F.grp[k] = make_uint2((uint32_t)i, m_cnt);
    DevLoc& L = F.locs[k];
    if (L.flags) continue;
    const uint32_t id = F.line_uid[k];
    const uint32_t line = (uint32_t)F.sort_key[i + id] - F.line_head[i + id] + 1;
    L.start_line = line;
    L.end_line = line;
  }
}


// The censor interval holding file-relative byte x, or -1, for x near
// interval h of the group (relative): a galloping search out from h, then a binary search of the bracket -- the
// line breaks k_find_spans looks up lie a few lines from the location, whose
// own interval is h, so a file with thousands of intervals costs ~2 loads a
// lookup instead of a full-depth binary search.
__device__ inline int64_t censor_holder_near(const uint64_t* iv, uint32_t g0, uint32_t m, uint64_t x, uint32_t h) {
  if (m == 0) return -1;
  if (h >= m) h = m - 1;
  uint32_t lo, hi;  // the first interval with a > x lies in [lo, hi]
  if (iv[2 * (g0 + h)] <= x) {
    lo = h + 1;
    hi = m;
    for (uint32_t d = 1;; d <<= 1) {
      const uint32_t t = lo - 1 + d;
      if (t >= m) break;
      if (iv[2 * (g0 + t)] > x) {
        hi = t;
        break;
      }
      lo = t + 1;
    }
  } else {
    lo = 0;
    hi = h;
    for (uint32_t d = 1; hi >= d; d <<= 1) {
      const uint32_t t = hi - d;
      if (iv[2 * (g0 + t)] <= x) {
        lo = t + 1;
        break;
      }
      hi = t;
    }
  }
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (iv[2 * (g0 + mid)] <= x) lo = mid + 1;
    else hi = mid;
  }
  if (lo == 0) return -1;
  return x < iv[2 * (g0 + lo - 1) + 1] ? (int64_t)(g0 + lo - 1) : -1;
}

// 16 bytes at p (zero past `end`): whole-vector load when it fits the buffer.
__device__ inline uint4 ld16_guard(const uint8_t* data, uint64_t p, uint64_t end) {
  if (p + 16 <= end) return *(const uint4*)(data + p);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k)  // (unrolled: constant indices, no scratch)
    if (p + k < end) w[k >> 2] |= (uint32_t)data[p + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Block holding newline number k (0-based, whole batch): the largest b with
// nl_pre[b] <= k (binary search over the prefix; wave-uniform).
__device__ inline uint64_t nl_block_of(const FindParams& F, uint64_t k) {
  uint64_t lo = 0, hi = F.n_nlb;  // nl_pre[lo] <= k < nl_pre[hi] (hi may be past the end)
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (F.nl_pre[mid] <= k) lo = mid;
    else hi = mid;
  }
  return lo;
}

// First raw '\n' in [A, B) within one 4 KiB block, or B: 1 KiB per wave step.
__device__ uint64_t wave_nl_fwd_blk(const FindParams& F, uint64_t A, uint64_t E, uint32_t lane) {
  while (A < E) {
    const uint64_t base = A & ~(uint64_t)15;
    const uint64_t p = base + 16ull * lane;
    uint32_t m = p < E ? nl_mask16(ld16_guard(F.data, p, F.data_end)) : 0u;
    if (p < A) m &= ~0u << (uint32_t)(A - p);
    if (p + 16 > E) m &= (E > p) ? ((1u << (uint32_t)(E - p)) - 1u) : 0u;
    const uint64_t hit = __ballot(m != 0);
    if (hit) {
      const uint32_t l = (uint32_t)__builtin_ctzll(hit);
      const uint32_t ml = __shfl(m, l);
      return base + 16ull * l + (uint32_t)__builtin_ctz(ml);
    }
    A = base + 1024;
  }
  return E;
}

// Last raw '\n' in [S, B), or -1: 1 KiB per wave step, backwards.
__device__ int64_t wave_nl_bwd_blk(const FindParams& F, uint64_t S, uint64_t B, uint32_t lane) {
  while (B > S) {
    const uint64_t top = ((B - 1) & ~(uint64_t)15) + 16;  // chunk [top - 1024, top)
    const int64_t base = (int64_t)top - 1024;
    const int64_t p = base + 16ll * lane;
    uint32_t m = 0;  // (p is 16-aligned: a lane with p < 0 lies wholly before S)
    if (p >= 0 && p + 16 > (int64_t)S) {
      m = nl_mask16(ld16_guard(F.data, (uint64_t)p, F.data_end));
      if (p < (int64_t)S) m &= ~0u << (uint32_t)((int64_t)S - p);
    }
    if (p + 16 > (int64_t)B) m &= (int64_t)B > p ? ((1u << (uint32_t)((int64_t)B - p)) - 1u) : 0u;
    const uint64_t hit = __ballot(m != 0);
    if (hit) {
      const uint32_t l = 63u - (uint32_t)__builtin_clzll(hit);
      const uint32_t ml = __shfl(m, l);
      return base + 16ll * l + (31 - __builtin_clz(ml));
    }
    B = base > (int64_t)S ? (uint64_t)base : S;
  }
  return -1;
}

// First raw '\n' in [A, E) (absolute), or E: the rest of A's 4 KiB block,
// then the block of the next newline by its number (O(log n) however long
// the line: minified files hold multi-MiB lines).
__device__ uint64_t wave_nl_fwd(const FindParams& F, uint64_t A, uint64_t E, uint32_t lane) {
  if (A >= E) return E;
  const uint64_t blk = A / kNlBlock;
  const uint64_t bend = (blk + 1) * kNlBlock;
  if (F.nl_blocks[blk]) {
    const uint64_t i = wave_nl_fwd_blk(F, A, bend < E ? bend : E, lane);
    if (i < (bend < E ? bend : E)) return i;
  }
  if (bend >= E || blk + 1 >= F.n_nlb) return E;
  const uint64_t b = nl_block_of(F, F.nl_pre[blk + 1]);  // block of the next newline after blk
  if (b * kNlBlock >= E || b >= F.n_nlb - 1 || F.nl_pre[b + 1] == F.nl_pre[b]) return E;
  return wave_nl_fwd_blk(F, b * kNlBlock, (b + 1) * kNlBlock < E ? (b + 1) * kNlBlock : E, lane);
}

// Last raw '\n' in [S, B) (absolute), or -1 (same two steps backwards).
__device__ int64_t wave_nl_bwd(const FindParams& F, uint64_t S, uint64_t B, uint32_t lane) {
  if (B <= S) return -1;
  const uint64_t blk = (B - 1) / kNlBlock;
  const uint64_t b0 = blk * kNlBlock;
  if (F.nl_blocks[blk]) {
    const int64_t i = wave_nl_bwd_blk(F, b0 > S ? b0 : S, B, lane);
    if (i >= 0) return i;
  }
  if (b0 <= S || F.nl_pre[blk] == 0) return -1;
  const uint64_t b = nl_block_of(F, F.nl_pre[blk] - 1);  // block of the last newline before blk
  const uint64_t e = (b + 1) * kNlBlock;
  if (e <= S) return -1;
  return wave_nl_bwd_blk(F, b * kNlBlock > S ? b * kNlBlock : S, e, lane);
}

// Censored-buffer line breaks of file [fs, fs + n) with intervals (g0, m):
// first '\n' at or after `from` (n if none) / start of the line holding pos.
__device__ uint64_t cens_next_nl(const FindParams& F, uint64_t fs, uint64_t n, uint32_t g0, uint32_t m, uint32_t h,
                                 uint64_t from, uint32_t lane) {
  while (from < n) {
    const uint64_t i = wave_nl_fwd(F, fs + from, fs + n, lane) - fs;
    if (i >= n) return n;
    const int64_t hold = censor_holder_near(F.iv, g0, m, i, h);
    if (hold < 0) return i;
    from = F.iv[2 * hold + 1];
  }
  return n;
}

__device__ uint64_t cens_line_begin(const FindParams& F, uint64_t fs, uint32_t g0, uint32_t m, uint32_t h, uint64_t pos,
                                    uint32_t lane) {
  while (pos) {
    const int64_t a = wave_nl_bwd(F, fs, fs + pos, lane);
    if (a < 0) return 0;
    const uint64_t i = (uint64_t)a - fs;
    const int64_t hold = censor_holder_near(F.iv, g0, m, i, h);
    if (hold < 0) return i + 1;
    pos = F.iv[2 * hold];
  }
  return 0;
}

// Dense files: a file with at most kDenseBytesPerLoc bytes per kept location
// (configs[4]'s stress files: a rule instance every ~4 lines, so the 4-line
// Code windows cover every line) goes into the arena WHOLE, censored, in a
// region of its own: its Code lines and Match windows are offsets into it
// (kArenaDense), no per-line segments.  The region is known once k_censor has
// merged the intervals, so it is filled and copied back on the side stream
// under k_find_spans and the rest of the findings stage, instead of after the
// arena fill (the results' ~200 MB of D2H were configs[4]'s critical path).
constexpr uint64_t kDenseBytesPerLoc = 384;
constexpr uint32_t kDenseLaneBytes = 256;  // k_dense_fill: bytes per lane step (one group search each)

__global__ void k_dense_heads(FindParams F, uint32_t* head) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < F.n_locs) head[w] = (w == 0 || F.locs[w].file != F.locs[w - 1].file) ? 1u : 0u;
}
// gid: inclusive prefix of the heads (1-based group of each location)
__global__ void k_dense_groups(FindParams F, const uint32_t* gid, uint32_t* gstart) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < F.n_locs && (w == 0 || gid[w] != gid[w - 1])) gstart[gid[w] - 1] = (uint32_t)w;
}
__global__ void k_dense_size(FindParams F, const uint32_t* gid, const uint32_t* gstart, uint64_t* dsize) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t G = gid[F.n_locs - 1];
  if (g >= G) return;  // (the rest stay 0: memset)
  const uint64_t s0 = gstart[g], s1 = g + 1 < G ? gstart[g + 1] : F.n_locs;
  const uint32_t file = F.locs[s0].file;
  const uint64_t bytes = F.off[file + 1] - 1 - F.off[file];
  dsize[g] = bytes && bytes <= kDenseBytesPerLoc * (s1 - s0) ? (bytes + 15) & ~15ull : 0;  // (16-byte aligned files)
}
__global__ void k_dense_at(FindParams F, const uint32_t* gid, const uint64_t* dsize, const uint64_t* doff,
                           uint64_t* dense_at) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= F.n_locs) return;
  const uint32_t g = gid[w] - 1;
  dense_at[w] = dsize[g] ? doff[g] : ~0ull;
  if (w == 0) {
    F.ctrl->dense_bytes = doff[F.n_locs - 1] + dsize[F.n_locs - 1];
    F.ctrl->dense_groups = gid[F.n_locs - 1];
  }
}

// Locations outside dense files: flags for their exclusive prefix (their
// Code slots' keys are packed at 4 x that index, so the distinct-line sort
// takes only theirs), and the total.
__global__ void k_dense_sparse_flags(FindParams F, const uint64_t* dense_at, uint32_t* flag) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < F.n_locs) flag[w] = dense_at[w] == ~0ull ? 1u : 0u;
}
__global__ void k_dense_sparse_total(FindParams F, const uint32_t* flag, const uint32_t* idx) {
  if (blockIdx.x == 0 && threadIdx.x == 0) F.ctrl->sparse_locs = (uint64_t)idx[F.n_locs - 1] + flag[F.n_locs - 1];
}

// Per location: file << 40 | its end (0 for a location k_censor skips); an
// inclusive max-scan makes it the running maximum end within the file (files
// ascend in the high bits), i.e. the censored bytes' union up to it.
constexpr uint32_t kPmaxShift = 40;
__global__ void k_dense_pmax_keys(FindParams F, uint64_t* keys) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= F.n_locs) return;
  const DevLoc& L = F.locs[w];
  keys[w] = ((uint64_t)L.file << kPmaxShift) | (L.flags ? 0ull : L.end);
}

// The dense region: kDenseLaneBytes per lane step, the file group by binary
// search over the G group offsets, 16 bytes at a time.  A byte is censored
// ('*') iff some valid location [start, end) of its file holds it -- the
// union k_censor merges (censorLocation, scanner.go:454-462): the running
// maximum end of the locations starting at or before the chunk (pmax) and
// the locations starting inside it.  Needs only the sorted locations, so it
// runs before k_lines / k_censor.
__global__ __launch_bounds__(256) void k_dense_fill(FindParams F, const uint32_t* gstart, const uint64_t* dsize,
                                                    const uint64_t* doff, const uint64_t* pmax, uint32_t G,
                                                    uint64_t total, uint8_t* out) {
  constexpr uint64_t kEndMask = (1ull << kPmaxShift) - 1;
  for (uint64_t a0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kDenseLaneBytes; a0 < total;
       a0 += (uint64_t)gridDim.x * blockDim.x * kDenseLaneBytes) {
    uint32_t lo = 0, hi = G;  // the last group with doff <= a0 (non-empty: it holds byte a0)
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (doff[mid] <= a0) lo = mid;
      else hi = mid;
    }
    uint32_t g = lo;
    uint64_t gend = 0, fbase = 0, x0 = 0, s0 = 0, s1 = 0, k = 0;
    bool fresh = true;
    for (uint64_t a = a0; a < a0 + kDenseLaneBytes && a < total; a += 16) {
      if (!fresh && a >= gend) {
        do ++g;
        while (g < G && doff[g] + dsize[g] <= a);
        fresh = true;
      }
      const uint64_t x = a - (fresh ? doff[g] : x0);  // file-relative
      if (fresh) {
        fresh = false;
        gend = doff[g] + dsize[g];
        x0 = doff[g];
        s0 = gstart[g];
        s1 = g + 1 < G ? gstart[g + 1] : F.n_locs;
        fbase = F.off[F.locs[s0].file];
        uint64_t l2 = s0, h2 = s1;  // k = the first location starting after x
        while (l2 < h2) {
          const uint64_t mid = (l2 + h2) >> 1;
          if (F.locs[mid].start <= x) l2 = mid + 1;
          else h2 = mid;
        }
        k = l2;
      }
      while (k < s1 && F.locs[k].start <= x) ++k;
      // bytes before the running maximum end of the locations starting <= x
      const uint64_t cover = k > s0 ? (pmax[k - 1] & kEndMask) : 0;
      uint32_t cmask = cover > x ? (cover >= x + 16 ? 0xFFFFu : (1u << (uint32_t)(cover - x)) - 1u) : 0u;
      for (uint64_t j = k; j < s1; ++j) {  // the locations starting inside the chunk
        const DevLoc& L = F.locs[j];
        if (L.start >= x + 16) break;
        if (L.flags || L.end <= L.start) continue;
        const uint32_t b = (uint32_t)(L.start - x), e2 = L.end < x + 16 ? (uint32_t)(L.end - x) : 16u;
        cmask |= ((1u << (e2 - b)) - 1u) << b;
      }
      const uint64_t src = fbase + x;
      const uint64_t b0 = src & ~15ull;
      const uint32_t sh = (uint32_t)(src - b0);
      const uint4 u = ld16_guard(F.data, b0, F.data_end);
      uint32_t r[4] = {u.x, u.y, u.z, u.w};
      if (sh) {
        const uint4 v = ld16_guard(F.data, b0 + 16, F.data_end);
        const uint32_t d[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        const uint32_t q = sh >> 2, bs = 8 * (sh & 3);
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          const uint32_t lo32 = q == 0 ? d[z] : q == 1 ? d[z + 1] : q == 2 ? d[z + 2] : d[z + 3];
          const uint32_t hi32 = q == 0 ? d[z + 1] : q == 1 ? d[z + 2] : q == 2 ? d[z + 3] : d[z + 4];
          r[z] = bs ? (lo32 >> bs) | (hi32 << (32 - bs)) : lo32;
        }
      }
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const uint32_t m4 = (cmask >> (4 * z)) & 0xFu;
        const uint32_t bm = ((m4 & 1u) ? 0xFFu : 0u) | ((m4 & 2u) ? 0xFF00u : 0u) | ((m4 & 4u) ? 0xFF0000u : 0u) |
                            ((m4 & 8u) ? 0xFF000000u : 0u);
        r[z] = (r[z] & ~bm) | (0x2A2A2A2Au & bm);  // '*'
      }
      *(uint4*)(out + a) = make_uint4(r[0], r[1], r[2], r[3]);
    }
  }
}

constexpr uint64_t kMatchInLine = 1ull << 63, kMatchInLineOff = (1ull << 48) - 1;  // FindRec::m_off before k_find_finalize

// The Match window and Code line spans of location w (one wave, or one
// lane, per location: `Srch` supplies the censored-buffer line searches).
// Returns false when the searcher gave up (a lane's window): nothing written.
template <class Srch>
__device__ __forceinline__ bool find_spans_one(const FindParams& F, uint64_t w, bool writer, Srch& srch) {
  const DevLoc L = F.locs[w];
  FindRec r{};
  r.file = L.file;
  r.loc = (uint32_t)w;
  const uint64_t fs = F.off[L.file];
  const uint64_t n = F.off[L.file + 1] - 1 - fs;
  const uint64_t dz = F.dense_at ? F.dense_at[w] : ~0ull;  // the file's place in the dense region
  // where this location's line keys go: its slots, or packed among the sparse locations'
  const uint64_t kb = F.dense_at ? (uint64_t)F.slot_base[w] * kCodeLines : w * kCodeLines;
  uint64_t m_src = 0;  // the Match window's file-relative start
  uint64_t keys[kCodeLines] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (!L.flags && L.start <= L.end && L.end <= n) {
    const uint2 g = F.grp[w];
    srch.begin(fs, n, g.x, g.y, F.line_uid[w], L.start, L.end);  // (line_uid: the location's own interval, k_censor)
    // match window (scanner.go:484-502)
    // the (censored) line holding the start: the Match window's and the first
    // cause Code line's bounds, searched once (a search on a multi-MiB line
    // costs a binary search over the newline prefix)
    const uint64_t ls0 = srch.line_begin(L.start);
    const uint64_t le0 = srch.next_nl(L.start);
    uint64_t ls = ls0, le = le0;
    if (le - ls > 100) {
      ls = L.start >= 30 ? L.start - 30 : 0;
      le = L.end + 20 > n ? n : L.end + 20;
    }
    m_src = ls;
    r.m_len = (uint32_t)(le - ls);
    // code lines (scanner.go:505-534), 0-based numbers [sl - 2, el + 2)
    const uint32_t sl = L.start_line - 1, el = L.end_line - 1;
    const uint32_t cs = sl >= 2 ? sl - 2 : 0, ce = el + 2;
    uint64_t p = ls0;
    for (uint32_t cur = sl; cur > cs && p > 0; --cur) p = srch.line_begin(p - 1);
    uint32_t nk = 0, kc = kCodeLines;  // kc: the Code slot of the line [ls0, le0)
#pragma unroll
    for (uint32_t k = 0; k < kCodeLines; ++k) {  // (unrolled: c_len stays in registers)
      if (cs + k >= ce || p > n) break;
      if (p == ls0) kc = k;
      const uint64_t q = p == ls0 ? le0 : srch.next_nl(p);
      r.c_len[k] = (uint32_t)(q - p);
      if (k == 0 && dz != ~0ull) r.c_off = kArenaDense | (dz + p);  // (final: no line segments)
      keys[k] = ((uint64_t)L.file << kKeyPosBits) | p;
      p = q + 1;
      nk = k + 1;
    }
    if (srch.failed()) return false;
    r.n_lines = nk;
    r.line = L.start_line;
    // a Match window inside the line holding the start (always when that
    // line is <= 100 bytes: then it IS the line) is that Code line's text:
    // no segment of its own, k_find_finalize points it into the line's
    // (configs[4]: most Match bytes, all of them PCIe D2H)
    if (dz != ~0ull) r.m_off = kArenaDense | (dz + ls);
    else if (kc < kCodeLines && ls >= ls0 && le <= le0) r.m_off = kMatchInLine | ((uint64_t)kc << 48) | (ls - ls0);
  }
  if (writer) {
    F.rec[w] = r;
    if (dz == ~0ull) {  // (a dense file's lines are offsets into its region: no keys)
#pragma unroll
      for (uint32_t k = 0; k < kCodeLines; ++k) {
        F.line_key[kb + k] = k < r.n_lines ? keys[k] : ~0ull;
        F.line_slot[kb + k] = (uint32_t)(w * kCodeLines + k);
      }
    }
    F.seg_file[w] = r.file;
    F.seg_grp[w] = F.grp[w];
    F.seg_src[w] = m_src;
    F.seg_len[w] = (r.m_off & (kMatchInLine | kArenaDense)) ? 0 : r.m_len;
  }
  return true;
}

// The wave's searches: 1 KiB per wave step, 4 KiB blocks without '\n'
// skipped by the newline prefix (any line length).
struct WaveSrch {
  const FindParams& F;
  uint32_t lane;
  uint64_t fs = 0, n = 0;
  uint32_t g0 = 0, gm = 0, h = 0;
  __device__ WaveSrch(const FindParams& f, uint32_t l) : F(f), lane(l) {}
  __device__ void begin(uint64_t fs_, uint64_t n_, uint32_t g0_, uint32_t gm_, uint32_t h_, uint64_t, uint64_t) {
    fs = fs_, n = n_, g0 = g0_, gm = gm_, h = h_;
  }
  __device__ __forceinline__ uint64_t line_begin(uint64_t pos) { return cens_line_begin(F, fs, g0, gm, h, pos, lane); }
  __device__ __forceinline__ uint64_t next_nl(uint64_t from) { return cens_next_nl(F, fs, n, g0, gm, h, from, lane); }
  __device__ bool failed() const { return false; }
};

// One lane's searches, 16 bytes per load, inside a window of kLaneSpanWin
// bytes either side of the location (the file's ends count as found); a
// search that would leave the window fails the location, which then goes to
// the wave search (k_find_spans over long_list).
constexpr uint64_t kLaneSpanWin = 512;
struct LaneSrch {
  const FindParams& F;
  uint64_t fs = 0, n = 0, lo = 0, hi = 0;
  uint32_t g0 = 0, gm = 0, h = 0;
  bool bad = false;
  __device__ explicit LaneSrch(const FindParams& f) : F(f) {}
  __device__ void begin(uint64_t fs_, uint64_t n_, uint32_t g0_, uint32_t gm_, uint32_t h_, uint64_t start,
                        uint64_t end) {
    fs = fs_, n = n_, g0 = g0_, gm = gm_, h = h_;
    lo = start > kLaneSpanWin ? start - kLaneSpanWin : 0;
    hi = end + kLaneSpanWin < n ? end + kLaneSpanWin : n;
  }
  // last raw '\n' in [lo, b) (file-relative), or -1
  __device__ int64_t raw_bwd(uint64_t b) {
    while (b > lo) {
      const uint64_t a0 = (fs + b - 1) & ~15ull;  // the 16-byte chunk holding byte b - 1
      uint32_t m = nl_mask16(ld16_guard(F.data, a0, F.data_end));
      const uint64_t first = a0 - fs;  // (may lie before lo or the file: masked below)
      const uint32_t top = (uint32_t)(fs + b - a0);  // bytes of the chunk before b
      m &= top >= 16 ? 0xFFFFu : ((1u << top) - 1u);
      if (a0 < fs + lo) m &= ~0u << (uint32_t)(fs + lo - a0);
      if (m) return (int64_t)(first + (31 - __builtin_clz(m)));
      b = a0 > fs + lo ? a0 - fs : lo;
    }
    return -1;
  }
  // first raw '\n' in [a, hi), or hi
  __device__ uint64_t raw_fwd(uint64_t a) {
    while (a < hi) {
      const uint64_t a0 = (fs + a) & ~15ull;
      uint32_t m = nl_mask16(ld16_guard(F.data, a0, F.data_end));
      m &= ~0u << (uint32_t)(fs + a - a0);
      const uint64_t end = fs + hi;
      if (a0 + 16 > end) m &= end > a0 ? ((1u << (uint32_t)(end - a0)) - 1u) : 0u;
      if (m) return a0 - fs + __builtin_ctz(m);
      a = a0 + 16 - fs;
    }
    return hi;
  }
  __device__ uint64_t line_begin(uint64_t pos) {  // cens_line_begin within [lo, ...)
    while (pos) {
      const int64_t i = raw_bwd(pos);
      if (i < 0) {
        if (lo > 0) bad = true;  // (the window ends before the file does)
        return 0;
      }
      const int64_t hold = censor_holder_near(F.iv, g0, gm, (uint64_t)i, h);
      if (hold < 0) return (uint64_t)i + 1;
      pos = F.iv[2 * hold];
    }
    return 0;
  }
  __device__ uint64_t next_nl(uint64_t from) {  // cens_next_nl within [..., hi)
    while (from < n) {
      const uint64_t i = raw_fwd(from);
      if (i >= hi) {
        if (hi < n) bad = true;
        return n;
      }
      const int64_t hold = censor_holder_near(F.iv, g0, gm, i, h);
      if (hold < 0) return i;
      from = F.iv[2 * hold + 1];
    }
    return n;
  }
  __device__ bool failed() const { return bad; }
};

// One lane per location; a location whose lines run past the lane's window
// is listed for the wave search.
__global__ __launch_bounds__(256) void k_find_spans_lane(FindParams F) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool go_long = false;
  if (w < F.n_locs) {
    // a location inside a 4 KiB block without newlines (a minified line) goes
    // straight to the wave search (a stale count only sends it there early)
    const DevLoc& L = F.locs[w];
    const uint64_t blk = (F.off[L.file] + L.start) / kNlBlock;
    LaneSrch srch(F);
    go_long = (blk < F.n_nlb && F.nl_blocks[blk] == 0) || !find_spans_one(F, w, true, srch);
  }
  // one list reservation per wave
  const uint64_t b = __ballot(go_long);
  if (b) {
    const uint32_t lead = (uint32_t)__builtin_ctzll(b);
    unsigned long long base = 0;
    if (__lane_id() == lead) base = atomicAdd(&F.ctrl->n_long_spans, (unsigned long long)__popcll(b));
    base = __shfl(base, lead);
    if (go_long) F.long_list[base + __popcll(b & ((1ull << __lane_id()) - 1))] = (uint32_t)w;
  }
}

// One wave per location: every location (long_list null), or those
// k_find_spans_lane listed (the count read on the device; a fixed grid).
__global__ __launch_bounds__(256) void k_find_spans(FindParams F) {
  const uint64_t wv = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (!F.long_list) {
    if (wv >= F.n_locs) return;
    WaveSrch srch(F, lane);
    (void)find_spans_one(F, wv, lane == 0, srch);
    return;
  }
  const uint64_t n_long = F.ctrl->n_long_spans;
  const uint64_t n_waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t i = wv; i < n_long; i += n_waves) {
    WaveSrch srch(F, lane);
    (void)find_spans_one(F, F.long_list[i], lane == 0, srch);
  }
}

// Distinct Code lines: the code slots sorted by (file, line start); the first
// slot of each run is a head (line_head), its inclusive prefix numbers them.
__global__ void k_line_heads(const uint64_t* keys, uint64_t n, uint32_t* head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = keys[i] != ~0ull && (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_line_map(FindParams F, const uint64_t* keys, const uint32_t* slots, const uint32_t* scan,
                           const uint32_t* head, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || keys[i] == ~0ull) return;
  const uint32_t slot = slots[i], uid = scan[i] - 1;
  F.line_uid[slot] = uid;
  if (head[i]) {
    const uint64_t sg = F.n_locs + uid;
    F.seg_file[sg] = (uint32_t)(keys[i] >> kKeyPosBits);
    F.seg_src[sg] = keys[i] & kKeyPosMask;
    F.seg_len[sg] = F.rec[slot / kCodeLines].c_len[slot % kCodeLines];
    F.seg_grp[sg] = F.grp[slot / kCodeLines];
  }
}

__global__ void k_seg_total(FindParams F) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    F.ctrl->find_bytes = F.seg_off[F.n_seg_cap - 1] + F.seg_len[F.n_seg_cap - 1];
    F.ctrl->match_bytes = F.n_locs < F.n_seg_cap ? F.seg_off[F.n_locs] : F.ctrl->find_bytes;
  }
}

// Arena granule index: a non-empty segment k records itself at the first
// granule whose start byte it covers (at most one segment covers a byte), and
// an inclusive max-scan spreads it over the later granules it covers --
// segments ascend with their offsets.  Per block of 1024 granules here, the
// blocks' maxima carried by k_arena_gran_carry.
constexpr uint32_t kArenaGran = 256;
__global__ void k_arena_gran_mark(FindParams F) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F.n_seg_cap) return;
  const uint64_t o = F.seg_off[k], len = F.seg_len[k];
  if (!len) return;
  const uint64_t g = (o + kArenaGran - 1) / kArenaGran;
  if (g * kArenaGran < o + len && g < F.n_gran) F.gran_seg[g] = (uint32_t)k;
}
__global__ __launch_bounds__(1024) void k_arena_gran_scan(FindParams F) {
  __shared__ uint64_t s64[16];
  const uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t v = g < F.n_gran ? F.gran_seg[g] : 0u;
  uint64_t tot;
  const uint64_t incl = block_incl_max64(v, s64, &tot);
  if (g < F.n_gran) F.gran_seg[g] = (uint32_t)incl;
  if (threadIdx.x == 0) F.gran_carry[blockIdx.x + 1] = (uint32_t)tot;  // (exclusive carries after the next pass)
}
__global__ __launch_bounds__(1024) void k_arena_gran_carry(FindParams F, uint32_t n_blocks) {
  __shared__ uint64_t s64[16];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < n_blocks ? F.gran_carry[b + 1] : 0u;
    uint64_t tot;
    uint64_t incl = block_incl_max64(v, s64, &tot);
    incl = incl > carry ? incl : carry;
    if (b < n_blocks) F.gran_carry[b + 1] = (uint32_t)incl;  // carry into block b + 1
    carry = carry > tot ? carry : tot;
  }
  if (threadIdx.x == 0) F.gran_carry[0] = 0;
}
__device__ inline uint64_t arena_gran_seg(const FindParams& F, uint64_t g, uint64_t total) {
  if (g >= F.n_gran || g * kArenaGran >= total) return F.n_seg_cap - 1;
  const uint32_t a = F.gran_seg[g], c = F.gran_carry[g >> 10];
  return a > c ? a : c;
}

// The string arena, 16 bytes per lane over all segments (a multi-MiB line is
// spread over the whole grid): the segment by binary search over seg_off
// between the covering segments of the chunk's granule and the next one,
// source bytes from the batch, bytes inside the file's censor intervals as '*'.
__global__ __launch_bounds__(256) void k_arena_fill(FindParams F) {
  const uint64_t total = F.ctrl->find_bytes < F.arena_cap ? F.ctrl->find_bytes : F.arena_cap;  // (cap: redone larger)
  for (uint64_t a = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; a < total;
       a += (uint64_t)gridDim.x * blockDim.x * 16) {
    // last segment with seg_off <= a: in [covering(g), covering(g + 1)]
    uint64_t lo = arena_gran_seg(F, a / kArenaGran, total), hi = arena_gran_seg(F, a / kArenaGran + 1, total) + 1;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (F.seg_off[mid] <= a) lo = mid;
      else hi = mid;
    }
    uint64_t k = lo;
    if (a + 16 <= total && a + 16 <= F.seg_off[k] + F.seg_len[k]) {
      // fast path: the 16 bytes lie in one segment -- two aligned 16-byte
      // loads and a funnel shift, the censor intervals overlapping them (0-2,
      // sorted) applied as a byte mask, one store
      const uint64_t x = F.seg_src[k] + (a - F.seg_off[k]);
      const uint32_t g0 = F.seg_grp[k].x, gm = F.seg_grp[k].y;
      uint32_t l2 = 0, h2 = gm;  // first interval ending after x
      while (l2 < h2) {
        const uint32_t mid = (l2 + h2) >> 1;
        if (F.iv[2 * (g0 + mid) + 1] <= x) l2 = mid + 1;
        else h2 = mid;
      }
      uint32_t cmask = 0;  // bit j: byte x + j is censored
      for (uint32_t t2 = l2; t2 < gm; ++t2) {
        const uint64_t is = F.iv[2 * (g0 + t2)], ie = F.iv[2 * (g0 + t2) + 1];
        if (is >= x + 16) break;
        const uint32_t b = is > x ? (uint32_t)(is - x) : 0u, e2 = ie < x + 16 ? (uint32_t)(ie - x) : 16u;
        if (e2 > b) cmask |= ((1u << (e2 - b)) - 1u) << b;
      }
      const uint64_t src = F.off[F.seg_file[k]] + x;
      const uint64_t b0 = src & ~15ull;
      const uint32_t sh = (uint32_t)(src - b0);
      const uint4 u = *(const uint4*)(F.data + b0);
      uint32_t r[4] = {u.x, u.y, u.z, u.w};
      if (sh) {
        const uint4 v = ld16_guard(F.data, b0 + 16, F.data_end);
        const uint32_t d[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        const uint32_t q = sh >> 2, bs = 8 * (sh & 3);
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          const uint32_t lo32 = q == 0 ? d[z] : q == 1 ? d[z + 1] : q == 2 ? d[z + 2] : d[z + 3];
          const uint32_t hi32 = q == 0 ? d[z + 1] : q == 1 ? d[z + 2] : q == 2 ? d[z + 3] : d[z + 4];
          r[z] = bs ? (lo32 >> bs) | (hi32 << (32 - bs)) : lo32;
        }
      }
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const uint32_t m4 = (cmask >> (4 * z)) & 0xFu;
        const uint32_t bm = ((m4 & 1u) ? 0xFFu : 0u) | ((m4 & 2u) ? 0xFF00u : 0u) | ((m4 & 4u) ? 0xFF0000u : 0u) |
                            ((m4 & 8u) ? 0xFF000000u : 0u);
        r[z] = (r[z] & ~bm) | (0x2A2A2A2Au & bm);  // '*'
      }
      *(uint4*)(F.arena + a) = make_uint4(r[0], r[1], r[2], r[3]);
      continue;
    }
    uint32_t w[4] = {0, 0, 0, 0};
    uint64_t kk = ~0ull, fbase = 0;
    uint32_t g0 = 0, gm = 0, t = 0;  // the segment's file intervals, t = first one ending after x
    for (uint32_t j = 0; j < 16 && a + j < total; ++j) {
      if (a + j >= F.seg_off[k] + F.seg_len[k]) {
        // the next segment holding byte a + j: galloping then binary search --
        // runs of empty segments (Match windows kept inside their lines, blank
        // lines) can be 10^5 long, one dependent load each when walked
        uint64_t lo = k, d = 1;
        while (lo + d < F.n_seg_cap && F.seg_off[lo + d] <= a + j) {
          lo += d;
          d <<= 1;
        }
        uint64_t hi = lo + d < F.n_seg_cap ? lo + d : F.n_seg_cap;  // seg_off[hi] > a + j (or the end)
        while (hi - lo > 1) {
          const uint64_t mid = (lo + hi) >> 1;
          if (F.seg_off[mid] <= a + j) lo = mid;
          else hi = mid;
        }
        k = lo;  // the last segment starting at or before a + j: non-empty (it covers a + j)
      }
      const uint64_t x = F.seg_src[k] + (a + j - F.seg_off[k]);  // file-relative
      if (k != kk) {  // a new segment: its intervals and the first one ending after x (binary search)
        kk = k;
        fbase = F.off[F.seg_file[k]];
        g0 = F.seg_grp[k].x;
        gm = F.seg_grp[k].y;
        uint32_t l2 = 0, h2 = gm;
        while (l2 < h2) {
          const uint32_t mid = (l2 + h2) >> 1;
          if (F.iv[2 * (g0 + mid) + 1] <= x) l2 = mid + 1;
          else h2 = mid;
        }
        t = l2;
      }
      while (t < gm && F.iv[2 * (g0 + t) + 1] <= x) ++t;
      const bool cens = t < gm && F.iv[2 * (g0 + t)] <= x;
      const uint32_t byte = cens ? (uint32_t)'*' : F.data[fbase + x];
      w[j >> 2] |= byte << (8 * (j & 3));
    }
    if (a + 16 <= total) {
      *(uint4*)(F.arena + a) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (uint32_t j = 0; a + j < total; ++j) F.arena[a + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
  }
}

// Arena offsets into the records, and the (file, RuleID rank) sort keys.
__global__ void k_find_finalize(FindParams F) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= F.n_locs) return;
  FindRec& r = F.rec[w];
  if (r.m_off & kMatchInLine)  // (k_find_spans: the Match window inside Code slot kc's line, at offset d)
    r.m_off = F.seg_off[F.n_locs + F.line_uid[w * kCodeLines + ((r.m_off >> 48) & 0xFF)]] + (r.m_off & kMatchInLineOff);
  else if (!(r.m_off & kArenaDense))
    r.m_off = F.seg_off[w];
  if (r.n_lines && !(r.c_off & kArenaDense))  // (the window's lines are adjacent segments: consecutive line ids)
    r.c_off = F.seg_off[F.n_locs + F.line_uid[w * kCodeLines]];
  const uint32_t rank = F.rules[F.locs[w].rule].id_rank;
  r.rank = rank;
  F.sort_key[w] = ((uint64_t)r.file << F.rank_bits) | rank;
  F.sort_idx[w] = (uint32_t)w;
}

__global__ void k_find_gather(const FindRec* in, const uint32_t* idx, uint64_t n, FindRec* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}

// Scan's sort (scanner.go:441-446) is by (RuleID, Match): the first 16 bytes
// of each Match window (from the filled arena, zero-padded, big-endian) are
// two sort keys, so the device orders (file, RuleID rank, Match prefix) and
// the host only breaks ties of equal prefixes.  (8 bytes left 19 k ties on
// configs[4] -- lines opening with the same assignment -- and 2.7 ms of host
// sorting.)
__global__ void k_match_prefix(const FindRec* rec, const uint8_t* arena, const uint8_t* dense, uint64_t n,
                               uint64_t* key, uint64_t* key_b, uint32_t* idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FindRec& r = rec[i];
  const uint8_t* m = (r.m_off & kArenaDense) ? dense + (r.m_off & ~kArenaDense) : arena + r.m_off;
  uint64_t k = 0, kb = 0;
  for (uint32_t j = 0; j < 8; ++j) k = (k << 8) | (j < r.m_len ? m[j] : 0u);
  for (uint32_t j = 8; j < 16; ++j) kb = (kb << 8) | (j < r.m_len ? m[j] : 0u);
  key[i] = k;
  key_b[i] = kb;
  idx[i] = (uint32_t)i;
}

__global__ void k_gather_u64(const uint64_t* in, const uint32_t* idx, uint64_t n, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}

// Small key-value sorts (u64 keys on bits [0, end_bit), u32 values), tried
// for the post-scan lists of configs[2] (candidates, locations, Match keys:
// 29-35 K each), which hipcub's radix sort runs as a cascade of a block sort,
// five to seven merge passes and two trampolines -- ~9 launches per sort, 50
// of the tail's 150 kernels -- and measured slower (sort_pairs): not the
// product's path.  Two launches: k_tile_sort orders each tile of
// kSortTile (masked key, index) pairs in LDS (bitonic; the index breaks ties,
// so the order equals the stable radix sort's), and k_tile_merge places every
// element at its rank: its index in its own tile plus, per other tile, how
// many of that tile's pairs precede it (the tiles' binary searches advance
// level by level together, so a thread waits ~13 L2 latencies, not 13 per
// tile).  Larger lists go to hipcub (sort_pairs).
constexpr uint32_t kSortTile = 4096;
constexpr uint32_t kSortTiles = 16;  // up to 64 K pairs
constexpr uint32_t kSortSmall = kSortTile * kSortTiles;

__global__ __launch_bounds__(1024) void k_tile_sort(const uint64_t* kin, uint64_t n, uint64_t mask, uint64_t* skey,
                                                    uint32_t* sidx) {
  __shared__ uint64_t k[kSortTile];
  __shared__ uint32_t x[kSortTile];
  const uint32_t base = blockIdx.x * kSortTile;
  for (uint32_t i = threadIdx.x; i < kSortTile; i += blockDim.x) {
    const bool in = base + i < n;
    k[i] = in ? kin[base + i] & mask : ~0ull;
    x[i] = in ? base + i : 0xFFFFFFFFu;  // (padding sorts last: its index beats every real one)
  }
  __syncthreads();
  // a stage of distance j <= 64 keeps each wave inside its own two 128-pair
  // segments (pairs q = tid and tid + 1024): 63 of the 78 stages then need
  // only the wave's own ordering, the rest a block barrier (one barrier per
  // stage cost the sort ~2x hipcub's time on configs[2]'s 34 K candidates)
  for (uint32_t len = 2; len <= kSortTile; len <<= 1) {
    for (uint32_t j = len >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t q = threadIdx.x + h * (kSortTile / 4);
        const uint32_t a = 2 * j * (q / j) + (q % j), b = a + j;
        const bool up = (a & len) == 0;
        const uint64_t ka = k[a], kb = k[b];
        const uint32_t xa = x[a], xb = x[b];
        const bool gt = ka > kb || (ka == kb && xa > xb);
        if (gt == up) {
          k[a] = kb;
          k[b] = ka;
          x[a] = xb;
          x[b] = xa;
        }
      }
      const uint32_t jn = j > 1 ? j >> 1 : len;  // the next stage's distance
      if (j > 64 || jn > 64) {
        __syncthreads();
      } else {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kSortTile; i += blockDim.x) {
    skey[base + i] = k[i];
    sidx[base + i] = x[i];
  }
}

__global__ __launch_bounds__(256) void k_tile_merge(const uint64_t* kin, const uint32_t* vin, uint64_t n,
                                                    const uint64_t* skey, const uint32_t* sidx, uint32_t n_tiles,
                                                    uint64_t* kout, uint32_t* vout) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t t = g / kSortTile, r = g % kSortTile;
  if (t >= n_tiles) return;
  const uint32_t len_t = (uint32_t)min<uint64_t>(kSortTile, n - (uint64_t)t * kSortTile);
  if (r >= len_t) return;
  const uint64_t mk = skey[g];
  const uint32_t ix = sidx[g];
  uint32_t lo[kSortTiles], hi[kSortTiles];
#pragma unroll
  for (uint32_t u = 0; u < kSortTiles; ++u) {
    lo[u] = 0;
    hi[u] = u < n_tiles && u != t ? (uint32_t)min<uint64_t>(kSortTile, n - (uint64_t)u * kSortTile) : 0u;
  }
  for (int level = 0; level < 13; ++level) {  // (4096 = 2^12: 13 halvings empty any range)
    // all 16 probes loaded before any compare, unconditionally (an empty
    // range reads a stale slot of the scratch and ignores it): one L2
    // latency per level, not one per tile
    uint64_t pk[kSortTiles];
    uint32_t px[kSortTiles];
#pragma unroll
    for (uint32_t u = 0; u < kSortTiles; ++u) {
      const uint32_t m = (lo[u] + hi[u]) >> 1;
      pk[u] = skey[u * kSortTile + min(m, kSortTile - 1)];
      px[u] = sidx[u * kSortTile + min(m, kSortTile - 1)];
    }
#pragma unroll
    for (uint32_t u = 0; u < kSortTiles; ++u) {
      const uint32_t m = (lo[u] + hi[u]) >> 1;
      const bool less = pk[u] < mk || (pk[u] == mk && px[u] < ix);
      const bool open = lo[u] < hi[u];
      lo[u] = open && less ? m + 1 : lo[u];
      hi[u] = open && !less ? m : hi[u];
    }
  }
  uint32_t rank = r;
#pragma unroll
  for (uint32_t u = 0; u < kSortTiles; ++u) rank += lo[u];
  kout[rank] = kin[ix];
  vout[rank] = vin[ix];
}

// Positions i (> 0) of the ordered findings whose (file, rank) key AND Match
// prefix equal those of i - 1: the only places the host has to compare whole
// Match strings (appended unordered; the host sorts the short list).
__global__ void k_tie_list(const uint64_t* fr_key, const uint64_t* prefix, const uint64_t* prefix_b,
                           const uint32_t* order, uint64_t n, uint32_t* ties, uint64_t cap, Ctrl* ctrl) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 || i >= n) return;
  const uint32_t a = order[i], b = order[i - 1];
  if (fr_key[i] != fr_key[i - 1] || prefix[a] != prefix[b] || prefix_b[a] != prefix_b[b]) return;
  const unsigned long long k = atomicAdd(&ctrl->n_ties, 1ull);
  if (k < cap) ties[k] = (uint32_t)i;
}

// The kept locations as the ABI's tsg_loc records, in (file, start) order;
// a secret group that did not participate (the reference panics) is counted.
__global__ void k_out_locs(const DevLoc* locs, uint64_t n, tsg_loc* out, Ctrl* ctrl) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DevLoc L = locs[i];
  out[i] = tsg_loc{L.file, L.rule, L.start, L.end, L.start_line, L.end_line};
  if (L.flags & 1) atomicAdd(&ctrl->n_panic, 1ull);
}

// ---- SecretAnalyzer front end (tsg_analyze) --------------------------------
// utils.IsBinary (utils.go:77-95) per byte of the head.
__device__ inline bool is_binary_byte(uint32_t b) {
  return b < 7 || b == 11 || (b > 13 && b < 27) || (b > 27 && b < 0x20) || b == 0x7F;
}

// One wave per file: the first min(len, 300) bytes decide IsBinary; a binary
// file's bytes become '\r', so the compaction drops it to an empty file.
__global__ __launch_bounds__(256) void k_binary(uint8_t* data, const uint64_t* off, uint32_t n_files,
                                                uint8_t* bin_flags, unsigned long long* n_drop) {
  const uint32_t f = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63;
  if (f >= n_files) return;
  const uint64_t s = off[f], len = off[f + 1] - 1 - s;
  const uint32_t head = len < 300 ? (uint32_t)len : 300u;
  bool bin = false;
  for (uint32_t i = lane; i < head; i += 64) bin |= is_binary_byte(data[s + i]);
  bin = __ballot(bin) != 0;
  if (lane == 0) {
    bin_flags[f] = bin ? 1 : 0;
    if (bin && len) atomicAdd(n_drop, 1ull);
  }
  if (bin)
    for (uint64_t i = lane; i < len; i += 64) data[s + i] = '\r';
}

__device__ inline uint32_t cr_count_dword(uint32_t w) {  // bytes == 0x0D (exact SWAR)
  const uint32_t t = w ^ 0x0D0D0D0Du;
  const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
  return __builtin_popcount(z);
}

constexpr uint32_t kStripBlock = 4096;  // bytes per block (256 threads x 16)

// 16 bytes of the batch for thread t of block b (zero past the end) and how
// many of them survive the '\r' deletion.
__device__ inline uint32_t strip_chunk(const uint8_t* data, uint64_t nbytes, uint64_t g, uint4* v) {
  if (g + 16 <= nbytes) {
    *v = *(const uint4*)(data + g);
    return 16 - cr_count_dword(v->x) - cr_count_dword(v->y) - cr_count_dword(v->z) - cr_count_dword(v->w);
  }
  uint8_t tmp[16] = {0};
  uint32_t kept = 0;
  for (uint32_t i = 0; i < 16; ++i) {
    const uint64_t q = g + i;
    tmp[i] = q < nbytes ? data[q] : '\r';
    kept += tmp[i] != '\r';
  }
  memcpy(v, tmp, 16);
  return kept;
}

__device__ inline uint32_t block_excl_scan(uint32_t x, uint32_t* total) {
  __shared__ uint32_t wsum[4];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    if (k < w) base += wsum[k];
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return base + inc - x;
}

__global__ __launch_bounds__(256) void k_strip_count(const uint8_t* data, uint64_t nbytes, uint64_t* blk_kept) {
  const uint64_t g = (uint64_t)blockIdx.x * kStripBlock + threadIdx.x * 16;
  uint4 v;
  const uint32_t kept = strip_chunk(data, nbytes, g, &v);
  uint32_t total;
  (void)block_excl_scan(kept, &total);
  if (threadIdx.x == 0) blk_kept[blockIdx.x] = total;
}

// Writes the kept bytes at their compacted positions and, per 16-byte chunk,
// the compacted position of its first byte (for the file offsets).
__global__ __launch_bounds__(256) void k_strip_compact(const uint8_t* data, uint64_t nbytes, const uint64_t* blk_base,
                                                       uint8_t* out, uint64_t* chunk_pos) {
  const uint64_t chunk = (uint64_t)blockIdx.x * (kStripBlock / 16) + threadIdx.x;
  const uint64_t g = chunk * 16;
  uint4 v;
  const uint32_t kept = strip_chunk(data, nbytes, g, &v);
  uint32_t total;
  const uint64_t pos = blk_base[blockIdx.x] + block_excl_scan(kept, &total);
  if (g < nbytes) chunk_pos[chunk] = pos;
  const uint8_t* b = (const uint8_t*)&v;
  uint64_t o = pos;
  for (uint32_t i = 0; i < 16; ++i)
    if (b[i] != '\r' && g + i < nbytes) out[o++] = b[i];
}

// off'[f] = compacted position of byte off[f].
__global__ void k_strip_offsets(const uint8_t* data, const uint64_t* off, uint32_t n_files, const uint64_t* chunk_pos,
                                uint64_t total_kept, uint64_t* off_out) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f > n_files) return;
  if (f == n_files) {
    off_out[f] = total_kept;
    return;
  }
  const uint64_t p = off[f], c = p / 16;
  uint64_t q = chunk_pos[c];
  for (uint64_t i = c * 16; i < p; ++i) q += data[i] != '\r';
  off_out[f] = q;
}

}  // namespace

// =========================================================== host side ======


namespace {

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t want) {
    if (want <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t cap = want + want / 4 + 64;
    hipError_t e = hipMalloc(&p, cap * sizeof(T));
    if (e == hipSuccess) n = cap;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// k_scan_big's LDS blob for automaton `ac` (BigDev layout) and its state
// numbering; false when even one dense row does not fit.  Host only, so
// tsg_ruleset_big_check can replay it on the CPU.
struct BigBlobHost {
  std::vector<uint8_t> blob;
  std::vector<uint16_t> ac_of;  // blob state id -> automaton state id
  uint32_t nd = 0, cold = 0, o_cold = 0, o_eval = 0;
  uint32_t lds_bytes = 0, cold_lds = 0;  // the LDS prefix: classes, dense rows, lists, cold records [0, cold_lds)
};
static bool build_big_blob(const AcHost& ac, bool bfs, BigBlobHost* out) {
  if (ac.fail.size() != ac.nstates || ac.nclasses > kBigMore || ac.nstates > 0x8000u || !ac.nstates) return false;
  const uint32_t S = ac.nstates, K = ac.nclasses;
  // blob numbering (the first nd states get the dense rows): breadth first,
  // output states in place (the automaton's own numbering puts them last),
  // and inside a depth the likelier labels first -- a label's probability
  // under independent bytes of a text byte model (big_byte_weight), the
  // parent's times the edge class's (a state is first reached from its trie
  // parent).  Cold records read per byte, CPU replay of the stress corpora
  // (tests/test_big_blob.py): 0.0149 / 0.0084 -> 0.0140 / 0.0072; by
  // probability alone, 0.0181 / 0.0128.
  std::vector<uint32_t> order(S), at(S);  // blob id -> automaton id, and back
  for (uint32_t k = 0; k < S; ++k) order[k] = k;
  if (!bfs) {
    double wsum = 0;
    for (int b = 0; b < 256; ++b) wsum += big_byte_weight((uint8_t)b);
    std::vector<double> pc(K, 0.0);
    for (int b = 0; b < 256; ++b) pc[ac.cls[b]] += big_byte_weight((uint8_t)b) / wsum;
    std::vector<double> prob(S, -1.0);
    std::vector<int> depth(S, 0);
    std::vector<uint32_t> q{0};
    prob[0] = 1.0;
    for (size_t h = 0; h < q.size(); ++h) {
      const uint32_t st = q[h];
      for (uint32_t c = 0; c < K; ++c) {
        const uint32_t t = ac.delta[(size_t)st * K + c] & 0x7FFFu;
        if (prob[t] < 0) {
          prob[t] = prob[st] * pc[c];
          depth[t] = depth[st] + 1;
          q.push_back(t);
        }
      }
    }
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      return depth[a] != depth[b] ? depth[a] < depth[b] : prob[a] > prob[b];
    });
    if (order[0] != 0) return false;  // (k_scan_big starts every lane in blob state 0)
  }
  for (uint32_t k = 0; k < S; ++k) at[order[k]] = k;
  auto entry = [&](uint32_t st, uint32_t c) {  // delta in blob ids (bit 15 kept)
    const uint16_t v = ac.delta[(size_t)st * K + c];
    return (uint32_t)((v & 0x8000u) | at[v & 0x7FFFu]);
  };
  // A cold state's record is flat: its entries where they differ from its
  // first dense ancestor d on the failure chain (delta(s,c) = delta(d,c) for
  // every other class, since every state between s and d defers to its own
  // failure state there), and d itself -- one record and one dense row per
  // cold byte, no failure-chain walk.
  auto dense_anc = [&](uint32_t n, uint32_t nd) {  // blob id of n's first dense ancestor
    uint32_t a = at[ac.fail[order[n]]];
    while (a >= nd) a = at[ac.fail[order[a]]];
    return a;
  };
  auto flat_edges = [&](uint32_t n, uint32_t d, std::vector<uint32_t>* E) {  // class << 16 | entry
    E->clear();
    const uint32_t st = order[n], ds = order[d];
    for (uint32_t c = 0; c < K; ++c)
      if (ac.delta[(size_t)st * K + c] != ac.delta[(size_t)ds * K + c]) E->push_back((c << 16) | entry(st, c));
  };
  std::vector<uint32_t> E;
  auto list_words = [&](uint32_t nd) {
    uint64_t w = 0;
    for (uint32_t n = nd; n < S; ++n) {
      flat_edges(n, dense_anc(n, nd), &E);
      if (E.size() > 2) w += E.size() + 1;
    }
    return w;
  };
  auto a8 = [](uint64_t x) { return (x + 7) & ~7ull; };
  // layout: classes | dense rows | lists | cold records; LDS holds the prefix
  // through the first kBigColdLdsMin records (or all of them)
  uint32_t cold_min = g_big_cold_floor.load();
  if (const char* e = experiment_env("TSG_BIG_COLD_LDS")) cold_min = (uint32_t)atoi(e);
  cold_min = std::max(cold_min, 1u);  // (the device walk reads record min(j, CL - 1) in every lane)
  auto lds_for = [&](uint32_t nd) {
    return a8(a8(256 + (uint64_t)nd * K * 2) + list_words(nd) * 4) + (uint64_t)std::min<uint32_t>(S - nd, cold_min) * 8;
  };
  // the largest nd that fits: dense bytes grow with nd while the flat
  // records' lists shrink (few dense ancestors = long lists), so step down
  // from the most rows the dense part alone allows, coarse then fine
  uint32_t nd = (uint32_t)std::min<uint64_t>(S, (kBigLdsMax - 256) / (2 * (uint64_t)K));
  while (nd > 16 && lds_for(nd) > kBigLdsMax) nd -= 16;
  while (nd > 1 && lds_for(nd) > kBigLdsMax) --nd;
  if (!nd || lds_for(nd) > kBigLdsMax) return false;
  while (nd < S && lds_for(nd + 1) <= kBigLdsMax) ++nd;
  {
    const uint32_t cold = S - nd;
    const uint32_t o_eval = (uint32_t)a8(256 + (uint64_t)nd * K * 2);
    const uint32_t o_cold = (uint32_t)a8(o_eval + list_words(nd) * 4);
    const uint32_t cold_lds = (uint32_t)std::min<uint64_t>(cold, (kBigLdsMax - o_cold) / 8);
    std::vector<uint8_t> blob(o_cold + (size_t)cold * 8, 0);
    memcpy(blob.data(), ac.cls, 256);
    uint16_t* dense = (uint16_t*)(blob.data() + 256);
    for (uint32_t n = 0; n < nd; ++n)
      for (uint32_t c = 0; c < K; ++c) dense[(size_t)n * K + c] = (uint16_t)entry(order[n], c);
    uint32_t* rec = (uint32_t*)(blob.data() + o_cold);
    uint32_t* ev = (uint32_t*)(blob.data() + o_eval);
    uint32_t k = 0;
    for (uint32_t j = 0; j < cold; ++j) {
      const uint32_t d = dense_anc(nd + j, nd);
      flat_edges(nd + j, d, &E);
      if (E.size() <= 2) {
        const uint32_t c1 = E.size() > 0 ? E[0] >> 16 : kBigNone, c2 = E.size() > 1 ? E[1] >> 16 : kBigNone;
        const uint32_t n1 = E.size() > 0 ? E[0] & 0xFFFFu : 0, n2 = E.size() > 1 ? E[1] & 0xFFFFu : 0;
        rec[2 * j] = c1 | c2 << 8 | n1 << 16;
        rec[2 * j + 1] = n2 | d << 16;
      } else {
        rec[2 * j] = kBigMore | kBigMore << 8 | (k & 0xFFFFu) << 16;
        rec[2 * j + 1] = (k >> 16) | d << 16;
        for (uint32_t v : E) ev[k++] = v;
        ev[k++] = 0xFFFFFFFFu;
      }
    }
    out->lds_bytes = o_cold + cold_lds * 8;
    out->cold_lds = cold_lds;
    out->ac_of.assign(S, 0);
    for (uint32_t n = 0; n < S; ++n) out->ac_of[n] = (uint16_t)order[n];
    out->blob.swap(blob);
    out->nd = nd;
    out->cold = cold;
    out->o_cold = o_cold;
    out->o_eval = o_eval;
  }
  return true;
}

// Invariants that keep big_next (and k_big_walk's replay) inside the blob
// and finite, checked on every blob before it is uploaded, and at
// tsg_ruleset_compile: state 0 is the root and has a dense row; every class
// byte is < K; every entry (dense, inline, listed) names a state < S; every
// cold record's ancestor row is a dense row (so a cold byte reads one record
// and one dense row); at least one cold record sits in LDS when there are any;
// every overflow list lies inside the blob and is terminated.  Returns an
// empty string, or what is violated.
static std::string validate_big_blob(const BigBlobHost& bb, uint32_t K, uint32_t S) {
  if (K == 0 || K >= kBigMore || S == 0 || S > 0x8000u) return "class or state count out of range";
  if (bb.nd == 0 || bb.nd + bb.cold != S || bb.ac_of.size() != S || bb.ac_of[0] != 0)
    return "state 0 is not the dense root";
  if (bb.o_eval < 256 + (uint64_t)bb.nd * K * 2 || bb.o_cold < bb.o_eval || (bb.o_cold - bb.o_eval) % 4 ||
      bb.blob.size() != bb.o_cold + (uint64_t)bb.cold * 8 || bb.cold_lds > bb.cold || (bb.cold && !bb.cold_lds) ||
      bb.lds_bytes != bb.o_cold + (uint64_t)bb.cold_lds * 8 || bb.lds_bytes > kBigLdsMax)
    return "blob sections overlap or exceed the LDS budget";
  for (int b = 0; b < 256; ++b)
    if (bb.blob[b] >= K) return "byte class out of range";
  const uint16_t* dense = (const uint16_t*)(bb.blob.data() + 256);
  for (uint64_t i = 0; i < (uint64_t)bb.nd * K; ++i)
    if ((dense[i] & 0x7FFFu) >= S) return "dense entry out of range";
  const uint32_t* rec = (const uint32_t*)(bb.blob.data() + bb.o_cold);
  const uint32_t* ev = (const uint32_t*)(bb.blob.data() + bb.o_eval);
  const uint64_t n_ev = (bb.o_cold - bb.o_eval) / 4;  // (every list sits in the LDS prefix)
  for (uint32_t j = 0; j < bb.cold; ++j) {
    const uint32_t st = bb.nd + j, x = rec[2 * j], y = rec[2 * j + 1];
    if ((y >> 16) >= bb.nd) return "a cold record's ancestor row is not a dense row";
    (void)st;
    const uint32_t c1 = x & 0xFFu, c2 = (x >> 8) & 0xFFu;
    if (c1 == kBigMore) {
      uint64_t k = (x >> 16) | ((uint64_t)(y & 0xFFFFu) << 16);
      for (;; ++k) {
        if (k >= n_ev) return "an overflow list is not terminated inside the blob";
        const uint32_t v = ev[k];
        if (v == 0xFFFFFFFFu) break;
        if ((v >> 16) >= K || (v & 0x7FFFu) >= S) return "overflow list entry out of range";
      }
    } else {
      if ((c1 != kBigNone && c1 >= K) || (c2 != kBigNone && c2 >= K)) return "cold record class out of range";
      if ((c1 != kBigNone && ((x >> 16) & 0x7FFFu) >= S) || (c2 != kBigNone && (y & 0x7FFFu) >= S))
        return "cold record entry out of range";
    }
  }
  return std::string();
}

// The blob the engine would upload for this ruleset (none when k_scan_fast's
// image or an LDS table holds the automaton), validated: TSG_ERR_INTERNAL with
// the violated invariant rather than a device walk that could not end.
static bool needs_big_blob(const AcHost& ac) {
  return ac.fast.empty() && (size_t)ac.nstates * ac.nclasses * 2 > (size_t)kLdsTableMax;
}

}  // namespace

int tsg::big_blob_precheck(const AcHost& ac, std::string* err) {
  if (!needs_big_blob(ac)) return TSG_OK;
  BigBlobHost bb;
  if (!build_big_blob(ac, experiment_env("TSG_BIG_BFS") != nullptr, &bb)) return TSG_OK;  // (generic kernel)
  const std::string why = validate_big_blob(bb, ac.nclasses, ac.nstates);
  if (why.empty()) return TSG_OK;
  *err = "k_scan_big automaton blob is malformed: " + why;
  return TSG_ERR_INTERNAL;
}

namespace {

// big_next on the host copy of the blob (the device walk, for the CPU check);
// *hops = cold records read.
static uint32_t big_next_host(const BigBlobHost& bb, uint32_t K, uint32_t st, uint32_t c, uint32_t* hops) {
  const uint16_t* dense = (const uint16_t*)(bb.blob.data() + 256);
  const uint32_t* rec = (const uint32_t*)(bb.blob.data() + bb.o_cold);
  const uint32_t* ev = (const uint32_t*)(bb.blob.data() + bb.o_eval);
  const size_t n_ev = (bb.o_cold - bb.o_eval) / 4;
  if (st >= bb.nd) {
    ++*hops;
    const uint32_t x = rec[2 * (st - bb.nd)], y = rec[2 * (st - bb.nd) + 1];
    if (c == (x & 0xFFu)) return x >> 16;
    if (c == ((x >> 8) & 0xFFu)) return y & 0xFFFFu;
    if ((x & 0xFFu) == kBigMore) {
      for (size_t k = (x >> 16) | ((y & 0xFFFFu) << 16);; ++k) {
        if (k >= n_ev) return 0xFFFFFFFEu;  // (list runs off the blob)
        const uint32_t v = ev[k];
        if (v == 0xFFFFFFFFu) break;
        if ((v >> 16) == c) return v & 0xFFFFu;
      }
    }
    st = y >> 16;
    if (st >= bb.nd) return 0xFFFFFFFFu;  // (not a dense row: the device would read past the table)
  }
  return dense[st * K + c];
}

// Run acceleration of a verify DFA: a state whose entry is the same on a
// set of at least kAccelMinStay ASCII bytes (its "stay" set), and that entry
// keeps the state with the same flags, steps over runs of stay bytes with a
// bitmap test per byte and no table lookups (a private key's base64 body,
// `[a-z0-9]{17,}` tails).  Records (32 B): the stay bitmap (4 u32), the class
// of a stay byte, padding; per state a record index or ~0.
constexpr int kAccelMinStay = 16;
struct DfaAccel {
  std::vector<uint32_t> idx;   // per state
  std::vector<uint32_t> recs;  // 8 u32 per record
};
static DfaAccel dfa_accel_records(const DfaHost& D) {
  const uint32_t K = std::max<uint32_t>(1, D.ncls), S = (uint32_t)(D.delta.size() / K);
  DfaAccel A;
  A.idx.assign(S, 0xFFFFFFFFu);
  for (uint32_t st = 1; st < S; ++st) {
    std::map<uint16_t, int> cnt;
    for (int b = 0; b < 128; ++b) ++cnt[D.delta[(size_t)st * K + D.cls[b]]];
    uint16_t self = 0;
    int best = -1;
    for (auto& kv : cnt)
      if ((kv.first & kDfaStateMask) == st && kv.second > best) {
        best = kv.second;
        self = kv.first;
      }
    if (best < kAccelMinStay) continue;
    uint32_t bm[4] = {0, 0, 0, 0}, scls = 0;
    for (int b = 0; b < 128; ++b)
      if (D.delta[(size_t)st * K + D.cls[b]] == self) {
        bm[b >> 5] |= 1u << (b & 31);
        scls = D.cls[b];
      }
    A.idx[st] = (uint32_t)(A.recs.size() / 8);
    A.recs.insert(A.recs.end(), {bm[0], bm[1], bm[2], bm[3], scls, 0, 0, 0});
  }
  return A;
}

struct DevImage {
  uint64_t rs_id = 0;
  DBuf<uint8_t> big;  // k_scan_big blob (empty unless the automaton needs it)
  DBuf<uint16_t> big_ac_of;  // its state numbering -> the automaton's
  BigDev big_view{};
  DBuf<gre::Inst> inst;
  DBuf<gre::ClassDesc> classes;
  DBuf<uint32_t> ranges;
  DBuf<gre::ProgView> progs;
  DBuf<RuleDev> rules;
  DBuf<uint32_t> u32;  // kw_ids | group_slots | allow_progs | global_allow | gpath | rule_apath_off | rule_apath | full_rules
  DBuf<int32_t> rule_path;
  DBuf<uint16_t> delta;
  DBuf<uint8_t> cls;
  DBuf<uint32_t> out_off;
  DBuf<uint16_t> out_pat;
  DBuf<PatDev> pats;
  DBuf<uint8_t> pat_bytes;
  DBuf<uint32_t> pat_rules;
  DBuf<uint8_t> fast;
  DBuf<uint32_t> prog_lit_off;
  DBuf<uint8_t> prog_lits;
  DBuf<uint16_t> follow_delta;
  DBuf<uint8_t> follow_cls;
  DBuf<uint8_t> pac;  // path literal automaton blob (k_path_gate)
  DBuf<uint16_t> dfa_delta;
  DBuf<uint8_t> dfa_bytes;
  DBuf<uint8_t> nfa;         // bit-parallel NFA records (nfa.cpp)
  DBuf<uint8_t> uni_bytes;   // lowercased non-ASCII keywords (k_uni_keywords)
  DBuf<uint32_t> uni_meta;   // per such keyword: byte offset, byte length, keyword id
  DBuf<uint32_t> lower_map;  // kLowerMap: {rune, lowercase} pairs
  uint32_t n_uni = 0, uni_back = 0;
  uint32_t pac_states = 0, pac_classes = 0, pac_bytes = 0;
  std::vector<uint8_t> pac_prog_bit;  // per regex: its bit in k_path_gate's literal mask (0xFF: none)
  uint32_t o_pac_cls = 0, o_pac_out_off = 0, o_pac_out = 0, o_pac_lits = 0, o_pac_req = 0, o_pac_bit = 0;
  uint64_t pac_always = 0;
  RuleSetDev view{};
  // offsets into u32
  uint32_t o_gpath = 0, n_gpath = 0, o_apoff = 0, o_ap = 0, o_full = 0, n_full = 0, o_prules = 0, n_prules = 0;
  uint32_t o_fold = 0, n_fold_items = 0;  // k_fold_windows work items
  uint32_t o_xoff = 0, o_xprog = 0, o_gx = 0, n_gx = 0, max_x = 0;  // exclude blocks (ExclDev)
  uint32_t o_pdfa = 0;  // path-regex MatchString DFA records (kPathDfaRec u32 per program)
  void release() {
    big.release();
    inst.release(); classes.release(); ranges.release(); progs.release(); rules.release();
    u32.release(); rule_path.release(); delta.release(); cls.release(); out_off.release();
    out_pat.release(); pats.release(); pat_bytes.release(); pat_rules.release(); fast.release();
    prog_lit_off.release(); prog_lits.release(); follow_delta.release(); follow_cls.release(); pac.release(); dfa_delta.release(); dfa_bytes.release(); nfa.release();
    uni_bytes.release(); uni_meta.release(); lower_map.release();
  }
};

}  // namespace

struct tsg_engine {
  int device = 0;
  int verify_split = 0;  // 1: every job list through k_verify_fast (tests; tsg_engine_force_verify_split)
  // launch_scan: the scan kernels skip the per-span newline counts (nl_lazy,
  // set by the caller), and nl_deferred records that the last scan did, so
  // k_nl_spans counts the spans of the files that have locations
  bool nl_lazy = false, nl_deferred = false;
  uint64_t nl_big = 0;  // the last scan's span_scan_counted threshold (k_nl_spans skips those spans)
  DBuf<uint32_t> fbase;  // newline prefix at each location file's start (k_file_base)
  DBuf<unsigned long long> nl_last;  // per file: counted bound + 1 (0: none) | kNlFull (k_nl_cands / _check / _tail)
  hipEvent_t ev_nl[2] = {nullptr, nullptr};  // candidates ready -> phase-0 count done (side stream)
  hipEvent_t ev_pg[2] = {nullptr, nullptr};  // the side-stream path gate: start, end
  bool nl_pending = false;                   // a phase-0 count was issued on the side stream
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevImage img;
  DBuf<uint8_t> data;
  DBuf<uint64_t> off;
  DBuf<uint8_t> paths;
  DBuf<uint64_t> path_off;
  DBuf<uint32_t> file_kw, file_flags, path_mask;
  DBuf<uint64_t> hits;
  DBuf<uint64_t> keys, keys2;
  DBuf<uint32_t> vals, vals2;
  DBuf<uint8_t> flags8;
  DBuf<uint32_t> job_start;
  DBuf<uint32_t> nsel;
  DBuf<uint8_t> cub_tmp;
  DBuf<uint64_t> ss_key;  // sort_pairs: the tile-sorted (masked key, index) pairs
  DBuf<uint32_t> ss_idx;
  DBuf<uint64_t> hit_seg, hit_pre, ev_pre;  // k_report's per-wave hit regions, their exclusive offsets (+ the base)
  DBuf<uint32_t> hit_seg_n;
  DBuf<DevLoc> locs, locs2;
  DBuf<unsigned long long> loc_cnt;  // sharded location counters (kLocShards + the overflow region's)
  DBuf<uint8_t> scratch;
  DBuf<Ctrl> ctrl;
  DBuf<uint32_t> nl_blocks, nl_pre;
  DBuf<uint8_t> tail;
  DBuf<uint32_t> region_file, region_tmp;
  DBuf<FastEvent> ev_buf, ev_overflow;
  DBuf<uint64_t> vprof;
  DBuf<uint8_t> span_hi;
  DBuf<uint64_t> fold_pos;    // fold-special rune occurrences (k_fold_windows)
  uint64_t fold_need = 0;     // fold-position capacity learnt from a lost scan
  DBuf<CapJob> caps, caps_big, caps_run;
  DBuf<uint64_t> job_fms, job_lme;  // speculative jobs (k_chain_fix)
  DBuf<uint8_t> job_bad;
  DBuf<RedoRec> redo;
  DBuf<uint32_t> defer;  // k_verify_fast -> k_verify_slow job list
  DBuf<CapJob> matches;  // k_verify_fast -> k_allow
  DBuf<uint32_t> ev_counts;
  uint64_t ev_ovf_need = 0;  // overflow-event capacity learnt from a lost scan
  DBuf<uint64_t> big_outs;   // k_big_walk's output records
  uint64_t big_out_need = 0;  // their capacity learnt from a lost scan
  bool fast_timed = false;   // ev[10..11] bracket the last k_scan_fast launch
  DBuf<uint8_t> fflags8;     // per-file result flags, u8
  uint32_t num_cus = 0;
  DBuf<ExclRange> excl_out;
  DBuf<uint8_t> part_buf;  // byte-range split: a part's packed scan state (export / import)
  uint32_t vm_threads = 0;
  uint64_t scratch_stride = 0;
  hipEvent_t ev[12];
  bool events = false;
  hipStream_t side = nullptr;  // D2H of the findings' Code records and strings under the last sorts
  hipEvent_t ev_code = nullptr, ev_fill = nullptr, ev_side = nullptr;
  DBuf<uint32_t> gate_out, gate_rules;  // tsg_gate_device: rule gate words, rule -> keyword-id CSR
  // tsg_analyze: IsBinary flags, '\r'-stripped batch and its offsets, block sums, chunk positions
  DBuf<uint8_t> bin8, strip_out;
  DBuf<uint64_t> strip_off, blk_kept, blk_base, chunk_pos;
  DBuf<unsigned long long> n_drop;
  uint8_t* h_stage = nullptr;  // pinned host staging of tsg_scan / tsg_analyze (grow-only)
  size_t h_stage_n = 0;
  double stage_ms[2] = {0, 0};  // last stage_host_batch: pack (+ overlapped H2D), H2D tail (host clock)
  std::vector<double> gate_tm;          // timings of the last tsg_gate_device call
  // device findings (build_findings_dev)
  DBuf<uint64_t> f_iv, f_lkey, f_lkey2, f_ssrc, f_slen, f_soff;
  DBuf<uint32_t> f_lslot, f_lslot2, f_lhead, f_lscan, f_luid, f_sfile;
  DBuf<uint2> f_sgrp;
  DBuf<uint2> f_grp;
  DBuf<FindRec> f_rec, f_rec2;
  DBuf<uint32_t> f_ties;   // k_tie_list
  DBuf<tsg_loc> out_locs;  // k_out_locs
  DBuf<uint32_t> gate_defer;  // k_path_gate: files for its DFA / VM pass ([0] = count)
  DBuf<uint8_t> f_arena;
  DBuf<uint32_t> f_gran, f_gcarry;  // arena granule index (k_arena_gran_*)
  DBuf<uint64_t> f_lkeyb;            // Match bytes 8..15 (k_match_prefix)
  // dense files' region of the arena (k_dense_*): per file group its size and
  // offset, per location its file's offset; the censored contents
  DBuf<uint64_t> f_dsize, f_doff, f_dense_at;
  DBuf<uint32_t> f_gstart;
  DBuf<uint8_t> f_dense;
  uint64_t* h_dense = nullptr;  // page-locked: the region's bytes and file groups, read mid-pipeline
  uint64_t* h_find = nullptr;   // page-locked: the arena's find_bytes / match_bytes, read under the arena fill
  uint64_t arena_need = 0;      // arena capacity the next call starts with (the last need + 1/4)
  uint64_t cand_need = 0;       // candidate capacity of the next call's speculative k_expand (the last count + 1/4)
  uint64_t hit_need = 0;        // hits the next call's speculative k_expand grid covers (the last count + 1/4)
  hipEvent_t ev_dense = nullptr, ev_dfill = nullptr, ev_frec = nullptr, ev_fb = nullptr;
  bool dense_active = false;   // this call's locations have dense_at (dense_begin)
  DBuf<uint64_t> f_pmax;       // per location: (file << 40 | max end so far in its file), k_dense_fill's censoring
  DBuf<uint32_t> f_spidx;      // per location: exclusive prefix of the sparse ones (FindParams::slot_base)
  DBuf<uint32_t> f_long;       // k_find_spans_lane's list of long-line locations
  uint64_t n_line_slots = 0;   // Code slots the distinct-line sort takes (4 per sparse location)
  hsa_signal_t dma_sig{0};  // dma_d2h's completion signal
  bool dma_pending = false;
  std::shared_ptr<PinnedPool> pinned = std::make_shared<PinnedPool>();
};

namespace {

// Rule gate words of tsg_gate_device, one lane per file: rule r passes iff it
// has no keywords or one of its keyword ids is set in the file's keyword bits
// (Rule.MatchKeywords, scanner.go:169-181).  `rules` is a CSR: rules[0..R]
// offsets into rules[R+1..], a keyword id or 0xFFFFFFFF for "always".
__global__ void k_rule_gates(const uint32_t* __restrict__ file_kw, uint32_t kw_words, uint32_t n_files,
                             const uint32_t* __restrict__ rules, uint32_t n_rules, uint32_t* __restrict__ out,
                             uint32_t words) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_files) return;
  const uint32_t* kw = file_kw + (uint64_t)f * kw_words;
  const uint32_t* ids = rules + n_rules + 1;
  uint32_t w = 0;
  for (uint32_t r = 0; r < n_rules; ++r) {
    bool pass = rules[r] == rules[r + 1];
    for (uint32_t k = rules[r]; k < rules[r + 1] && !pass; ++k) {
      const uint32_t id = ids[k];
      pass = id == 0xFFFFFFFFu || ((kw[id >> 5] >> (id & 31)) & 1);
    }
    if (pass) w |= 1u << (r & 31);
    if ((r & 31) == 31 || r + 1 == n_rules) {
      if ((r >> 5) < words) out[(uint64_t)f * words + (r >> 5)] = w;
      w = 0;
    }
  }
  for (uint32_t j = (n_rules + 31) >> 5; j < words; ++j) out[(uint64_t)f * words + j] = 0;
}

// The same gates from per-rule keyword masks (host-built: rule r passes when
// it has no keyword, has the empty keyword, or shares a bit with the file's
// keyword words), the file's words held in registers: one AND-OR per word and
// rule instead of k_rule_gates' dependent CSR walk per keyword (0.12 ms on
// configs[1]'s 0.9 M files).  Up to kGateMaskWords keyword words.
constexpr uint32_t kGateMaskWords = 8;
__global__ __launch_bounds__(256) void k_rule_gates_mask(const uint32_t* __restrict__ file_kw, uint32_t kw_words,
                                                         uint32_t n_files, const uint32_t* __restrict__ masks,
                                                         uint32_t n_rules, uint32_t* __restrict__ out, uint32_t words) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_files) return;
  uint32_t kw[kGateMaskWords];
#pragma unroll
  for (uint32_t w = 0; w < kGateMaskWords; ++w) kw[w] = w < kw_words ? file_kw[(uint64_t)f * kw_words + w] : 0u;
  // masks: per rule kw_words masks, then one word per 32 rules of always-pass bits
  const uint32_t* always = masks + (size_t)n_rules * kw_words;
  for (uint32_t j = 0; j < words; ++j) {
    uint32_t bits = 0;
    if (j * 32 < n_rules) {
      bits = always[j];
      const uint32_t r1 = min(n_rules, j * 32 + 32);
      for (uint32_t r = j * 32; r < r1; ++r) {
        uint32_t any = 0;
#pragma unroll
        for (uint32_t w = 0; w < kGateMaskWords; ++w)
          if (w < kw_words) any |= kw[w] & masks[(size_t)r * kw_words + w];
        bits |= any ? 1u << (r - j * 32) : 0u;
      }
    }
    out[(uint64_t)f * words + j] = bits;
  }
}

int upload_ruleset(tsg_engine* e, const tsg_ruleset* rs) {
  DevImage& im = e->img;
  if (im.rs_id == rs->id) return TSG_OK;
  // ---- programs
  std::vector<gre::Inst> inst;
  std::vector<gre::ClassDesc> classes;
  std::vector<uint32_t> ranges;
  struct Off { size_t i, c, r; };
  std::vector<Off> offs;
  uint32_t max_ninst = 1, max_ncap = 2, max_ninst_cap = 1;
  for (auto& rx : rs->regexes) {
    const gre::Prog& p = rx.c.prog;
    offs.push_back({inst.size(), classes.size(), ranges.size()});
    inst.insert(inst.end(), p.inst.begin(), p.inst.end());
    for (auto cd : p.classes) {
      cd.range_off += (uint32_t)ranges.size();
      classes.push_back(cd);
    }
    ranges.insert(ranges.end(), p.ranges.begin(), p.ranges.end());
    max_ninst = std::max<uint32_t>(max_ninst, (uint32_t)p.inst.size());
  }
  for (auto& r : rs->rules)
    if (!r.group_name.empty() && r.regex >= 0)
    {
      max_ncap = std::max<uint32_t>(max_ncap, (uint32_t)rs->regexes[r.regex].c.prog.ncap);
      max_ninst_cap = std::max<uint32_t>(max_ninst_cap, (uint32_t)rs->regexes[r.regex].c.prog.inst.size());
    }
  HIP_TRY(im.inst.ensure(inst.size() + 1));
  HIP_TRY(im.classes.ensure(classes.size() + 1));
  HIP_TRY(im.ranges.ensure(ranges.size() + 1));
  HIP_TRY(hipMemcpy(im.inst.p, inst.data(), inst.size() * sizeof(gre::Inst), hipMemcpyHostToDevice));
  if (!classes.empty())
    HIP_TRY(hipMemcpy(im.classes.p, classes.data(), classes.size() * sizeof(gre::ClassDesc), hipMemcpyHostToDevice));
  if (!ranges.empty())
    HIP_TRY(hipMemcpy(im.ranges.p, ranges.data(), ranges.size() * 4, hipMemcpyHostToDevice));
  std::vector<gre::ProgView> views;
  for (size_t k = 0; k < rs->regexes.size(); ++k) {
    const gre::Prog& p = rs->regexes[k].c.prog;
    views.push_back(gre::ProgView{im.inst.p + offs[k].i, im.classes.p + offs[k].c, im.ranges.p,
                                  (uint32_t)p.inst.size(), p.start, (uint32_t)p.ncap, p.nvis});
  }
  // per-program anchor literals for the MatchString prefilter
  std::vector<uint32_t> lit_off{0};
  std::vector<uint8_t> lits;
  for (auto& rx : rs->regexes) {
    const gre::Anchor& a = rx.c.anchor;
    if (a.valid && a.lits.size() <= 32) {
      // only a case-free k / s can be matched by a non-ASCII rune (U+212A, U+017F)
      bool fold_lits = false;
      for (auto& l : a.lits)
        for (size_t j = 0; j < l.lower.size(); ++j)
          fold_lits |= (l.lower[j] == 'k' || l.lower[j] == 's') && l.req[j] == 0;
      for (auto& l : a.lits) {
        uint8_t rec[kLitRec] = {0};
        rec[0] = (uint8_t)l.lower.size();
        memcpy(rec + 1, l.lower.data(), l.lower.size());
        memcpy(rec + 17, l.req.data(), l.req.size());
        rec[kLitExactByte] = rx.c.literal_exact ? 1 : 0;
        rec[kLitFoldByte] = fold_lits ? 1 : 0;
        lits.insert(lits.end(), rec, rec + kLitRec);
      }
    }
    lit_off.push_back((uint32_t)(lits.size() / kLitRec));
  }
  HIP_TRY(im.prog_lit_off.ensure(lit_off.size()));
  HIP_TRY(hipMemcpy(im.prog_lit_off.p, lit_off.data(), lit_off.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(im.prog_lits.ensure(lits.size() + kLitRec));
  if (!lits.empty()) HIP_TRY(hipMemcpy(im.prog_lits.p, lits.data(), lits.size(), hipMemcpyHostToDevice));
  HIP_TRY(im.progs.ensure(views.size() + 1));
  if (!views.empty())
    HIP_TRY(hipMemcpy(im.progs.p, views.data(), views.size() * sizeof(gre::ProgView), hipMemcpyHostToDevice));
  // ---- rules + u32 side tables
  std::vector<uint32_t> u32;
  std::vector<RuleDev> rules;
  std::vector<int32_t> rule_path;
  std::map<std::string, uint32_t> kwid;
  for (size_t k = 0; k < rs->keywords.size(); ++k) kwid[rs->keywords[k]] = (uint32_t)k;
  std::vector<uint32_t> kw_ids, group_slots, allow_progs, apath_off, apath, full_rules, path_rules;
  std::vector<uint16_t> fdelta, ddelta;
  std::vector<uint8_t> fcls, dbytes, nbytes;
  std::set<uint32_t> kw_needed_ids;
  std::vector<std::string> ids;  // sorted distinct rule IDs: the findings' RuleID order
  for (auto& r : rs->rules) ids.push_back(r.id);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  for (size_t ri = 0; ri < rs->rules.size(); ++ri) {
    const RuleHost& r = rs->rules[ri];
    RuleDev d{};
    d.id_rank = (uint32_t)(std::lower_bound(ids.begin(), ids.end(), r.id) - ids.begin());
    d.follow_off = kNoFollow;
    d.dfa_off = kNoFollow;
    if (r.dfa.valid) {
      if (ddelta.size() & 1) ddelta.push_back(0);  // even offsets: k_verify stages tables as dwords
      d.dfa_off = (uint32_t)ddelta.size();
      d.dfa_ncls = r.dfa.ncls;
      d.dfa_cls_off = (uint32_t)dbytes.size();
      dbytes.insert(dbytes.end(), r.dfa.cls, r.dfa.cls + 128);
      d.dfa_match_off = (uint32_t)dbytes.size();
      dbytes.insert(dbytes.end(), r.dfa.match.begin(), r.dfa.match.end());
      d.dfa_start0 = r.dfa.start[0];
      d.dfa_start1 = r.dfa.start[1];
      for (int q = 0; q < 4; ++q) d.dfa_first[q] = r.dfa.first[q];
      d.dfa_size = (uint32_t)r.dfa.delta.size();
      d.dfa_smatch = (r.dfa.match[r.dfa.start[0]] ? 1u : 0u) | (r.dfa.match[r.dfa.start[1]] ? 2u : 0u);
      d.dfa_sym = r.dfa.sym_base | (r.dfa.na_ok ? 0x80000000u : 0u);
      // accelerable states (a private key's body, `.{0,N}` runs): the entry
      // on all but <= 3 ASCII bytes keeps the state with the same flags, so
      // the device skips such runs with vector compares (dfa_accel_skip)
#ifdef TSG_EXPERIMENTS
      const DfaAccel acc = dfa_accel_records(r.dfa);
#else
      const DfaAccel acc{std::vector<uint32_t>(r.dfa.delta.size() / std::max<uint32_t>(1, r.dfa.ncls), 0xFFFFFFFFu), {}};
#endif
      while (dbytes.size() & 15) dbytes.push_back(0);
      d.dfa_accel_off = (uint32_t)dbytes.size();  // per-state record index (u32), then the 32-byte records
      dbytes.insert(dbytes.end(), (const uint8_t*)acc.idx.data(), (const uint8_t*)(acc.idx.data() + acc.idx.size()));
      while (dbytes.size() & 15) dbytes.push_back(0);
      d.dfa_accel_recs = (uint32_t)dbytes.size();
      dbytes.insert(dbytes.end(), (const uint8_t*)acc.recs.data(), (const uint8_t*)(acc.recs.data() + acc.recs.size()));
      const size_t at = ddelta.size();
      ddelta.insert(ddelta.end(), r.dfa.delta.begin(), r.dfa.delta.end());
      for (size_t i = at; i < ddelta.size(); ++i)
        if (acc.idx[ddelta[i] & kDfaStateMask] != 0xFFFFFFFFu) ddelta[i] |= kDfaAccel;
    }
    d.nfa_off = kNoFollow;
    if (r.nfa.valid) {  // (records are multiples of 16 bytes: every one stays 16-byte aligned)
      d.nfa_off = (uint32_t)nbytes.size();
      d.nfa_bytes = (uint32_t)r.nfa.blob.size();
      nbytes.insert(nbytes.end(), r.nfa.blob.begin(), r.nfa.blob.end());
    }
    if (r.follow.valid) {
      d.follow_off = (uint32_t)fdelta.size();
      d.follow_ncls = r.follow.ncls;
      d.follow_cls_off = (uint32_t)fcls.size();
      fdelta.insert(fdelta.end(), r.follow.delta.begin(), r.follow.delta.end());
      fcls.insert(fcls.end(), r.follow.cls, r.follow.cls + 128);
    }
    d.prog = r.regex >= 0 ? (uint32_t)r.regex : 0;
    d.mode = r.mode;
    d.kw_off = (uint32_t)kw_ids.size();
    for (auto& kw : r.keywords) {
      if (kw.empty()) d.gate_always = 1;
      else kw_ids.push_back(kwid[kw]);
    }
    d.kw_n = (uint32_t)kw_ids.size() - d.kw_off;
    if (r.keywords.empty()) d.kw_n = 0;
    if (r.regex >= 0) {
      const gre::Compiled& c = rs->regexes[r.regex].c;
      if (c.anchor.valid) {
        d.off_min = c.anchor.off_min;
        d.off_max = c.anchor.off_max;
        for (int q = 0; q < 4; ++q) d.alpha[q] = c.anchor.alpha.w[q];
      }
      d.use_groups = !r.group_name.empty();
      d.max_len = c.max_len;
      d.no_nl = 1;
      for (auto& in : c.prog.inst) {
        const bool nl = in.op == gre::I_ANY || (in.op == gre::I_RUNE1 && in.arg == '\n') ||
                        (in.op == gre::I_RUNE && ((c.prog.classes[in.arg].ascii['\n' >> 5] >> ('\n' & 31)) & 1));
        if (nl) d.no_nl = 0;
      }
      d.group_off = (uint32_t)group_slots.size();
      if (d.use_groups)
        for (size_t g = 0; g < c.prog.cap_names.size(); ++g)
          if (c.prog.cap_names[g] == r.group_name) group_slots.push_back((uint32_t)g);
      d.group_n = (uint32_t)group_slots.size() - d.group_off;
      if (d.use_groups && r.grp.valid) {  // ruleset.cpp: gre::group_span of the one named group
        d.grp_fast = 1;
        d.grp_pre = r.grp.pre;
        d.grp_len = r.grp.len;
        d.grp_suf = r.grp.suf;
      } else if (d.use_groups && r.grun.valid) {  // else gre::group_run
        d.grp_run = 1;
        d.grp_run_len = r.grun.len;
        for (int k = 0; k < 4; ++k) {
          d.grp_s[k] = r.grun.s_alpha[k];
          d.grp_b[k] = r.grun.b_alpha[k];
        }
      }
    }
    d.gate_implied = r.gate_implied;  // ruleset.cpp: every anchor literal contains a keyword
    if (!d.gate_implied || r.fold_gate)  // exact keyword bits: non-implied gates, K/ſ-spelled hits
      for (auto& kw : r.keywords)
        if (!kw.empty()) kw_needed_ids.insert(kwid[kw]);
    d.allow_off = (uint32_t)allow_progs.size();
    for (int x : r.allow_regex) allow_progs.push_back((uint32_t)x);
    d.allow_n = (uint32_t)allow_progs.size() - d.allow_off;
    rules.push_back(d);
    rule_path.push_back(r.path);
    apath_off.push_back((uint32_t)apath.size());
    for (int x : r.allow_path) apath.push_back((uint32_t)x);
    if (r.mode == MODE_FULL) full_rules.push_back((uint32_t)ri);
    if (r.path >= 0 || !r.allow_path.empty()) path_rules.push_back((uint32_t)ri);
  }
  apath_off.push_back((uint32_t)apath.size());
  auto append = [&](const std::vector<uint32_t>& v) {
    uint32_t o = (uint32_t)u32.size();
    u32.insert(u32.end(), v.begin(), v.end());
    return o;
  };
  uint32_t o_kw = append(kw_ids), o_gs = append(group_slots), o_ap = append(allow_progs);
  std::vector<uint32_t> gallow(rs->global_allow_regex.begin(), rs->global_allow_regex.end());
  std::vector<uint32_t> gpath(rs->global_allow_path.begin(), rs->global_allow_path.end());
  uint32_t o_ga = append(gallow);
  im.o_gpath = append(gpath);
  im.n_gpath = (uint32_t)gpath.size();
  im.o_apoff = append(apath_off);
  im.o_ap = append(apath);
  im.o_prules = append(path_rules);
  im.n_prules = (uint32_t)path_rules.size();
  im.o_full = append(full_rules);
  im.n_full = (uint32_t)full_rules.size();
  {  // exclude blocks: per rule offsets into its regex list, the global list
    std::vector<uint32_t> xoff, xprog;
    im.max_x = (uint32_t)rs->global_exclude.size();
    for (const auto& r : rs->rules) {
      xoff.push_back((uint32_t)xprog.size());
      for (int x : r.exclude) xprog.push_back((uint32_t)x);
      im.max_x = std::max<uint32_t>(im.max_x, (uint32_t)r.exclude.size());
    }
    xoff.push_back((uint32_t)xprog.size());
    std::vector<uint32_t> gx(rs->global_exclude.begin(), rs->global_exclude.end());
    im.o_xoff = append(xoff);
    im.o_xprog = append(xprog);
    im.o_gx = append(gx);
    im.n_gx = (uint32_t)gx.size();
  }
  {
    // k_fold_windows items: keywords a fold rune can spell (İ -> i, K -> k in
    // bytes.ToLower) and anchor literals with a case-free k / s ((?i) K, ſ)
    std::vector<uint32_t> fold;
    for (size_t pi = 0; pi < rs->patterns.size(); ++pi) {
      const PatternHost& p = rs->patterns[pi];
      if (p.special) continue;
      const bool gate = p.kw >= 0 && p.lower.find_first_of("ik") != std::string::npos;
      bool hit = !p.rules.empty() && !rs->ac.fast.empty() && rs->ac.fast_ext[pi] > 0;
      if (!p.rules.empty())
        for (size_t j = 0; j < p.lower.size(); ++j)
          hit |= (p.lower[j] == 'k' || p.lower[j] == 's') && (!p.confirm || p.req[j] == 0);
      if (gate || hit) fold.push_back((uint32_t)pi | (gate ? kFoldItemGate : 0u) | (hit ? kFoldItemHit : 0u));
    }
    im.o_fold = append(fold);
    im.n_fold_items = (uint32_t)fold.size();
  }
  {  // path-regex MatchString DFAs (k_path_gate): kPathDfaRec u32 per program
    std::vector<uint32_t> pd(rs->regexes.size() * kPathDfaRec, 0);
    for (size_t x = 0; x < rs->path_dfa.size(); ++x) {
      const DfaHost& D = rs->path_dfa[x];
      if (!D.valid) continue;
      if (ddelta.size() & 1) ddelta.push_back(0);
      uint32_t* q = pd.data() + x * kPathDfaRec;
      q[0] = (uint32_t)ddelta.size();
      q[1] = D.ncls;
      q[2] = (uint32_t)dbytes.size();
      dbytes.insert(dbytes.end(), D.cls, D.cls + 128);
      dbytes.insert(dbytes.end(), D.match.begin(), D.match.end());
      q[3] = D.start[0];
      q[4] = D.start[1];
      q[5] = (D.match[D.start[0]] ? 1u : 0u) | (D.match[D.start[1]] ? 2u : 0u);
      q[6] = D.sym_base | (D.na_ok ? 0x80000000u : 0u);
      q[7] = 1;
      ddelta.insert(ddelta.end(), D.delta.begin(), D.delta.end());
    }
    im.o_pdfa = (uint32_t)u32.size();
    u32.insert(u32.end(), pd.begin(), pd.end());
  }
  HIP_TRY(im.u32.ensure(u32.size() + 1));
  if (!u32.empty()) HIP_TRY(hipMemcpy(im.u32.p, u32.data(), u32.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(im.rules.ensure(rules.size() + 1));
  if (!rules.empty())
    HIP_TRY(hipMemcpy(im.rules.p, rules.data(), rules.size() * sizeof(RuleDev), hipMemcpyHostToDevice));
  HIP_TRY(im.follow_delta.ensure(fdelta.size() + 1));
  if (!fdelta.empty())
    HIP_TRY(hipMemcpy(im.follow_delta.p, fdelta.data(), fdelta.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(im.dfa_delta.ensure(ddelta.size() + 1));
  if (!ddelta.empty())
    HIP_TRY(hipMemcpy(im.dfa_delta.p, ddelta.data(), ddelta.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(im.dfa_bytes.ensure(dbytes.size() + 1));
  if (!dbytes.empty()) HIP_TRY(hipMemcpy(im.dfa_bytes.p, dbytes.data(), dbytes.size(), hipMemcpyHostToDevice));
  HIP_TRY(im.nfa.ensure(nbytes.size() + 16));
  if (!nbytes.empty()) HIP_TRY(hipMemcpy(im.nfa.p, nbytes.data(), nbytes.size(), hipMemcpyHostToDevice));
  HIP_TRY(im.follow_cls.ensure(fcls.size() + 1));
  if (!fcls.empty()) HIP_TRY(hipMemcpy(im.follow_cls.p, fcls.data(), fcls.size(), hipMemcpyHostToDevice));
  HIP_TRY(im.rule_path.ensure(rule_path.size() + 1));
  if (!rule_path.empty())
    HIP_TRY(hipMemcpy(im.rule_path.p, rule_path.data(), rule_path.size() * 4, hipMemcpyHostToDevice));
  // ---- automaton
  const AcHost& ac = rs->ac;
  HIP_TRY(im.delta.ensure(ac.delta.size()));
  HIP_TRY(hipMemcpy(im.delta.p, ac.delta.data(), ac.delta.size() * 2, hipMemcpyHostToDevice));
  HIP_TRY(im.cls.ensure(256));
  HIP_TRY(hipMemcpy(im.cls.p, ac.cls, 256, hipMemcpyHostToDevice));
  // k_scan_big blob: only for an automaton that neither k_scan_fast's image
  // nor an LDS table holds (see BigDev); the most dense rows that fit
  im.big_view = BigDev{};
  if (needs_big_blob(ac)) {
    BigBlobHost bb;
    if (build_big_blob(ac, experiment_env("TSG_BIG_BFS") != nullptr, &bb)) {
      const std::string why = validate_big_blob(bb, ac.nclasses, ac.nstates);
      if (!why.empty()) {  // never launch a walk that might not end
        set_last_error("k_scan_big automaton blob is malformed: " + why);
        return TSG_ERR_INTERNAL;
      }
      HIP_TRY(im.big.ensure(bb.blob.size()));
      HIP_TRY(hipMemcpy(im.big.p, bb.blob.data(), bb.blob.size(), hipMemcpyHostToDevice));
      HIP_TRY(im.big_ac_of.ensure(bb.ac_of.size()));
      HIP_TRY(hipMemcpy(im.big_ac_of.p, bb.ac_of.data(), bb.ac_of.size() * 2, hipMemcpyHostToDevice));
      im.big_view = BigDev{im.big.p, (uint32_t)bb.blob.size(), bb.nd, bb.cold, bb.o_cold, bb.o_eval, bb.lds_bytes,
                           bb.cold_lds, im.big_ac_of.p};
    }
  }
  HIP_TRY(im.out_off.ensure(ac.out_off.size()));
  HIP_TRY(hipMemcpy(im.out_off.p, ac.out_off.data(), ac.out_off.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(im.out_pat.ensure(ac.out_pat.size() + 1));
  if (!ac.out_pat.empty())
    HIP_TRY(hipMemcpy(im.out_pat.p, ac.out_pat.data(), ac.out_pat.size() * 2, hipMemcpyHostToDevice));
  std::vector<PatDev> pats;
  std::vector<uint8_t> pbytes;
  std::vector<uint32_t> prules;
  for (auto& p : rs->patterns) {
    PatDev d{};
    d.len = (uint32_t)p.lower.size();
    d.kw = p.kw >= 0 ? (uint32_t)p.kw : kNoKw;
    d.bytes_off = (uint32_t)pbytes.size();
    pbytes.insert(pbytes.end(), p.lower.begin(), p.lower.end());
    d.req_off = (uint32_t)pbytes.size();
    pbytes.insert(pbytes.end(), p.req.begin(), p.req.end());
    d.rule_off = (uint32_t)prules.size();
    prules.insert(prules.end(), p.rules.begin(), p.rules.end());
    d.rule_n = (uint32_t)p.rules.size();
    d.special = p.special;
    d.confirm = p.confirm;
    d.kw_needed = p.kw >= 0 && kw_needed_ids.count((uint32_t)p.kw);
    d.trunc = p.lower.size() > (size_t)ac.depth;
    d.ext = ac.fast.empty() ? 0 : ac.fast_ext[pats.size()];
    {
      // window = the 8 bytes ending at the automaton's output byte: the
      // literal sits `ext` class positions before it
      const size_t tl = std::min<size_t>(p.lower.size(), ac.depth);
      for (size_t k = 0; k < tl; ++k) {
        const int sh = 8 * (int)(8 - d.ext - tl + k);
        d.lo64 |= (uint64_t)(uint8_t)p.lower[k] << sh;
        d.m64 |= 0xFFull << sh;
        if (p.confirm && p.req[k]) {
          d.rq64 |= (uint64_t)(uint8_t)p.req[k] << sh;
          d.rqm64 |= 0xFFull << sh;
        }
      }
    }
    pats.push_back(d);
  }
  HIP_TRY(im.pats.ensure(pats.size() + 1));
  HIP_TRY(hipMemcpy(im.pats.p, pats.data(), pats.size() * sizeof(PatDev), hipMemcpyHostToDevice));
  HIP_TRY(im.pat_bytes.ensure(pbytes.size() + 1));
  if (!pbytes.empty()) HIP_TRY(hipMemcpy(im.pat_bytes.p, pbytes.data(), pbytes.size(), hipMemcpyHostToDevice));
  HIP_TRY(im.pat_rules.ensure(prules.size() + 1));
  if (!prules.empty())
    HIP_TRY(hipMemcpy(im.pat_rules.p, prules.data(), prules.size() * 4, hipMemcpyHostToDevice));
  // ---- path literal automaton (k_path_gate)
  im.pac_bytes = 0;
  {
    std::vector<uint32_t> pprogs(rs->global_allow_path.begin(), rs->global_allow_path.end());
    for (auto& r : rs->rules) {
      if (r.path >= 0) pprogs.push_back((uint32_t)r.path);
      for (int x : r.allow_path) pprogs.push_back((uint32_t)x);
    }
    std::sort(pprogs.begin(), pprogs.end());
    pprogs.erase(std::unique(pprogs.begin(), pprogs.end()), pprogs.end());
    if (!pprogs.empty() && pprogs.size() <= 64) {
      std::vector<uint8_t> bit(rs->regexes.size(), 0xFF);
      uint64_t always = 0;
      std::vector<std::string> lit_lower, lit_req;
      std::vector<uint32_t> lit_bit;
      for (size_t i = 0; i < pprogs.size(); ++i) {
        bit[pprogs[i]] = (uint8_t)i;
        const gre::Anchor& a = rs->regexes[pprogs[i]].c.anchor;
        bool ascii = a.valid && a.lits.size() <= 32;
        for (auto& l : a.lits)
          for (unsigned char c : l.lower) ascii &= c < 0x80 && c != 0;
        if (!ascii) {
          always |= 1ull << i;
          continue;
        }
        for (auto& l : a.lits) {
          lit_lower.push_back(l.lower);
          lit_req.push_back(l.req);
          lit_bit.push_back((uint32_t)i);
        }
      }
      // trie over lowercased literals; classes: literal bytes, 'A'-'Z' share lower case
      int cmap[256] = {0};
      int K = 1;
      for (auto& l : lit_lower)
        for (unsigned char c : l)
          if (!cmap[c]) cmap[c] = K++;
      for (int b = 'A'; b <= 'Z'; ++b) cmap[b] = cmap[b + 32];
      std::vector<std::vector<int>> go(1, std::vector<int>(K, -1));
      std::vector<std::vector<uint16_t>> term(1);
      for (size_t li = 0; li < lit_lower.size(); ++li) {
        int st = 0;
        for (unsigned char c : lit_lower[li]) {
          const int k = cmap[c];
          if (go[st][k] < 0) {
            go[st][k] = (int)go.size();
            go.emplace_back(K, -1);
            term.emplace_back();
          }
          st = go[st][k];
        }
        term[st].push_back((uint16_t)li);
      }
      const int S = (int)go.size();
      std::vector<int> fail(S, 0);
      std::vector<std::vector<uint16_t>> outs(S);
      std::deque<int> q;
      for (int k = 0; k < K; ++k) {
        if (go[0][k] < 0) go[0][k] = 0;
        else q.push_back(go[0][k]);
      }
      while (!q.empty()) {
        const int st = q.front();
        q.pop_front();
        outs[st] = term[st];
        for (auto x : outs[fail[st]]) outs[st].push_back(x);
        for (int k = 0; k < K; ++k) {
          const int t2 = go[st][k];
          if (t2 >= 0) {
            fail[t2] = go[fail[st]][k];
            q.push_back(t2);
          } else {
            go[st][k] = go[fail[st]][k];
          }
        }
      }
      if (S < 32768 && lit_lower.size() < 65536) {
        std::vector<uint8_t> blob;
        auto put = [&](const void* p, size_t n) {
          blob.resize((blob.size() + 15) & ~(size_t)15);
          const uint32_t o = (uint32_t)blob.size();
          blob.insert(blob.end(), (const uint8_t*)p, (const uint8_t*)p + n);
          return o;
        };
        std::vector<uint16_t> delta((size_t)S * K);
        for (int st = 0; st < S; ++st)
          for (int k = 0; k < K; ++k) {
            const int t2 = go[st][k];
            delta[(size_t)st * K + k] = (uint16_t)(t2 | (outs[t2].empty() ? 0 : 0x8000));
          }
        put(delta.data(), delta.size() * 2);
        uint8_t cl[256];
        for (int b = 0; b < 256; ++b) cl[b] = (uint8_t)cmap[b];
        im.o_pac_cls = put(cl, 256);
        std::vector<uint32_t> ooff(S + 1, 0);
        std::vector<uint16_t> oo;
        for (int st = 0; st < S; ++st) {
          ooff[st] = (uint32_t)oo.size();
          oo.insert(oo.end(), outs[st].begin(), outs[st].end());
        }
        ooff[S] = (uint32_t)oo.size();
        im.o_pac_out_off = put(ooff.data(), ooff.size() * 4);
        im.o_pac_out = put(oo.data(), oo.size() * 2 + 2);
        std::vector<uint8_t> reqb;
        std::vector<PacLit> pls;
        for (size_t li = 0; li < lit_lower.size(); ++li) {
          pls.push_back(PacLit{lit_bit[li], (uint32_t)lit_lower[li].size(), (uint32_t)reqb.size()});
          reqb.insert(reqb.end(), lit_req[li].begin(), lit_req[li].end());
        }
        im.o_pac_lits = put(pls.data(), pls.size() * sizeof(PacLit) + 4);
        im.o_pac_req = put(reqb.data(), reqb.size() + 1);
        im.o_pac_bit = put(bit.data(), bit.size());
        blob.resize((blob.size() + 15) & ~(size_t)15);
        HIP_TRY(im.pac.ensure(blob.size()));
        HIP_TRY(hipMemcpy(im.pac.p, blob.data(), blob.size(), hipMemcpyHostToDevice));
        im.pac_bytes = (uint32_t)blob.size();
        im.pac_states = (uint32_t)S;
        im.pac_classes = (uint32_t)K;
        im.pac_always = always;
        im.pac_prog_bit = bit;
      }
    }
  }
  // ---- view
  RuleSetDev& v = im.view;
  v.follow_delta = im.follow_delta.p;
  v.follow_cls = im.follow_cls.p;
  v.dfa_delta = im.dfa_delta.p;
  v.dfa_bytes = im.dfa_bytes.p;
  v.nfa_bytes = im.nfa.p;
  v.progs = im.progs.p;
  v.prog_lit_off = im.prog_lit_off.p;
  v.prog_lits = im.prog_lits.p;
  v.rules = im.rules.p;
  v.kw_ids = im.u32.p + o_kw;
  v.group_slots = im.u32.p + o_gs;
  v.allow_progs = im.u32.p + o_ap;
  v.global_allow = im.u32.p + o_ga;
  v.n_global_allow = (uint32_t)gallow.size();
  v.pdfa = im.u32.p + im.o_pdfa;
  v.n_rules = (uint32_t)rs->rules.size();
  v.kw_words = std::max<uint32_t>(1, ((uint32_t)rs->keywords.size() + 31) / 32);
  v.max_ninst = max_ninst;
  v.max_ncap = max_ncap;
  v.max_ninst_cap = max_ninst_cap;
  const uint8_t* fast = nullptr;
  uint32_t o_out_off = 0, o_out_pat = 0, o_pats = 0, o_pbytes = 0, rep_bytes = 0, o_pair = 0, o_fkw = 0;
  if (!ac.fast.empty()) {
    // k_report blob: the scan image followed by the small output tables
    std::vector<uint8_t> blob(ac.fast.begin(), ac.fast.end());
    auto put = [&](const void* p, size_t n) {
      blob.resize((blob.size() + 15) & ~(size_t)15);
      const uint32_t o = (uint32_t)blob.size();
      blob.insert(blob.end(), (const uint8_t*)p, (const uint8_t*)p + n);
      return o;
    };
    o_out_off = put(ac.fast_out_off.data(), ac.fast_out_off.size() * 4);
    o_out_pat = put(ac.fast_out_pat.data(), ac.fast_out_pat.size() * 2);
    o_pats = put(pats.data(), pats.size() * sizeof(PatDev));
    o_pbytes = put(pbytes.data(), pbytes.size());
    blob.resize((blob.size() + 15) & ~(size_t)15);
    rep_bytes = (uint32_t)blob.size();  // (k_report stages [0, rep_bytes); the pair table follows)
    if (!ac.fast_pair.empty()) o_pair = put(ac.fast_pair.data(), ac.fast_pair.size() * 2);
    // the keyword states' records and the local bits' keyword ids (k_scan_fast stages them in LDS)
    o_fkw = put(ac.fast_kw.data(), ac.fast_kw.size());
    std::vector<uint16_t> kw_map(ac.fast_kw_map);
    kw_map.resize(kFastKwBits, 0);  // (the scan stages all kFastKwBits entries)
    put(kw_map.data(), kw_map.size() * 2);
    HIP_TRY(im.fast.ensure(blob.size() + 16));
    HIP_TRY(hipMemcpy(im.fast.p, blob.data(), blob.size(), hipMemcpyHostToDevice));
    fast = im.fast.p;
  }
  v.ac = AcDev{im.delta.p, im.cls.p, im.out_off.p, im.out_pat.p, im.pats.p, im.pat_bytes.p, im.pat_rules.p,
               ac.nstates, ac.nclasses, fast, (uint32_t)ac.fast.size(), ac.fast_out_entry,
               fast ? ac.fast_ev_entry : ac.fast_out_entry, fast ? ac.fast_ev_entry - ac.fast_out_entry : 0u,
               fast ? fast + o_fkw : nullptr, ac.depth, rep_bytes, o_out_off, o_out_pat, o_pats, o_pbytes, o_pair};
  // keywords whose lowercase holds a non-ASCII rune (k_uni_keywords)
  {
    std::vector<uint8_t> ub;
    std::vector<uint32_t> um;
    uint32_t max_len = 0;
    for (size_t k = 0; k < rs->keywords.size(); ++k) {
      if (!rs->kw_uni[k]) continue;
      um.push_back((uint32_t)ub.size());
      um.push_back((uint32_t)rs->keywords[k].size());
      um.push_back((uint32_t)k);
      ub.insert(ub.end(), rs->keywords[k].begin(), rs->keywords[k].end());
      max_len = std::max<uint32_t>(max_len, (uint32_t)rs->keywords[k].size());
    }
    im.n_uni = (uint32_t)(um.size() / 3);
    // an occurrence in the content is at most 4 bytes per keyword rune (a lone
    // invalid byte lowers to the 3-byte U+FFFD): <= 4 * its byte length
    im.uni_back = 4 * max_len;
    if (im.n_uni) {
      HIP_TRY(im.uni_bytes.ensure(ub.size() + 1));
      HIP_TRY(im.uni_meta.ensure(um.size() + 1));
      HIP_TRY(im.lower_map.ensure(2 * kLowerMapLen + 2));
      HIP_TRY(hipMemcpy(im.uni_bytes.p, ub.data(), ub.size(), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(im.uni_meta.p, um.data(), um.size() * 4, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(im.lower_map.p, kLowerMap, sizeof(kLowerMap), hipMemcpyHostToDevice));
    }
  }
  im.rs_id = rs->id;
  // VM scratch
  e->scratch_stride = (scratch_bytes(max_ninst, max_ncap, max_ninst_cap) + 255) & ~255ull;
  return TSG_OK;
}


// Ablation / diagnostic switches: read only in a
// -DTSG_EXPERIMENTS build; the product library ignores the environment.
inline const char* experiment_env(const char* name) {
#ifdef TSG_EXPERIMENTS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// Sort n (key, value) pairs by key bits [0, end_bit), stable, kin/vin ->
// kout/vout (distinct buffers): hipcub::DeviceRadixSort::SortPairs, or with
// `small` (TSG_SORT_SMALL in the exp build; tsg_diag_sort_pairs) the two
// launches k_tile_sort + k_tile_merge up to kSortSmall pairs.  Measured on
// configs[2] (profiles/r06r): 45 + 23 us per 34 K-pair sort against ~25 us
// for hipcub's cascade unprofiled (sort_jobs 0.102 vs 0.078 ms, lines 0.98 vs
// 0.89 ms, step +0.06 ms over two alternating runs): the LDS bitonic's 78
// stages and the merge's 13 dependent L2 levels cost more than the ~8 launches
// they replace, so the product keeps hipcub.
hipError_t sort_pairs(tsg_engine* e, const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, int end_bit, hipStream_t s, bool small = false) {
  if (!n) return hipSuccess;
  if (n <= kSortSmall && (small || experiment_env("TSG_SORT_SMALL"))) {
    hipError_t r = e->ss_key.ensure(kSortSmall);
    if (r == hipSuccess) r = e->ss_idx.ensure(kSortSmall);
    if (r != hipSuccess) return r;
    const uint64_t mask = end_bit >= 64 ? ~0ull : (1ull << end_bit) - 1;
    const uint32_t nt = (uint32_t)((n + kSortTile - 1) / kSortTile);
    hipLaunchKernelGGL(k_tile_sort, dim3(nt), dim3(1024), 0, s, kin, n, mask, e->ss_key.p, e->ss_idx.p);
    hipLaunchKernelGGL(k_tile_merge, dim3(nt * kSortTile / 256), dim3(256), 0, s, kin, vin, n, e->ss_key.p,
                       e->ss_idx.p, nt, kout, vout);
    return hipGetLastError();
  }
  size_t tmp = 0;
  hipError_t r = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, (int)n, 0, end_bit, s);
  if (r == hipSuccess) r = e->cub_tmp.ensure(tmp + 1);
  if (r == hipSuccess) r = hipcub::DeviceRadixSort::SortPairs(e->cub_tmp.p, tmp, kin, kout, vin, vout, (int)n, 0, end_bit, s);
  return r;
}

// The side stream (D2H of the findings, the phase-0 newline count) and its events.
hipError_t ensure_side(tsg_engine* e) {
  if (e->side) return hipSuccess;
  // (a lowest-priority side stream left k_verify as slow under the phase-0
  // newline count: 0.74 vs 0.76 ms, profiles/r04v)
  hipError_t r = hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_code, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_fill, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_side, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_dense, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_dfill, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_frec, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_fb, hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_nl[0], hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreateWithFlags(&e->ev_nl[1], hipEventDisableTiming);
  if (r == hipSuccess) r = hipEventCreate(&e->ev_pg[0]);  // (timed: the path gate's stage time)
  if (r == hipSuccess) r = hipEventCreate(&e->ev_pg[1]);
  return r;
}

// D2H on a DMA engine (hsa_amd_memory_async_copy), ordered by the caller
// (the source is complete when it is issued).  hipMemcpyAsync runs a D2H into
// page-locked memory as blit kernels on the CUs: the ~200 MB dense region's
// copy beside k_find_spans made that kernel 1.9 -> 5.8 ms (profiles/r05i).
// false: not issued (the caller copies with hipMemcpyAsync).
hsa_status_t find_cpu_agent(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *(hsa_agent_t*)out = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
bool dma_d2h(tsg_engine* e, void* dst, const void* src, size_t n) {
  if (experiment_env("TSG_DMA_OFF")) return false;  // (A/B: blit copies)
  static hsa_agent_t cpu{0};
  static std::once_flag once;
  std::call_once(once, [] { (void)hsa_iterate_agents(find_cpu_agent, &cpu); });
  if (!cpu.handle) return false;
  if (!e->dma_sig.handle && hsa_signal_create(1, 0, nullptr, &e->dma_sig) != HSA_STATUS_SUCCESS) return false;
  hsa_amd_pointer_info_t pd{};
  pd.size = sizeof(pd);
  if (hsa_amd_pointer_info(src, &pd, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
      pd.type == HSA_EXT_POINTER_TYPE_UNKNOWN)
    return false;
  // one signal counts the call's copies down (each completion subtracts 1)
  if (e->dma_pending) hsa_signal_add_screlease(e->dma_sig, 1);
  else hsa_signal_store_screlease(e->dma_sig, 1);
  if (hsa_amd_memory_async_copy(dst, cpu, src, pd.agentOwner, n, 0, nullptr, e->dma_sig) != HSA_STATUS_SUCCESS) {
    if (e->dma_pending) hsa_signal_subtract_screlease(e->dma_sig, 1);
    return false;
  }
  e->dma_pending = true;
  return true;
}
// Waits for the call's dma_d2h copies (every exit of a call that issued one).
int dma_wait(tsg_engine* e) {
  if (!e->dma_pending) return TSG_OK;
  const hsa_signal_value_t v =
      hsa_signal_wait_scacquire(e->dma_sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  e->dma_pending = false;
  if (v < 0) {
    set_last_error("a DMA copy of the findings failed");
    return TSG_ERR_DEVICE;
  }
  return TSG_OK;
}
struct DmaGuard {  // (the copy's destination belongs to the result: never outlive the call)
  tsg_engine* e;
  ~DmaGuard() { (void)dma_wait(e); }
};

int read_ctrl(tsg_engine* e, Ctrl* h) {
  HIP_TRY(hipMemcpyAsync(h, e->ctrl.p, sizeof(Ctrl), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return TSG_OK;
}

// Launch the AC pass: k_scan_fast when the automaton fits its LDS image,
// else the generic kernel (transition table in LDS or, if too large, global).
int launch_scan(tsg_engine* e, ScanParams& P, bool kw_mid = false) {
  hipStream_t s = e->stream;
  bool nl_skipped = false;
  P.n_regions = P.nbytes / kNlBlock + 1;
  HIP_TRY(e->region_file.ensure(P.n_regions + 1));
  P.region_file = e->region_file.p;
  if (P.n_files) {
    hipLaunchKernelGGL(k_region_fill, dim3((P.n_files + 255) / 256), dim3(256), 0, s, P.off, P.n_files, P.n_regions,
                       e->region_file.p, P.ctrl);
    HIP_TRY(hipGetLastError());
  }
  if (!e->num_cus) {
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, e->device));
    e->num_cus = (uint32_t)prop.multiProcessorCount;
  }
  const AcDev& ac = P.rs.ac;
  if (ac.fast_lds) {
    // final partial region: zero-padded copy (with 8 bytes of warm-up context)
    // product shape: one chain per lane, 8 x 16-byte vectors per chain step,
    // one event check per kFastEventWin groups.  The other shapes, ablation
    // modes and event windows (all measured slower; modes give
    // wrong results) exist only in a -DTSG_EXPERIMENTS build.
    int chains = kFastChains;
    [[maybe_unused]] int vecs = kFastVecs;
    bool ring = false;
#ifdef TSG_EXPERIMENTS
    int deep_v = 0, deep_d = 0;  // TSG_FAST_VARIANT=d<V>x<D>: k_scan_deep
    int mode = 0;                // TSG_SCAN_MODE: timing experiments only (see fast_group)
    if (const char* m = getenv("TSG_SCAN_MODE")) mode = atoi(m);
    int win = kFastEventWin;     // groups per event check (fast_window; A/B via TSG_EVENT_WIN)
    if (const char* w = getenv("TSG_EVENT_WIN")) win = atoi(w);
    bool pair = false;  // TSG_FAST_VARIANT=pair: root pair table (fstep2)
    if (const char* v = getenv("TSG_FAST_VARIANT")) {
      pair = strcmp(v, "pair") == 0;
      if (pair) {
      } else if (sscanf(v, "d%dx%d", &deep_v, &deep_d) != 2) {
        deep_v = 0;
        ring = sscanf(v, "%dx%d", &chains, &vecs) != 2;
      }
    }
    if (!((chains == 1 && (vecs == 8 || vecs == 4)) || (chains == 2 && (vecs == 4 || vecs == 2)))) {
      chains = kFastChains;
      vecs = kFastVecs;
    }
#endif
    // the scan resolving its own events (kFuse) measured slower: 14.4 ms for
    // the fused scan against 10.7 + 0.64 (k_report) on configs[2], 13.9 ms with
    // the resolution after each wave's last span only (profiles/r05c) -- the
    // out-of-line resolution's call frame and spills sit on the streaming
    // loop, and inlined (128 VGPRs) it cost 11.5 ms (profiles/r05b).  Exp
    // build only (TSG_FUSE=1).
    bool fuse = false;
#ifdef TSG_EXPERIMENTS
    if (const char* f = getenv("TSG_FUSE")) fuse = ac.rep_bytes <= kReportLds && atoi(f) != 0;
#endif
    const uint64_t unit = ring ? (uint64_t)kNlBlock : (uint64_t)chains * kNlBlock;
    P.tail_base = (P.nbytes / unit) * unit;
    const uint64_t lead = P.tail_base >= 8 ? 8 : P.tail_base;
    HIP_TRY(e->tail.ensure(8 + kFastUnitMax + 64));
    HIP_TRY(hipMemsetAsync(e->tail.p, 0, 8 + kFastUnitMax + 64, s));
    if (P.nbytes - P.tail_base + lead)
      HIP_TRY(hipMemcpyAsync(e->tail.p + 8 - lead, P.data + P.tail_base - lead, P.nbytes - P.tail_base + lead,
                             hipMemcpyDeviceToDevice, s));
    P.tail = e->tail.p + 8 - P.tail_base;
    const uint64_t units = (P.nbytes + unit - 1) / unit;
    const uint64_t n_spans = (P.nbytes + kNlBlock - 1) / kNlBlock;
    HIP_TRY(e->span_hi.ensure(n_spans + 1));
    P.span_hi = e->span_hi.p;
    // 1024 threads, one block per CU (the image takes most of the LDS)
    const uint32_t nt = 1024;
    const uint32_t per_cu = 1;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((units + nt - 1) / nt, (uint64_t)e->num_cus * per_cu));
    // per-wave event segments (an output group per ~KiB of source text; 4x headroom)
    const uint64_t n_waves = (uint64_t)blocks * (nt / 64);
    P.ev_cap_per_wave = std::max<uint64_t>(1024, (P.nbytes / 256) / n_waves + 256);
    HIP_TRY(e->ev_buf.ensure(n_waves * P.ev_cap_per_wave));
    HIP_TRY(e->ev_counts.ensure(n_waves + 1));
    HIP_TRY(e->ev_overflow.ensure(std::max<uint64_t>(1 << 20, e->ev_ovf_need)));
    P.events = e->ev_buf.p;
    P.ev_counts = e->ev_counts.p;
    P.ev_overflow = e->ev_overflow.p;
    P.ev_overflow_cap = e->ev_overflow.n;
    HIP_TRY(hipMemsetAsync(&P.ctrl->ev_overflow, 0, 8, s));
    // (the image lives in the kernel's static kFastImgMax array: no dynamic LDS)
    if (e->events) HIP_TRY(hipEventRecord(e->ev[10], s));
#ifdef TSG_EXPERIMENTS
    bool fused = false;  // (only the product shape has a fused instantiation)
    if (ring) hipLaunchKernelGGL(k_scan_ring, dim3(blocks), dim3(nt), 0, s, P);
#define TSG_DEEP(VV, DD, M)                                                                 \
  else if (deep_v == VV && deep_d == DD && mode == M)                                      \
      hipLaunchKernelGGL((k_scan_deep<VV, DD, 1024, M>), dim3(blocks), dim3(nt), 0, s, P);
    TSG_DEEP(8, 1, 0) TSG_DEEP(4, 3, 0) TSG_DEEP(4, 1, 0) TSG_DEEP(2, 3, 0)
#undef TSG_DEEP
    else if (mode == 8) hipLaunchKernelGGL(k_scan_tri, dim3(blocks), dim3(nt), 0, s, P);  // trigram filter timing bound
#define TSG_MODE(M) \
  else if (chains == 1 && vecs == 8 && mode == M) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, M>), dim3(blocks), dim3(nt), 0, s, P);
    TSG_MODE(1) TSG_MODE(2) TSG_MODE(3) TSG_MODE(4) TSG_MODE(5) TSG_MODE(6) TSG_MODE(7)
#undef TSG_MODE
    else if (chains == 1 && vecs == 8 && win == 2) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 0, 2>), dim3(blocks), dim3(nt), 0, s, P);
    else if (chains == 1 && vecs == 8 && win == 8) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 0, 8>), dim3(blocks), dim3(nt), 0, s, P);
    else if (chains == 1 && vecs == 8 && win == 4 && pair && P.rs.ac.o_pair)
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 0, 4, true>), dim3(blocks), dim3(nt), 0, s, P);
    else if (chains == 1 && vecs == 8 && win == 4 && e->nl_lazy && fuse) {
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2, 4, false, true>), dim3(blocks), dim3(nt), 0, s, P);
      nl_skipped = true;
      fused = true;
    }
    else if (chains == 1 && vecs == 8 && win == 4 && e->nl_lazy && kw_mid) {
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2 | kScanKwMid, 4>), dim3(blocks), dim3(nt), 0, s, P);
      nl_skipped = true;
    }
    else if (chains == 1 && vecs == 8 && win == 4 && e->nl_lazy) {
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2, 4>), dim3(blocks), dim3(nt), 0, s, P);
      nl_skipped = true;
    }
    else if (chains == 1 && vecs == 8 && win == 4) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 0, 4>), dim3(blocks), dim3(nt), 0, s, P);
    else if (chains == 1 && vecs == 8) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024>), dim3(blocks), dim3(nt), 0, s, P);
    else if (chains == 1) hipLaunchKernelGGL((k_scan_fast<1, 4, 1024>), dim3(blocks), dim3(nt), 0, s, P);
    else if (vecs == 4) hipLaunchKernelGGL((k_scan_fast<2, 4, 1024>), dim3(blocks), dim3(nt), 0, s, P);
    else hipLaunchKernelGGL((k_scan_fast<2, 2, 1024>), dim3(blocks), dim3(nt), 0, s, P);
    fuse = fused;
#else
    // (kMode 2: no newline counts -- the engine counts them lazily, k_nl_spans)
    // (kw_mid: the prefilter-only scan, whose outputs are all keywords;
    // kScanNoCount: no span of this batch is counted in the scan, so the
    // kernel carries no count code -- its per-group test cost ~1.6 % of the
    // scan, configs[2] 11.97 -> 11.78 ms over three alternating runs,
    // profiles/r06zq_c2)
    if (e->nl_lazy && kw_mid && !P.nl_big)
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2 | kScanKwMid | kScanNoCount, kFastEventWin>), dim3(blocks), dim3(nt), 0,
                         s, P);
    else if (e->nl_lazy && kw_mid)
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2 | kScanKwMid, kFastEventWin>), dim3(blocks), dim3(nt), 0, s, P);
    else if (e->nl_lazy && !P.nl_big)
      hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2 | kScanNoCount, kFastEventWin>), dim3(blocks), dim3(nt), 0, s, P);
    else if (e->nl_lazy) hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 2, kFastEventWin>), dim3(blocks), dim3(nt), 0, s, P);
    else hipLaunchKernelGGL((k_scan_fast<1, 8, 1024, 0, kFastEventWin>), dim3(blocks), dim3(nt), 0, s, P);
    nl_skipped = e->nl_lazy;
#endif
    HIP_TRY(hipGetLastError());
    if (e->events) HIP_TRY(hipEventRecord(e->ev[11], s));
    e->fast_timed = e->events;
    // the wave segments (unless the scan resolved them) and the overflow bucket
    // (with n_waves 0, k_report returns at once when the bucket is empty);
    // each report wave stages its hits in a region of its own, packed into
    // P.hits afterwards with one reservation
    const uint32_t rep_blocks = (uint32_t)std::min<uint64_t>(fuse ? 1 : n_waves + 1, e->num_cus);
    const uint32_t n_rw = rep_blocks * (kReportThreads / 64);
    P.hit_seg_cap = kHitSegCap;
    HIP_TRY(e->hit_seg.ensure((uint64_t)n_rw * kHitSegCap));
    HIP_TRY(e->hit_seg_n.ensure(n_rw));
    HIP_TRY(e->hit_pre.ensure(n_rw + 1));
    P.hit_seg = e->hit_seg.p;
    P.hit_seg_n = e->hit_seg_n.p;
    HIP_TRY(hipMemsetAsync(e->hit_seg_n.p, 0, (size_t)n_rw * 4, s));
    if (!fuse) {  // the events' index space: exclusive prefix of the segments' counts
      HIP_TRY(e->ev_pre.ensure(n_waves + 1));
      HIP_TRY(hipMemsetAsync(e->ev_counts.p + n_waves, 0, 4, s));
      size_t tmp = 0;
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->ev_counts.p, e->ev_pre.p, (int)(n_waves + 1), s));
      HIP_TRY(e->cub_tmp.ensure(tmp + 1));
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->ev_counts.p, e->ev_pre.p, (int)(n_waves + 1), s));
    }
    hipLaunchKernelGGL(k_report, dim3(rep_blocks), dim3(kReportThreads), 0, s, P, fuse ? 0u : (uint32_t)n_waves,
                       (const uint64_t*)e->ev_pre.p);
    HIP_TRY(hipGetLastError());
    {
      size_t tmp = 0;
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->hit_seg_n.p, e->hit_pre.p, (int)n_rw, s));
      HIP_TRY(e->cub_tmp.ensure(tmp + 1));
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->hit_seg_n.p, e->hit_pre.p, (int)n_rw, s));
      unsigned long long* base = (unsigned long long*)(e->hit_pre.p + n_rw);
      hipLaunchKernelGGL(k_hits_reserve, dim3(1), dim3(1), 0, s, P, n_rw, e->hit_pre.p, base);
      hipLaunchKernelGGL(k_hits_pack, dim3(n_rw), dim3(256), 0, s, P, e->hit_pre.p, base);
      HIP_TRY(hipGetLastError());
    }
    P.hit_seg = nullptr;  // (the later passes reserve on ctrl->hits)
    hipLaunchKernelGGL(k_fold_special, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_spans + 255) / 256, 2048))),
                       dim3(256), 0, s, P, n_spans);
  } else if (P.big.blob && !experiment_env("TSG_NO_BIG")) {
    // k_scan_fast's span / tail / event layout (one 4 KiB span per lane)
    const uint32_t nt = kBigThreads;
    P.tail_base = (P.nbytes / kNlBlock) * kNlBlock;
    const uint64_t lead = P.tail_base >= 8 ? 8 : P.tail_base;
    HIP_TRY(e->tail.ensure(8 + kFastUnitMax + 64));
    HIP_TRY(hipMemsetAsync(e->tail.p, 0, 8 + kFastUnitMax + 64, s));
    if (P.nbytes - P.tail_base + lead)
      HIP_TRY(hipMemcpyAsync(e->tail.p + 8 - lead, P.data + P.tail_base - lead, P.nbytes - P.tail_base + lead,
                             hipMemcpyDeviceToDevice, s));
    P.tail = e->tail.p + 8 - P.tail_base;
    const uint64_t units = (P.nbytes + kNlBlock - 1) / kNlBlock;
    HIP_TRY(e->span_hi.ensure(units + 1));
    P.span_hi = e->span_hi.p;
    // one unit per lane: CH spans (kBigChains)
    // (newline counts stay in this kernel: they cost it ~0.1 ms on configs[4],
    // against ~0.9 ms for counting its many location files afterwards --
    // TSG_BIG_VARIANT=40x2v2 skips them, exp build)
    // product: the coalesced whole-line shape, one chain per lane (k_scan_lines;
    // configs[4]: 5.05 ms and 1.006x FETCH against 7.33 ms and 3.63x for the
    // span-per-lane k_scan_big, profiles/r05e_big)
    const void* big_fn = (const void*)k_scan_lines<kBigMode, 1>;
    int big_mode = kBigMode, big_ch = kBigChains;
    int lines = 2;  // 0: k_scan_big (exp: TSG_BIG_VARIANT), 1 / 2: k_scan_lines with 2 / 1 chains
#ifdef TSG_EXPERIMENTS
    int big_v = kBigRing;
    if (const char* v = getenv("TSG_BIG_VARIANT")) {  // "<mode>[x<chains>][v<ring uint4s>]"
      big_mode = atoi(v);
      big_ch = strchr(v, 'x') ? atoi(strchr(v, 'x') + 1) : 1;
      big_v = strchr(v, 'v') ? atoi(strchr(v, 'v') + 1) : 8 / big_ch;
    }
    using BigFn = void (*)(ScanParams);
    struct BigV { int mode, ch, v; BigFn fn; };
    static const BigV kBigVariants[] = {
        {0, 1, 8, k_scan_big<0, 1>},     {1, 1, 8, k_scan_big<1, 1>},     {2, 1, 8, k_scan_big<2, 1>},
        {3, 1, 8, k_scan_big<3, 1>},     {4, 1, 8, k_scan_big<4, 1>},     {0, 2, 4, k_scan_big<0, 2>},
        {8, 2, 4, k_scan_big<8, 2>},     {0, 2, 2, k_scan_big<0, 2, 2>},  {8, 2, 2, k_scan_big<8, 2, 2>},
        {8, 1, 8, k_scan_big<8, 1>},
        {12, 2, 2, k_scan_big<12, 2, 2>}, {2, 2, 2, k_scan_big<2, 2, 2>}, {4, 1, 4, k_scan_big<4, 1, 4>},
        {9, 2, 2, k_scan_big<9, 2, 2>},  {3, 2, 2, k_scan_big<3, 2, 2>},  {24, 2, 2, k_scan_big<24, 2, 2>},
        {25, 2, 2, k_scan_big<25, 2, 2>}, {40, 2, 2, k_scan_big<40, 2, 2>}};
    BigFn pick = nullptr;
    for (const BigV& x : kBigVariants)
      if (x.mode == big_mode && x.ch == big_ch && x.v == big_v) pick = x.fn;
    if (!pick) {
      set_last_error("TSG_BIG_VARIANT: no such k_scan_big instantiation");
      return TSG_ERR_INVALID_ARG;
    }
    if (getenv("TSG_BIG_VARIANT")) {
      big_fn = (const void*)pick;
      nl_skipped = e->nl_lazy && (big_mode & kBigNoNl);
      lines = 0;
    }
    if (const char* v = getenv("TSG_BIG_LINES")) {  // the coalesced whole-line shape: "1" = 2 chains, "2" = 1 chain
      lines = atoi(v);
      if (lines == 1) big_fn = (const void*)k_scan_lines<8, 2>;
      if (lines == 2) big_fn = (const void*)k_scan_lines<8, 1>;
      nl_skipped = false;
    }
#endif
    const uint64_t big_units = lines ? (P.nbytes + 127) / 128 / 64 * 64 : (units + big_ch - 1) / big_ch;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((big_units + nt - 1) / nt, e->num_cus));
    const uint64_t n_waves = (uint64_t)blocks * (nt / 64);
    P.ev_cap_per_wave = std::max<uint64_t>(1024, (P.nbytes / 256) / n_waves + 256);
    HIP_TRY(e->ev_buf.ensure(n_waves * P.ev_cap_per_wave));
    HIP_TRY(e->ev_counts.ensure(n_waves + 1));
    HIP_TRY(e->ev_overflow.ensure(std::max<uint64_t>(1 << 20, e->ev_ovf_need)));
    P.events = e->ev_buf.p;
    P.ev_counts = e->ev_counts.p;
    P.ev_overflow = e->ev_overflow.p;
    P.ev_overflow_cap = e->ev_overflow.n;
    HIP_TRY(hipMemsetAsync(&P.ctrl->ev_overflow, 0, 8, s));
    HIP_TRY(hipFuncSetAttribute(big_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.big.lds_bytes));
    if (e->events) HIP_TRY(hipEventRecord(e->ev[10], s));
    (void)big_mode;
    void* big_args[] = {&P};
    HIP_TRY(hipLaunchKernel(big_fn, dim3(blocks), dim3(nt), big_args, P.big.lds_bytes, s));
    HIP_TRY(hipGetLastError());
    if (e->events) HIP_TRY(hipEventRecord(e->ev[11], s));
    e->fast_timed = e->events;
    HIP_TRY(e->big_outs.ensure(std::max<uint64_t>({1 << 20, P.nbytes / 256, e->big_out_need})));
    P.big_outs = e->big_outs.p;
    P.big_out_cap = e->big_outs.n;
    HIP_TRY(hipFuncSetAttribute((const void*)k_big_walk, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)P.big.lds_bytes));
    hipLaunchKernelGGL(k_big_walk, dim3((uint32_t)std::min<uint64_t>(n_waves + 1, e->num_cus)), dim3(1024),
                       P.big.lds_bytes, s, P, (uint32_t)n_waves);
    hipLaunchKernelGGL(k_big_resolve, dim3(e->num_cus * 8), dim3(kResolveThreads), 0, s, P);
    HIP_TRY(hipGetLastError());
  } else {
    const size_t table_bytes = (size_t)ac.nstates * ac.nclasses * 2;
    const bool lds_table = table_bytes <= (size_t)kLdsTableMax;
    // a table too large for LDS is read from global memory (L2-resident).
    // Measured on configs[4] (6669 states x 46 classes): staging its 445
    // shallowest rows in LDS is slower (46.7 vs 35.8 ms / 10 GB) -- a wave
    // still waits on the rare lane in a deep state at almost every byte, and
    // the LDS halves the blocks per CU.  TSG_GEN_LDS_KB re-enables it for A/B.
    P.gen_lds_rows = lds_table ? ac.nstates : 0;
    if (!lds_table)
      if (const char* kb = experiment_env("TSG_GEN_LDS_KB"))
        P.gen_lds_rows = (uint32_t)std::min<size_t>(ac.nstates, ((size_t)atoi(kb) << 10) / (2u * ac.nclasses));
    const size_t lds = 256 + kTileLds + (size_t)P.gen_lds_rows * ac.nclasses * 2;
    const uint64_t nsteps = (P.nbytes + kBlockBytes - 1) / kBlockBytes;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nsteps, (uint64_t)e->num_cus * 8));
    if (lds_table) {
      HIP_TRY(hipFuncSetAttribute((const void*)k_scan_generic<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(k_scan_generic<true>, dim3(blocks), dim3(kScanThreads), lds, s, P);
    } else {
      HIP_TRY(hipFuncSetAttribute((const void*)k_scan_generic<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(k_scan_generic<false>, dim3(blocks), dim3(kScanThreads), lds, s, P);
    }
  }
  HIP_TRY(hipGetLastError());
  e->nl_deferred = nl_skipped;
  return TSG_OK;
}

// Keywords / anchor literals spelled with fold-special runes, around each of
// the n_fold occurrences the scan recorded (k_fold_windows).
int launch_fold_windows(tsg_engine* e, const ScanParams& P, bool with_hits) {
  const DevImage& im = e->img;
  if (!im.n_fold_items) return TSG_OK;
  const FoldItems F{im.u32.p + im.o_fold, im.n_fold_items, with_hits ? 1u : 0u};
  hipLaunchKernelGGL(k_fold_windows, dim3(std::max(1u, e->num_cus) * 2), dim3(256), 0, e->stream, P, F);
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

// Non-ASCII keyword bits (k_uni_keywords), after the scan flagged its spans.
int launch_uni_keywords(tsg_engine* e, const ScanParams& P) {
  const DevImage& im = e->img;
  if (!im.n_uni || !P.nbytes) return TSG_OK;
  const UniKw U{im.uni_bytes.p, im.uni_meta.p, im.n_uni, im.uni_back, im.lower_map.p, (uint32_t)kLowerMapLen};
  const uint64_t n_spans = (P.nbytes + kNlBlock - 1) / kNlBlock;
  hipLaunchKernelGGL(k_uni_keywords, dim3(std::max(1u, e->num_cus) * 4), dim3(256), 0, e->stream, P, U, n_spans);
  HIP_TRY(hipGetLastError());
  return TSG_OK;
}

// ---- the dense files' region (k_dense_*), started right after the
// location sort: dense_begin sizes it on the device (no host wait);
// dense_issue -- after k_lines is enqueued -- reads the size, fills the region
// on the side stream and hands its D2H to a DMA engine, so ~200 MB of
// configs[4] results cross PCIe under k_lines, k_censor and k_find_spans.
int dense_begin(tsg_engine* e, const uint8_t* d_data, const uint64_t* d_off, uint64_t nbytes, uint64_t n_locs) {
  e->dense_active = false;
  if (!n_locs || experiment_env("TSG_DENSE_OFF")) return TSG_OK;  // (A/B)
  hipStream_t s = e->stream;
  HIP_TRY(ensure_side(e));
  const uint64_t n_slots = (uint64_t)kCodeLines * n_locs;
  HIP_TRY(e->f_dsize.ensure(n_locs));
  HIP_TRY(e->f_doff.ensure(n_locs));
  HIP_TRY(e->f_dense_at.ensure(n_locs));
  HIP_TRY(e->f_gstart.ensure(n_locs));
  HIP_TRY(e->f_pmax.ensure(n_locs));
  HIP_TRY(e->f_lhead.ensure(n_slots));  // (build_findings_dev's sizes: no reallocation under the side fill)
  HIP_TRY(e->f_lscan.ensure(n_slots));
  HIP_TRY(e->f_lkey.ensure(n_slots));
  if (!e->h_dense) HIP_TRY(hipHostMalloc((void**)&e->h_dense, 64, hipHostMallocDefault));
  FindParams F{};
  F.data = d_data;
  F.data_end = nbytes;
  F.off = d_off;
  F.locs = e->locs2.p;
  F.n_locs = n_locs;
  F.ctrl = e->ctrl.p;
  const uint32_t lane_blocks = (uint32_t)((n_locs + 255) / 256);
  // heads -> 1-based group ids
  hipLaunchKernelGGL(k_dense_heads, dim3(lane_blocks), dim3(256), 0, s, F, e->f_lhead.p);
  size_t tmp = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, e->f_lhead.p, e->f_lscan.p, (int)n_locs, s));
  HIP_TRY(e->cub_tmp.ensure(tmp + 1));
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(e->cub_tmp.p, tmp, e->f_lhead.p, e->f_lscan.p, (int)n_locs, s));
  HIP_TRY(hipMemsetAsync(e->f_dsize.p, 0, n_locs * 8, s));
  hipLaunchKernelGGL(k_dense_groups, dim3(lane_blocks), dim3(256), 0, s, F, e->f_lscan.p, e->f_gstart.p);
  hipLaunchKernelGGL(k_dense_size, dim3(lane_blocks), dim3(256), 0, s, F, e->f_lscan.p, e->f_gstart.p, e->f_dsize.p);
  tmp = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->f_dsize.p, e->f_doff.p, (int)n_locs, s));
  HIP_TRY(e->cub_tmp.ensure(tmp + 1));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->f_dsize.p, e->f_doff.p, (int)n_locs, s));
  hipLaunchKernelGGL(k_dense_at, dim3(lane_blocks), dim3(256), 0, s, F, e->f_lscan.p, e->f_dsize.p, e->f_doff.p,
                     e->f_dense_at.p);
  // the sparse locations' packed index (f_lhead is free again: the group ids are in f_lscan)
  HIP_TRY(e->f_spidx.ensure(n_locs));
  hipLaunchKernelGGL(k_dense_sparse_flags, dim3(lane_blocks), dim3(256), 0, s, F, e->f_dense_at.p, e->f_lhead.p);
  tmp = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->f_lhead.p, e->f_spidx.p, (int)n_locs, s));
  HIP_TRY(e->cub_tmp.ensure(tmp + 1));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->f_lhead.p, e->f_spidx.p, (int)n_locs, s));
  hipLaunchKernelGGL(k_dense_sparse_total, dim3(1), dim3(64), 0, s, F, e->f_lhead.p, e->f_spidx.p);
  // the censor cover: running maximum end per file
  hipLaunchKernelGGL(k_dense_pmax_keys, dim3(lane_blocks), dim3(256), 0, s, F, e->f_lkey.p);
  tmp = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tmp, e->f_lkey.p, e->f_pmax.p, hipcub::Max(), (int)n_locs, s));
  HIP_TRY(e->cub_tmp.ensure(tmp + 1));
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(e->cub_tmp.p, tmp, e->f_lkey.p, e->f_pmax.p, hipcub::Max(), (int)n_locs, s));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(e->h_dense, &e->ctrl.p->dense_bytes, 24, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(e->ev_dense, s));
  e->dense_active = true;
  return TSG_OK;
}

int dense_issue(tsg_engine* e, const uint8_t* d_data, const uint64_t* d_off, uint64_t nbytes, uint64_t n_locs,
                tsg_result* res) {
  if (!e->dense_active) return TSG_OK;
  auto& R = res->impl;
  HIP_TRY(hipEventSynchronize(e->ev_dense));  // (k_file_base / k_lines are queued behind it)
  const uint64_t dense_bytes = e->h_dense[0];
  const uint32_t groups = (uint32_t)e->h_dense[1];
  e->n_line_slots = (uint64_t)kCodeLines * e->h_dense[2];
  if (!dense_bytes) return TSG_OK;
  R.dense_block = pinned_get(e->pinned, dense_bytes);
  if (!R.dense_block) {
    set_last_error("hipHostMalloc failed for the findings' dense region");
    return TSG_ERR_DEVICE;
  }
  R.dense = (const char*)R.dense_block->p;
  HIP_TRY(e->f_dense.ensure(dense_bytes));
  FindParams F{};
  F.data = d_data;
  F.data_end = nbytes;
  F.off = d_off;
  F.locs = e->locs2.p;
  F.n_locs = n_locs;
  HIP_TRY(hipStreamWaitEvent(e->side, e->ev_dense, 0));
  const uint64_t lanes = (dense_bytes + kDenseLaneBytes - 1) / kDenseLaneBytes;
  hipLaunchKernelGGL(k_dense_fill, dim3((uint32_t)std::min<uint64_t>((lanes + 255) / 256, 4096)), dim3(256), 0,
                     e->side, F, e->f_gstart.p, e->f_dsize.p, e->f_doff.p, e->f_pmax.p, groups, dense_bytes,
                     e->f_dense.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(e->ev_dfill, e->side));  // (k_match_prefix reads the region)
  // the copy on a DMA engine once the fill is done (k_lines and the findings
  // kernels keep the CUs meanwhile), else on the side stream
  HIP_TRY(hipEventSynchronize(e->ev_dfill));
  if (!dma_d2h(e, (void*)R.dense, e->f_dense.p, dense_bytes))
    HIP_TRY(hipMemcpyAsync((void*)R.dense, e->f_dense.p, dense_bytes, hipMemcpyDeviceToHost, e->side));
  return TSG_OK;
}

// Findings of the sorted kept locations (e->locs2): k_censor, k_find_spans,
// the arena prefix, k_find_copy, the (file, RuleID rank) order; the records
// and the string arena come back with the caller's final synchronisation.
int build_findings_dev(tsg_engine* e, const uint8_t* d_data, const uint64_t* d_off, uint64_t nbytes, uint64_t n_files,
                       uint64_t n_locs, tsg_result* res) {
  hipStream_t s = e->stream;
  const uint64_t n_slots = (uint64_t)kCodeLines * n_locs, n_seg = n_locs + n_slots;
  HIP_TRY(e->f_iv.ensure(2 * n_locs));
  HIP_TRY(e->f_grp.ensure(n_locs));
  HIP_TRY(e->f_rec.ensure(n_locs));
  HIP_TRY(e->f_rec2.ensure(n_locs));
  HIP_TRY(e->f_lkey.ensure(n_slots));
  HIP_TRY(e->f_lkey2.ensure(n_slots));
  HIP_TRY(e->f_lslot.ensure(n_slots));
  HIP_TRY(e->f_lslot2.ensure(n_slots));
  HIP_TRY(e->f_lhead.ensure(n_slots));
  HIP_TRY(e->f_lscan.ensure(n_slots));
  HIP_TRY(e->f_luid.ensure(n_slots));
  HIP_TRY(e->f_sfile.ensure(n_seg));
  HIP_TRY(e->f_sgrp.ensure(n_seg));
  HIP_TRY(e->f_ssrc.ensure(n_seg));
  HIP_TRY(e->f_slen.ensure(n_seg));
  HIP_TRY(e->f_soff.ensure(n_seg));
  FindParams F{};
  F.data = d_data;
  F.data_end = nbytes;
  F.off = d_off;
  F.nl_blocks = e->nl_blocks.p;
  F.nl_pre = e->nl_pre.p;
  F.n_nlb = nbytes / kNlBlock + 2;
  F.rules = e->img.view.rules;
  F.locs = e->locs2.p;
  F.n_locs = n_locs;
  F.iv = e->f_iv.p;
  F.grp = e->f_grp.p;
  F.rec = e->f_rec.p;
  F.line_key = e->f_lkey.p;
  F.line_slot = e->f_lslot.p;
  F.line_head = e->f_lhead.p;
  F.line_uid = e->f_luid.p;
  F.seg_file = e->f_sfile.p;
  F.seg_grp = e->f_sgrp.p;
  F.seg_src = e->f_ssrc.p;
  F.seg_len = e->f_slen.p;
  F.seg_off = e->f_soff.p;
  F.n_seg_cap = n_seg;
  F.sort_key = e->keys.p;
  F.sort_idx = e->vals.p;
  F.ctrl = e->ctrl.p;
  F.rank_bits = 1;
  while ((1u << F.rank_bits) < e->img.view.n_rules + 1) ++F.rank_bits;
  int key_bits = (int)F.rank_bits + 1;
  while (key_bits < 64 && (1ull << (key_bits - F.rank_bits)) <= n_files) ++key_bits;
  const uint32_t lane_blocks = (uint32_t)((n_locs + 255) / 256), wave_blocks = (uint32_t)((n_locs * 64 + 255) / 256);
  HIP_TRY(hipMemsetAsync(e->f_slen.p, 0, n_seg * 8, s));  // unused line segments stay empty
  hipLaunchKernelGGL(k_censor, dim3(wave_blocks), dim3(256), 0, s, F);
  if (n_locs >= kCensorBig)
    hipLaunchKernelGGL(k_censor_big, dim3((uint32_t)((n_locs + kCensorBig - 1) / kCensorBig)), dim3(1024), 0, s, F);
  // the dense files' region: sizes and offsets now (k_dense_*), filled and
  // copied back on the side stream while k_find_spans runs
  auto& R = res->impl;
  HIP_TRY(ensure_side(e));
  F.dense_at = e->dense_active ? e->f_dense_at.p : nullptr;  // (dense_begin / dense_issue)
  F.slot_base = e->dense_active ? e->f_spidx.p : nullptr;
  const uint64_t n_lslots = e->dense_active ? e->n_line_slots : n_slots;  // the sparse locations' slots
  const uint32_t lslot_blocks = (uint32_t)std::max<uint64_t>((n_lslots + 255) / 256, 1);
  // spans: one lane per location, the long lines' locations then one wave each
  if (experiment_env("TSG_SPANS_WAVE")) {  // (A/B: every location one wave)
    hipLaunchKernelGGL(k_find_spans, dim3(wave_blocks), dim3(256), 0, s, F);
  } else {
    HIP_TRY(e->f_long.ensure(n_locs));
    F.long_list = e->f_long.p;
    hipLaunchKernelGGL(k_find_spans_lane, dim3(lane_blocks), dim3(256), 0, s, F);
    hipLaunchKernelGGL(k_find_spans, dim3(std::min<uint32_t>(wave_blocks, std::max(1u, e->num_cus) * 32)), dim3(256),
                       0, s, F);
  }
  HIP_TRY(hipGetLastError());
  // distinct Code lines: sort the slots by (file, line start), number the runs
  size_t tmp = 0;
  if (n_lslots) {
    HIP_TRY(sort_pairs(e, e->f_lkey.p, e->f_lkey2.p, e->f_lslot.p, e->f_lslot2.p, n_lslots, 64, s));
    hipLaunchKernelGGL(k_line_heads, dim3(lslot_blocks), dim3(256), 0, s, e->f_lkey2.p, n_lslots, e->f_lhead.p);
    tmp = 0;
    HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, e->f_lhead.p, e->f_lscan.p, (int)n_lslots, s));
    HIP_TRY(e->cub_tmp.ensure(tmp + 1));
    HIP_TRY(hipcub::DeviceScan::InclusiveSum(e->cub_tmp.p, tmp, e->f_lhead.p, e->f_lscan.p, (int)n_lslots, s));
    hipLaunchKernelGGL(k_line_map, dim3(lslot_blocks), dim3(256), 0, s, F, e->f_lkey2.p, e->f_lslot2.p, e->f_lscan.p,
                       e->f_lhead.p, n_lslots);
  }
  // arena offsets of the segments (Match windows, then distinct lines)
  tmp = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->f_slen.p, e->f_soff.p, (int)n_seg, s));
  HIP_TRY(e->cub_tmp.ensure(tmp + 1));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->f_slen.p, e->f_soff.p, (int)n_seg, s));
  hipLaunchKernelGGL(k_seg_total, dim3(1), dim3(64), 0, s, F);
  hipLaunchKernelGGL(k_find_finalize, dim3(lane_blocks), dim3(256), 0, s, F);
  HIP_TRY(hipGetLastError());
  // The arena's size (find_bytes) is known only on the device.  The arena
  // stage is queued at a capacity that covers it almost always (the last
  // call's need + 1/4, at least 16 MiB and 1 KiB per location) while the
  // size comes back by an async copy; the host lays out the result block
  // under that stage and redoes the stage, larger, in the rare case the
  // capacity was short.  (A blocking read here left the GPU idle for the
  // round trip and the next launches: ~0.1 ms on configs[2], profiles/r05zd.)
  const bool use_dma = experiment_env("TSG_DMA_OFF") == nullptr;
  HIP_TRY(e->out_locs.ensure(n_locs));
  if (!e->h_find) HIP_TRY(hipHostMalloc((void**)&e->h_find, sizeof(Ctrl), hipHostMallocDefault));
  HIP_TRY(hipMemcpyAsync(e->h_find, e->ctrl.p, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(e->ev_fb, s));
  uint64_t cap = std::max<uint64_t>({1ull << 24, n_locs * 1024, e->arena_need});
  if (!use_dma) {  // (exp A/B: the copies below are queued now and need the layout: read the size first)
    HIP_TRY(hipEventSynchronize(e->ev_fb));
    cap = ((const Ctrl*)e->h_find)->find_bytes;
  }
  const uint64_t tie_cap = std::max<uint64_t>(1024, n_locs / 8);
  const size_t rec_bytes = n_locs * sizeof(FindRec);
  HIP_TRY(e->f_lkeyb.ensure(n_locs));
  HIP_TRY(e->f_ties.ensure(tie_cap));
  // k_out_locs, then the arena and the (file, RuleID rank, Match) order
  auto arena_stage = [&](uint64_t arena_cap) -> int {
    HIP_TRY(e->f_arena.ensure(arena_cap + 16));
    F.arena = e->f_arena.p;
    F.arena_cap = arena_cap;
    F.n_gran = arena_cap / kArenaGran + 2;
    const uint32_t gran_blocks = (uint32_t)((F.n_gran + 1023) / 1024);
    HIP_TRY(e->f_gran.ensure(F.n_gran));
    HIP_TRY(e->f_gcarry.ensure(gran_blocks + 1));
    F.gran_seg = e->f_gran.p;
    F.gran_carry = e->f_gcarry.p;
    HIP_TRY(hipMemsetAsync(F.gran_seg, 0, F.n_gran * 4, s));
    hipLaunchKernelGGL(k_arena_gran_mark, dim3((uint32_t)((n_seg + 255) / 256)), dim3(256), 0, s, F);
    hipLaunchKernelGGL(k_arena_gran_scan, dim3(gran_blocks), dim3(1024), 0, s, F);
    hipLaunchKernelGGL(k_arena_gran_carry, dim3(1), dim3(1024), 0, s, F, gran_blocks);
    hipLaunchKernelGGL(k_arena_fill, dim3((uint32_t)std::min<uint64_t>((arena_cap / 16 + 255) / 256 + 1, 8192)),
                       dim3(256), 0, s, F);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev_fill, s));
    // order: (file, RuleID rank) major, Match prefix minor -- two stable radix
    // sorts, least significant key first (f_lkey / f_lkey2 / f_lslot* are free now)
    if (R.dense) HIP_TRY(hipStreamWaitEvent(s, e->ev_dfill, 0));  // (the Match windows of dense files)
    hipLaunchKernelGGL(k_match_prefix, dim3(lane_blocks), dim3(256), 0, s, e->f_rec.p, e->f_arena.p, e->f_dense.p,
                       n_locs, e->f_lkey.p, e->f_lkeyb.p, e->f_lslot.p);
    // Match bytes 8..15, then (stable) bytes 0..7, then (file, RuleID rank)
    HIP_TRY(sort_pairs(e, e->f_lkeyb.p, e->f_lkey2.p, e->f_lslot.p, e->f_lslot2.p, n_locs, 64, s));
    hipLaunchKernelGGL(k_gather_u64, dim3(lane_blocks), dim3(256), 0, s, e->f_lkey.p, e->f_lslot2.p, n_locs, e->keys2.p);
    HIP_TRY(sort_pairs(e, e->keys2.p, e->f_lkey2.p, e->f_lslot2.p, e->f_lslot.p, n_locs, 64, s));
    hipLaunchKernelGGL(k_gather_u64, dim3(lane_blocks), dim3(256), 0, s, e->keys.p, e->f_lslot.p, n_locs, e->keys2.p);
    HIP_TRY(sort_pairs(e, e->keys2.p, e->keys.p, e->f_lslot.p, e->vals2.p, n_locs, key_bits, s));
    hipLaunchKernelGGL(k_find_gather, dim3(lane_blocks), dim3(256), 0, s, e->f_rec.p, e->vals2.p, n_locs, e->f_rec2.p);
    HIP_TRY(hipMemsetAsync(&e->ctrl.p->n_ties, 0, 8, s));
    hipLaunchKernelGGL(k_tie_list, dim3(lane_blocks), dim3(256), 0, s, e->keys.p, e->f_lkey.p, e->f_lkeyb.p, e->vals2.p,
                       n_locs, e->f_ties.p, tie_cap, e->ctrl.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev_frec, s));
    return TSG_OK;
  };
  // the kept locations as tsg_loc records
  hipLaunchKernelGGL(k_out_locs, dim3(lane_blocks), dim3(256), 0, s, e->locs2.p, n_locs, e->out_locs.p, e->ctrl.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(e->ev_code, s));
  if (int rc = arena_stage(cap)) return rc;
  HIP_TRY(hipEventSynchronize(e->ev_fb));  // (the GPU runs the arena stage meanwhile)
  const uint64_t find_bytes = ((const Ctrl*)e->h_find)->find_bytes;
  const uint64_t match_bytes = ((const Ctrl*)e->h_find)->match_bytes;
  e->arena_need = find_bytes + find_bytes / 4;
  if (find_bytes > cap) {  // short: the stage again at the size now known
    if (int rc = arena_stage(find_bytes)) return rc;
  }
  if (res->impl.timings.size() > 25) {
    res->impl.timings[24] = (double)find_bytes;
    res->impl.timings[25] = (double)match_bytes;
  }
  // the result's page-locked block
  const size_t o_locs = (rec_bytes + find_bytes + 15) & ~(size_t)15;
  const size_t o_flags = o_locs + n_locs * sizeof(tsg_loc);
  const size_t o_ties = (o_flags + n_files + 15) & ~(size_t)15;
  const size_t o_ctrl = (o_ties + tie_cap * 4 + 15) & ~(size_t)15;
  R.arena = pinned_get(e->pinned, o_ctrl + sizeof(Ctrl));
  if (!R.arena) {
    set_last_error("hipHostMalloc failed for the findings arena");
    return TSG_ERR_DEVICE;
  }
  uint8_t* base = (uint8_t*)R.arena->p;
  R.frec = {(FindRec*)base, n_locs};
  R.strs = (const char*)(base + rec_bytes);
  R.locs = {(tsg_loc*)(base + o_locs), n_locs};
  R.file_flags = {base + o_flags, n_files};
  R.ties = {(uint32_t*)(base + o_ties), 0};
  R.ctrl_off = o_ctrl;
  // The kept locations, the string arena and the ordered records go back on
  // a DMA engine (dma_d2h) once their producers are done -- the host waits
  // for each producer's event (the GPU has the rest of the stage queued);
  // without DMA as copies on the stream.  (hipMemcpyAsync into the
  // page-locked block ran as blit kernels on the CUs, even with
  // hipMemcpyDeviceToDeviceNoCU, profiles/r05h_c4.)
  auto d2h = [&](void* dst, const void* src, size_t bytes, hipEvent_t ev) -> int {
    if (!bytes) return TSG_OK;
    if (use_dma) {
      HIP_TRY(hipEventSynchronize(ev));
      if (dma_d2h(e, dst, src, bytes)) return TSG_OK;
    }
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    return TSG_OK;
  };
  if (int rc = d2h(R.locs.p, e->out_locs.p, n_locs * sizeof(tsg_loc), e->ev_code)) return rc;
  if (int rc = d2h(base + rec_bytes, e->f_arena.p, find_bytes, e->ev_fill)) return rc;
  if (int rc = d2h(R.frec.p, e->f_rec2.p, rec_bytes, e->ev_frec)) return rc;
  if (int rc = d2h(R.ties.p, e->f_ties.p, tie_cap * 4, e->ev_frec)) return rc;
  // the caller's final synchronisation covers the side stream's copies (the
  // dense region's, when it did not go to a DMA engine)
  HIP_TRY(hipEventRecord(e->ev_side, e->side));
  HIP_TRY(hipStreamWaitEvent(s, e->ev_side, 0));
  R.ties_cap = tie_cap;
  return TSG_OK;
}

// Scan's final sort (scanner.go:441-446) is by (RuleID, Match); the device
// ordered the records by (file, RuleID rank) keeping (file, start) order, so
// only runs with an equal (file, RuleID) are ordered here, by Match and then
// (rule, start, end) -- the order the reference's matches arrive in.
void order_finding_ties(ResultImpl& R, bool all_runs) {
  auto less = [&](const FindRec& x, const FindRec& y) {
    const int c = memcmp(arena_at(R, x.m_off), arena_at(R, y.m_off), std::min(x.m_len, y.m_len));
    if (c != 0) return c < 0;
    if (x.m_len != y.m_len) return x.m_len < y.m_len;
    const tsg_loc &a = R.locs[x.loc], &b = R.locs[y.loc];
    if (a.rule != b.rule) return a.rule < b.rule;
    if (a.start != b.start) return a.start < b.start;
    return a.end < b.end;
  };
  // the device ordered (file, RuleID, Match prefix); runs of equal
  // (file, RuleID, prefix) -- the positions k_tie_list flagged, each equal to
  // its predecessor -- are ordered here, on up to 16 host threads when large
  std::vector<std::pair<size_t, size_t>> runs;
  size_t work = 0;
  if (all_runs) {  // the tie list overflowed: every run of equal (file, RuleID)
    for (size_t i = 0; i < R.frec.size();) {
      size_t j = i + 1;
      while (j < R.frec.size() && R.frec[j].file == R.frec[i].file && R.frec[j].rank == R.frec[i].rank) ++j;
      if (j - i > 1) {
        runs.push_back({i, j});
        work += j - i;
      }
      i = j;
    }
  } else {
    std::vector<uint32_t> t(R.ties.p, R.ties.p + R.ties.n);
    std::sort(t.begin(), t.end());
    for (size_t k = 0; k < t.size();) {
      size_t q = k + 1;
      while (q < t.size() && t[q] == t[q - 1] + 1) ++q;
      runs.push_back({(size_t)t[k] - 1, (size_t)t[q - 1] + 1});  // a run starts at its first flag's predecessor
      work += q - k + 1;
      k = q;
    }
  }
  // the records and Match strings of the runs were just written by DMA and
  // are cold: each batch of runs is prefetched first (records, then their
  // strings: independent misses overlap; compared one by one they cost
  // ~170 ns per tie, 1.4 ms for configs[4]'s 8 K ties, 0.77 ms prefetched on
  // one thread, profiles/r05n)
  auto prefetch = [&](size_t k0, size_t k1) {
    for (size_t k = k0; k < k1; ++k)
      for (size_t i = runs[k].first; i < runs[k].second; ++i) __builtin_prefetch(&R.frec[i]);
    for (size_t k = k0; k < k1; ++k)
      for (size_t i = runs[k].first; i < runs[k].second; ++i) {
        const char* m = arena_at(R, R.frec[i].m_off);
        __builtin_prefetch(m);
        if (R.frec[i].m_len > 64) __builtin_prefetch(m + 64);
        __builtin_prefetch(&R.locs[R.frec[i].loc]);
      }
  };
  auto sort_run = [&](const std::pair<size_t, size_t>& r) {
    if (r.second - r.first <= 16) {  // short runs (most): stable insertion sort, no temporary buffer
      for (size_t a = r.first + 1; a < r.second; ++a) {
        const FindRec x = R.frec[a];
        size_t b = a;
        for (; b > r.first && less(x, R.frec[b - 1]); --b) R.frec[b] = R.frec[b - 1];
        R.frec[b] = x;
      }
      return;
    }
    std::stable_sort(R.frec.begin() + r.first, R.frec.begin() + r.second, less);
  };
  constexpr size_t kBatch = 256;  // runs per prefetch batch
  auto batch = [&](size_t k0) {
    const size_t k1 = std::min(runs.size(), k0 + kBatch);
    prefetch(k0, k1);
    for (size_t k = k0; k < k1; ++k) sort_run(runs[k]);
  };
  // threads: ~30 us each to start and join, so one per ~2 K records of work
  // (at most 16; configs[4]'s 8 K ties take 4)
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned nt = (unsigned)std::min<size_t>(std::min(16u, hw), work / 2048);
  if (nt <= 1 || runs.size() < 2 * kBatch) {
    for (size_t k0 = 0; k0 < runs.size(); k0 += kBatch) batch(k0);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (size_t k0; (k0 = next.fetch_add(kBatch)) < runs.size();) batch(k0);
    });
  for (auto& t : th) t.join();
}

// CPU replay of k_scan_big's walk (test hook): the text through the
// automaton's own table and through the LDS blob's dense rows / cold records
// (breadth-first or frequency numbering) must visit the same states with the
// same output bits.
extern "C" int tsg_ruleset_big_check(const tsg_ruleset* rs, const uint8_t* text, size_t len, int bfs,
                                     uint64_t* mismatches, uint64_t* cold_hops, uint32_t* n_dense) {
  if (!rs || (!text && len) || !mismatches || !cold_hops || !n_dense) return TSG_ERR_INVALID_ARG;
  const AcHost& ac = rs->ac;
  BigBlobHost bb;
  *mismatches = *cold_hops = 0;
  *n_dense = 0;
  if (!build_big_blob(ac, bfs != 0, &bb)) return TSG_ERR_UNSUPPORTED;
  *n_dense = bb.nd;
  const uint32_t K = ac.nclasses;
  uint32_t a = 0, b = 0;  // automaton state, blob state
  for (size_t i = 0; i < len; ++i) {
    const uint32_t c = ac.cls[text[i]];
    const uint32_t va = ac.delta[(size_t)a * K + c];
    uint32_t hops = 0;
    const uint32_t vb = big_next_host(bb, K, b, c, &hops);
    *cold_hops += hops;
    if (vb >= 0xFFFFFFFEu || (vb & 0x8000u) != (va & 0x8000u) || bb.ac_of[vb & 0x7FFFu] != (va & 0x7FFFu)) {
      ++*mismatches;
      a = b = 0;  // resynchronise
      continue;
    }
    a = va & 0x7FFFu;
    b = vb & 0x7FFFu;
  }
  return TSG_OK;
}

// The verify DFA walk with k_verify's run acceleration (dfa_accel_skip),
// restated on the host for tests: must give tsg_ruleset_dfa_check's answer
// for every start; *skipped = bytes the accelerated runs stepped over.
extern "C" int tsg_ruleset_dfa_accel_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s,
                                           int* result, size_t* me, uint64_t* skipped) {
  if (!rs || i >= rs->rules.size() || !result || !me || !skipped || (len && !text)) return TSG_ERR_INVALID_ARG;
  const DfaHost& d = rs->rules[i].dfa;
  *skipped = 0;
  if (!d.valid || s >= len) {
    *result = 2;
    return TSG_OK;
  }
  const DfaAccel acc = dfa_accel_records(d);
  const size_t n = len;
  uint32_t st = d.start[s == 0 ? 1 : 0];
  int64_t last = d.match[st] ? (int64_t)s : -1;
  for (size_t q = s; q < n && st;) {
    const uint8_t c = text[q];
    uint32_t w = 1, k = d.cls[c & 0x7F];
    if (c >= 0x80) {
      const int sym = dfa_rune_sym(d, text, n, q, &w);
      if (sym < 0) {
        *result = 2;
        return TSG_OK;
      }
      k = (uint32_t)sym;
    }
    const uint16_t e = d.delta[(size_t)st * d.ncls + k];
    if (q + w == n) {
      if (e & 0x8000) last = (int64_t)n;
      break;
    }
    st = e & kDfaStateMask;
    q += w;
    if (e & 0x4000) last = (int64_t)q;
    if (acc.idx[st] != 0xFFFFFFFFu) {
      const uint32_t* rec = acc.recs.data() + 8 * (size_t)acc.idx[st];
      size_t q2 = q;
      while (q2 < n && text[q2] < 0x80 && ((rec[text[q2] >> 5] >> (text[q2] & 31)) & 1)) ++q2;
      if (q2 > q) {
        const uint16_t es = d.delta[(size_t)st * d.ncls + rec[4]];
        *skipped += q2 - q;
        if (q2 == n) {
          if (n - 1 > q && (es & 0x4000)) last = (int64_t)n - 1;
          if (es & 0x8000) last = (int64_t)n;
          break;
        }
        if (es & 0x4000) last = (int64_t)q2;
        q = q2;
      }
    }
  }
  *result = last < 0 ? 0 : 1;
  if (last >= 0) *me = (size_t)last;
  return TSG_OK;
}

// Visits per state of the keyword / anchor automaton over a host text
// (diagnostics: dense-row selection studies); counts[blob order] with the
// blob's numbering when blob != 0, else automaton ids.  n = states.
extern "C" int tsg_big_cold_lds_floor(uint32_t n, uint32_t* previous) {
  const uint32_t was = g_big_cold_floor.exchange(n);
  if (previous) *previous = was;
  return TSG_OK;
}

extern "C" int tsg_ruleset_ac_visits(const tsg_ruleset* rs, const uint8_t* text, size_t len, int blob,
                                     uint64_t* counts, size_t n, uint32_t* n_dense) {
  if (!rs || (!text && len) || !counts || !n_dense) return TSG_ERR_INVALID_ARG;
  const AcHost& ac = rs->ac;
  if (n < ac.nstates) return TSG_ERR_INVALID_ARG;
  BigBlobHost bb;
  std::vector<uint32_t> at(ac.nstates);
  for (uint32_t k = 0; k < ac.nstates; ++k) at[k] = k;
  *n_dense = 0;
  if (blob) {
    if (!build_big_blob(ac, false, &bb)) return TSG_ERR_UNSUPPORTED;
    for (uint32_t k = 0; k < ac.nstates; ++k) at[bb.ac_of[k]] = k;
    *n_dense = bb.nd;
  }
  memset(counts, 0, n * sizeof(uint64_t));
  const uint32_t K = ac.nclasses;
  uint32_t a = 0;
  for (size_t i = 0; i < len; ++i) {
    a = ac.delta[(size_t)a * K + ac.cls[text[i]]] & 0x7FFFu;
    ++counts[at[a]];
  }
  return TSG_OK;
}

// The blob validator against forged blobs (tests): the ruleset's blob with
// one invariant broken -- kind 1: a cold state's failure link pointed at
// itself (a cycle), 2: an overflow list's terminator removed, 3: a dense
// entry past the last state, 4: a cold record's class past the class count,
// 0: unmodified.  *rc = what the validator (the product's pre-launch check)
// returns for it: TSG_OK or TSG_ERR_INTERNAL.
extern "C" int tsg_ruleset_big_forge_check(const tsg_ruleset* rs, int kind, int* rc) {
  if (!rs || !rc || kind < 0 || kind > 4) return TSG_ERR_INVALID_ARG;
  const AcHost& ac = rs->ac;
  BigBlobHost bb;
  if (!build_big_blob(ac, false, &bb)) return TSG_ERR_UNSUPPORTED;
  uint32_t* rec = (uint32_t*)(bb.blob.data() + bb.o_cold);
  uint32_t* ev = (uint32_t*)(bb.blob.data() + bb.o_eval);
  const uint64_t n_ev = (bb.o_cold - bb.o_eval) / 4;
  if (kind == 1) {
    if (!bb.cold) return TSG_ERR_UNSUPPORTED;
    const uint32_t j = bb.cold / 2;
    rec[2 * j + 1] = (rec[2 * j + 1] & 0xFFFFu) | ((bb.nd + j) << 16);
  } else if (kind == 2) {
    uint64_t last = n_ev;
    for (uint64_t k = 0; k < n_ev; ++k)
      if (ev[k] == 0xFFFFFFFFu) last = k;
    if (last == n_ev) return TSG_ERR_UNSUPPORTED;
    ev[last] = 0;  // the last list now runs off the blob's end
  } else if (kind == 3) {
    ((uint16_t*)(bb.blob.data() + 256))[1] = (uint16_t)ac.nstates;
  } else if (kind == 4) {
    if (!bb.cold) return TSG_ERR_UNSUPPORTED;
    uint32_t j = 0;
    while (j < bb.cold && (rec[2 * j] & 0xFFu) == kBigMore) ++j;
    if (j == bb.cold) return TSG_ERR_UNSUPPORTED;
    rec[2 * j] = (rec[2 * j] & ~0xFFu) | (ac.nclasses & 0xFFu);
  }
  *rc = validate_big_blob(bb, ac.nclasses, ac.nstates).empty() ? TSG_OK : TSG_ERR_INTERNAL;
  return TSG_OK;
}

// ------------------------------------------------- byte-range split (§8(e)) --
// One large file scanned by several GPUs: every rank runs the scan pass (the
// HBM-bound part) over its byte range [own_lo, own_hi) and exports the scan
// state that range owns; the file's owner imports the union and runs the rest
// of the pipeline (candidates, FindAll, exclude, lines, findings) over the
// whole file, so the result is the single-GPU result by construction.  The
// scan state is position-local: keyword bits (OR), anchor hits owned by their
// literal start, and per-4 KiB-span newline counts and >= 0x80 flags.
constexpr uint64_t kPartMagic = 0x3274726170677374ull;  // "tsgpart2"
// Blob body after the header, packed and unpacked on the device: kw_words u32
// keyword words | n_spans u16 newline counts | ceil(n_spans / 8) bytes of
// ">= 0x80" span bits | n_hits u64 owned anchor hits (file-relative starts).
__host__ __device__ inline uint64_t part_fixed_bytes(uint32_t kw_words, uint64_t n_spans) {
  return (uint64_t)kw_words * 4 + n_spans * 2 + (n_spans + 7) / 8;
}
// Part export on the device: the owned anchor hits compacted (any order: the
// candidates are sorted later) with file-relative starts, the keyword words,
// per-span newline counts as u16 (<= 4096 per 4 KiB span) and the >= 0x80
// flags as bits -- one buffer, one D2H.  out[0] (u64) counts the kept hits.
struct PartPack {
  const uint64_t* hits;
  uint64_t n_hits;
  const uint32_t* kw;
  uint32_t kw_words;
  const uint32_t* nl;
  const uint8_t* span_hi;  // may be null
  uint64_t sp0, n_spans;
  uint64_t base, own_lo, own_hi;  // view base, owned range (file-relative)
  uint8_t* out;                   // u64 count | fixed body | hits
};

__global__ void k_part_pack(PartPack K) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  uint8_t* body = K.out + 8;
  uint32_t* kw = (uint32_t*)body;
  uint16_t* nl = (uint16_t*)(body + (uint64_t)K.kw_words * 4);
  uint8_t* hib = body + (uint64_t)K.kw_words * 4 + K.n_spans * 2;
  uint64_t* hits = (uint64_t*)(K.out + 8 + ((part_fixed_bytes(K.kw_words, K.n_spans) + 7) & ~7ull));
  for (uint64_t i = t; i < K.kw_words; i += nt) kw[i] = K.kw[i];
  for (uint64_t i = t; i < K.n_spans; i += nt) nl[i] = (uint16_t)K.nl[K.sp0 + i];
  for (uint64_t i = t; i < (K.n_spans + 7) / 8; i += nt) {
    uint32_t b = 0;
    if (K.span_hi)
      for (uint32_t k = 0; k < 8 && 8 * i + k < K.n_spans; ++k) b |= (K.span_hi[K.sp0 + 8 * i + k] ? 1u : 0u) << k;
    hib[i] = (uint8_t)b;
  }
  for (uint64_t i = t; i < K.n_hits; i += nt) {
    const uint64_t h = K.hits[i];
    const uint64_t start = ((h & ~kFoldHit) >> 16) + K.base;
    if (start < K.own_lo || start >= K.own_hi) continue;
    const unsigned long long k = atomicAdd((unsigned long long*)K.out, 1ull);
    hits[k] = (start << 16) | (h & (kFoldHit | 0xFFFFull));
  }
}

// Part import on the device: one blob body (already in device memory) into
// the merge's scan state; a hit outside the part's owned range sets *bad.
struct PartUnpack {
  const uint8_t* body;
  uint32_t kw_words;
  uint64_t n_spans, s0, n_hits;
  uint64_t own_lo, own_hi;
  uint32_t* kw;
  uint32_t* nl;
  uint8_t* span_hi;
  uint64_t* hits;  // at this part's offset
  unsigned int* bad;
};

__global__ void k_part_unpack(PartUnpack U) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t* kw = (const uint32_t*)U.body;
  const uint16_t* nl = (const uint16_t*)(U.body + (uint64_t)U.kw_words * 4);
  const uint8_t* hib = U.body + (uint64_t)U.kw_words * 4 + U.n_spans * 2;
  const uint64_t* hits = (const uint64_t*)(U.body + ((part_fixed_bytes(U.kw_words, U.n_spans) + 7) & ~7ull));
  for (uint64_t i = t; i < U.kw_words; i += nt)
    if (kw[i]) atomicOr(&U.kw[i], kw[i]);
  for (uint64_t i = t; i < U.n_spans; i += nt) {
    U.nl[U.s0 + i] = nl[i];
    U.span_hi[U.s0 + i] = (hib[i >> 3] >> (i & 7)) & 1u;
  }
  for (uint64_t i = t; i < U.n_hits; i += nt) {
    const uint64_t h = hits[i];
    const uint64_t start = (h & ~kFoldHit) >> 16;
    if (start < U.own_lo || start >= U.own_hi) atomicOr(U.bad, 1u);
    U.hits[i] = h;
  }
}

struct PartHeader {
  uint64_t magic, ruleset_id, file_len, own_lo, own_hi, n_hits;
  uint32_t kw_words, flags, n_spans, has_span_hi;
};
struct SplitIo {
  int mode = 0;  // 1: export the part [own_lo, own_hi) of a view; 2: merge parts
  uint64_t text_base = 0, own_lo = 0, own_hi = 0, file_len = 0;
  uint8_t** blob_out = nullptr;                                // mode 1 output (page-locked, tsg_part_free)
  size_t* blob_len = nullptr;
  const std::vector<std::pair<const uint8_t*, size_t>>* parts = nullptr;  // mode 2 input
};

uint64_t part_right_halo(const tsg_ruleset* rs) {
  // a literal (with its class extension) starting before own_hi lies wholly
  // inside the view; k_fold_windows reads a pattern length around a rune
  size_t m = 0;
  for (auto& p : rs->patterns) m = std::max(m, p.lower.size() + p.ext_cols.size());
  return ((m + 64 + kNlBlock - 1) / kNlBlock) * kNlBlock;
}

// Part blobs come from a process-wide pool of page-locked blocks:
// hipHostMalloc of a blob (~5 MB of newline counts per 10 GB part) took
// 1.2 ms of a 10 GB part's 10.4 ms (profiles/r05f).  tsg_part_free returns a
// block to the pool; at most kBlobPoolBytes stay parked there.
constexpr size_t kBlobPoolBytes = 256ull << 20;
struct BlobPool {
  std::mutex mu;
  std::multimap<size_t, uint8_t*> parked;        // capacity -> block
  std::unordered_map<uint8_t*, size_t> cap_of;   // every block handed out or parked
  size_t parked_bytes = 0;
};
BlobPool& blob_pool() {
  static BlobPool* p = new BlobPool;  // (never destroyed: frees may come at exit)
  return *p;
}
uint8_t* blob_alloc(size_t n) {
  BlobPool& bp = blob_pool();
  {
    std::lock_guard<std::mutex> lk(bp.mu);
    auto it = bp.parked.lower_bound(n);
    if (it != bp.parked.end() && it->first <= 4 * n + (1 << 20)) {  // (no huge block for a small blob)
      uint8_t* b = it->second;
      bp.parked_bytes -= it->first;
      bp.parked.erase(it);
      return b;
    }
  }
  const size_t cap = std::max<size_t>((n + (n >> 2) + 4095) & ~(size_t)4095, 64 << 10);
  uint8_t* b = nullptr;
  if (hipHostMalloc((void**)&b, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(bp.mu);
  bp.cap_of[b] = cap;
  return b;
}
void blob_release(uint8_t* b) {
  BlobPool& bp = blob_pool();
  std::unique_lock<std::mutex> lk(bp.mu);
  auto it = bp.cap_of.find(b);
  if (it == bp.cap_of.end()) return;  // (not a blob of this library)
  const size_t cap = it->second;
  bp.parked.emplace(cap, b);
  bp.parked_bytes += cap;
  std::vector<uint8_t*> drop;
  while (bp.parked_bytes > kBlobPoolBytes && !bp.parked.empty()) {  // the largest go first
    auto last = std::prev(bp.parked.end());
    bp.parked_bytes -= last->first;
    drop.push_back(last->second);
    bp.cap_of.erase(last->second);
    bp.parked.erase(last);
  }
  lk.unlock();
  for (uint8_t* d : drop) (void)hipHostFree(d);
}

int export_part(tsg_engine* e, const tsg_ruleset* rs, const ScanParams& P, uint64_t n_hits, const SplitIo& sp) {
  hipStream_t s = e->stream;
  const uint64_t base = sp.text_base;
  const uint64_t sp0 = (sp.own_lo - base) / kNlBlock, sp1 = (sp.own_hi - base + kNlBlock - 1) / kNlBlock;
  const uint64_t n_spans = sp1 - sp0;
  const bool has_hi = P.span_hi != nullptr;
  const uint64_t fixed = part_fixed_bytes(P.rs.kw_words, n_spans);
  const uint64_t cap = 8 + ((fixed + 7) & ~7ull) + n_hits * 8;
  HIP_TRY(e->part_buf.ensure(cap));
  HIP_TRY(hipMemsetAsync(e->part_buf.p, 0, 8, s));
  PartPack K{e->hits.p, n_hits, e->file_kw.p, P.rs.kw_words, e->nl_blocks.p, has_hi ? P.span_hi : nullptr,
             sp0, n_spans, base, sp.own_lo, sp.own_hi, e->part_buf.p};
  const uint64_t work = std::max<uint64_t>(std::max<uint64_t>(n_hits, n_spans), 1);
  hipLaunchKernelGGL(k_part_pack, dim3((uint32_t)std::min<uint64_t>((work + 255) / 256, e->num_cus * 8ull)), dim3(256),
                     0, s, K);
  HIP_TRY(hipGetLastError());
  // one D2H of the packed buffer into page-locked memory (the blob itself)
  uint8_t* blob = blob_alloc(sizeof(PartHeader) + cap);
  if (!blob) {
    set_last_error("hipHostMalloc failed for a part blob");
    return TSG_ERR_DEVICE;
  }
  uint32_t flags = 0;
  hipError_t he = hipMemcpyAsync(blob + sizeof(PartHeader) - 8, e->part_buf.p, cap, hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipMemcpyAsync(&flags, e->file_flags.p, 4, hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess) {  // the blob is not handed out: free it here
    blob_release(blob);
    set_last_error(std::string("HIP error in export_part: ") + hipGetErrorString(he));
    return TSG_ERR_DEVICE;
  }
  uint64_t kept = 0;
  memcpy(&kept, blob + sizeof(PartHeader) - 8, 8);  // (the count sits where the header's tail goes)
  PartHeader H{kPartMagic, rs->id, sp.file_len, sp.own_lo, sp.own_hi, kept, P.rs.kw_words, flags, (uint32_t)n_spans,
               has_hi ? 1u : 0u};
  memcpy(blob, &H, sizeof(H));
  *sp.blob_out = blob;
  *sp.blob_len = sizeof(PartHeader) + ((fixed + 7) & ~7ull) + kept * 8;
  return TSG_OK;
}

// The owner's side: parts must tile [0, file_len) of this ruleset's scans.
int import_parts(tsg_engine* e, const tsg_ruleset* rs, ScanParams& P, const SplitIo& sp, uint64_t* n_hits_out) {
  hipStream_t s = e->stream;
  const auto& parts = *sp.parts;
  std::vector<const PartHeader*> hs;
  for (auto& pr : parts) {
    if (pr.second < sizeof(PartHeader)) {
      set_last_error("split: a part blob is truncated");
      return TSG_ERR_INVALID_ARG;
    }
    const PartHeader* H = (const PartHeader*)pr.first;
    // every size field checked against the file and the blob before any
    // arithmetic with it (blobs travel over arbitrary transports)
    const size_t body = pr.second - sizeof(PartHeader);
    bool ok = H->magic == kPartMagic && H->ruleset_id == rs->id && H->kw_words == P.rs.kw_words &&
              H->file_len == sp.file_len && H->own_lo < H->own_hi && H->own_hi <= sp.file_len &&
              H->own_lo % kNlBlock == 0 && (H->own_hi % kNlBlock == 0 || H->own_hi == sp.file_len) &&
              H->n_spans == (H->own_hi - H->own_lo + kNlBlock - 1) / kNlBlock && H->n_hits <= body / 8;
    if (ok) {  // (every hit's start is checked on the device: k_part_unpack)
      const uint64_t fixed = (part_fixed_bytes(H->kw_words, H->n_spans) + 7) & ~7ull;
      ok = body == fixed + (size_t)H->n_hits * 8;
    }
    if (!ok) {
      set_last_error("split: a part blob belongs to another file or ruleset, or is corrupt");
      return TSG_ERR_INVALID_ARG;
    }
    hs.push_back(H);
  }
  std::vector<size_t> order(hs.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return hs[a]->own_lo < hs[b]->own_lo; });
  uint64_t at = 0, total = 0;
  for (size_t i : order) {
    if (hs[i]->own_lo != at || hs[i]->own_hi <= hs[i]->own_lo) {
      set_last_error("split: the parts do not tile the file");
      return TSG_ERR_INVALID_ARG;
    }
    at = hs[i]->own_hi;
    total += hs[i]->n_hits;
  }
  if (at != sp.file_len && !(sp.file_len == 0 && hs.empty())) {
    set_last_error("split: the parts do not tile the file");
    return TSG_ERR_INVALID_ARG;
  }
  const uint64_t n_nlb = P.nbytes / kNlBlock + 2, n_spans = (P.nbytes + kNlBlock - 1) / kNlBlock;
  // every body to the device (one H2D each, straight from the caller's
  // blob), then unpacked there: keyword words OR'd, newline counts and span
  // bits at their spans, hits appended part after part
  uint64_t body_total = 0;  // each body starts 16-byte aligned (at_body below)
  for (size_t i : order) body_total += (parts[i].second - sizeof(PartHeader) + 15) & ~(uint64_t)15;
  HIP_TRY(e->part_buf.ensure(body_total + 8));
  HIP_TRY(e->hits.ensure(std::max<uint64_t>(total, 1)));
  HIP_TRY(e->nl_blocks.ensure(n_nlb));
  HIP_TRY(e->span_hi.ensure(n_spans + 1));
  HIP_TRY(hipMemsetAsync(e->nl_blocks.p, 0, n_nlb * 4, s));
  HIP_TRY(hipMemsetAsync(e->span_hi.p, 0, n_spans + 1, s));
  HIP_TRY(hipMemsetAsync(&e->ctrl.p->err, 0, 4, s));
  uint32_t flags = 0;
  bool all_hi = true;
  uint64_t at_body = 0, at_hit = 0;
  for (size_t i : order) {
    const PartHeader* H = hs[i];
    const size_t blen = parts[i].second - sizeof(PartHeader);
    HIP_TRY(hipMemcpyAsync(e->part_buf.p + at_body, (const uint8_t*)(H + 1), blen, hipMemcpyHostToDevice, s));
    PartUnpack U{e->part_buf.p + at_body, H->kw_words, H->n_spans, H->own_lo / kNlBlock, H->n_hits, H->own_lo,
                 H->own_hi, e->file_kw.p, e->nl_blocks.p, e->span_hi.p, e->hits.p + at_hit, &e->ctrl.p->err};
    const uint64_t work = std::max<uint64_t>(std::max<uint64_t>(H->n_hits, H->n_spans), 1);
    hipLaunchKernelGGL(k_part_unpack, dim3((uint32_t)std::min<uint64_t>((work + 255) / 256, e->num_cus * 8ull)),
                       dim3(256), 0, s, U);
    HIP_TRY(hipGetLastError());
    at_body += (blen + 15) & ~(size_t)15;
    at_hit += H->n_hits;
    flags |= H->flags & ~kFileAllowed;  // the owner's path gate decides AllowPath
    all_hi = all_hi && H->has_span_hi;
  }
  P.span_hi = all_hi ? e->span_hi.p : nullptr;  // (no flags: k_uni_keywords searches every span)
  const uint64_t n_regions = P.nbytes / kNlBlock + 1;
  HIP_TRY(e->region_file.ensure(n_regions + 1));
  HIP_TRY(hipMemsetAsync(e->region_file.p, 0, (n_regions + 1) * 4, s));  // one file
  P.n_regions = n_regions;  // (k_uni_keywords' file lookup reads them through P)
  P.region_file = e->region_file.p;
  uint32_t f0 = 0, bad = 0;
  HIP_TRY(hipMemcpyAsync(&f0, e->file_flags.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&bad, &e->ctrl.p->err, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (bad) {
    set_last_error("split: a part blob belongs to another file or ruleset, or is corrupt");
    return TSG_ERR_INVALID_ARG;
  }
  f0 |= flags;
  HIP_TRY(hipMemcpy(e->file_flags.p, &f0, 4, hipMemcpyHostToDevice));
  *n_hits_out = total;
  return TSG_OK;
}

// Run the device pipeline on a batch already in HBM.  Fills r->impl.locs and flags.
int run_pipeline(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data, const uint64_t* d_off,
                 const uint8_t* d_paths, const uint64_t* d_path_off, size_t n_files, uint64_t nbytes,
                 tsg_result* res, const SplitIo* sp = nullptr) {
  const auto wall0 = std::chrono::steady_clock::now();
  DmaGuard dma_guard{e};
  e->fast_timed = false;
  e->dense_active = false;
  int rc = upload_ruleset(e, rs);
  if (rc) return rc;
  const DevImage& im = e->img;
  const RuleSetDev& RS = im.view;
  hipStream_t s = e->stream;
  if (n_files >= kMaxBatchFiles) {
    set_last_error("a batch holds fewer than 2^24 files (40-bit positions in the sort keys)");
    return TSG_ERR_UNSUPPORTED;
  }
  const uint32_t nf = (uint32_t)n_files;
  const uint32_t rule_words = std::max<uint32_t>(1, (RS.n_rules + 31) / 32);
  HIP_TRY(e->ctrl.ensure(1));
  HIP_TRY(e->file_kw.ensure((size_t)nf * RS.kw_words + 1));
  HIP_TRY(e->file_flags.ensure(nf + 1));
  if (rs->any_path_rules) HIP_TRY(e->path_mask.ensure((size_t)nf * rule_words + 1));
  HIP_TRY(hipMemsetAsync(e->ctrl.p, 0, sizeof(Ctrl), s));
  HIP_TRY(hipMemsetAsync(e->file_kw.p, 0, ((size_t)nf * RS.kw_words + 1) * 4, s));
  HIP_TRY(hipMemsetAsync(e->file_flags.p, 0, (nf + 1) * 4, s));
  if (rs->any_path_rules) HIP_TRY(hipMemsetAsync(e->path_mask.p, 0, ((size_t)nf * rule_words + 1) * 4, s));
  // VM thread pool for path gate / verify / exclude
  if (!e->vm_threads) {
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, e->device));
    e->vm_threads = (uint32_t)prop.multiProcessorCount * 512;  // 8 waves per CU
  }
  HIP_TRY(e->scratch.ensure((size_t)e->vm_threads * e->scratch_stride));
  std::vector<double>& tm = res->impl.timings;
  tm.assign(26, 0.0);  // [18..22]: tsg_analyze's host stages, [23]: jobs k_verify_fast deferred, [24..25] arena bytes
  if (!e->events) {
    for (auto& ev : e->ev) HIP_TRY(hipEventCreate(&ev));
    e->events = true;
  }
  HIP_TRY(hipEventRecord(e->ev[0], s));
  // ---- 1. path gates (per file), before the scan on the main stream.  Not
  // overlapped with the scan (it fills every CU's VGPRs and LDS); beside
  // k_report on the side stream (TSG_GATE_SIDE, exp) it slowed k_report more
  // than it saved: step 14.86 vs 14.72 ms over three alternating runs each
  // (`profiles/r05q_gate`).
  const bool path_gates = nf && (im.n_gpath || rs->any_path_rules);
  const bool merge_mode = sp && sp->mode == 2;
  const bool gate_on_side = path_gates && !merge_mode && nbytes > 0 && experiment_env("TSG_GATE_SIDE") != nullptr;
  GateParams G{};
  uint32_t gate_blocks = 0;
  if (path_gates) {
    G.off = d_off;
    G.paths = d_paths;
    G.path_off = d_path_off;
    G.n_files = nf;
    G.rs = RS;
    G.gpath = im.u32.p + im.o_gpath;
    G.n_gpath = im.n_gpath;
    G.rule_path = im.rule_path.p;
    G.rule_apath_off = im.u32.p + im.o_apoff;
    G.rule_apath = im.u32.p + im.o_ap;
    G.path_rules = im.u32.p + im.o_prules;
    G.n_path_rules = im.n_prules;
    G.any_rule_paths = rs->any_path_rules;
    G.file_flags = e->file_flags.p;
    G.path_mask = e->path_mask.p;
    G.rule_words = rule_words;
    G.scratch = e->scratch.p;
    G.scratch_stride = e->scratch_stride;
    G.pac = im.pac_bytes ? im.pac.p : nullptr;
    G.pac_states = im.pac_states;
    G.pac_classes = im.pac_classes;
    G.pac_bytes = im.pac_bytes;
    G.o_pac_cls = im.o_pac_cls;
    G.o_pac_out_off = im.o_pac_out_off;
    G.o_pac_out = im.o_pac_out;
    G.o_pac_lits = im.o_pac_lits;
    G.o_pac_req = im.o_pac_req;
    G.o_pac_bit = im.o_pac_bit;
    G.pac_always = im.pac_always;
    G.n_progs = (uint32_t)rs->regexes.size();
    G.pdfa = im.u32.p + im.o_pdfa;
    gate_blocks = std::max(1u, std::min<uint32_t>((nf + 255) / 256, e->vm_threads / 256));
    if (!gate_on_side) {
      // the literal pass over every file at full occupancy, then the files a
      // path program may match with the DFA / VM (grid: one scratch slot per lane)
      HIP_TRY(e->gate_defer.ensure((size_t)nf + 1));
      HIP_TRY(hipMemsetAsync(e->gate_defer.p, 0, 4, s));
      G.defer = e->gate_defer.p;
      if (!e->num_cus) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, e->device));
        e->num_cus = (uint32_t)prop.multiProcessorCount;
      }
      G.pac_lds = G.pac && G.pac_bytes <= 64 * 1024 ? (G.pac_bytes + 15) & ~15u : 0;
      auto prog_bit = [&](int prog, uint64_t* bits, uint32_t* nobit) {
        const uint8_t b = prog >= 0 && (size_t)prog < im.pac_prog_bit.size() ? im.pac_prog_bit[prog] : 0xFF;
        if (b == 0xFF) *nobit = 1;
        else *bits |= 1ull << b;
      };
      G.gpath_bits = G.rpath_bits = 0;
      G.gpath_nobit = G.rpath_nobit = 0;
      for (int x : rs->global_allow_path) prog_bit(x, &G.gpath_bits, &G.gpath_nobit);
      for (auto& r : rs->rules) {
        if (r.path >= 0) prog_bit(r.path, &G.rpath_bits, &G.rpath_nobit);
        for (int x : r.allow_path) prog_bit(x, &G.rpath_bits, &G.rpath_nobit);
      }
      const uint32_t ac_blocks = std::max(1u, std::min<uint32_t>((nf + 255) / 256, e->num_cus * 8));
      hipLaunchKernelGGL((k_path_gate<true, 1>), dim3(ac_blocks), dim3(256), G.pac_lds, s, G);
      hipLaunchKernelGGL((k_path_gate<true, 2>), dim3(gate_blocks), dim3(256), G.pac_lds, s, G);
      HIP_TRY(hipGetLastError());
    } else {
      HIP_TRY(ensure_side(e));
    }
  }
  bool gate_pending = false;  // the side-stream gate has been launched and not yet waited for
  HIP_TRY(hipEventRecord(e->ev[1], s));
  // ---- 2. keyword/anchor scan
  uint64_t hit_cap = std::max<uint64_t>(1 << 20, nbytes / 256);
  HIP_TRY(e->hits.ensure(hit_cap));
  hit_cap = e->hits.n;
  ScanParams P{};
  P.big = e->img.big_view;
  P.data = d_data;
  P.off = d_off;
  P.nbytes = nbytes;
  P.n_files = nf;
  P.rs = RS;
  P.file_kw = e->file_kw.p;
  P.file_flags = e->file_flags.p;
  P.hits = e->hits.p;
  P.hit_cap = hit_cap;
  P.ctrl = e->ctrl.p;

  HIP_TRY(e->fold_pos.ensure(std::max<uint64_t>(1 << 16, e->fold_need)));
  P.fold_pos = e->fold_pos.p;
  P.fold_cap = e->fold_pos.n;
  if (const char* m = experiment_env("TSG_REPORT_MODE")) P.report_mode = (uint32_t)atoi(m);
  const uint64_t n_nlb = nbytes / kNlBlock + 2;
  HIP_TRY(e->nl_blocks.ensure(n_nlb));
  HIP_TRY(e->nl_pre.ensure(n_nlb));
  P.nl_blocks = e->nl_blocks.p;
  // the scan counts the newlines of big files' spans itself (span_scan_counted)
  e->nl_big = kNlBig;
  if (const char* v = experiment_env("TSG_NL_BIG")) e->nl_big = strtoull(v, nullptr, 10);  // (A/B; 0 = all lazy)
  P.nl_big = e->nl_big;
  P.kw_plain = kKwReadFirst;
  if (const char* v = experiment_env("TSG_KW_PLAIN")) P.kw_plain = strtoull(v, nullptr, 10);  // (A/B)
  P.kw_drain_at = kKwDrainAt;
  if (const char* v = experiment_env("TSG_KW_DRAIN")) P.kw_drain_at = (uint32_t)strtoul(v, nullptr, 10);  // (A/B)
  P.kw_off = experiment_env("TSG_KW_OFF") != nullptr;  // (A/B)
  const bool merge = sp && sp->mode == 2;
  // newline counts: counted lazily after the locations (k_nl_spans), except
  // for a part scan, whose blob exports its range's counts, and a batch of
  // one file the scan would count anyway (span_scan_counted: every span)
  e->nl_lazy = !(sp && sp->mode == 1) && !(nf == 1 && e->nl_big && nbytes > e->nl_big);
  // a lazy scan counts nothing itself (the count-free kernel): the files of
  // nl_big bytes or more inside a multi-file batch are counted by k_nl_spans
  // like the rest (one file that large is its own, counted batch above;
  // TSG_NL_INSCAN keeps the round-5 in-scan counting for A/B)
  if (e->nl_lazy && !experiment_env("TSG_NL_INSCAN")) e->nl_big = P.nl_big = 0;
  e->nl_deferred = false;
  if (e->nl_pending) {  // (an earlier call ended before its lines stage: its side count must not overlap this one)
    HIP_TRY(hipStreamWaitEvent(s, e->ev_nl[1], 0));
    e->nl_pending = false;
  }
  bool scanned = nbytes == 0 || merge;
  if (merge) {  // the scan state comes from the parts (ev[8..9] bracket the import)
    HIP_TRY(hipEventRecord(e->ev[8], s));
    uint64_t nh = 0;
    if ((rc = import_parts(e, rs, P, *sp, &nh))) return rc;
    P.nl_blocks = e->nl_blocks.p;
    P.hits = e->hits.p;
    HIP_TRY(hipMemcpyAsync(&e->ctrl.p->hits, &nh, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(e->ev[9], s));
  }
  Ctrl c_scan{};
  bool have_c = false;  // c_scan holds the counters after the scan (k_uni_keywords changes none)
  // ---- 3. candidates (set up here: k_expand is queued speculatively behind
  // the scan, before the host has read the hit count -- one counter read for
  // both passes instead of one after each; a scan whose buffers overflowed is
  // redone with its candidates, and a candidate list over the speculative
  // capacity is expanded again once the count is known)
  ExpandParams E{};
  auto launch_expand = [&](uint64_t n_hits_host, bool on_device, uint64_t cap) -> int {
    // (every engine buffer read at launch time: launch_scan may have grown
    // region_file / file_kw since this lambda was made)
    E.data = d_data;
    E.off = d_off;
    E.region_file = e->region_file.p;
    E.n_regions = nbytes / kNlBlock + 1;
    E.n_files = nf;
    E.rs = RS;
    E.file_kw = e->file_kw.p;
    E.file_flags = e->file_flags.p;
    E.path_mask = rs->any_path_rules ? e->path_mask.p : nullptr;
    E.rule_words = rule_words;
    E.ctrl = e->ctrl.p;
    E.full_rules = im.u32.p + im.o_full;
    E.n_full_rules = im.n_full;
    HIP_TRY(e->keys.ensure(cap));
    HIP_TRY(e->vals.ensure(cap));
    E.keys = e->keys.p;
    E.vals = e->vals.p;
    E.cand_cap = e->keys.n;
    E.hits = e->hits.p;
    E.hit_cap = hit_cap;
    E.n_hits = n_hits_host;
    E.n_hits_dev = on_device ? &e->ctrl.p->hits : nullptr;
    E.nl_last = nullptr;
    if (e->nl_deferred) {  // the lazy newline counts' reach per file, marked by the candidates' kernels
      HIP_TRY(ensure_side(e));
      HIP_TRY(e->nl_last.ensure(nf));
      E.nl_last = e->nl_last.p;
    }
    HIP_TRY(hipMemsetAsync(&e->ctrl.p->cands, 0, 8, s));
    if (E.nl_last) HIP_TRY(hipMemsetAsync(e->nl_last.p, 0, (size_t)nf * 8, s));
    if (on_device)  // (grid: the last call's hit count + 1/4, the stride covers more; configs[4]'s 2.3 M
                    // hits on a 16-blocks-per-CU grid: k_expand 0.76 -> 0.89 ms, profiles/r06s_ab)
      hipLaunchKernelGGL(k_expand,
                         dim3((uint32_t)std::min<uint64_t>((hit_cap + 255) / 256,
                                                           std::max<uint64_t>(e->num_cus * 16ull, (e->hit_need + 255) / 256))),
                         dim3(256), 0, s, E);
    else if (n_hits_host)
      hipLaunchKernelGGL(k_expand, dim3((uint32_t)((n_hits_host + 255) / 256)), dim3(256), 0, s, E);
    if (nf) hipLaunchKernelGGL(k_full_jobs, dim3((nf + 255) / 256), dim3(256), 0, s, E);
    HIP_TRY(hipGetLastError());
    return TSG_OK;
  };
  const bool spec = !(sp && sp->mode == 1) && !experiment_env("TSG_SPEC_OFF");
  const uint64_t spec_cap = std::max<uint64_t>(1 << 20, e->cand_need);
  bool spec_done = false;  // the successful scan attempt's candidates were expanded with it
  for (int attempt = 0; attempt < 3 && !scanned; ++attempt) {
    HIP_TRY(hipMemsetAsync(e->nl_blocks.p, 0, n_nlb * 4, s));
    HIP_TRY(hipEventRecord(e->ev[8], s));
    if ((rc = launch_scan(e, P))) return rc;
    HIP_TRY(hipEventRecord(e->ev[9], s));
    if (gate_on_side && !gate_pending) {  // (once: a rescan leaves the gates as they are)
      // right after the scan kernel (ev[11]), beside k_report (whose blocks
      // leave VGPRs and wave slots but no LDS: the gate's automaton stays in
      // global memory)
      HIP_TRY(hipStreamWaitEvent(e->side, e->fast_timed ? e->ev[11] : e->ev[9], 0));
      HIP_TRY(hipEventRecord(e->ev_pg[0], e->side));
      G.pac_lds = 0;
      hipLaunchKernelGGL(k_path_gate<false>, dim3(gate_blocks), dim3(256), 0, e->side, G);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(e->ev_pg[1], e->side));
      gate_pending = true;
    }
    // the fold-window pass reads the scan's rune count on the device; one
    // read of the counters afterwards checks every buffer of both passes
    if ((rc = launch_fold_windows(e, P, true))) return rc;
    if (spec) {
      if ((rc = launch_uni_keywords(e, P))) return rc;
      if (gate_pending) HIP_TRY(hipStreamWaitEvent(s, e->ev_pg[1], 0));  // file flags and path masks complete
      HIP_TRY(hipEventRecord(e->ev[2], s));
      if ((rc = launch_expand(0, true, spec_cap))) return rc;
      HIP_TRY(hipEventRecord(e->ev[3], s));
    }
    Ctrl& c = c_scan;
    if ((rc = read_ctrl(e, &c))) return rc;
    have_c = true;
    spec_done = spec;
    const bool ev_lost = (rs->ac.fast.size() || P.big.blob) && c.ev_overflow > e->ev_overflow.n;
    const bool fold_lost = c.n_fold > P.fold_cap;
    const bool outs_lost = P.big.blob && c.outputs > P.big_out_cap;  // (k_big_walk's records)
    if (c.hits <= hit_cap && !ev_lost && !fold_lost && !outs_lost) {
      scanned = true;
      break;
    }
    // overflow: grow and rescan (keyword bits are idempotent)
    if (ev_lost) e->ev_ovf_need = c.ev_overflow + (c.ev_overflow >> 2);
    if (outs_lost) e->big_out_need = c.outputs + (c.outputs >> 2);
    if (fold_lost) {
      e->fold_need = c.n_fold + (c.n_fold >> 2);
      HIP_TRY(e->fold_pos.ensure(e->fold_need));
      P.fold_pos = e->fold_pos.p;
      P.fold_cap = e->fold_pos.n;
    }
    if (c.hits > hit_cap) {
      HIP_TRY(e->hits.ensure(c.hits + (c.hits >> 2)));
      hit_cap = P.hit_cap = e->hits.n;
      P.hits = e->hits.p;
    }
    HIP_TRY(hipMemsetAsync(e->ctrl.p, 0, offsetof(Ctrl, n_caps), s));
  }
  if (!scanned) {
    set_last_error("internal: scan buffers still overflowed after regrowing them twice");
    return TSG_ERR_INTERNAL;
  }
  if (!spec_done) {
    if ((rc = launch_uni_keywords(e, P))) return rc;
    if (gate_pending) HIP_TRY(hipStreamWaitEvent(s, e->ev_pg[1], 0));  // file flags and path masks complete
    HIP_TRY(hipEventRecord(e->ev[2], s));
  }
  Ctrl c = c_scan;
  if (!have_c && (rc = read_ctrl(e, &c))) return rc;  // (one host round trip fewer after a scan)
  const uint64_t n_hits = c.hits;
  const uint64_t scan_overflow = c.ev_overflow;
  const uint64_t n_outputs = c.outputs;
  const uint64_t n_events = scan_overflow + c.events;
  if (sp && sp->mode == 1) return export_part(e, rs, P, n_hits, *sp);
  // files past kMaxVerifyFile: their jobs run the 64-bit instantiations of the
  // search kernels (launched only then)
  const bool any_long = c.long_files != 0 || (merge && sp->file_len > kMaxVerifyFile);
  uint64_t cand_cap = std::max<uint64_t>(1 << 16, n_hits * 2 + nf / 4);
  uint64_t n_cands = 0;
  if (spec_done && c.cands <= E.cand_cap) {
    n_cands = c.cands;
  } else {
    if (spec_done) cand_cap = std::max<uint64_t>(cand_cap, c.cands);
    for (int attempt = 0; attempt < 3; ++attempt) {
      if ((rc = launch_expand(n_hits, false, cand_cap))) return rc;
      if ((rc = read_ctrl(e, &c))) return rc;
      n_cands = c.cands;
      if (n_cands <= E.cand_cap) break;
      if (attempt == 2) {
        set_last_error("internal: candidate buffers still overflowed after regrowing them");
        return TSG_ERR_INTERNAL;
      }
      cand_cap = n_cands;
    }
    HIP_TRY(hipEventRecord(e->ev[3], s));
  }
  e->cand_need = n_cands + n_cands / 4;
  e->hit_need = n_hits + n_hits / 4;
  const bool nl_early = experiment_env("TSG_NL_EARLY") != nullptr;  // (A/B: the count under the candidate sort too)
  if (e->nl_deferred && n_cands && nl_early) {
    HIP_TRY(hipEventRecord(e->ev_nl[0], s));
    HIP_TRY(hipStreamWaitEvent(e->side, e->ev_nl[0], 0));
    const uint64_t n_spans = (nbytes + kNlBlock - 1) / kNlBlock;
    hipLaunchKernelGGL(k_nl_spans, dim3((uint32_t)((n_spans + 255) / 256)), dim3(256), 0, e->side, d_data, nbytes, d_off,
                       e->region_file.p, nbytes / kNlBlock + 1, nf, e->nl_last.p, e->nl_blocks.p, 0u, e->nl_big);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev_nl[1], e->side));
    e->nl_pending = true;
  }
  // ---- 4. sort by (rule, position) and segment into jobs
  uint32_t n_jobs = 0;
  if (n_cands) {
    HIP_TRY(e->keys2.ensure(n_cands));
    HIP_TRY(e->vals2.ensure(n_cands));
    int end_bit = kPosBits;
    while ((1ull << (end_bit - kPosBits)) < RS.n_rules + 1ull) ++end_bit;
    HIP_TRY(sort_pairs(e, e->keys.p, e->keys2.p, e->vals.p, e->vals2.p, n_cands, end_bit, s));
    HIP_TRY(e->flags8.ensure(n_cands));
    HIP_TRY(e->job_start.ensure(n_cands));
    HIP_TRY(e->nsel.ensure(1));
    hipLaunchKernelGGL(k_mark_jobs, dim3((uint32_t)((n_cands + 255) / 256)), dim3(256), 0, s, e->keys2.p,
                       e->vals2.p, n_cands, RS.rules, d_data, e->flags8.p);
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    size_t tmp2 = 0;
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tmp2, cnt, e->flags8.p, e->job_start.p, e->nsel.p,
                                          (int)n_cands, s));
    HIP_TRY(e->cub_tmp.ensure(tmp2 + 1));
    HIP_TRY(hipcub::DeviceSelect::Flagged(e->cub_tmp.p, tmp2, cnt, e->flags8.p, e->job_start.p, e->nsel.p,
                                          (int)n_cands, s));
  }
  if (e->nl_deferred && n_cands && !nl_early) {
    // phase-0 newline counts of the candidate files on the side stream, under
    // the verify (the reach comes from k_expand / k_full_jobs).  Not under the
    // candidate sort: the count's blocks starved its short kernels (0.09 ->
    // 0.6 ms, profiles/r05d)
    HIP_TRY(hipEventRecord(e->ev_nl[0], s));
    HIP_TRY(hipStreamWaitEvent(e->side, e->ev_nl[0], 0));
    const uint64_t n_spans = (nbytes + kNlBlock - 1) / kNlBlock;
    uint32_t nl_blocks0 = (uint32_t)((n_spans + 255) / 256);
    if (const char* v = experiment_env("TSG_NL_BLOCKS_PER_CU"))  // (A/B: a thinner phase-0 grid under k_verify)
      nl_blocks0 = std::min<uint32_t>(nl_blocks0, std::max(1, atoi(v)) * std::max(1u, e->num_cus));
    hipLaunchKernelGGL(k_nl_spans, dim3(nl_blocks0), dim3(256), 0, e->side, d_data, nbytes, d_off,
                       e->region_file.p, nbytes / kNlBlock + 1, nf, e->nl_last.p, e->nl_blocks.p, 0u, e->nl_big);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev_nl[1], e->side));
    e->nl_pending = true;
  }
  // the job count stays on the device: k_verify reads it, and its grid and
  // the location lists are sized from n_cands (>= jobs); the host reads the
  // count with the verify counters
  HIP_TRY(hipEventRecord(e->ev[4], s));
  // ---- 5. verify
  uint64_t loc_cap = std::max<uint64_t>(1 << 16, n_cands);
  uint64_t caps_cap = std::max<uint64_t>(1 << 14, n_cands / 2), caps_big_cap = std::max<uint64_t>(1 << 12, n_cands / 16);
  uint64_t caps_run_cap = std::max<uint64_t>(1 << 14, n_cands);
  uint64_t redo_cap = std::max<uint64_t>(1 << 12, n_cands / 64);
  uint64_t n_locs = 0, n_dropped = 0, n_deferred = 0;
  bool verified = n_cands == 0;
  bool shard_locs = true;  // (A/B: TSG_LOC_SHARDS=0, exp build: one location counter)
#ifdef TSG_EXPERIMENTS
  if (const char* v = getenv("TSG_LOC_SHARDS")) shard_locs = atoi(v) != 0;
#endif
  for (int attempt = 0; attempt < 4 && !verified; ++attempt) {
    // sharded: kLocShards regions of loc_cap / kLocShards (at least 256) and
    // an overflow region of loc_cap; the dense copy goes to locs2
    // (both lists sized from loc_total, never from each other's capacity: they
    // swap roles after every call)
    const uint64_t shard_cap = std::max<uint64_t>(256, loc_cap / kLocShards);
    const uint64_t loc_total = shard_locs ? kLocShards * shard_cap + loc_cap : loc_cap;
    HIP_TRY(e->locs.ensure(loc_total));
    if (shard_locs) {
      HIP_TRY(e->locs2.ensure(loc_total));
      HIP_TRY(e->loc_cnt.ensure(kLocShards + 1));
    }
    HIP_TRY(e->caps.ensure(caps_cap));
    HIP_TRY(e->caps_big.ensure(caps_big_cap));
    HIP_TRY(e->caps_run.ensure(caps_run_cap));
    HIP_TRY(e->job_fms.ensure(n_cands));
    HIP_TRY(e->job_lme.ensure(n_cands));
    HIP_TRY(e->job_bad.ensure(n_cands));
    HIP_TRY(e->redo.ensure(redo_cap));
    HIP_TRY(e->defer.ensure(n_cands));
    HIP_TRY(e->matches.ensure(loc_cap));
    // the verify counters, the location shards and the job flags: one launch
    // (was six fills)
    hipLaunchKernelGGL(k_verify_reset, dim3((uint32_t)std::min<uint64_t>((n_cands + 4095) / 4096 + 1, 4096)), dim3(256),
                       0, s, e->ctrl.p, shard_locs ? e->loc_cnt.p : nullptr, e->job_bad.p, n_cands);
    VerifyParams V{};
    V.data = d_data;
    V.off = d_off;
    V.rs = RS;
    V.keys = e->keys2.p;
    V.vals = e->vals2.p;
    V.n_cands = n_cands;
    V.job_start = e->job_start.p;
    V.n_jobs_dev = e->nsel.p;
    V.locs = e->locs.p;
    V.loc_cap = shard_locs ? loc_total : e->locs.n;
    V.loc_shards = shard_locs ? e->loc_cnt.p : nullptr;
    V.loc_shard_cap = shard_cap;
    V.ctrl = e->ctrl.p;
    V.scratch = e->scratch.p;
    V.scratch_stride = e->scratch_stride;
    V.caps = e->caps.p;
    V.cap_cap = e->caps.n;
    V.caps_big = e->caps_big.p;
    V.cap_big_cap = e->caps_big.n;
    V.caps_run = e->caps_run.p;
    V.cap_run_cap = e->caps_run.n;
    V.job_fms = e->job_fms.p;
    V.job_lme = e->job_lme.p;
    V.split = e->flags8.p;
    V.job_bad = e->job_bad.p;
    V.redo = e->redo.p;
    V.redo_cap = e->redo.n;
    V.defer = e->defer.p;
    V.matches = e->matches.p;
    V.match_cap = e->matches.n;
    V.span_hi = (rs->ac.fast.size() || P.big.blob) && nbytes ? e->span_hi.p : nullptr;
    const bool prof = experiment_env("TSG_PROFILE_VERIFY") != nullptr;
    V.no_accel = experiment_env("TSG_ACCEL") == nullptr;
    V.jpw = 64;
    if (prof) {  // diagnostics only: the job count on the host
      HIP_TRY(hipMemcpyAsync(&n_jobs, e->nsel.p, 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
    }
    if (prof) HIP_TRY(e->vprof.ensure(4ull * n_jobs + 16));
    if (prof) HIP_TRY(hipMemsetAsync(e->vprof.p, 0, (4ull * n_jobs + 16) * 8, s));
    V.prof = prof ? e->vprof.p : nullptr;
    V.tck = prof ? (uint32_t*)(e->vprof.p + 2ull * n_jobs) : nullptr;
    // rule tables back into L2, then the match search (no LDS: full occupancy)
    if (attempt == 0) {
      WarmRanges W{};
      auto add = [&](const void* ptr, uint64_t bytes) {
        if (ptr && bytes && W.k < 10) {
          W.p[W.k] = (const uint8_t*)ptr;
          W.n[W.k++] = bytes;
        }
      };
      add(im.inst.p, im.inst.n * sizeof(gre::Inst));
      add(im.classes.p, im.classes.n * sizeof(gre::ClassDesc));
      add(im.ranges.p, im.ranges.n * 4);
      add(im.progs.p, im.progs.n * sizeof(gre::ProgView));
      add(im.rules.p, im.rules.n * sizeof(RuleDev));
      add(im.dfa_delta.p, im.dfa_delta.n * 2);
      add(im.dfa_bytes.p, im.dfa_bytes.n);
      add(im.u32.p, im.u32.n * 4);
      add(im.nfa.p, im.nfa.n);
      hipLaunchKernelGGL(k_warm, dim3(8 * kWarmParts), dim3(256), 0, s, W, (uint32_t*)e->nsel.p);
      HIP_TRY(hipGetLastError());
    }
    // fast / slow split (k_verify_fast) for long job lists, where occupancy
    // sets the time (configs[4]: 5.09 -> 1.07 ms).  A short list (a few jobs
    // per lane of one wave per CU: configs[2]) ends with its slowest job, and
    // there the single VM-capable kernel with its 64 KiB staged table is
    // quicker (0.43 vs 0.62 ms, profiles/r04e); it also serves the per-job
    // profile (TSG_PROFILE_VERIFY) and A/B (TSG_VERIFY_SINGLE).
    const bool long_list = n_cands > (uint64_t)e->num_cus * kVerifyBlockWide * 4;
    const bool force_split = experiment_env("TSG_VERIFY_SPLIT") != nullptr;  // (A/B: the split on a short list)
    const bool single = (!long_list && !e->verify_split && !force_split) || prof ||
                        experiment_env("TSG_VERIFY_SINGLE") != nullptr;
    if (!single) {
      {
        const uint32_t blocks = (uint32_t)((n_cands + kVerifyBlockWide - 1) / kVerifyBlockWide);
        hipLaunchKernelGGL((k_verify_fast<kVerifyBlockWide, uint32_t>), dim3(std::max(1u, blocks)),
                           dim3(kVerifyBlockWide), 0, s, V);
        if (any_long)
          hipLaunchKernelGGL((k_verify_fast<kVerifyBlockWide, uint64_t>), dim3(std::max(1u, blocks)),
                             dim3(kVerifyBlockWide), 0, s, V);
      }
      // the deferred jobs with the VM-capable paths, then the allow rules of
      // the fast matches (grids: one VM scratch slot per lane)
      hipLaunchKernelGGL(k_verify_slow<uint32_t>, dim3(e->vm_threads / 64), dim3(64), 0, s, V);
      if (any_long) hipLaunchKernelGGL(k_verify_slow<uint64_t>, dim3(e->vm_threads / 64), dim3(64), 0, s, V);
      hipLaunchKernelGGL(k_allow, dim3(e->vm_threads / 64), dim3(64), 0, s, V);
    } else if (n_cands > (uint64_t)e->num_cus * kVerifyBlockWide * 4) {
      const uint32_t blocks = (uint32_t)std::min<uint64_t>((n_cands + kVerifyBlockWide - 1) / kVerifyBlockWide,
                                                           e->vm_threads / kVerifyBlockWide);  // (VM scratch per lane)
      hipLaunchKernelGGL((k_verify<kVerifyBlockWide, uint32_t>), dim3(std::max(1u, blocks)), dim3(kVerifyBlockWide), 0,
                         s, V);
      if (any_long)
        hipLaunchKernelGGL((k_verify<kVerifyBlockWide, uint64_t>), dim3(std::max(1u, blocks)), dim3(kVerifyBlockWide),
                           0, s, V);
    } else {
      // a short list: 64-lane blocks, every lane a job.  Fewer jobs per wave
      // (more waves, 256-lane blocks sharing one staged table) measured
      // slower: 0.75 / 0.81 / 0.95 ms at 32 / 17 / 8 jobs per wave against
      // 0.57 ms (configs[2], profiles/r06b_ab) -- the jobs' own dependent
      // chains, not the wave's lock-step union of them, set the time
      uint32_t blk = kVerifyBlock;
#ifdef TSG_EXPERIMENTS
      if (const char* v = getenv("TSG_VERIFY_JPW")) {  // (A/B: 256-lane blocks, jpw jobs per wave)
        blk = kVerifyBlockWide;
        V.jpw = (uint32_t)std::max(1, std::min(64, atoi(v)));
      }
#endif
      const uint32_t per_block = blk / 64 * V.jpw;
      const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_cands + per_block - 1) / per_block,
                                                                                  e->vm_threads / per_block));
      if (blk == kVerifyBlockWide) {
        hipLaunchKernelGGL((k_verify<kVerifyBlockWide, uint32_t>), dim3(blocks), dim3(kVerifyBlockWide), 0, s, V);
        if (any_long)
          hipLaunchKernelGGL((k_verify<kVerifyBlockWide, uint64_t>), dim3(blocks), dim3(kVerifyBlockWide), 0, s, V);
      } else {
        hipLaunchKernelGGL((k_verify<kVerifyBlock, uint32_t>), dim3(blocks), dim3(kVerifyBlock), 0, s, V);
        if (any_long) hipLaunchKernelGGL((k_verify<kVerifyBlock, uint64_t>), dim3(blocks), dim3(kVerifyBlock), 0, s, V);
      }
    }
    // speculative chains: conflicts re-run in order (grid: one lane per job
    // start at most; the re-run grid keeps every lane's VM scratch slot below
    // vm_threads)
    hipLaunchKernelGGL(k_chain_fix, dim3((uint32_t)((n_cands + 255) / 256)), dim3(256), 0, s, V);
    hipLaunchKernelGGL(k_verify_redo<uint32_t>, dim3(e->num_cus * 2), dim3(64), 0, s, V);
    if (any_long) hipLaunchKernelGGL(k_verify_redo<uint64_t>, dim3(e->num_cus * 2), dim3(64), 0, s, V);
    HIP_TRY(hipGetLastError());
    // capture stages over the device-side lists: 8 searching lanes per wave with
    // 560-word arenas, then one lane per wave with 36 KiB for what does not fit
    // (grids keep every lane's VM scratch slot below vm_threads: 512 / 256 per CU)
    hipLaunchKernelGGL(k_group_runs<uint32_t>, dim3(e->num_cus * 4), dim3(256), 0, s, V);
    if (any_long) hipLaunchKernelGGL(k_group_runs<uint64_t>, dim3(e->num_cus * 4), dim3(256), 0, s, V);
    hipLaunchKernelGGL((k_captures<64, kCapActive, kBsWords, false, uint32_t>), dim3(e->num_cus * 8), dim3(64), 0, s, V);
    if (any_long)
      hipLaunchKernelGGL((k_captures<64, kCapActive, kBsWords, false, uint64_t>), dim3(e->num_cus * 8), dim3(64), 0, s,
                         V);
    hipLaunchKernelGGL((k_captures<64, 1, kBigBsWords, true, uint32_t>), dim3(e->num_cus * 4), dim3(64), 0, s, V);
    if (any_long)
      hipLaunchKernelGGL((k_captures<64, 1, kBigBsWords, true, uint64_t>), dim3(e->num_cus * 4), dim3(64), 0, s, V);
    if (shard_locs) {  // the shard regions packed densely into locs2; k_drop_spec works on that
      hipLaunchKernelGGL(k_loc_compact, dim3(kLocShards + 1), dim3(256), 0, s, V, e->locs2.p);
      VerifyParams D = V;
      D.locs = e->locs2.p;
      D.loc_cap = loc_total;
      D.loc_shards = nullptr;
      hipLaunchKernelGGL(k_drop_spec, dim3(e->num_cus * 4), dim3(256), 0, s, D);
    } else {
      hipLaunchKernelGGL(k_drop_spec, dim3(e->num_cus * 4), dim3(256), 0, s, V);
    }
    HIP_TRY(hipGetLastError());
    if (prof) {  // the jobs that end last (their waves set k_verify's length), per-rule totals
      std::vector<uint64_t> hp(4ull * n_jobs);
      std::vector<uint32_t> hjs(n_jobs);
      HIP_TRY(hipMemcpyAsync(hp.data(), e->vprof.p, hp.size() * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(hjs.data(), e->job_start.p, n_jobs * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      auto dur = [&](uint32_t q) { return hp[2 * q] & 0xFFFFFFFFull; };
      auto end = [&](uint32_t q) { return hp[2 * q] >> 32; };
      uint64_t tmin = ~0ull;
      for (uint32_t q = 0; q < n_jobs; ++q) tmin = std::min<uint64_t>(tmin, end(q) - dur(q));
      std::vector<uint32_t> idx(n_jobs);
      for (uint32_t q = 0; q < n_jobs; ++q) idx[q] = q;
      std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return end(a) > end(b); });
      fprintf(stderr, "[verify] kernel span %.3f ms\n", (end(idx[0]) - tmin) / 1e5);
      {  // job end times and durations by percentile (a tail-bound kernel ends late for a few jobs)
        std::vector<uint64_t> ends(n_jobs), durs(n_jobs);
        for (uint32_t q = 0; q < n_jobs; ++q) {
          ends[q] = end(q) - tmin;
          durs[q] = dur(q);
        }
        std::sort(ends.begin(), ends.end());
        std::sort(durs.begin(), durs.end());
        auto pct = [&](const std::vector<uint64_t>& v, double f) { return v[std::min<size_t>(v.size() - 1, (size_t)(f * v.size()))] / 1e5; };
        fprintf(stderr, "[verify] job ends p50 %.3f p90 %.3f p99 %.3f p99.9 %.3f max %.3f ms; durations p50 %.3f p90 %.3f p99 %.3f max %.3f ms\n",
                pct(ends, 0.5), pct(ends, 0.9), pct(ends, 0.99), pct(ends, 0.999), ends.back() / 1e5, pct(durs, 0.5),
                pct(durs, 0.9), pct(durs, 0.99), durs.back() / 1e5);
      }
      for (uint32_t q = 0; q < std::min<uint32_t>(16, n_jobs); ++q) {
        const uint32_t jq = idx[q];
        const uint64_t c0 = hjs[jq], c1 = jq + 1 < n_jobs ? hjs[jq + 1] : n_cands;
        const uint32_t* tk = (const uint32_t*)(hp.data() + 2ull * n_jobs) + 4 * jq;
        fprintf(stderr,
                "[verify] job %u dur %.3f ms end %.3f ms rule %s full %llu dfa steps %llu cands %llu dfa %.3f emit %.3f "
                "(global allow %.3f)\n",
                jq, dur(jq) / 1e5, (end(jq) - tmin) / 1e5, rs->rules[hp[2 * jq + 1] >> 32].id.c_str(),
                (unsigned long long)(hp[2 * jq + 1] & 1), (unsigned long long)((hp[2 * jq + 1] & 0xFFFFFFFFull) >> 1),
                (unsigned long long)(c1 - c0), tk[0] / 1e5, tk[1] / 1e5, tk[2] / 1e5);
      }
      {  // the jobs with the most DFA steps and the most candidates (the work, not the wave's wait)
        std::vector<uint32_t> by(n_jobs);
        for (uint32_t q = 0; q < n_jobs; ++q) by[q] = q;
        auto steps = [&](uint32_t q) { return (hp[2 * q + 1] & 0xFFFFFFFFull) >> 1; };
        auto cands = [&](uint32_t q) { return (uint64_t)((q + 1 < n_jobs ? hjs[q + 1] : n_cands) - hjs[q]); };
        std::partial_sort(by.begin(), by.begin() + std::min<uint32_t>(8, n_jobs), by.end(),
                          [&](uint32_t a, uint32_t b) { return steps(a) > steps(b); });
        for (uint32_t q = 0; q < std::min<uint32_t>(8, n_jobs); ++q)
          fprintf(stderr, "[verify] top-steps job %u rule %s file %u steps %llu cands %llu dur %.3f ms\n", by[q],
                  rs->rules[hp[2 * by[q] + 1] >> 32].id.c_str(), 0u, (unsigned long long)steps(by[q]),
                  (unsigned long long)cands(by[q]), dur(by[q]) / 1e5);
        std::partial_sort(by.begin(), by.begin() + std::min<uint32_t>(8, n_jobs), by.end(),
                          [&](uint32_t a, uint32_t b) { return dur(a) > dur(b); });
        for (uint32_t q = 0; q < std::min<uint32_t>(8, n_jobs); ++q) {
          const uint32_t* tk = (const uint32_t*)(hp.data() + 2ull * n_jobs) + 4 * by[q];
          fprintf(stderr, "[verify] top-dur job %u rule %s steps %llu cands %llu dur %.3f ms dfa %.3f emit %.3f allow %.3f full %llu\n",
                  by[q], rs->rules[hp[2 * by[q] + 1] >> 32].id.c_str(), (unsigned long long)steps(by[q]),
                  (unsigned long long)cands(by[q]), dur(by[q]) / 1e5, tk[0] / 1e5, tk[1] / 1e5, tk[2] / 1e5,
                  (unsigned long long)(hp[2 * by[q] + 1] & 1));
        }
        std::partial_sort(by.begin(), by.begin() + std::min<uint32_t>(8, n_jobs), by.end(),
                          [&](uint32_t a, uint32_t b) { return cands(a) > cands(b); });
        for (uint32_t q = 0; q < std::min<uint32_t>(8, n_jobs); ++q)
          fprintf(stderr, "[verify] top-cands job %u rule %s steps %llu cands %llu dur %.3f ms full %llu\n", by[q],
                  rs->rules[hp[2 * by[q] + 1] >> 32].id.c_str(), (unsigned long long)steps(by[q]),
                  (unsigned long long)cands(by[q]), dur(by[q]) / 1e5, (unsigned long long)(hp[2 * by[q] + 1] & 1));
      }
      std::map<uint32_t, std::pair<uint64_t, uint64_t>> per_rule;
      std::map<uint32_t, std::pair<uint64_t, uint64_t>> per_rule_n;  // jobs, DFA / NFA steps
      for (uint32_t q = 0; q < n_jobs; ++q) {
        auto& pr = per_rule[(uint32_t)(hp[2 * q + 1] >> 32)];
        pr.first += dur(q);
        pr.second = std::max<uint64_t>(pr.second, dur(q));
        auto& pn = per_rule_n[(uint32_t)(hp[2 * q + 1] >> 32)];
        pn.first += 1;
        pn.second += (hp[2 * q + 1] & 0xFFFFFFFFull) >> 1;
      }
      for (auto& kv : per_rule)
        fprintf(stderr, "[verify] rule %s total %.3f ms max %.3f ms jobs %llu steps %llu\n",
                rs->rules[kv.first].id.c_str(), kv.second.first / 1e5, kv.second.second / 1e5,
                (unsigned long long)per_rule_n[kv.first].first, (unsigned long long)per_rule_n[kv.first].second);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&n_jobs, e->nsel.p, 4, hipMemcpyDeviceToHost, s));  // (read by read_ctrl's sync)
    if ((rc = read_ctrl(e, &c))) return rc;
    n_locs = c.locs;
    n_dropped = c.n_dropped;
    n_deferred = c.n_defer;
    if (n_locs <= V.loc_cap && c.n_caps <= e->caps.n && c.n_caps_big <= e->caps_big.n &&
        c.n_redo <= e->redo.n && c.n_caps_run <= e->caps_run.n && c.n_match <= e->matches.n) {
      verified = true;
      if (shard_locs) std::swap(e->locs, e->locs2);  // the dense list is the location list from here on
      break;
    }
    // a list overflowed: grow it and re-run the search and the capture stages
    loc_cap = std::max<uint64_t>({loc_cap, n_locs, c.n_match});
    caps_cap = std::max<uint64_t>(caps_cap, c.n_caps);
    caps_big_cap = std::max<uint64_t>(caps_big_cap, c.n_caps_big);
    redo_cap = std::max<uint64_t>(redo_cap, c.n_redo);
    caps_run_cap = std::max<uint64_t>(caps_run_cap, c.n_caps_run);
  }
  if (!verified) {
    set_last_error("internal: location buffers still overflowed after regrowing them");
    return TSG_ERR_INTERNAL;
  }
  if (c.err & 2u) {
    set_last_error("a match of 4 GiB or more: its allow regexes would run past 32-bit match strings");
    return TSG_ERR_UNSUPPORTED;
  }
  if (c.err) {
    set_last_error("internal: capture re-run disagreed with the whole-match run");
    return TSG_ERR_INTERNAL;
  }
  if (n_dropped) {  // the conflicting speculative jobs' locations out (rare): compact in order
    HIP_TRY(e->locs2.ensure(n_locs));
    HIP_TRY(e->flags8.ensure(n_locs));
    HIP_TRY(e->nsel.ensure(2));
    hipLaunchKernelGGL(k_keep_flags, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p, n_locs,
                       e->flags8.p);
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tmp, e->locs.p, e->flags8.p, e->locs2.p, e->nsel.p + 1,
                                          (int)n_locs, s));
    HIP_TRY(e->cub_tmp.ensure(tmp + 1));
    HIP_TRY(hipcub::DeviceSelect::Flagged(e->cub_tmp.p, tmp, e->locs.p, e->flags8.p, e->locs2.p, e->nsel.p + 1,
                                          (int)n_locs, s));
    n_locs -= n_dropped;
    HIP_TRY(hipMemcpyAsync(e->locs.p, e->locs2.p, n_locs * sizeof(DevLoc), hipMemcpyDeviceToDevice, s));
  }
  HIP_TRY(hipEventRecord(e->ev[5], s));
  // ---- 6. exclude blocks (only when the config has any)
  if (n_locs && rs->any_exclude) {
    // (device-only: the (file, scope) groups, their FindAll ranges and the
    // containment filter; the host reads two counts)
    ExclDev X{im.u32.p + im.o_xoff, im.u32.p + im.o_xprog, im.u32.p + im.o_gx, im.n_gx, std::max(1u, im.max_x)};
    const uint64_t nk = 2 * n_locs;
    if (nk >= (1ull << (64 - kKeyPosBits))) {  // group ids share the range sort key with 40-bit starts
      set_last_error("exclude blocks: more than 2^23 locations in one batch");
      return TSG_ERR_UNSUPPORTED;
    }
    HIP_TRY(e->keys.ensure(nk));
    HIP_TRY(e->keys2.ensure(nk));
    HIP_TRY(e->vals.ensure(nk));
    HIP_TRY(e->vals2.ensure(nk));
    HIP_TRY(e->job_start.ensure(nk));
    HIP_TRY(e->flags8.ensure(std::max<uint64_t>(nk, n_locs)));
    HIP_TRY(e->nsel.ensure(2));
    hipLaunchKernelGGL(k_excl_keys, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p, n_locs, X,
                       e->keys.p, e->vals.p);
    size_t tmp = 0;
    HIP_TRY(sort_pairs(e, e->keys.p, e->keys2.p, e->vals.p, e->vals2.p, nk, 64, s));
    hipLaunchKernelGGL(k_excl_uniq, dim3((uint32_t)((nk + 255) / 256)), dim3(256), 0, s, e->keys2.p, nk,
                       e->flags8.p);
    HIP_TRY(hipGetLastError());
    // the groups: indices of the unique sorted keys (tidx = job_start[0, n_tags));
    // n_tags stays on the device
    {
      hipcub::CountingInputIterator<uint32_t> cnt(0);
      HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tmp, cnt, e->flags8.p, e->job_start.p, e->nsel.p, (int)nk, s));
      HIP_TRY(e->cub_tmp.ensure(tmp + 1));
      HIP_TRY(hipcub::DeviceSelect::Flagged(e->cub_tmp.p, tmp, cnt, e->flags8.p, e->job_start.p, e->nsel.p, (int)nk,
                                            s));
    }
    uint64_t cap = std::max<uint64_t>(1 << 16, n_locs);
    for (int attempt = 0; attempt < 3; ++attempt) {
      HIP_TRY(e->excl_out.ensure(cap));
      HIP_TRY(hipMemsetAsync(&e->ctrl.p->excl, 0, 8, s));
      const uint32_t blocks = std::min<uint32_t>((uint32_t)((nk * X.max_x + 255) / 256), e->vm_threads / 256);
      hipLaunchKernelGGL(k_exclude_tags, dim3(std::max(1u, blocks)), dim3(256), 0, s, d_data, d_off, RS, X,
                         (const uint64_t*)e->keys2.p, (const uint32_t*)e->job_start.p, (const uint32_t*)e->nsel.p,
                         e->excl_out.p, (uint64_t)e->excl_out.n, e->ctrl.p, e->scratch.p, e->scratch_stride);
      HIP_TRY(hipGetLastError());
      if ((rc = read_ctrl(e, &c))) return rc;
      if (c.excl <= e->excl_out.n) break;
      if (attempt == 2) {
        set_last_error("internal: exclude-block buffers still overflowed after regrowing them");
        return TSG_ERR_INTERNAL;
      }
      cap = c.excl;
    }
    const uint64_t n_r = c.excl;
    // ranges sorted by (group, start), running max of the ends per group
    HIP_TRY(e->f_iv.ensure(n_r + 1));     // keys
    HIP_TRY(e->f_lkey2.ensure(n_r + 1));  // sorted keys
    HIP_TRY(e->f_ssrc.ensure(n_r + 1));   // running max of the ends
    HIP_TRY(e->f_lslot.ensure(n_r + 1));  // range index
    HIP_TRY(e->f_lslot2.ensure(n_r + 1)); // ... in sorted order
    if (n_r) {
      hipLaunchKernelGGL(k_excl_rkeys, dim3((uint32_t)((n_r + 255) / 256)), dim3(256), 0, s, e->excl_out.p, n_r,
                         e->f_iv.p, e->f_lslot.p);
      HIP_TRY(sort_pairs(e, e->f_iv.p, e->f_lkey2.p, e->f_lslot.p, e->f_lslot2.p, n_r, 64, s));
      hipLaunchKernelGGL(k_excl_pmax, dim3((uint32_t)((n_r + 255) / 256)), dim3(256), 0, s, e->f_lkey2.p,
                         e->f_lslot2.p, e->excl_out.p, e->f_ssrc.p, n_r);
    }
    hipLaunchKernelGGL(k_excl_filter, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p, n_locs,
                       X, (const uint64_t*)e->keys2.p, (const uint32_t*)e->job_start.p, (const uint32_t*)e->nsel.p,
                       e->f_lkey2.p, e->f_ssrc.p, n_r, e->flags8.p);
    HIP_TRY(hipGetLastError());
    // the kept locations, compacted in order (a non-participating group never
    // reaches censoring in Go if excluded)
    HIP_TRY(e->locs2.ensure(n_locs));
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tmp, e->locs.p, e->flags8.p, e->locs2.p, e->nsel.p + 1,
                                          (int)n_locs, s));
    HIP_TRY(e->cub_tmp.ensure(tmp + 1));
    HIP_TRY(hipcub::DeviceSelect::Flagged(e->cub_tmp.p, tmp, e->locs.p, e->flags8.p, e->locs2.p, e->nsel.p + 1,
                                          (int)n_locs, s));
    uint32_t kept = 0;
    HIP_TRY(hipMemcpyAsync(&kept, e->nsel.p + 1, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    n_locs = kept;
    if (n_locs)
      HIP_TRY(hipMemcpyAsync(e->locs.p, e->locs2.p, n_locs * sizeof(DevLoc), hipMemcpyDeviceToDevice, s));
  }
  HIP_TRY(hipEventRecord(e->ev[6], s));
  if (!n_locs && e->nl_pending) {  // no lines stage: the side count reads the caller's batch, so the call's
    HIP_TRY(hipStreamWaitEvent(s, e->ev_nl[1], 0));  // final synchronisation must cover it
    e->nl_pending = false;
  }
  // ---- 7. line numbers
  if (n_locs) {
    const int n_nlb = (int)(nbytes / kNlBlock + 2);
    if (e->nl_deferred) {  // the scan skipped the newline counts: what the location files' searches reach
      const uint64_t n_spans = (nbytes + kNlBlock - 1) / kNlBlock;
      const uint32_t span_blocks = (uint32_t)((n_spans + 255) / 256);
      if (!e->nl_pending) {  // (no candidate pass ran: count every location file whole)
        HIP_TRY(e->nl_last.ensure(nf));
        HIP_TRY(hipMemsetAsync(e->nl_last.p, 0, (size_t)nf * 8, s));
      } else {
        HIP_TRY(hipStreamWaitEvent(s, e->ev_nl[1], 0));
        e->nl_pending = false;
      }
      hipLaunchKernelGGL(k_nl_check, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p, n_locs,
                         d_off, e->nl_last.p);
      hipLaunchKernelGGL(k_nl_tail, dim3((nf + 255) / 256), dim3(256), 0, s, d_off, nf, e->nl_blocks.p, n_spans,
                         e->nl_last.p);
      hipLaunchKernelGGL(k_nl_spans, dim3(span_blocks), dim3(256), 0, s, d_data, nbytes, d_off, e->region_file.p,
                         nbytes / kNlBlock + 1, nf, e->nl_last.p, e->nl_blocks.p, 1u, e->nl_big);
      HIP_TRY(hipGetLastError());
    }
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->nl_blocks.p, e->nl_pre.p, n_nlb, s));
    HIP_TRY(e->cub_tmp.ensure(tmp + 1));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->nl_blocks.p, e->nl_pre.p, n_nlb, s));
    // order by (file, start) on the device (censored_lines walks files in order)
    HIP_TRY(e->keys.ensure(n_locs));
    HIP_TRY(e->keys2.ensure(n_locs));
    HIP_TRY(e->vals.ensure(n_locs));
    HIP_TRY(e->vals2.ensure(n_locs));
    HIP_TRY(e->locs2.ensure(n_locs));
    hipLaunchKernelGGL(k_loc_keys, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p, n_locs,
                       e->keys.p, e->vals.p);
    HIP_TRY(sort_pairs(e, e->keys.p, e->keys2.p, e->vals.p, e->vals2.p, n_locs, 64, s));
    hipLaunchKernelGGL(k_loc_gather, dim3((uint32_t)((n_locs + 255) / 256)), dim3(256), 0, s, e->locs.p,
                       e->vals2.p, n_locs, e->locs2.p);
    if ((rc = dense_begin(e, d_data, d_off, nbytes, n_locs))) return rc;
    HIP_TRY(e->fbase.ensure(nf + 1));
    hipLaunchKernelGGL(k_file_base, dim3((uint32_t)((n_locs * 64 + 255) / 256)), dim3(256), 0, s, d_data, d_off,
                       e->nl_pre.p, e->locs2.p, n_locs, e->fbase.p);
    hipLaunchKernelGGL(k_lines, dim3((uint32_t)((n_locs * 64 + 255) / 256)), dim3(256), 0, s, d_data, d_off,
                       e->nl_pre.p, e->fbase.p, e->locs2.p, n_locs);
    HIP_TRY(hipGetLastError());
    if ((rc = dense_issue(e, d_data, d_off, nbytes, n_locs, res))) {
      if (e->side) (void)hipStreamSynchronize(e->side);
      return rc;
    }
    // ---- 8. findings (censored lines, Match, Code, order) on the device
    if ((rc = build_findings_dev(e, d_data, d_off, nbytes, nf, n_locs, res))) {
      if (e->side) (void)hipStreamSynchronize(e->side);  // no side copy may outlive the result block
      return rc;
    }
  }
  HIP_TRY(hipEventRecord(e->ev[7], s));
  auto& R = res->impl;
  if (!n_locs) {  // no findings: the block holds the flags and the counters
    R.arena = pinned_get(e->pinned, ((size_t)nf + 15) / 16 * 16 + sizeof(Ctrl));
    if (!R.arena) {
      set_last_error("hipHostMalloc failed for the result block");
      return TSG_ERR_DEVICE;
    }
    R.file_flags = {(uint8_t*)R.arena->p, nf};
    R.ctrl_off = ((size_t)nf + 15) / 16 * 16;
  }
  // per-file flags as bytes, and the counters, into the result's block
  if (nf) {
    HIP_TRY(e->fflags8.ensure(nf));
    hipLaunchKernelGGL(k_flags8, dim3((nf + 255) / 256), dim3(256), 0, s, e->file_flags.p, e->fflags8.p, nf);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(R.file_flags.p, e->fflags8.p, nf, hipMemcpyDeviceToHost, s));
  }
  Ctrl* hc = (Ctrl*)((uint8_t*)R.arena->p + R.ctrl_off);
  HIP_TRY(hipMemcpyAsync(hc, e->ctrl.p, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if ((rc = dma_wait(e))) return rc;
  const auto wall1 = std::chrono::steady_clock::now();
  for (int k = 0; k < 7; ++k) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev[k], e->ev[k + 1]));
    tm[k] = ms;
  }
  if (gate_pending) {  // the path gate ran on the side stream: its own time
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev_pg[0], e->ev_pg[1]));
    tm[0] = ms;
  }

  tm[8] = (double)n_hits;
  tm[9] = (double)n_cands;
  tm[10] = (double)n_jobs;
  tm[11] = (double)n_locs;
  tm[12] = (double)scan_overflow;
  tm[13] = (double)n_events;
  tm[14] = (double)n_outputs;
  tm[23] = (double)n_deferred;
  if (nbytes) {  // k_scan alone (the dominant, HBM-bound kernel)
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev[8], e->ev[9]));
    tm[7] = ms;
  }
  if (e->fast_timed) {  // k_scan_fast alone
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev[10], e->ev[11]));
    tm[17] = ms;
  }
  if (hc->n_panic) {
    set_last_error("secret group did not participate in the match (the Go reference panics here)");
    return TSG_ERR_PANIC;
  }
  R.ties.n = n_locs ? (size_t)std::min<unsigned long long>(hc->n_ties, R.ties_cap) : 0;
#ifdef TSG_EXPERIMENTS
  const auto wall_t = std::chrono::steady_clock::now();
#endif
  order_finding_ties(R, hc->n_ties > R.ties_cap);
  R.have_findings = true;
  const auto wall2 = std::chrono::steady_clock::now();
#ifdef TSG_EXPERIMENTS
  fprintf(stderr, "[post] locs %.3f ms, tie order %.3f ms (%zu records, %zu ties)\n",
          std::chrono::duration<double, std::milli>(wall_t - wall1).count(),
          std::chrono::duration<double, std::milli>(wall2 - wall_t).count(), R.frec.size(), R.ties.n);
#endif
  tm[15] = std::chrono::duration<double, std::milli>(wall2 - wall0).count();  // whole call, host clock
  tm[16] = std::chrono::duration<double, std::milli>(wall2 - wall1).count();  // host post-processing
  return TSG_OK;
}

}  // namespace

namespace tsg {
PinnedPool::~PinnedPool() {
  for (auto& b : free_blocks) (void)hipHostFree(b.first);
}
PinnedBlock::~PinnedBlock() {
  if (!p) return;
  std::lock_guard<std::mutex> lk(pool->mu);
  if (pool->free_blocks.size() < 4) pool->free_blocks.push_back({p, n});
  else (void)hipHostFree(p);
}
std::shared_ptr<PinnedBlock> pinned_get(const std::shared_ptr<PinnedPool>& pool, size_t bytes) {
  auto b = std::make_shared<PinnedBlock>();
  b->pool = pool;
  {
    std::lock_guard<std::mutex> lk(pool->mu);
    size_t best = (size_t)-1;
    for (size_t i = 0; i < pool->free_blocks.size(); ++i)
      if (pool->free_blocks[i].second >= bytes && (best == (size_t)-1 || pool->free_blocks[i].second < pool->free_blocks[best].second))
        best = i;
    if (best != (size_t)-1) {
      b->p = pool->free_blocks[best].first;
      b->n = pool->free_blocks[best].second;
      pool->free_blocks.erase(pool->free_blocks.begin() + best);
      return b;
    }
  }
  const size_t n = std::max<size_t>(1 << 20, bytes + bytes / 4);
  if (hipHostMalloc(&b->p, n, hipHostMallocDefault) != hipSuccess) {
    b->p = nullptr;
    return nullptr;
  }
  b->n = n;
  return b;
}
}  // namespace tsg

extern "C" {

const char* tsg_version(void) { return "trivy-secret-mi355x 0.1 (gfx950)"; }

int tsg_engine_create(int device, tsg_engine** out) {
  if (!out) return TSG_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
    set_last_error("no HIP device available: the MI355X engine has no CPU fallback");
    return TSG_ERR_NO_DEVICE;
  }
  auto* e = new tsg_engine();
  e->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    set_last_error("hipSetDevice/hipStreamCreate failed");
    delete e;
    return TSG_ERR_DEVICE;
  }
  *out = e;
  return TSG_OK;
}

void tsg_engine_free(tsg_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  e->img.release();
  e->data.release(); e->off.release(); e->paths.release(); e->path_off.release();
  e->file_kw.release(); e->file_flags.release(); e->path_mask.release(); e->hits.release();
  e->keys.release(); e->keys2.release(); e->vals.release(); e->vals2.release(); e->flags8.release();
  e->job_start.release(); e->nsel.release(); e->cub_tmp.release(); e->locs.release(); e->locs2.release();
  e->hit_seg.release(); e->hit_pre.release(); e->hit_seg_n.release(); e->loc_cnt.release(); e->ev_pre.release();
  e->scratch.release(); e->ctrl.release(); e->excl_out.release(); e->part_buf.release(); e->caps_run.release();
  e->nl_blocks.release(); e->nl_pre.release(); e->tail.release(); e->region_file.release(); e->region_tmp.release();
  e->ev_buf.release(); e->ev_overflow.release(); e->ev_counts.release(); e->span_hi.release(); e->fold_pos.release(); e->caps.release(); e->caps_big.release();
  e->job_fms.release(); e->job_lme.release(); e->job_bad.release(); e->redo.release(); e->vprof.release(); e->fflags8.release();
  if (e->h_stage) (void)hipHostFree(e->h_stage);
  e->gate_out.release(); e->gate_rules.release(); e->bin8.release(); e->strip_out.release();
  e->strip_off.release(); e->blk_kept.release(); e->blk_base.release(); e->chunk_pos.release(); e->n_drop.release();
  e->f_iv.release(); e->f_lkey.release(); e->f_lkey2.release(); e->f_ssrc.release(); e->f_slen.release();
  e->f_soff.release(); e->f_lslot.release(); e->f_lslot2.release(); e->f_lhead.release(); e->f_lscan.release();
  e->f_luid.release(); e->f_sfile.release(); e->f_sgrp.release(); e->f_grp.release();
  e->f_rec.release(); e->f_rec2.release(); e->f_arena.release();
  e->f_gran.release(); e->f_gcarry.release(); e->big_outs.release(); e->f_lkeyb.release();
  e->f_ties.release(); e->out_locs.release(); e->gate_defer.release();
  e->f_dsize.release(); e->f_doff.release(); e->f_dense_at.release(); e->f_gstart.release(); e->f_dense.release();
  e->f_pmax.release(); e->f_spidx.release(); e->f_long.release();
  if (e->h_dense) (void)hipHostFree(e->h_dense);
  if (e->h_find) (void)hipHostFree(e->h_find);
  if (e->dma_sig.handle) {
    (void)dma_wait(e);
    (void)hsa_signal_destroy(e->dma_sig);
  }
  if (e->events)
    for (auto& ev : e->ev) (void)hipEventDestroy(ev);
  if (e->side) {
    (void)hipStreamSynchronize(e->side);
    (void)hipEventDestroy(e->ev_code);
    (void)hipEventDestroy(e->ev_fill);
    (void)hipEventDestroy(e->ev_side);
    (void)hipEventDestroy(e->ev_dense);
    (void)hipEventDestroy(e->ev_dfill);
    (void)hipEventDestroy(e->ev_frec);
    (void)hipEventDestroy(e->ev_fb);
    (void)hipEventDestroy(e->ev_nl[0]);
    (void)hipEventDestroy(e->ev_nl[1]);
    (void)hipEventDestroy(e->ev_pg[0]);
    (void)hipEventDestroy(e->ev_pg[1]);
    (void)hipStreamDestroy(e->side);
  }
  (void)hipStreamDestroy(e->stream);
  delete e;
}

static int scan_impl(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files,
                     tsg_result** out);
static int scan_device_impl(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data,
                            const uint64_t* d_offsets, const uint8_t* d_paths,
                            const uint64_t* d_path_offsets, size_t n_files, tsg_result** out);

// The C ABI never lets a C++ exception escape (never abort).
int tsg_scan(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files, tsg_result** out) {
  try {
    return scan_impl(e, rs, files, n_files, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

int tsg_scan_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data, const uint64_t* d_offsets,
                    const uint8_t* d_paths, const uint64_t* d_path_offsets, size_t n_files, tsg_result** out) {
  try {
    return scan_device_impl(e, rs, d_data, d_offsets, d_paths, d_path_offsets, n_files, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

// One-file batch layout for the split entry points: offsets {0, len + 1} and
// the path, in the engine's own staging buffers.
static int stage_one_file(tsg_engine* e, uint64_t len, const char* path) {
  const uint64_t off[2] = {0, len + 1};
  const size_t plen = path ? strlen(path) : 0;
  const uint64_t poff[2] = {0, plen};
  if (e->off.ensure(2) != hipSuccess || e->paths.ensure(plen + 16) != hipSuccess || e->path_off.ensure(2) != hipSuccess) {
    set_last_error("hipMalloc failed");
    return TSG_ERR_DEVICE;
  }
  HIP_TRY(hipMemcpy(e->off.p, off, 16, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->path_off.p, poff, 16, hipMemcpyHostToDevice));
  if (plen) HIP_TRY(hipMemcpy(e->paths.p, path, plen, hipMemcpyHostToDevice));
  return TSG_OK;
}

int tsg_part_halo(const tsg_ruleset* rs, uint64_t* left, uint64_t* right) {
  if (!rs || !left || !right) return TSG_ERR_INVALID_ARG;
  *left = kNlBlock;
  *right = part_right_halo(rs);
  return TSG_OK;
}

static int scan_part_impl(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_text, uint64_t text_base,
                          uint64_t text_len, uint64_t own_lo, uint64_t own_hi, uint64_t file_len, const char* path,
                          uint8_t** blob, size_t* blob_len) {
  if (!e || !rs || !blob || !blob_len || (text_len && !d_text)) return TSG_ERR_INVALID_ARG;
  *blob = nullptr;
  *blob_len = 0;
  const uint64_t left = kNlBlock, right = part_right_halo(rs);
  const bool aligned = text_base % kNlBlock == 0 && own_lo % kNlBlock == 0 && (own_hi % kNlBlock == 0 || own_hi == file_len);
  const bool covers = own_lo < own_hi && own_hi <= file_len && text_base + std::min(own_lo, left) <= own_lo &&
                      text_base + text_len >= std::min(file_len, own_hi + right) && text_base + text_len <= file_len;
  if (!aligned || !covers || text_len >= kMaxFileBytes) {
    set_last_error("split: the part's view does not satisfy tsg_part_halo / 4 KiB alignment");
    return TSG_ERR_INVALID_ARG;
  }
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  if (text_base + text_len == file_len) {  // the view reaches the file end: its extra byte is the NUL separator
    uint8_t sep = 1;
    HIP_TRY(hipMemcpy(&sep, d_text + text_len, 1, hipMemcpyDeviceToHost));
    if (sep != 0) {
      set_last_error("split: a view that ends at the file end must be followed by the NUL separator");
      return TSG_ERR_INVALID_ARG;
    }
  }
  int rc = stage_one_file(e, text_len, path);
  if (rc) return rc;
  SplitIo sp;
  sp.mode = 1;
  sp.text_base = text_base;
  sp.own_lo = own_lo;
  sp.own_hi = own_hi;
  sp.file_len = file_len;
  sp.blob_out = blob;
  sp.blob_len = blob_len;
  tsg_result tmp;
  return run_pipeline(e, rs, d_text, e->off.p, e->paths.p, e->path_off.p, 1, text_len + 1, &tmp, &sp);
}

int tsg_scan_part_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_text, uint64_t text_base,
                         uint64_t text_len, uint64_t own_lo, uint64_t own_hi, uint64_t file_len, const char* path,
                         uint8_t** blob, size_t* blob_len) {
  try {
    return scan_part_impl(e, rs, d_text, text_base, text_len, own_lo, own_hi, file_len, path, blob, blob_len);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

void tsg_part_free(uint8_t* blob) {
  if (blob) blob_release(blob);
}

static int scan_merge_impl(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_file, uint64_t file_len,
                           const char* path, const uint8_t* const* blobs, const size_t* blob_lens, size_t n_parts,
                           tsg_result** out) {
  if (!e || !rs || !out || !d_file || (n_parts && (!blobs || !blob_lens))) return TSG_ERR_INVALID_ARG;
  *out = nullptr;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  uint8_t sep = 1;
  HIP_TRY(hipMemcpy(&sep, d_file + file_len, 1, hipMemcpyDeviceToHost));
  if (sep != 0) {
    set_last_error("split: d_file[file_len] must be the NUL separator");
    return TSG_ERR_INVALID_ARG;
  }
  int rc = stage_one_file(e, file_len, path);
  if (rc) return rc;
  std::vector<std::pair<const uint8_t*, size_t>> parts;
  for (size_t i = 0; i < n_parts; ++i) {
    if (!blobs[i]) return TSG_ERR_INVALID_ARG;
    parts.push_back({blobs[i], blob_lens[i]});
  }
  SplitIo sp;
  sp.mode = 2;
  sp.file_len = file_len;
  sp.parts = &parts;
  auto* res = new tsg_result();
  rc = run_pipeline(e, rs, d_file, e->off.p, e->paths.p, e->path_off.p, 1, file_len + 1, res, &sp);
  if (rc) {
    delete res;
    return rc;
  }
  *out = res;
  return TSG_OK;
}

int tsg_scan_merge_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_file, uint64_t file_len,
                          const char* path, const uint8_t* const* blobs, const size_t* blob_lens, size_t n_parts,
                          tsg_result** out) {
  try {
    return scan_merge_impl(e, rs, d_file, file_len, path, blobs, blob_lens, n_parts, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

// Host files -> device batch layout (contents each followed by one NUL, then
// paths) in e->data / e->off / e->paths / e->path_off: packed into the
// engine's pinned staging buffer by up to 16 threads (the copy, not PCIe,
// bounds a single-threaded pack), then one H2D per array.
static int stage_host_batch(tsg_engine* e, const tsg_file* files, size_t n_files, uint64_t* nbytes_out) {
  std::vector<uint64_t> off(n_files + 1, 0), poff(n_files + 1, 0);
  for (size_t i = 0; i < n_files; ++i) {
    off[i + 1] = off[i] + files[i].len + 1;
    poff[i + 1] = poff[i] + (files[i].path ? strlen(files[i].path) : 0);
  }
  const uint64_t nbytes = off[n_files], pbytes = poff[n_files];
  const size_t need = nbytes + pbytes + 16;
  if (e->h_stage_n < need) {
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    e->h_stage = nullptr;
    e->h_stage_n = 0;
    const size_t cap = need + need / 4;
    unsigned flags = hipHostMallocDefault;
    if (const char* v = experiment_env("TSG_STAGE_NC")) flags = atoi(v) ? hipHostMallocNonCoherent : flags;
    HIP_TRY(hipHostMalloc((void**)&e->h_stage, cap, flags));
    e->h_stage_n = cap;
  }
  uint8_t* h = e->h_stage;
  if (e->data.ensure(nbytes + 16) != hipSuccess || e->off.ensure(n_files + 1) != hipSuccess ||
      e->paths.ensure(pbytes + 16) != hipSuccess || e->path_off.ensure(n_files + 1) != hipSuccess) {
    set_last_error("hipMalloc failed");
    return TSG_ERR_DEVICE;
  }
  hipStream_t s = e->stream;
  const auto t0 = std::chrono::steady_clock::now();
  // bytes [lo, hi) of the packed batch: the parts of the files (and their
  // NUL separators) that fall inside
  auto pack_range = [&](uint64_t lo, uint64_t hi) {
    size_t i = (size_t)(std::upper_bound(off.begin(), off.end(), lo) - off.begin());
    i = i ? i - 1 : 0;
    for (; i < n_files && off[i] < hi; ++i) {
      const uint64_t fs = off[i], fe = fs + files[i].len;  // separator at fe
      const uint64_t a = std::max(fs, lo), b = std::min(fe, hi);
      if (a < b) memcpy(h + a, files[i].data + (a - fs), b - a);
      if (fe >= lo && fe < hi) h[fe] = 0;
    }
  };
  const unsigned nt = nbytes < (64u << 20) ? 1u : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  // chunk DMAs alternate over this many streams (A/B: TSG_DMA_STREAMS, exp build)
  int n_dma = 1;
  if (const char* v = experiment_env("TSG_DMA_STREAMS")) n_dma = atoi(v) == 2 ? 2 : 1;
  if (n_dma == 2) HIP_TRY(ensure_side(e));
  auto dma_stream = [&](uint64_t c) { return (n_dma == 2 && (c & 1)) ? e->side : s; };
  // chunks: the DMA of chunk k is issued as soon as every worker has packed
  // its slice of it, while the workers go on to the next chunks (one set of
  // threads per call: a spawn / join per 64 MiB chunk cost ~0.3 ms each)
  uint64_t kStageChunk = 64ull << 20;
  if (const char* v = experiment_env("TSG_STAGE_CHUNK_MB")) kStageChunk = std::max(1, atoi(v)) * (1ull << 20);
  const uint64_t n_chunks = (nbytes + kStageChunk - 1) / kStageChunk;
  bool ok = true;
  if (nt == 1 || n_chunks == 0) {
    for (uint64_t lo = 0; lo < nbytes && ok; lo += kStageChunk) {
      const uint64_t hi = std::min(nbytes, lo + kStageChunk);
      pack_range(lo, hi);
      ok = hipMemcpyAsync(e->data.p + lo, h + lo, hi - lo, hipMemcpyHostToDevice, dma_stream(lo / kStageChunk)) ==
           hipSuccess;
    }
  } else {
    std::unique_ptr<std::atomic<unsigned>[]> done(new std::atomic<unsigned>[n_chunks]);
    for (uint64_t c = 0; c < n_chunks; ++c) done[c].store(0, std::memory_order_relaxed);
    std::atomic<bool> stop{false};
    auto worker = [&](unsigned t) {
      for (uint64_t c = 0; c < n_chunks && !stop.load(std::memory_order_relaxed); ++c) {
        const uint64_t lo = c * kStageChunk, hi = std::min(nbytes, lo + kStageChunk);
        pack_range(lo + (hi - lo) * t / nt, lo + (hi - lo) * (t + 1) / nt);
        done[c].fetch_add(1, std::memory_order_release);
      }
    };
    std::vector<std::thread> th;
    unsigned started = 0;
    try {
      for (; started < nt; ++started) th.emplace_back(worker, started);
    } catch (const std::system_error&) {
    }
    for (unsigned t = started; t < nt; ++t) {  // slices of threads that could not start: done here, up front
      for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t lo = c * kStageChunk, hi = std::min(nbytes, lo + kStageChunk);
        pack_range(lo + (hi - lo) * t / nt, lo + (hi - lo) * (t + 1) / nt);
        done[c].fetch_add(1, std::memory_order_release);
      }
    }
    for (uint64_t c = 0; c < n_chunks && ok; ++c) {
      while (done[c].load(std::memory_order_acquire) < nt) std::this_thread::yield();
      const uint64_t lo = c * kStageChunk, hi = std::min(nbytes, lo + kStageChunk);
      ok = hipMemcpyAsync(e->data.p + lo, h + lo, hi - lo, hipMemcpyHostToDevice, dma_stream(c)) == hipSuccess;
    }
    if (!ok) stop.store(true);
    for (auto& t : th) t.join();
  }
  for (size_t i = 0; i < n_files; ++i)
    if (files[i].path) memcpy(h + nbytes + poff[i], files[i].path, poff[i + 1] - poff[i]);
  const auto t1 = std::chrono::steady_clock::now();
  if (ok && n_dma == 2)  // (the side stream's chunks before anything on the main stream reads the batch)
    ok = hipEventRecord(e->ev_side, e->side) == hipSuccess && hipStreamWaitEvent(s, e->ev_side, 0) == hipSuccess;
  ok = ok && hipMemcpyAsync(e->paths.p, h + nbytes, pbytes, hipMemcpyHostToDevice, s) == hipSuccess &&
       hipMemcpyAsync(e->off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
       hipMemcpyAsync(e->path_off.p, poff.data(), poff.size() * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
       hipStreamSynchronize(s) == hipSuccess;
  if (!ok) {
    set_last_error("host-to-device copy failed");
    return TSG_ERR_DEVICE;
  }
  const auto t2 = std::chrono::steady_clock::now();
  e->stage_ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
  e->stage_ms[1] = std::chrono::duration<double, std::milli>(t2 - t1).count();
  *nbytes_out = nbytes;
  return TSG_OK;
}

static int scan_impl(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files,
                     tsg_result** out) {
  if (!e || !rs || !out || (n_files && !files)) return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  *out = nullptr;
  HIP_TRY(hipSetDevice(e->device));
  uint64_t nbytes = 0;
  int src = stage_host_batch(e, files, n_files, &nbytes);
  if (src) return src;
  auto* res = new tsg_result();
  int rc = run_pipeline(e, rs, e->data.p, e->off.p, e->paths.p, e->path_off.p, n_files, nbytes, res);
  if (rc) {
    delete res;
    return rc;
  }
  res->impl.timings.resize(std::max<size_t>(res->impl.timings.size(), 20), 0.0);
  res->impl.timings[18] = e->stage_ms[0];  // host pack into pinned staging
  res->impl.timings[19] = e->stage_ms[1];  // H2D
  *out = res;
  return TSG_OK;
}

static int scan_device_impl(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data,
                            const uint64_t* d_offsets, const uint8_t* d_paths,
                            const uint64_t* d_path_offsets, size_t n_files, tsg_result** out) {
  if (!e || !rs || !out || !d_offsets || !d_path_offsets) return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  *out = nullptr;
  HIP_TRY(hipSetDevice(e->device));
  uint64_t nbytes = 0;
  HIP_TRY(hipMemcpy(&nbytes, d_offsets + n_files, 8, hipMemcpyDeviceToHost));
  auto* res = new tsg_result();
  int rc = run_pipeline(e, rs, d_data, d_offsets, d_paths, d_path_offsets, n_files, nbytes, res);
  if (rc) {
    delete res;
    return rc;
  }
  *out = res;
  return TSG_OK;
}

// SecretAnalyzer.Analyze over raw files (secret.go:79-113): pack -> H2D ->
// IsBinary (k_binary) -> '\r' deletion by compaction (k_strip_*) -> scan.
// The batch is in e->data / e->off / e->paths / e->path_off (staged by the
// caller of this function, under e->mu, since w0).
static int analyze_staged_batch(tsg_engine* e, const tsg_ruleset* rs, size_t n_files, uint64_t nbytes,
                                std::chrono::steady_clock::time_point w0, tsg_result** out) {
  hipStream_t s = e->stream;
  const uint32_t nf = (uint32_t)n_files;
  const uint64_t n_blk = (nbytes + kStripBlock - 1) / kStripBlock;
  if (e->bin8.ensure(n_files + 1) != hipSuccess || e->n_drop.ensure(1) != hipSuccess ||
      e->blk_kept.ensure(n_blk + 1) != hipSuccess || e->blk_base.ensure(n_blk + 1) != hipSuccess) {
    set_last_error("hipMalloc failed");
    return TSG_ERR_DEVICE;
  }
  const uint8_t* d_data = e->data.p;
  const uint64_t* d_off = e->off.p;
  uint64_t kept = nbytes;
  std::vector<uint8_t> bin(n_files, 0);
  if (nf) {
    HIP_TRY(hipMemsetAsync(e->n_drop.p, 0, 8, s));
    hipLaunchKernelGGL(k_binary, dim3((uint32_t)(((uint64_t)nf * 64 + 255) / 256)), dim3(256), 0, s, e->data.p,
                       e->off.p, nf, e->bin8.p, e->n_drop.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_strip_count, dim3((uint32_t)n_blk), dim3(256), 0, s, e->data.p, nbytes, e->blk_kept.p);
    HIP_TRY(hipGetLastError());
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, e->blk_kept.p, e->blk_base.p, (int)n_blk, s));
    HIP_TRY(e->cub_tmp.ensure(tmp + 1));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(e->cub_tmp.p, tmp, e->blk_kept.p, e->blk_base.p, (int)n_blk, s));
    uint64_t last[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&last[0], e->blk_base.p + n_blk - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&last[1], e->blk_kept.p + n_blk - 1, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(bin.data(), e->bin8.p, n_files, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    kept = last[0] + last[1];
    if (kept != nbytes) {  // some '\r' or a binary file: compact
      const uint64_t n_chunks = (nbytes + 15) / 16;
      HIP_TRY(e->strip_out.ensure(kept + 16));
      HIP_TRY(e->strip_off.ensure(n_files + 1));
      HIP_TRY(e->chunk_pos.ensure(n_chunks + 1));
      hipLaunchKernelGGL(k_strip_compact, dim3((uint32_t)n_blk), dim3(256), 0, s, e->data.p, nbytes,
                         e->blk_base.p, e->strip_out.p, e->chunk_pos.p);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_strip_offsets, dim3((nf + 1 + 255) / 256), dim3(256), 0, s, e->data.p, e->off.p, nf,
                         e->chunk_pos.p, kept, e->strip_off.p);
      HIP_TRY(hipGetLastError());
      d_data = e->strip_out.p;
      d_off = e->strip_off.p;
    }
  }
  const auto w1 = std::chrono::steady_clock::now();
  auto* res = new tsg_result();
  int rc = run_pipeline(e, rs, d_data, d_off, e->paths.p, e->path_off.p, n_files, kept, res);
  if (rc) {
    delete res;
    return rc;
  }
  const auto w2 = std::chrono::steady_clock::now();
  auto& R = res->impl;
  for (size_t i = 0; i < n_files && i < R.file_flags.size(); ++i)
    if (bin[i]) R.file_flags[i] |= TSG_FILE_BINARY;
  // findings were built on the device from the CR-stripped batch Scan saw

  res->impl.timings.resize(std::max<size_t>(res->impl.timings.size(), 23), 0.0);
  res->impl.timings[18] = e->stage_ms[0];  // host pack into pinned staging
  res->impl.timings[19] = e->stage_ms[1];  // H2D
  {
    const auto w3 = std::chrono::steady_clock::now();
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    res->impl.timings[20] = ms(w0, w1);  // staging + front end (IsBinary, strip)
    res->impl.timings[21] = ms(w1, w2);  // scan pipeline
    res->impl.timings[22] = ms(w2, w3);  // findings
  }
  *out = res;
  return TSG_OK;
}

static int analyze_impl(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files,
                        tsg_result** out) {
  if (!e || !rs || !out || (n_files && !files)) return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  *out = nullptr;
  HIP_TRY(hipSetDevice(e->device));
  const auto w0 = std::chrono::steady_clock::now();
  uint64_t nbytes = 0;
  int src = stage_host_batch(e, files, n_files, &nbytes);
  if (src) return src;
  return analyze_staged_batch(e, rs, n_files, nbytes, w0, out);
}

// ---- caller-filled staging (tsg_staging_*): files read straight into
// page-locked memory in the batch layout, so a staged call needs no host pack
struct tsg_staging {
  uint8_t* buf = nullptr;  // hipHostMalloc'd, `cap` bytes: contents, each followed by its NUL separator
  size_t cap = 0;
  std::vector<uint64_t> off{0};   // n + 1 batch offsets
  std::vector<uint64_t> poff{0};  // n + 1 path offsets
  std::string paths;
};

int tsg_staging_create(size_t capacity_bytes, tsg_staging** out) {
  if (!out || capacity_bytes == 0) return TSG_ERR_INVALID_ARG;
  *out = nullptr;
  try {
    auto* st = new tsg_staging();
    if (hipHostMalloc((void**)&st->buf, capacity_bytes, hipHostMallocDefault) != hipSuccess) {
      delete st;
      set_last_error("hipHostMalloc failed");
      return TSG_ERR_DEVICE;
    }
    st->cap = capacity_bytes;
    *out = st;
    return TSG_OK;
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

int tsg_staging_add(tsg_staging* st, const char* path, uint64_t len, uint8_t** dst) {
  if (!st || !dst) return TSG_ERR_INVALID_ARG;
  *dst = nullptr;
  const uint64_t at = st->off.back();
  if (len >= kMaxFileBytes || at + len + 1 > st->cap) {
    set_last_error(st->off.size() == 1 ? "staging: the file is larger than the staging buffer"
                                       : "staging: buffer full (run the batch, reset, add again)");
    return TSG_ERR_FULL;
  }
  try {
    const size_t plen = path ? strlen(path) : 0;
    st->paths.append(path ? path : "", plen);
    st->poff.push_back(st->paths.size());
    st->off.push_back(at + len + 1);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
  st->buf[at + len] = 0;  // the separator
  *dst = st->buf + at;
  return TSG_OK;
}

size_t tsg_staging_count(const tsg_staging* st) { return st ? st->off.size() - 1 : 0; }
size_t tsg_staging_bytes(const tsg_staging* st) { return st ? st->off.back() : 0; }

void tsg_staging_reset(tsg_staging* st) {
  if (!st) return;
  st->off.assign(1, 0);
  st->poff.assign(1, 0);
  st->paths.clear();
}

void tsg_staging_free(tsg_staging* st) {
  if (!st) return;
  if (st->buf) (void)hipHostFree(st->buf);
  delete st;
}

// The staged batch -> e->data / e->off / e->paths / e->path_off: one H2D per
// array straight from the page-locked buffer.
static int upload_staging(tsg_engine* e, const tsg_staging* st, uint64_t* nbytes_out) {
  const size_t n = st->off.size() - 1;
  const uint64_t nbytes = st->off.back(), pbytes = st->paths.size();
  if (e->data.ensure(nbytes + 16) != hipSuccess || e->off.ensure(n + 1) != hipSuccess ||
      e->paths.ensure(pbytes + 16) != hipSuccess || e->path_off.ensure(n + 1) != hipSuccess) {
    set_last_error("hipMalloc failed");
    return TSG_ERR_DEVICE;
  }
  hipStream_t s = e->stream;
  const auto t0 = std::chrono::steady_clock::now();
  bool ok = (nbytes == 0 || hipMemcpyAsync(e->data.p, st->buf, nbytes, hipMemcpyHostToDevice, s) == hipSuccess) &&
            (pbytes == 0 || hipMemcpyAsync(e->paths.p, st->paths.data(), pbytes, hipMemcpyHostToDevice, s) == hipSuccess) &&
            hipMemcpyAsync(e->off.p, st->off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemcpyAsync(e->path_off.p, st->poff.data(), (n + 1) * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  if (!ok) {
    set_last_error("host-to-device copy failed");
    return TSG_ERR_DEVICE;
  }
  e->stage_ms[0] = 0.0;  // nothing packed: the caller read the files into place
  e->stage_ms[1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *nbytes_out = nbytes;
  return TSG_OK;
}

static int staged_impl(tsg_engine* e, const tsg_ruleset* rs, const tsg_staging* st, bool analyze, tsg_result** out) {
  if (!e || !rs || !st || !out) return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  *out = nullptr;
  HIP_TRY(hipSetDevice(e->device));
  const auto w0 = std::chrono::steady_clock::now();
  uint64_t nbytes = 0;
  int rc = upload_staging(e, st, &nbytes);
  if (rc) return rc;
  const size_t n = st->off.size() - 1;
  if (analyze) return analyze_staged_batch(e, rs, n, nbytes, w0, out);
  auto* res = new tsg_result();
  rc = run_pipeline(e, rs, e->data.p, e->off.p, e->paths.p, e->path_off.p, n, nbytes, res);
  if (rc) {
    delete res;
    return rc;
  }
  res->impl.timings.resize(std::max<size_t>(res->impl.timings.size(), 20), 0.0);
  res->impl.timings[18] = e->stage_ms[0];
  res->impl.timings[19] = e->stage_ms[1];
  *out = res;
  return TSG_OK;
}

int tsg_analyze_staged(tsg_engine* e, const tsg_ruleset* rs, const tsg_staging* st, tsg_result** out) {
  try {
    return staged_impl(e, rs, st, true, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

int tsg_scan_staged(tsg_engine* e, const tsg_ruleset* rs, const tsg_staging* st, tsg_result** out) {
  try {
    return staged_impl(e, rs, st, false, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

int tsg_analyze(tsg_engine* e, const tsg_ruleset* rs, const tsg_file* files, size_t n_files, tsg_result** out) {
  try {
    return analyze_impl(e, rs, files, n_files, out);
  } catch (const std::exception& ex) {
    set_last_error(std::string("internal error: ") + ex.what());
    return TSG_ERR_INTERNAL;
  }
}

int tsg_gate_device(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* d_data, const uint64_t* d_offsets,
                    size_t n_files, uint32_t* h_gates_out, size_t gate_words_per_file) {
  if (!e || !rs || !d_offsets) return TSG_ERR_INVALID_ARG;
  {
    std::string err;
    const tsg_ruleset* g = gate_ruleset(rs, &err);
    if (!g) {
      set_last_error(err);
      return TSG_ERR_INTERNAL;
    }
    rs = g;
  }
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  int rc = upload_ruleset(e, rs);
  if (rc) return rc;
  const RuleSetDev& RS = e->img.view;
  const uint32_t nf = (uint32_t)n_files;
  uint64_t nbytes = 0;
  HIP_TRY(hipMemcpy(&nbytes, d_offsets + n_files, 8, hipMemcpyDeviceToHost));
  hipStream_t s = e->stream;
  const auto wall0 = std::chrono::steady_clock::now();
  if (!e->events) {
    for (auto& ev : e->ev) HIP_TRY(hipEventCreate(&ev));
    e->events = true;
  }
  e->fast_timed = false;
  if (e->nl_pending) {  // (an earlier scan's side newline count still writes nl_blocks)
    HIP_TRY(hipStreamWaitEvent(s, e->ev_nl[1], 0));
    e->nl_pending = false;
  }
  HIP_TRY(e->ctrl.ensure(1));
  HIP_TRY(e->file_kw.ensure((size_t)nf * RS.kw_words + 1));
  HIP_TRY(e->file_flags.ensure(nf + 1));
  HIP_TRY(hipMemsetAsync(e->ctrl.p, 0, sizeof(Ctrl), s));
  HIP_TRY(hipMemsetAsync(e->file_kw.p, 0, ((size_t)nf * RS.kw_words + 1) * 4, s));
  HIP_TRY(hipMemsetAsync(e->file_flags.p, 0, (nf + 1) * 4, s));
  HIP_TRY(e->hits.ensure(1));
  ScanParams P{};
  P.big = e->img.big_view;
  P.data = d_data;
  P.off = d_offsets;
  P.nbytes = nbytes;
  P.n_files = nf;
  P.rs = RS;
  P.file_kw = e->file_kw.p;
  P.file_flags = e->file_flags.p;
  P.hits = e->hits.p;
  P.hit_cap = 0;  // prefilter only: hits are counted, not stored
  e->nl_lazy = true;  // (no line numbers here)
  P.ctrl = e->ctrl.p;
  HIP_TRY(e->fold_pos.ensure(std::max<uint64_t>(1 << 16, e->fold_need)));
  P.fold_pos = e->fold_pos.p;
  P.fold_cap = e->fold_pos.n;
  const uint64_t n_nlb = nbytes / kNlBlock + 2;
  HIP_TRY(e->nl_blocks.ensure(n_nlb));
  HIP_TRY(hipMemsetAsync(e->nl_blocks.p, 0, n_nlb * 4, s));
  P.nl_blocks = e->nl_blocks.p;
  P.kw_plain = kKwReadFirst;
  if (const char* v = experiment_env("TSG_KW_PLAIN")) P.kw_plain = strtoull(v, nullptr, 10);  // (A/B)
  P.kw_drain_at = kKwDrainAt;
  if (const char* v = experiment_env("TSG_KW_DRAIN")) P.kw_drain_at = (uint32_t)strtoul(v, nullptr, 10);  // (A/B)
  P.kw_off = experiment_env("TSG_KW_OFF") != nullptr;  // (A/B)
  const bool want_gates = h_gates_out && nf && gate_words_per_file;
  const uint32_t R = (uint32_t)rs->rules.size();
  std::vector<uint32_t> csr;
  if (want_gates) {
    // rule -> keyword-id CSR (host, per ruleset: not per byte), gates on the GPU
    csr.resize(R + 1);
    std::vector<uint32_t> ids;
    for (uint32_t r = 0; r < R; ++r) {
      csr[r] = (uint32_t)ids.size();
      for (auto& k : rs->rules[r].keywords) {
        if (k.empty()) { ids.push_back(0xFFFFFFFFu); continue; }
        ids.push_back((uint32_t)(std::find(rs->keywords.begin(), rs->keywords.end(), k) - rs->keywords.begin()));
      }
    }
    csr[R] = (uint32_t)ids.size();
    if (RS.kw_words <= kGateMaskWords) {  // k_rule_gates_mask's table instead of the CSR
      const uint32_t W = RS.kw_words;
      std::vector<uint32_t> masks((size_t)R * W + (R + 31) / 32, 0u);
      uint32_t* always = masks.data() + (size_t)R * W;
      for (uint32_t r = 0; r < R; ++r) {
        bool all = csr[r] == (r + 1 < R ? csr[r + 1] : (uint32_t)ids.size());
        for (uint32_t k = csr[r]; k < (r + 1 < R ? csr[r + 1] : (uint32_t)ids.size()); ++k) {
          if (ids[k] == 0xFFFFFFFFu) all = true;
          else masks[(size_t)r * W + (ids[k] >> 5)] |= 1u << (ids[k] & 31);
        }
        if (all) always[r >> 5] |= 1u << (r & 31);
      }
      csr.swap(masks);
    } else {
      csr.insert(csr.end(), ids.begin(), ids.end());
    }
    HIP_TRY(e->gate_rules.ensure(csr.size()));
    HIP_TRY(hipMemcpyAsync(e->gate_rules.p, csr.data(), csr.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(e->gate_out.ensure((size_t)nf * gate_words_per_file));
  }
  // The whole pass -- scan, fold windows, non-ASCII keywords, rule gates and
  // their D2H -- is queued before the one host wait, which then checks the
  // scan's buffers: every kernel after the scan clamps to them (k_fold_windows
  // to fold_cap), keyword bits are idempotent and the gate words are
  // rewritten, so an overflowed attempt is simply redone with grown buffers.
  // (One host round trip fewer than checking between the scan and the rest.)
  HIP_TRY(hipEventRecord(e->ev[8], s));
  bool scanned = false;
  for (int attempt = 0; attempt < 3 && !scanned; ++attempt) {
    if (nbytes) {
      if ((rc = launch_scan(e, P, true))) return rc;
      if ((rc = launch_fold_windows(e, P, false))) return rc;
      if ((rc = launch_uni_keywords(e, P))) return rc;
    }
    if (e->events) HIP_TRY(hipEventRecord(e->ev[9], s));
    if (want_gates) {
      const size_t words = gate_words_per_file;
      if (RS.kw_words <= kGateMaskWords)
        hipLaunchKernelGGL(k_rule_gates_mask, dim3((nf + 255) / 256), dim3(256), 0, s, e->file_kw.p, RS.kw_words, nf,
                           e->gate_rules.p, R, e->gate_out.p, (uint32_t)words);
      else
        hipLaunchKernelGGL(k_rule_gates, dim3((nf + 255) / 256), dim3(256), 0, s, e->file_kw.p, RS.kw_words, nf,
                           e->gate_rules.p, R, e->gate_out.p, (uint32_t)words);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(h_gates_out, e->gate_out.p, (size_t)nf * words * 4, hipMemcpyDeviceToHost, s));
    }
    Ctrl c;
    if ((rc = read_ctrl(e, &c))) return rc;  // (the stream's one synchronisation)
    if (!nbytes) {
      scanned = true;
      break;
    }
    const bool ev_lost = (rs->ac.fast.size() || P.big.blob) && c.ev_overflow > e->ev_overflow.n;
    const bool outs_lost = P.big.blob && c.outputs > P.big_out_cap;  // (k_big_walk's records)
    if (outs_lost) e->big_out_need = c.outputs + (c.outputs >> 2);
    if (!ev_lost && !outs_lost && c.n_fold <= P.fold_cap) {
      scanned = true;
      break;
    }
    if (ev_lost) e->ev_ovf_need = c.ev_overflow + (c.ev_overflow >> 2);  // events were lost: grow and rescan
    if (c.n_fold > P.fold_cap) {
      e->fold_need = c.n_fold + (c.n_fold >> 2);
      HIP_TRY(e->fold_pos.ensure(e->fold_need));
      P.fold_pos = e->fold_pos.p;
      P.fold_cap = e->fold_pos.n;
    }
    HIP_TRY(hipMemsetAsync(e->ctrl.p, 0, offsetof(Ctrl, n_caps), s));
  }
  if (!scanned) {
    set_last_error("internal: scan buffers still overflowed after regrowing them twice");
    return TSG_ERR_INTERNAL;
  }
  e->gate_tm.assign(18, 0.0);
  if (e->events && nbytes) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e->ev[8], e->ev[9]));
    e->gate_tm[0] = ms;  // scan + report + special gate
    if (e->fast_timed) {
      HIP_TRY(hipEventElapsedTime(&ms, e->ev[10], e->ev[11]));
      e->gate_tm[17] = ms;
    } else {
      e->gate_tm[7] = e->gate_tm[0];
    }
  }
  e->gate_tm[15] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
  return TSG_OK;
}

int tsg_diag_sort_pairs(tsg_engine* e, const uint64_t* keys, const uint32_t* vals, size_t n, int end_bit,
                        uint64_t* out_keys, uint32_t* out_vals, int small) {
  if (!e || (n && (!keys || !vals || !out_keys || !out_vals)) || end_bit < 1 || end_bit > 64)
    return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  if (!n) return TSG_OK;
  DBuf<uint64_t> k[2];
  DBuf<uint32_t> v[2];
  int rc = TSG_OK;
  auto run = [&]() -> int {
    for (int i = 0; i < 2; ++i) {
      HIP_TRY(k[i].ensure(n));
      HIP_TRY(v[i].ensure(n));
    }
    HIP_TRY(hipMemcpyAsync(k[0].p, keys, n * 8, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(v[0].p, vals, n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(sort_pairs(e, k[0].p, k[1].p, v[0].p, v[1].p, n, end_bit, e->stream, small != 0));
    HIP_TRY(hipMemcpyAsync(out_keys, k[1].p, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(out_vals, v[1].p, n * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return TSG_OK;
  };
  rc = run();
  for (int i = 0; i < 2; ++i) {
    k[i].release();
    v[i].release();
  }
  return rc;
}

int tsg_engine_force_verify_split(tsg_engine* e, int on) {
  if (!e) return TSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(e->mu);
  e->verify_split = on ? 1 : 0;
  return TSG_OK;
}

int tsg_engine_gate_timings(const tsg_engine* e, double* ms, size_t n, size_t* n_out) {
  if (!e || (!ms && n)) return TSG_ERR_INVALID_ARG;
  const size_t k = std::min(n, e->gate_tm.size());
  for (size_t i = 0; i < k; ++i) ms[i] = e->gate_tm[i];
  if (n_out) *n_out = k;
  return TSG_OK;
}

size_t tsg_result_loc_count(const tsg_result* r) { return r ? r->impl.locs.size() : 0; }
const tsg_loc* tsg_result_locs(const tsg_result* r) { return r ? r->impl.locs.data() : nullptr; }
size_t tsg_result_file_count(const tsg_result* r) { return r ? r->impl.file_flags.size() : 0; }
const uint8_t* tsg_result_file_flags(const tsg_result* r) { return r ? r->impl.file_flags.data() : nullptr; }
size_t tsg_result_findings(const tsg_result* r, size_t file, const tsg_finding** out) {
  if (out) *out = nullptr;
  if (!r || !out || !r->impl.have_findings) return 0;
  const auto& R = r->impl;
  auto lo = std::lower_bound(R.frec.begin(), R.frec.end(), (uint32_t)file,
                             [](const FindRec& a, uint32_t f) { return a.file < f; });
  if (lo == R.frec.end() || lo->file != file) return 0;
  auto hi = lo;
  while (hi != R.frec.end() && hi->file == file) ++hi;
  std::lock_guard<std::mutex> lk(R.fmu);
  auto it = R.fcache.find((uint32_t)file);
  if (it == R.fcache.end()) {  // views into the result's string arena, built once per file
    auto& slot = R.fcache[(uint32_t)file];
    size_t nl = 0;
    for (auto q = lo; q != hi; ++q) nl += q->n_lines;
    slot.second.reserve(nl);
    for (auto q = lo; q != hi; ++q) {
      tsg_finding fd{};
      fd.file = q->file;
      const tsg_loc& lq = R.locs[q->loc];
      fd.rule = lq.rule;
      fd.start_line = q->line;
      fd.end_line = q->line;
      fd.match = arena_at(R, q->m_off);
      fd.match_len = q->m_len;
      fd.start = lq.start;
      fd.end = lq.end;
      fd.n_lines = q->n_lines;
      // (FindRec: lines [first, first + n_lines), consecutive in the arena)
      const uint32_t first = q->line >= 3 ? q->line - 3 : 0;
      const uint64_t sep = (q->c_off & kArenaDense) ? 1 : 0;
      uint64_t off = q->c_off;
      for (uint32_t k = 0; k < q->n_lines; ++k) {
        tsg_line tl{};
        tl.number = first + k + 1;
        tl.content = arena_at(R, off);
        tl.content_len = q->c_len[k];
        const bool cause = tl.number == q->line;
        tl.is_cause = cause;
        tl.first_cause = cause;
        tl.last_cause = cause;
        slot.second.push_back(tl);
        off += q->c_len[k] + sep;
      }
      slot.first.push_back(fd);
    }
    size_t k = 0;  // line pointers after the vector stopped growing
    for (auto& fd : slot.first) {
      fd.lines = fd.n_lines ? slot.second.data() + k : nullptr;
      k += fd.n_lines;
    }
    it = R.fcache.find((uint32_t)file);
  }
  *out = it->second.first.data();
  return it->second.first.size();
}
int tsg_result_timings(const tsg_result* r, double* ms, size_t n, size_t* n_out) {
  if (!r) return TSG_ERR_INVALID_ARG;
  size_t k = std::min(n, r->impl.timings.size());
  for (size_t i = 0; i < k; ++i) ms[i] = r->impl.timings[i];
  if (n_out) *n_out = r->impl.timings.size();
  return TSG_OK;
}
void tsg_result_free(tsg_result* r) { delete r; }

}  // extern "C"
